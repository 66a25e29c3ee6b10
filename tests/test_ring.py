"""Host IQ ring: pypanadapter_thread.py's `Data` (T:1400-1483) as the pinned
double-buffered zfft_ring.  Oracle: oracle/iqring.py (the reference class restated without
QtCore / the NewtRap pacer)."""
import threading

import numpy as np
import pytest

from oracle.iqring import Data


def _ring(chunk=64, dtype="complex64"):
    from pypanadapter_amd import IQRing
    return IQRing(chunk, dtype)


def test_add_take_sequence_matches_reference_data():
    rng = np.random.default_rng(1)
    chunk = 64
    ring, ref = _ring(chunk), Data(chunk)
    for step in range(400):
        if rng.random() < 0.8:
            n = int(rng.integers(0, 3 * chunk))
            x = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
            ring.add(x)
            ref.add(x)
            assert ring.state() == (ref.size, ref.real_size, ref.total_size), step
        else:
            got, tot = ring.take()
            want, wtot = ref.take()
            assert tot == wtot
            np.testing.assert_array_equal(got, want)
    ring.close()


def test_fold_back_keeps_the_reference_frame_order():
    """A chunk that would pass max_size is written at 0: the frame is then the newest chunk
    followed by the older tail, as data[:real_size] is in the reference."""
    ring, ref = _ring(4), Data(4)  # max_size 64
    for k in range(3):
        x = np.full(25, k + 1, dtype=np.complex64)
        ring.add(x)
        ref.add(x)
    got, tot = ring.take()
    want, _ = ref.take()
    np.testing.assert_array_equal(got, want)
    assert tot == 75 and len(got) == 50 and got[0] == 3 and got[30] == 2
    with pytest.raises(ValueError):
        ring.add(np.zeros(65, np.complex64))  # longer than the ring
    ring.close()


def test_raw_uint8_iq_ring():
    ring, ref = _ring(32, "cu8"), Data(32, dtype=np.uint16)
    rng = np.random.default_rng(3)
    for _ in range(30):
        b = rng.integers(0, 256, size=2 * int(rng.integers(1, 80)), dtype=np.uint8)
        ring.add(b)
        ref.add(b.view(np.uint16))  # one I,Q byte pair per sample
    got, tot = ring.take()
    want, wtot = ref.take()
    assert tot == wtot
    np.testing.assert_array_equal(got.view(np.uint16), want)
    ring.close()


def test_frames_are_never_torn_by_a_concurrent_producer():
    """The reference hands the worker a view the reader keeps writing into;
    here a drained frame stays intact while add() continues: every frame is whole chunks
    in the order the Data semantics give, and the counts add up."""
    chunk = 256
    ring = _ring(chunk)
    n_chunks = 3000
    stop = threading.Event()
    frames = []

    def consumer():
        while not stop.is_set() or ring.state()[1]:
            f, tot = ring.take()
            if len(f):
                frames.append((f.copy(), tot))

    th = threading.Thread(target=consumer)
    th.start()
    for k in range(n_chunks):
        ring.add(np.full(chunk, k + 1, dtype=np.complex64))
    stop.set()
    th.join()
    assert sum(t for _, t in frames) == n_chunks * chunk
    seen = 0
    for f, tot in frames:
        v = f.real.astype(np.int64)
        assert len(v) % chunk == 0
        blocks = v.reshape(-1, chunk)
        assert np.all(blocks == blocks[:, :1])  # whole chunks only
        seen += tot
    assert seen == n_chunks * chunk
    ring.close()


@pytest.mark.gpu
def test_ring_process_is_psd_update(oracle_lib):
    """zfft_ring_process = PSD.update (T:1513-1548): the drained frame's row, bit-identical
    to the plan's own row of that frame; frames shorter than fft_size give no row."""
    from pypanadapter_amd import ZoomFFT
    from pypanadapter_amd import synth
    N, z, W = 1024, 4, 256
    x = synth.make_iq(40000, 2.4e6, 77, n_fft=N, zoom=z, n_win=W).astype(np.complex64)
    ring = _ring(2500)
    with ZoomFFT(N, z, 2.4e6, n_win=W) as plan:
        ring.add(x[:1000])
        assert ring.process(plan) is None  # 1000 < fft_size
        for i in range(0, 40000, 2500):
            ring.add(x[i:i + 2500])
        row = ring.process(plan)
        np.testing.assert_array_equal(row, plan.rows(x))
        from conftest import assert_row_close
        assert_row_close(row, oracle_lib.psd_row(x, 2.4e6, N, z, W), "ring frame")
    ring.close()


def test_data_facade_reference_calls():
    """The reference's own call sequence (T:2191, T:1516-1520) on the facade."""
    from pypanadapter_amd import Data as RingData
    d = RingData(16).new_complex()
    ref = Data(16)
    rng = np.random.default_rng(9)
    for _ in range(50):
        x = (rng.standard_normal(40) + 1j * rng.standard_normal(40)).astype(np.complex64)
        d.add(x)
        ref.add(x)
        if rng.random() < 0.3:
            d.get_data_start()
            size = d.real_size
            chunk = d.data[:size]
            d.get_data_end()
            want, _ = ref.take()
            np.testing.assert_array_equal(chunk, want)
    assert d.maxsize == 256
