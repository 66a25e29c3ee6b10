"""The host IQ ring against sequences of the reference's OWN `Data` class
(pypanadapter_thread.py:1400-1483, driven by tools/gen_golden.py through T's module with
the Qt stubs): add / fold-back / over-long chunks / the PSD worker's drain (T:1516-1520) /
the target setter (T:1474-1479) and add's target clip (T:1445).  CPU only: without a device
the ring's buffers are ordinary memory."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

RING = np.load(os.path.join(GOLDEN, "ring.npz"))
META = json.load(open(os.path.join(GOLDEN, "cases.json")))["ring"]


def _replay(m, make, check_target=True):
    name = m["name"]
    ops, states = RING[f"{name}/ops"], RING[f"{name}/states"]
    targets = RING[f"{name}/targets"]
    d = make(m)
    for i, op in enumerate(ops):
        if op == 0:
            d.add(RING[f"{name}/in{i}"])
        elif op == 3:
            with pytest.raises(ValueError):
                d.add(RING[f"{name}/in{i}"])
        elif op == 2:
            d.target = float(targets[i])
        else:
            d.get_data_start()
            size = d.real_size
            chunk = d.data[:size]
            total = d.total_size
            d.get_data_end()
            np.testing.assert_array_equal(chunk, RING[f"{name}/frame{i}"], err_msg=f"{name} op {i}")
            assert total == RING[f"{name}/frame_total{i}"][0], (name, i)
        st = states[i]
        assert (d.size, d.ring_real_size, d.ring_total_size) == tuple(int(v) for v in st[:3]), (name, i)
        if check_target:
            assert float(d.target_size) == st[3], (name, i, d.target_size, st[3])


class _Facade:
    """pypanadapter_amd.Data plus the ring's live counts (the reference's attributes)."""

    def __init__(self, m):
        from pypanadapter_amd import Data
        self.d = Data(m["chunk_size"], fft_size=m["fft_size"])
        (self.d.new_real if m["real"] else self.d.new_complex)()

    def __getattr__(self, k):
        return getattr(self.d, k)

    def __setattr__(self, k, v):
        if k == "d":
            object.__setattr__(self, k, v)
        else:
            setattr(self.d, k, v)

    @property
    def ring_real_size(self):
        return self.d._ring.state()[1]

    @property
    def ring_total_size(self):
        return self.d._ring.state()[2]


@pytest.mark.parametrize("m", META, ids=[m["name"] for m in META])
def test_data_facade_replays_reference_sequences(m):
    _replay(m, _Facade)


class _Restated:
    """oracle/iqring.py (the checker's restatement) under the same replay: pinned too."""

    def __init__(self, m):
        from oracle.iqring import Data as R
        self.r = R(m["chunk_size"], dtype=np.float32 if m["real"] else np.complex64)
        self.data = None
        self.real_size = self.total_size = 0

    def add(self, x):
        if len(x) > self.r.max_size:
            self.r.size = 0
            raise ValueError("chunk longer than the ring")
        self.r.add(x)

    def get_data_start(self):
        self.data, self.total_size = self.r.take()
        self.real_size = len(self.data)

    def get_data_end(self):
        pass

    @property
    def size(self):
        return self.r.size

    @property
    def ring_real_size(self):
        return self.r.real_size

    @property
    def ring_total_size(self):
        return self.r.total_size


@pytest.mark.parametrize("m", META, ids=[m["name"] for m in META])
def test_restated_ring_oracle_replays_reference_sequences(m):
    _replay(m, _Restated, check_target=False)


def test_fixture_covers_the_reference_paths():
    """Fold-back, target clip above 8192, the setter's refusals, over-long chunks, real data."""
    by = {m["name"]: m for m in META}
    assert by["real64"]["real"] and by["c520"]["max_size"] > 8192
    st = RING["c520/states"][:, 3]
    assert st.max() == 8320.0 and 8192.0 in st  # clip(…, 8192, max_size) seen at both ends
    assert (RING["c64_overlong/ops"] == 3).any()
    folds = 0
    for m in META:
        s = RING[f"{m['name']}/states"]
        ops = RING[f"{m['name']}/ops"]
        folds += int(((ops == 0)[1:] & (s[1:, 0] < s[:-1, 0])).sum())
    assert folds > 10
