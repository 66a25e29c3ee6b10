"""Multi-rank path on CPU (gloo, world_size 2): partition + ordered row gather.

The GPU ranks run ZoomFFT plans; here each rank's rows come from the float64 oracle
(the checker), which exercises exactly the sharding/gather logic the GPU path uses."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from pypanadapter_amd.shard import frame_range, lo_for_rank, run_sharded


def test_frame_range_partitions():
    for n in (0, 1, 7, 8, 4096, 4099):
        for world in (1, 2, 3, 8):
            covered = []
            for r in range(world):
                rg = frame_range(n, r, world)
                covered.extend(rg)
                assert abs(len(rg) - n / world) < 1
            assert covered == list(range(n))
    with pytest.raises(ValueError):
        frame_range(10, 2, 2)
    assert lo_for_rank(3) == 1.0 + 450e3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, frames, out_path):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import coracle

    def rows_fn(x):
        return np.stack([coracle.psd_row(f, 2.4e6, 256, 4, 64) for f in x]) if len(x) else \
            np.zeros((0, 64), np.float32)

    rows = run_sharded(frames, rows_fn, rank, world, dist=dist)
    if rank == 0:
        np.save(out_path, rows)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n_frames", [5, 2])
def test_gloo_two_ranks_match_single_process(tmp_path, n_frames):
    from oracle import coracle
    from pypanadapter_amd import synth
    coracle.build()
    frames = np.stack([synth.make_iq(16384, 2.4e6, 60 + f, n_fft=256, zoom=4, n_win=64)
                       for f in range(n_frames)])
    out = str(tmp_path / "rows.npy")
    mp.spawn(_worker, args=(2, _free_port(), frames, out), nprocs=2, join=True)
    got = np.load(out)
    ref = np.stack([coracle.psd_row(f, 2.4e6, 256, 4, 64) for f in frames]).astype(np.float32)
    np.testing.assert_array_equal(got, ref)


def _gpu_worker(rank, world, port, frames, path, out_path):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from pypanadapter_amd import ZoomFFT, device_count
    dev = rank % device_count()  # rank r on GPU r on a node; both on device 0 on a 1-GPU box
    with ZoomFFT(1024, 8, 2.4e6, device=dev) as plan:
        assert plan.device == dev
        plan.set_path(path)
        rows = run_sharded(frames, plan.rows, rank, world, dist=dist)
    if rank == 0:
        np.save(out_path, rows)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("path", [0, 3])
def test_hip_two_ranks_bit_equal_single_process(tmp_path, path):
    """rows of frames sharded over two rank processes (HIP plans, gloo
    gather) equal the single-process rows bit for bit."""
    from pypanadapter_amd import ZoomFFT, synth
    frames = np.stack([synth.make_iq(65536, 2.4e6, 300 + f, n_fft=1024, zoom=8, n_win=128)
                       for f in range(7)])
    with ZoomFFT(1024, 8, 2.4e6) as plan:
        plan.set_path(path)
        ref = plan.rows(frames)
    out = str(tmp_path / "rows.npy")
    mp.spawn(_gpu_worker, args=(2, _free_port(), frames, path, out), nprocs=2, join=True)
    np.testing.assert_array_equal(np.load(out), ref)
