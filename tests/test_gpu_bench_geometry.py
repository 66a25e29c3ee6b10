"""Parity at the benchmarked geometry itself ("what's weak" 1): the exact batch
sizes bench.py times -- cfg2 and cfg3 at F = 4096 frames, cfg5 at F = 2048 (9.8 / 9.7 / 17 GB
of IQ built on the device by bench.make_frames) -- through the auto schedule (round 6: the PC walk for every one of them), with
sampled frames including the first, both sides of a 64-frame boundary, the middle and the
last two compared against the float64 oracle under the fp32 gate.  Reaches the
> 4 GiB input offsets and the grid's last workgroup."""
import numpy as np
import pytest

import bench
from conftest import assert_row_close

pytestmark = pytest.mark.gpu

PICK = lambda F: sorted({0, 1, 63, 64, F // 2, F - 2, F - 1})  # noqa: E731


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    from pypanadapter_amd import device_count
    assert device_count() >= 1
    return torch, torch.device("cuda", 0)


@pytest.mark.parametrize("config,in_dtype", [("cfg2", "complex64"), ("cfg3", "complex64"),
                                             ("cfg5", "complex64"), ("cfg2", "cu8"),
                                             ("cfg5", "complex32"), ("cfg1", "complex64")])
def test_bench_batch_rows_vs_oracle(oracle_lib, torch_dev, config, in_dtype):
    torch, dev = torch_dev
    from pypanadapter_amd import ZoomFFT
    cfg = bench.CONFIGS[config]
    F, N, z, fs = cfg["frames"], cfg["n_fft"], cfg["zoom"], cfg["fs"]
    L, W = N * cfg["n_avg"], N // cfg["zoom"]
    x = bench.make_frames(torch, F, L, cfg, dev, 1234)
    xe = bench.encode(torch, x, in_dtype)
    del x
    rows = torch.empty((F, W), dtype=torch.float32, device=dev)
    with ZoomFFT(N, z, fs, n_win=W, in_dtype=in_dtype) as plan:
        plan.set_timing(True)
        st = torch.cuda.current_stream()
        plan.process_device(xe.data_ptr(), L, F, rows.data_ptr(), st.cuda_stream)
        torch.cuda.synchronize()
        names = plan.launch_names()
    assert names[0] in ("xa_stage_mix", "pc_fir", "pc_walk", "pc_walk4", "fc_decim"), names  # the schedule the bench times
    if config == "cfg1":
        assert names[0] == "fc_decim", names  # zoom 4 at F = 4096: FC (round 6, r06fc8)
    if config in ("cfg2", "cfg3", "cfg5"):
        assert names[0] == "fc_decim", names  # zoom 8 from 16 frames per call: FC (round 6, r06fc3)
    host = rows.cpu().numpy()
    assert np.isfinite(host).all()
    for f in PICK(F):
        xf = bench.decoded_host(torch, xe, f, in_dtype)
        assert_row_close(host[f], oracle_lib.psd_row(xf, fs, N, z, W), f"{config} {in_dtype} frame {f}")
    del xe, rows
    torch.cuda.empty_cache()
