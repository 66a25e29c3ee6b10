"""Frame sharding across GPUs.

Every frame is self-contained in the reference: the LO phase restarts, filtfilt pads and
initialises per frame, Welch segments never cross frames (pypanadapter_spectrum.py:
2091-2111; pypanadapter_thread.py:1516-1538).  So G ranks (one process per GPU, launched
by torch.distributed.run) each take a contiguous block of frames and run their own plan
with no collective on the data path.  The only cross-rank step is the ordered gather of
the finished rows (a few KB per line) to the rank that owns the display, which then
pushes them into its waterfall in frame order.  Config 4 (one IF stream per GPU) is the
same partition with a per-rank f_LO.
"""
from __future__ import annotations

from typing import Callable, Sequence

import numpy as np


def frame_range(n_frames: int, rank: int, world: int) -> range:
    """Contiguous, balanced block of frames for `rank` (sizes differ by at most one)."""
    if not (0 <= rank < world) or n_frames < 0:
        raise ValueError("bad rank/world/n_frames")
    base, extra = divmod(n_frames, world)
    start = rank * base + min(rank, extra)
    return range(start, start + base + (1 if rank < extra else 0))


def lo_for_rank(rank: int, f0: float = 1.0, spacing: float = 150e3) -> float:
    """Config 4: f_LO,k = 1 Hz + k * 150 kHz, one IF centre frequency per GPU."""
    return f0 + rank * spacing


def run_sharded(frames: np.ndarray, rows_fn: Callable[[np.ndarray], np.ndarray],
                rank: int, world: int, dist=None, dst: int = 0):
    """Compute this rank's rows, then gather all rows to `dst` in frame order.

    `rows_fn` maps (F_local, L) IQ -> (F_local, W) rows (a ZoomFFT plan's `rows` on a GPU
    rank).  Returns the (F, W) rows on `dst` and None elsewhere.  With dist=None (single
    process) it is just rows_fn(frames).
    """
    if dist is None or world == 1:
        return rows_fn(frames)
    import torch
    mine = frame_range(len(frames), rank, world)
    local = np.asarray(rows_fn(frames[mine.start:mine.stop]), dtype=np.float32)
    W = local.shape[1] if local.ndim == 2 and local.size else 0
    sizes = [len(frame_range(len(frames), r, world)) for r in range(world)]
    width = torch.tensor([W], dtype=torch.int64)
    dist.all_reduce(width, op=dist.ReduceOp.MAX)
    W = int(width.item())
    pad = max(sizes)
    buf = torch.zeros((pad, W), dtype=torch.float32)
    if len(local):
        buf[:len(local)] = torch.from_numpy(local)
    gathered = [torch.zeros((pad, W), dtype=torch.float32) for _ in range(world)] if rank == dst else None
    dist.gather(buf, gather_list=gathered, dst=dst)
    if rank != dst:
        return None
    return np.concatenate([g[:s].numpy() for g, s in zip(gathered, sizes)], axis=0)


def push_in_order(waterfall, rows: Sequence[np.ndarray]) -> None:
    """Feed gathered rows to a reference-shaped Waterfall in frame order."""
    for r in rows:
        waterfall.image_update(np.array(r, dtype=np.float64))
