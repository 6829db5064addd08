"""Frame-parallel execution across GPUs: one process per GPU, no data-path
collective.

The reference converts one video per ffmpeg process and never shards
(SURVEY.md §8e): frames are independent, S1-S8 are per-pixel, and the peak
comes from static metadata, so there is no cross-frame state.  Ranks
therefore take contiguous frame ranges (C4: frame i -> rank i // ceil(F/N))
and run the same kernel on their own HBM.  The only collectives are:

* init: broadcast of the tone-map parameters and the LUT lattice
  (65^3 x 3 fp32 = 3,295,500 B) from rank 0 — RCCL on GPU ranks, gloo on CPU;
* end: SUM of {pixels, output checksum} and MAX of the elapsed time;
* dynamic peak detection only (BT.2390 / spline, peak_detect=1): the peak
  is smoothed by a recurrence over the whole sequence, which is the one real
  exchange step.  Each rank measures its own frames' statistics (two floats
  per frame), all ranks all-gather them, and each replays the frames before
  its range into its context (h2s_peak_feed) before converting, so the
  sharded output equals the sequential one (sync_peak_state).

Everything here works with either backend; the CPU tests run it under gloo
with world_size 2 (tests/test_dist.py).
"""
from __future__ import annotations

import math
from typing import Any, Optional, Tuple

import numpy as np

from .chain import TonemapParams


def shard_range(nframes: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [start, stop) of the frames ``rank`` owns.

    ceil-sized blocks, so frame i belongs to rank i // ceil(F/N); trailing
    ranks may get fewer (or zero) frames when F is not a multiple of N."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f'bad rank {rank} for world {world}')
    if nframes < 0:
        raise ValueError(f'nframes must be >= 0, got {nframes}')
    per = math.ceil(nframes / world) if nframes else 0
    start = min(rank * per, nframes)
    return start, min(start + per, nframes)


def owner_of(frame: int, nframes: int, world: int) -> int:
    per = math.ceil(nframes / world)
    return frame // per


def _dist():
    import torch.distributed as dist
    return dist


def _comm_device(device: Any):
    """gloo moves CPU tensors, RCCL device tensors."""
    import torch
    if _dist().get_backend() == 'gloo':
        return torch.device('cpu')
    return torch.device(device)


def broadcast_setup(params: Optional[TonemapParams], lattice: Optional[np.ndarray], lut_size: int,
                    device: Any = 'cpu', src: int = 0) -> Tuple[TonemapParams, np.ndarray]:
    """Rank ``src`` supplies params + lattice ([N^3, 3] fp32, r fastest);
    every rank returns identical copies.  ``lut_size`` must be known on all
    ranks (it sizes the receive buffer)."""
    import torch
    dist = _dist()
    rank = dist.get_rank()
    obj = [params if rank == src else None]
    dev = _comm_device(device)
    dist.broadcast_object_list(obj, src=src, device=None if dev.type == 'cpu' else dev)
    params = obj[0]
    if not isinstance(params, TonemapParams):
        raise RuntimeError('parameter broadcast failed')
    buf = torch.empty((lut_size ** 3, 3), dtype=torch.float32, device=dev)
    if rank == src:
        if lattice is None or lattice.shape != (lut_size ** 3, 3):
            raise ValueError(f'rank {src} must supply a [{lut_size}^3, 3] lattice')
        buf.copy_(torch.from_numpy(np.ascontiguousarray(lattice, dtype=np.float32)))
    dist.broadcast(buf, src=src)
    return params, buf.cpu().numpy()


def frame_checksum(buf: Any, first_index: int) -> int:
    """Order-sensitive checksum of a [F, samples] batch whose first row is
    global frame ``first_index``: sum_i (i + 1) * sum(frame_i).  Summing it
    over ranks gives the single-process checksum of the whole sequence."""
    import torch
    if not isinstance(buf, torch.Tensor):
        buf = torch.from_numpy(np.asarray(buf, dtype=np.int64))
    if buf.shape[0] == 0:
        return 0
    per = buf.to(torch.int64).sum(dim=1)    # 10/12-bit samples are < 2^15: int16 is exact
    w = torch.arange(first_index + 1, first_index + 1 + buf.shape[0], dtype=torch.int64, device=per.device)
    return int((per * w).sum().item())


def reduce_run(pixels: int, checksum: int, elapsed_s: float, device: Any = 'cpu') -> Tuple[int, int, float]:
    """SUM pixels and checksums, MAX elapsed time over ranks."""
    import torch
    dist = _dist()
    dev = _comm_device(device)
    s = torch.tensor([pixels, checksum], dtype=torch.int64, device=dev)
    t = torch.tensor([elapsed_s], dtype=torch.float64, device=dev)
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return int(s[0].item()), int(s[1].item()), float(t[0].item())


def gather_peak_stats(fmax: np.ndarray, favg: np.ndarray, nframes: int, device: Any = 'cpu') -> np.ndarray:
    """All-gather every rank's per-frame (max, mean) statistics into the whole
    sequence's [nframes, 2] array (ranks own contiguous shard_range blocks)."""
    import torch
    dist = _dist()
    world, rank = dist.get_world_size(), dist.get_rank()
    per = math.ceil(nframes / world) if nframes else 0
    a, b = shard_range(nframes, world, rank)
    if len(fmax) != b - a or len(favg) != b - a:
        raise ValueError(f'rank {rank} owns {b - a} frames, got {len(fmax)} statistics')
    dev = _comm_device(device)
    mine = torch.zeros((per, 2), dtype=torch.float64, device=dev)
    if b > a:
        mine[:b - a, 0] = torch.as_tensor(np.asarray(fmax, dtype=np.float64), device=dev)
        mine[:b - a, 1] = torch.as_tensor(np.asarray(favg, dtype=np.float64), device=dev)
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine)
    return torch.cat(parts).cpu().numpy()[:nframes]


def sync_peak_state(tm: Any, shard: Any, nframes: int, device: Any = 'cpu') -> np.ndarray:
    """Before converting this rank's shard under dynamic peak detection: its
    frames' statistics (``tm.peak_stats``) are gathered from every rank and
    the frames before its range are fed into ``tm``'s smoothing state
    (``tm.feed_peak``).  Returns the gathered [nframes, 2] statistics."""
    dist = _dist()
    a, _ = shard_range(nframes, dist.get_world_size(), dist.get_rank())
    fmax, favg = tm.peak_stats(shard) if shard.nframes else (np.zeros(0), np.zeros(0))
    stats = gather_peak_stats(fmax, favg, nframes, device)
    tm.reset_peak()
    if a:
        tm.feed_peak(stats[:a, 0], stats[:a, 1])
    return stats
