"""Multi-GPU work split of the path tracer (one process per GPU, torch.distributed over RCCL).

Two decompositions, both without any data-path exchange until the single merge:
  * sample sharding (bench.py, weak scaling): every rank renders the whole frame with its
    own disjoint range of sample indices; the per-pixel accumulators (SampleSet: sum RGB,
    samples, misses -- RaytracerCore/Raytracing/SampleSet.cs:8-44) are summed onto rank 0
    with one reduce.  Perfect load balance; the result equals a single render of all ranges
    (the RNG is keyed by (seed, pixel, sample index), include/rtcore_rng.h).
  * row bands (rt_render_frame_multi, tiles of one frame): rank r owns 16-row bands
    r, r+N, r+2N, ...; interleaving balances background-heavy rows
    (FullRaytracer.cs:71-72 makes contiguous tiles instead, which is imbalanced).
"""
from __future__ import annotations

from typing import List, Sequence


def sample_base(step: int, rank: int, world: int, spp: int) -> int:
    """First sample index rank `rank` renders in step `step` (disjoint across ranks and steps)."""
    return (step * world + rank) * spp


def band_rows(height: int, world: int, rank: int, band: int = 16) -> List[int]:
    """Frame rows owned by `rank` under the row-interleaved band split."""
    rows = []
    for b in range((height + band - 1) // band):
        if b % world == rank:
            rows.extend(range(b * band, min(height, (b + 1) * band)))
    return rows


def merge_accumulators(tensors: Sequence, dist=None, dst: int = 0, async_op: bool = False) -> list:
    """Sum each rank's step accumulators onto `dst` (one reduce per tensor; no-op for 1 rank).
    With async_op the work handles are returned; wait() on them before reading the result."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return []
    works = [dist.reduce(t, dst=dst, async_op=async_op) for t in tensors]
    return [w for w in works if w is not None]
