"""Multi-GPU work split of the path tracer (one process per GPU, torch.distributed over RCCL).

Two decompositions, both without any data-path exchange until the single merge per step:
  * row bands (bench.py default; the BASELINE north star's "image tiled across the GPUs with an
    RCCL gather of per-tile sample accumulators"): rank r owns the band set (band, N, r), i.e.
    the `band`-row bands r, r+N, r+2N, ... of the frame, interleaved so every rank gets the same
    mix of background-heavy and scene-heavy rows (FullRaytracer.cs:71-72 makes contiguous tiles
    instead, which is imbalanced).  Each rank renders its rows with all of the step's samples
    into a gather slot (rt_render_bands_device), the slots are gathered onto rank 0 and added
    into the frame's accumulators (SampleSet: sum RGB, samples, misses --
    RaytracerCore/Raytracing/SampleSet.cs:8-44; the merge of FullRaytracer.cs:326-344).
  * sample sharding (bench.py --split samples): every rank renders the whole frame with its own
    disjoint range of sample indices, and the accumulators are summed onto rank 0 with one
    reduce.  The result equals a single render of all ranges (the RNG is keyed by (seed, pixel,
    sample index), include/rtcore_rng.h).

Slot layout (the device layout of rt_render_bands_device / rt_frame): plane = rows of the
tallest band set x width; a float64 slot of 4 * plane elements holds the R | G | B sum planes,
then (viewed as int32) the samples plane and the misses plane, each row-major over the rank's
rows in frame order.
"""
from __future__ import annotations

from typing import List, Sequence

BAND = 8  # rows per band: with 8, every split of 1080 or 2160 rows is within one band of even


def sample_base(step: int, rank: int, world: int, spp: int) -> int:
    """First sample index rank `rank` renders in step `step` (disjoint across ranks and steps)."""
    return (step * world + rank) * spp


def band_rows(height: int, world: int, rank: int, band: int = BAND) -> List[int]:
    """Frame rows owned by `rank` under the row-interleaved band split (band set (band, world, rank))."""
    rows = []
    for b in range(rank, (height + band - 1) // band, world):
        rows.extend(range(b * band, min(height, (b + 1) * band)))
    return rows


def slot_rows(height: int, world: int, band: int = BAND) -> int:
    """Rows of the tallest band set: a gather slot's plane is slot_rows * width."""
    return max(len(band_rows(height, world, r, band)) for r in range(world))


def slot_views(slot, plane: int):
    """(sum planes f64 [3*plane], samples int32 [plane], misses int32 [plane]) views of a float64 slot."""
    import torch

    counts = slot[3 * plane:4 * plane].view(dtype=torch.int32)
    return slot[:3 * plane], counts[:plane], counts[plane:]


def row_index(height: int, world: int, band: int = BAND, device=None) -> list:
    """Per rank: a long tensor of its frame rows (for the scatter of gathered slots)."""
    import torch

    return [torch.tensor(band_rows(height, world, r, band), dtype=torch.long, device=device) for r in range(world)]


def scatter_slots(frame_sum, frame_n, frame_m, slots: Sequence, rows: Sequence, width: int, plane: int) -> None:
    """Adds every rank's slot into the frame accumulators (frame_sum: 3*H*W f64 planes, frame_n /
    frame_m: H*W int32, all row-major): rank g's slot row i is frame row rows[g][i]."""
    height = frame_n.numel() // width
    if len(slots) == 1 and plane == height * width:  # one rank owns every row, in order
        s, n, m = slot_views(slots[0], plane)
        frame_sum.add_(s)
        frame_n.add_(n)
        frame_m.add_(m)
        return
    fs = frame_sum.view(3, height, width)
    fn = frame_n.view(height, width)
    fm = frame_m.view(height, width)
    p_rows = plane // width
    for slot, idx in zip(slots, rows):
        k = idx.numel()
        if k == 0:
            continue
        s, n, m = slot_views(slot, plane)
        fs.index_add_(1, idx, s.view(3, p_rows, width)[:, :k])
        fn.index_add_(0, idx, n.view(p_rows, width)[:k])
        fm.index_add_(0, idx, m.view(p_rows, width)[:k])


def gather_slots(slot, gather_list, dist=None, dst: int = 0, async_op: bool = False) -> list:
    """Gathers each rank's slot into gather_list on `dst` (one collective; no-op for 1 rank, where
    gather_list[0] must be the slot itself).  With async_op the work handles are returned."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return []
    mine = dist.get_rank() == dst
    if slot.is_cuda and dist.get_backend() == "gloo":  # bench.py's one-GPU rehearsal: gloo gathers host tensors
        host = [t.cpu() for t in gather_list] if mine else None
        dist.gather(slot.cpu(), host, dst=dst)
        if mine:
            for t, h in zip(gather_list, host):
                t.copy_(h)
        return []
    w = dist.gather(slot, gather_list if mine else None, dst=dst, async_op=async_op)
    return [w] if w is not None else []


def merge_accumulators(tensors: Sequence, dist=None, dst: int = 0, async_op: bool = False) -> list:
    """Sum each rank's step accumulators onto `dst` (one reduce per tensor; no-op for 1 rank).
    With async_op the work handles are returned; wait() on them before reading the result."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return []
    works = [dist.reduce(t, dst=dst, async_op=async_op) for t in tensors]
    return [w for w in works if w is not None]
