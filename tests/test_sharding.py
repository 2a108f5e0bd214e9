"""Gloo rehearsals (world size 2 and 3) of bench.py's multi-GPU splits (CPU only).

The CPU oracle stands in for the GPU.  Row bands (the default): each rank renders its band set
into a gather slot, the slots are gathered onto rank 0 and scattered into the frame exactly as
bench.py does over RCCL, and the frame must equal one whole-frame render.  Sample sharding:
each rank renders its sample range, the accumulators are reduced onto rank 0, and the merged
frame must equal one render of all sample ranges.  Also checks the band split covers the frame.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from raytracercore_amd import sharding
from raytracercore_amd.sharding import band_rows, merge_accumulators, sample_base

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H, SPP, STEPS = 12, 10, 3, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path, async_merge=False):
    import sys

    sys.path.insert(0, ROOT)
    from oracle.oracle import OracleScene

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    orc = OracleScene.from_file(os.path.join(ROOT, "tests", "golden", "scenes", "die.txt"))
    orc.set_size(W, H)
    f_sum = torch.zeros((W, H, 3), dtype=torch.float64)
    f_n = torch.zeros((W, H), dtype=torch.int64)
    f_m = torch.zeros((W, H), dtype=torch.int64)
    for step in range(STEPS):
        s, n, m, _ = orc.render_tile(0, 0, W, H, SPP, seed=5, sample_base=sample_base(step, rank, world, SPP))
        ts, tn, tm = torch.from_numpy(s), torch.from_numpy(n.astype(np.int64)), torch.from_numpy(m.astype(np.int64))
        works = merge_accumulators([ts, tn, tm], dist, async_op=async_merge)
        for w in works:
            w.wait()
        if rank == 0:
            f_sum += ts
            f_n += tn
            f_m += tm
    if rank == 0:
        np.savez(out_path, s=f_sum.numpy(), n=f_n.numpy(), m=f_m.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("async_merge", [False, True])
def test_sample_sharded_reduce_equals_single_render(tmp_path, async_merge):
    """bench.py's merge: reduce each step's accumulators onto rank 0 (async as in bench.py)."""
    out = str(tmp_path / "merged.npz")
    mp.spawn(_worker, args=(2, _free_port(), out, async_merge), nprocs=2, join=True)
    got = np.load(out)
    from oracle.oracle import OracleScene

    orc = OracleScene.from_file(os.path.join(ROOT, "tests", "golden", "scenes", "die.txt"))
    orc.set_size(W, H)
    s, n, m, _ = orc.render_tile(0, 0, W, H, SPP * 2 * STEPS, seed=5, sample_base=0)
    assert np.array_equal(got["n"], n) and np.array_equal(got["m"], m)
    assert np.allclose(got["s"], s, rtol=1e-12, atol=1e-12)


BW, BH = 10, 27  # 4 bands of 8 rows and one of 3: ragged band sets at world 2 and 3


def _band_slot(orc, rank, world, spp, seed):
    """The rank's gather slot (sharding slot layout) rendered band by band by the oracle."""
    plane = sharding.slot_rows(BH, world) * BW
    slot = torch.zeros(4 * plane, dtype=torch.float64)
    s_, n_, m_ = sharding.slot_views(slot, plane)
    s3, n2, m2 = s_.view(3, -1, BW), n_.view(-1, BW), m_.view(-1, BW)
    i = 0
    for b in range(rank, (BH + sharding.BAND - 1) // sharding.BAND, world):
        y0 = b * sharding.BAND
        bh = min(sharding.BAND, BH - y0)
        s, n, m, _ = orc.render_tile(0, y0, BW, bh, spp, seed=seed, sample_base=0)  # [x, y] order
        s3[:, i:i + bh] = torch.from_numpy(s.transpose(2, 1, 0).copy())
        n2[i:i + bh] = torch.from_numpy(n.T.astype(np.int32))
        m2[i:i + bh] = torch.from_numpy(m.T.astype(np.int32))
        i += bh
    return slot, plane


def _band_worker(rank, world, port, out_path):
    import sys

    sys.path.insert(0, ROOT)
    from oracle.oracle import OracleScene

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    orc = OracleScene.from_file(os.path.join(ROOT, "tests", "golden", "scenes", "bounce.txt"))
    orc.set_size(BW, BH)
    slot, plane = _band_slot(orc, rank, world, 4, 3)
    glist = [torch.empty_like(slot) for _ in range(world)] if rank == 0 else None
    for w in sharding.gather_slots(slot, glist, dist, async_op=True):
        w.wait()
    if rank == 0:
        f_sum = torch.zeros(3 * BW * BH, dtype=torch.float64)
        f_n = torch.zeros(BW * BH, dtype=torch.int32)
        f_m = torch.zeros(BW * BH, dtype=torch.int32)
        sharding.scatter_slots(f_sum, f_n, f_m, glist, sharding.row_index(BH, world), BW, plane)
        np.savez(out_path, s=f_sum.numpy(), n=f_n.numpy(), m=f_m.numpy())
    dist.barrier()
    dist.destroy_process_group()


def _whole_frame(spp, seed):
    from oracle.oracle import OracleScene

    orc = OracleScene.from_file(os.path.join(ROOT, "tests", "golden", "scenes", "bounce.txt"))
    orc.set_size(BW, BH)
    s, n, m, _ = orc.render_tile(0, 0, BW, BH, spp, seed=seed, sample_base=0)
    return s.transpose(2, 1, 0).reshape(-1), n.T.reshape(-1), m.T.reshape(-1)


@pytest.mark.parametrize("world", [2, 3])
def test_band_gather_equals_whole_frame(tmp_path, world):
    """bench.py's default merge: band-set slots gathered onto rank 0 and scattered into the frame
    equal one whole-frame render bit for bit (ragged sets: 27 rows in bands of 8)."""
    out = str(tmp_path / "bands.npz")
    mp.spawn(_band_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    got = np.load(out)
    s, n, m = _whole_frame(4, 3)
    assert np.array_equal(got["n"], n) and np.array_equal(got["m"], m)
    assert np.array_equal(got["s"], s)


def test_band_scatter_single_rank():
    """World size 1 (bench.py at N = 1): the rank's own slot is scattered without a collective."""
    import sys

    sys.path.insert(0, ROOT)
    from oracle.oracle import OracleScene

    orc = OracleScene.from_file(os.path.join(ROOT, "tests", "golden", "scenes", "bounce.txt"))
    orc.set_size(BW, BH)
    slot, plane = _band_slot(orc, 0, 1, 4, 3)
    assert sharding.gather_slots(slot, [slot], None) == []
    f_sum = torch.zeros(3 * BW * BH, dtype=torch.float64)
    f_n = torch.zeros(BW * BH, dtype=torch.int32)
    f_m = torch.zeros(BW * BH, dtype=torch.int32)
    sharding.scatter_slots(f_sum, f_n, f_m, [slot], sharding.row_index(BH, 1), BW, plane)
    s, n, m = _whole_frame(4, 3)
    assert np.array_equal(f_n.numpy(), n) and np.array_equal(f_m.numpy(), m)
    assert np.array_equal(f_sum.numpy(), s)


@pytest.mark.parametrize("h,world", [(1080, 8), (1080, 3), (2160, 8), (37, 2), (16, 4)])
def test_band_rows_partition_the_frame(h, world):
    owned = [band_rows(h, world, r) for r in range(world)]
    allrows = sorted(r for rows in owned for r in rows)
    assert allrows == list(range(h))
    sizes = [len(o) for o in owned]
    assert max(sizes) - min(sizes) <= sharding.BAND
    assert max(sizes) == sharding.slot_rows(h, world)


@pytest.mark.parametrize("h,world", [(1080, 8), (1080, 3), (2160, 8), (37, 2), (16, 4), (27, 3)])
def test_band_rows_match_library(rc, h, world):
    """The Python split and the library's band sets (rt_band_rows, host only) agree."""
    for r in range(world):
        assert rc.band_rows_count(h, sharding.BAND, world, r) == len(band_rows(h, world, r))


def test_sample_bases_disjoint():
    seen = set()
    for step in range(3):
        for rank in range(4):
            b = sample_base(step, rank, 4, 256)
            rng = set(range(b, b + 256))
            assert not (seen & rng)
            seen |= rng


@pytest.mark.parametrize("h,w,world", [(27, 5, 2), (27, 5, 3), (37, 11, 2), (40, 7, 3), (1080, 16, 3)])
def test_frame_path_layout_matches_sharding(rc, h, w, world):
    """The two multi-GPU paths share one band layout.  The product path is the
    library's rt_frame (one process drives every GPU: render each band set into a gather slot,
    ncclGather to device 0, scatter on the host -- rt_frame_render); bench.py's per-rank path
    renders the same slots through rt_render_bands_device and scatters them with sharding.py.
    Here random slots in that layout are scattered both ways and must give the same frame bit for
    bit: the library's rt_scatter_band_slot (rt_frame_render's merge, [x, y] order) against
    sharding.scatter_slots (row-major planes); and both size the slot alike."""
    torch = pytest.importorskip("torch")
    plane = sharding.slot_rows(h, world) * w
    assert rc.band_slot_rows(h, sharding.BAND, world) * w == plane
    gen = torch.Generator().manual_seed(h * 100 + world)
    slots = []
    for r in range(world):
        slot = torch.zeros(4 * plane, dtype=torch.float64)
        s_, n_, m_ = sharding.slot_views(slot, plane)
        k = len(band_rows(h, world, r)) * w  # the set's rows; the rest of each plane stays unused (0)
        s_.view(3, plane)[:, :k] = torch.rand(3, k, generator=gen, dtype=torch.float64)
        n_[:k] = torch.randint(0, 1000, (k,), generator=gen, dtype=torch.int32)
        m_[:k] = torch.randint(0, 1000, (k,), generator=gen, dtype=torch.int32)
        slots.append(slot)
    # the per-rank host's merge (bench.py rank 0)
    f_sum = torch.zeros(3 * h * w, dtype=torch.float64)
    f_n = torch.zeros(h * w, dtype=torch.int32)
    f_m = torch.zeros(h * w, dtype=torch.int32)
    sharding.scatter_slots(f_sum, f_n, f_m, slots, sharding.row_index(h, world), w, plane)
    # the frame path's merge, into SampleSet[w, h] order
    out = (np.zeros((w, h, 3)), np.zeros((w, h), np.uint32), np.zeros((w, h), np.uint32))
    for r in range(world):
        rc.scatter_band_slot(slots[r].numpy(), plane, w, h, sharding.BAND, world, r, out)
    assert np.array_equal(out[0].transpose(2, 1, 0), f_sum.view(3, h, w).numpy())
    assert np.array_equal(out[1].T.astype(np.int64), f_n.view(h, w).numpy().astype(np.int64))
    assert np.array_equal(out[2].T.astype(np.int64), f_m.view(h, w).numpy().astype(np.int64))
    # every frame row owned by exactly one rank
    assert np.all(out[1].T.sum(axis=1) == f_n.view(h, w).numpy().sum(axis=1))
