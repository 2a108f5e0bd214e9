"""World-size-2 gloo rehearsal of the multi-GPU split (CPU only).

Each rank renders its sample range with the CPU oracle (standing in for the GPU), the
accumulators are reduced onto rank 0 exactly as bench.py does over RCCL, and the merged frame
must equal one render of all sample ranges.  Also checks the row-band split covers the frame.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

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


@pytest.mark.parametrize("h,world", [(1080, 8), (1080, 3), (37, 2), (16, 4)])
def test_band_rows_partition_the_frame(h, world):
    owned = [band_rows(h, world, r) for r in range(world)]
    allrows = sorted(r for rows in owned for r in rows)
    assert allrows == list(range(h))
    sizes = [len(o) for o in owned]
    assert max(sizes) - min(sizes) <= 16


def test_sample_bases_disjoint():
    seen = set()
    for step in range(3):
        for rank in range(4):
            b = sample_base(step, rank, 4, 256)
            rng = set(range(b, b + 256))
            assert not (seen & rng)
            seen |= rng
