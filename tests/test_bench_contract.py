"""bench.py's output contract on the GPU: one JSON line with the driver's keys, the roofline and
the CPU baseline, at N = 1 and on the N > 1 path (two ranks on one device over gloo, the rehearsal
mode; RCCL refuses two ranks on one GPU).  Small spp keeps each run to seconds."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"}


def _last_json(out: str) -> dict:
    lines = [l for l in out.strip().splitlines() if l.startswith("{")]
    assert len(lines) == 1, out[-2000:]  # rank 0 prints exactly one line
    return json.loads(lines[0])


def test_bench_line_single_gpu():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--spp", "16"], cwd=ROOT,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert KEYS <= set(d)
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["scaling"] == "weak" and d["vs_baseline"] is None and d["value"] > 0 and d["ms_per_step"] > 0
    assert d["config"]["workload"].startswith("bounce.txt")
    rf = d["roofline"]
    assert {"bound", "achieved", "peak", "unit", "frac", "traffic"} <= set(rf)
    assert 0 < rf["frac"] < 1 and rf["achieved"] == pytest.approx(rf["frac"] * rf["peak"], rel=1e-2)
    cb = d["cpu_baseline"]
    assert {"value", "unit", "cores", "kind", "sample"} <= set(cb) and cb["value"] > 0 and cb["kind"] == "port"
    assert cb["host"]["nproc"] >= cb["cores"] >= 1 and cb["host"]["cpu_model"]
    # C2 is VALU-bound: SURVEY 8(d)'s FLOP formula (1095 per ray segment on bounce.txt's flat order)
    assert rf["bound"] == "valu_fp32" and d["path_stats"]["flop_per_ray"] == pytest.approx(1095, abs=1)
    assert d["multi_gpu"] is None
    # value: rays over the timed wall clock; kernel time is within it
    assert d["kernel_ms"] <= d["ms_per_step"] * 1.001


def test_bench_two_ranks_one_device():
    env = dict(os.environ, RTCORE_BENCH_SAME_DEVICE="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", "29561", "bench.py", "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--spp", "8", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert "x2" in d["config"]["parallelism"]
    mg = d["multi_gpu"]  # the N > 1 line explains itself: ranks' kernel times, collective and merge phases
    assert mg["world_size"] == 2 and len(mg["kernel_ms_per_rank"]) == 2
    assert mg["kernel_ms_min"] <= mg["kernel_ms_max"] and mg["gather_ms"] >= 0 and mg["scatter_ms"] >= 0


def test_bench_frame_split_single_process():
    """`--split frame`: the product multi-GPU path (rt_frame, one process) timed at N = 1; one JSON
    line, the per-GPU workload, and the sample bookkeeping check inside bench.py passed (rc 0)."""
    r = subprocess.run([sys.executable, "bench.py", "--split", "frame", "--gpus", "1", "--steps", "2", "--warmup", "1",
                        "--spp", "8"], cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 1 and d["value"] > 0 and d["steps"] == 2 and d["scaling"] == "weak"
    assert "rt_frame" in d["config"]["parallelism"] and d["config"]["workload"].startswith("bounce.txt")


def test_bench_gpus2_without_launcher_starts_its_ranks(tmp_path):
    """`bench.py --gpus 2` with no WORLD_SIZE starts its own two ranks (fresh processes) instead of
    quietly measuring one GPU: the line says n_gpus 2, and the gathered frame of the two ranks'
    band sets (gloo, both on device 0) equals, bit for bit, one rank rendering the same frame."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["RTCORE_BENCH_SAME_DEVICE"] = "1"
    common = ["--config", "bounce256", "--steps", "2", "--warmup", "1", "--no-cpu-baseline"]
    two, one = tmp_path / "two.npz", tmp_path / "one.npz"
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--spp", "4", "--dump", str(two)] + common,
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _last_json(r.stdout)
    assert d["n_gpus"] == 2 and d["multi_gpu"]["world_size"] == 2
    # one rank, the same frame: 2 x 4 samples per pixel per step, the same sample indices
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "1", "--spp", "8", "--dump", str(one)] + common,
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    assert _last_json(r.stdout)["n_gpus"] == 1
    a, b = np.load(two), np.load(one)
    assert int(a["samples"].sum() + a["misses"].sum()) == 256 * 256 * 8 * 3
    for k in ("sum", "samples", "misses"):
        assert np.array_equal(a[k], b[k]), k


def test_bench_world_size_must_match_gpus():
    """A launcher world that disagrees with --gpus is refused (rc != 0), never reported as n_gpus 1."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "1", "--warmup", "0", "--spp", "4",
                        "--config", "bounce256", "--no-cpu-baseline"], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode != 0 and '"n_gpus"' not in r.stdout
