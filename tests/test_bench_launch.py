"""bench.py's launch contract on the CPU (no GPU needed): `--gpus N` without a launcher starts
N rank processes instead of measuring one GPU and calling it N, and a launcher world that
disagrees with --gpus is refused.  Here the ranks fail (no device), so the run must fail too --
never exit 0 with an `n_gpus: 1` line."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--steps", "1", "--warmup", "0", "--spp", "1", "--config", "bounce256", "--no-cpu-baseline"]


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = env.get("HIP_VISIBLE_DEVICES", "")
    env.update(kw)
    return env


def test_gpus2_without_launcher_is_not_one_gpu():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2"] + ARGS, cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert '"n_gpus": 1' not in r.stdout
    if r.returncode == 0:  # only possible where two devices exist: then it measured two
        assert '"n_gpus": 2' in r.stdout


def test_world_size_mismatch_refused():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2"] + ARGS, cwd=ROOT,
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True,
                       timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr and '"n_gpus"' not in r.stdout
