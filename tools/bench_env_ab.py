"""A/B of bench.py under environment settings, each setting a child process of its own (this
process never touches the GPU), in the order given, so that run-to-run drift shows up as a
difference between the repeats of one setting.
usage: tools/bench_env_ab.py "VAR=a" "VAR=b;OTHER=c d" "" "VAR=a" -- [bench.py args]
("" = the default environment).  Prints one line per run: setting, ms_per_step, kernel_ms and the instrumented launch's tests per ray."""
import json
import os
import subprocess
import sys


def main():
    argv = sys.argv[1:]
    cut = argv.index("--") if "--" in argv else len(argv)
    settings, bench_args = argv[:cut], argv[cut + 1:]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for setting in settings:
        env = dict(os.environ)
        for kv in setting.split(";"):  # "A=1;B=x y": variables separated by ';' (values may hold spaces)
            if kv.strip():
                k, v = kv.strip().split("=", 1)
                env[k] = v
        r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--no-cpu-baseline"] + bench_args,
                           env=env, capture_output=True, text=True, timeout=600)
        lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
        if r.returncode != 0 or not lines:
            print(f"{setting or 'default'}: failed rc={r.returncode}\n{r.stderr[-2000:]}", flush=True)
            sys.exit(1)
        d = json.loads(lines[-1])
        per_ray = (d.get("path_stats") or {}).get("per_ray", {})
        print(f"{setting or 'default':32s} ms_per_step {d['ms_per_step']:.3f} kernel_ms {d['kernel_ms']:.3f} "
              f"per_ray {json.dumps(per_ray)}", flush=True)


if __name__ == "__main__":
    main()
