"""Rates through the host-buffer entry points (the PCIe-inclusive view; bench.py's `value` keeps the
accumulators in HBM): rt_render_tile (spp samples per call into host SampleSet buffers; column bands whose copies overlap
the next band's launch, and one launch for comparison) and
rt_render_tile_1spp (Raytracer.Render's one-pass contract, DoubleColor[w, h] per pass), 1080p
bounce.txt camera 0.  Prints one JSON line.

The one-pass figure is taken into one reused output array (a C# caller's pinned DoubleColor[w, h],
zeroed by the runtime, has its pages mapped); `render_tile_1spp_fresh` allocates a new numpy array
per pass, whose first-touch page faults the call then pays (Raytracer.Render's own pattern,
Raytracer.cs:305); `render_tile_1spp_recycled` is INTEGRATION.md §3's worker: a pool of arrays that
the update loop hands back after its merge (FullRaytracer.cs:326-344), three of them in rotation
here (the pass is queued while the previous ones wait for the merge), each allocated fresh on its
first use and timed from then on, first touches included."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import raytracercore_amd as rc  # noqa: E402

W, H = 1920, 1080
scene = rc.SceneLoader.from_file(rc.scene_path("bounce.txt"))
g = rc.GpuRaytracer(scene, 0, size=(W, H))
out = {}
BANDS = os.environ.get("HOST_TIMING_BANDS", "1").split(",")  # e.g. "1,2,4": band counts to compare
for spp in (256, 64, 16):
    # the default band count for the call against the forced counts (RTCORE_TILE_BANDS, read per call)
    for bands in BANDS + [None]:
        if bands:
            os.environ["RTCORE_TILE_BANDS"] = bands
        else:
            os.environ.pop("RTCORE_TILE_BANDS", None)
        # the caller's SampleSet arrays persist across calls (FullRaytracer.SampleSets): one set of
        # arrays, touched once by the warm-up call, then added into
        acc = (np.zeros((W, H, 3), np.float64), np.zeros((W, H), np.uint32), np.zeros((W, H), np.uint32))
        g.render_tile(0, 0, W, H, spp, seed=1, out=acc)  # warm-up (buffers, specialised build, pages)
        t0 = time.perf_counter()
        rays = 0
        n = 5
        for k in range(n):
            s, ns, ms, r = g.render_tile(0, 0, W, H, spp, seed=1, sample_base=(k + 1) * spp, out=acc)
            rays += r
        dt = (time.perf_counter() - t0) / n
        rec = {"ms_per_call": round(dt * 1e3, 2), "mrays_per_s": round(rays / n / dt / 1e6, 1)}
        nb = int(bands) if bands else (1 if W * H * spp >= 2.5e8 else 4 if W * H * spp >= 1.6e7 else 2 if W * H * spp >= 4e6 else 1)
        rec["kernel_ms"] = round(float(np.sum(g.kernel_times(nb))), 2)  # the call's launches
        rec["launches"] = nb
        # a fresh set of arrays per call (np.zeros: pages mapped by the call's first touch)
        t0 = time.perf_counter()
        for k in range(n):
            g.render_tile(0, 0, W, H, spp, seed=1, sample_base=(k + 1) * spp)
        rec["ms_per_call_fresh_arrays"] = round((time.perf_counter() - t0) / n * 1e3, 2)
        out[f"render_tile_{spp}spp" + (f"_bands{bands}" if bands else "")] = rec
buf = np.zeros((W, H, 3), np.float64)
g.render_tile_1spp(0, 0, W, H, seed=1, sample_index=0, out=buf)
for label, mode in (("render_tile_1spp", "reuse"), ("render_tile_1spp_fresh", "fresh"),
                    ("render_tile_1spp_recycled", "pool")):
    n = 40
    pool = []  # the arrays the merge has handed back
    t0 = time.perf_counter()
    for k in range(n):
        if mode == "pool":
            arr = pool.pop(0) if len(pool) >= 3 else np.zeros((W, H, 3), np.float64)
            g.render_tile_1spp(0, 0, W, H, seed=1, sample_index=k + 1, out=arr)
            pool.append(arr)  # merged, returned to the pool
        else:
            g.render_tile_1spp(0, 0, W, H, seed=1, sample_index=k + 1, out=buf if mode == "reuse" else None)
    dt = (time.perf_counter() - t0) / n
    kt = g.kernel_times(min(n, g.KERNEL_TIME_RING))
    out[label] = {"ms_per_pass": round(dt * 1e3, 3), "msamples_per_s": round(W * H / dt / 1e6, 1),
                  "kernel_ms": round(float(np.mean(kt)), 3)}
g.close()
print(json.dumps(out), flush=True)
