"""The C# drop-in's host loop, natively: tests/host/worker_host.cpp is the GpuRaytracer worker and
FullRaytracer's tile hand-out and update merge of INTEGRATION.md §3 (FullRaytracer.cs:66-72,
219-229, 297-302, 326-344; Raytracer.cs:294-330), in C++ against include/rtcore.h only.  Several
worker threads, one scene handle each, take tiles round-robin and render passes that an update
loop merges into per-pixel sums; the merged frame must match single-threaded whole-frame renders
of the same sample indices (see the source for the exact bars).  Mode "frame" runs the whole-frame
loop of the same section instead: rt_frame_submit one pass ahead of rt_frame_collect.  It is built next to the library
by the library's Makefile (`all`)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "raytracercore_amd", "worker_host")
SCENES = os.path.join(ROOT, "tests", "golden", "scenes")


def _run(*args, timeout=240):
    assert os.path.exists(BIN), "raytracercore_amd/worker_host is built by the library's Makefile"
    return subprocess.run([BIN, *map(str, args)], capture_output=True, text=True, timeout=timeout)


def test_worker_host_loads_the_library_and_refuses_without_a_device(has_gpu):
    """CPU: the binary links the library and reports a missing device instead of crashing."""
    if has_gpu:
        pytest.skip("a device is present")
    r = _run(os.path.join(SCENES, "bounce.txt"), 64, 48, 4, 2, "1spp", 1)
    assert r.returncode == 1 and "no device" in r.stdout, (r.returncode, r.stdout, r.stderr)


@pytest.mark.gpu
@pytest.mark.parametrize("scene,size,threads,passes,mode,spp", [
    ("bounce.txt", (320, 240), 4, 24, "1spp", 1),  # Raytracer.Render's one-pass contract, Placeholder misses
    ("die.txt", (320, 240), 3, 16, "1spp", 1),     # 1 x 3 tiles; depth of field, misses at the background
    ("bounce.txt", (320, 240), 4, 6, "bulk", 16),  # the recommended multi-spp calls + bulk merge
    ("die.txt", (333, 217), 6, 4, "bulk", 8),      # 3 x 2 tiles of ragged sizes
    ("bounce.txt", (320, 240), 1, 5, "frame", 16), # rt_frame: submit one pass ahead, collect, merge
    ("die.txt", (333, 217), 1, 4, "frame", 8),
])
def test_worker_host_matches_whole_frame_renders(scene, size, threads, passes, mode, spp):
    r = _run(os.path.join(SCENES, scene), size[0], size[1], threads, passes, mode, spp)
    print(r.stdout)
    last = r.stdout.strip().splitlines()[-1:]  # RCCL prints its version banner first in frame mode
    assert r.returncode == 0 and last and last[0].startswith("ok "), (r.returncode, r.stdout, r.stderr)
