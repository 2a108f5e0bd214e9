"""Device memory returned per create / render / destroy cycle, by kind (hipMemGetInfo deltas).
usage: python tools/leak_probe.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import raytracercore_amd as rc  # noqa: E402
from raytracercore_amd.scenes import mesh_scene_text  # noqa: E402

bounce = rc.SceneLoader.from_file(rc.scene_path("bounce.txt"))
die = rc.SceneLoader.from_file(rc.scene_path("die.txt"))
mesh = rc.SceneLoader.from_text(mesh_scene_text(nx=41, ny=41))


def scene(sc, trav, render=True):
    g = rc.GpuRaytracer(sc, 0, size=(96, 64), traversal=trav)
    if render:
        g.render_tile(0, 0, 96, 64, 4, seed=1)
    g.close()


def frame():
    fr = rc.GpuFrame(bounce, 0, n_gpus=1, size=(96, 64))
    fr.render(4, seed=2)
    fr.close()


kinds = {
    "bounce brute (jit)": lambda: scene(bounce, rc.RT_TRAVERSAL_AUTO),
    "bounce create only": lambda: scene(bounce, rc.RT_TRAVERSAL_AUTO, render=False),
    "die grouped (jit)": lambda: scene(die, rc.RT_TRAVERSAL_AUTO),
    "mesh bvh": lambda: scene(mesh, rc.RT_TRAVERSAL_BVH),
    "frame": frame,
}
for name, fn in kinds.items():
    fn()
    torch.cuda.synchronize()
    f0 = torch.cuda.mem_get_info(0)[0]
    deltas = []
    for _ in range(6):
        fn()
        torch.cuda.synchronize()
        f = torch.cuda.mem_get_info(0)[0]
        deltas.append((f0 - f) / 2**20)
    print(f"{name:22s} MiB held after 1..6 more cycles: " + " ".join(f"{d:.1f}" for d in deltas), flush=True)
