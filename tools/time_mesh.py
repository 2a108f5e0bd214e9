"""Times the mesh config with and without the instrumented kernel (diagnostic)."""
import os, sys, time
sys.path.insert(0, os.getcwd())
import torch
import raytracercore_amd as rc
from raytracercore_amd.scenes import mesh_scene_text
spp = int(sys.argv[1]) if len(sys.argv) > 1 else 64
trav = {"bvh": rc.RT_TRAVERSAL_BVH, "bvh2": rc.RT_TRAVERSAL_BVH2}[sys.argv[2] if len(sys.argv) > 2 else "bvh"]
sc = rc.SceneLoader.from_text(mesh_scene_text())
W, H = 1920, 1080
g = rc.GpuRaytracer(sc, 0, size=(W, H), traversal=trav)
dev = torch.device("cuda", 0)
s = torch.zeros(3 * W * H, dtype=torch.float64, device=dev)
n = torch.zeros(W * H, dtype=torch.int32, device=dev)
m = torch.zeros_like(n)
r = torch.zeros(1, dtype=torch.int64, device=dev)
for stats in (False, True, False):
    g.set_stats(stats)
    r.zero_()
    g.render_device(0, 0, W, H, spp, 0, 0, s.data_ptr(), n.data_ptr(), m.data_ptr(), r.data_ptr(), 0)
    torch.cuda.synchronize()
    st = g.get_stats() if stats else {}
    print("stats" if stats else "plain", "kernel ms", round(g.last_kernel_ms(), 2), "rays", int(r.item()), st, flush=True)
