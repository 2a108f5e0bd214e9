"""Diagnostic: one GPU's share of the N-GPU bench step -- band set (8, N, 0) of bounce.txt 1080p
at N x 256 spp -- timed for N = 1, 2, 4, 8 (weak scaling: the kernel time should stay flat).
usage: python tools/band_timing.py [config]"""
import os
import sys

sys.path.insert(0, os.getcwd())
import torch

import raytracercore_amd as rc
from raytracercore_amd import sharding

scene = rc.SceneLoader.from_file(rc.scene_path(sys.argv[1] if len(sys.argv) > 1 else "bounce.txt"))
W, H = 1920, 1080
g = rc.GpuRaytracer(scene, 0, size=(W, H))
dev = torch.device("cuda", 0)
rays = torch.zeros(1, dtype=torch.int64, device=dev)
for n in (1, 2, 4, 8):
    plane = sharding.slot_rows(H, n) * W
    slot = torch.zeros(4 * plane, dtype=torch.float64, device=dev)
    s_, n_, m_ = sharding.slot_views(slot, plane)
    ms = []
    for rep in range(4):
        slot.zero_()
        rays.zero_()
        g.render_bands_device(8, n, 0, 256 * n, 0, rep * 256 * n, s_.data_ptr(), n_.data_ptr(), m_.data_ptr(), plane,
                              rays.data_ptr(), 0)
        torch.cuda.synchronize()
        ms.append(g.last_kernel_ms())
    print(f"N={n} band set 0: kernel ms {[round(x, 2) for x in ms]} rays {int(rays.item())}", flush=True)
