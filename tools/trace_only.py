#!/usr/bin/env python3
"""Wavefront-split measurement: how fast would C4's traversal stage run on its own?

1. The instrumented wide-BVH megakernel renders the C4 mesh at 1080p x SPP and logs every finished
   query (rt_debug_ray_log: origin, previous primitive, direction, closest hit).
2. The trace-only kernel (rt_debug_trace_rays: the same speculative traversal, no shading phase,
   a lane takes the next ray as soon as its query ends) re-traces the logged queries at 6, 7 and 8
   waves per SIMD; its hits must equal the logged ones.
3. Printed: the megakernel's timed rate at the bench launch (64 spp) and the trace-only rate,
   both in Grays/s, and the trace-only kernel's lane-slot split.
4. Round 5 (ray coherence): the same queries sorted the way a ray-binning step
   would group them -- by direction octant then origin Morton code, by a finer direction bin
   (cube-map face x 8 x 8) then origin, and by origin then direction -- bound what regrouping the
   megakernel's secondary rays could gain in the traversal itself.
usage: python tools/trace_only.py [SPP]
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import raytracercore_amd as rc
    from raytracercore_amd.scenes import mesh_scene_text

    spp = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    W, H = 1920, 1080
    dev = torch.device("cuda", 0)
    scene = rc.SceneLoader.from_text(mesh_scene_text())
    gpu = rc.GpuRaytracer(scene, 0, size=(W, H), traversal=rc.RT_TRAVERSAL_BVH)
    lib = gpu.lib
    d_sum = torch.zeros(3 * W * H, dtype=torch.float64, device=dev)
    d_n = torch.zeros(W * H, dtype=torch.int32, device=dev)
    d_m = torch.zeros(W * H, dtype=torch.int32, device=dev)
    d_r = torch.zeros(1, dtype=torch.int64, device=dev)

    def render(s, base):
        gpu.render_device(0, 0, W, H, s, 0, base, d_sum.data_ptr(), d_n.data_ptr(), d_m.data_ptr(), d_r.data_ptr(), 0)

    # the megakernel at the bench launch shape (64 spp), timed
    render(64, 0)
    d_r.zero_()
    render(64, 64)
    torch.cuda.synchronize()
    mk_ms = gpu.last_kernel_ms()
    mk_rays = int(d_r.item())
    out = {"megakernel": {"spp": 64, "rays": mk_rays, "kernel_ms": round(mk_ms, 3),
                          "grays_s": round(mk_rays / mk_ms / 1e6, 3)}}

    # log the queries of an instrumented launch
    cap = W * H * spp * 4
    log = torch.empty(cap * 12, dtype=torch.float32, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    assert lib.rt_debug_ray_log(gpu.handle, C.c_void_p(log.data_ptr()), cap, C.c_void_p(cnt.data_ptr())) == 0
    gpu.set_stats(True)
    d_r.zero_()
    render(spp, 1 << 30)
    torch.cuda.synchronize()
    gpu.set_stats(False)
    assert lib.rt_debug_ray_log(gpu.handle, None, 0, None) == 0
    n = int(cnt.item())
    assert n <= cap and n == int(d_r.item()), (n, cap, int(d_r.item()))
    logged = log[: n * 12].view(n, 3, 4)
    hits = torch.empty(n * 2, dtype=torch.float32, device=dev)
    stats = torch.zeros(3, dtype=torch.int64, device=dev)
    out["logged_rays"] = n
    orders = {"completion": None}
    # the order a wavefront split would trace in: bounce by bounce, paths in pixel order (the
    # megakernel's waves hold neighbouring pixels); and pixel order alone
    key_pix = logged[:, 1, 3].view(torch.int32).to(torch.int64)
    key_bounce = logged[:, 2, 2].view(torch.int32).to(torch.int64)
    orders["bounce_then_pixel"] = torch.argsort(key_bounce * (W * H) + key_pix)
    orders["pixel_then_bounce"] = torch.argsort(key_pix * 16 + key_bounce)
    # coherent orders: origin Morton code (10 bits per axis over the logged origins' bounds) and
    # direction bins (octant, or cube-map face x 8 x 8 cells)
    o = logged[:, 0, :3]
    d = logged[:, 1, :3]
    lo, hi = o.min(0).values, o.max(0).values
    q = ((o - lo) / (hi - lo).clamp_min(1e-9) * 1023).clamp(0, 1023).to(torch.int64)

    def spread(v):  # 10 bits -> every third bit of 30
        v = (v | (v << 16)) & 0x030000FF
        v = (v | (v << 8)) & 0x0300F00F
        v = (v | (v << 4)) & 0x030C30C3
        return (v | (v << 2)) & 0x09249249

    morton = spread(q[:, 0]) | (spread(q[:, 1]) << 1) | (spread(q[:, 2]) << 2)
    octant = ((d[:, 0] < 0).to(torch.int64) | ((d[:, 1] < 0).to(torch.int64) << 1) |
              ((d[:, 2] < 0).to(torch.int64) << 2))
    ad = d.abs()
    face = ad.argmax(1)
    major = ad.gather(1, face[:, None])[:, 0].clamp_min(1e-9)
    sgn = (d.gather(1, face[:, None])[:, 0] < 0).to(torch.int64)
    uv = torch.stack([d.gather(1, ((face + 1) % 3)[:, None])[:, 0], d.gather(1, ((face + 2) % 3)[:, None])[:, 0]],
                     1) / major[:, None]  # in [-1, 1]
    cell = ((uv + 1) * 4).clamp(0, 7.999).to(torch.int64)
    dirbin = ((face * 2 + sgn) * 8 + cell[:, 0]) * 8 + cell[:, 1]  # 384 bins
    orders["octant_then_origin"] = torch.argsort((octant << 30) | morton)
    orders["dirbin_then_origin"] = torch.argsort((dirbin << 30) | morton)
    orders["origin_then_octant"] = torch.argsort((morton << 3) | octant)
    base_log = log

    def trace(order, waves, rays):
        n_rays_log = rays.view(n, 3, 4)
        hits.fill_(-1)
        stats.zero_()
        ms = C.c_float(0)
        assert lib.rt_debug_trace_rays(gpu.handle, C.c_void_p(rays.data_ptr()), n, C.c_void_p(hits.data_ptr()), waves,
                                       C.c_void_p(stats.data_ptr()), None, C.byref(ms)) == 0
        torch.cuda.synchronize()
        h = hits.view(n, 2)
        same = bool(torch.equal(h[:, 0], n_rays_log[:, 2, 0])) and \
            bool(torch.equal(h[:, 1].view(torch.int32), n_rays_log[:, 2, 1].view(torch.int32)))
        st = stats.cpu().tolist()
        ms2 = C.c_float(0)  # a second, uninstrumented launch for the time
        assert lib.rt_debug_trace_rays(gpu.handle, C.c_void_p(rays.data_ptr()), n, C.c_void_p(hits.data_ptr()), waves,
                                       None, None, C.byref(ms2)) == 0
        return {"order": order, "waves": waves, "kernel_ms": round(ms2.value, 3),
                "grays_s": round(n / ms2.value / 1e6, 3), "hits_equal": same,
                "lane_slots_per_ray": {"node_step": round(st[0] / n, 3), "leaf_step": round(st[1] / n, 3),
                                       "all": round(st[2] / n, 3)}}

    out["trace_only"] = []
    pick = os.environ.get("TRACE_ORDERS")  # e.g. "pixel_then_bounce,octant_then_origin" (PMC passes)
    wv = [int(v) for v in os.environ.get("TRACE_WAVES", "6,8").split(",")]
    for oname, perm in orders.items():
        if pick and oname not in pick.split(","):
            continue
        rays = base_log[: n * 12] if perm is None else base_log[: n * 12].view(n, 12)[perm].contiguous().view(-1)
        for waves in wv:
            out["trace_only"].append(trace(oname, waves, rays))
    print(json.dumps(out, indent=1))
    gpu.close()


if __name__ == "__main__":
    main()
