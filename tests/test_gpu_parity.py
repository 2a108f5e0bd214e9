"""GPU parity: the HIP path (through the C ABI) against the CPU oracle on the same inputs.

* primary-ray hit IDs (DebugRaycaster Primitives mode, exact fp64 kernel): bit-exact at
  1920x1080 for Scenes/bounce.txt and Scenes/die.txt;
* accumulated colour (fp32 path kernel vs fp64 oracle, shared RNG): mean over pixels of the
  squared L2 RGB error of the per-pixel mean < 1e-4 (BASELINE.json tolerance), plus the
  divergence bookkeeping the fp32 restatement allows;
* size-independent properties at the full 1080p x 256 spp workload: every pixel gets exactly
  spp samples, results are bit-reproducible, and the ray count per sample is bounded by
  Recursion + 1.
"""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _oracle(rc, scene, size, cam=0):
    from oracle.oracle import OracleScene

    params = rc.rt_scene_params.from_buffer_copy(scene.params)
    params.width, params.height = size
    orc = OracleScene.from_abi(params, list(scene.prims), list(scene.cameras))
    orc.select_camera(cam)
    return orc


@pytest.mark.parametrize("name", ["bounce.txt", "die.txt"])
def test_primary_ids_bitexact_1080p(rc, scenes, name):
    scene = scenes[name]
    gpu = rc.GpuRaytracer(scene, 0, size=(1920, 1080))
    ids = gpu.primary_ids()
    orc = _oracle(rc, scene, (1920, 1080))
    ref = orc.primary_ids()
    assert ids.shape == (1920, 1080)
    bad = int((ids != ref).sum())
    assert bad == 0, f"{bad} pixels differ"
    assert (ids >= 0).any() and (ids == -1).any()


@pytest.mark.parametrize("cam", [0, 2])
@pytest.mark.parametrize("name", ["bounce.txt", "die.txt"])
def test_bvh_counts_bitexact(rc, scenes, name, cam):
    """DebugRaycaster BoundingVolumes mode: reference-BVH node counts, exact."""
    scene = scenes[name]
    gpu = rc.GpuRaytracer(scene, cam, size=(640, 360))
    got = gpu.bvh_counts()
    ref = _oracle(rc, scene, (640, 360), cam).bvh_counts()
    assert np.array_equal(got, ref)
    assert got.max() > 3 and (got == 0).any() == (ref == 0).any()


def test_mesh_primary_ids_bitexact(rc):
    """1M-triangle mesh (config C4): grazing rays pierce more leaves than the exact kernel's list
    holds, so this also covers its selection fallback; IDs must still be exact."""
    from raytracercore_amd.scenes import mesh_scene_text

    scene = rc.SceneLoader.from_text(mesh_scene_text())
    size = (120, 68)
    gpu = rc.GpuRaytracer(scene, 0, size=size)
    ids = gpu.primary_ids()
    ref = _oracle(rc, scene, size).primary_ids()
    assert int((ids != ref).sum()) == 0
    assert (ids >= 11).mean() > 0.02  # the height field (IDs after the room and light box) is in view
    counts = gpu.bvh_counts(40, 20, 24, 16)
    assert np.array_equal(counts, _oracle(rc, scene, size).bvh_counts(40, 20, 24, 16))
    # the room's and light box's 11 rectangles are outer records; the tree holds the 1M triangles
    bs = gpu.build_stats()
    assert bs["outer_prims"] == 11 and bs["flat_tris"] == 1000000 and bs["flat_boxes"] == 2
    gpu.check_bvh()
    # 1M triangles do not fit the brute-force group's 16-bit count: refused, the BVH mode kept
    with pytest.raises(rc.RtError):
        gpu.set_traversal(rc.RT_TRAVERSAL_BRUTE)
    assert gpu.info().traversal == rc.RT_TRAVERSAL_BVH
    gpu.close()


@pytest.mark.parametrize("name", ["bounce.txt", "die.txt"])
def test_primary_ids_tile_offsets(rc, scenes, name):
    """A sub-tile equals the same window of the full frame (tile origin handling)."""
    scene = scenes[name]
    gpu = rc.GpuRaytracer(scene, 0, size=(320, 240))
    full = gpu.primary_ids()
    tile = gpu.primary_ids(37, 51, 101, 77)
    assert np.array_equal(tile, full[37:138, 51:128])


@pytest.mark.parametrize("name,cam", [("bounce.txt", 0), ("bounce.txt", 2), ("die.txt", 0), ("die.txt", 2)])
def test_accumulation_parity(rc, scenes, name, cam):
    """fp32 kernel vs fp64 oracle under the shared RNG on a 48x48 window, 32 spp."""
    scene = scenes[name]
    size = (192, 144)
    gpu = rc.GpuRaytracer(scene, cam, size=size)
    orc = _oracle(rc, scene, size, cam)
    x0, y0, w, h, spp = 72, 48, 48, 48, 32
    s, n, m, rays = gpu.render_tile(x0, y0, w, h, spp, seed=11)
    so, no, mo, rays_o = orc.render_tile(x0, y0, w, h, spp, seed=11)
    assert np.all(n + m == spp) and np.all(no + mo == spp)
    # primary misses come from fp32 vs fp64 jittered camera rays: equal except at silhouettes
    assert np.abs(m.astype(int) - mo.astype(int)).sum() <= 0.002 * w * h * spp
    mean_g = s / np.maximum(n, 1)[..., None]
    mean_o = so / np.maximum(no, 1)[..., None]
    both = (n > 0) & (no > 0)
    err = np.sum((mean_g - mean_o) ** 2, axis=-1)[both]
    assert float(err.mean()) < 1e-4, f"mean squared L2 error {err.mean():.3g} (max {err.max():.3g})"
    assert abs(rays - rays_o) <= 0.01 * rays_o


def test_sample_level_agreement(rc, scenes):
    """Most individual samples take the same path: compare single-sample colours (1 spp pass)."""
    scene = scenes["bounce.txt"]
    size = (128, 128)
    gpu = rc.GpuRaytracer(scene, 0, size=size)
    orc = _oracle(rc, scene, size)
    g = gpu.render_tile_1spp(32, 32, 64, 64, seed=5, sample_index=3)
    o = np.zeros_like(g)
    for x in range(64):
        for y in range(64):
            col, miss, _ = orc.sample(32 + x, 32 + y, seed=5, sample=3)
            o[x, y] = (-1.0, -1.0, -1.0) if miss else col
    close = np.all(np.abs(g - o) <= 1e-3 * np.maximum(1.0, np.abs(o)), axis=-1)
    assert close.mean() > 0.97, f"only {close.mean():.3f} of samples agree"
    # misses are reported as DoubleColor.Placeholder exactly
    assert set(np.unique(g[np.all(g < 0, axis=-1)])) <= {-1.0}


@pytest.mark.parametrize("tile", [(0, 0, 1920, 1080, 1), (0, 0, 1920, 1080, 4), (0, 0, 1920, 1080, 32),
                                  (3, 5, 1001, 777, 96)])
def test_host_tile_equals_device_render_1080p(rc, scenes, tile):
    """rt_render_tile (host arrays, SampleSet [x, y] order, added to) equals the device-resident
    render of the same samples in one launch, transposed, bit for bit; a second call adds.  1080p at
    1 spp is one launch, at 4 spp 2 column bands; 1080p at 32 spp and a ragged 1001 x 777 tile at
    96 spp render in 4 (band edges on multiples of 8 columns), each band's copy overlapping the next
    band's launch (calls of 2.5e8 samples and more are one launch again)."""
    import torch

    x0, y0, W, H, spp = tile
    gpu = rc.GpuRaytracer(scenes["die.txt"], 0, size=(1920, 1080))
    dev = torch.device("cuda", 0)
    d_sum = torch.zeros(3 * W * H, dtype=torch.float64, device=dev)
    d_n = torch.zeros(W * H, dtype=torch.int32, device=dev)
    d_m = torch.zeros(W * H, dtype=torch.int32, device=dev)
    d_r = torch.zeros(1, dtype=torch.int64, device=dev)
    gpu.render_device(x0, y0, W, H, spp, 5, 7, d_sum.data_ptr(), d_n.data_ptr(), d_m.data_ptr(), d_r.data_ptr(), 0)
    torch.cuda.synchronize(dev)
    s, n, m, rays = gpu.render_tile(x0, y0, W, H, spp, seed=5, sample_base=7)
    ds = d_sum.cpu().numpy().reshape(3, H, W).transpose(2, 1, 0)  # -> [x, y, rgb]
    assert np.array_equal(s, ds)
    assert np.array_equal(n, d_n.cpu().numpy().reshape(H, W).T.astype(np.uint32))
    assert np.array_equal(m, d_m.cpu().numpy().reshape(H, W).T.astype(np.uint32))
    assert rays == int(d_r.item())
    lib, C_ = gpu.lib, __import__("ctypes")
    r2 = C_.c_uint64(0)
    assert lib.rt_render_tile(gpu.handle, x0, y0, W, H, spp, 5, 7, s.ctypes.data_as(C_.POINTER(rc.rt_color)),
                              n.ctypes.data_as(C_.POINTER(C_.c_uint32)), m.ctypes.data_as(C_.POINTER(C_.c_uint32)),
                              C_.byref(r2)) == 0
    assert np.array_equal(s, 2 * ds) and np.all(n + m == 2 * spp) and r2.value == rays
    gpu.close()


@pytest.mark.parametrize("tile", [(0, 0, 1920, 1080), (3, 5, 1001, 777), (3, 5, 1601, 777)])
def test_one_pass_equals_device_render(rc, scenes, tile):
    """rt_render_tile_1spp (Raytracer.Render's one pass, copied in chunks as fp32 and widened on the
    host) equals the device-resident 1-spp render of the same sample: the colour where the sample
    hit, Placeholder (-1) where it missed, bit for bit; a whole 1080p frame and ragged tiles whose
    pixel counts split unevenly over the copy chunks."""
    import torch

    x0, y0, w, h = tile
    gpu = rc.GpuRaytracer(scenes["bounce.txt"], 0, size=(1920, 1080))
    dev = torch.device("cuda", 0)
    d_sum = torch.zeros(3 * w * h, dtype=torch.float64, device=dev)
    d_n = torch.zeros(w * h, dtype=torch.int32, device=dev)
    d_m = torch.zeros(w * h, dtype=torch.int32, device=dev)
    d_r = torch.zeros(1, dtype=torch.int64, device=dev)
    gpu.render_device(x0, y0, w, h, 1, 9, 41, d_sum.data_ptr(), d_n.data_ptr(), d_m.data_ptr(), d_r.data_ptr(), 0)
    torch.cuda.synchronize(dev)
    ds = d_sum.cpu().numpy().reshape(3, h, w).transpose(2, 1, 0)  # -> [x, y, rgb]
    miss = (d_m.cpu().numpy().reshape(h, w).T == 1)
    want = np.where(miss[..., None], -1.0, ds)
    buf = np.full((w, h, 3), 7.0)
    for _ in range(2):  # into a reused array, twice (no accumulation: the pass overwrites)
        got = gpu.render_tile_1spp(x0, y0, w, h, seed=9, sample_index=41, out=buf)
        assert got is buf and np.array_equal(got, want)
    assert np.array_equal(gpu.render_tile_1spp(x0, y0, w, h, seed=9, sample_index=41), want)
    gpu.close()


def test_full_1080p_properties(rc, scenes):
    """Full configs[1] workload: bookkeeping, reproducibility, rays per sample."""
    import torch

    scene = scenes["bounce.txt"]
    W, H, spp = 1920, 1080, 256
    gpu = rc.GpuRaytracer(scene, 0, size=(W, H))
    dev = torch.device("cuda", 0)
    outs = []
    for _ in range(2):
        d_sum = torch.zeros(3 * W * H, dtype=torch.float64, device=dev)
        d_n = torch.zeros(W * H, dtype=torch.int32, device=dev)
        d_m = torch.zeros(W * H, dtype=torch.int32, device=dev)
        d_r = torch.zeros(1, dtype=torch.int64, device=dev)
        gpu.render_device(0, 0, W, H, spp, 0, 0, d_sum.data_ptr(), d_n.data_ptr(), d_m.data_ptr(), d_r.data_ptr(),
                          torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
        outs.append((d_sum.cpu().numpy(), d_n.cpu().numpy(), d_m.cpu().numpy(), int(d_r.item())))
    (s0, n0, m0, r0), (s1, n1, m1, r1) = outs
    assert np.all(n0 + m0 == spp)
    assert np.array_equal(s0, s1) and np.array_equal(n0, n1) and r0 == r1, "not bit-reproducible"
    samples = W * H * spp
    assert samples <= r0 <= samples * (scene.params.recursion + 1)
    assert np.all(np.isfinite(s0))
    # misses are only where the camera ray leaves the scene: the oracle's primary-ID map at
    # pixel centres agrees with "all samples missed" away from silhouettes
    ids = gpu.primary_ids()
    full_miss = (m0.reshape(H, W).T == spp)
    assert (full_miss == (ids < 0)).mean() > 0.99


@pytest.mark.parametrize("config", ["die1080", "die4k", "mesh1080"])
def test_bench_configs_full_size_properties(rc, scenes, config):
    """The other bench workloads at their full sizes (C3 die 1080p x 1024 spp, C5 die 4K x 512 spp
    per GPU, C4 the 1 M-triangle mesh 1080p x 64 spp), through size-independent properties:
    every pixel gets exactly spp samples, radiance is finite and non-negative, the launch is
    bit-reproducible, and the ray count lies within [samples, samples x (Recursion + 1)]."""
    import torch

    if config == "mesh1080":
        from raytracercore_amd.scenes import mesh_scene_text

        scene, (W, H, spp) = rc.SceneLoader.from_text(mesh_scene_text()), (1920, 1080, 64)
    else:
        scene = scenes["die.txt"]
        W, H, spp = (1920, 1080, 1024) if config == "die1080" else (3840, 2160, 512)
    gpu = rc.GpuRaytracer(scene, 0, size=(W, H))
    dev = torch.device("cuda", 0)
    outs = []
    for _ in range(2):
        d_sum = torch.zeros(3 * W * H, dtype=torch.float64, device=dev)
        d_n = torch.zeros(W * H, dtype=torch.int32, device=dev)
        d_m = torch.zeros(W * H, dtype=torch.int32, device=dev)
        d_r = torch.zeros(1, dtype=torch.int64, device=dev)
        gpu.render_device(0, 0, W, H, spp, 0, 0, d_sum.data_ptr(), d_n.data_ptr(), d_m.data_ptr(), d_r.data_ptr(),
                          torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize(dev)
        ok = bool(torch.all(d_n + d_m == spp).item()) and bool(torch.all(torch.isfinite(d_sum)).item())
        outs.append((ok, bool(torch.all(d_sum >= 0).item()), d_sum, d_n, int(d_r.item())))
    (ok0, nn0, s0, n0, r0), (ok1, _, s1, n1, r1) = outs
    assert ok0 and ok1 and nn0
    assert torch.equal(s0, s1) and torch.equal(n0, n1) and r0 == r1, "not bit-reproducible"
    samples = W * H * spp
    assert samples <= r0 <= samples * (scene.params.recursion + 1)
    gpu.close()


def test_sample_ranges_compose(rc, scenes):
    """Rendering samples [0, a) and [a, a+b) accumulates the same samples as [0, a+b)."""
    scene = scenes["die.txt"]
    gpu = rc.GpuRaytracer(scene, 0, size=(160, 120))
    s1, n1, m1, r1 = gpu.render_tile(0, 0, 160, 120, 24, seed=3, sample_base=0)
    s2, n2, m2, r2 = gpu.render_tile(0, 0, 160, 120, 40, seed=3, sample_base=24)
    s, n, m, r = gpu.render_tile(0, 0, 160, 120, 64, seed=3, sample_base=0)
    assert np.array_equal(n1 + n2, n) and np.array_equal(m1 + m2, m) and r1 + r2 == r
    assert np.allclose(s1 + s2, s, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("mode", ["BVH", "BVH2", "GROUPED"])
@pytest.mark.parametrize("name", ["die.txt", "bounce.txt"])
def test_traversal_modes_agree(rc, scenes, name, mode):
    """Brute force and BVH traversal (wide and binary) return the same closest hits."""
    scene = scenes[name]
    a = rc.GpuRaytracer(scene, 0, size=(128, 96), traversal=rc.RT_TRAVERSAL_BRUTE)
    b = rc.GpuRaytracer(scene, 0, size=(128, 96), traversal=getattr(rc, "RT_TRAVERSAL_" + mode))
    sa, na, ma, ra = a.render_tile(0, 0, 128, 96, 16, seed=9)
    sb, nb, mb, rb = b.render_tile(0, 0, 128, 96, 16, seed=9)
    assert np.array_equal(na, nb) and np.array_equal(ma, mb)
    assert abs(ra - rb) <= 1e-4 * ra
    assert np.allclose(sa, sb, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("mode,nx,builder", [("BVH", 41, "HOST"), ("BVH2", 41, "HOST"), ("GROUPED", 41, "HOST"),
                                             ("BVH", 71, "HOST"), ("BVH2", 71, "HOST"), ("BVH", 71, "GPU"),
                                             ("BVH2", 71, "GPU")])
def test_traversal_modes_agree_mesh(rc, mode, nx, builder):
    """The same on a small procedural height field (3,200 triangles; 5,600 at nx = 71, where the
    BVH kernels test the room and the light box as outer records, with either builder's tree):
    BVH == brute force up to ties on shared triangle edges."""
    from raytracercore_amd.scenes import mesh_scene_text

    scene = rc.SceneLoader.from_text(mesh_scene_text(nx=nx, ny=41))
    a = rc.GpuRaytracer(scene, 0, size=(96, 64), traversal=rc.RT_TRAVERSAL_BRUTE)
    b = rc.GpuRaytracer(scene, 0, size=(96, 64), traversal=getattr(rc, "RT_TRAVERSAL_" + mode),
                        builder=getattr(rc, "RT_BVH_BUILDER_" + builder))
    assert b.info().traversal == getattr(rc, "RT_TRAVERSAL_" + mode)
    assert b.info().bvh_builder == getattr(rc, "RT_BVH_BUILDER_" + builder)
    assert (b.build_stats()["outer_prims"] == 11) == (nx == 71)
    b.check_bvh()
    sa, na, ma, ra = a.render_tile(0, 0, 96, 64, 16, seed=4)
    sb, nb, mb, rb = b.render_tile(0, 0, 96, 64, 16, seed=4)
    assert abs(int(ma.sum()) - int(mb.sum())) <= 2
    assert abs(ra - rb) <= 2e-3 * ra
    same = np.isclose(sa, sb, rtol=1e-4, atol=1e-4).all(axis=-1).mean()
    assert same > 0.99, same


def test_outer_records_leave_small_cubes_in_the_tree(rc):
    """Outer records are only the large axis-aligned rectangles: 300 small cubes
    (1,800 axis-aligned faces) beside a 3,200-triangle height field in the bounce room stay in the
    tree, while the room's walls and the light box's faces (11) leave it; the render still equals
    brute force up to ties."""
    from raytracercore_amd.scenes import mesh_scene_text

    rng = np.random.default_rng(5)
    cubes = ["\ndiffuse .3 .5 .7\nspecular .1 .1 .1\n"]
    for x, y, z in rng.uniform([-1.8, -1.8, -1.6], [1.8, 1.8, -0.5], size=(300, 3)):
        cubes.append(f"cube {x:.4f} {y:.4f} {z:.4f} .06 .06 .06 all\n")
    scene = rc.SceneLoader.from_text(mesh_scene_text(nx=41, ny=41) + "".join(cubes))
    assert scene.n_prims == 5 + 6 + 3200 + 1800  # light box, room, field, cubes
    a = rc.GpuRaytracer(scene, 0, size=(96, 64), traversal=rc.RT_TRAVERSAL_BRUTE)
    for builder in ("HOST", "GPU"):
        b = rc.GpuRaytracer(scene, 0, size=(96, 64), traversal=rc.RT_TRAVERSAL_BVH,
                            builder=getattr(rc, "RT_BVH_BUILDER_" + builder))
        st = b.build_stats()
        assert st["outer_prims"] == 11, st["outer_prims"]
        b.check_bvh()
        sa, na, ma, ra = a.render_tile(0, 0, 96, 64, 16, seed=4)
        sb, nb, mb, rb = b.render_tile(0, 0, 96, 64, 16, seed=4)
        assert abs(int(ma.sum()) - int(mb.sum())) <= 2
        assert abs(ra - rb) <= 2e-3 * ra
        same = np.isclose(sa, sb, rtol=1e-4, atol=1e-4).all(axis=-1).mean()
        assert same > 0.99, same
        b.close()


def _builder_scene(rc, scenes, name):
    from raytracercore_amd.scenes import mesh_scene_text, soup_scene_text

    if name == "MESH200":
        return rc.SceneLoader.from_text(mesh_scene_text(nx=201, ny=101))
    if name == "SOUP":
        return rc.SceneLoader.from_text(soup_scene_text(3000, 7))
    if name == "ONE":  # a single BVH primitive beside a plane: the root is a leaf
        return rc.SceneLoader.from_text("size 16 12\ncamera 0 -4 1, 0 0 0, 0 0 1, 50\nplane 0 0 1 0\nsphere 0 0 0 1\n")
    return scenes[name]


@pytest.mark.parametrize("name", ["MESH200", "SOUP", "bounce.txt", "die.txt", "ONE"])
def test_gpu_bvh_builder_structure(rc, scenes, name):
    """The GPU (PLOC) builder's BVH2 and 4-wide quantised tree pass the same structural check as
    the host builder's: boxes contain every primitive below them, each primitive in one leaf,
    depth and stack within the recorded figures."""
    scene = _builder_scene(rc, scenes, name)
    for b in (rc.RT_BVH_BUILDER_HOST, rc.RT_BVH_BUILDER_GPU):
        g = rc.GpuRaytracer(scene, 0, size=(32, 24), builder=b)
        assert g.info().bvh_builder == b
        g.check_bvh()
        st = g.build_stats()
        if b == rc.RT_BVH_BUILDER_GPU and name != "ONE":
            assert st["ploc_rounds"] >= 1 and st["wide_nodes"] >= 1


@pytest.mark.parametrize("mode", ["BVH", "BVH2"])
@pytest.mark.parametrize("name", ["MESH41", "SOUP"])
def test_gpu_bvh_builder_renders(rc, scenes, name, mode):
    """Renders through the GPU-built trees agree with brute force (ties on shared triangle
    edges aside) and the build is deterministic: two builds render bit-identically."""
    from raytracercore_amd.scenes import mesh_scene_text

    scene = (rc.SceneLoader.from_text(mesh_scene_text(nx=41, ny=41)) if name == "MESH41"
             else _builder_scene(rc, scenes, name))
    size = (96, 64)
    a = rc.GpuRaytracer(scene, 0, size=size, traversal=rc.RT_TRAVERSAL_BRUTE)
    trav = getattr(rc, "RT_TRAVERSAL_" + mode)
    b1 = rc.GpuRaytracer(scene, 0, size=size, traversal=trav, builder=rc.RT_BVH_BUILDER_GPU)
    b2 = rc.GpuRaytracer(scene, 0, size=size, traversal=trav, builder=rc.RT_BVH_BUILDER_GPU)
    assert b1.info().traversal == trav
    sa, na, ma, ra = a.render_tile(0, 0, *size, 16, seed=4)
    s1, n1, m1, r1 = b1.render_tile(0, 0, *size, 16, seed=4)
    s2, n2, m2, r2 = b2.render_tile(0, 0, *size, 16, seed=4)
    assert np.array_equal(s1, s2) and np.array_equal(n1, n2) and np.array_equal(m1, m2) and r1 == r2
    assert abs(int(ma.sum()) - int(m1.sum())) <= 2
    assert abs(ra - r1) <= 2e-3 * ra
    same = np.isclose(sa, s1, rtol=1e-4, atol=1e-4).all(axis=-1).mean()
    assert same > 0.99, same


@pytest.mark.parametrize("builder", ["HOST", "GPU"])
@pytest.mark.parametrize("name", ["MESH200", "SOUP", "bounce.txt"])
def test_compact_leaves_render_identically(rc, scenes, name, builder, monkeypatch):
    """Compact leaves (rt_internal.h kLeafCompact: the primitives' kind and test flags in the leaf
    reference, 48-B records) render bit for bit what generic leaves (64-B records, flags per
    record) render, through both trees and both builders.  The scenes mix triangles, spheres,
    transformed spheres, one-sided, inverted and parallelogram faces, so that leaves of either kind
    occur; rt_scene_check_bvh checks every compact leaf's flags against its primitives."""
    scene = _builder_scene(rc, scenes, name)
    b = getattr(rc, "RT_BVH_BUILDER_" + builder)
    size = (64, 48)
    for trav in (rc.RT_TRAVERSAL_BVH, rc.RT_TRAVERSAL_BVH2):
        monkeypatch.setenv("RTCORE_COMPACT_LEAVES", "0")
        g0 = rc.GpuRaytracer(scene, 0, size=size, traversal=trav, builder=b)
        monkeypatch.delenv("RTCORE_COMPACT_LEAVES")
        g1 = rc.GpuRaytracer(scene, 0, size=size, traversal=trav, builder=b)
        st0, st1 = g0.build_stats(), g1.build_stats()
        assert st0["compact_leaves"] == 0 and st1["wide_leaves"] == st0["wide_leaves"] > 0
        assert st1["compact_leaves"] > 0.5 * st1["wide_leaves"], st1
        g1.check_bvh()
        r0 = g0.render_tile(0, 0, *size, 16, seed=6)
        r1 = g1.render_tile(0, 0, *size, 16, seed=6)
        for x, y in zip(r0, r1):
            assert np.array_equal(x, y)


@pytest.mark.parametrize("name,mode", [("bounce.txt", "BRUTE"), ("die.txt", "GROUPED"), ("MESH200", "BVH")])
def test_xcd_item_ranges_render_identically(rc, scenes, name, mode, monkeypatch):
    """The XCD-local item ranges (8 dispensers, each strip of 8x8 blocks dealt first to one XCD's
    workgroups, then stolen by the others) change which wave renders an item, never what the item
    computes: a 256 x 160 frame (640 blocks, 8 ranges) renders bit for bit as with one dispenser,
    and so does a tile too small to split (16 blocks)."""
    scene = _builder_scene(rc, scenes, name)
    g = rc.GpuRaytracer(scene, 0, size=(256, 160), traversal=getattr(rc, "RT_TRAVERSAL_" + mode))
    for tile in ((0, 0, 256, 160), (40, 24, 32, 32)):
        monkeypatch.setenv("RTCORE_XCD_SPLIT", "0")
        a = g.render_tile(*tile, 8, seed=11)
        monkeypatch.delenv("RTCORE_XCD_SPLIT")
        b = g.render_tile(*tile, 8, seed=11)
        for x, y in zip(a, b):
            assert np.array_equal(x, y)


def test_frame_multi_single_device(rc, scenes):
    """rt_render_frame_multi on one device equals a whole-frame tile render."""
    scene = scenes["die.txt"]
    s, n, m, r = rc.render_frame_multi(scene, 0, 1, 8, seed=4, size=(96, 80))
    gpu = rc.GpuRaytracer(scene, 0, size=(96, 80))
    s2, n2, m2, r2 = gpu.render_tile(0, 0, 96, 80, 8, seed=4)
    assert np.array_equal(n, n2) and np.array_equal(m, m2) and r == r2
    assert np.array_equal(s, s2)


@pytest.mark.parametrize("stride", [2, 3, 8])
@pytest.mark.parametrize("size", [(100, 84), (64, 40), (40, 16)])
def test_band_sets_compose_ragged(rc, scenes, stride, size):
    """Every band set of a frame, rendered on one device through the rt_frame slot layout
    (planes spaced for the tallest set) and scattered into one frame, equals a whole-frame
    render bit for bit -- including splits whose sets differ in height (a short last band,
    a set with fewer bands) and sets with no rows at all."""
    scene = scenes["bounce.txt"]
    W, H = size
    gpu = rc.GpuRaytracer(scene, 0, size=size)
    out = (np.zeros((W, H, 3)), np.zeros((W, H), np.uint32), np.zeros((W, H), np.uint32))
    rays = 0
    for off in range(stride):
        rays += gpu.render_bands(16, stride, off, 6, seed=11, sample_base=5, out=out)[3]
    s2, n2, m2, r2 = gpu.render_tile(0, 0, W, H, 6, seed=11, sample_base=5)
    assert np.array_equal(out[1], n2) and np.array_equal(out[2], m2) and rays == r2
    assert np.array_equal(out[0], s2)
    assert np.all(n2 + m2 == 6)


@pytest.mark.parametrize("world", [1, 3])
def test_band_sets_device_gather_layout(rc, scenes, world):
    """bench.py's band split on the device: each band set rendered by rt_render_bands_device into a
    gather slot and scattered into the frame (raytracercore_amd.sharding) equals a whole-frame
    render bit for bit."""
    import torch

    from raytracercore_amd import sharding

    scene = scenes["bounce.txt"]
    W, H, spp = 100, 84, 6
    gpu = rc.GpuRaytracer(scene, 0, size=(W, H))
    dev = torch.device("cuda", 0)
    plane = sharding.slot_rows(H, world) * W
    d_r = torch.zeros(1, dtype=torch.int64, device=dev)
    slots = []
    for r in range(world):
        slot = torch.zeros(4 * plane, dtype=torch.float64, device=dev)
        s_, n_, m_ = sharding.slot_views(slot, plane)
        gpu.render_bands_device(sharding.BAND, world, r, spp, 11, 5, s_.data_ptr(), n_.data_ptr(), m_.data_ptr(),
                                plane, d_r.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
        slots.append(slot)
    f_sum = torch.zeros(3 * W * H, dtype=torch.float64, device=dev)
    f_n = torch.zeros(W * H, dtype=torch.int32, device=dev)
    f_m = torch.zeros(W * H, dtype=torch.int32, device=dev)
    sharding.scatter_slots(f_sum, f_n, f_m, slots, sharding.row_index(H, world, device=dev), W, plane)
    torch.cuda.synchronize(dev)
    s2, n2, m2, r2 = gpu.render_tile(0, 0, W, H, spp, seed=11, sample_base=5)
    assert np.array_equal(f_n.cpu().numpy().reshape(H, W).T, n2)
    assert np.array_equal(f_m.cpu().numpy().reshape(H, W).T, m2)
    assert np.array_equal(f_sum.cpu().numpy().reshape(3, H, W).transpose(2, 1, 0), s2)
    assert int(d_r.item()) == r2


def test_frame_refuses_more_gpus_than_devices(rc, scenes):
    """rt_frame_create / rt_render_frame_multi with more GPUs than rt_device_count(): RT_ERR_NODEVICE
    with a message, no communicator attempted; the library still renders afterwards."""
    n = rc.device_count()
    for bad in (n + 1, 64):
        with pytest.raises(rc.RtError, match="error -"):
            rc.GpuFrame(scenes["die.txt"], 0, n_gpus=bad, size=(32, 24))
        with pytest.raises(rc.RtError):
            rc.render_frame_multi(scenes["die.txt"], 0, bad, 2, size=(32, 24))
    f = rc.GpuFrame(scenes["die.txt"], 0, n_gpus=1, size=(32, 24))
    s, n_, m, r = f.render(2, seed=1)
    f.close()
    assert (n_ + m == 2).all() and r > 0


def test_frame_progressive_sample_base(rc, scenes):
    """A persistent rt_frame called twice with disjoint sample ranges accumulates the same samples
    as one call over both ranges (FullRaytracer's progressive refinement)."""
    scene = scenes["die.txt"]
    f = rc.GpuFrame(scene, 0, n_gpus=1, size=(72, 56))
    out = f.render(8, seed=2, sample_base=0)
    s, n, m, r = f.render(8, seed=2, sample_base=8, out=out[:3])
    f.close()
    gpu = rc.GpuRaytracer(scene, 0, size=(72, 56))
    s2, n2, m2, r2 = gpu.render_tile(0, 0, 72, 56, 16, seed=2)
    assert np.array_equal(n, n2) and np.array_equal(m, m2) and out[3] + r == r2
    assert np.allclose(s, s2, rtol=1e-5, atol=1e-5)


def test_frame_submit_collect_pipeline(rc, scenes):
    """rt_frame_submit / rt_frame_collect with render k+1 submitted before render k is collected
    (the two-stage pipeline) accumulate bit for bit what sequential rt_frame_render calls do; a
    third submit with two in flight is refused (RT_ERR_STATE) and the pipeline still works."""
    scene = scenes["bounce.txt"]
    W, H = 80, 48
    f = rc.GpuFrame(scene, 0, n_gpus=1, size=(W, H))
    zero = lambda: (np.zeros((W, H, 3)), np.zeros((W, H), np.uint32), np.zeros((W, H), np.uint32))
    seq = zero()
    rays_seq = sum(f.render(4, seed=3, sample_base=4 * k, out=seq)[3] for k in range(5))
    pip = zero()
    rays_pip = 0
    f.submit(4, seed=3, sample_base=0)
    for k in range(5):
        if k + 1 < 5:
            f.submit(4, seed=3, sample_base=4 * (k + 1))
        if k == 2:
            with pytest.raises(rc.RtError, match="in flight"):
                f.submit(4, seed=3, sample_base=999)
        rays_pip += f.collect(pip)[3]
    with pytest.raises(rc.RtError, match="nothing submitted"):
        f.collect(pip)
    f.close()
    assert rays_pip == rays_seq
    for a, b in zip(pip, seq):
        assert np.array_equal(a, b)
    assert np.all(seq[1] + seq[2] == 20)


def test_frame_fault_inside_gather_group_then_renders(rc, scenes):
    """A failure inside rt_frame_render's RCCL gather group (rt_frame_inject_fault) returns an
    error with the group closed: the next render on the same frame gathers again and equals a
    fresh frame's render bit for bit (an open group would swallow its gather)."""
    scene = scenes["die.txt"]
    W, H = 64, 40
    f = rc.GpuFrame(scene, 0, n_gpus=1, size=(W, H))
    f.inject_fault(1)
    with pytest.raises(rc.RtError, match="injected fault"):
        f.render(4, seed=5, sample_base=0)
    s, n, m, r = f.render(4, seed=5, sample_base=0)
    f.close()
    g = rc.GpuFrame(scene, 0, n_gpus=1, size=(W, H))
    s2, n2, m2, r2 = g.render(4, seed=5, sample_base=0)
    g.close()
    assert r == r2 and np.array_equal(n, n2) and np.array_equal(m, m2) and np.array_equal(s, s2)
    assert np.all(n + m == 4)


def test_many_launches_two_streams(rc, scenes):
    """More launches than the launch-parameter ring holds (256), queued without a sync and
    alternating between two streams into one set of device accumulators: every launch gets its
    own parameters and the scene's shared scratch is never used by two launches at once."""
    import torch

    scene = scenes["bounce.txt"]
    W, H, N = 32, 24, 300
    gpu = rc.GpuRaytracer(scene, 0, size=(W, H))
    dev = torch.device("cuda", 0)
    d_sum = torch.zeros(3 * W * H, dtype=torch.float64, device=dev)
    d_n = torch.zeros(W * H, dtype=torch.int32, device=dev)
    d_m = torch.zeros(W * H, dtype=torch.int32, device=dev)
    d_r = torch.zeros(1, dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    for k in range(N):
        gpu.render_device(0, 0, W, H, 1, 6, k, d_sum.data_ptr(), d_n.data_ptr(), d_m.data_ptr(), d_r.data_ptr(),
                          streams[k % 2].cuda_stream)
    torch.cuda.synchronize(dev)
    s2, n2, m2, r2 = gpu.render_tile(0, 0, W, H, N, seed=6)
    n = d_n.cpu().numpy().reshape(H, W).T
    m = d_m.cpu().numpy().reshape(H, W).T
    s = d_sum.cpu().numpy().reshape(3, H, W).transpose(2, 1, 0)
    assert np.array_equal(n, n2) and np.array_equal(m, m2) and int(d_r.item()) == r2
    assert np.allclose(s, s2, rtol=1e-5, atol=1e-5)


def test_kernel_times_ring(rc, scenes):
    """rt_kernel_times: launches queued without a host sync keep their own event pairs (a ring of
    64); the last entry is rt_last_kernel_ms, a longer launch times longer, bad counts fail."""
    import torch

    scene = scenes["bounce.txt"]
    W, H = 256, 192
    gpu = rc.GpuRaytracer(scene, 0, size=(W, H))
    with pytest.raises(rc.RtError):
        gpu.last_kernel_ms()  # nothing launched yet
    dev = torch.device("cuda", 0)
    d_sum = torch.zeros(3 * W * H, dtype=torch.float64, device=dev)
    d_n = torch.zeros(W * H, dtype=torch.int32, device=dev)
    d_m = torch.zeros(W * H, dtype=torch.int32, device=dev)
    d_r = torch.zeros(1, dtype=torch.int64, device=dev)
    spps = [1, 256, 1, 256] * 17  # 68 launches: the ring wraps
    for k, spp in enumerate(spps):
        gpu.render_device(0, 0, W, H, spp, 2, 100 * k, d_sum.data_ptr(), d_n.data_ptr(), d_m.data_ptr(),
                          d_r.data_ptr(), 0)
    t = gpu.kernel_times(64)
    assert len(t) == 64 and all(v > 0 for v in t)
    assert t[-1] == gpu.last_kernel_ms()
    # the ring holds the last 64 launches, oldest first: launches 4..67, spp 1, 256, 1, 256, ...
    assert min(t[1::2]) > 1.5 * max(t[0::2])
    for bad in (0, 65):
        with pytest.raises(rc.RtError):
            gpu.kernel_times(bad)
    g2 = rc.GpuRaytracer(scene, 0, size=(W, H))
    g2.render_tile(0, 0, 8, 8, 1)
    assert len(g2.kernel_times(1)) == 1
    with pytest.raises(rc.RtError):
        g2.kernel_times(2)  # only one launch so far


def test_errors_fail_loudly(rc, scenes):
    scene = scenes["bounce.txt"]
    gpu = rc.GpuRaytracer(scene, 0, size=(64, 64))
    with pytest.raises(rc.RtError):
        gpu.render_tile(60, 60, 8, 8, 1)  # outside the frame
    with pytest.raises(rc.RtError):
        gpu.primary_ids(0, 0, 0, 4)
    with pytest.raises(rc.RtError):
        gpu.render_tile(0, 0, 8, 8, -1)
    s0, n0, m0, r0 = gpu.render_tile(0, 0, 8, 8, 0)  # zero samples: a no-op
    assert not n0.any() and not m0.any() and not s0.any() and r0 == 0
    with pytest.raises(rc.RtError):
        gpu.render_tile(0, 0, 64, 64, 1 << 27)  # more work items than the 32-bit dispenser counts
    s, n, m, rays = gpu.render_tile(0, 0, 8, 8, 2)  # the scene still renders after the refusals
    assert (n + m == 2).all() and rays > 0


def test_tonemap_device_matches_sample_output(rc, scenes):
    """SampleSet.GetOutput on the device (rt_tonemap_device) against the oracle's per-pixel
    restatement on the same accumulators: ARGB codes equal, up to a 1-LSB truncation flip where
    device and host pow differ in the last ulp."""
    import torch
    from oracle.oracle import sample_output

    W, H = 64, 48
    gpu = rc.GpuRaytracer(scenes["die.txt"], 0, size=(W, H))
    dev = torch.device("cuda", 0)
    s = torch.zeros(3 * W * H, dtype=torch.float64, device=dev)
    n = torch.zeros(W * H, dtype=torch.int32, device=dev)
    m = torch.zeros_like(n)
    r = torch.zeros(1, dtype=torch.int64, device=dev)
    gpu.render_device(0, 0, W, H, 8, 3, 0, s.data_ptr(), n.data_ptr(), m.data_ptr(), r.data_ptr(), 0)
    out = torch.zeros(W * H, dtype=torch.int32, device=dev)
    back, alpha, expo = (0.2, 0.3, 0.4), 0.5, 1.7
    rc.tonemap_device(s.data_ptr(), n.data_ptr(), m.data_ptr(), W, H, out.data_ptr(), back, alpha, expo)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    sh, nh, mh = s.cpu().numpy().reshape(3, -1), n.cpu().numpy(), m.cpu().numpy()
    ref = np.array([sample_output(tuple(sh[:, i]), int(nh[i]), int(mh[i]), back, alpha, expo) & 0xFFFFFFFF
                    for i in range(W * H)], dtype=np.uint32)
    assert (mh > 0).any() and (nh > 0).any()
    diff = got != ref
    assert diff.mean() < 1e-3
    for k in range(4):  # any difference is one code step in one channel
        ch = lambda a: (a >> (8 * k)) & 255
        assert np.abs(ch(got).astype(int) - ch(ref).astype(int)).max() <= 1


EDGE_SCENES = {
    # no primitives at all: every primary ray misses
    "empty": "size 16 12\ncamera 0 -4 1, 0 0 0, 0 0 1, 50\n",
    # one plane (outside any BVH), seen from above; ambient returns for escaping bounces
    "plane": "size 16 12\nambient color .2 .3 .4\ncamera 0 -4 3, 0 0 0, 0 0 1, 60\ndiffuse .5 .5 .5\nplane 0 0 0 1\n",
    # one sphere, orthographic camera, emissive
    "sphere": "size 16 12\northographic 0 -4 0 0 0 0 0 0 1 1.5\nemission 1 .5 .25\nsphere 0 0 0 1\n",
}


@pytest.mark.parametrize("name", sorted(EDGE_SCENES))
def test_edge_scenes_match_oracle(rc, name):
    """Degenerate scenes (no primitives, a lone plane, a lone sphere under an ortho camera):
    exact primary IDs and per-sample agreement with the oracle."""
    scene = rc.SceneLoader.from_text(EDGE_SCENES[name])
    gpu = rc.GpuRaytracer(scene, 0)
    orc = _oracle(rc, scene, (16, 12))
    assert np.array_equal(gpu.primary_ids(), orc.primary_ids())
    s, n, m, rays = gpu.render_tile(0, 0, 16, 12, 8, seed=2)
    s2, n2, m2, rays2 = orc.render_tile(0, 0, 16, 12, 8, seed=2)
    assert np.array_equal(n, n2) and np.array_equal(m, m2)
    assert np.allclose(s, s2, rtol=1e-4, atol=1e-5)
    if name == "empty":
        assert (m == 8).all() and rays == 16 * 12 * 8


@pytest.mark.parametrize("w,h,spp", [(1, 1, 1), (9, 7, 3), (13, 1, 200), (3, 17, 1000)])
def test_ragged_tiles_and_spp(rc, scenes, w, h, spp):
    """Tiles that are not multiples of the 8x8 pixel blocks, single pixels, spp that is not a
    multiple of the chunking (and spp above the 64-sample chunk cap): every pixel gets exactly
    spp samples and the result equals the sum of two half renders."""
    gpu = rc.GpuRaytracer(scenes["bounce.txt"], 0, size=(64, 48))
    x0, y0 = 64 - w, 48 - h
    s, n, m, rays = gpu.render_tile(x0, y0, w, h, spp, seed=5)
    assert ((n + m) == spp).all()
    if spp > 1:  # fp32 per-item partials regroup, hence the fp32-level tolerance
        a = gpu.render_tile(x0, y0, w, h, spp // 2, seed=5, sample_base=0)
        b = gpu.render_tile(x0, y0, w, h, spp - spp // 2, seed=5, sample_base=spp // 2)
        assert np.array_equal(a[1] + b[1], n) and np.array_equal(a[2] + b[2], m)
        assert np.allclose(a[0] + b[0], s, rtol=1e-5, atol=1e-6)


# Closed boxes under every culling rule the box test folds into its keep masks: one-sided seen
# from outside (entry faces), inverted one-sided in a rotated frame (exit faces only), two-sided
# in a skewed frame (both), an open emissive box (five faces: a placeholder slot), a plane after
# the box slots (per-order plane offsets), and an inverted room around everything (exit faces).
BOX_SCENE = """size 48 36
camera 0 -6 1.5, 0 0 0, 0 0 1, 70
ambient color .3 .3 .3
diffuse .6 .5 .4
specular .2 .2 .2
shininess 50
twosided false
cube 0 0 0 1 1 1 all
pushtransform
translate 2 0 0
rotate 0 0 1 30
invert true
cube 0 0 0 1 1.2 .8 all
invert false
poptransform
twosided true
pushtransform
translate -2 0 .5
rotate 1 1 0 20
scale 1 .7 1.3
emission 1 .8 .6
cube 0 0 0 1 1 1 all
emission 0 0 0
poptransform
emission .6 .6 .6
twosided true
cube 0 1.5 -.5 1 .5 .5 not -z
emission 0 0 0
diffuse .3 .3 .3
plane 3 0 1 0
invert true
twosided false
cube 0 0 0 12 12 12 all
"""


@pytest.mark.parametrize("mode", ["BVH", "GROUPED"])
def test_closed_boxes_agree(rc, mode):
    """The flat brute-force order tests closed boxes by one slab test (BoxRec); the BVH and
    grouped orders test the same faces one by one.  Same closest hits, same samples."""
    scene = rc.SceneLoader.from_text(BOX_SCENE)
    a = rc.GpuRaytracer(scene, 0, traversal=rc.RT_TRAVERSAL_BRUTE)
    b = rc.GpuRaytracer(scene, 0, traversal=getattr(rc, "RT_TRAVERSAL_" + mode))
    sa, na, ma, ra = a.render_tile(0, 0, 48, 36, 32, seed=4)
    sb, nb, mb, rb = b.render_tile(0, 0, 48, 36, 32, seed=4)
    assert np.array_equal(na, nb) and np.array_equal(ma, mb)
    assert abs(ra - rb) <= 1e-3 * ra
    mean_a = sa / np.maximum(na, 1)[..., None]
    mean_b = sb / np.maximum(nb, 1)[..., None]
    assert float(np.mean(np.sum((mean_a - mean_b) ** 2, axis=-1))) < 1e-5


def test_closed_boxes_match_oracle(rc):
    """Box scene: fp32 kernel (box slab tests) vs the fp64 oracle (faces one by one)."""
    scene = rc.SceneLoader.from_text(BOX_SCENE)
    gpu = rc.GpuRaytracer(scene, 0, traversal=rc.RT_TRAVERSAL_BRUTE)
    orc = _oracle(rc, scene, (48, 36))
    assert np.array_equal(gpu.primary_ids(), orc.primary_ids())
    s, n, m, rays = gpu.render_tile(0, 0, 48, 36, 32, seed=6)
    so, no, mo, rays_o = orc.render_tile(0, 0, 48, 36, 32, seed=6)
    assert np.abs(m.astype(int) - mo.astype(int)).sum() <= 0.002 * 48 * 36 * 32
    mean_g = s / np.maximum(n, 1)[..., None]
    mean_o = so / np.maximum(no, 1)[..., None]
    both = (n > 0) & (no > 0)
    err = np.sum((mean_g - mean_o) ** 2, axis=-1)[both]
    assert float(err.mean()) < 1e-4, f"mean squared L2 error {err.mean():.3g}"
    assert abs(rays - rays_o) <= 0.01 * rays_o


@pytest.mark.parametrize("name,expect", [
    # the cut-out corner's two faces stay rectangles; the inverted room and the open light box are
    # world boxes; the rotated cube is one frame with its box; three spheres (one transformed)
    ("bounce.txt", dict(flat_rects=2, flat_boxes=2, flat_frames=1, flat_frame_boxes=1, flat_frame_rects=0,
                        flat_tris=0, flat_spheres=3)),
    # the die is one world box; 2 light spheres and 21 pips
    ("die.txt", dict(flat_rects=0, flat_boxes=1, flat_frames=0, flat_tris=0, flat_spheres=23)),
    ("BOX", dict(flat_rects=0, flat_boxes=3, flat_frames=2, flat_frame_boxes=2, flat_frame_rects=0, flat_tris=0,
                 flat_spheres=0)),
])
def test_brute_layout(rc, scenes, name, expect):
    """The flat brute-force order's decomposition into rectangles, boxes and frames."""
    scene = rc.SceneLoader.from_text(BOX_SCENE) if name == "BOX" else scenes[name]
    st = rc.GpuRaytracer(scene, 0, size=(32, 24), traversal=rc.RT_TRAVERSAL_BRUTE).build_stats()
    assert {k: int(st[k]) for k in expect} == expect


@pytest.mark.parametrize("name", ["bounce.txt", "die.txt"])
def test_full_frame_1080p_against_oracle(rc, scenes, name):
    """The BASELINE tolerance on the bench workload itself (configs[1]): bounce.txt at 1920x1080,
    camera 0, 256 samples per pixel (and die.txt, with depth of field, at the same size), fp32
    kernel against the fp64 oracle under the shared RNG (the oracle renders with the reference's
    tile scheduler on the host cores, ~25 s and ~7 s on 16 threads).  Mean over pixels of the squared L2 RGB
    error of the per-pixel mean < 1e-4; the largest single-pixel error is reported."""
    import os

    scene = scenes[name]
    W, H, spp = 1920, 1080, 256
    gpu = rc.GpuRaytracer(scene, 0, size=(W, H))
    s, n, m, rays = gpu.render_tile(0, 0, W, H, spp, seed=0)
    orc = _oracle(rc, scene, (W, H))
    so, no, mo, rays_o, secs, used = orc.render_frame(spp, seed=0, threads=min(16, os.cpu_count() or 1))
    assert np.all(n + m == spp) and np.all(no + mo == spp)
    assert np.abs(m.astype(np.int64) - mo.astype(np.int64)).sum() <= 0.002 * W * H * spp
    both = (n > 0) & (no > 0)
    mean_g = s / np.maximum(n, 1)[..., None]
    mean_o = so / np.maximum(no, 1)[..., None]
    err = np.sum((mean_g - mean_o) ** 2, axis=-1)[both]
    print(f"{name} 1080p x {spp} spp: mean squared L2 error {err.mean():.3g}, max {err.max():.3g}, "
          f"rays gpu {rays} oracle {rays_o} ({secs:.1f} s on {used} threads)")
    assert float(err.mean()) < 1e-4
    assert abs(rays - rays_o) <= 0.01 * rays_o


def _random_box_scene(seed: int) -> str:
    """Random cubes (rotated, scaled, one-sided, inverted, open) and spheres in a room."""
    rng = np.random.default_rng(seed)
    lines = ["size 40 30", "camera 0 -7 2, 0 0 0, 0 0 1, 70", "ambient color .2 .25 .3",
             "diffuse .5 .5 .5", "specular .3 .3 .3", "shininess 80"]
    faces = ["+x", "-x", "+y", "-y", "+z", "-z"]
    for k in range(6):
        lines.append(f"twosided {'true' if rng.random() < 0.5 else 'false'}")
        lines.append(f"invert {'true' if rng.random() < 0.3 else 'false'}")
        lines.append(f"emission {rng.random() * 2:.3f} {rng.random() * 2:.3f} {rng.random():.3f}"
                     if rng.random() < 0.3 else "emission 0 0 0")
        c = rng.uniform(-2.5, 2.5, 3)
        s = rng.uniform(0.4, 1.5, 3)
        which = rng.random()
        sel = "all" if which < 0.5 else ("not " + faces[rng.integers(6)]) if which < 0.8 else \
            "only " + " ".join(rng.choice(faces, size=int(rng.integers(1, 5)), replace=False))
        if rng.random() < 0.5:
            ax = rng.normal(size=3)
            lines += ["pushtransform", f"translate {c[0]:.3f} {c[1]:.3f} {c[2]:.3f}",
                      f"rotate {ax[0]:.3f} {ax[1]:.3f} {ax[2]:.3f} {rng.uniform(5, 80):.2f}",
                      f"cube 0 0 0 {s[0]:.3f} {s[1]:.3f} {s[2]:.3f} {sel}", "poptransform"]
        else:
            lines.append(f"cube {c[0]:.3f} {c[1]:.3f} {c[2]:.3f} {s[0]:.3f} {s[1]:.3f} {s[2]:.3f} {sel}")
    lines += ["twosided true", "invert false", "emission 0 0 0"]
    for k in range(3):
        c = rng.uniform(-2.5, 2.5, 3)
        lines.append(f"sphere {c[0]:.3f} {c[1]:.3f} {c[2]:.3f} {rng.uniform(0.2, 0.8):.3f}")
    lines += ["emission 3 3 3", "sphere 0 0 4 .6", "emission 0 0 0", "invert true", "twosided false",
              "cube 0 0 0 10 10 10 all"]
    return "\n".join(lines) + "\n"


@pytest.mark.parametrize("seed", range(8))
def test_random_box_scenes_agree(rc, seed):
    """Fuzz: random cubes under every transform/culling/open-face combination; the flat order's
    box and frame tests against the BVH order's face-by-face tests, and the oracle's IDs."""
    scene = rc.SceneLoader.from_text(_random_box_scene(seed))
    a = rc.GpuRaytracer(scene, 0, traversal=rc.RT_TRAVERSAL_BRUTE)
    b = rc.GpuRaytracer(scene, 0, traversal=rc.RT_TRAVERSAL_BVH)
    sa, na, ma, ra = a.render_tile(0, 0, 40, 30, 16, seed=seed)
    sb, nb, mb, rb = b.render_tile(0, 0, 40, 30, 16, seed=seed)
    assert np.array_equal(na + ma, nb + mb)
    assert abs(ra - rb) <= 2e-3 * ra
    mean_a = sa / np.maximum(na, 1)[..., None]
    mean_b = sb / np.maximum(nb, 1)[..., None]
    both = (na > 0) & (nb > 0)
    assert float(np.mean(np.sum((mean_a - mean_b) ** 2, axis=-1)[both])) < 1e-4
    orc = _oracle(rc, scene, (40, 30))
    assert (a.primary_ids() == orc.primary_ids()).all()


@pytest.mark.parametrize("name,mode", [("bounce.txt", "BRUTE"), ("die.txt", "GROUPED"), ("die.txt", "BRUTE"),
                                       ("BOXES3", "BRUTE"), ("BOXES5", "GROUPED"), ("VN", "BRUTE")])
def test_scene_specialised_kernel_matches_generic(rc, scenes, name, mode):
    """The hiprtc build with the scene's records as constants (rt_set_jit) computes exactly what the
    generic brute-force kernel computes: bit-identical sums, counts and ray totals."""
    if name.startswith("BOXES"):
        scene = rc.SceneLoader.from_text(_random_box_scene(int(name[5:])))
    elif name == "VN":  # vertex-normal triangles: the kernels' fp64 re-hit test (vn_rehit_test)
        from test_gpu_oracle_paths import VN_SCENE

        scene = rc.SceneLoader.from_text(VN_SCENE)
    else:
        scene = scenes[name]
    trav = getattr(rc, "RT_TRAVERSAL_" + mode)
    out = {}
    try:
        for on in (True, False):
            rc.set_jit(on)
            g = rc.GpuRaytracer(scene, 0, size=(96, 64), traversal=trav)
            out[on] = g.render_tile(8, 4, 80, 56, 24, seed=11, sample_base=5)
            st = g.build_stats()
            assert st["jit_status"] == (1.0 if on else 0.0), g.jit_error()
            g.close()
    finally:
        rc.set_jit(True)
    (sa, na, ma, ra), (sb, nb, mb, rb) = out[True], out[False]
    assert ra == rb and np.array_equal(na, nb) and np.array_equal(ma, mb)
    assert np.array_equal(sa, sb)


def test_scene_specialised_kernel_follows_camera_group_order(rc, scenes):
    """Grouped order: the groups are re-sorted per camera, and the specialised build follows."""
    g = rc.GpuRaytracer(scenes["die.txt"], 0, size=(64, 48), traversal=rc.RT_TRAVERSAL_GROUPED)
    a0 = g.render_tile(0, 0, 64, 48, 8, seed=3)
    cam2 = rc.rt_camera.from_buffer_copy(scenes["die.txt"].cameras[2])
    C_ = __import__("ctypes")
    assert g.lib.rt_scene_set_camera(g.handle, C_.byref(cam2)) == 0
    a2 = g.render_tile(0, 0, 64, 48, 8, seed=3)
    assert g.build_stats()["jit_status"] == 1.0
    rc.set_jit(False)
    try:
        b2 = g.render_tile(0, 0, 64, 48, 8, seed=3)
    finally:
        rc.set_jit(True)
    assert a2[3] == b2[3] and np.array_equal(a2[0], b2[0]) and np.array_equal(a2[1], b2[1])
    assert not np.array_equal(a0[0], a2[0])


def test_scene_specialised_many_cameras_evicts_and_matches(rc, scenes):
    """The grouped order's build is per camera (its group order is): after more camera changes than
    the process keeps unreferenced modules (kJitKeep = 16), the least recently used are unloaded and
    the current build still renders exactly what the generic kernel does."""
    C_ = __import__("ctypes")
    g = rc.GpuRaytracer(scenes["die.txt"], 0, size=(32, 24), traversal=rc.RT_TRAVERSAL_GROUPED)
    cam = rc.rt_camera.from_buffer_copy(scenes["die.txt"].cameras[0])
    for k in range(20):
        cam.position.x += 0.01  # a new camera: a new specialised build, the previous one released
        assert g.lib.rt_scene_set_camera(g.handle, C_.byref(cam)) == 0
        a = g.render_tile(0, 0, 32, 24, 2, seed=k)
        assert g.build_stats()["jit_status"] == 1.0
    rc.set_jit(False)
    try:
        b = g.render_tile(0, 0, 32, 24, 2, seed=19)
    finally:
        rc.set_jit(True)
    g.close()
    assert a[3] == b[3] and np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_scene_specialised_flat_build_is_camera_independent(rc, scenes):
    """The flat order's build compiles in the camera's kind and depth-of-field switch only, so a
    camera change (MainWindow.cs:262-269 restarts the render with another scene camera) does no
    hiprtc build: build statistic 16 (compile ms) reads 0 after it, and the render equals the
    generic kernel's and a scene created with that camera from the start, bit for bit."""
    C_ = __import__("ctypes")
    scene = scenes["bounce.txt"]
    size = (64, 48)
    g = rc.GpuRaytracer(scene, 0, size=size, traversal=rc.RT_TRAVERSAL_BRUTE)
    g.render_tile(0, 0, *size, 2, seed=1)
    assert g.build_stats()["jit_status"] == 1.0
    outs = []
    for ci in (1, 2, 3, 0):
        cam = rc.rt_camera.from_buffer_copy(scene.cameras[ci])
        assert g.lib.rt_scene_set_camera(g.handle, C_.byref(cam)) == 0
        st = g.build_stats()
        assert st["jit_status"] == 1.0 and st["jit_compile_ms"] == 0.0 and st["jit_cached"] == 1.0, st
        outs.append((ci, g.render_tile(0, 0, *size, 8, seed=4)))
    for ci, a in outs[:2]:
        f = rc.GpuRaytracer(scene, ci, size=size, traversal=rc.RT_TRAVERSAL_BRUTE)
        b = f.render_tile(0, 0, *size, 8, seed=4)
        f.close()
        assert a[3] == b[3] and np.array_equal(a[1], b[1]) and np.array_equal(a[0], b[0])
    rc.set_jit(False)
    try:
        c = g.render_tile(0, 0, *size, 8, seed=4)
    finally:
        rc.set_jit(True)
    g.close()
    a = outs[-1][1]
    assert a[3] == c[3] and np.array_equal(a[1], c[1]) and np.array_equal(a[0], c[0])


def test_scene_specialised_build_failure_falls_back(rc, scenes, monkeypatch):
    """A failing run-time build (here: a bad compiler flag) leaves the generic kernel in charge:
    the render is unchanged, build statistic 15 reads -1 and rt_scene_get_jit_error says why."""
    monkeypatch.setenv("RTCORE_JIT_FLAGS", "-DRT_JIT_BROKEN_FLAG=( -include rt_no_such_header.h")
    g = rc.GpuRaytracer(scenes["bounce.txt"], 0, size=(48, 32), traversal=rc.RT_TRAVERSAL_BRUTE)
    a = g.render_tile(0, 0, 48, 32, 8, seed=2)
    st = g.build_stats()
    err = g.jit_error()
    g.close()
    assert st["jit_status"] == -1.0 and "hiprtc" in err
    monkeypatch.delenv("RTCORE_JIT_FLAGS")
    rc.set_jit(False)
    try:
        h = rc.GpuRaytracer(scenes["bounce.txt"], 0, size=(48, 32), traversal=rc.RT_TRAVERSAL_BRUTE)
        b = h.render_tile(0, 0, 48, 32, 8, seed=2)
        h.close()
    finally:
        rc.set_jit(True)
    assert a[3] == b[3] and np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


_CACHE_PROBE = r"""
import json, sys
import numpy as np
import raytracercore_amd as rc
g = rc.GpuRaytracer(rc.SceneLoader.from_file(rc.scene_path("bounce.txt")), 0, size=(48, 32),
                    traversal=rc.RT_TRAVERSAL_BRUTE)
s = g.render_tile(0, 0, 48, 32, 4, seed=3)
st = g.build_stats()
print(json.dumps({"status": st["jit_status"], "cached": st["jit_cached"], "rays": int(s[3]),
                  "sum": float(np.asarray(s[0], dtype=np.float64).sum()), "err": g.jit_error()}))
g.close()
"""


def _cache_probe(cache_dir, salt):
    """One scene-specialised render in a fresh child process (so the in-process module cache does
    not hide the disk), with the code-object cache in cache_dir."""
    import json
    import subprocess
    import sys

    env = dict(os.environ, RTCORE_JIT_CACHE=str(cache_dir), RTCORE_JIT_FLAGS=f"-DRT_CACHE_TEST_SALT={salt}")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _CACHE_PROBE], env=env, cwd=root, capture_output=True, text=True,
                       timeout=150)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_scene_specialised_cache_file_damage_recovers(tmp_path):
    """The on-disk code-object cache: a second process loads the first one's build; a damaged cache
    file is dropped and rebuilt, never fatal."""
    os.chmod(tmp_path, 0o700)

    def probe():
        return _cache_probe(tmp_path, 1)

    first = probe()
    assert first["status"] == 1.0 and first["cached"] == 0.0, first
    files = [f for f in os.listdir(tmp_path) if f.endswith(".co")]
    assert len(files) == 1, files
    second = probe()
    assert second["status"] == 1.0 and second["cached"] == 1.0, second
    with open(tmp_path / files[0], "wb") as f:
        f.write(b"not a code object" * 64)
    third = probe()
    assert third["status"] == 1.0 and third["cached"] == 0.0, third
    for r in (second, third):
        assert r["rays"] == first["rays"] and r["sum"] == first["sum"]
    assert os.path.getsize(tmp_path / files[0]) > 4096  # rewritten with the fresh build


def test_scene_specialised_cache_untrusted_dir_is_not_used(tmp_path):
    """A cache directory others can write into is neither read nor written: every process builds
    afresh (a planted code object would otherwise be loaded and run); a new directory is created
    private (0700)."""
    import stat

    shared = tmp_path / "shared"
    shared.mkdir()
    os.chmod(shared, 0o777)
    for _ in range(2):
        r = _cache_probe(shared, 2)
        assert r["status"] == 1.0 and r["cached"] == 0.0, r
    assert not [f for f in os.listdir(shared) if f.endswith(".co")]
    fresh = tmp_path / "new" / "cache"
    r = _cache_probe(fresh, 3)
    assert r["status"] == 1.0 and stat.S_IMODE(os.stat(fresh).st_mode) == 0o700
    assert len([f for f in os.listdir(fresh) if f.endswith(".co")]) == 1
    assert _cache_probe(fresh, 3)["cached"] == 1.0


@pytest.mark.parametrize("nx", [41, 71])
def test_trace_only_kernel_reproduces_logged_hits(rc, nx):
    """rt_debug_ray_log + rt_debug_trace_rays (the wavefront-split measurement): the
    instrumented wide-BVH kernel logs every finished query of a small mesh render, and the
    trace-only kernel re-traces them at 6, 7 and 8 waves per SIMD with bit-identical closest hits.
    nx = 71 (5.7k BVH primitives) has the room's walls as outer records, nx = 41 in the tree."""
    import torch

    from raytracercore_amd.scenes import mesh_scene_text

    W, H, spp = 96, 64, 4
    scene = rc.SceneLoader.from_text(mesh_scene_text(nx=nx, ny=41))
    gpu = rc.GpuRaytracer(scene, 0, size=(W, H), traversal=rc.RT_TRAVERSAL_BVH)
    assert (gpu.build_stats()["outer_prims"] > 0) == (nx == 71)
    dev = torch.device("cuda", 0)
    cap = W * H * spp * 12
    log = torch.zeros(cap * 12, dtype=torch.float32, device=dev)
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    lib = gpu.lib
    assert lib.rt_debug_ray_log(gpu.handle, C.c_void_p(log.data_ptr()), cap, C.c_void_p(cnt.data_ptr())) == 0
    gpu.set_stats(True)
    s, n_, m, rays = gpu.render_tile(0, 0, W, H, spp, seed=3)
    n = int(cnt.item())
    gpu.render_tile(0, 0, W, H, spp, seed=4)  # logging armed one launch only: nothing more is written
    gpu.set_stats(False)
    assert int(cnt.item()) == n
    assert n == rays > W * H * spp
    logged = log[: n * 12].view(n, 3, 4)
    assert int((logged[:, 2, 1].view(torch.int32) >= 0).sum()) > 0.5 * n  # most queries meet the room or the field
    for waves in (6, 7, 8):
        hits = torch.full((n, 2), -7.0, dtype=torch.float32, device=dev)
        ms = C.c_float(0)
        stats = torch.zeros(3, dtype=torch.int64, device=dev)
        assert lib.rt_debug_trace_rays(gpu.handle, C.c_void_p(log.data_ptr()), n, C.c_void_p(hits.data_ptr()), waves,
                                       C.c_void_p(stats.data_ptr()), None, C.byref(ms)) == 0
        torch.cuda.synchronize()
        assert torch.equal(hits[:, 0], logged[:, 2, 0])
        assert torch.equal(hits[:, 1].view(torch.int32), logged[:, 2, 1].view(torch.int32))
        assert ms.value > 0 and int(stats[2].item()) >= int(stats[0].item()) + int(stats[1].item()) > 0
    with pytest.raises(rc.RtError):
        rc._check(lib.rt_debug_trace_rays(gpu.handle, C.c_void_p(log.data_ptr()), n, C.c_void_p(hits.data_ptr()), 5,
                                          None, None, C.byref(ms)))
    gpu.close()


def test_scene_and_frame_lifecycle_returns_device_memory(rc, scenes):
    """A long-running host (the UI re-renders on every scene or camera edit) creates and destroys
    scenes and frames many times: every one of the library's device allocations -- scene records,
    BVHs, launch scratch, per-launch partials, event rings, the frame's slots and its RCCL
    communicator -- must be returned.  hipMemGetInfo after 12 create / render / destroy rounds of a
    brute-force, a grouped and a BVH scene (and 3 of rt_frame) against the same after a warm-up
    round (which loads the scene-specialised builds once per process) with two frames: RCCL keeps
    ~176 MiB from its second communicator on for reuse (tools/leak_probe.py: flat over further
    create / destroy cycles, so a cache, not a leak)."""
    import torch

    from raytracercore_amd.scenes import mesh_scene_text

    mesh = rc.SceneLoader.from_text(mesh_scene_text(nx=41, ny=41))
    work = [(scenes["bounce.txt"], rc.RT_TRAVERSAL_AUTO), (scenes["die.txt"], rc.RT_TRAVERSAL_AUTO),
            (mesh, rc.RT_TRAVERSAL_BVH)]

    def round_trip(frames):
        for sc, trav in work:
            g = rc.GpuRaytracer(sc, 0, size=(96, 64), traversal=trav)
            g.render_tile(0, 0, 96, 64, 4, seed=1)
            g.close()
        for _ in range(frames):
            fr = rc.GpuFrame(scenes["bounce.txt"], 0, n_gpus=1, size=(96, 64))
            fr.render(4, seed=2)
            fr.close()
        torch.cuda.synchronize()

    round_trip(2)
    free0, total = torch.cuda.mem_get_info(0)
    for k in range(12):
        round_trip(1 if k < 3 else 0)
    free1, _ = torch.cuda.mem_get_info(0)
    assert free1 >= free0 - (32 << 20), (free0 - free1) / 2**20  # MiB not returned


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["bounce.txt", "die.txt"])
def test_small_launch_grid_does_not_change_results(rc, scenes, name, monkeypatch):
    """A small brute-force launch runs fewer blocks per CU (run_path: >= 6 samples per lane); which
    lane renders an item never changes what it computes, so the full grid (RTCORE_GRID_BPC=8, read
    per launch) and the capped ones give the same bits."""
    gpu = rc.GpuRaytracer(scenes[name], 0, size=(256, 256))
    out = []
    for bpc in ("8", "3", "1", None):
        if bpc is None:
            monkeypatch.delenv("RTCORE_GRID_BPC", raising=False)
        else:
            monkeypatch.setenv("RTCORE_GRID_BPC", bpc)
        out.append(gpu.render_tile(0, 0, 256, 256, 16, seed=3))
    for r in out[1:]:
        for a, b in zip(out[0][:3], r[:3]):
            assert np.array_equal(a, b)
        assert r[3] == out[0][3]
