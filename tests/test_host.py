"""Host side of the library, no GPU needed: the C ABI exports, the scene loader and the
reference-BVH build, each checked bit for bit against the oracle's independent restatement.
"""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from oracle.oracle import OracleScene, sample_output as orc_sample_output

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_functions():
    text = open(os.path.join(ROOT, "include", "rtcore.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|void|int32_t|const char\s*\*)\s*(rt_\w+)\s*\(", text, flags=re.M)))


def test_library_exports_every_declared_symbol(rc):
    lib = rc.load_library()
    names = _declared_functions()
    assert len(names) >= 18
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    out = subprocess.run(["nm", "-D", "--defined-only", rc.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (rt_\w+)", out))
    assert set(names) <= exported
    assert lib.rt_abi_version() == rc.ABI_VERSION


def test_library_has_gfx950_code_object(rc):
    blob = open(rc.LIB_PATH, "rb").read()
    assert b"gfx950" in blob, "librtcore_hip.so carries no gfx950 code object"


SYNTH = """size 64 48
recursion 5
ambient color .1 .2 .3
dof .05 3 at 0 0 0
camera 0 -4 1, 0 0 0, 0 0 1, 50
orthographic 0 -4 1 0 0 0 0 0 1 3
pushtransform
translate .5 -.25 .1
rotate 1 2 3 30
scale 1 2 .5
shininess 10 2
emission .5 .4 .3
sphere 0 0 0 .7
cube 0 0 0 1 1 1 not -x +z
poptransform
refraction .8 .8 .8, 1.33
twosided no
vertex 0 0 0
vertex 1 0 0
vertex 0 1 .2
tri 0 1 2
tri 0 2 1 mirrored
refraction off
vertexnormal 0 0 1 0 0 1
vertexnormal 1 0 1 0 1 1
vertexnormal 0 1 1 1 0 1
trinormal 0 1 2
plane 2 0 0 1   # comment
debug off
"""


def _bytes(arr):
    return [bytes(x) for x in arr]


def _scene_text(rc, name):
    if name == "SYNTH":
        return SYNTH
    if name == "MESH":  # config C4's generator at 20 x 10 vertices (342 triangles)
        from raytracercore_amd.scenes import mesh_scene_text

        return mesh_scene_text(nx=20, ny=10)
    return open(rc.scene_path(name)).read()


@pytest.mark.parametrize("name", ["bounce.txt", "die.txt", "SYNTH", "MESH"])
def test_loader_matches_oracle(rc, name):
    text = _scene_text(rc, name)
    ps = rc.SceneLoader.from_text(text)
    orc = OracleScene.from_text(text)
    params, prims, cams = orc.export()
    assert ps.n_prims == orc.n_prims and len(ps.cameras) == orc.n_cameras
    assert bytes(ps.params) == bytes(params)
    assert _bytes(ps.prims) == _bytes(prims)
    assert _bytes(ps.cameras) == _bytes(cams)


@pytest.mark.parametrize("name", ["bounce.txt", "die.txt", "SYNTH", "MESH"])
def test_reference_bvh_matches_oracle(rc, name):
    text = _scene_text(rc, name)
    ps = rc.SceneLoader.from_text(text)
    orc = OracleScene.from_text(text)
    order, boxes, nodes, depth = rc.ref_bvh_export(list(ps.prims))
    assert (nodes, depth) == orc.bvh_info()
    assert np.array_equal(order, orc.bvh_leaf_order())
    b2 = orc.bvh_boxes()
    assert np.array_equal(boxes, b2) or np.array_equal(np.isnan(boxes), np.isnan(b2))


@pytest.mark.parametrize("n,seed", [(5, 1), (20, 2), (21, 3), (64, 4), (300, 5)])
def test_reference_bvh_regimes(rc, n, seed):
    """Brute force (n <= 20) and heap agglomeration (21..200000) agree with the oracle."""
    rng = np.random.default_rng(seed)
    lines = ["size 16 16", "camera 0 0 -10 0 0 0 0 1 0 60"]
    nv = 0
    for i in range(n):
        c = rng.uniform(-5, 5, 3)
        if rng.random() < 0.5:
            lines.append("sphere %.6f %.6f %.6f %.4f" % (c[0], c[1], c[2], rng.uniform(0.05, 0.8)))
        else:
            for _ in range(3):
                v = c + rng.uniform(-0.7, 0.7, 3)
                lines.append("vertex %.6f %.6f %.6f" % tuple(v))
            lines.append("tri %d %d %d" % (nv, nv + 1, nv + 2))
            nv += 3
    # duplicated centres stress the k-d tree's introsort ties
    lines.append("sphere 1 1 1 .2")
    lines.append("sphere 1 1 1 .3")
    text = "\n".join(lines)
    ps = rc.SceneLoader.from_text(text)
    orc = OracleScene.from_text(text)
    assert _bytes(ps.prims) == _bytes(orc.export()[1])
    order, boxes, nodes, depth = rc.ref_bvh_export(list(ps.prims))
    assert (nodes, depth) == orc.bvh_info()
    assert np.array_equal(order, orc.bvh_leaf_order())


@pytest.mark.parametrize("bad", ["size 10", "camera 1 2 3", "cube 0 0 0 1 1 1 some", "instance x",
                                 "tri 0 1 2", "sphere 1,2 3 4", "size 1.5 2", "ambient foo", "  ,x"])
def test_loader_errors(rc, bad):
    with pytest.raises(rc.RtError):
        rc.SceneLoader.from_text(bad + "\n")
    with pytest.raises(ValueError):
        OracleScene.from_text(bad + "\n")


def test_loader_ignores_unknown_and_comments(rc):
    ps = rc.SceneLoader.from_text("# comment\n\n   \noutput x.png\npoint 0 0 0 1 1 1\nmaxverts 3\n")
    assert ps.n_prims == 0 and len(ps.cameras) == 0
    assert ps.params.recursion == 3 and ps.params.air_ior == 1.000293


@pytest.mark.parametrize("args", [((1.0, 0.5, 0.25), 4, 1, (0, 0, 0), 0.0, 1.0), ((3, 3, 3), 2, 0, (0, 0, 0), 0, 1.7),
                                  ((0.2, 0.1, 0.05), 1, 3, (0.5, 0.2, 0.9), 0.8, 1.0), ((0, 0, 0), 0, 3, (1, 1, 1), 1, 2),
                                  ((-1, -1, -1), 1, 0, (0, 0, 0), 0, 1)])
def test_sample_output_matches_oracle(rc, args):
    assert rc.sample_output(*args) == orc_sample_output(*args)


def test_mesh_generator_shape(rc):
    """C4: 1001 x 501 vertices -> 1,000,000 triangles in the bounce room (counted on a small grid)."""
    from raytracercore_amd.scenes import heightfield_text, mesh_scene_text

    t = heightfield_text(nx=31, ny=11)
    assert t.count("\nvertex ") == 31 * 11 and t.count("\ntri ") == 2 * 30 * 10
    ps = rc.SceneLoader.from_text(mesh_scene_text(nx=31, ny=11))
    room = rc.SceneLoader.from_text(mesh_scene_text(nx=2, ny=2))
    assert ps.n_prims - room.n_prims == 2 * 30 * 10 - 2
    zs = np.array([[p.p[k].z for k in range(3)] for p in list(ps.prims)[room.n_prims:]])
    assert zs.min() > -0.47 and zs.max() < -0.13  # -0.3 +- (0.15 + 0.01)


@pytest.fixture(scope="module")
def bvh_check_bin():
    import subprocess

    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "raytracercore_amd", "csrc"), "bvh_check"], check=True)
    return os.path.join(ROOT, "raytracercore_amd", "csrc", "_obj", "bvh_check")


@pytest.mark.parametrize("name", ["bounce.txt", "die.txt", "SYNTH", "MESH200", "SOUP"])
def test_wide_bvh_structure(rc, bvh_check_bin, tmp_path, name):
    """Host checks of the fast path's BVH: every primitive referenced once, every 4-wide node's
    8-bit dequantised child planes contain the primitives below them, stack bound honoured."""
    import subprocess
    from raytracercore_amd.scenes import mesh_scene_text, soup_scene_text

    if name == "MESH200":
        text = mesh_scene_text(nx=201, ny=101)
    elif name == "SOUP":
        text = soup_scene_text(3000, 7)
    else:
        text = _scene_text(rc, name)
    path = tmp_path / "scene.txt"
    path.write_text(text)
    out = subprocess.run([bvh_check_bin, str(path)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.startswith("ok"), out.stdout + out.stderr


@pytest.fixture(scope="module")
def bvh_check_asan_bin():
    import subprocess

    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "raytracercore_amd", "csrc"), "bvh_check_asan"], check=True)
    return os.path.join(ROOT, "raytracercore_amd", "csrc", "_obj_asan", "bvh_check")


@pytest.mark.parametrize("name", ["bounce.txt", "die.txt", "SYNTH", "MESH200", "SOUP"])
def test_host_builders_under_sanitizers(rc, bvh_check_asan_bin, tmp_path, name):
    """The host side of scene creation -- SceneLoader restatement, primitive preparation, the
    reference agglomerative BVH (heap + k-d tree), the binned-SAH BVH2, both wide collapses, the
    camera setup, the host thread pool -- built with AddressSanitizer and UndefinedBehaviorSanitizer
    (`make bvh_check_asan`), on the shipped scenes, the synthetic loader scene, a 40,000-triangle
    mesh and a 3,000-primitive soup: the structural checks pass and the sanitizers report nothing
    (leaks included)."""
    import subprocess
    from raytracercore_amd.scenes import mesh_scene_text, soup_scene_text

    if name == "MESH200":
        text = mesh_scene_text(nx=201, ny=101)
    elif name == "SOUP":
        text = soup_scene_text(3000, 7)
    else:
        text = _scene_text(rc, name)
    path = tmp_path / "scene.txt"
    path.write_text(text)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1")
    out = subprocess.run([bvh_check_asan_bin, str(path), "--ref"], capture_output=True, text=True, env=env,
                         timeout=300)
    assert out.returncode == 0 and out.stdout.startswith("ok") and "\nref " in out.stdout, out.stdout + out.stderr
    assert "Sanitizer" not in out.stderr and "runtime error" not in out.stderr, out.stderr


def test_library_host_entry_points_under_sanitizers(rc, tmp_path):
    """The library's host code -- every source, the HIP files' host side included -- built with
    AddressSanitizer and UndefinedBehaviorSanitizer (`make abi_host_check_asan`) and driven from C++
    through its host-only entry points (tests/host/abi_host_check.cpp: rt_parse_scene's two calls,
    rt_debug_brute_layout, rt_ref_bvh_export, rt_debug_jit_header, the band-set rows and merge,
    rt_sample_output, refused arguments) on the shipped scenes, the synthetic loader scene, an
    empty scene, a 40,000-triangle mesh, 5,000 small cubes and 1,000 rotated cubes (the finders'
    caps): every call succeeds and the sanitizers report nothing, leaks included."""
    import subprocess
    from raytracercore_amd.scenes import mesh_scene_text

    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "raytracercore_amd", "csrc"), "-j8", "abi_host_check_asan"],
                   check=True)
    exe = os.path.join(ROOT, "raytracercore_amd", "csrc", "_obj_asan", "abi_host_check")
    rng = np.random.default_rng(4)
    head = "size 64 48\ncamera 0 -8 0, 0 0 0, 0 0 1, 60\ndiffuse .5 .5 .5\n"
    texts = {
        "synth": SYNTH, "empty": "", "mesh": mesh_scene_text(nx=201, ny=101),
        "cubes": head + "".join(f"cube {x:.3f} {y:.3f} {z:.3f} .05 .05 .05 all\n"
                                for x, y, z in rng.uniform(-3, 3, (5000, 3))),
        "rotated": head + "".join(f"pushtransform\ntranslate {x:.3f} {y:.3f} {z:.3f}\nrotate 0 0 1 {a:.2f}\n"
                                  f"cube 0 0 0 .05 .05 .05 all\npoptransform\n"
                                  for x, y, z, a in np.c_[rng.uniform(-3, 3, (1000, 3)), rng.uniform(1, 89, 1000)]),
    }
    paths = [rc.scene_path("bounce.txt"), rc.scene_path("die.txt")]
    for k, t in texts.items():
        (tmp_path / f"{k}.txt").write_text(t)
        paths.append(str(tmp_path / f"{k}.txt"))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1")
    out = subprocess.run([exe] + paths, capture_output=True, text=True, env=env, timeout=600)
    assert out.returncode == 0 and out.stdout.count("ok ") == len(paths), out.stdout + out.stderr[-3000:]
    assert "Sanitizer" not in out.stderr and "runtime error" not in out.stderr, out.stderr[-3000:]


# --- brute-force layout (host code): rectangles, boxes and frames --------------------------

def _layout(rc, text):
    return rc.brute_layout(list(rc.SceneLoader.from_text(text).prims))


def test_brute_layout_shipped_scenes(rc):
    """bounce.txt: the inverted room and the open light box are world boxes, the rotated cube a
    frame box, the cut-out corner two single rectangles; die.txt: the die is one box."""
    b = rc.brute_layout(list(rc.SceneLoader.from_file(rc.scene_path("bounce.txt")).prims))
    assert (b["rects"], b["boxes"], b["frames"], b["frame_boxes"], b["frame_rects"], b["tris"], b["spheres"]) == \
        (2, 2, 1, 1, 0, 0, 3)
    d = rc.brute_layout(list(rc.SceneLoader.from_file(rc.scene_path("die.txt")).prims))
    assert (d["rects"], d["boxes"], d["frames"], d["tris"], d["spheres"]) == (0, 1, 0, 0, 23)
    assert d["groups"] > 1 and d["grouped_slots"] >= 29


def test_brute_layout_counts_past_16_bits(rc):
    """A flat order of 80,000 triangles: the layout reports the true count (GroupRec packs
    triangles and spheres into 16 + 15 bits, so the brute-force kernels refuse such an order,
    rt_scene_set_traversal; the statistic used to show the truncated 14,464)."""
    from raytracercore_amd.scenes import mesh_scene_text

    got = _layout(rc, mesh_scene_text(nx=201, ny=201))
    assert (got["tris"], got["boxes"], got["rects"], got["spheres"]) == (80000, 2, 0, 0)


HEAD = "size 16 12\ncamera 0 -6 1, 0 0 0, 0 0 1, 60\n"


@pytest.mark.parametrize("text,expect", [
    ("cube 0 0 0 1 1 1 all\n", dict(boxes=1, rects=0)),                     # closed box
    ("cube 0 0 0 1 2 3 not -z\n", dict(boxes=1, rects=0)),                  # open box (5 faces)
    ("cube 0 0 0 1 1 1 only +x -x +y -y\n", dict(boxes=0, rects=4)),       # 4 faces: rectangles
    ("cube 0 0 0 1 1 1 only +x -y\n", dict(boxes=0, rects=2)),
    ("cube 0 0 0 1 1 1 all\ncube 3 0 0 1 1 1 all\n", dict(boxes=2, rects=0)),
    ("pushtransform\nrotate 1 2 3 30\ncube 0 0 0 1 2 3 all\npoptransform\n",
     dict(boxes=0, rects=0, frames=1, frame_boxes=1, frame_rects=0)),      # box in a rotated frame
    ("pushtransform\nrotate 0 0 1 30\ncube 0 0 0 1 1 1 only +x -x +y\npoptransform\n",
     dict(frames=1, frame_boxes=0, frame_rects=3)),                        # frame, too few faces for a box
    ("pushtransform\nrotate 0 0 1 30\ncube 0 0 0 1 1 1 only +x\npoptransform\n",
     dict(frames=0, tris=1)),                                              # a lone parallelogram stays a triangle
    ("plane 3 0 1 0\ncube 0 0 0 1 1 1 not -z\n", dict(boxes=1, planes=1)),
])
def test_brute_layout_detection(rc, text, expect):
    got = _layout(rc, HEAD + text)
    assert {k: got[k] for k in expect} == expect


@pytest.mark.parametrize("grouped", [False, True])
def test_scene_specialised_build_compiles(rc, grouped):
    """The kernel sources embedded in the library compile with hiprtc for gfx950 (host only: the
    run-time build of rt_set_jit, here for an empty scene)."""
    assert rc.jit_compile_check("gfx950", grouped) > 1000


@pytest.mark.parametrize("name,grouped", [("bounce.txt", False), ("die.txt", True)])
def test_scene_specialised_header_of_shipped_scenes(rc, name, grouped, tmp_path):
    """rt_debug_jit_header (host only): the generated header of the shipped scenes' specialised
    builds.  The flat order's carries only the camera's kind and depth-of-field switch (one build
    serves every camera of those), the grouped order's the camera itself; both compile for gfx950
    with the embedded sources (tools/jit_isa.py, the run-time build's options)."""
    import subprocess
    import sys

    scene = rc.SceneLoader.from_file(rc.scene_path(name))
    h = rc.jit_header(scene, 0, size=(1920, 1080), grouped=grouped)
    assert "kSceneW" in h and "kRectsW" in h
    if grouped:
        assert "#define RT_SCENE_CONST_CAMERA 1" in h and "kCameraW" in h
    else:
        assert "#define RT_SCENE_CONST_CAMERA 0" in h and "kCameraW" not in h
        assert "#define RT_SCENE_CAMERA_KIND 0" in h and "#define RT_SCENE_CAMERA_DOF 0" in h
        # another camera of the same kind: the same header, so no new build
        assert rc.jit_header(scene, 1, size=(1920, 1080)) == h
    hdr = tmp_path / "hdr.h"
    hdr.write_text(h)
    tool = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "jit_isa.py")
    out = subprocess.run([sys.executable, tool, str(hdr), "1" if grouped else "0", str(tmp_path / "k")],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "rt_path_const" in (tmp_path / "k.s").read_text()


def _group_records(h):
    import re
    import struct

    w = [int(x, 16) for x in re.search(r"kGroupsW\[\d+\][^{]*\{([^}]*)\}", h).group(1).split(",")]
    recs = []
    for k in range(0, len(w), 16):
        r = w[k:k + 16]
        f = [struct.unpack("f", struct.pack("I", v))[0] for v in r[:8]]
        recs.append({"lo": f[0:3], "hi": f[4:7], "n_rect": sum(r[8:11]), "n_tri": r[11] & 0xFFFF,
                     "n_sph": r[11] >> 16, "n_frames": r[13] & 0xFFFF, "n_boxes": r[13] >> 16,
                     "extra": r[14], "skip": r[15]})
    return recs


@pytest.mark.parametrize("name", ["die.txt", "bounce.txt"])
def test_grouped_order_records(rc, name):
    """The grouped order's records, as the scene-specialised header carries them for each camera:
    super records (a box, no primitives, skip > 0) hold the records right behind them, are not
    nested, and their box contains every record they hold; the groups together test every
    non-plane primitive once (the flat order's count).  Only under RTCORE_GROUP_BOXES=1 (the
    box-aware cut, off by default: DESIGN §6.1) are the scene's closed boxes whole groups' boxes,
    so that die.txt's cube is one box test; that check runs only then."""
    scene = rc.SceneLoader.from_file(rc.scene_path(name))
    flat = _group_records(rc.jit_header(scene, 0, size=(1920, 1080), grouped=False))
    assert len(flat) == 1 and flat[0]["skip"] == 0
    total = lambda g: g["n_rect"] + g["n_tri"] + g["n_sph"] + g["extra"]
    for cam in range(3 if name == "die.txt" else 1):
        recs = _group_records(rc.jit_header(scene, cam, size=(1920, 1080), grouped=True))
        i = 0
        while i < len(recs):
            g = recs[i]
            if g["skip"] > 0:
                assert total(g) == 0 and g["n_frames"] == 0 and g["n_boxes"] == 0
                held = recs[i + 1:i + 1 + g["skip"]]
                assert len(held) == g["skip"] >= 2
                for c in held:
                    assert c["skip"] == 0  # one level
                    assert all(g["lo"][k] <= c["lo"][k] and c["hi"][k] <= g["hi"][k] for k in range(3))
            i += 1
        assert sum(total(g) for g in recs if g["skip"] == 0) == total(flat[0])
        if name == "die.txt" and os.environ.get("RTCORE_GROUP_BOXES", "0") != "0":
            assert sum(g["n_boxes"] for g in recs) == 1 and sum(g["n_rect"] for g in recs) == 0
        if name == "die.txt" and os.environ.get("RTCORE_GROUP_SUPER", "3") != "0":
            assert sum(g["skip"] > 0 for g in recs) == 1


def test_experiment_patches_apply():
    """Cost experiments live in tools/exp_patch.py, not in the product kernel: every patch's anchors
    occur exactly once in kernels_path.hip, and the kernel holds no experiment switches."""
    import importlib.util

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("exp_patch", os.path.join(root, "tools", "exp_patch.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    src = open(os.path.join(root, "raytracercore_amd", "csrc", "kernels_path.hip")).read()
    assert "RT_EXP_" not in src and "exp_sink" not in src
    for name in mod.PATCHES:
        assert mod.apply(src, [name]) != src, name


def test_vertexnormal_rehit_test_matches_oracle(rc):
    """The kernels' fp64 re-hit test of a vertex-normal triangle (rt_debug_vn_rehit, the host build of
    vn_rehit_test) against the oracle's own Triangle.RayTraceAVXFaster restatement on
    the same ray: from the hit point fma(e01, u, fma(e02, v, v0)), along random directions, the same
    hit / no-hit outcome -- a rounding residual of t decides it -- and the same t, bit for bit."""
    import ctypes as C

    from oracle.oracle import OracleScene

    rng = np.random.default_rng(7)
    lib = rc.load_library()
    D3 = C.c_double * 3
    hits = misses = 0
    for tri in range(12):
        v = rng.uniform(-2, 2, (3, 3))
        n = rng.normal(size=(3, 3))
        text = "size 8 8\ncamera 0 -5 0, 0 0 0, 0 0 1, 60\n" + "".join(
            f"vertexnormal {v[k, 0]:.17g} {v[k, 1]:.17g} {v[k, 2]:.17g} {n[k, 0]:.17g} {n[k, 1]:.17g} {n[k, 2]:.17g}\n"
            for k in range(3)) + "trinormal 0 1 2\n"
        orc = OracleScene.from_text(text)
        v0, e01, e02 = D3(*v[0]), D3(*(v[1] - v[0])), D3(*(v[2] - v[0]))
        for _ in range(150):
            a, b = rng.uniform(0.01, 0.99, 2)
            if a + b > 0.99:
                a, b = 1 - a, 1 - b
            d = rng.normal(size=3).astype(np.float32)
            d /= np.float32(np.linalg.norm(d))
            inside, t, o = C.c_int32(), C.c_double(), D3()
            got = lib.rt_debug_vn_rehit(v0, e01, e02, 0, float(a), float(b), d.ctypes.data_as(C.POINTER(C.c_float)),
                                        C.byref(inside), C.byref(t), o)
            pid, dist = orc.raytrace((o[0], o[1], o[2], 1.0), (float(d[0]), float(d[1]), float(d[2]), 0.0))
            assert got == (1 if pid == 0 else 0), (tri, a, b, d, t.value, pid, dist)
            if got:
                assert dist == t.value
                hits += 1
            else:
                misses += 1
    # both outcomes occur: the residual's sign is data-dependent
    print(f"re-hit test: {hits} hits, {misses} misses, all equal to the oracle")
    assert hits > 100 and misses > 100, (hits, misses)


def test_host_pool_survives_fork(rc):
    """a fork()ed child inherits the persistent host pool's pointer but not its
    worker threads.  The child's first pool-backed call must build a pool of its own instead of
    waiting forever for workers that do not exist.  The parent runs one host-only pass large enough
    for the pool (scene preparation of a 20,000-triangle mesh goes through parallel_for) so the pool
    exists; a forked child then runs the same pass, which must finish and agree with the parent's."""
    import multiprocessing as mp

    from raytracercore_amd import scenes

    prims = rc.SceneLoader.from_text(scenes.mesh_scene_text(101, 101)).prims
    assert len(prims) > 20000
    ref = rc.brute_layout(prims)
    ctx = mp.get_context("fork")
    q = ctx.Queue()

    def child():
        q.put(rc.brute_layout(prims) == ref)

    p = ctx.Process(target=child)
    p.start()
    p.join(120)
    alive = p.is_alive()
    if alive:
        p.kill()
    assert not alive, "forked child hung in the host pool"
    assert p.exitcode == 0 and q.get(timeout=5)


def test_library_built_from_these_sources():
    """The library carries the hash of the sources it was built from (rt_build_info, Makefile +
    csrc/source_hash.py): it equals the hash of the tree's sources, with no extra compiler flags,
    so the library every test loads is the committed source's build, not a stale or variant one."""
    import raytracercore_amd as rc
    from raytracercore_amd.csrc.source_hash import build_info

    assert rc.load_library().rt_build_info().decode() == build_info("")


def test_brute_layout_linear_on_large_rectangle_scenes():
    """The flat brute-force order is built for every scene; its box and frame finders pair
    rectangles by search, so a group with more than 4,096 candidates keeps its rectangles as they
    are (rtcore_api.hip kFindMax): 30,000 axis-aligned single faces and 6,000 rotated cube faces lay
    out in well under a second instead of minutes, while a small scene still finds its boxes."""
    import time

    import raytracercore_amd as rc

    rng = np.random.default_rng(3)
    head = "size 64 48\ncamera 0 -8 0, 0 0 0, 0 0 1, 60\ndiffuse .5 .5 .5\n"
    faces = "".join(f"cube {x:.4f} {y:.4f} {z:.4f} .05 .05 .05 only +x\n" for x, y, z in rng.uniform(-3, 3, (30000, 3)))
    sc = rc.SceneLoader.from_text(head + faces)
    t = time.perf_counter()
    lay = rc.brute_layout(sc.prims)
    assert time.perf_counter() - t < 3.0 and lay["rects"] == 30000 and lay["boxes"] == 0
    rot = "".join(f"pushtransform\ntranslate {x:.3f} {y:.3f} {z:.3f}\nrotate 0 0 1 {a:.2f}\ncube 0 0 0 .05 .05 .05 all\n"
                  "poptransform\n" for x, y, z, a in np.c_[rng.uniform(-3, 3, (1000, 3)), rng.uniform(1, 89, 1000)])
    sc = rc.SceneLoader.from_text(head + rot)
    t = time.perf_counter()
    lay = rc.brute_layout(sc.prims)
    assert time.perf_counter() - t < 3.0 and lay["frames"] == 0 and lay["tris"] == 6000
    small = rc.SceneLoader.from_text(head + "cube 0 0 0 1 1 1 all\ncube 2 0 0 1 1 1 all\n")
    assert rc.brute_layout(small.prims)["boxes"] == 2


def test_scene_create_refuses_frames_past_16_bit_coordinates(rc):
    """The BVH kernels hold a pixel's x and y in 16 bits each (kernels_path.hip lane_fx / lane_fy):
    rt_scene_create refuses a width or height above 65535 with RT_ERR_ARG and a message, before it
    touches a device (so this runs without one)."""
    lib = rc.load_library()
    sc = rc.SceneLoader.from_text(SYNTH)
    for w, h in ((65536, 16), (16, 70000)):
        params = rc.rt_scene_params.from_buffer_copy(sc.params)
        params.width, params.height = w, h
        handle = C.c_void_p()
        assert lib.rt_scene_create(C.byref(params), sc.prims, sc.n_prims, 0, C.byref(handle)) == -1
        buf = C.create_string_buffer(256)
        lib.rt_last_error(buf, 256)
        assert b"65535" in buf.value and not handle.value
