"""The CPU oracle against known answers, its committed golden vectors, and loader facts.

The reference ships no tests or fixtures, so the known answers here are
analytic (Fresnel at normal incidence, the TIR critical angle, exact sphere and
parallelogram hits) or follow from the scene files and the loader semantics
(primitive counts and ID order, BVH node counts).
"""
import math
import os

import numpy as np
import pytest

from oracle.oracle import OracleScene, fresnel, sample_output

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _scene(name):
    return OracleScene.from_file(os.path.join(GOLDEN, "scenes", name))


def test_fresnel_normal_incidence():
    # Raytracer.cs:136-153 at cos = 1, air (Scene.cs:35) -> glass 1.52 (bounce.txt:104)
    r0 = ((1.52 - 1.000293) / (1.52 + 1.000293)) ** 2
    assert fresnel(1.0, 1.000293, 1.52) == pytest.approx(r0, rel=1e-14)
    assert r0 == pytest.approx(0.0425221354, rel=1e-9)


def test_total_internal_reflection_angle():
    crit = math.asin(1.000293 / 1.52)
    assert math.degrees(crit) == pytest.approx(41.154, abs=1e-3)
    # inside the glass: beyond the critical angle the ratio is 1 (TIR), just inside it is < 1
    assert fresnel(math.cos(crit + 1e-6), 1.52, 1.000293) == 1.0
    assert fresnel(math.cos(crit - 1e-4), 1.52, 1.000293) < 1.0


SPHERE_SCENE = """size 8 8
camera 0 0 -5 0 0 0 0 1 0 45
sphere 0 0 0 1
"""


def test_sphere_hit_exact():
    s = OracleScene.from_text(SPHERE_SCENE)
    pid, dist = s.raytrace((0, 0, -5, 1), (0, 0, 1, 0))
    assert pid == 0 and dist == 4.0
    pid, dist = s.raytrace((0, 0, 0, 1), (0, 0, 1, 0))  # from the centre: the far root
    assert pid == 0 and dist == 1.0
    pid, _ = s.raytrace((0, 2, -5, 1), (0, 0, 1, 0))
    assert pid == -1


def test_parallelogram_hit():
    # cube face +z of a unit cube at the origin: z = 0.5, u, v in [0, 1]^2 (Triangle.cs:13-20)
    s = OracleScene.from_text("size 8 8\ncamera 0 0 5 0 0 0 0 1 0 45\ncube 0 0 0 1 1 1 only +z\n")
    pid, dist = s.raytrace((0.4, 0.4, 5, 1), (0, 0, -1, 0))
    assert pid == 0 and dist == pytest.approx(4.5, rel=1e-15)
    pid, _ = s.raytrace((0.6, 0.4, 5, 1), (0, 0, -1, 0))  # just outside the square
    assert pid == -1


def test_one_sided_inverted_room():
    # bounce.txt's room faces are `invert true` + `twosided false`: seen from outside they
    # are culled (Primitive.cs:60-64), so camera 0 looks through the near walls
    s = OracleScene.from_text("size 8 8\ncamera 0 0 5 0 0 0 0 1 0 45\ntwosided false\ninvert true\n"
                              "cube 0 0 0 2 2 2 all\n")
    pid, dist = s.raytrace((0, 0, 5, 1), (0, 0, -1, 0))
    assert pid == 5 and dist == pytest.approx(5.0 + 1.0)  # the far (-z) face, seen from inside


@pytest.mark.parametrize("name,prims,nodes,cams", [("bounce.txt", 22, 43, 8), ("die.txt", 29, 57, 3)])
def test_scene_facts(name, prims, nodes, cams):
    s = _scene(name)
    assert s.n_prims == prims and s.n_cameras == cams
    assert s.bvh_info()[0] == nodes  # 2n - 1 nodes
    p, pr, c = s.export()
    kinds = [q.kind for q in pr]
    if name == "bounce.txt":
        assert kinds.count(0) == 19 and kinds.count(1) == 3 and (p.width, p.height, p.recursion) == (700, 700, 10)
        assert pr[20].flags & 16 and pr[20].refractive_index == 1.52  # the lens: transformed sphere
        assert all(pr[i].emission.r == 5 for i in range(5))  # light box faces 0-4
        assert all(pr[i].flags & 4 and not pr[i].flags & 2 for i in range(5, 11))  # room: invert, one-sided
    else:
        assert kinds.count(0) == 6 and kinds.count(1) == 23 and (p.width, p.height, p.recursion) == (1280, 960, 3)
        assert c[0].dof_amount == 1000 and c[0].image_plane == pytest.approx(0.1) and c[0].focal_length == 3
        assert all(q.refractive_index == 0 for q in pr)  # no refraction in die.txt (SURVEY finding 5)


@pytest.mark.parametrize("name", ["bounce", "die"])
def test_golden_primary_ids(name):
    s = _scene(name + ".txt")
    s.set_size(64, 64)
    ref = np.load(os.path.join(GOLDEN, f"primary_ids_{name}_64x64.npy"))
    assert np.array_equal(s.primary_ids(), ref)


@pytest.mark.parametrize("name", ["bounce", "die"])
def test_golden_accumulators(name):
    s = _scene(name + ".txt")
    s.set_size(32, 32)
    ref = np.load(os.path.join(GOLDEN, f"accum_{name}_32x32_16spp_seed0.npz"))
    got = s.render_tile(0, 0, 32, 32, 16, seed=0, sample_base=0)
    assert np.array_equal(got[0], ref["sum"]) and np.array_equal(got[1], ref["samples"])
    assert np.array_equal(got[2], ref["misses"]) and got[3] == int(ref["rays"][0])


def test_sample_output_tonemap():
    # SampleSet.GetOutput: no samples -> background; gamma 1/2.2; misses blend alpha
    assert sample_output((0, 0, 0), 0, 5, (0, 0, 0), 0.0, 1.0) == 0
    c = sample_output((2.0, 2.0, 2.0), 4, 0) & 0xFFFFFFFF
    v = int(0.5 ** (1 / 2.2) * 255)
    assert c == (255 << 24) | (v << 16) | (v << 8) | v
    c = sample_output((4.0, 0, 0), 4, 4) & 0xFFFFFFFF
    assert (c >> 24) == int(0.5 * 255) and ((c >> 16) & 255) == 255


def test_threaded_frame_matches_sequential():
    """FullRaytracer-style tiling (1 spp per pass) gives the same per-pixel samples."""
    s = _scene("die.txt")
    s.set_size(40, 30)
    a = s.render_frame(3, seed=2, threads=4)
    b = s.render_tile(0, 0, 40, 30, 3, seed=2)
    assert np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2]) and a[3] == b[3]
    assert np.allclose(a[0], b[0], rtol=1e-12, atol=0)


def test_c1_plumbing_config():
    """BASELINE configs[0] (C1): bounce.txt 256x256 x 16 spp, camera 0, on the oracle's FullRaytracer
    restatement (T threads, TilesY = floor(sqrt(T)), TilesX = T / TilesY, 1 spp per tile pass,
    FullRaytracer.cs:66-72, 219-229): every pixel gets 16 samples, the result does not depend on
    the thread count (1 vs all host cores) up to the order of the fp64 additions (passes of one tile
    merge as they finish, FullRaytracer.cs:326-344, so two passes of a tile may land in either order),
    a pixel mean is the same whatever the tiling, and the ray count per sample lies in
    [1, Recursion + 1]."""
    import os

    s = _scene("bounce.txt")
    s.set_size(256, 256)
    s.select_camera(0)
    a = s.render_frame(16, seed=0, threads=os.cpu_count() or 1)
    b = s.render_frame(16, seed=0, threads=1)
    assert np.all(a[1] + a[2] == 16)
    assert np.array_equal(a[1], b[1]) and np.array_equal(a[2], b[2]) and a[3] == b[3]
    np.testing.assert_allclose(a[0], b[0], rtol=1e-12, atol=1e-12)
    assert 256 * 256 * 16 <= a[3] <= 256 * 256 * 16 * 11
    t = s.render_tile(100, 120, 16, 16, 16, seed=0)
    np.testing.assert_allclose(t[0], a[0][100:116, 120:136], rtol=1e-12, atol=1e-12)


def _h32(x):
    x &= 0xFFFFFFFF
    x ^= x >> 16
    x = (x * 0x7FEB352D) & 0xFFFFFFFF
    x ^= x >> 15
    x = (x * 0x846CA68B) & 0xFFFFFFFF
    x ^= x >> 16
    return x


def _spec_draws(seed, pixel, sample, n):
    """include/rtcore_rng.h's stream definition, restated in Python."""
    m = 0xFFFFFFFF
    s0 = _h32((seed & m) + 0x9E3779B9)
    s1 = _h32((seed >> 32) ^ 0x85EBCA6B ^ s0)
    p0 = _h32((pixel & m) ^ s0)
    p1 = _h32((pixel >> 32) + p0 + s1)
    x = (_h32((sample & m) ^ p0) ^ ((p1 + (sample >> 32) * 0x9E3779B9) & m)) | 1
    out = []
    for _ in range(n):  # xorshift32 (13, 17, 5)
        x ^= (x << 13) & m
        x ^= x >> 17
        x ^= (x << 5) & m
        out.append((x >> 8) * 2.0 ** -24)
    return out


@pytest.mark.parametrize("seed,pixel,sample", [(0, 0, 0), (1, 12345, 7), (2**40 + 3, 2**33 + 5, 2**35 + 11)])
def test_rng_matches_its_definition(seed, pixel, sample):
    from oracle.oracle import rng_draws

    assert list(rng_draws(seed, pixel, sample, 12)) == _spec_draws(seed, pixel, sample, 12)


def test_rng_statistics():
    """Uniformity (chi-square over 64 bins) and no lag-1 / cross-sample correlation for the draws
    a path consumes: 20 draws of 4,000 samples over 4 pixels."""
    from oracle.oracle import rng_draws

    d = np.array([rng_draws(9, px, s, 20) for px in range(4) for s in range(1000)])
    u = d.ravel()
    hist = np.histogram(u, bins=64, range=(0, 1))[0]
    exp = u.size / 64
    chi2 = ((hist - exp) ** 2 / exp).sum()
    assert chi2 < 120, chi2  # 63 dof: p ~ 1e-5
    for a, b in [(d[:, :-1].ravel(), d[:, 1:].ravel()), (d[:-1].ravel(), d[1:].ravel())]:
        assert abs(np.corrcoef(a, b)[0, 1]) < 0.02
    assert abs(u.mean() - 0.5) < 0.005


def test_rng_pairs_and_lags():
    """The xorshift32 stream's consecutive draws are used as 2-D points (theta with the pow draw,
    the camera's sub-pixel x and y, the diffuse acos and angle): 16x16 chi-square of (U_n, U_n+1)
    at every draw index a path reaches, correlations at lags 1-4, and the first draws of
    neighbouring pixels and samples."""
    from oracle.oracle import rng_draws

    d = np.array([rng_draws(3, px, s, 24) for px in range(8) for s in range(1500)])
    for j in range(0, 23, 2):
        h = np.histogram2d(d[:, j], d[:, j + 1], bins=16, range=[[0, 1], [0, 1]])[0]
        exp = d.shape[0] / 256
        chi2 = ((h - exp) ** 2 / exp).sum()
        assert chi2 < 360, (j, chi2)  # 255 dof: p ~ 1e-5
    for lag in range(1, 5):
        assert abs(np.corrcoef(d[:, :-lag].ravel(), d[:, lag:].ravel())[0, 1]) < 0.01
    # the same sample index of neighbouring pixels, and neighbouring samples of one pixel
    first = d[:, :2].reshape(8, 1500, 2)
    assert abs(np.corrcoef(first[:-1, :, 0].ravel(), first[1:, :, 0].ravel())[0, 1]) < 0.02
    assert abs(np.corrcoef(first[:, :-1, 1].ravel(), first[:, 1:, 1].ravel())[0, 1]) < 0.02
