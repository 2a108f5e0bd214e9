"""Pins the oracle to the reference's own output: the screenshots it rendered.

The reference cannot run here (C# WinForms) and has no fixtures; its only outputs are the
tonemapped screenshots in Screenshots/ (unseeded RNG, 8-bit).  The committed sparse samples
(tests/golden/screenshot_*.npz, from tests/golden/make_golden.py) pin:
  * geometry: which pixels see the scene at all, i.e. the loader's transforms, the camera model
    and the closest-hit query;
  * radiometry: mean linear radiance of fully covered, unsaturated pixels, i.e. the bounce loop's
    estimator, RandomShine, Fresnel, the specular/diffuse split and the tint rule.
Radiance is compared in the linear domain: the oracle's per-pixel mean sum/samples against the
screenshot's code linearised at the middle of its truncation interval, ((v + 0.5) / 255)^2.2
(SampleSet.GetOutput truncates, SampleSet.cs:61-113).  Tonemapping a noisy few-hundred-spp mean
and clipping it at 1 would bias the comparison downwards (die.png read 0.96-0.99 that way at
48 spp); the linear means are unbiased, so only sampling noise remains: about 1 % at 192 spp
over a few thousand pixels (seeds 1-3: die.png 0.990-1.002, app.png 0.991-1.010).

* die.png (1280x960): captured at the file's exposure; radiance within 2 %.
* app.png: bounce.txt in the application window at the UI's exposure 1.000 (MainWindow.cs:40)
  after 4,826 spp, camera 0, recursion 10; its 700x700 viewport pins bounce.txt's radiance
  within 2 % (FullRaytracer.cs:179-205).
* Region by region (both screenshots): pixels grouped by the oracle's primary-ID map (the
  DebugRaycaster Primitives mode, DebugRaycaster.cs:193-199), so that paths which cover few pixels
  -- the Fresnel / TIR lens (primitive 20, Raytracer.cs:115-161), the spheres, the cut-out faces,
  the die's faces and pips -- are each pinned on their own instead of inside one frame mean.
* bounce-with-lens.png (1200x1200) was captured at an unknown exposure/recursion setting (its
  linear radiance is ~1.4x the file's recursion-10 render): geometry plus one uniform factor.
"""
import functools
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from oracle.oracle import OracleScene, sample_output

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _render_sparse(scene_file, size, xs, ys, spp, seed=1):
    """The oracle at the sparse pixels: ARGB codes (exposure 1, no background) as [y, x, (r, g, b, a)],
    the linear per-pixel means [y, x, 3] and the miss counts [y, x]."""
    orc = OracleScene.from_file(os.path.join(GOLDEN, "scenes", scene_file))
    orc.set_size(*size)
    codes = np.zeros((len(ys), len(xs), 4), np.int64)
    lin = np.zeros((len(ys), len(xs), 3))
    miss = np.zeros((len(ys), len(xs)), np.int64)

    def row(j):  # ctypes releases the GIL: rows render on the host cores in parallel
        for i, x in enumerate(xs):
            s, n, m, _ = orc.render_tile(int(x), int(ys[j]), 1, 1, spp, seed=seed)
            c = sample_output(tuple(s[0, 0]), int(n[0, 0]), int(m[0, 0])) & 0xFFFFFFFF
            codes[j, i] = ((c >> 16) & 255, (c >> 8) & 255, c & 255, c >> 24)
            lin[j, i] = s[0, 0] / max(1, int(n[0, 0]))
            miss[j, i] = m[0, 0]

    with ThreadPoolExecutor(min(16, os.cpu_count() or 1)) as ex:
        list(ex.map(row, range(len(ys))))
    return codes, lin, miss


def _load(key):
    d = np.load(os.path.join(GOLDEN, f"screenshot_{key}.npz"))
    return d["rgba"].astype(np.int64), d["xs"], d["ys"], tuple(int(v) for v in d["size"])


def _linear_ratio(ref_rgb, lin, ok):
    """Per-channel mean linear radiance, oracle / screenshot, over the pixels `ok`."""
    return lin[ok].mean(axis=0) / (((ref_rgb[ok] + 0.5) / 255.0) ** 2.2).mean(axis=0)


def _render_points(scene_file, size, pts, spp, seed):
    """The oracle's linear per-pixel means [n, 3] and miss counts [n] at the pixels pts [(x, y)]."""
    orc = OracleScene.from_file(os.path.join(GOLDEN, "scenes", scene_file))
    orc.set_size(*size)
    lin = np.zeros((len(pts), 3))
    miss = np.zeros(len(pts), np.int64)
    chunks = np.array_split(np.arange(len(pts)), 64)

    def run(idx):  # ctypes releases the GIL: chunks render on the host cores in parallel
        for k in idx:
            s, n, m, _ = orc.render_tile(int(pts[k][0]), int(pts[k][1]), 1, 1, spp, seed=seed)
            lin[k] = s[0, 0] / max(1, int(n[0, 0]))
            miss[k] = m[0, 0]

    with ThreadPoolExecutor(min(16, os.cpu_count() or 1)) as ex:
        list(ex.map(run, chunks))
    return lin, miss


def _region_ids(scene_file, size, xs, ys):
    """The oracle's primary-ID map (exact; integer pixel, no jitter or depth of field) at the sparse
    pixels, and whether each one's 3x3 neighbourhood holds one ID (away from region edges)."""
    orc = OracleScene.from_file(os.path.join(GOLDEN, "scenes", scene_file))
    orc.set_size(*size)
    ids = orc.primary_ids()  # [x, y]
    w, h = size
    rid = ids[np.ix_(xs, ys)].T  # [y, x]
    inner = np.ones_like(rid, bool)
    for dx in (-1, 0, 1):
        for dy in (-1, 0, 1):
            inner &= ids[np.ix_(np.clip(xs + dx, 0, w - 1), np.clip(ys + dy, 0, h - 1))].T == rid
    return rid, inner


LUMA = np.array([0.299, 0.587, 0.114])  # DoubleColor.GetLuminance (DoubleColor.cs:76-79)


def _check_regions(label, ref, lin, ok, rid, regions, tol, min_pixels=200, tol_of=None):
    """Region by region: the oracle's mean linear radiance against the screenshot's, where a pixel's
    code v only says its value lies in [v, v + 1) / 255 before the 2.2 power (truncation,
    SampleSet.cs:61-113).  The deviation is the distance of the oracle's mean from the region's
    interval [mean ((v / 255)^2.2), mean (((v + 1) / 255)^2.2)], relative; it is asserted within
    `tol` for the region's luminance (0.299 R + 0.587 G + 0.114 B) and for every channel whose
    mean code is at least 48.  A darker channel is only reported: one 8-bit step there is 4.5 % and
    more of the linear value, and in die.png such channels are the light blurred in by the depth of
    field from neighbouring regions (the -x face has no red albedo, die.txt:44-46, yet its pixels
    carry red codes near its edges).  Returns {region: (pixels, deviation R, G, B, luminance)}."""
    lo = (ref / 255.0) ** 2.2
    hi = ((ref + 1.0) / 255.0) ** 2.2
    out = {}
    t_of = tol_of or {}
    for name, m in regions:
        m = m & ok & (ref.max(axis=-1) >= 16)  # near-black pixels say nothing of the radiance
        n = int(m.sum())
        if n < min_pixels:
            continue
        o, a, b = lin[m].mean(0), lo[m].mean(0), hi[m].mean(0)
        o, a, b = np.append(o, o @ LUMA), np.append(a, a @ LUMA), np.append(b, b @ LUMA)
        dev = np.where(o > b, o / b - 1, np.where(o < a, o / a - 1, 0.0))
        code = np.append(ref[m].mean(0), 255.0)
        t = t_of.get(name, tol)
        checked = code >= 48
        out[name] = (n, dev)
        print(f"{label} region {name}: {n} px, mean code {np.round(code[:3], 1)}, deviation R G B Y "
              f"{np.round(100 * dev, 2)} % (bound {100 * t:.0f} % on {''.join(c for c, k in zip('RGBY', checked) if k)})")
        bad = checked & ~(np.abs(dev) <= t)
        assert not bad.any(), f"{label} region {name}: deviation {dev} beyond {t}"
    return out


def test_die_screenshot_geometry_and_radiance():
    """die.png: coverage (32 spp over every sampled pixel) and mean linear radiance of the fully
    covered, unsaturated pixels within 2 % of the oracle (768 spp); then region by region: each die
    face and each pip with at least 200 usable pixels, and the 21 pips together, within 4 %."""
    ref, xs, ys, size = _load("die")
    assert size == (1280, 960) and ref.shape[:2] == (240, 320)
    got, _, _ = _render_sparse("die.txt", size, xs, ys, 32)
    agree = ((ref[..., 3] > 0) == (got[..., 3] > 0)).mean()
    assert agree > 0.985, f"coverage agreement {agree:.4f}"
    cand = (ref[..., 3] == 255) & np.all(ref[..., :3] < 250, axis=-1)
    jj, ii = np.nonzero(cand)
    pts = list(zip(xs[ii], ys[jj]))
    lin_p, miss_p = _render_points("die.txt", size, pts, 768, seed=1)
    lin = np.zeros(ref.shape[:2] + (3,))
    miss = np.ones(ref.shape[:2], np.int64)
    lin[jj, ii], miss[jj, ii] = lin_p, miss_p
    ok = cand & (miss == 0)
    assert ok.sum() > 8000
    ratio = _linear_ratio(ref[..., :3], lin, ok)
    print("die.png radiance ratio (R, G, B):", ratio, "pixels", int(ok.sum()))
    assert np.all(np.abs(ratio - 1) < 0.02), ratio
    # regions: die faces 2-7 (-y, +y, +x, -x, -z, +z) and pips 8-28 (die.txt:32-87)
    rid, inner = _region_ids("die.txt", size, xs, ys)
    regions = [(int(r), rid == r) for r in range(2, 29)] + [("pips", (rid >= 8) & (rid <= 28))]
    out = _check_regions("die.png", ref[..., :3], lin, ok & inner, rid, regions, 0.04)
    assert {7, "pips"} <= set(out) and len(out) >= 6, sorted(map(str, out))


def test_bounce_screenshot_geometry_and_uniform_exposure():
    ref, xs, ys, size = _load("bounce1200")
    assert size == (1200, 1200)
    got, lin, miss = _render_sparse("bounce.txt", size, xs, ys, 32)
    agree = ((ref[..., 3] > 0) == (got[..., 3] > 0)).mean()
    assert agree > 0.985, f"coverage agreement {agree:.4f}"
    # radiance: one global factor (the capture's exposure) explains the image -- the block
    # ratios are uniform across walls, floor, lens and mirror sphere
    lr = ((ref[..., :3] + 0.5) / 255.0) ** 2.2
    ok = (ref[..., 3] == 255) & (miss == 0) & np.all(ref[..., :3] < 250, axis=-1)
    ratios = []
    for by in range(0, 150, 25):
        for bx in range(0, 150, 25):
            m = ok[by:by + 25, bx:bx + 25]
            if m.sum() >= 50:
                ratios.append(lr[by:by + 25, bx:bx + 25][m].mean() / lin[by:by + 25, bx:bx + 25][m].mean())
    ratios = np.array(ratios)
    print("bounce-with-lens.png block ratios: median", np.median(ratios), "CoV", ratios.std() / ratios.mean())
    assert len(ratios) >= 20
    assert 1.2 < np.median(ratios) < 1.7
    assert ratios.std() / ratios.mean() < 0.15, ratios


# app.png's viewport sits at (5, 86) of the window (tests/golden/make_golden.py APP_OFFSET): the
# light box's saturated footprint pins it to the pixel (test_bounce_app_viewport_offset_from_light_box).
# Until round 6 the fixture was cut at (4, 85), one pixel off in x and y; that alone put sphere 13
# (bounce.txt:88) 3.5 % below the screenshot -- -7 to -16 % R in its upper cells, where the one-pixel
# shift slides its bright rim over the darker shading -- and the ceiling ring around the light box
# 12 % above it.  At (5, 86) both read within 0.3 % at full resolution (tools/app_offset_diag.py,
# DESIGN.md §4.1), and every region is held to 2 % instead of 4 %.


@functools.lru_cache(maxsize=None)
def _app_regions(spp, seed=1):
    d = np.load(os.path.join(GOLDEN, "screenshot_app_bounce700.npz"))
    ref, xs, ys = d["rgb"].astype(np.int64), d["xs"], d["ys"]
    assert tuple(d["size"]) == (700, 700) and float(d["exposure"][0]) == 1.0 and ref.shape[:2] == (175, 175)
    got, lin, miss = _render_sparse("bounce.txt", (700, 700), xs, ys, spp, seed=seed)
    panel = np.all(ref == d["panel"], axis=-1)  # a transparent (all-miss) pixel shows the panel grey
    ok = (miss == 0) & ~panel & np.all(ref < 250, axis=-1)
    rid, inner = _region_ids("bounce.txt", (700, 700), xs, ys)
    return ref, got, lin, panel, ok, rid, inner


def test_bounce_app_screenshot_exposure1_radiance():
    """bounce.txt at exposure 1.000 (Screenshots/app.png viewport, every 4th pixel): coverage, the
    per-channel mean linear radiance of the fully covered, unsaturated pixels within 1 % of the
    oracle (1,024 spp), and region by region: every primitive with at least 200 usable pixels --
    the room's walls, floor and ceiling, the cut-out faces, sphere 13, the rotated cube's faces and
    the Fresnel / TIR lens (20) -- within 2 %."""
    ref, got, lin, panel, ok, rid, inner = _app_regions(1024)
    agree = (panel != (got[..., 3] > 0)).mean()
    assert agree > 0.995, f"coverage agreement {agree:.4f}"
    assert ok.sum() > 10000
    ratio = _linear_ratio(ref, lin, ok)
    print("app.png exposure-1 radiance ratio (R, G, B):", ratio, "pixels", int(ok.sum()))
    assert np.all(np.abs(ratio - 1) < 0.01), ratio
    regions = [(int(r), rid == r) for r in range(22)]
    out = _check_regions("app.png", ref, lin, ok & inner, rid, regions, 0.02)
    # the lens, sphere 13, the floor (10), the far walls (6, 9) and a rotated-cube face must be among them
    assert {6, 9, 10, 13, 20} <= set(out) and len(out) >= 8, sorted(out)


def _app_crop(key):
    d = np.load(os.path.join(GOLDEN, "screenshot_app_bounce700.npz"))
    return d[key].astype(np.int64), tuple(int(v) for v in d[key + "_window"])


def _window_mean(x0, y0, w, h, spp, seed=1):
    """The oracle's linear per-pixel means [h, w, 3] over a window of the 700 x 700 frame."""
    orc = OracleScene.from_file(os.path.join(GOLDEN, "scenes", "bounce.txt"))
    orc.set_size(700, 700)
    out = np.zeros((h, w, 3))

    def row(j):
        s, n, _, _ = orc.render_tile(x0, y0 + j, w, 1, spp, seed=seed)
        out[j] = s[:, 0] / np.maximum(n[:, 0], 1)[:, None]

    with ThreadPoolExecutor(min(16, os.cpu_count() or 1)) as ex:
        list(ex.map(row, range(h)))
    return out


def test_bounce_app_viewport_offset_from_light_box():
    """The light box (bounce.txt:29-32, emission 5) in app.png: its saturated footprint (the box and
    the ceiling next to it, which it lights above 1) equals the oracle's at the fixture's viewport
    offset and at no shift within 3 pixels -- the screenshot is registered to the pixel, and the
    box's position, size and visible faces (+x, -y and the bottom +z, IDs 0, 3, 4) are the
    reference's."""
    crop, (x0, y0, w, h) = _app_crop("light")
    m = 3  # the crop's margin on every side
    lin = _window_mean(x0 + m, y0 + m, w - 2 * m, h - 2 * m, 512)
    ours = (np.clip(lin, 0, 1) ** (1 / 2.2) * 255).astype(np.int64).max(-1) >= 250  # GetOutput's truncation
    diff = {}
    for dy in range(-m, m + 1):
        for dx in range(-m, m + 1):
            sat = crop[m + dy:m + dy + h - 2 * m, m + dx:m + dx + w - 2 * m].max(-1) >= 250
            diff[(dx, dy)] = int((sat ^ ours).sum())
    best = min(diff, key=diff.get)
    print("light box saturated pixels", int(ours.sum()), "differing at shift (0, 0):", diff[(0, 0)],
          "next best:", sorted(diff.values())[1])
    assert best == (0, 0) and diff[(0, 0)] <= 0.03 * ours.sum(), diff
    assert sorted(diff.values())[1] >= 1.5 * diff[(0, 0)] + 10
    orc = OracleScene.from_file(os.path.join(GOLDEN, "scenes", "bounce.txt"))
    orc.set_size(700, 700)
    ids = orc.primary_ids(x0, y0, w, h).T  # [y, x]
    light = (ids >= 0) & (ids <= 4)
    assert set(np.unique(ids[light]).tolist()) == {0, 3, 4}
    # every pixel the box covers whole (its 3 x 3 neighbourhood's corner IDs all on the box; a primary-ID
    # pixel is sampled at its corner) is saturated in the screenshot
    from scipy.ndimage import binary_erosion

    whole = binary_erosion(light, np.ones((3, 3), bool))
    assert whole.sum() > 1500 and (crop[whole].max(-1) >= 250).all()


def test_bounce_app_subregions_sphere13_and_ceiling_ring():
    """Sub-regions that a region average could hide: sphere 13's upper and lower halves
    (every 4th pixel) and the ceiling ring 2-10 pixels around the light box (full resolution) --
    the sphere's upper half faces the ceiling and the light, the ring is lit by the box's sides at
    grazing angles -- each within 2 % of the screenshot, as every region is."""
    ref, got, lin, panel, ok, rid, inner = _app_regions(1024)
    d = np.load(os.path.join(GOLDEN, "screenshot_app_bounce700.npz"))
    ys = d["ys"]
    usable = ok & inner & (rid == 13) & (ref.max(-1) >= 16)
    rows = np.nonzero(usable)[0]
    mid_row = np.median(rows)
    upper = usable & (np.arange(usable.shape[0])[:, None] < mid_row)  # image up is the scene's -z: the ceiling
    lower = usable & ~upper
    print("sphere 13 halves split at screen row", int(ys[int(mid_row)]))
    out = _check_regions("app.png sphere 13", ref, lin, usable, rid, [("upper", upper), ("lower", lower)], 0.02,
                         min_pixels=150)
    assert set(out) == {"upper", "lower"}
    # the ceiling ring: the ceiling (9) 2-10 pixels from the light box's primary-ID footprint, unsaturated
    from scipy.ndimage import distance_transform_edt

    crop, (x0, y0, w, h) = _app_crop("ring")
    orc = OracleScene.from_file(os.path.join(GOLDEN, "scenes", "bounce.txt"))
    orc.set_size(700, 700)
    ids = orc.primary_ids(x0, y0, w, h).T
    dist = distance_transform_edt(~((ids >= 0) & (ids <= 4)))
    ring = (ids == 9) & (dist >= 2) & (dist <= 10) & (crop.max(-1) < 250)
    jj, ii = np.nonzero(ring)
    lin_p, miss_p = _render_points("bounce.txt", (700, 700), list(zip(x0 + ii, y0 + jj)), 512, seed=1)
    assert (miss_p == 0).all() and len(jj) > 1000
    lin_r = np.zeros((h, w, 3))
    lin_r[jj, ii] = lin_p
    out = _check_regions("app.png ceiling ring", crop, lin_r, ring, ids, [("ring", ring)], 0.02)
    assert set(out) == {"ring"}
