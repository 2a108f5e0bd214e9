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

* die.png (1280x960): captured at the file's exposure; radiance within 2.5 %.
* app.png: bounce.txt in the application window at the UI's exposure 1.000 (MainWindow.cs:40)
  after 4,826 spp, camera 0, recursion 10; its 700x700 viewport pins bounce.txt's radiance
  within 3 % (FullRaytracer.cs:179-205).
* bounce-with-lens.png (1200x1200) was captured at an unknown exposure/recursion setting (its
  linear radiance is ~1.4x the file's recursion-10 render): geometry plus one uniform factor.
"""
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


def test_die_screenshot_geometry_and_radiance():
    ref, xs, ys, size = _load("die")
    assert size == (1280, 960)
    got, lin, miss = _render_sparse("die.txt", size, xs, ys, 192)
    agree = ((ref[..., 3] > 0) == (got[..., 3] > 0)).mean()
    assert agree > 0.985, f"coverage agreement {agree:.4f}"
    ok = (ref[..., 3] == 255) & (miss == 0) & np.all(ref[..., :3] < 250, axis=-1)
    assert ok.sum() > 1000
    ratio = _linear_ratio(ref[..., :3], lin, ok)
    print("die.png radiance ratio (R, G, B):", ratio, "pixels", int(ok.sum()))
    assert np.all(np.abs(ratio - 1) < 0.025), ratio


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


def test_bounce_app_screenshot_exposure1_radiance():
    """bounce.txt at exposure 1.000 (Screenshots/app.png viewport): coverage, and per-channel mean
    linear radiance of the fully covered, unsaturated pixels within 3 % of the oracle."""
    d = np.load(os.path.join(GOLDEN, "screenshot_app_bounce700.npz"))
    ref, xs, ys = d["rgb"].astype(np.int64), d["xs"], d["ys"]
    assert tuple(d["size"]) == (700, 700) and float(d["exposure"][0]) == 1.0
    got, lin, miss = _render_sparse("bounce.txt", (700, 700), xs, ys, 192)
    panel = np.all(ref == d["panel"], axis=-1)  # a transparent (all-miss) pixel shows the panel grey
    agree = (panel != (got[..., 3] > 0)).mean()
    assert agree > 0.99, f"coverage agreement {agree:.4f}"
    ok = (miss == 0) & ~panel & np.all(ref < 250, axis=-1)
    assert ok.sum() > 2000
    ratio = _linear_ratio(ref, lin, ok)
    print("app.png exposure-1 radiance ratio (R, G, B):", ratio, "pixels", int(ok.sum()))
    assert np.all(np.abs(ratio - 1) < 0.03), ratio
