"""Pins the oracle to the reference's own output: the screenshots it rendered.

The reference cannot run here (C# WinForms) and has no fixtures; its only outputs are the
tonemapped screenshots in Screenshots/ (unknown spp, unseeded RNG, 8-bit).  The committed
sparse samples (tests/golden/screenshot_*.npz, from tests/golden/make_golden.py) pin:
  * geometry: which pixels see the scene at all (alpha > 0 = at least one camera hit), i.e.
    the loader's transforms, the camera model and the closest-hit query;
  * radiometry (die.png): mean linear radiance of fully-covered pixels, i.e. the bounce
    loop's estimator, RandomShine, Fresnel-free specular/diffuse split and tint rule.
bounce-with-lens.png was captured at an unknown exposure/recursion setting (its linear
radiance is ~1.4x the file's recursion-10 render); only its geometry is asserted.
"""
import os

import numpy as np
import pytest

from oracle.oracle import OracleScene, sample_output

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _render_sparse(scene_file, size, xs, ys, spp):
    orc = OracleScene.from_file(os.path.join(GOLDEN, "scenes", scene_file))
    orc.set_size(*size)
    out = np.zeros((len(ys), len(xs), 4), np.int64)
    for j, y in enumerate(ys):
        for i, x in enumerate(xs):
            s, n, m, _ = orc.render_tile(int(x), int(y), 1, 1, spp, seed=1)
            c = sample_output(tuple(s[0, 0]), int(n[0, 0]), int(m[0, 0])) & 0xFFFFFFFF
            out[j, i] = ((c >> 16) & 255, (c >> 8) & 255, c & 255, c >> 24)
    return out


def _load(key):
    d = np.load(os.path.join(GOLDEN, f"screenshot_{key}.npz"))
    return d["rgba"].astype(np.int64), d["xs"], d["ys"], tuple(int(v) for v in d["size"])


def test_die_screenshot_geometry_and_radiance():
    ref, xs, ys, size = _load("die")
    assert size == (1280, 960)
    got = _render_sparse("die.txt", size, xs, ys, 48)
    cov_ref, cov_got = ref[..., 3] > 0, got[..., 3] > 0
    agree = (cov_ref == cov_got).mean()
    assert agree > 0.985, f"coverage agreement {agree:.4f}"
    full = (ref[..., 3] == 255) & (got[..., 3] == 255)
    assert full.sum() > 1000
    lin_ref = ((ref[full][:, :3] / 255.0) ** 2.2).mean(axis=0)
    lin_got = ((got[full][:, :3] / 255.0) ** 2.2).mean(axis=0)
    ratio = lin_got / lin_ref
    # per-channel mean linear radiance within 8% (48 spp + 8-bit quantisation + clipping)
    assert np.all(np.abs(ratio - 1) < 0.08), ratio


def test_bounce_screenshot_geometry_and_uniform_exposure():
    ref, xs, ys, size = _load("bounce1200")
    assert size == (1200, 1200)
    got = _render_sparse("bounce.txt", size, xs, ys, 32)
    cov_ref, cov_got = ref[..., 3] > 0, got[..., 3] > 0
    agree = (cov_ref == cov_got).mean()
    assert agree > 0.985, f"coverage agreement {agree:.4f}"
    # radiance: one global factor (the capture's exposure) explains the image -- the block
    # ratios are uniform across walls, floor, lens and mirror sphere
    lr, lg = (ref[..., :3] / 255.0) ** 2.2, (got[..., :3] / 255.0) ** 2.2
    full = (ref[..., 3] == 255) & (got[..., 3] == 255)
    ratios = []
    for by in range(0, 150, 25):
        for bx in range(0, 150, 25):
            m = full[by:by + 25, bx:bx + 25]
            if m.sum() >= 50:
                ratios.append(lr[by:by + 25, bx:bx + 25][m].mean() / lg[by:by + 25, bx:bx + 25][m].mean())
    ratios = np.array(ratios)
    assert len(ratios) >= 20
    assert 1.2 < np.median(ratios) < 1.7
    assert ratios.std() / ratios.mean() < 0.15, ratios
