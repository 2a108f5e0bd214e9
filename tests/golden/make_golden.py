#!/usr/bin/env python3
"""Regenerates the committed fixtures in tests/golden/.

Two kinds of data:
  * oracle vectors (primary_ids_*, accum_*): the CPU oracle's output on the reference's own
    scene files; they pin the oracle against regressions and give GPU tests a frozen target;
  * screenshot samples (screenshot_*.npz): sparse pixels of the reference's rendered
    screenshots (Screenshots/die.png 1280x960, Screenshots/bounce-with-lens.png 1200x1200),
    i.e. outputs of the reference itself, used to pin the oracle statistically
    (tests/test_oracle_pin.py).  Reading them needs /root/reference (this container only);
    the tests read only the .npz files.

usage: python tests/golden/make_golden.py [--screenshots /root/reference/Screenshots]
"""
import argparse
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)


def oracle_vectors():
    from oracle.oracle import OracleScene

    for name in ("bounce", "die"):
        orc = OracleScene.from_file(os.path.join(HERE, "scenes", name + ".txt"))
        orc.set_size(64, 64)
        ids = orc.primary_ids()
        np.save(os.path.join(HERE, f"primary_ids_{name}_64x64.npy"), ids)
        orc.set_size(32, 32)
        s, n, m, rays = orc.render_tile(0, 0, 32, 32, 16, seed=0, sample_base=0)
        np.savez(os.path.join(HERE, f"accum_{name}_32x32_16spp_seed0.npz"), sum=s, samples=n, misses=m,
                 rays=np.array([rays], np.uint64))
        print(name, "ids", np.unique(ids).size, "rays", rays)


def screenshots(src: str):
    from PIL import Image

    # die.png every 4th pixel (coverage, global and per-region radiance); bounce-with-lens.png every 8th
    for fname, key, step in (("die.png", "die", 4), ("bounce-with-lens.png", "bounce1200", 8)):
        img = np.asarray(Image.open(os.path.join(src, fname)))  # RGBA uint8, row-major [y, x]
        ys = np.arange(step // 2, img.shape[0], step)
        xs = np.arange(step // 2, img.shape[1], step)
        sub = img[np.ix_(ys, xs)]
        np.savez_compressed(os.path.join(HERE, f"screenshot_{key}.npz"), rgba=sub, xs=xs, ys=ys,
                            size=np.array([img.shape[1], img.shape[0]]))
        print(fname, sub.shape)
    # Screenshots/app.png: the WinForms window rendering bounce.txt (camera 0, 700x700, recursion 10)
    # at UI exposure 1.000 after 4,826.37 spp (status bar).  The 700x700 viewport sits at (4, 85) of
    # the window (coverage agreement with the oracle's primary-ID map 0.995, best over nearby
    # offsets); misses are transparent (background alpha 0) over the panel grey (240, 240, 240).
    img = np.asarray(Image.open(os.path.join(src, "app.png")))[..., :3]
    ox, oy, step = 4, 85, 4  # every 4th pixel: regions of a few hundred pixels (tests/test_oracle_pin.py)
    view = img[oy:oy + 700, ox:ox + 700]
    ys = np.arange(step // 2, 700, step)
    xs = np.arange(step // 2, 700, step)
    np.savez_compressed(os.path.join(HERE, "screenshot_app_bounce700.npz"), rgb=view[np.ix_(ys, xs)], xs=xs, ys=ys,
                        size=np.array([700, 700]), offset=np.array([ox, oy]), exposure=np.array([1.0]),
                        spp=np.array([4826.37]), panel=np.array([240, 240, 240]))
    print("app.png viewport", view[np.ix_(ys, xs)].shape)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--screenshots", default="")
    a = ap.parse_args()
    oracle_vectors()
    if a.screenshots:
        screenshots(a.screenshots)
