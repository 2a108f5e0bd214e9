"""Where the reference's app.png viewport sits, and sphere 13 / the ceiling ring against the oracle
(CPU only, diagnostic; needs /root/reference/Screenshots/app.png).

VERDICT r5 item 2.  The light box (bounce.txt:29-32, emission 5, IDs 0-4) is the sharpest feature
of the screenshot: every pixel it covers by more than ~1/6 saturates (5 x coverage >= 0.96).  The
oracle predicts that mask exactly from its primary-ID map at 4 x 4 sub-pixel positions
(FrustumCamera.GetRay is linear in the pixel coordinate, so pixel (x, y) of a 2800 x 2800 frame is
(x / 4, y / 4) of the 700 x 700 one).  Matching it against the screenshot's saturated pixels over
nearby viewport offsets says where the 700 x 700 image sits in the window (the oracle's own
rendered saturation is used: the ceiling right next to the box is lit above 1 and saturates too).  Then, at the old
(4, 85) and the matched offset: sphere 13 split 5 x 5 over its screen footprint, its upper and lower
halves, and the ceiling ring around the light box, oracle against screenshot in linear radiance; and
the "selection artefact" check of the ring: a second oracle frame (another seed) quantised like a
screenshot and put through the same >= 250 drop and ring selection.

    python tools/app_offset_diag.py [spp]
"""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
from oracle.oracle import OracleScene  # noqa: E402

SCENE = os.path.join(ROOT, "tests", "golden", "scenes", "bounce.txt")
W = H = 700
LUMA = np.array([0.299, 0.587, 0.114])


def light_coverage(x0, y0, w, h, sub=4):
    """Fraction of each pixel of the window covered by the light box (IDs 0-4), [h, w]."""
    orc = OracleScene.from_file(SCENE)
    orc.set_size(W * sub, H * sub)
    ids = orc.primary_ids(x0 * sub, y0 * sub, w * sub, h * sub)  # [x, y]
    lit = ((ids >= 0) & (ids <= 4)).T.reshape(h, sub, w, sub)
    return lit.mean(axis=(1, 3))


def render_window(x0, y0, w, h, spp, seed):
    """The oracle's per-pixel linear mean [h, w, 3] over the window (rows in parallel)."""
    orc = OracleScene.from_file(SCENE)
    orc.set_size(W, H)
    out = np.zeros((h, w, 3))

    def row(j):
        s, n, m, _ = orc.render_tile(x0, y0 + j, w, 1, spp, seed=seed)
        out[j] = s[:, 0] / np.maximum(n[:, 0], 1)[:, None]

    with ThreadPoolExecutor(os.cpu_count() or 1) as ex:
        list(ex.map(row, range(h)))
    return out


def codes(lin):
    """SampleSet.GetOutput at exposure 1 without misses: truncated 8-bit codes of x^(1/2.2)."""
    return (np.clip(lin, 0, 1) ** (1 / 2.2) * 255).astype(np.int64)


def main():
    from PIL import Image

    spp = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    img = np.asarray(Image.open("/root/reference/Screenshots/app.png"))[..., :3].astype(np.int64)
    # 1. the light box's footprint and the viewport offset: the oracle's own saturated pixels (the
    # box and the ceiling right next to it, which it lights to > 1) against the screenshot's
    x0, y0, w, h = 274, 218, 152, 92
    ring_lin = render_window(x0, y0, w, h, spp, 1)
    pred = (codes(ring_lin) >= 250).any(-1)
    cov = light_coverage(x0, y0, w, h)
    best = None
    print("viewport offset -> pixels where the screenshot's and the oracle's saturated masks differ")
    for oy in range(82, 90):
        row = []
        for ox in range(1, 9):
            sat = (img[oy + y0:oy + y0 + h, ox + x0:ox + x0 + w] >= 250).any(-1)
            d = int((sat ^ pred).sum())
            row.append(f"({ox},{oy}) {d:4d}")
            if best is None or d < best[0]:
                best = (d, ox, oy)
        print("  " + "  ".join(row))
    print(f"light box: {int((cov > 0).sum())} pixels it touches, {int(pred.sum())} saturated in the oracle; "
          f"best offset ({best[1]}, {best[2]}), {best[0]} differ")
    ids = OracleScene.from_file(SCENE)
    ids.set_size(W, H)
    pid = ids.primary_ids().T  # [y, x]
    faces = sorted(int(f) for f in np.unique(pid) if 0 <= f <= 4)
    print("light-box faces the camera sees:", faces)
    # 2. sphere 13 and the ceiling ring at both offsets
    sy, sx = np.nonzero(pid == 13)
    bx0, bx1, by0, by1 = sx.min(), sx.max() + 1, sy.min(), sy.max() + 1
    lin13 = render_window(int(bx0), int(by0), int(bx1 - bx0), int(by1 - by0), spp, 1)
    ring_lin2 = render_window(x0, y0, w, h, spp, 2)
    inner = np.ones_like(pid, bool)
    for dx in (-1, 0, 1):
        for dy in (-1, 0, 1):
            inner &= np.roll(np.roll(pid, dy, 0), dx, 1) == pid
    light = (pid >= 0) & (pid <= 4)
    from scipy.ndimage import distance_transform_edt
    dist = distance_transform_edt(~light)
    for ox, oy in ((4, 85), (best[1], best[2])):
        view = img[oy:oy + H, ox:ox + W]
        print(f"--- viewport offset ({ox}, {oy})")
        m13 = (pid == 13) & inner & (view < 250).all(-1) & (view.max(-1) >= 16)
        m13w = m13[by0:by1, bx0:bx1]
        ref = view[by0:by1, bx0:bx1]
        mid = ((ref + 0.5) / 255) ** 2.2
        yy, xx = np.nonzero(m13w)
        print(f"sphere 13: {len(yy)} px, oracle/screenshot R G B {np.round(lin13[m13w].mean(0) / mid[m13w].mean(0), 4)}")
        for name, sel in (("upper half", yy < np.median(yy)), ("lower half", yy >= np.median(yy))):
            q = (yy[sel], xx[sel])
            print(f"  {name}: {sel.sum()} px, R G B {np.round(lin13[q].mean(0) / mid[q].mean(0), 4)}")
        print("  5 x 5 split (rows top to bottom), luminance ratio:")
        ey = np.linspace(yy.min(), yy.max() + 1, 6)
        ex = np.linspace(xx.min(), xx.max() + 1, 6)
        for a in range(5):
            cells = []
            for b in range(5):
                c = (yy >= ey[a]) & (yy < ey[a + 1]) & (xx >= ex[b]) & (xx < ex[b + 1])
                if c.sum() >= 10:
                    q = (yy[c], xx[c])
                    cells.append(f"{(lin13[q] @ LUMA).mean() / (mid[q] @ LUMA).mean():6.3f}")
                else:
                    cells.append("   -  ")
            print("   " + " ".join(cells))
        # ceiling (9) 2..10 px from the light box, unsaturated
        ring = (pid == 9) & (dist >= 2) & (dist <= 10)
        rw = ring[y0:y0 + h, x0:x0 + w] & (view[y0:y0 + h, x0:x0 + w] < 250).all(-1)
        refr = view[y0:y0 + h, x0:x0 + w]
        midr = ((refr + 0.5) / 255) ** 2.2
        print(f"ceiling ring 2-10 px: {int(rw.sum())} px, oracle/screenshot R G B "
              f"{np.round(ring_lin[rw].mean(0) / midr[rw].mean(0), 4)}")
        if (ox, oy) != (4, 85):
            # selection artefact check: seed 2 as the "screenshot", quantised, same drop and selection
            fake = codes(ring_lin2)
            rw2 = ring[y0:y0 + h, x0:x0 + w] & (fake < 250).all(-1)
            midf = ((fake + 0.5) / 255) ** 2.2
            print(f"ring, oracle seed 1 / quantised oracle seed 2 (selection alone): {int(rw2.sum())} px, "
                  f"R G B {np.round(ring_lin[rw2].mean(0) / midf[rw2].mean(0), 4)}")


if __name__ == "__main__":
    main()
