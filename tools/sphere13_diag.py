"""Sphere 13 of app.png against the oracle, pixel group by pixel group (CPU only, diagnostic).

VERDICT r4 item 1: sphere 13 (bounce.txt:88) read 3-4 % darker in the oracle than in the
reference's own screenshot while the cut-out face 11 next to it read 1.4-2.1 % brighter.  Round 6
found the cause: the fixture had been cut one pixel off (tools/app_offset_diag.py); with the
fixture at its registered offset (5, 86) this tool reads sphere 13 within noise.  This
splits the sphere's usable pixels by the direction of the surface normal at the primary hit and
prints, per bin, oracle / screenshot in linear radiance (the screenshot linearised at the middle
of its 8-bit truncation interval, as tests/test_oracle_pin.py does).

    python tools/sphere13_diag.py [spp] [seed]
"""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from oracle.oracle import OracleScene  # noqa: E402

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")
W = H = 700
CENTER = np.array([-1.0, -1.25, -1.0])
RADIUS = 0.5


def camera_dir(x, y):
    """FrustumCamera.GetRay (FrustumCamera.cs:33-41) for camera 0 of bounce.txt at 700 x 700."""
    pos = np.array([2.8, -2.8, -1.0])
    look = np.array([0.0, 0.0, -1.0]) - pos
    look /= np.linalg.norm(look)
    up0 = np.array([0.0, 0.0, -1.0])
    side = np.cross(look, -up0)
    side /= np.linalg.norm(side)
    up = np.cross(look, side)
    up /= np.linalg.norm(up)
    side = -side
    t = np.tan(np.radians(90) / 2)
    tx, ty = t * W / H, -t
    d = look + side * tx * ((x - W / 2) / (W / 2)) + up * ty * ((y - H / 2) / (H / 2))
    return pos, d / np.linalg.norm(d)


def main():
    spp = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    net = len(sys.argv) > 3 and sys.argv[3] == "net"  # draws from .NET System.Random, one stream per pixel
    d = np.load(os.path.join(GOLDEN, "screenshot_app_bounce700.npz"))
    ref, xs, ys = d["rgb"].astype(np.int64), d["xs"], d["ys"]
    orc = OracleScene.from_file(os.path.join(GOLDEN, "scenes", "bounce.txt"))
    orc.set_size(W, H)
    ids = orc.primary_ids()
    rid = ids[np.ix_(xs, ys)].T
    inner = np.ones_like(rid, bool)
    for dx in (-1, 0, 1):
        for dy in (-1, 0, 1):
            inner &= ids[np.ix_(np.clip(xs + dx, 0, W - 1), np.clip(ys + dy, 0, H - 1))].T == rid
    sel = {}
    for prim in (13, 11, 12):
        m = (rid == prim) & inner & np.all(ref < 250, axis=-1) & (ref.max(-1) >= 16)
        jj, ii = np.nonzero(m)
        sel[prim] = (jj, ii)
    pts = [(xs[i], ys[j], p) for p, (jj, ii) in sel.items() for j, i in zip(jj, ii)]
    lin = np.zeros((len(pts), 3))

    def run(idx):
        for k in idx:
            if net:
                s, n, m, _ = orc.render_tile_netrandom(int(pts[k][0]), int(pts[k][1]), 1, 1, spp,
                                                       seed=(seed * 1000003 + k * 7919) & 0x7fffffff)
            else:
                s, n, m, _ = orc.render_tile(int(pts[k][0]), int(pts[k][1]), 1, 1, spp, seed=seed)
            lin[k] = s[0, 0] / max(1, int(n[0, 0]))

    with ThreadPoolExecutor(os.cpu_count() or 1) as ex:
        list(ex.map(run, np.array_split(np.arange(len(pts)), 64)))
    k = 0
    for prim, (jj, ii) in sel.items():
        n = len(jj)
        o = lin[k:k + n]
        k += n
        r = ref[jj, ii]
        lo, hi, mid = (r / 255.0) ** 2.2, ((r + 1.0) / 255.0) ** 2.2, ((r + 0.5) / 255.0) ** 2.2
        print(f"prim {prim}: {n} px  oracle/mid R G B = {np.round(o.mean(0) / mid.mean(0), 4)}")
        if prim != 13:
            # split by screen x (distance along the face)
            xsv = xs[ii]
            for q in np.array_split(np.argsort(xsv), 4):
                print(f"   x {xsv[q].min():3d}-{xsv[q].max():3d}: {len(q):4d} px ratio "
                      f"{np.round(o[q].mean(0) / mid[q].mean(0), 4)}  code {np.round(r[q].mean(0), 1)}")
            continue
        nrm = []
        for j, i in zip(jj, ii):
            p0, dd = camera_dir(xs[i] + 0.5, ys[j] + 0.5)
            oc = p0 - CENTER
            b = oc @ dd
            c = oc @ oc - RADIUS ** 2
            t = -b - np.sqrt(max(b * b - c, 0.0))
            nrm.append((p0 + t * dd - CENTER) / RADIUS)
        nrm = np.array(nrm)
        for axis, name in ((0, "nx"), (1, "ny"), (2, "nz (+ = down)")):
            print(f"  by {name}:")
            for q in np.array_split(np.argsort(nrm[:, axis]), 4):
                print(f"   {nrm[q, axis].min():+.2f}..{nrm[q, axis].max():+.2f}: {len(q):4d} px ratio "
                      f"{np.round(o[q].mean(0) / mid[q].mean(0), 4)}  code {np.round(r[q].mean(0), 1)}"
                      f"  interval-dev lum {100 * ((o[q] @ [.299, .587, .114]).mean() / (mid[q] @ [.299, .587, .114]).mean() - 1):+.2f} %")
        # brightness split: dim vs bright pixels (highlight)
        lum = mid @ np.array([.299, .587, .114])
        print("  by screenshot luminance:")
        for q in np.array_split(np.argsort(lum), 4):
            print(f"   lum {lum[q].min():.3f}..{lum[q].max():.3f}: {len(q):4d} px ratio "
                  f"{np.round(o[q].mean(0) / mid[q].mean(0), 4)}")


if __name__ == "__main__":
    main()
