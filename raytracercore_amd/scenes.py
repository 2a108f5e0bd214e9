"""Procedural scenes of the measurement configs and of the BVH tests.

C4 ("M1M"): the bounce.txt Cornell room, light box and cameras, with the corner cut-out, cube,
lens and spheres replaced by a displaced height field of 1001 x 501 vertices = 1,000,000
triangles. The field spans x in [-1.9, 1.9], y in [-1.9, 1.9], at
z = -0.3 + 0.15 sin(7x) cos(5y) + 0.01 noise(i, j), where noise is the shared counter hash
(include/rtcore_rng.h lowbias32) mapped to [-1, 1) with seed 42. The room spans z in [-2, 0];
its floor is the +z face at z = 0 and "up" is -z, so the field floats 0.3 above the floor.
Material: diffuse .7, specular .2, shininess 250, two-sided. It is emitted as `vertex` / `tri`
scene text, so the reference's loader semantics apply (SceneLoader.cs:305-318).
"""
from __future__ import annotations

import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def _lowbias32(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint32)
    x ^= x >> np.uint32(16)
    x *= np.uint32(0x7FEB352D)
    x ^= x >> np.uint32(15)
    x *= np.uint32(0x846CA68B)
    x ^= x >> np.uint32(16)
    return x


def _room_header(bounce_text: str) -> str:
    """bounce.txt up to (excluding) the corner cut-out: size, cameras, light box and room."""
    cut = bounce_text.index("# corner cutout")
    return bounce_text[:cut]


def heightfield_text(nx: int = 1001, ny: int = 501, seed: int = 42) -> str:
    """`vertex` / `tri` lines of the displaced height field: (nx-1)*(ny-1)*2 triangles."""
    xs = np.linspace(-1.9, 1.9, nx)
    ys = np.linspace(-1.9, 1.9, ny)
    X, Y = np.meshgrid(xs, ys, indexing="xy")  # [ny, nx]
    jj, ii = np.meshgrid(np.arange(ny, dtype=np.uint64), np.arange(nx, dtype=np.uint64), indexing="ij")
    h = _lowbias32(((jj * np.uint64(nx) + ii) ^ np.uint64(seed)).astype(np.uint32))
    noise = (h >> np.uint32(8)).astype(np.float64) * 2.0 ** -23 - 1.0
    Z = -0.3 + 0.15 * np.sin(7 * X) * np.cos(5 * Y) + 0.01 * noise
    verts = np.stack([X.ravel(), Y.ravel(), Z.ravel()], axis=1)
    out = ["\n# procedural height field (SURVEY.md 8(d) C4)\n", "diffuse .7 .7 .7\n", "specular .2 .2 .2\n",
           "emission 0 0 0\n", "shininess 250\n", "invert false\n", "twosided true\n"]
    out.append("".join(f"vertex {x:.9g} {y:.9g} {z:.9g}\n" for x, y, z in verts))
    j, i = np.meshgrid(np.arange(ny - 1), np.arange(nx - 1), indexing="ij")
    v00 = (j * nx + i).ravel()
    v10, v01, v11 = v00 + 1, v00 + nx, v00 + nx + 1
    tris = np.empty((v00.size * 2, 3), dtype=np.int64)
    tris[0::2] = np.stack([v00, v10, v11], axis=1)
    tris[1::2] = np.stack([v00, v11, v01], axis=1)
    out.append("".join(f"tri {a} {b} {c}\n" for a, b, c in tris))
    return "".join(out)


def mesh_scene_text(nx: int = 1001, ny: int = 501, seed: int = 42, bounce_text: str | None = None) -> str:
    """Scene text of config C4 (nx=1001, ny=501: 1M triangles); smaller nx/ny for tests."""
    if bounce_text is None:
        from . import scene_path

        bounce_text = open(scene_path("bounce.txt")).read()
    return _room_header(bounce_text) + heightfield_text(nx, ny, seed)


def soup_scene_text(n: int, seed: int) -> str:
    """Random triangles and spheres (every fifth) over six orders of magnitude of size: a stress
    case for BVH builders and the wide tree's 8-bit quantisation."""
    rng = np.random.default_rng(seed)
    lines = ["size 32 32", "camera 0 -50 0, 0 0 0, 0 0 1, 60"]
    for i in range(n):
        c = rng.uniform(-20, 20, 3)
        s = 10.0 ** rng.uniform(-4, 1)
        if i % 5 == 0:
            lines.append(f"sphere {c[0]:.9g} {c[1]:.9g} {c[2]:.9g} {s:.9g}")
        else:
            for _ in range(3):
                v = c + rng.normal(0, s, 3)
                lines.append(f"vertex {v[0]:.9g} {v[1]:.9g} {v[2]:.9g}")
            b = 3 * (i - i // 5 - 1)
            lines.append(f"tri {b} {b + 1} {b + 2}")
    return "\n".join(lines) + "\n"
