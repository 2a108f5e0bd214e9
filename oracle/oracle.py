"""ctypes binding of the CPU oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, always as the checker.  The product (raytracercore_amd) never imports it.

Parity status: the reference (C# / WinForms, netcoreapp3.1) cannot be built or run here and
has no tests or fixtures; this oracle is pinned by analytic known-answer tests and by a
statistical comparison with the reference's own screenshots (tests/test_oracle_pin.py).
The RNG and libm boundary is "parity unpinned" (System.Random is unseeded, Raytracer.cs:48).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import Optional, Tuple

import numpy as np

from raytracercore_amd import rt_camera, rt_color, rt_prim, rt_scene_params  # ABI structs only

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE, "-j8"], check=True)


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        P = C.POINTER
        sig = {
            "orc_load_text": (C.c_void_p, [C.c_char_p, C.c_char_p, C.c_int32]),
            "orc_from_prims": (C.c_void_p, [P(rt_scene_params), P(rt_prim), C.c_int32, P(rt_camera), C.c_int32]),
            "orc_destroy": (None, [C.c_void_p]),
            "orc_num_prims": (C.c_int32, [C.c_void_p]),
            "orc_num_cameras": (C.c_int32, [C.c_void_p]),
            "orc_export": (C.c_int32, [C.c_void_p, P(rt_scene_params), P(rt_prim), P(rt_camera)]),
            "orc_background": (C.c_int32, [C.c_void_p, P(rt_color), P(C.c_double)]),
            "orc_set_size": (C.c_int32, [C.c_void_p, C.c_int32, C.c_int32]),
            "orc_select_camera": (C.c_int32, [C.c_void_p, C.c_int32]),
            "orc_bvh_info": (C.c_int32, [C.c_void_p, P(C.c_int32), P(C.c_int32)]),
            "orc_bvh_leaf_order": (C.c_int32, [C.c_void_p, P(C.c_int32)]),
            "orc_bvh_boxes": (C.c_int32, [C.c_void_p, P(C.c_double)]),
            "orc_primary_ids": (C.c_int32, [C.c_void_p] + [C.c_int32] * 4 + [P(C.c_int32)]),
            "orc_bvh_counts": (C.c_int32, [C.c_void_p] + [C.c_int32] * 4 + [P(C.c_int32)]),
            "orc_raytrace": (C.c_int32, [C.c_void_p, P(C.c_double), P(C.c_double), P(C.c_double)]),
            "orc_sample": (C.c_int32, [C.c_void_p, C.c_int32, C.c_int32, C.c_uint64, C.c_uint64, P(rt_color),
                                       P(C.c_int32)]),
            "orc_render_tile": (C.c_int32, [C.c_void_p] + [C.c_int32] * 5 + [C.c_uint64, C.c_uint64, P(rt_color),
                                                                               P(C.c_uint32), P(C.c_uint32),
                                                                               P(C.c_uint64)]),
            "orc_sample_trace": (C.c_int32, [C.c_void_p, C.c_int32, C.c_int32, C.c_uint64, C.c_uint64, P(rt_color),
                                             P(C.c_int32)]),
            "orc_render_tile_netrandom": (C.c_int32, [C.c_void_p] + [C.c_int32] * 6 + [P(rt_color), P(C.c_uint32),
                                                                                   P(C.c_uint32), P(C.c_uint64)]),
            "orc_render_frame": (C.c_int32, [C.c_void_p, C.c_int32, C.c_uint64, C.c_int32, P(rt_color), P(C.c_uint32),
                                              P(C.c_uint32), P(C.c_uint64), P(C.c_double), P(C.c_int32)]),
            "orc_sample_output": (C.c_int32, [rt_color, C.c_uint32, C.c_uint32, rt_color, C.c_double, C.c_double]),
            "orc_fresnel": (C.c_double, [C.c_double, C.c_double, C.c_double]),
            "orc_rng_draws": (C.c_int32, [C.c_uint64, C.c_uint64, C.c_uint64, C.c_int32, C.POINTER(C.c_double)]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


class OracleScene:
    """An oracle scene (its own loader + reference BVH), mirroring RaytracerCore.Scene."""

    def __init__(self, handle: int):
        if not handle:
            raise ValueError("oracle scene creation failed")
        self.h = C.c_void_p(handle)

    @classmethod
    def from_text(cls, text: str) -> "OracleScene":
        err = C.create_string_buffer(512)
        h = lib().orc_load_text(text.encode(), err, 512)
        if not h:
            raise ValueError(err.value.decode())
        return cls(h)

    @classmethod
    def from_file(cls, path: str) -> "OracleScene":
        with open(path, encoding="utf-8") as f:
            return cls.from_text(f.read())

    @classmethod
    def from_abi(cls, params: rt_scene_params, prims, cameras) -> "OracleScene":
        n = len(prims)
        parr = (rt_prim * max(1, n))(*prims)
        carr = (rt_camera * max(1, len(cameras)))(*cameras)
        return cls(lib().orc_from_prims(C.byref(params), parr, n, carr, len(cameras)))

    def __del__(self):
        try:
            if self.h:
                lib().orc_destroy(self.h)
                self.h = None
        except Exception:
            pass

    @property
    def n_prims(self) -> int:
        return lib().orc_num_prims(self.h)

    @property
    def n_cameras(self) -> int:
        return lib().orc_num_cameras(self.h)

    def export(self):
        n, nc = self.n_prims, self.n_cameras
        params = rt_scene_params()
        prims = (rt_prim * max(1, n))()
        cams = (rt_camera * max(1, nc))()
        lib().orc_export(self.h, C.byref(params), prims, cams)
        return params, prims[:n], cams[:nc]

    def background(self) -> Tuple[Tuple[float, float, float], float]:
        c, a = rt_color(), C.c_double()
        lib().orc_background(self.h, C.byref(c), C.byref(a))
        return (c.r, c.g, c.b), a.value

    def set_size(self, w: int, h: int) -> None:
        assert lib().orc_set_size(self.h, w, h) == 0

    def select_camera(self, i: int) -> None:
        assert lib().orc_select_camera(self.h, i) == 0

    def size(self) -> Tuple[int, int]:
        p, _, _ = self.export()
        return p.width, p.height

    def bvh_info(self) -> Tuple[int, int]:
        n, d = C.c_int32(), C.c_int32()
        lib().orc_bvh_info(self.h, C.byref(n), C.byref(d))
        return n.value, d.value

    def bvh_leaf_order(self) -> np.ndarray:
        out = np.zeros(max(1, self.n_prims), np.int32)
        k = lib().orc_bvh_leaf_order(self.h, out.ctypes.data_as(C.POINTER(C.c_int32)))
        return out[:k]

    def bvh_boxes(self) -> np.ndarray:
        nodes, _ = self.bvh_info()
        out = np.zeros((max(1, nodes), 8), np.float64)
        lib().orc_bvh_boxes(self.h, out.ctypes.data_as(C.POINTER(C.c_double)))
        return out[:nodes]

    def primary_ids(self, x0=0, y0=0, w=None, h=None) -> np.ndarray:
        W, H = self.size()
        w = W - x0 if w is None else w
        h = H - y0 if h is None else h
        ids = np.empty((w, h), np.int32)
        assert lib().orc_primary_ids(self.h, x0, y0, w, h, ids.ctypes.data_as(C.POINTER(C.c_int32))) == 0
        return ids

    def bvh_counts(self, x0=0, y0=0, w=None, h=None) -> np.ndarray:
        """DebugRaycaster BoundingVolumes mode: BVH.GetIntersectionCount per pixel, [x, y]."""
        W, H = self.size()
        w = W - x0 if w is None else w
        h = H - y0 if h is None else h
        out = np.empty((w, h), np.int32)
        assert lib().orc_bvh_counts(self.h, x0, y0, w, h, out.ctypes.data_as(C.POINTER(C.c_int32))) == 0
        return out

    def raytrace(self, o, d) -> Tuple[int, float]:
        oa = (C.c_double * 4)(*o)
        da = (C.c_double * 4)(*d)
        dist = C.c_double()
        pid = lib().orc_raytrace(self.h, oa, da, C.byref(dist))
        return pid, dist.value

    def sample(self, x, y, seed=0, sample=0):
        c, r = rt_color(), C.c_int32()
        miss = lib().orc_sample(self.h, x, y, seed, sample, C.byref(c), C.byref(r))
        return (c.r, c.g, c.b), bool(miss), r.value

    def render_tile(self, x0, y0, w, h, spp, seed=0, sample_base=0):
        s = np.zeros((w, h, 3), np.float64)
        n = np.zeros((w, h), np.uint32)
        m = np.zeros((w, h), np.uint32)
        rays = C.c_uint64(0)
        assert lib().orc_render_tile(self.h, x0, y0, w, h, spp, seed, sample_base,
                                     s.ctypes.data_as(C.POINTER(rt_color)), n.ctypes.data_as(C.POINTER(C.c_uint32)),
                                     m.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(rays)) == 0
        return s, n, m, rays.value

    def sample_trace(self, x, y, seed=0, sample=0, recursion=32):
        """Diagnostic: one sample's colour, miss flag and path [(primitive, event)] (oracle.h)."""
        c = rt_color()
        tr = (C.c_int32 * (2 * (recursion + 1)))()
        miss = lib().orc_sample_trace(self.h, x, y, seed, sample, C.byref(c), tr)
        path = [(tr[2 * i], tr[2 * i + 1]) for i in range(recursion + 1) if tr[2 * i] != -2]
        return (c.r, c.g, c.b), bool(miss), path

    def render_tile_netrandom(self, x0, y0, w, h, spp, seed=0):
        """Diagnostic: the draws of one reference worker (.NET System.Random(seed), passes row by row)."""
        s = np.zeros((w, h, 3), np.float64)
        n = np.zeros((w, h), np.uint32)
        m = np.zeros((w, h), np.uint32)
        rays = C.c_uint64(0)
        assert lib().orc_render_tile_netrandom(self.h, x0, y0, w, h, spp, seed,
                                               s.ctypes.data_as(C.POINTER(rt_color)), n.ctypes.data_as(C.POINTER(C.c_uint32)),
                                               m.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(rays)) == 0
        return s, n, m, rays.value

    def render_frame(self, spp, seed=0, threads=0):
        W, H = self.size()
        s = np.zeros((W, H, 3), np.float64)
        n = np.zeros((W, H), np.uint32)
        m = np.zeros((W, H), np.uint32)
        rays = C.c_uint64(0)
        secs = C.c_double(0)
        used = C.c_int32(0)
        assert lib().orc_render_frame(self.h, spp, seed, threads, s.ctypes.data_as(C.POINTER(rt_color)),
                                      n.ctypes.data_as(C.POINTER(C.c_uint32)), m.ctypes.data_as(C.POINTER(C.c_uint32)),
                                      C.byref(rays), C.byref(secs), C.byref(used)) == 0
        return s, n, m, rays.value, secs.value, used.value


def fresnel(cos_in: float, ior_in: float, ior_out: float) -> float:
    return lib().orc_fresnel(cos_in, ior_in, ior_out)


def rng_draws(seed: int, pixel: int, sample: int, n: int) -> np.ndarray:
    """The first n uniforms of the shared stream (include/rtcore_rng.h) for (seed, pixel, sample)."""
    out = np.zeros(n, np.float64)
    lib().orc_rng_draws(seed, pixel, sample, n, out.ctypes.data_as(C.POINTER(C.c_double)))
    return out


def sample_output(sum_rgb, samples, misses, background=(0, 0, 0), background_alpha=0.0, exposure=1.0) -> int:
    return lib().orc_sample_output(rt_color(*sum_rgb), samples, misses, rt_color(*background), background_alpha,
                                   exposure)
