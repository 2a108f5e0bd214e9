"""raytracercore_amd -- MI355X (gfx950) path-tracing core behind RaytracerCore's render seam.

The product is ``librtcore_hip.so`` (HIP kernels + the C ABI of ``include/rtcore.h``).  This
module is the Python host mirror used by the tests and the benchmark: ctypes structs that
match the ABI, a ``SceneLoader`` over ``rt_parse_scene`` (SceneLoader.FromFile,
RaytracerCore/SceneLoader.cs:112-440) and a ``GpuRaytracer`` that owns one device scene and
renders tile passes with the semantics of ``Raytracer.Render`` (Raytracer.cs:294-330).

There is no CPU fallback: if the shared library is missing or no HIP device is present the
calls raise ``RtError``.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "librtcore_hip.so")
REPO_ROOT = os.path.dirname(_HERE)

RT_OK = 0
ABI_VERSION = 5  # RTCORE_ABI_VERSION of include/rtcore.h
RT_PRIM_TRIANGLE, RT_PRIM_SPHERE, RT_PRIM_PLANE = 0, 1, 2
RT_FLAG_MIRROR, RT_FLAG_TWOSIDED, RT_FLAG_INVERT, RT_FLAG_HASNORMALS, RT_FLAG_TRANSFORMED = 1, 2, 4, 8, 16
RT_CAMERA_FRUSTUM, RT_CAMERA_ORTHO = 0, 1
RT_TRAVERSAL_AUTO, RT_TRAVERSAL_BRUTE, RT_TRAVERSAL_BVH, RT_TRAVERSAL_BVH2, RT_TRAVERSAL_GROUPED = 0, 1, 2, 3, 4
RT_BVH_BUILDER_AUTO, RT_BVH_BUILDER_HOST, RT_BVH_BUILDER_GPU = 0, 1, 2
BUILD_STAT_NAMES = ("prepare_ms", "bvh_ms", "upload_ms", "gpu_build_ms", "ploc_rounds", "wide_nodes", "stack_need",
                    "flat_rects", "flat_boxes", "flat_frames", "flat_frame_boxes", "flat_frame_rects", "flat_tris",
                    "flat_spheres", "hot_nodes", "jit_status", "jit_compile_ms", "jit_cached", "group_max",
                    "wide_leaves", "compact_leaves", "outer_prims")


def set_jit(on: bool) -> None:
    """rt_set_jit: scene-specialised brute-force kernels (hiprtc) on or off, process-wide."""
    _check(load_library().rt_set_jit(1 if on else 0))


def jit_compile_check(arch: str = "gfx950", grouped: bool = False) -> int:
    """rt_debug_jit_compile (host only): code-object bytes of a scene-specialised build of the
    embedded kernel sources for `arch`; raises RtError with the compiler log on failure."""
    buf = C.create_string_buffer(8192)
    n = load_library().rt_debug_jit_compile(arch.encode(), 1 if grouped else 0, buf, len(buf))
    if n < 0:
        raise RtError(f"scene-specialised build failed: {buf.value.decode(errors='replace')}")
    return n


class RtError(RuntimeError):
    """A negative rt_status from the library (message from rt_last_error)."""


class rt_vec4d(C.Structure):
    _fields_ = [("x", C.c_double), ("y", C.c_double), ("z", C.c_double), ("w", C.c_double)]


class rt_color(C.Structure):
    _fields_ = [("r", C.c_double), ("g", C.c_double), ("b", C.c_double)]


class rt_prim(C.Structure):
    _fields_ = [
        ("kind", C.c_int32), ("flags", C.c_int32),
        ("p", rt_vec4d * 3), ("n", rt_vec4d * 3),
        ("radius", C.c_double),
        ("to_obj", C.c_double * 16), ("to_world", C.c_double * 16), ("to_normal", C.c_double * 16),
        ("emission", rt_color), ("diffuse", rt_color), ("specular", rt_color), ("refraction", rt_color),
        ("shininess", C.c_double), ("refractive_index", C.c_double),
    ]


class rt_camera(C.Structure):
    _fields_ = [
        ("kind", C.c_int32), ("reserved", C.c_int32),
        ("position", rt_vec4d), ("look_at", rt_vec4d), ("up", rt_vec4d),
        ("fov_y", C.c_double), ("size_mult", C.c_double),
        ("image_plane", C.c_double), ("dof_amount", C.c_double), ("focal_length", C.c_double),
    ]


class rt_scene_params(C.Structure):
    _fields_ = [
        ("width", C.c_int32), ("height", C.c_int32), ("recursion", C.c_int32), ("debug_geom", C.c_int32),
        ("air_ior", C.c_double), ("ambient", rt_color),
    ]


class rt_scene_info(C.Structure):
    _fields_ = [
        ("n_prims", C.c_int32), ("ref_bvh_nodes", C.c_int32), ("ref_bvh_depth", C.c_int32),
        ("sah_bvh_nodes", C.c_int32), ("sah_bvh_depth", C.c_int32), ("traversal", C.c_int32),
        ("device", C.c_int32), ("bvh_builder", C.c_int32), ("device_bytes", C.c_uint64),
    ]


_lib: Optional[C.CDLL] = None


def load_library(path: str = "") -> C.CDLL:
    """Load librtcore_hip.so (built by __graft_entry__.build()).  Raises if it is missing.

    RTCORE_LIB may name an alternative build of the same library (e.g. a tuning variant).
    """
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("RTCORE_LIB", "") or LIB_PATH
    if not os.path.exists(path):
        raise RtError(f"{path} is missing: run __graft_entry__.build() (make -C raytracercore_amd/csrc)")
    # torch-ROCm wheels carry their own HIP runtime; when torch is present it must be loaded
    # first so that this library binds to the same runtime instance (one HIP runtime per process)
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    P = C.POINTER
    sig = {
        "rt_abi_version": (C.c_int, []),
        "rt_build_info": (C.c_char_p, []),
        "rt_device_count": (C.c_int, []),
        "rt_last_error": (C.c_int, [C.c_char_p, C.c_int32]),
        "rt_scene_create": (C.c_int, [P(rt_scene_params), P(rt_prim), C.c_int32, C.c_int32, P(C.c_void_p)]),
        "rt_scene_set_camera": (C.c_int, [C.c_void_p, P(rt_camera)]),
        "rt_scene_set_traversal": (C.c_int, [C.c_void_p, C.c_int32]),
        "rt_scene_get_info": (C.c_int, [C.c_void_p, P(rt_scene_info)]),
        "rt_scene_destroy": (None, [C.c_void_p]),
        "rt_set_bvh_builder": (C.c_int, [C.c_int32]),
        "rt_scene_get_build_stats": (C.c_int, [C.c_void_p, P(C.c_double), C.c_int32]),
        "rt_scene_check_bvh": (C.c_int, [C.c_void_p]),
        "rt_set_jit": (C.c_int, [C.c_int32]),
        "rt_scene_get_jit_error": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int32]),
        "rt_debug_jit_compile": (C.c_int, [C.c_char_p, C.c_int32, C.c_char_p, C.c_int32]),
        "rt_debug_jit_header": (C.c_int, [P(rt_scene_params), P(rt_prim), C.c_int32, P(rt_camera), C.c_int32,
                                          C.c_char_p, C.c_int64]),
        "rt_render_tile": (C.c_int, [C.c_void_p] + [C.c_int32] * 5 + [C.c_uint64, C.c_uint64,
                                     P(rt_color), P(C.c_uint32), P(C.c_uint32), P(C.c_uint64)]),
        "rt_render_tile_1spp": (C.c_int, [C.c_void_p] + [C.c_int32] * 4 + [C.c_uint64, C.c_uint64, P(rt_color)]),
        "rt_primary_ids": (C.c_int, [C.c_void_p] + [C.c_int32] * 4 + [P(C.c_int32)]),
        "rt_bvh_counts": (C.c_int, [C.c_void_p] + [C.c_int32] * 4 + [P(C.c_int32)]),
        "rt_render_device": (C.c_int, [C.c_void_p] + [C.c_int32] * 5 + [C.c_uint64, C.c_uint64] +
                             [C.c_void_p] * 4 + [C.c_void_p]),
        "rt_primary_ids_device": (C.c_int, [C.c_void_p] + [C.c_int32] * 4 + [C.c_void_p, C.c_void_p]),
        "rt_last_kernel_ms": (C.c_int, [C.c_void_p, P(C.c_float)]),
        "rt_kernel_times": (C.c_int, [C.c_void_p, C.c_int32, P(C.c_float)]),
        "rt_scene_set_stats": (C.c_int, [C.c_void_p, C.c_int32]),
        "rt_scene_get_stats": (C.c_int, [C.c_void_p, P(C.c_uint64), C.c_int32]),
        "rt_render_frame_multi": (C.c_int, [P(rt_scene_params), P(rt_prim), C.c_int32, P(rt_camera), C.c_int32,
                                            C.c_int32, C.c_uint64, C.c_uint64, P(rt_color), P(C.c_uint32),
                                            P(C.c_uint32), P(C.c_uint64)]),
        "rt_render_bands": (C.c_int, [C.c_void_p] + [C.c_int32] * 4 + [C.c_uint64, C.c_uint64, P(rt_color),
                                      P(C.c_uint32), P(C.c_uint32), P(C.c_uint64)]),
        "rt_render_bands_device": (C.c_int, [C.c_void_p] + [C.c_int32] * 4 + [C.c_uint64, C.c_uint64] +
                                   [C.c_void_p] * 3 + [C.c_uint64, C.c_void_p, C.c_void_p]),
        "rt_band_rows": (C.c_int, [C.c_int32] * 4),
        "rt_band_slot_rows": (C.c_int, [C.c_int32] * 3),
        "rt_scatter_band_slot": (C.c_int, [C.c_void_p, C.c_uint64] + [C.c_int32] * 5 + [P(rt_color), P(C.c_uint32),
                                                                                       P(C.c_uint32)]),
        "rt_frame_create": (C.c_int, [P(rt_scene_params), P(rt_prim), C.c_int32, P(rt_camera), C.c_int32,
                                      P(C.c_void_p)]),
        "rt_frame_set_camera": (C.c_int, [C.c_void_p, P(rt_camera)]),
        "rt_frame_render": (C.c_int, [C.c_void_p, C.c_int32, C.c_uint64, C.c_uint64, P(rt_color), P(C.c_uint32),
                                      P(C.c_uint32), P(C.c_uint64)]),
        "rt_frame_submit": (C.c_int, [C.c_void_p, C.c_int32, C.c_uint64, C.c_uint64]),
        "rt_frame_collect": (C.c_int, [C.c_void_p, P(rt_color), P(C.c_uint32), P(C.c_uint32), P(C.c_uint64)]),
        "rt_frame_inject_fault": (C.c_int, [C.c_void_p, C.c_int32]),
        "rt_frame_destroy": (None, [C.c_void_p]),
        "rt_parse_scene": (C.c_int, [C.c_char_p, P(rt_scene_params), P(rt_prim), P(C.c_int32), P(rt_camera),
                                     P(C.c_int32)]),
        "rt_sample_output": (C.c_int32, [rt_color, C.c_uint32, C.c_uint32, rt_color, C.c_double, C.c_double]),
        "rt_tonemap_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, rt_color, C.c_double,
                                        C.c_double, C.c_void_p, C.c_void_p]),
        "rt_ref_bvh_export": (C.c_int, [P(rt_prim), C.c_int32, P(C.c_int32), P(C.c_double), P(C.c_int32),
                                        P(C.c_int32)]),
        "rt_debug_ray_log": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p]),
        "rt_debug_vn_rehit": (C.c_int, [P(C.c_double), P(C.c_double), P(C.c_double), C.c_int32, C.c_double,
                                        C.c_double, P(C.c_float), P(C.c_int32), P(C.c_double), P(C.c_double)]),
        "rt_debug_trace_rays": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_int32, C.c_void_p,
                                          C.c_void_p, P(C.c_float)]),
    }
    for name, (res, args) in sig.items():
        if name.startswith("rt_debug_") and not hasattr(lib, name):
            continue  # an older build (RTCORE_LIB, A/B measurements) without a newer debug entry point
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.rt_abi_version() != ABI_VERSION:
        raise RtError(f"{path}: ABI version {lib.rt_abi_version()}, this module binds {ABI_VERSION} (rebuild)")
    _lib = lib
    return lib


def _check(rc: int) -> None:
    if rc != RT_OK:
        buf = C.create_string_buffer(1024)
        _lib.rt_last_error(buf, 1024)
        raise RtError(f"rtcore error {rc}: {buf.value.decode(errors='replace')}")


@dataclass
class ParsedScene:
    """SceneLoader.FromFile output in ABI form (Scene.cs fields + Primitives + Cameras)."""
    params: rt_scene_params
    prims: "C.Array[rt_prim]"
    cameras: "C.Array[rt_camera]"

    @property
    def n_prims(self) -> int:
        return len(self.prims)


class SceneLoader:
    """Mirror of RaytracerCore.SceneLoader (SceneLoader.cs:28-440) over rt_parse_scene."""

    @staticmethod
    def from_text(text: str) -> ParsedScene:
        lib = load_library()
        n_p, n_c = C.c_int32(0), C.c_int32(0)
        params = rt_scene_params()
        _check(lib.rt_parse_scene(text.encode(), C.byref(params), None, C.byref(n_p), None, C.byref(n_c)))
        prims = (rt_prim * max(1, n_p.value))()
        cams = (rt_camera * max(1, n_c.value))()
        _check(lib.rt_parse_scene(text.encode(), C.byref(params), prims, C.byref(n_p), cams, C.byref(n_c)))
        return ParsedScene(params, (rt_prim * n_p.value).from_buffer(prims), (rt_camera * n_c.value).from_buffer(cams))

    @staticmethod
    def from_file(path: str) -> ParsedScene:
        with open(path, "r", encoding="utf-8") as f:
            return SceneLoader.from_text(f.read())


LAYOUT_NAMES = ("rects", "boxes", "frames", "frame_boxes", "frame_rects", "tris", "spheres", "planes",
                "groups", "grouped_slots")


def jit_header(scene: "SceneLoader", camera: int = 0, size: Optional[Tuple[int, int]] = None,
               grouped: bool = False) -> str:
    """rt_debug_jit_header (host code, no GPU): the generated header of the scene-specialised build
    for this scene and camera (tools/jit_isa.py compiles it and writes the listing)."""
    lib = load_library()
    params = rt_scene_params.from_buffer_copy(scene.params)
    if size:
        params.width, params.height = size
    n = len(scene.prims)
    arr = (rt_prim * max(1, n))(*scene.prims)
    cam = rt_camera.from_buffer_copy(scene.cameras[camera])
    k = lib.rt_debug_jit_header(C.byref(params), arr, n, C.byref(cam), 1 if grouped else 0, None, 0)
    if k < 0:
        _check(k)
    buf = C.create_string_buffer(k + 1)
    k2 = lib.rt_debug_jit_header(C.byref(params), arr, n, C.byref(cam), 1 if grouped else 0, buf, k + 1)
    if k2 < 0:
        _check(k2)
    return buf.value.decode()


def brute_layout(prims: Sequence[rt_prim]) -> dict:
    """rt_debug_brute_layout (host code, no GPU): how the brute-force kernels would test these
    primitives -- world rectangles, boxes, frames, triangles, spheres, planes, and the grouping."""
    lib = load_library()
    n = len(prims)
    arr = (rt_prim * max(1, n))(*prims)
    out = (C.c_int32 * len(LAYOUT_NAMES))()
    _check(lib.rt_debug_brute_layout(arr, n, out, len(LAYOUT_NAMES)))
    return dict(zip(LAYOUT_NAMES, (int(v) for v in out)))


def ref_bvh_export(prims: Sequence[rt_prim]) -> Tuple[np.ndarray, np.ndarray, int, int]:
    """The library's reference-BVH build (host code, no GPU): (leaf prim order, node boxes, nodes, depth)."""
    lib = load_library()
    n = len(prims)
    arr = (rt_prim * max(1, n))(*prims)
    order = np.zeros(max(1, n), np.int32)
    boxes = np.zeros((max(1, 2 * n), 8), np.float64)
    nodes, depth = C.c_int32(0), C.c_int32(0)
    _check(lib.rt_ref_bvh_export(arr, n, order.ctypes.data_as(C.POINTER(C.c_int32)),
                                 boxes.ctypes.data_as(C.POINTER(C.c_double)), C.byref(nodes), C.byref(depth)))
    return order[:n], boxes[:nodes.value], nodes.value, depth.value


def sample_output(sum_rgb: Tuple[float, float, float], samples: int, misses: int,
                  background=(0.0, 0.0, 0.0), background_alpha: float = 0.0, exposure: float = 1.0) -> int:
    """SampleSet.GetOutput (SampleSet.cs:61-113): ARGB int32."""
    lib = load_library()
    return lib.rt_sample_output(rt_color(*sum_rgb), samples, misses, rt_color(*background), background_alpha, exposure)


def device_count() -> int:
    return load_library().rt_device_count()


class GpuRaytracer:
    """One device scene: the drop-in for a `Raytracer` worker (Raytracer.cs:12-49, 294-330).

    Tile buffers follow the C# DoubleColor[w, h] order: element (x, y) at x*h + y.
    """

    def __init__(self, scene: ParsedScene, camera_index: int = 0, device: int = 0,
                 size: Optional[Tuple[int, int]] = None, traversal: int = RT_TRAVERSAL_AUTO,
                 builder: Optional[int] = None):
        lib = load_library()
        self.lib = lib
        self.params = rt_scene_params.from_buffer_copy(scene.params)
        if size is not None:
            self.params.width, self.params.height = int(size[0]), int(size[1])
        self.width, self.height = self.params.width, self.params.height
        self.handle = C.c_void_p()
        n = scene.n_prims
        prims = scene.prims if isinstance(scene.prims, C.Array) and n > 0 else (rt_prim * max(1, n))(*scene.prims)
        if builder is not None:  # process-wide in the library: set for this create only
            _check(lib.rt_set_bvh_builder(builder))
        try:
            _check(lib.rt_scene_create(C.byref(self.params), prims, n, device, C.byref(self.handle)))
        finally:
            if builder is not None:
                lib.rt_set_bvh_builder(RT_BVH_BUILDER_AUTO)
        self.device = device
        if len(scene.cameras) == 0:
            raise RtError("scene has no camera")
        self.camera = rt_camera.from_buffer_copy(scene.cameras[camera_index])
        _check(lib.rt_scene_set_camera(self.handle, C.byref(self.camera)))
        if traversal != RT_TRAVERSAL_AUTO:
            self.set_traversal(traversal)

    def close(self) -> None:
        if self.handle:
            self.lib.rt_scene_destroy(self.handle)
            self.handle = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_traversal(self, traversal: int) -> None:
        _check(self.lib.rt_scene_set_traversal(self.handle, traversal))

    def info(self) -> rt_scene_info:
        inf = rt_scene_info()
        _check(self.lib.rt_scene_get_info(self.handle, C.byref(inf)))
        return inf

    def check_bvh(self) -> None:
        """rt_scene_check_bvh: structural validation of the device BVHs (raises RtError)."""
        _check(self.lib.rt_scene_check_bvh(self.handle))

    def jit_error(self) -> str:
        """rt_scene_get_jit_error: why the last scene-specialised build failed ("" if it did not)."""
        buf = C.create_string_buffer(4096)
        self.lib.rt_scene_get_jit_error(self.handle, buf, len(buf))
        return buf.value.decode(errors="replace")

    def build_stats(self) -> dict:
        """rt_scene_get_build_stats: scene-creation timings and the BVH builder's figures."""
        out = (C.c_double * len(BUILD_STAT_NAMES))()
        _check(self.lib.rt_scene_get_build_stats(self.handle, out, len(BUILD_STAT_NAMES)))
        return dict(zip(BUILD_STAT_NAMES, (float(v) for v in out)))

    def primary_ids(self, x0: int = 0, y0: int = 0, w: Optional[int] = None, h: Optional[int] = None) -> np.ndarray:
        """DebugRaycaster Primitives-mode IDs as an int32 array indexed [x, y]."""
        w = self.width - x0 if w is None else w
        h = self.height - y0 if h is None else h
        ids = np.empty((w, h), np.int32)
        _check(self.lib.rt_primary_ids(self.handle, x0, y0, w, h, ids.ctypes.data_as(C.POINTER(C.c_int32))))
        return ids

    def bvh_counts(self, x0: int = 0, y0: int = 0, w: Optional[int] = None, h: Optional[int] = None) -> np.ndarray:
        """DebugRaycaster BoundingVolumes mode: reference-BVH node counts as int32 [x, y]."""
        w = self.width - x0 if w is None else w
        h = self.height - y0 if h is None else h
        out = np.empty((w, h), np.int32)
        _check(self.lib.rt_bvh_counts(self.handle, x0, y0, w, h, out.ctypes.data_as(C.POINTER(C.c_int32))))
        return out

    def render_tile(self, x0: int, y0: int, w: int, h: int, spp: int, seed: int = 0, sample_base: int = 0, out=None):
        """Accumulators (sum[w,h,3] f64, samples[w,h] u32, misses[w,h] u32, rays): new zeroed arrays, or
        the caller's `out` = (sum, samples, misses), which the call adds into (SampleSet's merge)."""
        if out is None:
            out = (np.zeros((w, h, 3), np.float64), np.zeros((w, h), np.uint32), np.zeros((w, h), np.uint32))
        s, n, m = out
        for a, shape, dt in ((s, (w, h, 3), np.float64), (n, (w, h), np.uint32), (m, (w, h), np.uint32)):
            if a.shape != shape or a.dtype != dt or not a.flags.c_contiguous:
                raise ValueError("out must be C-contiguous (sum f64 [w, h, 3], samples u32 [w, h], misses u32 [w, h])")
        rays = C.c_uint64(0)
        _check(self.lib.rt_render_tile(self.handle, x0, y0, w, h, spp, seed, sample_base,
                                       s.ctypes.data_as(C.POINTER(rt_color)),
                                       n.ctypes.data_as(C.POINTER(C.c_uint32)),
                                       m.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(rays)))
        return s, n, m, rays.value

    def render_bands(self, band: int, band_stride: int, band_offset: int, spp: int, seed: int = 0,
                     sample_base: int = 0, out=None):
        """rt_render_bands: one band set of the frame added into whole-frame accumulators
        (sum[W,H,3] f64, samples[W,H] u32, misses[W,H] u32; new zeroed arrays unless `out`), plus rays."""
        W, H = self.width, self.height
        if out is None:
            out = (np.zeros((W, H, 3), np.float64), np.zeros((W, H), np.uint32), np.zeros((W, H), np.uint32))
        s, n, m = out
        rays = C.c_uint64(0)
        _check(self.lib.rt_render_bands(self.handle, band, band_stride, band_offset, spp, seed, sample_base,
                                        s.ctypes.data_as(C.POINTER(rt_color)), n.ctypes.data_as(C.POINTER(C.c_uint32)),
                                        m.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(rays)))
        return s, n, m, rays.value

    def render_bands_device(self, band, band_stride, band_offset, spp, seed, sample_base, d_sum, d_samples, d_misses,
                            plane, d_rays, stream: int = 0) -> None:
        """rt_render_bands_device: asynchronous band-set render into device accumulators (pointers)."""
        _check(self.lib.rt_render_bands_device(self.handle, band, band_stride, band_offset, spp, seed, sample_base,
                                               C.c_void_p(d_sum), C.c_void_p(d_samples), C.c_void_p(d_misses), plane,
                                               C.c_void_p(d_rays), C.c_void_p(stream)))

    def render_tile_1spp(self, x0: int, y0: int, w: int, h: int, seed: int = 0, sample_index: int = 0,
                         out: Optional[np.ndarray] = None) -> np.ndarray:
        """Raytracer.Render one pass: DoubleColor[w, h] with Placeholder (-1) for misses (into `out`,
        a C-contiguous float64 [w, h, 3] array, when given)."""
        if out is None:
            out = np.empty((w, h, 3), np.float64)
        elif out.shape != (w, h, 3) or out.dtype != np.float64 or not out.flags.c_contiguous:
            raise ValueError("out must be a C-contiguous float64 array of shape (w, h, 3)")
        _check(self.lib.rt_render_tile_1spp(self.handle, x0, y0, w, h, seed, sample_index,
                                            out.ctypes.data_as(C.POINTER(rt_color))))
        return out

    def render_device(self, x0, y0, w, h, spp, seed, sample_base, d_sum, d_samples, d_misses, d_rays,
                      stream: int = 0) -> None:
        """Asynchronous device-resident render; d_* are device pointers (e.g. torch data_ptr())."""
        _check(self.lib.rt_render_device(self.handle, x0, y0, w, h, spp, seed, sample_base,
                                         C.c_void_p(d_sum), C.c_void_p(d_samples), C.c_void_p(d_misses),
                                         C.c_void_p(d_rays), C.c_void_p(stream)))

    def last_kernel_ms(self) -> float:
        ms = C.c_float(0)
        _check(self.lib.rt_last_kernel_ms(self.handle, C.byref(ms)))
        return float(ms.value)

    KERNEL_TIME_RING = 64

    def kernel_times(self, n: int) -> List[float]:
        """rt_kernel_times: durations (ms) of the last n path kernels on this scene, oldest first
        (n <= 64): launches queued without a host sync, timed afterwards."""
        out = (C.c_float * max(n, 1))()
        _check(self.lib.rt_kernel_times(self.handle, n, out))
        return [float(v) for v in out[:n]]

    STAT_NAMES = ("node_visits", "tri_tests", "sph_tests", "cyc_start", "cyc_trace", "cyc_shade", "wave_iters",
                  "max_query_steps", "stack_overflow_pushes", "max_stack_depth", "outer_tests")

    def set_stats(self, enable: bool) -> None:
        """rt_scene_set_stats: run the instrumented kernel variant (profiling only)."""
        _check(self.lib.rt_scene_set_stats(self.handle, 1 if enable else 0))

    def get_stats(self) -> dict:
        """rt_scene_get_stats: counters accumulated since the last read (then zeroed)."""
        out = (C.c_uint64 * len(self.STAT_NAMES))()
        _check(self.lib.rt_scene_get_stats(self.handle, out, len(self.STAT_NAMES)))
        return dict(zip(self.STAT_NAMES, (int(v) for v in out)))


def tonemap_device(d_sum: int, d_samples: int, d_misses: int, w: int, h: int, d_argb: int,
                   background=(0.0, 0.0, 0.0), background_alpha: float = 0.0, exposure: float = 1.0,
                   stream: int = 0) -> None:
    """rt_tonemap_device: SampleSet.GetOutput for every pixel of device accumulators (pointers)."""
    _check(load_library().rt_tonemap_device(d_sum, d_samples, d_misses, w, h, rt_color(*background),
                                            background_alpha, exposure, d_argb, stream))


def _frame_inputs(scene: ParsedScene, camera_index: int, size: Optional[Tuple[int, int]]):
    params = rt_scene_params.from_buffer_copy(scene.params)
    if size is not None:
        params.width, params.height = size
    prims = (rt_prim * max(1, scene.n_prims))(*scene.prims)
    cam = rt_camera.from_buffer_copy(scene.cameras[camera_index])
    return params, prims, cam


class GpuFrame:
    """rt_frame: persistent whole-frame renderer over devices 0..n_gpus-1 of this process (row-band
    split, one RCCL gather to device 0 per render).  Replaces FullRaytracer's worker pool
    (FullRaytracer.cs:297-302) on a multi-GPU host; accumulators in the [x, y] order of SampleSet[w, h]."""

    def __init__(self, scene: ParsedScene, camera_index: int = 0, n_gpus: int = 1,
                 size: Optional[Tuple[int, int]] = None):
        self.lib = load_library()
        params, prims, cam = _frame_inputs(scene, camera_index, size)
        self.width, self.height = params.width, params.height
        self.handle = C.c_void_p()
        _check(self.lib.rt_frame_create(C.byref(params), prims, scene.n_prims, C.byref(cam), n_gpus,
                                        C.byref(self.handle)))

    def set_camera(self, camera: rt_camera) -> None:
        _check(self.lib.rt_frame_set_camera(self.handle, C.byref(camera)))

    def render(self, spp: int, seed: int = 0, sample_base: int = 0, out=None):
        """Adds spp samples of every pixel into (sum[W,H,3], samples[W,H], misses[W,H]) (new if out is None)."""
        W, H = self.width, self.height
        if out is None:
            out = (np.zeros((W, H, 3), np.float64), np.zeros((W, H), np.uint32), np.zeros((W, H), np.uint32))
        s, n, m = self._check_out(out)
        rays = C.c_uint64(0)
        _check(self.lib.rt_frame_render(self.handle, spp, seed, sample_base, s.ctypes.data_as(C.POINTER(rt_color)),
                                        n.ctypes.data_as(C.POINTER(C.c_uint32)),
                                        m.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(rays)))
        return s, n, m, rays.value

    def submit(self, spp: int, seed: int = 0, sample_base: int = 0) -> None:
        """rt_frame_submit: queue a render (band sets, gather, host copy) and return at once."""
        _check(self.lib.rt_frame_submit(self.handle, spp, seed, sample_base))

    def collect(self, out):
        """rt_frame_collect: wait for the oldest submitted render and add it into out = (sum[W,H,3],
        samples[W,H], misses[W,H]); returns (sum, samples, misses, rays)."""
        s, n, m = self._check_out(out)
        rays = C.c_uint64(0)
        _check(self.lib.rt_frame_collect(self.handle, s.ctypes.data_as(C.POINTER(rt_color)),
                                         n.ctypes.data_as(C.POINTER(C.c_uint32)),
                                         m.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(rays)))
        return s, n, m, rays.value

    def inject_fault(self, point: int) -> None:
        """rt_frame_inject_fault (test hook): 1 = the next gather fails inside its RCCL group."""
        _check(self.lib.rt_frame_inject_fault(self.handle, point))

    def _check_out(self, out):
        W, H = self.width, self.height
        s, n, m = out
        for a, dt, shape in ((s, np.float64, (W, H, 3)), (n, np.uint32, (W, H)), (m, np.uint32, (W, H))):
            if not (isinstance(a, np.ndarray) and a.dtype == dt and a.shape == shape and a.flags.c_contiguous):
                raise ValueError(f"GpuFrame: outputs must be C-contiguous {np.dtype(dt).name}{shape} arrays")
        return s, n, m

    def close(self) -> None:
        if self.handle:
            self.lib.rt_frame_destroy(self.handle)
            self.handle = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def band_rows_count(height: int, band: int, band_stride: int, band_offset: int) -> int:
    """rt_band_rows: rows of band set (band, band_stride, band_offset) of a frame (host only)."""
    n = load_library().rt_band_rows(height, band, band_stride, band_offset)
    _check(min(n, 0))
    return n


def band_slot_rows(height: int, band: int, band_stride: int) -> int:
    """rt_band_slot_rows: rows of the tallest band set of the split (host only)."""
    n = load_library().rt_band_slot_rows(height, band, band_stride)
    _check(min(n, 0))
    return n


def scatter_band_slot(slot: np.ndarray, plane: int, width: int, height: int, band: int, band_stride: int,
                      band_offset: int, out) -> None:
    """rt_scatter_band_slot (host only): rt_frame_render's merge of one device's gathered slot (a
    float64 array of 4 * plane: sum planes, then the samples / misses u32 planes) into
    (sum[W,H,3], samples[W,H], misses[W,H])."""
    s, n, m = out
    slot = np.ascontiguousarray(slot, dtype=np.float64)
    # the C side writes through raw pointers: refuse anything but the exact layouts it assumes
    for a, dt, shape in ((s, np.float64, (width, height, 3)), (n, np.uint32, (width, height)),
                         (m, np.uint32, (width, height))):
        if not (isinstance(a, np.ndarray) and a.dtype == dt and a.shape == shape and a.flags.c_contiguous
                and a.flags.writeable):
            raise ValueError(f"scatter_band_slot: outputs must be writeable C-contiguous {np.dtype(dt).name}"
                             f"{shape} arrays")
    if plane < 0 or slot.size < 4 * plane:
        raise ValueError(f"scatter_band_slot: slot holds {slot.size} float64, needs 4 * plane = {4 * plane}")
    _check(load_library().rt_scatter_band_slot(slot.ctypes.data_as(C.c_void_p), plane, width, height, band,
                                               band_stride, band_offset, s.ctypes.data_as(C.POINTER(rt_color)),
                                               n.ctypes.data_as(C.POINTER(C.c_uint32)),
                                               m.ctypes.data_as(C.POINTER(C.c_uint32))))


def render_frame_multi(scene: ParsedScene, camera_index: int, n_gpus: int, spp: int, seed: int = 0,
                       size: Optional[Tuple[int, int]] = None, sample_base: int = 0):
    """rt_render_frame_multi: row-interleaved bands on n_gpus devices + RCCL gather (one shot)."""
    lib = load_library()
    params, prims, cam = _frame_inputs(scene, camera_index, size)
    W, H = params.width, params.height
    s = np.zeros((W, H, 3), np.float64)
    n = np.zeros((W, H), np.uint32)
    m = np.zeros((W, H), np.uint32)
    rays = C.c_uint64(0)
    _check(lib.rt_render_frame_multi(C.byref(params), prims, scene.n_prims, C.byref(cam), n_gpus, spp, seed,
                                     sample_base, s.ctypes.data_as(C.POINTER(rt_color)),
                                     n.ctypes.data_as(C.POINTER(C.c_uint32)), m.ctypes.data_as(C.POINTER(C.c_uint32)),
                                     C.byref(rays)))
    return s, n, m, rays.value


def scene_path(name: str) -> str:
    """Path of a scene fixture shipped in tests/golden/scenes (bounce.txt, die.txt, ...)."""
    return os.path.join(REPO_ROOT, "tests", "golden", "scenes", name)
