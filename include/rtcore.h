/*
 * rtcore.h -- C ABI of the MI355X (gfx950) path-tracing core: the drop-in for
 * RaytracerCore's render worker.
 *
 * Reference seam (all paths relative to the reference repository):
 *   FullRaytracer constructs `Raytracer(this, Scene)` workers
 *   (RaytracerCore/Raytracing/FullRaytracer.cs:297-302).  Each worker loops
 *   GetWorkingTile() (FullRaytracer.cs:219-229) -> one sample per pixel of the tile
 *   into DoubleColor[tile.Width, tile.Height] with DoubleColor.Placeholder marking a
 *   primary miss (Raytracer.cs:294-330) -> OnTileFinished(tile, samples, elapsed)
 *   (FullRaytracer.cs:210-214).  The library replaces the body of that loop; the C#
 *   host keeps Scene / SceneLoader / Camera / SampleSet and calls this ABI through
 *   P/Invoke.
 *
 * Conventions
 *   - extern "C", cdecl, blittable structs only; every function returns RT_OK (0) or
 *     a negative rt_status; details via rt_last_error() (thread-local).
 *   - Host tile buffers use the C# rectangular-array order of DoubleColor[w, h]:
 *     element (x, y) of a w*h tile lives at offset x*h + y (y fastest),
 *     as in Raytracer.cs:305,317 and FullRaytracer.cs:328-339.
 *   - The library owns scene handles and device memory; callers own every output
 *     buffer and nothing is retained after a call returns.
 *   - A scene handle is bound to one device and is not re-entrant: calls on one handle
 *     are serialised by the caller.  Device-side calls may be queued on any stream; the
 *     library orders an operation on a stream other than the previous one after it
 *     (the launches share per-scene scratch), and any number of launches may be queued
 *     without a synchronisation.
 */
#ifndef RTCORE_H
#define RTCORE_H

#ifndef __HIPCC_RTC__
#include <stdint.h>
#include <stddef.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define RTCORE_ABI_VERSION 5 /* 2: rt_frame_*, rt_render_bands, sample_base in rt_render_frame_multi;
                                3: rt_set_jit, rt_scene_get_jit_error, build stats [15..17];
                                4: rt_kernel_times;
                                5: rt_frame_submit / rt_frame_collect / rt_frame_inject_fault */

typedef enum rt_status {
    RT_OK = 0,
    RT_ERR_ARG = -1,      /* bad argument (null pointer, bad size, unknown kind)      */
    RT_ERR_HIP = -2,      /* a HIP runtime call failed                               */
    RT_ERR_OOM = -3,      /* device or host allocation failed                         */
    RT_ERR_NCCL = -4,     /* an RCCL call failed                                      */
    RT_ERR_PARSE = -5,    /* scene text could not be parsed (SceneLoader.cs:417-422) */
    RT_ERR_NODEVICE = -6, /* no HIP device available                                  */
    RT_ERR_STATE = -7     /* call out of order (e.g. render before a camera is set)   */
} rt_status;

/* Vec4D (RaytracerCore/Vectors/Vec4D.cs:16-91): 4 x fp64, 32 B, w=1 points, w=0 directions. */
typedef struct rt_vec4d { double x, y, z, w; } rt_vec4d;

/* DoubleColor (RaytracerCore/DoubleColor.cs:8-45): 3 x fp64, 24 B.  Placeholder = (-1,-1,-1). */
typedef struct rt_color { double r, g, b; } rt_color;

typedef enum rt_prim_kind {
    RT_PRIM_TRIANGLE = 0, /* Primitives/Triangle.cs */
    RT_PRIM_SPHERE = 1,   /* Primitives/Sphere.cs   */
    RT_PRIM_PLANE = 2     /* Primitives/Plane.cs    */
} rt_prim_kind;

typedef enum rt_prim_flags {
    RT_FLAG_MIRROR = 1,      /* Triangle.Mirror: parallelogram, u,v in [0,1]^2 (Triangle.cs:13-20)    */
    RT_FLAG_TWOSIDED = 2,    /* Primitive.TwoSided (Primitive.cs:78)                                   */
    RT_FLAG_INVERT = 4,      /* Primitive.Invert: flips Hit.Inside only (Primitive.cs:60-61)           */
    RT_FLAG_HASNORMALS = 8,  /* Triangle.HasNormals: per-vertex normals (Triangle.cs:45-52,209-219)   */
    RT_FLAG_TRANSFORMED = 16 /* Sphere.Transformed: ellipsoid via matrices (Sphere.cs:29-37)           */
} rt_prim_flags;

/*
 * One primitive as the C# Scene holds it after SceneLoader finalisation
 * (SceneLoader.cs:388-413), i.e. after Primitive.Transform.  Derived data
 * (triangle edges / face normal, bounding boxes, BVH) is computed by the library
 * with the reference's arithmetic.
 *   triangle: p[0..2] = Vert0..2.Position (world), n[0..2] = Vert0..2.Normal
 *   sphere:   p[0] = Center (object space), radius = Radius,
 *             to_obj = MatrixToObject, to_world = MatrixToWorld, to_normal = MatrixToNormal
 *             (row-major D00..D33; only read when RT_FLAG_TRANSFORMED is set)
 *   plane:    p[0] = Normal (unit, w=0), radius = OriginDistance
 * Materials are the raw backing fields; the library applies the Shininess<=0 gating of
 * the Specular / Refraction getters (Primitive.cs:111-129).
 */
typedef struct rt_prim {
    int32_t kind;
    int32_t flags;
    rt_vec4d p[3];
    rt_vec4d n[3];
    double radius;
    double to_obj[16];
    double to_world[16];
    double to_normal[16];
    rt_color emission, diffuse, specular, refraction;
    double shininess;
    double refractive_index;
} rt_prim;

typedef enum rt_camera_kind {
    RT_CAMERA_FRUSTUM = 0, /* Cameras/FrustumCamera.cs */
    RT_CAMERA_ORTHO = 1    /* Cameras/OrthoCamera.cs   */
} rt_camera_kind;

/*
 * The public fields of Camera (Cameras/Camera.cs:10-27) before InitRender.  The library
 * runs InitRender(width, height) itself (Camera.cs:54-63, FrustumCamera.cs:24-31,
 * OrthoCamera.cs:22-31) with the reference's arithmetic.
 */
typedef struct rt_camera {
    int32_t kind;
    int32_t reserved;
    rt_vec4d position, look_at, up;
    double fov_y;     /* FrustumCamera.fovY, radians                   */
    double size_mult; /* OrthoCamera.sizeMult                          */
    double image_plane, dof_amount, focal_length;
} rt_camera;

/* Scene-wide fields read on the hot path (Scene.cs:16-35). */
typedef struct rt_scene_params {
    int32_t width, height; /* Scene.Width / Height: the whole frame                        */
    int32_t recursion;     /* Scene.Recursion (default 3)                                  */
    int32_t debug_geom;    /* Scene.DebugGeom                                              */
    double air_ior;        /* Scene.AirRefractiveIndex (default 1.000293)                  */
    rt_color ambient;      /* Scene.AmbientRGB; (-1,-1,-1) = "ambient miss"                */
} rt_scene_params;

typedef struct rt_scene rt_scene; /* opaque */

/* Traversal strategy of the path-tracing kernel. */
typedef enum rt_traversal {
    RT_TRAVERSAL_AUTO = 0,  /* small scenes: brute force, grouped where a cost model
                               favours it; large scenes: the wide BVH                  */
    RT_TRAVERSAL_BRUTE = 1, /* every primitive, scene read through the scalar cache   */
    RT_TRAVERSAL_BVH = 2,   /* 4-wide quantised BVH (binned SAH, collapsed), LDS stack */
    RT_TRAVERSAL_BVH2 = 3,  /* the binary binned-SAH BVH it is collapsed from          */
    RT_TRAVERSAL_GROUPED = 4 /* brute force over groups of <= 8 primitives, a group
                                skipped when no ray of the wave meets its box          */
} rt_traversal;

typedef struct rt_scene_info {
    int32_t n_prims;
    int32_t ref_bvh_nodes;   /* nodes of the reference agglomerative BVH (BVH.cs:193-236); 0 until
                                the first exact debug pass builds it                         */
    int32_t ref_bvh_depth;
    int32_t sah_bvh_nodes;   /* nodes of the kernel's BVH2                                */
    int32_t sah_bvh_depth;
    int32_t traversal;       /* resolved rt_traversal of the path kernel                  */
    int32_t device;
    int32_t bvh_builder;     /* rt_bvh_builder that built the kernel's BVHs               */
    uint64_t device_bytes;   /* scene bytes resident in HBM                               */
} rt_scene_info;

/* Who builds the path kernel's BVH2 and its wide collapse at rt_scene_create. */
typedef enum rt_bvh_builder {
    RT_BVH_BUILDER_AUTO = 0, /* the GPU from 2^22 BVH primitives on, the host below
                                (RTCORE_BVH_BUILDER=host|gpu overrides AUTO)          */
    RT_BVH_BUILDER_HOST = 1, /* binned SAH on the host, collapsed to 4-wide            */
    RT_BVH_BUILDER_GPU = 2   /* PLOC on the device (Morton order, nearest-neighbour
                                merges by merged-box area), collapsed on the device   */
} rt_bvh_builder;

/* rt_scene_get_build_stats: [0] host preparation ms, [1] BVH build ms (wall, either
   builder), [2] upload ms, [3] GPU builder device ms, [4] PLOC rounds, [5] wide nodes,
   [6] wide-tree stack need; flat brute-force layout: [7] single world rectangles,
   [8] world boxes, [9] frames, [10] frame boxes, [11] rectangles tested one by one in
   frames, [12] other triangles, [13] spheres, [14] hot wide nodes staged in LDS;
   scene-specialised kernel of the last brute-force launch (rt_set_jit): [15] status (1 in use,
   0 not used, -1 build failed: see rt_scene_get_jit_error), [16] its hiprtc compile ms (0 when
   it came from the cache), [17] 1 if it came from the in-process or on-disk cache,
   [18] primitives per group of the grouped brute-force order (fixed at creation: 8 when the
   scene-specialised build was on then, else 4); [19] leaves of the wide tree, [20] of them compact
   (primitives of one kind and one set of test flags, read as 48-B records); [21] outer
   primitives: axis-aligned rectangles the BVH leaves out and tests as one group of rects and
   closed boxes when a query ends (host builder, scenes of more than 4096 BVH primitives) */
#define RT_BUILD_STATS_COUNT 22

/* ---------------------------------------------------------------- library ---- */
int rt_abi_version(void);
/* "src-sha256=<hex> extra=<flags>": the hash of the sources the library was built from and the
 * extra compiler flags of its build (raytracercore_amd/csrc/source_hash.py recomputes the hash). */
const char* rt_build_info(void);
int rt_device_count(void);
/* Copies the calling thread's last error message (NUL-terminated); returns its length. */
int rt_last_error(char* buf, int32_t cap);

/* ----------------------------------------------------------------- scenes ---- */
int rt_scene_create(const rt_scene_params* params, const rt_prim* prims, int32_t n_prims,
                    int32_t device, rt_scene** out_scene);
int rt_scene_set_camera(rt_scene* scene, const rt_camera* camera);
/* RT_ERR_ARG (the scene's mode unchanged) for a mode the scene cannot run: brute force over more
   than 65535 triangles or 32767 spheres, a BVH deeper than the kernel's traversal stack. */
int rt_scene_set_traversal(rt_scene* scene, int32_t traversal);
int rt_scene_get_info(const rt_scene* scene, rt_scene_info* info);
void rt_scene_destroy(rt_scene* scene);
/* Process-wide builder choice for later rt_scene_create calls (default AUTO). */
int rt_set_bvh_builder(int32_t builder);
/* Copies min(n, RT_BUILD_STATS_COUNT) build statistics of the scene (see above). */
int rt_scene_get_build_stats(const rt_scene* scene, double* out, int32_t n);
/* Scene-specialised brute-force kernels (no reference counterpart: an MI355X code-generation
   choice).  With on = 1 (the default; the environment variable RTCORE_JIT=0 makes the default
   0) the brute-force traversals of scenes of <= 48 primitives launch a build of the path kernel
   whose primitive records are compile-time constants, made with hiprtc on the first launch per
   scene (and per camera for the grouped order) and cached in-process and on disk
   (RTCORE_JIT_CACHE, else $HOME/.cache/rtcore_jit).  Same arithmetic and results as the generic
   kernel, which runs when on = 0 or a build fails.  Process-wide; applies to later launches. */
int rt_set_jit(int32_t on);
/* The reason the last scene-specialised build of this scene failed ("" if none). */
int rt_scene_get_jit_error(const rt_scene* scene, char* buf, int32_t cap);
/* Host only (no device needed): compiles the embedded kernel sources for `arch` (e.g. "gfx950")
   as a scene-specialised build of an empty scene; returns the code object size, or a negative
   rt_status with the compiler log in `log` (may be NULL). */
int rt_debug_jit_compile(const char* arch, int32_t grouped, char* log, int32_t cap);
/* Host only (no device needed): the generated header of the scene-specialised build that
   rt_scene_create + rt_scene_set_camera would make for these primitives and camera (grouped = 0
   flat order, 1 grouped order; brute-force scenes of <= 48 primitives), for reading its code
   without a GPU (tools/jit_isa.py).  Returns the header length; copies it NUL-terminated into buf
   when cap exceeds the length. */
int rt_debug_jit_header(const rt_scene_params* params, const rt_prim* prims, int32_t n_prims, const rt_camera* camera,
                        int32_t grouped, char* buf, int64_t cap);
/* Validation: checks the device-resident BVH2 and wide tree against the primitives (every
   child box contains the primitives below it, each primitive in exactly one leaf, depth and
   stack within what the kernels were sized for).  RT_ERR_STATE with the finding otherwise. */
int rt_scene_check_bvh(rt_scene* scene);
/* Host only (no device needed): the decomposition the brute-force kernels would test for these
   primitives -- out[0..9] = flat order: single world rectangles, world boxes (five or six faces of
   an axis-aligned box), frames (parallelograms along one affine frame's axes), frame boxes,
   rectangles tested one by one in frames, other triangles, spheres, planes; then the grouped
   order's group count and its slot count.  Copies min(n_out, 10) values. */
#define RT_LAYOUT_COUNT 10
int rt_debug_brute_layout(const rt_prim* prims, int32_t n_prims, int32_t* out, int32_t n_out);
/* Measurement of a wavefront split's traversal stage.  rt_debug_ray_log: while
   the next instrumented launch of a BVH kernel runs (rt_scene_set_stats; one launch only, then
   logging is off again), the kernel appends every finished query
   to d_log as 3 float4 (origin, previous primitive ID | direction, frame pixel index | closest t,
   hit slot, bounce) at the
   device counter *d_count, up to cap records (d_log = NULL turns logging off).
   rt_debug_trace_rays: the trace-only kernel (wide BVH, no shading) over n logged queries on
   `stream`, with waves_per_simd 6, 7 or 8; writes (t, slot) per query to d_hits, optional
   counters to d_stats[3] (node-step lane slots, leaf-step lane slots, lane slots in all) and the
   kernel's time (hipEvents) to *ms.  BVH traversal modes of a scene without planes only. */
int rt_debug_ray_log(rt_scene* scene, void* d_log, uint32_t cap, void* d_count);
/* Host only: the kernels' vertex-normal re-hit test -- Triangle.RayTraceAVXFaster in
   fp64 on the ray that leaves the triangle (v0, e01, e02) from its point fma(e01, u, fma(e02, v, v0))
   along dir (fp32, as the kernel holds it).  Returns 1 if that query meets the triangle again, 0 if
   not (negative rt_status on bad arguments); *inside = its Inside flag, *t its distance, origin[3]
   the start point used. */
int rt_debug_vn_rehit(const double* v0, const double* e01, const double* e02, int32_t mirror, double u, double v,
                      const float* dir, int32_t* inside, double* t, double* origin);
int rt_debug_trace_rays(rt_scene* scene, const void* d_rays, uint32_t n, void* d_hits, int32_t waves_per_simd,
                        void* d_stats, void* stream, float* ms);

/* ------------------------------------------------------- host-buffer renders --- */
/*
 * Accumulate spp samples (sample indices sample_base .. sample_base+spp-1) for every
 * pixel of the tile [x0, x0+w) x [y0, y0+h) into caller buffers laid out x*h + y:
 *   sum_rgb[i] += sum of non-miss sample colours   (SampleSet.AddSample, SampleSet.cs:32-36)
 *   samples[i] += non-miss samples, misses[i] += misses (SampleSet.AddMiss, :41-44)
 * rays_out (may be NULL) receives the number of Scene.RayTrace-equivalents (Mrays unit).
 */
int rt_render_tile(rt_scene* scene, int32_t x0, int32_t y0, int32_t w, int32_t h, int32_t spp,
                   uint64_t seed, uint64_t sample_base, rt_color* sum_rgb, uint32_t* samples,
                   uint32_t* misses, uint64_t* rays_out);

/*
 * Exactly Raytracer.Render's one-pass contract (Raytracer.cs:305-320): one sample per
 * pixel (index sample_index), written (not accumulated) to out[x*h + y];
 * primary misses are DoubleColor.Placeholder (-1,-1,-1).
 */
int rt_render_tile_1spp(rt_scene* scene, int32_t x0, int32_t y0, int32_t w, int32_t h,
                        uint64_t seed, uint64_t sample_index, rt_color* out);

/*
 * DebugRaycaster Primitives mode (DebugRaycaster.cs:193-199,241): integer-pixel primary
 * ray, no jitter / DOF, closest hit by the reference's BVH query in fp64
 * (Scene.cs:65-111).  ids_out[x*h + y] = Primitive.ID (insertion order) or -1 on a miss.
 */
int rt_primary_ids(rt_scene* scene, int32_t x0, int32_t y0, int32_t w, int32_t h, int32_t* ids_out);

/*
 * DebugRaycaster BoundingVolumes mode (DebugRaycaster.cs:200-212): for the same integer-pixel
 * primary rays, BVH<T>.GetIntersectionCount (BVH.cs:352-363) over the reference BVH in fp64 --
 * the number of nodes whose own box the ray meets (Volume.Intersect(ray).far >= 0), descending
 * only through those.  counts_out[x*h + y]; 0 where the root is missed.
 */
int rt_bvh_counts(rt_scene* scene, int32_t x0, int32_t y0, int32_t w, int32_t h, int32_t* counts_out);

/* -------------------------------------------------- device-resident renders --- */
/*
 * The same work as rt_render_tile on device buffers (framebuffer stays in HBM).
 * Device layout is row-major over the tile, i = y*w + x, with planar accumulators:
 *   d_sum    : 3 * w*h doubles, planes R | G | B
 *   d_samples, d_misses : w*h uint32
 *   d_rays   : one uint64 counter (added to)
 * `stream` is a hipStream_t (NULL = default stream).  Asynchronous: returns after launch.
 */
int rt_render_device(rt_scene* scene, int32_t x0, int32_t y0, int32_t w, int32_t h, int32_t spp,
                     uint64_t seed, uint64_t sample_base, double* d_sum, uint32_t* d_samples,
                     uint32_t* d_misses, unsigned long long* d_rays, void* stream);

/* Device-side DebugRaycaster Primitives pass: d_ids[y*w + x].  Asynchronous. */
int rt_primary_ids_device(rt_scene* scene, int32_t x0, int32_t y0, int32_t w, int32_t h,
                          int32_t* d_ids, void* stream);

/* Duration in ms of the last path-tracing kernel launched on this scene (hipEvent pair).
 * Waits for that kernel.  RT_ERR_ARG before the first launch. */
int rt_last_kernel_ms(rt_scene* scene, float* ms);

/* Durations in ms of the last n path-tracing kernels launched on this scene, oldest first
 * (1 <= n <= 64 and n <= the launches so far, else RT_ERR_ARG).  Each launch records its own
 * event pair in a ring of 64, so a caller can queue up to 64 launches without a host sync and
 * read their times afterwards.  Waits for those kernels. */
int rt_kernel_times(rt_scene* scene, int32_t n, float* ms);

/*
 * Instrumentation (profiling builds of the measurement, not the render): while enabled, the
 * path kernel's instrumented variant runs and adds up, over all launches since the last read,
 *   [0] BVH node visits  [1] triangle tests  [2] sphere tests           (per ray segment)
 *   [3] wave cycles in work fetch + camera ray  [4] in traversal  [5] in shading
 *   [6] wave loop iterations  [7] BVH kernels: the most traversal steps one query took (max)
 *   [8] wide BVH kernel: traversal-stack entries written past the LDS part (global overflow)
 *   [9] wide BVH kernel: the deepest traversal stack of any lane (max)
 *   [10] BVH kernels: faces of the outer records tested (rectangles and closed boxes' faces left
 *        out of the tree, build statistic [21]; wave-uniform records, not in [1])
 * rt_scene_get_stats synchronises the device, copies min(n, RT_STATS_COUNT) counters and zeroes them.
 */
#define RT_STATS_COUNT 11
int rt_scene_set_stats(rt_scene* scene, int32_t enable);
int rt_scene_get_stats(rt_scene* scene, uint64_t* out, int32_t n);

/* ------------------------------------------------------------- multi-GPU ---- */
/*
 * Row bands.  A band set (band, stride, offset) is the frame rows y with
 * (y / band) % stride == offset.  rt_frame deals the rows of a frame to n devices as the sets
 * (8, n, g), g = 0..n-1: interleaved bands balance background-heavy rows, where the
 * reference's contiguous tiles (FullRaytracer.cs:71-72) would not.
 *
 * rt_render_bands renders one band set on one scene and adds it into whole-frame buffers
 * (x*height + y order, every row outside the set untouched): the per-device step of
 * rt_frame_render, with the same device layout, callable on one device.
 */
int rt_render_bands(rt_scene* scene, int32_t band, int32_t band_stride, int32_t band_offset, int32_t spp,
                    uint64_t seed, uint64_t sample_base, rt_color* sum_rgb, uint32_t* samples,
                    uint32_t* misses, uint64_t* rays_out);

/*
 * Device-resident band-set render for hosts that run one process (or worker) per GPU: adds spp
 * samples of every pixel of the set into planar accumulators, row-major over the set's rows in
 * frame order: d_sum planes R | G | B each `plane` doubles apart, d_samples / d_misses `plane`
 * elements each (plane = 0: rows of the tallest set of the split x width, the gather-slot layout
 * of rt_frame).  Asynchronous on `stream`, like rt_render_device.
 */
int rt_render_bands_device(rt_scene* scene, int32_t band, int32_t band_stride, int32_t band_offset,
                           int32_t spp, uint64_t seed, uint64_t sample_base, double* d_sum,
                           uint32_t* d_samples, uint32_t* d_misses, uint64_t plane,
                           unsigned long long* d_rays, void* stream);
/* Rows of a frame of `height` rows in band set (band, band_stride, band_offset); host only. */
int rt_band_rows(int32_t height, int32_t band, int32_t band_stride, int32_t band_offset);
/* Rows of the tallest band set of the split (band, band_stride, *): a gather slot's plane is
 * this x width (host only). */
int rt_band_slot_rows(int32_t height, int32_t band, int32_t band_stride);
/* Host only: rt_frame_render's merge step for one device's gathered slot -- the slot (Σr | Σg | Σb
 * fp64 planes, then samples and misses u32 planes, each `plane` elements, row-major over the band
 * set's rows in frame order) added into frame buffers in the x*height + y order.  Exposed so that
 * the single-process frame path's band layout can be checked against a per-rank host's (the
 * torch.distributed split of bench.py, raytracercore_amd/sharding.py) without devices. */
int rt_scatter_band_slot(const void* slot, uint64_t plane, int32_t width, int32_t height, int32_t band,
                         int32_t band_stride, int32_t band_offset, rt_color* sum_rgb, uint32_t* samples,
                         uint32_t* misses);

/*
 * Persistent whole-frame renderer over devices 0..n_gpus-1 of this process (replaces the
 * FullRaytracer worker pool, FullRaytracer.cs:297-302, for a multi-GPU host): one scene per
 * device and one RCCL communicator, created once.  Each rt_frame_render call renders spp
 * samples (indices sample_base .. sample_base+spp-1) of every pixel: each device its band set,
 * then one RCCL gather over xGMI to device 0, and adds the result into the caller's frame
 * buffers (x*height + y; SampleSet semantics as rt_render_tile).  Progressive callers pass
 * disjoint sample_base ranges with the same seed.
 */
typedef struct rt_frame rt_frame; /* opaque */
int rt_frame_create(const rt_scene_params* params, const rt_prim* prims, int32_t n_prims,
                    const rt_camera* camera, int32_t n_gpus, rt_frame** out_frame);
int rt_frame_set_camera(rt_frame* frame, const rt_camera* camera);
int rt_frame_render(rt_frame* frame, int32_t spp, uint64_t seed, uint64_t sample_base,
                    rt_color* sum_rgb, uint32_t* samples, uint32_t* misses, uint64_t* rays_out);
/*
 * rt_frame_render in two phases, for a host that keeps the devices busy while it merges: submit
 * queues a render (every device's band set, the RCCL gather to device 0 and the copy of the
 * gathered slots into pinned host memory) and returns at once; collect waits for the oldest
 * submitted render and adds it into the caller's buffers (as rt_frame_render).  At most two
 * renders are in flight (RT_ERR_STATE otherwise), so submit(k+1) before collect(k) overlaps
 * render k+1 with the gather, copy and merge of render k -- FullRaytracer's update loop
 * (FullRaytracer.cs:326-344) merging finished passes while the workers render the next.  No
 * caller buffer is held between calls.  After an error every queued render is dropped.
 */
int rt_frame_submit(rt_frame* frame, int32_t spp, uint64_t seed, uint64_t sample_base);
int rt_frame_collect(rt_frame* frame, rt_color* sum_rgb, uint32_t* samples, uint32_t* misses,
                     uint64_t* rays_out);
/* Test hook: point 1 makes the next gather fail inside its RCCL group (the group is still closed). */
int rt_frame_inject_fault(rt_frame* frame, int32_t point);
void rt_frame_destroy(rt_frame* frame);

/* One-shot rt_frame_create + rt_frame_render + rt_frame_destroy. */
int rt_render_frame_multi(const rt_scene_params* params, const rt_prim* prims, int32_t n_prims,
                          const rt_camera* camera, int32_t n_gpus, int32_t spp, uint64_t seed,
                          uint64_t sample_base, rt_color* sum_rgb, uint32_t* samples, uint32_t* misses,
                          uint64_t* rays_out);

/* ------------------------------------------------------------- scene text ---- */
/*
 * SceneLoader.FromFile restatement (SceneLoader.cs:112-440): parses scene text into
 * primitives (insertion order = Primitive.ID), cameras and scene params.  Two-call
 * protocol: pass NULL arrays to query the counts, then call again with arrays of at
 * least that size.  Returns RT_ERR_PARSE with the line number in rt_last_error().
 */
int rt_parse_scene(const char* text, rt_scene_params* params, rt_prim* prims, int32_t* n_prims,
                   rt_camera* cameras, int32_t* n_cameras);

/*
 * Diagnostic, host only (no device needed): the reference agglomerative BVH the exact pass
 * uses (BVH.cs:193-236), flattened depth-first.  leaf_order[n] receives primitive indices in
 * depth-first leaf order; boxes (may be NULL, room for 2n-1 nodes) receives 8 doubles per node
 * (min xyzw, max xyzw) in pre-order.
 */
int rt_ref_bvh_export(const rt_prim* prims, int32_t n_prims, int32_t* leaf_order, double* boxes,
                      int32_t* n_nodes, int32_t* depth);

/*
 * SampleSet.GetOutput (SampleSet.cs:61-113) on the device, for every pixel of accumulators in
 * rt_render_device's layout (row-major w*h, d_sum planes R | G | B): d_argb[y*w + x] receives the
 * Color.ToArgb code the UI bitmap stores.  Uses the calling thread's current device.  Asynchronous.
 */
int rt_tonemap_device(const double* d_sum, const uint32_t* d_samples, const uint32_t* d_misses, int32_t w, int32_t h,
                      rt_color background, double background_alpha, double exposure, int32_t* d_argb, void* stream);

/* SampleSet.GetOutput (SampleSet.cs:61-113): tonemap accumulators to ARGB. */
int32_t rt_sample_output(rt_color sum, uint32_t samples, uint32_t misses, rt_color background,
                         double background_alpha, double exposure);

#ifdef __cplusplus
}
#endif

#endif /* RTCORE_H */
