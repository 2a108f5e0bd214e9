/*
 * oracle.h -- C API of the CPU oracle (TEST INFRASTRUCTURE ONLY).
 *
 * The oracle is a plain C++17 fp64 restatement of RaytracerCore's hot path
 * (SURVEY.md §8(c)), following the AVX2+FMA code paths the reference takes on hosts
 * with SIMDHelpers.Enabled (RaytracerCore/Vectors/SIMDHelpers.cs:15).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only as the
 * checker -- never as the thing measured or shipped.
 *
 * Parity status: the reference is C# / WinForms (netcoreapp3.1) and cannot be built or
 * run in this image, and it ships no tests, fixtures or golden vectors.  The oracle is
 * therefore pinned only by (a) analytic known-answer tests and (b) a statistical check
 * against the reference's own rendered screenshots (Screenshots/die.png,
 * Screenshots/bounce-with-lens.png); RNG and libm are "parity unpinned" (the reference
 * RNG is unseeded, Raytracer.cs:48).  See DESIGN.md §Oracle.
 */
#ifndef RTCORE_ORACLE_H
#define RTCORE_ORACLE_H

#include "../include/rtcore.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_scene orc_scene;

/* SceneLoader.FromFile restatement (SceneLoader.cs:112-440).  NULL on error (message in err). */
orc_scene* orc_load_text(const char* text, char* err, int32_t errcap);
/* Build from the ABI structs the GPU library consumes ("same inputs"). */
orc_scene* orc_from_prims(const rt_scene_params* params, const rt_prim* prims, int32_t n,
                          const rt_camera* cameras, int32_t n_cameras);
void orc_destroy(orc_scene* s);

int32_t orc_num_prims(const orc_scene* s);
int32_t orc_num_cameras(const orc_scene* s);
/* Export loader output as ABI structs (to cross-check the library's loader). */
int32_t orc_export(const orc_scene* s, rt_scene_params* params, rt_prim* prims, rt_camera* cameras);
/* Background colour/alpha of the scene (scene text `background`). */
int32_t orc_background(const orc_scene* s, rt_color* rgb, double* alpha);

/* Scene.Width/Height override and camera selection; both re-run Camera.InitRender. */
int32_t orc_set_size(orc_scene* s, int32_t w, int32_t h);
int32_t orc_select_camera(orc_scene* s, int32_t index);

/* Reference BVH (BVH.cs:193-236) statistics and its depth-first leaf order (prim IDs). */
int32_t orc_bvh_info(const orc_scene* s, int32_t* nodes, int32_t* depth);
int32_t orc_bvh_leaf_order(const orc_scene* s, int32_t* prim_ids);
/* Node boxes in depth-first (pre-)order: 8 doubles per node (min xyzw, max xyzw). */
int32_t orc_bvh_boxes(const orc_scene* s, double* boxes);

/* DebugRaycaster Primitives mode, ids[x*h + y] (-1 = miss). */
int32_t orc_primary_ids(const orc_scene* s, int32_t x0, int32_t y0, int32_t w, int32_t h, int32_t* ids);
/* DebugRaycaster BoundingVolumes mode: BVH<T>.GetIntersectionCount per integer-pixel ray (x*h + y). */
int32_t orc_bvh_counts(const orc_scene* s, int32_t x0, int32_t y0, int32_t w, int32_t h, int32_t* counts);
/* Closest hit of an arbitrary ray with no skip hit: returns prim ID or -1; dist may be NULL. */
int32_t orc_raytrace(const orc_scene* s, const double o[4], const double d[4], double* dist);

/* One camera sample (GetCameraRay + GetColor).  Returns 1 if it counts as a miss. */
int32_t orc_sample(const orc_scene* s, int32_t x, int32_t y, uint64_t seed, uint64_t sample,
                   rt_color* color, int32_t* rays);

/* Sequential, deterministic accumulation (sample order) into x*h + y buffers (+=). */
int32_t orc_render_tile(const orc_scene* s, int32_t x0, int32_t y0, int32_t w, int32_t h, int32_t spp,
                        uint64_t seed, uint64_t sample_base, rt_color* sum, uint32_t* samples,
                        uint32_t* misses, uint64_t* rays);

/* Diagnostic: one sample (as orc_sample) and its path: trace[2i] = primitive met by bounce i (-1 miss),
 * trace[2i+1] = event chosen there (1 diffuse, 2 specular, 3 specular fail, 4 transmitted,
 * 5 emission); 2 * (recursion + 1) entries, -2 past the path's end. */
int32_t orc_sample_trace(const orc_scene* s, int32_t x, int32_t y, uint64_t seed, uint64_t sample,
                         rt_color* color, int32_t* trace);

/* Diagnostic: the same accumulation with the draws of one reference worker thread: one .NET Core
 * 3.1 System.Random(seed) stream, spp passes over the tile row by row (Raytracer.cs:48,302-320). */
int32_t orc_render_tile_netrandom(const orc_scene* s, int32_t x0, int32_t y0, int32_t w, int32_t h, int32_t spp,
                                  int32_t seed, rt_color* sum, uint32_t* samples, uint32_t* misses,
                                  uint64_t* rays);

/*
 * FullRaytracer-style frame render (FullRaytracer.cs:66-72,219-229,271-302): `threads`
 * workers (0 = hardware_concurrency), TilesY = floor(sqrt(T)), TilesX = T / TilesY,
 * tiles handed out round-robin, one pass = 1 spp for one tile.  Buffers are whole-frame
 * x*height + y.  The pass budget is spp passes per tile.  *seconds gets the wall time
 * from the first tile to the last (Prepare/BVH excluded); *threads_used the worker count.
 */
int32_t orc_render_frame(const orc_scene* s, int32_t spp, uint64_t seed, int32_t threads,
                         rt_color* sum, uint32_t* samples, uint32_t* misses, uint64_t* rays,
                         double* seconds, int32_t* threads_used);

/* SampleSet.GetOutput (SampleSet.cs:61-113). */
int32_t orc_sample_output(rt_color sum, uint32_t samples, uint32_t misses, rt_color back,
                          double back_alpha, double exposure);

/* Fresnel helper for known-answer tests: the ratio Raytracer.cs:136-153 computes
 * (returns 1 on total internal reflection). */
double orc_fresnel(double cos_in, double ior_in, double ior_out);

/* The shared random stream (include/rtcore_rng.h): the first n uniforms of (seed, pixel, sample). */
int32_t orc_rng_draws(uint64_t seed, uint64_t pixel, uint64_t sample, int32_t n, double* out);

#ifdef __cplusplus
}
#endif

#endif
