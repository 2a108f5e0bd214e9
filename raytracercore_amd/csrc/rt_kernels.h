// rt_kernels.h -- launch interface between the C ABI (rtcore_api.hip) and the kernels.
#pragma once
#include "../../include/rtcore_rng.h"
#include "rt_internal.h"

namespace rtc {

constexpr int kMaxSplit = 8;     // item ranges of a launch: one per XCD of the MI355X
constexpr int kSplitStride = 32; // dispenser words apart (one 128-B line each)

// Work decomposition of one path-tracing launch over a w x h tile.
struct PathParams {
    int x0, y0, w, h;           // tile within the frame
    int band, band_stride, band_offset; // band > 0: tile row r is frame row
                                        // y0 + ((r / band) * band_stride + band_offset) * band + r % band
    int band_log2;              // log2(band) for a power-of-two band, else -1 (divide by inv_band)
    float inv_band;             // fp32 1 / band
    int spp;                    // samples per pixel in this launch
    int chunk;                  // samples per work item (a lane owns one item at a time)
    int n_chunks;               // ceil(spp / chunk) rounded up to a power of two (empty chunks are skipped)
    int log2_chunks;
    int blocks_x;               // 8x8 pixel blocks per tile row
    int n_pad;                  // padded pixels per chunk (blocks * 64)
    int refill;                 // BVH kernel: waiting lanes (of 64) that trigger the shading phase
    int spec;                   // BVH kernel (RT_BVH_SPEC): lanes blocked on a pending leaf that trigger a leaf step
    int pool;                   // work items a wave takes per atomic: 64 x a power of two <= n_chunks
                                // (all from one 8x8 block, so a wave's lanes stay on neighbouring pixels)
    float inv_blocks_x;         // fp32 reciprocal for the item decode (when magic_bx == 0)
    unsigned magic_bx;          // ceil(2^32 / blocks_x) when block / blocks_x = umulhi(block, magic_bx) for
                                // every block of the launch (make_params checks), else 0
    unsigned long long seed;
    rt_key2 seed_key;           // rt_rng_seed_key(seed) (rtcore_rng.h)
    unsigned long long sample_base;
    const rt_key2* pkeys;       // brute-force kernels: rt_rng_pixel_key(seed_key, pixel) per frame pixel
                                // (cached per scene and seed, pixel_keys_kernel), or null: hashed per item
    unsigned int* counter;      // work-item dispensers (zeroed before launch), one per item range, kSplitStride apart
    int n_split;                // item ranges (1 or kMaxSplit): range g = blocks [split_start[g], split_start[g + 1])
                                // in item units, dealt first to the workgroups b with b % n_split == g (the
                                // workgroups that share one XCD and its L2), then to any wave once theirs is spent
    unsigned split_start[9];
    float4* partial;            // [block][chunk][64 pixels]: rgb sums, (samples | misses << 16)
    unsigned long long* rays;   // Scene.RayTrace-equivalents (added to)
    int* stack_ovf;             // BVH kernels: traversal-stack overflow, RT_STACK_OVF entries per lane of the grid
    unsigned long long* stats;  // optional [7]: node visits, triangle tests, sphere tests (per lane);
                                //   wave cycles in sample start, traversal, shading; wave iterations
    // The scene as this launch's kernel variant walks it (fill_launch).  The brute-force kernels read
    // these from the launch record by scalar loads where they are used, instead of holding them in
    // SGPRs as kernel arguments for the whole kernel (which spilled into VGPR lanes).
    PathScene scene;
    const TestRec* tests;
    const float4* rows;         // BVH kernels: 3 float4 per slot, the compact leaves' records (DevScene::rows_bvh)
    const RectRec* rects;
    const FrameRec* frames;
    const PrimF* prims;
    const GroupRec* groups;
    const NodeF* nodes;         // BVH kernels: the BVH2 and the wide tree
    const Node4Q* nodes4;
    const XformF* xf;
    const MatF* mats;
    const float4* vnormals;
    const PrimD* prims_d;       // the exact fp64 records by primitive ID (the vertex-normal re-hit test)
    float4* ray_log;            // BVH kernels, instrumented launch only (rt_debug_ray_log): every finished
    unsigned int* ray_log_n;    //   query as 3 float4 (o, prev | d | t, sg) appended at ray_log_n, up to
    unsigned int ray_log_cap;   //   ray_log_cap records
};

// Trace-only kernel over a ray list (rt_debug_trace_rays): the wide BVH's speculative traversal
// without the shading phase, for measuring what a wavefront split's traversal stage would take.
struct TraceRaysParams {
    const float4* rays;         // 3 float4 per ray as the ray log writes them
    float2* hits;               // (t, bitcast sg) per ray
    unsigned int n;
    unsigned int* counter;      // ray dispenser (zeroed before the launch)
    int* stack_ovf;
    const TestRec* tests;
    const float4* rows;
    const Node4Q* nodes4;
    const XformF* xf;
    int root4;
    int spec;                   // blocked lanes that trigger a leaf step (as PathParams.spec)
    const GroupRec* outer;      // the BVH order's outer group (DevScene::groups_bvh) or null
    const RectRec* outer_rects;
    const FrameRec* outer_boxes;
    unsigned long long* stats;  // optional [3]: node visits, leaf-step lane slots, lane slots in all
};

#ifndef __HIPCC_RTC__ // host-side launch interface (not part of a hiprtc-compiled kernel)
// Sets p.scene and the record pointers of the given kernel variant's slot order.
void fill_launch(const DevScene& s, int variant, PathParams& p);

// mode 0: primary hit IDs, mode 1: reference-BVH node counts (DebugRaycaster BoundingVolumes)
hipError_t launch_primary_ids(const DevScene& s, const CameraD& cam, int x0, int y0, int w, int h, int mode,
                              int32_t* d_ids, hipStream_t stream);

// Kernel variant: kernel 0 brute force, 1 grouped brute force, 2 BVH2 (24-entry stack), 3 wide BVH
// (RT_WIDE_STACK = 16-entry stack), both + kStackOverflow entries in global memory;
// lds stages the shading records in LDS.
int path_variant(int kernel, bool lds);
constexpr int kStackOverflow = 44; // = RT_STACK_OVF (kernels_path.hip)
constexpr int kTestSpares = 3;     // zero TestRecs after the BVH-order records (leaf steps of up to 4 loads)
int path_wide_stack();              // LDS entries of the wide BVH kernel's stack (RT_WIDE_STACK)
size_t path_lds_bytes(const DevScene& s);   // dynamic LDS of the staged (lds) variants
size_t path_dyn_lds(const DevScene& s, int variant); // all dynamic LDS of a variant (+ the wide kernel's hot nodes)
// Launch the persistent kernel; stats counts node visits / primitive tests (slower build).
// The camera and the launch parameters are read from device memory (d_cam, d_params).
hipError_t launch_path(const DevScene& s, const CameraF* d_cam, const PathParams* d_params, int variant,
                       int grid_blocks, hipStream_t stream, bool stats);
int path_blocks_per_cu(int variant, size_t dyn_lds, bool stats, bool vn); // vn: scene has vertex-normal triangles
// The trace-only kernel (waves per SIMD 6 / 7 / 8 with LDS stacks of 20 / 16 / 16 entries): blocks
// per CU and launch (grid blocks of 256).
int trace_rays_blocks_per_cu(int waves);
// Host evaluation of the kernels' vertex-normal re-hit test (vn_rehit_test): Triangle.RayTraceAVXFaster
// in fp64 from the hit point fma(e01, u, fma(e02, v, v0)) along dir; returns 1 on a hit, with its
// Inside flag, t and the origin used.
int debug_vn_rehit(const double v0[3], const double e01[3], const double e02[3], int mirror, double u, double v,
                   const float dir[3], int* inside, double* t, double o[3]);
hipError_t launch_trace_rays(const TraceRaysParams& p, int waves, int grid_blocks, hipStream_t stream);
// out[y * w + x] = rt_rng_pixel_key(seed_key, y * w + x) for a w x h frame
hipError_t launch_pixel_keys(rt_key2 seed_key, int w, int h, rt_key2* out, hipStream_t stream);
// The BVH order's rows (3 float4 per record, n_records including the spares) from its TestRecs and,
// with rewrite, every homogeneous leaf reference of the BVH2 and the wide tree made compact
// (rt_internal.h, kLeafCompact).
hipError_t compact_leaves(const TestRec* d_tests, int n_records, float4* d_rows, NodeF* d_nodes, int n_nodes,
                          Node4Q* d_nodes4, int n_nodes4, bool rewrite, hipStream_t stream);

// partial -> fp64 planar accumulators (d_sum planes R | G | B, each `plane` doubles apart;
// 0 = w*h), d_samples, d_misses (row-major w*h), added to.
hipError_t launch_accumulate(const PathParams& p, double* d_sum, uint32_t* d_samples, uint32_t* d_misses,
                             hipStream_t stream, size_t plane = 0);
// SampleSet.GetOutput over planar accumulators (row-major w*h) -> ARGB codes.
hipError_t launch_tonemap(int w, int h, const double* d_sum, const uint32_t* d_samples, const uint32_t* d_misses,
                          rt_color back, double back_alpha, double exposure, int32_t* d_argb, hipStream_t stream);
// One pixel of the host-buffer entry point's layout (rt_render_tile): the accumulated DoubleColor,
// samples and misses, in the caller's x*h + y order.
struct TileRec {
    double r, g, b;
    uint32_t samples, misses;
};
// planar row-major accumulators (w*h) -> TileRec[w*h] in x*h + y order
hipError_t launch_tile_host_layout(int w, int h, const double* d_sum, const uint32_t* d_samples,
                                  const uint32_t* d_misses, TileRec* d_out, hipStream_t stream);
// partial (1 spp) -> the DoubleColor[w, h] values as fp32 rgb in x*h + y order, Placeholder(-1) on a miss.
hipError_t launch_colors_1spp(const PathParams& p, float* d_out, hipStream_t stream);

#endif

} // namespace rtc
