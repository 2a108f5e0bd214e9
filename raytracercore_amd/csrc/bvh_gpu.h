// bvh_gpu.h -- GPU BVH builder (PLOC) for large scenes.
//
// Builds, on the device, the same two fast-path structures the host builder makes
// (bvh_sah.cpp): a BVH2 of NodeF records in depth-first order whose leaves hold <= max_leaf
// primitives contiguous in `order`, and its 4-wide quantised collapse (Node4Q, the same
// opening rule and the same quantisation, quantize_node4).  The binary tree comes from
// Parallel Locally-Ordered Clustering (Meister & Bittner 2018): primitives sorted by the Morton
// code of their centroid, then rounds in which every cluster finds the neighbour within a
// window of +-16 clusters whose merged box has the smallest surface area, and mutual nearest
// neighbours merge.  That is the reference's own agglomerative rule (merge the pair with the
// smallest combined surface area, BVH.cs:50-191) restricted to a Morton window so that each
// round is one data-parallel pass.
#pragma once
#include <hip/hip_runtime.h>

#include "rt_internal.h"

namespace rtc {

struct GpuBvh {
    // device arrays, allocated with hipMalloc; the caller owns (and frees) them
    NodeF* nodes = nullptr;   // n_nodes BVH2 internal nodes, root = index 0 (if any)
    Node4Q* nodes4 = nullptr; // n_nodes4 wide nodes, root = index 0 (if any)
    int32_t* order = nullptr; // n_order entries: primitive IDs in leaf order (capacity n + extra)
    int n_nodes = 0, n_nodes4 = 0, n_order = 0;
    int root = 0, root4 = 0;  // child references of the roots (>= 0 node index, < 0 leaf code)
    int depth = 0;            // deepest BVH2 node (root 0), as SahBvh::depth
    int depth4 = 0;           // deepest wide node, as Bvh4::depth
    int stack_need = 0;       // as Bvh4::stack_need
    int rounds = 0;           // PLOC rounds
    float ms = 0.0f;          // device build time (Morton codes to the last wide node)
};

// boxes: n primitive boxes (lo, hi; fp32, already rounded outward); ids: the primitive ID of
// each box.  `order` gets capacity n + extra so the caller can append records behind the BVH's.
// Returns hipSuccess or the first HIP error; on error nothing stays allocated.
hipError_t build_bvh_gpu(const float4* h_lo, const float4* h_hi, const int32_t* h_ids, int n, int max_leaf, int extra,
                         hipStream_t stream, GpuBvh& out);

// prims[k] = prims_id[order[k]], tests[k] = tests_id[order[k]] for k < n (records in leaf order)
hipError_t gather_bvh_records(const int32_t* d_order, int n, const PrimF* d_prims_id, const TestRec* d_tests_id,
                              PrimF* d_prims, TestRec* d_tests, hipStream_t stream);

} // namespace rtc
