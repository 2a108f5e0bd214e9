// bvh_gpu.hip -- PLOC BVH builder on the GPU (bvh_gpu.h).
//
// Pipeline (all on one stream):
//   1. centroid bounds (wave reductions + ordered-int atomics), 63-bit Morton codes,
//      rocPRIM radix sort of (code, index) pairs (stable: equal codes keep index order);
//   2. PLOC rounds over the cluster array (Morton order, compacted every round):
//        nn     -- each cluster's nearest neighbour in a +-kRadius window (LDS-staged boxes),
//                  metric = surface area of the merged box, ties -> the smaller index; that is
//                  a total order on pairs, so the globally best pair is always mutual and every
//                  round merges at least one pair;
//        flags  -- per-block counts of surviving clusters and of merges (wave ballots);
//        scan   -- one block scans the per-block counts;
//        merge  -- mutual pairs become a node (at the left cluster's position), the right
//                  cluster is dropped, survivors are compacted in order.  A new node records
//                  its primitive count, the number of internal nodes its collapsed subtree
//                  keeps (subtrees of <= max_leaf primitives become leaves), and -- for the
//                  4-wide collapse -- its wide children, wide-subtree size, stack need and
//                  depth, all from children that earlier rounds finished;
//   3. emission, rounds in reverse (a node's parent is always made in a later round, so this
//      is top-down): each kept node receives its pre-order index P and primitive offset O from
//      its parent, writes its NodeF, hands (P, O) to its kept children and writes the IDs of
//      leaf children into `order`; a wide-tree root also writes its Node4Q and hands wide
//      indices (pre-order, from the subtree sizes) to its wide children.
// The tree is a deterministic function of the boxes: no atomics decide any index.
#include "bvh_gpu.h"

#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace rtc {
namespace {

constexpr int kBlock = 256;
constexpr int kRadius = 16;    // default search radius (RTCORE_PLOC_RADIUS, up to kMaxRadius, for tuning)
constexpr int kMaxRadius = 64;
constexpr int kMaxRounds = 100000;

// ---- small helpers -------------------------------------------------------------------
__device__ __forceinline__ unsigned f2o(float f)
{
    const unsigned u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__host__ __device__ inline float o2f(unsigned u)
{
    const unsigned v = (u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u;
    float f;
    __builtin_memcpy(&f, &v, 4);
    return f;
}
__device__ __forceinline__ float area3(float4 lo, float4 hi) // FBox::area (bvh_sah.cpp)
{
    const float dx = fmaxf(0.0f, hi.x - lo.x), dy = fmaxf(0.0f, hi.y - lo.y), dz = fmaxf(0.0f, hi.z - lo.z);
    return 2.0f * (dx * dy + dy * dz + dz * dx);
}
__device__ __forceinline__ float4 min4(float4 a, float4 b)
{
    return make_float4(fminf(a.x, b.x), fminf(a.y, b.y), fminf(a.z, b.z), 0.0f);
}
__device__ __forceinline__ float4 max4(float4 a, float4 b)
{
    return make_float4(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z), 0.0f);
}
__device__ __forceinline__ uint64_t expand21(uint64_t x)
{
    x &= 0x1FFFFFull;
    x = (x | (x << 32)) & 0x1F00000000FFFFull;
    x = (x | (x << 16)) & 0x1F0000FF0000FFull;
    x = (x | (x << 8)) & 0x100F00F00F00F00Full;
    x = (x | (x << 4)) & 0x10C30C30C30C30C3ull;
    x = (x | (x << 2)) & 0x1249249249249249ull;
    return x;
}
__host__ __device__ inline int leaf_code(int first, int count) { return ~((first << 3) | (count - 1)); }

// Node records, unified index: 0..n-1 leaves (one primitive each, Morton order), n.. internal
// nodes in creation order.  lo.w = primitive count, hi.w = kept internal nodes (both int bits).
struct Tree {
    float4* lo;
    float4* hi;
    int2* child;   // [X - n]
    int4* wide;    // [X - n]: wide-subtree size, stack need, wide depth
    int4* pos;     // [X - n]: P, O, D (BVH2 depth)
    int* widx;     // [X - n]: wide-node index, -1 unless a wide root
    int* leaf_id;  // [leaf]: primitive ID
    int n, max_leaf;
    __device__ int count(int x) const { return __float_as_int(lo[x].w); }
    __device__ int kept(int x) const { return __float_as_int(hi[x].w); }
    __device__ bool real(int x) const { return count(x) > max_leaf; }
};

// The wide children of a kept node (BVH2 children l, r): open the kept child of largest box
// area (first on ties) until four children or none left to open (bvh_sah.cpp W4Builder::emit).
// off[] carries primitive offsets along (offset of l = o).
__device__ int wide_children(const Tree& T, int l, int r, int o, int ch[4], int off[4])
{
    ch[0] = l;
    ch[1] = r;
    off[0] = o;
    off[1] = o + T.count(l);
    int nc = 2;
    while (nc < 4) {
        int best = -1;
        float ba = -1.0f;
        for (int k = 0; k < nc; k++)
            if (T.real(ch[k])) {
                const float a = area3(T.lo[ch[k]], T.hi[ch[k]]);
                if (a > ba) {
                    ba = a;
                    best = k;
                }
            }
        if (best < 0) break;
        const int c = ch[best], oc = off[best];
        const int2 cc = T.child[c - T.n];
        for (int k = nc; k > best + 1; k--) {
            ch[k] = ch[k - 1];
            off[k] = off[k - 1];
        }
        ch[best] = cc.x;
        off[best] = oc;
        ch[best + 1] = cc.y;
        off[best + 1] = oc + T.count(cc.x);
        nc++;
    }
    return nc;
}

// ---- 1. Morton order ---------------------------------------------------------------------
__global__ void k_bounds_init(unsigned* b)
{
    if (threadIdx.x < 3) b[threadIdx.x] = 0xFFFFFFFFu;
    else if (threadIdx.x < 6) b[threadIdx.x] = 0u;
}

__global__ void __launch_bounds__(kBlock) k_bounds(const float4* lo, const float4* hi, int n, unsigned* b)
{
    unsigned mn[3] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}, mx[3] = {0u, 0u, 0u};
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        const float4 a = lo[i], c = hi[i];
        const float ce[3] = {0.5f * (a.x + c.x), 0.5f * (a.y + c.y), 0.5f * (a.z + c.z)};
        for (int k = 0; k < 3; k++) {
            const unsigned o = f2o(ce[k]);
            mn[k] = min(mn[k], o);
            mx[k] = max(mx[k], o);
        }
    }
    for (int k = 0; k < 3; k++)
        for (int s = 32; s > 0; s >>= 1) {
            mn[k] = min(mn[k], (unsigned)__shfl_xor((int)mn[k], s));
            mx[k] = max(mx[k], (unsigned)__shfl_xor((int)mx[k], s));
        }
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < 3; k++) {
            atomicMin(&b[k], mn[k]);
            atomicMax(&b[3 + k], mx[k]);
        }
}

__global__ void __launch_bounds__(kBlock) k_morton(const float4* lo, const float4* hi, int n, const unsigned* b,
                                                   uint64_t* keys, int* vals)
{
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float4 a = lo[i], c = hi[i];
    const float ce[3] = {0.5f * (a.x + c.x), 0.5f * (a.y + c.y), 0.5f * (a.z + c.z)};
    uint64_t code = 0; // 63-bit Morton code, 21 bits per axis
    for (int k = 0; k < 3; k++) {
        const float l = o2f(b[k]), h = o2f(b[3 + k]);
        const float ext = h - l;
        const float x = ext > 0.0f ? (ce[k] - l) / ext : 0.0f;
        const uint64_t q = (uint64_t)fminf(2097151.0f, fmaxf(0.0f, x * 2097152.0f));
        code |= expand21(q) << (2 - k);
    }
    keys[i] = code;
    vals[i] = i;
}

__global__ void __launch_bounds__(kBlock) k_init(Tree T, const float4* lo, const float4* hi, const int* ids,
                                                 const int* sorted, int* cref, float4* clo, float4* chi)
{
    const int s = blockIdx.x * kBlock + threadIdx.x;
    if (s >= T.n) return;
    const int p = sorted[s];
    const float4 a = lo[p], c = hi[p];
    T.lo[s] = make_float4(a.x, a.y, a.z, __int_as_float(1));
    T.hi[s] = make_float4(c.x, c.y, c.z, __int_as_float(0));
    T.leaf_id[s] = ids[p];
    cref[s] = s;
    clo[s] = a;
    chi[s] = c;
}

// ---- 2. PLOC rounds ----------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock) k_nn(int m, int radius, const float4* clo, const float4* chi, int* nn)
{
    __shared__ float4 s_lo[kBlock + 2 * kMaxRadius], s_hi[kBlock + 2 * kMaxRadius];
    const int base = blockIdx.x * kBlock - radius;
    for (int t = threadIdx.x; t < kBlock + 2 * radius; t += kBlock) {
        const int g = base + t;
        if (g >= 0 && g < m) {
            s_lo[t] = clo[g];
            s_hi[t] = chi[g];
        }
    }
    __syncthreads();
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= m) return;
    const float4 a = s_lo[i - base], b = s_hi[i - base];
    const int j0 = max(0, i - radius), j1 = min(m - 1, i + radius);
    float best = 0.0f;
    int bj = -1;
    for (int j = j0; j <= j1; j++) {
        if (j == i) continue;
        const float ar = area3(min4(a, s_lo[j - base]), max4(b, s_hi[j - base]));
        if (bj < 0 || ar < best) { // ascending j with a strict '<': ties go to the smaller index
            best = ar;
            bj = j;
        }
    }
    nn[i] = bj;
}

struct Flags {
    bool keep, lead;
};
__device__ __forceinline__ Flags flags_of(int i, int m, const int* nn)
{
    if (i >= m) return {false, false};
    const int j = nn[i];
    const bool mutual = nn[j] == i;
    return {!(mutual && i > j), mutual && i < j};
}

// exclusive in-block ranks of keep / lead and the block totals (256 threads = 4 waves)
__device__ __forceinline__ void block_ranks(Flags f, int& rk, int& rl, int& tk, int& tl)
{
    __shared__ int wk[kBlock / 64], wl[kBlock / 64];
    const unsigned long long bk = __ballot(f.keep), bl = __ballot(f.lead);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned long long lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    rk = __popcll(bk & lt);
    rl = __popcll(bl & lt);
    if (lane == 0) {
        wk[wave] = __popcll(bk);
        wl[wave] = __popcll(bl);
    }
    __syncthreads();
    tk = tl = 0;
    for (int w = 0; w < kBlock / 64; w++) {
        if (w < wave) {
            rk += wk[w];
            rl += wl[w];
        }
        tk += wk[w];
        tl += wl[w];
    }
}

__global__ void __launch_bounds__(kBlock) k_flags(int m, const int* nn, int2* bsum)
{
    const int i = blockIdx.x * kBlock + threadIdx.x;
    const Flags f = flags_of(i, m, nn);
    int rk, rl, tk, tl;
    block_ranks(f, rk, rl, tk, tl);
    if (threadIdx.x == 0) bsum[blockIdx.x] = make_int2(tk, tl);
}

// exclusive scan of the per-block counts in place; totals[0] = survivors, totals[1] = merges
__global__ void __launch_bounds__(1024) k_scan_blocks(int nb, int2* bsum, int* totals)
{
    __shared__ int sk[1024], sl[1024];
    const int per = (nb + 1023) / 1024;
    const int b0 = threadIdx.x * per, b1 = min(nb, b0 + per);
    int k = 0, l = 0;
    for (int b = b0; b < b1; b++) {
        k += bsum[b].x;
        l += bsum[b].y;
    }
    sk[threadIdx.x] = k;
    sl[threadIdx.x] = l;
    __syncthreads();
    for (int s = 1; s < 1024; s <<= 1) { // Hillis-Steele inclusive scan
        const int ak = threadIdx.x >= s ? sk[threadIdx.x - s] : 0;
        const int al = threadIdx.x >= s ? sl[threadIdx.x - s] : 0;
        __syncthreads();
        sk[threadIdx.x] += ak;
        sl[threadIdx.x] += al;
        __syncthreads();
    }
    int ok = sk[threadIdx.x] - k, ol = sl[threadIdx.x] - l;
    for (int b = b0; b < b1; b++) {
        const int2 v = bsum[b];
        bsum[b] = make_int2(ok, ol);
        ok += v.x;
        ol += v.y;
    }
    if (threadIdx.x == 1023) {
        totals[0] = sk[1023];
        totals[1] = sl[1023];
    }
}

__global__ void __launch_bounds__(kBlock) k_merge(Tree T, int m, int node_base, const int* nn, const int2* boff,
                                                  const int* cref, const float4* clo, const float4* chi, int* cref2,
                                                  float4* clo2, float4* chi2)
{
    const int i = blockIdx.x * kBlock + threadIdx.x;
    const Flags f = flags_of(i, m, nn);
    int rk, rl, tk, tl;
    block_ranks(f, rk, rl, tk, tl);
    if (!f.keep) return;
    const int2 o = boff[blockIdx.x];
    const int pos = o.x + rk;
    if (!f.lead) {
        cref2[pos] = cref[i];
        clo2[pos] = clo[i];
        chi2[pos] = chi[i];
        return;
    }
    const int j = nn[i];
    const int X = T.n + node_base + o.y + rl;
    const int l = cref[i], r = cref[j];
    const float4 lo = min4(clo[i], clo[j]), hi = max4(chi[i], chi[j]);
    const int cnt = T.count(l) + T.count(r);
    const bool real = cnt > T.max_leaf;
    const int kept = real ? 1 + T.kept(l) + T.kept(r) : 0;
    T.lo[X] = make_float4(lo.x, lo.y, lo.z, __int_as_float(cnt));
    T.hi[X] = make_float4(hi.x, hi.y, hi.z, __int_as_float(kept));
    T.child[X - T.n] = make_int2(l, r);
    if (real) {
        int ch[4], off[4];
        const int nc = wide_children(T, l, r, 0, ch, off);
        int w = 1, sn = 0, wd = 0;
        for (int k = 0; k < nc; k++)
            if (T.real(ch[k])) {
                const int4 c = T.wide[ch[k] - T.n];
                w += c.x;
                sn = max(sn, c.y);
                wd = max(wd, c.z + 1);
            }
        T.wide[X - T.n] = make_int4(w, nc - 1 + sn, wd, 0);
    }
    cref2[pos] = X;
    clo2[pos] = lo;
    chi2[pos] = hi;
}

// ---- 3. emission -------------------------------------------------------------------------
__device__ void write_leaf(const Tree& T, int c, int first, int* order)
{
    int st[8];
    int sp = 0, k = 0;
    st[sp++] = c;
    while (sp > 0) {
        const int x = st[--sp];
        if (x < T.n) {
            order[first + k++] = T.leaf_id[x];
        } else {
            const int2 cc = T.child[x - T.n];
            st[sp++] = cc.y;
            st[sp++] = cc.x;
        }
    }
}

__global__ void __launch_bounds__(kBlock) k_emit(Tree T, int first, int count, NodeF* out2, Node4Q* out4, int* order,
                                                 int* depth)
{
    const int t = blockIdx.x * kBlock + threadIdx.x;
    if (t >= count) return;
    const int X = T.n + first + t;
    if (!T.real(X)) return;
    const int4 ps = T.pos[X - T.n];
    const int P = ps.x, O = ps.y, D = ps.z;
    const int2 c = T.child[X - T.n];
    const int cs[2] = {c.x, c.y};
    const int Os[2] = {O, O + T.count(c.x)};
    const int Ps[2] = {P + 1, P + 1 + T.kept(c.x)};
    int refs2[2];
    for (int s = 0; s < 2; s++) {
        const int x = cs[s];
        if (T.real(x)) {
            refs2[s] = Ps[s];
            T.pos[x - T.n] = make_int4(Ps[s], Os[s], D + 1, 0);
        } else {
            refs2[s] = leaf_code(Os[s], T.count(x));
            write_leaf(T, x, Os[s], order);
        }
    }
    atomicMax(depth, D + 1);
    NodeF nf;
    const float4 a = T.lo[c.x], b = T.hi[c.x], e = T.lo[c.y], g = T.hi[c.y];
    nf.lmin = make_float4(a.x, a.y, a.z, __int_as_float(refs2[0]));
    nf.lmax = make_float4(b.x, b.y, b.z, 0.0f);
    nf.rmin = make_float4(e.x, e.y, e.z, __int_as_float(refs2[1]));
    nf.rmax = make_float4(g.x, g.y, g.z, 0.0f);
    out2[P] = nf;
    const int W = T.widx[X - T.n];
    if (W < 0) return;
    int ch[4], off[4];
    const int nc = wide_children(T, c.x, c.y, O, ch, off);
    float lo[4][3], hi[4][3];
    int refs[4];
    int next = W + 1;
    for (int k = 0; k < nc; k++) {
        const int x = ch[k];
        const float4 l = T.lo[x], h = T.hi[x];
        lo[k][0] = l.x;
        lo[k][1] = l.y;
        lo[k][2] = l.z;
        hi[k][0] = h.x;
        hi[k][1] = h.y;
        hi[k][2] = h.z;
        if (T.real(x)) {
            refs[k] = next;
            T.widx[x - T.n] = next;
            next += T.wide[x - T.n].x;
        } else {
            refs[k] = leaf_code(off[k], T.count(x));
        }
    }
    out4[W] = quantize_node4(lo, hi, refs, nc);
}

__global__ void k_root(Tree T, int root, int* order)
{
    if (threadIdx.x != 0) return;
    if (T.real(root)) {
        T.pos[root - T.n] = make_int4(0, 0, 0, 0);
        T.widx[root - T.n] = 0;
    } else {
        write_leaf(T, root, 0, order);
    }
}

template <class T>
struct Scratch {
    T* p = nullptr;
    ~Scratch()
    {
        if (p) (void)hipFree(p);
    }
    hipError_t alloc(size_t n) { return hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)); }
};

#define BVH_TRY(expr)                                                                                     \
    do {                                                                                                  \
        const hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess) return e_;                                                                  \
    } while (0)

hipError_t build(const float4* h_lo, const float4* h_hi, const int32_t* h_ids, int n, int max_leaf, int extra,
                 hipStream_t st, GpuBvh& out, Scratch<NodeF>& nodes, Scratch<Node4Q>& nodes4, Scratch<int>& order)
{
    const int nn2 = std::max(1, n - 1);
    int radius = kRadius;
    if (const char* e = getenv("RTCORE_PLOC_RADIUS")) radius = std::max(1, std::min(kMaxRadius, atoi(e)));
    Scratch<float4> lo_in, hi_in, clo[2], chi[2], tlo, thi;
    Scratch<int> ids, vals_in, vals, cref[2], nnb, leaf_id, widx, totals, depth;
    Scratch<uint64_t> keys_in, keys;
    Scratch<unsigned> bounds;
    Scratch<int2> child, bsum;
    Scratch<int4> wide, pos;
    BVH_TRY(lo_in.alloc(n));
    BVH_TRY(hi_in.alloc(n));
    BVH_TRY(ids.alloc(n));
    BVH_TRY(order.alloc((size_t)n + extra));
    BVH_TRY(hipMemcpyAsync(lo_in.p, h_lo, n * sizeof(float4), hipMemcpyHostToDevice, st));
    BVH_TRY(hipMemcpyAsync(hi_in.p, h_hi, n * sizeof(float4), hipMemcpyHostToDevice, st));
    BVH_TRY(hipMemcpyAsync(ids.p, h_ids, n * sizeof(int), hipMemcpyHostToDevice, st));
    for (int b = 0; b < 2; b++) {
        BVH_TRY(clo[b].alloc(n));
        BVH_TRY(chi[b].alloc(n));
        BVH_TRY(cref[b].alloc(n));
    }
    BVH_TRY(tlo.alloc(2 * (size_t)n));
    BVH_TRY(thi.alloc(2 * (size_t)n));
    BVH_TRY(vals_in.alloc(n));
    BVH_TRY(vals.alloc(n));
    BVH_TRY(keys_in.alloc(n));
    BVH_TRY(keys.alloc(n));
    BVH_TRY(bounds.alloc(6));
    BVH_TRY(nnb.alloc(n));
    BVH_TRY(leaf_id.alloc(n));
    BVH_TRY(widx.alloc(nn2));
    BVH_TRY(child.alloc(nn2));
    BVH_TRY(wide.alloc(nn2));
    BVH_TRY(pos.alloc(nn2));
    BVH_TRY(totals.alloc(2));
    BVH_TRY(depth.alloc(1));
    const int nb_max = (n + kBlock - 1) / kBlock;
    BVH_TRY(bsum.alloc(nb_max));

    hipEvent_t e0, e1;
    BVH_TRY(hipEventCreate(&e0));
    BVH_TRY(hipEventCreate(&e1));
    struct EvGuard {
        hipEvent_t a, b;
        ~EvGuard()
        {
            (void)hipEventDestroy(a);
            (void)hipEventDestroy(b);
        }
    } evg{e0, e1};
    BVH_TRY(hipEventRecord(e0, st));

    // 1. Morton order
    k_bounds_init<<<1, 64, 0, st>>>(bounds.p);
    k_bounds<<<std::min(nb_max, 2048), kBlock, 0, st>>>(lo_in.p, hi_in.p, n, bounds.p);
    k_morton<<<nb_max, kBlock, 0, st>>>(lo_in.p, hi_in.p, n, bounds.p, keys_in.p, vals_in.p);
    size_t tmp_bytes = 0;
    BVH_TRY(rocprim::radix_sort_pairs(nullptr, tmp_bytes, keys_in.p, keys.p, vals_in.p, vals.p, (size_t)n, 0, 63, st));
    Scratch<char> tmp;
    BVH_TRY(tmp.alloc(tmp_bytes));
    BVH_TRY(rocprim::radix_sort_pairs(tmp.p, tmp_bytes, keys_in.p, keys.p, vals_in.p, vals.p, (size_t)n, 0, 63, st));

    Tree T{tlo.p, thi.p, child.p, wide.p, pos.p, widx.p, leaf_id.p, n, max_leaf};
    k_init<<<nb_max, kBlock, 0, st>>>(T, lo_in.p, hi_in.p, ids.p, vals.p, cref[0].p, clo[0].p, chi[0].p);
    BVH_TRY(hipMemsetAsync(widx.p, 0xFF, nn2 * sizeof(int), st));
    BVH_TRY(hipMemsetAsync(depth.p, 0, sizeof(int), st));

    // 2. PLOC rounds
    std::vector<int> created;
    int m = n, cur = 0, node_base = 0;
    int h_tot[2];
    while (m > 1) {
        if ((int)created.size() >= kMaxRounds) return hipErrorUnknown;
        const int nb = (m + kBlock - 1) / kBlock;
        k_nn<<<nb, kBlock, 0, st>>>(m, radius, clo[cur].p, chi[cur].p, nnb.p);
        k_flags<<<nb, kBlock, 0, st>>>(m, nnb.p, bsum.p);
        k_scan_blocks<<<1, 1024, 0, st>>>(nb, bsum.p, totals.p);
        k_merge<<<nb, kBlock, 0, st>>>(T, m, node_base, nnb.p, bsum.p, cref[cur].p, clo[cur].p, chi[cur].p,
                                       cref[cur ^ 1].p, clo[cur ^ 1].p, chi[cur ^ 1].p);
        BVH_TRY(hipGetLastError());
        BVH_TRY(hipMemcpyAsync(h_tot, totals.p, sizeof h_tot, hipMemcpyDeviceToHost, st));
        BVH_TRY(hipStreamSynchronize(st));
        if (h_tot[1] <= 0 || h_tot[0] != m - h_tot[1]) return hipErrorUnknown; // no progress: cannot happen
        created.push_back(h_tot[1]);
        node_base += h_tot[1];
        m = h_tot[0];
        cur ^= 1;
    }
    int root = 0;
    BVH_TRY(hipMemcpyAsync(&root, cref[cur].p, sizeof(int), hipMemcpyDeviceToHost, st));
    BVH_TRY(hipStreamSynchronize(st));

    // sizes of the two trees
    int n_nodes = 0, n_nodes4 = 0, stack_need = 0, depth4 = 0, root_count = 1;
    if (root >= n) {
        float4 rl, rh;
        int4 rw;
        BVH_TRY(hipMemcpy(&rl, tlo.p + root, sizeof rl, hipMemcpyDeviceToHost));
        BVH_TRY(hipMemcpy(&rh, thi.p + root, sizeof rh, hipMemcpyDeviceToHost));
        BVH_TRY(hipMemcpy(&rw, wide.p + (root - n), sizeof rw, hipMemcpyDeviceToHost));
        std::memcpy(&root_count, &rl.w, 4);
        std::memcpy(&n_nodes, &rh.w, 4);
        if (root_count > max_leaf) {
            n_nodes4 = rw.x;
            stack_need = rw.y;
            depth4 = rw.z;
        }
    }
    BVH_TRY(nodes.alloc(n_nodes));
    BVH_TRY(nodes4.alloc(n_nodes4));

    // 3. emission, top-down
    k_root<<<1, 64, 0, st>>>(T, root, order.p);
    int first = node_base;
    for (int r = (int)created.size() - 1; r >= 0; r--) {
        first -= created[r];
        k_emit<<<(created[r] + kBlock - 1) / kBlock, kBlock, 0, st>>>(T, first, created[r], nodes.p, nodes4.p, order.p,
                                                                       depth.p);
    }
    BVH_TRY(hipGetLastError());
    BVH_TRY(hipEventRecord(e1, st));
    int h_depth = 0;
    BVH_TRY(hipMemcpyAsync(&h_depth, depth.p, sizeof(int), hipMemcpyDeviceToHost, st));
    BVH_TRY(hipStreamSynchronize(st));
    BVH_TRY(hipEventElapsedTime(&out.ms, e0, e1));

    out.n_nodes = n_nodes;
    out.n_nodes4 = n_nodes4;
    out.n_order = n;
    out.root = root_count > max_leaf ? 0 : leaf_code(0, root_count);
    out.root4 = out.root;
    out.depth = h_depth;
    out.depth4 = depth4;
    out.stack_need = stack_need;
    out.rounds = (int)created.size();
    return hipSuccess;
}

__global__ void __launch_bounds__(kBlock) k_gather(const int* order, int n, const PrimF* pi, const TestRec* ti,
                                                   PrimF* po, TestRec* to)
{
    const int k = blockIdx.x * kBlock + threadIdx.x;
    if (k >= n) return;
    const int id = order[k];
    po[k] = pi[id];
    to[k] = ti[id];
}

} // namespace

hipError_t gather_bvh_records(const int32_t* d_order, int n, const PrimF* d_prims_id, const TestRec* d_tests_id,
                              PrimF* d_prims, TestRec* d_tests, hipStream_t stream)
{
    if (n <= 0) return hipSuccess;
    k_gather<<<(n + kBlock - 1) / kBlock, kBlock, 0, stream>>>(d_order, n, d_prims_id, d_tests_id, d_prims, d_tests);
    return hipGetLastError();
}

hipError_t build_bvh_gpu(const float4* h_lo, const float4* h_hi, const int32_t* h_ids, int n, int max_leaf, int extra,
                         hipStream_t stream, GpuBvh& out)
{
    out = GpuBvh{};
    if (n <= 0 || max_leaf < 1 || max_leaf > 8) return hipErrorInvalidValue;
    Scratch<NodeF> nodes;
    Scratch<Node4Q> nodes4;
    Scratch<int> order;
    const hipError_t e = build(h_lo, h_hi, h_ids, n, max_leaf, extra, stream, out, nodes, nodes4, order);
    if (e != hipSuccess) {
        out = GpuBvh{};
        return e;
    }
    out.nodes = nodes.p;
    out.nodes4 = nodes4.p;
    out.order = order.p;
    nodes.p = nullptr; // ownership passes to the caller
    nodes4.p = nullptr;
    order.p = nullptr;
    return hipSuccess;
}

} // namespace rtc
