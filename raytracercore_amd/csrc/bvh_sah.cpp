// bvh_sah.cpp -- binned-SAH BVH2 for the fp32 path-tracing kernel.
//
// The kernel's own acceleration structure (the reference's agglomerative tree is kept only
// for the exact primary-ID pass, bvh_ref.cpp).  Leaf boxes start from the reference's fp64
// bounds (AABB.CreateFromBounded) rounded outward to fp32, so every primitive the fp64 query
// could reach is still reached.  Nodes store both children's boxes (64 B per visit, one
// cache line) and child references encode leaves inline (rt_internal.h NodeF).
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "host_scene.h"

namespace rtc {
namespace {

struct FBox {
    float lo[3], hi[3];
    void empty()
    {
        for (int i = 0; i < 3; i++) {
            lo[i] = __builtin_huge_valf();
            hi[i] = -__builtin_huge_valf();
        }
    }
    void grow(const FBox& b)
    {
        for (int i = 0; i < 3; i++) {
            lo[i] = std::min(lo[i], b.lo[i]);
            hi[i] = std::max(hi[i], b.hi[i]);
        }
    }
    float area() const
    {
        float d[3];
        for (int i = 0; i < 3; i++) d[i] = std::max(0.0f, hi[i] - lo[i]);
        return 2.0f * (d[0] * d[1] + d[1] * d[2] + d[2] * d[0]);
    }
};

float round_down(double v)
{
    float f = (float)v;
    if ((double)f > v) f = std::nextafter(f, -__builtin_huge_valf());
    return f;
}
float round_up(double v)
{
    float f = (float)v;
    if ((double)f < v) f = std::nextafter(f, __builtin_huge_valf());
    return f;
}

struct BNode {
    FBox box;
    int left = -1, right = -1;
    int first = 0, count = 0;
    bool cut = false; // a leaf of the BVH2 (count <= max_leaf); with `full` its subtree is built on
};

struct Ref {
    int prim;
    FBox box;
    float c[3];
};

struct SahBuilder {
    std::vector<Ref> refs;
    std::vector<BNode> nodes;
    int max_leaf;
    bool full = false; // build on below the BVH2 leaves down to single primitives (for the wide collapse)
    int max_depth = 0;

    int build(int first, int count, int depth, bool below = false)
    {
        if (!below) max_depth = std::max(max_depth, depth);
        BNode n;
        n.first = first;
        n.count = count;
        n.box.empty();
        FBox cb;
        cb.empty();
        for (int i = first; i < first + count; i++) {
            n.box.grow(refs[i].box);
            for (int k = 0; k < 3; k++) {
                cb.lo[k] = std::min(cb.lo[k], refs[i].c[k]);
                cb.hi[k] = std::max(cb.hi[k], refs[i].c[k]);
            }
        }
        int me = (int)nodes.size();
        const bool cut = count <= max_leaf;
        n.cut = cut;
        nodes.push_back(n);
        if (cut && (!full || count == 1)) return me;
        // binned SAH over the centroid bounds
        const int B = 32;
        int best_axis = -1, best_split = -1;
        float best_cost = __builtin_huge_valf();
        for (int axis = 0; axis < 3; axis++) {
            float ext = cb.hi[axis] - cb.lo[axis];
            if (!(ext > 0)) continue;
            FBox bb[B];
            int bc[B];
            for (int b = 0; b < B; b++) {
                bb[b].empty();
                bc[b] = 0;
            }
            float k = B / ext;
            for (int i = first; i < first + count; i++) {
                int b = std::min(B - 1, std::max(0, (int)((refs[i].c[axis] - cb.lo[axis]) * k)));
                bb[b].grow(refs[i].box);
                bc[b]++;
            }
            float rarea[B];
            int rcount[B];
            FBox acc;
            acc.empty();
            int cnt = 0;
            for (int b = B - 1; b > 0; b--) {
                acc.grow(bb[b]);
                cnt += bc[b];
                rarea[b] = acc.area();
                rcount[b] = cnt;
            }
            acc.empty();
            cnt = 0;
            for (int b = 0; b < B - 1; b++) {
                acc.grow(bb[b]);
                cnt += bc[b];
                if (cnt == 0 || rcount[b + 1] == 0) continue;
                float cost = acc.area() * cnt + rarea[b + 1] * rcount[b + 1];
                if (cost < best_cost) {
                    best_cost = cost;
                    best_axis = axis;
                    best_split = b;
                }
            }
        }
        int mid;
        if (best_axis < 0) {
            // all centroids coincide (or no useful split): median split by index
            mid = first + count / 2;
        } else {
            float ext = cb.hi[best_axis] - cb.lo[best_axis];
            float k = B / ext;
            auto it = std::partition(refs.begin() + first, refs.begin() + first + count, [&](const Ref& r) {
                int b = std::min(B - 1, std::max(0, (int)((r.c[best_axis] - cb.lo[best_axis]) * k)));
                return b <= best_split;
            });
            mid = (int)(it - refs.begin());
            if (mid == first || mid == first + count) mid = first + count / 2;
        }
        int l = build(first, mid - first, depth + 1, below || cut);
        int r = build(mid, first + count - mid, depth + 1, below || cut);
        nodes[me].left = l;
        nodes[me].right = r;
        return me;
    }
};

int leaf_ref(int first, int count) { return ~((first << 3) | (count - 1)); }

} // namespace

void sah_prim_box(const HostPrim& p, float lo[3], float hi[3])
{
    const double l[3] = {p.box.mn.x, p.box.mn.y, p.box.mn.z}, h[3] = {p.box.mx.x, p.box.mx.y, p.box.mx.z};
    for (int k = 0; k < 3; k++) {
        // outward rounding plus a relative pad of 2^-20 against fp32 traversal rounding
        const double pad = (std::fabs(l[k]) + std::fabs(h[k])) * 9.5367431640625e-07 + 1e-30;
        lo[k] = round_down(l[k] - pad);
        hi[k] = round_up(h[k] + pad);
    }
}

SahBvh build_sah_bvh(const std::vector<HostPrim>& prims, int max_leaf, bool full, const std::vector<char>* skip)
{
    SahBvh out;
    SahBuilder b;
    b.max_leaf = std::max(1, std::min(8, max_leaf));
    b.full = full;
    for (int i = 0; i < (int)prims.size(); i++) {
        const HostPrim& p = prims[i];
        if (p.kind == RT_PRIM_PLANE || (skip && (*skip)[i])) continue;
        Ref r;
        r.prim = i;
        sah_prim_box(p, r.box.lo, r.box.hi);
        for (int k = 0; k < 3; k++) r.c[k] = 0.5f * (r.box.lo[k] + r.box.hi[k]);
        b.refs.push_back(r);
    }
    if (b.refs.empty()) {
        out.root = 0;
        return out;
    }
    b.nodes.reserve(b.refs.size() * 2);
    int root = b.build(0, (int)b.refs.size(), 0);
    out.depth = b.max_depth;
    for (const Ref& r : b.refs) out.order.push_back(r.prim);
    // Emit internal nodes depth-first; the root gets index 0.
    std::vector<int> remap(b.nodes.size(), -1);
    std::vector<int> stack{root};
    std::vector<int> internal;
    while (!stack.empty()) {
        int i = stack.back();
        stack.pop_back();
        if (b.nodes[i].left < 0 || b.nodes[i].cut) continue;
        remap[i] = (int)internal.size();
        internal.push_back(i);
        stack.push_back(b.nodes[i].right);
        stack.push_back(b.nodes[i].left);
    }
    auto ref_of = [&](int i) {
        const BNode& n = b.nodes[i];
        return (n.left < 0 || n.cut) ? leaf_ref(n.first, n.count) : remap[i];
    };
    out.root = ref_of(root);
    for (int i : internal) {
        const BNode& n = b.nodes[i];
        const BNode& l = b.nodes[n.left];
        const BNode& r = b.nodes[n.right];
        NodeF f;
        int lr = ref_of(n.left), rr = ref_of(n.right);
        float lw, rw;
        std::memcpy(&lw, &lr, 4);
        std::memcpy(&rw, &rr, 4);
        f.lmin = make_float4(l.box.lo[0], l.box.lo[1], l.box.lo[2], lw);
        f.lmax = make_float4(l.box.hi[0], l.box.hi[1], l.box.hi[2], 0.0f);
        f.rmin = make_float4(r.box.lo[0], r.box.lo[1], r.box.lo[2], rw);
        f.rmax = make_float4(r.box.hi[0], r.box.hi[1], r.box.hi[2], 0.0f);
        out.nodes.push_back(f);
    }
    if (full) { // the whole tree down to single primitives, pre-order (children after their parent)
        out.full.resize(b.nodes.size());
        for (size_t i = 0; i < b.nodes.size(); i++) {
            const BNode& n = b.nodes[i];
            SahFullNode& f = out.full[i];
            for (int k = 0; k < 3; k++) {
                f.lo[k] = n.box.lo[k];
                f.hi[k] = n.box.hi[k];
            }
            f.left = n.left;
            f.right = n.right;
            f.first = n.first;
            f.count = n.count;
        }
        out.full_root = root;
    }
    return out;
}

// ---- 4-wide quantised BVH (Node4Q) -------------------------------------------------
// Collapse the BVH2: each wide node opens the largest-area internal child until it holds four
// children.  Child boxes are stored as 8-bit offsets from the node's origin in steps of 2^e
// per axis, rounded outward (every child box is contained in its dequantised box, checked in
// fp32), so a wide-node visit is one 64-B record as in the BVH2 and the depth halves.
namespace {

struct WChild {
    FBox box;
    int ref; // BVH2 child reference (>= 0 internal NodeF index, < 0 leaf code)
};

FBox nodef_box(const NodeF& n, bool right)
{
    FBox b;
    const float4 lo = right ? n.rmin : n.lmin, hi = right ? n.rmax : n.lmax;
    b.lo[0] = lo.x;
    b.lo[1] = lo.y;
    b.lo[2] = lo.z;
    b.hi[0] = hi.x;
    b.hi[1] = hi.y;
    b.hi[2] = hi.z;
    return b;
}
int nodef_ref(const NodeF& n, bool right)
{
    int r;
    std::memcpy(&r, right ? &n.rmin.w : &n.lmin.w, 4);
    return r;
}

struct W4Builder {
    const std::vector<NodeF>& n2;
    std::vector<Node4Q> out;
    int stack_need = 0;
    int depth = 0;
    bool siblings = false; // sibling-adjacent order: a node's internal children get consecutive indices

    std::vector<WChild> children(int i) const
    {
        std::vector<WChild> ch{{nodef_box(n2[i], false), nodef_ref(n2[i], false)},
                               {nodef_box(n2[i], true), nodef_ref(n2[i], true)}};
        while (ch.size() < 4) {
            int best = -1;
            float ba = -1.0f;
            for (int k = 0; k < (int)ch.size(); k++)
                if (ch[k].ref >= 0 && ch[k].box.area() > ba) {
                    ba = ch[k].box.area();
                    best = k;
                }
            if (best < 0) break;
            const NodeF& m = n2[ch[best].ref];
            WChild a{nodef_box(m, false), nodef_ref(m, false)}, b{nodef_box(m, true), nodef_ref(m, true)};
            ch[best] = a;
            ch.insert(ch.begin() + best + 1, b);
        }
        return ch;
    }

    // Emit the wide node for BVH2 node i at index `me` (already allocated); pre-order, or with its
    // internal children allocated as one consecutive block before any of their subtrees.
    void emit_at(int me, int i, int level, int pushes)
    {
        depth = std::max(depth, level);
        const std::vector<WChild> ch = children(i);
        const int nc = (int)ch.size();
        stack_need = std::max(stack_need, pushes + nc - 1);
        int refs[4] = {RT_NODE4_EMPTY, RT_NODE4_EMPTY, RT_NODE4_EMPTY, RT_NODE4_EMPTY};
        if (siblings) {
            for (int k = 0; k < nc; k++)
                if (ch[k].ref >= 0) {
                    refs[k] = (int)out.size();
                    out.push_back(Node4Q{});
                }
            for (int k = 0; k < nc; k++) {
                if (ch[k].ref >= 0) emit_at(refs[k], ch[k].ref, level + 1, pushes + nc - 1);
                else refs[k] = ch[k].ref;
            }
        } else {
            for (int k = 0; k < nc; k++)
                refs[k] = ch[k].ref >= 0 ? emit(ch[k].ref, level + 1, pushes + nc - 1) : ch[k].ref;
        }
        float lo[4][3], hi[4][3];
        for (int k = 0; k < nc; k++)
            for (int a = 0; a < 3; a++) {
                lo[k][a] = ch[k].box.lo[a];
                hi[k][a] = ch[k].box.hi[a];
            }
        out[me] = quantize_node4(lo, hi, refs, nc);
    }
    int emit(int i, int level, int pushes)
    {
        const int me = (int)out.size();
        out.push_back(Node4Q{});
        emit_at(me, i, level, pushes);
        return me;
    }
    // Emit the wide node for BVH2 node i (pre-order); returns its index.
    int emit_pre(int i, int level, int pushes)
    {
        depth = std::max(depth, level);
        const std::vector<WChild> ch = children(i);
        const int me = (int)out.size();
        out.push_back(Node4Q{});
        const int nc = (int)ch.size();
        stack_need = std::max(stack_need, pushes + nc - 1);
        int refs[4] = {RT_NODE4_EMPTY, RT_NODE4_EMPTY, RT_NODE4_EMPTY, RT_NODE4_EMPTY};
        for (int k = 0; k < nc; k++)
            refs[k] = ch[k].ref >= 0 ? emit_pre(ch[k].ref, level + 1, pushes + nc - 1) : ch[k].ref;
        float lo[4][3], hi[4][3];
        for (int k = 0; k < nc; k++)
            for (int a = 0; a < 3; a++) {
                lo[k][a] = ch[k].box.lo[a];
                hi[k][a] = ch[k].box.hi[a];
            }
        const Node4Q q = quantize_node4(lo, hi, refs, nc);
        out[me] = q;
        return me;
    }
};

// SAH-optimal collapse of the whole tree.  C[i][j] is the least cost of node i's subtree when it
// may fill up to j child slots of its parent wide node: one slot (i itself as a leaf or as a wide
// node) or i opened and its slots shared by its two children.
struct W4Sah {
    const std::vector<SahFullNode>& t;
    WideCosts w;
    std::vector<std::array<float, 5>> C;
    std::vector<std::array<int8_t, 5>> use;   // use[i][j]: slots actually taken (1 = i itself)
    std::vector<std::array<int8_t, 5>> split; // split[i][j]: slots of the left child when opened with j
    std::vector<uint8_t> leaf;                // i itself (one slot) is a leaf, not a wide node
    std::vector<Node4Q> out;
    int stack_need = 0;
    int depth = 0;

    static float area(const SahFullNode& n)
    {
        float d[3];
        for (int k = 0; k < 3; k++) d[k] = std::max(0.0f, n.hi[k] - n.lo[k]);
        return 2.0f * (d[0] * d[1] + d[1] * d[2] + d[2] * d[0]);
    }
    void solve()
    {
        const int n = (int)t.size();
        C.resize(n);
        use.resize(n);
        split.resize(n);
        leaf.resize(n);
        for (int i = n - 1; i >= 0; i--) { // children come after their parent (pre-order)
            const SahFullNode& s = t[i];
            const float a = area(s);
            if (s.left < 0) {
                for (int j = 1; j <= 4; j++) {
                    C[i][j] = w.c_prim * a * (float)s.count;
                    use[i][j] = 1;
                }
                leaf[i] = 1;
                continue;
            }
            float dist[5];
            for (int j = 2; j <= 4; j++) {
                dist[j] = __builtin_huge_valf();
                for (int k = 1; k < j; k++) {
                    const float c = C[s.left][k] + C[s.right][j - k];
                    if (c < dist[j]) {
                        dist[j] = c;
                        split[i][j] = (int8_t)k;
                    }
                }
            }
            const float c_node = w.c_node * a + dist[4];
            const float c_leaf = s.count <= w.max_leaf ? w.c_prim * a * (float)s.count : __builtin_huge_valf();
            leaf[i] = c_leaf <= c_node;
            C[i][1] = leaf[i] ? c_leaf : c_node;
            use[i][1] = 1;
            for (int j = 2; j <= 4; j++) {
                if (dist[j] < C[i][j - 1]) {
                    C[i][j] = dist[j];
                    use[i][j] = (int8_t)j;
                } else {
                    C[i][j] = C[i][j - 1];
                    use[i][j] = use[i][j - 1];
                }
            }
        }
    }
    void expand(int i, int j, std::vector<int>& ch) const
    {
        const int u = use[i][j];
        if (u == 1) {
            ch.push_back(i);
            return;
        }
        expand(t[i].left, split[i][u], ch);
        expand(t[i].right, u - split[i][u], ch);
    }
    int ref_of_leaf(int i) const { return leaf_ref(t[i].first, t[i].count); }
    // the wide node of tree node i (pre-order, as the greedy collapse); returns its index
    int emit(int i, int level, int pushes)
    {
        depth = std::max(depth, level);
        std::vector<int> ch;
        expand(t[i].left, split[i][4], ch);
        expand(t[i].right, 4 - split[i][4], ch);
        const int me = (int)out.size();
        out.push_back(Node4Q{});
        const int nc = (int)ch.size();
        stack_need = std::max(stack_need, pushes + nc - 1);
        int refs[4] = {RT_NODE4_EMPTY, RT_NODE4_EMPTY, RT_NODE4_EMPTY, RT_NODE4_EMPTY};
        float lo[4][3], hi[4][3];
        for (int k = 0; k < nc; k++) {
            const int c = ch[k];
            refs[k] = leaf[c] ? ref_of_leaf(c) : emit(c, level + 1, pushes + nc - 1);
            for (int a = 0; a < 3; a++) {
                lo[k][a] = t[c].lo[a];
                hi[k][a] = t[c].hi[a];
            }
        }
        out[me] = quantize_node4(lo, hi, refs, nc);
        return me;
    }
};

} // namespace

Bvh4 build_bvh4(const SahBvh& b2, const WideCosts* sah)
{
    Bvh4 r;
    if (sah && !b2.full.empty()) {
        W4Sah w{b2.full, *sah, {}, {}, {}, {}, {}, 0, 0};
        w.w.max_leaf = std::max(1, std::min(8, w.w.max_leaf));
        w.solve();
        const int root = b2.full_root;
        if (w.leaf[root]) {
            r.root = w.ref_of_leaf(root);
            return r;
        }
        w.out.reserve(b2.full.size() / 4 + 1);
        r.root = w.emit(root, 0, 0);
        r.nodes = std::move(w.out);
        r.stack_need = w.stack_need;
        r.depth = w.depth;
        return r;
    }
    if (b2.nodes.empty()) { // a single leaf (or nothing)
        r.root = b2.root;
        return r;
    }
    W4Builder w{b2.nodes, {}, 0, 0};
    if (const char* e = getenv("RTCORE_WIDE_ORDER")) w.siblings = e[0] == 's'; // A/B: sibling-adjacent order
    w.out.reserve(b2.nodes.size() / 2 + 1);
    r.root = w.siblings ? w.emit(0, 0, 0) : w.emit_pre(0, 0, 0);
    r.nodes = std::move(w.out);
    r.stack_need = w.stack_need;
    r.depth = w.depth;
    return r;
}

} // namespace rtc
