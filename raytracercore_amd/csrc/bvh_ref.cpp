// bvh_ref.cpp -- the reference's agglomerative BVH (Acceleration/BVH.cs:12-236), built
// with index arrays and flattened depth-first for the exact primary-ID kernel.
//
// Why the product rebuilds the reference's tree instead of using its own SAH BVH: the
// reference's closest hit (Scene.cs:65-111) breaks ties between equal-distance hits by the
// order of the near-sorted pierced-leaf list, whose tie order is this tree's depth-first
// leaf order.  Reproducing primary-ray IDs bit for bit needs the same tree.
//
// Pieces restated: KDTree (KDTree.cs:9-453) incl. the .NET Core 3.1 introsort that
// Array.Sort applies to it, the binary Heap (Heap.cs), the three construction regimes
// (brute force n<=20 with HashSet slot order, heap agglomeration 21..200000, local
// nearest-neighbour agglomeration >200000) and BVH.MakeParent's SkipVolume flags.
// Element identity stands in for BVH<T>.Equals (live tree elements are disjoint).
#include <algorithm>
#include <cmath>
#include <functional>

#include "host_scene.h"

namespace rtc {
namespace {

struct BNode {
    int left = -1, right = -1, prim = -1;
    Box box;
    double cost = -1;
    bool skip = false;
    bool leaf() const { return prim >= 0; }
};

struct Builder {
    const std::vector<HostPrim>& prims;
    std::vector<BNode> n;
    explicit Builder(const std::vector<HostPrim>& p) : prims(p) { n.reserve(p.size() * 4 + 8); }

    int leaf(int i)
    {
        BNode b;
        b.prim = i;
        b.box = prims[i].box;
        n.push_back(b);
        return (int)n.size() - 1;
    }
    int pair(int l, int r)
    {
        BNode b;
        b.left = l;
        b.right = r;
        b.box = box_combine(n[l].box, n[r].box);
        n.push_back(b);
        return (int)n.size() - 1;
    }
    void make_parent(int p)
    {
        n[n[p].left].skip = box_equals(n[n[p].left].box, n[p].box);
        n[n[p].right].skip = box_equals(n[n[p].right].box, n[p].box);
    }
    double cost(int i)
    {
        if (n[i].cost == -1) n[i].cost = box_sa(n[i].box);
        return n[i].cost;
    }
    int child_leaves(int i) const { return (n[n[i].left].leaf() ? 1 : 0) + (n[n[i].right].leaf() ? 1 : 0); }
    Vec4d center(int i) const { return n[i].leaf() ? prims[n[i].prim].center_pt : n[i].box.ctr; }
};

int cmp_double(double a, double b) // double.CompareTo
{
    if (a < b) return -1;
    if (a > b) return 1;
    if (a == b) return 0;
    bool an = a != a, bn = b != b;
    return an ? (bn ? 0 : -1) : 1;
}
double comp(Vec4d v, int axis) { return axis == 0 ? v.x : axis == 1 ? v.y : v.z; }

// .NET Core 3.1 ArraySortHelper<T>.IntrospectiveSort over an index range.
template <class Cmp>
void net_introsort(std::vector<int>& k, Cmp cmp)
{
    auto swap_if = [&](int a, int b) {
        if (a != b && cmp(k[a], k[b]) > 0) std::swap(k[a], k[b]);
    };
    std::function<void(int, int, int)> intro = [&](int lo, int hi, int depth) {
        while (hi > lo) {
            int size = hi - lo + 1;
            if (size <= 16) {
                if (size == 1) return;
                if (size == 2) { swap_if(lo, hi); return; }
                if (size == 3) { swap_if(lo, hi - 1); swap_if(lo, hi); swap_if(hi - 1, hi); return; }
                for (int i = lo; i < hi; i++) { // InsertionSort
                    int j = i, t = k[i + 1];
                    while (j >= lo && cmp(t, k[j]) < 0) { k[j + 1] = k[j]; j--; }
                    k[j + 1] = t;
                }
                return;
            }
            if (depth == 0) { // Heapsort
                int cnt = size;
                auto down = [&](int i, int m) {
                    int d = k[lo + i - 1];
                    while (i <= m / 2) {
                        int c = 2 * i;
                        if (c < m && cmp(k[lo + c - 1], k[lo + c]) < 0) c++;
                        if (!(cmp(d, k[lo + c - 1]) < 0)) break;
                        k[lo + i - 1] = k[lo + c - 1];
                        i = c;
                    }
                    k[lo + i - 1] = d;
                };
                for (int i = cnt / 2; i >= 1; i--) down(i, cnt);
                for (int i = cnt; i > 1; i--) { std::swap(k[lo], k[lo + i - 1]); down(1, i - 1); }
                return;
            }
            depth--;
            int mid = lo + ((hi - lo) >> 1); // PickPivotAndPartition
            swap_if(lo, mid);
            swap_if(lo, hi);
            swap_if(mid, hi);
            int pivot = k[mid];
            std::swap(k[mid], k[hi - 1]);
            int l = lo, r = hi - 1;
            while (l < r) {
                while (cmp(k[++l], pivot) < 0) {}
                while (cmp(pivot, k[--r]) < 0) {}
                if (l >= r) break;
                std::swap(k[l], k[r]);
            }
            if (l != hi - 1) std::swap(k[l], k[hi - 1]);
            intro(l + 1, hi, depth);
            hi = l - 1;
        }
    };
    int cnt = (int)k.size();
    if (cnt < 2) return;
    int lg = 0;
    for (int m = cnt; m >= 1; m /= 2) lg++;
    intro(0, cnt - 1, 2 * lg);
}

// k-d tree over BVH node centres (KDTree<T>), node pool with in-place MergeTo / SplitWith.
struct Kd {
    struct N {
        bool leaf = false;
        int axis = 0;
        double median = 0;
        int left = -1, right = -1;
        int elem = -1;
        Vec4d ctr{0, 0, 0, 0};
    };
    Builder& b;
    std::vector<N> t;
    int root = -1;
    explicit Kd(Builder& bb) : b(bb) {}

    int mk_leaf(int e)
    {
        N x;
        x.leaf = true;
        x.elem = e;
        x.ctr = b.center(e);
        t.push_back(x);
        return (int)t.size() - 1;
    }
    int construct(std::vector<int> set, int depth) // KDTree.Construct (KDTree.cs:11-33)
    {
        if (set.size() == 1) return set[0];
        int axis = depth % 3;
        net_introsort(set, [&](int a, int c) { return cmp_double(comp(t[a].ctr, axis), comp(t[c].ctr, axis)); });
        size_t half = set.size() / 2;
        std::vector<int> l(set.begin(), set.begin() + half), r(set.begin() + half, set.end());
        double median = (comp(t[l.back()].ctr, axis) + comp(t[r[0]].ctr, axis)) / 2;
        int a = construct(l, depth + 1), c = construct(r, depth + 1);
        N x;
        x.axis = axis;
        x.median = median;
        x.left = a;
        x.right = c;
        t.push_back(x);
        return (int)t.size() - 1;
    }
    bool contains(int k, int e, Vec4d p) const
    {
        const N& x = t[k];
        if (x.leaf) return x.elem == e;
        double c = comp(p, x.axis);
        return (c <= x.median && contains(x.left, e, p)) || (c >= x.median && contains(x.right, e, p));
    }
    bool contains(int e) const { return contains(root, e, b.center(e)); }
    void nn(int k, int e, Vec4d p, int& best, double& bd) const
    {
        const N& x = t[k];
        if (x.leaf) {
            if (x.elem != e) {
                double d = sqlen_s(sub(x.ctr, p));
                if (d < bd) { best = k; bd = d; }
            }
            return;
        }
        double c = comp(p, x.axis);
        int pri = c <= x.median ? x.left : x.right, sec = c <= x.median ? x.right : x.left;
        nn(pri, e, p, best, bd);
        double bdist = fabs(c - x.median);
        bdist *= bdist;
        if (bdist < bd) nn(sec, e, p, best, bd);
    }
    int nearest(int e) const
    {
        int best = -1;
        double bd = __builtin_huge_val();
        nn(root, e, b.center(e), best, bd);
        return best >= 0 ? t[best].elem : -1;
    }
    bool parent_of(int k, int e, Vec4d p, int& parent) const
    {
        const N& x = t[k];
        if (x.leaf) return x.elem == e;
        int gp = parent;
        double c = comp(p, x.axis);
        if (c <= x.median) { parent = k; if (parent_of(x.left, e, p, parent)) return true; }
        if (c >= x.median) { parent = k; if (parent_of(x.right, e, p, parent)) return true; }
        parent = gp;
        return false;
    }
    void remove(int e)
    {
        int parent = root;
        parent_of(root, e, b.center(e), parent);
        const N& l = t[t[parent].left];
        int keep = (l.leaf && l.elem == e) ? t[parent].right : t[parent].left;
        t[parent] = t[keep];
    }
    void add(int e)
    {
        Vec4d p = b.center(e);
        int parent = root, node = root;
        while (!t[node].leaf) {
            parent = node;
            node = comp(p, t[node].axis) <= t[node].median ? t[node].left : t[node].right;
        }
        int axis = (t[parent].axis + 1) % 3;
        N copy = t[node];
        t.push_back(copy);
        int l = (int)t.size() - 1;
        int r = mk_leaf(e);
        double lc = comp(t[l].ctr, axis), rc = comp(t[r].ctr, axis);
        double median = (lc + rc) / 2;
        if (lc > rc) std::swap(l, r);
        N s;
        s.axis = axis;
        s.median = median;
        s.left = l;
        s.right = r;
        t[node] = s;
    }
    void build(const std::vector<int>& elems)
    {
        std::vector<int> set;
        for (int e : elems) set.push_back(mk_leaf(e));
        root = construct(set, 0);
    }
};

int build_heap(Builder& b, int np)
{
    std::vector<int> leaves(np);
    for (int i = 0; i < np; i++) leaves[i] = b.leaf(i);
    Kd kd(b);
    kd.build(leaves);
    auto cmp = [&](int x, int y) { // pairComparer (BVH.cs:100-115)
        if (x == y) return 0;
        int c = cmp_double(b.cost(x), b.cost(y));
        if (c) return c;
        int lx = b.child_leaves(x), ly = b.child_leaves(y);
        return (ly > lx) - (ly < lx);
    };
    std::vector<int> h;
    for (int i = 0; i < np; i++) h.push_back(b.pair(leaves[i], kd.nearest(leaves[i])));
    auto down = [&](int i) {
        while (true) {
            int l = 2 * i + 1, r = l + 1, c = i;
            if (l < (int)h.size() && cmp(h[c], h[l]) > 0) c = l;
            if (r < (int)h.size() && cmp(h[c], h[r]) > 0) c = r;
            if (c == i) break;
            std::swap(h[i], h[c]);
            i = c;
        }
    };
    auto push = [&](int x) {
        h.push_back(x);
        int i = (int)h.size() - 1, p = (i - 1) / 2;
        while (i != 0 && cmp(x, h[p]) <= 0) { h[i] = h[p]; i = p; p = (i - 1) / 2; }
        h[i] = x;
    };
    for (int i = (int)h.size() / 2 - 1; i >= 0; i--) down(i);
    while (true) {
        int ch = h[0];
        h[0] = h.back();
        h.pop_back();
        down(0);
        if (!kd.contains(b.n[ch].left)) continue;
        if (!kd.contains(b.n[ch].right)) {
            push(b.pair(b.n[ch].left, kd.nearest(b.n[ch].left)));
            continue;
        }
        b.make_parent(ch);
        kd.remove(b.n[ch].left);
        if (kd.t[kd.root].leaf) return ch;
        kd.remove(b.n[ch].right);
        kd.add(ch);
        push(b.pair(ch, kd.nearest(ch)));
    }
}

int build_local(Builder& b, int np)
{
    std::vector<int> leaves(np);
    for (int i = 0; i < np; i++) leaves[i] = b.leaf(i);
    Kd kd(b);
    kd.build(leaves);
    int a = leaves[0], c2 = kd.nearest(a);
    while (true) {
        int c = kd.nearest(c2);
        if (a == c) {
            kd.remove(a);
            a = b.pair(a, c2);
            b.make_parent(a);
            if (kd.t[kd.root].leaf) return a;
            kd.remove(c2);
            kd.add(a);
            c2 = kd.nearest(a);
        } else {
            a = c2;
            c2 = c;
        }
    }
}

int build_brute(Builder& b, int np)
{
    std::vector<int> slot(np), free_slots;
    for (int i = 0; i < np; i++) slot[i] = b.leaf(i);
    int live = np;
    while (live > 1) {
        int bi = -1, bj = -1;
        double best = __builtin_huge_val();
        for (int i = 0; i < (int)slot.size(); i++) {
            if (slot[i] < 0) continue;
            for (int j = 0; j < (int)slot.size(); j++) {
                if (slot[j] < 0 || i == j) continue;
                int x = slot[i], y = slot[j];
                double c = box_sa(box_combine(b.n[x].box, b.n[y].box));
                if (bi < 0 || c < best || (c == best && b.n[x].leaf() && b.n[y].leaf())) { bi = i; bj = j; best = c; }
            }
        }
        int p = b.pair(slot[bi], slot[bj]);
        b.make_parent(p);
        slot[bi] = -1;
        free_slots.push_back(bi);
        slot[bj] = -1;
        free_slots.push_back(bj);
        slot[free_slots.back()] = p;
        free_slots.pop_back();
        live--;
    }
    for (int s : slot)
        if (s >= 0) return s;
    return -1;
}

void flatten(const Builder& b, int i, int depth, RefBvh& out)
{
    out.depth = std::max(out.depth, depth);
    int me = (int)out.nodes.size();
    RefNode r{};
    r.mn = b.n[i].box.mn;
    r.mx = b.n[i].box.mx;
    r.skip = b.n[i].skip ? 1 : 0;
    r.prim = b.n[i].prim;
    r.right = -1;
    out.nodes.push_back(r);
    if (b.n[i].leaf()) return;
    flatten(b, b.n[i].left, depth + 1, out);
    out.nodes[me].right = (int)out.nodes.size();
    flatten(b, b.n[i].right, depth + 1, out);
}

} // namespace

RefBvh build_ref_bvh(const std::vector<HostPrim>& prims)
{
    RefBvh out;
    int np = (int)prims.size();
    if (np == 0) return out;
    Builder b(prims);
    int root = np > 200000 ? build_local(b, np) : np > 20 ? build_heap(b, np) : build_brute(b, np);
    // Iterative flatten would be needed for degenerate deep trees; depth is bounded by np.
    flatten(b, root, 0, out);
    return out;
}

} // namespace rtc
