// oracle_bvh.cpp -- the reference's agglomerative BVH construction and leaf query.
// TEST INFRASTRUCTURE (see oracle.h).  Restates Acceleration/BVH.cs:12-331,
// Acceleration/KDTree.cs:9-453, Acceleration/Heap.cs:9-143 and the .NET Core 3.1
// Array.Sort (introsort) the k-d tree build relies on.  Node identity stands in for the
// reference's structural BVH<T>.Equals: tree elements partition the leaves, so two
// distinct live elements can never be structurally equal.
#include <algorithm>
#include <functional>

#include "oracle_scene.h"

namespace orc {

double BNode::cost()
{
    if (cost_cache == -1) cost_cache = aabb_sa(vol); // BVH.GetCost -> GetSurfaceArea
    return cost_cache;
}

V4 BNode::center(const std::vector<Prim>& prims) const
{
    return leaf ? prims[prim].get_center() : vol.ctr; // BVH.GetCenter (BVH.cs:283-288)
}

// AABB.CreateFromBounded (AABB.cs:22-36)
static AABB aabb_from_prim(const Prim& p)
{
    V4 c = p.get_center();
    V4 lo = v4(p.max_center_distance(v4(-1, 0, 0, 0)), p.max_center_distance(v4(0, -1, 0, 0)),
               p.max_center_distance(v4(0, 0, -1, 0)), 0);
    V4 hi = v4(p.max_center_distance(v4(1, 0, 0, 0)), p.max_center_distance(v4(0, 1, 0, 0)),
               p.max_center_distance(v4(0, 0, 1, 0)), 0);
    return aabb_make(c - lo, c + hi);
}
// AABB.Combine (AABB.cs:38-43)
static AABB aabb_combine(const AABB& a, const AABB& b) { return aabb_make(vmin(a.mn, b.mn), vmax(a.mx, b.mx)); }

// ------------------------------------------------------- .NET introsort ----
template <class T, class Cmp>
struct NetSort {
    std::vector<T>& k;
    Cmp cmp;
    void swap_if_greater(int a, int b)
    {
        if (a != b && cmp(k[a], k[b]) > 0) std::swap(k[a], k[b]);
    }
    void insertion(int lo, int hi)
    {
        for (int i = lo; i < hi; i++) {
            int j = i;
            T t = k[i + 1];
            while (j >= lo && cmp(t, k[j]) < 0) {
                k[j + 1] = k[j];
                j--;
            }
            k[j + 1] = t;
        }
    }
    void down_heap(int i, int n, int lo)
    {
        T d = k[lo + i - 1];
        while (i <= n / 2) {
            int child = 2 * i;
            if (child < n && cmp(k[lo + child - 1], k[lo + child]) < 0) child++;
            if (!(cmp(d, k[lo + child - 1]) < 0)) break;
            k[lo + i - 1] = k[lo + child - 1];
            i = child;
        }
        k[lo + i - 1] = d;
    }
    void heapsort(int lo, int hi)
    {
        int n = hi - lo + 1;
        for (int i = n / 2; i >= 1; i--) down_heap(i, n, lo);
        for (int i = n; i > 1; i--) {
            std::swap(k[lo], k[lo + i - 1]);
            down_heap(1, i - 1, lo);
        }
    }
    int pick_pivot_and_partition(int lo, int hi)
    {
        int mid = lo + ((hi - lo) >> 1);
        swap_if_greater(lo, mid);
        swap_if_greater(lo, hi);
        swap_if_greater(mid, hi);
        T pivot = k[mid];
        std::swap(k[mid], k[hi - 1]);
        int left = lo, right = hi - 1;
        while (left < right) {
            while (cmp(k[++left], pivot) < 0) {
            }
            while (cmp(pivot, k[--right]) < 0) {
            }
            if (left >= right) break;
            std::swap(k[left], k[right]);
        }
        if (left != hi - 1) std::swap(k[left], k[hi - 1]);
        return left;
    }
    void intro(int lo, int hi, int depth)
    {
        while (hi > lo) {
            int size = hi - lo + 1;
            if (size <= 16) {
                if (size == 1) return;
                if (size == 2) {
                    swap_if_greater(lo, hi);
                    return;
                }
                if (size == 3) {
                    swap_if_greater(lo, hi - 1);
                    swap_if_greater(lo, hi);
                    swap_if_greater(hi - 1, hi);
                    return;
                }
                insertion(lo, hi);
                return;
            }
            if (depth == 0) {
                heapsort(lo, hi);
                return;
            }
            depth--;
            int p = pick_pivot_and_partition(lo, hi);
            intro(p + 1, hi, depth);
            hi = p - 1;
        }
    }
    void sort()
    {
        int n = (int)k.size();
        if (n < 2) return;
        int lg = 0;
        for (int m = n; m >= 1; m /= 2) lg++; // FloorLog2PlusOne
        intro(0, n - 1, 2 * lg);
    }
};

// double.CompareTo (NaN sorts first)
static int dcompare(double a, double b)
{
    if (a < b) return -1;
    if (a > b) return 1;
    if (a == b) return 0;
    if (std::isnan(a)) return std::isnan(b) ? 0 : -1;
    return 1;
}
static double axis_of(V4 v, int axis) { return axis == 0 ? v.x : axis == 1 ? v.y : axis == 2 ? v.z : v.w; }

// -------------------------------------------------------------- k-d tree ----
struct KD {
    bool leaf = false;
    int axis = 0;
    double median = 0;
    KD *left = nullptr, *right = nullptr;
    BNode* elem = nullptr;
    V4 ctr{0, 0, 0, 0};
};

struct KDTree {
    std::deque<KD>& pool;
    const std::vector<Prim>& prims;
    KD* root = nullptr;

    KD* make_leaf(BNode* e)
    {
        pool.emplace_back();
        KD* k = &pool.back();
        k->leaf = true;
        k->elem = e;
        k->ctr = e->center(prims);
        return k;
    }
    // KDTree.Construct(set, depth) (KDTree.cs:11-33)
    KD* construct(std::vector<KD*> set, int depth)
    {
        if (set.size() == 1) return set[0];
        int axis = depth % 3;
        auto cmp = [axis](KD* a, KD* b) { return dcompare(axis_of(a->ctr, axis), axis_of(b->ctr, axis)); };
        NetSort<KD*, decltype(cmp)>{set, cmp}.sort();
        size_t half = set.size() / 2;
        std::vector<KD*> l(set.begin(), set.begin() + half), r(set.begin() + half, set.end());
        double median = (axis_of(l.back()->ctr, axis) + axis_of(r[0]->ctr, axis)) / 2;
        KD* a = construct(l, depth + 1);
        KD* b = construct(r, depth + 1);
        pool.emplace_back();
        KD* k = &pool.back();
        k->axis = axis;
        k->median = median;
        k->left = a;
        k->right = b;
        return k;
    }
    static bool contains(const KD* k, const BNode* e, V4 pt) // KDTree.cs:254-268
    {
        if (k->leaf) return e == k->elem;
        double c = axis_of(pt, k->axis);
        if (c <= k->median && contains(k->left, e, pt)) return true;
        if (c >= k->median && contains(k->right, e, pt)) return true;
        return false;
    }
    bool contains(const BNode* e) const { return contains(root, e, e->center(prims)); }
    static void nn(const KD* k, const BNode* e, V4 pt, const KD*& best, double& bd) // KDTree.cs:275-316
    {
        if (k->leaf) {
            if (e != k->elem) {
                double cd = sqlen(k->ctr - pt);
                if (cd < bd) {
                    best = k;
                    bd = cd;
                }
            }
            return;
        }
        double c = axis_of(pt, k->axis);
        const KD *pri, *sec;
        if (c <= k->median) {
            pri = k->left;
            sec = k->right;
        } else {
            pri = k->right;
            sec = k->left;
        }
        nn(pri, e, pt, best, bd);
        double bdist = std::fabs(c - k->median);
        bdist *= bdist;
        if (bdist < bd) nn(sec, e, pt, best, bd);
    }
    BNode* nearest(const BNode* e) const
    {
        const KD* best = nullptr;
        double bd = kInf;
        nn(root, e, e->center(prims), best, bd);
        return best ? best->elem : nullptr;
    }
    static bool get_parent(KD* k, const BNode* e, V4 pt, KD*& parent) // KDTree.cs:364-389
    {
        if (k->leaf) return e == k->elem;
        KD* gp = parent;
        double c = axis_of(pt, k->axis);
        if (c <= k->median) {
            parent = k;
            if (get_parent(k->left, e, pt, parent)) return true;
        }
        if (c >= k->median) {
            parent = k;
            if (get_parent(k->right, e, pt, parent)) return true;
        }
        parent = gp;
        return false;
    }
    void remove(const BNode* e) // KDTree.cs:407-411
    {
        KD* parent = root;
        get_parent(root, e, e->center(prims), parent);
        KD* child = (parent->left->elem == e && parent->left->leaf) ? parent->right : parent->left;
        *parent = *child; // MergeTo -> CopyFrom
    }
    void add(BNode* e) // KDTree.cs:413-453
    {
        KD* parent = root;
        V4 pt = e->center(prims);
        KD* node = root;
        while (!node->leaf) {
            parent = node;
            node = (axis_of(pt, node->axis) <= node->median) ? node->left : node->right;
        }
        int axis = (parent->axis + 1) % 3;
        // SplitWith (KDTree.cs:216-232)
        pool.emplace_back(*node);
        KD* l = &pool.back();
        KD* r = make_leaf(e);
        double lc = axis_of(l->ctr, axis), rc = axis_of(r->ctr, axis);
        double median = (lc + rc) / 2;
        if (lc > rc) std::swap(l, r);
        *node = KD{};
        node->leaf = false;
        node->axis = axis;
        node->median = median;
        node->left = l;
        node->right = r;
    }
};

// ------------------------------------------------------------------ heap ----
struct PairHeap { // Heap<T> (Heap.cs)
    std::vector<BNode*> c;
    static int cmp(BNode* a, BNode* b)
    {
        if (a == b) return 0;
        int k = dcompare(a->cost(), b->cost());
        if (k != 0) return k;
        k = (b->child_leaves() > a->child_leaves()) - (b->child_leaves() < a->child_leaves());
        return k;
    }
    void down(int i)
    {
        while (true) {
            int l = i * 2 + 1, r = l + 1, ch = i;
            if (l < (int)c.size() && cmp(c[ch], c[l]) > 0) ch = l;
            if (r < (int)c.size() && cmp(c[ch], c[r]) > 0) ch = r;
            if (ch == i) break;
            std::swap(c[i], c[ch]);
            i = ch;
        }
    }
    void up(int i)
    {
        BNode* it = c[i];
        int p = (i - 1) / 2;
        while (i != 0 && cmp(it, c[p]) <= 0) {
            c[i] = c[p];
            i = p;
            p = (i - 1) / 2;
        }
        c[i] = it;
    }
    void build()
    {
        for (int i = (int)c.size() / 2 - 1; i >= 0; i--) down(i);
    }
    void add(BNode* n)
    {
        c.push_back(n);
        up((int)c.size() - 1);
    }
    BNode* extract()
    {
        BNode* m = c[0];
        c[0] = c.back();
        c.pop_back();
        down(0);
        return m;
    }
};

// ---------------------------------------------------------------- builders ----
static BNode* new_leaf(std::deque<BNode>& pool, const std::vector<Prim>& prims, int i)
{
    pool.emplace_back();
    BNode* n = &pool.back();
    n->leaf = true;
    n->prim = i;
    n->vol = aabb_from_prim(prims[i]);
    return n;
}
static BNode* new_pair(std::deque<BNode>& pool, BNode* l, BNode* r)
{
    pool.emplace_back();
    BNode* n = &pool.back();
    n->left = l;
    n->right = r;
    n->vol = aabb_combine(l->vol, r->vol);
    return n;
}
static void make_parent(BNode* p) // BVH.MakeParent (BVH.cs:44-48)
{
    p->left->skip = aabb_equals(p->left->vol, p->vol);
    p->right->skip = aabb_equals(p->right->vol, p->vol);
}

static KD* kd_build(KDTree& t, const std::vector<BNode*>& leaves)
{
    std::vector<KD*> set;
    for (BNode* b : leaves) set.push_back(t.make_leaf(b));
    return t.construct(set, 0);
}

static BNode* construct_heap(std::deque<BNode>& pool, const std::vector<Prim>& prims) // BVH.cs:89-191
{
    int n = (int)prims.size();
    std::vector<BNode*> nodes(n);
    for (int i = 0; i < n; i++) nodes[i] = new_leaf(pool, prims, i);
    std::deque<KD> kpool;
    KDTree tree{kpool, prims};
    tree.root = kd_build(tree, nodes);
    PairHeap heap;
    for (int i = 0; i < n; i++) heap.c.push_back(new_pair(pool, nodes[i], tree.nearest(nodes[i])));
    heap.build();
    while (true) {
        BNode* ch = heap.extract();
        if (!tree.contains(ch->left)) continue;
        if (!tree.contains(ch->right)) {
            heap.add(new_pair(pool, ch->left, tree.nearest(ch->left)));
            continue;
        }
        make_parent(ch);
        tree.remove(ch->left);
        if (tree.root->leaf) return ch;
        tree.remove(ch->right);
        tree.add(ch);
        heap.add(new_pair(pool, ch, tree.nearest(ch)));
    }
}

static BNode* construct_local(std::deque<BNode>& pool, const std::vector<Prim>& prims) // BVH.cs:50-87
{
    int n = (int)prims.size();
    std::vector<BNode*> leaves(n);
    for (int i = 0; i < n; i++) leaves[i] = new_leaf(pool, prims, i);
    std::deque<KD> kpool;
    KDTree tree{kpool, prims};
    tree.root = kd_build(tree, leaves);
    BNode* a = leaves[0];
    BNode* b = tree.nearest(a);
    while (true) {
        BNode* c = tree.nearest(b);
        if (a == c) {
            tree.remove(a);
            a = new_pair(pool, a, b);
            make_parent(a);
            if (tree.root->leaf) return a;
            tree.remove(b);
            tree.add(a);
            b = tree.nearest(a);
        } else {
            a = b;
            b = c;
        }
    }
}

static BNode* construct_brute(std::deque<BNode>& pool, const std::vector<Prim>& prims) // BVH.cs:201-235
{
    // HashSet<T> enumeration order: slot order, freed slots reused LIFO.
    int n = (int)prims.size();
    std::vector<BNode*> slots;
    std::vector<int> free_list;
    for (int i = 0; i < n; i++) slots.push_back(new_leaf(pool, prims, i));
    int count = n;
    while (count > 1) {
        int bi = -1, bj = -1;
        double best = kInf;
        for (int i = 0; i < (int)slots.size(); i++) {
            if (!slots[i]) continue;
            for (int j = 0; j < (int)slots.size(); j++) {
                if (!slots[j] || i == j) continue;
                BNode *a = slots[i], *b = slots[j];
                double c = aabb_sa(aabb_combine(a->vol, b->vol));
                if (bi < 0 || c < best || (c == best && a->leaf && b->leaf)) {
                    bi = i;
                    bj = j;
                    best = c;
                }
            }
        }
        BNode *a = slots[bi], *b = slots[bj];
        slots[bi] = nullptr;
        free_list.push_back(bi);
        slots[bj] = nullptr;
        free_list.push_back(bj);
        BNode* p = new_pair(pool, a, b);
        make_parent(p);
        int s = free_list.back();
        free_list.pop_back();
        slots[s] = p;
        count--;
    }
    for (BNode* s : slots)
        if (s) return s;
    return nullptr;
}

void Scene::prepare()
{
    pool.clear();
    root = nullptr;
    int n = (int)prims.size();
    if (n == 0) return;
    if (n > 200000)
        root = construct_local(pool, prims);
    else if (n > 20)
        root = construct_heap(pool, prims);
    else
        root = construct_brute(pool, prims);
}

// BVH<T>.IntersectLeaves (BVH.cs:295-331): every pierced leaf, DFS order, then the stable
// insertion sort by Near (Util.InsertSort, Util.cs:262-280).
static void intersect_leaves(const BNode* n, const Ray& r, std::vector<Leaf>& out, double nr, double fr)
{
    if (!n->skip) {
        aabb_intersect(n->vol, r, nr, fr);
        if (!(fr >= 0)) return;
    }
    if (n->leaf) {
        out.push_back(Leaf{n, nr, fr});
        return;
    }
    intersect_leaves(n->left, r, out, nr, fr);
    intersect_leaves(n->right, r, out, nr, fr);
}

// Scene.RayTracePrimitives BVH branch (Scene.cs:65-92).
Hit Scene::raytrace(const Ray& r, const Hit* skip, std::vector<Leaf>& list) const
{
    Hit hit;
    if (!root) return hit;
    list.clear();
    intersect_leaves(root, r, list, 0, 0);
    for (int i = 1; i < (int)list.size(); i++) {
        Leaf a = list[i];
        int j = i - 1;
        while (j >= 0 && dcompare(a.near_, list[j].near_) < 0) {
            list[j + 1] = list[j];
            j--;
        }
        list[j + 1] = a;
    }
    const Leaf* prev = nullptr;
    for (const Leaf& cur : list) {
        if (prev && cur.near_ > prev->far_) break;
        Hit h = prim_raytrace(prims[cur.node->prim], r, skip);
        if (h.prim >= 0 && (hit.prim < 0 || h.dist < hit.dist)) {
            hit = h;
            prev = &cur;
        }
    }
    return hit;
}

} // namespace orc
