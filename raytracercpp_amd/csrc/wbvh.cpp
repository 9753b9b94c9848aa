// wbvh.cpp -- host build of the 4-wide SAH BVH (wbvh.hpp) over the octree's triangle
// records: binned SAH binary tree (16 bins per axis, parallel over subtrees), collapsed
// to 4-wide nodes by repeatedly opening the child with the largest surface area.
#include "wbvh.hpp"
#include "pool.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>

#include <emmintrin.h>   // SSE2 (x86-64 baseline): the builder's box min / max four lanes at a time

namespace rt {

namespace {

struct Box {
    float lo[3], hi[3];
};

inline Box empty_box() { return Box{{INFINITY, INFINITY, INFINITY}, {-INFINITY, -INFINITY, -INFINITY}}; }
inline void grow(Box& b, const Box& o)
{
    for (int a = 0; a < 3; a++) {
        b.lo[a] = std::min(b.lo[a], o.lo[a]);
        b.hi[a] = std::max(b.hi[a], o.hi[a]);
    }
}
inline float area(const Box& b)
{
    float dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
    if (!(dx >= 0 && dy >= 0 && dz >= 0))
        return 0.0f;
    return 2.0f * (dx * dy + dy * dz + dz * dx);
}

// float lower / upper bound of a double
inline float down(double x)
{
    float f = (float)x;
    return (double)f > x ? std::nextafter(f, -INFINITY) : f;
}
inline float up(double x)
{
    float f = (float)x;
    return (double)f < x ? std::nextafter(f, INFINITY) : f;
}

// the box of a record's vertices a, a + ab, a + ac (exact sums in double, rounded outward)
Box tri_box(const GTri& g)
{
    Box b;
    for (int c = 0; c < 3; c++) {
        double a = g.a[c], p = a + (double)g.ab[c], q = a + (double)g.ac[c];
        b.lo[c] = down(std::min(a, std::min(p, q)));
        b.hi[c] = up(std::max(a, std::max(p, q)));
    }
    return b;
}

struct BNode {
    Box box;
    int32_t left, right;   // left < 0: leaf
    int32_t first, count;  // primitives [first, first + count) of the final order
    double ns[3];          // sum of the subtree's stored triangle normals (the slab normal, wbvh.hpp)
};

// A primitive during the build: its box (a record's vertices, rounded outward) and the
// octree slot it came from; its centroid is 0.5 lo + 0.5 hi.  The builder partitions these
// 32-B records in place, so every level of the build reads them sequentially, and keeps
// boxes in SSE registers (lane 3 unused).
struct alignas(16) Prim {
    float lo[3];
    int32_t id;
    float hi[3];
    float pad;
};
inline __m128 plo(const Prim& p) { return _mm_load_ps(p.lo); }
inline __m128 phi(const Prim& p) { return _mm_load_ps(p.hi); }
// (lane 3 of lo holds the id's bits -- a denormal as a float, slow in arithmetic: masked out)
inline __m128 pcen(const Prim& p)
{
    const __m128 xyz = _mm_castsi128_ps(_mm_setr_epi32(-1, -1, -1, 0));
    return _mm_add_ps(_mm_mul_ps(_mm_and_ps(plo(p), xyz), _mm_set1_ps(0.5f)), _mm_mul_ps(phi(p), _mm_set1_ps(0.5f)));
}

// a box as two SSE registers (lane 3 ignored)
struct VBox {
    __m128 lo, hi;
    static VBox empty() { return VBox{_mm_set1_ps(INFINITY), _mm_set1_ps(-INFINITY)}; }
    void grow(__m128 l, __m128 h)
    {
        lo = _mm_min_ps(lo, l);
        hi = _mm_max_ps(hi, h);
    }
    void grow(const VBox& o) { grow(o.lo, o.hi); }
    Box box() const
    {
        alignas(16) float l[4], h[4];
        _mm_store_ps(l, lo);
        _mm_store_ps(h, hi);
        return Box{{l[0], l[1], l[2]}, {h[0], h[1], h[2]}};
    }
    static VBox of(const Box& b)
    {
        return VBox{_mm_setr_ps(b.lo[0], b.lo[1], b.lo[2], 0.0f), _mm_setr_ps(b.hi[0], b.hi[1], b.hi[2], 0.0f)};
    }
};

constexpr int NBINS = 16;
constexpr int32_t PAR_BIN = 1 << 14;   // nodes with more primitives are binned and partitioned by every thread
constexpr int32_t PAR_CHUNK = 1 << 13; // primitives per chunk of a cooperative pass

struct Bins {
    int32_t cnt[3][NBINS];
    VBox box[3][NBINS];
    void clear()
    {
        for (int a = 0; a < 3; a++)
            for (int i = 0; i < NBINS; i++) {
                cnt[a][i] = 0;
                box[a][i] = VBox::empty();
            }
    }
    void add(const Bins& o)
    {
        for (int a = 0; a < 3; a++)
            for (int i = 0; i < NBINS; i++) {
                cnt[a][i] += o.cnt[a][i];
                box[a][i].grow(o.box[a][i]);
            }
    }
};

inline int bin_of(float c, float lo, float scale)
{
    int k = (int)((c - lo) * scale);
    return k < 0 ? 0 : (k >= NBINS ? NBINS - 1 : k);
}
// the three axes' bins of a centroid at once: trunc(clamp((c - lo) scale, 0, NBINS - 1)), the
// same integers as bin_of (no NaN: the triangles are finite)
inline __m128i bins_of(__m128 c, __m128 lo, __m128 scale)
{
    __m128 k = _mm_mul_ps(_mm_sub_ps(c, lo), scale);
    k = _mm_min_ps(_mm_max_ps(k, _mm_setzero_ps()), _mm_set1_ps((float)(NBINS - 1)));
    return _mm_cvttps_epi32(k);
}
inline float lane(__m128 v, int a)
{
    alignas(16) float f[4];
    _mm_store_ps(f, v);
    return f[a];
}

// Binned SAH (16 bins per axis) over the primitive records; the children's boxes and centroid
// boxes come out of the partition pass, so no node re-reads its primitives for its bounds.
struct Builder {
    std::vector<Prim, DefaultInitAlloc<Prim>>& P;
    std::vector<Prim, DefaultInitAlloc<Prim>>& tmp;
    std::vector<BNode, DefaultInitAlloc<BNode>>& nodes;    // preallocated, 2n - 1 nodes at most
    const GTri* tris;             // octree records by slot (leaf normal sums)
    Pool& pool;
    int32_t next = 1;             // the cooperative phase's node counter (one thread)
    float ct = 1.0f;              // SAH cost of a node visit, in triangle tests (r02: 2 and 3 were slower)
    int32_t maxleaf = W_MAX_LEAF; // primitives per leaf at most
    struct Task {
        int32_t ni, b, e;
        Box box, cbox;
        double sah;      // sum of (leaf ? count : 1) x area over the subtree's nodes
    };
    double sah_big = 0;
    std::vector<Task> tasks;      // subtrees below PAR_BIN, built one per thread
    std::vector<int32_t> big;     // nodes built cooperatively (their normal sums are filled last)

    Builder(std::vector<Prim, DefaultInitAlloc<Prim>>& p, std::vector<Prim, DefaultInitAlloc<Prim>>& t,
            std::vector<BNode, DefaultInitAlloc<BNode>>& n, const GTri* tr, Pool& pl)
        : P(p), tmp(t), nodes(n), tris(tr), pool(pl)
    {
    }

    // best split of a node from its bins: axis (-1: none), bin, cost
    void best_split(const Bins& B, const float* scale, const Box& box, int& axis, int& split, float& cost) const
    {
        axis = split = -1;
        cost = INFINITY;
        const float pa = area(box);
        for (int a = 0; a < 3; a++) {
            if (scale[a] == 0.0f)
                continue;
            float ra[NBINS];
            int32_t rc[NBINS];
            Box acc = empty_box();
            int32_t c = 0;
            for (int i = NBINS - 1; i >= 1; i--) {
                grow(acc, B.box[a][i].box());
                c += B.cnt[a][i];
                ra[i] = area(acc);
                rc[i] = c;
            }
            acc = empty_box();
            c = 0;
            for (int i = 0; i < NBINS - 1; i++) {
                grow(acc, B.box[a][i].box());
                c += B.cnt[a][i];
                if (c == 0 || rc[i + 1] == 0)
                    continue;
                float k = ct + (area(acc) * (float)c + ra[i + 1] * (float)rc[i + 1]) / (pa > 0 ? pa : 1.0f);
                if (k < cost) {
                    cost = k;
                    axis = a;
                    split = i;
                }
            }
        }
    }

    static void bin_range(const Prim* p, int32_t n, const float* clo, const float* scale, Bins& B)
    {
        const __m128 lo = _mm_setr_ps(clo[0], clo[1], clo[2], 0.0f), sc = _mm_setr_ps(scale[0], scale[1], scale[2], 0.0f);
        for (int32_t i = 0; i < n; i++) {
            const Prim& q = p[i];
            const __m128 l = plo(q), h = phi(q);
            alignas(16) int32_t k[4];
            _mm_store_si128(reinterpret_cast<__m128i*>(k), bins_of(pcen(q), lo, sc));
            for (int a = 0; a < 3; a++) {
                B.cnt[a][k[a]]++;
                B.box[a][k[a]].grow(l, h);
            }
        }
    }

    // is primitive i left of the split (axis >= 0), or in the first half (axis < 0)
    struct Pred {
        int axis, split;
        float lo, sc;
        bool operator()(const Prim& q) const { return bin_of(lane(pcen(q), axis), lo, sc) <= split; }
    };

    void make_leaf(BNode& N) const
    {
        N.left = N.right = -1;
        N.ns[0] = N.ns[1] = N.ns[2] = 0.0;
        for (int32_t i = N.first; i < N.first + N.count; i++) {
            const GTri& t = tris[(size_t)P[(size_t)i].id];
            for (int a = 0; a < 3; a++)
                N.ns[a] += t.n[a];
        }
    }

    // the split decision shared by both build paths: false -> the node is a leaf; else the
    // predicate's axis / bin (axis -1: halves in order)
    bool decide(int32_t n, const Box& box, const Box& cb, float* scale, Bins* B, int& axis, int& split)
    {
        bool any = false;
        for (int a = 0; a < 3; a++) {
            const float ext = cb.hi[a] - cb.lo[a];
            scale[a] = ext > 0 ? (float)NBINS / ext : 0.0f;
            any |= ext > 0;
        }
        axis = split = -1;
        if (n <= 1)
            return false;
        if (!any)
            return n > maxleaf;   // every centroid equal: halves in order
        float cost;
        best_split(*B, scale, box, axis, split, cost);
        if (axis >= 0 && n <= maxleaf && (float)n <= cost)
            return false;   // a leaf is no more expensive than the best split
        if (axis < 0)
            return n > maxleaf;
        return true;
    }

    // serial subtree build (a task); its nodes' normal sums post-order.  Node indices come from
    // the task's own counter (a region of its own: no shared atomic per node).
    void build_serial(int32_t ni, int32_t b, int32_t e, const Box& box, const Box& cb, int32_t& alloc, double& sah)
    {
        BNode& N = nodes[(size_t)ni];
        const int32_t n = e - b;
        N.box = box;
        N.first = b;
        N.count = n;
        float scale[3];
        Bins B;
        bool anyext = false;
        for (int a = 0; a < 3; a++)
            anyext |= cb.hi[a] - cb.lo[a] > 0;
        if (n > 1 && anyext) {
            for (int a = 0; a < 3; a++) {
                const float ext = cb.hi[a] - cb.lo[a];
                scale[a] = ext > 0 ? (float)NBINS / ext : 0.0f;
            }
            B.clear();
            bin_range(&P[(size_t)b], n, cb.lo, scale, B);
        }
        int axis, split;
        if (!decide(n, box, cb, scale, &B, axis, split)) {
            make_leaf(N);
            sah += (double)n * area(box);
            return;
        }
        sah += area(box);
        // partition (two-sided, every primitive visited once) with the children's bounds
        VBox lb = VBox::empty(), lc = VBox::empty(), rb = VBox::empty(), rc = VBox::empty();
        int32_t mid;
        if (axis >= 0) {
            const Pred left{axis, split, cb.lo[axis], scale[axis]};
            int32_t i = b, j = e - 1;
            for (;;) {
                while (i <= j && left(P[(size_t)i])) {
                    lb.grow(plo(P[(size_t)i]), phi(P[(size_t)i]));
                    const __m128 c = pcen(P[(size_t)i]);
                    lc.grow(c, c);
                    i++;
                }
                while (i <= j && !left(P[(size_t)j])) {
                    rb.grow(plo(P[(size_t)j]), phi(P[(size_t)j]));
                    const __m128 c = pcen(P[(size_t)j]);
                    rc.grow(c, c);
                    j--;
                }
                if (i >= j)
                    break;
                std::swap(P[(size_t)i], P[(size_t)j]);
            }
            mid = i;
        } else
            mid = b + n / 2;
        if (mid == b || mid == e || axis < 0) {
            mid = b + n / 2;
            lb = lc = rb = rc = VBox::empty();
            for (int32_t i = b; i < e; i++) {
                VBox& bb = i < mid ? lb : rb;
                VBox& cc = i < mid ? lc : rc;
                bb.grow(plo(P[(size_t)i]), phi(P[(size_t)i]));
                const __m128 c = pcen(P[(size_t)i]);
                cc.grow(c, c);
            }
        }
        const int32_t l = alloc;
        alloc += 2;
        N.left = l;
        N.right = l + 1;
        build_serial(l, b, mid, lb.box(), lc.box(), alloc, sah);
        build_serial(l + 1, mid, e, rb.box(), rc.box(), alloc, sah);
        const BNode &L = nodes[(size_t)l], &R = nodes[(size_t)l + 1];
        for (int a = 0; a < 3; a++)
            nodes[(size_t)ni].ns[a] = L.ns[a] + R.ns[a];
    }

    // cooperative build of the large nodes: binning and a stable partition (through tmp) by
    // every thread; subtrees below PAR_BIN become tasks
    void build_big(int32_t ni, int32_t b, int32_t e, const Box& box, const Box& cb)
    {
        const int32_t n = e - b;
        if (n < PAR_BIN) {
            tasks.push_back(Task{ni, b, e, box, cb, 0.0});
            return;
        }
        big.push_back(ni);
        sah_big += area(box);
        BNode& N = nodes[(size_t)ni];
        N.box = box;
        N.first = b;
        N.count = n;
        float scale[3];
        for (int a = 0; a < 3; a++) {
            const float ext = cb.hi[a] - cb.lo[a];
            scale[a] = ext > 0 ? (float)NBINS / ext : 0.0f;
        }
        const int32_t nch = (n + PAR_CHUNK - 1) / PAR_CHUNK;
        std::vector<Bins> part((size_t)nch);
        parallel_for(pool, nch, 1, [&](int64_t k) {
            const int32_t cb0 = b + (int32_t)k * PAR_CHUNK, ce = std::min(e, cb0 + PAR_CHUNK);
            part[(size_t)k].clear();
            bin_range(&P[(size_t)cb0], ce - cb0, cb.lo, scale, part[(size_t)k]);
        });
        Bins B = part[0];
        for (int32_t k = 1; k < nch; k++)
            B.add(part[(size_t)k]);
        int axis, split;
        if (!decide(n, box, cb, scale, &B, axis, split)) {
            make_leaf(N);   // (never for n >= PAR_BIN > W_MAX_LEAF)
            return;
        }
        // stable partition: per chunk, the count going left and both sides' bounds
        struct Side {
            int32_t nl;
            VBox lb, lc, rb, rc;
        };
        std::vector<Side> side((size_t)nch);
        const Pred pred{axis, split, axis >= 0 ? cb.lo[axis] : 0.0f, axis >= 0 ? scale[axis] : 0.0f};
        const int32_t half = b + n / 2;
        auto left_of = [&](int32_t i) { return axis >= 0 ? pred(P[(size_t)i]) : i < half; };
        auto sides = [&](bool halves) {
            parallel_for(pool, nch, 1, [&](int64_t k) {
                const int32_t c0 = b + (int32_t)k * PAR_CHUNK, c1 = std::min(e, c0 + PAR_CHUNK);
                Side& S = side[(size_t)k];
                S.nl = 0;
                S.lb = S.lc = S.rb = S.rc = VBox::empty();
                for (int32_t i = c0; i < c1; i++) {
                    const bool l = halves ? i < half : left_of(i);
                    S.nl += l;
                    const __m128 c = pcen(P[(size_t)i]);
                    (l ? S.lb : S.rb).grow(plo(P[(size_t)i]), phi(P[(size_t)i]));
                    (l ? S.lc : S.rc).grow(c, c);
                }
            });
        };
        sides(false);
        std::vector<int32_t> loff((size_t)nch), roff((size_t)nch);
        int32_t nl = 0;
        for (int32_t k = 0; k < nch; k++) {
            loff[(size_t)k] = nl;
            nl += side[(size_t)k].nl;
        }
        if (nl == 0 || nl == n) {
            sides(true);   // a degenerate split: halves in order
            nl = n / 2;
        } else {
            int32_t nr = 0;
            for (int32_t k = 0; k < nch; k++) {
                roff[(size_t)k] = nl + nr;
                nr += std::min(e, b + (k + 1) * PAR_CHUNK) - (b + k * PAR_CHUNK) - side[(size_t)k].nl;
            }
            parallel_for(pool, nch, 1, [&](int64_t k) {
                const int32_t c0 = b + (int32_t)k * PAR_CHUNK, c1 = std::min(e, c0 + PAR_CHUNK);
                int32_t li = b + loff[(size_t)k], ri = b + roff[(size_t)k];
                for (int32_t i = c0; i < c1; i++)
                    tmp[(size_t)(left_of(i) ? li++ : ri++)] = P[(size_t)i];
            });
            parallel_for(pool, nch, 1, [&](int64_t k) {
                const int32_t c0 = b + (int32_t)k * PAR_CHUNK, c1 = std::min(e, c0 + PAR_CHUNK);
                std::copy(tmp.begin() + c0, tmp.begin() + c1, P.begin() + c0);
            });
        }
        VBox lb = VBox::empty(), lc = VBox::empty(), rb = VBox::empty(), rc = VBox::empty();
        for (const Side& S : side) {
            lb.grow(S.lb);
            lc.grow(S.lc);
            rb.grow(S.rb);
            rc.grow(S.rc);
        }
        const int32_t mid = b + nl;
        const int32_t l = next;
        next += 2;
        N.left = l;
        N.right = l + 1;
        build_big(l, b, mid, lb.box(), lc.box());
        build_big(l + 1, mid, e, rb.box(), rc.box());
    }

    void run(int32_t n)
    {
        VBox vb = VBox::empty(), vc = VBox::empty();
        {
            const int32_t nch = (n + PAR_CHUNK - 1) / PAR_CHUNK;
            std::vector<VBox> pb((size_t)nch), pc((size_t)nch);
            parallel_for(pool, nch, 1, [&](int64_t k) {
                const int32_t c0 = (int32_t)k * PAR_CHUNK, c1 = std::min(n, c0 + PAR_CHUNK);
                VBox a = VBox::empty(), c = VBox::empty();
                for (int32_t i = c0; i < c1; i++) {
                    a.grow(plo(P[(size_t)i]), phi(P[(size_t)i]));
                    const __m128 q = pcen(P[(size_t)i]);
                    c.grow(q, q);
                }
                pb[(size_t)k] = a;
                pc[(size_t)k] = c;
            });
            for (int32_t k = 0; k < nch; k++) {
                vb.grow(pb[(size_t)k]);
                vc.grow(pc[(size_t)k]);
            }
        }
        const Box box = vb.box(), cb = vc.box();
        build_big(0, 0, n, box, cb);
        if (std::getenv("RT_BUILD_PROFILE"))
            fprintf(stderr, "[wbvh]   cooperative part done: %zu big nodes, %zu tasks\n", big.size(), tasks.size());
        auto tt0 = std::chrono::steady_clock::now();
        // the subtrees, largest first, one per thread at a time; the task over primitives [b, e)
        // allocates its nodes from [next + 2 b, next + 2 e) (a subtree of m primitives has 2 m - 1
        // nodes at most, its root allocated above)
        if (nodes.size() < (size_t)next + 2 * (size_t)n)   // (only after many uneven cooperative splits)
            nodes.resize((size_t)next + 2 * (size_t)n);
        std::sort(tasks.begin(), tasks.end(), [](const Task& x, const Task& y) { return x.e - x.b > y.e - y.b; });
        std::atomic<size_t> ti{0};
        const int32_t base = next;
        pool.run([&](int) {
            for (;;) {
                const size_t k = ti.fetch_add(1);
                if (k >= tasks.size())
                    return;
                Task& T = tasks[k];
                int32_t alloc = base + 2 * T.b;
                build_serial(T.ni, T.b, T.e, T.box, T.cbox, alloc, T.sah);
            }
        });
        if (std::getenv("RT_BUILD_PROFILE"))
            fprintf(stderr, "[wbvh]   tasks %.2f ms\n",
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tt0).count());
        // the cooperative nodes' normal sums, children before parents (they were pushed top-down)
        for (size_t k = big.size(); k-- > 0;) {
            BNode& N = nodes[(size_t)big[k]];
            if (N.left < 0)
                continue;
            for (int a = 0; a < 3; a++)
                N.ns[a] = nodes[(size_t)N.left].ns[a] + nodes[(size_t)N.right].ns[a];
        }
    }
};

// The conditioning bytes (wbvh.hpp wq_val): the largest code whose value is <= x (a lower
// bound on a sine in [0, 1]), and the smallest code whose value is >= x (an upper bound; for
// lengths 255 = no bound).
uint32_t wq_code_lb(double x)
{
    if (!(x > 0))
        return 0u;
    if (x >= 1)
        return 255u;
    float f = (float)x;
    if ((double)f > x)
        f = std::nextafter(f, 0.0f);
    uint32_t bits;
    std::memcpy(&bits, &f, 4);
    if (bits < WQ_UNIT + (1u << 20))
        return 0u;
    const uint32_t k = (bits - WQ_UNIT) >> 20;
    return k > 255u ? 255u : k;
}

uint32_t wq_code_ub(double x, uint32_t base)
{
    if (!(x > 0))
        return x == 0 ? 0u : 255u;   // (NaN: no bound)
    float f = (float)x;
    if ((double)f < x)
        f = std::nextafter(f, INFINITY);
    uint32_t bits;
    std::memcpy(&bits, &f, 4);
    if (bits <= base + (1u << 20))
        return 1u;
    const uint32_t k = (bits - base + (1u << 20) - 1u) >> 20;
    if (base == WQ_UNIT)
        return k > 255u ? 255u : k;
    return k > 254u ? 255u : k;
}

// One 4-wide node: the children's float boxes quantised to 8 bits per plane against the
// node box's low corner, low planes rounded down and high planes up (exact in double:
// origin, q and the power-of-two step are all representable), so each decoded box holds
// its float box.
// Per child: the sum of its subtree's stored triangle normals (for the orientation slab's
// normal, wbvh.hpp) and its triangles [first, first + count) of the final order.
struct ChildGeom {
    double n[3];
    int32_t first, count;
};

// Per triangle of the final order, for the cone codes: the unit normal in double, or a flag.
struct UnitN {
    double u[3];
    int state;   // 0: |n| in (1e-30, 1e27); 1: n = 0 (never hit: Mdet = 0); 2: out of range (no cone)
};

// Backface cone code of a child (wbvh.hpp): theta = the largest angle between N and a triangle
// normal n below (triangles with n = 0 never hit: Mdet = 0); a ray with angle(N, d) < psi =
// acos(eps) - theta has angle(n, d) < acos(eps) for every n, i.e. exact n . d > eps |n| |d|,
// and the float Mdet = n . (-d) is then negative (its rounding is below 2^-22 |n| |d| for |n|
// in (1e-30, 1e27)).  cos(angle(N, d)) > cos psi  <=>  N . d > cos(psi) |N| |d|: the code is
// the threshold cos(psi) |N| + 0.01 (the kernel's rounding margin) rounded up in steps of
// W_CONE_STEP; 255 = no cone (psi <= 0, or a normal out of range).  The largest angle is the
// arccosine of the smallest cosine.
int cone_code(const int* nq, const ChildGeom& g, const UnitN* un)
{
    const double Nl = std::sqrt((double)nq[0] * nq[0] + (double)nq[1] * nq[1] + (double)nq[2] * nq[2]);
    double cmin = 1.0;
    for (int32_t i = g.first; i < g.first + g.count; i++) {
        const UnitN& t = un[i];
        if (t.state == 1)
            continue;
        if (t.state == 2)
            return 255;
        cmin = std::min(cmin, (t.u[0] * nq[0] + t.u[1] * nq[1] + t.u[2] * nq[2]) / Nl);
    }
    const double theta = std::acos(std::max(-1.0, std::min(1.0, cmin)));
    const double psi = std::acos(W_CONE_EPS) - theta - 1e-9;
    if (!(psi > 0))
        return 255;
    const double code = std::ceil((std::cos(psi) * Nl + 0.01) / ((double)W_CONE_STEP * (1 - 1e-9)));
    return code <= 254 ? (int)code : 255;
}

WNode quantise(const Box* cb, const uint32_t* link, int nc, const ChildGeom* cg, const GTri* tris, const UnitN* un)
{
    WNode w;
    std::memset(&w, 0, sizeof(w));
    Box nb = empty_box();
    for (int j = 0; j < nc; j++)
        grow(nb, cb[j]);
    const float org[3] = {nb.lo[0], nb.lo[1], nb.lo[2]};
    w.ox = org[0];
    w.oy = org[1];
    w.oz = org[2];
    w.exps = 0;
    for (int a = 0; a < 3; a++) {
        const double ext = (double)nb.hi[a] - (double)org[a];
        int k = -100;
        if (ext > 0) {
            int e;
            std::frexp(ext / 255.0, &e);   // ext / 255 <= 2^e
            k = std::max(-100, std::min(127, e - 1));
            while (k < 127 && std::ldexp(255.0, k) < ext)
                k++;
        }
        w.exps |= (uint32_t)(127 + k) << (8 * a);
        const double st = std::ldexp(1.0, k);
        for (int j = 0; j < W_WIDTH; j++) {
            if (j >= nc) {
                w.qlo[a][j] = 0;
                w.qhi[a][j] = 0;
                continue;
            }
            double lo = std::floor(((double)cb[j].lo[a] - org[a]) / st);
            double hi = std::ceil(((double)cb[j].hi[a] - org[a]) / st);
            w.qlo[a][j] = (uint8_t)std::max(0.0, std::min(255.0, lo));
            w.qhi[a][j] = (uint8_t)std::max(0.0, std::min(255.0, hi));
        }
    }
    for (int j = 0; j < W_WIDTH; j++)
        w.child[j] = link[j];
    // slabs: N_j = round(127 n / |n|) (integer), range of N_j . (v - origin) over the vertices
    // in double (exact: integer N, float vertices and origin), quantised outward on 16 bits
    double smin[W_WIDTH], smax[W_WIDTH];
    int nq[W_WIDTH][3];
    double lo_all = INFINITY, hi_all = -INFINITY;
    for (int j = 0; j < nc; j++) {
        const ChildGeom& g = cg[j];
        double len = std::sqrt(g.n[0] * g.n[0] + g.n[1] * g.n[1] + g.n[2] * g.n[2]);
        for (int a = 0; a < 3; a++)
            nq[j][a] = len > 0 ? (int)std::lround(127.0 * g.n[a] / len) : (a == 0 ? 1 : 0);
        if (nq[j][0] == 0 && nq[j][1] == 0 && nq[j][2] == 0)
            nq[j][0] = 1;
        const double n0 = nq[j][0], n1 = nq[j][1], n2 = nq[j][2];
        const double o0 = org[0], o1 = org[1], o2 = org[2];
        double mn = INFINITY, mx = -INFINITY;
        for (int32_t i = g.first; i < g.first + g.count; i++) {
            const GTri& t = tris[(size_t)i];
            const double a0 = t.a[0], a1 = t.a[1], a2 = t.a[2];
            const double s0 = n0 * (a0 - o0) + n1 * (a1 - o1) + n2 * (a2 - o2);
            const double s1 = n0 * ((a0 + (double)t.ab[0]) - o0) + n1 * ((a1 + (double)t.ab[1]) - o1) +
                              n2 * ((a2 + (double)t.ab[2]) - o2);
            const double s2 = n0 * ((a0 + (double)t.ac[0]) - o0) + n1 * ((a1 + (double)t.ac[1]) - o1) +
                              n2 * ((a2 + (double)t.ac[2]) - o2);
            mn = std::min(mn, std::min(s0, std::min(s1, s2)));
            mx = std::max(mx, std::max(s0, std::max(s1, s2)));
        }
        smin[j] = mn;
        smax[j] = mx;
        lo_all = std::min(lo_all, smin[j]);
        hi_all = std::max(hi_all, smax[j]);
    }
    // slo: a float at or below every smin; s: a power of two with 65535 s covering the range
    float slo = down(lo_all);
    double ext = hi_all - (double)slo;
    int k = -100;
    if (ext > 0) {
        int e;
        std::frexp(ext / 65535.0, &e);
        k = std::max(-100, std::min(127, e - 1));
        while (k < 127 && std::ldexp(65535.0, k) < ext)
            k++;
    }
    const double st = std::ldexp(1.0, k);
    w.s = (float)st;
    w.slo = slo;
    for (int j = 0; j < W_WIDTH; j++) {
        if (j >= nc) {
            w.nrm[j] = 0;
            w.slab[j] = 0;
            continue;
        }
        // signed bytes (two's complement), the cone code in byte 3
        w.nrm[j] = (uint32_t)(uint8_t)(int8_t)nq[j][0] | ((uint32_t)(uint8_t)(int8_t)nq[j][1] << 8) |
                   ((uint32_t)(uint8_t)(int8_t)nq[j][2] << 16) | ((uint32_t)cone_code(nq[j], cg[j], un) << 24);
        double q0 = std::floor((smin[j] - (double)slo) / st), q1 = std::ceil((smax[j] - (double)slo) / st);
        q0 = std::max(0.0, std::min(65535.0, q0));
        q1 = std::max(0.0, std::min(65535.0, q1));
        w.slab[j] = (uint32_t)q0 | ((uint32_t)q1 << 16);
    }
    return w;
}

// the decoded box of child j (double, exact)
Box decode(const WNode& w, int j, double lo[3], double hi[3])
{
    const float org[3] = {w.ox, w.oy, w.oz};
    Box b;
    for (int a = 0; a < 3; a++) {
        const double st = std::ldexp(1.0, (int)((w.exps >> (8 * a)) & 0xffu) - 127);
        lo[a] = org[a] + w.qlo[a][j] * st;
        hi[a] = org[a] + w.qhi[a][j] * st;
        b.lo[a] = down(lo[a]);
        b.hi[a] = up(hi[a]);
    }
    return b;
}

// The 4-wide topology: each wide node opens the binary child with the largest surface area
// until it has four children (leaves stay leaves).  The top of the tree is planned on one
// thread; subtrees of at most PLAN_CUT triangles are planned in parallel, each in depth-first
// preorder into a contiguous range of wide nodes after the top ones.  The geometry (quantise)
// of every wide node is computed afterwards, in parallel.
constexpr int32_t PLAN_CUT = 1 << 12;

struct Planner {
    const std::vector<BNode, DefaultInitAlloc<BNode>>& bn;
    struct Plan {
        int32_t c[W_WIDTH];   // binary nodes of the children
        uint32_t link[W_WIDTH];
        int nc;
    };
    struct Stats {
        int64_t leaves = 0, max_leaf = 0, max_depth = 0;
        void add(const Stats& o)
        {
            leaves += o.leaves;
            max_leaf = std::max(max_leaf, o.max_leaf);
            max_depth = std::max(max_depth, o.max_depth);
        }
    };
    struct Cut {
        int32_t bi;       // the subtree's binary root
        uint32_t node;    // the top wide node linking to it ...
        int j;            // ... through its child j
        int depth;
        std::vector<Plan> local;
        Stats st;
    };
    std::vector<Plan> plans;
    std::vector<Cut> cuts;
    Stats st;

    // the children of the wide node for binary node bi
    void open(int32_t bi, Plan& p) const
    {
        p.nc = 0;
        const BNode& N = bn[(size_t)bi];
        if (N.left < 0) {
            p.c[p.nc++] = bi;   // a leaf root: one child
            return;
        }
        p.c[p.nc++] = N.left;
        p.c[p.nc++] = N.right;
        while (p.nc < W_WIDTH) {
            int pick = -1;
            float pa = -1.0f;
            for (int j = 0; j < p.nc; j++) {
                const BNode& C = bn[(size_t)p.c[j]];
                if (C.left >= 0 && area(C.box) > pa) {
                    pa = area(C.box);
                    pick = j;
                }
            }
            if (pick < 0)
                break;
            const BNode& C = bn[(size_t)p.c[pick]];
            p.c[pick] = C.left;
            p.c[p.nc++] = C.right;
        }
    }

    // plan the subtree of binary node bi into 'out' (indices local to it); top: children of at
    // most PLAN_CUT triangles become cuts instead of being planned here
    uint32_t plan(int32_t bi, int depth, std::vector<Plan>& out, Stats& s, bool top)
    {
        s.max_depth = std::max<int64_t>(s.max_depth, depth);
        Plan p;
        open(bi, p);
        const uint32_t me = (uint32_t)out.size();
        out.push_back(p);
        uint32_t link[W_WIDTH];
        for (int j = 0; j < W_WIDTH; j++)
            link[j] = W_EMPTY;
        for (int j = 0; j < p.nc; j++) {
            const BNode& C = bn[(size_t)p.c[j]];
            if (C.left < 0) {
                link[j] = W_LEAF | ((uint32_t)C.first << 3) | (uint32_t)(C.count - 1);
                s.leaves++;
                s.max_leaf = std::max<int64_t>(s.max_leaf, C.count);
            } else if (top && C.count <= PLAN_CUT) {
                cuts.push_back(Cut{p.c[j], me, j, depth + 1, {}, {}});
                link[j] = W_EMPTY;   // patched once the cut has its place
            } else
                link[j] = plan(p.c[j], depth + 1, out, s, top);
        }
        for (int j = 0; j < W_WIDTH; j++)
            out[me].link[j] = link[j];
        return me;
    }

    void run(Pool& pool)
    {
        plan(0, 1, plans, st, true);
        parallel_for(pool, (int64_t)cuts.size(), 1, [&](int64_t k) {
            Cut& c = cuts[(size_t)k];
            plan(c.bi, c.depth, c.local, c.st, false);
        });
        size_t total = plans.size();
        std::vector<size_t> base(cuts.size());
        for (size_t k = 0; k < cuts.size(); k++) {
            base[k] = total;
            total += cuts[k].local.size();
            plans[cuts[k].node].link[cuts[k].j] = (uint32_t)base[k];
            st.add(cuts[k].st);
        }
        plans.resize(total);
        parallel_for(pool, (int64_t)cuts.size(), 1, [&](int64_t k) {
            const Cut& c = cuts[(size_t)k];
            for (size_t i = 0; i < c.local.size(); i++) {
                Plan p = c.local[i];
                for (int j = 0; j < W_WIDTH; j++)
                    if (p.link[j] != W_EMPTY && !(p.link[j] & W_LEAF))
                        p.link[j] += (uint32_t)base[(size_t)k];
                plans[base[(size_t)k] + i] = p;
            }
        });
    }
};

// Two-level build: a binary SAH tree over the octree's non-empty leaves (one leaf per top
// leaf, boxes = the leaf's triangles' boxes and its k-DOP's axis planes), then under each top
// leaf a binary SAH tree over that octree leaf's triangles.  Every node above the octree
// leaves then holds the k-DOP boxes of the octree leaves of all its triangles.
void build_two_level(const FlatOctree& oct, std::vector<Prim, DefaultInitAlloc<Prim>>& P,
                     std::vector<Prim, DefaultInitAlloc<Prim>>& tmp, std::vector<BNode, DefaultInitAlloc<BNode>>& bn,
                     Pool& pool)
{
    const bool prof = std::getenv("RT_BUILD_PROFILE") != nullptr;
    auto tick = std::chrono::steady_clock::now();
    auto phase = [&](const char* what) {
        if (!prof)
            return;
        auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[wbvh]   two-level %-8s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(now - tick).count());
        tick = now;
    };
    std::vector<uint32_t> leaves;
    for (size_t i = 0; i < oct.nodes.size(); i++)
        if ((oct.nodes[i].b & LEAF_BIT) && (oct.nodes[i].b & ~LEAF_BIT) > 0)
            leaves.push_back((uint32_t)i);
    const int32_t nl = (int32_t)leaves.size();
    std::vector<Prim, DefaultInitAlloc<Prim>> LP((size_t)nl), Ltmp((size_t)nl);
    parallel_for(pool, nl, 256, [&](int64_t k) {
        const GNode& g = oct.nodes[leaves[(size_t)k]];
        Box b = empty_box();
        for (int a = 0; a < 3; a++) {
            b.lo[a] = g.dn[a];
            b.hi[a] = g.df[a];
        }
        for (uint32_t s = g.a; s < g.a + (g.b & ~LEAF_BIT); s++)
            grow(b, Box{{P[s].lo[0], P[s].lo[1], P[s].lo[2]}, {P[s].hi[0], P[s].hi[1], P[s].hi[2]}});
        Prim& q = LP[(size_t)k];
        for (int a = 0; a < 3; a++) {
            q.lo[a] = b.lo[a];
            q.hi[a] = b.hi[a];
        }
        q.pad = 0.0f;
        q.id = (int32_t)k;
    });
    std::vector<BNode, DefaultInitAlloc<BNode>> tn((size_t)(2 * nl + 4 * (nl / PAR_BIN) + 64));
    std::vector<GTri> dummy((size_t)std::max<int32_t>(nl, 1));   // make_leaf's normal sums: recomputed below
    for (auto& t : dummy)
        std::memset(&t, 0, sizeof(t));
    {
        Builder T(LP, Ltmp, tn, dummy.data(), pool);
        T.maxleaf = 1;
        T.run(nl);
    }
    phase("top");
    // the top tree's nodes: those reachable from the root
    std::vector<int32_t> order;   // top nodes, preorder
    std::vector<int32_t> st{0};
    while (!st.empty()) {
        int32_t k = st.back();
        st.pop_back();
        order.push_back(k);
        if (tn[(size_t)k].left >= 0) {
            st.push_back(tn[(size_t)k].right);
            st.push_back(tn[(size_t)k].left);
        }
    }
    const int32_t ntop = (int32_t)tn.size();
    // the triangles in top-leaf order
    std::vector<int32_t> tb((size_t)nl), te((size_t)nl);
    {
        int32_t pos = 0;
        for (int32_t k : order) {
            const BNode& N = tn[(size_t)k];
            if (N.left >= 0)
                continue;
            for (int32_t i = N.first; i < N.first + N.count; i++) {
                const int32_t lk = LP[(size_t)i].id;
                const GNode& g = oct.nodes[leaves[(size_t)lk]];
                tb[(size_t)lk] = pos;
                for (uint32_t s = g.a; s < g.a + (g.b & ~LEAF_BIT); s++)
                    tmp[(size_t)pos++] = P[s];
                te[(size_t)lk] = pos;
            }
        }
        std::copy(tmp.begin(), tmp.begin() + pos, P.begin());
    }
    const size_t need = (size_t)ntop + 2 * P.size() + 64;
    if (bn.size() < need)
        bn.resize(need);
    for (int32_t k : order)
        bn[(size_t)k] = tn[(size_t)k];
    // bottom trees: each top leaf (one octree leaf) becomes the root of its triangles' tree, with
    // the top leaf's box (it holds the octree leaf's k-DOP box)
    std::vector<int32_t> top_leaves;
    for (int32_t k : order)
        if (tn[(size_t)k].left < 0)
            top_leaves.push_back(k);
    std::vector<GTri> none;
    Builder Bt(P, tmp, bn, oct.tris.data(), pool);
    parallel_for(pool, (int64_t)top_leaves.size(), 16, [&](int64_t q) {
        const int32_t k = top_leaves[(size_t)q];
        const BNode N0 = tn[(size_t)k];
        int32_t b = INT32_MAX, e = 0;
        for (int32_t i = N0.first; i < N0.first + N0.count; i++) {
            b = std::min(b, tb[(size_t)LP[(size_t)i].id]);
            e = std::max(e, te[(size_t)LP[(size_t)i].id]);
        }
        VBox vb = VBox::empty(), vc = VBox::empty();
        for (int32_t i = b; i < e; i++) {
            vb.grow(plo(P[(size_t)i]), phi(P[(size_t)i]));
            const __m128 c = pcen(P[(size_t)i]);
            vc.grow(c, c);
        }
        int32_t alloc = ntop + 2 * b;
        double sah = 0;
        Bt.build_serial(k, b, e, vb.box(), vc.box(), alloc, sah);
        bn[(size_t)k].box = N0.box;
    });
    phase("bottom");
    // top inner nodes: triangle ranges and normal sums, children first
    for (size_t q = order.size(); q-- > 0;) {
        BNode& N = bn[(size_t)order[q]];
        if (tn[(size_t)order[q]].left < 0)
            continue;
        const BNode &L = bn[(size_t)N.left], &R = bn[(size_t)N.right];
        N.first = L.first;
        N.count = L.count + R.count;
        for (int a = 0; a < 3; a++)
            N.ns[a] = L.ns[a] + R.ns[a];
    }
}

}  // namespace

void wbvh_fill_tris(const FlatOctree& oct, WBvh& w)
{
    const int64_t n = (int64_t)w.slot.size();
    w.tris.resize((size_t)n);
    parallel_for(build_pool(), n, 8192, [&](int64_t k) { w.tris[(size_t)k] = oct.tris[(size_t)w.slot[(size_t)k]]; });
}

void build_wbvh(const FlatOctree& oct, WBvh& out)
{
    if (const char* q = std::getenv("RT_WBVH_QUICK"))
        if (q[0] == '1') {   // (tests, probes: the quick tree in place of the SAH tree)
            build_wbvh_quick(oct, out);
            return;
        }
    const bool prof = std::getenv("RT_BUILD_PROFILE") != nullptr;
    auto tick = std::chrono::steady_clock::now();
    auto phase = [&](const char* what) {
        if (!prof)
            return;
        auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[wbvh] %-10s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(now - tick).count());
        tick = now;
    };
    out = WBvh();
    const int64_t n = (int64_t)oct.tris.size();
    Pool& pool = build_pool();
    out.leaf_of_slot.assign((size_t)n, 0u);
    parallel_for(pool, (int64_t)oct.nodes.size(), 4096, [&](int64_t i) {
        const GNode& g = oct.nodes[(size_t)i];
        if (g.b & LEAF_BIT)
            for (uint32_t s = g.a; s < g.a + (g.b & ~LEAF_BIT); s++)
                out.leaf_of_slot[s] = (uint32_t)i;
    });
    if (n == 0 || n >= ((int64_t)1 << 28))
        return;
    std::vector<Prim, DefaultInitAlloc<Prim>> P((size_t)n), tmp((size_t)n);
    parallel_for(pool, n, 8192, [&](int64_t i) {
        const Box b = tri_box(oct.tris[(size_t)i]);
        Prim& q = P[(size_t)i];
        for (int a = 0; a < 3; a++) {
            q.lo[a] = b.lo[a];
            q.hi[a] = b.hi[a];
        }
        q.pad = 0.0f;
        q.id = (int32_t)i;
    });
    // 2n for the tasks' regions plus room for the cooperative phase's nodes
    std::vector<BNode, DefaultInitAlloc<BNode>> bn((size_t)(2 * n + 4 * (n / PAR_BIN) + 64));
    phase("prep");
    // two levels (the default): every node above the octree's leaves holds the k-DOP boxes of the
    // octree leaves of all its triangles (the grazing-sound query's rho = 0 there)
    const bool two = !(std::getenv("RT_WBVH_TWOLEVEL") && std::atoi(std::getenv("RT_WBVH_TWOLEVEL")) == 0);
    if (!two) {
        Builder B(P, tmp, bn, oct.tris.data(), pool);
        B.run((int32_t)n);
        // SAH cost of the binary tree (diagnostic)
        const float ra = area(bn[0].box) > 0 ? area(bn[0].box) : 1.0f;
        double s = B.sah_big;
        for (const auto& T : B.tasks)
            s += T.sah;
        out.stats.sah = (float)(s / ra);
    } else
        build_two_level(oct, P, tmp, bn, pool);
    phase("binary");
    // the triangles in the final (leaf) order, and the cone codes' unit normals
    out.tris.resize((size_t)n);
    out.slot.resize((size_t)n);
    out.leaf_of_k.resize((size_t)n);
    std::vector<UnitN, DefaultInitAlloc<UnitN>> un((size_t)n);
    parallel_for(pool, n, 8192, [&](int64_t i) {
        const int32_t s = P[(size_t)i].id;
        const GTri& t = oct.tris[(size_t)s];
        out.tris[(size_t)i] = t;
        out.slot[(size_t)i] = s;
        out.leaf_of_k[(size_t)i] = out.leaf_of_slot[(size_t)s];
        const double n0 = t.n[0], n1 = t.n[1], n2 = t.n[2];
        const double len = std::sqrt(n0 * n0 + n1 * n1 + n2 * n2);
        UnitN& u = un[(size_t)i];
        u.state = len == 0 ? 1 : (len > 1e-30 && len < 1e27 ? 0 : 2);
        u.u[0] = u.state == 0 ? n0 / len : 0.0;
        u.u[1] = u.state == 0 ? n1 / len : 0.0;
        u.u[2] = u.state == 0 ? n2 / len : 0.0;
    });
    phase("order");
    Planner pl{bn};
    pl.plans.reserve(1024);
    pl.run(pool);
    phase("plan");
    out.nodes.resize(pl.plans.size());
    parallel_for(pool, (int64_t)pl.plans.size(), 64, [&](int64_t w) {
        const Planner::Plan& p = pl.plans[(size_t)w];
        Box cb[W_WIDTH];
        ChildGeom cg[W_WIDTH];
        for (int j = 0; j < W_WIDTH; j++)
            cb[j] = empty_box();
        for (int j = 0; j < p.nc; j++) {
            const BNode& C = bn[(size_t)p.c[j]];
            cb[j] = C.box;
            cg[j].first = C.first;
            cg[j].count = C.count;
            for (int a = 0; a < 3; a++)
                cg[j].n[a] = C.ns[a];
        }
        out.nodes[(size_t)w] = quantise(cb, p.link, p.nc, cg, out.tris.data(), un.data());
        // the conditioning bytes of the grazing-sound query (wbvh.hpp WNode::ext): per child the
        // triangles' shape and orientation bounds, and the octree leaves' reach
        WNode& WN = out.nodes[(size_t)w];
        for (int j = 0; j < W_WIDTH; j++) {
            WN.ext[j] = 0u;
            WN.ext2[j] = 0u;
            if (j >= p.nc)
                continue;
            double lo[3], hi[3];
            decode(WN, j, lo, hi);
            const double N0 = (int8_t)(WN.nrm[j] & 0xffu), N1 = (int8_t)((WN.nrm[j] >> 8) & 0xffu),
                         N2 = (int8_t)((WN.nrm[j] >> 16) & 0xffu);
            const double NLd = std::sqrt(N0 * N0 + N1 * N1 + N2 * N2);
            double smin = 1.0, s2 = 1.0, cmin = 1.0, lmax = 0.0;
            double ulo[3] = {lo[0], lo[1], lo[2]}, uhi[3] = {hi[0], hi[1], hi[2]};
            for (int32_t i = cg[j].first; i < cg[j].first + cg[j].count; i++) {
                const GTri& t = out.tris[(size_t)i];
                const GNode& L = oct.nodes[out.leaf_of_k[(size_t)i]];
                for (int a = 0; a < 3; a++) {
                    ulo[a] = std::min(ulo[a], (double)L.dn[a]);
                    uhi[a] = std::max(uhi[a], (double)L.df[a]);
                }
                if (t.n[0] == 0.0f && t.n[1] == 0.0f && t.n[2] == 0.0f)
                    continue;   // Mdet = 0: never a hit
                const double x0 = t.ab[0], x1 = t.ab[1], x2 = t.ab[2], y0 = t.ac[0], y1 = t.ac[1], y2 = t.ac[2];
                const double c0 = x1 * y2 - x2 * y1, c1 = x2 * y0 - x0 * y2, c2 = x0 * y1 - x1 * y0;
                const double la = std::sqrt(x0 * x0 + x1 * x1 + x2 * x2), lc = std::sqrt(y0 * y0 + y1 * y1 + y2 * y2);
                const double cl = std::sqrt(c0 * c0 + c1 * c1 + c2 * c2);
                lmax = std::max(lmax, std::max(la, lc) * (1 + 1e-12));
                smin = std::min(smin, sin_at_a_lb(t));
                if (!(la * lc > 0x1p-100) || !(cl > 0x1p-50 * la * lc) || !(NLd > 0)) {
                    s2 = 0.0;   // no bound: a zero-area record with Mdet != 0
                    cmin = -1.0;
                    continue;
                }
                const double ca = std::fabs(x0 * y0 + x1 * y1 + x2 * y2) / (la * lc);
                s2 = std::min(s2, std::sqrt(std::max(0.0, (1.0 - std::min(1.0, ca + 1e-12)) / 2.0)) * (1 - 1e-9));
                cmin = std::min(cmin, (c0 * N0 + c1 * N1 + c2 * N2) / (cl * NLd) - 1e-12);
            }
            double rho = 0.0;
            for (int a = 0; a < 3; a++)
                rho = std::max(rho, std::max(lo[a] - ulo[a], uhi[a] - hi[a]));
            cmin = std::max(-1.0, std::min(1.0, cmin));
            const double sth = cmin > 0 ? std::min(1.0, std::sqrt(1.0 - cmin * cmin) + 1e-12) : 1.0;
            WN.ext[j] = wq_code_lb(smin) | (wq_code_lb(s2) << 8) | (wq_code_ub(sth, WQ_UNIT) << 16) |
                        (wq_code_ub(lmax, WQ_LEN) << 24);
            WN.ext2[j] = wq_code_ub(rho, WQ_LEN);
        }
    });
    phase("geometry");
    // the risk walk's links (wbvh.hpp WBvh::tri_leaf / parent)
    out.tri_leaf.assign((size_t)n, W_EMPTY);
    out.parent.assign(out.nodes.size(), W_EMPTY);
    parallel_for(pool, (int64_t)out.nodes.size(), 256, [&](int64_t w) {
        const WNode& WN = out.nodes[(size_t)w];
        for (int j = 0; j < W_WIDTH; j++) {
            const uint32_t c = WN.child[j];
            const uint32_t e = (uint32_t)w << 2 | (uint32_t)j;
            if (c == W_EMPTY)
                continue;
            if (c & W_LEAF) {
                const uint32_t first = (c >> 3) & 0x0FFFFFFFu, cnt = (c & 7u) + 1u;
                for (uint32_t k = first; k < first + cnt; k++)
                    out.tri_leaf[k] = e;
            } else
                out.parent[c] = e;
        }
    });
    phase("links");
    out.stats.nodes = (int64_t)out.nodes.size();
    out.stats.leaves = pl.st.leaves;
    out.stats.max_leaf = pl.st.max_leaf;
    out.stats.depth = pl.st.max_depth;
    out.stats.tris = n;
    free_later(std::move(P), std::move(tmp), std::move(bn), std::move(un), std::move(pl.plans));
    phase("exit");
}

// ---- The quick wide BVH (r05): the octree itself as the tree -----------------------------------
// For the frames right after a geometry change: every octree inner node becomes a
// wide node (one with up to four children; with five to eight, the extra ones under one or two group
// nodes), an octree leaf of up to 8 triangles a leaf child, a larger one a small 4-ary tree over its
// triangles in runs of 8.  The triangles take the octree's depth-first leaf order, so every subtree is a
// range.  Everything is O(n): a leaf-level child's slab range, cones and conditioning come from its
// triangles exactly; an upper child's from its children, conservatively -- the slab from its box's
// corners, the cone half-angles by the triangle inequality (angle(n, N) <= angle(n, N_c) +
// angle(N_c, N)), min / max for the rest.  Its float box holds its octree node's axis box, so rho = 0
// above the octree leaves (as in the two-level SAH tree).  check_wbvh verifies all of it like the SAH
// tree's.
namespace {

struct QChild {
    Box box;
    uint32_t link = W_EMPTY;   // W_LEAF | first << 3 | (count - 1), or a node index
    double ns[3] = {0, 0, 0};  // sum of the stored normals (the slab normal's direction)
    int nq[3] = {1, 0, 0};     // the quantised slab normal (quantise's rule)
    double slo = INFINITY, shi = -INFINITY;   // range of nq . v over the triangles' vertices (absolute)
    double tc = 0, ts = 0;     // half-angles between nq and the stored normals / the exact normals below
    bool nocone = false, nosth = false;
    double smin = 1.0, s2 = 1.0, lmax = 0.0;
    int32_t leaf = -1;         // a run of an octree leaf's triangles: that leaf (rho against its axis box)
};

inline void q_normal(QChild& c)
{
    const double len = std::sqrt(c.ns[0] * c.ns[0] + c.ns[1] * c.ns[1] + c.ns[2] * c.ns[2]);
    for (int a = 0; a < 3; a++)
        c.nq[a] = len > 0 ? (int)std::lround(127.0 * c.ns[a] / len) : (a == 0 ? 1 : 0);
    if (c.nq[0] == 0 && c.nq[1] == 0 && c.nq[2] == 0)
        c.nq[0] = 1;
}

inline double q_len(const int* q) { return std::sqrt((double)q[0] * q[0] + (double)q[1] * q[1] + (double)q[2] * q[2]); }

// angle between two quantised normals, rounded up (acos near 1 turns the cosine's rounding, ~1e-16,
// into ~1.5e-8 of angle: 1e-7 of slack)
inline double q_angle(const int* a, const int* b)
{
    const double c = ((double)a[0] * b[0] + (double)a[1] * b[1] + (double)a[2] * b[2]) / (q_len(a) * q_len(b));
    return std::acos(std::max(-1.0, std::min(1.0, c))) + 1e-7;
}

// a run of triangles [first, first + cnt) of the wide order (record i: t[map[i]]): everything from the
// triangles themselves
void q_from_tris(QChild& c, const GTri* t, const int32_t* map, int32_t first, int32_t cnt)
{
    c.box = empty_box();
    for (int a = 0; a < 3; a++)
        c.ns[a] = 0;
    for (int32_t i = first; i < first + cnt; i++) {
        const GTri& T = t[map[i]];
        grow(c.box, tri_box(T));
        for (int a = 0; a < 3; a++)
            c.ns[a] += (double)T.n[a];
    }
    q_normal(c);
    const double n0 = c.nq[0], n1 = c.nq[1], n2 = c.nq[2], NL = q_len(c.nq);
    double cmin = 1.0, smn = 1.0;   // stored normals (cone), exact normals (sth)
    for (int32_t i = first; i < first + cnt; i++) {
        const GTri& T = t[map[i]];
        const double a0 = T.a[0], a1 = T.a[1], a2 = T.a[2];
        const double s0 = n0 * a0 + n1 * a1 + n2 * a2;
        const double s1 = n0 * (a0 + (double)T.ab[0]) + n1 * (a1 + (double)T.ab[1]) + n2 * (a2 + (double)T.ab[2]);
        const double sv = n0 * (a0 + (double)T.ac[0]) + n1 * (a1 + (double)T.ac[1]) + n2 * (a2 + (double)T.ac[2]);
        c.slo = std::min(c.slo, std::min(s0, std::min(s1, sv)));
        c.shi = std::max(c.shi, std::max(s0, std::max(s1, sv)));
        const double m0 = T.n[0], m1 = T.n[1], m2 = T.n[2];
        const double mlen = std::sqrt(m0 * m0 + m1 * m1 + m2 * m2);
        if (mlen == 0)
            continue;   // Mdet = 0: never a hit (no cone, no conditioning bound needed)
        if (!(mlen > 1e-30 && mlen < 1e27))
            c.nocone = true;
        else
            cmin = std::min(cmin, (m0 * n0 + m1 * n1 + m2 * n2) / (mlen * NL));
        const double x0 = T.ab[0], x1 = T.ab[1], x2 = T.ab[2], y0 = T.ac[0], y1 = T.ac[1], y2 = T.ac[2];
        const double c0 = x1 * y2 - x2 * y1, c1 = x2 * y0 - x0 * y2, c2 = x0 * y1 - x1 * y0;
        const double la = std::sqrt(x0 * x0 + x1 * x1 + x2 * x2), lc = std::sqrt(y0 * y0 + y1 * y1 + y2 * y2);
        const double cl = std::sqrt(c0 * c0 + c1 * c1 + c2 * c2);
        c.lmax = std::max(c.lmax, std::max(la, lc) * (1 + 1e-12));
        c.smin = std::min(c.smin, sin_at_a_lb(T));
        if (!(la * lc > 0x1p-100) || !(cl > 0x1p-50 * la * lc)) {
            c.s2 = 0.0;
            c.nosth = true;
            continue;
        }
        const double ca = std::fabs(x0 * y0 + x1 * y1 + x2 * y2) / (la * lc);
        c.s2 = std::min(c.s2, std::sqrt(std::max(0.0, (1.0 - std::min(1.0, ca + 1e-12)) / 2.0)) * (1 - 1e-9));
        smn = std::min(smn, (c0 * n0 + c1 * n1 + c2 * n2) / (cl * NL) - 1e-12);
    }
    c.tc = std::acos(std::max(-1.0, std::min(1.0, cmin))) + 1e-7;
    c.ts = std::acos(std::max(-1.0, std::min(1.0, smn))) + 1e-7;
}

// an upper child from its children (and the octree node's axis box, which it holds)
void q_combine(QChild& p, const QChild* ch, int nc, const Box* extra)
{
    p.box = empty_box();
    if (extra)
        p.box = *extra;
    for (int a = 0; a < 3; a++)
        p.ns[a] = 0;
    p.nocone = p.nosth = false;
    p.smin = p.s2 = 1.0;
    p.lmax = 0.0;
    for (int i = 0; i < nc; i++) {
        grow(p.box, ch[i].box);
        for (int a = 0; a < 3; a++)
            p.ns[a] += ch[i].ns[a];
        p.nocone |= ch[i].nocone;
        p.nosth |= ch[i].nosth;
        p.smin = std::min(p.smin, ch[i].smin);
        p.s2 = std::min(p.s2, ch[i].s2);
        p.lmax = std::max(p.lmax, ch[i].lmax);
    }
    q_normal(p);
    p.tc = p.ts = 0;
    for (int i = 0; i < nc; i++) {
        const double d = q_angle(p.nq, ch[i].nq);
        p.tc = std::max(p.tc, d + ch[i].tc);
        p.ts = std::max(p.ts, d + ch[i].ts);
    }
    // the slab: the range of nq . v over the box's corners (the box holds every vertex below)
    p.slo = INFINITY;
    p.shi = -INFINITY;
    for (int k = 0; k < 8; k++) {
        const double v0 = (k & 1) ? p.box.hi[0] : p.box.lo[0], v1 = (k & 2) ? p.box.hi[1] : p.box.lo[1],
                     v2 = (k & 4) ? p.box.hi[2] : p.box.lo[2];
        const double sv = p.nq[0] * v0 + p.nq[1] * v1 + p.nq[2] * v2;
        p.slo = std::min(p.slo, sv);
        p.shi = std::max(p.shi, sv);
    }
    p.leaf = -1;
}

// the node's boxes (quantise's rule), then per child the slab (absolute range shifted to the node's
// origin, widened by the rounding of that shift), the cone code, the conditioning bytes and rho
WNode q_node(const QChild* ch, int nc, const FlatOctree& oct)
{
    WNode w;
    std::memset(&w, 0, sizeof(w));
    Box nb = empty_box();
    for (int j = 0; j < nc; j++)
        grow(nb, ch[j].box);
    const float org[3] = {nb.lo[0], nb.lo[1], nb.lo[2]};
    w.ox = org[0];
    w.oy = org[1];
    w.oz = org[2];
    for (int a = 0; a < 3; a++) {
        const double ext = (double)nb.hi[a] - (double)org[a];
        int k = -100;
        if (ext > 0) {
            int e;
            std::frexp(ext / 255.0, &e);
            k = std::max(-100, std::min(127, e - 1));
            while (k < 127 && std::ldexp(255.0, k) < ext)
                k++;
        }
        w.exps |= (uint32_t)(127 + k) << (8 * a);
        const double st = std::ldexp(1.0, k);
        for (int j = 0; j < nc; j++) {
            const double lo = std::floor(((double)ch[j].box.lo[a] - org[a]) / st);
            const double hi = std::ceil(((double)ch[j].box.hi[a] - org[a]) / st);
            w.qlo[a][j] = (uint8_t)std::max(0.0, std::min(255.0, lo));
            w.qhi[a][j] = (uint8_t)std::max(0.0, std::min(255.0, hi));
        }
    }
    for (int j = 0; j < W_WIDTH; j++)
        w.child[j] = j < nc ? ch[j].link : W_EMPTY;
    double lo[W_WIDTH], hi[W_WIDTH], lo_all = INFINITY, hi_all = -INFINITY;
    for (int j = 0; j < nc; j++) {
        const double sh = (double)ch[j].nq[0] * org[0] + (double)ch[j].nq[1] * org[1] + (double)ch[j].nq[2] * org[2];
        // |rounding| of the absolute sums and of the shift: a few ulps of the largest magnitude
        const double slack = 0x1p-48 * (std::fabs(ch[j].slo) + std::fabs(ch[j].shi) + std::fabs(sh) +
                                        128.0 * (std::fabs((double)org[0]) + std::fabs((double)org[1]) + std::fabs((double)org[2])));
        lo[j] = ch[j].slo - sh - slack;
        hi[j] = ch[j].shi - sh + slack;
        lo_all = std::min(lo_all, lo[j]);
        hi_all = std::max(hi_all, hi[j]);
    }
    const float slo = down(lo_all);
    const double ext = hi_all - (double)slo;
    int k = -100;
    if (ext > 0) {
        int e;
        std::frexp(ext / 65535.0, &e);
        k = std::max(-100, std::min(127, e - 1));
        while (k < 127 && std::ldexp(65535.0, k) < ext)
            k++;
    }
    const double st = std::ldexp(1.0, k);
    w.s = (float)st;
    w.slo = slo;
    for (int j = 0; j < nc; j++) {
        const QChild& c = ch[j];
        // the cone code (cone_code's rule) from the half-angle
        int code = 255;
        const double NL = q_len(c.nq);
        const double psi = std::acos(W_CONE_EPS) - c.tc - 1e-9;
        if (!c.nocone && psi > 0) {
            const double cd = std::ceil((std::cos(psi) * NL + 0.01) / ((double)W_CONE_STEP * (1 - 1e-9)));
            code = cd <= 254 ? (int)cd : 255;
        }
        w.nrm[j] = (uint32_t)(uint8_t)(int8_t)c.nq[0] | ((uint32_t)(uint8_t)(int8_t)c.nq[1] << 8) |
                   ((uint32_t)(uint8_t)(int8_t)c.nq[2] << 16) | ((uint32_t)code << 24);
        double q0 = std::floor((lo[j] - (double)slo) / st), q1 = std::ceil((hi[j] - (double)slo) / st);
        q0 = std::max(0.0, std::min(65535.0, q0));
        q1 = std::max(0.0, std::min(65535.0, q1));
        w.slab[j] = (uint32_t)q0 | ((uint32_t)q1 << 16);
        const double sth = c.nosth || c.ts >= M_PI / 2 ? 1.0 : std::min(1.0, std::sin(c.ts) + 1e-12);
        w.ext[j] = wq_code_lb(c.smin) | (wq_code_lb(c.s2) << 8) | (wq_code_ub(sth, WQ_UNIT) << 16) |
                   (wq_code_ub(c.lmax, WQ_LEN) << 24);
        double rho = 0.0;
        if (c.leaf >= 0) {
            double dlo[3], dhi[3];
            decode(w, j, dlo, dhi);
            const GNode& L = oct.nodes[(size_t)c.leaf];
            for (int a = 0; a < 3; a++)
                rho = std::max(rho, std::max(dlo[a] - (double)L.dn[a], (double)L.df[a] - dhi[a]));
        }
        w.ext2[j] = wq_code_ub(rho, WQ_LEN);
    }
    return w;
}

}  // namespace

void build_wbvh_quick(const FlatOctree& oct, WBvh& out, bool tris)
{
    const bool prof = std::getenv("RT_BUILD_PROFILE") != nullptr;
    auto tick = std::chrono::steady_clock::now();
    auto phase = [&](const char* what) {
        if (!prof)
            return;
        auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[wbvh quick] %-10s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(now - tick).count());
        tick = now;
    };
    out = WBvh();
    const int64_t n = (int64_t)oct.tris.size();
    Pool& pool = build_pool();
    out.leaf_of_slot.assign((size_t)n, 0u);
    parallel_for(pool, (int64_t)oct.nodes.size(), 4096, [&](int64_t i) {
        const GNode& g = oct.nodes[(size_t)i];
        if (g.b & LEAF_BIT)
            for (uint32_t s = g.a; s < g.a + (g.b & ~LEAF_BIT); s++)
                out.leaf_of_slot[s] = (uint32_t)i;
    });
    if (n == 0 || n >= ((int64_t)1 << 28))
        return;
    // wide nodes, planned depth first (the root is node 0; a node's children have higher indices)
    struct Plan {
        int nc = 0;
        int kind[W_WIDTH];      // 0: a run of triangles (first, cnt); 1: a wide node
        int32_t a[W_WIDTH], b[W_WIDTH];   // run: first, count; node: index, -
        int32_t leaf[W_WIDTH];  // run: the octree leaf it belongs to (rho), or -1 when the run is the whole leaf
        int32_t oct = -1;       // the octree node whose axis box the node's parent entry holds (-1: none)
        int32_t runleaf = -1;   // a node over runs of octree leaf L's triangles: L (its entry's rho against L)
        int32_t depth = 0;
    };
    std::vector<Plan> plans;
    plans.reserve((size_t)(n / 4 + 16));
    std::vector<int32_t> order;   // wide order -> slot
    order.reserve((size_t)n);
    int32_t maxd = 0;
    // a 4-ary tree over the runs [first, first + cnt) in runs of 8 of octree leaf L
    std::function<int32_t(int32_t, int32_t, int32_t, int32_t)> runs = [&](int32_t first, int32_t cnt, int32_t L, int32_t depth) {
        const int32_t me = (int32_t)plans.size();
        plans.emplace_back();
        plans[(size_t)me].depth = depth;
        plans[(size_t)me].runleaf = L;
        maxd = std::max(maxd, depth);
        const int32_t nr = (cnt + W_MAX_LEAF - 1) / W_MAX_LEAF;   // runs
        // split the runs over up to four children as evenly as possible
        const int parts = (int)std::min<int32_t>(W_WIDTH, nr);
        int32_t r0 = 0;
        for (int p = 0; p < parts; p++) {
            const int32_t r1 = (int32_t)((int64_t)nr * (p + 1) / parts);
            const int32_t f = first + r0 * W_MAX_LEAF, c = std::min(cnt, r1 * W_MAX_LEAF) - r0 * W_MAX_LEAF;
            Plan& P = plans[(size_t)me];
            const int j = P.nc++;
            if (r1 - r0 == 1) {
                P.kind[j] = 0;
                P.a[j] = f;
                P.b[j] = c;
                P.leaf[j] = L;
            } else {
                const int32_t child = runs(f, c, L, depth + 1);
                Plan& Q = plans[(size_t)me];
                Q.kind[j] = 1;
                Q.a[j] = child;
                Q.b[j] = 0;
                Q.leaf[j] = -1;
            }
            r0 = r1;
        }
        return me;
    };
    // the entry for octree node u: fills (kind, a, b, leaf) of child slot j of plan p
    std::function<void(int32_t, int32_t, int, int32_t)> entry;
    std::function<int32_t(int32_t, int32_t)> inner = [&](int32_t u, int32_t depth) {
        // a wide node for octree inner node u (children c0 .. c0 + cn - 1, up to 8)
        const GNode& g = oct.nodes[(size_t)u];
        const int32_t c0 = (int32_t)g.a, cn = (int32_t)g.b;
        const int32_t me = (int32_t)plans.size();
        plans.emplace_back();
        plans[(size_t)me].depth = depth;
        maxd = std::max(maxd, depth);
        // direct children and groups: 1-4 direct; 5-7: 3 direct + 1 group; 8: 2 direct + 2 groups of 3
        int direct = cn <= W_WIDTH ? cn : (cn <= 7 ? 3 : 2);
        for (int i = 0; i < direct; i++)
            entry(c0 + i, me, plans[(size_t)me].nc++, depth);
        int32_t rest = cn - direct, at = c0 + direct;
        const int groups = rest == 0 ? 0 : (cn <= 7 ? 1 : 2);
        for (int gi = 0; gi < groups; gi++) {
            const int32_t gs = gi == groups - 1 ? rest : (rest + 1) / 2;
            const int32_t gnode = (int32_t)plans.size();
            plans.emplace_back();
            plans[(size_t)gnode].depth = depth + 1;
            maxd = std::max(maxd, depth + 1);
            for (int32_t i = 0; i < gs; i++)
                entry(at + i, gnode, plans[(size_t)gnode].nc++, depth + 1);
            Plan& P = plans[(size_t)me];
            const int j = P.nc++;
            P.kind[j] = 1;
            P.a[j] = gnode;
            P.b[j] = 0;
            P.leaf[j] = -1;
            at += gs;
            rest -= gs;
        }
        return me;
    };
    entry = [&](int32_t u, int32_t p, int j, int32_t depth) {
        const GNode& g = oct.nodes[(size_t)u];
        if (g.b & LEAF_BIT) {
            const int32_t cnt = (int32_t)(g.b & ~LEAF_BIT), first = (int32_t)order.size();
            for (int32_t s = 0; s < cnt; s++)
                order.push_back((int32_t)g.a + s);
            if (cnt <= W_MAX_LEAF) {
                Plan& P = plans[(size_t)p];
                P.kind[j] = 0;
                P.a[j] = first;
                P.b[j] = cnt;
                P.leaf[j] = u;
            } else {
                const int32_t child = runs(first, cnt, u, depth + 1);
                Plan& P = plans[(size_t)p];
                P.kind[j] = 1;
                P.a[j] = child;
                P.b[j] = 0;
                P.leaf[j] = -1;
                plans[(size_t)child].oct = u;   // (the runs' node holds the leaf's axis box: rho = 0 above it)
            }
        } else {
            const int32_t child = inner(u, depth + 1);
            Plan& P = plans[(size_t)p];
            P.kind[j] = 1;
            P.a[j] = child;
            P.b[j] = 0;
            P.leaf[j] = -1;
            plans[(size_t)child].oct = u;
        }
    };
    if (oct.nodes[0].b & LEAF_BIT) {
        // a single leaf: one node over its runs (with one run, a node with one leaf child)
        const GNode& g = oct.nodes[0];
        const int32_t cnt = (int32_t)(g.b & ~LEAF_BIT);
        for (int32_t s = 0; s < cnt; s++)
            order.push_back((int32_t)g.a + s);
        runs(0, cnt, 0, 0);
        plans[0].oct = 0;
    } else {
        inner(0, 0);
        plans[0].oct = 0;
    }
    phase("plan");
    if ((int64_t)order.size() != n)
        return;   // (cannot happen: every slot is in one leaf)
    out.slot.resize((size_t)n);
    out.leaf_of_k.resize((size_t)n);
    parallel_for(pool, n, 8192, [&](int64_t k) {
        const int32_t s = order[(size_t)k];
        out.slot[(size_t)k] = s;
        out.leaf_of_k[(size_t)k] = out.leaf_of_slot[(size_t)s];
    });
    if (tris)
        wbvh_fill_tris(oct, out);
    phase("order");
    // geometry, deepest nodes first (each level in parallel): a node's children are complete when it runs
    const size_t np = plans.size();
    out.nodes.resize(np);
    std::vector<QChild> agg(np);   // each node as its parent's child
    std::vector<std::vector<int32_t>> by_depth((size_t)maxd + 1);
    for (size_t w = 0; w < np; w++)
        by_depth[(size_t)plans[w].depth].push_back((int32_t)w);
    for (int32_t d = maxd; d >= 0; d--) {
        const std::vector<int32_t>& lv = by_depth[(size_t)d];
        parallel_for(pool, (int64_t)lv.size(), 64, [&](int64_t q) {
            const int32_t w = lv[(size_t)q];
            const Plan& P = plans[(size_t)w];
            QChild ch[W_WIDTH];
            for (int j = 0; j < P.nc; j++) {
                if (P.kind[j] == 0) {
                    q_from_tris(ch[j], oct.tris.data(), out.slot.data(), P.a[j], P.b[j]);
                    ch[j].link = W_LEAF | ((uint32_t)P.a[j] << 3) | (uint32_t)(P.b[j] - 1);
                    ch[j].leaf = P.leaf[j];
                } else {
                    ch[j] = agg[(size_t)P.a[j]];
                    ch[j].link = (uint32_t)P.a[j];
                }
            }
            out.nodes[(size_t)w] = q_node(ch, P.nc, oct);
            // the node's entry in its parent holds the axis boxes of the octree leaves below (rho = 0
            // there): its octree node's, and those of its leaf-run children (their record boxes can sit
            // an ulp inside the leaf's k-DOP, which the original vertices set)
            Box ax = empty_box();
            auto axis = [&](int32_t u) {
                const GNode& g = oct.nodes[(size_t)u];
                Box b;
                for (int a = 0; a < 3; a++) {
                    b.lo[a] = g.dn[a];
                    b.hi[a] = g.df[a];
                }
                grow(ax, b);
            };
            if (P.oct >= 0)
                axis(P.oct);
            for (int j = 0; j < P.nc; j++)
                if (P.kind[j] == 0 && P.leaf[j] >= 0)
                    axis(P.leaf[j]);
            q_combine(agg[(size_t)w], ch, P.nc, &ax);
            agg[(size_t)w].leaf = P.runleaf;   // (0 reach for the top one: it holds the leaf's axis box)
        });
    }
    phase("geometry");
    // the risk walk's links
    out.tri_leaf.assign((size_t)n, W_EMPTY);
    out.parent.assign(np, W_EMPTY);
    parallel_for(pool, (int64_t)np, 256, [&](int64_t w) {
        const WNode& WN = out.nodes[(size_t)w];
        for (int j = 0; j < W_WIDTH; j++) {
            const uint32_t c = WN.child[j];
            const uint32_t e = (uint32_t)w << 2 | (uint32_t)j;
            if (c == W_EMPTY)
                continue;
            if (c & W_LEAF) {
                const uint32_t first = (c >> 3) & 0x0FFFFFFFu, cnt = (c & 7u) + 1u;
                for (uint32_t k = first; k < first + cnt; k++)
                    out.tri_leaf[k] = e;
            } else
                out.parent[c] = e;
        }
    });
    int64_t leaves = 0, maxleaf = 0;
    for (const Plan& P : plans)
        for (int j = 0; j < P.nc; j++)
            if (P.kind[j] == 0) {
                leaves++;
                maxleaf = std::max<int64_t>(maxleaf, P.b[j]);
            }
    out.stats.nodes = (int64_t)np;
    out.stats.leaves = leaves;
    out.stats.max_leaf = maxleaf;
    out.stats.depth = maxd + 1;
    out.stats.tris = n;
    phase("links");
}

// The conditioning bytes of child j of node N (WNode::ext / ext2, read as the query's values:
// wq_val, a code 0 being 0) against wide-BVH triangle k below it, recomputed independently of the
// build in x87 long double (64-bit significands: the products of float coordinates are exact, each
// sum rounds at 2^-64 relative) from the record's float edges, i.e. for the triangle (a, a + ab,
// a + ac) Moller-Trumbore tests (triangle.cpp:25-91):
//   smin <= sin(alpha), s2 <= sin(alpha' / 2), alpha' = min(alpha, pi - alpha) (alpha: the angle at a);
//   sth >= sin of the angle between the child's slab normal N and the exact normal ab x ac (1 when
//        that angle is 90 degrees or more, or the exact normal is 0);
//   lmax >= |ab|, |ac|;
//   rho >= how far the axis box of the triangle's octree leaf (its k-DOP's axis slabs) reaches past
//        the child's decoded box.
// The slack 2^-60 on the sines is far below every build margin (sin_at_a_lb subtracts 2^-50).
// Records whose stored normal is 0 never report a hit (Mdet = 0) and need no bound.  Returns the
// number of violated bounds.
// (RT_CHECK_VERBOSE=1: each violation's source line on stderr, the first 40)
static void w_viol_note(int line)
{
    static const bool on = std::getenv("RT_CHECK_VERBOSE") != nullptr;
    static std::atomic<int> shown{0};
    if (on && shown.fetch_add(1) < 40)
        fprintf(stderr, "[check_wbvh] violation at wbvh.cpp:%d\n", line);
}
#define W_VIOL() (bad++, w_viol_note(__LINE__))

static int64_t check_conditioning(const FlatOctree& oct, const WBvh& w, const WNode& N, int j, uint32_t k)
{
    const GTri& t = w.tris[k];
    int64_t bad = 0;
    const uint32_t e = N.ext[j], e2 = N.ext2[j];
    const long double smin = wq_val(e & 0xffu, WQ_UNIT), s2 = wq_val((e >> 8) & 0xffu, WQ_UNIT);
    const long double sth = wq_val((e >> 16) & 0xffu, WQ_UNIT);
    const long double L = (e >> 24) == 255u ? INFINITY : wq_val(e >> 24, WQ_LEN);
    const long double rho = wq_len(e2 & 0xffu);
    // rho: the octree leaf's axis box within the decoded child box widened by rho
    {
        double lo[3], hi[3];
        decode(N, j, lo, hi);
        const GNode& OL = oct.nodes[w.leaf_of_k[k]];
        for (int a = 0; a < 3; a++)
            if (!((long double)OL.dn[a] >= (long double)lo[a] - rho && (long double)OL.df[a] <= (long double)hi[a] + rho)) {
                W_VIOL();
                if (std::getenv("RT_CHECK_VERBOSE"))
                    fprintf(stderr, "  rho: node %ld child %d (link %08x) tri %u leaf %u axis %d: leaf [%.9g, %.9g] box [%.9g, %.9g] rho %.3Lg\n",
                            (long)(&N - w.nodes.data()), j, N.child[j], k, w.leaf_of_k[k], a, OL.dn[a], OL.df[a], lo[a], hi[a], rho);
            }
    }
    if (t.n[0] == 0.0f && t.n[1] == 0.0f && t.n[2] == 0.0f)
        return bad;
    const long double x0 = t.ab[0], x1 = t.ab[1], x2 = t.ab[2], y0 = t.ac[0], y1 = t.ac[1], y2 = t.ac[2];
    const long double c0 = x1 * y2 - x2 * y1, c1 = x2 * y0 - x0 * y2, c2 = x0 * y1 - x1 * y0;
    const long double la = sqrtl(x0 * x0 + x1 * x1 + x2 * x2), lc = sqrtl(y0 * y0 + y1 * y1 + y2 * y2);
    const long double cl = sqrtl(c0 * c0 + c1 * c1 + c2 * c2);
    if (!(L >= fmaxl(la, lc)))
        W_VIOL();
    if (la > 0 && lc > 0) {
        const long double sa = cl / (la * lc);
        if (!(smin <= sa + 0x1p-60L))
            W_VIOL();
        const long double ca = fabsl(x0 * y0 + x1 * y1 + x2 * y2) / (la * lc);
        if (!(s2 <= sqrtl(fmaxl(0.0L, (1.0L - ca) / 2.0L) + 0x1p-60L)))
            W_VIOL();
    } else if (smin > 0 || s2 > 0)
        W_VIOL();
    const long double N0 = (int8_t)(N.nrm[j] & 0xffu), N1 = (int8_t)((N.nrm[j] >> 8) & 0xffu),
                      N2 = (int8_t)((N.nrm[j] >> 16) & 0xffu);
    const long double NL = sqrtl(N0 * N0 + N1 * N1 + N2 * N2);
    const long double cs = cl > 0 && NL > 0 ? (c0 * N0 + c1 * N1 + c2 * N2) / (cl * NL) : -1.0L;
    if (cs > 0) {
        if (!(sth >= sqrtl(fmaxl(0.0L, 1.0L - cs * cs)) - 0x1p-60L))
            W_VIOL();
    } else if (!(sth >= 1.0L))
        W_VIOL();
    return bad;
}

int64_t check_risk_words(const FlatOctree& oct, const WBvh& w, const WRiskArgs& A, int sel, const uint64_t* risk)
{
    int64_t bad = 0;
    if (!A.on[sel]) {
        for (size_t v = 0; v < w.nodes.size(); v++)
            for (int j = 0; j < W_WIDTH; j++)
                bad += risk[(2 * v + sel) * W_WIDTH + j] != wrisk_pack(0.0f, 0xFFFFFF000000ull);
        return bad;
    }
    for (size_t k = 0; k < w.tris.size(); k++) {
        const float Kt = wbvh_risk_key(w.tris[k], A.p[sel][0], A.p[sel][1], A.p[sel][2], A.G[sel], A.nu[sel],
                                       A.slack[sel], A.QS[sel]);
        if (!(Kt < INFINITY))
            continue;
        const GNode& OL = oct.nodes[w.leaf_of_k[k]];
        for (uint32_t e = w.tri_leaf[k], hops = 0; e != W_EMPTY && hops < 1024; e = w.parent[e >> 2], hops++) {
            const WNode& N = w.nodes[e >> 2];
            const int j = (int)(e & 3u);
            const uint64_t word = risk[(2 * (size_t)(e >> 2) + sel) * W_WIDTH + j];
            if (!(wrisk_key(word) <= Kt))
                W_VIOL();
            // the at-risk box (in the node's frame) widened by rho holds the triangle's octree leaf
            const double org[3] = {N.ox, N.oy, N.oz};
            const double rho = wq_len(N.ext2[j] & 0xffu);
            for (int a = 0; a < 3; a++) {
                const double st = std::ldexp(1.0, (int)((N.exps >> (8 * a)) & 0xffu) - 127);
                const double lo = org[a] + (double)((word >> (8 * a)) & 0xffu) * st;
                const double hi = org[a] + (double)((word >> (8 * (a + 3))) & 0xffu) * st;
                if (!((double)OL.dn[a] >= lo - rho && (double)OL.df[a] <= hi + rho))
                    W_VIOL();
            }
        }
    }
    return bad;
}

int64_t check_wbvh(const FlatOctree& oct, const WBvh& w)
{
    int64_t bad = 0;
    const size_t n = oct.tris.size();
    if (w.tris.size() != n || w.slot.size() != n || w.leaf_of_slot.size() != n || w.leaf_of_k.size() != n)
        return 1;
    for (size_t k = 0; k < n; k++)
        if (w.slot[k] >= 0 && (size_t)w.slot[k] < n && w.leaf_of_k[k] != w.leaf_of_slot[(size_t)w.slot[k]])
            W_VIOL();
    if (n == 0)
        return w.nodes.empty() ? 0 : 1;
    std::vector<uint8_t> seen(n, 0), used(w.tris.size(), 0);
    for (size_t i = 0; i < n; i++) {
        int32_t s = w.slot[i];
        if (s < 0 || (size_t)s >= n || seen[(size_t)s]++)
            W_VIOL();
        else if (std::memcmp(&w.tris[i], &oct.tris[(size_t)s], sizeof(GTri)))
            W_VIOL();
    }
    for (size_t s = 0; s < n; s++) {
        uint32_t L = w.leaf_of_slot[s];
        if (L >= oct.nodes.size() || !(oct.nodes[L].b & LEAF_BIT) || s < oct.nodes[L].a ||
            s >= oct.nodes[L].a + (oct.nodes[L].b & ~LEAF_BIT))
            W_VIOL();
    }
    // the risk walk's links: each triangle's leaf entry names it, each node's parent entry names it,
    // and every walk reaches the root
    if (w.tri_leaf.size() != n || w.parent.size() != w.nodes.size() || w.parent[0] != W_EMPTY)
        return bad + 1;
    for (size_t k = 0; k < n; k++) {
        const uint32_t e = w.tri_leaf[k];
        if (e == W_EMPTY || (e >> 2) >= w.nodes.size()) {
            W_VIOL();
            continue;
        }
        const uint32_t c = w.nodes[e >> 2].child[e & 3u];
        const uint32_t first = (c >> 3) & 0x0FFFFFFFu, cnt = (c & 7u) + 1u;
        if (c == W_EMPTY || !(c & W_LEAF) || k < first || k >= first + cnt)
            W_VIOL();
    }
    for (size_t v = 1; v < w.nodes.size(); v++) {
        const uint32_t e = w.parent[v];
        if (e == W_EMPTY || (e >> 2) >= w.nodes.size() || w.nodes[e >> 2].child[e & 3u] != (uint32_t)v)
            W_VIOL();
    }
    // every child box holds its subtree: node boxes and triangle vertices (a, a + ab, a + ac);
    // every slab and cone on the path holds each triangle below (checked at the leaves)
    constexpr int MAXP = 64;
    struct Item {
        uint32_t ref;
        Box box;
        int np;
        uint32_t path[MAXP];   // node << 3 | child of every inner node on the way
    };
    std::vector<Item> stack;
    Box all = {{-INFINITY, -INFINITY, -INFINITY}, {INFINITY, INFINITY, INFINITY}};
    {
        Item root{};
        root.ref = 0u;
        root.box = all;
        stack.push_back(root);
    }
    auto inside = [](const Box& b, const Box& outer) {
        for (int a = 0; a < 3; a++)
            if (!(b.lo[a] >= outer.lo[a] && b.hi[a] <= outer.hi[a]))
                return false;
        return true;
    };
    size_t visited = 0;
    while (!stack.empty()) {
        Item it = stack.back();
        stack.pop_back();
        if (it.ref & W_LEAF) {
            uint32_t first = (it.ref >> 3) & 0x0FFFFFFFu, cnt = (it.ref & 7u) + 1u;
            if ((size_t)first + cnt > n) {
                W_VIOL();
                continue;
            }
            for (uint32_t k = first; k < first + cnt; k++) {
                if (used[k]++)
                    W_VIOL();
                if (!inside(tri_box(w.tris[k]), it.box))
                    W_VIOL();
                const GTri& T = w.tris[k];
                for (int q = 0; q < it.np; q++) {
                    const WNode& N = w.nodes[it.path[q] >> 3];
                    const int j = (int)(it.path[q] & 7u);
                    const double org[3] = {N.ox, N.oy, N.oz};
                    const double nv[3] = {(double)(int8_t)(N.nrm[j] & 0xffu), (double)(int8_t)((N.nrm[j] >> 8) & 0xffu),
                                          (double)(int8_t)((N.nrm[j] >> 16) & 0xffu)};
                    const double lo = (double)N.slo + (double)(N.slab[j] & 0xffffu) * (double)N.s;
                    const double hi = (double)N.slo + (double)(N.slab[j] >> 16) * (double)N.s;
                    for (int v = 0; v < 3; v++) {
                        double sp = 0;
                        for (int a = 0; a < 3; a++)
                            sp += nv[a] * ((double)T.a[a] + (v == 1 ? (double)T.ab[a] : v == 2 ? (double)T.ac[a] : 0.0) - org[a]);
                        if (!(sp >= lo && sp <= hi))
                            W_VIOL();
                    }
                    bad += check_conditioning(oct, w, N, j, k);
                    const uint32_t code = N.nrm[j] >> 24;
                    const double nn = std::sqrt((double)T.n[0] * T.n[0] + (double)T.n[1] * T.n[1] + (double)T.n[2] * T.n[2]);
                    if (code < 255 && nn > 0) {
                        // the kernel skips the child only for d with N . d > (code STEP - 0.01) |d|;
                        // every such d must meet n at cos > eps
                        const double Nl = std::sqrt(nv[0] * nv[0] + nv[1] * nv[1] + nv[2] * nv[2]);
                        const double kap = (code * (double)W_CONE_STEP - 0.01) / Nl;
                        const double c = (T.n[0] * nv[0] + T.n[1] * nv[1] + T.n[2] * nv[2]) / (nn * Nl);
                        const double ang = std::acos(std::max(-1.0, std::min(1.0, c)));
                        if (!(nn > 1e-30 && nn < 1e27) || !(kap > -1.0) ||
                            !(std::acos(std::min(1.0, kap)) + ang < std::acos(W_CONE_EPS)))
                            W_VIOL();
                    }
                }
            }
            continue;
        }
        if (it.ref >= w.nodes.size() || ++visited > w.nodes.size()) {
            W_VIOL();
            continue;
        }
        const WNode& N = w.nodes[it.ref];
        for (int j = 0; j < W_WIDTH; j++) {
            if (N.child[j] == W_EMPTY)
                continue;
            double lo[3], hi[3];
            Box cb = decode(N, j, lo, hi);
            // the decoded box (outward-rounded to float) need not sit inside the parent's, but the
            // triangles below must sit inside every decoded box on their path: tested at the leaves
            // against the intersection of the path's boxes
            Item ch = it;
            ch.ref = N.child[j];
            for (int a = 0; a < 3; a++) {
                ch.box.lo[a] = std::max(cb.lo[a], it.box.lo[a]);
                ch.box.hi[a] = std::min(cb.hi[a], it.box.hi[a]);
            }
            if (ch.np >= MAXP) {
                W_VIOL();
                continue;
            }
            ch.path[ch.np++] = (it.ref << 3) | (uint32_t)j;
            stack.push_back(ch);
        }
    }
    for (size_t k = 0; k < n; k++)
        if (!used[k])
            W_VIOL();
    return bad;
}

}  // namespace rt
