// wbvh.cpp -- host build of the 4-wide SAH BVH (wbvh.hpp) over the octree's triangle
// records: binned SAH binary tree (16 bins per axis, parallel over subtrees), collapsed
// to 4-wide nodes by repeatedly opening the child with the largest surface area.
#include "wbvh.hpp"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <thread>

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
    int32_t first, count;
};

constexpr int NBINS = 16;
constexpr int64_t PAR_BIN = 1 << 17;     // nodes with more primitives bin with all threads
constexpr int64_t PAR_TASK = 1 << 14;    // subtrees at least this large run on their own thread

int wbvh_threads()
{
    if (const char* e = std::getenv("RT_BUILD_THREADS")) {
        int v = std::atoi(e);
        if (v >= 1)
            return v;
    }
    unsigned hc = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(hc, 16u));
}

struct Builder {
    const std::vector<Box>& pb;      // primitive boxes
    const std::vector<float>& pc;    // primitive centroids [3 * i]
    std::vector<int32_t>& idx;
    std::vector<BNode>& nodes;       // preallocated, 2n - 1 nodes at most
    std::atomic<int32_t> next{1};
    std::atomic<int> spare;          // threads that may still be started
    float ct = 1.0f;                 // SAH cost of a node visit, in triangle tests (r02: 2 and 3 were slower)

    struct Bins {
        int32_t cnt[3][NBINS];
        Box box[3][NBINS];
        void clear()
        {
            for (int a = 0; a < 3; a++)
                for (int i = 0; i < NBINS; i++) {
                    cnt[a][i] = 0;
                    box[a][i] = empty_box();
                }
        }
        void add(const Bins& o)
        {
            for (int a = 0; a < 3; a++)
                for (int i = 0; i < NBINS; i++) {
                    cnt[a][i] += o.cnt[a][i];
                    grow(box[a][i], o.box[a][i]);
                }
        }
    };

    Builder(const std::vector<Box>& b, const std::vector<float>& c, std::vector<int32_t>& i, std::vector<BNode>& n,
            int threads)
        : pb(b), pc(c), idx(i), nodes(n), spare(threads - 1)
    {
    }

    static int bin_of(float c, float lo, float scale)
    {
        int k = (int)((c - lo) * scale);
        return k < 0 ? 0 : (k >= NBINS ? NBINS - 1 : k);
    }

    void bin_range(int32_t b, int32_t e, const float* clo, const float* scale, Bins& B) const
    {
        B.clear();
        for (int32_t i = b; i < e; i++) {
            const int32_t p = idx[(size_t)i];
            for (int a = 0; a < 3; a++) {
                int k = bin_of(pc[3 * (size_t)p + a], clo[a], scale[a]);
                B.cnt[a][k]++;
                grow(B.box[a][k], pb[(size_t)p]);
            }
        }
    }

    void build(int32_t ni, int32_t b, int32_t e)
    {
        BNode& N = nodes[(size_t)ni];
        const int32_t n = e - b;
        Box box = empty_box(), cb = empty_box();
        for (int32_t i = b; i < e; i++) {
            const int32_t p = idx[(size_t)i];
            grow(box, pb[(size_t)p]);
            for (int a = 0; a < 3; a++) {
                cb.lo[a] = std::min(cb.lo[a], pc[3 * (size_t)p + a]);
                cb.hi[a] = std::max(cb.hi[a], pc[3 * (size_t)p + a]);
            }
        }
        N.box = box;
        N.first = b;
        N.count = n;
        N.left = N.right = -1;
        if (n <= 1)
            return;
        float scale[3];
        bool any = false;
        for (int a = 0; a < 3; a++) {
            float ext = cb.hi[a] - cb.lo[a];
            scale[a] = ext > 0 ? (float)NBINS / ext : 0.0f;
            any |= ext > 0;
        }
        int best_axis = -1, best_split = -1;
        float best_cost = INFINITY;
        if (any) {
            Bins B;
            if (n >= PAR_BIN) {
                const int nt = wbvh_threads();
                std::vector<Bins> part((size_t)nt);
                std::vector<std::thread> th;
                const int32_t chunk = (n + nt - 1) / nt;
                for (int t = 0; t < nt; t++)
                    th.emplace_back([&, t] {
                        int32_t cb0 = b + t * chunk, ce = std::min(e, cb0 + chunk);
                        if (cb0 < ce)
                            bin_range(cb0, ce, cb.lo, scale, part[(size_t)t]);
                        else
                            part[(size_t)t].clear();
                    });
                for (auto& t : th)
                    t.join();
                B = part[0];
                for (int t = 1; t < nt; t++)
                    B.add(part[(size_t)t]);
            } else
                bin_range(b, e, cb.lo, scale, B);
            const float pa = area(box);
            for (int a = 0; a < 3; a++) {
                if (scale[a] == 0.0f)
                    continue;
                float ra[NBINS];
                int32_t rc[NBINS];
                Box acc = empty_box();
                int32_t c = 0;
                for (int i = NBINS - 1; i >= 1; i--) {
                    grow(acc, B.box[a][i]);
                    c += B.cnt[a][i];
                    ra[i] = area(acc);
                    rc[i] = c;
                }
                acc = empty_box();
                c = 0;
                for (int i = 0; i < NBINS - 1; i++) {
                    grow(acc, B.box[a][i]);
                    c += B.cnt[a][i];
                    if (c == 0 || rc[i + 1] == 0)
                        continue;
                    float cost = ct + (area(acc) * (float)c + ra[i + 1] * (float)rc[i + 1]) / (pa > 0 ? pa : 1.0f);
                    if (cost < best_cost) {
                        best_cost = cost;
                        best_axis = a;
                        best_split = i;
                    }
                }
            }
        }
        int32_t mid;
        if (best_axis >= 0) {
            if (n <= W_MAX_LEAF && (float)n <= best_cost)
                return;   // a leaf is no more expensive than the best split
            const int a = best_axis;
            const float lo = cb.lo[a], sc = scale[a];
            auto it = std::partition(idx.begin() + b, idx.begin() + e,
                                     [&](int32_t p) { return bin_of(pc[3 * (size_t)p + a], lo, sc) <= best_split; });
            mid = (int32_t)(it - idx.begin());
        } else {
            // every centroid equal: a leaf if it fits, else halves in index order
            if (n <= W_MAX_LEAF)
                return;
            mid = b + n / 2;
        }
        if (mid == b || mid == e)
            mid = b + n / 2;
        const int32_t l = next.fetch_add(2);
        N.left = l;
        N.right = l + 1;
        const bool big = (mid - b) >= PAR_TASK && (e - mid) >= PAR_TASK;
        const bool par = big && spare.fetch_sub(1) > 0;
        if (big && !par)
            spare.fetch_add(1);   // no thread left: give the claim back
        if (par) {
            std::thread t([&, l, b, mid] { build(l, b, mid); });
            build(l + 1, mid, e);
            t.join();
            spare.fetch_add(1);
        } else {
            build(l, b, mid);
            build(l + 1, mid, e);
        }
    }
};

// One 4-wide node: the children's float boxes quantised to 8 bits per plane against the
// node box's low corner, low planes rounded down and high planes up (exact in double:
// origin, q and the power-of-two step are all representable), so each decoded box holds
// its float box.
// Per child: the area-weighted normal of its subtree's triangles and its vertices (for the
// orientation slabs, wbvh.hpp)
struct ChildGeom {
    double n[3];
    const int32_t* idx;   // the subtree's triangles: idx[first .. first + count)
    int32_t first, count;
};

// Backface cone code of a child (wbvh.hpp): theta = the largest angle between N and a triangle
// normal n below (triangles with n = 0 never hit: Mdet = 0); a ray with angle(N, d) < psi =
// acos(eps) - theta has angle(n, d) < acos(eps) for every n, i.e. exact n . d > eps |n| |d|,
// and the float Mdet = n . (-d) is then negative (its rounding is below 2^-22 |n| |d| for |n|
// in (1e-30, 1e27)).  cos(angle(N, d)) > cos psi  <=>  N . d > cos(psi) |N| |d|: the code is
// the threshold cos(psi) |N| + 0.01 (the kernel's rounding margin) rounded up in steps of
// W_CONE_STEP; 255 = no cone (psi <= 0, or a normal out of range).
int cone_code(const int* nq, const ChildGeom& g, const std::vector<GTri, DefaultInitAlloc<GTri>>& tris)
{
    const double Nl = std::sqrt((double)nq[0] * nq[0] + (double)nq[1] * nq[1] + (double)nq[2] * nq[2]);
    double theta = 0;
    for (int32_t i = g.first; i < g.first + g.count; i++) {
        const GTri& t = tris[(size_t)g.idx[i]];
        const double n0 = t.n[0], n1 = t.n[1], n2 = t.n[2];
        const double len = std::sqrt(n0 * n0 + n1 * n1 + n2 * n2);
        if (len == 0)
            continue;
        if (!(len > 1e-30 && len < 1e27))
            return 255;
        const double c = (n0 * nq[0] + n1 * nq[1] + n2 * nq[2]) / (len * Nl);
        theta = std::max(theta, std::acos(std::max(-1.0, std::min(1.0, c))));
    }
    const double psi = std::acos(W_CONE_EPS) - theta - 1e-9;
    if (!(psi > 0))
        return 255;
    const double code = std::ceil((std::cos(psi) * Nl + 0.01) / ((double)W_CONE_STEP * (1 - 1e-9)));
    return code <= 254 ? (int)code : 255;
}

WNode quantise(const Box* cb, const uint32_t* link, int nc, const ChildGeom* cg,
               const std::vector<GTri, DefaultInitAlloc<GTri>>* tris)
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
        smin[j] = INFINITY;
        smax[j] = -INFINITY;
        for (int32_t i = g.first; i < g.first + g.count; i++) {
            const GTri& t = (*tris)[(size_t)g.idx[i]];
            for (int v = 0; v < 3; v++) {
                double s = 0;
                for (int a = 0; a < 3; a++) {
                    double x = (double)t.a[a] + (v == 1 ? (double)t.ab[a] : v == 2 ? (double)t.ac[a] : 0.0);
                    s += nq[j][a] * (x - (double)org[a]);
                }
                smin[j] = std::min(smin[j], s);
                smax[j] = std::max(smax[j], s);
            }
        }
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
                   ((uint32_t)(uint8_t)(int8_t)nq[j][2] << 16) | ((uint32_t)cone_code(nq[j], cg[j], *tris) << 24);
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

struct Collapser {
    const std::vector<BNode>& bn;
    WBvh& out;
    const std::vector<int32_t>& idx;
    const std::vector<GTri, DefaultInitAlloc<GTri>>& tris;
    int64_t max_depth = 0;

    uint32_t leaf_ref(const BNode& L) const
    {
        return W_LEAF | ((uint32_t)L.first << 3) | (uint32_t)(L.count - 1);
    }

    uint32_t emit(int32_t bi, int depth)
    {
        max_depth = std::max<int64_t>(max_depth, depth);
        int32_t c[W_WIDTH];
        int nc = 0;
        const BNode& N = bn[(size_t)bi];
        if (N.left < 0)
            c[nc++] = bi;   // a leaf root: one child
        else {
            c[nc++] = N.left;
            c[nc++] = N.right;
            while (nc < W_WIDTH) {
                int pick = -1;
                float pa = -1.0f;
                for (int j = 0; j < nc; j++) {
                    const BNode& C = bn[(size_t)c[j]];
                    if (C.left >= 0 && area(C.box) > pa) {
                        pa = area(C.box);
                        pick = j;
                    }
                }
                if (pick < 0)
                    break;
                const BNode& C = bn[(size_t)c[pick]];
                c[pick] = C.left;
                c[nc++] = C.right;
            }
        }
        const uint32_t me = (uint32_t)out.nodes.size();
        out.nodes.emplace_back();
        Box cb[W_WIDTH];
        uint32_t link[W_WIDTH];
        for (int j = 0; j < W_WIDTH; j++) {
            cb[j] = empty_box();
            link[j] = W_EMPTY;
        }
        for (int j = 0; j < nc; j++) {
            const BNode& C = bn[(size_t)c[j]];
            cb[j] = C.box;
            if (C.left < 0) {
                link[j] = leaf_ref(C);
                out.stats.leaves++;
                out.stats.max_leaf = std::max<int64_t>(out.stats.max_leaf, C.count);
            } else
                link[j] = emit(c[j], depth + 1);
        }
        ChildGeom cg[W_WIDTH];
        for (int j = 0; j < nc; j++) {
            const BNode& C = bn[(size_t)c[j]];
            cg[j].idx = idx.data();
            cg[j].first = C.first;
            cg[j].count = C.count;
            cg[j].n[0] = cg[j].n[1] = cg[j].n[2] = 0;
            for (int32_t i = C.first; i < C.first + C.count; i++) {
                const GTri& t = tris[(size_t)idx[(size_t)i]];
                for (int a = 0; a < 3; a++)
                    cg[j].n[a] += t.n[a];
            }
        }
        WNode w = quantise(cb, link, nc, cg, &tris);
        out.nodes[me] = w;
        return me;
    }
};

}  // namespace

void build_wbvh(const FlatOctree& oct, WBvh& out)
{
    out = WBvh();
    const int64_t n = (int64_t)oct.tris.size();
    out.leaf_of_slot.assign((size_t)n, 0u);
    for (size_t i = 0; i < oct.nodes.size(); i++) {
        const GNode& g = oct.nodes[i];
        if (g.b & LEAF_BIT)
            for (uint32_t s = g.a; s < g.a + (g.b & ~LEAF_BIT); s++)
                out.leaf_of_slot[s] = (uint32_t)i;
    }
    if (n == 0 || n >= ((int64_t)1 << 28))
        return;
    std::vector<Box> pb((size_t)n);
    std::vector<float> pc(3 * (size_t)n);
    std::vector<int32_t> idx((size_t)n);
    for (int64_t i = 0; i < n; i++) {
        pb[(size_t)i] = tri_box(oct.tris[(size_t)i]);
        for (int a = 0; a < 3; a++)
            pc[3 * (size_t)i + a] = 0.5f * pb[(size_t)i].lo[a] + 0.5f * pb[(size_t)i].hi[a];
        idx[(size_t)i] = (int32_t)i;
    }
    std::vector<BNode> bn((size_t)(2 * n));
    const int nt = wbvh_threads();
    Builder B(pb, pc, idx, bn, nt);
    B.build(0, 0, (int32_t)n);
    bn.resize((size_t)B.next.load());
    // SAH cost of the binary tree (diagnostic)
    {
        const float ra = area(bn[0].box) > 0 ? area(bn[0].box) : 1.0f;
        double s = 0;
        for (const BNode& N : bn)
            s += (N.left < 0 ? (double)N.count : 1.0) * area(N.box) / ra;
        out.stats.sah = (float)s;
    }
    Collapser C{bn, out, idx, oct.tris};
    out.nodes.reserve(bn.size() / 2 + 1);
    C.emit(0, 1);
    out.stats.nodes = (int64_t)out.nodes.size();
    out.stats.depth = C.max_depth;
    out.stats.tris = n;
    out.tris.resize((size_t)n);
    out.slot.resize((size_t)n);
    out.leaf_of_k.resize((size_t)n);
    for (int64_t i = 0; i < n; i++) {
        out.tris[(size_t)i] = oct.tris[(size_t)idx[(size_t)i]];
        out.slot[(size_t)i] = idx[(size_t)i];
        out.leaf_of_k[(size_t)i] = out.leaf_of_slot[(size_t)idx[(size_t)i]];
    }
}

int64_t check_wbvh(const FlatOctree& oct, const WBvh& w)
{
    int64_t bad = 0;
    const size_t n = oct.tris.size();
    if (w.tris.size() != n || w.slot.size() != n || w.leaf_of_slot.size() != n || w.leaf_of_k.size() != n)
        return 1;
    for (size_t k = 0; k < n; k++)
        if (w.slot[k] >= 0 && (size_t)w.slot[k] < n && w.leaf_of_k[k] != w.leaf_of_slot[(size_t)w.slot[k]])
            bad++;
    if (n == 0)
        return w.nodes.empty() ? 0 : 1;
    std::vector<uint8_t> seen(n, 0), used(w.tris.size(), 0);
    for (size_t i = 0; i < n; i++) {
        int32_t s = w.slot[i];
        if (s < 0 || (size_t)s >= n || seen[(size_t)s]++)
            bad++;
        else if (std::memcmp(&w.tris[i], &oct.tris[(size_t)s], sizeof(GTri)))
            bad++;
    }
    for (size_t s = 0; s < n; s++) {
        uint32_t L = w.leaf_of_slot[s];
        if (L >= oct.nodes.size() || !(oct.nodes[L].b & LEAF_BIT) || s < oct.nodes[L].a ||
            s >= oct.nodes[L].a + (oct.nodes[L].b & ~LEAF_BIT))
            bad++;
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
                bad++;
                continue;
            }
            for (uint32_t k = first; k < first + cnt; k++) {
                if (used[k]++)
                    bad++;
                if (!inside(tri_box(w.tris[k]), it.box))
                    bad++;
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
                            bad++;
                    }
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
                            bad++;
                    }
                }
            }
            continue;
        }
        if (it.ref >= w.nodes.size() || ++visited > w.nodes.size()) {
            bad++;
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
                bad++;
                continue;
            }
            ch.path[ch.np++] = (it.ref << 3) | (uint32_t)j;
            stack.push_back(ch);
        }
    }
    for (size_t k = 0; k < n; k++)
        if (!used[k])
            bad++;
    return bad;
}

}  // namespace rt
