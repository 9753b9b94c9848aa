// octree.cpp -- see octree.hpp.  Host-side build stays faithful to the
// reference's insertion order and floating-point expressions so that the k-DOP
// slab distances, the octant assignment and the leaf triangle order are
// bit-identical to BVH(&triangles, max_depth, leaf_max_obj_count).
#include "octree.hpp"
#include "pool.hpp"

#include <algorithm>
#include <array>
#include <chrono>
#include <cstdio>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <utility>

namespace rt {

void plane_normals(v3 out[NPLANES])
{
    // bvh.cpp:8-16: std::sqrt(3.0f) / 3 and -std::sqrt(3.0f) / 3
    float s = std::sqrt(3.0f) / 3;
    float ms = -std::sqrt(3.0f) / 3;
    out[0] = mk(1, 0, 0);
    out[1] = mk(0, 1, 0);
    out[2] = mk(0, 0, 1);
    out[3] = mk(s, s, s);
    out[4] = mk(ms, s, s);
    out[5] = mk(ms, ms, s);
    out[6] = mk(s, ms, s);
}

namespace {

struct BTri {
    v3 v[3];
    v3 centroid;
    float dn[NPLANES], df[NPLANES];
};

struct BNode {
    v3 bmin, bmax;
    bool leaf = true;
    int child[8];
    std::vector<int> tris;
    float dn[NPLANES], df[NPLANES];
};

class Builder {
public:
    Builder(const std::vector<BTri, DefaultInitAlloc<BTri>>& t, int max_depth, int leaf)
        : T(t), max_depth(max_depth), leaf(leaf) {}

    const std::vector<BTri, DefaultInitAlloc<BTri>>& T;
    int max_depth, leaf;
    std::vector<BNode> nodes;

    int new_node(v3 mn, v3 mx)
    {
        BNode n;
        n.bmin = mn;
        n.bmax = mx;
        for (int i = 0; i < NPLANES; i++) {   // BoundingVolume(), bvh.h:24-31
            n.dn[i] = INFINITY;
            n.df[i] = -INFINITY;
        }
        nodes.push_back(std::move(n));
        return (int)nodes.size() - 1;
    }

    // OctreeNode::create_children, bvh.h:153-167 (children 2/4/6 use _min + Point(...))
    void create_children(int ni)
    {
        v3 mn = nodes[ni].bmin, mx = nodes[ni].bmax;
        float cx = (mn.x + mx.x) / 2;
        float cy = (mn.y + mx.y) / 2;
        float cz = (mn.z + mx.z) / 2;
        v3 lo[8] = {mn,
                    mk(cx, mn.y, mn.z),
                    mn + mk(0, cy, 0),
                    mk(cx, cy, mn.z),
                    mn + mk(0, 0, cz),
                    mk(cx, mn.y, cz),
                    mn + mk(0, cy, cz),
                    mk(cx, cy, cz)};
        v3 hi[8] = {mk(cx, cy, cz),     mk(mx.x, cy, cz),   mk(cx, mx.y, cz),   mk(mx.x, mx.y, cz),
                    mk(cx, cy, mx.z),   mk(mx.x, cy, mx.z), mk(cx, mx.y, mx.z), mk(mx.x, mx.y, mx.z)};
        for (int i = 0; i < 8; i++) {
            int c = new_node(lo[i], hi[i]);
            nodes[ni].child[i] = c;
        }
    }

    // OctreeNode::insert_to_children, bvh.h:195-210
    void insert_to_children(int ni, int t, int depth)
    {
        v3 c = T[t].centroid;
        v3 mn = nodes[ni].bmin, mx = nodes[ni].bmax;
        float cx = (mn.x + mx.x) / 2;
        float cy = (mn.y + mx.y) / 2;
        float cz = (mn.z + mx.z) / 2;
        int oct = 0;
        if (c.x > cx) oct += 1;
        if (c.y > cy) oct += 2;
        if (c.z > cz) oct += 4;
        insert(nodes[ni].child[oct], t, depth + 1);
    }

    // OctreeNode::insert, bvh.h:169-193
    void insert(int ni, int t, int depth)
    {
        bool depth_exceeded = depth == max_depth;
        if (nodes[ni].leaf || depth_exceeded) {
            nodes[ni].tris.push_back(t);
            if (nodes[ni].tris.size() > (size_t)(long)leaf && !depth_exceeded) {
                nodes[ni].leaf = false;
                create_children(ni);
                std::vector<int> list = std::move(nodes[ni].tris);
                nodes[ni].tris.clear();
                for (int k : list)
                    insert_to_children(ni, k, depth);
            }
        } else
            insert_to_children(ni, t, depth);
    }

    // OctreeNode::compute_volume, bvh.h:141-151
    void compute_volume(int ni)
    {
        if (nodes[ni].leaf) {
            for (int t : nodes[ni].tris)
                for (int i = 0; i < NPLANES; i++) {
                    nodes[ni].dn[i] = smin(nodes[ni].dn[i], T[t].dn[i]);
                    nodes[ni].df[i] = smax(nodes[ni].df[i], T[t].df[i]);
                }
        } else {
            for (int k = 0; k < 8; k++) {
                int c = nodes[ni].child[k];
                compute_volume(c);
                for (int i = 0; i < NPLANES; i++) {
                    nodes[ni].dn[i] = smin(nodes[ni].dn[i], nodes[c].dn[i]);
                    nodes[ni].df[i] = smax(nodes[ni].df[i], nodes[c].df[i]);
                }
            }
        }
    }

    void stats(int ni, int depth, OctreeStats& s) const
    {
        const BNode& n = nodes[ni];
        if (depth > s.max_depth) s.max_depth = depth;
        if (n.leaf) {
            s.leaves++;
            if (n.tris.empty()) s.empty_leaves++;
            if ((int64_t)n.tris.size() > s.max_leaf) s.max_leaf = (int64_t)n.tris.size();
            return;
        }
        s.inner++;
        for (int k = 0; k < 8; k++) stats(n.child[k], depth + 1, s);
    }
};

}  // namespace

namespace {

// Triangle prep for [b, e): Triangle::bbox_centroid, BoundingVolume::triangle_volume
// and the BVH::BVH root box (running min / max over the vertices; never NaN, so
// the order of the partial boxes does not matter).
using BTriVec = std::vector<BTri, DefaultInitAlloc<BTri>>;

void prep_triangles(const float* tri9, int64_t b, int64_t e, BTriVec& T, v3& mn_io, v3& mx_io)
{
    v3 PN[NPLANES];
    plane_normals(PN);
    v3 mn = mn_io, mx = mx_io;   // locals: the callers' partial boxes share cache lines
    for (int64_t i = b; i < e; i++) {
        const float* p = tri9 + 9 * i;
        BTri& t = T[(size_t)i];
        for (int k = 0; k < 3; k++) t.v[k] = mk(p[3 * k], p[3 * k + 1], p[3 * k + 2]);
        // Triangle::bbox_centroid, triangle.cpp:162-165: (min(a, min(b, c)) + max(a, max(b, c))) / 2
        v3 lo = mk(smin(t.v[0].x, smin(t.v[1].x, t.v[2].x)), smin(t.v[0].y, smin(t.v[1].y, t.v[2].y)),
                   smin(t.v[0].z, smin(t.v[1].z, t.v[2].z)));
        v3 hi = mk(smax(t.v[0].x, smax(t.v[1].x, t.v[2].x)), smax(t.v[0].y, smax(t.v[1].y, t.v[2].y)),
                   smax(t.v[0].z, smax(t.v[1].z, t.v[2].z)));
        float kk = 1.f / 2;   // Point / float, vec.cpp:56-60
        t.centroid = kk * (lo + hi);
        // BoundingVolume::triangle_volume, bvh.h:33-45
        for (int p2 = 0; p2 < NPLANES; p2++) {
            float dn = INFINITY, df = -INFINITY;
            for (int k = 0; k < 3; k++) {
                float dist = dot(PN[p2], t.v[k]);
                dn = smin(dn, dist);
                df = smax(df, dist);
            }
            t.dn[p2] = dn;
            t.df[p2] = df;
        }
        // BVH::BVH root box, bvh.cpp:27-36
        for (int k = 0; k < 3; k++) {
            mn = mk(smin(mn.x, t.v[k].x), smin(mn.y, t.v[k].y), smin(mn.z, t.v[k].z));
            mx = mk(smax(mx.x, t.v[k].x), smax(mx.y, t.v[k].y), smax(mx.z, t.v[k].z));
        }
    }
    mn_io = mn;
    mx_io = mx;
}

GTri make_gtri(const BTri& bt)
{
    GTri gt;
    v3 ab = bt.v[1] - bt.v[0];
    v3 ac = bt.v[2] - bt.v[0];
    v3 nn = cross(bt.v[1] - bt.v[0], bt.v[2] - bt.v[0]);
    gt.a[0] = bt.v[0].x; gt.a[1] = bt.v[0].y; gt.a[2] = bt.v[0].z;
    gt.ab[0] = ab.x; gt.ab[1] = ab.y; gt.ab[2] = ab.z;
    gt.ac[0] = ac.x; gt.ac[1] = ac.y; gt.ac[2] = ac.z;
    gt.n[0] = nn.x; gt.n[1] = nn.y; gt.n[2] = nn.z;
    return gt;
}

void finish_checks(FlatOctree& out)
{
    // the kernels' slab test relies on d_near <= d_far for every stored volume
    // (true for any node holding a triangle with finite vertices)
    out.ordered_slabs = true;
    for (const GNode& g : out.nodes)
        for (int i = 0; i < NPLANES; i++)
            if (!(g.dn[i] <= g.df[i]))
                out.ordered_slabs = false;
}

}  // namespace

// The reference's insertion-order build, restated one insert at a time (kept as
// the executable specification the parallel build is tested against).
void build_flat_octree_serial(const float* tri9, int64_t n, int max_depth, int leaf_max_obj_count, FlatOctree& out)
{
    out = FlatOctree();
    if (n <= 0)
        return;
    BTriVec T((size_t)n);
    v3 mn = mk(INFINITY, INFINITY, INFINITY), mx = mk(-INFINITY, -INFINITY, -INFINITY);
    prep_triangles(tri9, 0, n, T, mn, mx);

    Builder B(T, max_depth, leaf_max_obj_count);
    B.nodes.reserve((size_t)(n / 2 + 64));
    int root = B.new_node(mn, mx);
    for (int64_t i = 0; i < n; i++)
        B.insert(root, (int)i, 0);
    B.compute_volume(root);
    B.stats(root, 0, out.stats);
    out.stats.nodes = (int64_t)B.nodes.size();

    // ---- flatten (breadth-first; non-empty children contiguous, in octant order) ----
    out.nodes.reserve(B.nodes.size());
    out.tris.reserve((size_t)n);
    out.tri_id.reserve((size_t)n);
    std::deque<std::pair<int, int>> q;   // (builder node, depth)
    auto emit = [&](int bi) {
        GNode g;
        for (int i = 0; i < NPLANES; i++) {
            g.dn[i] = B.nodes[bi].dn[i];
            g.df[i] = B.nodes[bi].df[i];
        }
        g.a = 0;
        g.b = 0;
        out.nodes.push_back(g);
    };
    const BNode& r = B.nodes[root];
    if (r.leaf && r.tris.empty())
        return;   // no geometry
    emit(root);
    q.emplace_back(root, 0);
    size_t fi = 0;
    int maxd = 0;
    while (!q.empty()) {
        auto [bi, depth] = q.front();
        q.pop_front();
        GNode& g = out.nodes[fi];
        const BNode& bn = B.nodes[bi];
        if (depth > maxd) maxd = depth;
        if (bn.leaf) {
            g.a = (uint32_t)out.tris.size();
            g.b = LEAF_BIT | (uint32_t)bn.tris.size();
            for (int t : bn.tris) {
                out.tris.push_back(make_gtri(T[(size_t)t]));
                out.tri_id.push_back(t);
            }
        } else {
            uint32_t mask = 0;
            for (int k = 0; k < 8; k++) {
                const BNode& c = B.nodes[bn.child[k]];
                if (!(c.leaf && c.tris.empty()))
                    mask |= 1u << k;
            }
            // g may dangle after emit(): write a/b first
            out.nodes[fi].a = (uint32_t)out.nodes.size();
            out.nodes[fi].b = (uint32_t)__builtin_popcount(mask);
            for (int k = 0; k < 8; k++)
                if (mask & (1u << k)) {
                    emit(bn.child[k]);
                    q.emplace_back(bn.child[k], depth + 1);
                }
        }
        fi++;
    }
    out.levels = maxd + 1;
    finish_checks(out);
}


// ---------------------------------------------------------------------------
// Parallel build with the same output.  The insertion-order build has a closed
// form: a node at depth d that receives c triangles is inner iff c > leaf and
// d != max_depth (bvh.h:179-185: a leaf splits on the insert that makes its size
// exceed `leaf`, and its list is then re-inserted in order), and each child
// receives its parent's triangles in insertion order (octant of the bbox centroid
// against the node's cell centre, bvh.h:195-210).  So the tree is a top-down,
// stable partition by octant, level by level; every level's nodes are processed
// in parallel.  BFS order of the flattened tree is level order (children of
// earlier nodes first, octant order), exactly what the serial flatten emits.
// ---------------------------------------------------------------------------
namespace {

struct Item {
    v3 c;        // Triangle::bbox_centroid
    int32_t t;   // caller triangle index
};

struct LNode {
    int64_t begin = 0, end = 0;   // its triangles: idx[begin, end), insertion order
    v3 mn, mx;                    // OctreeNode::_min / _max
    int64_t child = -1;           // first of its 8 children in the next level (inner)
    bool leaf = true;
    float dn[NPLANES], df[NPLANES];
};

}  // namespace

void build_flat_octree(const float* tri9, int64_t n, int max_depth, int leaf_max_obj_count, FlatOctree& out)
{
    out = FlatOctree();
    if (n <= 0)
        return;
    const int nt = build_threads();
    const bool prof = std::getenv("RT_BUILD_PROFILE") != nullptr;
    auto tick = std::chrono::steady_clock::now();
    auto phase = [&](const char* what) {
        if (!prof)
            return;
        auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[octree] %-10s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(now - tick).count());
        tick = now;
    };
    struct ExitPhase {   // the locals' destructors, reported after them
        decltype(phase)& ph;
        ~ExitPhase() { ph("exit"); }
    } exit_phase{phase};
    Pool& pool = build_pool();
    phase("pool");

    // ---- triangle prep + root box ----
    BTriVec T((size_t)n);
    std::vector<v3> pmn((size_t)nt, mk(INFINITY, INFINITY, INFINITY)), pmx((size_t)nt, mk(-INFINITY, -INFINITY, -INFINITY));
    {
        std::atomic<int64_t> next{0};
        const int64_t chunk = 16384;
        pool.run([&](int w) {
            for (;;) {
                int64_t b = next.fetch_add(chunk);
                if (b >= n)
                    return;
                prep_triangles(tri9, b, std::min(n, b + chunk), T, pmn[(size_t)w], pmx[(size_t)w]);
            }
        });
    }
    v3 mn = pmn[0], mx = pmx[0];
    for (int w = 1; w < nt; w++) {
        mn = mk(smin(mn.x, pmn[(size_t)w].x), smin(mn.y, pmn[(size_t)w].y), smin(mn.z, pmn[(size_t)w].z));
        mx = mk(smax(mx.x, pmx[(size_t)w].x), smax(mx.y, pmx[(size_t)w].y), smax(mx.z, pmx[(size_t)w].z));
    }

    phase("prep");
    // ---- structure, level by level ----
    // (centroid, triangle) items, partitioned level by level; a node's items stay
    // contiguous and in insertion order
    std::vector<Item, DefaultInitAlloc<Item>> idx((size_t)n);
    parallel_for(pool, n, 65536, [&](int64_t i) {
        idx[(size_t)i].c = T[(size_t)i].centroid;
        idx[(size_t)i].t = (int32_t)i;
    });
    std::vector<std::vector<LNode>> L(1);
    L[0].resize(1);
    L[0][0].begin = 0;
    L[0][0].end = n;
    L[0][0].mn = mn;
    L[0][0].mx = mx;
    const size_t lim = (size_t)(long)leaf_max_obj_count;   // bvh.h:181: size() > leaf_max_obj_count
    std::vector<std::vector<Item>> scratch((size_t)nt);
    for (int d = 0;; d++) {
        std::vector<LNode>& cur = L[(size_t)d];
        int64_t ninner = 0;
        for (LNode& nd : cur) {
            nd.leaf = !((size_t)(nd.end - nd.begin) > lim && d != max_depth);
            if (!nd.leaf)
                nd.child = 8 * ninner++;
        }
        if (ninner == 0)
            break;
        std::vector<LNode> next((size_t)(8 * ninner));
        // insert_to_children (bvh.h:195-210): octant of the bbox centroid vs the cell centre
        auto octant = [&](const Item& it, float cx, float cy, float cz) {
            const v3& c = it.c;
            int oct = 0;
            if (c.x > cx) oct += 1;
            if (c.y > cy) oct += 2;
            if (c.z > cz) oct += 4;
            return oct;
        };
        // create_children (bvh.h:153-167), children 2/4/6 from _min + Point(...)
        auto make_children = [&](const LNode& nd, float cx, float cy, float cz, const int64_t* start,
                                 const int64_t* cnt) {
            v3 cmn = nd.mn, cmx = nd.mx;
            v3 lo[8] = {cmn,
                        mk(cx, cmn.y, cmn.z),
                        cmn + mk(0, cy, 0),
                        mk(cx, cy, cmn.z),
                        cmn + mk(0, 0, cz),
                        mk(cx, cmn.y, cz),
                        cmn + mk(0, cy, cz),
                        mk(cx, cy, cz)};
            v3 hi[8] = {mk(cx, cy, cz),      mk(cmx.x, cy, cz),    mk(cx, cmx.y, cz),    mk(cmx.x, cmx.y, cz),
                        mk(cx, cy, cmx.z),   mk(cmx.x, cy, cmx.z), mk(cx, cmx.y, cmx.z), mk(cmx.x, cmx.y, cmx.z)};
            for (int o = 0; o < 8; o++) {
                LNode& c = next[(size_t)(nd.child + o)];
                c.begin = start[o];
                c.end = start[o] + cnt[o];
                c.mn = lo[o];
                c.mx = hi[o];
            }
        };
        const int64_t BIG = 1 << 17;
        // big nodes: one at a time, every worker on a contiguous chunk (counts per chunk,
        // then ordered scatters: stable)
        for (size_t i = 0; i < cur.size(); i++) {
            const LNode& nd = cur[i];
            if (nd.leaf || nd.end - nd.begin < BIG)
                continue;
            float cx = (nd.mn.x + nd.mx.x) / 2, cy = (nd.mn.y + nd.mx.y) / 2, cz = (nd.mn.z + nd.mx.z) / 2;
            const int64_t len = nd.end - nd.begin;
            std::vector<Item> seg(idx.begin() + nd.begin, idx.begin() + nd.end);
            std::vector<uint8_t> oc((size_t)len);
            std::vector<std::array<int64_t, 8>> wc((size_t)nt);
            auto chunk_of = [&](int w, int64_t& b, int64_t& e) {
                b = len * w / nt;
                e = len * (w + 1) / nt;
            };
            pool.run([&](int w) {
                int64_t b, e;
                chunk_of(w, b, e);
                std::array<int64_t, 8> c{};
                for (int64_t k = b; k < e; k++) {
                    int o = octant(seg[(size_t)k], cx, cy, cz);
                    oc[(size_t)k] = (uint8_t)o;
                    c[(size_t)o]++;
                }
                wc[(size_t)w] = c;
            });
            int64_t cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0}, start[8];
            for (int w = 0; w < nt; w++)
                for (int o = 0; o < 8; o++) cnt[o] += wc[(size_t)w][(size_t)o];
            int64_t acc = nd.begin;
            for (int o = 0; o < 8; o++) {
                start[o] = acc;
                acc += cnt[o];
            }
            std::vector<std::array<int64_t, 8>> wpos((size_t)nt);
            for (int o = 0; o < 8; o++) {
                int64_t p = start[o];
                for (int w = 0; w < nt; w++) {
                    wpos[(size_t)w][(size_t)o] = p;
                    p += wc[(size_t)w][(size_t)o];
                }
            }
            pool.run([&](int w) {
                int64_t b, e;
                chunk_of(w, b, e);
                std::array<int64_t, 8> pos = wpos[(size_t)w];
                for (int64_t k = b; k < e; k++)
                    idx[(size_t)pos[oc[(size_t)k]]++] = seg[(size_t)k];
            });
            make_children(nd, cx, cy, cz, start, cnt);
        }
        std::atomic<int64_t> cursor{0};
        const int64_t ncur = (int64_t)cur.size();
        const int64_t grab = std::max<int64_t>(1, ncur / (16 * nt));
        pool.run([&](int w) {
            std::vector<Item>& seg = scratch[(size_t)w];
            std::vector<uint8_t> oc;
            int64_t i = 0, iend = 0;
            for (;; i++) {
                if (i >= iend) {
                    i = cursor.fetch_add(grab);
                    if (i >= ncur)
                        return;
                    iend = std::min(ncur, i + grab);
                }
                const LNode& nd = cur[(size_t)i];
                if (nd.leaf || nd.end - nd.begin >= BIG)
                    continue;
                float cx = (nd.mn.x + nd.mx.x) / 2;
                float cy = (nd.mn.y + nd.mx.y) / 2;
                float cz = (nd.mn.z + nd.mx.z) / 2;
                int64_t cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                seg.assign(idx.begin() + nd.begin, idx.begin() + nd.end);
                oc.resize(seg.size());
                for (size_t k = 0; k < seg.size(); k++) {
                    int o = octant(seg[k], cx, cy, cz);
                    oc[k] = (uint8_t)o;
                    cnt[o]++;
                }
                int64_t start[8], pos[8];
                int64_t acc = nd.begin;
                for (int o = 0; o < 8; o++) {
                    start[o] = pos[o] = acc;
                    acc += cnt[o];
                }
                // stable scatter
                for (size_t k = 0; k < seg.size(); k++)
                    idx[(size_t)pos[oc[k]]++] = seg[k];
                make_children(nd, cx, cy, cz, start, cnt);
            }
        });
        L.push_back(std::move(next));   // (invalidates cur)
    }

    phase("structure");
    // ---- compute_volume (bvh.h:141-151), bottom-up ----
    for (int d = (int)L.size() - 1; d >= 0; d--) {
        std::vector<LNode>& cur = L[(size_t)d];
        const std::vector<LNode>* below = d + 1 < (int)L.size() ? &L[(size_t)d + 1] : nullptr;
        parallel_for(pool, (int64_t)cur.size(), 256, [&](int64_t i) {
            LNode& nd = cur[(size_t)i];
            for (int p = 0; p < NPLANES; p++) {
                nd.dn[p] = INFINITY;
                nd.df[p] = -INFINITY;
            }
            if (nd.leaf) {
                for (int64_t k = nd.begin; k < nd.end; k++) {
                    const BTri& t = T[(size_t)idx[(size_t)k].t];
                    for (int p = 0; p < NPLANES; p++) {
                        nd.dn[p] = smin(nd.dn[p], t.dn[p]);
                        nd.df[p] = smax(nd.df[p], t.df[p]);
                    }
                }
            } else {
                for (int o = 0; o < 8; o++) {
                    const LNode& c = (*below)[(size_t)(nd.child + o)];
                    for (int p = 0; p < NPLANES; p++) {
                        nd.dn[p] = smin(nd.dn[p], c.dn[p]);
                        nd.df[p] = smax(nd.df[p], c.df[p]);
                    }
                }
            }
        });
    }

    phase("volumes");
    // ---- statistics of the unflattened tree ----
    OctreeStats& st = out.stats;
    for (size_t d = 0; d < L.size(); d++)
        for (const LNode& nd : L[d]) {
            if ((int64_t)d > st.max_depth) st.max_depth = (int64_t)d;
            if (nd.leaf) {
                st.leaves++;
                int64_t c = nd.end - nd.begin;
                if (c == 0) st.empty_leaves++;
                if (c > st.max_leaf) st.max_leaf = c;
            } else
                st.inner++;
        }
    st.nodes = 1 + 8 * st.inner;

    // ---- flatten in level order, empty leaves dropped ----
    auto kept = [](const LNode& nd) { return !(nd.leaf && nd.begin == nd.end); };
    std::vector<std::vector<int64_t>> flat(L.size());   // flat index per node (-1: dropped)
    int64_t nflat = 0, ntri = 0;
    int maxd = 0;
    std::vector<std::vector<int64_t>> slot(L.size());   // first triangle slot per kept leaf
    for (size_t d = 0; d < L.size(); d++) {
        flat[d].assign(L[d].size(), -1);
        slot[d].assign(L[d].size(), -1);
        for (size_t i = 0; i < L[d].size(); i++)
            if (kept(L[d][i])) {
                flat[d][i] = nflat++;
                maxd = (int)d;
                if (L[d][i].leaf) {
                    slot[d][i] = ntri;
                    ntri += L[d][i].end - L[d][i].begin;
                }
            }
    }
    out.nodes.resize((size_t)nflat);
    out.tris.resize((size_t)ntri);
    out.tri_id.resize((size_t)ntri);
    for (size_t d = 0; d < L.size(); d++) {
        const std::vector<LNode>& cur = L[d];
        parallel_for(pool, (int64_t)cur.size(), 256, [&](int64_t i) {
            const LNode& nd = cur[(size_t)i];
            int64_t fi = flat[d][(size_t)i];
            if (fi < 0)
                return;
            GNode& g = out.nodes[(size_t)fi];
            for (int p = 0; p < NPLANES; p++) {
                g.dn[p] = nd.dn[p];
                g.df[p] = nd.df[p];
            }
            if (nd.leaf) {
                int64_t s0 = slot[d][(size_t)i];
                g.a = (uint32_t)s0;
                g.b = LEAF_BIT | (uint32_t)(nd.end - nd.begin);
                for (int64_t k = nd.begin; k < nd.end; k++) {
                    int32_t t = idx[(size_t)k].t;
                    out.tris[(size_t)(s0 + k - nd.begin)] = make_gtri(T[(size_t)t]);
                    out.tri_id[(size_t)(s0 + k - nd.begin)] = t;
                }
            } else {
                // first kept child: children of earlier nodes precede, so it is the
                // lowest flat index among this node's kept children
                uint32_t k = 0;
                int64_t first = -1;
                for (int o = 0; o < 8; o++) {
                    int64_t f = flat[d + 1][(size_t)(nd.child + o)];
                    if (f >= 0) {
                        if (first < 0) first = f;
                        k++;
                    }
                }
                g.a = (uint32_t)first;
                g.b = k;
            }
        });
    }
    phase("flatten");
    out.levels = maxd + 1;
    finish_checks(out);
    phase("checks");
    free_later(std::move(T), std::move(idx), std::move(L), std::move(scratch), std::move(flat), std::move(slot));
}

}  // namespace rt
