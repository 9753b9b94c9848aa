// octree.cpp -- see octree.hpp.  Host-side build stays faithful to the
// reference's insertion order and floating-point expressions so that the k-DOP
// slab distances, the octant assignment and the leaf triangle order are
// bit-identical to BVH(&triangles, max_depth, leaf_max_obj_count).
#include "octree.hpp"

#include <cmath>
#include <deque>
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
    Builder(const std::vector<BTri>& t, int max_depth, int leaf) : T(t), max_depth(max_depth), leaf(leaf) {}

    const std::vector<BTri>& T;
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

void build_flat_octree(const float* tri9, int64_t n, int max_depth, int leaf_max_obj_count, FlatOctree& out)
{
    out = FlatOctree();
    if (n <= 0)
        return;
    v3 PN[NPLANES];
    plane_normals(PN);

    std::vector<BTri> T((size_t)n);
    v3 mn = mk(INFINITY, INFINITY, INFINITY), mx = mk(-INFINITY, -INFINITY, -INFINITY);
    for (int64_t i = 0; i < n; i++) {
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
                const BTri& bt = T[(size_t)t];
                GTri gt;
                v3 ab = bt.v[1] - bt.v[0];
                v3 ac = bt.v[2] - bt.v[0];
                v3 nn = cross(bt.v[1] - bt.v[0], bt.v[2] - bt.v[0]);
                gt.a[0] = bt.v[0].x; gt.a[1] = bt.v[0].y; gt.a[2] = bt.v[0].z;
                gt.ab[0] = ab.x; gt.ab[1] = ab.y; gt.ab[2] = ab.z;
                gt.ac[0] = ac.x; gt.ac[1] = ac.y; gt.ac[2] = ac.z;
                gt.n[0] = nn.x; gt.n[1] = nn.y; gt.n[2] = nn.z;
                out.tris.push_back(gt);
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
    // the kernels' slab test relies on d_near <= d_far for every stored volume
    // (true for any node holding a triangle with finite vertices)
    out.ordered_slabs = true;
    for (const GNode& g : out.nodes)
        for (int i = 0; i < NPLANES; i++)
            if (!(g.dn[i] <= g.df[i]))
                out.ordered_slabs = false;
}

}  // namespace rt
