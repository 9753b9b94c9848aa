// octree.hpp -- host-side octree BVH build (the reference's algorithm, restated)
// and its flattening into the gfx950 traversal layout.
//
// Build: BVH::BVH / build_bvh (tp2/projets/bvh.cpp:19-66), OctreeNode::insert /
// insert_to_children / create_children / compute_volume (tp2/projets/bvh.h:141-210),
// BoundingVolume (bvh.h:15-74), PLANE_NORMALS (bvh.cpp:8-16).
//
// Flattened layout (HBM):
//   GNode[ ]  64 B each: 7 near + 7 far k-DOP slab distances, then
//             a = first child (inner) or first triangle (leaf),
//             b = LEAF_BIT | triangle count (leaf) or the number of
//                 non-empty child octants (inner; children a .. a+b-1 in octant order).
//             The non-empty children of an inner node are contiguous, in octant
//             order, so heap insertion order (bvh.h:251-256) is rank order.
//             Empty leaves are dropped: their empty volume (+inf / -inf) can
//             never pass BoundingVolume::intersect for a non-NaN ray.
//   GTri[ ]   48 B each, leaf-contiguous: a, b - a, c - a, cross(b - a, c - a)
//             (Triangle::_normal, triangle.cpp:11-12), plus tri_id[ ] mapping
//             back to the caller's triangle index.
#pragma once

#include <stdint.h>

#include <memory>
#include <utility>
#include <vector>

#include "rt_math.hpp"

namespace rt {

constexpr int NPLANES = 7;
// BVH::BoundingVolume::PLANE_NORMALS (bvh.cpp:8-16) as literals: sqrtf(3) / 3 in
// fp32 is 0x3f13cd3a; plane_normals() computes them the reference's way and the
// renderer checks the two agree (kernels read the literals).
constexpr float PN_S = 0x1.279a74p-1f;
constexpr float PLANE_N[NPLANES][3] = {{1, 0, 0},           {0, 1, 0},           {0, 0, 1},
                                       {PN_S, PN_S, PN_S},  {-PN_S, PN_S, PN_S}, {-PN_S, -PN_S, PN_S},
                                       {PN_S, -PN_S, PN_S}};
constexpr uint32_t LEAF_BIT = 0x80000000u;

struct alignas(16) GNode {
    float dn[NPLANES];
    float df[NPLANES];
    uint32_t a;
    uint32_t b;
};
static_assert(sizeof(GNode) == 64, "GNode must be 64 B");

struct alignas(16) GTri {
    float a[3];
    float ab[3];
    float ac[3];
    float n[3];
};
static_assert(sizeof(GTri) == 48, "GTri must be 48 B");

// PLANE_NORMALS (bvh.cpp:8-16), in float, with the reference's expressions.
void plane_normals(v3 out[NPLANES]);

// std::allocator that default-initialises (no zero fill of arrays about to be overwritten)
template <class T>
struct DefaultInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = DefaultInitAlloc<U>;
    };
    DefaultInitAlloc() = default;
    template <class U>
    DefaultInitAlloc(const DefaultInitAlloc<U>&) {}
    template <class U>
    void construct(U* p)
    {
        ::new (static_cast<void*>(p)) U;
    }
    template <class U, class... A>
    void construct(U* p, A&&... a)
    {
        ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
    }
};

struct OctreeStats {
    int64_t inner = 0, leaves = 0, empty_leaves = 0, max_leaf = 0, max_depth = 0, nodes = 0;
};

struct FlatOctree {
    std::vector<GNode, DefaultInitAlloc<GNode>> nodes;       // nodes[0] = root (empty when there are no triangles)
    std::vector<GTri, DefaultInitAlloc<GTri>> tris;          // leaf-contiguous
    std::vector<int32_t, DefaultInitAlloc<int32_t>> tri_id;  // GTri slot -> caller triangle index
    int levels = 0;                // max depth + 1 of the flattened tree
    bool ordered_slabs = true;     // every node has dn[i] <= df[i] (kernels.hip vol_test)
    OctreeStats stats;             // of the unflattened (reference) tree
};

// Builds the reference octree over tri9 ([n][9] world-space vertices) and flattens it
// (parallel level-by-level build; RT_BUILD_THREADS threads, default min(cores, 16)).
void build_flat_octree(const float* tri9, int64_t n, int max_depth, int leaf_max_obj_count, FlatOctree& out);
// The same tree by the reference's one-insert-at-a-time algorithm (the specification
// the parallel build is tested against: rt_octree_digest).
void build_flat_octree_serial(const float* tri9, int64_t n, int max_depth, int leaf_max_obj_count, FlatOctree& out);

}  // namespace rt
