// kernels.hip -- gfx950 (CDNA4) kernels for the primary-ray + shadow-ray hot path.
//
// One 64-lane wavefront renders one 8x8 pixel tile (one lane per pixel).  Each
// lane runs the reference's best-first octree traversal
// (OctreeNode::intersect, tp2/projets/bvh.h:212-287) as an iterative state
// machine whose visit order is exactly the reference's recursion:
//   * children that pass BoundingVolume::intersect (bvh.h:79-105) are ordered
//     as std::priority_queue<..., std::greater<>> pops them (bvh.h:250-256):
//     ascending t_near; when two t_near compare equal the libstdc++ heap is
//     emulated move for move, so ties pop in the same order;
//   * after a child returns true, the remaining siblings are skipped as soon as
//     the closest hit is nearer than the next t_near (bvh.h:264-276);
//   * a leaf "returns" hit.t > 0 of the query-global hit record (bvh.h:235-248).
// The per-depth pending-children queues live in LDS (one 8-byte entry per depth
// per lane: first child index + packed 3-bit child ranks + count); the next
// sibling's t_near is recomputed from its 64-byte node when needed instead of
// being stored.  Node and triangle records are 64 B / 48 B and read with
// 16-byte loads.  All arithmetic follows the reference expression trees with
// no contraction (-ffp-contract=off) and IEEE division / sqrt, so results are
// bit-identical to the reference compiled with -ffp-contract=off.
#include <hip/hip_runtime.h>
#include <stdint.h>
#if defined(RT_COUNT) && RT_COUNT
// diagnostic builds: per wave iteration of the wide-BVH loop, the lanes in its node (leaf)
// branch and whether they share one node (leaf) -- how often a scalar-cache path could
// serve the step.  g_wsteps: [0] node steps, [1] of them uniform, [2] leaf steps, [3]
// uniform, [4] / [5] lanes, [6] / [7] distinct nodes / leaves (tools/count_gpu_work.py)
__device__ unsigned long long g_wsteps[8];
__device__ __forceinline__ void w_step_hook(uint32_t cur, int leaf)
{
    const uint64_t act = __ballot(1);
    uint64_t left = act;
    unsigned distinct = 0;
    while (left) {
        const uint32_t f = (uint32_t)__builtin_amdgcn_readlane((int)cur, __ffsll((unsigned long long)left) - 1);
        left &= ~__ballot(cur == f);
        distinct++;
    }
    if ((int)__lane_id() == __ffsll((unsigned long long)act) - 1) {
        atomicAdd(&g_wsteps[2 * leaf], 1ull);
        if (distinct == 1)
            atomicAdd(&g_wsteps[2 * leaf + 1], 1ull);
        atomicAdd(&g_wsteps[4 + leaf], (unsigned long long)__popcll(act));
        atomicAdd(&g_wsteps[6 + leaf], (unsigned long long)distinct);
    }
}
#define W_STEP_HOOK(cur, leaf) w_step_hook(cur, leaf)
#endif
#include "kparams.hpp"
#include "rt_math.hpp"
#include "wbvh.hpp"

namespace rt {

constexpr int WAVES_PER_BLOCK = 4;
constexpr int BLOCK = 64 * WAVES_PER_BLOCK;

#ifndef RT_OCC
#define RT_OCC 5
#endif
#ifndef RT_OCC_PLAIN
#define RT_OCC_PLAIN 3   // the plain kernel: 168 VGPRs (r04, the sound wide query: 4.31 ms vs 5.4 at 4 waves with
                         // 103 spills, 5.17 at 2; r02's unsound query: 0.67 ms at 4 vs 0.71 at 5, 0.69 at 3)
#endif
#ifndef RT_OCC_OCT
#define RT_OCC_OCT 5     // ray_trace_kernel<false, true, true>: the octree walk alone (first frames, exact mode)
#endif
// RT_COUNT=1 (diagnostic builds only, tools/count_gpu_work.py): every traversal adds
// its k-DOP and Moller-Trumbore test counts to P.counters[4..7] (whole-line queries:
// 4 / 5, segment queries: 6 / 7), the work the kernel actually did
#ifndef RT_COUNT
#define RT_COUNT 0
#endif
// RT_PHASE_TIME=1 (diagnostic builds, tools/phase_time.py): shader cycles per wave spent in
// each phase of the plain kernel's pixel loop (ph_mark), written to P.dbg
#ifndef RT_PHASE_TIME
#define RT_PHASE_TIME 0
#endif

struct TRay {
    v3 o, d;
    float den[NPLANES], num[NPLANES];   // num[i] = NaN where den[i] == 0 (see vol_test)
    bool nan;
    float lo, hi;   // query segment of a SEG traversal (seg_margin): volumes outside [lo, hi] are not entered
};


// HitInfo (hitInfo.h:8-24) reduced to what the kernels need.
struct Rec {
    int tri;      // caller triangle index (HitInfo::triangle), -1 == nullptr
    float t, u, v;
    int mat;
    v3 normal, tangent;
};

__device__ __forceinline__ Rec rec_fresh()
{
    Rec r;
    r.tri = -1; r.t = -1.0f; r.u = 1.0f; r.v = 0.0f; r.mat = -1;
    r.normal = mk(0, 0, 0); r.tangent = mk(0, 0, 0);
    return r;
}

// OctreeNode::intersect(ray, hit) prologue, bvh.h:216-223
__device__ __forceinline__ TRay make_ray(const KParams& P, v3 o, v3 d)
{
    TRay R;
    R.o = o;
    R.d = d;
    bool nan = false;
#pragma unroll
    for (int i = 0; i < NPLANES; i++) {
        v3 n = mk(PLANE_N[i][0], PLANE_N[i][1], PLANE_N[i][2]);
        R.den[i] = dot(n, d);
        R.num[i] = dot(n, o);
        nan |= (R.den[i] != R.den[i]) || (R.num[i] != R.num[i]);
        // a plane with denom == 0 is skipped (bvh.h:86-87): a NaN numerator makes
        // both of its quotients NaN, which the max / min below ignore
        if (R.den[i] == 0.0f)
            R.num[i] = __int_as_float(0x7fc00000);
    }
    R.nan = nan;
    R.lo = -INFINITY;
    R.hi = INFINITY;
    return R;
}

// make_ray's R.nan alone (the primary pass needs no plane products)
// A copy of v the compiler cannot prove equal to v: the exact path's ray setup (make_ray) is
// then computed inside that rarely taken branch instead of being merged with an earlier
// one and held in registers across the wide-BVH query.
__device__ __forceinline__ v3 opaque(v3 v)
{
    asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z));
    return v;
}

__device__ __forceinline__ bool ray_is_nan(v3 o, v3 d)
{
    bool nan = false;
#pragma unroll
    for (int i = 0; i < NPLANES; i++) {
        v3 n = mk(PLANE_N[i][0], PLANE_N[i][1], PLANE_N[i][2]);
        float den = dot(n, d), num = dot(n, o);
        nan |= (den != den) || (num != num);
    }
    return nan;
}

struct NodeBox {
    float dn[NPLANES], df[NPLANES];
    uint32_t a, b;
};

__device__ __forceinline__ NodeBox load_node(const GNode* nodes, uint32_t i)
{
    const float4* p = reinterpret_cast<const float4*>(nodes + i);
    float4 q0 = ldg(p), q1 = ldg(p + 1), q2 = ldg(p + 2), q3 = ldg(p + 3);
    NodeBox n;
    n.dn[0] = q0.x; n.dn[1] = q0.y; n.dn[2] = q0.z; n.dn[3] = q0.w;
    n.dn[4] = q1.x; n.dn[5] = q1.y; n.dn[6] = q1.z;
    n.df[0] = q1.w;
    n.df[1] = q2.x; n.df[2] = q2.y; n.df[3] = q2.z; n.df[4] = q2.w;
    n.df[5] = q3.x; n.df[6] = q3.y;
    n.a = __float_as_uint(q3.z);
    n.b = __float_as_uint(q3.w);
    return n;
}

__device__ __forceinline__ uint2 load_node_link(const GNode* nodes, uint32_t i)
{
    const uint4* p = reinterpret_cast<const uint4*>(nodes + i);
    uint4 q3 = ldg(p + 3);
    return make_uint2(q3.z, q3.w);
}

// BoundingVolume::intersect, bvh.h:79-105, branch-free.  Exactly the
// reference's decision and t_near:
//  * t_near only grows and t_far only shrinks (std::max / std::min never return
//    a NaN second operand), so one t_far < t_near test after the loop equals the
//    early exit inside it;
//  * every stored volume has d_near[i] <= d_far[i] (a min / max over its
//    triangles' projections, checked when the octree is flattened), so the
//    quotient pair ordered by the sign of denom (the std::swap) is (min, max);
//  * a skipped plane (denom == 0) has num = NaN, its quotients are NaN and
//    fmaxf / fminf keep the running bound, as std::max / std::min do.
// fmaxf / fminf differ from std::max / std::min only in the sign of a zero
// result, which no comparison sees.
// SEG (segment queries): a volume that passes but lies
// wholly outside [R.lo, R.hi] is treated as missed.
template <bool SEG = false>
__device__ __forceinline__ bool vol_test(const NodeBox& n, const TRay& R, float& t_near_out)
{
    float t_near = -INFINITY, t_far = INFINITY;
#pragma unroll
    for (int i = 0; i < NPLANES; i++) {
        float d0 = (n.dn[i] - R.num[i]) / R.den[i];
        float d1 = (n.df[i] - R.num[i]) / R.den[i];
        t_near = fmaxf(t_near, fminf(d0, d1));
        t_far = fminf(t_far, fmaxf(d0, d1));
    }
    t_near_out = t_near;
    if (SEG)
        return !(t_far < t_near) & !(t_far < R.lo) & !(t_near > R.hi);
    return !(t_far < t_near);
}

// Triangle::intersect (Moller-Trumbore, backface culling), triangle.cpp:25-91,
// split into the 48-byte record load and the test so loads can be batched.
struct TriRec {
    float4 q0, q1, q2;
};

__device__ __forceinline__ TriRec load_tri(const GTri* tris, uint32_t k)
{
    const float4* p = reinterpret_cast<const float4*>(tris + k);
    TriRec r;
    r.q0 = ldg(p);
    r.q1 = ldg(p + 1);
    r.q2 = ldg(p + 2);
    return r;
}

__device__ __forceinline__ bool tri_test_rec(const TriRec& T, const TRay& R, float& t_out, float& u_out,
                                             float& v_out)
{
    // the reference's early returns become one predicate over the same values
    // (same expressions, same comparisons, so NaNs behave identically)
    v3 a = mk(T.q0.x, T.q0.y, T.q0.z);
    v3 ab = mk(T.q0.w, T.q1.x, T.q1.y);
    v3 ac = mk(T.q1.z, T.q1.w, T.q2.x);
    v3 n = mk(T.q2.y, T.q2.z, T.q2.w);
    v3 OA = R.o - a;
    v3 nd = -R.d;
    v3 m = cross(nd, OA);
    float Mdet = dot(n, nd);
    // coherent waves often reject a back-facing triangle together: skip the rest
    if (Mdet <= 0)
        return false;
    float inv = 1 / Mdet;
    float u = dot(m, ac) * inv;
    if (u < 0 || u > 1)
        return false;
    float v = dot(m, -ab) * inv;
    if (v < 0 || u + v > 1)
        return false;
    float t = dot(n, OA) * inv;
    t_out = t;
    u_out = u;
    v_out = v;
    return !(Mdet <= 0) & !(u < 0 || u > 1) & !(v < 0 || u + v > 1) & !(t < 0);
}

__device__ __forceinline__ bool tri_test(const GTri* tris, uint32_t k, const TRay& R, float& t_out, float& u_out,
                                         float& v_out)
{
    return tri_test_rec(load_tri(tris, k), R, t_out, u_out, v_out);
}

struct THit {
    float t, u, v;
    int k;   // GTri slot, -1 none
};

// Leaf slabs.  P.lslab[a] for the leaf whose triangles start at
// slot a: the box of its vertices (lo, hi) and the range [smin, smax] of their projections
// on the leaf's cone axis (P.cones[a].xyz).  A curved-surface patch is thin along its mean
// normal, so a line that grazes the surface (a silhouette ray) passes above most patches
// near it: if the line's parameter intervals inside the box and inside the slab, both
// widened by a margin, do not overlap (within the query segment), no triangle of the leaf
// can be hit.  The margin holds every point Moller-Trumbore can report: it lies within
// 2^-17 (|o|_inf + S) / Q of its triangle, Q = sin(angle at a) |cos(n, d)|,
// bounded below by P.lsin[a] and the leaf's cone; a leaf without a Q bound >= 2^-16 (no
// cone, or a ray within a few degrees of grazing it) is never skipped.
__device__ __forceinline__ bool leaf_missed(const KParams& P, uint32_t a, const TRay& R)
{
    if (!P.lslab)
        return false;
    const float4 c = ldg(reinterpret_cast<const float4*>(P.cones) + a);
    const float om = fmaxf(fabsf(R.o.x), fmaxf(fabsf(R.o.y), fabsf(R.o.z)));
    const float dd = R.d.x * R.d.x + R.d.y * R.d.y + R.d.z * R.d.z;
    if (!(c.w > 0.0f && om <= 0x1p30f && dd >= 0x1p-60f && dd <= 0x1p60f))
        return false;
    // cos(n, -d) >= cos(phi + theta): phi = angle(axis, -d), theta the cone's half-angle
    const float cb = -(c.x * R.d.x + c.y * R.d.y + c.z * R.d.z) / sqrtf(dd);
    const float lb = c.w * cb - sqrtf(fmaxf(0.0f, 1.0f - c.w * c.w)) * sqrtf(fmaxf(0.0f, 1.0f - cb * cb)) - 0x1p-18f;
    const float Q = ldg(P.lsin + a) * lb;
    if (!(Q >= 0x1p-16f))
        return false;
    const float4* L = reinterpret_cast<const float4*>(P.lslab) + 2 * (size_t)a;
    const float4 lo = ldg(L), hi = ldg(L + 1);
    const float Sc = om + P.scene_scale;
    const float m = 0x1p-16f * Sc + 0x1p-17f * Sc / Q * (1.0f + 0x1p-20f);
    const float ix = 1.0f / R.d.x, iy = 1.0f / R.d.y, iz = 1.0f / R.d.z;
    float tx0 = (lo.x - m - R.o.x) * ix, tx1 = (hi.x + m - R.o.x) * ix;
    float ty0 = (lo.y - m - R.o.y) * iy, ty1 = (hi.y + m - R.o.y) * iy;
    float tz0 = (lo.z - m - R.o.z) * iz, tz1 = (hi.z + m - R.o.z) * iz;
    const float da = c.x * R.d.x + c.y * R.d.y + c.z * R.d.z;
    const float oa = c.x * R.o.x + c.y * R.o.y + c.z * R.o.z;
    float s0 = (lo.w - m - oa) / da, s1 = (hi.w + m - oa) / da;
    // NaN quotients (a zero component on a boundary) constrain nothing
    float tmin = fmaxf(fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), fminf(s0, s1))), R.lo);
    float tmax = fminf(fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), fmaxf(s0, s1))), R.hi);
    return tmax < tmin;
}

// Leaf normal cones.  P.cones[a] for the leaf whose triangles
// start at slot a: a unit axis and the cosine c of a cone holding every normalised
// triangle normal of the leaf (c = -2: no cone).  If the ray direction's angle to the
// axis plus the cone's half-angle stays below 90 degrees by a margin, every triangle
// of the leaf has n.d > 1e-4 |n| |d|, so the computed Mdet = dot(n, -d) of
// Triangle::intersect (triangle.cpp:39-40) is negative for each of them and the whole
// leaf is rejected exactly as the reference's loop rejects it, one triangle at a time.
__device__ __forceinline__ bool leaf_backfacing(const KParams& P, uint32_t a, const TRay& R)
{
    if (!P.cones)
        return false;
    const float4 c = ldg(reinterpret_cast<const float4*>(P.cones) + a);
    const float dd = R.d.x * R.d.x + R.d.y * R.d.y + R.d.z * R.d.z;
    // |d| in [1e-10, 1e10]: the products of dot(n, -d) neither underflow nor overflow
    if (!(c.w > 0.0f && dd > 1.0e-20f && dd < 1.0e20f))
        return false;
    const float ad = (c.x * R.d.x + c.y * R.d.y + c.z * R.d.z) / sqrtf(dd);   // cos(phi)
    // n.d / |d| >= cos(theta + phi) = cos(theta) cos(phi) - sin(theta) sin(phi) for theta, phi < 90 deg
    const float lb = c.w * ad - sqrtf(fmaxf(0.0f, 1.0f - c.w * c.w)) * sqrtf(fmaxf(0.0f, 1.0f - ad * ad));
    return ad > 0.0f && lb > 1.0e-4f;
}

// ---- libstdc++ binary heap (push_heap / pop_heap with std::greater), only
// used when two pending children have equal t_near. ----
// Children are pushed in octant order, which is their slot order a + j.
__device__ __noinline__ uint32_t heap_order(float k0, float k1, float k2, float k3, float k4, float k5, float k6,
                                            float k7, uint32_t validmask, int n)
{
    // keys arrive in registers; the arrays below exist only on this (rare) path
    float key[8] = {k0, k1, k2, k3, k4, k5, k6, k7};
    bool valid[8];
    uint32_t rank[8];
    for (int s = 0; s < 8; s++) {
        valid[s] = (validmask >> s) & 1u;
        rank[s] = (uint32_t)s;
    }
    float hk[8];
    uint32_t hr[8];
    int len = 0;
    for (int s = 0; s < 8; s++) {
        if (!valid[s])
            continue;
        // push_back + __push_heap(first, len, 0, value)
        float vk = key[s];
        uint32_t vr = rank[s];
        int hole = len, parent = (hole - 1) / 2;
        while (hole > 0 && hk[parent] > vk) {
            hk[hole] = hk[parent];
            hr[hole] = hr[parent];
            hole = parent;
            parent = (hole - 1) / 2;
        }
        hk[hole] = vk;
        hr[hole] = vr;
        len++;
    }
    uint32_t order = 0;
    for (int i = 0; i < n; i++) {
        order |= hr[0] << (3 * i);
        // pop_heap: value = last; last = first; __adjust_heap(first, 0, len - 1, value)
        if (len > 1) {
            int l = len - 1;
            float vk = hk[l];
            uint32_t vr = hr[l];
            int hole = 0, second = 0;
            while (second < (l - 1) / 2) {
                second = 2 * (second + 1);
                if (hk[second] > hk[second - 1])
                    second--;
                hk[hole] = hk[second];
                hr[hole] = hr[second];
                hole = second;
            }
            if ((l & 1) == 0 && second == (l - 2) / 2) {
                second = 2 * (second + 1);
                hk[hole] = hk[second - 1];
                hr[hole] = hr[second - 1];
                hole = second - 1;
            }
            int parent = (hole - 1) / 2;
            while (hole > 0 && hk[parent] > vk) {
                hk[hole] = hk[parent];
                hr[hole] = hr[parent];
                hole = parent;
                parent = (hole - 1) / 2;
            }
            hk[hole] = vk;
            hr[hole] = vr;
        }
        len--;
    }
    return order;
}

// BVH::intersect (bvh.cpp:68-71) -> OctreeNode::intersect, iteratively, as a
// resumable traversal: trav_begin runs the root prologue, each trav_step VISITs
// one node (a leaf's triangles, or an inner node's children) and performs the
// RETURN unwinding that follows it.  T.live turns false once the root returned;
// T.r is then the reference's boolean and h the query-global HitInfo
// (t, u, v, GTri slot).  lv: this lane's LDS level stack, entry d at lv[d * BLOCK].
struct Trav {
    uint32_t a, b;       // link word of the node to VISIT next
    int depth;
    uint32_t any_true;   // bit d: closest_inter != INFINITY in the node whose children are at depth d
    bool r, live;
#if RT_COUNT
    uint32_t nvol, ntri;
#endif
};

template <bool SEG = false>
__device__ __forceinline__ void trav_begin(const KParams& P, const TRay& R, THit& h, Trav& T)
{
    h.t = -1.0f;
    h.u = 1.0f;
    h.v = 0.0f;
    h.k = -1;
    T.r = false;
    T.live = false;
#if RT_COUNT
    T.nvol = 1;
    T.ntri = 0;
#endif
    if (P.nnodes == 0)
        return;
    if (R.nan) {
        // every volume passes with t_near = -inf, every triangle "hits" with
        // t = NaN and no leaf ever returns true: the query returns false with
        // a NaN record (NaN rays).
        h.t = __int_as_float(0x7fc00000);
        return;
    }
    float tn;
    NodeBox nb = load_node(P.nodes, 0);
    if (!vol_test<SEG>(nb, R, tn))
        return;
    T.a = nb.a;
    T.b = nb.b;
    T.depth = 0;
    T.any_true = 0;
    T.live = true;
}

template <bool SEG = false>
__device__ __forceinline__ void trav_step(const KParams& P, const TRay& R, THit& h, Trav& T, uint2* lv)
{
    uint32_t a = T.a, b = T.b;
    int depth = T.depth;
    uint32_t any_true = T.any_true;
    bool r = false;
    // ---- VISIT the node whose link word is (a, b) at 'depth' ----
    if (b & LEAF_BIT) {
        uint32_t end = a + (b & ~LEAF_BIT);
        if (leaf_backfacing(P, a, R) || leaf_missed(P, a, R))
            end = a;   // every triangle back-facing, or the line misses them all: no Triangle::intersect succeeds
#if RT_COUNT
        T.ntri += end - a;
#endif
        // triangles in leaf order, h updated as in bvh.h:237-243
        // the next triangle's record is loaded while this one is tested
        TriRec cur;
        if (a < end)
            cur = load_tri(P.tris, a);
        for (uint32_t k = a; k < end; k++) {
            TriRec nxt = load_tri(P.tris, k + 1 < end ? k + 1 : k);
            float t, u, v;
            if (tri_test_rec(cur, R, t, u, v))
                if (t < h.t || h.t == -1) {
                    h.t = t;
                    h.u = u;
                    h.v = v;
                    h.k = (int)k;
                }
            cur = nxt;
        }
        r = h.t > 0;
    } else {
        // the k non-empty children are nodes a .. a+k-1, in octant order; a
        // child that is missed keeps a NaN key (no comparison counts it)
        const uint32_t k = b;
#if RT_COUNT
        T.nvol += k;
#endif
        float key[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            key[j] = __int_as_float(0x7fc00000);
            if ((uint32_t)j < k) {
                NodeBox c = load_node(P.nodes, a + j);
                float t;
                if (vol_test<SEG>(c, R, t))
                    key[j] = t;
            }
        }
        // pop position of child j = number of hit children before it in a
        // stable sort by t_near; equal keys need the heap's own order
        uint32_t pos[8];
        uint32_t vm = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            pos[j] = 0;
            vm |= (key[j] == key[j] ? 1u : 0u) << j;
        }
        bool tie = false;
#pragma unroll
        for (int j = 0; j < 8; j++)
#pragma unroll
            for (int j2 = j + 1; j2 < 8; j2++) {
                pos[j] += key[j2] < key[j] ? 1u : 0u;
                pos[j2] += key[j] <= key[j2] ? 1u : 0u;
                tie |= key[j] == key[j2];
            }
        const int n = __popc(vm);
        if (n > 0) {
            uint32_t order = 0;
#pragma unroll
            for (int j = 0; j < 8; j++)
                order |= ((vm >> j) & 1u) ? (uint32_t)j << (3 * pos[j]) : 0u;
            if (tie)
                order = heap_order(key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7], vm, n);
            depth++;
            any_true &= ~(1u << depth);
            uint32_t first = a + (order & 7u);
            lv[depth * BLOCK] = make_uint2(a, (order >> 3) | ((uint32_t)(n - 1) << 24));
            uint2 link = load_node_link(P.nodes, first);
            T.a = link.x;
            T.b = link.y;
            T.depth = depth;
            T.any_true = any_true;
            return;
        }
        r = false;
    }
    // ---- RETURN r from the node at 'depth' to its parent ----
    for (;;) {
        if (depth == 0) {
            T.r = r;
            T.live = false;
            return;
        }
        uint2 e = lv[depth * BLOCK];
        uint32_t cnt = e.y >> 24;
        uint32_t ord = e.y & 0xffffffu;
        if (r) {
            // closest_inter = min(closest_inter, child t_near); the child's t_near is
            // the query-global hit t, and a child returning true with t = +inf
            // (overflow) leaves closest_inter == INFINITY (bvh.h:267, 280-281)
            if (h.t < INFINITY)
                any_true |= 1u << depth;
            if (cnt == 0) {
                depth--;
                continue;   // queue empty: parent returns true
            }
            NodeBox nx = load_node(P.nodes, e.x + (ord & 7u));
            float t_next;
            vol_test(nx, R, t_next);
#if RT_COUNT
            T.nvol++;
#endif
            if (h.t < t_next) {
                depth--;    // closest hit nearer than the next child: parent returns true
                continue;
            }
            lv[depth * BLOCK] = make_uint2(e.x, (ord >> 3) | ((cnt - 1) << 24));
            a = nx.a;
            b = nx.b;
            break;
        } else {
            if (cnt == 0) {
                r = (any_true >> depth) & 1u;   // closest_inter != INFINITY
                depth--;
                continue;
            }
            uint2 link = load_node_link(P.nodes, e.x + (ord & 7u));
            lv[depth * BLOCK] = make_uint2(e.x, (ord >> 3) | ((cnt - 1) << 24));
            a = link.x;
            b = link.y;
            break;
        }
    }
    T.a = a;
    T.b = b;
    T.depth = depth;
    T.any_true = any_true;
}

template <bool SEG = false>
__device__ bool bvh_closest(const KParams& P, const TRay& R, THit& h, uint2* lv)
{
    Trav T;
    trav_begin<SEG>(P, R, h, T);
    // while-while: lanes at inner nodes keep expanding until every lane of the
    // wave sits on a leaf (or is done), then the leaves are tested together
    while (T.live) {
        while (T.live && !(T.b & LEAF_BIT))
            trav_step<SEG>(P, R, h, T, lv);
        if (T.live)
            trav_step<SEG>(P, R, h, T, lv);
    }
#if RT_COUNT
    if (P.counters) {
        atomicAdd(&P.counters[SEG ? 6 : 4], (unsigned long long)T.nvol);
        atomicAdd(&P.counters[SEG ? 7 : 5], (unsigned long long)T.ntri);
    }
#endif
    return T.r;
}

// Segment queries.  A shadow query's answer depends only on
// hits in front of its origin and not beyond the light; a reflection sample's closest
// hit only on hits in front of its origin.  Under the assumption the reference's own
// early-out makes (bvh.h:270: a triangle's hit t lies inside its volumes' [t_near,
// t_far]), a volume wholly outside the query segment holds no hit that changes the
// query-global record or the root's return value, so it need not be entered.  The
// segment is widened on both sides by seg_margin, a bound on the rounding of a k-DOP
// quotient and of a Moller-Trumbore t in a scene of scale P.seg_scale.  Queries that
// end with the record at t == 0, +inf or NaN (where the reference's return value
// depends on the leaves visited) are re-run over the whole line.
__device__ __forceinline__ float seg_margin(const KParams& P, const TRay& R)
{
    float dmin = INFINITY;
#pragma unroll
    for (int i = 0; i < NPLANES; i++)
        if (R.den[i] != 0.0f)
            dmin = fminf(dmin, fabsf(R.den[i]));
    float om = fmaxf(fabsf(R.o.x), fmaxf(fabsf(R.o.y), fabsf(R.o.z)));
    return 0x1p-8f * P.seg_scale + 0x1p-14f * (P.seg_scale + om) / dmin;
}

__device__ __forceinline__ bool bvh_closest_seg(const KParams& P, TRay& R, THit& h, uint2* lv)
{
    bool r = bvh_closest<true>(P, R, h, lv);
    if (h.k >= 0 && !(h.t > 0.0f && h.t < INFINITY)) {
        R.lo = -INFINITY;
        R.hi = INFINITY;
        r = bvh_closest<true>(P, R, h, lv);
    }
    return r;
}

// HitInfo filled by Triangle::intersect for slot k (triangle.cpp:81-88)
// The record of a hit on triangle record T (caller index id, material mat).
__device__ __forceinline__ Rec rec_of(const KParams& P, const GTri& T, int id, int mat, const THit& h)
{
    Rec r;
    v3 ab = mk(T.ab[0], T.ab[1], T.ab[2]);
    v3 ac = mk(T.ac[0], T.ac[1], T.ac[2]);
    v3 n = mk(T.n[0], T.n[1], T.n[2]);
    r.tri = id;
    r.t = h.t;
    r.u = h.u;
    r.v = h.v;
    r.mat = mat;
    r.normal = normalize(n);
    // Triangle::get_tangent, triangle.cpp:134-153
    float u1 = -1, v1 = -1, u2 = -1, v2 = -1, u3 = -1, v3_ = -1;
    if (P.tri_uv) {
        const float* uv = P.tri_uv + 6 * (size_t)id;
        u1 = uv[0]; u2 = uv[1]; u3 = uv[2];
        v1 = uv[3]; v2 = uv[4]; v3_ = uv[5];
    }
    float dU1 = u2 - u1, dV1 = v2 - v1, dU2 = u3 - u1, dV2 = v3_ - v1;
    float f = 1.0f / (dU1 * dV2 - dU2 * dV1);
    r.tangent.x = f * (dV2 * ab.x - dV1 * ac.x);
    r.tangent.y = f * (dV2 * ab.y - dV1 * ac.y);
    r.tangent.z = f * (dV2 * ab.z - dV1 * ac.z);
    return r;
}

__device__ __forceinline__ Rec tri_record(const KParams& P, const THit& h)
{
    const int id = P.tri_id[h.k];
    return rec_of(P, load_gtri(P.tris + h.k), id, P.tri_mat[id], h);
}

// Sphere::intersect, analyticShape.cpp:9-60 (compute_uv forced true; reads a stale hit.t when delta>0 and t1>=t2)
__device__ __forceinline__ bool sphere_test(const float* s, int mat, v3 o, v3 d, Rec& h)
{
    v3 c = mk(s[0], s[1], s[2]);
    float r2 = s[3] * s[3];
    v3 L = o - c;
    const float a = 1;
    float b = 2 * dot(d, L);
    float cc = dot(L, L) - r2;
    float delta = b * b - 4 * a * cc;
    if (delta < 0)
        return false;
    const float a2 = 2 * a;
    if (delta == 0.0f)
        h.t = -b / a2;
    else {
        float sq = sqrtf(delta);
        float t1 = (-b - sq) / a2;
        float t2 = (-b + sq) / a2;
        if (t1 < t2) {
            h.t = t1;
            if (h.t < 0)
                h.t = t2;
        }
    }
    if (h.t < 0)
        return false;
    h.normal = normalize((o + d * h.t) - c);
    h.u = 0.5f + atan2f(-h.normal.z, -h.normal.x) / (2.0f * (float)M_PI);
    h.v = 0.5f + asinf(-h.normal.y) / (float)M_PI;
    h.tangent = cross(mk(0, 1, 0), h.normal);
    h.mat = mat;
    return true;
}

// Plane::intersect, analyticShape.cpp:64-76
__device__ __forceinline__ bool plane_test(const float* p, int mat, v3 o, v3 d, Rec& h)
{
    v3 n = mk(p[3], p[4], p[5]);
    float t = dot(mk(p[0], p[1], p[2]) - o, n) / dot(d, n);
    if (t < 0)
        return false;
    h.t = t;
    h.mat = mat;
    h.normal = n;
    return true;
}

// Image::offset clamp + texel (image.h:122-134)
__device__ __forceinline__ float4 texel(const KTex& T, int x, int y)
{
    int px = x;
    if (px < 0) px = 0;
    if (px > T.w - 1) px = T.w - 1;
    int py = y;
    if (py < 0) py = 0;
    if (py > T.h - 1) py = T.h - 1;
    return T.px[(unsigned)(py * T.w + px)];
}

// Image::texture_floor -> sample_floor, image.h:79-86, 94-97 (alpha optional)
__device__ __forceinline__ c3 tex_floor(const KTex& T, float x, float y, float* alpha = nullptr)
{
    float u = floorf(x * T.w);
    float v = floorf(y * T.h);
    float4 p = texel(T, f2i(u), f2i(v));
    if (alpha) *alpha = p.w;
    return col(p.x, p.y, p.z);
}

// Image::texture_bilinear -> sample_bilinear, image.h:66-77, 89-92
__device__ __forceinline__ c3 tex_bilinear(const KTex& T, float xx, float yy, float* alpha)
{
    float x = xx * T.w, y = yy * T.h;
    float u = x - floorf(x);
    float v = y - floorf(y);
    int ix = f2i(x), iy = f2i(y);
    float4 p00 = texel(T, ix, iy), p10 = texel(T, ix + 1, iy), p01 = texel(T, ix, iy + 1), p11 = texel(T, ix + 1, iy + 1);
    float w00 = (1 - u) * (1 - v), w10 = u * (1 - v), w01 = (1 - u) * v, w11 = u * v;
    *alpha = p00.w * w00 + p10.w * w10 + p01.w * w01 + p11.w * w11;
    return col(p00.x * w00 + p10.x * w10 + p01.x * w01 + p11.x * w11,
               p00.y * w00 + p10.y * w10 + p01.y * w01 + p11.y * w11,
               p00.z * w00 + p10.z * w10 + p01.z * w01 + p11.z * w11);
}

// Skybox::sample, skybox.cpp:12-51
__device__ c3 skybox_sample(const KParams& P, v3 dir, float* alpha)
{
    v3 d2 = mk(dir.x, dir.y, -dir.z);
    v3 da = mk(fabsf(d2.x), fabsf(d2.y), fabsf(d2.z));
    int face;
    float nf, u, v;
    if (da.z >= da.x && da.z >= da.y) {
        face = d2.z < 0.0f ? 4 : 5;
        nf = (float)(0.5 / (double)da.z);
        u = d2.z < 0.0f ? -d2.x : d2.x;
        v = -d2.y;
    } else if (da.y >= da.x) {
        face = d2.y < 0.0f ? 3 : 2;
        nf = (float)(0.5 / (double)da.y);
        u = d2.x;
        v = d2.y < 0.0f ? -d2.z : d2.z;
    } else {
        face = d2.x < 0.0f ? 1 : 0;
        nf = (float)(0.5 / (double)da.x);
        u = d2.x < 0.0f ? d2.z : -d2.z;
        v = -d2.y;
    }
    u = (float)((double)(u * nf) + 0.5);
    v = (float)((double)(v * nf) + 0.5);
    return tex_bilinear(P.sky[face], u, v, alpha);
}

__device__ __forceinline__ const float* mat_of(const KParams& P, int id) { return P.mats + (size_t)MAT_STRIDE * id; }
__device__ __forceinline__ c3 mat_col(const float* m, int off) { return col(m[off], m[off + 1], m[off + 2]); }

// Triangle::interpolate_texcoords (triangle.cpp:155-160) / get_tex_coords (renderer.cpp:436-445)
__device__ __forceinline__ void get_tex_coords(const KParams& P, int tri, float u, float v, float& tu, float& tv)
{
    if (tri >= 0) {
        float u0 = -1, u1 = -1, u2 = -1, v0 = -1, v1 = -1, v2 = -1;
        if (P.tri_uv) {
            const float* uv = P.tri_uv + 6 * (size_t)tri;
            u0 = uv[0]; u1 = uv[1]; u2 = uv[2];
            v0 = uv[3]; v1 = uv[4]; v2 = uv[5];
        }
        tu = (1 - u - v) * u0 + u * u1 + v * u2;
        tv = (1 - u - v) * v0 + u * v1 + v * v2;
    } else {
        tu = u;
        tv = v;
    }
}

// renderer.cpp:464-478
__device__ v3 normal_mapping(const KParams& P, const Rec& h, float u, float v)
{
    float tu, tv;
    get_tex_coords(P, h.tri, u, v, tu, tv);
    v3 T = h.tangent;
    v3 B = cross(T, h.normal);
    v3 N = h.normal;
    c3 nc = tex_floor(P.tex[TEX_NORMAL], tu, tv);
    v3 nm = mk(nc.r, nc.g, nc.b) * 2.0f - mk(1, 1, 1);
    v3 q = normalize(nm);
    v3 p = mk(T.x * q.x + B.x * q.y + N.x * q.z, T.y * q.x + B.y * q.y + N.y * q.z, T.z * q.x + B.z * q.y + N.z * q.z);
    return normalize(p);
}

// renderer.cpp:518-554
__device__ void parallax_occlusion_mapping(const KParams& P, int tri, float u, float v, v3 view, float& nu, float& nv)
{
    float tu, tv;
    get_tex_coords(P, tri, u, v, tu, tv);
    const KTex& D = P.tex[TEX_DISPLACEMENT];
    int steps = P.parallax_mapping_steps;
    float current_depth;
    float depth_step = 1.0f / steps;
    float sampled = tex_floor(D, tu, tv).r;
    v3 search = -view * P.displacement_mapping_strength;
    float du = search.x / steps;
    float dv = search.y / steps;
    current_depth = 0.0f;
    float u2 = tu, v2 = tv;
    while (current_depth < sampled) {
        u2 += du;
        v2 += dv;
        sampled = tex_floor(D, u2, v2).r;
        current_depth += depth_step;
    }
    float pu = u2 - du, pv = v2 - dv;
    float after = sampled - current_depth;
    float before = tex_floor(D, pu, pv).r - (current_depth - depth_step);
    float w = after / (after - before);
    nu = (1 - w) * u2 + w * pu;
    nv = (1 - w) * v2 + w * pv;
}

#if RT_PHASE_TIME
// per wave: [0..6] cycles per phase, [7] the last mark (LDS; the wave's first active lane updates)
__shared__ unsigned long long g_phase[WAVES_PER_BLOCK][8];
__device__ __forceinline__ void ph_mark(int k)
{
    const unsigned long long now = __builtin_amdgcn_s_memtime();
    const uint64_t act = __ballot(1);
    if ((int)__lane_id() == __ffsll((unsigned long long)act) - 1) {
        const int w = threadIdx.x >> 6;
        g_phase[w][k] += now - g_phase[w][7];
        g_phase[w][7] = now;
    }
}
#define PH_MARK(k) ph_mark(k)
#else
#define PH_MARK(k)
#endif

// The lane's wide-BVH traversal stack: entry i at lv[i * BLOCK] (the LDS of the octree
// level stack, which is not live during the wide-BVH query).
// A lane's LDS entries (uint2, entry i at lane + i * BLOCK): the octree walk's level stack (P.levels) or
// the wide query's stack (W_STACK), then LDS_SAVE_ENTRIES more from lds_save_slot (trace_pixel)
constexpr int LDS_SAVE_ENTRIES = 3;
__host__ __device__ __forceinline__ int lds_save_slot(const KParams& P) { return P.levels > W_STACK ? P.levels : W_STACK; }
// The plain kernel (3 blocks of 4 waves per CU by its 168 VGPRs) may take up to 160 KB / 3 / 256 lanes = 26
// LDS entries per lane: its one-lane queries get a deeper stack than W_STACK, so that fewer of them overflow
// into the 64-entry scratch stack of wide_closest_deep (hair1m: 0.5% of its queries at 16 entries, the
// longest ones); its lane groups keep the W_STACK ring.  The octree-only plain kernel has no wide stack.
#ifndef RT_W_STACK_PLAIN
#define RT_W_STACK_PLAIN 22
#endif
constexpr int W_STACK_PLAIN = RT_W_STACK_PLAIN;
static_assert(W_STACK_PLAIN >= W_STACK && W_STACK_PLAIN + LDS_SAVE_ENTRIES <= 26, "the plain kernel's LDS entries");
template <bool OCT>
__host__ __device__ __forceinline__ int lds_save_slot_plain(const KParams& P)
{
    const int w = OCT ? 0 : W_STACK_PLAIN;
    return P.levels > w ? P.levels : w;
}

template <int N = W_STACK>
struct WStackLdsN {
    static constexpr int CAP = N;
    uint2* base;
    __device__ __forceinline__ void put(int i, uint2 v) { base[i * BLOCK] = v; }
    __device__ __forceinline__ uint2 get(int i) const { return base[i * BLOCK]; }
    // entry i of the lane 'delta' lanes away (a lane group's steal, wbvh_closest<.., G>)
    __device__ __forceinline__ uint2 get_lane(int delta, int i) const { return base[delta + i * BLOCK]; }
};
using WStackLds = WStackLdsN<W_STACK>;

#if RT_COUNT
// counters[base]: the wave's longest lane's loop iterations, [base + 1]: every lane's, [base + 2]:
// wave calls (SIMD efficiency of the if-if loop; diagnostic builds only)
__device__ void count_wave_steps(const KParams& P, int base, uint32_t steps)
{
    if (!P.counters)
        return;
    uint64_t act = __ballot(1), a = act;
    uint32_t mx = 0;
    while (a) {
        const int l = __ffsll((unsigned long long)a) - 1;
        a &= a - 1;
        mx = max(mx, (uint32_t)__builtin_amdgcn_readlane((int)steps, l));
    }
    if ((int)__lane_id() == __ffsll((unsigned long long)act) - 1) {
        atomicAdd(&P.counters[base], (unsigned long long)mx);
        atomicAdd(&P.counters[base + 2], 1ull);
    }
    atomicAdd(&P.counters[base + 1], (unsigned long long)steps);
}
#endif


// A query whose LDS stack overflowed (wbvh_closest returned W_DEEP, ~0.03% of C4's primary rays:
// grazing rays with many case-(b) children) runs again with a 64-entry stack in private memory, out
// of line so that its frame stays out of the traversal loop's registers; the exact octree walk is
// left for what that cannot certify.
// The record comes back by value (WDeep, in registers): a WHit passed by reference would live in
// scratch in every caller, and each query's record went through it (r05: the plain kernel's HBM writes).
struct WDeep {
    int st;
    WHit w;
};
__device__ __noinline__ WDeep wide_closest_deep(const WNode* wnodes, const GTri* wtris, v3 o, v3 d, float m, float hi,
                                                bool ties, float QS, const uint64_t* rk, int rsel, float rsub)
{
    WStackArr<W_DEEP_STACK> stk;
    WDeep r;
    const int st = wbvh_closest(wnodes, wtris, o, d, m, stk, r.w, nullptr, hi, ties, QS, rk, rsel, rsub);
    r.st = st == W_DEEP ? W_UNCERT : st;
    return r;
}

// BVH::intersect through the wide BVH and its certificate (wbvh.hpp).
// Returns true with (h, r) = the reference's record and boolean when the query is
// certified; false when it must be traced through the octree.
// rec (optional): on a certified hit, the record built from the wide BVH's own copies (the
// triangle from wtris, index and material from wmeta), with no further dependent loads.
template <int G = 1, int CAP = W_STACK>
__device__ __forceinline__ bool wide_closest(const KParams& P, v3 o, v3 d, THit& h, bool& r, uint2* lv,
                                             Rec* rec = nullptr, uint32_t max_steps = 0, bool* longq = nullptr)
{
    using Stk = WStackLdsN<G == 1 ? CAP : W_STACK>;   // (a lane group's ring: W_STACK entries)
    const float om = fmaxf(fabsf(o.x), fmaxf(fabsf(o.y), fabsf(o.z)));
    Stk stk{lv};
    WHit w;
    // a ray from the camera position reads the frame's camera risk keys
    const uint64_t* rk = P.wrisk && o.x == P.cam_pos[0] && o.y == P.cam_pos[1] && o.z == P.cam_pos[2] ? P.wrisk : nullptr;
    // the camera's risk cap: a ray into the silhouette's interior meets no at-risk triangle in case (b)
    const bool nob = rk && P.risk_cap && risk_cap_skip(P.risk_cap[0], P.cap_dir[0], d, W_QS_CLOSEST);
#if RT_COUNT
    uint32_t wk[4] = {0, 0, 0, 0};
    int st = wbvh_closest<Stk, G>(P.wnodes, P.wtris, o, d, 0x1p-16f * (om + P.scene_scale), stk, w, wk, INFINITY, true,
                          W_QS_CLOSEST, rk, 0, 0.0f, 0u, (WNoFeed*)nullptr, nob);
    count_wave_steps(P, 22, wk[3]);
    if (P.counters) {
        atomicAdd(&P.counters[10], (unsigned long long)wk[0]);
        atomicAdd(&P.counters[11], (unsigned long long)wk[1]);
        for (int c = 0; c < 5; c++)
            if ((wk[2] >> c) & 1u)
                atomicAdd(&P.counters[16 + c], 1ull);   // uncertified, by reason (wbvh_closest)
    }
#else
    int st = wbvh_closest<Stk, G>(P.wnodes, P.wtris, o, d, 0x1p-16f * (om + P.scene_scale), stk, w, nullptr, INFINITY,
                          true, W_QS_CLOSEST, rk, 0, 0.0f, max_steps, (WNoFeed*)nullptr, nob);
#endif
    if (st == W_LONG) {
        *longq = true;
        return false;
    }
    if (st == W_DEEP) {
        const WDeep r = wide_closest_deep(P.wnodes, P.wtris, o, d, 0x1p-16f * (om + P.scene_scale), INFINITY, true,
                                          W_QS_CLOSEST, rk, 0, 0.0f);
        st = r.st;
        w = r.w;
    }
    if (st == W_MISS) {
        h.t = -1.0f;
        h.u = 1.0f;
        h.v = 0.0f;
        h.k = -1;
        r = false;
        return true;
    }
#if RT_COUNT
    if (st == W_HIT && P.counters)
        atomicAdd(&P.counters[14], 1ull);   // the certificate's k-DOP test
#endif
    if (st == W_HIT) {
        // one 16-B load names the slot, the certificate's leaf, the index and the material
        const uint4 M = ldg(P.wmeta + w.k);
        const GNode leaf = load_gnode(P.nodes + M.y);
        if (kdop_certifies(leaf, o, d, w.t)) {
            h.t = w.t;
            h.u = w.u;
            h.v = w.v;
            h.k = (int32_t)M.x;
            r = true;
            if (rec)
                *rec = rec_of(P, load_gtri(P.wtris + w.k), (int)M.z, (int)M.w, h);
            return true;
        }
    }
#if RT_COUNT
    if (P.counters) {
        atomicAdd(&P.counters[12], 1ull);
        if (st == W_HIT)
            atomicAdd(&P.counters[21], 1ull);   // the certificate's k-DOP test failed
    }
#endif
    return false;
}

// is_shadowed's BVH part through the wide BVH: the decision depends only
// on the reference's record t.  No hit at t <= hi: every hit lies beyond the segment
// end, which fails the distance test, so the point is lit whatever the record is.  A
// minimum hit t* <= hi whose octree leaf certifies it is the reference's record t.
// Returns true when decided (shadowed in *sh); false: take the octree segment query.
// light: the ray is one of the frame's shadow rays towards P.light that may read its risk keys
// (KParams::wrisk; hi >= |light - o|)
template <int G = 1, int CAP = W_STACK>
__device__ __forceinline__ bool wide_shadow(const KParams& P, v3 o, v3 d, float hi, v3 p, v3 lp, uint2* lv, bool* sh,
                                            bool light)
{
    using Stk = WStackLdsN<G == 1 ? CAP : W_STACK>;
    const float om = fmaxf(fabsf(o.x), fmaxf(fabsf(o.y), fabsf(o.z)));
    Stk stk{lv};
    WHit w;
    const uint64_t* rk = light ? P.wrisk : nullptr;
    const float rsub = light ? wrisk_sub(W_QS_SHADOW, hi, P.risk_nu) : 0.0f;
    // the origin cones (a lit point's shadow ray leaves its surface: the triangles whose planes pass near
    // the origin face away from it; ocone.hpp, built for W_QS_CLOSEST >= W_QS_SHADOW, so for a superset)
    static_assert(W_QS_SHADOW <= W_QS_CLOSEST, "the origin cones hold the at-risk triangles for the larger split");
    const bool nob = ocone_skip(P.ocone, o, d, W_QS_SHADOW) || (light && P.risk_cap && risk_cap_skip(P.risk_cap[1], P.cap_dir[1], d, W_QS_SHADOW));
#if RT_COUNT
    uint32_t wk[4] = {0, 0, 0, 0};
    int st = wbvh_closest<Stk, G>(P.wnodes, P.wtris, o, d, 0x1p-16f * (om + P.scene_scale), stk, w, wk, hi, false,
                          W_QS_SHADOW, rk, 1, rsub, 0u, (WNoFeed*)nullptr, nob);
    count_wave_steps(P, 25, wk[3]);
    if (P.counters) {
        atomicAdd(&P.counters[10], (unsigned long long)wk[0]);
        atomicAdd(&P.counters[11], (unsigned long long)wk[1]);
        for (int c = 0; c < 5; c++)
            if ((wk[2] >> c) & 1u)
                atomicAdd(&P.counters[16 + c], 1ull);   // uncertified, by reason (wbvh_closest)
    }
#else
    int st = wbvh_closest<Stk, G>(P.wnodes, P.wtris, o, d, 0x1p-16f * (om + P.scene_scale), stk, w, nullptr, hi, false,
                          W_QS_SHADOW, rk, 1, rsub, 0u, (WNoFeed*)nullptr, nob);
#endif
    if (st == W_DEEP) {
        const WDeep r = wide_closest_deep(P.wnodes, P.wtris, o, d, 0x1p-16f * (om + P.scene_scale), hi, false, W_QS_SHADOW,
                                          rk, 1, rsub);
        st = r.st;
        w = r.w;
    }
    if (st == W_MISS) {
        *sh = false;
        return true;
    }
#if RT_COUNT
    if (st == W_HIT && P.counters)
        atomicAdd(&P.counters[14], 1ull);
#endif
    if (st == W_HIT && kdop_certifies(load_gnode(P.nodes + ldg(P.wmeta + w.k).y), o, d, w.t)) {
        v3 q = o + d * w.t;
        *sh = length2(p - q) < length2(p - lp);
        return true;
    }
#if RT_COUNT
    if (P.counters) {
        atomicAdd(&P.counters[12], 1ull);
        if (st == W_HIT)
            atomicAdd(&P.counters[21], 1ull);   // the certificate's k-DOP test failed
    }
#endif
    return false;
}

// The analytic-shape part of is_shadowed (renderer.cpp:385-399); the shapes
// read the HitInfo the BVH query left behind (t_stale).
__device__ __forceinline__ bool shapes_shadow(const KParams& P, v3 o, v3 d, float t_stale, v3 p, v3 lp)
{
    if (P.nshape > 0) {
        Rec hi = rec_fresh();
        hi.t = t_stale;
        for (int k = 0; k < P.nshape; k++) {
            bool hk = P.shape_kind[k] == 0 ? sphere_test(P.shape[k], P.shape_mat[k], o, d, hi)
                                           : plane_test(P.shape[k], P.shape_mat[k], o, d, hi);
            if (hk) {
                v3 q = o + d * hi.t;
                if (length2(p - q) < length2(p - lp))
                    return true;
            }
        }
    }
    return false;
}

// The exact octree traversal (BVH::intersect): the wide BVH's rare fallback, and the path of
// every query when the wide BVH is off (exact mode, frames before it is adopted).  The plain
// kernel calls it as a function of its own, so that its large state (the ray's k-DOP products,
// the traversal record, the heap) stays out of the register allocation of the hot loop (inlined
// there it made the loop spill on every tile); the result comes back in registers.  Every other
// kernel inlines it (their queries may all take it).  seg: the segment query [lo, hi]
// (bvh_closest_seg), else the whole line.
struct OctQ {
    THit h;
    bool r;
};

__device__ __forceinline__ OctQ octree_query_inl(const KParams& P, v3 o, v3 d, float lo, float hi, bool seg, uint2* lv)
{
    TRay R = make_ray(P, opaque(o), opaque(d));
    OctQ q;
    if (seg) {
        R.lo = lo;
        R.hi = hi;
        q.r = bvh_closest_seg(P, R, q.h, lv);
    } else
        q.r = bvh_closest<false>(P, R, q.h, lv);
    return q;
}

__device__ __noinline__ OctQ octree_query_call(const KParams& P, v3 o, v3 d, float lo, float hi, bool seg, uint2* lv)
{
    return octree_query_inl(P, o, d, lo, hi, seg, lv);
}

// The launch's KParams where the kernel received it (the plain kernel takes KParams as its first
// argument, at offset 0 of the kernel-argument segment): passing the kernel's by-value copy to a
// call would copy all of it into scratch first.
__device__ __forceinline__ const KParams& kernel_params()
{
    return *reinterpret_cast<const KParams*>((const void*)__builtin_amdgcn_kernarg_segment_ptr());
}

template <bool CALL>
__device__ __forceinline__ OctQ octree_query(const KParams& P, v3 o, v3 d, float lo, float hi, bool seg, uint2* lv)
{
    if (CALL)
        return octree_query_call(kernel_params(), o, d, lo, hi, seg, lv);
    return octree_query_inl(P, o, d, lo, hi, seg, lv);
}

// renderer.cpp:340-402
// OCT: the octree walk only (ray_trace_kernel's octree specialisation: no wide-BVH code)
template <bool PLAIN = false, int G = 1, bool CALL = PLAIN, bool OCT = false>
__device__ bool is_shadowed(const KParams& P, v3 p, v3 n, v3 lp, uint2* lv)
{
    if (!P.compute_shadows)
        return false;
    v3 o = p + n * 1.0e-4f;
    v3 d = normalize(lp - p);
    THit h;
    bool r;
    if ((PLAIN || P.enable_bvh) && P.seg_scale > 0.0f) {
        // segment [-m, past the light]: a hit beyond hi fails the distance test below
        // (|p - q| >= t - |n| * 1e-4), one behind the origin does not exist (t >= 0)
        float m, hi;
        bool nan, light;
        {
            const TRay R0 = make_ray(P, o, d);
            m = seg_margin(P, R0);
            nan = R0.nan;
            const float nl = fabsf(n.x) + fabsf(n.y) + fabsf(n.z);
            hi = (sqrtf(length2(p - lp)) + 1.0e-4f * nl) * (1.0f + 0x1p-10f) + m;
            // the frame's light risk keys hold for this ray (wbvh.hpp WRiskArgs)
            light = P.wrisk && lp.x == P.light[0] && lp.y == P.light[1] && lp.z == P.light[2] && hi <= P.risk_G &&
                    nl <= P.risk_nl;
        }
        // (seg_scale > 0: no analytic shapes, so shapes_shadow below has nothing to add)
        bool sh;
        if (!OCT && P.wnodes && P.nnodes > 0 && !nan &&
            wide_shadow<G, PLAIN ? W_STACK_PLAIN : W_STACK>(P, o, d, hi, p, lp, lv, &sh, light))
            return sh;
        const OctQ q = octree_query<CALL>(P, o, d, -m, hi, P.seg_oct != 0, lv);
        h = q.h;
        r = q.r;
        if (r) {
            v3 q = o + d * h.t;
            if (length2(p - q) < length2(p - lp))
                return true;
        }
        if (PLAIN)
            return false;
        return shapes_shadow(P, o, d, h.t, p, lp);
    }
    if (PLAIN || P.enable_bvh) {
        // whole-line query (segment queries off)
        const OctQ oq = octree_query<CALL>(P, o, d, 0.0f, 0.0f, false, lv);
        h = oq.h;
        r = oq.r;
        if (r) {
            v3 q = o + d * h.t;
            if (length2(p - q) < length2(p - lp))
                return true;
        }
    } else {
        TRay R = make_ray(P, o, d);
        h.t = -1.0f;
        for (int k = 0; k < P.ntri_slots; k++) {
            float t, u, v;
            if (tri_test(P.tris, (uint32_t)k, R, t, u, v)) {
                h.t = t;
                v3 q = o + d * h.t;
                if (length2(p - q) < length2(p - lp))
                    return true;
            }
        }
    }
    if (PLAIN)
        return false;   // no analytic shapes
    return shapes_shadow(P, o, d, h.t, p, lp);
}

// BACKGROUND_COLOR, renderer.cpp:19
__device__ __forceinline__ c3 background() { return col(135.0f / 255.0f, 206.0f / 255.0f, 235.0f / 255.0f); }

// The BVH branch of trace_ray (renderer.cpp:1015-1020): the query-global
// HitInfo becomes 'local'; fin takes it when the query returned true and it is nearer.
__device__ __forceinline__ void bvh_record(const KParams& P, const THit& h, bool r, Rec& local, Rec& fin, int& src)
{
    if (h.k >= 0)
        local = tri_record(P, h);
    else
        local.t = h.t != h.t ? h.t : local.t;   // NaN ray: stale NaN record (a select: a conditional
                                                // partial store kept the record in scratch)
    if (r && (local.t < fin.t || fin.t == -1)) {
        fin = local;
        src = local.tri;
    }
}

// The analytic-shape loop of trace_ray (renderer.cpp:1029-1036), reusing 'local'.
__device__ __forceinline__ void shapes_closest(const KParams& P, v3 o, v3 d, Rec& local, Rec& fin, int& src)
{
    for (int k = 0; k < P.nshape; k++) {
        bool hk = P.shape_kind[k] == 0 ? sphere_test(P.shape[k], P.shape_mat[k], o, d, local)
                                       : plane_test(P.shape[k], P.shape_mat[k], o, d, local);
        if (hk && (local.t < fin.t || fin.t == -1)) {
            fin = local;
            src = -2 - k;
        }
    }
}

// Closest hit over the BVH then the analytic shapes (renderer.cpp:1015-1037).
// fin is the caller's HitInfo; returns the source (-1 none, >=0 triangle, -2-k shape k).
// With the wide BVH (P.wnodes), a certified query takes its answer; one it cannot certify
// is traced through the octree here.
template <bool PLAIN = false, int G = 1, bool OCT = false>
__device__ int closest_hit(const KParams& P, v3 o, v3 d, Rec& fin, uint2* lv)
{
    Rec local = rec_fresh();
    int src = -1;
    if (PLAIN || P.enable_bvh) {
        THit h;
        bool r = false;
        const bool wide = !OCT && P.wnodes && P.nnodes > 0 && !ray_is_nan(o, d);
        if (wide && wide_closest<G, PLAIN ? W_STACK_PLAIN : W_STACK>(P, o, d, h, r, lv, &local)) {
            // certified: a hit's record is already in local (a miss leaves it fresh)
            if (r && (local.t < fin.t || fin.t == -1)) {
                fin = local;
                src = local.tri;
            }
        } else {
            const OctQ q = octree_query<PLAIN && !OCT>(P, o, d, 0.0f, 0.0f, false, lv);
            bvh_record(P, q.h, q.r, local, fin, src);
        }
    } else {
        TRay R = make_ray(P, o, d);
        // brute-force loop, renderer.cpp:1021-1027: fin takes every hit nearer
        // than itself; local keeps the last triangle that was hit.
        THit best, last;
        best.k = -1;
        last.k = -1;
        float bt = fin.t;
        for (int k = 0; k < P.ntri_slots; k++) {
            float t, u, v;
            if (tri_test(P.tris, (uint32_t)k, R, t, u, v)) {
                last.t = t; last.u = u; last.v = v; last.k = k;
                if (t < bt || bt == -1) {
                    bt = t;
                    best = last;
                }
            }
        }
        if (best.k >= 0) {
            fin = tri_record(P, best);
            src = fin.tri;
        }
        if (last.k >= 0)
            local = tri_record(P, last);
    }
    if (!PLAIN)
        shapes_closest(P, o, d, local, fin, src);
    return src;
}

// shade_ray_inter_point (renderer.cpp:556-617) up to (not including) the
// reflection term: for RT_SHADING, fc = diffuse + specular, halved when
// shadowed, plus emission; for the debug modes fc is the final colour.  The
// caller adds "+ compute_reflection(..) * reflection" and the ambient term
// (shade_finish).  Normal mapping overwrites h.normal, which persists in the
// caller's HitInfo exactly as in the reference (renderer.cpp:571-572).
struct Direct {
    c3 fc;
    v3 ip;
    bool shadowed;
};

// RT_SHADING up to the shadow test: diffuse + specular at the hit (renderer.cpp:556-590).
// PLAIN: the scene enables no texture map (the kernel's plain specialisation).
template <bool PLAIN = false>
__device__ c3 shade_lit(const KParams& P, v3 ro, v3 rd, Rec& h, v3& ip_out)
{
    c3 fc = col(0.0f, 0.0f, 0.0f);
    float u = h.u, v = h.v;
    v3 ip = ro + rd * h.t;
    ip_out = ip;
    v3 cam = mk(P.cam_pos[0], P.cam_pos[1], P.cam_pos[2]);
    v3 light = mk(P.light[0], P.light[1], P.light[2]);
    if (!PLAIN && P.enable_displacement_mapping)
        parallax_occlusion_mapping(P, h.tri, h.u, h.v, normalize(cam - ip), u, v);
    v3 dl = normalize(light - ip);
    if (!PLAIN && P.enable_normal_mapping)
        h.normal = normal_mapping(P, h, u, v);
    const float* m = mat_of(P, h.mat);
    float ao = 1.0f;
    if (!PLAIN && P.enable_ao_mapping) {
        float tu, tv;
        get_tex_coords(P, h.tri, u, v, tu, tv);
        ao = tex_floor(P.tex[TEX_AO], tu, tv).r;
    }
    c3 dc;
    if (!PLAIN && P.enable_diffuse_mapping) {
        float tu, tv;
        get_tex_coords(P, h.tri, u, v, tu, tv);
        dc = tex_floor(P.tex[TEX_DIFFUSE], tu, tv);
        float f = smax(0.5f, dot(h.normal, normalize(cam - ip)));
        dc = dc * col(f, f, f);
    } else {
        float f = smax(0.0f, dot(h.normal, dl));   // compute_diffuse, :263-266
        dc = mat_col(m, 3) * col(f, f, f);
    }
    fc = fc + (dc * ao) * (float)(P.enable_diffuse != 0);
    c3 spec;   // compute_specular, :270-280
    {
        v3 hv = normalize(dl - rd);
        float angle = dot(hv, h.normal);
        if (angle <= m[15])
            spec = col(0, 0, 0);
        else {
            float pw = powf(smax(0.0f, angle), m[14]);
            spec = mat_col(m, 6) * col(pw, pw, pw);
        }
    }
    fc = fc + spec * (float)(P.enable_specular != 0);
    return fc;
}

// renderer.cpp:591-593: halve when shadowed, add the emission.
__device__ __forceinline__ c3 shade_shadow_emit(const KParams& P, c3 fc, const float* m, bool shadowed)
{
    if (shadowed)
        fc = fc * col(0.5f, 0.5f, 0.5f);
    return fc + mat_col(m, 9) * (float)(P.enable_emissive != 0);
}

// debug shading methods (renderer.cpp:596-613); the returned colour is final.
__device__ c3 shade_debug(const KParams& P, const Rec& h)
{
    c3 fc = col(0.0f, 0.0f, 0.0f);
    if (P.shading_method == ABS_NORMALS) {
        fc = col(fabsf(h.normal.x), fabsf(h.normal.y), fabsf(h.normal.z));
    } else if (P.shading_method == PASTEL_NORMALS) {
        fc = (col(h.normal.x, h.normal.y, h.normal.z) + col(1.0f, 1.0f, 1.0f)) * 0.5f;
    } else if (P.shading_method == BARYCENTRIC) {
        fc = (col(1, 0, 0) * h.u + col(0, 1.0f, 0) * h.v) + col(0, 0, 1) * (1 - h.u - h.v);
    } else if (P.shading_method == VISUALIZE_AO) {
        c3 c = col(0.9f, 0.9f, 0.9f);
        if (P.enable_ao_mapping) {
            float tu, tv;
            get_tex_coords(P, h.tri, h.u, h.v, tu, tv);
            float a = tex_floor(P.tex[TEX_AO], tu, tv).r;
            c = c * col(a, a, a);
        }
        fc = c;
    }
    return fc;
}

template <bool PLAIN = false, int G = 1, bool OCT = false>
__device__ Direct shade_direct(const KParams& P, v3 ro, v3 rd, Rec& h, uint2* lv, unsigned& nshadow)
{
    Direct out;
    out.shadowed = false;
    out.ip = mk(0, 0, 0);
    if (PLAIN || P.shading_method == RT_SHADING) {
        c3 fc = shade_lit<PLAIN>(P, ro, rd, h, out.ip);
        if (P.compute_shadows)
            nshadow++;
        v3 light = mk(P.light[0], P.light[1], P.light[2]);
        if (PLAIN) PH_MARK(3);
        out.shadowed = is_shadowed<PLAIN, G, PLAIN && !OCT, OCT>(P, out.ip, h.normal, light, lv);
        if (PLAIN) PH_MARK(4);
        out.fc = shade_shadow_emit(P, fc, mat_of(P, h.mat), out.shadowed);
    } else
        out.fc = shade_debug(P, h);
    return out;
}

__device__ __forceinline__ c3 clamp3(c3 c) { return col(clamp01(c.r), clamp01(c.g), clamp01(c.b)); }

// renderer.cpp:594-616: "+ reflection * reflection" (refl > 0 only), "+ ambient", clamp.
__device__ __forceinline__ c3 shade_finish(const KParams& P, c3 fc, const float* m, c3 refl_color)
{
    float refl = m[12];
    if (refl > 0.0f)
        fc = fc + refl_color * refl;
    fc = fc + (col(0.1f, 0.1f, 0.1f) * mat_col(m, 0)) * (1 - refl) * (float)(P.enable_ambient != 0);
    return clamp3(fc);
}

// trace_ray miss colour (renderer.cpp:1052-1065); alpha of the returned Color
template <bool PLAIN = false>
__device__ c3 miss_color(const KParams& P, v3 d, float& alpha)
{
    alpha = 1.0f;
    if (PLAIN)
        return background();
    if (P.enable_skysphere) {
        float u = (float)(0.5 + (double)atan2f(-d.z, -d.x) / (2 * M_PI));
        float v = (float)(0.5 + (double)asinf(-d.y) / M_PI);
        return tex_floor(P.tex[TEX_SKYSPHERE], u, v, &alpha);
    } else if (P.enable_skybox)
        return skybox_sample(P, d, &alpha);
    return background();
}

// XorShiftGenerator::get_rand / get_rand_bilateral (xorshift.h:43-57) on a
// per-pixel stream seeded from the pixel index (the reference seeds one stream
// per OpenMP thread with std::rand()).
__device__ __forceinline__ uint32_t pixel_seed(uint32_t pixel, uint32_t seed)
{
    uint32_t x = pixel * 0x9E3779B9u ^ seed;
    x ^= x >> 16; x *= 0x7feb352dU;
    x ^= x >> 15; x *= 0x846ca68bU;
    x ^= x >> 16;
    return x ? x : 0x9E3779B9u;
}

// Path-keyed streams (oracle/ref_harness.cpp HRng): the frame of a primary hit is
// keyed pixel_seed(pixel, seed); sample i of a frame draws from sample_state(key, i)
// and the frame its hit spawns is keyed child_key(key, i).
__device__ __forceinline__ uint32_t mix32(uint32_t x)
{
    x ^= x >> 16; x *= 0x7feb352dU;
    x ^= x >> 15; x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

__device__ __forceinline__ uint32_t sample_state(uint32_t key, uint32_t i)
{
    uint32_t x = mix32(key ^ (0x9E3779B9u * (2u * i + 1u)));
    return x ? x : 0x9E3779B9u;
}

__device__ __forceinline__ uint32_t child_key(uint32_t key, uint32_t i)
{
    return mix32(key ^ (0x85EBCA6Bu * (2u * i + 2u)));
}

__device__ __forceinline__ float rng_bilateral(uint32_t& s)
{
    uint32_t x = s;
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    s = x;
    return (float)x / (float)UINT32_MAX * 2 - 1;
}

// One pending Renderer::compute_reflection call (renderer.cpp:283-338) of the
// trace at depth d: its samples are traced at depth d + 1 into the shared
// reflection_hit_info 'rhi' (renderer.cpp:286).
struct Frame {
    c3 fc;          // shade_direct colour of the hit that reflects
    c3 total;
    v3 ro, perfect, n;
    float rough;
    int mat, i, sc;
    uint32_t key;   // RNG key of this compute_reflection call
    Rec rhi;
};

constexpr int MAX_FRAMES = 16;   // max_recursion_depth <= 15 with reflective materials

struct PixelOut {
    c3 color;
    float alpha;
    Rec fin;
    int src;
    bool found, shadowed;
};

// Renderer::trace_ray (renderer.cpp:1008-1066) for one primary ray, with the
// compute_reflection recursion (when REFL) unrolled onto an explicit stack.
template <bool REFL, bool PLAIN = false, int G = 1, bool OCT = false>
__device__ PixelOut trace_pixel(const KParams& P, v3 cam, v3 rd0, uint2* lv, uint32_t pixel_key, unsigned& nshadow,
                                unsigned& nrefl)
{
    PixelOut po;
    po.fin = rec_fresh();
    po.found = po.shadowed = false;
    po.alpha = 1.0f;
    po.src = closest_hit<PLAIN && !REFL, REFL ? 1 : G, OCT>(P, cam, rd0, po.fin, lv);
    if (PLAIN) PH_MARK(2);
    if (!REFL) {
        if (PLAIN && po.fin.t > 0.1f) {
            // shade_direct<true> with what the pixel needs after its shadow query (the lit colour, the
            // material, the record's t and the source) waiting in the lane's LDS slots past the traversal
            // stack: the query's loop takes every register, and values held across it were spilled to
            // scratch (HBM writes)
            po.found = true;
            v3 ip;
            const c3 fc = shade_lit<true>(P, cam, rd0, po.fin, ip);
            if (P.compute_shadows)
                nshadow++;
            uint2* sv = lv + (size_t)lds_save_slot_plain<OCT>(P) * BLOCK;
            sv[0] = make_uint2(fbits(fc.r), fbits(fc.g));
            sv[BLOCK] = make_uint2(fbits(fc.b), (uint32_t)po.fin.mat);
            sv[2 * BLOCK] = make_uint2(fbits(po.fin.t), (uint32_t)po.src);
            asm volatile("" ::: "memory");
            const v3 light = mk(P.light[0], P.light[1], P.light[2]);
            if (PLAIN) PH_MARK(3);
            po.shadowed = is_shadowed<true, G, !OCT, OCT>(P, ip, po.fin.normal, light, lv);
            if (PLAIN) PH_MARK(4);
            asm volatile("" ::: "memory");
            const uint2 s0 = sv[0], s1 = sv[BLOCK], s2 = sv[2 * BLOCK];
            po.fin.mat = (int)s1.y;
            po.fin.t = bitsf(s2.x);
            po.src = (int)s2.y;
            const float* m = mat_of(P, po.fin.mat);
            po.color = shade_finish(P, shade_shadow_emit(P, col(bitsf(s0.x), bitsf(s0.y), bitsf(s1.x)), m, po.shadowed), m,
                                    col(0, 0, 0));
            return po;
        }
        if (po.fin.t > 0.1f) {
            po.found = true;
            Direct D = shade_direct<PLAIN, G, OCT>(P, cam, rd0, po.fin, lv, nshadow);
            po.shadowed = D.shadowed;
            po.color = PLAIN || P.shading_method == RT_SHADING
                           ? shade_finish(P, D.fc, mat_of(P, po.fin.mat), col(0, 0, 0))
                           : clamp3(D.fc);
        } else
            po.color = miss_color<PLAIN>(P, rd0, po.alpha);
        return po;
    }

    Frame fr[MAX_FRAMES];
    const int N = P.rough_reflections_sample_count;
    enum { S_TRACE, S_RET, S_NEXT };
    int state, depth = 0, f = 0;
    v3 ro = cam, rd = rd0;
    c3 ret = col(0, 0, 0);
    bool first = true;   // the depth-0 closest hit is already in po.fin
    uint32_t next_key = pixel_key;   // key of a frame spawned by the trace in progress
    state = S_TRACE;
    for (;;) {
        if (state == S_TRACE) {
            // ---- trace_ray(ray, fin, depth) ----
            Rec& fin = depth == 0 ? po.fin : fr[depth - 1].rhi;
            if (depth > P.max_recursion_depth) {
                ret = col(0.0f, 0.0f, 0.0f);
                state = S_RET;
                continue;
            }
            if (!first)
                closest_hit(P, ro, rd, fin, lv);
            first = false;
            if (fin.t > 0.1f) {
                if (depth == 0)
                    po.found = true;
                Direct D = shade_direct(P, ro, rd, fin, lv, nshadow);
                if (depth == 0)
                    po.shadowed = D.shadowed;
                if (P.shading_method != RT_SHADING) {
                    ret = clamp3(D.fc);
                    state = S_RET;
                    continue;
                }
                const float* m = mat_of(P, fin.mat);
                if (!(m[12] > 0.0f)) {
                    ret = shade_finish(P, D.fc, m, col(0, 0, 0));
                    state = S_RET;
                    continue;
                }
                // compute_reflection prologue, renderer.cpp:285-296
                Frame& F = fr[depth];
                F.fc = D.fc;
                F.mat = fin.mat;
                F.n = fin.normal;
                F.ro = D.ip + F.n * 0.01f;
                F.perfect = rd - (2 * dot(rd, F.n)) * F.n;
                if (P.enable_roughness_mapping) {
                    float tu, tv;
                    get_tex_coords(P, fin.tri, fin.u, fin.v, tu, tv);
                    F.rough = tex_floor(P.tex[TEX_ROUGHNESS], tu, tv).r;
                } else
                    F.rough = m[13];
                F.i = 0;
                F.sc = 0;
                F.total = col(0.0f, 0.0f, 0.0f);
                F.key = next_key;
                F.rhi = rec_fresh();
                f = depth;
                state = S_NEXT;
            } else {
                float a;
                ret = miss_color(P, rd, a);
                if (depth == 0)
                    po.alpha = a;
                state = S_RET;
            }
        } else if (state == S_RET) {
            // ---- the trace at 'depth' returned ret ----
            if (depth == 0)
                break;
            Frame& F = fr[depth - 1];
            F.total = F.total + ret;
            if (F.rough > 0) {
                F.sc++;
                F.i++;
            } else {
                F.sc = 1;
                F.i = N;   // pure specular: break
            }
            f = depth - 1;
            state = S_NEXT;
        } else {
            // ---- frame f: next sample, or return the reflection colour ----
            Frame& F = fr[f];
            if (F.i < N) {
                v3 dir;
                next_key = child_key(F.key, (uint32_t)F.i);
                if (F.rough > 0) {
                    uint32_t rng = sample_state(F.key, (uint32_t)F.i);
                    float rx = rng_bilateral(rng);
                    float ry = rng_bilateral(rng);
                    float rz = rng_bilateral(rng);
                    v3 rdir = normalize(mk(rx, ry, rz));
                    if (dot(rdir, F.n) < 0)
                        rdir = -rdir;
                    dir = F.rough * rdir + (1 - F.rough) * F.perfect;
                } else
                    dir = F.perfect;
                nrefl++;
                ro = F.ro;
                rd = dir;
                depth = f + 1;
                state = S_TRACE;
            } else {
                const float* m = mat_of(P, F.mat);
                float sc = (float)F.sc, rf = m[12];
                c3 R = (F.total / col(sc, sc, sc)) * col(rf, rf, rf);
                ret = shade_finish(P, F.fc, m, R);
                depth = f;
                state = S_RET;
            }
        }
    }
    po.color = ret;
    return po;
}

// renderer.cpp:1104-1110: a primary hit writes _z_buffer = -(o.z + d.z * t) and the
// (normal-mapped) hit normal; other pixels keep the cleared INFINITY / Vector(0)
// (the UI clears both before every render, mainwindow.cpp:184-185).
__device__ __forceinline__ void write_ssao_buffers(const KParams& P, size_t o, bool found, v3 cam, v3 rd,
                                                   const Rec& fin)
{
    P.zbuf[o] = found ? -(cam.z + rd.z * fin.t) : INFINITY;
    P.nbuf[o] = found ? make_float4(fin.normal.x, fin.normal.y, fin.normal.z, 0.0f) : make_float4(0, 0, 0, 0);
}

// tile -> (tile column, tile row) without an integer division: the float quotient through
// 1 / tiles_x is within one of the true one for tile < 2^24, then corrected
__device__ __forceinline__ void tile_xy(const KParams& P, int tile, int& tx, int& ty)
{
    const int W = P.tiles_x;
    if (tile >= (1 << 24)) {
        tx = tile % W;
        ty = tile / W;
        return;
    }
    int q = (int)((float)tile * (1.0f / (float)W));
    int r = tile - q * W;
    if (r < 0) {
        q--;
        r += W;
    } else if (r >= W) {
        q++;
        r -= W;
    }
    tx = r;
    ty = q;
}

// Global internal row of a launch-local row (interleaved bands across ranks, or a band list).
__device__ __forceinline__ int global_row(const KParams& P, int lr)
{
    if (P.nranks == 1)
        return lr;   // (band * 1 + 0) * band_rows + lr - band * band_rows
    int band = lr / P.band_rows;
    const int g = P.band_map ? ldg(P.band_map + band) : band * P.nranks + P.rank;
    return g * P.band_rows + (lr - band * P.band_rows);
}

// The persistent tile queue, sharded: shard s owns the tile rows [s Y / 8, (s + 1) Y / 8)
// (a band of the image) and its head counter sits on its own 128-B line.  A wave starts on the
// shard of its block's XCD group (blockIdx % 8: blocks b and b + 8 share an XCD, so a
// band's rays share that XCD's L2) and moves to the next shard when its own is empty;
// it is done once it has found all eight empty.  One head word serves ~88 dequeues per
// microsecond (MI355X_MICROARCH.md, dequeue row), under the frame's 130K tiles at ~2 ms.
constexpr int BQ_BATCH = 4;   // tickets per block dequeue (<= 255)

// Ticket t of shard s -> tile index (row-major), or -1 past the shard's end.  Measured
// against alternatives (r02): guided chunks of 2-4 adjacent tiles per wave dequeue, tickets
// taken one tile ahead, blocked orders (patches of 8x8 .. 32x16 tiles), 2x2 tile quads per
// block batch and 8-ticket block batches were all slower.
__device__ __forceinline__ int shard_tile(const KParams& P, int s, int t)
{
    const int r0 = (int)((long long)P.tiles_y * s / TILE_SHARDS), r1 = (int)((long long)P.tiles_y * (s + 1) / TILE_SHARDS);
    return t < (r1 - r0) * P.tiles_x ? r0 * P.tiles_x + t : -1;
}


// Block-shared dequeue.  One global atomic takes WAVES_PER_BLOCK consecutive tickets of the
// block's shard, and the block's waves hand them out among themselves through one LDS word
//   bit 31 done | bits 30..24 generation | bits 23..16 tickets in the batch | bits 15..0 next;
// a wave's LDS add returns (generation g, count c, index i): i < c -> the batch's i-th ticket
// (base and shard in slot g & 3); i == c -> this wave takes the next batch (the global atomic,
// moving to the next shard when its own is empty) and publishes generation g + 1 with its own
// ticket already taken; i > c -> it waits for generation g + 1.  The four waves of a block
// then work on four adjacent tiles (one CU's L1), and the frame needs a quarter of the
// global dequeues (a global round trip was ~7 % of a wave's time per tile, MI355X r02).
struct BlockQueue {
    unsigned int word;
    int shard, empty;
    int base[4], sh[4];
    int heavy_done;   // the heavy list is exhausted (any wave may set it)
    int split_done;   // the split tiles' parts are exhausted
    // the block's share of the launch's tile-cost sum and max (KParams::tile_stats; the last wave of
    // the block to finish adds it to the launch's)
    unsigned long long cost_sum;
    unsigned int cost_max;
    int waves_done;
};
__shared__ BlockQueue g_bq;

__device__ __forceinline__ void tile_queue_init()
{
    if (threadIdx.x == 0) {
        g_bq.word = 0u;   // generation 0 with no tickets: the first wave refills
        g_bq.shard = (int)(blockIdx.x & (TILE_SHARDS - 1));
        g_bq.empty = 0;
        g_bq.heavy_done = 0;
        g_bq.split_done = 0;
        g_bq.cost_sum = 0;
        g_bq.cost_max = 0;
        g_bq.waves_done = 0;
    }
    __syncthreads();
}

// A tile's (or a split part's: its cost x G stands for the tile's in the max) cost into the block's sums.
__device__ __forceinline__ void tile_stats_add(uint32_t c, uint32_t cmax)
{
    __hip_atomic_fetch_add(&g_bq.cost_sum, (unsigned long long)c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __hip_atomic_fetch_max(&g_bq.cost_max, cmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// At a wave's exit: the last wave of the block adds the block's sums to the launch's (2 global atomics
// per block instead of one per tile; heavy_prep_kernel reads them for the next launch).
__device__ __forceinline__ void tile_stats_flush(const KParams& P, int lane)
{
    if (!P.tile_stats || lane != 0)
        return;
    const int k = __hip_atomic_fetch_add(&g_bq.waves_done, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (k != (int)(blockDim.x >> 6) - 1)
        return;
    const unsigned long long s = __hip_atomic_load(&g_bq.cost_sum, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
    const unsigned int m = __hip_atomic_load(&g_bq.cost_max, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
    if (s) atomicAdd(P.tile_stats, s);
    if (m) atomicMax(P.tile_stats + 1, (unsigned long long)m);
}

__device__ __forceinline__ int tile_queue_next_shards(const KParams& P);

// The next tile: first the heavy list (one global ticket per tile), then the sharded queue with the
// heavy tiles skipped (each tile exactly once; the split tiles of heavy_prep_kernel are
// trace_split_part's).
__device__ __forceinline__ int tile_queue_next(const KParams& P)
{
    const int lane = threadIdx.x & 63;
    if (P.heavy_list) {
        if (!__builtin_amdgcn_readfirstlane(__hip_atomic_load(&g_bq.heavy_done, __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_WORKGROUP))) {
            int t = 0;
            if (lane == 0)
                t = atomicAdd(P.heavy_ctr + 1, 1);
            t = __builtin_amdgcn_readfirstlane(t);
            if (t < min(ldg(P.heavy_ctr), P.tiles_x * P.tiles_y / 16))   // (heavy_prep_kernel counts past its cap)
                return ldg(P.heavy_list + t);
            if (lane == 0)
                __hip_atomic_store(&g_bq.heavy_done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        for (;;) {
            const int tile = tile_queue_next_shards(P);
            if (tile < 0 || !((ldg(P.heavy_bits + (tile >> 5)) >> (tile & 31)) & 1u))
                return tile;
        }
    }
    return tile_queue_next_shards(P);
}

__device__ __forceinline__ int tile_queue_next_shards(const KParams& P)
{
    const int lane = threadIdx.x & 63;
    for (;;) {
        unsigned int w = 0;
        if (lane == 0)
            w = __hip_atomic_fetch_add(&g_bq.word, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
        w = __builtin_amdgcn_readfirstlane(w);
        if (w & 0x80000000u)
            return -1;
        const unsigned int g = (w >> 24) & 0x7fu, c = (w >> 16) & 0xffu, i = w & 0xffffu;
        if (i < c) {
            const int slot = (int)(g & 3u);
            return shard_tile(P, g_bq.sh[slot], g_bq.base[slot] + (int)i);
        }
        if (i == c) {
            // this wave refills: WAVES_PER_BLOCK tickets of the first non-empty shard
            int shard = g_bq.shard, empty = g_bq.empty, b = 0, n = 0;
            while (empty < TILE_SHARDS) {
                int t = 0;
                if (lane == 0)
                    t = (int)atomicAdd(reinterpret_cast<unsigned int*>(&P.counters[NCOUNTERS + 16 * shard]),
                                       (unsigned)BQ_BATCH);
                b = __builtin_amdgcn_readfirstlane(t);
                n = 0;
                while (n < BQ_BATCH && shard_tile(P, shard, b + n) >= 0)
                    n++;
                if (n > 0)
                    break;
                empty++;
                shard = (shard + 1) & (TILE_SHARDS - 1);
            }
            const unsigned int g1 = (g + 1u) & 0x7fu;
            if (lane == 0) {
                g_bq.shard = shard;
                g_bq.empty = empty;
                g_bq.base[g1 & 3u] = b;
                g_bq.sh[g1 & 3u] = shard;
                // publish: the batch's fields are visible before the word that names them
                __hip_atomic_store(&g_bq.word, n > 0 ? (g1 << 24) | ((unsigned)n << 16) | 1u : 0x80000000u,
                                   __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            return n > 0 ? shard_tile(P, shard, b) : -1;
        }
        // another wave is taking the next batch
        for (;;) {
            unsigned int v = 0;
            if (lane == 0)
                v = __hip_atomic_load(&g_bq.word, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            v = __builtin_amdgcn_readfirstlane(v);
            if ((v & 0x80000000u) || ((v >> 24) & 0x7fu) != g)
                break;
            __builtin_amdgcn_s_sleep(2);
        }
    }
}

// The wave's instruction-issue priority among the waves of its SIMD: heavy-list tiles carry a level
// (heavy_prep_kernel, from the tile's cost in the previous launch) so that the few tiles whose single
// wave spans most of the launch (grazing silhouette and terminator rays) issue ahead
// of the cheap tiles sharing their SIMD; every other tile runs at level 0.
__device__ __forceinline__ void set_wave_prio(int level)
{
    switch (level) {
    case 3: __builtin_amdgcn_s_setprio(3); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    default: __builtin_amdgcn_s_setprio(0); break;
    }
}

// ImageUtils::downscale_image_qt_ARGB32 (imageUtils.h:98-147) fused into the tile: the
// wave holds its 8x8 tile's ARGB values one per lane (lane = 8 * row + column), every
// lane active; the f x f blocks (f = 1 << P.ds_shift, f | 8, rows f-aligned in the band)
// are summed per 8-bit channel across lanes, divided by f * f with truncation (the sums
// are non-negative: a shift) and written by the block's first lane, as downscale_kernel.
// G > 1 (trace_split_part): pixel i of the wave's C-wide block is held by lanes G i .. G i + G - 1
// (f <= the block's columns and rows, checked on the host).
template <int G = 1, int C0 = 8>
__device__ __forceinline__ void downscale_tile(const KParams& P, int lane, int lr, int px, uint32_t c, int C = C0)
{
    int r = (int)((c >> 16) & 0xffu), g = (int)((c >> 8) & 0xffu), b = (int)(c & 0xffu);
    const int f = 1 << P.ds_shift;
    for (int m = 1; m < f; m <<= 1) {   // columns, within the lane's row of C
        r += __shfl_xor(r, G * m);
        g += __shfl_xor(g, G * m);
        b += __shfl_xor(b, G * m);
    }
    for (int m = C; m < C * f; m <<= 1) {   // rows
        r += __shfl_xor(r, G * m);
        g += __shfl_xor(g, G * m);
        b += __shfl_xor(b, G * m);
    }
    const int pl = lane / G;   // the lane's pixel: C row + column
    if ((lane & (G - 1)) == 0 && ((pl % C) & (f - 1)) == 0 && ((pl / C) & (f - 1)) == 0) {
        const int s2 = 2 * P.ds_shift;
        P.ds_out[(size_t)(lr >> P.ds_shift) * (size_t)(P.rw >> P.ds_shift) + (size_t)(px >> P.ds_shift)] =
            qrgb(r >> s2, g >> s2, b >> s2);
    }
}

// Renderer::ray_trace's ray generation (renderer.cpp:1086-1098) for pixel (px, py): the two
// Transform::operator()(Point) (mat.cpp:83-100) skip their division when the host found w
// constant (KParams::proj_mode, c2w_affine); the direction is bit for bit the general path's.
__device__ __forceinline__ v3 camera_dir(const KParams& P, int px, int py, v3 cam)
{
    const float y_world = ((float)py + 0.5f) / P.rh * 2 - 1;
    const float x_world = ((float)px + 0.5f) / P.rw * 2 - 1;
    v3 vs;
    if (P.proj_mode != 0) {
        const float* m = P.proj_inv;
        const float x = x_world, y = y_world, z = -1.0f;
        const float xt = m[0] * x + m[1] * y + m[2] * z + m[3];
        const float yt = m[4] * x + m[5] * y + m[6] * z + m[7];
        const float zt = m[8] * x + m[9] * y + m[10] * z + m[11];
        const float w = P.proj_w;
        vs = P.proj_mode == 1 ? mk(xt, yt, zt) : mk(xt * w, yt * w, zt * w);
    } else
        vs = xform_point(P.proj_inv, mk(x_world, y_world, -1));
    v3 ws;
    if (P.c2w_affine && fabsf(vs.x) < INFINITY && fabsf(vs.y) < INFINITY && fabsf(vs.z) < INFINITY) {
        const float* m = P.cam_to_world;
        ws = mk(m[0] * vs.x + m[1] * vs.y + m[2] * vs.z + m[3], m[4] * vs.x + m[5] * vs.y + m[6] * vs.z + m[7],
                m[8] * vs.x + m[9] * vs.y + m[10] * vs.z + m[11]);
    } else
        ws = xform_point(P.cam_to_world, vs);
    return normalize(ws - cam);
}

// The split tiles (KParams::heavy_group = G, heavy_prep_kernel's second list): a tile whose one wave
// would outlast the launch's mean wave (grazing silhouette rays walk 100-170 wide nodes)
// is traced as G parts of 8 / G rows, each part by one wave of ray_trace_kernel with G lanes per pixel
// (a lane group: wbvh_closest<.., G> walks the pixel's tree on its G lanes together).  The parts are
// taken first, by the ticket heavy_ctr[2] over the list's G * heavy_ctr[3] parts, so they run on
// different waves at the same time; each adds its cycles to the tile's cost (heavy_prep_kernel zeroed
// it).  Plain scenes over the wide BVH only, fused SSAA factors up to 8 / G (the host checks).  Per
// pixel the results are trace_pixel<false, true>'s: the group's query returns the one-lane answer.
template <int G>
__device__ __forceinline__ void trace_split_part(const KParams& P, uint2* lv, int t, int lane, unsigned& nshadow)
{
    static_assert(G > 1 && G <= 8 && (G & (G - 1)) == 0, "2, 4 or 8 lanes per pixel");
    const int cap = P.tiles_x * P.tiles_y / 16;   // (heavy_prep_kernel: the split list at list + cap)
    const int np = P.split_parts;                 // parts per tile: G (every lane busy) or 2G (half the lanes)
    const int tq = ldg(P.heavy_list + cap + t / np), part = t % np;
    const int tile = tq & 0x0fffffff;
    set_wave_prio(tq >> 28);
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    int tx, ty;
    tile_xy(P, tile, tx, ty);
    // part p: columns (p % (8 / C)) C .. + C, rows (p / (8 / C)) R .. + R of the tile (C x R = 64 / np
    // pixels: C = 8 and R = 64 / np / 8 down to 16 pixels, then 4 x 2 and 2 x 2 blocks)
    const int npix = 64 / np;
    const int C = npix >= 16 ? 8 : npix / 2, R = npix / C;
    const int pl = lane / G;   // the lane's pixel among the part's, row-major C wide
    const int px = tx * 8 + (part % (8 / C)) * C + pl % C;
    const int lr = ty * 8 + (part / (8 / C)) * R + pl / C;
    const int py = lr < P.local_rows ? global_row(P, lr) : P.rh;
    if (pl < npix && px < P.rw && py < P.rh) {   // (the same for the G lanes of a pixel)
        const v3 cam = mk(P.cam_pos[0], P.cam_pos[1], P.cam_pos[2]);
        const v3 rd = camera_dir(P, px, py, cam);
        unsigned ns = 0, nr = 0;
        PixelOut po = trace_pixel<false, true, G>(P, cam, rd, lv, 0u, ns, nr);
        if ((lane & (G - 1)) == 0)
            nshadow += ns;   // (one count per pixel)
        const size_t o = (size_t)lr * P.rw + px;
        const uint32_t c = color_to_argb(po.color);
        if (P.ds_out) downscale_tile<G>(P, lane, lr, px, c, C);
        if ((lane & (G - 1)) == 0) {
            if (P.argb) P.argb[o] = c;
            if (P.rgba) P.rgba[o] = make_float4(po.color.r, po.color.g, po.color.b, po.alpha);
            if (P.hit_id) P.hit_id[o] = po.found ? po.src : -1;
            if (P.hit_t) P.hit_t[o] = po.fin.t;
            if (P.shadow) P.shadow[o] = (uint8_t)(po.found && po.shadowed);
        }
    }
    const uint64_t c = __builtin_amdgcn_s_memtime() - t0;
    if (lane == 0) {
        const uint32_t c32 = c > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)c;
        atomicAdd(P.tile_cost + tile, c32);
        tile_stats_add(c32, c32 > 0xFFFFFFFFu / G ? 0xFFFFFFFFu : c32 * G);
    }
}

// Renderer::ray_trace (renderer.cpp:1068-1116): one lane per pixel, one wave
// per 8x8 tile.  Waves are persistent and pull tiles from the sharded device-scope
// queue (tile_queue_next): shadow-ray-heavy tiles cluster around the object, so
// a static block -> tile (-> XCD) mapping leaves whole XCDs idle while others
// still trace; dynamic pulling keeps every CU busy until the queue drains.
// PLAIN: no texture map, sky, analytic shape, debug shading or SSAO buffer (host-checked,
// KParams::plain): those code paths are compiled out.
// OCT (with PLAIN): frames before the wide BVH is resident -- the octree walk in line, no
// wide-BVH code, at its own occupancy
template <bool REFL, bool PLAIN = false, bool OCT = false>
__global__ __launch_bounds__(BLOCK, OCT ? RT_OCC_OCT : PLAIN ? RT_OCC_PLAIN : RT_OCC) void ray_trace_kernel(KParams P_arg)
{
    // The kernel reads its parameters where the kernel received them, through a pointer
    // the compiler cannot hoist out of the tile loop: each field is loaded (scalar cache) where
    // a tile uses it instead of ~100 of them being held in registers across the loop, which
    // spilled (register budget).
    auto kp = __builtin_amdgcn_kernarg_segment_ptr();
    (void)P_arg;
    const KParams& P = *reinterpret_cast<const KParams*>((const void*)kp);
    extern __shared__ uint2 lds_levels[];
    uint2* lv = lds_levels + threadIdx.x;
    int lane = threadIdx.x & 63;
    unsigned nshadow = 0, nrefl = 0;
    tile_queue_init();
#if RT_PHASE_TIME
    if (PLAIN && lane == 0) {
        for (int k = 0; k < 7; k++)
            g_phase[threadIdx.x >> 6][k] = 0;
        g_phase[threadIdx.x >> 6][7] = __builtin_amdgcn_s_memtime();
    }
#endif
    for (;;) {
        auto kpl = kp;
        asm volatile("" : "+s"(kpl));   // (the loop's loads depend on it: not hoisted)
        const KParams& P = *reinterpret_cast<const KParams*>((const void*)kpl);
        const v3 cam = mk(P.cam_pos[0], P.cam_pos[1], P.cam_pos[2]);
        if (PLAIN && !REFL && !OCT && P.heavy_group == SPLIT_G &&
            !__builtin_amdgcn_readfirstlane(__hip_atomic_load(&g_bq.split_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))) {
            // the split tiles' parts first (trace_split_part)
            int t = 0;
            if (lane == 0)
                t = atomicAdd(P.heavy_ctr + 2, 1);
            t = __builtin_amdgcn_readfirstlane(t);
            if (t < P.split_parts * min(ldg(P.heavy_ctr + 3), P.tiles_x * P.tiles_y / 16)) {
                trace_split_part<SPLIT_G>(P, lv, t, lane, nshadow);
                continue;
            }
            if (lane == 0)
                __hip_atomic_store(&g_bq.split_done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        const int tq = tile_queue_next(P);
        if (PLAIN) PH_MARK(6);
        if (tq < 0)
            break;
        const int tile = tq & 0x0fffffff;
        if (P.heavy_list)
            set_wave_prio(tq >> 28);
        const uint64_t tile_t0 = __builtin_amdgcn_s_memtime();
        int tx, ty;
        tile_xy(P, tile, tx, ty);
        int px = tx * 8 + (lane & 7);
        int lr = ty * 8 + (lane >> 3);
        int py = lr < P.local_rows ? global_row(P, lr) : P.rh;
        if (PLAIN) PH_MARK(0);
        if (px >= P.rw || py >= P.rh) {
            if (P.tile_cost && lane == 0)
                P.tile_cost[tile] = 0u;
            continue;
        }
        // ray generation, renderer.cpp:1086-1098
        const v3 rd = camera_dir(P, px, py, cam);
        if (PLAIN) PH_MARK(1);

        uint32_t rng = REFL ? pixel_seed((uint32_t)(py * P.rw + px), P.rng_seed) : 0u;
        PixelOut po = trace_pixel<REFL, PLAIN, 1, OCT>(P, cam, rd, lv, rng, nshadow, nrefl);
        size_t o = (size_t)lr * P.rw + px;
        if (P.argb) P.argb[o] = color_to_argb(po.color);
        if (!REFL && P.ds_out) downscale_tile(P, lane, lr, px, color_to_argb(po.color));
        if (P.rgba) P.rgba[o] = make_float4(po.color.r, po.color.g, po.color.b, po.alpha);
        if (P.hit_id) P.hit_id[o] = po.found ? po.src : -1;
        if (P.hit_t) P.hit_t[o] = po.fin.t;
        if (P.shadow) P.shadow[o] = (uint8_t)(po.found && po.shadowed);
        if (!PLAIN && P.zbuf) write_ssao_buffers(P, o, po.found, cam, rd, po.fin);
        if (PLAIN) PH_MARK(5);
        if (P.tile_cost) {   // the tile's shader cycles (heavy-first order of the next launch)
            const uint64_t c = __builtin_amdgcn_s_memtime() - tile_t0;
            if (lane == 0) {
                const uint32_t c32 = c > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)c;
                P.tile_cost[tile] = c32;
                tile_stats_add(c32, c32);
            }
        }
    }
    tile_stats_flush(P, lane);
#if RT_PHASE_TIME
    if (PLAIN) {
        PH_MARK(0);   // the final (empty) dequeues
        const int wid = (int)(blockIdx.x * WAVES_PER_BLOCK + (threadIdx.x >> 6));
        if (P.dbg && lane == 0 && wid < DBG_WAVES)
            for (int k = 0; k < 7; k++)
                P.dbg[DBG_WORDS * wid + k] = g_phase[threadIdx.x >> 6][k];
    }
#endif
    if (nshadow) atomicAdd(&P.counters[0], (unsigned long long)nshadow);
    if (nrefl) atomicAdd(&P.counters[1], (unsigned long long)nrefl);
}

// ===========================================================================
// Reflections as frames.  trace_pixel<true> walks one pixel's compute_reflection
// recursion on one lane, ray after ray: with rough reflections a pixel owns up to
// N^depth rays and the frame time is set by the costliest pixel's chain.  Here
// every compute_reflection call is a frame record and the recursion runs level by
// level (host loop in renderer.cpp, chunks of frames, depth-first over chunks):
//   gen:    the N sample directions of each frame (path-keyed RNG: no draw
//           depends on another sample)                 renderer.cpp:296-315
//   trace:  every sample's closest-hit query, one lane per sample
//   pass1:  per frame, in sample order: the samples' hits merged into the shared
//           reflection_hit_info, shade_lit (normal mapping rewrites the shared
//           record, as in the reference)               renderer.cpp:286, 1015-1044
//   shadow: every shaded sample's is_shadowed query, one lane per sample
//   spawn:  reflective hits become the next level's frames
//   resolve (after the next level): the samples' colours summed in sample order,
//           (total / sc) * reflection, shade_finish    renderer.cpp:316-337, 594-616
// Per pixel the results are trace_pixel<true>'s, bit for bit.
// ===========================================================================
__device__ __forceinline__ v3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }
__device__ __forceinline__ void st3(float* p, v3 v) { p[0] = v.x; p[1] = v.y; p[2] = v.z; }
__device__ __forceinline__ void st3(float* p, c3 c) { p[0] = c.r; p[1] = c.g; p[2] = c.b; }
__device__ __forceinline__ c3 ldc(const float* p) { return col(p[0], p[1], p[2]); }

__device__ __forceinline__ void wave_count_add(unsigned long long* ctr, unsigned v)
{
    for (int off = 32; off > 0; off >>= 1)
        v += __shfl_xor(v, off);
    if ((threadIdx.x & 63) == 0 && v)
        atomicAdd(ctr, (unsigned long long)v);
}

// compute_reflection prologue (renderer.cpp:285-296) for the hit record h
__device__ __forceinline__ float frame_roughness(const KParams& P, const Rec& h, const float* m)
{
    if (P.enable_roughness_mapping) {
        float tu, tv;
        get_tex_coords(P, h.tri, h.u, h.v, tu, tv);
        return tex_floor(P.tex[TEX_ROUGHNESS], tu, tv).r;
    }
    return m[13];
}

__device__ __forceinline__ int frame_nsamp(const KParams& P, float rough)
{
    int N = P.rough_reflections_sample_count;
    return N <= 0 ? 0 : (rough > 0 ? N : 1);
}

__device__ __forceinline__ void make_frame(const KParams& P, FrameRec& F, v3 ip, v3 n, v3 rd, c3 fc, float rough,
                                           int mat, uint32_t key, int parent)
{
    st3(F.ro, ip + n * 0.01f);
    st3(F.perfect, rd - (2 * dot(rd, n)) * n);
    st3(F.n, n);
    st3(F.fc, fc);
    F.rough = rough;
    F.mat = mat;
    F.key = key;
    F.nsamp = frame_nsamp(P, rough);
    F.parent = parent;
}

// Level 0: the primary ray of every pixel, shaded (with its shadow query); a
// reflective hit becomes a level-1 frame, any other pixel is finished here.
__global__ __launch_bounds__(BLOCK, RT_OCC) void refl_level0_kernel(KParams P_arg, FrameRec* fr1, unsigned int* nfr1)
{
    // the parameters where the kernel received them (not a copy: passing the by-value argument to a
    // call made every lane copy it to scratch, r05: C5's shadow pass wrote ~90 GB per launch)
    const KParams& P = kernel_params();
    (void)P_arg;
    extern __shared__ uint2 lds_levels[];
    uint2* lv = lds_levels + threadIdx.x;
    int lane = threadIdx.x & 63;
    const int ntiles = P.tiles_x * P.tiles_y;
    v3 cam = mk(P.cam_pos[0], P.cam_pos[1], P.cam_pos[2]);
    unsigned nshadow = 0;
    for (;;) {
        int tile = 0;
        if (lane == 0)
            tile = (int)atomicAdd(reinterpret_cast<unsigned int*>(&P.counters[2]), 1u);
        tile = __builtin_amdgcn_readfirstlane(tile);
        if (tile >= ntiles)
            break;
        int tx, ty;
        tile_xy(P, tile, tx, ty);
        int px = tx * 8 + (lane & 7);
        int lr = ty * 8 + (lane >> 3);
        int py = lr < P.local_rows ? global_row(P, lr) : P.rh;
        if (px >= P.rw || py >= P.rh)
            continue;
        // ray generation, renderer.cpp:1086-1098
        const v3 rd = camera_dir(P, px, py, cam);

        Rec fin = rec_fresh();
        int src = closest_hit(P, cam, rd, fin, lv);
        bool found = false, shadowed = false, deferred = false;
        c3 color;
        float alpha = 1.0f;
        size_t o = (size_t)lr * P.rw + px;
        if (0 > P.max_recursion_depth) {
            color = col(0.0f, 0.0f, 0.0f);   // trace_pixel: the depth test after the first closest hit
        } else if (fin.t > 0.1f) {
            found = true;
            Direct D = shade_direct(P, cam, rd, fin, lv, nshadow);
            shadowed = D.shadowed;
            const float* m = mat_of(P, fin.mat);
            if (m[12] > 0.0f) {
                unsigned idx = atomicAdd(nfr1, 1u);
                make_frame(P, fr1[idx], D.ip, fin.normal, rd, D.fc, frame_roughness(P, fin, m), fin.mat,
                           pixel_seed((uint32_t)(py * P.rw + px), P.rng_seed), (int)o);
                deferred = true;
            } else
                color = shade_finish(P, D.fc, m, col(0, 0, 0));
        } else
            color = miss_color(P, rd, alpha);
        if (!deferred) {
            if (P.argb) P.argb[o] = color_to_argb(color);
            if (P.rgba) P.rgba[o] = make_float4(color.r, color.g, color.b, alpha);
        }
        if (P.hit_id) P.hit_id[o] = found ? src : -1;
        if (P.hit_t) P.hit_t[o] = fin.t;
        if (P.shadow) P.shadow[o] = (uint8_t)(found && shadowed);
        if (P.zbuf) write_ssao_buffers(P, o, found, cam, rd, fin);
    }
    if (nshadow) atomicAdd(&P.counters[0], (unsigned long long)nshadow);
}

// keys: 30-bit Morton code of each frame's origin in the scene box (the root's
// axis slabs), so that a level's frames can be sorted for ray coherence
__device__ __forceinline__ uint32_t spread10(uint32_t v)
{
    v &= 0x3ffu;
    v = (v | (v << 16)) & 0x030000ffu;
    v = (v | (v << 8)) & 0x0300f00fu;
    v = (v | (v << 4)) & 0x030c30c3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}

__global__ __launch_bounds__(BLOCK) void refl_keys_kernel(KParams P, const FrameRec* fr, int n, uint32_t* keys,
                                                          int32_t* idx)
{
    int f = blockIdx.x * BLOCK + threadIdx.x;
    if (f >= n)
        return;
    uint32_t q[3];
    for (int a = 0; a < 3; a++) {
        float lo = P.nodes[0].dn[a], hi = P.nodes[0].df[a];
        float t = (fr[f].ro[a] - lo) / (hi - lo);
        t = t == t ? fminf(fmaxf(t, 0.0f), 1.0f) : 0.0f;
        q[a] = (uint32_t)(t * 1023.0f);
    }
    keys[f] = spread10(q[0]) | (spread10(q[1]) << 1) | (spread10(q[2]) << 2);
    idx[f] = f;
}

// keys of the shadow list (ReflArgs::list, RT_REFL_SHADOW_SORT): the 30-bit Morton code of each entry's hit
// point in the scene box, so that the shadow pass takes its segments in spatial order (adjacent lanes
// start from nearby points toward the one light)
__global__ __launch_bounds__(BLOCK) void refl_shadow_keys_kernel(KParams P, const SampleRec* sm, const int32_t* list, int n,
                                                                 uint32_t* keys)
{
    int t = blockIdx.x * BLOCK + threadIdx.x;
    if (t >= n)
        return;
    const SampleRec& S = sm[list[t]];
    uint32_t q[3];
    for (int a = 0; a < 3; a++) {
        float lo = P.nodes[0].dn[a], hi = P.nodes[0].df[a];
        float u = (S.ip[a] - lo) / (hi - lo);
        u = u == u ? fminf(fmaxf(u, 0.0f), 1.0f) : 0.0f;
        q[a] = (uint32_t)(u * 1023.0f);
    }
    keys[t] = spread10(q[0]) | (spread10(q[1]) << 1) | (spread10(q[2]) << 2);
}

// The chunk's sample slots (ReflArgs::sample_major): slot = i * nfr + (p - c0), nfr = c1 - c0, the i-th
// samples of consecutive frames side by side, so that the per-frame passes (pass1, resolve: one lane per
// frame, its samples in order) read their records coalesced; 0: slot = (p - c0) * stride + i, a frame's
// samples side by side
// the frame at sorted position p: the level's sorted copy (ReflArgs::frs, refl_sort_frames_kernel) when
// there is one, else through the order
__device__ __forceinline__ const FrameRec& refl_frame(const ReflArgs& A, int p)
{
    return A.frs ? A.frs[p] : A.fr[A.order[p]];
}

__device__ __forceinline__ int slot_pos(const ReflArgs& A, int slot)
{
    return A.sample_major ? A.c0 + slot % (A.c1 - A.c0) : A.c0 + slot / A.stride;
}
__device__ __forceinline__ int slot_sample(const ReflArgs& A, int slot)
{
    return A.sample_major ? slot / (A.c1 - A.c0) : slot % A.stride;
}
__device__ __forceinline__ int slot_of(const ReflArgs& A, int p, int i)
{
    return A.sample_major ? i * (A.c1 - A.c0) + (p - A.c0) : (p - A.c0) * A.stride + i;
}

// the i-th sample's direction of a frame (renderer.cpp:296-315: path-keyed RNG, no draw depends on another
// sample)
__device__ __forceinline__ v3 refl_dir(const FrameRec& F, int i)
{
    if (F.rough > 0) {
        uint32_t rng = sample_state(F.key, (uint32_t)i);
        float rx = rng_bilateral(rng);
        float ry = rng_bilateral(rng);
        float rz = rng_bilateral(rng);
        v3 rdir = normalize(mk(rx, ry, rz));
        if (dot(rdir, ld3(F.n)) < 0)
            rdir = -rdir;
        return F.rough * rdir + (1 - F.rough) * ld3(F.perfect);
    }
    return ld3(F.perfect);
}

// keys of the feed's tickets (ReflArgs::perm, RT_REFL_DIR_SORT): each slot's direction binned by its
// cube-map face and a 2 x 2 cell of the face (the slots without a ray last); a stable sort by these keys
// keeps the slots' order (the frames' Morton order) inside each bin, so that a wave's lanes take rays of
// nearby origins and similar directions
__global__ __launch_bounds__(BLOCK) void refl_dir_keys_kernel(KParams P, ReflArgs A, uint32_t* keys, int32_t* vals)
{
    const int slot = (int)(blockIdx.x * BLOCK + threadIdx.x);
    const int nslot = (A.c1 - A.c0) * A.stride;
    if (slot >= nslot)
        return;
    const int i = slot_sample(A, slot);
    const FrameRec& F = refl_frame(A, slot_pos(A, slot));
    uint32_t key = 127u;
    if (i < F.nsamp && A.level <= P.max_recursion_depth) {
        const v3 d = refl_dir(F, i);
        const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
        int face;
        float u, v, m;
        if (ax >= ay && ax >= az) {
            face = d.x < 0 ? 1 : 0;
            u = d.y, v = d.z, m = ax;
        } else if (ay >= az) {
            face = d.y < 0 ? 3 : 2;
            u = d.x, v = d.z, m = ay;
        } else {
            face = d.z < 0 ? 5 : 4;
            u = d.x, v = d.y, m = az;
        }
        const uint32_t cu = m > 0 && u > 0 ? 1u : 0u, cv = m > 0 && v > 0 ? 1u : 0u;
        key = d.x == d.x && d.y == d.y && d.z == d.z ? (uint32_t)face << 2 | cu << 1 | cv : 126u;
    }
    keys[slot] = key;
    vals[slot] = slot;
}

// keys of the deferred queries (ReflArgs::defer, RT_REFL_DEFER_SORT): each slot's frame position, so that
// refl_trace_long_kernel takes them in the frames' Morton order (nearby origins in a wave)
__global__ __launch_bounds__(BLOCK) void refl_defer_keys_kernel(ReflArgs A, int n, uint32_t* keys)
{
    int t = blockIdx.x * BLOCK + threadIdx.x;
    if (t < n)
        keys[t] = (uint32_t)(slot_pos(A, A.defer[t]) - A.c0);
}

// gen: one thread per sample slot of the chunk
// gen + trace: each sample slot's direction (path-keyed RNG: no draw depends on another
// sample, renderer.cpp:296-315) written to its record, then the sample's closest-hit query.
// One kernel, so that the record writes overlap the traversals.
__device__ __forceinline__ bool refl_gen(const KParams& P, const ReflArgs& A, int slot, v3& dir, unsigned& count)
{
    const int i = slot_sample(A, slot);
    const FrameRec& F = refl_frame(A, slot_pos(A, slot));
    SampleRec& S = A.sm[slot];
    // fused: a sample's direction and ray flag go to its 32-B RawHit (written by the trace
    // kernel, coalesced) and nothing to the 72-B record, which only shaded samples fill
    if (i >= F.nsamp) {
        if (!A.fused) {
            S.kind = 2;
            S.ray = 0;
            S.sh = 0;
            S.child = -1;
        }
        return false;
    }
    dir = refl_dir(F, i);
    if (!A.fused)
        st3(S.d, dir);
    if (i == 0)
        count = (unsigned)F.nsamp;   // reflection rays
    if (A.level > P.max_recursion_depth) {   // trace_ray's depth guard (renderer.cpp:1012-1013)
        if (A.fused) {
            A.res[slot] = make_float4(0.0f, 0.0f, 0.0f, __int_as_float(-1));
        } else {
            S.kind = 0;
            st3(S.fc, col(0.0f, 0.0f, 0.0f));
            S.ray = 0;
            S.sh = 0;
            S.child = -1;
        }
        return false;
    }
    if (!A.fused) {
        S.kind = 1;
        S.ray = 1;
    }
    return true;
}

#ifndef RT_REFL_G
#define RT_REFL_G 1   // lanes per reflection sample in refl_trace_kernel
#endif
#ifndef RT_OCC_REFL
#define RT_OCC_REFL 4   // waves per SIMD of the reflection trace / shadow / pass1 kernels (r04, the sound query:
                        // C5 689 vs 656 Mrays/s at 5 (31 spills), 691 at 3; r03: 4 -> 5 about -0.6%)
#endif
template <int G = 1>
__device__ __forceinline__ void refl_trace_one(const KParams& P, const ReflArgs& A, int slot, v3 dir, uint2* lv,
                                               uint32_t max_steps);

__global__ __launch_bounds__(BLOCK, RT_OCC_REFL) void refl_trace_kernel(KParams P_arg, ReflArgs A)
{
    // the parameters where the kernel received them (not a copy: passing the by-value argument to a
    // call made every lane copy it to scratch, r05: C5's shadow pass wrote ~90 GB per launch)
    const KParams& P = kernel_params();
    (void)P_arg;
    extern __shared__ uint2 lds_levels[];
    uint2* lv = lds_levels + threadIdx.x;
    constexpr int G = RT_REFL_G;   // lanes per sample (the launch has G threads per slot)
    const bool lead = G == 1 || (threadIdx.x & (G - 1)) == 0;
    int slot = (int)((blockIdx.x * BLOCK + threadIdx.x) / G);
    int nslot = (A.c1 - A.c0) * A.stride;
    unsigned count = 0;
    v3 dir = mk(0, 0, 0);
    bool ray = slot < nslot && refl_gen(P, A, slot, dir, count);
    wave_count_add(&P.counters[1], lead ? count : 0u);
    if (!ray) {
        if (A.fused && slot < nslot && lead) {   // no ray (pass1 skips it: bit 1 clear)
            RawHit H;
            H.t = H.u = H.v = 0.0f;
            H.k = -1;
            st3(H.d, dir);
            H.r = 0;
            A.hit[slot] = H;
        }
        return;
    }
    refl_trace_one<G>(P, A, slot, dir, lv, (uint32_t)A.max_steps);
}

// Lane refill for the reflection queries (ReflArgs::feed; Aila and Laine's persistent threads with
// dynamic ray fetch).  Most reflection queries end in a few steps and a few run long: with one query
// per lane, a wave ran to its longest lane (up to the deferral threshold) with ~15% of its lanes busy
// (RT_COUNT SIMD efficiency, profiles/r05/c5/work_counts_c5.log).  Here the waves are persistent: a
// lane whose query ended waits until threshold lanes of its wave wait, then each of them writes its
// result and takes the next sample slot (one atomic per wave), so that the wave keeps working on fresh
// queries while its long ones run on.  Per query the wide query is wbvh_closest's (the same state, reset
// per query, the same steps) and the record the certificate's; the queries it cannot certify (a stack
// overflow, a tie, a NaN ray) go to the defer list, which refl_trace_long_kernel runs as before (deep
// retry, octree walk).  The result per slot is refl_trace_one's, bit for bit.
#ifndef RT_OCC_FEED
#define RT_OCC_FEED 3   // waves per SIMD of refl_trace_feed_kernel (its persistent grid; r06, C5 ms per frame:
                        // 3 waves with a 26-entry stack 903-904, 4 / 20 entries 913-915, 2 / 32 912, 3 / 20 921-923,
                        // 5 / 16 1,077: the deeper stack defers fewer queries, more waves thrash the L1)
#endif
#ifndef RT_STACK_REFL_FEED
#define RT_STACK_REFL_FEED 26   // (160 KB / 3 blocks / 256 lanes / 8 B)
#endif
static_assert(RT_OCC_FEED * RT_STACK_REFL_FEED * 256 * 8 <= 160 * 1024, "the feed's stacks fit the CU's LDS");
constexpr int W_STACK_REFL_FEED = RT_STACK_REFL_FEED;
static_assert(W_STACK_REFL_FEED >= W_STACK, "the feed's stack");

struct ReflFeed {
    static constexpr bool on = true;
    bool busy = false;      // the lane holds a query (slot) not yet finished
    bool drained = false;   // (wave-uniform) every slot has been handed out
    int threshold;
    int slot = -1;
    int part = 0;        // (feed_parts, wave-uniform) eighths of the slots this wave has found exhausted
    unsigned count = 0;  // reflection rays of the lane's slots (refl_gen)
    const KParams* P;
    const ReflArgs* A;
    int nslot;

    // defer the lanes' slots (divergent lanes: one atomic per wave)
    __device__ __forceinline__ void defer() const
    {
        const uint64_t mk = __ballot(1);
        const int leader = __ffsll((unsigned long long)mk) - 1;
        uint32_t base = 0;
        if ((int)(threadIdx.x & 63) == leader)
            base = atomicAdd(A->defer_count, (unsigned)__popcll(mk));
        base = __shfl(base, leader);
        A->defer[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u))] = slot;
    }

    __device__ __forceinline__ void finish(int st, WHit& w, v3 o, v3 d)
    {
        busy = false;
        RawHit H;
        H.k = -1;
        H.t = -1.0f;
        H.u = 1.0f;
        H.v = 0.0f;
        bool r = false, ok = st == W_MISS;
        if (st == W_HIT) {
            // the certificate (wide_closest): the octree leaf holding the triangle passes the reference's
            // k-DOP test at t* (bvh.h:79-105)
            const uint4 M = ldg(P->wmeta + w.k);
            if (kdop_certifies(load_gnode(P->nodes + M.y), o, d, w.t)) {
                H.t = w.t;
                H.u = w.u;
                H.v = w.v;
                H.k = (int32_t)M.x;
                r = ok = true;
            }
        }
        if (!ok) {
            defer();
            return;
        }
        st3(H.d, d);
        H.r = (r ? 1 : 0) | (A->fused ? 2 : 0);
        A->hit[slot] = H;
    }

    // wave-uniform: the waiting lanes (want) take the next slots; true for a lane given a ray (hi, risk and
    // rsub stay the call's: INFINITY, none, 0; nob: the origin cones, ocone.hpp)
    __device__ __forceinline__ bool fetch(bool want, v3& o, v3& d, float& m, float&, const uint64_t*&, float&, bool& nob)
    {
        const uint64_t wb = __ballot(want);
        if (!wb)
            return false;
        const int leader = __ffsll((unsigned long long)wb) - 1;
        const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(wb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)wb, 0u));
        if (A->feed_parts) {
            // the slots in eighths, one ticket each: a wave starts on its XCD's eighth (workgroups go to the
            // 8 XCDs round robin), so that each XCD's L2 holds the nodes of one part of the frames' Morton
            // order, and moves on to the next eighths when its own is exhausted
            const int xcd = (int)(blockIdx.x & 7);
            int base = 0, lim = 0;
            for (;;) {
                if (part >= 8) {
                    drained = true;
                    return false;
                }
                const int x = (xcd + part) & 7;
                const int lo = (int)((long long)nslot * x / 8), hi = (int)((long long)nslot * (x + 1) / 8);
                int b = 0;
                if ((int)(threadIdx.x & 63) == leader)
                    b = (int)atomicAdd(A->feed_parts + x, (unsigned)__popcll(wb));
                b = __shfl(b, leader);
                if (lo + b < hi) {
                    base = lo + b;
                    lim = hi;
                    break;
                }
                part++;
            }
            drained = false;
            if (!want)
                return false;
            slot = base + rank;
            if (slot >= lim)
                return false;
        } else {
            int base = 0;
            if ((int)(threadIdx.x & 63) == leader)
                base = (int)atomicAdd(A->feed_ticket, (unsigned)__popcll(wb));
            base = __shfl(base, leader);
            drained = base + __popcll(wb) >= nslot;
            if (!want)
                return false;
            slot = base + rank;
            if (slot >= nslot)
                return false;
        }
        // the tickets in frame order (a frame's samples on adjacent lanes: one origin, coherent first
        // steps), whatever the slots' order
        if (A->perm)
            slot = A->perm[slot];
        else if (A->sample_major && A->feed_frame_order)
            slot = slot_of(*A, A->c0 + slot / A->stride, slot % A->stride);
        v3 dir = mk(0, 0, 0);
        unsigned c = 0;   // (refl_gen sets it for a frame's first sample: the frame's reflection rays)
        const bool gen = refl_gen(*P, *A, slot, dir, c);
        count += c;
        if (!gen) {
            if (A->fused) {   // no ray (pass1 skips it: bit 1 clear)
                RawHit H;
                H.t = H.u = H.v = 0.0f;
                H.k = -1;
                st3(H.d, dir);
                H.r = 0;
                A->hit[slot] = H;
            }
            return false;
        }
        const FrameRec& F = refl_frame(*A, slot_pos(*A, slot));
        o = ld3(F.ro);
        d = dir;
        if (ray_is_nan(o, d) || !(P->wnodes && P->nnodes > 0)) {   // (refl_trace_one's octree path)
            defer();
            return false;
        }
        const float om = fmaxf(fabsf(o.x), fmaxf(fabsf(o.y), fabsf(o.z)));
        m = 0x1p-16f * (om + P->scene_scale);
        nob = ocone_skip(P->ocone, o, d, W_QS_CLOSEST);
        busy = true;
        return true;
    }
};

__global__ __launch_bounds__(BLOCK, RT_OCC_FEED) void refl_trace_feed_kernel(KParams P_arg, ReflArgs A)
{
    const KParams& P = kernel_params();
    (void)P_arg;
    extern __shared__ uint2 lds_levels[];
    uint2* lv = lds_levels + threadIdx.x;
    ReflFeed feed;
    feed.threshold = A.feed;
    feed.P = &P;
    feed.A = &A;
    feed.nslot = (A.c1 - A.c0) * A.stride;
    // its one-lane queries take the CU's LDS at RT_OCC_FEED blocks (3 blocks per CU: 52 KB, 26 entries per
    // lane): fewer overflow into the defer list
    WStackLdsN<W_STACK_REFL_FEED> stk{lv};
    WHit w;
#if RT_COUNT
    uint32_t wk[4] = {0, 0, 0, 0};   // (the lane's queries' node visits and triangle tests)
#else
    uint32_t* wk = nullptr;
#endif
    wbvh_closest<WStackLdsN<W_STACK_REFL_FEED>, 1, ReflFeed>(P.wnodes, P.wtris, mk(0, 0, 0), mk(1, 0, 0), 0.0f, stk, w,
                                                             wk, INFINITY, true, W_QS_CLOSEST, nullptr, 0, 0.0f, 0u,
                                                             &feed);
    wave_count_add(&P.counters[1], feed.count);
#if RT_COUNT
    if (P.counters) {
        atomicAdd(&P.counters[10], (unsigned long long)wk[0]);
        atomicAdd(&P.counters[11], (unsigned long long)wk[1]);
    }
#endif
}

#ifndef RT_REFL_LONG_QUEUE
#define RT_REFL_LONG_QUEUE 1   // refl_trace_long_kernel: waves take batches from a ticket (0: grid stride)
#endif
#ifndef RT_REFL_LONG_G
#define RT_REFL_LONG_G 8   // lanes per deferred reflection query (refl_trace_long_kernel; r06: with lane refill only
                           // the overflowed / uncertified queries come here, the longest: C5 1,105 -> 1,078 ms at 8)
#endif
// The queries refl_trace_kernel deferred (ReflArgs::defer): traced to the end in waves of long
// queries only, each by a lane group of RT_REFL_LONG_G lanes (wbvh_closest<.., G>: one stack shared
// by steals, so that the few longest queries do not hold the wave alone).
__global__ __launch_bounds__(BLOCK, RT_OCC_REFL) void refl_trace_long_kernel(KParams P_arg, ReflArgs A)
{
    constexpr int G = RT_REFL_LONG_G;
    static_assert(G == 1 || G == 2 || G == 4 || G == 8, "lane groups of 1, 2, 4 or 8");
    // the parameters where the kernel received them (not a copy: passing the by-value argument to a
    // call made every lane copy it to scratch, r05: C5's shadow pass wrote ~90 GB per launch)
    const KParams& P = kernel_params();
    (void)P_arg;
    extern __shared__ uint2 lds_levels[];
    uint2* lv = lds_levels + threadIdx.x;
    const int n = (int)ldg(A.defer_count);
#if RT_REFL_LONG_QUEUE
    // a wave takes the next 64 / G queries from a ticket (defer_count[1], zeroed with the count) when it
    // is done with its last ones: the waves' batches differ in length, a fixed grid stride left the
    // kernel to its slowest wave's sum of batches
    const int lane = (int)(threadIdx.x & 63);
    for (;;) {
        int base = 0;
        if (lane == 0)
            base = (int)atomicAdd(A.defer_count + 1, (unsigned)(64 / G));
        base = __builtin_amdgcn_readfirstlane(base);
        if (base >= n)
            break;
        const int i = base + lane / G;   // query i: lanes G i .. G i + G - 1 of the batch
        if (i >= n)
            continue;
#else
    // query i is held by lanes G i .. G i + G - 1 of the grid (whole groups inside one wave)
    for (int i = (int)((blockIdx.x * BLOCK + threadIdx.x) / G); i < n; i += (int)(gridDim.x * BLOCK / G)) {
#endif
        const int slot = A.defer[i];
        unsigned count = 0;
        v3 dir = mk(0, 0, 0);
        if (refl_gen(P, A, slot, dir, count))   // (the same direction: path-keyed RNG; every lane of the group)
            refl_trace_one<G>(P, A, slot, dir, lv, 0u);
    }
}

// One reflection sample's closest hit into A.hit[slot]; a query past max_steps (> 0) goes to the
// deferred list instead.
// In line, with the octree fallback behind the out-of-line octree_query_call (results by value): a
// ray record or hit record whose address reached a call lived in scratch for every sample (r05).
// G > 1 (refl_trace_long_kernel): the G lanes of a group hold the same slot and run the query
// together; the group's first lane writes the result.
template <int G>
__device__ __forceinline__ void refl_trace_one(const KParams& P, const ReflArgs& A, int slot, v3 dir, uint2* lv,
                                               uint32_t max_steps)
{
    const FrameRec& F = refl_frame(A, slot_pos(A, slot));
    const v3 ro = ld3(F.ro);
    THit h;
    bool r;
    bool longq = false;
    if (P.wnodes && P.nnodes > 0 && !ray_is_nan(ro, dir) && wide_closest<G>(P, ro, dir, h, r, lv, nullptr, max_steps, &longq))
        ;   // certified by the wide BVH
    else if (longq) {
        // the groups deferring now (their first lanes): one atomic per wave
        const bool lead = G == 1 || (threadIdx.x & (G - 1)) == 0;
        const uint64_t m = __ballot(lead);
        const int leader = __ffsll((unsigned long long)m) - 1;
        uint32_t base = 0;
        if ((int)(threadIdx.x & 63) == leader)
            base = atomicAdd(A.defer_count, (unsigned)__popcll(m));
        base = __shfl(base, leader);
        if (lead)
            A.defer[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = slot;
        return;
    } else {
        const bool seg = P.seg_scale > 0.0f && P.seg_oct;
        // (seg: nothing behind the origin can be hit, t >= 0)
        const float lo = seg ? -seg_margin(P, make_ray(P, ro, dir)) : 0.0f;
        const OctQ q = octree_query<true>(P, ro, dir, lo, INFINITY, seg, lv);
        h = q.h;
        r = q.r;
    }
    RawHit H;
    H.t = h.t;
    H.u = h.u;
    H.v = h.v;
    H.k = h.k;
    st3(H.d, dir);
    H.r = (r ? 1 : 0) | (A.fused ? 2 : 0);
    if (G == 1 || (threadIdx.x & (G - 1)) == 0)
        A.hit[slot] = H;
}

// append slot to the shadow list from (possibly divergent) lanes: one atomic per wave
__device__ __forceinline__ void list_append(const ReflArgs& A, int slot)
{
    const uint64_t m = __ballot(1);   // the lanes appending now
    const int leader = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if ((int)(threadIdx.x & 63) == leader)
        base = atomicAdd(A.list_count, (unsigned)__popcll(m));
    base = __shfl(base, leader);
    A.list[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = slot;
}

// pass1: per frame, the samples' trace_ray up to the shadow query, in sample order
__global__ __launch_bounds__(BLOCK, RT_OCC_REFL) void refl_pass1_kernel(KParams P_arg, ReflArgs A)
{
    // the parameters where the kernel received them (not a copy: passing the by-value argument to a
    // call made every lane copy it to scratch, r05: C5's shadow pass wrote ~90 GB per launch)
    const KParams& P = kernel_params();
    (void)P_arg;
    int p = A.c0 + blockIdx.x * BLOCK + threadIdx.x;
    unsigned nshadow = 0;
    if (p < A.c1) {
        const FrameRec& F = refl_frame(A, p);
        v3 ro = ld3(F.ro);
        Rec rhi = rec_fresh();   // reflection_hit_info, renderer.cpp:286
        for (int i = 0; i < F.nsamp; i++) {
            int slot = slot_of(A, p, i);
            SampleRec& S = A.sm[slot];
            const RawHit H = A.hit[slot];
            if (A.fused ? !(H.r & 2) : !S.ray)
                continue;   // depth limit: trace_ray returns before touching the record
            const v3 d = A.fused ? ld3(H.d) : ld3(S.d);
            THit h;
            h.t = H.t;
            h.u = H.u;
            h.v = H.v;
            h.k = H.k;
            Rec local = rec_fresh();
            int s = -1;
            bvh_record(P, h, (H.r & 1) != 0, local, rhi, s);
            shapes_closest(P, ro, d, local, rhi, s);
            if (!A.fused) {
                S.sh = 0;
                S.child = -1;
            }
            if (rhi.t > 0.1f) {
                v3 ip;
                c3 fc = shade_lit(P, ro, d, rhi, ip);   // may normal-map rhi.normal (persists)
                if (A.fused)
                    list_append(A, slot);   // a shaded sample: its shadow query (and spawn)
                S.kind = 1;
                st3(S.fc, fc);
                st3(S.ip, ip);
                st3(S.nrm, rhi.normal);
                S.mat = rhi.mat;
                const float* m = mat_of(P, rhi.mat);
                S.crough = m[12] > 0.0f ? frame_roughness(P, rhi, m) : 0.0f;
                if (P.compute_shadows)
                    nshadow++;
            } else {
                float a;
                const c3 mc = miss_color(P, d, a);
                if (A.fused) {
                    A.res[slot] = make_float4(mc.r, mc.g, mc.b, __int_as_float(-1));
                } else {
                    S.kind = 0;
                    st3(S.fc, mc);
                }
            }
        }
    }
    wave_count_add(&P.counters[0], nshadow);
}

// list: the shaded samples (the only ones with a shadow query), compacted so that
// the shadow pass runs on full waves (one atomic per wave)
__global__ __launch_bounds__(BLOCK) void refl_list_kernel(KParams P, ReflArgs A)
{
    int slot = blockIdx.x * BLOCK + threadIdx.x;
    int nslot = (A.c1 - A.c0) * A.stride;
    bool need = slot < nslot && A.sm[slot].ray && A.sm[slot].kind == 1;
    if (slot < nslot && !need)
        A.sm[slot].sh = 0;
    uint64_t m = __ballot(need);
    if (!m)
        return;
    uint32_t base = 0;
    int leader = __ffsll((unsigned long long)m) - 1;
    if ((threadIdx.x & 63) == leader)
        base = atomicAdd(A.list_count, (unsigned)__popcll(m));
    base = __shfl(base, leader);
    if (need)
        A.list[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = slot;
}

__device__ __forceinline__ int spawn_sample(const KParams& P, const ReflArgs& A, int slot, SampleRec& S, bool sh);

// a sample's shadow decided: its record, and (fused) the child frame it spawns and the colour it returns
__device__ __forceinline__ void refl_shadow_done(const KParams& P, const ReflArgs& A, int slot, bool sh)
{
    SampleRec& S = A.sm[slot];
    S.sh = sh ? 1 : 0;
    if (A.fused) {
        // the colour this sample returns (resolve, below): its child frame's, or its own finished shade
        const int child = spawn_sample(P, A, slot, S, sh);
        c3 c = col(0.0f, 0.0f, 0.0f);
        if (child < 0) {
            const float* m = mat_of(P, S.mat);
            c = shade_finish(P, shade_shadow_emit(P, ldc(S.fc), m, sh), m, col(0, 0, 0));
        }
        A.res[slot] = make_float4(c.r, c.g, c.b, __int_as_float(child));
    }
}

// shadow: is_shadowed (renderer.cpp:340-402) for every shaded sample (via the list)
#ifndef RT_REFL_SHADOW_CALL
#define RT_REFL_SHADOW_CALL 1   // the shadow pass's octree fallback out of line (octree_query_call)
#endif
__global__ __launch_bounds__(BLOCK, RT_OCC_REFL) void refl_shadow_kernel(KParams P_arg, ReflArgs A)
{
    // the parameters where the kernel received them (not a copy: passing the by-value argument to a
    // call made every lane copy it to scratch, r05: C5's shadow pass wrote ~90 GB per launch)
    const KParams& P = kernel_params();
    (void)P_arg;
    extern __shared__ uint2 lds_levels[];
    uint2* lv = lds_levels + threadIdx.x;
    unsigned t = blockIdx.x * BLOCK + threadIdx.x;
    if (t >= *A.list_count)
        return;
    const int slot = A.list[t];
    SampleRec& S = A.sm[slot];
    v3 light = mk(P.light[0], P.light[1], P.light[2]);
    refl_shadow_done(P, A, slot, is_shadowed<false, 1, RT_REFL_SHADOW_CALL != 0>(P, ld3(S.ip), ld3(S.nrm), light, lv));
}

// Lane refill for the shadow pass (ReflArgs::shadow_feed; the reflection queries' ReflFeed, above): most
// shadow segments end in a few steps and a few run long (lane utilisation ~0.2 with one segment per
// lane).  Per list entry the query is is_shadowed's wide part (wide_shadow: the segment [0, hi], no ties,
// the light's risk words when they hold for the ray) and the decision its; the entries it does not decide
// (a stack overflow, an uncertified hit, a NaN ray, no segment query) go to the deferred list, which
// refl_shadow_kernel runs as before (deep retry, octree segment query).  Each entry's result is
// refl_shadow_kernel's, bit for bit.
struct ShadowFeed {
    static constexpr bool on = true;
    bool busy = false;
    bool drained = false;
    int threshold;
    int slot = -1;
    const KParams* P;
    const ReflArgs* A;
    int nlist;
    v3 light;

    __device__ __forceinline__ void defer() const
    {
        const uint64_t mk = __ballot(1);
        const int leader = __ffsll((unsigned long long)mk) - 1;
        uint32_t base = 0;
        if ((int)(threadIdx.x & 63) == leader)
            base = atomicAdd(A->sdefer_count, (unsigned)__popcll(mk));
        base = __shfl(base, leader);
        A->sdefer[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(mk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk, 0u))] = slot;
    }

    __device__ __forceinline__ void finish(int st, WHit& w, v3 o, v3 d)
    {
        busy = false;
        bool sh = false;
        if (st == W_HIT) {
            // wide_shadow: a certified minimum hit t* <= hi is the reference's record t
            if (!kdop_certifies(load_gnode(P->nodes + ldg(P->wmeta + w.k).y), o, d, w.t)) {
                defer();
                return;
            }
            const v3 p = ld3(A->sm[slot].ip);
            const v3 q = o + d * w.t;
            sh = length2(p - q) < length2(p - light);
        } else if (st != W_MISS) {   // (a miss: lit)
            defer();
            return;
        }
        refl_shadow_done(*P, *A, slot, sh);
    }

    __device__ __forceinline__ bool fetch(bool want, v3& o, v3& d, float& m, float& hi, const uint64_t*& risk, float& rsub,
                                          bool&)
    {
        const uint64_t wb = __ballot(want);
        if (!wb)
            return false;
        const int leader = __ffsll((unsigned long long)wb) - 1;
        int base = 0;
        if ((int)(threadIdx.x & 63) == leader)
            base = (int)atomicAdd(A->shadow_ticket, (unsigned)__popcll(wb));
        base = __shfl(base, leader);
        drained = base + __popcll(wb) >= nlist;
        if (!want)
            return false;
        const int t = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(wb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)wb, 0u));
        if (t >= nlist)
            return false;
        slot = A->list[t];
        if (!P->compute_shadows) {   // (is_shadowed: lit)
            refl_shadow_done(*P, *A, slot, false);
            return false;
        }
        const SampleRec& S = A->sm[slot];
        const v3 p = ld3(S.ip), n = ld3(S.nrm);
        o = p + n * 1.0e-4f;
        d = normalize(light - p);
        if (!(P->enable_bvh && P->seg_scale > 0.0f && P->wnodes && P->nnodes > 0)) {
            defer();
            return false;
        }
        // is_shadowed's segment end and risk words, the same expressions
        const TRay R0 = make_ray(*P, o, d);
        const float ms = seg_margin(*P, R0);
        const float nl = fabsf(n.x) + fabsf(n.y) + fabsf(n.z);
        hi = (sqrtf(length2(p - light)) + 1.0e-4f * nl) * (1.0f + 0x1p-10f) + ms;
        if (R0.nan) {
            defer();
            return false;
        }
        const bool lr = P->wrisk && hi <= P->risk_G && nl <= P->risk_nl;
        risk = lr ? P->wrisk : nullptr;
        rsub = lr ? wrisk_sub(W_QS_SHADOW, hi, P->risk_nu) : 0.0f;
        const float om = fmaxf(fabsf(o.x), fmaxf(fabsf(o.y), fabsf(o.z)));
        m = 0x1p-16f * (om + P->scene_scale);
        busy = true;
        return true;
    }
};

__global__ __launch_bounds__(BLOCK, RT_OCC_REFL) void refl_shadow_feed_kernel(KParams P_arg, ReflArgs A)
{
    const KParams& P = kernel_params();
    (void)P_arg;
    extern __shared__ uint2 lds_levels[];
    uint2* lv = lds_levels + threadIdx.x;
    ShadowFeed feed;
    feed.threshold = A.shadow_feed;
    feed.P = &P;
    feed.A = &A;
    feed.nlist = (int)*A.list_count;
    feed.light = mk(P.light[0], P.light[1], P.light[2]);
    WStackLdsN<W_STACK_REFL_FEED> stk{lv};
    WHit w;
    wbvh_closest<WStackLdsN<W_STACK_REFL_FEED>, 1, ShadowFeed>(P.wnodes, P.wtris, mk(0, 0, 0), mk(1, 0, 0), 0.0f, stk, w,
                                                               nullptr, INFINITY, false, W_QS_SHADOW, nullptr, 1, 0.0f, 0u,
                                                               &feed);
}

// a shaded sample with a reflective material becomes a frame of the next level (its
// compute_reflection call); the frame's index goes into S.child
__device__ __forceinline__ int spawn_sample(const KParams& P, const ReflArgs& A, int slot, SampleRec& S, bool sh)
{
    const float* m = mat_of(P, S.mat);
    if (!(m[12] > 0.0f))
        return -1;
    const int i = slot_sample(A, slot);
    const FrameRec& F = refl_frame(A, slot_pos(A, slot));
    unsigned idx = atomicAdd(A.child_count, 1u);
    c3 dfc = shade_shadow_emit(P, ldc(S.fc), m, sh);
    make_frame(P, A.child_fr[idx], ld3(S.ip), ld3(S.nrm), A.fused ? ld3(A.hit[slot].d) : ld3(S.d), dfc, S.crough, S.mat,
               child_key(F.key, (uint32_t)i), -1);
    S.child = (int)idx;
    return (int)idx;
}

// spawn: reflective hits become frames of the next level (A.fused == 0; else the shadow pass)
__global__ __launch_bounds__(BLOCK) void refl_spawn_kernel(KParams P_arg, ReflArgs A)
{
    // the parameters where the kernel received them (not a copy: passing the by-value argument to a
    // call made every lane copy it to scratch, r05: C5's shadow pass wrote ~90 GB per launch)
    const KParams& P = kernel_params();
    (void)P_arg;
    int slot = blockIdx.x * BLOCK + threadIdx.x;
    int nslot = (A.c1 - A.c0) * A.stride;
    if (slot >= nslot)
        return;
    SampleRec& S = A.sm[slot];
    S.child = -1;
    if (!S.ray || S.kind != 1)
        return;
    spawn_sample(P, A, slot, S, S.sh != 0);
}

// resolve: compute_reflection's sum in sample order, then the frame's hit colour
__global__ __launch_bounds__(BLOCK) void refl_resolve_kernel(KParams P_arg, ReflArgs A)
{
    // the parameters where the kernel received them (not a copy: passing the by-value argument to a
    // call made every lane copy it to scratch, r05: C5's shadow pass wrote ~90 GB per launch)
    const KParams& P = kernel_params();
    (void)P_arg;
    int p = A.c0 + blockIdx.x * BLOCK + threadIdx.x;
    if (p >= A.c1)
        return;
    const int f = A.order[p];
    const FrameRec& F = refl_frame(A, p);
    c3 total = col(0.0f, 0.0f, 0.0f);
    for (int i = 0; i < F.nsamp; i++) {
        const int slot = slot_of(A, p, i);
        c3 ret;
        if (A.fused) {   // 16 B per sample instead of its 72-B record
            const float4 r = A.res[slot];
            const int child = __float_as_int(r.w);
            ret = child >= 0 ? ldc(A.child_ret + 3 * (size_t)child) : col(r.x, r.y, r.z);
            total = total + ret;
            continue;
        }
        const SampleRec& S = A.sm[slot];
        if (S.kind == 0)
            ret = ldc(S.fc);
        else if (S.child >= 0)
            ret = ldc(A.child_ret + 3 * (size_t)S.child);
        else {
            const float* m = mat_of(P, S.mat);
            ret = shade_finish(P, shade_shadow_emit(P, ldc(S.fc), m, S.sh != 0), m, col(0, 0, 0));
        }
        total = total + ret;
    }
    const float* m = mat_of(P, F.mat);
    float sc = (float)F.nsamp, rf = m[12];
    c3 R = (total / col(sc, sc, sc)) * col(rf, rf, rf);
    c3 c = shade_finish(P, ldc(F.fc), m, R);
    if (A.level == 1) {
        size_t o = (size_t)F.parent;
        if (P.argb) P.argb[o] = color_to_argb(c);
        if (P.rgba) P.rgba[o] = make_float4(c.r, c.g, c.b, 1.0f);
    } else
        st3(A.ret + 3 * (size_t)f, c);
}

// ===========================================================================
// Renderer::raster_trace (renderer.cpp:869-1006): hybrid rasterisation of the
// primary visibility, then trace_triangle's shading (shadows / reflections through
// the octree).  The reference's OpenMP triangle loop races on the z-buffer; the
// defined result is the sequential one (triangles and their clipped pieces in
// order, strict z-test), which the per-pixel 64-bit atomicMin of
// (order-preserving z, piece index) reproduces: pieces are numbered in
// (triangle, piece) order, so among equal z the first one wins.
// ===========================================================================
struct V4 {
    float x, y, z, w;
};
__device__ __forceinline__ V4 v4(float x, float y, float z, float w) { V4 r = {x, y, z, w}; return r; }
__device__ __forceinline__ V4 v4add(V4 a, V4 b) { return v4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }   // vec.cpp:123
__device__ __forceinline__ V4 v4sub(V4 a, V4 b) { return v4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }   // vec.cpp:128
__device__ __forceinline__ V4 v4mul(float t, V4 u) { return v4(u.x * t, u.y * t, u.z * t, u.w * t); }       // vec.cpp:133-141
__device__ __forceinline__ float v4c(V4 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
// Transform::operator()(vec4), mat.cpp:118-131
__device__ __forceinline__ V4 xform4(const float* m, V4 v)
{
    return v4(m[0] * v.x + m[1] * v.y + m[2] * v.z + m[3] * v.w, m[4] * v.x + m[5] * v.y + m[6] * v.z + m[7] * v.w,
              m[8] * v.x + m[9] * v.y + m[10] * v.z + m[11] * v.w, m[12] * v.x + m[13] * v.y + m[14] * v.z + m[15] * v.w);
}
// Renderer::matrix_transform_z, renderer.cpp:856-867 (a division, not a reciprocal)
__device__ __forceinline__ float xform_z(const float* m, v3 p)
{
    float zt = m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11];
    float wt = m[12] * p.x + m[13] * p.y + m[14] * p.z + m[15];
    if (wt == 1.0f)
        return zt;
    return zt / wt;
}

struct Tri4 {   // Triangle4, triangle.h:24-40
    V4 a, b, c;
    v3 tu, tv;
};

constexpr int CLIP_MAX = 12;   // std::array<Triangle4, 12>: more pieces are UB in the reference, dropped here

__device__ __forceinline__ bool in_half(V4 p, int i, int sgn) { return sgn > 0 ? v4c(p, i) < p.w : v4c(p, i) > -p.w; }

// clip_triangles_to_plane<i, sgn>, renderer.cpp:669-850 (in may alias out when n == 1)
__device__ int clip_plane(const Tri4* in, int n, Tri4* out, int i, int sgn)
{
    int k = 0;
    const float fs = (float)sgn;
    for (int t = 0; t < n; t++) {
        const Tri4 T = in[t];
        bool ia = in_half(T.a, i, sgn), ib = in_half(T.b, i, sgn), ic = in_half(T.c, i, sgn);
        int cnt = (int)ia + (int)ib + (int)ic;
        if (cnt == 3) {
            if (k < CLIP_MAX) out[k] = T;
            k++;
        } else if (cnt == 1) {
            V4 p0 = ia ? T.a : (ib ? T.b : T.c), p1 = ia ? T.b : (ib ? T.c : T.a), p2 = ia ? T.c : (ib ? T.a : T.b);
            float u0 = ia ? T.tu.x : (ib ? T.tu.y : T.tu.z), u1 = ia ? T.tu.y : (ib ? T.tu.z : T.tu.x),
                  u2 = ia ? T.tu.z : (ib ? T.tu.x : T.tu.y);
            float w0 = ia ? T.tv.x : (ib ? T.tv.y : T.tv.z), w1 = ia ? T.tv.y : (ib ? T.tv.z : T.tv.x),
                  w2 = ia ? T.tv.z : (ib ? T.tv.x : T.tv.y);
            float d0 = v4c(p0, i) - p0.w * fs, d1 = v4c(p1, i) - p1.w * fs, d2 = v4c(p2, i) - p2.w * fs;
            float t1 = d1 / (d1 - d0), t2 = d2 / (d2 - d0);
            Tri4 R;
            R.a = p0;
            R.b = v4add(p1, v4mul(t1 - 0.0f, v4sub(p0, p1)));
            R.c = v4add(p2, v4mul(t2 - 0.0f, v4sub(p0, p2)));
            R.tu = mk(u0, u1 + (t1 - 0.0f) * (u0 - u1), u2 + (t2 - 0.0f) * (u0 - u2));
            R.tv = mk(w0, w1 + (t1 - 0.0f) * (w0 - w1), w2 + (t2 - 0.0f) * (w0 - w2));
            if (k < CLIP_MAX) out[k] = R;
            k++;
        } else if (cnt == 2) {
            V4 q0 = !ia ? T.a : (!ib ? T.b : T.c), q1 = !ia ? T.b : (!ib ? T.c : T.a), q2 = !ia ? T.c : (!ib ? T.a : T.b);
            float u0 = !ia ? T.tu.y : (!ib ? T.tu.z : T.tu.x), u1 = !ia ? T.tu.z : (!ib ? T.tu.x : T.tu.y),
                  u2 = !ia ? T.tu.x : (!ib ? T.tu.y : T.tu.z);
            float w0 = !ia ? T.tv.y : (!ib ? T.tv.z : T.tv.x), w1 = !ia ? T.tv.z : (!ib ? T.tv.x : T.tv.y),
                  w2 = !ia ? T.tv.x : (!ib ? T.tv.y : T.tv.z);
            float e1 = v4c(q1, i) - q1.w * fs, e2 = v4c(q2, i) - q2.w * fs, e0 = v4c(q0, i) - q0.w * fs;
            float t1 = e0 / (e0 - e1), t2 = e0 / (e0 - e2);
            V4 P1 = v4add(q0, v4mul(t1 - 0.0f, v4sub(q1, q0)));
            V4 P2 = v4add(q0, v4mul(t2 - 0.0f, v4sub(q2, q0)));
            Tri4 R1, R2;
            R1.a = q1; R1.b = q2; R1.c = P2;
            R1.tu = mk(u0, u1, u2 + (t2 - 0.0f) * (u1 - u2));
            R1.tv = mk(w0, w1, w2 + (t2 - 0.0f) * (w1 - w2));
            R2.a = q1; R2.b = P2; R2.c = P1;
            R2.tu = mk(u0, u2 + (t2 - 0.0f) * (u1 - u2), u2 + (t1 - 0.0f) * (u0 - u2));
            R2.tv = mk(w0, w2 + (t2 - 0.0f) * (w1 - w2), w2 + (t1 - 0.0f) * (w0 - w2));
            if (k < CLIP_MAX) out[k] = R1;
            k++;
            if (k < CLIP_MAX) out[k] = R2;
            k++;
        }
    }
    return k < CLIP_MAX ? k : CLIP_MAX;
}

// _world_to_camera_mat(triangle), perspective_projection(vec4(vertex)), clip_triangle (renderer.cpp:833-854)
__device__ int clip_triangle(const KParams& P, const RasterArgs& A, int64_t t, Tri4* buf0, Tri4* buf1, const Tri4** res)
{
    const float* q = A.tri9 + 9 * t;
    v3 ca = xform_point(A.w2c, mk(q[0], q[1], q[2]));
    v3 cb = xform_point(A.w2c, mk(q[3], q[4], q[5]));
    v3 cc = xform_point(A.w2c, mk(q[6], q[7], q[8]));
    buf0[0].a = xform4(A.proj, v4(ca.x, ca.y, ca.z, 1.0f));
    buf0[0].b = xform4(A.proj, v4(cb.x, cb.y, cb.z, 1.0f));
    buf0[0].c = xform4(A.proj, v4(cc.x, cc.y, cc.z, 1.0f));
    if (P.tri_uv) {
        const float* uv = P.tri_uv + 6 * t;
        buf0[0].tu = mk(uv[0], uv[1], uv[2]);
        buf0[0].tv = mk(uv[3], uv[4], uv[5]);
    } else {
        buf0[0].tu = mk(-1, -1, -1);
        buf0[0].tv = mk(-1, -1, -1);
    }
    int n = 1;
    *res = buf0;
    if (A.clipping) {
        n = clip_plane(buf0, n, buf0, 0, 1);
        n = clip_plane(buf0, n, buf1, 0, -1);
        n = clip_plane(buf1, n, buf0, 1, 1);
        n = clip_plane(buf0, n, buf1, 1, -1);
        n = clip_plane(buf1, n, buf0, 2, 1);
        n = clip_plane(buf0, n, buf1, 2, -1);
        *res = buf1;
    }
    return n;
}

__global__ __launch_bounds__(BLOCK) void raster_count_kernel(KParams P, RasterArgs A)
{
    int64_t t = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (t >= A.ntri)
        return;
    Tri4 b0[CLIP_MAX], b1[CLIP_MAX];
    const Tri4* res;
    A.count[t] = clip_triangle(P, A, t, b0, b1, &res);
}

// (int)(double), x86 cvttsd2si semantics: INT_MIN out of range / NaN
__device__ __forceinline__ int d2i(double d) { return (d > -2147483649.0 && d < 2147483648.0) ? (int)d : INT_MIN; }

__global__ __launch_bounds__(BLOCK) void raster_write_kernel(KParams P, RasterArgs A)
{
    int64_t t = (int64_t)blockIdx.x * BLOCK + threadIdx.x;
    if (t >= A.ntri)
        return;
    Tri4 b0[CLIP_MAX], b1[CLIP_MAX];
    const Tri4* res;
    int n = clip_triangle(P, A, t, b0, b1, &res);
    for (int k = 0; k < n; k++) {
        const Tri4& Q = res[k];
        int idx = A.offset[t] + k;
        RasterPiece& R = A.pieces[idx];
        // Triangle(Triangle4), triangle.cpp:12-23
        float iaw = 1.0f / Q.a.w, ibw = 1.0f / Q.b.w, icw = 1.0f / Q.c.w;
        v3 a = mk(Q.a.x * iaw, Q.a.y * iaw, Q.a.z * iaw);
        v3 b = mk(Q.b.x * ibw, Q.b.y * ibw, Q.b.z * ibw);
        v3 c = mk(Q.c.x * icw, Q.c.y * icw, Q.c.z * icw);
        st3(R.na, a);
        st3(R.nb, b);
        st3(R.nc, c);
        v3 pa = xform_point(P.proj_inv, a), pb = xform_point(P.proj_inv, b), pc = xform_point(P.proj_inv, c);
        st3(R.wa, xform_point(P.cam_to_world, pa));
        st3(R.wb, xform_point(P.cam_to_world, pb));
        st3(R.wc, xform_point(P.cam_to_world, pc));
        R.inv_area = 1 / ((b.x - a.x) * (c.y - a.y) - (b.y - a.y) * (c.x - a.x));
        float mnx = smin(a.x, smin(b.x, c.x)), mny = smin(a.y, smin(b.y, c.y));
        float mxx = smax(a.x, smax(b.x, c.x)), mxy = smax(a.y, smax(b.y, c.y));
        int x0 = d2i((double)(mnx + 1) * 0.5 * P.rw), y0 = d2i((double)(mny + 1) * 0.5 * P.rh);
        int x1 = d2i((double)(mxx + 1) * 0.5 * P.rw), y1 = d2i((double)(mxy + 1) * 0.5 * P.rh);
        R.x0 = x0 > 0 ? x0 : 0;
        R.y0 = y0 > 0 ? y0 : 0;
        R.x1 = P.rw - 1 < x1 ? P.rw - 1 : x1;
        R.y1 = P.rh - 1 < y1 ? P.rh - 1 : y1;
        R.za = xform_z(P.cam_to_world, pa);
        R.zb = xform_z(P.cam_to_world, pb);
        R.zc = xform_z(P.cam_to_world, pc);
        R.tri = (int32_t)t;
        float* uv = A.piece_uv + 6 * (size_t)idx;
        uv[0] = Q.tu.x; uv[1] = Q.tu.y; uv[2] = Q.tu.z;
        uv[3] = Q.tv.x; uv[4] = Q.tv.y; uv[5] = Q.tv.z;
    }
}

// Triangle::edge_function, triangle.h:65-68
__device__ __forceinline__ float edge_fn(float px, float py, v3 a, v3 b)
{
    return (b.x - a.x) * (py - a.y) - (b.y - a.y) * (px - a.x);
}

// launch-local row of a global row (-1: another rank's band)
__device__ __forceinline__ int local_row(const KParams& P, int py)
{
    int band = py / P.band_rows;
    if (P.band_inv) {
        const int lb = ldg(P.band_inv + band);
        return lb < 0 ? -1 : lb * P.band_rows + (py - band * P.band_rows);
    }
    if (band % P.nranks != P.rank)
        return -1;
    return (band / P.nranks) * P.band_rows + (py - band * P.band_rows);
}

__device__ __forceinline__ uint32_t z_order(float z)
{
    if (z == 0.0f)
        z = 0.0f;   // -0 == +0 in the reference's z-test
    uint32_t u = __float_as_uint(z);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

constexpr int RASTER_BIG = 2048;   // bounding-box pixels above which a piece gets a workgroup

// raster_trace's loops over rows y_first, y_first + ystep, .. of one piece's bounding
// box: every covered sample's candidate goes into the z-key buffer.  The sample
// coordinates accumulate exactly as the reference's loops do (iy += hs per row from
// y0, ix += ws per column from x0).
__device__ void raster_rows(const KParams& P, const RasterArgs& A, int idx, int y_first, int ystep)
{
    const RasterPiece& R = A.pieces[idx];
    v3 a = ld3(R.na), b = ld3(R.nb), c = ld3(R.nc);
    const float inv_area = R.inv_area, za = R.za, zb = R.zb, zc = R.zc;
    const int x0 = R.x0, x1 = R.x1, y0 = R.y0, y1 = R.y1;
    const float hs = 1.0f / P.rh * 2, ws = 1.0f / P.rw * 2;
    float iy = y0 * hs - 1;
    int yc = y0;
    for (int py = y_first; py <= y1; py += ystep) {
        for (; yc < py; yc++) iy += hs;
        int lr = local_row(P, py);
        if (lr < 0)
            continue;
        unsigned long long* zrow = A.zkey + (size_t)lr * P.rw;
        float ix = x0 * ws - 1;
        for (int px = x0; px <= x1; px++, ix += ws) {
            float sx = ix + ws * 0.5f, sy = iy + hs * 0.5f;
            float u = edge_fn(sx, sy, c, a);
            if (u < 0) continue;
            float v = edge_fn(sx, sy, a, b);
            if (v < 0) continue;
            float w = edge_fn(sx, sy, b, c);
            if (w < 0) continue;
            u *= inv_area;
            v *= inv_area;
            w *= inv_area;
            float z = -1 / (1 / za * w + 1 / zb * u + 1 / zc * v);
            if (!(z < INFINITY))
                continue;   // NaN / +inf never pass the z-test against the INFINITY-filled buffer
            unsigned long long key = ((unsigned long long)z_order(z) << 32) | (uint32_t)idx;
            atomicMin(&zrow[px], key);
        }
    }
}

// the raster loops of raster_trace for one piece: candidates into the z-key buffer
__global__ __launch_bounds__(BLOCK) void raster_fill_kernel(KParams P, RasterArgs A, int npieces)
{
    int idx = blockIdx.x * BLOCK + threadIdx.x;
    if (idx >= npieces)
        return;
    const RasterPiece& R = A.pieces[idx];
    if (R.y1 >= R.y0 && R.x1 >= R.x0 && (int64_t)(R.y1 - R.y0 + 1) * (R.x1 - R.x0 + 1) > RASTER_BIG) {
        A.big[atomicAdd(A.nbig, 1u)] = idx;
        return;
    }
    raster_rows(P, A, idx, R.y0, 1);
}

// big pieces: the workgroup's threads take the bounding box's rows round-robin
__global__ __launch_bounds__(BLOCK) void raster_fill_big_kernel(KParams P, RasterArgs A)
{
    const unsigned n = *A.nbig;
    for (unsigned k = blockIdx.x; k < n; k += gridDim.x) {
        const int idx = A.big[k];
        raster_rows(P, A, idx, A.pieces[idx].y0 + (int)threadIdx.x, BLOCK);
    }
}

// per pixel: the winning piece's shading (trace_triangle / debug shadings), reflective
// hits become level-1 frames of the reflection engine.  P.tri_uv is the piece_uv table
// and Rec::tri a piece index here (trace_triangle's temporary triangle).
__global__ __launch_bounds__(BLOCK, RT_OCC) void raster_shade_kernel(KParams P_arg, RasterArgs A,
                                                                     FrameRec* fr1, unsigned int* nfr1)
{
    // the parameters where the kernel received them (not a copy: passing the by-value argument to a
    // call made every lane copy it to scratch, r05: C5's shadow pass wrote ~90 GB per launch)
    const KParams& P = kernel_params();
    (void)P_arg;
    extern __shared__ uint2 lds_levels[];
    uint2* lv = lds_levels + threadIdx.x;
    int lane = threadIdx.x & 63;
    const int ntiles = P.tiles_x * P.tiles_y;
    v3 cam = mk(P.cam_pos[0], P.cam_pos[1], P.cam_pos[2]);
    const float hs = 1.0f / P.rh * 2, ws = 1.0f / P.rw * 2;
    unsigned nshadow = 0;
    for (;;) {
        int tile = 0;
        if (lane == 0)
            tile = (int)atomicAdd(reinterpret_cast<unsigned int*>(&P.counters[2]), 1u);
        tile = __builtin_amdgcn_readfirstlane(tile);
        if (tile >= ntiles)
            break;
        int tx, ty;
        tile_xy(P, tile, tx, ty);
        int px = tx * 8 + (lane & 7);
        int lr = ty * 8 + (lane >> 3);
        int py = lr < P.local_rows ? global_row(P, lr) : P.rh;
        if (px >= P.rw || py >= P.rh)
            continue;
        size_t o = (size_t)lr * P.rw + px;
        unsigned long long key = A.zkey[o];
        c3 color = background();
        bool sh = false, deferred = false;
        int hit = -1;
        float zt = INFINITY;
        if (key != ~0ull) {
            int idx = (int)(uint32_t)key;
            uint32_t zo = (uint32_t)(key >> 32);
            zt = __uint_as_float((zo & 0x80000000u) ? (zo & 0x7fffffffu) : ~zo);
            const RasterPiece& R = A.pieces[idx];
            hit = R.tri;
            float iy = R.y0 * hs - 1;
            for (int y = R.y0; y < py; y++) iy += hs;
            float ix = R.x0 * ws - 1;
            for (int x = R.x0; x < px; x++) ix += ws;
            float sx = ix + ws * 0.5f, sy = iy + hs * 0.5f;
            v3 a = ld3(R.na), b = ld3(R.nb), c = ld3(R.nc);
            float u = edge_fn(sx, sy, c, a) * R.inv_area;
            float v = edge_fn(sx, sy, a, b) * R.inv_area;
            const float* q = A.tri9 + 9 * (size_t)R.tri;
            if (P.shading_method == RT_SHADING) {
                // trace_triangle (renderer.cpp:619-628): Triangle::intersect with the world piece
                v3 pw = xform_point(P.cam_to_world, xform_point(P.proj_inv, mk(sx, sy, -1)));
                v3 rd = normalize(pw - cam);
                v3 wa = ld3(R.wa), wb = ld3(R.wb), wc = ld3(R.wc);
                v3 ab = wb - wa, ac = wc - wa;
                v3 nn = cross(wb - wa, wc - wa);
                TriRec T;
                T.q0 = make_float4(wa.x, wa.y, wa.z, ab.x);
                T.q1 = make_float4(ab.y, ab.z, ac.x, ac.y);
                T.q2 = make_float4(ac.z, nn.x, nn.y, nn.z);
                TRay Rr = make_ray(P, cam, rd);
                float tt, uu, vv;
                color = col(0, 0, 0);
                if (tri_test_rec(T, Rr, tt, uu, vv)) {
                    // the HitInfo Triangle::intersect fills (triangle.cpp:81-88), texcoords of the piece
                    Rec fin = rec_fresh();
                    fin.tri = idx;
                    fin.t = tt;
                    fin.u = uu;
                    fin.v = vv;
                    fin.mat = P.tri_mat[R.tri];
                    fin.normal = normalize(nn);
                    const float* uvp = P.tri_uv + 6 * (size_t)idx;
                    float u1 = uvp[0], u2 = uvp[1], u3 = uvp[2], v1 = uvp[3], v2 = uvp[4], v3_ = uvp[5];
                    float dU1 = u2 - u1, dV1 = v2 - v1, dU2 = u3 - u1, dV2 = v3_ - v1;
                    float f = 1.0f / (dU1 * dV2 - dU2 * dV1);
                    fin.tangent.x = f * (dV2 * ab.x - dV1 * ac.x);
                    fin.tangent.y = f * (dV2 * ab.y - dV1 * ac.y);
                    fin.tangent.z = f * (dV2 * ab.z - dV1 * ac.z);
                    Direct D = shade_direct(P, cam, rd, fin, lv, nshadow);
                    sh = D.shadowed;
                    const float* m = mat_of(P, fin.mat);
                    if (m[12] > 0.0f) {
                        unsigned fi = atomicAdd(nfr1, 1u);
                        make_frame(P, fr1[fi], D.ip, fin.normal, rd, D.fc, frame_roughness(P, fin, m), fin.mat,
                                   pixel_seed((uint32_t)(py * P.rw + px), P.rng_seed), (int)o);
                        deferred = true;
                    } else
                        color = shade_finish(P, D.fc, m, col(0, 0, 0));
                }
            } else if (P.shading_method == ABS_NORMALS || P.shading_method == PASTEL_NORMALS) {
                v3 ta = mk(q[0], q[1], q[2]), tb = mk(q[3], q[4], q[5]), tc = mk(q[6], q[7], q[8]);
                v3 nn = normalize(cross(tb - ta, tc - ta));
                color = P.shading_method == ABS_NORMALS ? col(fabsf(nn.x), fabsf(nn.y), fabsf(nn.z))
                                                         : (col(nn.x, nn.y, nn.z) + col(1.0f, 1.0f, 1.0f)) * 0.5f;
            } else if (P.shading_method == BARYCENTRIC) {
                color = (col(1, 0, 0) * u + col(0, 1.0f, 0) * v) + col(0, 0, 1) * (1 - u - v);
            } else if (P.shading_method == VISUALIZE_AO) {
                color = col(0.9f, 0.9f, 0.9f);
                if (P.enable_ao_mapping) {
                    float tu, tv;
                    get_tex_coords(P, idx, u, v, tu, tv);
                    float ao = tex_floor(P.tex[TEX_AO], tu, tv).r;
                    color = color * col(ao, ao, ao);
                }
            }
        }
        if (!deferred) {
            if (P.argb) P.argb[o] = color_to_argb(color);
            if (P.rgba) P.rgba[o] = make_float4(color.r, color.g, color.b, 1.0f);
        }
        if (P.hit_id) P.hit_id[o] = hit;
        if (P.hit_t) P.hit_t[o] = zt;
        if (P.shadow) P.shadow[o] = (uint8_t)sh;
        if (P.zbuf) {
            // renderer.cpp:975-979: the z-test winner's z and original_triangle._normal
            // (cross(b - a, c - a), triangle.cpp:9-10, unnormalised)
            P.zbuf[o] = zt;
            v3 nn = mk(0, 0, 0);
            if (hit >= 0) {
                const float* q = A.tri9 + 9 * (size_t)hit;
                v3 ta = mk(q[0], q[1], q[2]), tb = mk(q[3], q[4], q[5]), tc = mk(q[6], q[7], q[8]);
                nn = cross(tb - ta, tc - ta);
            }
            P.nbuf[o] = make_float4(nn.x, nn.y, nn.z, 0.0f);
        }
    }
    if (nshadow) atomicAdd(&P.counters[0], (unsigned long long)nshadow);
}

// ===========================================================================
// Renderer::post_process_ssao_SIMD (renderer.cpp:1229-1434): screen-space
// ambient occlusion on the internal image, before the SSAA downscale.  One
// lane per pixel.  Columns x < w - w % 8 follow the 8-lane AVX2 loop's
// arithmetic (signed-lane randoms, the fused __m256Point::transform,
// round-to-nearest _mm256_cvtps_epi32), the w % 8 tail columns follow the
// scalar loop (unsigned randoms, Transform::operator(), truncating double ->
// int).  The reference's per-thread std::rand()-seeded generators are not
// reproducible; each pixel here owns the xorshift32 stream ssao_state(pixel),
// drawn x, y, z then lateral per sample, as the oracle and the reference
// harness do.  Then the 7x7 box blur of the counts is
// applied to the image (renderer.cpp:1416-1431).
// ===========================================================================
__device__ __forceinline__ uint32_t ssao_state(uint32_t pixel, uint32_t seed)
{
    uint32_t x = mix32(pixel * 0x9E3779B9u ^ seed ^ 0x5A0C1D3Bu);
    return x ? x : 0x9E3779B9u;
}

__device__ __forceinline__ uint32_t xs32(uint32_t& s)   // xorshift.h:13-22 / 43-52
{
    uint32_t x = s;
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    s = x;
    return x;
}

// _mm256_cvtps_epi32 under the default MXCSR: nearest-even; NaN / out of range -> INT_MIN
__device__ __forceinline__ int cvt_rne(float f)
{
    if (!(f >= -2147483648.0f && f < 2147483648.0f))
        return INT_MIN;
    return (int)__builtin_rintf(f);
}

__device__ int ssao_simd_pixel(const SsaoArgs& A, int x, int y, float view_z, uint32_t st)
{
    const bool valid = view_z != INFINITY && view_z == view_z;   // _CMP_NEQ_OQ against INFINITY
    float y_ndc = (float)y / (float)A.h * 2.0f - 1.0f;
    float x_ndc = (float)x / (float)A.w * 2.0f - 1.0f;
    float vrx = x_ndc * (A.fovm * A.aspect);
    float vry = y_ndc * A.fovm;
    v3 csp = mk(view_z * vrx, view_z * vry, view_z * -1.0f);
    float4 nq = A.n[(size_t)y * A.w + x];
    v3 n = mk(nq.x, nq.y, nq.z);
    {   // _mm256_normalize (m256Vector.cpp:73-108): a * (1 / sqrt(x*x + (y*y + z*z)))
        float inv = 1.0f / sqrtf(n.x * n.x + (n.y * n.y + n.z * n.z));
        n = mk(n.x * inv, n.y * inv, n.z * inv);
    }
    const float* pm = A.proj;
    const int wm1 = cvt_rne((float)A.w - 1.0f), hm1 = cvt_rne((float)A.h - 1.0f), wi = cvt_rne((float)A.w);
    int occ = 0;
    for (int i = 0; i < A.count; i++) {
        float rx = (float)(int32_t)xs32(st) / 2147483648.0f;
        float ry = (float)(int32_t)xs32(st) / 2147483648.0f;
        float rz = (float)(int32_t)xs32(st) / 2147483648.0f;
        float inv = 1.0f / sqrtf(rx * rx + (ry * ry + rz * rz));
        v3 rs = mk(rx * inv, ry * inv, rz * inv);
        float k = ((float)(int32_t)xs32(st) / 2147483648.0f + 1.0f) * 0.5f + 0.0001f;
        rs = mk(rs.x * k, rs.y * k, rs.z * k);
        rs = mk(rs.x * A.radius, rs.y * A.radius, rs.z * A.radius);
        rs = mk(rs.x + csp.x, rs.y + csp.y, rs.z + csp.z);
        v3 vd = mk(rs.x - csp.x, rs.y - csp.y, rs.z - csp.z);
        float dt = vd.x * n.x + (vd.y * n.y + vd.z * n.z);
        float flip = dt < 0.0f ? 1.0f : 0.0f;
        v3 bf = mk((csp.x - rs.x) * 2.0f, (csp.y - rs.y) * 2.0f, (csp.z - rs.z) * 2.0f);
        rs = mk(rs.x + bf.x * flip, rs.y + bf.y * flip, rs.z + bf.z * flip);
        // __m256Point::transform (m256Point.cpp:3-37): fused multiply-adds, w = 1 / wt
        float xt = __builtin_fmaf(pm[0], rs.x, __builtin_fmaf(pm[1], rs.y, __builtin_fmaf(pm[2], rs.z, pm[3])));
        float yt = __builtin_fmaf(pm[4], rs.x, __builtin_fmaf(pm[5], rs.y, __builtin_fmaf(pm[6], rs.z, pm[7])));
        float wt = __builtin_fmaf(pm[12], rs.x, __builtin_fmaf(pm[13], rs.y, __builtin_fmaf(pm[14], rs.z, pm[15])));
        float w = 1.0f / wt;
        int px = cvt_rne(((xt * w + 1.0f) * 0.5f) * (float)A.w);
        int py = cvt_rne(((yt * w + 1.0f) * 0.5f) * (float)A.h);
        px = px < wm1 ? px : wm1;
        px = px > 0 ? px : 0;
        py = py < hm1 ? py : hm1;
        py = py > 0 ? py : 0;
        float sgd = -1.0f * A.z[(int)((uint32_t)px + (uint32_t)py * (uint32_t)wi)];
        occ += (fabsf(sgd - csp.z) <= A.radius && rs.z < sgd && valid) ? 1 : 0;
    }
    return occ;
}

__device__ int ssao_scalar_pixel(const SsaoArgs& A, int x, int y, float view_z, uint32_t st)
{
    if (view_z == INFINITY)
        return 0;
    float x_ndc = (float)x / A.w * 2 - 1;
    float y_ndc = (float)y / A.h * 2 - 1;
    float vrx = x_ndc * A.aspect * A.tanv;
    float vry = y_ndc * A.tanv;
    v3 csp = mk(vrx * view_z, vry * view_z, -view_z);
    float4 nq = A.n[(size_t)y * A.w + x];
    v3 n = normalize(mk(nq.x, nq.y, nq.z));
    int16_t occ = 0;
    for (int i = 0; i < A.count; i++) {
        float rx = xs32(st) / (float)UINT32_MAX * 2 - 1;
        float ry = xs32(st) / (float)UINT32_MAX * 2 - 1;
        float rz = xs32(st) / (float)UINT32_MAX * 2 - 1;
        v3 rs = normalize(mk(rx, ry, rz));
        rs = rs * (xs32(st) / (float)UINT32_MAX + 0.0001f);
        rs = rs * A.radius;
        rs = rs + csp;
        if (dot(rs - csp, n) < 0)
            rs = rs + 2.0f * (csp - rs);
        v3 ndc = xform_point(A.proj, rs);
        int px = d2i((ndc.x + 1) * 0.5 * A.w);
        int py = d2i((ndc.y + 1) * 0.5 * A.h);
        px = px > 0 ? px : 0;
        px = px < A.w - 1 ? px : A.w - 1;
        py = py > 0 ? py : 0;
        py = py < A.h - 1 ? py : A.h - 1;
        float sgd = -A.z[(size_t)py * A.w + px];
        if (fabsf(sgd - csp.z) > A.radius)
            continue;
        if (rs.z < sgd)
            occ = (int16_t)(occ + 1);
    }
    return occ;
}

constexpr int SSAO_TX = 16, SSAO_TY = 16;   // 16x4-pixel waves: the sample gathers stay local

__global__ __launch_bounds__(256) void ssao_occlusion_kernel(SsaoArgs A)
{
    int x = blockIdx.x * SSAO_TX + threadIdx.x, y = blockIdx.y * SSAO_TY + threadIdx.y;
    if (x >= A.w || y >= A.h)
        return;
    size_t o = (size_t)y * A.w + x;
    float view_z = A.z[o];
    uint32_t st = ssao_state((uint32_t)o, A.seed);
    A.ao[o] = x < A.simd_w ? ssao_simd_pixel(A, x, y, view_z, st) : ssao_scalar_pixel(A, x, y, view_z, st);
}

// 7x7 box blur of the counts (integer sums: separable in LDS, exact), applied to
// the interior pixels with a hit: c * (1 - sum / 49 / count * amount) per channel,
// written as QColor(int, int, int) -- an out-of-range channel makes the colour
// invalid and QImage::setPixelColor leaves the pixel.
constexpr int BLUR_X = 32, BLUR_Y = 8, BLUR_H = 3;

__global__ __launch_bounds__(256) void ssao_blur_kernel(SsaoArgs A)
{
    __shared__ int tile[BLUR_Y + 2 * BLUR_H][BLUR_X + 2 * BLUR_H];
    __shared__ int rows[BLUR_Y + 2 * BLUR_H][BLUR_X];
    const int x0 = blockIdx.x * BLUR_X, y0 = blockIdx.y * BLUR_Y;
    const int tid = threadIdx.y * BLUR_X + threadIdx.x;
    constexpr int TW = BLUR_X + 2 * BLUR_H, TH = BLUR_Y + 2 * BLUR_H;
    for (int i = tid; i < TW * TH; i += BLUR_X * BLUR_Y) {
        int ly = i / TW, lx = i - ly * TW;
        int gx = x0 + lx - BLUR_H, gy = y0 + ly - BLUR_H;
        tile[ly][lx] = (gx >= 0 && gx < A.w && gy >= 0 && gy < A.h) ? A.ao[(size_t)gy * A.w + gx] : 0;
    }
    __syncthreads();
    for (int i = tid; i < BLUR_X * TH; i += BLUR_X * BLUR_Y) {
        int ly = i / BLUR_X, lx = i - ly * BLUR_X;
        int s = 0;
        for (int k = 0; k < 2 * BLUR_H + 1; k++) s += tile[ly][lx + k];
        rows[ly][lx] = s;
    }
    __syncthreads();
    int x = x0 + threadIdx.x, y = y0 + threadIdx.y;
    if (x < BLUR_H || x >= A.w - BLUR_H || y < BLUR_H || y >= A.h - BLUR_H)
        return;
    size_t o = (size_t)y * A.w + x;
    if (A.z[o] == INFINITY)
        return;
    int sum = 0;
    for (int k = 0; k < 2 * BLUR_H + 1; k++) sum += rows[threadIdx.y + k][threadIdx.x];
    const int bs = 2 * BLUR_H + 1;
    float cm = 1 - ((float)sum / (float)(bs * bs) / (float)A.count * A.amount);
    uint32_t p = A.argb[o];
    int r = f2i((float)((p >> 16) & 0xff) * cm), g = f2i((float)((p >> 8) & 0xff) * cm), b = f2i((float)(p & 0xff) * cm);
    if (r < 0 || r > 255 || g < 0 || g > 255 || b < 0 || b > 255)
        return;
    A.argb[o] = qrgb(r, g, b);
}

// ImageUtils::downscale_image_qt_ARGB32 (imageUtils.h:98-147): integer box
// filter of 8-bit channels, truncating division.
__global__ __launch_bounds__(256) void downscale_kernel(const uint32_t* __restrict__ in, int w, int h_rows, int f,
                                                        uint32_t* __restrict__ out)
{
    int dw = w / f, dh = h_rows / f;
    int x = blockIdx.x * blockDim.x + threadIdx.x;
    int y = blockIdx.y;
    if (x >= dw || y >= dh)
        return;
    int ar = 0, ag = 0, ab = 0;
    for (int i = 0; i < f; i++)
        for (int j = 0; j < f; j++) {
            uint32_t p = in[(size_t)(y * f + i) * w + (x * f + j)];
            ar += (p >> 16) & 0xff;
            ag += (p >> 8) & 0xff;
            ab += p & 0xff;
        }
    out[(size_t)y * dw + x] = qrgb(ar / (f * f), ag / (f * f), ab / (f * f));
}

// BVH::intersect (bvh.cpp:68-71) for a batch of arbitrary rays: the closest-hit
// query the reference's trace_ray / is_shadowed issue, exposed for callers and
// for ray-level parity tests.  Brute-force loop when enable_bvh is off.
__global__ __launch_bounds__(BLOCK) void trace_rays_kernel(KParams P_arg, const float* __restrict__ orig,
                                                           const float* __restrict__ dir, int n,
                                                           int32_t* __restrict__ out_id, float* __restrict__ out_t,
                                                           float* __restrict__ out_u, float* __restrict__ out_v,
                                                           uint8_t* __restrict__ out_ret)
{
    // the parameters where the kernel received them (not a copy: passing the by-value argument to a
    // call made every lane copy it to scratch, r05: C5's shadow pass wrote ~90 GB per launch)
    const KParams& P = kernel_params();
    (void)P_arg;
    extern __shared__ uint2 lds_levels[];
    uint2* lv = lds_levels + threadIdx.x;
    int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n)
        return;
    v3 o = mk(orig[3 * i], orig[3 * i + 1], orig[3 * i + 2]);
    v3 d = mk(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]);
    TRay R = make_ray(P, o, d);
    THit h;
    bool r;
    if (P.enable_bvh) {
        r = bvh_closest(P, R, h, lv);
    } else {
        h.t = -1.0f; h.u = 1.0f; h.v = 0.0f; h.k = -1;
        for (int k = 0; k < P.ntri_slots; k++) {
            float t, u, v;
            if (tri_test(P.tris, (uint32_t)k, R, t, u, v))
                if (t < h.t || h.t == -1) {
                    h.t = t; h.u = u; h.v = v; h.k = k;
                }
        }
        r = h.k >= 0;
    }
    out_id[i] = h.k >= 0 ? P.tri_id[h.k] : -1;
    out_t[i] = h.t;
    out_u[i] = h.u;
    out_v[i] = h.v;
    out_ret[i] = r ? 1 : 0;
}

// The wide-BVH query of the frames (wbvh.hpp wbvh_closest + kdop_certifies) for a
// batch of rays, with its status: the device build of what rt_wbvh_query_ex runs on the host (the
// hardware reciprocal and square root, the GPU-computed risk words of KParams::wrisk), so that the
// adversarial grazing cases can be checked on the GPU build itself (rt_wide_query).  kind 0: no risk
// words (reflection rays, rt_trace_ray); 1: rays from the camera read its words when their origin is
// the camera position, as wide_closest does; 2: (hit point, normal) pairs traced as is_shadowed's ray
// towards P.light (renderer.cpp:340-402), reading the light's words when the ray qualifies, and, in
// out_sh, the frame's own decision through wide_shadow (0 lit, 1 shadowed, 2 not decided: the frame
// takes the octree's segment query).  Every kind is also answered as a closest-hit query over the
// whole line (status 0 certified miss, 1 certified hit with the record, 2 not certified).
// (The occupancy bound is the plain kernel's: wide_closest_deep is compiled once for all its callers,
// within the loosest caller's register budget, and the plain kernel inherits what it uses.)
template <int G>
__global__ __launch_bounds__(BLOCK, RT_OCC_PLAIN) void wide_query_kernel(KParams P_arg, const float* __restrict__ orig,
                                                           const float* __restrict__ dir, int n, int kind,
                                                           float* __restrict__ o_out, float* __restrict__ d_out,
                                                           int32_t* __restrict__ status, int32_t* __restrict__ out_id,
                                                           float* __restrict__ out_t, float* __restrict__ out_u,
                                                           float* __restrict__ out_v, uint8_t* __restrict__ out_sh)
{
    // the parameters where the kernel received them (not a copy: passing the by-value argument to a
    // call made every lane copy it to scratch, r05: C5's shadow pass wrote ~90 GB per launch)
    const KParams& P = kernel_params();
    (void)P_arg;
    extern __shared__ uint2 lds_levels[];
    uint2* lv = lds_levels + threadIdx.x;
    // G > 1: the G lanes of a lane group trace ray i together (wbvh_closest<.., G>)
    const int i = (blockIdx.x * BLOCK + threadIdx.x) / G;
    const bool writer = (threadIdx.x & (G - 1)) == 0;
    if (i >= n)
        return;
    v3 o = mk(orig[3 * i], orig[3 * i + 1], orig[3 * i + 2]);
    v3 d = mk(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]);
    const uint64_t* rk = nullptr;
    int rsel = 0;
    float rsub = 0.0f, QS = W_QS_CLOSEST;
    uint8_t sh = 2;
    if (kind == 2) {
        const v3 p = o, nrm = d, lp = mk(P.light[0], P.light[1], P.light[2]);
        o = p + nrm * 1.0e-4f;
        d = normalize(lp - p);
        QS = W_QS_SHADOW;
        const TRay R0 = make_ray(P, o, d);
        const float m = seg_margin(P, R0);
        const float nl = fabsf(nrm.x) + fabsf(nrm.y) + fabsf(nrm.z);
        const float hi = (sqrtf(length2(p - lp)) + 1.0e-4f * nl) * (1.0f + 0x1p-10f) + m;
        const bool light = P.wrisk && hi <= P.risk_G && nl <= P.risk_nl;
        if (light) {
            rk = P.wrisk;
            rsel = 1;
            rsub = wrisk_sub(W_QS_SHADOW, hi, P.risk_nu);
        }
        bool s;
        if (P.wnodes && P.nnodes > 0 && P.seg_scale > 0.0f && !R0.nan && wide_shadow<G>(P, o, d, hi, p, lp, lv, &s, light))
            sh = s ? 1 : 0;
    } else if (kind == 1 && P.wrisk && o.x == P.cam_pos[0] && o.y == P.cam_pos[1] && o.z == P.cam_pos[2]) {
        rk = P.wrisk;
    }
    if (writer) {
        o_out[3 * i] = o.x;
        o_out[3 * i + 1] = o.y;
        o_out[3 * i + 2] = o.z;
        d_out[3 * i] = d.x;
        d_out[3 * i + 1] = d.y;
        d_out[3 * i + 2] = d.z;
    }
    int st = W_UNCERT;
    int32_t id = -1;
    WHit w;
    w.t = -1.0f;
    w.u = 1.0f;
    w.v = 0.0f;
    if (P.wnodes && P.nnodes > 0 && !ray_is_nan(o, d)) {
        const float om = fmaxf(fabsf(o.x), fmaxf(fabsf(o.y), fabsf(o.z)));
        const float m = 0x1p-16f * (om + P.scene_scale);
        WStackLds stk{lv};
        st = wbvh_closest<WStackLds, G>(P.wnodes, P.wtris, o, d, m, stk, w, nullptr, INFINITY, true, QS, rk, rsel, rsub);
        if (st == W_DEEP) {
            const WDeep r = wide_closest_deep(P.wnodes, P.wtris, o, d, m, INFINITY, true, QS, rk, rsel, rsub);
            st = r.st;
            w = r.w;
        }
        if (st == W_HIT) {
            const uint4 M = ldg(P.wmeta + w.k);
            if (kdop_certifies(load_gnode(P.nodes + M.y), o, d, w.t))
                id = (int32_t)M.z;
            else
                st = W_UNCERT;
        }
        if (st == W_MISS)
            w.t = -1.0f;
    }
    if (!writer)
        return;
    status[i] = st;
    out_id[i] = id;
    out_t[i] = st == W_HIT ? w.t : -1.0f;
    out_u[i] = st == W_HIT ? w.u : 1.0f;
    out_v[i] = st == W_HIT ? w.v : 0.0f;
    out_sh[i] = sh;
}

// Renderer::trace_ray (renderer.cpp:1008-1066) for a batch of arbitrary rays, one lane per
// ray, each with a fresh HitInfo: the colour trace_ray returns (shading, shadow ray, the
// compute_reflection recursion when REFL), and the record it leaves.  The host folds
// current_recursion_depth into P.max_recursion_depth (only their difference is read).  Ray
// i's rough-reflection stream is keyed as pixel i of a frame.
template <bool REFL>
__global__ __launch_bounds__(BLOCK, RT_OCC) void trace_colors_kernel(KParams P_arg, const float* __restrict__ orig,
                                                                     const float* __restrict__ dir, int n,
                                                                     float4* __restrict__ out_rgba,
                                                                     int32_t* __restrict__ out_src,
                                                                     float* __restrict__ out_t,
                                                                     uint8_t* __restrict__ out_found,
                                                                     uint8_t* __restrict__ out_shadow)
{
    // the parameters where the kernel received them (not a copy: passing the by-value argument to a
    // call made every lane copy it to scratch, r05: C5's shadow pass wrote ~90 GB per launch)
    const KParams& P = kernel_params();
    (void)P_arg;
    extern __shared__ uint2 lds_levels[];
    uint2* lv = lds_levels + threadIdx.x;
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    unsigned nshadow = 0, nrefl = 0;
    if (i < n) {
        const v3 o = mk(orig[3 * i], orig[3 * i + 1], orig[3 * i + 2]);
        const v3 d = mk(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]);
        const uint32_t key = REFL ? pixel_seed((uint32_t)i, P.rng_seed) : 0u;
        PixelOut po = trace_pixel<REFL>(P, o, d, lv, key, nshadow, nrefl);
        out_rgba[i] = make_float4(po.color.r, po.color.g, po.color.b, po.alpha);
        out_src[i] = po.found ? po.src : -1;
        out_t[i] = po.fin.t;
        out_found[i] = po.found ? 1 : 0;
        out_shadow[i] = (uint8_t)(po.found && po.shadowed);
    }
    if (nshadow) atomicAdd(&P.counters[0], (unsigned long long)nshadow);
    if (nrefl) atomicAdd(&P.counters[1], (unsigned long long)nrefl);
}

// The wide BVH's triangle records and their metadata, gathered on the device from the octree's
// (already uploaded) instead of uploading 64 B per triangle again: wide-BVH triangle k is octree
// slot s = slot[k]; wmeta[k] = {s, its octree leaf, its caller index, that triangle's material}.
// The frame's grazing-risk words (wbvh.hpp wbvh_risk_key / wrisk_pack / wbvh_risk_host, DESIGN.md
// 5.6): one thread per wide-BVH triangle; a triangle at risk for point sel takes the minimum of its
// key and its leaf child's and the union of its octree leaf's axis box with the child's, then its
// parent entries', stopping where both are already there (the walk that put them there goes on to
// the root).  K (float bits; non-negative floats compare as their bit patterns) is filled with
// INFINITY, B's lows with +INFINITY and highs with -INFINITY before the launch; wide_risk_pack_kernel
// then packs them into the risk words.  A point with no bound (A.on 0) gives every child key 0 and its
// whole frame.  Vector atomics on global memory.
__device__ __forceinline__ float atomic_min_float(float* p, float v)
{
    return v >= 0.0f ? __int_as_float(atomicMin(reinterpret_cast<int*>(p), __float_as_int(v)))
                     : __uint_as_float(atomicMax(reinterpret_cast<unsigned int*>(p), __float_as_uint(v)));
}
__device__ __forceinline__ float atomic_max_float(float* p, float v)
{
    return v >= 0.0f ? __int_as_float(atomicMax(reinterpret_cast<int*>(p), __float_as_int(v)))
                     : __uint_as_float(atomicMin(reinterpret_cast<unsigned int*>(p), __float_as_uint(v)));
}

struct RiskCapDirs {
    float c[2][3];
};
__global__ __launch_bounds__(256) void wide_risk_kernel(const GTri* __restrict__ wtris, const uint4* __restrict__ wmeta,
                                                        const GNode* __restrict__ onodes,
                                                        const uint32_t* __restrict__ tri_leaf,
                                                        const uint32_t* __restrict__ parent, uint32_t* K, float* B, int n,
                                                        WRiskArgs A, uint32_t* cap, RiskCapDirs cd)
{
    const int k = (int)(blockIdx.x * 256 + threadIdx.x);
    if (k >= n)
        return;
    const GTri t = load_gtri(wtris + k);
    for (int sel = 0; sel < 2; sel++) {
        if (!A.on[sel])
            continue;
        const float Kt = wbvh_risk_key(t, A.p[sel][0], A.p[sel][1], A.p[sel][2], A.G[sel], A.nu[sel], A.slack[sel],
                                       A.QS[sel]);
        if (!(Kt < INFINITY))
            continue;
        if (cap) {   // the point's risk cap: the least |cos(N, c)| over its at-risk triangles
            const double c[3] = {cd.c[sel][0], cd.c[sel][1], cd.c[sel][2]};
            atomicMin(cap + sel, __builtin_bit_cast(uint32_t, risk_cap_tri(t, c)));
        }
        const GNode L = load_gnode(onodes + ldg(wmeta + k).y);   // the octree leaf of its certificate
        const uint32_t kb = __builtin_bit_cast(uint32_t, Kt);
        uint32_t e = tri_leaf[k];
        for (int it = 0; it < 1024 && e != W_EMPTY; it++) {   // (a walk ends at the root)
            const size_t i = (2 * (size_t)(e >> 2) + sel) * 4 + (e & 3u);
            bool has = atomicMin(K + i, kb) <= kb;
            float* b = B + 6 * i;
            for (int a = 0; a < 3; a++) {
                has = (atomic_min_float(b + a, L.dn[a]) <= L.dn[a]) & has;
                has = (atomic_max_float(b + 3 + a, L.df[a]) >= L.df[a]) & has;
            }
            if (has)
                break;
            e = parent[e >> 2];
        }
    }
}

__global__ __launch_bounds__(256) void wide_risk_pack_kernel(const WNode* __restrict__ wnodes,
                                                             const uint32_t* __restrict__ K,
                                                             const float* __restrict__ B, unsigned long long* risk,
                                                             int nentries, WRiskArgs A)
{
    const int i = (int)(blockIdx.x * 256 + threadIdx.x);
    if (i >= nentries)
        return;
    const int sel = (i >> 2) & 1;
    const float Ki = __builtin_bit_cast(float, K[i]);
    if (!A.on[sel])
        risk[i] = wrisk_pack(0.0f, 0xFFFFFF000000ull);
    else if (Ki < INFINITY) {
        const WNode nd = wnodes[i >> 3];
        risk[i] = wrisk_pack(Ki, wrisk_qbox(nd, B + 6 * (size_t)i, B + 6 * (size_t)i + 3));
    } else
        risk[i] = wrisk_pack(INFINITY, 0);
}

__global__ __launch_bounds__(256) void wide_gather_kernel(const GTri* __restrict__ tris, const int32_t* __restrict__ slot,
                                                          const uint32_t* __restrict__ leaf_of_slot,
                                                          const int32_t* __restrict__ tri_id,
                                                          const int32_t* __restrict__ tri_mat, int n, GTri* wtris,
                                                          uint4* wmeta)
{
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k >= n)
        return;
    const int32_t s = slot[k];
    const float4* src = reinterpret_cast<const float4*>(tris + s);
    float4* dst = reinterpret_cast<float4*>(wtris + k);
    dst[0] = src[0];
    dst[1] = src[1];
    dst[2] = src[2];
    const int32_t id = tri_id[s];
    wmeta[k] = make_uint4((uint32_t)s, leaf_of_slot[s], (uint32_t)id, (uint32_t)tri_mat[id]);
}

// dynamic LDS of the traversal kernels: the octree level stack, or the wide-BVH stack
// (the same memory; a lane uses one at a time)
// plain_pixel: the launch runs trace_pixel<false, true> (the plain ray_trace_kernel instances and their
// split parts), whose pixel values wait in LDS_SAVE_ENTRIES more slots across the shadow query; the
// other kernels do not take them (32 -> 38 KB per block cost the 5-wave kernels a block)
size_t lds_bytes(const KParams& P, bool plain_pixel = false)
{
    if (plain_pixel)   // (the plain kernel over the wide BVH, or its octree-only instance without one)
        return (size_t)((P.wnodes ? lds_save_slot_plain<false>(P) : lds_save_slot_plain<true>(P)) + LDS_SAVE_ENTRIES) *
               BLOCK * sizeof(uint2);
    return (size_t)lds_save_slot(P) * BLOCK * sizeof(uint2);
}

}  // namespace rt

extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_trace_rays(const rt::KParams* P, const float* o, const float* d, int n, int32_t* id,
                                           float* t, float* u, float* v, uint8_t* ret, hipStream_t stream)
{
    if (n <= 0)
        return hipSuccess;
    size_t lds = rt::lds_bytes(*P);
    hipLaunchKernelGGL(rt::trace_rays_kernel, dim3((n + rt::BLOCK - 1) / rt::BLOCK), dim3(rt::BLOCK), lds, stream, *P,
                       o, d, n, id, t, u, v, ret);
    return hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_wide_query(const rt::KParams* P, const float* o,
                                                                                 const float* d, int n, int kind,
                                                                                 float* o_out, float* d_out,
                                                                                 int32_t* status, int32_t* id, float* t,
                                                                                 float* u, float* v, uint8_t* sh,
                                                                                 hipStream_t stream)
{
    if (n <= 0)
        return hipSuccess;
    size_t lds = rt::lds_bytes(*P);
    // RT_WIDE_QUERY_GROUP=2 / 4 / 8 (tests, tools): each ray traced by a lane group (wbvh_closest<.., G>)
    const char* gv = getenv("RT_WIDE_QUERY_GROUP");
    const int G = gv && (atoi(gv) == 2 || atoi(gv) == 4 || atoi(gv) == 8) ? atoi(gv) : 1;
    const dim3 grid((unsigned)(((int64_t)n * G + rt::BLOCK - 1) / rt::BLOCK));
#define RT_WQ(g) hipLaunchKernelGGL(rt::wide_query_kernel<g>, grid, dim3(rt::BLOCK), lds, stream, *P, o, d, n, kind, \
                                    o_out, d_out, status, id, t, u, v, sh)
    if (G == 1) RT_WQ(1);
    else if (G == 2) RT_WQ(2);
    else if (G == 4) RT_WQ(4);
    else RT_WQ(8);
#undef RT_WQ
    return hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_trace_colors(const rt::KParams* P, bool refl,
                                                                                   const float* o, const float* d,
                                                                                   int n, float4* rgba, int32_t* src,
                                                                                   float* t, uint8_t* found,
                                                                                   uint8_t* shadow, hipStream_t stream)
{
    if (n <= 0)
        return hipSuccess;
    size_t lds = rt::lds_bytes(*P);
    dim3 grid((n + rt::BLOCK - 1) / rt::BLOCK), block(rt::BLOCK);
    if (refl)
        hipLaunchKernelGGL(rt::trace_colors_kernel<true>, grid, block, lds, stream, *P, o, d, n, rgba, src, t, found,
                           shadow);
    else
        hipLaunchKernelGGL(rt::trace_colors_kernel<false>, grid, block, lds, stream, *P, o, d, n, rgba, src, t, found,
                           shadow);
    return hipGetLastError();
}

// The heavy list of a launch (KParams::heavy_list) from the previous launch's tile costs of the same
// layout: the tiles costing at least max(4 x the mean, the largest / 8), at most ntiles / 16 of them.
// With group G > 1, those that also cost at least split x the launch's mean cycles per wave (the sum
// over nwaves, the plain kernel's waves: a tile that would outlast the mean wave) go to the split list
// list[cap .. cap + ctr[3]) of trace_split_part (cap = ntiles / 16), the others to list[0 .. ctr[0])
// of ray_trace_kernel (the consumers clamp the counts to cap).  One lane per tile over the whole grid:
// the sum and the largest cost come from the previous launch itself (KParams::tile_stats, stats_prev),
// the list slots from one atomic per wave and list, each wave writes its 64 tiles' two bit words, and
// block 0 clears the launch's counter words, the sums the coming launch accumulates (stats_next) and the
// counts of the slot's next heavy_prep (ctr_next; ctr was cleared by the previous one).  r05 ran this
// as one 1,024-thread block: 83-91 us per launch at C4.
#ifndef RT_HEAVY_PRIO
#define RT_HEAVY_PRIO 1   // heavy tiles at raised wave priority (set_wave_prio)
#endif
__global__ __launch_bounds__(64) void heavy_prep_kernel(uint32_t* __restrict__ cost, int ntiles, int32_t* list,
                                                        uint32_t* bits, int32_t* ctr, int32_t* ctr_next,
                                                        const unsigned long long* stats_prev,
                                                        unsigned long long* stats_next,
                                                        unsigned long long* counters, int ncounters, int nwaves,
                                                        float split, int group)
{
    if (blockIdx.x == 0) {
        // for the coming launch: its counter words (the memset the launch would need otherwise: one
        // dispatch fewer per frame, each waiting for a free wave slot among the frames in flight), and
        // for the slot's next heavy_prep its list counts and tickets (this launch's are ctr)
        for (int i = (int)threadIdx.x; i < ncounters; i += (int)blockDim.x)
            counters[i] = 0ull;
        if (threadIdx.x < 4)
            ctr_next[threadIdx.x] = 0;
        if (threadIdx.x < 2)
            stats_next[threadIdx.x] = 0ull;
    }
    const unsigned long long sum = stats_prev[0];
    const unsigned int mx = (unsigned int)min(stats_prev[1], 0xFFFFFFFFull);
    const unsigned long long mean = ntiles > 0 ? sum / (unsigned long long)ntiles : 0;
    const unsigned long long thr = max(4 * mean, (unsigned long long)(mx / 8));
    // split: at least split x the mean cycles per wave (never, without a group)
    const unsigned long long thr2 = group > 1 && nwaves > 0 ? max(thr, (unsigned long long)((double)split * (double)sum / nwaves))
                                                            : ~0ull;
    const int cap = ntiles / 16;
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    const int lane = (int)(threadIdx.x & 63);
    const uint32_t c = i < ntiles ? cost[i] : 0u;
    const bool heavy = mx > 0 && c >= thr && c > 0;
    const bool two = heavy && c >= thr2;
    const uint64_t b1 = __ballot(heavy && !two), b2 = __ballot(two);
    int base1 = 0, base2 = 0;
    if (lane == 0) {
        if (b1) base1 = atomicAdd(ctr, __popcll(b1));
        if (b2) base2 = atomicAdd(ctr + 3, __popcll(b2));
    }
    base1 = __builtin_amdgcn_readfirstlane(base1);
    base2 = __builtin_amdgcn_readfirstlane(base2);
    const uint64_t below = (1ull << lane) - 1ull;   // (lane < 64)
    const int k = two ? base2 + __popcll(b2 & below) : base1 + __popcll(b1 & below);
    const bool listed = heavy && k < cap;
    if (listed) {
        // the wave's issue priority while it traces the tile (bits 28-29, ray_trace_kernel)
        const int prio = !RT_HEAVY_PRIO || ntiles >= (1 << 28) ? 0 : c >= mx / 2 ? 3 : c >= mx / 4 ? 2 : 1;
        list[two ? cap + k : k] = i | (prio << 28);
        if (two)
            cost[i] = 0u;   // (the parts add theirs; ray_trace_kernel stores a tile's own)
    }
    const uint64_t bl = __ballot(listed);
    if ((lane & 31) == 0 && i < ntiles)
        bits[i >> 5] = (uint32_t)(bl >> lane);
}

// ---- host-side launch wrappers (called from renderer.cpp) ----
// the plain kernel's grid (rt_launch_ray_trace): exactly its residency
static int plain_blocks(const rt::KParams& P)
{
    const int tiles = P.tiles_x * P.tiles_y;
    const int blocks = (tiles + rt::WAVES_PER_BLOCK - 1) / rt::WAVES_PER_BLOCK;
    return P.max_blocks > 0 ? std::max(1, std::min(blocks, P.max_blocks / 8 * RT_OCC_PLAIN)) : blocks;
}

extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_heavy_prep(const rt::KParams* P, uint32_t* cost,
                                                                                 int ntiles, int32_t* list,
                                                                                 uint32_t* bits, int32_t* ctr,
                                                                                 int32_t* ctr_next,
                                                                                 const unsigned long long* stats_prev,
                                                                                 unsigned long long* stats_next,
                                                                                 float split, int group,
                                                                                 hipStream_t stream)
{
    if (ntiles <= 0)
        return hipSuccess;
    // one-wave blocks: each finds a slot beside the persistent grids of the frames in flight
    hipLaunchKernelGGL(heavy_prep_kernel, dim3((ntiles + 63) / 64), dim3(64), 0, stream, cost, ntiles, list, bits,
                       ctr, ctr_next, stats_prev, stats_next, P->counters, rt::NCOUNTER_WORDS,
                       plain_blocks(*P) * rt::WAVES_PER_BLOCK, split, group);
    return hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_ray_trace(const rt::KParams* P, hipStream_t stream)
{
    int tiles = P->tiles_x * P->tiles_y;
    int blocks = (tiles + rt::WAVES_PER_BLOCK - 1) / rt::WAVES_PER_BLOCK;
    // persistent waves: enough blocks to fill every CU (surplus blocks find the queue empty)
    if (blocks > P->max_blocks && P->max_blocks > 0)
        blocks = P->max_blocks;
    if (blocks < 1)
        return hipSuccess;
    const bool plain = !P->has_reflection && P->plain && !P->zbuf && !P->nbuf;
    size_t lds = rt::lds_bytes(*P, plain);
    if (P->has_reflection)
        hipLaunchKernelGGL((rt::ray_trace_kernel<true, false>), dim3(blocks), dim3(rt::BLOCK), lds, stream, *P);
    else if (plain) {
        // the plain kernel's grid is exactly its residency (RT_OCC_PLAIN blocks of 4 waves per
        // CU): with two frames in flight, surplus blocks of one frame would be dispatched ahead
        // of the next frame's only to find the queue empty (C4 +1.3%: r02_bench98_*.log)
        if (!P->wnodes) {   // the octree specialisation (its residency differs: the generic grid)
            hipLaunchKernelGGL((rt::ray_trace_kernel<false, true, true>), dim3(blocks), dim3(rt::BLOCK), lds, stream, *P);
            return hipGetLastError();
        }
        const int pblocks = plain_blocks(*P);
        hipLaunchKernelGGL((rt::ray_trace_kernel<false, true>), dim3(pblocks), dim3(rt::BLOCK), lds, stream, *P);
    } else
        hipLaunchKernelGGL((rt::ray_trace_kernel<false, false>), dim3(blocks), dim3(rt::BLOCK), lds, stream, *P);
    return hipGetLastError();
}

// the walk's boxes: lows +INFINITY, highs -INFINITY
__global__ __launch_bounds__(256) void risk_box_init_kernel(float* B, size_t n)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < 6 * n)
        B[i] = (i % 6) < 3 ? INFINITY : -INFINITY;
}

extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_risk_box_init(float* B, size_t nentries,
                                                                                    hipStream_t stream)
{
    if (nentries > 0)
        hipLaunchKernelGGL(risk_box_init_kernel, dim3((unsigned)((6 * nentries + 255) / 256)), dim3(256), 0, stream, B,
                           nentries);
    return hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_wide_risk(
    const rt::GTri* wtris, const uint4* wmeta, const rt::GNode* onodes, const rt::WNode* wnodes, const uint32_t* tri_leaf,
    const uint32_t* parent, uint32_t* K, float* B, unsigned long long* risk, int n, int nnodes, const rt::WRiskArgs* A,
    uint32_t* cap, const float* cap_dir, hipStream_t stream)
{
    rt::RiskCapDirs cd;
    for (int i = 0; i < 6; i++)
        cd.c[i / 3][i % 3] = cap_dir ? cap_dir[i] : 0.0f;
    if (n > 0)
        hipLaunchKernelGGL(rt::wide_risk_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, wtris, wmeta, onodes,
                           tri_leaf, parent, K, B, n, *A, cap, cd);
    const int ne = 8 * nnodes;
    if (ne > 0)
        hipLaunchKernelGGL(rt::wide_risk_pack_kernel, dim3((ne + 255) / 256), dim3(256), 0, stream, wnodes, K, B, risk,
                           ne, *A);
    return hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_wide_gather(
    const rt::GTri* tris, const int32_t* slot, const uint32_t* leaf_of_slot, const int32_t* tri_id,
    const int32_t* tri_mat, int n, rt::GTri* wtris, uint4* wmeta, hipStream_t stream)
{
    if (n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(rt::wide_gather_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, tris, slot, leaf_of_slot,
                       tri_id, tri_mat, n, wtris, wmeta);
    return hipGetLastError();
}

// ---- origin cones (ocone.hpp): each listed cell's word, one lane per cell; the rest OC_NOSKIP ----
namespace rt {
__global__ void ocone_fill_kernel(uint2* cells, size_t n)
{
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n)
        cells[i] = make_uint2(0u, OC_NOSKIP << 16);
}

struct OConeArgs {
    float lo[3];
    int32_t dim[3];
    double h, r, slack, QS, cos_cap;
};

__global__ __launch_bounds__(256) void ocone_kernel(const OConeEnt* E, const GTri* tris, const uint32_t* todo, int n,
                                                    OConeArgs A, uint2* cells)
{
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n)
        return;
    const uint32_t id = todo[i];
    double c[3];
    ocone_center(A.lo, A.dim, A.h, id, c);
    cells[id] = ocone_cell<OC_STACK>(E, tris, c, A.r, A.slack, A.QS, A.cos_cap);
}
}  // namespace rt

extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_ocone(const rt::OConeEnt* E, const rt::GTri* tris,
                                                                     const uint32_t* todo, int n, const float lo[3],
                                                                     const int32_t dim[3], double h, double r, double slack,
                                                                     double QS, double cos_cap, uint2* cells,
                                                                     size_t ncells, hipStream_t stream)
{
    if (ncells == 0)
        return hipSuccess;
    hipLaunchKernelGGL(rt::ocone_fill_kernel, dim3((unsigned)((ncells + 255) / 256)), dim3(256), 0, stream, cells, ncells);
    if (n > 0) {
        rt::OConeArgs A;
        for (int a = 0; a < 3; a++) {
            A.lo[a] = lo[a];
            A.dim[a] = dim[a];
        }
        A.h = h;
        A.r = r;
        A.slack = slack;
        A.QS = QS;
        A.cos_cap = cos_cap;
        hipLaunchKernelGGL(rt::ocone_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, E, tris, todo, n, A,
                           cells);
    }
    return hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_downscale(const uint32_t* in, int w, int h_rows, int f, uint32_t* out,
                                          hipStream_t stream)
{
    int dw = w / f, dh = h_rows / f;
    if (dw <= 0 || dh <= 0)
        return hipSuccess;
    dim3 grid((dw + 255) / 256, dh);
    hipLaunchKernelGGL(rt::downscale_kernel, grid, dim3(256), 0, stream, in, w, h_rows, f, out);
    return hipGetLastError();
}

// ---- reflection engine launchers (renderer.cpp drives the levels) ----
extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_refl_level0(const rt::KParams* P, rt::FrameRec* fr1,
                                                                           unsigned int* nfr1, hipStream_t stream)
{
    int tiles = P->tiles_x * P->tiles_y;
    int blocks = (tiles + rt::WAVES_PER_BLOCK - 1) / rt::WAVES_PER_BLOCK;
    if (blocks > P->max_blocks && P->max_blocks > 0)
        blocks = P->max_blocks;
    if (blocks < 1)
        return hipSuccess;
    size_t lds = rt::lds_bytes(*P);
    hipLaunchKernelGGL(rt::refl_level0_kernel, dim3(blocks), dim3(rt::BLOCK), lds, stream, *P, fr1, nfr1);
    return hipGetLastError();
}

// stage: 1 gen + trace, 2 pass1, 3 shadow, 4 spawn, 5 resolve, 6 list, 7 the deferred long traces
extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_refl_stage(int stage, const rt::KParams* P,
                                                                          const rt::ReflArgs* A, hipStream_t stream)
{
    int nframes = A->c1 - A->c0;
    if (nframes <= 0)
        return hipSuccess;
    int nslot = nframes * A->stride;
    dim3 gs((nslot + rt::BLOCK - 1) / rt::BLOCK), gf((nframes + rt::BLOCK - 1) / rt::BLOCK);
    size_t lds = rt::lds_bytes(*P);
    switch (stage) {
    case 1:
        if (A->feed > 0)   // persistent waves (lane refill): the reflection kernels' residency
            hipLaunchKernelGGL(rt::refl_trace_feed_kernel,
                               dim3(std::max(1u, std::min<unsigned>(gs.x, (unsigned)(P->max_blocks / 8 * RT_OCC_FEED)))),
                               dim3(rt::BLOCK), (size_t)std::max(P->levels, rt::W_STACK_REFL_FEED) * rt::BLOCK * sizeof(uint2),
                               stream, *P, *A);
        else
            hipLaunchKernelGGL(rt::refl_trace_kernel, dim3(gs.x * RT_REFL_G), dim3(rt::BLOCK), lds, stream, *P, *A);
        break;
    case 7: hipLaunchKernelGGL(rt::refl_trace_long_kernel, dim3(std::min<unsigned>(gs.x, 2048u)), dim3(rt::BLOCK), lds,
                               stream, *P, *A); break;
    case 2: hipLaunchKernelGGL(rt::refl_pass1_kernel, gf, dim3(rt::BLOCK), 0, stream, *P, *A); break;
    case 3:
        if (A->shadow_feed > 0 && A->fused && !RT_COUNT) {
            // persistent waves (lane refill), then the entries they deferred by the one-query kernel
            hipLaunchKernelGGL(rt::refl_shadow_feed_kernel,
                               dim3(std::max(1u, std::min<unsigned>(gs.x, (unsigned)(P->max_blocks / 8 * RT_OCC_REFL)))),
                               dim3(rt::BLOCK), (size_t)std::max(P->levels, rt::W_STACK_REFL_FEED) * rt::BLOCK * sizeof(uint2),
                               stream, *P, *A);
            rt::ReflArgs D = *A;
            D.list = A->sdefer;
            D.list_count = A->sdefer_count;
            hipLaunchKernelGGL(rt::refl_shadow_kernel, gs, dim3(rt::BLOCK), lds, stream, *P, D);
        } else
            hipLaunchKernelGGL(rt::refl_shadow_kernel, gs, dim3(rt::BLOCK), lds, stream, *P, *A);
        break;
    case 4: hipLaunchKernelGGL(rt::refl_spawn_kernel, gs, dim3(rt::BLOCK), 0, stream, *P, *A); break;
    case 6: hipLaunchKernelGGL(rt::refl_list_kernel, gs, dim3(rt::BLOCK), 0, stream, *P, *A); break;
    default: hipLaunchKernelGGL(rt::refl_resolve_kernel, gf, dim3(rt::BLOCK), 0, stream, *P, *A); break;
    }
    return hipGetLastError();
}

namespace rt {
// the level's frames copied in their sorted order (ReflArgs::frs): the passes that walk the sorted
// positions read adjacent records
__global__ __launch_bounds__(256) void refl_sort_frames_kernel(const FrameRec* __restrict__ fr, const int32_t* __restrict__ order,
                                                               int n, FrameRec* __restrict__ frs)
{
    const int p = (int)(blockIdx.x * 256 + threadIdx.x);
    if (p < n)
        frs[p] = fr[order[p]];
}
}  // namespace rt

extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_refl_sort_frames(const rt::FrameRec* fr, const int32_t* order,
                                                                                int n, rt::FrameRec* frs, hipStream_t stream)
{
    if (n > 0)
        hipLaunchKernelGGL(rt::refl_sort_frames_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, fr, order, n, frs);
    return hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_refl_shadow_keys(const rt::KParams* P, const rt::SampleRec* sm,
                                                                                 const int32_t* list, int n, uint32_t* keys,
                                                                                 hipStream_t stream)
{
    if (n > 0)
        hipLaunchKernelGGL(rt::refl_shadow_keys_kernel, dim3((n + rt::BLOCK - 1) / rt::BLOCK), dim3(rt::BLOCK), 0, stream, *P,
                           sm, list, n, keys);
    return hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_refl_dir_keys(const rt::KParams* P, const rt::ReflArgs* A,
                                                                              uint32_t* keys, int32_t* vals, hipStream_t stream)
{
    const int n = (A->c1 - A->c0) * A->stride;
    if (n > 0)
        hipLaunchKernelGGL(rt::refl_dir_keys_kernel, dim3((n + rt::BLOCK - 1) / rt::BLOCK), dim3(rt::BLOCK), 0, stream, *P,
                           *A, keys, vals);
    return hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_refl_defer_keys(const rt::ReflArgs* A, int n, uint32_t* keys,
                                                                                hipStream_t stream)
{
    if (n > 0)
        hipLaunchKernelGGL(rt::refl_defer_keys_kernel, dim3((n + rt::BLOCK - 1) / rt::BLOCK), dim3(rt::BLOCK), 0, stream, *A, n,
                           keys);
    return hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_refl_keys(const rt::KParams* P, const rt::FrameRec* fr,
                                                                         int n, uint32_t* keys, int32_t* idx,
                                                                         hipStream_t stream)
{
    if (n <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(rt::refl_keys_kernel, dim3((n + rt::BLOCK - 1) / rt::BLOCK), dim3(rt::BLOCK), 0, stream, *P, fr,
                       n, keys, idx);
    return hipGetLastError();
}

// ---- raster launchers (renderer.cpp raster path) ----
// stage: 0 count, 1 write, 2 fill (small pieces), 3 fill (big pieces)
extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_raster_stage(int stage, const rt::KParams* P,
                                                                            const rt::RasterArgs* A, int npieces,
                                                                            hipStream_t stream)
{
    if (stage < 2) {
        if (A->ntri <= 0)
            return hipSuccess;
        dim3 g((unsigned)((A->ntri + rt::BLOCK - 1) / rt::BLOCK));
        if (stage == 0)
            hipLaunchKernelGGL(rt::raster_count_kernel, g, dim3(rt::BLOCK), 0, stream, *P, *A);
        else
            hipLaunchKernelGGL(rt::raster_write_kernel, g, dim3(rt::BLOCK), 0, stream, *P, *A);
    } else if (stage == 2) {
        if (npieces <= 0)
            return hipSuccess;
        hipLaunchKernelGGL(rt::raster_fill_kernel, dim3((npieces + rt::BLOCK - 1) / rt::BLOCK), dim3(rt::BLOCK), 0,
                           stream, *P, *A, npieces);
    } else {
        if (npieces <= 0)
            return hipSuccess;
        hipLaunchKernelGGL(rt::raster_fill_big_kernel, dim3(P->max_blocks > 0 ? P->max_blocks : 1024),
                           dim3(rt::BLOCK), 0, stream, *P, *A);
    }
    return hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_raster_shade(const rt::KParams* P,
                                                                            const rt::RasterArgs* A,
                                                                            rt::FrameRec* fr1,
                                                                            unsigned int* nfr1, hipStream_t stream)
{
    int tiles = P->tiles_x * P->tiles_y;
    int blocks = (tiles + rt::WAVES_PER_BLOCK - 1) / rt::WAVES_PER_BLOCK;
    if (blocks > P->max_blocks && P->max_blocks > 0)
        blocks = P->max_blocks;
    if (blocks < 1)
        return hipSuccess;
    size_t lds = rt::lds_bytes(*P);
    hipLaunchKernelGGL(rt::raster_shade_kernel, dim3(blocks), dim3(rt::BLOCK), lds, stream, *P, *A, fr1, nfr1);
    return hipGetLastError();
}

extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_ssao(const rt::SsaoArgs* A, hipStream_t stream)
{
    if (A->w <= 0 || A->h <= 0)
        return hipSuccess;
    hipLaunchKernelGGL(rt::ssao_occlusion_kernel,
                       dim3((A->w + rt::SSAO_TX - 1) / rt::SSAO_TX, (A->h + rt::SSAO_TY - 1) / rt::SSAO_TY),
                       dim3(rt::SSAO_TX, rt::SSAO_TY), 0, stream, *A);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        return e;
    hipLaunchKernelGGL(rt::ssao_blur_kernel, dim3((A->w + rt::BLUR_X - 1) / rt::BLUR_X, (A->h + rt::BLUR_Y - 1) / rt::BLUR_Y),
                       dim3(rt::BLUR_X, rt::BLUR_Y), 0, stream, *A);
    return hipGetLastError();
}

#if defined(RT_COUNT) && RT_COUNT
// diagnostic builds: read and clear g_wsteps (tools/count_gpu_work.py)
extern "C" __attribute__((visibility("default"))) int rt_diag_wave_steps(unsigned long long* out)
{
    unsigned long long z[8] = {};
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wsteps), sizeof(z)) != hipSuccess) return -1;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_wsteps), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
