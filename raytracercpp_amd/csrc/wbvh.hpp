// wbvh.hpp -- a 4-wide SAH bounding-volume hierarchy over the octree's triangle records,
// used to find primary-ray hits fast, and the certificate that makes its answer the
// reference's.
//
// The reference's BVH::intersect (tp2/projets/bvh.h:212-287) returns the closest hit
// among the triangles of the octree leaves it visits, folded in its visit order.  The
// wide BVH below finds the minimum-t hit t* over ALL triangles (its boxes contain every
// point Moller-Trumbore can report as a hit; the kernel widens them by a margin far above
// the rounding of the test).  That is the reference's record when
//   (1) t* is finite and > 0, no other triangle hits at exactly t*, and no tested hit is NaN;
//   (2) the octree leaf L holding t*'s triangle passes the reference's own k-DOP test
//       (BoundingVolume::intersect, bvh.h:79-105, the same IEEE arithmetic) with t_near <= t*.
// Every ancestor's slabs contain L's (min / max over more triangles), and rounding is
// monotone, so each ancestor's computed t_near is <= L's and its t_far >= L's: every node
// on the path passes and none is skipped by the early-out (bvh.h:270: that needs an
// earlier record t_A < t_near <= t*, and t* is the minimum).  The reference therefore
// tests t*'s triangle and its record ends at t* with the same (t, u, v), and every node on
// the path returns true.  A query the certificate does not cover (ties, t* <= 0 or
// infinite, a NaN hit, a traversal stack overflow, (2) failing) is re-traced by the exact
// octree traversal.  With no hit at all, the reference finds none either and returns false
// with a fresh record.
//
// Layout (HBM): WNode 128 B (struct WNode below), the four children's boxes quantised to 8 bits
// per plane against the node's own frame (Ylitie et al.'s compressed wide nodes, 4-wide):
//   float4 0: origin x, y, z (the node box's low corner) and the three scale exponents
//             (byte a = biased exponent of the power-of-two step s_a along axis a);
//   float4 1: q_lo x[4], q_lo y[4], q_lo z[4], q_hi x[4] (one byte per child);
//   float4 2: q_hi y[4], q_hi z[4], the slab scale and offset;
//   float4 3 / 4: the slab normals and cones / the slab ranges;
//   float4 5: the four child links:
//     inner child:  node index (bit 31 clear);
//     leaf child:   W_LEAF | first << 3 | (count - 1), triangles first .. first + count - 1
//                   of the wide BVH's own triangle order (count <= 8);
//     no child:     W_EMPTY.
//   float4 6 / 7: the conditioning bytes of the sound child test (ext, ext2).
// Child box = [origin + q_lo s, origin + q_hi s] with q_lo rounded down and q_hi up, so
// it holds the float box exactly (checked in double by check_wbvh).
// Triangles: GTri records (octree.hpp) copied in leaf order, plus slot[] = the octree GTri
// slot of each, and leaf_of_slot[] = the flattened octree leaf node holding each slot.
#pragma once

#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <vector>

#include "octree.hpp"

namespace rt {

constexpr uint32_t W_LEAF = 0x80000000u;
constexpr uint32_t W_EMPTY = 0xFFFFFFFFu;
constexpr int W_MAX_LEAF = 8;
#ifndef W_GROUP_ILP
#define W_GROUP_ILP 0   // lane groups: the four children's tests interleaved by the scheduler (wbvh_closest)
#endif
#ifndef W_STACK_N
#define W_STACK_N 16
#endif
constexpr int W_STACK = W_STACK_N;   // traversal stack entries per lane (a child dropped by a full stack
                                     // whose key is at most the final best hit: the query is not certified)
constexpr int W_WIDTH = 4;    // children per node

// the grazing split QS of the wide query's child test per query kind (wbvh_closest, wbvh_risk_key):
// (a)'s reach grows as 1 / QS (wq_reach: its D term is 10.87u D / QS), the risk set of case (b) as QS.
// r05, with the correlated reach (tools/visit_probe.py, host wide-node visits per C4 ray, every 8th
// tile row): camera 2^-8 / 2^-10 / 2^-12 / 2^-14: 5.71 / 5.15 / 4.83 / 52 (at 2^-14 the pole slivers'
// s q falls below the bound's 5.86u: no reach); shadow 2^-11 / 2^-12 / 2^-13 / 2^-14: 7.72 / 7.06 /
// 8.61 / 8.55.  On the GPU (three scenes, so that the choice is not the headline sphere's alone,
// profiles/r05/qs_scenes.log): camera 2^-10 is ahead of 2^-8 on C4 (+7.8%), hair1m (+5%) and robot
// (+1%); 2^-12 is ahead on C4 only (hair1m -6%, robot -4%)
#ifndef W_QS_CLOSEST
#define W_QS_CLOSEST 0x1p-10f
#endif
#ifndef W_QS_SHADOW
#define W_QS_SHADOW 0x1p-12f
#endif

// case (b)'s D (wbvh_closest): the farthest corner of the child's box (sound either way; 0: the node's
// frame for every ray, 1: per child for rays without risk words, 2: per child for every ray)
#ifndef W_B_CHILD_D
#define W_B_CHILD_D 2
#endif
#ifndef W_A_CHILD_D
#define W_A_CHILD_D 0   // case (a)'s D per child as well (sound either way)
#endif

// timing-only switches (tools/variants.py; never sound when off)
#ifndef W_CASE_B
#define W_CASE_B 1
#endif
#ifndef W_STEP_CAP
#define W_STEP_CAP 0
#endif
#ifndef W_LAZY_EXT2
#define W_LAZY_EXT2 0
#endif
#ifndef W_PRIO_ORDER
#define W_PRIO_ORDER 1   // children visited by their unwidened entry t (wbvh_closest)
#endif
#ifndef W_SOUND_A
#define W_SOUND_A 1
#endif
#ifndef W_SMIN_FLOOR
#define W_SMIN_FLOOR 0.0f   // (diagnostic builds: a floor on the children's smin, to price the slivers' widening)
#endif
#ifndef W_R_SCALE
#define W_R_SCALE 1.0f      // (diagnostic builds: case (a)'s widening R scaled, to price its constants)
#endif

// host diagnostic counters (tools/variants.py build diag="-DW_DIAG=1"; rt_diag_read)
#if defined(W_DIAG) && !defined(__HIP_DEVICE_COMPILE__)
inline std::atomic<long long> g_wdiag[8];
#define W_DIAG_ADD(i, v) rt::g_wdiag[i].fetch_add((long long)(v), std::memory_order_relaxed)
#else
#define W_DIAG_ADD(i, v) ((void)0)
#endif

#ifndef W_STEP_HOOK
#define W_STEP_HOOK(cur, leaf)   // diagnostic builds (kernels.hip): per-step wave statistics
#endif

// cone threshold step: c in 0..254 encodes c * 224 / 254 >= |N| (|N| <= 127 sqrt 3 < 220), so 255
// can never pass.  W_CONE_EPS: the triangles' minimum cos(normal, d) the build guarantees
constexpr float W_CONE_STEP = 224.0f / 254.0f;
constexpr double W_CONE_EPS = 1e-4;

struct alignas(16) WNode {
    float ox, oy, oz;
    uint32_t exps;        // byte a: biased exponent (127 + k) of the step 2^k along axis a
    uint8_t qlo[3][W_WIDTH];    // [axis][child]
    uint8_t qhi[3][W_WIDTH];
    // Orientation slab of child j: every vertex v below it has
    //   slo + q0 s  <=  N_j . (v - origin)  <=  slo + q1 s,
    // N_j = nrm bytes 0..2 as signed 8-bit integers (the subtree's area-weighted normal,
    // quantised to [-127, 127]), q0 / q1 the low / high 16 bits of slab[j].  A curved patch is thin
    // along its mean normal, so a ray that grazes the surface misses most patches' slabs
    // although it crosses their boxes (silhouette rays).
    // Backface cone of child j: nrm byte 3 = c, 255 = none.  Every triangle
    // below j that Moller-Trumbore could ever hit faces away from a ray whose direction d has
    //   N_j . d  >  c * W_CONE_STEP * |d|
    // (the test rejects it on Mdet <= 0 before anything else), so such a ray skips j.
    float s, slo;
    uint32_t nrm[W_WIDTH];
    uint32_t slab[W_WIDTH];
    uint32_t child[W_WIDTH];
    // Conditioning of child j's triangles (the grazing-sound query), one byte each,
    // as 8-bit minifloats (wn_code / wn_decode):
    //   ext[j]  byte 0: smin, a lower bound on sin(alpha) (alpha: the triangle's angle at a);
    //           byte 1: s2, a lower bound on sin(alpha' / 2), alpha' = min(alpha, pi - alpha);
    //           byte 2: sth, an upper bound on sin(angle(N_j, n)) over the triangles' exact normals;
    //           byte 3: lmax, an upper bound on their edges |ab|, |ac|;
    //   ext2[j] byte 0: rho, how far the k-DOP boxes of the octree leaves holding them reach past
    //           the child's box (0 when the child holds whole octree leaves); bytes 1-3 unused.
    uint32_t ext[W_WIDTH];
    uint32_t ext2[W_WIDTH];
};
static_assert(sizeof(WNode) == 128, "WNode size");
// word offsets inside a node (the kernel loads it as 16-B rows and picks words)
constexpr int WN_QLO = 4;                           // qlo[a] starts at word WN_QLO + a * W_WIDTH / 4
constexpr int WN_QHI = 4 + 3 * W_WIDTH / 4;         // qhi[a] at WN_QHI + a * W_WIDTH / 4
constexpr int WN_SS = 4 + 6 * W_WIDTH / 4;          // s, slo
constexpr int WN_NRM = ((4 + 6 * W_WIDTH / 4 + 2 + 3) / 4) * 4;
constexpr int WN_SLAB = WN_NRM + W_WIDTH;
constexpr int WN_CHILD = WN_SLAB + W_WIDTH;
constexpr int WN_EXT = WN_CHILD + W_WIDTH;
constexpr int WN_EXT2 = WN_EXT + W_WIDTH;
constexpr int WN_ROWS = (int)(sizeof(WNode) / 16);

// The conditioning bytes: value(k) = float with bits (k << 20) + base for k > 0 (three mantissa
// bits, an octave per 8 codes); k = 0 is 0.  Unit quantities (sines) use WQ_UNIT (k = 255 is
// 1.0), lengths WQ_LEN (2^-16 .. 2^16; k = 255 stands for "no bound", infinity).
constexpr uint32_t WQ_UNIT = 0x3F800000u - (255u << 20);
constexpr uint32_t WQ_LEN = 111u << 23;
RT_HD float wq_val(uint32_t k, uint32_t base)
{
    return k == 0u ? 0.0f : __builtin_bit_cast(float, (k << 20) + base);
}
RT_HD float wq_len(uint32_t k)
{
    return k == 255u ? INFINITY : wq_val(k, WQ_LEN);
}
// code k read as if k = 0 stood for the smallest nonzero value (2^-19 x the top value for WQ_UNIT,
// 2^-16 for WQ_LEN): a larger upper bound, or, for a lower bound used only as a divisor whose tiny
// values already mean "no bound" (the query's smin, s2), the same decision as 0
RT_HD float wq_val_nz(uint32_t k, uint32_t base)
{
    return __builtin_bit_cast(float, (k << 20) + base);
}

struct WStats {
    int64_t nodes = 0, leaves = 0, tris = 0, max_leaf = 0, depth = 0;
    float sah = 0.0f;   // SAH cost of the binary tree (traversal 1, triangle 1), for diagnostics
};

struct WBvh {
    std::vector<WNode> nodes;          // nodes[0] = root (empty when there are no triangles)
    std::vector<GTri> tris;            // octree records in leaf order
    std::vector<int32_t> slot;         // wide-BVH triangle -> octree GTri slot
    std::vector<uint32_t> leaf_of_slot;   // octree GTri slot -> flattened octree leaf node
    std::vector<uint32_t> leaf_of_k;      // wide-BVH triangle -> flattened octree leaf node (= leaf_of_slot[slot])
    // the grazing-risk walk (wbvh_risk_tri): wide-BVH triangle -> its leaf child (node << 2 | slot),
    // node -> its parent's child entry (parent << 2 | slot; W_EMPTY for the root)
    std::vector<uint32_t> tri_leaf, parent;
    WStats stats;
};

// A lower bound on sin(angle at a) of the record's edges ab, ac (floats) from the exact cross
// product: the double products of floats are exact, each difference rounds once (2^-53 of the
// larger term), so |ab x ac| >= |cross_double| - 2^-51 |ab| |ac|.  1 for a zero cross product
// of non-zero edges is not claimed: 0 then (never skipped by the query's margins).
inline double sin_at_a_lb(const GTri& t)
{
    const double x0 = t.ab[0], x1 = t.ab[1], x2 = t.ab[2], y0 = t.ac[0], y1 = t.ac[1], y2 = t.ac[2];
    const double c0 = x1 * y2 - x2 * y1, c1 = x2 * y0 - x0 * y2, c2 = x0 * y1 - x1 * y0;
    const double ab = std::sqrt(x0 * x0 + x1 * x1 + x2 * x2), ac = std::sqrt(y0 * y0 + y1 * y1 + y2 * y2);
    const double lam = ab * ac;
    if (!(lam > 0x1p-100) || !(lam < 0x1p100))
        return 0.0;
    const double c = std::sqrt(c0 * c0 + c1 * c1 + c2 * c2);
    return std::max(0.0, (c - 0x1p-50 * lam) / lam * (1 - 1e-12));
}

// sin of the triangle's angle at a (Moller-Trumbore's vertex) as a float rounded down, from the
// exact cross product of the record's edges (sin_at_a_lb; the stored normal's own rounding could
// make |n| / (|ab| |ac|) overestimate it); 1 for n = 0 (never hit: Mdet = 0); 0 where the
// rounding analysis of DESIGN.md 5.6 does not apply (|n| outside [2^-60, 2^60], |ab| |ac|
// outside (2^-100, 2^100)).  Host only (kernels.hip leaf_missed's margin).
inline float sin_at_a_f(const GTri& t)
{
    const double n = std::sqrt((double)t.n[0] * t.n[0] + (double)t.n[1] * t.n[1] + (double)t.n[2] * t.n[2]);
    if (n == 0)
        return 1.0f;
    if (!(n >= 0x1p-60 && n <= 0x1p60))
        return 0.0f;
    const double sl = sin_at_a_lb(t);
    const float f = (float)sl;
    return (double)f > sl ? std::nextafter(f, 0.0f) : f;
}

// Binned-SAH binary build over the octree's triangle records, collapsed to 4-wide nodes
// (RT_BUILD_THREADS threads, as the octree build).  Boxes are the records' vertices a,
// a + ab, a + ac rounded outward to float.
void build_wbvh(const FlatOctree& oct, WBvh& out);
// The quick tree (r05, wbvh.cpp): the octree's own hierarchy as the wide BVH, O(n) to build, for the
// frames right after a geometry change while the SAH tree builds; RT_WBVH_QUICK=1 makes
// build_wbvh build it instead.
// tris = false: WBvh::tris left empty (the renderer gathers the records on the device; wbvh_fill_tris
// makes the host copy when a host check needs it).
void build_wbvh_quick(const FlatOctree& oct, WBvh& out, bool tris = true);
void wbvh_fill_tris(const FlatOctree& oct, WBvh& w);

// Structural check (CPU tests): every octree slot exactly once, each child box holds its
// subtree's boxes / its triangles' vertices, leaf sizes within W_MAX_LEAF, leaf_of_slot
// consistent with the octree.  Returns the number of violations.
int64_t check_wbvh(const FlatOctree& oct, const WBvh& w);

// ---------------------------------------------------------------------------------
// Traversal (host and device).  One query: the closest Moller-Trumbore hit over the
// wide BVH, then the certificate against the octree.

// Triangle::intersect, triangle.cpp:25-91 (backface culling), on a GTri record: the
// same expressions in the same order as the reference (and kernels.hip tri_test_rec).
RT_HD bool mt_record(const GTri& T, v3 o, v3 d, float& t_out, float& u_out, float& v_out)
{
    v3 a = mk(T.a[0], T.a[1], T.a[2]);
    v3 ab = mk(T.ab[0], T.ab[1], T.ab[2]);
    v3 ac = mk(T.ac[0], T.ac[1], T.ac[2]);
    v3 n = mk(T.n[0], T.n[1], T.n[2]);
    v3 OA = o - a;
    v3 nd = -d;
    v3 m = cross(nd, OA);
    float Mdet = dot(n, nd);
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
    return !(t < 0);
}

RT_HD GTri load_gtri(const GTri* p)
{
    const float4* q = reinterpret_cast<const float4*>(p);
    float4 a = ldg(q), b = ldg(q + 1), c = ldg(q + 2);
    GTri g;
    g.a[0] = a.x; g.a[1] = a.y; g.a[2] = a.z;
    g.ab[0] = a.w; g.ab[1] = b.x; g.ab[2] = b.y;
    g.ac[0] = b.z; g.ac[1] = b.w; g.ac[2] = c.x;
    g.n[0] = c.y; g.n[1] = c.z; g.n[2] = c.w;
    return g;
}

RT_HD GNode load_gnode(const GNode* p)
{
    const float4* q = reinterpret_cast<const float4*>(p);
    float4 a = ldg(q), b = ldg(q + 1), c = ldg(q + 2), d = ldg(q + 3);
    GNode g;
    g.dn[0] = a.x; g.dn[1] = a.y; g.dn[2] = a.z; g.dn[3] = a.w;
    g.dn[4] = b.x; g.dn[5] = b.y; g.dn[6] = b.z;
    g.df[0] = b.w; g.df[1] = c.x; g.df[2] = c.y; g.df[3] = c.z; g.df[4] = c.w;
    g.df[5] = d.x; g.df[6] = d.y;
    g.a = __builtin_bit_cast(uint32_t, d.z);
    g.b = __builtin_bit_cast(uint32_t, d.w);
    return g;
}

// sqrt within 1 ulp on the device (the hardware instruction), correctly rounded on the host; callers
// round up by far more than 1 ulp where they need an upper bound
RT_HD float fast_sqrt(float a)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_sqrtf(a);
#else
    return std::sqrt(a);
#endif
}

RT_HD float fast_rcp(float a)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcpf(a);
#elif defined(RT_TEST_RCP_HOOK)
    return RT_TEST_RCP_HOOK(a);   // tests/c/kdop_fast.cpp: a reciprocal a few ulps off
#else
    // host emulation: the correctly rounded reciprocal (the device's is within 1 ulp of it;
    // both stay inside the slab margin)
    return 1.0f / a;
#endif
}

// BoundingVolume::intersect (bvh.h:79-105) with the ray's plane products as
// OctreeNode::intersect computes them (bvh.h:216-223), branch-free as kernels.hip
// vol_test: returns pass && t_near <= t.
// Case (b)'s bound on the origin's distance from a triangle's plane: with q = |cos(n,
// d)| < QS, s = sin(alpha) (the angle at a), s2 = sin(alpha' / 2), L >= the edges, D >= |o - a| and u =
// 2^-24, a hit Moller-Trumbore reports (u', v' in [0, 1]; triangle.cpp:25-91) puts the origin within
//   H0 = 1.01 [QS (2L + D) + u (24.2 L + 48 D) / s + u (30 L + 12 D + 24 D / s) / s2]
// of the plane: for q s >= 24u the exact line-plane point P0 has barycentrics within 1 + (12.1u + 24u
// D / |e|) / (q s) of [0, 1] (numerator and Mdet rounding), so |P0 - a| <= 2L + u (24.2 L + 48 D) / (q s),
// and the distance is q |P0 - o| <= q (|P0 - a| + D); below, Mdet < 30u |ab||ac||d| bounds both
// barycentric numerators U = -alpha d.n - gamma d.(n x ac), V = -beta d.n + gamma d.(n x ab), and the
// larger of |d.(n x ab)| / |ab|, |d.(n x ac)| / |ac| is at least s2 |d|.  Device: the hardware
// reciprocal (1 ulp), inside the 1.01.
RT_HD float wq_h0(float QS, float L, float D, float s, float s2)
{
    constexpr float U = 0x1p-24f;
    const float is = fast_rcp(s), is2 = fast_rcp(s2);
    const float a = __builtin_fmaf(QS, 2.0f * L + D, U * __builtin_fmaf(24.2f, L, 48.0f * D) * is);
    return 1.01f * __builtin_fmaf(U * __builtin_fmaf(30.0f, L, __builtin_fmaf(24.0f, D * is, 12.0f * D)), is2, a);
}

RT_HD bool kdop_certifies_exact(const GNode& nd, v3 o, v3 d, float t)
{
    float t_near = -INFINITY, t_far = INFINITY;
#pragma unroll
    for (int i = 0; i < NPLANES; i++) {
        v3 n = mk(PLANE_N[i][0], PLANE_N[i][1], PLANE_N[i][2]);
        float den = dot(n, d);
        float num = dot(n, o);
        if (den == 0.0f)
            num = __builtin_nanf("");   // skipped plane (bvh.h:86-87): NaN quotients are ignored
        float d0 = (nd.dn[i] - num) / den;
        float d1 = (nd.df[i] - num) / den;
        t_near = fmaxf(t_near, fminf(d0, d1));
        t_far = fminf(t_far, fmaxf(d0, d1));
    }
    return !(t_far < t_near) && t_near <= t;
}

// The same decision, first from quotients through the hardware reciprocal (1 ulp): each is
// within 2^-21 of the correctly rounded one (relative), a max / min of them within 2^-21 of its
// exact counterpart's magnitude, so a comparison won by more than 2^-19 (|t_near| + |t_far| + |t|)
// is the exact comparison's.  Closer calls, a denominator below 2^-100 (reciprocal range) and
// infinite bounds take the correctly rounded divisions.  The numerators are the reference's.
RT_HD bool kdop_certifies(const GNode& nd, v3 o, v3 d, float t)
{
    float t_near = -INFINITY, t_far = INFINITY;
    bool tiny = false;
#pragma unroll
    for (int i = 0; i < NPLANES; i++) {
        v3 n = mk(PLANE_N[i][0], PLANE_N[i][1], PLANE_N[i][2]);
        float den = dot(n, d);
        float num = dot(n, o);
        if (den == 0.0f)
            num = __builtin_nanf("");
        tiny |= den != 0.0f && !(fabsf(den) >= 0x1p-100f);
        const float r = fast_rcp(den);
        float d0 = (nd.dn[i] - num) * r;
        float d1 = (nd.df[i] - num) * r;
        t_near = fmaxf(t_near, fminf(d0, d1));
        t_far = fminf(t_far, fmaxf(d0, d1));
    }
    const float e = (fabsf(t_near) + fabsf(t_far) + fabsf(t)) * 0x1p-19f;
    if (!tiny && fabsf(t_near) < INFINITY && fabsf(t_far) < INFINITY && e < INFINITY) {
        if (t_far - t_near > e && t - t_near > e)
            return true;
        if (t_near - t_far > e || t_near - t > e)
            return false;
    }
    return kdop_certifies_exact(nd, o, d, t);
}

RT_HD uint32_t fbits(float f) { return __builtin_bit_cast(uint32_t, f); }
RT_HD float bitsf(uint32_t u) { return __builtin_bit_cast(float, u); }

// Grazing risk of a triangle for a point X ("risk keys"): INFINITY when no ray of the
// kind X stands for can make the triangle report a hit in case (b) of wbvh_closest (|cos(n, d)| = q <
// QS); otherwise a key K >= 0 such that every hit it reports in case (b) has
//   t' >= (K - QS hi - nu) / (QS |d|)      (camera: t' >= K / (QS |d|)).
// Case (b) puts the ray's origin o within H0(D = |o - a|) of the triangle's plane (wq_h0; s2 =
// sin(alpha' / 2) as the build's ext byte 1, L = the longer edge).  And with s = sin(alpha)
// and u = 2^-24, Moller-Trumbore's float quantities (triangle.cpp:25-91; stored normal n within
// 2.83u |ab||ac| of the exact one) satisfy |Mdet| <= (q + 6u/s) |n~||d| and |n . OA| >= |n~| (dist(o) -
// cN |o - a|), cN = (6/s + 1.2)u, so a reported t' >= (dist(o) - cN |o - a|) / ((QS + 6u/s) |d|) (1 - 2.01u).
//   camera (G = 0, nu = 0): the rays start at X itself: K = (dist(X) - cN |X - a|) / f, f = 1 + 6u/(s QS);
//   light: the rays start at o with |X - o| <= hi <= G and their lines pass within nu of X, so
//          dist(o) >= dist(X) - QS hi - nu and |o - a| <= |X - a| + G: K = (dist(X) - cN (|X - a| + G)) / f;
//          X lies within H0(|X - a| + G) + QS G + nu of the plane when it is at risk at all.
// slack >= the query's box margin m for those rays.  In double from the record's float edges (the
// products exact, each difference rounded once); the key is rounded down to float (0 when negative).
// A degenerate record (no s2 bound) is always at risk with key 0, one whose stored normal is zero
// never (Mdet = 0: never a hit).
RT_HD float wbvh_risk_key(const GTri& t, double px, double py, double pz, double G, double nu, double slack, double QS)
{
    if (t.n[0] == 0.0f && t.n[1] == 0.0f && t.n[2] == 0.0f)
        return INFINITY;
    const double x0 = t.ab[0], x1 = t.ab[1], x2 = t.ab[2], y0 = t.ac[0], y1 = t.ac[1], y2 = t.ac[2];
    const double c0 = x1 * y2 - x2 * y1, c1 = x2 * y0 - x0 * y2, c2 = x0 * y1 - x1 * y0;
    const double la = sqrt(x0 * x0 + x1 * x1 + x2 * x2), lc = sqrt(y0 * y0 + y1 * y1 + y2 * y2);
    const double cl = sqrt(c0 * c0 + c1 * c1 + c2 * c2);
    if (!(la * lc > 0x1p-100) || !(cl > 0x1p-50 * la * lc))
        return 0.0f;

    const double ca = fabs(x0 * y0 + x1 * y1 + x2 * y2) / (la * lc);
    const double s2 = sqrt(fmax(0.0, (1.0 - fmin(1.0, ca + 1e-12)) / 2.0)) * (1 - 1e-9);
    const double sa = cl / (la * lc) * (1 - 1e-9);
    if (!(s2 > 0.0) || !(sa > 0.0))
        return 0.0f;
    const double ax = px - (double)t.a[0], ay = py - (double)t.a[1], az = pz - (double)t.a[2];
    const double Da = sqrt(ax * ax + ay * ay + az * az);
    const double dist = fabs(c0 * ax + c1 * ay + c2 * az) / cl;
    const double L = fmax(la, lc) * (1 + 1e-12);
    const double sa0 = cl / (la * lc);
    const double Dx = Da + G + slack, u = 0x1p-24;
    const double H0 = 1.01 * (QS * (2 * L + Dx) + u * (24.2 * L + 48 * Dx) / sa0 + u * (30 * L + 12 * Dx + 24 * Dx / sa0) / s2);
    const double rhs = (H0 + QS * G + nu) * (1 + 1e-6);
    if (dist > rhs)
        return INFINITY;
    if (!(dist <= rhs))
        return 0.0f;   // NaN
    const double cN = (6.0 / sa + 1.2) * 0x1p-24 * 1.01;
    const double K = (dist * (1 - 1e-9) - cN * (Da + G + slack)) / (1.0 + 6.0 * 0x1p-24 / (sa * QS)) * (1 - 1e-6);
    if (!(K > 0.0))
        return 0.0f;
    const float f = (float)K;
    return (double)f > K ? nextafterf(f, 0.0f) : f;
}

// Case (a)'s reach (r05, DESIGN.md 5.6 "The correlated bound"): how far a point Moller-Trumbore reports
// (triangle.cpp:25-91) can lie from its triangle T = (a, a + ab, a + ac), and from T's plane.  With u =
// 2^-24, N = ab x ac, s = |N| / (|ab| |ac|), q = cos(N, -d), L >= |ab|, |ac|, D >= |o - x| for every x of T,
// the computed m, Mdet, U = m.ac, V = -m.ab, T = n.OA carry errors dm, eM, eu, ev, eT (|n - N| <= 2.83u
// |ab||ac|, |dm| <= 3.84u |d| |o - a|, |eM| <= 3.01u |n||d|, |eu| <= 3.01u |m||ac|, |ev| <= 3.01u |m||ab|,
// |eT| <= 4.02u |n| |o - a|).  For P' = a + u' ab + v' ac (in T: u', v' were accepted) and p' = o + t' d,
// the identities U ab + V ac = m x N and (o - a) x d = M give
//   Mdet (p' - P') = -(n - N) x M + eM (o - a) + eT d - dm x N - eu ab - ev ac   (+ the final roundings),
// where |M| = |d| h, h = dist(a, line) <= L + |p' - P'|, and Mdet >= |d||N| G, G = q - 3.01u - 2.84u / s.
// So the D terms come with 1 / G only and 1 / s meets only L (the former bound had D / (q s)):
//   E = |p' - P'| <= [8.85u (L + E) / (s G) + 10.87u D / G + 43u^2 D / (s G) + 2.011u (D + E + L)]
// and, by Binet-Cauchy on Mdet (p' - a).N, the distance of p' from T's plane
//   eta <= [2.83u (L + E) / (s G) + (3.01 (D + E) + 4.02 D) u kq + 2.011u (D + E)] / (1 - 3.02u / G - 9u^2 / (s G))
// with kq = (1 + 2.83u / (s G))(1 + 5.85u / (s G)) >= (|n| / |N|)(q / G).  tests/c/wq_lemma.cpp checks both
// on 10^7 accepted hits (largest |p' - P'| / E 0.33, eta ratio 0.47).  Inputs: lower bounds smin <= s, qa
// <= q; G >= qa - 5.85u / smin.  wq_reach: E (INFINITY: no bound); wq_eta: eta.  Float evaluation: every
// constant is rounded up, every step a product or sum of non-negative terms (relative error a few u,
// inside the final 2^-16).
struct WReach {
    float E, isG, iG;   // the reach, >= 1 / (s G), >= 1 / G
};
RT_HD WReach wq_reach(float qa, float smin, float L, float D)
{
    constexpr float U = 0x1p-24f;
    WReach r;
    const float X = __builtin_fmaf(smin, qa, -5.86f * U);   // <= s G (one rounding)
    r.isG = X > 0.0f ? fast_rcp(X) * (1.0f + 0x1p-18f) : INFINITY;
    r.iG = smin * r.isG * (1.0f + 0x1p-20f);
    const float beta = __builtin_fmaf(8.86f * U, r.isG, 2.012f * U);
    // 1 / (1 - beta) <= 1 + 2 beta for beta <= 1/2
    const float num = U * __builtin_fmaf(8.86f, L * r.isG, __builtin_fmaf(10.88f, D * r.iG, __builtin_fmaf(43.1f * U, D * r.isG,
                                                                                                       2.012f * (D + L))));
    r.E = !(beta <= 0.5f) ? INFINITY : num * __builtin_fmaf(2.0f, beta, 1.0f) * (1.0f + 0x1p-16f);
    return r;
}
// The same error split into a lateral part and a part along d: p' - P' = lat + par, par parallel to d.
// Only the terms eT d, the d-component of eM (o - a) (o - a = (P' - a) + (p' - P') - t' d) and the final
// rounding of t' lie along d; so P' + lat, a point of the line, lies within Rlat of T (the line crosses
// the box widened by Rlat) and p' lies within Rpar of it along the line:
//   Rlat <= 8.85u (L + E) / (s G) + 3.01u kn (L + E) / G + 3.84u D / G + 23.2u^2 D / (s G) + 2.012u L,
//   Rpar <= (4.02 D + 3.01 (D + E)) u kn / G + 2.011u (D + E),   kn = 1 + 2.83u / (s G) >= |n| / |N|.
// The D / q term of the lateral reach is 3.84u D / G against 10.87u D / G for E (tests/c/wq_lemma.cpp:
// largest lat / Rlat 0.38).
RT_HD void wq_split(const WReach& r, float L, float D, float& Rlat, float& Rpar)
{
    constexpr float U = 0x1p-24f;
    const float E = r.E;
    const float kn = __builtin_fmaf(2.84f * U, r.isG, 1.0f);
    const float LE = (L + E) * (1.0f + 0x1p-22f);
    Rlat = U * __builtin_fmaf(8.86f * LE, r.isG,
                              __builtin_fmaf(__builtin_fmaf(3.03f * LE, kn, 3.85f * D), r.iG,
                                             __builtin_fmaf(23.3f * U * D, r.isG, 2.013f * L))) * (1.0f + 0x1p-16f);
    Rpar = U * __builtin_fmaf(__builtin_fmaf(4.03f, D, 3.02f * (D + E)) * kn, r.iG, 2.012f * (D + E)) * (1.0f + 0x1p-16f);
}

RT_HD float wq_eta(const WReach& r, float L, float D)
{
    constexpr float U = 0x1p-24f;
    const float E = r.E;
    const float kq = __builtin_fmaf(2.84f * U, r.isG, 1.0f) * __builtin_fmaf(5.86f * U, r.isG, 1.0f);
    const float x = __builtin_fmaf(3.03f * U, r.iG, 9.1f * U * U * r.isG);   // <= 0.17 when E is finite
    const float n2 = U * __builtin_fmaf(2.85f * (L + E), r.isG,
                                        __builtin_fmaf(__builtin_fmaf(3.02f, D + E, 4.03f * D), kq, 2.012f * (D + E)));
    return n2 * __builtin_fmaf(2.0f, x, 1.0f) * (1.0f + 0x1p-16f);
}

// A frame's two risk points (kernels.hip wide_risk_kernel): sel 0 the camera (rays start at it), sel
// 1 the light (shadow rays: o = p + 1e-4 n, d = normalize(light - p), renderer.cpp:340-402, for hit
// points p in the scene box [lo, hi]).  The shadow rays that may use the light's keys are the ones
// whose segment bound hi (kernels.hip is_shadowed, >= |light - o|) is <= ray_G and whose normal has
// |n|_1 <= ray_nl: their lines pass within nu = 1.001e-4 ray_nl + 16u G of the light (the offset
// and normalize's rounding; ray_nu: nu rounded up).  slack >= the query's margin m for the kind's
// origins.
struct WRiskArgs {
    double p[2][3];
    double G[2], nu[2], slack[2], QS[2];
    int32_t on[2];
    float ray_G, ray_nl, ray_nu;
};

inline WRiskArgs wbvh_risk_args(const float lo[3], const float hi[3], float S, const float cam[3], const float light[3],
                                float qs_cam, float qs_light)
{
    WRiskArgs A{};
    double cm = 0, lm = 0, gc = 0;
    for (int a = 0; a < 3; a++) {
        A.p[0][a] = cam[a];
        A.p[1][a] = light[a];
        cm = std::max(cm, std::fabs((double)cam[a]));
        lm = std::max(lm, std::fabs((double)light[a]));
    }
    for (int c = 0; c < 8; c++) {
        double g = 0;
        for (int a = 0; a < 3; a++) {
            const double x = ((c >> a) & 1) ? hi[a] : lo[a];
            g += (x - light[a]) * (x - light[a]);
        }
        gc = std::max(gc, std::sqrt(g));
    }
    A.ray_nl = 2.0f;
    const double G = 1.01 * (gc + 1e-4 * A.ray_nl) + 0x1p-10 * (S + lm);
    A.ray_G = std::nextafter((float)G, 0.0f);
    A.G[0] = 0.0;
    A.nu[0] = 0.0;
    A.slack[0] = 1.01 * 0x1p-16 * (cm + S);
    A.QS[0] = qs_cam;
    A.G[1] = G;
    A.nu[1] = 1.001e-4 * A.ray_nl + 16.0 * 0x1p-24 * G;
    A.ray_nu = std::nextafter((float)(A.nu[1] * (1 + 1e-6)), INFINITY);
    A.slack[1] = 1.01 * 0x1p-16 * (lm + G + S);
    A.QS[1] = qs_light;
    const bool fin = std::isfinite(cm) && std::isfinite(lm) && std::isfinite(G);
    A.on[0] = A.on[1] = fin ? 1 : 0;
    return A;
}

// The risk cap of a frame's point X (camera or light): s <= |cos(N, c)| for the exact normal N of every
// triangle at risk for X's rays (wbvh_risk_key < INFINITY), c a unit direction (from X towards the scene).
// A ray of X's kind at angle g to the line of c has, for each of them, |cos(N, d)| >= s cos g - sqrt(1 -
// s^2) sin g (N = a c + b e with |a| >= s, e normal to c): when that is >= QS (plus a margin over the float
// evaluation) none of them is in case (b) for the ray, and the others cannot report there (their key is
// INFINITY), so the query skips case (b).  For a convex object seen from X the at-risk triangles are its
// silhouette, whose normals are all at 90 degrees + the silhouette's angle from the direction to its
// centre: every ray into the silhouette's interior skips.
RT_HD bool risk_cap_skip(float s, const float c[3], v3 d, float QS)
{
    const float dl = sqrtf(d.x * d.x + d.y * d.y + d.z * d.z);
    const float cg = fabsf(c[0] * d.x + c[1] * d.y + c[2] * d.z) / dl;
    const float x = c[1] * d.z - c[2] * d.y, y = c[2] * d.x - c[0] * d.z, z = c[0] * d.y - c[1] * d.x;
    const float sg = sqrtf(x * x + y * y + z * z) / dl;
    return s * cg - sqrtf(fmaxf(0.0f, 1.0f - s * s)) * sg >= QS + 0x1p-14f;
}
// A triangle's lower bound on |cos(N, c)| (risk_cap_skip), in double from the record's float edges; 0 for
// a degenerate record (no normal: it counts as at risk for every ray)
RT_HD float risk_cap_tri(const GTri& t, const double c[3])
{
    const double x0 = t.ab[0], x1 = t.ab[1], x2 = t.ab[2], y0 = t.ac[0], y1 = t.ac[1], y2 = t.ac[2];
    const double c0 = x1 * y2 - x2 * y1, c1 = x2 * y0 - x0 * y2, c2 = x0 * y1 - x1 * y0;
    const double la = sqrt(x0 * x0 + x1 * x1 + x2 * x2), lc = sqrt(y0 * y0 + y1 * y1 + y2 * y2);
    const double cl = sqrt(c0 * c0 + c1 * c1 + c2 * c2);
    if (!(la * lc > 0x1p-100) || !(cl > 0x1p-50 * la * lc) || !(cl < INFINITY))
        return 0.0f;
    const double v = fabs(c0 * c[0] + c1 * c[1] + c2 * c[2]) / cl - 1e-9;
    if (!(v > 0.0))
        return 0.0f;
    const float f = (float)v;
    return (double)f > v ? nextafterf(f, 0.0f) : f;
}

// rsub of wbvh_closest for a shadow ray with |light - o| <= h (rounded up)
RT_HD float wrisk_sub(float QS, float h, float nu)
{
    return __builtin_fmaf(QS, h, nu) * (1.0f + 0x1p-20f);
}

// The per-point risk words of the wide BVH, one 64-bit word per child (risk[(2 node + sel) 4 + j]):
// bits 0-47 = the box of the octree leaves holding its at-risk triangles (the reference tests such a
// triangle only where the line crosses its leaf's k-DOP, inside that box), quantised like the child
// boxes against the node's frame (6 bytes: lo x y z, hi x y z; lo rounded down, hi up, clamped to the
// frame: the box lies within rho of the child's, so the decoded box widened by rho holds it), bits
// 48-63 = the smallest key (wbvh_risk_key) of them as a bfloat16 rounded down (INFINITY: none at risk).
RT_HD uint64_t wrisk_pack(float K, uint64_t box48)
{
    return ((uint64_t)(fbits(K) >> 16) << 48) | (box48 & 0xFFFFFFFFFFFFull);
}
RT_HD float wrisk_key(uint64_t w)
{
    return bitsf((uint32_t)(w >> 48) << 16);
}
// the 6 bytes of a float box [lo, hi] against a node's frame (origin, power-of-two steps)
RT_HD uint64_t wrisk_qbox(const WNode& nd, const float lo[3], const float hi[3])
{
    const double org[3] = {nd.ox, nd.oy, nd.oz};
    uint64_t q = 0;
    for (int a = 0; a < 3; a++) {
        const double st = ldexp(1.0, (int)((nd.exps >> (8 * a)) & 0xffu) - 127);
        const double l = floor(((double)lo[a] - org[a]) / st), h = ceil(((double)hi[a] - org[a]) / st);
        const uint64_t ql = (uint64_t)fmin(255.0, fmax(0.0, l)), qh = (uint64_t)fmin(255.0, fmax(0.0, h));
        q |= ql << (8 * a);
        q |= qh << (8 * (a + 3));
    }
    return q;
}

// Host version of kernels.hip wide_risk_kernel (tests, rt_wbvh_query_ex): a triangle's key and its
// octree leaf's axis box go up its leaf entry's parent chain (minimum, union), stopping where both are
// already there (aggregates over subtrees: what an entry holds its ancestors hold too).  leaf_box:
// per wide-BVH triangle, its octree leaf's axis box (lo xyz, hi xyz).
inline void wbvh_risk_host(const WBvh& w, const std::vector<float>& leaf_box, const WRiskArgs& A, int sel,
                           std::vector<uint64_t>& risk)
{
    risk.resize(w.nodes.size() * 8, wrisk_pack(INFINITY, 0));
    const size_t ne = w.nodes.size() * 4;
    std::vector<float> K(ne, INFINITY), B(ne * 6);
    for (size_t i = 0; i < ne; i++)
        for (int a = 0; a < 3; a++) {
            B[6 * i + a] = INFINITY;
            B[6 * i + 3 + a] = -INFINITY;
        }
    if (!A.on[sel]) {   // no bound: every child at risk, key 0, its whole frame
        for (size_t v = 0; v < w.nodes.size(); v++)
            for (int j = 0; j < 4; j++)
                risk[(2 * v + sel) * 4 + j] = wrisk_pack(0.0f, 0xFFFFFF000000ull);
        return;
    }
    for (size_t k = 0; k < w.tris.size(); k++) {
        const float Kt = wbvh_risk_key(w.tris[k], A.p[sel][0], A.p[sel][1], A.p[sel][2], A.G[sel], A.nu[sel],
                                       A.slack[sel], A.QS[sel]);
        if (!(Kt < INFINITY))
            continue;
        const float* lb = &leaf_box[6 * k];
        uint32_t e = w.tri_leaf[k];
        while (e != W_EMPTY) {
            const size_t i = (size_t)(e >> 2) * 4 + (e & 3u);
            float* b = &B[6 * i];
            const bool has = K[i] <= Kt && b[0] <= lb[0] && b[1] <= lb[1] && b[2] <= lb[2] && b[3] >= lb[3] &&
                             b[4] >= lb[4] && b[5] >= lb[5];
            if (has)
                break;
            K[i] = std::min(K[i], Kt);
            for (int a = 0; a < 3; a++) {
                b[a] = std::min(b[a], lb[a]);
                b[3 + a] = std::max(b[3 + a], lb[3 + a]);
            }
            e = w.parent[e >> 2];
        }
    }
    for (size_t v = 0; v < w.nodes.size(); v++)
        for (int j = 0; j < 4; j++) {
            const size_t i = v * 4 + j;
            risk[(2 * v + sel) * 4 + j] = K[i] < INFINITY ? wrisk_pack(K[i], wrisk_qbox(w.nodes[v], &B[6 * i], &B[6 * i + 3]))
                                                          : wrisk_pack(INFINITY, 0);
        }
}

// Checks a frame's risk words of point sel (host or GPU-computed) against the tree (CPU tests,
// rt_risk_words): for every triangle with a finite key (wbvh_risk_key), every entry on its leaf's
// parent chain must hold a key <= it and an at-risk box that, widened by the entry's rho, holds the
// triangle's octree leaf (what wbvh_closest's case (b) relies on).  Returns the number of violations.
int64_t check_risk_words(const FlatOctree& oct, const WBvh& w, const WRiskArgs& A, int sel, const uint64_t* risk);

// W_DEEP: not certified only because the stack overflowed (callers may retry with a deeper stack)
// W_LONG: stopped after max_steps loop iterations (the caller defers the query to a later pass)
enum WStatus : int { W_MISS = 0, W_HIT = 1, W_UNCERT = 2, W_DEEP = 3, W_LONG = 4 };
constexpr int W_DEEP_STACK = 64;   // the retry's stack (private memory, kernels.hip wide_closest_deep)

struct WHit {
    float t, u, v;
    int32_t k;   // wide-BVH triangle index (W_HIT)
};

// A lane's traversal stack: entry (child link, entry t); CAP entries.
template <int N>
struct WStackArr {
    static constexpr int CAP = N;
    uint2 e[N];
    RT_HD void put(int i, uint2 v) { e[i] = v; }
    RT_HD uint2 get(int i) const { return e[i]; }
};
using WStackLocal = WStackArr<W_STACK>;   // host

// A lane group: G adjacent lanes of a wave (lanes g0 .. g0 + G - 1, g0 a multiple of G) trace one ray
// together (wbvh_closest<Stack, G>, kernels.hip trace_split_part and refl_trace_long_kernel).  Device only; on the host
// (G = 1) these are the identity.
template <int G>
RT_HD uint32_t wg_lane()
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __lane_id() & (uint32_t)(G - 1);
#else
    return 0u;
#endif
}
// the group's lanes where p holds (bit i: group lane i)
template <int G>
RT_HD uint32_t wg_bits(bool p)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return (uint32_t)(__ballot(p) >> (__lane_id() & ~(uint32_t)(G - 1))) & ((1u << G) - 1u);
#else
    return p ? 1u : 0u;
#endif
}
#if defined(__HIP_DEVICE_COMPILE__)
// a 32-bit value from the lane the DPP quad permutation names (within each group of 4 lanes; all active)
template <int PERM>
__device__ __forceinline__ uint32_t wg_quad(uint32_t x)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, PERM, 0xF, 0xF, false);
}
#endif
template <int G>
RT_HD float wg_min(float x)
{
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (G <= 4) {   // DPP quad permutations (lane ^ 1, lane ^ 2), no LDS round trip
        x = fminf(x, __uint_as_float(wg_quad<0xB1>(__float_as_uint(x))));
        if (G == 4)
            x = fminf(x, __uint_as_float(wg_quad<0x4E>(__float_as_uint(x))));
    } else {
        for (int m = 1; m < G; m <<= 1)
            x = fminf(x, __shfl_xor(x, m));
    }
#endif
    return x;
}
// x of group lane i (i may differ per lane)
template <int G, class T>
RT_HD T wg_read(T x, int i)
{
    static_assert(sizeof(T) == 4, "32-bit values");
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (G <= 4) {   // the group's G values by DPP quad broadcasts, then a select
        uint32_t u;
        __builtin_memcpy(&u, &x, 4);
        uint32_t r;
        if (G == 4) {   // quad lane 0 / 1 / 2 / 3 to every lane of the quad
            const uint32_t b0 = wg_quad<0x00>(u), b1 = wg_quad<0x55>(u), b2 = wg_quad<0xAA>(u), b3 = wg_quad<0xFF>(u);
            r = i == 0 ? b0 : i == 1 ? b1 : i == 2 ? b2 : b3;
        } else {        // pairs: (0, 0, 2, 2) and (1, 1, 3, 3)
            const uint32_t b0 = wg_quad<0xA0>(u), b1 = wg_quad<0xF5>(u);
            r = i == 0 ? b0 : b1;
        }
        T y;
        __builtin_memcpy(&y, &r, 4);
        return y;
    } else {
        return __shfl(x, (int)(__lane_id() & ~(uint32_t)(G - 1)) + i);
    }
#else
    (void)i;
    return x;
#endif
}

// Closest hit over the wide BVH for the ray (o, d) among hits with t <= hi.  m: box margin
// (2^-16 (max|o| + scene scale), the leaf-slab margin of kernels.hip leaf_missed).
// Returns W_MISS (no triangle reports a hit at t <= hi), W_HIT (h = the minimum-t hit, finite
// and > 0, unique when ties: still to be certified by kdop_certifies on its octree leaf) or
// W_UNCERT (W_DEEP when only the stack overflowed).  Shadow queries (hi = the segment end of kernels.hip is_shadowed, ties false) read
// only the record's t.  work (optional, 4 entries): {nodes, triangles} added, [2] = the reasons
// a query is not certified, [3] = loop iterations added.
//
// The query is sound for every ray: a child is skipped only when no triangle
// below it can REPORT a hit (Moller-Trumbore's rounded t, u, v; triangle.cpp:25-91) that the
// reference could record at t <= the best hit so far.  With q = |cos(n, d)| of a triangle, s =
// sin(alpha), u = 2^-24 and D >= |o - a| (the node frame's farthest corner):
//   (a) every reported point p' lies within R = wq_reach's E of its triangle (r05: D / q and L / (q s)
//       terms, L the longest edge) and within eta (wq_eta) of its plane,
//       which is tilted by theta from the child's slab normal: the child's box widened by R and
//       its slab widened by eta + R sin(theta) hold p' (q is bounded below by the cone: q >=
//       cos(phi) - sin(theta) (1 + sin(theta)), phi the angle between N and -d);
//   (b) for the triangles with q < QS that bound is not used: their reported points can lie
//       anywhere on their plane, but the origin is then within H0 (wq_h0) of
//       that plane (the barycentric numerators must be small), and the reference tests such a
//       triangle only where the line crosses its octree leaf's k-DOP (inside the child box
//       widened by rho).  A child passing both is entered, keyed by its risk key's t bound (0
//       without risk keys).
// Robustly back-facing children (the cone) report nothing and are skipped as before.
// nob: no triangle with q < QS can report a hit for this ray (ocone.hpp ocone_skip, the origin cones),
// so case (b) is skipped (with or without risk words).
// risk (optional): the risk words of the ray's kind rsel (wrisk_pack / wbvh_risk_host / kernels.hip
// wide_risk_kernel): a child whose key is INFINITY holds no triangle that can report a hit in case (b)
// for this ray; its (b) triangles lie in octree leaves inside its at-risk box (so the line must cross
// that box, widened by rho), and none of their reports has t' below (key - rsub) / (QS |d|), so (b) is
// skipped for it when that exceeds the best hit.  rsub: 0 for the camera (rsel 0); for the light (rsel 1), at least
// QS h + nu with h >= |light - o| and nu the frame's (WRiskArgs::ray_nu; wrisk_sub).  The caller
// guarantees the ray is of that kind.
//
// G > 1 (device, Stack = kernels.hip WStackLds, max_steps 0): the G lanes of a lane group (wg_lane)
// hold the same ray and walk its tree together.  Group lane 0 starts at the root, the others idle; after
// every step the group shares its best hit bound (best_s, the minimum over the group), and each idle lane
// takes the bottom entry of a busy lane's stack (the stack is then a ring [bot, sp): pushes and pops at
// sp, steals at bot; the i-th idle lane in lane order takes from the i-th lane with entries).  Every
// child pushed is visited by one lane or skipped because its key exceeds the group's best (never below
// the final best: skipped soundly), so the group's lanes together test every triangle the G = 1 query
// would need; the answer (minimum over the lanes' records, a tie when two lanes hold it or one lane saw
// two) is the same on every lane of the group.
// No lane refill (the default): one query per call.
struct WNoFeed {
    static constexpr bool on = false;
    bool busy = false;
    bool drained = true;   // (wave-uniform) the feed has no query left to hand out
    int threshold = 64;
    template <class H> RT_HD void finish(int, H&, v3, v3) {}
    RT_HD bool fetch(bool, v3&, v3&, float&, float&, const uint64_t*&, float&, bool&) { return false; }
};

template <class Stack, int G = 1, class Feed = WNoFeed>
RT_HD int wbvh_closest(const WNode* nodes, const GTri* tris, v3 o, v3 d, float m, Stack& stk, WHit& h,
                       uint32_t* work = nullptr, float hi = INFINITY, bool ties = true, float QS = 0x1p-8f,
                       const uint64_t* risk = nullptr, int rsel = 0, float rsub = 0.0f, uint32_t max_steps = 0,
                       Feed* feed = nullptr, bool nob = false)
{
    static_assert(G == 1 || ((G & (G - 1)) == 0 && G <= 8 && (Stack::CAP & (Stack::CAP - 1)) == 0),
                  "a lane group: a power of two up to 8 lanes, a ring stack of 2^k entries");
    static_assert(G == 1 || !W_STEP_CAP, "a lane group leaves the loop together");
    // Feed::on (device, one lane per query): lane refill.  The wave stays in the loop; a lane whose query
    // ended waits, and when at least feed->threshold lanes (or every lane) wait, each hands its query's
    // status and record to feed->finish and takes the next ray from feed->fetch (o, d, m, hi, the risk
    // words, rsub and nob, which it may leave as they are; ties, QS and rsel are the same for every query of
    // the feed).  The per-query work is the one-query
    // call's: the same state, reset per query, the same steps.  Returns W_MISS once the feed is drained.
    constexpr bool FEED = Feed::on;
    static_assert(!FEED || (G == 1 && !W_STEP_CAP), "lane refill: one lane per query");
    // the stack index of entry i (a ring in a lane group)
    auto slot = [](int i) { return G > 1 ? (i & (Stack::CAP - 1)) : i; };
    h.t = INFINITY;
    h.u = 1.0f;
    h.v = 0.0f;
    h.k = -1;
    // slab parameters: t = (lo - (o + M)) / d and (hi - (o - M)) / d over the box widened by M.
    // A direction component below 2^-100 in magnitude (or 0) is treated as +-2^-100: the
    // slab's t range then exceeds 2^70 m / |d| on the far side, far beyond the scene's, so
    // it constrains only as much as the true one does (the margin covers the origin's side).
    const float DMIN = 0x1p-100f;
    constexpr float SL = 0x1p-20f;   // relative slack over the rounding of a slab parameter (<= 3 ulp)
    constexpr float NLH = 127.9f;    // |N| of a quantised slab normal: 127 +- sqrt(3) / 2 (wbvh.cpp quantise)
    float ix, iy, iz, aix, aiy, aiz, dl, cstep, idl, icp, iqd;
    bool nx_lo, ny_lo, nz_lo;
    auto setup = [&]() {
        ix = 1.0f / (fabsf(d.x) < DMIN ? copysignf(DMIN, d.x) : d.x);
        iy = 1.0f / (fabsf(d.y) < DMIN ? copysignf(DMIN, d.y) : d.y);
        iz = 1.0f / (fabsf(d.z) < DMIN ? copysignf(DMIN, d.z) : d.z);
        // per axis, the byte row of the entry (near) planes: q_lo where the direction is positive,
        // q_hi where it is negative; the near plane is widened by -M sign(d), the far one by +M sign(d)
        nx_lo = !(ix < 0.0f);
        ny_lo = !(iy < 0.0f);
        nz_lo = !(iz < 0.0f);
        aix = fabsf(ix);
        aiy = fabsf(iy);
        aiz = fabsf(iz);
        // |d| rounded up (sqrt and dot within 2^-22), times the cone step: threshold = c * cstep
        dl = sqrtf(d.x * d.x + d.y * d.y + d.z * d.z) * (1.0f + 0x1p-20f);
        cstep = dl * W_CONE_STEP;
        // 1 / |d| rounded up (|d| rounded down, the hardware reciprocal within 1 ulp)
        idl = fast_rcp(sqrtf(d.x * d.x + d.y * d.y + d.z * d.z) * (1.0f - 0x1p-20f)) * (1.0f + 0x1p-18f);
        icp = (1.0f - 0x1p-18f) / (NLH * dl);   // cos(angle(N, -d)) >= -a icp
        iqd = (1.0f - 0x1p-20f) / (QS * dl);    // a risk key's t bound: key / (QS |d|)
    };
    setup();
    float best_s = hi + fabsf(hi) * SL;   // h.t (or hi) plus slack: a child entered at or below it may hold a hit
    bool tie = false, nanhit = false, infhit = false;
    float dropped = INFINITY;   // the smallest key of the children a full stack could not take
    int sp = 0, bot = 0;        // the stack's entries [bot, sp) (bot > 0: entries taken by the group)
    uint32_t cur = FEED || (G > 1 && wg_lane<G>() != 0) ? W_EMPTY : 0u;   // root node (FEED: no query yet)
    uint32_t nn = 0, nt = 0;
    uint32_t steps = 0;   // loop iterations (node or leaf visits)
    // the status of the lane's query once its loop is over (G = 1; the tail below for every G)
    auto status = [&]() -> int {
        const bool ovf = dropped < INFINITY && dropped <= best_s;
        if (nanhit)
            return W_UNCERT;
        if (h.k < 0) {
            if (infhit)
                return W_UNCERT;
            if (ovf)
                return W_DEEP;
            h.t = -1.0f;   // HitInfo() (hitInfo.h:8-24): t = -1, u = 1, v = 0
            return W_MISS;
        }
        if ((ties && tie) || !(h.t > 0.0f && h.t < INFINITY))
            return W_UNCERT;
        return ovf ? W_DEEP : W_HIT;
    };
    // FEED: at the loop's head, with the wave together; false once the feed is drained and no lane runs
    (void)status;
    auto refill = [&]() -> bool {
        if constexpr (FEED) {
#if defined(__HIP_DEVICE_COMPILE__)
            const bool idle_lane = cur == W_EMPTY;
            const uint64_t idle = __ballot(idle_lane);
            if (idle != 0ull && (idle == __ballot(1) || __popcll(idle) >= feed->threshold)) {
                if (idle_lane && feed->busy)
                    feed->finish(status(), h, o, d);
                if (feed->fetch(idle_lane, o, d, m, hi, risk, rsub, nob)) {   // (wave-uniform call; true for the lanes given a ray)
                    setup();
                    h.t = INFINITY;
                    h.u = 1.0f;
                    h.v = 0.0f;
                    h.k = -1;
                    best_s = hi + fabsf(hi) * SL;
                    tie = nanhit = infhit = false;
                    dropped = INFINITY;
                    sp = bot = 0;
                    cur = 0u;
                }
                return __ballot(cur != W_EMPTY) != 0ull || !feed->drained;
            }
#endif
        }
        return true;
    };
    while (FEED ? refill() : (G > 1 ? wg_bits<G>(cur != W_EMPTY) != 0u : cur != W_EMPTY)) {
        if constexpr (FEED) {
            if (cur == W_EMPTY)
                continue;   // (waits for the refill)
        }
        ++steps;
        if (max_steps && steps > max_steps)
            return W_LONG;
#if W_STEP_CAP
        if (steps > W_STEP_CAP) {   // a very long query: the exact octree walk instead
            nanhit = true;
            break;
        }
#endif
        // ---- inner nodes: test the four child boxes, go to the nearest, push the others ----
        // if-if: every lane takes one step (inner node or leaf) per iteration
        if (!(cur & W_LEAF)) {
            nn++;
            W_DIAG_ADD(0, 1);
            W_STEP_HOOK(cur, 0);
            const uint4* p = reinterpret_cast<const uint4*>(nodes + cur);
#if W_LAZY_EXT2
            // every row but the last (ext2: rho, read by case (b) alone, per lane when it runs)
            constexpr int NR = WN_EXT2 / 4;
            static_assert(WN_EXT2 % 4 == 0 && NR == WN_ROWS - 1, "ext2 is the node's last row");
#else
            constexpr int NR = WN_ROWS;
#endif
            uint4 Rw[NR];
#pragma unroll
            for (int i = 0; i < NR; i++)
                Rw[i] = ldg(p + i);
            // word i of the node (compile-time i)
            auto wd = [&](int i) -> uint32_t {
                const uint4 r = Rw[i >> 2];
                return (i & 3) == 0 ? r.x : (i & 3) == 1 ? r.y : (i & 3) == 2 ? r.z : r.w;
            };
            const float ss = bitsf(wd(WN_SS)), slo = bitsf(wd(WN_SS + 1));
            const uint32_t ex = wd(3);
            const float stx = bitsf((ex & 0xffu) << 23), sty = bitsf(((ex >> 8) & 0xffu) << 23),
                        stz = bitsf(((ex >> 16) & 0xffu) << 23);
            // t of a plane origin + q s (widened by M) = q (s / d) + (origin - o -+ M) / d
            const float sx = stx * ix, sy = sty * iy, sz = stz * iz;
            const float Dx = bitsf(wd(0)) - o.x, Dy = bitsf(wd(1)) - o.y, Dz = bitsf(wd(2)) - o.z;
            const float bx = Dx * ix, by = Dy * iy, bz = Dz * iz;
            // per axis, the byte rows of the entry (near) and exit (far) planes: q_lo where the direction
            // is positive, q_hi where it is negative (one select per node and row)
            constexpr int QW = W_WIDTH / 4;   // words per axis row of quantised planes
            uint32_t nwx[QW], fwx[QW], nwy[QW], fwy[QW], nwz[QW], fwz[QW];
#pragma unroll
            for (int jw = 0; jw < QW; jw++) {
                const uint32_t lx = wd(WN_QLO + 0 * QW + jw), hx = wd(WN_QHI + 0 * QW + jw);
                const uint32_t ly = wd(WN_QLO + 1 * QW + jw), hy = wd(WN_QHI + 1 * QW + jw);
                const uint32_t lz = wd(WN_QLO + 2 * QW + jw), hz = wd(WN_QHI + 2 * QW + jw);
                nwx[jw] = nx_lo ? lx : hx;
                fwx[jw] = nx_lo ? hx : lx;
                nwy[jw] = ny_lo ? ly : hy;
                fwy[jw] = ny_lo ? hy : ly;
                nwz[jw] = nz_lo ? lz : hz;
                fwz[jw] = nz_lo ? hz : lz;
            }
            // D: o to the farthest corner of the node's frame [origin, origin + 255 step]
            float Dn;
            {
                const float fx = fmaxf(fabsf(Dx), fabsf(__builtin_fmaf(255.0f, stx, Dx)));
                const float fy = fmaxf(fabsf(Dy), fabsf(__builtin_fmaf(255.0f, sty, Dy)));
                const float fz = fmaxf(fabsf(Dz), fabsf(__builtin_fmaf(255.0f, stz, Dz)));
                Dn = fast_sqrt(fx * fx + fy * fy + fz * fz) * (1.0f + 0x1p-16f) + m;
            }
            // the children's risk words for this ray's kind (wrisk_pack): key and at-risk box
            uint32_t rw[2 * W_WIDTH];
            if (risk) {
                const uint4* rp = reinterpret_cast<const uint4*>(risk + (2 * (size_t)cur + rsel) * W_WIDTH);
                const uint4 r0 = ldg(rp), r1 = ldg(rp + 1);
                rw[0] = r0.x; rw[1] = r0.y; rw[2] = r0.z; rw[3] = r0.w;
                rw[4] = r1.x; rw[5] = r1.y; rw[6] = r1.z; rw[7] = r1.w;
            } else {
#pragma unroll
                for (int i = 0; i < 2 * W_WIDTH; i++)
                    rw[i] = 0u;   // key 0 (unused: the full test runs)
            }
            float key[W_WIDTH];
            uint32_t ref[W_WIDTH];
#if W_PRIO_ORDER
            float pri[W_WIDTH];   // visiting order (key: the cull bound kept on the stack)
#endif
#pragma unroll
            for (int j = 0; j < W_WIDTH; j++) {
                const int sh = 8 * (j & 3), jw = j >> 2;
                const uint32_t chj = wd(WN_CHILD + j);
                ref[j] = chj;
                key[j] = INFINITY;
#if W_PRIO_ORDER
                pri[j] = INFINITY;
#endif
                const uint32_t nrj = wd(WN_NRM + j);
                const float nx = (float)(int8_t)(nrj & 0xffu), ny = (float)(int8_t)((nrj >> 8) & 0xffu),
                            nz = (float)(int8_t)((nrj >> 16) & 0xffu);
                const float a = nx * d.x + ny * d.y + nz * d.z;
                // every triangle below faces away when a exceeds the cone threshold (rounding of
                // a and of the threshold: < 1e-4 |d|, inside the build's 0.01 |d|): none reports a hit
                if (chj != W_EMPTY && !(a > (float)(nrj >> 24) * cstep)) {
                    const uint32_t e = wd(WN_EXT + j);
                    const float smin = fmaxf(wq_val_nz(e & 0xffu, WQ_UNIT), W_SMIN_FLOOR);
                    const float sth = wq_val_nz((e >> 16) & 0xffu, WQ_UNIT);
                    const float L = (e >> 24) == 255u ? INFINITY : wq_val_nz(e >> 24, WQ_LEN);
                    const float qlb = __builtin_fmaf(-sth, 1.0f + sth, -a * icp) - 0x1p-20f;
                    const float qa = fmaxf(qlb, QS);
                    const float qnx = (float)((nwx[jw] >> sh) & 0xffu), qfx = (float)((fwx[jw] >> sh) & 0xffu);
                    const float qny = (float)((nwy[jw] >> sh) & 0xffu), qfy = (float)((fwy[jw] >> sh) & 0xffu);
                    const float qnz = (float)((nwz[jw] >> sh) & 0xffu), qfz = (float)((fwz[jw] >> sh) & 0xffu);
                    // D for case (b) (and (a), W_A_CHILD_D): o to the farthest corner of child j's box (it holds the child's
                    // vertices; Dn's frame can be several times larger, and near the origin (b) is priced
                    // by D sin(theta))
                    auto dchild = [&]() -> float {
#if W_B_CHILD_D
                        const float fx = fmaxf(fabsf(__builtin_fmaf(qnx, stx, Dx)), fabsf(__builtin_fmaf(qfx, stx, Dx)));
                        const float fy = fmaxf(fabsf(__builtin_fmaf(qny, sty, Dy)), fabsf(__builtin_fmaf(qfy, sty, Dy)));
                        const float fz = fmaxf(fabsf(__builtin_fmaf(qnz, stz, Dz)), fabsf(__builtin_fmaf(qfz, stz, Dz)));
                        return fast_sqrt(fx * fx + fy * fy + fz * fz) * (1.0f + 0x1p-16f) + m;
#else
                        return Dn;
#endif
                    };
                    // (a): the box widened by R, the slab by eta + R sin(theta) (wq_reach: the correlated bound of
                    // Moller-Trumbore's reports, D = Dn)
#if W_SOUND_A
                    const float Da = W_A_CHILD_D ? dchild() : Dn;
                    const WReach wr = wq_reach(qa, smin, L, Da);
                    const float R = __builtin_fmaf(W_R_SCALE, wr.E, m);
                    // the box test: the line crosses the box widened by the lateral reach, and a report lies
                    // within Rpar of that crossing along the line (wq_split)
                    float Rlat, Rpar;
                    wq_split(wr, L, Da, Rlat, Rpar);
                    const float Rb = __builtin_fmaf(W_R_SCALE, Rlat, m);
                    const float dtp = W_R_SCALE * Rpar * idl;
#else
                    const float R = m, Rb = m, dtp = 0.0f;   // (timing only)
#endif
                    // the entry / exit planes' t of this child's box widened by M:
                    // q (s / d) + (origin - o) / d -+ M / |d| per axis
                    auto box = [&](float M, float& tmin, float& tmax) {
                        const float tnx = __builtin_fmaf(-M, aix, __builtin_fmaf(qnx, sx, bx));
                        const float tny = __builtin_fmaf(-M, aiy, __builtin_fmaf(qny, sy, by));
                        const float tnz = __builtin_fmaf(-M, aiz, __builtin_fmaf(qnz, sz, bz));
                        const float tfx = __builtin_fmaf(M, aix, __builtin_fmaf(qfx, sx, bx));
                        const float tfy = __builtin_fmaf(M, aiy, __builtin_fmaf(qfy, sy, by));
                        const float tfz = __builtin_fmaf(M, aiz, __builtin_fmaf(qfz, sz, bz));
                        tmin = fmaxf(fmaxf(tnx, tny), tnz);
                        tmax = fminf(fminf(tfx, tfy), tfz);
                    };
                    const uint32_t sbj = wd(WN_SLAB + j);
                    const float C0 = __builtin_fmaf((float)(sbj & 0xffffu), ss, slo);
                    const float C1 = __builtin_fmaf((float)(sbj >> 16), ss, slo);
                    const float b = nx * Dx + ny * Dy + nz * Dz;   // N . (origin - o)
                    float tmin, tmax;
                    box(Rb, tmin, tmax);
                    tmin -= dtp;
                    tmax += dtp;
                    // enter when max(tmin, 0) <= min(tmax (1 + SL), best_s); a NaN tmin (every
                    // slab NaN) enters too.  The key orders the children; misses get INFINITY.
                    bool ok = fmaxf(tmin, 0.0f) <= fminf(__builtin_fmaf(fabsf(tmax), SL, tmax), best_s);
                    // the slab only narrows the box's interval: skipped when no lane's box passes
                    if (ok && R < INFINITY) {
                        // N . (o + t d - origin) in [C0, C1] widened by w: t between
                        // (C0 - w + b) / a and (C1 + w + b) / a
#if W_SOUND_A
                        const float eta = wq_eta(wr, L, Da);
#else
                        const float eta = 0.0f;
#endif
                        const float w = NLH * __builtin_fmaf(R, sth, eta) * (1.0f + 0x1p-16f) + 384.0f * m;
                        // the hardware reciprocal (1 ulp): its error moves the slab's t by a relative
                        // 2^-23, a distance far inside the margin over the scene
                        const float ia = fast_rcp(a);
                        const float s0 = (C0 - w + b) * ia, s1 = (C1 + w + b) * ia;
                        tmin = fmaxf(tmin, fminf(s0, s1));
                        tmax = fminf(tmax, fmaxf(s0, s1));
                        ok = fmaxf(tmin, 0.0f) <= fminf(__builtin_fmaf(fabsf(tmax), SL, tmax), best_s);
                    }
                    if (ok)
                        key[j] = fminf(fmaxf(tmin, 0.0f), 3.0e38f);
#if defined(W_TRACE) && !defined(__HIP_DEVICE_COMPILE__)
                    {
                        // the r03 test (box and slab widened by m only) for comparison: why the child is entered
                        float t0, t1;
                        box(m, t0, t1);
                        bool ok0 = fmaxf(t0, 0.0f) <= fminf(__builtin_fmaf(fabsf(t1), SL, t1), best_s);
                        bool okbox = ok0;
                        if (ok0) {
                            const float ia = fast_rcp(a);
                            const float s0 = (C0 - 384.0f * m + b) * ia, s1 = (C1 + 384.0f * m + b) * ia;
                            t0 = fmaxf(t0, fminf(s0, s1));
                            t1 = fminf(t1, fmaxf(s0, s1));
                            ok0 = fmaxf(t0, 0.0f) <= fminf(__builtin_fmaf(fabsf(t1), SL, t1), best_s);
                        }
                        float b0, b1;
                        box(Rb, b0, b1);
                        const bool okRbox = fmaxf(b0 - dtp, 0.0f) <= fminf(b1 + dtp, best_s);
                        printf("node %u child %d leaf %d: qlb %.4g smin %.3g sth %.3g L %.3g Dn %.3g R %.3g Rlat %.3g Rpar %.3g "
                               "tmin %.5g tmax %.5g ok %d (tight box %d, tight %d, widened box %d) best %.5g\n",
                               cur, j, (int)((chj & W_LEAF) != 0), qlb, smin, sth, L, Dn, R, Rlat, Rpar, tmin, tmax, (int)ok,
                               (int)okbox, (int)ok0, (int)okRbox, best_s);
                    }
#endif
                    W_DIAG_ADD(1, 1);
                    W_DIAG_ADD(2, ok);
                    // (b): triangles that may lie nearly parallel to d (q < QS), none of whose reports
                    // precedes kbl (the risk key): the line must cross the octree leaves holding them
                    // (the child box widened by rho, any t), and the origin must lie within H0
                    // (wq_h0) of a triangle's plane, so within H0 + D sin(theta)
                    // of the child's slab (D = Dn >= |o - a|)
                    const float rkj = bitsf(rw[2 * j + 1] & 0xFFFF0000u);   // wrisk_key
                    const float kbl = (rkj - rsub) * iqd;
                    if (W_CASE_B && !risk && !nob && qlb < QS) {
                        // no risk words (reflection rays, rt_trace_ray):
                        W_DIAG_ADD(4, 1);
                        // the child box widened by m + rho (any t) and the origin within H0 + D sin(theta) of
                        // the slab; keyed 0 (no risk key bounds the reports' t)
                        float umin, umax;
#if W_LAZY_EXT2
                        const uint32_t e2 = ldg(reinterpret_cast<const uint32_t*>(nodes + cur) + WN_EXT2 + j);
#else
                        const uint32_t e2 = wd(WN_EXT2 + j);
#endif
                        box(m + wq_len(e2 & 0xffu), umin, umax);
                        bool okb = !(umin > __builtin_fmaf(fabsf(umax), SL, umax));
                        if (okb) {
                            const float s2 = wq_val_nz((e >> 8) & 0xffu, WQ_UNIT);
                            const float Dc = dchild();
                            const float H0 = wq_h0(QS, L, Dc, smin, s2);
                            const float w = NLH * (H0 + __builtin_fmaf(Dc, sth, m)) * (1.0f + 0x1p-16f) + 384.0f * m;
                            okb = !(-b < C0 - w || -b > C1 + w);
#if defined(W_TRACE) && !defined(__HIP_DEVICE_COMPILE__)
                            printf("  (b0) node %u child %d: umin %.4g umax %.4g -b %.4g slab [%.4g, %.4g] w %.4g H0 %.3g Dc %.3g sth %.3g okb %d\n",
                                   cur, j, umin, umax, -b, C0, C1, w, H0, Dc, sth, (int)okb);
#endif
                        }
                        if (okb)
                            key[j] = 0.0f;
                    } else if (W_CASE_B && risk && !nob && qlb < QS && rkj < INFINITY && !(kbl > best_s)) {
                        W_DIAG_ADD(4, 1);
#if W_LAZY_EXT2
                        const uint32_t e2 = ldg(reinterpret_cast<const uint32_t*>(nodes + cur) + WN_EXT2 + j);
#else
                        const uint32_t e2 = wd(WN_EXT2 + j);
#endif
                        // the at-risk octree leaves' box widened by m + rho (any t)
                        const float Mb = m + wq_len(e2 & 0xffu);
                        const uint32_t r0 = rw[2 * j], r1 = rw[2 * j + 1];   // lo x y z, hi x y z bytes
                        const float blx = (float)(r0 & 0xffu), bly = (float)((r0 >> 8) & 0xffu),
                                    blz = (float)((r0 >> 16) & 0xffu), bhx = (float)(r0 >> 24),
                                    bhy = (float)(r1 & 0xffu), bhz = (float)((r1 >> 8) & 0xffu);
                        const float umin = fmaxf(fmaxf(__builtin_fmaf(-Mb, aix, __builtin_fmaf(nx_lo ? blx : bhx, sx, bx)),
                                                       __builtin_fmaf(-Mb, aiy, __builtin_fmaf(ny_lo ? bly : bhy, sy, by))),
                                                 __builtin_fmaf(-Mb, aiz, __builtin_fmaf(nz_lo ? blz : bhz, sz, bz)));
                        const float umax = fminf(fminf(__builtin_fmaf(Mb, aix, __builtin_fmaf(nx_lo ? bhx : blx, sx, bx)),
                                                       __builtin_fmaf(Mb, aiy, __builtin_fmaf(ny_lo ? bhy : bly, sy, by))),
                                                 __builtin_fmaf(Mb, aiz, __builtin_fmaf(nz_lo ? bhz : blz, sz, bz)));
                        bool okb = !(umin > __builtin_fmaf(fabsf(umax), SL, umax));
                        if (okb) {
                            const float s2 = wq_val_nz((e >> 8) & 0xffu, WQ_UNIT);
                            const float Dc = W_B_CHILD_D >= 2 ? dchild() : Dn;
                            const float H0 = wq_h0(QS, L, Dc, smin, s2);
                            const float w = NLH * (H0 + __builtin_fmaf(Dc, sth, m)) * (1.0f + 0x1p-16f) + 384.0f * m;
                            okb = !(-b < C0 - w || -b > C1 + w);   // N . (o - origin) = -b
                        }
#if defined(W_TRACE) && !defined(__HIP_DEVICE_COMPILE__)
                        printf("  (b) node %u child %d: okb %d kbl %.5g key %.5g\n", cur, j, (int)okb, kbl, key[j]);
#endif
                        if (okb) {
                            W_DIAG_ADD(3, !ok);
                            W_DIAG_ADD(6, !ok && (chj & W_LEAF));
                            W_DIAG_ADD(7, !ok && kbl > 0.0f);
                            W_DIAG_ADD(5, ok && kbl < key[j]);
                            key[j] = fminf(key[j], fminf(fmaxf(kbl, 0.0f), 3.0e38f));
                        }
                    }
#if W_PRIO_ORDER
                    // visit order: the entry t of the child's unwidened box (not below the key).  A child
                    // holding ill-conditioned triangles (UV-sphere pole slivers) has a box widened by a
                    // large R whose entry t precedes the actual hit; ordered by that key the query walked
                    // such subtrees first, with no best hit to cull them yet (grazing C4 rays: 144 of 156
                    // entered children before the hit).  The order does not change the answer.
                    if (key[j] < INFINITY)
                        pri[j] = fmaxf(key[j], fmaxf(fmaxf(__builtin_fmaf(qnx, sx, bx), __builtin_fmaf(qny, sy, by)),
                                                     __builtin_fmaf(qnz, sz, bz)));
#endif
                }
#if defined(__HIP_DEVICE_COMPILE__)
                // one child at a time: the scheduler would interleave the children's
                // temporaries (VALU latency is hidden by the other waves anyway); a lane group
                // (the few long queries of split tiles, W_GROUP_ILP) may interleave them
                if (G == 1 || !W_GROUP_ILP)
                    __builtin_amdgcn_sched_barrier(0);
#endif
            }
            // sort the (key, ref) pairs ascending: misses (INFINITY) go last
#if W_PRIO_ORDER
#define W_CSWAP(a, b)                                                              \
    if (pri[b] < pri[a]) {                                                         \
        float tp = pri[a]; pri[a] = pri[b]; pri[b] = tp;                           \
        float tk = key[a]; key[a] = key[b]; key[b] = tk;                           \
        uint32_t tr = ref[a]; ref[a] = ref[b]; ref[b] = tr;                        \
    }
#else
#define W_CSWAP(a, b)                                                              \
    if (key[b] < key[a]) {                                                         \
        float tk = key[a]; key[a] = key[b]; key[b] = tk;                           \
        uint32_t tr = ref[a]; ref[a] = ref[b]; ref[b] = tr;                        \
    }
#endif
            W_CSWAP(0, 1) W_CSWAP(2, 3) W_CSWAP(0, 2) W_CSWAP(1, 3) W_CSWAP(1, 2)
#undef W_CSWAP
            if (key[0] < INFINITY) {
                cur = ref[0];
#pragma unroll
                for (int j = W_WIDTH - 1; j >= 1; j--)
                    if (key[j] < INFINITY) {
                        if (sp - bot < Stack::CAP)
                            stk.put(slot(sp++), make_uint2(ref[j], fbits(key[j])));
                        else {
                            // full: the entry with the largest key goes (the new child or one on the
                            // stack, which it replaces); the query stays certified if the dropped key
                            // exceeds the final best hit
                            int im = -1;
                            float km = key[j];
                            for (int i = 0; i < Stack::CAP; i++) {
                                const float ki = bitsf(stk.get(i).y);
                                if (ki > km) {
                                    km = ki;
                                    im = i;
                                }
                            }
                            if (im >= 0)
                                stk.put(im, make_uint2(ref[j], fbits(key[j])));
                            dropped = fminf(dropped, km);
                        }
                    }
            } else {
                cur = W_EMPTY;
                while (sp > bot) {
                    uint2 e = stk.get(slot(--sp));
                    if (bitsf(e.y) <= best_s) {
                        cur = e.x;
                        break;
                    }
                }
            }
        }
        else if (G == 1 || cur != W_EMPTY) {   // (an idle lane of a group: no step)
        // ---- a leaf: its triangles, closest hit kept; equal t from another triangle is a tie ----
        W_STEP_HOOK(cur, 1);
        const uint32_t first = (cur >> 3) & 0x0FFFFFFFu, cnt = (cur & 7u) + 1u;
        const uint32_t kend = first + cnt;
        // the leaf's triangles in order (loading two records at a time was measured slower)
        auto fold = [&](const GTri& T, uint32_t k) {
            nt++;
            float t, u, v;
            if (mt_record(T, o, d, t, u, v)) {
                if (t != t)
                    nanhit = true;
                else if (!(t <= hi))
                    ;   // beyond the segment
                else if (t == INFINITY)
                    infhit = true;   // overflowed t: only matters when no finite hit exists
                else if (t < h.t) {
                    h.t = t;
                    h.u = u;
                    h.v = v;
                    h.k = (int32_t)k;
                    tie = false;
                    best_s = t + fabsf(t) * SL;
                } else if (t == h.t)
                    tie = true;
            }
        };
        for (uint32_t k = first; k < kend; k++)
            fold(load_gtri(tris + k), k);
        cur = W_EMPTY;
        while (sp > bot) {
            uint2 e = stk.get(slot(--sp));
            if (bitsf(e.y) <= best_s) {
                cur = e.x;
                break;
            }
        }
        }
        if constexpr (G > 1) {
            // the group's best bound, then the idle lanes take work: the i-th idle lane the bottom
            // (oldest: the largest subtree) entry of the i-th lane holding entries
            best_s = wg_min<G>(best_s);
            const uint32_t idle = wg_bits<G>(cur == W_EMPTY), busy = wg_bits<G>(sp > bot);
            if (idle && busy) {
                const uint32_t gl = wg_lane<G>(), below = (1u << gl) - 1u;
                int src = -1;
                if (cur == W_EMPTY) {
                    uint32_t b = busy;
                    for (int r = __builtin_popcount(idle & below); r > 0 && b; r--)
                        b &= b - 1u;
                    src = b ? __builtin_ctz(b) : -1;
                }
                const int sbot = wg_read<G>(bot, src >= 0 ? src : (int)gl);
                if (sp > bot && __builtin_popcount(busy & below) < __builtin_popcount(idle))
                    bot++;   // (the taker reads the entry below before any later push can reuse its slot)
                if (src >= 0) {
                    const uint2 e = stk.get_lane(src - (int)gl, slot(sbot));
                    if (bitsf(e.y) <= best_s)
                        cur = e.x;
                }
            }
        }
    }
    if constexpr (G > 1) {
        // the group's answer: the least t over its lanes' records; a tie when two lanes hold it (each
        // triangle is tested by one lane at most) or the lane holding it saw two
        const float T = wg_min<G>(h.t);
        const uint32_t at = wg_bits<G>(h.k >= 0 && h.t == T);
        const int w = at ? __builtin_ctz(at) : 0;
        tie = __builtin_popcount(at) > 1 || wg_bits<G>(h.k >= 0 && h.t == T && tie) != 0u;
        h.t = wg_read<G>(h.t, w);
        h.u = wg_read<G>(h.u, w);
        h.v = wg_read<G>(h.v, w);
        h.k = wg_read<G>(h.k, w);
        nanhit = wg_bits<G>(nanhit) != 0u;
        infhit = wg_bits<G>(infhit) != 0u;
        dropped = wg_min<G>(dropped);
        best_s = wg_min<G>(best_s);
    }
    // a dropped child matters only if it could hold a hit at t <= the final best (a pop would have
    // skipped it otherwise)
    const bool overflow = dropped < INFINITY && dropped <= best_s;
    if (work) {
        work[0] += nn;
        work[1] += nt;
        work[3] += steps;
        // why a query is not certified (diagnostics): 1 stack overflow, 2 NaN hit,
        // 4 only overflowed hits, 8 tie, 16 minimum t not in (0, inf)
        work[2] = (overflow ? 1u : 0u) | (nanhit ? 2u : 0u) | (h.k < 0 && infhit ? 4u : 0u) |
                  (h.k >= 0 && ties && tie ? 8u : 0u) | (h.k >= 0 && !(h.t > 0.0f && h.t < INFINITY) ? 16u : 0u);
    }
    if constexpr (FEED)
        return W_MISS;   // (every query went to feed->finish)
    if (nanhit)
        return W_UNCERT;
    if (h.k < 0) {
        if (infhit)
            return W_UNCERT;
        if (overflow)
            return W_DEEP;
        h.t = -1.0f;   // HitInfo() (hitInfo.h:8-24): t = -1, u = 1, v = 0
        return W_MISS;
    }
    if ((ties && tie) || !(h.t > 0.0f && h.t < INFINITY))
        return W_UNCERT;
    return overflow ? W_DEEP : W_HIT;
}

}  // namespace rt
