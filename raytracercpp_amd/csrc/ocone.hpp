// ocone.hpp -- origin cones: when a ray without risk words (a reflection ray, rt_trace_ray) may skip
// case (b) of the wide query (wbvh.hpp wbvh_closest).
//
// Case (b) covers the triangles nearly parallel to the ray (q = |cos(N, d)| < QS), whose reports the
// box-and-slab test of case (a) cannot bound.  Such a triangle reports a hit only when the ray's origin
// lies within H0(|o - a|) of its plane (wq_h0, the lemma behind the camera's risk keys), and no
// triangle reports one when Moller-Trumbore's computed Mdet = n~ . (-d) is <= 0 (triangle.cpp:37-40,
// BACKFACE_CULLING; n~ the stored normal).  A uniform grid over the scene holds, per cell X, a cone
// (axis A, half-angle beta) around the stored unit normals of every triangle that is "at risk" for
// some origin in X (wbvh_risk_key with the cell's ball as the spread of origins: the lemma's distance
// test fails for no other triangle).  A ray from o in X with angle(A, -d) - beta >= pi/2 + asin(EPS)
// has n~ . (-d) <= -EPS |n~||d| for every at-risk triangle: with the dot product's rounding (<= 3u |n~||d|)
// the computed Mdet is negative and none of them reports.  The other triangles with q < QS cannot
// report either (the lemma), so case (b) has nothing to find and the query skips it: the same answer,
// fewer node visits (a reflection ray leaving the surface faces the back of the triangles near its
// origin, which are the ones whose planes pass near it).
//
// The cone holds the exact unit normals N = ab x ac of the at-risk triangles too, which gives a second
// route: a ray with angle(A, -d) + beta <= acos(QS + EPS) has |cos(N, d)| >= QS for every at-risk triangle,
// so none of them is in case (b) (a ray entering the surface its origin is above: a reflection sample that
// turns back into a bumpy surface).  A degenerate at-risk record (no N) closes that route (OC_NOFRONT).
//
// Cell word (uint2): x = A.x | A.y << 16, y = A.z | code << 16 (A as signed 16-bit integers, the axis
// A / |A|); code = beta in units of (pi/2) / OC_BMAX rounded up (| OC_NOFRONT), OC_NOSKIP (no bound: case
// (b) runs), OC_EMPTY (no triangle at risk: every ray may skip).
#pragma once

#include <stdint.h>

#include <vector>

#include "wbvh.hpp"

namespace rt {

constexpr uint32_t OC_BMAX = 0x7FFDu, OC_EMPTY = 0x7FFEu, OC_NOSKIP = 0x7FFFu, OC_NOFRONT = 0x8000u;
constexpr float OC_EPS = 0x1p-12f;   // the test's margin in cos(angle(n~, -d)) (rounding: < 1e-5)
// the grid search's shortcut (ocone_cell): entries of half-angle <= 2 degrees reaching <= 1 degree past the cone
constexpr double OC_SIN_TAU = 0.034899496702500969, OC_COS_TAU2 = 0.99984769515639127, OC_SIN_TAU2 = 0.017452406437283512;

// The grid the device reads (KParams::ocone): cell (ix, iy, iz) holds the origins o with
// floor(fl(fl(o - lo) * ih)) = (ix, iy, iz) per axis, in float as ocone_skip computes it.
struct OConeView {
    const uint2* cells;
    float lo[3];
    float ih;
    int32_t dim[3];
};

// True: the ray (o, d) may skip case (b) (no triangle of it can report a hit, see above).
RT_HD bool ocone_skip(const OConeView& g, v3 o, v3 d, float QS)
{
    if (!g.cells)
        return false;
    const float fx = (o.x - g.lo[0]) * g.ih, fy = (o.y - g.lo[1]) * g.ih, fz = (o.z - g.lo[2]) * g.ih;
    if (!(fx >= 0.0f && fx < (float)g.dim[0] && fy >= 0.0f && fy < (float)g.dim[1] && fz >= 0.0f && fz < (float)g.dim[2]))
        return false;
    const int ix = (int)fx, iy = (int)fy, iz = (int)fz;
    const uint2 w = g.cells[((size_t)iz * (size_t)g.dim[1] + (size_t)iy) * (size_t)g.dim[0] + (size_t)ix];
    const uint32_t word = w.y >> 16, code = word & 0x7FFFu;
    if (code == OC_NOSKIP)
        return false;
    if (code == OC_EMPTY)
        return true;
    const float ax = (float)(int16_t)(w.x & 0xffffu), ay = (float)(int16_t)(w.x >> 16), az = (float)(int16_t)(w.y & 0xffffu);
    const float beta = (float)code * (float)(1.5707963267948966 / OC_BMAX);
    const float sb = sinf(beta), cb = cosf(beta);
    const float inv = 1.0f / (sqrtf(ax * ax + ay * ay + az * az) * sqrtf(d.x * d.x + d.y * d.y + d.z * d.z));
    const float c = -(ax * d.x + ay * d.y + az * d.z) * inv;   // cos(angle(A, -d))
    const float cx = ay * d.z - az * d.y, cy = az * d.x - ax * d.z, cz = ax * d.y - ay * d.x;
    const float s = sqrtf(cx * cx + cy * cy + cz * cz) * inv;   // sin(angle(A, -d))
    // cos(angle(A, -d) - beta) <= -EPS: every at-risk stored normal is past pi/2 + asin(EPS) from -d; or
    // cos(angle(A, -d) + beta) >= QS + EPS: every at-risk exact normal within acos(QS + EPS) of -d
    return c * cb + s * sb <= -OC_EPS || (!(word & OC_NOFRONT) && c * cb - s * sb >= QS + OC_EPS);
}

// One child entry (node v, slot j) of the wide BVH for the grid's search (ocone.cpp oc_entries): what
// its triangles' planes and stored normals span, in double.  Cones as unit axis and cos / sin of the
// half-angle, rounded outwards; pc <= 0: the plane cone reaches pi / 2 or more (no distance bound),
// sc <= 0: the stored-normal cone does.
struct OConeEnt {
    double lo[3], hi[3];
    double pa[3], pc, ps;   // exact normals N = ab x ac of the non-degenerate triangles
    double sa[3], sc, ss;   // stored normals n~, the non-zero ones
    double lmax, smin, s2min;   // the lemma's L, s, s2 (smin = s2min = 0: a degenerate triangle below)
    uint32_t link;          // the node's child link: W_LEAF | first << 3 | (count - 1), a node index, W_EMPTY
    uint32_t any;           // a triangle with a non-zero stored normal below
};

// H0 (wq_h0 / wbvh_risk_key) in double; infinite without an s / s2 bound
RT_HD double oc_h0(double QS, double L, double D, double s, double s2)
{
    if (!(s > 0) || !(s2 > 0))
        return INFINITY;
    const double u = 0x1p-24;
    return 1.01 * (QS * (2 * L + D) + u * (24.2 * L + 48 * D) / s + u * (30 * L + 12 * D + 24 * D / s) / s2);
}

// May the entry hold a triangle at risk for the origins within r of c?  Its planes have unit normals n
// within the plane cone's half-angle th of its axis a and pass through points x of its box: |n . (c -
// x)| >= cos(th) |a . (c - x)| - sin(th) |c - x|, against the lemma's H0(|c - x| + r + slack) + QS r + r
// (wbvh_risk_key with G = nu = r).
RT_HD bool oc_may_risk(const OConeEnt& g, const double c[3], double r, double slack, double QS)
{
    if (!g.any)
        return false;
    double dmax2 = 0, pc = 0, pm = 0, ph = 0;
    for (int i = 0; i < 3; i++) {
        const double e = fmax(fabs(c[i] - g.lo[i]), fabs(c[i] - g.hi[i]));
        dmax2 += e * e;
        pc += g.pa[i] * c[i];
        pm += g.pa[i] * 0.5 * (g.lo[i] + g.hi[i]);
        ph += fabs(g.pa[i]) * 0.5 * (g.hi[i] - g.lo[i]);
    }
    const double dmax = sqrt(dmax2) * (1 + 1e-12);
    const double rhs = (oc_h0(QS, g.lmax, dmax + r + slack, g.smin, g.s2min) + QS * r + r) * (1 + 1e-6);
    if (!(rhs < INFINITY) || !(g.pc > 0))
        return true;
    const double gap = fmax(0.0, fabs(pc - pm) - ph * (1 + 1e-12)) * (1 - 1e-12);
    const double lb = g.pc * gap - g.ps * dmax;
    return !(lb > rhs * (1 + 1e-9));
}

// The word of the cell whose origins lie within r of c (ocone.hpp top): the axis is the stored normal
// of the triangle whose centroid is nearest to c, quantised; the cone's half-angle the largest angle
// from it to the stored normal of a triangle at risk, found by a depth-first branch and bound over the
// entries E (children ordered by their normals' reach; an entry whose normals all lie within the
// half-angle found so far, or whose planes stay away from the ball, is skipped).  Half-angles beyond
// acos(cos_cap) and a full stack give OC_NOSKIP.
template <int CAP>
RT_HD uint2 ocone_cell(const OConeEnt* E, const GTri* tris, const double c[3], double r, double slack, double QS,
                       double cos_cap)
{
    auto pack = [](const int32_t q[3], uint32_t code) {
        uint2 o;
        o.x = (uint32_t)(uint16_t)q[0] | ((uint32_t)(uint16_t)q[1] << 16);
        o.y = (uint32_t)(uint16_t)q[2] | (code << 16);
        return o;
    };
    int32_t q[3] = {0, 0, 0};
    uint32_t stk[CAP];
    int sp = 0;
    auto boxd2 = [&](const OConeEnt& g) {
        double s = 0;
        for (int i = 0; i < 3; i++) {
            const double e = fmax(0.0, fmax(g.lo[i] - c[i], c[i] - g.hi[i]));
            s += e * e;
        }
        return s;
    };
    // 1. the axis
    double best = INFINITY, A[3] = {0, 0, 0};
    for (int j = W_WIDTH - 1; j >= 0; j--)
        if (E[j].any)
            stk[sp++] = (uint32_t)j;
    while (sp > 0) {
        const OConeEnt& g = E[stk[--sp]];
        if (!(boxd2(g) < best))
            continue;
        if (g.link & W_LEAF) {
            const uint32_t first = (g.link & ~W_LEAF) >> 3, cnt = (g.link & 7u) + 1;
            for (uint32_t k = first; k < first + cnt; k++) {
                const GTri& t = tris[k];
                const double nn = sqrt((double)t.n[0] * t.n[0] + (double)t.n[1] * t.n[1] + (double)t.n[2] * t.n[2]);
                if (!(nn > 0) || !(nn < INFINITY))
                    continue;
                double d2 = 0;
                for (int i = 0; i < 3; i++) {
                    const double m = t.a[i] + ((double)t.ab[i] + (double)t.ac[i]) / 3.0 - c[i];
                    d2 += m * m;
                }
                if (d2 < best) {
                    best = d2;
                    for (int i = 0; i < 3; i++)
                        A[i] = t.n[i] / nn;
                }
            }
        } else if (sp + W_WIDTH <= CAP) {   // (a full stack only makes the axis worse)
            // the nearest box popped first
            double dk[W_WIDTH];
            uint32_t ek[W_WIDTH];
            int nk = 0;
            for (int j = 0; j < W_WIDTH; j++) {
                const uint32_t e = g.link * W_WIDTH + (uint32_t)j;
                if (!E[e].any)
                    continue;
                const double dd = boxd2(E[e]);
                if (!(dd < best))
                    continue;
                int i = nk++;
                for (; i > 0 && dk[i - 1] < dd; i--) {
                    dk[i] = dk[i - 1];
                    ek[i] = ek[i - 1];
                }
                dk[i] = dd;
                ek[i] = e;
            }
            for (int i = 0; i < nk; i++)
                stk[sp++] = ek[i];
        }
    }
    if (!(best < INFINITY))
        return pack(q, OC_EMPTY);   // no triangle can report a hit at all
    for (int i = 0; i < 3; i++)
        q[i] = (int32_t)rint(A[i] * 32767.0);
    double Aq[3] = {(double)q[0], (double)q[1], (double)q[2]};
    const double ql = sqrt(Aq[0] * Aq[0] + Aq[1] * Aq[1] + Aq[2] * Aq[2]);
    if (!(ql > 0))
        return pack(q, OC_NOSKIP);
    for (int i = 0; i < 3; i++)
        Aq[i] /= ql;
    // 2. the half-angle: cb = cos of the largest angle found (any: a triangle at risk found)
    bool any = false, nofront = false;
    double cb = 2.0, sb = 0.0;
    // cos of the largest angle from Aq an entry's stored normals may make (-2: no bound)
    auto cub = [&](const OConeEnt& g) {
        if (!(g.sc > 0))
            return -2.0;
        const double ca = Aq[0] * g.sa[0] + Aq[1] * g.sa[1] + Aq[2] * g.sa[2];
        const double x = Aq[1] * g.sa[2] - Aq[2] * g.sa[1], y = Aq[2] * g.sa[0] - Aq[0] * g.sa[2],
                     z = Aq[0] * g.sa[1] - Aq[1] * g.sa[0];
        return ca * g.sc - sqrt(x * x + y * y + z * z) * g.ss - 1e-12;
    };
    // An inner entry whose normals lie within OC_TAU of its axis and whose reach exceeds the half-angle
    // found by at most OC_TAU2 is not searched: its reach joins the cone instead (cabs, the cos of the
    // largest such reach), so the triangles just past the at-risk rim cost no walk to their leaves.
    double cabs = 2.0, clim = 2.0;   // clim: cos(half-angle found + OC_TAU2)
    sp = 0;
    for (int j = 0; j < W_WIDTH; j++)
        if (E[j].any)
            stk[sp++] = (uint32_t)j;
    while (sp > 0) {
        const OConeEnt& g = E[stk[--sp]];
        const double kg = cub(g);
        if (any && kg >= fmin(cb, cabs)) {
            nofront |= g.smin == 0;   // (a degenerate record below, at risk or not: the front route closes)
            continue;                 // every normal below within the cone so far
        }
        if (!oc_may_risk(g, c, r, slack, QS))
            continue;
        if (any && !(g.link & W_LEAF) && g.sc > 0 && g.ss <= OC_SIN_TAU && kg >= clim) {
            cabs = fmin(cabs, kg);
            nofront |= g.smin == 0;
            continue;
        }
        if (g.link & W_LEAF) {
            const uint32_t first = (g.link & ~W_LEAF) >> 3, cnt = (g.link & 7u) + 1;
            for (uint32_t k = first; k < first + cnt; k++) {
                const GTri& t = tris[k];
                const double nn = sqrt((double)t.n[0] * t.n[0] + (double)t.n[1] * t.n[1] + (double)t.n[2] * t.n[2]);
                if (nn == 0)
                    continue;   // Mdet = 0: never a hit
                if (!(nn < INFINITY))
                    return pack(q, OC_NOSKIP);
                // the stored normal and (non-degenerate records) the exact one: the farther from the axis
                double u[3] = {t.n[0] / nn, t.n[1] / nn, t.n[2] / nn};
                double cu = Aq[0] * u[0] + Aq[1] * u[1] + Aq[2] * u[2];
                bool degen = false;
                {
                    const double x0 = t.ab[0], x1 = t.ab[1], x2 = t.ab[2], y0 = t.ac[0], y1 = t.ac[1], y2 = t.ac[2];
                    const double n0 = x1 * y2 - x2 * y1, n1 = x2 * y0 - x0 * y2, n2 = x0 * y1 - x1 * y0;
                    const double la = sqrt(x0 * x0 + x1 * x1 + x2 * x2), lc = sqrt(y0 * y0 + y1 * y1 + y2 * y2);
                    const double cl = sqrt(n0 * n0 + n1 * n1 + n2 * n2);
                    degen = !(la * lc > 0x1p-100) || !(cl > 0x1p-50 * la * lc) || !(cl < INFINITY);
                    if (!degen) {
                        const double cN = (Aq[0] * n0 + Aq[1] * n1 + Aq[2] * n2) / cl;
                        if (cN < cu) {
                            cu = cN;
                            u[0] = n0 / cl;
                            u[1] = n1 / cl;
                            u[2] = n2 / cl;
                        }
                    }
                }
                if (any && !(cu < cb) && !degen)
                    continue;   // within the half-angle found: at risk or not, it changes nothing
                if (!(wbvh_risk_key(t, c[0], c[1], c[2], r, r, slack, QS) < INFINITY))
                    continue;   // no origin of the cell lies near its plane
                nofront |= degen;
                if (!any || cu < cb) {
                    const double x = Aq[1] * u[2] - Aq[2] * u[1], y = Aq[2] * u[0] - Aq[0] * u[2], z = Aq[0] * u[1] - Aq[1] * u[0];
                    cb = cu;
                    sb = sqrt(x * x + y * y + z * z);
                    any = true;
                    clim = cb * OC_COS_TAU2 - sb * OC_SIN_TAU2;
                    if (!(cb >= cos_cap))
                        return pack(q, OC_NOSKIP);
                }
            }
        } else {
            if (sp + W_WIDTH > CAP)
                return pack(q, OC_NOSKIP);
            // the widest-reaching child popped first (it may raise the half-angle most)
            double kk[W_WIDTH];
            uint32_t ek[W_WIDTH];
            int nk = 0;
            for (int j = 0; j < W_WIDTH; j++) {
                const uint32_t e = g.link * W_WIDTH + (uint32_t)j;
                if (!E[e].any)
                    continue;
                const double kc = cub(E[e]);
                int i = nk++;
                for (; i > 0 && kk[i - 1] < kc; i--) {
                    kk[i] = kk[i - 1];
                    ek[i] = ek[i - 1];
                }
                kk[i] = kc;
                ek[i] = e;
            }
            for (int i = 0; i < nk; i++)
                stk[sp++] = ek[i];
        }
    }
    if (!any)
        return pack(q, OC_EMPTY);
    // rounded up: the angle's own rounding (1e-9) and the float test's margin (OC_EPS)
    const double beta = fmax(atan2(sb, cb), cabs <= 1.0 ? acos(fmax(-1.0, cabs)) : 0.0);
    const double code = ceil((beta * (1 + 1e-9) + 1e-9) / 1.5707963267948966 * OC_BMAX);
    if (!(code <= OC_BMAX))
        return pack(q, OC_NOSKIP);
    return pack(q, (uint32_t)code | (nofront ? OC_NOFRONT : 0u));
}

struct OConeGrid {
    float lo[3] = {0, 0, 0};
    float ih = 0.0f;
    int32_t dim[3] = {0, 0, 0};
    std::vector<uint2> cells;   // dim[0] * dim[1] * dim[2], x fastest
    int64_t computed = 0, empty = 0, noskip = 0;   // cells with a cone / with no triangle at risk / no bound
    float ms = 0.0f;
};

// The grid for the wide BVH's triangles (its tree prunes the search): cells within `reach` of a
// triangle get a cone (origins farther away read OC_NOSKIP), at most max_dim cells along the longest
// axis.  QS: the query's grazing split for these rays (W_QS_CLOSEST); S: the scene scale (the query's
// margin m = 2^-16 (max|o| + S)).  beta_cap: larger cones are stored as OC_NOSKIP.  threads <= 0: all.
void build_origin_cones(const WBvh& w, float S, double QS, double reach, int max_dim, double beta_cap, int threads,
                        OConeGrid& g);

// The same in two halves for a device build (renderer.cpp start_accel, kernels.hip ocone_kernel): the
// host's part (the entries, the grid's frame and its cells within reach, g.cells left empty), then each
// listed cell's word from ocone_cell.  OConeJob carries what the device needs.
constexpr int OC_STACK = 96;
struct OConeJob {
    std::vector<OConeEnt> ent;
    std::vector<uint32_t> todo;   // the cells within reach (x + dim0 (y + dim1 z))
    double h = 0, r = 0, slack = 0, QS = 0, cos_cap = 0;
};
// cells' tallies (empty / noskip) of a finished grid
void origin_cones_count(OConeGrid& g);
void origin_cones_plan(const WBvh& w, float S, double QS, double reach, int max_dim, double beta_cap, OConeGrid& g,
                       OConeJob& job);

// the centre of cell id (x + dim0 (y + dim1 z)) of a grid with origin lo and cell size h
RT_HD void ocone_center(const float lo[3], const int32_t dim[3], double h, uint32_t id, double c[3])
{
    const uint32_t x = id % (uint32_t)dim[0], y = id / (uint32_t)dim[0] % (uint32_t)dim[1],
                   z = id / ((uint32_t)dim[0] * (uint32_t)dim[1]);
    c[0] = (double)lo[0] + ((double)x + 0.5) * h;
    c[1] = (double)lo[1] + ((double)y + 0.5) * h;
    c[2] = (double)lo[2] + ((double)z + 0.5) * h;
}

}  // namespace rt
