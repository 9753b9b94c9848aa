/*
 * oracle.c -- TEST INFRASTRUCTURE ONLY: CPU restatement of the reference's
 * primary-ray + shadow-ray hot path (TomClabault/RayTracerCPP @ 2024-08-07).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * liboracle.so.  It is the checker, never the thing measured as the product.
 *
 * Every function cites the reference file:line it restates (paths relative to
 * /root/reference/tp2).  Floating-point expressions keep the reference's
 * operation order; the file is compiled with -ffp-contract=off so that no
 * multiply-add is contracted (the portable parity target).
 *
 * Pinning: tests/test_oracle_pinning.py checks this restatement bit-for-bit
 * against the reference's own compiled BVH / Triangle / Transform code
 * (oracle/_ref/libref_harness.so, built from the unmodified sources), and the
 * committed golden vectors in tests/golden/ were produced by that harness.
 *
 * Divergences from the reference, all documented in DESIGN.md:
 *   - rough-reflection random numbers come from a per-pixel counter-seeded
 *     xorshift32 stream (the reference seeds one stream per OpenMP thread with
 *     std::rand(), renderer.cpp:51-61, so it is not reproducible run to run);
 *   - the three bilateral randoms of one reflection sample are drawn x, y, z in
 *     order (C++ leaves the order of renderer.cpp:313's arguments unspecified).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "orc_scene.h"

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

#define ORC_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------------- */
/* vec.cpp / color.cpp restated (tp2/src/vec.cpp:41-177, tp2/src/color.cpp)   */
/* ------------------------------------------------------------------------- */
typedef struct { float x, y, z; } v3;

static inline v3 V(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 vsub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }      /* vec.cpp:41-44, 97-100 */
static inline v3 vadd(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }      /* vec.cpp:72-75, 92-95 */
static inline v3 vneg(v3 a) { return V(-a.x, -a.y, -a.z); }                           /* vec.cpp:67-70 */
static inline v3 vscale(float k, v3 v) { return V(k * v.x, k * v.y, k * v.z); }       /* vec.cpp:102-110 */
static inline float vdot(v3 u, v3 v) { return u.x * v.x + u.y * v.y + u.z * v.z; }    /* vec.cpp:164-167 */
static inline v3 vcross(v3 u, v3 v)                                                     /* vec.cpp:156-162 */
{
    return V((u.y * v.z) - (u.z * v.y), (u.z * v.x) - (u.x * v.z), (u.x * v.y) - (u.y * v.x));
}
static inline float vlength2(v3 v) { return v.x * v.x + v.y * v.y + v.z * v.z; }      /* vec.cpp:174-177 */
static inline float vlength(v3 v) { return sqrtf(vlength2(v)); }                      /* vec.cpp:169-172 */
static inline v3 vnormalize(v3 v)                                                       /* vec.cpp:150-154 */
{
    float kk = 1 / vlength(v);
    return vscale(kk, v);
}
/* std::min / std::max semantics: min(a,b) = (b < a) ? b : a ; max(a,b) = (a < b) ? b : a */
static inline float smin(float a, float b) { return (b < a) ? b : a; }
static inline float smax(float a, float b) { return (a < b) ? b : a; }
static inline float sclamp01(float v) { return (v < 0.0f) ? 0.0f : ((1.0f < v) ? 1.0f : v); } /* std::clamp */

typedef struct { float r, g, b; } c3;   /* Color; alpha never reaches RGB */
static inline c3 C(float r, float g, float b) { c3 c = {r, g, b}; return c; }
static inline c3 cadd(c3 a, c3 b) { return C(a.r + b.r, a.g + b.g, a.b + b.b); }     /* color.cpp:48-51 */
static inline c3 cmul(c3 a, c3 b) { return C(a.r * b.r, a.g * b.g, a.b * b.b); }     /* color.cpp:63-66 */
static inline c3 cmulf(c3 c, float k) { return C(c.r * k, c.g * k, c.b * k); }       /* color.cpp:68-76 */
static inline c3 cdiv(c3 a, c3 b) { return C(a.r / b.r, a.g / b.g, a.b / b.b); }     /* color.cpp:78-81 */

/* Transform::operator()(Point) (tp2/src/mat.cpp:83-100); m row-major m[i][j] */
static inline v3 xform_point(const float *m, v3 p)
{
    float x = p.x, y = p.y, z = p.z;
    float xt = m[0] * x + m[1] * y + m[2] * z + m[3];
    float yt = m[4] * x + m[5] * y + m[6] * z + m[7];
    float zt = m[8] * x + m[9] * y + m[10] * z + m[11];
    float wt = m[12] * x + m[13] * y + m[14] * z + m[15];
    float w = 1.f / wt;
    if (wt == 1.f)
        return V(xt, yt, zt);
    return V(xt * w, yt * w, zt * w);
}

/* x86-64 cvttss2si: out-of-range and NaN give INT_MIN (0x80000000) */
static inline int f2i(float f)
{
    if (!(f > -2147483648.0f && f < 2147483648.0f))
        return INT32_MIN;
    return (int)f;
}

static inline uint32_t qrgb(int r, int g, int b)
{
    return 0xff000000u | ((uint32_t)(r & 0xff) << 16) | ((uint32_t)(g & 0xff) << 8) | (uint32_t)(b & 0xff);
}

/* ------------------------------------------------------------------------- */
/* Triangle (tp2/projets/triangle.{h,cpp})                                     */
/* ------------------------------------------------------------------------- */
typedef struct {
    v3 a, b, c, n;  /* n = cross(b - a, c - a), triangle.cpp:11-12 */
    int mat;
    v3 tu, tv;      /* _tex_coords_u, _tex_coords_v */
} otri;

typedef struct {
    int tri;        /* HitInfo::triangle as index, -1 == nullptr */
    float t, u, v;
    int mat;
    v3 normal, tangent;
} ohit;

static inline ohit hit_fresh(void)  /* HitInfo defaults, hitInfo.h:8-24 */
{
    ohit h;
    h.tri = -1; h.t = -1; h.u = 1.0f; h.v = 0.0f; h.mat = -1;
    h.normal = V(0, 0, 0); h.tangent = V(0, 0, 0);
    return h;
}

/* Triangle::get_tangent, triangle.cpp:134-153 */
static v3 tri_tangent(const otri *T, v3 ab, v3 ac)
{
    float u1 = T->tu.x, v1 = T->tv.x;
    float u2 = T->tu.y, v2 = T->tv.y;
    float u3 = T->tu.z, v3_ = T->tv.z;
    float dU1 = u2 - u1, dV1 = v2 - v1, dU2 = u3 - u1, dV2 = v3_ - v1;
    float f = 1.0f / (dU1 * dV2 - dU2 * dV1);
    v3 t;
    t.x = f * (dV2 * ab.x - dV1 * ac.x);
    t.y = f * (dV2 * ab.y - dV1 * ac.y);
    t.z = f * (dV2 * ab.z - dV1 * ac.z);
    return t;
}

/* Triangle::intersect (Moller-Trumbore, BACKFACE_CULLING 1), triangle.cpp:25-91 */
static int tri_intersect(const otri *T, int id, v3 o, v3 d, ohit *h)
{
    v3 ab = vsub(T->b, T->a);
    v3 ac = vsub(T->c, T->a);
    v3 OA = vsub(o, T->a);
    v3 m = vcross(vneg(d), OA);
    float Mdet = vdot(T->n, vneg(d));
    if (Mdet <= 0)
        return 0;
    Mdet = 1 / Mdet;
    float u = vdot(m, ac) * Mdet;
    if (u < 0 || u > 1)
        return 0;
    float v = vdot(m, vneg(ab)) * Mdet;
    if (v < 0 || u + v > 1)
        return 0;
    float t = vdot(T->n, OA) * Mdet;
    if (t < 0)
        return 0;
    h->t = t;
    h->u = u;
    h->v = v;
    h->tangent = tri_tangent(T, ab, ac);
    h->mat = T->mat;
    h->normal = vnormalize(T->n);
    h->tri = id;
    return 1;
}

/* Triangle::interpolate_texcoords, triangle.cpp:155-160 */
static void tri_interp(const otri *T, float u, float v, float *ou, float *ov)
{
    *ou = (1 - u - v) * T->tu.x + u * T->tu.y + v * T->tu.z;
    *ov = (1 - u - v) * T->tv.x + u * T->tv.y + v * T->tv.z;
}

/* ------------------------------------------------------------------------- */
/* BVH (tp2/projets/bvh.{h,cpp})                                               */
/* ------------------------------------------------------------------------- */
#define NPLANES 7
static v3 PN[NPLANES];   /* PLANE_NORMALS, bvh.cpp:8-16 */

static void init_plane_normals(void)
{
    float s = sqrtf(3.0f) / 3;
    float ms = -sqrtf(3.0f) / 3;
    PN[0] = V(1, 0, 0);
    PN[1] = V(0, 1, 0);
    PN[2] = V(0, 0, 1);
    PN[3] = V(s, s, s);
    PN[4] = V(ms, s, s);
    PN[5] = V(ms, ms, s);
    PN[6] = V(s, ms, s);
}

typedef struct {
    v3 bmin, bmax;
    int is_leaf;
    int child[8];
    int *tris, ntris, cap;
    float dn[NPLANES], df[NPLANES];
} onode;

typedef struct {
    onode *nodes;
    int nnodes, cap;
    const otri *tris;
    int max_depth, leaf;
} obvh;

static int node_new(obvh *B, v3 mn, v3 mx)
{
    if (B->nnodes == B->cap) {
        B->cap = B->cap ? B->cap * 2 : 1024;
        B->nodes = (onode *)realloc(B->nodes, sizeof(onode) * B->cap);
    }
    onode *n = &B->nodes[B->nnodes];
    memset(n, 0, sizeof(*n));
    n->bmin = mn;
    n->bmax = mx;
    n->is_leaf = 1;
    for (int i = 0; i < NPLANES; i++) {   /* BoundingVolume(), bvh.h:24-31 */
        n->dn[i] = INFINITY;
        n->df[i] = -INFINITY;
    }
    return B->nnodes++;
}

static void node_push_tri(onode *n, int t)
{
    if (n->ntris == n->cap) {
        n->cap = n->cap ? n->cap * 2 : 8;
        n->tris = (int *)realloc(n->tris, sizeof(int) * n->cap);
    }
    n->tris[n->ntris++] = t;
}

/* OctreeNode::create_children, bvh.h:153-167 (child 2/4/6 minima are _min + Point(...), kept as-is) */
static void create_children(obvh *B, int ni)
{
    v3 mn = B->nodes[ni].bmin, mx = B->nodes[ni].bmax;
    float mx_ = (mn.x + mx.x) / 2;
    float my_ = (mn.y + mx.y) / 2;
    float mz_ = (mn.z + mx.z) / 2;
    v3 lo[8], hi[8];
    lo[0] = mn;                                       hi[0] = V(mx_, my_, mz_);
    lo[1] = V(mx_, mn.y, mn.z);                       hi[1] = V(mx.x, my_, mz_);
    lo[2] = vadd(mn, V(0, my_, 0));                   hi[2] = V(mx_, mx.y, mz_);
    lo[3] = V(mx_, my_, mn.z);                        hi[3] = V(mx.x, mx.y, mz_);
    lo[4] = vadd(mn, V(0, 0, mz_));                   hi[4] = V(mx_, my_, mx.z);
    lo[5] = V(mx_, mn.y, mz_);                        hi[5] = V(mx.x, my_, mx.z);
    lo[6] = vadd(mn, V(0, my_, mz_));                 hi[6] = V(mx_, mx.y, mx.z);
    lo[7] = V(mx_, my_, mz_);                         hi[7] = V(mx.x, mx.y, mx.z);
    for (int i = 0; i < 8; i++) {
        int c = node_new(B, lo[i], hi[i]);
        B->nodes[ni].child[i] = c;
    }
}

/* Triangle::bbox_centroid, triangle.cpp:162-165 */
static v3 bbox_centroid(const otri *T)
{
    v3 mn = V(smin(T->a.x, smin(T->b.x, T->c.x)), smin(T->a.y, smin(T->b.y, T->c.y)), smin(T->a.z, smin(T->b.z, T->c.z)));
    v3 mx = V(smax(T->a.x, smax(T->b.x, T->c.x)), smax(T->a.y, smax(T->b.y, T->c.y)), smax(T->a.z, smax(T->b.z, T->c.z)));
    float kk = 1.f / 2;  /* Point / float, vec.cpp:56-60 */
    v3 s = vadd(mn, mx);
    return vscale(kk, s);
}

static void node_insert(obvh *B, int ni, int t, int depth);

/* OctreeNode::insert_to_children, bvh.h:195-210 */
static void insert_to_children(obvh *B, int ni, int t, int depth)
{
    v3 c = bbox_centroid(&B->tris[t]);
    v3 mn = B->nodes[ni].bmin, mx = B->nodes[ni].bmax;
    float mx_ = (mn.x + mx.x) / 2;
    float my_ = (mn.y + mx.y) / 2;
    float mz_ = (mn.z + mx.z) / 2;
    int oct = 0;
    if (c.x > mx_) oct += 1;
    if (c.y > my_) oct += 2;
    if (c.z > mz_) oct += 4;
    node_insert(B, B->nodes[ni].child[oct], t, depth + 1);
}

/* OctreeNode::insert, bvh.h:169-193 */
static void node_insert(obvh *B, int ni, int t, int depth)
{
    int depth_exceeded = depth == B->max_depth;
    if (B->nodes[ni].is_leaf || depth_exceeded) {
        node_push_tri(&B->nodes[ni], t);
        if ((size_t)B->nodes[ni].ntris > (size_t)(long)B->leaf && !depth_exceeded) {
            B->nodes[ni].is_leaf = 0;
            create_children(B, ni);
            int n = B->nodes[ni].ntris;
            int *list = B->nodes[ni].tris;
            for (int k = 0; k < n; k++)
                insert_to_children(B, ni, list[k], depth);
            free(B->nodes[ni].tris);
            B->nodes[ni].tris = NULL;
            B->nodes[ni].ntris = 0;
            B->nodes[ni].cap = 0;
        }
    } else
        insert_to_children(B, ni, t, depth);
}

/* BoundingVolume::triangle_volume + extend_volume, bvh.h:33-74 */
static void extend_with_triangle(onode *n, const otri *T)
{
    float dn[NPLANES], df[NPLANES];
    for (int i = 0; i < NPLANES; i++) {
        dn[i] = INFINITY;
        df[i] = -INFINITY;
    }
    const v3 *vs[3] = {&T->a, &T->b, &T->c};
    for (int i = 0; i < NPLANES; i++)
        for (int j = 0; j < 3; j++) {
            float dist = vdot(PN[i], *vs[j]);
            dn[i] = smin(dn[i], dist);
            df[i] = smax(df[i], dist);
        }
    for (int i = 0; i < NPLANES; i++) {
        n->dn[i] = smin(n->dn[i], dn[i]);
        n->df[i] = smax(n->df[i], df[i]);
    }
}

/* OctreeNode::compute_volume, bvh.h:141-151 */
static void compute_volume(obvh *B, int ni)
{
    if (B->nodes[ni].is_leaf) {
        for (int k = 0; k < B->nodes[ni].ntris; k++)
            extend_with_triangle(&B->nodes[ni], &B->tris[B->nodes[ni].tris[k]]);
    } else {
        for (int i = 0; i < 8; i++) {
            int c = B->nodes[ni].child[i];
            compute_volume(B, c);
            for (int p = 0; p < NPLANES; p++) {
                B->nodes[ni].dn[p] = smin(B->nodes[ni].dn[p], B->nodes[c].dn[p]);
                B->nodes[ni].df[p] = smax(B->nodes[ni].df[p], B->nodes[c].df[p]);
            }
        }
    }
}

/* BVH::BVH + build_bvh, bvh.cpp:19-66 */
static void bvh_build(obvh *B, const otri *tris, int64_t ntri, int max_depth, int leaf)
{
    memset(B, 0, sizeof(*B));
    B->tris = tris;
    B->max_depth = max_depth;
    B->leaf = leaf;
    v3 mn = V(INFINITY, INFINITY, INFINITY), mx = V(-INFINITY, -INFINITY, -INFINITY);
    for (int64_t i = 0; i < ntri; i++) {
        const v3 *vs[3] = {&tris[i].a, &tris[i].b, &tris[i].c};
        for (int k = 0; k < 3; k++) {
            mn = V(smin(mn.x, vs[k]->x), smin(mn.y, vs[k]->y), smin(mn.z, vs[k]->z));
            mx = V(smax(mx.x, vs[k]->x), smax(mx.y, vs[k]->y), smax(mx.z, vs[k]->z));
        }
    }
    int root = node_new(B, mn, mx);
    for (int64_t i = 0; i < ntri; i++)
        node_insert(B, root, (int)i, 0);
    compute_volume(B, root);
}

static void bvh_free(obvh *B)
{
    for (int i = 0; i < B->nnodes; i++)
        free(B->nodes[i].tris);
    free(B->nodes);
    memset(B, 0, sizeof(*B));
}

typedef struct {
    v3 o, d;
    float denoms[NPLANES], numers[NPLANES];
} oray;

/* OctreeNode::intersect(ray, hit) precompute, bvh.h:212-226 */
static oray make_ray(v3 o, v3 d)
{
    oray r;
    r.o = o;
    r.d = d;
    for (int i = 0; i < NPLANES; i++) {
        r.denoms[i] = vdot(PN[i], d);
        r.numers[i] = vdot(PN[i], o);
    }
    return r;
}

/* BoundingVolume::intersect, bvh.h:79-105 */
static int vol_intersect(const onode *n, const oray *r, float *t_near_out, float *t_far_out)
{
    float t_near = -INFINITY, t_far = INFINITY;
    *t_near_out = t_near;
    *t_far_out = t_far;
    for (int i = 0; i < NPLANES; i++) {
        float denom = r->denoms[i];
        if (denom == 0.0)
            continue;
        float dn = (n->dn[i] - r->numers[i]) / denom;
        float df = (n->df[i] - r->numers[i]) / denom;
        if (denom < 0) {
            float tmp = dn;
            dn = df;
            df = tmp;
        }
        t_near = smax(t_near, dn);
        t_far = smin(t_far, df);
        *t_near_out = t_near;
        *t_far_out = t_far;
        if (t_far < t_near)
            return 0;
    }
    return 1;
}

/* std::priority_queue<QueueElement, vector, std::greater<QueueElement>> on
 * at most 8 elements: libstdc++ push_heap / pop_heap (bits/stl_heap.h),
 * comparator a > b on _t_near (bvh.h:110-123, 250). */
typedef struct { int node; float key; } qel;
typedef struct { qel e[8]; int len; } oheap;

static inline int qgt(qel a, qel b) { return a.key > b.key; }

static void heap_push_hole(qel *first, int hole, int top, qel value)
{
    int parent = (hole - 1) / 2;
    while (hole > top && qgt(first[parent], value)) {
        first[hole] = first[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    first[hole] = value;
}

static void heap_push(oheap *h, qel e)
{
    h->e[h->len] = e;
    heap_push_hole(h->e, h->len, 0, e);
    h->len++;
}

static void heap_adjust(qel *first, int hole, int len, qel value)
{
    int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (qgt(first[second], first[second - 1]))
            second--;
        first[hole] = first[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        first[hole] = first[second - 1];
        hole = second - 1;
    }
    heap_push_hole(first, hole, top, value);
}

static void heap_pop(oheap *h)
{
    if (h->len > 1) {
        int last = h->len - 1;
        qel value = h->e[last];
        h->e[last] = h->e[0];
        heap_adjust(h->e, 0, last, value);
    }
    h->len--;
}

typedef struct {
    int64_t vol, tri, child;
} tcount;

/* OctreeNode::intersect(ray, hit, t_near, denoms, numers), bvh.h:228-287 */
static int node_intersect(const obvh *B, int ni, const oray *r, ohit *hit, float *t_near_out, tcount *tc)
{
    float t_far, trash;
    const onode *n = &B->nodes[ni];
    tc->vol++;
    if (!vol_intersect(n, r, &trash, &t_far))
        return 0;
    if (n->is_leaf) {
        for (int k = 0; k < n->ntris; k++) {
            ohit local = hit_fresh();
            int ti = n->tris[k];
            tc->tri++;
            if (tri_intersect(&B->tris[ti], ti, r->o, r->d, &local))
                if (local.t < hit->t || hit->t == -1)
                    *hit = local;
        }
        *t_near_out = hit->t;
        return *t_near_out > 0;
    }
    oheap q;
    q.len = 0;
    for (int i = 0; i < 8; i++) {
        float inter;
        tc->vol++;
        tc->child++;
        if (vol_intersect(&B->nodes[n->child[i]], r, &inter, &t_far)) {
            qel e = {n->child[i], inter};
            heap_push(&q, e);
        }
    }
    float closest = INFINITY, inter_distance = INFINITY;
    while (q.len > 0) {
        qel top = q.e[0];
        heap_pop(&q);
        if (node_intersect(B, top.node, r, hit, &inter_distance, tc)) {
            closest = smin(closest, inter_distance);
            if (q.len == 0 || closest < q.e[0].key) {
                *t_near_out = closest;
                return 1;
            }
        }
    }
    if (closest == INFINITY)
        return 0;
    *t_near_out = closest;
    return 1;
}

/* BVH::intersect, bvh.cpp:68-71 */
static int bvh_intersect(const obvh *B, v3 o, v3 d, ohit *hit, tcount *tc)
{
    if (B->nnodes == 0)
        return 0;
    oray r = make_ray(o, d);
    float trash;
    tc->child++;   /* the root's own test */
    return node_intersect(B, 0, &r, hit, &trash, tc);
}

/* ------------------------------------------------------------------------- */
/* Analytic shapes (tp2/projets/analyticShape.cpp)                             */
/* ------------------------------------------------------------------------- */
/* Sphere::intersect, analyticShape.cpp:9-60 (hit->t may be read stale) */
static int sphere_intersect(const float *s, int mat, v3 o, v3 d, ohit *h)
{
    v3 c = V(s[0], s[1], s[2]);
    float r2 = s[3] * s[3];
    v3 L = vsub(o, c);
    const float a = 1;
    float b = 2 * vdot(d, L);
    float cc = vdot(L, L) - r2;
    float delta = b * b - 4 * a * cc;
    if (delta < 0)
        return 0;
    const float a2 = 2 * a;
    if (delta == 0.0)
        h->t = -b / a2;
    else {
        float sq = sqrtf(delta);
        float t1 = (-b - sq) / a2;
        float t2 = (-b + sq) / a2;
        if (t1 < t2) {
            h->t = t1;
            if (h->t < 0)
                h->t = t2;
        }
    }
    if (h->t < 0)
        return 0;
    v3 p = vadd(o, vscale(h->t, d));
    h->normal = vnormalize(vsub(p, c));
    h->u = 0.5f + atan2f(-h->normal.z, -h->normal.x) / (2.0f * (float)M_PI);
    h->v = 0.5f + asinf(-h->normal.y) / (float)M_PI;
    h->tangent = vcross(V(0, 1, 0), h->normal);
    h->mat = mat;
    return 1;
}

/* Plane::intersect, analyticShape.cpp:64-76 */
static int plane_intersect(const float *p, int mat, v3 o, v3 d, ohit *h)
{
    v3 n = V(p[3], p[4], p[5]);
    float t = vdot(vsub(V(p[0], p[1], p[2]), o), n) / vdot(d, n);
    if (t < 0)
        return 0;
    h->t = t;
    h->mat = mat;
    h->normal = n;
    return 1;
}

/* ------------------------------------------------------------------------- */
/* Images (tp2/src/image.h) and Skybox (tp2/projets/renderer/skybox.cpp)      */
/* ------------------------------------------------------------------------- */
typedef struct { int w, h; const float *px; } oimg;

/* Image::offset, image.h:122-134 */
static inline const float *img_at(const oimg *I, int x, int y)
{
    int px = x;
    if (px < 0) px = 0;
    if (px > I->w - 1) px = I->w - 1;
    int py = y;
    if (py < 0) py = 0;
    if (py > I->h - 1) py = I->h - 1;
    unsigned p = (unsigned)(py * I->w + px);
    return I->px + 4 * (size_t)p;
}

/* Image::texture_floor -> sample_floor, image.h:79-86, 94-97 */
static c3 tex_floor_a(const oimg *I, float x, float y, float *alpha)
{
    float u = floorf(x * I->w);
    float v = floorf(y * I->h);
    const float *p = img_at(I, f2i(u), f2i(v));
    if (alpha) *alpha = p[3];
    return C(p[0], p[1], p[2]);
}
static c3 tex_floor(const oimg *I, float x, float y) { return tex_floor_a(I, x, y, NULL); }

/* Image::texture_bilinear -> sample_bilinear, image.h:66-77, 89-92 */
static c3 tex_bilinear(const oimg *I, float xx, float yy, float *alpha)
{
    float x = xx * I->w, y = yy * I->h;
    float u = x - floorf(x);
    float v = y - floorf(y);
    int ix = f2i(x);
    int iy = f2i(y);
    const float *p00 = img_at(I, ix, iy), *p10 = img_at(I, ix + 1, iy);
    const float *p01 = img_at(I, ix, iy + 1), *p11 = img_at(I, ix + 1, iy + 1);
    float w00 = (1 - u) * (1 - v), w10 = u * (1 - v), w01 = (1 - u) * v, w11 = u * v;
    c3 r;
    r.r = p00[0] * w00 + p10[0] * w10 + p01[0] * w01 + p11[0] * w11;
    r.g = p00[1] * w00 + p10[1] * w10 + p01[1] * w01 + p11[1] * w11;
    r.b = p00[2] * w00 + p10[2] * w10 + p01[2] * w01 + p11[2] * w11;
    if (alpha) *alpha = p00[3] * w00 + p10[3] * w10 + p01[3] * w01 + p11[3] * w11;
    return r;
}

/* Skybox::sample, skybox.cpp:12-51 */
static c3 skybox_sample(const oimg *faces, v3 dir, float *alpha)
{
    v3 d2 = V(dir.x, dir.y, -dir.z);
    v3 da = V(fabsf(d2.x), fabsf(d2.y), fabsf(d2.z));
    int face;
    float nf, u, v;
    if (da.z >= da.x && da.z >= da.y) {
        face = d2.z < 0.0 ? 4 : 5;
        nf = 0.5 / da.z;
        u = d2.z < 0.0 ? -d2.x : d2.x;
        v = -d2.y;
    } else if (da.y >= da.x) {
        face = d2.y < 0.0 ? 3 : 2;
        nf = 0.5 / da.y;
        u = d2.x;
        v = d2.y < 0.0 ? -d2.z : d2.z;
    } else {
        face = d2.x < 0.0 ? 1 : 0;
        nf = 0.5 / da.x;
        u = d2.x < 0.0 ? d2.z : -d2.z;
        v = -d2.y;
    }
    u = u * nf + 0.5;
    v = v * nf + 0.5;
    return tex_bilinear(&faces[face], u, v, alpha);
}

/* ------------------------------------------------------------------------- */
/* Renderer (tp2/projets/renderer/renderer.cpp)                                */
/* ------------------------------------------------------------------------- */
#define ORC_RASTER_SLOTS 256
struct orc_ctx {
    orc_scene sc;
    orc_settings s;
    otri *tris;
    int64_t ntri;
    obvh bvh;
    oimg tex[ORC_TEX_COUNT];
    oimg sky[6];
    int rw, rh;
};

typedef struct {
    const struct orc_ctx *X;
    uint32_t rng;
    uint32_t frame_key;   /* key of the next compute_reflection frame (see pixel_seed) */
    orc_counters *cnt;
    int ray_kind;   /* 0 primary, 1 shadow, 2 reflection (for counters) */
    float alpha;    /* Color::a of the last trace_ray result (sky textures carry theirs) */
} otracer;

static const float EPS_SHADOW = 1.0e-4f;       /* Renderer::EPSILON, renderer.h:23 */
static const float SHADOW_INTENSITY = 0.5f;    /* renderer.h:24 */

static c3 ambient_color(void) { return C(0.1f, 0.1f, 0.1f); }                                 /* renderer.cpp:18 */
static c3 background_color(void) { return C(135.0f / 255.0f, 206.0f / 255.0f, 235.0f / 255.0f); } /* renderer.cpp:19 */

static uint32_t pixel_seed(uint32_t pixel, uint32_t seed)
{
    uint32_t x = pixel * 0x9E3779B9u ^ seed;
    x ^= x >> 16; x *= 0x7feb352dU;
    x ^= x >> 15; x *= 0x846ca68bU;
    x ^= x >> 16;
    return x ? x : 0x9E3779B9u;
}

/* Path-keyed streams (ref_harness.cpp HRng): the frame of a primary hit is keyed
 * pixel_seed(pixel, seed); sample i of a frame draws from sample_state(key, i) and
 * the frame its hit spawns is keyed child_key(key, i). */
static uint32_t mix32(uint32_t x)
{
    x ^= x >> 16; x *= 0x7feb352dU;
    x ^= x >> 15; x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

static uint32_t sample_state(uint32_t key, uint32_t i)
{
    uint32_t x = mix32(key ^ (0x9E3779B9u * (2u * i + 1u)));
    return x ? x : 0x9E3779B9u;
}

static uint32_t child_key(uint32_t key, uint32_t i) { return mix32(key ^ (0x85EBCA6Bu * (2u * i + 2u))); }

/* XorShiftGenerator::get_rand / get_rand_bilateral, xorshift.h:43-57 */
static float rng_bilateral(otracer *T)
{
    uint32_t x = T->rng;
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    T->rng = x;
    return (float)x / (float)UINT32_MAX * 2 - 1;
}

static void count_traversal(otracer *T, const tcount *tc)
{
    if (!T->cnt)
        return;
    if (T->ray_kind == 0) {
        T->cnt->vol_tests_primary += tc->vol;
        T->cnt->tri_tests_primary += tc->tri;
        T->cnt->child_tests_primary += tc->child;
    } else if (T->ray_kind == 1) {
        T->cnt->vol_tests_shadow += tc->vol;
        T->cnt->tri_tests_shadow += tc->tri;
        T->cnt->child_tests_shadow += tc->child;
    } else {
        T->cnt->vol_tests_refl += tc->vol;
        T->cnt->tri_tests_refl += tc->tri;
    }
}

static const float *mat_of(const struct orc_ctx *X, int id) { return X->sc.mat + (size_t)ORC_MAT_STRIDE * id; }
static c3 mat_color(const float *m, int off) { return C(m[off], m[off + 1], m[off + 2]); }

/* renderer.cpp:436-445 */
static void get_tex_coords(const struct orc_ctx *X, int tri, float u, float v, float *tu, float *tv)
{
    if (tri >= 0)
        tri_interp(&X->tris[tri], u, v, tu, tv);
    else {
        *tu = u;
        *tv = v;
    }
}

/* renderer.cpp:464-478 */
static v3 normal_mapping(const struct orc_ctx *X, const ohit *h, float u, float v)
{
    float tu, tv;
    get_tex_coords(X, h->tri, u, v, &tu, &tv);
    v3 T = h->tangent;
    v3 Bt = vcross(T, h->normal);
    v3 N = h->normal;
    c3 nc = tex_floor(&X->tex[ORC_TEX_NORMAL], tu, tv);
    v3 nm = vsub(vscale(2, V(nc.r, nc.g, nc.b)), V(1, 1, 1));
    v3 q = vnormalize(nm);
    /* Transform(T, B, N, 0) applied to a Vector (mat.cpp:67-73, 103-115) */
    float m00 = T.x, m01 = Bt.x, m02 = N.x;
    float m10 = T.y, m11 = Bt.y, m12 = N.y;
    float m20 = T.z, m21 = Bt.z, m22 = N.z;
    v3 p = V(m00 * q.x + m01 * q.y + m02 * q.z, m10 * q.x + m11 * q.y + m12 * q.z, m20 * q.x + m21 * q.y + m22 * q.z);
    return vnormalize(p);
}

/* renderer.cpp:518-554 */
static void parallax_occlusion_mapping(const struct orc_ctx *X, int tri, float u, float v, v3 view, float *nu, float *nv)
{
    float tu, tv;
    get_tex_coords(X, tri, u, v, &tu, &tv);
    const oimg *D = &X->tex[ORC_TEX_DISPLACEMENT];
    int steps = X->s.parallax_mapping_steps;
    float current_depth;
    float depth_step = 1.0f / steps;
    float sampled = tex_floor(D, tu, tv).r;
    v3 search = vscale(X->s.displacement_mapping_strength, vneg(view));
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
    *nu = (1 - w) * u2 + w * pu;
    *nv = (1 - w) * v2 + w * pv;
}

static c3 trace_ray(otracer *T, v3 ro, v3 rd, ohit *fin, int depth, int *found, int *src_out, int *shadowed_out);

/* renderer.cpp:340-402 */
static int is_shadowed(otracer *T, v3 p, v3 n, v3 lp)
{
    const struct orc_ctx *X = T->X;
    if (!X->s.compute_shadows)
        return 0;
    if (T->cnt) T->cnt->shadow_rays++;
    v3 o = vadd(p, vscale(EPS_SHADOW, n));
    v3 d = vnormalize(vsub(lp, p));
    ohit hi = hit_fresh();
    if (X->s.enable_bvh) {
        tcount tc = {0, 0, 0};
        int saved = T->ray_kind;
        T->ray_kind = 1;
        int r = bvh_intersect(&X->bvh, o, d, &hi, &tc);
        count_traversal(T, &tc);
        T->ray_kind = saved;
        if (r) {
            v3 q = vadd(o, vscale(hi.t, d));
            if (vlength2(vsub(p, q)) < vlength2(vsub(p, lp)))
                return 1;
        }
    } else {
        for (int64_t i = 0; i < X->ntri; i++)
            if (tri_intersect(&X->tris[i], (int)i, o, d, &hi)) {
                v3 q = vadd(o, vscale(hi.t, d));
                if (vlength2(vsub(p, q)) < vlength2(vsub(p, lp)))
                    return 1;
            }
    }
    for (int k = 0; k < X->sc.nshape; k++) {
        int hitk = X->sc.shape_kind[k] == 0 ? sphere_intersect(X->sc.shape + 6 * k, X->sc.shape_mat[k], o, d, &hi)
                                            : plane_intersect(X->sc.shape + 6 * k, X->sc.shape_mat[k], o, d, &hi);
        if (hitk) {
            v3 q = vadd(o, vscale(hi.t, d));
            if (vlength2(vsub(p, q)) < vlength2(vsub(p, lp)))
                return 1;
        }
    }
    return 0;
}

/* renderer.cpp:283-338 */
static c3 compute_reflection(otracer *T, v3 rd_in, v3 ip, const ohit *h, int depth)
{
    const struct orc_ctx *X = T->X;
    int found = 0;
    ohit rhi = hit_fresh();
    const float *m = mat_of(X, h->mat);
    v3 nn = h->normal;
    v3 ro = vadd(ip, vscale(0.01f, nn));
    v3 perfect = vsub(rd_in, vscale(2 * vdot(rd_in, nn), nn));
    int sample_count = 0;
    c3 total = C(0.0f, 0.0f, 0.0f);
    const uint32_t key = T->frame_key;
    for (int i = 0; i < X->s.rough_reflections_sample_count; i++) {
        T->rng = sample_state(key, (uint32_t)i);
        T->frame_key = child_key(key, (uint32_t)i);
        float roughness;
        if (X->s.enable_roughness_mapping) {
            float tu, tv;
            get_tex_coords(X, h->tri, h->u, h->v, &tu, &tv);
            roughness = tex_floor(&X->tex[ORC_TEX_ROUGHNESS], tu, tv).r;
        } else
            roughness = m[ORC_MAT_ROUGHNESS];
        if (roughness > 0) {
            float rx = rng_bilateral(T);
            float ry = rng_bilateral(T);
            float rz = rng_bilateral(T);
            v3 rdir = vnormalize(V(rx, ry, rz));
            if (vdot(rdir, h->normal) < 0)
                rdir = vneg(rdir);
            v3 lerped = vadd(vscale(roughness, rdir), vscale(1 - roughness, perfect));
            if (T->cnt) T->cnt->reflection_rays++;
            total = cadd(total, trace_ray(T, ro, lerped, &rhi, depth + 1, &found, NULL, NULL));
            sample_count++;
        } else {
            if (T->cnt) T->cnt->reflection_rays++;
            total = cadd(total, trace_ray(T, ro, perfect, &rhi, depth + 1, &found, NULL, NULL));
            sample_count = 1;
            break;
        }
    }
    float sc = (float)sample_count;
    float rf = m[ORC_MAT_REFLECTION];
    return cmul(cdiv(total, C(sc, sc, sc)), C(rf, rf, rf));
}

/* renderer.cpp:556-617 */
static c3 shade(otracer *T, v3 ro, v3 rd, ohit *h, int depth, int *shadowed_out)
{
    const struct orc_ctx *X = T->X;
    const orc_settings *S = &X->s;
    c3 fc = C(0.0f, 0.0f, 0.0f);
    if (S->shading_method == ORC_RT_SHADING) {
        float u = h->u, v = h->v;
        v3 ip = vadd(ro, vscale(h->t, rd));
        v3 cam = V(X->sc.cam_pos[0], X->sc.cam_pos[1], X->sc.cam_pos[2]);
        v3 light = V(X->sc.light[0], X->sc.light[1], X->sc.light[2]);
        if (S->enable_displacement_mapping)
            parallax_occlusion_mapping(X, h->tri, h->u, h->v, vnormalize(vsub(cam, ip)), &u, &v);
        v3 dl = vnormalize(vsub(light, ip));
        if (S->enable_normal_mapping)
            h->normal = normal_mapping(X, h, u, v);
        const float *m = mat_of(X, h->mat);
        float ao = 1.0f;
        if (S->enable_ao_mapping) {
            float tu, tv;
            get_tex_coords(X, h->tri, u, v, &tu, &tv);
            ao = tex_floor(&X->tex[ORC_TEX_AO], tu, tv).r;
        }
        c3 dc;
        if (S->enable_diffuse_mapping) {
            float tu, tv;
            get_tex_coords(X, h->tri, u, v, &tu, &tv);
            dc = tex_floor(&X->tex[ORC_TEX_DIFFUSE], tu, tv);
            float f = smax(0.5f, vdot(h->normal, vnormalize(vsub(cam, ip))));
            dc = cmul(dc, C(f, f, f));
        } else {
            float f = smax(0.0f, vdot(h->normal, dl));     /* compute_diffuse, :263-266 */
            dc = cmul(mat_color(m, ORC_MAT_DIFFUSE), C(f, f, f));
        }
        fc = cadd(fc, cmulf(cmulf(dc, ao), (float)(S->enable_diffuse != 0)));
        /* compute_specular, :270-280 */
        c3 spec;
        {
            v3 hv = vnormalize(vsub(dl, rd));
            float angle = vdot(hv, h->normal);
            if (angle <= m[ORC_MAT_SPEC_THRESHOLD])
                spec = C(0, 0, 0);
            else {
                float p = powf(smax(0.0f, angle), m[ORC_MAT_NS]);
                spec = cmul(mat_color(m, ORC_MAT_SPECULAR), C(p, p, p));
            }
        }
        fc = cadd(fc, cmulf(spec, (float)(S->enable_specular != 0)));
        int sh = is_shadowed(T, ip, h->normal, light);
        if (shadowed_out) *shadowed_out = sh;
        if (sh)
            fc = cmul(fc, C(SHADOW_INTENSITY, SHADOW_INTENSITY, SHADOW_INTENSITY));
        fc = cadd(fc, cmulf(mat_color(m, ORC_MAT_EMISSION), (float)(S->enable_emissive != 0)));
        float refl = m[ORC_MAT_REFLECTION];
        if (refl > 0.0f)
            fc = cadd(fc, cmulf(compute_reflection(T, rd, ip, h, depth), refl));
        fc = cadd(fc, cmulf(cmulf(cmul(ambient_color(), mat_color(m, ORC_MAT_AMBIENT)), 1 - refl),
                            (float)(S->enable_ambient != 0)));
    } else if (S->shading_method == ORC_ABS_NORMALS_SHADING) {          /* :404-407 */
        fc = C(fabsf(h->normal.x), fabsf(h->normal.y), fabsf(h->normal.z));
    } else if (S->shading_method == ORC_PASTEL_NORMALS_SHADING) {       /* :409-412 */
        fc = cmulf(cadd(C(h->normal.x, h->normal.y, h->normal.z), C(1.0f, 1.0f, 1.0f)), 0.5);
    } else if (S->shading_method == ORC_BARYCENTRIC_COORDINATES_SHADING) { /* :414-417 */
        fc = cadd(cadd(cmulf(C(1, 0, 0), h->u), cmulf(C(0, 1.0, 0), h->v)), cmulf(C(0, 0, 1), 1 - h->u - h->v));
    } else if (S->shading_method == ORC_VISUALIZE_AO) {                 /* :419-434 */
        c3 c = C(0.9f, 0.9f, 0.9f);
        if (S->enable_ao_mapping) {
            float tu, tv;
            tri_interp(&X->tris[h->tri], h->u, h->v, &tu, &tv);
            float a = tex_floor(&X->tex[ORC_TEX_AO], tu, tv).r;
            c = cmul(c, C(a, a, a));
        }
        fc = c;
    }
    fc.r = sclamp01(fc.r);
    fc.g = sclamp01(fc.g);
    fc.b = sclamp01(fc.b);
    return fc;
}

/* renderer.cpp:1008-1066 */
static c3 trace_ray(otracer *T, v3 ro, v3 rd, ohit *fin, int depth, int *found, int *src_out, int *shadowed_out)
{
    const struct orc_ctx *X = T->X;
    const orc_settings *S = &X->s;
    ohit local = hit_fresh();
    if (depth > S->max_recursion_depth) {
        T->alpha = 1.0f;
        return C(0.0f, 0.0f, 0.0f);
    }
    int src = -1;
    T->ray_kind = depth == 0 ? 0 : 2;
    if (S->enable_bvh) {
        tcount tc = {0, 0, 0};
        int r = bvh_intersect(&X->bvh, ro, rd, &local, &tc);
        count_traversal(T, &tc);
        if (r)
            if (local.t < fin->t || fin->t == -1) {
                *fin = local;
                src = local.tri;
            }
    } else {
        for (int64_t i = 0; i < X->ntri; i++)
            if (tri_intersect(&X->tris[i], (int)i, ro, rd, &local))
                if (local.t < fin->t || fin->t == -1) {
                    *fin = local;
                    src = (int)i;
                }
    }
    for (int k = 0; k < X->sc.nshape; k++) {
        int hitk = X->sc.shape_kind[k] == 0 ? sphere_intersect(X->sc.shape + 6 * k, X->sc.shape_mat[k], ro, rd, &local)
                                            : plane_intersect(X->sc.shape + 6 * k, X->sc.shape_mat[k], ro, rd, &local);
        if (hitk)
            if (local.t < fin->t || fin->t == -1) {
                *fin = local;
                src = -2 - k;
            }
    }
    if (src_out) *src_out = src;
    float min_t = 0.1;
    if (fin->t > min_t) {
        *found = 1;
        int saved = T->ray_kind;
        c3 c = shade(T, ro, rd, fin, depth, shadowed_out);
        T->ray_kind = saved;
        c.r = sclamp01(c.r);
        c.g = sclamp01(c.g);
        c.b = sclamp01(c.b);
        T->alpha = 1.0f;
        return c;
    }
    if (S->enable_skysphere) {
        float u = 0.5 + atan2f(-rd.z, -rd.x) / (2 * M_PI);
        float v = 0.5 + asinf(-rd.y) / M_PI;
        return tex_floor_a(&X->tex[ORC_TEX_SKYSPHERE], u, v, &T->alpha);
    } else if (S->enable_skybox)
        return skybox_sample(X->sky, rd, &T->alpha);
    T->alpha = 1.0f;
    return background_color();
}

/* ------------------------------------------------------------------------- */
/* Public (test-only) API                                                      */
/* ------------------------------------------------------------------------- */
ORC_API struct orc_ctx *orc_create(const orc_scene *sc, const orc_settings *s)
{
    init_plane_normals();
    struct orc_ctx *X = (struct orc_ctx *)calloc(1, sizeof(struct orc_ctx));
    X->sc = *sc;
    X->s = *s;
    X->ntri = sc->ntri;
    /* + ORC_RASTER_SLOTS: per-thread temporary triangles of raster_trace's shading */
    X->tris = (otri *)calloc((size_t)sc->ntri + ORC_RASTER_SLOTS, sizeof(otri));
    for (int64_t i = 0; i < sc->ntri; i++) {
        const float *t = sc->tri + 9 * i;
        otri *T = &X->tris[i];
        T->a = V(t[0], t[1], t[2]);
        T->b = V(t[3], t[4], t[5]);
        T->c = V(t[6], t[7], t[8]);
        T->n = vcross(vsub(T->b, T->a), vsub(T->c, T->a));
        T->mat = sc->tri_mat ? sc->tri_mat[i] : -1;
        if (sc->tri_uv) {
            const float *uv = sc->tri_uv + 6 * i;
            T->tu = V(uv[0], uv[1], uv[2]);
            T->tv = V(uv[3], uv[4], uv[5]);
        } else {
            T->tu = V(-1, -1, -1);
            T->tv = V(-1, -1, -1);
        }
    }
    if (s->enable_bvh)
        bvh_build(&X->bvh, X->tris, X->ntri, s->bvh_max_depth, s->bvh_leaf_object_count);
    for (int i = 0; i < ORC_TEX_COUNT; i++) {
        X->tex[i].w = sc->tex_w[i];
        X->tex[i].h = sc->tex_h[i];
        X->tex[i].px = sc->tex[i];
    }
    for (int i = 0; i < 6; i++) {
        X->sky[i].w = sc->sky_w[i];
        X->sky[i].h = sc->sky_h[i];
        X->sky[i].px = sc->sky[i];
    }
    X->rw = s->enable_ssaa ? s->image_width * s->ssaa_factor : s->image_width;
    X->rh = s->enable_ssaa ? s->image_height * s->ssaa_factor : s->image_height;
    return X;
}

ORC_API void orc_destroy(struct orc_ctx *X)
{
    if (!X)
        return;
    bvh_free(&X->bvh);
    free(X->tris);
    free(X);
}

static void add_counters(orc_counters *a, const orc_counters *b)
{
    a->primary_rays += b->primary_rays;
    a->shadow_rays += b->shadow_rays;
    a->reflection_rays += b->reflection_rays;
    a->vol_tests_primary += b->vol_tests_primary;
    a->tri_tests_primary += b->tri_tests_primary;
    a->vol_tests_shadow += b->vol_tests_shadow;
    a->tri_tests_shadow += b->tri_tests_shadow;
    a->vol_tests_refl += b->vol_tests_refl;
    a->tri_tests_refl += b->tri_tests_refl;
    a->child_tests_primary += b->child_tests_primary;
    a->child_tests_shadow += b->child_tests_shadow;
}

/* ------------------------------------------------------------------------- */
/* Renderer::raster_trace (renderer.cpp:869-1006): hybrid rasterisation.       */
/* The reference runs the triangle loop under OpenMP with an unsynchronised    */
/* z-test-and-write, so overlapping triangles race; the oracle (like the GPU)  */
/* defines the sequential result: triangles (and their clipped pieces) in      */
/* order, a pixel keeps the first candidate with the smallest z (strict <).    */
/* Every z-test pass shades the pixel in the reference; only the last one      */
/* survives, so only the winner is shaded here (its shading is per-pixel       */
/* deterministic, rough reflections included).                                 */
/* ------------------------------------------------------------------------- */
typedef struct { float x, y, z, w; } v4;
static inline v4 V4(float x, float y, float z, float w) { v4 r = {x, y, z, w}; return r; }
static inline v4 v4add(v4 a, v4 b) { return V4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }  /* vec.cpp:123-126 */
static inline v4 v4sub(v4 a, v4 b) { return V4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }  /* vec.cpp:128-131 */
static inline v4 v4mul(float t, v4 u) { return V4(u.x * t, u.y * t, u.z * t, u.w * t); }      /* vec.cpp:133-141 */
static inline float v4c(v4 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }

/* Transform::operator()(vec4), mat.cpp:118-131 */
static inline v4 xform4(const float *m, v4 v)
{
    return V4(m[0] * v.x + m[1] * v.y + m[2] * v.z + m[3] * v.w, m[4] * v.x + m[5] * v.y + m[6] * v.z + m[7] * v.w,
              m[8] * v.x + m[9] * v.y + m[10] * v.z + m[11] * v.w,
              m[12] * v.x + m[13] * v.y + m[14] * v.z + m[15] * v.w);
}

typedef struct { v4 a, b, c; v3 tu, tv; } otri4;   /* Triangle4, triangle.h:24-40 */

#define ORC_CLIP_MAX 12   /* std::array<Triangle4, 12> (renderer.h:304-309); more pieces are UB there and dropped here */

static inline int in_half(v4 p, int i, int sgn) { return sgn > 0 ? v4c(p, i) < p.w : v4c(p, i) > -p.w; }

/* clip_triangles_to_plane<i, sgn> (renderer.cpp:669-850); in may alias out when n == 1 */
static int clip_plane(const otri4 *in, int n, otri4 *out, int i, int sgn)
{
    int k = 0;
    const float fs = (float)sgn;
    for (int t = 0; t < n; t++) {
        const otri4 T = in[t];
        int ia = in_half(T.a, i, sgn), ib = in_half(T.b, i, sgn), ic = in_half(T.c, i, sgn);
        int cnt = ia + ib + ic;
        if (cnt == 3) {
            if (k < ORC_CLIP_MAX) out[k] = T;
            k++;
        } else if (cnt == 1) {
            /* (kept, lost1, lost2) rotated so the kept vertex leads, texcoords alike */
            v4 p0, p1, p2;
            float u0, u1, u2, w0, w1, w2;
            if (ia) { p0 = T.a; p1 = T.b; p2 = T.c; u0 = T.tu.x; u1 = T.tu.y; u2 = T.tu.z; w0 = T.tv.x; w1 = T.tv.y; w2 = T.tv.z; }
            else if (ib) { p0 = T.b; p1 = T.c; p2 = T.a; u0 = T.tu.y; u1 = T.tu.z; u2 = T.tu.x; w0 = T.tv.y; w1 = T.tv.z; w2 = T.tv.x; }
            else { p0 = T.c; p1 = T.a; p2 = T.b; u0 = T.tu.z; u1 = T.tu.x; u2 = T.tu.y; w0 = T.tv.z; w1 = T.tv.x; w2 = T.tv.y; }
            float d0 = v4c(p0, i) - p0.w * fs, d1 = v4c(p1, i) - p1.w * fs, d2 = v4c(p2, i) - p2.w * fs;
            float t1 = d1 / (d1 - d0), t2 = d2 / (d2 - d0);
            otri4 R;
            R.a = p0;
            R.b = v4add(p1, v4mul(t1 - 0.0f, v4sub(p0, p1)));
            R.c = v4add(p2, v4mul(t2 - 0.0f, v4sub(p0, p2)));
            R.tu = V(u0, u1 + (t1 - 0.0f) * (u0 - u1), u2 + (t2 - 0.0f) * (u0 - u2));
            R.tv = V(w0, w1 + (t1 - 0.0f) * (w0 - w1), w2 + (t2 - 0.0f) * (w0 - w2));
            if (k < ORC_CLIP_MAX) out[k] = R;
            k++;
        } else if (cnt == 2) {
            /* (kept1, kept2, lost): the lost vertex's successors lead */
            v4 q1, q2, q0;
            float u0, u1, u2, w0, w1, w2;
            if (!ia) { q0 = T.a; q1 = T.b; q2 = T.c; u0 = T.tu.y; u1 = T.tu.z; u2 = T.tu.x; w0 = T.tv.y; w1 = T.tv.z; w2 = T.tv.x; }
            else if (!ib) { q0 = T.b; q1 = T.c; q2 = T.a; u0 = T.tu.z; u1 = T.tu.x; u2 = T.tu.y; w0 = T.tv.z; w1 = T.tv.x; w2 = T.tv.y; }
            else { q0 = T.c; q1 = T.a; q2 = T.b; u0 = T.tu.x; u1 = T.tu.y; u2 = T.tu.z; w0 = T.tv.x; w1 = T.tv.y; w2 = T.tv.z; }
            float e1 = v4c(q1, i) - q1.w * fs, e2 = v4c(q2, i) - q2.w * fs, e0 = v4c(q0, i) - q0.w * fs;
            float t1 = e0 / (e0 - e1), t2 = e0 / (e0 - e2);
            v4 P1 = v4add(q0, v4mul(t1 - 0.0f, v4sub(q1, q0)));
            v4 P2 = v4add(q0, v4mul(t2 - 0.0f, v4sub(q2, q0)));
            otri4 R1, R2;
            R1.a = q1; R1.b = q2; R1.c = P2;
            R1.tu = V(u0, u1, u2 + (t2 - 0.0f) * (u1 - u2));
            R1.tv = V(w0, w1, w2 + (t2 - 0.0f) * (w1 - w2));
            R2.a = q1; R2.b = P2; R2.c = P1;
            R2.tu = V(u0, u2 + (t2 - 0.0f) * (u1 - u2), u2 + (t1 - 0.0f) * (u0 - u2));
            R2.tv = V(w0, w2 + (t2 - 0.0f) * (w1 - w2), w2 + (t1 - 0.0f) * (w0 - w2));
            if (k < ORC_CLIP_MAX) out[k] = R1;
            k++;
            if (k < ORC_CLIP_MAX) out[k] = R2;
            k++;
        }
    }
    return k < ORC_CLIP_MAX ? k : ORC_CLIP_MAX;
}

/* one clipped piece, everything raster_trace derives from it */
typedef struct {
    int tri, piece;
    v3 na, nb, nc;           /* Triangle(Triangle4) in NDC (triangle.cpp:12-23) */
    v3 tu, tv;
    float inv_area;
    int x0, y0, x1, y1;      /* pixel bounding box */
    float za, zb, zc;        /* matrix_transform_z(cam_to_world, proj_inv(vertex)) */
    otri world;              /* _camera_to_world_mat(proj_inv(NDC triangle)) */
    otri cam;                /* proj_inv(NDC triangle) */
} opiece;

/* (int)(double): cvttsd2si, INT_MIN out of range / NaN */
static inline int d2i(double d)
{
    if (!(d > -2147483649.0 && d < 2147483648.0))
        return INT32_MIN;
    return (int)d;
}

/* Renderer::matrix_transform_z, renderer.cpp:856-867 (a division, not a reciprocal) */
static inline float xform_z(const float *m, v3 p)
{
    float zt = m[8] * p.x + m[9] * p.y + m[10] * p.z + m[11];
    float wt = m[12] * p.x + m[13] * p.y + m[14] * p.z + m[15];
    if (wt == 1.0f)
        return zt;
    return zt / wt;
}

static otri tri_from(v3 a, v3 b, v3 c, int mat, v3 tu, v3 tv)   /* Triangle(Point...) ctor */
{
    otri t;
    t.a = a; t.b = b; t.c = c;
    t.n = vcross(vsub(b, a), vsub(c, a));
    t.mat = mat;
    t.tu = tu; t.tv = tv;
    return t;
}

static int make_pieces(const struct orc_ctx *X, int64_t ti, opiece *out)
{
    const otri *O = &X->tris[ti];
    const float *W2C = X->sc.world_to_cam, *PR = X->sc.proj, *PI = X->sc.proj_inv, *C2W = X->sc.cam_to_world;
    /* _world_to_camera_mat(original_triangle), then perspective_projection(vec4(point)) */
    v3 ca = xform_point(W2C, O->a), cb = xform_point(W2C, O->b), cc = xform_point(W2C, O->c);
    otri4 A[ORC_CLIP_MAX], B[ORC_CLIP_MAX];
    A[0].a = xform4(PR, V4(ca.x, ca.y, ca.z, 1.0f));
    A[0].b = xform4(PR, V4(cb.x, cb.y, cb.z, 1.0f));
    A[0].c = xform4(PR, V4(cc.x, cc.y, cc.z, 1.0f));
    A[0].tu = O->tu;
    A[0].tv = O->tv;
    int n = 1;
    const otri4 *res = A;
    if (X->s.enable_clipping) {   /* clip_triangle, renderer.cpp:833-854 */
        n = clip_plane(A, n, A, 0, 1);
        n = clip_plane(A, n, B, 0, -1);
        n = clip_plane(B, n, A, 1, 1);
        n = clip_plane(A, n, B, 1, -1);
        n = clip_plane(B, n, A, 2, 1);
        n = clip_plane(A, n, B, 2, -1);
        res = B;
    }
    const int rw = X->rw, rh = X->rh;
    for (int k = 0; k < n; k++) {
        const otri4 *Q = &res[k];
        opiece *P = &out[k];
        P->tri = (int)ti;
        P->piece = k;
        float iaw = 1.0f / Q->a.w, ibw = 1.0f / Q->b.w, icw = 1.0f / Q->c.w;
        P->na = V(Q->a.x * iaw, Q->a.y * iaw, Q->a.z * iaw);
        P->nb = V(Q->b.x * ibw, Q->b.y * ibw, Q->b.z * ibw);
        P->nc = V(Q->c.x * icw, Q->c.y * icw, Q->c.z * icw);
        P->tu = Q->tu;
        P->tv = Q->tv;
        P->cam = tri_from(xform_point(PI, P->na), xform_point(PI, P->nb), xform_point(PI, P->nc), O->mat, Q->tu, Q->tv);
        P->world = tri_from(xform_point(C2W, P->cam.a), xform_point(C2W, P->cam.b), xform_point(C2W, P->cam.c), O->mat,
                            Q->tu, Q->tv);
        v3 a = P->na, b = P->nb, c = P->nc;
        P->inv_area = 1 / ((b.x - a.x) * (c.y - a.y) - (b.y - a.y) * (c.x - a.x));
        float mnx = smin(a.x, smin(b.x, c.x)), mny = smin(a.y, smin(b.y, c.y));
        float mxx = smax(a.x, smax(b.x, c.x)), mxy = smax(a.y, smax(b.y, c.y));
        int x0 = d2i((double)(mnx + 1) * 0.5 * rw), y0 = d2i((double)(mny + 1) * 0.5 * rh);
        int x1 = d2i((double)(mxx + 1) * 0.5 * rw), y1 = d2i((double)(mxy + 1) * 0.5 * rh);
        P->x0 = x0 > 0 ? x0 : 0;
        P->y0 = y0 > 0 ? y0 : 0;
        P->x1 = rw - 1 < x1 ? rw - 1 : x1;
        P->y1 = rh - 1 < y1 ? rh - 1 : y1;
        P->za = xform_z(C2W, xform_point(PI, P->na));
        P->zb = xform_z(C2W, xform_point(PI, P->nb));
        P->zc = xform_z(C2W, xform_point(PI, P->nc));
    }
    return n;
}

/* Triangle::edge_function, triangle.h:65-68 */
static inline float edge_fn(float px, float py, v3 a, v3 b) { return (b.x - a.x) * (py - a.y) - (b.y - a.y) * (px - a.x); }

/* the sample point of pixel (px, py) as raster_trace's incremental loops reach it for piece P */
static void piece_sample(const opiece *P, int rw, int rh, int px, int py, float *sx, float *sy)
{
    const float hs = 1.0f / rh * 2, ws = 1.0f / rw * 2;
    float iy = P->y0 * hs - 1;
    for (int y = P->y0; y < py; y++)
        iy += hs;
    float ix = P->x0 * ws - 1;
    for (int x = P->x0; x < px; x++)
        ix += ws;
    *sx = ix + ws * 0.5f;
    *sy = iy + hs * 0.5f;
}

static int piece_bary(const opiece *P, float sx, float sy, float *u, float *v, float *w)
{
    float U = edge_fn(sx, sy, P->nc, P->na);
    if (U < 0) return 0;
    float Vv = edge_fn(sx, sy, P->na, P->nb);
    if (Vv < 0) return 0;
    float Ww = edge_fn(sx, sy, P->nb, P->nc);
    if (Ww < 0) return 0;
    *u = U * P->inv_area;
    *v = Vv * P->inv_area;
    *w = Ww * P->inv_area;
    return 1;
}

static inline float piece_z(const opiece *P, float u, float v, float w)
{
    return -1 / (1 / P->za * w + 1 / P->zb * u + 1 / P->zc * v);
}

/* raster_trace over the whole render: outputs are internal rows 0..rh-1.  hit_id =
 * winning triangle (-1: background), hit_t = its z, shadow = the shaded hit's flag. */
ORC_API int orc_raster(const struct orc_ctx *X, orc_outputs *out, orc_counters *counters, int nthreads)
{
    const int rw = X->rw, rh = X->rh;
    const size_t npx = (size_t)rw * rh;
    float *zb = (float *)malloc(npx * sizeof(float));
    int64_t *win = (int64_t *)malloc(npx * sizeof(int64_t));
    size_t cap = (size_t)(X->ntri > 0 ? X->ntri : 1) + 16, np = 0;
    opiece *pieces = (opiece *)malloc(cap * sizeof(opiece));
    if (!zb || !win || !pieces) {
        free(zb); free(win); free(pieces);
        return -1;
    }
    for (size_t i = 0; i < npx; i++) {
        zb[i] = INFINITY;
        win[i] = -1;
    }
    opiece tmp[ORC_CLIP_MAX];
    const float hs = 1.0f / rh * 2, ws = 1.0f / rw * 2;
    for (int64_t ti = 0; ti < X->ntri; ti++) {
        int n = make_pieces(X, ti, tmp);
        for (int k = 0; k < n; k++) {
            if (np == cap) {
                cap *= 2;
                opiece *np2 = (opiece *)realloc(pieces, cap * sizeof(opiece));
                if (!np2) { free(zb); free(win); free(pieces); return -1; }
                pieces = np2;
            }
            const opiece *P = &tmp[k];
            pieces[np] = *P;
            float iy = P->y0 * hs - 1;
            for (int py = P->y0; py <= P->y1; py++, iy += hs) {
                float ix = P->x0 * ws - 1;
                for (int px = P->x0; px <= P->x1; px++, ix += ws) {
                    float u, v, w;
                    if (!piece_bary(P, ix + ws * 0.5f, iy + hs * 0.5f, &u, &v, &w))
                        continue;
                    float z = piece_z(P, u, v, w);
                    size_t o = (size_t)py * rw + px;
                    if (z < zb[o]) {
                        zb[o] = z;
                        win[o] = (int64_t)np;
                    }
                }
            }
            np++;
        }
    }
    orc_counters total;
    memset(&total, 0, sizeof(total));
    v3 cam = V(X->sc.cam_pos[0], X->sc.cam_pos[1], X->sc.cam_pos[2]);
#ifdef _OPENMP
    if (nthreads <= 0)
        nthreads = omp_get_max_threads();
    if (nthreads > ORC_RASTER_SLOTS)
        nthreads = ORC_RASTER_SLOTS;
#pragma omp parallel num_threads(nthreads)
#endif
    {
        orc_counters local;
        memset(&local, 0, sizeof(local));
        int slot = 0;
#ifdef _OPENMP
        slot = omp_get_thread_num();
#endif
        otri *temp = (otri *)&X->tris[X->ntri + slot];
        otracer T;
        T.X = X;
        T.cnt = &local;
        T.ray_kind = 0;
        T.rng = 1;
        T.frame_key = 0;
#ifdef _OPENMP
#pragma omp for schedule(dynamic)
#endif
        for (int py = 0; py < rh; py++) {
            for (int px = 0; px < rw; px++) {
                size_t o = (size_t)py * rw + px;
                c3 c = background_color();
                int sh = 0;
                int64_t wi = win[o];
                if (wi >= 0) {
                    const opiece *P = &pieces[wi];
                    float sx, sy, u = 0, v = 0, w = 0;
                    piece_sample(P, rw, rh, px, py, &sx, &sy);
                    piece_bary(P, sx, sy, &u, &v, &w);
                    const otri *O = &X->tris[P->tri];
                    const orc_settings *S = &X->s;
                    if (S->shading_method == ORC_RT_SHADING) {
                        /* trace_triangle(Ray(cam, normalize(c2w(proj_inv(p)) - cam)), world piece, 0) */
                        v3 pw = xform_point(X->sc.cam_to_world, xform_point(X->sc.proj_inv, V(sx, sy, -1)));
                        v3 rd = vnormalize(vsub(pw, cam));
                        *temp = P->world;
                        ohit h = hit_fresh();
                        c = C(0, 0, 0);
                        if (tri_intersect(temp, (int)(X->ntri + slot), cam, rd, &h)) {
                            T.frame_key = pixel_seed((uint32_t)(py * rw + px), S->rng_seed);
                            local.primary_rays++;
                            c = shade(&T, cam, rd, &h, 0, &sh);
                        }
                    } else if (S->shading_method == ORC_ABS_NORMALS_SHADING) {
                        v3 nn = vnormalize(O->n);
                        c = C(fabsf(nn.x), fabsf(nn.y), fabsf(nn.z));
                    } else if (S->shading_method == ORC_PASTEL_NORMALS_SHADING) {
                        v3 nn = vnormalize(O->n);
                        c = cmulf(cadd(C(nn.x, nn.y, nn.z), C(1.0f, 1.0f, 1.0f)), 0.5f);
                    } else if (S->shading_method == ORC_BARYCENTRIC_COORDINATES_SHADING) {
                        c = cadd(cadd(cmulf(C(1, 0, 0), u), cmulf(C(0, 1.0f, 0), v)), cmulf(C(0, 0, 1), 1 - u - v));
                    } else if (S->shading_method == ORC_VISUALIZE_AO) {
                        c = C(0.9f, 0.9f, 0.9f);
                        if (S->enable_ao_mapping) {
                            float tu, tv;
                            tri_interp(&P->cam, u, v, &tu, &tv);
                            float a = tex_floor(&X->tex[ORC_TEX_AO], tu, tv).r;
                            c = cmul(c, C(a, a, a));
                        }
                    }
                }
                if (out->argb) out->argb[o] = qrgb(f2i(c.r * 255), f2i(c.g * 255), f2i(c.b * 255));
                if (out->rgba) {
                    out->rgba[4 * o] = c.r;
                    out->rgba[4 * o + 1] = c.g;
                    out->rgba[4 * o + 2] = c.b;
                    out->rgba[4 * o + 3] = 1.0f;
                }
                if (out->hit_id) out->hit_id[o] = wi >= 0 ? pieces[wi].tri : -1;
                if (out->hit_t) out->hit_t[o] = zb[o];
                if (out->shadow) out->shadow[o] = (uint8_t)sh;
                /* renderer.cpp:975-979: the z-test winner's z and original_triangle._normal */
                if (out->zbuf) out->zbuf[o] = zb[o];
                if (out->nbuf) {
                    v3 nn = wi >= 0 ? X->tris[pieces[wi].tri].n : V(0, 0, 0);
                    out->nbuf[3 * o] = nn.x;
                    out->nbuf[3 * o + 1] = nn.y;
                    out->nbuf[3 * o + 2] = nn.z;
                }
            }
        }
#ifdef _OPENMP
#pragma omp critical
#endif
        add_counters(&total, &local);
    }
    if (counters) *counters = total;
    free(zb);
    free(win);
    free(pieces);
    return 0;
}

/* One pixel of Renderer::ray_trace (renderer.cpp:1086-1113) into output slot o */
static void render_pixel(otracer *T, int px, int py, orc_outputs *out, size_t o)
{
    const struct orc_ctx *X = T->X;
    int rw = X->rw, rh = X->rh;
    v3 cam = V(X->sc.cam_pos[0], X->sc.cam_pos[1], X->sc.cam_pos[2]);
    float y_world = ((float)py + 0.5f) / rh * 2 - 1;
    float x_world = ((float)px + 0.5f) / rw * 2 - 1;
    v3 vs = xform_point(X->sc.proj_inv, V(x_world, y_world, -1));
    v3 ws = xform_point(X->sc.cam_to_world, vs);
    v3 rd = vnormalize(vsub(ws, cam));
    int found = 0, src = -1, shadowed = 0;
    ohit hi = hit_fresh();
    T->frame_key = pixel_seed((uint32_t)(py * rw + px), X->s.rng_seed);
    T->ray_kind = 0;
    T->cnt->primary_rays++;
    c3 c = trace_ray(T, cam, rd, &hi, 0, &found, &src, &shadowed);
    if (out->argb) out->argb[o] = qrgb(f2i(c.r * 255), f2i(c.g * 255), f2i(c.b * 255));
    if (out->rgba) {
        out->rgba[4 * o] = c.r;
        out->rgba[4 * o + 1] = c.g;
        out->rgba[4 * o + 2] = c.b;
        out->rgba[4 * o + 3] = T->alpha;
    }
    if (out->hit_id) out->hit_id[o] = found ? src : -1;
    if (out->hit_t) out->hit_t[o] = hi.t;
    if (out->shadow) out->shadow[o] = (uint8_t)(found && shadowed);
    /* renderer.cpp:1104-1110: hits write the z / normal buffers; the others keep
     * the cleared values (the UI clears both before every render, mainwindow.cpp:184-185) */
    if (out->zbuf) out->zbuf[o] = found ? -(cam.z + rd.z * hi.t) : INFINITY;
    if (out->nbuf) {
        v3 nn = found ? hi.normal : V(0, 0, 0);
        out->nbuf[3 * o] = nn.x;
        out->nbuf[3 * o + 1] = nn.y;
        out->nbuf[3 * o + 2] = nn.z;
    }
}

/* Renderer::ray_trace, renderer.cpp:1068-1116, rows [row_begin, row_begin+row_count) */
ORC_API int orc_render_rows(const struct orc_ctx *X, int row_begin, int row_count, orc_outputs *out,
                            orc_counters *counters, int nthreads)
{
    int rw = X->rw, rh = X->rh;
    if (row_begin < 0 || row_count < 0 || row_begin + row_count > rh)
        return -1;
    orc_counters total;
    memset(&total, 0, sizeof(total));
#ifdef _OPENMP
    if (nthreads <= 0)
        nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads)
#endif
    {
        orc_counters local;
        memset(&local, 0, sizeof(local));
        otracer T;
        T.X = X;
        T.cnt = &local;
        T.ray_kind = 0;
        T.rng = 1;
        T.frame_key = 0;
#ifdef _OPENMP
#pragma omp for schedule(dynamic)
#endif
        for (int py = row_begin; py < row_begin + row_count; py++)
            for (int px = 0; px < rw; px++)
                render_pixel(&T, px, py, out, (size_t)(py - row_begin) * rw + px);
#ifdef _OPENMP
#pragma omp critical
#endif
        add_counters(&total, &local);
    }
    if (counters)
        *counters = total;
    return 0;
}

/* The same pixels for an arbitrary set of rows (rows[i] -> output rows i), spread over the
 * threads in runs of 16 pixels: a few rows of an expensive frame (rough reflections) keep
 * every thread busy.  Pixels are independent (path-keyed RNG), so the result equals
 * orc_render_rows on each row. */
ORC_API int orc_render_row_set(const struct orc_ctx *X, const int *rows, int nrows, orc_outputs *out,
                               orc_counters *counters, int nthreads)
{
    int rw = X->rw, rh = X->rh;
    for (int i = 0; i < nrows; i++)
        if (rows[i] < 0 || rows[i] >= rh)
            return -1;
    orc_counters total;
    memset(&total, 0, sizeof(total));
    const int64_t runs = ((int64_t)rw + 15) / 16;
#ifdef _OPENMP
    if (nthreads <= 0)
        nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads)
#endif
    {
        orc_counters local;
        memset(&local, 0, sizeof(local));
        otracer T;
        T.X = X;
        T.cnt = &local;
        T.ray_kind = 0;
        T.rng = 1;
        T.frame_key = 0;
#ifdef _OPENMP
#pragma omp for schedule(dynamic)
#endif
        for (int64_t k = 0; k < (int64_t)nrows * runs; k++) {
            const int i = (int)(k / runs);
            const int px0 = (int)(k % runs) * 16;
            for (int px = px0; px < px0 + 16 && px < rw; px++)
                render_pixel(&T, px, rows[i], out, (size_t)i * rw + px);
        }
#ifdef _OPENMP
#pragma omp critical
#endif
        add_counters(&total, &local);
    }
    if (counters)
        *counters = total;
    return 0;
}

/* ------------------------------------------------------------------------- */
/* Renderer::post_process_ssao_SIMD (renderer.cpp:1229-1434)                   */
/* ------------------------------------------------------------------------- */
/* The reference seeds one 8-lane xorshift32 generator (xorshift.h:8-35) and one
 * scalar generator (:37-65) per OpenMP thread with std::rand() (renderer.cpp:1250-
 * 1261), so its occlusion noise is not reproducible run to run.  Here every pixel
 * owns a fresh xorshift32 state ssao_state(pixel, seed); the SIMD columns draw from
 * it as their 8-lane generator's lane would (signed conversion, / (float)INT32_MAX),
 * the leftover columns (render_width % 8) as the scalar generator would.  Per
 * sample the draws are x, y, z, then the lateral one, as renderer.cpp:1299-1304.  */
static uint32_t ssao_state(uint32_t pixel, uint32_t seed)
{
    uint32_t x = mix32(pixel * 0x9E3779B9u ^ seed ^ 0x5A0C1D3Bu);
    return x ? x : 0x9E3779B9u;
}

static inline uint32_t xs32(uint32_t *s)   /* xorshift.h:13-22 / :43-52 */
{
    uint32_t x = *s;
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    return *s = x;
}

/* _mm256_cvtps_epi32 under the default MXCSR: round to nearest even; NaN and
 * out-of-range values give INT_MIN */
static inline int cvt_rne(float f)
{
    if (!(f >= -2147483648.0f && f < 2147483648.0f))
        return INT32_MIN;
    return (int)rintf(f);
}

/* one lane of the SIMD loop body, renderer.cpp:1263-1361 */
static int ssao_simd_pixel(const struct orc_ctx *X, const float *zb, const float *nb, int x, int y, uint32_t st,
                           float fovm)
{
    const int W = X->rw, H = X->rh;
    const orc_settings *S = &X->s;
    const float *pm = X->sc.proj;
    float view_z = zb[(size_t)y * W + x];
    int valid = view_z != INFINITY && view_z == view_z;   /* _CMP_NEQ_OQ */
    float y_ndc = (float)y / (float)H;
    y_ndc = y_ndc * 2.0f;
    y_ndc = y_ndc - 1.0f;
    float x_ndc = (float)x / (float)W;
    x_ndc = x_ndc * 2.0f;
    x_ndc = x_ndc - 1.0f;
    float vrx = x_ndc * (fovm * X->sc.cam_aspect);
    float vry = y_ndc * fovm;
    v3 csp = V(view_z * vrx, view_z * vry, view_z * -1.0f);
    const float *np = nb + 3 * ((size_t)y * W + x);
    v3 n = V(np[0], np[1], np[2]);
    {   /* _mm256_normalize: a * (1 / sqrt(x*x + (y*y + z*z))) (m256Vector.cpp:73-108) */
        float len = sqrtf(n.x * n.x + (n.y * n.y + n.z * n.z));
        float inv = 1.0f / len;
        n = V(n.x * inv, n.y * inv, n.z * inv);
    }
    int occ = 0;
    for (int i = 0; i < S->ssao_sample_count; i++) {
        float rx = (float)(int32_t)xs32(&st) / 2147483648.0f;
        float ry = (float)(int32_t)xs32(&st) / 2147483648.0f;
        float rz = (float)(int32_t)xs32(&st) / 2147483648.0f;
        float len = sqrtf(rx * rx + (ry * ry + rz * rz));
        float inv = 1.0f / len;
        v3 rs = V(rx * inv, ry * inv, rz * inv);
        float lat = ((float)(int32_t)xs32(&st) / 2147483648.0f + 1.0f) * 0.5f;
        float k = lat + 0.0001f;
        rs = V(rs.x * k, rs.y * k, rs.z * k);
        rs = V(rs.x * S->ssao_radius, rs.y * S->ssao_radius, rs.z * S->ssao_radius);
        rs = V(rs.x + csp.x, rs.y + csp.y, rs.z + csp.z);
        v3 vd = V(rs.x - csp.x, rs.y - csp.y, rs.z - csp.z);
        float dt = vd.x * n.x + (vd.y * n.y + vd.z * n.z);
        float mask = dt < 0.0f ? 1.0f : 0.0f;
        v3 bf = V((csp.x - rs.x) * 2.0f, (csp.y - rs.y) * 2.0f, (csp.z - rs.z) * 2.0f);
        rs = V(rs.x + bf.x * mask, rs.y + bf.y * mask, rs.z + bf.z * mask);
        /* __m256Point::transform (m256Point.cpp:3-37): fused multiply-adds, w = 1 / wt */
        float xt = fmaf(pm[0], rs.x, fmaf(pm[1], rs.y, fmaf(pm[2], rs.z, pm[3])));
        float yt = fmaf(pm[4], rs.x, fmaf(pm[5], rs.y, fmaf(pm[6], rs.z, pm[7])));
        float wt = fmaf(pm[12], rs.x, fmaf(pm[13], rs.y, fmaf(pm[14], rs.z, pm[15])));
        float w = 1.0f / wt;
        float ndx = xt * w, ndy = yt * w;
        int px = cvt_rne(((ndx + 1.0f) * 0.5f) * (float)W);
        int py = cvt_rne(((ndy + 1.0f) * 0.5f) * (float)H);
        int wm1 = cvt_rne((float)W - 1.0f), hm1 = cvt_rne((float)H - 1.0f);
        px = px < wm1 ? px : wm1;
        px = px > 0 ? px : 0;
        py = py < hm1 ? py : hm1;
        py = py > 0 ? py : 0;
        int off = (int)((uint32_t)px + (uint32_t)py * (uint32_t)cvt_rne((float)W));
        float sgd = -1.0f * zb[off];
        float dz = fabsf(sgd - csp.z);
        int range = dz <= S->ssao_radius;
        int depth = rs.z < sgd;
        occ += (range && depth && valid) ? 1 : 0;
    }
    return occ;
}

/* the scalar loop over the leftover columns, renderer.cpp:1363-1413 */
static int ssao_scalar_pixel(const struct orc_ctx *X, const float *zb, const float *nb, int x, int y, uint32_t st,
                             float tanv)
{
    const int W = X->rw, H = X->rh;
    const orc_settings *S = &X->s;
    float view_z = zb[(size_t)y * W + x];
    if (view_z == INFINITY)
        return 0;
    float x_ndc = (float)x / W * 2 - 1;
    float y_ndc = (float)y / H * 2 - 1;
    float vrx = x_ndc * X->sc.cam_aspect * tanv;
    float vry = y_ndc * tanv;
    v3 csp = V(vrx * view_z, vry * view_z, -view_z);
    const float *np = nb + 3 * ((size_t)y * W + x);
    v3 n = vnormalize(V(np[0], np[1], np[2]));
    int16_t occ = 0;
    for (int i = 0; i < S->ssao_sample_count; i++) {
        float rx = xs32(&st) / (float)UINT32_MAX * 2 - 1;
        float ry = xs32(&st) / (float)UINT32_MAX * 2 - 1;
        float rz = xs32(&st) / (float)UINT32_MAX * 2 - 1;
        v3 rs = vnormalize(V(rx, ry, rz));
        rs = vscale(xs32(&st) / (float)UINT32_MAX + 0.0001f, rs);
        rs = vscale(S->ssao_radius, rs);
        rs = vadd(rs, csp);
        if (vdot(vsub(rs, csp), n) < 0)
            rs = vadd(rs, vscale(2, vsub(csp, rs)));
        v3 ndc = xform_point(X->sc.proj, rs);
        int px = d2i((ndc.x + 1) * 0.5 * W);
        int py = d2i((ndc.y + 1) * 0.5 * H);
        px = px > 0 ? px : 0;
        px = px < W - 1 ? px : W - 1;
        py = py > 0 ? py : 0;
        py = py < H - 1 ? py : H - 1;
        float sgd = -zb[(size_t)py * W + px];
        if (fabsf(sgd - csp.z) > S->ssao_radius)
            continue;
        if (rs.z < sgd)
            occ = (int16_t)(occ + 1);
    }
    return occ;
}

/* SSAO on the internal ARGB image, before the SSAA downscale (renderer.cpp:1118-1124):
 * per-pixel occlusion counts, then the 7x7 box blur applied to the image
 * (renderer.cpp:1416-1431).  fovm = (float)tan(fov / 2 / 180 * M_PI) (renderer.cpp:1245)
 * and tanv = tan(radians(fov / 2)) (renderer.cpp:1379) come from the host libm. */
ORC_API int orc_ssao(const struct orc_ctx *X, const float *zb, const float *nb, uint32_t *argb, int32_t *ao_out,
                     int nthreads)
{
    const int W = X->rw, H = X->rh;
    const orc_settings *S = &X->s;
    const float fov = X->sc.cam_fov;
    const float fovm = (float)tan(fov / 2 / 180 * M_PI);
    const float tanv = tanf(((float)M_PI / 180) * (fov / 2));
    const int simd_w = W - W % 8;
    int32_t *ao = (int32_t *)calloc((size_t)W * H, sizeof(int32_t));
    if (!ao)
        return -1;
#ifdef _OPENMP
    if (nthreads <= 0)
        nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(static) num_threads(nthreads)
#endif
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            uint32_t st = ssao_state((uint32_t)(y * W + x), S->rng_seed);
            ao[(size_t)y * W + x] = x < simd_w ? ssao_simd_pixel(X, zb, nb, x, y, st, fovm)
                                               : ssao_scalar_pixel(X, zb, nb, x, y, st, tanv);
        }
    const int blur = 7, half = blur / 2;
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(nthreads)
#endif
    for (int y = half; y < H - half; y++)
        for (int x = half; x < W - half; x++) {
            size_t o = (size_t)y * W + x;
            if (zb[o] == INFINITY)
                continue;
            int sum = 0;
            for (int dy = -half; dy <= half; dy++)
                for (int dx = -half; dx <= half; dx++)
                    sum += ao[(size_t)(y + dy) * W + x + dx];
            float cm = 1 - ((float)sum / (float)(blur * blur) / (float)S->ssao_sample_count * S->ssao_amount);
            uint32_t p = argb[o];
            /* QColor(int, int, int) from float products (truncated); an out-of-range
             * channel makes the colour invalid and QImage::setPixelColor ignores it */
            int r = f2i((float)((p >> 16) & 0xff) * cm);
            int g = f2i((float)((p >> 8) & 0xff) * cm);
            int b = f2i((float)(p & 0xff) * cm);
            if (r < 0 || r > 255 || g < 0 || g > 255 || b < 0 || b > 255)
                continue;
            argb[o] = qrgb(r, g, b);
        }
    if (ao_out)
        memcpy(ao_out, ao, (size_t)W * H * sizeof(int32_t));
    free(ao);
    return 0;
}

/* ImageUtils::downscale_image_qt_ARGB32, imageUtils.h:98-147 */
ORC_API int orc_downscale_argb(const uint32_t *in, int w, int h, int factor, uint32_t *out)
{
    if (factor <= 0 || w % factor != 0 || h % factor != 0)
        return -1;
    int dw = w / factor, dh = h / factor;
    for (int y = 0; y < dh; y++)
        for (int x = 0; x < dw; x++) {
            int ar = 0, ag = 0, ab = 0;
            for (int i = 0; i < factor; i++)
                for (int j = 0; j < factor; j++) {
                    uint32_t p = in[(size_t)(y * factor + i) * w + (x * factor + j)];
                    ar += (p >> 16) & 0xff;
                    ag += (p >> 8) & 0xff;
                    ab += p & 0xff;
                }
            out[(size_t)y * dw + x] = qrgb(ar / (factor * factor), ag / (factor * factor), ab / (factor * factor));
        }
    return 0;
}

/* Closest-hit queries on the octree (BVH::intersect), for pinning against the reference. */
ORC_API void orc_bvh_query(const struct orc_ctx *X, const float *orig, const float *dir, int64_t n, int32_t *out_id,
                           float *out_t, float *out_u, float *out_v, uint8_t *out_ret, int64_t *out_counts)
{
    int64_t vol = 0, tri = 0, child = 0;
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : vol, tri, child)
    for (int64_t i = 0; i < n; i++) {
        ohit h = hit_fresh();
        tcount tc = {0, 0, 0};
        int r = bvh_intersect(&X->bvh, V(orig[3 * i], orig[3 * i + 1], orig[3 * i + 2]),
                              V(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]), &h, &tc);
        out_ret[i] = (uint8_t)r;
        out_id[i] = h.tri;
        out_t[i] = h.t;
        out_u[i] = h.u;
        out_v[i] = h.v;
        vol += tc.vol;
        tri += tc.tri;
        child += tc.child;
    }
    if (out_counts) {
        out_counts[0] = vol;
        out_counts[1] = tri;
        out_counts[2] = child;
    }
}

/* Renderer::trace_ray(ray, hit_info, current_recursion_depth, intersection_found)
 * (renderer.cpp:1008-1066) for n arbitrary rays, each with a fresh HitInfo: colour
 * (rgba), the record's source (triangle index, -2-k for analytic shape k, -1 when
 * intersection_found stays false), its t, intersection_found and the depth-0 shadow
 * flag.  Ray i's rough-reflection stream is keyed pixel_seed(i, rng_seed), as pixel i
 * of a frame. */
ORC_API void orc_trace_rays_shaded(const struct orc_ctx *X, const float *orig, const float *dir, int64_t n, int depth,
                                   float *rgba, int32_t *out_src, float *out_t, uint8_t *out_found,
                                   uint8_t *out_shadow, orc_counters *counters)
{
    orc_counters total;
    memset(&total, 0, sizeof(total));
#pragma omp parallel
    {
        orc_counters local;
        memset(&local, 0, sizeof(local));
        otracer T;
        T.X = X;
        T.cnt = &local;
        T.ray_kind = 0;
        T.rng = 1;
        T.frame_key = 0;
#pragma omp for schedule(dynamic, 16)
        for (int64_t i = 0; i < n; i++) {
            int found = 0, src = -1, shadowed = 0;
            ohit hi = hit_fresh();
            T.frame_key = pixel_seed((uint32_t)i, X->s.rng_seed);
            T.alpha = 1.0f;
            c3 c = trace_ray(&T, V(orig[3 * i], orig[3 * i + 1], orig[3 * i + 2]),
                             V(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]), &hi, depth, &found, &src, &shadowed);
            rgba[4 * i] = c.r;
            rgba[4 * i + 1] = c.g;
            rgba[4 * i + 2] = c.b;
            rgba[4 * i + 3] = T.alpha;
            out_src[i] = found ? src : -1;
            out_t[i] = hi.t;
            out_found[i] = (uint8_t)found;
            out_shadow[i] = (uint8_t)(found && shadowed);
        }
#pragma omp critical
        add_counters(&total, &local);
    }
    if (counters)
        *counters = total;
}

/* Octree statistics: [inner, leaves, empty_leaves, max_leaf_size, max_depth, node_count] */
static void stats_rec(const obvh *B, int ni, int depth, int64_t *st)
{
    const onode *n = &B->nodes[ni];
    if (depth > st[4]) st[4] = depth;
    if (n->is_leaf) {
        st[1]++;
        if (n->ntris == 0) st[2]++;
        if (n->ntris > st[3]) st[3] = n->ntris;
        return;
    }
    st[0]++;
    for (int i = 0; i < 8; i++)
        stats_rec(B, n->child[i], depth + 1, st);
}

ORC_API void orc_bvh_stats(const struct orc_ctx *X, int64_t *st)
{
    for (int i = 0; i < 6; i++) st[i] = 0;
    if (X->bvh.nnodes > 0)
        stats_rec(&X->bvh, 0, 0, st);
    st[5] = X->bvh.nnodes;
}

/* k-DOP of node i in DFS-creation order (for pinning the flattened layout) */
ORC_API int orc_bvh_node(const struct orc_ctx *X, int i, float *dn7, float *df7, int32_t *is_leaf, int32_t *children8,
                         int32_t *ntris)
{
    if (i < 0 || i >= X->bvh.nnodes)
        return -1;
    const onode *n = &X->bvh.nodes[i];
    for (int p = 0; p < NPLANES; p++) {
        dn7[p] = n->dn[p];
        df7[p] = n->df[p];
    }
    *is_leaf = n->is_leaf;
    for (int c = 0; c < 8; c++) children8[c] = n->is_leaf ? -1 : n->child[c];
    *ntris = n->ntris;
    return 0;
}

/* libstdc++ priority_queue pop order emulation, exposed for pinning */
ORC_API void orc_heap_order(const float *keys, int n, int32_t *out_order)
{
    oheap h;
    h.len = 0;
    for (int i = 0; i < n; i++) {
        qel e = {i, keys[i]};
        heap_push(&h, e);
    }
    for (int i = 0; i < n; i++) {
        out_order[i] = h.e[0].node;
        heap_pop(&h);
    }
}
