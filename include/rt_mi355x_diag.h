/*
 * rt_mi355x_diag.h -- diagnostic entry points of librt_mi355x.so (no reference counterpart).
 * Tests and tools use them to check and measure the hot path; a drop-in caller of the reference's
 * Renderer surface needs only rt_mi355x.h.  Same conventions and error codes as rt_mi355x.h.
 */
#ifndef RT_MI355X_DIAG_H
#define RT_MI355X_DIAG_H

#include "rt_mi355x.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Diagnostic builds (-DRT_PHASE_TIME=1, with RT_DEBUG_WAVES set in the environment when the
 * renderer is created): the last ray_trace's per-wave records of 8 words, n = 8 x waves values --
 * shader cycles per phase {tile setup, ray generation, primary query, shading, shadow query,
 * framebuffer, dequeue} of the plain kernel.  RT_EINVAL when no record buffer exists. */
int rt_debug_read(rt_renderer *r, uint64_t *out, int64_t n);
/* Diagnostics (no reference counterpart): the shader cycles of each 8x8 tile of the last launch --
 * rt_render / rt_ray_trace, or rt_render_bands_device (its launch-local tiles) -- (tile = ty * tiles_x
 * + tx; the heavy-first ordering's input; a split tile, the sum of its parts' cycles).
 * out == NULL: only the layout.  RT_EINVAL before a launch that records them (reflections, raster,
 * RT_HEAVY_FIRST=0). */
int rt_tile_costs(rt_renderer *r, uint32_t *out, int64_t n, int32_t *tiles_x, int32_t *tiles_y);

/* The frames' wide-BVH query on the GPU (kernels.hip wide_query_kernel), with its
 * status, for n rays: the device build (hardware reciprocal / square root, the GPU-computed risk
 * words of the current camera and light) of what rt_wbvh_query_ex runs on the host, answering
 * BVH::intersect (bvh.h:212-287) through the resident wide BVH and its certificate.  kind 0: plain
 * rays (no risk words: reflection rays, rt_trace_ray); 1: camera rays (a ray whose origin equals the
 * camera position bitwise reads the camera's words, as the frame's primary rays do); 2: each ray is
 * (hit point p in orig, normal n in dir), traced as is_shadowed's ray o = p + 1e-4 n, d =
 * normalize(light - p) (renderer.cpp:340-402) with the light's words when the frame's would apply.
 * o_out / d_out [n][3]: the rays queried.  status: 0 certified miss, 1 certified hit (tri_id / t /
 * u / v = BVH::intersect's record; it returned true), 2 not certified (a frame takes the exact
 * octree walk), each as a closest-hit query over the whole line.  shadowed (kind 2): the frame's
 * own decision through its segment query, 0 lit, 1 shadowed, 2 not decided (octree walk); 2 for the
 * other kinds.  Waits for the wide BVH's background build (rt_finish_accel); with no wide BVH
 * (exact mode, RT_WBVH=0, a scene scale outside its margins) every status is 2. */
int rt_wide_query(rt_renderer *r, const float *orig, const float *dir, int64_t n, int32_t kind, float *o_out,
                  float *d_out, int32_t *status, int32_t *tri_id, float *t, float *u, float *v, uint8_t *shadowed);
/* Diagnostics: the current frame's grazing-risk words (8 per wide-BVH node, wbvh.hpp wrisk_pack):
 * src 0 as the GPU computes them (wide_risk_kernel), src 1 by the host walk (wbvh_risk_host) over
 * the same resident wide BVH.  *count = the number of words; out (cap words) may be null to query
 * it.  violations (optional): the words checked against the tree (wbvh.hpp check_risk_words: every
 * at-risk triangle's key and octree leaf held by each entry above it).  Waits for the wide BVH's
 * build; RT_ESTATE when there is none. */
int rt_risk_words(rt_renderer *r, int32_t src, uint64_t *out, int64_t cap, int64_t *count, int64_t *violations);

/* ---- Host octree build (BVH::BVH, tp2/projets/bvh.cpp:19-66; bvh.h:141-210), no GPU ----
 * Builds and flattens the octree over tri9 and returns a 64-bit FNV-1a digest of the
 * flattened nodes, triangle records and slot -> triangle map, and stats[7] =
 * {inner, leaves, empty_leaves, max_leaf, max_depth, nodes, flattened levels}.
 * builder 0: the parallel level-by-level build the renderer uses; 1: the reference's
 * one-insert-at-a-time algorithm restated.  *ms (optional) gets the build time. */
int rt_octree_digest(const float *tri9, int64_t n, int32_t max_depth, int32_t leaf_max_obj_count, int32_t builder,
                     uint64_t *digest, int64_t stats[7], float *ms);

/* ---- Wide-BVH certified closest hit, on the host, no GPU ----
 * Builds the octree over tri9 and the 4-wide SAH BVH over its triangle records, then runs,
 * for each ray, the traversal and certificate the primary-ray kernel runs (wbvh.hpp).
 * status[i]: 0 = certified no hit (BVH::intersect returns false, record untouched),
 * 1 = certified hit (id / t / u / v = BVH::intersect's record, bvh.h:212-287, returns true),
 * 2 = not certified (the kernel re-traces it through the octree).  stats[8] = {wide nodes,
 * leaves, max leaf, depth, node visits, triangle tests, structural violations (check_wbvh),
 * SAH cost x 1000}; ms[2] (optional) = {octree build, wide-BVH build} milliseconds. */
int rt_wbvh_query(const float *tri9, int64_t n, int32_t max_depth, int32_t leaf_max_obj_count, const float *orig,
                  const float *dir, int64_t nrays, int32_t *status, int32_t *id, float *t, float *u, float *v,
                  int64_t stats[8], float *ms);
/* The same with the frame's grazing-risk bits of a camera and / or a light point:
 * rays whose origin equals cam (bitwise) read the camera's bits; with shadow_rays = 1 (light
 * required) each ray is given as (hit point p in orig, normal n in dir) and becomes is_shadowed's
 * ray o = p + 1e-4 n, d = normalize(light - p) (renderer.cpp:340-402), reading the light's bits when
 * its segment bound allows, and is answered as a closest-hit query over the whole line.  o_out /
 * d_out (optional, 3 floats per ray) receive the rays queried, ray_nodes (optional) each query's
 * wide-node visits (the retry's included).  ocone_dim > 0: the origin cones at that
 * resolution for the rays that read no risk words (the reflection queries' skip of case (b));
 * oc_stats[5] (optional) = {cells computed, cells with no triangle at risk, cells without a bound,
 * rays that skipped case (b), grid build ms}. */
int rt_wbvh_query_ex(const float *tri9, int64_t n, int32_t max_depth, int32_t leaf_max_obj_count, const float *orig,
                     const float *dir, int64_t nrays, const float *cam, const float *light, int32_t shadow_rays,
                     float *o_out, float *d_out, int32_t *status, int32_t *id, float *t, float *u, float *v,
                     int64_t stats[8], float *ms, int32_t *ray_nodes, int32_t ocone_dim, int64_t oc_stats[5]);

/* The origin cones' soundness by brute force (CPU tests): builds the octree, the wide
 * BVH and the origin-cone grid (ocone_dim cells along the longest axis) over tri9; for each ray whose
 * origin cone lets it skip case (b) (skip[i] = 1, optional), runs Moller-Trumbore (triangle.cpp:25-91)
 * on every triangle nearly parallel to it (|cos(N, d)| < the query's split, or degenerate): a reported
 * hit is a violation.  out[6] = {violations, rays skipping, grazing triangle tests, cells computed,
 * cells with no triangle at risk, cells without a bound}. */
int rt_ocone_check(const float *tri9, int64_t n, int32_t max_depth, int32_t leaf_max_obj_count, int32_t ocone_dim,
                   const float *orig, const float *dir, int64_t nrays, int32_t *skip, int64_t out[6],
                   const uint32_t *cells, const int32_t *dims, const float *lo_ih, uint32_t *cells_out);
/* cells / dims / lo_ih (optional, all or none): check that grid instead of building one (a renderer's,
 * rt_ocone_read; out[3] then counts its cells); cells_out (optional): the built grid's words, 2 per cell
 * (its frame: ocone_dim along the longest axis, as the renderer builds it).
 * The renderer's resident origin-cone grid (built on the device at the last geometry change when a
 * material reflects): dims[3], lo_ih[4] = {lo x, y, z, 1 / cell size}; out (optional) receives its
 * words, 2 per cell (n >= 2 dims[0] dims[1] dims[2]). */
int rt_ocone_read(rt_renderer *r, uint32_t *out, int64_t n, int32_t dims[3], float lo_ih[4]);
/* The camera's risk cap by brute force (CPU tests): rays from cam with directions dir; for
 * each that the cap (as the renderer computes it per frame, or cap_override >= 0) lets skip case (b) (skip[i]
 * = 1, optional), Moller-Trumbore runs on every triangle nearly parallel to it or degenerate: a reported hit
 * is a violation.  out[4] = {violations, rays skipping, grazing triangle tests, the cap x 1e9 (-1: none)}. */
int rt_risk_cap_check(const float *tri9, int64_t n, int32_t max_depth, int32_t leaf_max_obj_count, const float *cam,
                      const float *dir, int64_t nrays, float cap_override, int32_t *skip, int64_t out[4]);

#ifdef __cplusplus
}
#endif
#endif
