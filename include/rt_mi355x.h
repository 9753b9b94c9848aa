/*
 * rt_mi355x.h -- C ABI of the MI355X-native primary-ray + shadow-ray renderer
 * (librt_mi355x.so).  Drop-in for the hot path of TomClabault/RayTracerCPP:
 * each entry point replaces one member of the reference's Renderer class
 * (tp2/projets/renderer/renderer.h:20-355) or one free function it depends on;
 * the reference interface is cited next to each declaration.
 *
 * Conventions
 *   - plain pointers + sizes, no C++ types; every function is synchronous;
 *   - matrices are 16 floats, row-major (Transform::m[i][j] = m[4*i+j], tp2/src/mat.h:21-71);
 *   - triangles are [n][9] floats (a.xyz b.xyz c.xyz, world space as left by
 *     MeshIOUtils::create_triangles), material indices [n] int32, optional
 *     texture coordinates [n][6] floats (u0 u1 u2 v0 v1 v2 == Triangle::_tex_coords_u/_v);
 *   - materials are [n][16] floats: ambient_coeff rgb, diffuse rgb, specular rgb,
 *     emission rgb, reflection, roughness, ns, specular_threshold (Material, tp2/src/materials.h:14-38);
 *   - images are ARGB32 (0xAARRGGBB, QImage::Format_ARGB32), row-major, row 0 = NDC y = -1;
 *   - every function returns RT_OK (0) or a negative RT_E* code; rt_last_error()
 *     gives the message of the calling thread's last failure.  No exceptions
 *     cross this boundary.  The reference has no error reporting (asserts / UB):
 *     invalid material indices, absent textures and renders without geometry
 *     are rejected here up front with RT_EINVAL.
 *   - a handle belongs to one thread at a time (as Renderer does), except that rt_get_image,
 *     rt_lock_image and rt_unlock_image may be called from a second (display) thread while the
 *     owning thread renders (DisplayThread / RenderThread, QT/mainWindowThreads.cpp:6-65).
 */
#ifndef RT_MI355X_H
#define RT_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_OK 0
#define RT_EINVAL (-1)
#define RT_EHIP (-2)
#define RT_ENOMEM (-3)
#define RT_ESTATE (-4)
#define RT_EUNSUPPORTED (-5)
#define RT_EIO (-6)

/* RenderSettings::ShadingMethod (rendererSettings.h:8-25) */
#define RT_SHADING_RT 0
#define RT_SHADING_ABS_NORMALS 1
#define RT_SHADING_PASTEL_NORMALS 2
#define RT_SHADING_BARYCENTRIC 3
#define RT_SHADING_VISUALIZE_AO 4

/* texture slots: Renderer::set_{ao,diffuse,normal,displacement,roughness}_map, set_skysphere (renderer.h:77-84) */
#define RT_TEX_AO 0
#define RT_TEX_DIFFUSE 1
#define RT_TEX_NORMAL 2
#define RT_TEX_DISPLACEMENT 3
#define RT_TEX_ROUGHNESS 4
#define RT_TEX_SKYSPHERE 5

/* RenderSettings, field for field (tp2/projets/renderer/rendererSettings.h:6-105);
 * every field is honoured (SSAO: full-frame rendering only). */
typedef struct rt_settings {
    int32_t image_width, image_height;
    int32_t enable_ssaa, ssaa_factor;
    int32_t enable_clipping;
    int32_t hybrid_rasterization_tracing;   /* rt_render: raster_trace instead of ray_trace */
    int32_t shading_method;
    int32_t compute_shadows;
    int32_t max_recursion_depth;
    int32_t enable_bvh, bvh_max_depth, bvh_leaf_object_count;
    int32_t enable_ssao;                    /* post_process: SSAO before SSAA (not with rt_render_bands_device) */
    int32_t ssao_sample_count;
    float ssao_radius, ssao_amount;
    int32_t enable_ambient, enable_diffuse, enable_specular, enable_emissive;
    int32_t rough_reflections_sample_count;
    int32_t enable_ao_mapping, enable_diffuse_mapping, enable_normal_mapping, enable_displacement_mapping;
    float displacement_mapping_strength;
    int32_t parallax_mapping_steps;
    int32_t enable_roughness_mapping;
    int32_t enable_skysphere, enable_skybox;
    uint32_t rng_seed;                      /* counter-based rough-reflection RNG seed (no reference equivalent) */
} rt_settings;

/* Per-render statistics (no reference equivalent; Renderer prints timings only). */
typedef struct rt_stats {
    int64_t primary_rays;      /* render_w * render_h of the last ray_trace */
    int64_t shadow_rays;       /* one per shaded hit with compute_shadows */
    int64_t reflection_rays;
    float kernel_ms;           /* GPU time of the last ray_trace kernel (HIP events) */
    float post_ms;             /* GPU time of the last post_process */
    float build_ms;            /* the last geometry change's blocking part: octree build + flatten + upload */
    int64_t octree_inner, octree_leaves, octree_empty_leaves, octree_max_leaf, octree_max_depth;
    int64_t gpu_nodes, gpu_tris;
    int32_t render_width, render_height;
    float seg_scale;           /* scene scale of the last frame's segment queries (kernels.hip seg_margin);
                                  0: shadow / reflection queries walked the whole line */
    int64_t work[4];           /* diagnostic builds (-DRT_COUNT=1) only, else 0: the last frame's k-DOP and
                                  Moller-Trumbore tests of whole-line queries, then of segment queries */
    int64_t work_wide[4];      /* diagnostic builds only: wide-BVH node visits, triangle tests, the queries it could
                                  not certify (traced through the octree instead), and the
                                  certificates' octree k-DOP tests */
    int64_t uncertified[6];    /* diagnostic builds only: uncertified wide-BVH queries by reason -- stack overflow,
                                  NaN hit, only overflowed hits, tie, minimum t outside (0, inf), failed
                                  certificate */
    int64_t wave_steps[6];     /* diagnostic builds only: wide-BVH traversal loop iterations of primary queries --
                                  summed over waves (each wave's longest lane), summed over lanes, wave calls --
                                  then the same for shadow queries (SIMD efficiency = lanes / (64 waves)) */
    float build_split_ms[4];   /* the last scene build, host milliseconds: octree build + flatten; leaf cones and
                                  slabs, and the wide BVH with its upload (both on the background thread,
                                  rt_finish_accel; 0 until adopted); the octree's upload */
    int64_t host_builds;       /* host octree builds since rt_create, over every device of rt_set_devices (its
                                  helpers copy the lead's build: one per geometry change, renderer.cpp:214-224) */
    int32_t wide_tree;         /* the wide BVH serving frames: 0 none (octree walk), 1 the quick tree built with the
                                  octree, 2 the SAH tree adopted after the background build, -1 that build failed
                                  (rt_finish_accel returned the error) and the quick tree keeps serving */
} rt_stats;

typedef struct rt_renderer rt_renderer;

/* RenderSettings() defaults (rendererSettings.h:27-102) */
void rt_default_settings(rt_settings *s);

/* Renderer::Renderer() (renderer.cpp:80): default Scene (Camera at origin, fov 45,
 * near 0.1, far 1000; PointLight (3,3,2)), RenderSettings(), no geometry.
 * device: HIP device ordinal.  Returns NULL on failure (see rt_last_error). */
rt_renderer *rt_create(int device);
void rt_destroy(rt_renderer *r);
const char *rt_last_error(void);

/* Renderer::render_settings() (renderer.h:46): read / replace the settings.
 * Replacing them re-creates the image (init_buffers, renderer.cpp:122-135) when the
 * render size changed and rebuilds the octree when the BVH parameters changed. */
int rt_get_settings(rt_renderer *r, rt_settings *out);
int rt_set_settings(rt_renderer *r, const rt_settings *s);

/* Exact mode (no reference counterpart).  on != 0: every BVH query walks
 * the octree over the whole ray line as BVH::intersect does (bvh.h:212-287), so every
 * result is the reference's by construction.  Off (default): closest hits come from the
 * wide BVH, whose child test is sound for every ray (grazing rays included, r04-r05), and
 * each answer is certified on the reference's own octree leaf; the few queries it cannot
 * certify (ties, NaN hits, overflowed stacks) walk the octree in place.  Both give the
 * same images; exact mode is slower.  Also RT_EXACT=1 at rt_create. */
int rt_set_exact(rt_renderer *r, int on);

/* Acceleration structures beside the octree (no reference counterpart): after a
 * geometry change the octree (the reference's BVH, renderer.cpp:214-224) is built and uploaded
 * before the next frame, together with a quick wide BVH (the octree's own hierarchy, O(n)); the
 * leaf cones / slabs and the SAH wide BVH are built on a background thread and replace it when
 * resident.  Frames certify their answers on either tree (the same images; without a wide BVH, as
 * in exact mode, they take the octree traversal).  rt_finish_accel waits for the background build
 * (RT_ASYNC_ACCEL=0 at rt_create: every geometry change waits for it; RT_WBVH_QUICK_FIRST=0: no
 * quick tree). */
int rt_finish_accel(rt_renderer *r);

/* Single-process multi-device rendering (no reference counterpart: the reference renders on
 * one host, RenderThread::run, QT/mainWindowThreads.cpp:39-65).  ids[0] must be the handle's
 * device; n = 0 (or ids NULL) returns to one device.  rt_render then renders on every device
 * the interleaved bands of 8 output rows with band % n == its index in ids (the kernels of
 * rt_render_bands_device), sends them to ids[0] with RCCL (librccl, loaded at the first call
 * with n > 1) and re-assembles the frame there: rt_get_image returns the same image as on one
 * device.  Scene and settings changes on the handle reach the other devices before each
 * frame.  ids may instead repeat the handle's device n times (n renderers on one device, the
 * bands copied instead of sent: the same path without RCCL, for one-device machines).
 * Frames with enable_ssao render on ids[0] alone (SSAO reads across bands);
 * rt_ray_trace / rt_post_process / rt_get_internal are single-device as before.
 * The geometry is built once, on ids[0]; the other devices copy its device tables (rt_stats
 * host_builds).
 * EXPERIMENTAL: distinct device ids (the RCCL send / receive path) have not run on a multi-GPU
 * machine yet; they are refused with RT_EUNSUPPORTED unless RT_MULTIDEV_RCCL=1 is set in the
 * environment (tests/test_gpu_parity.py test_set_devices_distinct_rccl runs them where two or
 * more devices exist).  The repeated-device form is tested on every GPU run. */
int rt_set_devices(rt_renderer *r, const int32_t *ids, int32_t n);

/* Renderer::change_render_size (renderer.cpp:250-261) */
int rt_change_render_size(rt_renderer *r, int32_t width, int32_t height);

/* Renderer::set_triangles (renderer.cpp:137-144): copies, then builds the octree
 * BVH(&_triangles, bvh_max_depth, bvh_leaf_object_count) on the host, flattens
 * and uploads it.  uv6 may be NULL ((-1,-1,-1) texture coordinates). */
int rt_set_triangles(rt_renderer *r, const float *tri9, const int32_t *mat, const float *uv6, int64_t n);

/* Renderer::add_analytic_shape (renderer.cpp:146) with Sphere / Plane (analyticShape.h:20-53) */
int rt_add_sphere(rt_renderer *r, float cx, float cy, float cz, float radius, int32_t mat);
int rt_add_plane(rt_renderer *r, float px, float py, float pz, float nx, float ny, float nz, int32_t mat);

/* Renderer::clear_geometry (renderer.cpp:182-186) */
int rt_clear_geometry(rt_renderer *r);

/* Renderer::set_materials / get_materials (renderer.cpp:148-150) */
int rt_set_materials(rt_renderer *r, const float *mats16, int32_t n);
int rt_get_material_count(rt_renderer *r, int32_t *n);

/* Renderer::change_camera_fov / change_camera_aspect_ratio / set_light_position (renderer.cpp:188-190) */
int rt_change_camera_fov(rt_renderer *r, float fov);
int rt_change_camera_aspect_ratio(rt_renderer *r, float aspect);
int rt_set_light_position(rt_renderer *r, float x, float y, float z);

/* Renderer::set_camera_transform / apply_transformation_to_camera (renderer.cpp:226-241) */
int rt_set_camera_transform(rt_renderer *r, const float m[16]);
int rt_apply_transformation_to_camera(rt_renderer *r, const float m[16]);

/* Direct camera state (Camera::_position, _perspective_proj_mat_inv, _camera_to_world_mat,
 * scene/camera.h:19-30), for callers that computed the matrices themselves. */
int rt_set_camera_matrices(rt_renderer *r, const float pos[3], const float proj_inv[16], const float cam_to_world[16]);
int rt_get_camera_matrices(rt_renderer *r, float pos[3], float proj_inv[16], float cam_to_world[16]);

/* Camera::_perspective_proj_mat and Camera::_world_to_camera_mat (scene/camera.h:19-30),
 * which the raster path uses (renderer.cpp:833-838, 877-879), as the caller computed
 * them.  Default: perspective(fov, aspect) and the inverse of cam_to_world. */
int rt_set_camera_projection(rt_renderer *r, const float proj[16], const float world_to_cam[16]);

/* Camera::_fov and Camera::_aspect_ratio (scene/camera.h:22-23) as the caller holds them,
 * without recomputing any matrix: the SSAO pass reads them (renderer.cpp:1245, 1281-1282,
 * 1378-1379).  Default: the fov / aspect of the last change_camera_fov /
 * change_camera_aspect_ratio / change_render_size. */
int rt_set_camera_lens(rt_renderer *r, float fov, float aspect);

/* Renderer::set_object_transform / reset_previous_transform (renderer.cpp:212-224) */
int rt_set_object_transform(rt_renderer *r, const float m[16]);
int rt_reset_previous_transform(rt_renderer *r);

/* Renderer::set_*_map / set_skysphere and clear_*_map (renderer.cpp:192-205).
 * rgba: w*h*4 floats (Image texels); NULL clears the slot. */
int rt_set_texture(rt_renderer *r, int32_t slot, int32_t w, int32_t h, const float *rgba);

/* Renderer::set_skybox(Skybox(faces)) (renderer.cpp:199, skybox.h:12-16): faces
 * right, left, top, bottom, back, front. */
int rt_set_skybox(rt_renderer *r, const int32_t w[6], const int32_t h[6], const float *const faces[6]);

/* Renderer::reconstruct_bvh_new / destroy_bvh (renderer.cpp:243-248) */
int rt_reconstruct_bvh_new(rt_renderer *r);
int rt_destroy_bvh(rt_renderer *r);

/* Renderer::ray_trace (renderer.cpp:1068-1116): renders the render_w x render_h
 * internal image on the GPU (synchronous). */
int rt_ray_trace(rt_renderer *r);

/* Renderer::raster_trace (renderer.cpp:869-1006): the hybrid path -- primary visibility
 * by rasterising the clipped triangles (z-buffer; the sequential z-test's winner, first of
 * equal z), shading by trace_triangle (shadow and reflection rays through the octree).
 * Reflective materials need enable_bvh (RT_EUNSUPPORTED otherwise).  Same outputs as
 * rt_ray_trace: hit_id = the winning triangle, hit_t = its z-buffer depth. */
int rt_raster_trace(rt_renderer *r);

/* Diagnostics (no reference equivalent; Renderer::_z_buffer / _normal_buffer are private,
 * renderer.h:319-320): the internal-size z buffer, the normal buffer as 4 floats per pixel
 * (xyz, 0) and the occlusion counts of the last SSAO pass; any pointer may be NULL. */
int rt_get_ssao_buffers(rt_renderer *r, float *z, float *n4, int32_t *ao);

/* Renderer::post_process (renderer.cpp:1118-1124): post_process_ssao_SIMD (renderer.cpp:
 * 1229-1434) on the internal image when enable_ssao, then the SSAA downscale when enabled.
 * The z / normal buffers SSAO reads are those of the last rt_ray_trace / rt_raster_trace,
 * cleared before each (mainwindow.cpp:184-185); RT_ESTATE if that frame had SSAO off. */
int rt_post_process(rt_renderer *r);

/* Renderer::get_image (renderer.cpp:106-109): copies the current image
 * (image_width x image_height after post_process) to argb; w/h receive its size.
 * Progressive readback: from the start of a ray_trace / raster_trace the image is the frame's
 * internal (render_w x render_h) buffer, which the GPU fills tile by tile, as the reference's
 * ray_trace fills _image pixel by pixel.  Called from a display thread while the owning thread
 * renders, rt_get_image returns the image as it stands (finished tiles of the frame in progress,
 * elsewhere the previous frame or, for a re-created image -- size change, SSAA frame -- the
 * BACKGROUND_COLOR fill); it does not wait for the frame.  Frames rendered with rt_set_devices
 * appear whole, after their gather. */
int rt_get_image(rt_renderer *r, uint32_t *argb, int32_t *w, int32_t *h);

/* Renderer::lock_image_mutex / unlock_image_mutex (renderer.h:41-42, renderer.cpp:96-104): while a
 * thread holds the image lock, no frame of the handle switches or re-creates the image (the start
 * of a frame and post_process's SSAA swap wait for it); rt_get_image takes it too (recursive). */
int rt_lock_image(rt_renderer *r);
int rt_unlock_image(rt_renderer *r);

/* render(Renderer&) (utils/mainUtils.cpp:6-21): raster_trace (hybrid_rasterization_tracing)
 * or ray_trace, then post_process;
 * *ms receives the wall time in milliseconds (may be NULL). */
int rt_render(rt_renderer *r, float *ms);

/* Parity / debug buffers of the last ray_trace at internal resolution
 * (render_w x render_h); any pointer may be NULL.  Requesting them before the
 * render (rt_request_aux) makes the kernel write them. */
int rt_request_aux(rt_renderer *r, int32_t want_rgba, int32_t want_hit, int32_t want_shadow);
int rt_get_internal(rt_renderer *r, uint32_t *argb, float *rgba, int32_t *hit_id, float *hit_t, uint8_t *shadow);

int rt_get_stats(rt_renderer *r, rt_stats *out);

/* Image-strip rendering for multi-GPU (one process per GPU): renders the bands of
 * band_rows OUTPUT rows with band % nranks == rank into the device buffer d_out
 * (image_width x local_rows(...) ARGB32, final resolution, SSAA applied) on the
 * given HIP stream (NULL = the handle's stream).  Does not synchronise.
 *
 * Stream contract.  Every write to d_out is enqueued on hip_stream and ordered only by it:
 *   - the caller orders any earlier work on d_out (fills, copies, reads of the previous frame)
 *     before this call on hip_stream, e.g. with hipStreamWaitEvent; work that touches d_out
 *     on another stream afterwards must wait for an event recorded on hip_stream after this call;
 *   - launches on different streams may run concurrently (frames in flight); each stream has
 *     its own tile-queue counters and band buffer (up to 8 streams, the least recently used is
 *     recycled once its last launch is done);
 *   - the library orders its own shared state: a launch that uses buffers shared across
 *     launches (reflection engine, raster path) waits for every launch still in flight, and a
 *     scene, material or texture change waits for them on the host before it is uploaded. */
int rt_local_rows(rt_renderer *r, int32_t band_rows, int32_t rank, int32_t nranks, int32_t *rows_out);
int rt_render_bands_device(rt_renderer *r, int32_t band_rows, int32_t rank, int32_t nranks, uint32_t *d_out,
                           void *hip_stream);
/* Cost-balanced strips: renders the listed OUTPUT bands (bands[i] in [0, ceil(image_height /
 * band_rows)), each at most once) into d_out, local band i = rows [i * band_rows, (i + 1) *
 * band_rows) of an image_width x (nbands * band_rows) ARGB32 buffer; otherwise as
 * rt_render_bands_device (which renders the list rank, rank + nranks, ...), same stream contract.
 * A list that differs from the stream's previous one waits for that stream's last launch. */
int rt_render_band_list_device(rt_renderer *r, int32_t band_rows, const int32_t *bands, int32_t nbands,
                               uint32_t *d_out, void *hip_stream);
/* The cost of each OUTPUT band in the last band launch on hip_stream (NULL = the handle's stream):
 * the shader cycles of its 8x8 tiles (a tile is charged to the band of its first row), written to
 * costs[global band] for the bands that launch rendered; the others are left as they are, so that
 * ranks can sum their vectors.  Waits for that launch.  nbands >= ceil(image_height / band_rows).
 * RT_EINVAL before a band launch that records tile costs (reflections, raster, RT_HEAVY_FIRST=0). */
int rt_band_costs(rt_renderer *r, void *hip_stream, double *costs, int32_t nbands);

/* BVH::intersect (bvh.cpp:68-71; OctreeNode::intersect, bvh.h:212-287) for n arbitrary
 * rays (origins / directions [n][3]): the closest-hit query trace_ray and is_shadowed
 * issue, with the reference's visit order.  Outputs per ray: triangle index of the
 * query's HitInfo (-1 none), its t / u / v, and the boolean BVH::intersect returned.
 * Uses the brute-force loop when enable_bvh is 0. */
int rt_trace_rays(rt_renderer *r, const float *orig, const float *dir, int64_t n, int32_t *tri_id, float *t,
                  float *u, float *v, uint8_t *ret);

/* Renderer::trace_ray(ray, hit_info, current_recursion_depth, intersection_found)
 * (renderer.h:144, renderer.cpp:1008-1066) for n arbitrary rays (origins / directions [n][3]),
 * each with a fresh HitInfo: rgba [n][4] = the Color trace_ray returns (shading, shadow ray,
 * compute_reflection recursion down to max_recursion_depth, sky / background on a miss);
 * hit_src = the record's source when intersection_found (triangle index, -2 - k for analytic
 * shape k), else -1; t = the record's t; intersection_found; shadowed = the hit's shadow ray was
 * blocked.  Ray i's rough-reflection samples draw from the stream of pixel i of a frame (the
 * counter-based RNG of rt_settings::rng_seed).  rt_get_stats reports the call's shadow and
 * reflection ray counts. */
int rt_trace_ray(rt_renderer *r, const float *orig, const float *dir, int64_t n, int32_t current_recursion_depth,
                 float *rgba, int32_t *hit_src, float *t, uint8_t *intersection_found, uint8_t *shadowed);

/* GPU durations (ms) of the ray-trace kernel of the last n rt_render_bands_device
 * calls, from HIP events recorded around each launch on its stream (waits for them). */
int rt_kernel_times(rt_renderer *r, float *ms, int32_t n);
/* shadow / reflection ray counts of the last rt_render_bands_device (waits for that launch);
 * RT_ESTATE before the first rt_render_bands_device call */
int rt_band_counters(rt_renderer *r, int64_t *shadow_rays, int64_t *reflection_rays);

/* ---- tp2/src/mat.cpp restated (host) ---- */
/* kind: 0 Translation(x,y,z) 1 RotationX(x deg) 2 RotationY 3 RotationZ 4 Scale(x,y,z) 5 Identity */
void rt_make_transform(int32_t kind, float x, float y, float z, float out[16]);
void rt_compose(const float a[16], const float b[16], float out[16]);                      /* a(b), mat.cpp:363-371 */
void rt_inverse(const float m[16], float out[16]);                                          /* mat.cpp:378-447 */
void rt_perspective(float fov, float aspect, float znear, float zfar, float out[16]);       /* mat.cpp:307-319 */
void rt_transform_points(const float m[16], const float *pts, int64_t n, float *out);       /* mat.cpp:83-100 */

/* ---- OBJ / MTL loading: read_meshio_data (tp2/src/mesh_io.cpp:426-591) +
 * MeshIOUtils::create_triangles(data, mat_offset, xform) (utils/meshIOUtils.cpp:4-30).
 * Two-step: rt_obj_open parses, rt_obj_fetch copies out (arrays sized from the counts). */
typedef struct rt_obj rt_obj;
rt_obj *rt_obj_open(const char *path, const float xform[16], int32_t mat_offset);
int rt_obj_counts(const rt_obj *o, int64_t *ntri, int32_t *nmat, int32_t *has_uv);
int rt_obj_fetch(const rt_obj *o, float *tri9, int32_t *mat, float *uv6, float *mats16);
void rt_obj_close(rt_obj *o);

/* Diagnostics (tile costs, per-wave records, the wide query and its risk words on the GPU, the host
 * octree digest and wide-BVH query) are declared in rt_mi355x_diag.h; the same library exports them. */

#ifdef __cplusplus
}
#endif
#endif
