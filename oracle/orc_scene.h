/*
 * orc_scene.h -- TEST INFRASTRUCTURE ONLY (oracle side).
 *
 * Flat, plain-C description of a scene + render settings shared by the two
 * checkers under oracle/:
 *   - oracle.c          : CPU restatement of the reference hot path (the "port")
 *   - ref_harness.cpp   : harness linked against the reference's own Qt-free
 *                         translation units (built into oracle/_ref/)
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load anything built from this directory.  The product (raytracercpp_amd/)
 * never includes this header.
 *
 * Field meanings mirror RenderSettings (tp2/projets/renderer/rendererSettings.h:6-105),
 * Material (tp2/src/materials.h:14-38), Camera (tp2/projets/scene/camera.h:9-33)
 * and PointLight (tp2/projets/scene/light.h:6-12).
 */
#ifndef ORC_SCENE_H
#define ORC_SCENE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Material record: 16 floats, RGB colours (alpha never reaches RGB). */
enum {
    ORC_MAT_AMBIENT = 0,   /* ambient_coeff r,g,b */
    ORC_MAT_DIFFUSE = 3,   /* diffuse r,g,b */
    ORC_MAT_SPECULAR = 6,  /* specular r,g,b */
    ORC_MAT_EMISSION = 9,  /* emission r,g,b */
    ORC_MAT_REFLECTION = 12,
    ORC_MAT_ROUGHNESS = 13,
    ORC_MAT_NS = 14,
    ORC_MAT_SPEC_THRESHOLD = 15,
    ORC_MAT_STRIDE = 16
};

/* texture slots (Renderer::set_*_map, renderer.h:77-84) */
enum {
    ORC_TEX_AO = 0,
    ORC_TEX_DIFFUSE = 1,
    ORC_TEX_NORMAL = 2,
    ORC_TEX_DISPLACEMENT = 3,
    ORC_TEX_ROUGHNESS = 4,
    ORC_TEX_SKYSPHERE = 5,
    ORC_TEX_COUNT = 6
};

/* RenderSettings::ShadingMethod (rendererSettings.h:8-25) */
enum {
    ORC_RT_SHADING = 0,
    ORC_ABS_NORMALS_SHADING = 1,
    ORC_PASTEL_NORMALS_SHADING = 2,
    ORC_BARYCENTRIC_COORDINATES_SHADING = 3,
    ORC_VISUALIZE_AO = 4
};

typedef struct orc_scene {
    /* triangles, already in world space (MeshIOUtils::create_triangles applied) */
    int64_t ntri;
    const float *tri;       /* [ntri][9]  a.xyz b.xyz c.xyz */
    const int32_t *tri_mat; /* [ntri]     _materialIndex */
    const float *tri_uv;    /* [ntri][6]  _tex_coords_u.xyz, _tex_coords_v.xyz ; NULL => (-1,-1,-1) */

    /* analytic shapes, in add_analytic_shape order: kind 0 = Sphere, 1 = Plane */
    int32_t nshape;
    const int32_t *shape_kind; /* [nshape] */
    const float *shape;        /* [nshape][6] sphere: cx cy cz r - - ; plane: px py pz nx ny nz */
    const int32_t *shape_mat;  /* [nshape] */

    int32_t nmat;
    const float *mat; /* [nmat][ORC_MAT_STRIDE] */

    float cam_pos[3];
    float proj_inv[16];     /* Camera::_perspective_proj_mat_inv, row-major m[i][j] */
    float cam_to_world[16]; /* Camera::_camera_to_world_mat, row-major */
    float light[3];

    /* float RGBA textures (Image), row-major, 4 floats per texel */
    int32_t tex_w[ORC_TEX_COUNT], tex_h[ORC_TEX_COUNT];
    const float *tex[ORC_TEX_COUNT];
    /* skybox faces: right, left, top, bottom, back, front (skybox.h:12-16) */
    int32_t sky_w[6], sky_h[6];
    const float *sky[6];

    /* hybrid rasterisation (Renderer::raster_trace, renderer.cpp:869-1006) */
    float proj[16];         /* Camera::_perspective_proj_mat, row-major */
    float world_to_cam[16]; /* Camera::_world_to_camera_mat, row-major */

    /* Camera::_fov / _aspect_ratio (scene/camera.h:22-23), read by the SSAO pass
     * (renderer.cpp:1245, 1281-1282, 1378-1379) */
    float cam_fov, cam_aspect;
} orc_scene;

typedef struct orc_settings {
    int32_t image_width, image_height;
    int32_t enable_ssaa, ssaa_factor;
    int32_t shading_method;
    int32_t compute_shadows;
    int32_t max_recursion_depth;
    int32_t enable_bvh, bvh_max_depth, bvh_leaf_object_count;
    int32_t enable_ambient, enable_diffuse, enable_specular, enable_emissive;
    int32_t rough_reflections_sample_count;
    int32_t enable_ao_mapping, enable_diffuse_mapping, enable_normal_mapping;
    int32_t enable_displacement_mapping;
    float displacement_mapping_strength;
    int32_t parallax_mapping_steps;
    int32_t enable_roughness_mapping;
    int32_t enable_skysphere, enable_skybox;
    uint32_t rng_seed; /* counter-based RNG seed for rough reflections */
    int32_t enable_clipping; /* raster_trace: clip against the 6 frustum planes */
    /* post_process_ssao_SIMD (renderer.cpp:1229-1434), rendererSettings.h:66-73 */
    int32_t enable_ssao, ssao_sample_count;
    float ssao_radius, ssao_amount;
} orc_settings;

/* per-internal-pixel outputs; any pointer may be NULL.  Arrays cover the
 * rows [row_begin, row_begin+row_count) of the render_w x render_h image. */
typedef struct orc_outputs {
    uint32_t *argb;   /* qRgb(r*255, g*255, b*255) of trace_ray's colour */
    float *rgba;      /* trace_ray colour (4 floats) */
    int32_t *hit_id;  /* primary closest hit: triangle index, -2-k for shape k, -1 miss (t <= 0.1) */
    float *hit_t;     /* final_hit_info.t of the primary ray (-1 when nothing) */
    uint8_t *shadow;  /* 1 when the primary hit point is shadowed */
    /* Renderer::_z_buffer / _normal_buffer as ray_trace (renderer.cpp:1107-1110) or
     * raster_trace (:975-979) leave them for SSAO, starting from clear_z_buffer /
     * clear_normal_buffer (INFINITY / Vector(0,0,0), renderer.cpp:165-173) */
    float *zbuf;      /* [px] */
    float *nbuf;      /* [px][3] */
} orc_outputs;

/* counters (ray + traversal statistics) */
typedef struct orc_counters {
    int64_t primary_rays;
    int64_t shadow_rays;
    int64_t reflection_rays;
    int64_t vol_tests_primary, tri_tests_primary;   /* reference semantics */
    int64_t vol_tests_shadow, tri_tests_shadow;
    int64_t vol_tests_refl, tri_tests_refl;
    int64_t child_tests_primary, child_tests_shadow; /* k-DOP tests without the re-test on entry */
} orc_counters;

#ifdef __cplusplus
}
#endif
#endif
