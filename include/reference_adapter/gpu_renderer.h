/*
 * gpu_renderer.h -- the reference-side binding of librt_mi355x: a
 * header-only C++ class a maintainer of TomClabault/RayTracerCPP drops into
 * tp2/projets/renderer/ to render with the MI355X library through the reference's own types.
 *
 * It includes only the reference's Qt-free headers -- triangle.h, materials.h, camera.h,
 * mat.h, rendererSettings.h, vec.h, color.h -- and this repository's C ABI (rt_mi355x.h).
 * The method names and arguments are Renderer's (tp2/projets/renderer/renderer.h:20-355);
 * get_image returns the ARGB32 pixels that Renderer::get_image()'s QImage* holds
 * (QImage::Format_ARGB32, row 0 = NDC y = -1), so no Qt type crosses it.  Callers:
 *   RenderThread::run (QT/mainWindowThreads.cpp:39-65)  -> render()
 *   DisplayThread / MainWindow::update_image            -> lock_image_mutex(); get_image();
 *                                                           unlock_image_mutex()
 * Errors: every call that fails throws GpuRendererError with rt_last_error()'s message
 * (the C ABI itself never throws).
 *
 * Build (reference side): -I<repo>/include -I<repo>/include/reference_adapter
 * -I tp2/src -I tp2/projets -I tp2/projets/scene -I tp2/projets/renderer, link
 * -L<repo>/raytracercpp_amd -lrt_mi355x.  tests/test_reference_adapter.py compiles it against
 * /root/reference here and runs a golden scene through it on the GPU.
 */
#ifndef RT_MI355X_REFERENCE_ADAPTER_H
#define RT_MI355X_REFERENCE_ADAPTER_H

#include <stdint.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "rt_mi355x.h"

#include "camera.h"             // tp2/projets/scene: Camera (camera.h:9-33)
#include "color.h"              // tp2/src: Color
#include "mat.h"                // tp2/src: Transform (mat.h:21-71)
#include "materials.h"          // tp2/src: Material, Materials (materials.h:14-80)
#include "rendererSettings.h"   // tp2/projets/renderer: RenderSettings (rendererSettings.h:6-105)
#include "triangle.h"           // tp2/projets: Triangle (triangle.h:42-104)
#include "vec.h"                // tp2/src: Point, Vector

namespace rt_ref {

struct GpuRendererError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// Renderer::_image as plain pixels: QImage(width, height, Format_ARGB32) rows
struct ArgbImage {
    int32_t width = 0, height = 0;
    std::vector<uint32_t> argb;
};

class GpuRenderer {
public:
    explicit GpuRenderer(int device = 0) : h_(rt_create(device))
    {
        if (!h_)
            throw GpuRendererError(std::string("rt_create: ") + rt_last_error());
    }
    ~GpuRenderer() { rt_destroy(h_); }
    GpuRenderer(const GpuRenderer&) = delete;
    GpuRenderer& operator=(const GpuRenderer&) = delete;

    // Renderer::render_settings() = settings (renderer.h:46): every field by name
    void set_render_settings(const RenderSettings& s)
    {
        rt_settings r;
        rt_default_settings(&r);
        r.image_width = s.image_width;
        r.image_height = s.image_height;
        r.enable_ssaa = s.enable_ssaa;
        r.ssaa_factor = s.ssaa_factor;
        r.enable_clipping = s.enable_clipping;
        r.hybrid_rasterization_tracing = s.hybrid_rasterization_tracing;
        r.shading_method = (int32_t)s.shading_method;
        r.compute_shadows = s.compute_shadows;
        r.max_recursion_depth = s.max_recursion_depth;
        r.enable_bvh = s.enable_bvh;
        r.bvh_max_depth = s.bvh_max_depth;
        r.bvh_leaf_object_count = s.bvh_leaf_object_count;
        r.enable_ssao = s.enable_ssao;
        r.ssao_sample_count = s.ssao_sample_count;
        r.ssao_radius = s.ssao_radius;
        r.ssao_amount = s.ssao_amount;
        r.enable_ambient = s.enable_ambient;
        r.enable_diffuse = s.enable_diffuse;
        r.enable_specular = s.enable_specular;
        r.enable_emissive = s.enable_emissive;
        r.rough_reflections_sample_count = s.rough_reflections_sample_count;
        r.enable_ao_mapping = s.enable_ao_mapping;
        r.enable_diffuse_mapping = s.enable_diffuse_mapping;
        r.enable_normal_mapping = s.enable_normal_mapping;
        r.enable_displacement_mapping = s.enable_displacement_mapping;
        r.displacement_mapping_strength = s.displacement_mapping_strength;
        r.parallax_mapping_steps = s.parallax_mapping_steps;
        r.enable_roughness_mapping = s.enable_roughness_mapping;
        r.enable_skysphere = s.enable_skysphere;
        r.enable_skybox = s.enable_skybox;
        check(rt_set_settings(h_, &r), "rt_set_settings");
    }

    // Renderer::change_render_size (renderer.h:118)
    void change_render_size(int width, int height) { check(rt_change_render_size(h_, width, height), "rt_change_render_size"); }

    // Renderer::set_triangles (renderer.h:57): the triangles as MeshIOUtils::create_triangles
    // left them (world space), their material indices and texture coordinates
    void set_triangles(const std::vector<Triangle>& tris)
    {
        const size_t n = tris.size();
        std::vector<float> v(9 * n), uv(6 * n);
        std::vector<int32_t> m(n);
        for (size_t i = 0; i < n; i++) {
            const Triangle& t = tris[i];
            const Point* p[3] = {&t._a, &t._b, &t._c};
            for (int k = 0; k < 3; k++) {
                v[9 * i + 3 * k] = p[k]->x;
                v[9 * i + 3 * k + 1] = p[k]->y;
                v[9 * i + 3 * k + 2] = p[k]->z;
            }
            m[i] = t._materialIndex;
            const float u6[6] = {t._tex_coords_u.x, t._tex_coords_u.y, t._tex_coords_u.z,
                                 t._tex_coords_v.x, t._tex_coords_v.y, t._tex_coords_v.z};
            for (int k = 0; k < 6; k++)
                uv[6 * i + k] = u6[k];
        }
        check(rt_set_triangles(h_, v.data(), m.data(), uv.data(), (int64_t)n), "rt_set_triangles");
    }

    // Renderer::set_materials (renderer.h:62)
    void set_materials(const Materials& mats)
    {
        std::vector<float> f;
        f.reserve(16 * mats.materials.size());
        for (const Material& mt : mats.materials) {
            const float r[16] = {mt.ambient_coeff.r, mt.ambient_coeff.g, mt.ambient_coeff.b,
                                 mt.diffuse.r,       mt.diffuse.g,       mt.diffuse.b,
                                 mt.specular.r,      mt.specular.g,      mt.specular.b,
                                 mt.emission.r,      mt.emission.g,      mt.emission.b,
                                 mt.reflection,      mt.roughness,       mt.ns,
                                 mt.specular_threshold};
            f.insert(f.end(), r, r + 16);
        }
        check(rt_set_materials(h_, f.data(), (int32_t)mats.materials.size()), "rt_set_materials");
    }

    // The scene's camera (Scene::_camera, camera.h:9-33): its position and the two matrices the
    // reference's ray generation reads (renderer.cpp:1086-1098), the projection and view matrices
    // of raster_trace (renderer.cpp:869-1006), and the lens (SSAO, renderer.cpp:1229-1434)
    void set_camera(const Camera& c)
    {
        const float pos[3] = {c._position.x, c._position.y, c._position.z};
        check(rt_set_camera_matrices(h_, pos, &c._perspective_proj_mat_inv.m[0][0], &c._camera_to_world_mat.m[0][0]),
              "rt_set_camera_matrices");
        check(rt_set_camera_projection(h_, &c._perspective_proj_mat.m[0][0], &c._world_to_camera_mat.m[0][0]),
              "rt_set_camera_projection");
        check(rt_set_camera_lens(h_, c._fov, c._aspect_ratio), "rt_set_camera_lens");
    }

    // Renderer::set_light_position (renderer.h:75)
    void set_light_position(const Point& p) { check(rt_set_light_position(h_, p.x, p.y, p.z), "rt_set_light_position"); }

    // Renderer::ray_trace / raster_trace / post_process (renderer.h:149-154)
    void ray_trace() { check(rt_ray_trace(h_), "rt_ray_trace"); }
    void raster_trace() { check(rt_raster_trace(h_), "rt_raster_trace"); }
    void post_process() { check(rt_post_process(h_), "rt_post_process"); }

    // render(Renderer&) (utils/mainUtils.cpp:6-21): the frame and its post-process; milliseconds
    float render()
    {
        float ms = 0.0f;
        check(rt_render(h_, &ms), "rt_render");
        return ms;
    }

    // Renderer::lock_image_mutex / unlock_image_mutex (renderer.h:41-42)
    void lock_image_mutex() { check(rt_lock_image(h_), "rt_lock_image"); }
    void unlock_image_mutex() { check(rt_unlock_image(h_), "rt_unlock_image"); }

    // Renderer::get_image (renderer.h:44): the image's ARGB32 pixels (a copy)
    ArgbImage get_image()
    {
        ArgbImage img;
        check(rt_get_image(h_, nullptr, &img.width, &img.height), "rt_get_image");
        img.argb.resize((size_t)img.width * (size_t)img.height);
        check(rt_get_image(h_, img.argb.data(), &img.width, &img.height), "rt_get_image");
        return img;
    }

    // every GPU of the machine from this one process (no reference counterpart; rt_set_devices)
    void use_devices(const std::vector<int32_t>& ids)
    {
        check(rt_set_devices(h_, ids.empty() ? nullptr : ids.data(), (int32_t)ids.size()), "rt_set_devices");
    }

    rt_renderer* handle() const { return h_; }

private:
    static void check(int rc, const char* what)
    {
        if (rc != RT_OK)
            throw GpuRendererError(std::string(what) + ": " + rt_last_error());
    }
    rt_renderer* h_;
};

}  // namespace rt_ref

#endif
