// adapter_golden.cpp -- the reference-side binding (include/reference_adapter/gpu_renderer.h) driven
// with the reference's own types: the scene file written by tests/test_c_api.py write_scene
// (format: tests/c/render_golden.c) becomes a RenderSettings, a Camera, a Materials and a
// std::vector<Triangle> built by the reference's Triangle constructor (triangle.cpp, compiled
// from /root/reference by `make -C oracle ref`); GpuRenderer renders it (render(Renderer&)) and
// get_image's ARGB32 pixels are written out.
//
//   adapter_golden SCENE OUT
//
// OUT receives int32 width, int32 height, then width x height ARGB32 words.
#include <cstdio>
#include <cstring>
#include <vector>

#include "gpu_renderer.h"

namespace {

bool read_all(FILE* f, void* p, size_t n) { return std::fread(p, 1, n, f) == n; }

void set_transform(Transform& t, const float m[16])
{
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            t.m[i][j] = m[4 * i + j];
}

}  // namespace

int main(int argc, char** argv)
{
    if (argc != 3) {
        std::fprintf(stderr, "usage: %s SCENE OUT\n", argv[0]);
        return 2;
    }
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) {
        std::perror(argv[1]);
        return 1;
    }
    char magic[4];
    int32_t ssz = 0;
    rt_settings cs;
    if (!read_all(f, magic, 4) || std::memcmp(magic, "RTSC", 4) || !read_all(f, &ssz, 4) || ssz != (int32_t)sizeof cs ||
        !read_all(f, &cs, sizeof cs)) {
        std::fprintf(stderr, "bad scene header\n");
        return 1;
    }
    float pos[3], proj_inv[16], c2w[16], proj[16], w2c[16], lens[2], light[3];
    int32_t has_proj = 0, nmat = 0, has_uv = 0;
    int64_t ntri = 0;
    bool ok = read_all(f, pos, 12) && read_all(f, proj_inv, 64) && read_all(f, c2w, 64) && read_all(f, &has_proj, 4) &&
              read_all(f, proj, 64) && read_all(f, w2c, 64) && read_all(f, lens, 8) && read_all(f, light, 12) &&
              read_all(f, &nmat, 4);
    std::vector<float> mats16(ok ? 16 * (size_t)nmat : 0);
    ok = ok && read_all(f, mats16.data(), mats16.size() * 4) && read_all(f, &ntri, 8);
    std::vector<float> tri9(ok ? 9 * (size_t)ntri : 0);
    std::vector<int32_t> tmat(ok ? (size_t)ntri : 0);
    ok = ok && read_all(f, tri9.data(), tri9.size() * 4) && read_all(f, tmat.data(), tmat.size() * 4) &&
         read_all(f, &has_uv, 4);
    std::vector<float> uv6(ok && has_uv ? 6 * (size_t)ntri : 0);
    ok = ok && read_all(f, uv6.data(), uv6.size() * 4);
    std::fclose(f);
    if (!ok) {
        std::fprintf(stderr, "truncated scene file\n");
        return 1;
    }

    // the reference's types
    RenderSettings s;
    s.image_width = cs.image_width;
    s.image_height = cs.image_height;
    s.enable_ssaa = cs.enable_ssaa;
    s.ssaa_factor = cs.ssaa_factor;
    s.enable_clipping = cs.enable_clipping;
    s.hybrid_rasterization_tracing = cs.hybrid_rasterization_tracing;
    s.shading_method = (RenderSettings::ShadingMethod)cs.shading_method;
    s.compute_shadows = cs.compute_shadows;
    s.max_recursion_depth = cs.max_recursion_depth;
    s.enable_bvh = cs.enable_bvh;
    s.bvh_max_depth = cs.bvh_max_depth;
    s.bvh_leaf_object_count = cs.bvh_leaf_object_count;
    s.enable_ssao = cs.enable_ssao;
    s.ssao_sample_count = cs.ssao_sample_count;
    s.ssao_radius = cs.ssao_radius;
    s.ssao_amount = cs.ssao_amount;
    s.enable_ambient = cs.enable_ambient;
    s.enable_diffuse = cs.enable_diffuse;
    s.enable_specular = cs.enable_specular;
    s.enable_emissive = cs.enable_emissive;
    s.rough_reflections_sample_count = cs.rough_reflections_sample_count;
    s.enable_ao_mapping = cs.enable_ao_mapping;
    s.enable_diffuse_mapping = cs.enable_diffuse_mapping;
    s.enable_normal_mapping = cs.enable_normal_mapping;
    s.enable_displacement_mapping = cs.enable_displacement_mapping;
    s.displacement_mapping_strength = cs.displacement_mapping_strength;
    s.parallax_mapping_steps = cs.parallax_mapping_steps;
    s.enable_roughness_mapping = cs.enable_roughness_mapping;
    s.enable_skysphere = cs.enable_skysphere;
    s.enable_skybox = cs.enable_skybox;

    // Camera::set_aspect_ratio (camera.cpp:5-11, the reference's code) gives the projection for the
    // file's lens; the file's matrices then replace what it holds
    Camera cam(Point(pos[0], pos[1], pos[2]), lens[0]);
    cam.set_aspect_ratio(lens[1]);
    set_transform(cam._perspective_proj_mat_inv, proj_inv);
    set_transform(cam._camera_to_world_mat, c2w);
    if (has_proj) {
        set_transform(cam._perspective_proj_mat, proj);
        set_transform(cam._world_to_camera_mat, w2c);
    } else
        cam._world_to_camera_mat = cam._camera_to_world_mat.inverse();

    Materials mats;
    for (int32_t i = 0; i < nmat; i++) {
        const float* r = &mats16[16 * (size_t)i];
        Material m;
        m.ambient_coeff = Color(r[0], r[1], r[2]);
        m.diffuse = Color(r[3], r[4], r[5]);
        m.specular = Color(r[6], r[7], r[8]);
        m.emission = Color(r[9], r[10], r[11]);
        m.reflection = r[12];
        m.roughness = r[13];
        m.ns = r[14];
        m.specular_threshold = r[15];
        mats.materials.push_back(m);
    }

    std::vector<Triangle> tris;
    tris.reserve((size_t)ntri);
    for (int64_t i = 0; i < ntri; i++) {
        const float* t = &tri9[9 * (size_t)i];
        const Point tu = has_uv ? Point(uv6[6 * i], uv6[6 * i + 1], uv6[6 * i + 2]) : Point(-1, -1, -1);
        const Point tv = has_uv ? Point(uv6[6 * i + 3], uv6[6 * i + 4], uv6[6 * i + 5]) : Point(-1, -1, -1);
        tris.emplace_back(Point(t[0], t[1], t[2]), Point(t[3], t[4], t[5]), Point(t[6], t[7], t[8]), tmat[i], tu, tv);
    }

    try {
        rt_ref::GpuRenderer r(0);
        r.set_render_settings(s);
        r.set_camera(cam);
        r.set_light_position(Point(light[0], light[1], light[2]));
        r.set_materials(mats);
        r.set_triangles(tris);
        r.render();
        r.lock_image_mutex();   // the display thread's pattern (mainwindow.cpp:85-87)
        rt_ref::ArgbImage img = r.get_image();
        r.unlock_image_mutex();
        FILE* o = std::fopen(argv[2], "wb");
        if (!o || std::fwrite(&img.width, 4, 1, o) != 1 || std::fwrite(&img.height, 4, 1, o) != 1 ||
            std::fwrite(img.argb.data(), 4, img.argb.size(), o) != img.argb.size()) {
            std::perror(argv[2]);
            return 1;
        }
        std::fclose(o);
    } catch (const rt_ref::GpuRendererError& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 1;
    }
    return 0;
}
