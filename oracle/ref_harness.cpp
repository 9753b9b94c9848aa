/*
 * ref_harness.cpp -- TEST INFRASTRUCTURE ONLY (builds into oracle/_ref/).
 *
 * Links the reference's own, unmodified, Qt-free translation units (compiled
 * straight from /root/reference/tp2 by oracle/Makefile) and exposes them
 * through a small extern "C" surface so that tests/golden fixtures can be
 * generated from the reference itself:
 *
 *   - transforms / camera matrices   : Transform, Perspective, RotationX/Y/Z,
 *                                      Translation, Scale, inverse  (tp2/src/mat.cpp)
 *                                      Camera::set_aspect_ratio      (tp2/projets/scene/camera.cpp:5-11)
 *   - OBJ loading                    : read_meshio_data (tp2/src/mesh_io.cpp:426-591)
 *                                      + MeshIOUtils::create_triangles (tp2/projets/utils/meshIOUtils.cpp:4-30)
 *   - closest-hit queries            : BVH::BVH / BVH::intersect (tp2/projets/bvh.{h,cpp})
 *                                      Triangle::intersect (tp2/projets/triangle.cpp:25-91)
 *                                      Sphere/Plane::intersect (tp2/projets/analyticShape.cpp:9-76)
 *   - texture / sky sampling         : Image::texture_floor (tp2/src/image.h:94-97),
 *                                      Skybox::sample (tp2/projets/renderer/skybox.cpp:12-51)
 *
 * tp2/projets/renderer/renderer.cpp includes <QImage> (renderer.h:4) and Qt is
 * not in this image, so Renderer itself cannot be compiled here (writing a
 * stand-in QImage header is not allowed).  The per-pixel control flow of
 * Renderer::ray_trace / trace_ray / shade_ray_inter_point / is_shadowed /
 * compute_reflection is therefore restated below, line by line, on top of the
 * reference's own compiled primitives (vector / colour / material operators,
 * BVH, triangle and analytic-shape intersection, texture sampling), so every
 * floating-point operation is executed by reference code or by an expression
 * written with the reference's own operator overloads.
 *
 * Compiled with -ffp-contract=off (portable parity target).
 */
#include <cmath>
#include <cstdint>
#include <cstring>
#include <algorithm>
#include <variant>
#include <vector>

#include <omp.h>

#include "xorshift.h"   // the reference's XorShiftGenerator (sequential RNG mode)

#include "analyticShape.h"
#include "bvh.h"
#include "camera.h"
#include "color.h"
#include "image.h"
#include "mat.h"
#include "materials.h"
#include "meshIOUtils.h"
#include "mesh_io.h"
#include "skybox.h"
#include "triangle.h"

#include "orc_scene.h"

#ifndef M_PI
#define M_PI 3.141592653589793
#endif

namespace {

// Renderer constants (renderer.h:23-29, renderer.cpp:18-19)
const float H_EPSILON = 1.0e-4f;
const float H_SHADOW_INTENSITY = 0.5f;
const Color H_AMBIENT_COLOR = Color(0.1f, 0.1f, 0.1f);
const Color H_BACKGROUND_COLOR = Color(135.0f / 255.0f, 206.0f / 255.0f, 235.0f / 255.0f);

void to_transform(const float m[16], Transform& t)
{
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            t.m[i][j] = m[i * 4 + j];
}

void from_transform(const Transform& t, float m[16])
{
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            m[i * 4 + j] = t.m[i][j];
}

uint32_t h_qrgb(int r, int g, int b)
{
    // qRgb(r, g, b) = 0xff000000 | ((r & 0xff) << 16) | ((g & 0xff) << 8) | (b & 0xff)
    return 0xff000000u | ((uint32_t)(r & 0xff) << 16) | ((uint32_t)(g & 0xff) << 8) | (uint32_t)(b & 0xff);
}

// float -> int conversion as the x86-64 cvttss2si the reference compiles to
int h_f2i(float f)
{
    if (!(f > -2147483648.0f && f < 2147483648.0f))
        return INT32_MIN;
    return (int)f;
}

// ImageUtils::gkit_color_to_Qt_ARGB32_uint (imageUtils.h:149-152)
uint32_t h_color_to_argb(const Color& c)
{
    return h_qrgb(h_f2i(c.r * 255), h_f2i(c.g * 255), h_f2i(c.b * 255));
}

/* Path-keyed RNG for rough reflections (xorshift.h:37-65 draws).  The
 * reference seeds one generator per OpenMP thread with std::rand(), so its
 * stream is not reproducible; this one is shared verbatim by the oracle and the
 * HIP kernels.  Every compute_reflection call (a "frame") has a 32-bit key: the
 * frame of a primary hit is keyed by h_pixel_seed(pixel, seed); sample i of a
 * frame draws its three randoms from a fresh xorshift32 state
 * h_sample_state(key, i), and the frame its hit spawns is keyed
 * h_child_key(key, i).  No draw depends on how many randoms other samples used,
 * so the samples of a frame can be traced in any order. */
struct HRng {
    uint32_t state;
    uint32_t next()
    {
        uint32_t x = state;
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        return state = x;
    }
    float bilateral() { return next() / (float)UINT32_MAX * 2 - 1; }
};

uint32_t h_pixel_seed(uint32_t pixel, uint32_t seed)
{
    uint32_t x = pixel * 0x9E3779B9u ^ seed;
    x ^= x >> 16; x *= 0x7feb352dU;
    x ^= x >> 15; x *= 0x846ca68bU;
    x ^= x >> 16;
    return x ? x : 0x9E3779B9u;
}

uint32_t h_mix32(uint32_t x)
{
    x ^= x >> 16; x *= 0x7feb352dU;
    x ^= x >> 15; x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

uint32_t h_sample_state(uint32_t key, uint32_t i)
{
    uint32_t x = h_mix32(key ^ (0x9E3779B9u * (2u * i + 1u)));
    return x ? x : 0x9E3779B9u;
}

uint32_t h_child_key(uint32_t key, uint32_t i) { return h_mix32(key ^ (0x85EBCA6Bu * (2u * i + 2u))); }

/* Sequential mode (ref_set_rng_sequential): the reference's own stream at OMP_NUM_THREADS=1.
 * One XorShiftGenerator (the reference's struct, xorshift.h:37-65) seeded as
 * init_xorshift_generators seeds thread 0's (renderer.cpp:51-59: std::rand()), consumed in
 * the reference's order: pixels row by row (renderer.cpp:1082-1088, one thread), the three
 * draws of each rough sample, depth first through the recursion (renderer.cpp:294-313).
 * Used only to make the statistical fixtures of tests/golden/make_rng_stats.py. */
static bool g_seq = false;
static XorShiftGenerator g_seq_gen(1u);

struct HScene {
    std::vector<Triangle> tris;
    BVH bvh;
    std::vector<AnalyticShapesTypes> shapes;
    std::vector<int> shape_index;
    Materials materials;
    Point cam_pos;
    Transform proj_inv, cam_to_world;
    Transform proj, world_to_cam;   // raster_trace
    Point light;
    Image tex[ORC_TEX_COUNT];
    Skybox skybox;
    orc_settings s;
};

Image make_image(int w, int h, const float* rgba)
{
    if (!rgba || w <= 0 || h <= 0)
        return Image();
    Image img(w, h);
    for (int i = 0; i < w * h; i++)
        img((size_t)i) = Color(rgba[4 * i], rgba[4 * i + 1], rgba[4 * i + 2], rgba[4 * i + 3]);
    return img;
}

void build_scene(HScene& H, const orc_scene* sc, const orc_settings* st)
{
    H.s = *st;
    H.tris.reserve(sc->ntri);
    for (int64_t i = 0; i < sc->ntri; i++) {
        const float* t = sc->tri + 9 * i;
        Point uu(-1, -1, -1), vv(-1, -1, -1);
        if (sc->tri_uv) {
            const float* uv = sc->tri_uv + 6 * i;
            uu = Point(uv[0], uv[1], uv[2]);
            vv = Point(uv[3], uv[4], uv[5]);
        }
        H.tris.push_back(Triangle(Point(t[0], t[1], t[2]), Point(t[3], t[4], t[5]), Point(t[6], t[7], t[8]),
                                  sc->tri_mat ? sc->tri_mat[i] : -1, uu, vv));
    }
    if (st->enable_bvh)
        H.bvh = BVH(&H.tris, st->bvh_max_depth, st->bvh_leaf_object_count);   // Renderer::set_triangles, renderer.cpp:137-144
    for (int k = 0; k < sc->nshape; k++) {
        const float* p = sc->shape + 6 * k;
        if (sc->shape_kind[k] == 0)
            H.shapes.push_back(Sphere(Point(p[0], p[1], p[2]), p[3], sc->shape_mat[k]));
        else
            H.shapes.push_back(Plane(Point(p[0], p[1], p[2]), Vector(p[3], p[4], p[5]), sc->shape_mat[k]));
    }
    for (int m = 0; m < sc->nmat; m++) {
        const float* f = sc->mat + ORC_MAT_STRIDE * m;
        Material mat;
        mat.ambient_coeff = Color(f[ORC_MAT_AMBIENT], f[ORC_MAT_AMBIENT + 1], f[ORC_MAT_AMBIENT + 2]);
        mat.diffuse = Color(f[ORC_MAT_DIFFUSE], f[ORC_MAT_DIFFUSE + 1], f[ORC_MAT_DIFFUSE + 2]);
        mat.specular = Color(f[ORC_MAT_SPECULAR], f[ORC_MAT_SPECULAR + 1], f[ORC_MAT_SPECULAR + 2]);
        mat.emission = Color(f[ORC_MAT_EMISSION], f[ORC_MAT_EMISSION + 1], f[ORC_MAT_EMISSION + 2]);
        mat.reflection = f[ORC_MAT_REFLECTION];
        mat.roughness = f[ORC_MAT_ROUGHNESS];
        mat.ns = f[ORC_MAT_NS];
        mat.specular_threshold = f[ORC_MAT_SPEC_THRESHOLD];
        H.materials.materials.push_back(mat);
        H.materials.names.push_back("m");
    }
    H.cam_pos = Point(sc->cam_pos[0], sc->cam_pos[1], sc->cam_pos[2]);
    to_transform(sc->proj_inv, H.proj_inv);
    to_transform(sc->cam_to_world, H.cam_to_world);
    to_transform(sc->proj, H.proj);
    to_transform(sc->world_to_cam, H.world_to_cam);
    H.light = Point(sc->light[0], sc->light[1], sc->light[2]);
    for (int i = 0; i < ORC_TEX_COUNT; i++)
        H.tex[i] = make_image(sc->tex_w[i], sc->tex_h[i], sc->tex[i]);
    Image faces[6];
    for (int i = 0; i < 6; i++)
        faces[i] = make_image(sc->sky_w[i], sc->sky_h[i], sc->sky[i]);
    H.skybox = Skybox(faces);
}

struct Tracer {
    const HScene& H;
    HRng rng;
    uint32_t frame_key = 0;   // key of the next compute_reflection frame (see HRng)

    explicit Tracer(const HScene& h) : H(h), rng{1} {}

    Color sample_texture(const Image& t, float u, float v) const { return t.texture_floor(u, v); }

    // renderer.cpp:436-445
    void get_tex_coords(const Triangle* tri, float u, float v, float& tu, float& tv) const
    {
        if (tri != nullptr)
            tri->interpolate_texcoords(u, v, tu, tv);
        else {
            tu = u;
            tv = v;
        }
    }

    // renderer.cpp:263-266
    Color compute_diffuse(const Material& m, const Vector& n, const Vector& l) const
    {
        return m.diffuse * Color(std::max(0.0f, dot(n, l)));
    }

    // renderer.cpp:270-280
    Color compute_specular(const Material& m, const Vector& d, const Vector& n, const Vector& l) const
    {
        Vector h = normalize(l - d);
        float angle = dot(h, n);
        if (angle <= m.specular_threshold)
            return Color(0, 0, 0);
        return m.specular * Color(std::pow(std::max(0.0f, angle), m.ns));
    }

    // renderer.cpp:447-461
    float ao_mapping(const HitInfo& hi, float u, float v) const
    {
        float tu, tv;
        get_tex_coords(hi.triangle, u, v, tu, tv);
        return sample_texture(H.tex[ORC_TEX_AO], tu, tv).r;
    }
    Color diffuse_mapping(const HitInfo& hi, float u, float v) const
    {
        float tu, tv;
        get_tex_coords(hi.triangle, u, v, tu, tv);
        return sample_texture(H.tex[ORC_TEX_DIFFUSE], tu, tv);
    }

    // renderer.cpp:464-478
    Vector normal_mapping(const HitInfo& hi, float u, float v) const
    {
        float tu, tv;
        get_tex_coords(hi.triangle, u, v, tu, tv);
        Vector tangent = hi.tangent;
        Vector bitangent = cross(tangent, hi.normal_at_intersection);
        Transform btn(tangent, bitangent, hi.normal_at_intersection, Vector(0, 0, 0));
        Color nc = sample_texture(H.tex[ORC_TEX_NORMAL], tu, tv);
        Vector nmn = Vector(nc.r, nc.g, nc.b) * 2 - Vector(1, 1, 1);
        Vector pert = btn(normalize(nmn));
        return normalize(pert);
    }

    // renderer.cpp:518-554
    void parallax_occlusion_mapping(const Triangle* tri, float u, float v, const Vector& view, float& nu, float& nv) const
    {
        float tu, tv;
        get_tex_coords(tri, u, v, tu, tv);
        const Image& disp = H.tex[ORC_TEX_DISPLACEMENT];
        float current_depth;
        float depth_step = 1.0f / H.s.parallax_mapping_steps;
        float sampled_depth = sample_texture(disp, tu, tv).r;
        Vector search = -view * H.s.displacement_mapping_strength;
        float du = search.x / H.s.parallax_mapping_steps;
        float dv = search.y / H.s.parallax_mapping_steps;
        current_depth = 0.0f;
        nu = tu;
        nv = tv;
        while (current_depth < sampled_depth) {
            nu += du;
            nv += dv;
            sampled_depth = sample_texture(disp, nu, nv).r;
            current_depth += depth_step;
        }
        float pu = nu - du;
        float pv = nv - dv;
        float after = sampled_depth - current_depth;
        float before = sample_texture(disp, pu, pv).r - (current_depth - depth_step);
        float w = after / (after - before);
        nu = (1 - w) * nu + w * pu;
        nv = (1 - w) * nv + w * pv;
    }

    // renderer.cpp:340-402
    bool is_shadowed(const Point& p, const Vector& n, const Point& lp, orc_counters* cnt) const
    {
        if (!H.s.compute_shadows)
            return false;
        if (cnt) cnt->shadow_rays++;
        Ray ray(p + n * H_EPSILON, normalize(lp - p));
        HitInfo hi;
        if (H.s.enable_bvh) {
            if (H.bvh.intersect(ray, hi)) {
                Point q = ray._origin + ray._direction * hi.t;
                if (length2(Point(p) - Point(q)) < length2(Point(p) - Point(lp)))
                    return true;
            }
        } else {
            for (const Triangle& tri : H.tris)
                if (tri.intersect(ray, hi)) {
                    Point q = ray._origin + ray._direction * hi.t;
                    if (length2(Point(p) - Point(q)) < length2(Point(p) - Point(lp)))
                        return true;
                }
        }
        for (AnalyticShapesTypes shape : H.shapes) {
            bool found = false;
            std::visit([&](auto& sh) {
                if (sh.intersect(ray, hi)) {
                    Point q = ray._origin + ray._direction * hi.t;
                    if (length2(Point(p) - Point(q)) < length2(Point(p) - Point(lp)))
                        found = true;
                }
            }, shape);
            if (found)
                return true;
        }
        return false;
    }

    // renderer.cpp:283-338
    Color compute_reflection(const Ray& ray, const Point& ip, const HitInfo& hi, int depth, orc_counters* cnt)
    {
        bool found = false;
        HitInfo rhi;
        const Material& m = H.materials.material(hi.mat_index);
        Vector nn = hi.normal_at_intersection;
        Point ro = ip + nn * 0.01f;
        Vector perfect = ray._direction - 2 * dot(ray._direction, nn) * nn;
        int sample_count = 0;
        Color total = Color(0.0f);
        const uint32_t key = frame_key;
        for (int i = 0; i < H.s.rough_reflections_sample_count; i++) {
            rng.state = h_sample_state(key, (uint32_t)i);
            frame_key = h_child_key(key, (uint32_t)i);
            float roughness;
            if (H.s.enable_roughness_mapping) {
                float tu, tv;
                get_tex_coords(hi.triangle, hi.u, hi.v, tu, tv);
                roughness = sample_texture(H.tex[ORC_TEX_ROUGHNESS], tu, tv).r;
            } else
                roughness = m.roughness;
            if (roughness > 0) {
                float rx, ry, rz;
                if (g_seq) {
                    rx = g_seq_gen.get_rand_bilateral();
                    ry = g_seq_gen.get_rand_bilateral();
                    rz = g_seq_gen.get_rand_bilateral();
                } else {
                    rx = rng.bilateral();
                    ry = rng.bilateral();
                    rz = rng.bilateral();
                }
                Vector rd = normalize(Vector(rx, ry, rz));
                if (dot(rd, hi.normal_at_intersection) < 0)
                    rd = -rd;
                Vector lerped = roughness * rd + (1 - roughness) * perfect;
                if (cnt) cnt->reflection_rays++;
                total = total + trace_ray(Ray(ro, lerped), rhi, depth + 1, found, nullptr, cnt);
                sample_count++;
            } else {
                if (cnt) cnt->reflection_rays++;
                total = total + trace_ray(Ray(ro, perfect), rhi, depth + 1, found, nullptr, cnt);
                sample_count = 1;
                break;
            }
        }
        return total / Color(sample_count) * Color(m.reflection);
    }

    // renderer.cpp:556-617
    Color shade(const Ray& ray, HitInfo& hi, int depth, bool* shadowed_out, orc_counters* cnt)
    {
        Color fc = Color(0.0f, 0.0f, 0.0f);
        int sm = H.s.shading_method;
        if (sm == ORC_RT_SHADING) {
            float u = hi.u, v = hi.v;
            Point ip = ray._origin + ray._direction * hi.t;
            if (H.s.enable_displacement_mapping)
                parallax_occlusion_mapping(hi.triangle, hi.u, hi.v, normalize(H.cam_pos - ip), u, v);
            Vector dl = normalize(H.light - ip);
            if (H.s.enable_normal_mapping)
                hi.normal_at_intersection = normal_mapping(hi, u, v);
            Material m = H.materials(hi.mat_index);
            float ao = 1.0f;
            if (H.s.enable_ao_mapping)
                ao = ao_mapping(hi, u, v);
            Color dc;
            if (H.s.enable_diffuse_mapping) {
                dc = diffuse_mapping(hi, u, v);
                dc = dc * Color(std::max(0.5f, dot(hi.normal_at_intersection, normalize(H.cam_pos - ip))));
            } else
                dc = compute_diffuse(m, hi.normal_at_intersection, dl);
            fc = fc + dc * ao * (bool)H.s.enable_diffuse;
            fc = fc + compute_specular(m, ray._direction, hi.normal_at_intersection, dl) * (bool)H.s.enable_specular;
            bool sh = is_shadowed(ip, hi.normal_at_intersection, H.light, cnt);
            if (shadowed_out) *shadowed_out = sh;
            if (sh)
                fc = fc * Color(H_SHADOW_INTENSITY);
            fc = fc + m.emission * (bool)H.s.enable_emissive;
            if (m.reflection > 0.0f)
                fc = fc + compute_reflection(ray, ip, hi, depth, cnt) * m.reflection;
            fc = fc + H_AMBIENT_COLOR * m.ambient_coeff * (1 - m.reflection) * (bool)H.s.enable_ambient;
        } else if (sm == ORC_ABS_NORMALS_SHADING) {
            const Vector& n = hi.normal_at_intersection;
            fc = Color(std::abs(n.x), std::abs(n.y), std::abs(n.z));
        } else if (sm == ORC_PASTEL_NORMALS_SHADING) {
            const Vector& n = hi.normal_at_intersection;
            fc = (Color(n.x, n.y, n.z) + Color(1.0f, 1.0f, 1.0f)) * 0.5;
        } else if (sm == ORC_BARYCENTRIC_COORDINATES_SHADING) {
            fc = Color(1, 0, 0) * hi.u + Color(0, 1.0, 0) * hi.v + Color(0, 0, 1) * (1 - hi.u - hi.v);
        } else if (sm == ORC_VISUALIZE_AO) {
            Color c = Color(0.9f, 0.9f, 0.9f);
            if (H.s.enable_ao_mapping) {
                float tu, tv;
                hi.triangle->interpolate_texcoords(hi.u, hi.v, tu, tv);
                c = c * Color(sample_texture(H.tex[ORC_TEX_AO], tu, tv).r);
            }
            fc = c;
        }
        fc.r = std::clamp(fc.r, 0.0f, 1.0f);
        fc.g = std::clamp(fc.g, 0.0f, 1.0f);
        fc.b = std::clamp(fc.b, 0.0f, 1.0f);
        fc.a = 1.0f;
        return fc;
    }

    // renderer.cpp:1008-1066
    Color trace_ray(const Ray& ray, HitInfo& fin, int depth, bool& found, int* src_out, orc_counters* cnt,
                    bool* shadowed_out = nullptr)
    {
        HitInfo local;
        if (depth > H.s.max_recursion_depth)
            return Color(0.0f);
        int src = -1;
        if (H.s.enable_bvh) {
            if (H.bvh.intersect(ray, local))
                if (local.t < fin.t || fin.t == -1) {
                    fin = local;
                    src = (int)(local.triangle - H.tris.data());
                }
        } else {
            for (const Triangle& tri : H.tris)
                if (tri.intersect(ray, local))
                    if (local.t < fin.t || fin.t == -1) {
                        fin = local;
                        src = (int)(&tri - H.tris.data());
                    }
        }
        int k = 0;
        for (AnalyticShapesTypes shape : H.shapes) {
            std::visit([&](auto& sh) {
                if (sh.intersect(ray, local))
                    if (local.t < fin.t || fin.t == -1) {
                        fin = local;
                        src = -2 - k;
                    }
            }, shape);
            k++;
        }
        if (src_out) *src_out = src;
        float min_t = 0.1;
        if (fin.t > min_t) {
            found = true;
            Color c = shade(ray, fin, depth, shadowed_out, cnt);
            c.r = std::clamp(c.r, 0.0f, 1.0f);
            c.g = std::clamp(c.g, 0.0f, 1.0f);
            c.b = std::clamp(c.b, 0.0f, 1.0f);
            c.a = 1.0f;
            return c;
        }
        if (H.s.enable_skysphere) {
            float u = 0.5 + std::atan2(-ray._direction.z, -ray._direction.x) / (2 * M_PI);
            float v = 0.5 + std::asin(-ray._direction.y) / M_PI;
            return sample_texture(H.tex[ORC_TEX_SKYSPHERE], u, v);
        } else if (H.s.enable_skybox)
            return H.skybox.sample(ray._direction);
        return H_BACKGROUND_COLOR;
    }
};

void render_w_h(const orc_settings* s, int& w, int& h)
{
    // Renderer::get_render_width_height, renderer.cpp:116-120
    w = s->enable_ssaa ? s->image_width * s->ssaa_factor : s->image_width;
    h = s->enable_ssaa ? s->image_height * s->ssaa_factor : s->image_height;
}

}  // namespace

extern "C" {

/* Camera::set_aspect_ratio (camera.cpp:5-11): Perspective(fov, aspect, near, far).inverse() */
void ref_camera_matrices(float fov, float aspect, float znear, float zfar, float out_proj[16], float out_proj_inv[16])
{
    Camera cam(Point(0, 0, 0), fov, znear, zfar);
    cam.set_aspect_ratio(aspect);
    from_transform(cam._perspective_proj_mat, out_proj);
    from_transform(cam._perspective_proj_mat_inv, out_proj_inv);
}

/* kind: 0 Translation(x,y,z) 1 RotationX(a) 2 RotationY(a) 3 RotationZ(a) 4 Scale(x,y,z) 5 Identity */
void ref_make_transform(int kind, float x, float y, float z, float out[16])
{
    Transform t;
    switch (kind) {
    case 0: t = Translation(x, y, z); break;
    case 1: t = RotationX(x); break;
    case 2: t = RotationY(x); break;
    case 3: t = RotationZ(x); break;
    case 4: t = Scale(x, y, z); break;
    default: t = Identity(); break;
    }
    from_transform(t, out);
}

/* a(b): compose_transform (mat.cpp:363-371) */
void ref_compose(const float a[16], const float b[16], float out[16])
{
    Transform ta, tb;
    to_transform(a, ta);
    to_transform(b, tb);
    from_transform(ta(tb), out);
}

void ref_inverse(const float a[16], float out[16])
{
    Transform ta;
    to_transform(a, ta);
    from_transform(ta.inverse(), out);
}

/* Transform::operator()(Point) (mat.cpp:83-100) on n points */
void ref_transform_points(const float m[16], const float* pts, int64_t n, float* out)
{
    Transform t;
    to_transform(m, t);
    for (int64_t i = 0; i < n; i++) {
        Point p = t(Point(pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]));
        out[3 * i] = p.x;
        out[3 * i + 1] = p.y;
        out[3 * i + 2] = p.z;
    }
}

/* read_meshio_data + MeshIOUtils::create_triangles(data, mat_offset, xform).
 * Returns the triangle count (or -1 on error); fills up to cap triangles.
 * out_mats receives up to mat_cap materials as ORC_MAT_STRIDE floats
 * (specular_threshold left at 0). */
int64_t ref_load_obj(const char* path, const float xform[16], int mat_offset, float* out_tri9, int32_t* out_mat,
                     float* out_uv6, int64_t cap, int32_t* out_has_uv, float* out_mats, int32_t mat_cap,
                     int32_t* out_nmat)
{
    MeshIOData data = read_meshio_data(path);
    Transform t;
    to_transform(xform, t);
    std::vector<Triangle> tris = MeshIOUtils::create_triangles(data, mat_offset, t);
    *out_has_uv = data.texcoords.size() > 0;
    int64_t n = (int64_t)tris.size();
    for (int64_t i = 0; i < n && i < cap; i++) {
        const Triangle& tr = tris[i];
        const Point* v[3] = {&tr._a, &tr._b, &tr._c};
        for (int k = 0; k < 3; k++) {
            out_tri9[9 * i + 3 * k] = v[k]->x;
            out_tri9[9 * i + 3 * k + 1] = v[k]->y;
            out_tri9[9 * i + 3 * k + 2] = v[k]->z;
        }
        out_mat[i] = tr._materialIndex;
        out_uv6[6 * i + 0] = tr._tex_coords_u.x;
        out_uv6[6 * i + 1] = tr._tex_coords_u.y;
        out_uv6[6 * i + 2] = tr._tex_coords_u.z;
        out_uv6[6 * i + 3] = tr._tex_coords_v.x;
        out_uv6[6 * i + 4] = tr._tex_coords_v.y;
        out_uv6[6 * i + 5] = tr._tex_coords_v.z;
    }
    int nm = data.materials.count();
    *out_nmat = nm;
    for (int m = 0; m < nm && m < mat_cap; m++) {
        const Material& mt = data.materials.materials[m];
        float* f = out_mats + ORC_MAT_STRIDE * m;
        f[ORC_MAT_AMBIENT] = mt.ambient_coeff.r; f[ORC_MAT_AMBIENT + 1] = mt.ambient_coeff.g; f[ORC_MAT_AMBIENT + 2] = mt.ambient_coeff.b;
        f[ORC_MAT_DIFFUSE] = mt.diffuse.r; f[ORC_MAT_DIFFUSE + 1] = mt.diffuse.g; f[ORC_MAT_DIFFUSE + 2] = mt.diffuse.b;
        f[ORC_MAT_SPECULAR] = mt.specular.r; f[ORC_MAT_SPECULAR + 1] = mt.specular.g; f[ORC_MAT_SPECULAR + 2] = mt.specular.b;
        f[ORC_MAT_EMISSION] = mt.emission.r; f[ORC_MAT_EMISSION + 1] = mt.emission.g; f[ORC_MAT_EMISSION + 2] = mt.emission.b;
        f[ORC_MAT_REFLECTION] = mt.reflection;
        f[ORC_MAT_ROUGHNESS] = mt.roughness;
        f[ORC_MAT_NS] = mt.ns;
        f[ORC_MAT_SPEC_THRESHOLD] = 0.0f;
    }
    return n;
}

/* MainWindow::precompute_materials (mainwindow.cpp:240-249) */
float ref_specular_threshold(float sr, float sg, float sb, float ns)
{
    float luminance = 0.2126f * sr + 0.7152f * sg + 0.0722 * sb;
    float tau = std::pow(Material::SPECULAR_THRESHOLD_EPSILON / luminance, 1 / ns);
    return tau;
}

/* One Triangle::intersect call (triangle.cpp:25-91). Returns 1 on hit. */
int ref_triangle_intersect(const float tri9[9], const float o[3], const float d[3], float out_tuv[3])
{
    Triangle tr(Point(tri9[0], tri9[1], tri9[2]), Point(tri9[3], tri9[4], tri9[5]), Point(tri9[6], tri9[7], tri9[8]));
    Ray r(Point(o[0], o[1], o[2]), Vector(d[0], d[1], d[2]));
    float t = 0, u = 0, v = 0;
    int hit = tr.intersect(r, t, u, v) ? 1 : 0;
    out_tuv[0] = t;
    out_tuv[1] = u;
    out_tuv[2] = v;
    return hit;
}

/* Closest-hit query BVH::intersect for arbitrary rays over a triangle soup.
 * out_id: triangle index of the final HitInfo (-1 if none), out_ret: BVH::intersect return value. */
void ref_bvh_query(const float* tri9, int64_t ntri, int max_depth, int leaf, const float* orig, const float* dir,
                   int64_t nrays, int32_t* out_id, float* out_t, float* out_u, float* out_v, uint8_t* out_ret)
{
    std::vector<Triangle> tris;
    tris.reserve(ntri);
    for (int64_t i = 0; i < ntri; i++) {
        const float* t = tri9 + 9 * i;
        tris.push_back(Triangle(Point(t[0], t[1], t[2]), Point(t[3], t[4], t[5]), Point(t[6], t[7], t[8])));
    }
    BVH bvh(&tris, max_depth, leaf);
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t i = 0; i < nrays; i++) {
        Ray r(Point(orig[3 * i], orig[3 * i + 1], orig[3 * i + 2]), Vector(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]));
        HitInfo hi;
        bool ret = bvh.intersect(r, hi);
        out_ret[i] = ret;
        out_id[i] = hi.triangle ? (int32_t)(hi.triangle - tris.data()) : -1;
        out_t[i] = hi.t;
        out_u[i] = hi.u;
        out_v[i] = hi.v;
    }
}

/* Renderer::ray_trace (renderer.cpp:1068-1116) over internal rows
 * [row_begin, row_begin + row_count), restated on reference primitives. */
static double g_last_render_seconds = 0.0;

/* Sequential RNG mode (see g_seq): on != 0 renders on one thread in the reference's pixel
 * order with XorShiftGenerator(seed); 0 returns to the path-keyed stream. */
void ref_set_rng_sequential(int on, uint32_t seed)
{
    g_seq = on != 0;
    g_seq_gen = XorShiftGenerator(seed);
}

/* Wall time of the last ref_render_rows pixel loop (the octree build excluded). */
double ref_last_render_seconds(void) { return g_last_render_seconds; }

/* the OpenMP team size of the row loops (the reference forks omp_get_max_threads(), i.e.
   OMP_NUM_THREADS or every CPU, renderer.cpp:1082); n <= 0 leaves it unchanged */
void ref_set_threads(int n)
{
    if (n > 0)
        omp_set_num_threads(n);
}

static int render_rows_strided(const orc_scene* sc, const orc_settings* st, int row_begin, int row_count,
                               int row_stride, orc_outputs* out, orc_counters* counters);

int ref_render_rows(const orc_scene* sc, const orc_settings* st, int row_begin, int row_count, orc_outputs* out,
                    orc_counters* counters)
{
    return render_rows_strided(sc, st, row_begin, row_count, 1, out, counters);
}

/* Internal rows row_begin + i * row_stride, i < row_count (a frame-wide sample for
 * CPU timing), written as consecutive output rows. */
int ref_render_row_sample(const orc_scene* sc, const orc_settings* st, int row_begin, int row_count, int row_stride,
                          orc_outputs* out, orc_counters* counters)
{
    return render_rows_strided(sc, st, row_begin, row_count, row_stride, out, counters);
}

static int render_rows_strided(const orc_scene* sc, const orc_settings* st, int row_begin, int row_count,
                               int row_stride, orc_outputs* out, orc_counters* counters)
{
    HScene H;
    build_scene(H, sc, st);
    int rw, rh;
    render_w_h(st, rw, rh);
    if (row_begin < 0 || row_count < 0 || row_stride < 1 ||
        (row_count > 0 && row_begin + (int64_t)(row_count - 1) * row_stride >= rh))
        return -1;
    orc_counters total = {};
    const double t_start = omp_get_wtime();
#pragma omp parallel if (!g_seq)
    {
        orc_counters local = {};
#pragma omp for schedule(dynamic)
        for (int row = 0; row < row_count; row++) {
            const int py = row_begin + row * row_stride;
            Tracer tr(H);
            float y_world = ((float)py + 0.5f) / rh * 2 - 1;
            for (int px = 0; px < rw; px++) {
                float x_world = ((float)px + 0.5f) / rw * 2 - 1;
                Point vs = H.proj_inv(Point(x_world, y_world, -1));
                Point ws = H.cam_to_world(vs);
                Point cp = H.cam_pos;
                Vector rd = normalize(ws - cp);
                Ray ray(cp, rd);
                bool found = false;
                HitInfo hi;
                tr.frame_key = h_pixel_seed((uint32_t)(py * rw + px), st->rng_seed);
                int src = -1;
                bool shadowed = false;
                local.primary_rays++;
                Color c = tr.trace_ray(ray, hi, 0, found, &src, &local, &shadowed);
                size_t o = (size_t)row * rw + px;
                if (out->argb) out->argb[o] = h_color_to_argb(c);
                if (out->rgba) {
                    out->rgba[4 * o] = c.r;
                    out->rgba[4 * o + 1] = c.g;
                    out->rgba[4 * o + 2] = c.b;
                    out->rgba[4 * o + 3] = c.a;
                }
                if (out->hit_id) out->hit_id[o] = found ? src : -1;
                if (out->hit_t) out->hit_t[o] = hi.t;
                if (out->shadow) out->shadow[o] = found && shadowed;
                // renderer.cpp:1104-1110 (buffers cleared before the render, mainwindow.cpp:184-185)
                if (out->zbuf) out->zbuf[o] = found ? -(ray._origin.z + ray._direction.z * hi.t) : INFINITY;
                if (out->nbuf) {
                    Vector nn = found ? hi.normal_at_intersection : Vector(0, 0, 0);
                    out->nbuf[3 * o] = nn.x;
                    out->nbuf[3 * o + 1] = nn.y;
                    out->nbuf[3 * o + 2] = nn.z;
                }
            }
        }
#pragma omp critical
        {
            total.primary_rays += local.primary_rays;
            total.shadow_rays += local.shadow_rays;
            total.reflection_rays += local.reflection_rays;
        }
    }
    g_last_render_seconds = omp_get_wtime() - t_start;
    if (counters) *counters = total;
    return 0;
}

/* Renderer::raster_trace (renderer.cpp:869-1006) on the reference's own vec4 /
 * Triangle4 / Transform / Triangle code.  The reference's OpenMP triangle loop
 * races on the z-buffer; the sequential result is defined here: triangles and
 * their clipped pieces in order, strict z-test, only the winner shaded (see
 * oracle.c).  hit_id = winning triangle (-1 background), hit_t = its z. */
namespace {

bool h_in_half(const vec4& p, int i, int sgn) { return sgn > 0 ? p(i) < p.w : p(i) > -p.w; }

// clip_triangles_to_plane<i, sgn> (renderer.cpp:669-850); in may alias out when n == 1
int h_clip_plane(const Triangle4* in, int n, Triangle4* out, int i, int sgn)
{
    const int CAP = 12;   // std::array<Triangle4, 12>: more pieces are UB in the reference and dropped here
    int k = 0;
    for (int t = 0; t < n; t++) {
        const Triangle4 T = in[t];
        bool ia = h_in_half(T._a, i, sgn), ib = h_in_half(T._b, i, sgn), ic = h_in_half(T._c, i, sgn);
        int cnt = (int)ia + (int)ib + (int)ic;
        if (cnt == 3) {
            if (k < CAP) out[k] = T;
            k++;
        } else if (cnt == 1) {
            const vec4& p0 = ia ? T._a : (ib ? T._b : T._c);
            const vec4& p1 = ia ? T._b : (ib ? T._c : T._a);
            const vec4& p2 = ia ? T._c : (ib ? T._a : T._b);
            float u[3] = {ia ? T._tex_coords_u.x : (ib ? T._tex_coords_u.y : T._tex_coords_u.z),
                          ia ? T._tex_coords_u.y : (ib ? T._tex_coords_u.z : T._tex_coords_u.x),
                          ia ? T._tex_coords_u.z : (ib ? T._tex_coords_u.x : T._tex_coords_u.y)};
            float v[3] = {ia ? T._tex_coords_v.x : (ib ? T._tex_coords_v.y : T._tex_coords_v.z),
                          ia ? T._tex_coords_v.y : (ib ? T._tex_coords_v.z : T._tex_coords_v.x),
                          ia ? T._tex_coords_v.z : (ib ? T._tex_coords_v.x : T._tex_coords_v.y)};
            float d0 = p0(i) - p0.w * sgn, d1 = p1(i) - p1.w * sgn, d2 = p2(i) - p2.w * sgn;
            float t1 = d1 / (d1 - d0), t2 = d2 / (d2 - d0);
            const float eps = 0;
            vec4 q1 = p1 + (t1 - eps) * (p0 - p1);
            vec4 q2 = p2 + (t2 - eps) * (p0 - p2);
            Point nu(u[0], u[1] + (t1 - eps) * (u[0] - u[1]), u[2] + (t2 - eps) * (u[0] - u[2]));
            Point nv(v[0], v[1] + (t1 - eps) * (v[0] - v[1]), v[2] + (t2 - eps) * (v[0] - v[2]));
            if (k < CAP) out[k] = Triangle4(p0, q1, q2, nu, nv);
            k++;
        } else if (cnt == 2) {
            const vec4& lost = !ia ? T._a : (!ib ? T._b : T._c);
            const vec4& k1 = !ia ? T._b : (!ib ? T._c : T._a);
            const vec4& k2 = !ia ? T._c : (!ib ? T._a : T._b);
            float u[3] = {!ia ? T._tex_coords_u.y : (!ib ? T._tex_coords_u.z : T._tex_coords_u.x),
                          !ia ? T._tex_coords_u.z : (!ib ? T._tex_coords_u.x : T._tex_coords_u.y),
                          !ia ? T._tex_coords_u.x : (!ib ? T._tex_coords_u.y : T._tex_coords_u.z)};
            float v[3] = {!ia ? T._tex_coords_v.y : (!ib ? T._tex_coords_v.z : T._tex_coords_v.x),
                          !ia ? T._tex_coords_v.z : (!ib ? T._tex_coords_v.x : T._tex_coords_v.y),
                          !ia ? T._tex_coords_v.x : (!ib ? T._tex_coords_v.y : T._tex_coords_v.z)};
            float e1 = k1(i) - k1.w * sgn, e2 = k2(i) - k2.w * sgn, e0 = lost(i) - lost.w * sgn;
            float t1 = e0 / (e0 - e1), t2 = e0 / (e0 - e2);
            const float eps = 0;
            vec4 P1 = lost + (t1 - eps) * (k1 - lost);
            vec4 P2 = lost + (t2 - eps) * (k2 - lost);
            Point u1(u[0], u[1], u[2] + (t2 - eps) * (u[1] - u[2]));
            Point v1(v[0], v[1], v[2] + (t2 - eps) * (v[1] - v[2]));
            Point u2(u[0], u[2] + (t2 - eps) * (u[1] - u[2]), u[2] + (t1 - eps) * (u[0] - u[2]));
            Point v2(v[0], v[2] + (t2 - eps) * (v[1] - v[2]), v[2] + (t1 - eps) * (v[0] - v[2]));
            Triangle4 A(k1, k2, P2, u1, v1), B(k1, P2, P1, u2, v2);
            if (k < CAP) out[k] = A;
            k++;
            if (k < CAP) out[k] = B;
            k++;
        }
    }
    return k < CAP ? k : CAP;
}

int h_d2i(double d)
{
    if (!(d > -2147483649.0 && d < 2147483648.0))
        return INT32_MIN;
    return (int)d;
}

// Renderer::matrix_transform_z, renderer.cpp:856-867
float h_matrix_z(const Transform& m, const Point& p)
{
    const float* d = m.data();
    float zt = d[8] * p.x + d[9] * p.y + d[10] * p.z + d[11];
    float wt = d[12] * p.x + d[13] * p.y + d[14] * p.z + d[15];
    if (wt == 1.0f)
        return zt;
    return zt / wt;
}

struct HPiece {
    int tri;
    Triangle ndc, cam, world;
    float inv_area;
    int x0, y0, x1, y1;
    float za, zb, zc;
};

}  // namespace

int ref_raster(const orc_scene* sc, const orc_settings* st, orc_outputs* out, orc_counters* counters)
{
    HScene H;
    build_scene(H, sc, st);
    int rw, rh;
    render_w_h(st, rw, rh);
    const size_t npx = (size_t)rw * rh;
    std::vector<float> zb(npx, INFINITY);
    std::vector<int64_t> win(npx, -1);
    std::vector<HPiece> pieces;
    const float hs = 1.0f / rh * 2, ws = 1.0f / rw * 2;
    for (size_t ti = 0; ti < H.tris.size(); ti++) {
        const Triangle& O = H.tris[ti];
        Triangle tc = H.world_to_cam(O);
        Triangle4 A[12], B[12];
        A[0] = Triangle4(H.proj(vec4(tc._a)), H.proj(vec4(tc._b)), H.proj(vec4(tc._c)), tc._tex_coords_u,
                         tc._tex_coords_v);
        int n = 1;
        const Triangle4* res = A;
        if (st->enable_clipping) {
            n = h_clip_plane(A, n, A, 0, 1);
            n = h_clip_plane(A, n, B, 0, -1);
            n = h_clip_plane(B, n, A, 1, 1);
            n = h_clip_plane(A, n, B, 1, -1);
            n = h_clip_plane(B, n, A, 2, 1);
            n = h_clip_plane(A, n, B, 2, -1);
            res = B;
        }
        for (int k = 0; k < n; k++) {
            HPiece P;
            P.tri = (int)ti;
            P.ndc = Triangle(res[k], O._materialIndex, res[k]._tex_coords_u, res[k]._tex_coords_v);
            P.cam = H.proj_inv(P.ndc);
            P.world = H.cam_to_world(P.cam);
            const Point &a = P.ndc._a, &b = P.ndc._b, &c = P.ndc._c;
            P.inv_area = 1 / ((b.x - a.x) * (c.y - a.y) - (b.y - a.y) * (c.x - a.x));
            float mnx = std::min(a.x, std::min(b.x, c.x)), mny = std::min(a.y, std::min(b.y, c.y));
            float mxx = std::max(a.x, std::max(b.x, c.x)), mxy = std::max(a.y, std::max(b.y, c.y));
            P.x0 = std::max(h_d2i((mnx + 1) * 0.5 * rw), 0);
            P.y0 = std::max(h_d2i((mny + 1) * 0.5 * rh), 0);
            P.x1 = std::min(rw - 1, h_d2i((mxx + 1) * 0.5 * rw));
            P.y1 = std::min(rh - 1, h_d2i((mxy + 1) * 0.5 * rh));
            P.za = h_matrix_z(H.cam_to_world, H.proj_inv(a));
            P.zb = h_matrix_z(H.cam_to_world, H.proj_inv(b));
            P.zc = h_matrix_z(H.cam_to_world, H.proj_inv(c));
            float iy = P.y0 * hs - 1;
            for (int py = P.y0; py <= P.y1; py++, iy += hs) {
                float ix = P.x0 * ws - 1;
                for (int px = P.x0; px <= P.x1; px++, ix += ws) {
                    Point s(ix + ws * 0.5f, iy + hs * 0.5f, -1);
                    float u = Triangle::edge_function(s, c, a);
                    if (u < 0) continue;
                    float v = Triangle::edge_function(s, a, b);
                    if (v < 0) continue;
                    float w = Triangle::edge_function(s, b, c);
                    if (w < 0) continue;
                    u *= P.inv_area;
                    v *= P.inv_area;
                    w *= P.inv_area;
                    float z = -1 / (1 / P.za * w + 1 / P.zb * u + 1 / P.zc * v);
                    size_t o = (size_t)py * rw + px;
                    if (z < zb[o]) {
                        zb[o] = z;
                        win[o] = (int64_t)pieces.size();
                    }
                }
            }
            pieces.push_back(P);
        }
    }
    orc_counters total = {};
#pragma omp parallel
    {
        orc_counters local = {};
        Tracer tr(H);
#pragma omp for schedule(dynamic)
        for (int py = 0; py < rh; py++) {
            for (int px = 0; px < rw; px++) {
                size_t o = (size_t)py * rw + px;
                Color c = H_BACKGROUND_COLOR;
                bool sh = false;
                int64_t wi = win[o];
                if (wi >= 0) {
                    const HPiece& P = pieces[(size_t)wi];
                    float iy = P.y0 * hs - 1;
                    for (int y = P.y0; y < py; y++) iy += hs;
                    float ix = P.x0 * ws - 1;
                    for (int x = P.x0; x < px; x++) ix += ws;
                    Point s(ix + ws * 0.5f, iy + hs * 0.5f, -1);
                    const Point &a = P.ndc._a, &b = P.ndc._b, &cc = P.ndc._c;
                    float u = Triangle::edge_function(s, cc, a) * P.inv_area;
                    float v = Triangle::edge_function(s, a, b) * P.inv_area;
                    const Triangle& O = H.tris[(size_t)P.tri];
                    int sm = st->shading_method;
                    if (sm == ORC_RT_SHADING) {
                        // trace_triangle (renderer.cpp:619-628)
                        Ray ray(H.cam_pos, normalize(H.cam_to_world(H.proj_inv(s)) - H.cam_pos));
                        HitInfo hi;
                        c = Color(0, 0, 0);
                        if (P.world.intersect(ray, hi)) {
                            tr.frame_key = h_pixel_seed((uint32_t)(py * rw + px), st->rng_seed);
                            local.primary_rays++;
                            c = tr.shade(ray, hi, 0, &sh, &local);
                        }
                    } else if (sm == ORC_ABS_NORMALS_SHADING) {
                        Vector n = normalize(O._normal);
                        c = Color(std::abs(n.x), std::abs(n.y), std::abs(n.z));
                    } else if (sm == ORC_PASTEL_NORMALS_SHADING) {
                        Vector n = normalize(O._normal);
                        c = (Color(n.x, n.y, n.z) + Color(1.0f, 1.0f, 1.0f)) * 0.5;
                    } else if (sm == ORC_BARYCENTRIC_COORDINATES_SHADING) {
                        c = Color(1, 0, 0) * u + Color(0, 1.0, 0) * v + Color(0, 0, 1) * (1 - u - v);
                    } else if (sm == ORC_VISUALIZE_AO) {
                        c = Color(0.9f, 0.9f, 0.9f);
                        if (st->enable_ao_mapping) {
                            float tu, tv;
                            P.cam.interpolate_texcoords(u, v, tu, tv);
                            c = c * Color(tr.sample_texture(H.tex[ORC_TEX_AO], tu, tv).r);
                        }
                    }
                }
                if (out->argb) out->argb[o] = h_color_to_argb(c);
                if (out->rgba) {
                    out->rgba[4 * o] = c.r;
                    out->rgba[4 * o + 1] = c.g;
                    out->rgba[4 * o + 2] = c.b;
                    out->rgba[4 * o + 3] = 1.0f;
                }
                if (out->hit_id) out->hit_id[o] = wi >= 0 ? pieces[(size_t)wi].tri : -1;
                if (out->hit_t) out->hit_t[o] = zb[o];
                if (out->shadow) out->shadow[o] = (uint8_t)sh;
                // renderer.cpp:975-979: _z_buffer and _normal_buffer = original_triangle._normal
                if (out->zbuf) out->zbuf[o] = zb[o];
                if (out->nbuf) {
                    Vector nn = wi >= 0 ? H.tris[(size_t)pieces[(size_t)wi].tri]._normal : Vector(0, 0, 0);
                    out->nbuf[3 * o] = nn.x;
                    out->nbuf[3 * o + 1] = nn.y;
                    out->nbuf[3 * o + 2] = nn.z;
                }
            }
        }
#pragma omp critical
        {
            total.primary_rays += local.primary_rays;
            total.shadow_rays += local.shadow_rays;
            total.reflection_rays += local.reflection_rays;
        }
    }
    if (counters) *counters = total;
    return 0;
}

/* Pop order of the reference's per-node queue type (bvh.h:110-123, 250):
 * std::priority_queue<QueueElement, std::vector<QueueElement>, std::greater<QueueElement>>
 * filled with n elements in index order. */
void ref_heap_order(const float* keys, int n, int32_t* out_order)
{
    std::vector<BVH::OctreeNode> dummies;
    dummies.reserve(n);
    for (int i = 0; i < n; i++)
        dummies.emplace_back(Point(0, 0, 0), Point(0, 0, 0));
    std::priority_queue<BVH::OctreeNode::QueueElement, std::vector<BVH::OctreeNode::QueueElement>,
                        std::greater<BVH::OctreeNode::QueueElement>>
        q;
    for (int i = 0; i < n; i++)
        q.emplace(BVH::OctreeNode::QueueElement(&dummies[i], keys[i]));
    for (int i = 0; i < n; i++) {
        out_order[i] = (int32_t)(q.top()._node - dummies.data());
        q.pop();
    }
}

/* ImageUtils::downscale_image_qt_ARGB32 (imageUtils.h:98-147) */
int ref_downscale_argb(const uint32_t* in, int w, int h, int factor, uint32_t* out)
{
    if (w % factor != 0 || h % factor != 0)
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
            ar = ar / (factor * factor);
            ag = ag / (factor * factor);
            ab = ab / (factor * factor);
            out[(size_t)y * dw + x] = h_qrgb(ar, ag, ab);
        }
    return 0;
}

}  // extern "C"
