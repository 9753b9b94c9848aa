// capi.cpp -- extern "C" boundary (include/rt_mi355x.h).  No exception crosses it.
#include <atomic>
#include <chrono>
#include <cmath>
#include <thread>
#include <cstring>
#include <new>
#include <string>

#include "../../include/rt_mi355x_diag.h"   // (includes rt_mi355x.h)
#include "host_scene.hpp"
#include "octree.hpp"
#include "ocone.hpp"
#include "wbvh.hpp"
#include "renderer.hpp"

namespace {
thread_local std::string g_err;

int record(rt::Renderer* r, int rc)
{
    if (rc != RT_OK)
        g_err = r->error();
    return rc;
}

int bad(const char* msg)
{
    g_err = msg;
    return RT_EINVAL;
}

template <class F>
int guarded(rt::Renderer* r, F&& f)
{
    if (!r)
        return bad("null renderer handle");
    try {
        return record(r, f());
    } catch (const std::bad_alloc&) {
        g_err = "out of host memory";
        return RT_ENOMEM;
    } catch (const std::exception& e) {
        g_err = e.what();
        return RT_EINVAL;
    }
}

rt::Renderer* R(rt_renderer* r) { return reinterpret_cast<rt::Renderer*>(r); }
}  // namespace

extern "C" {

void rt_default_settings(rt_settings* s)
{
    std::memset(s, 0, sizeof(*s));
    s->image_width = 1024;
    s->image_height = 1024;
    s->enable_ssaa = 0;
    s->ssaa_factor = 2;
    s->enable_clipping = 1;
    s->hybrid_rasterization_tracing = 0;
    s->shading_method = RT_SHADING_RT;
    s->compute_shadows = 0;
    s->max_recursion_depth = 5;
    s->enable_bvh = 1;
    s->bvh_max_depth = 12;
    s->bvh_leaf_object_count = 40;
    s->enable_ssao = 0;
    s->ssao_sample_count = 64;
    s->ssao_radius = 0.5f;
    s->ssao_amount = 1.0f;
    s->enable_ambient = 1;
    s->enable_diffuse = 1;
    s->enable_specular = 1;
    s->enable_emissive = 1;
    s->rough_reflections_sample_count = 3;
    s->displacement_mapping_strength = 0.02f;
    s->parallax_mapping_steps = 32;
    s->rng_seed = 0x5EED1234u;
}

rt_renderer* rt_create(int device)
{
    try {
        rt::Renderer* r = new rt::Renderer(device);
        std::string err;
        if (r->init(err) != RT_OK) {
            g_err = err;
            delete r;
            return nullptr;
        }
        return reinterpret_cast<rt_renderer*>(r);
    } catch (const std::exception& e) {
        g_err = e.what();
        return nullptr;
    }
}

void rt_destroy(rt_renderer* r) { delete R(r); }

const char* rt_last_error(void) { return g_err.c_str(); }

int rt_get_settings(rt_renderer* r, rt_settings* out)
{
    return guarded(R(r), [&] {
        *out = R(r)->render_settings();
        return RT_OK;
    });
}
int rt_set_settings(rt_renderer* r, const rt_settings* s)
{
    return guarded(R(r), [&] { return s ? R(r)->set_settings(*s) : RT_EINVAL; });
}
int rt_set_devices(rt_renderer* r, const int32_t* ids, int32_t n)
{
    return guarded(R(r), [&] { return R(r)->set_devices(ids, n); });
}
int rt_finish_accel(rt_renderer* r)
{
    return guarded(R(r), [&] { return R(r)->finish_accel(); });
}
int rt_set_exact(rt_renderer* r, int on)
{
    return guarded(R(r), [&] { return R(r)->set_exact(on != 0); });
}
int rt_change_render_size(rt_renderer* r, int32_t w, int32_t h)
{
    return guarded(R(r), [&] { return R(r)->change_render_size(w, h); });
}
int rt_set_triangles(rt_renderer* r, const float* tri9, const int32_t* mat, const float* uv6, int64_t n)
{
    return guarded(R(r), [&] { return R(r)->set_triangles(tri9, mat, uv6, n); });
}
int rt_add_sphere(rt_renderer* r, float cx, float cy, float cz, float radius, int32_t mat)
{
    return guarded(R(r), [&] { return R(r)->add_sphere(cx, cy, cz, radius, mat); });
}
int rt_add_plane(rt_renderer* r, float px, float py, float pz, float nx, float ny, float nz, int32_t mat)
{
    return guarded(R(r), [&] { return R(r)->add_plane(px, py, pz, nx, ny, nz, mat); });
}
int rt_clear_geometry(rt_renderer* r)
{
    return guarded(R(r), [&] { return R(r)->clear_geometry(); });
}
int rt_set_materials(rt_renderer* r, const float* mats16, int32_t n)
{
    return guarded(R(r), [&] { return R(r)->set_materials(mats16, n); });
}
int rt_get_material_count(rt_renderer* r, int32_t* n)
{
    return guarded(R(r), [&] {
        *n = R(r)->material_count();
        return RT_OK;
    });
}
int rt_change_camera_fov(rt_renderer* r, float fov)
{
    return guarded(R(r), [&] { return R(r)->change_camera_fov(fov); });
}
int rt_change_camera_aspect_ratio(rt_renderer* r, float aspect)
{
    return guarded(R(r), [&] { return R(r)->change_camera_aspect_ratio(aspect); });
}
int rt_set_light_position(rt_renderer* r, float x, float y, float z)
{
    return guarded(R(r), [&] { return R(r)->set_light_position(x, y, z); });
}
int rt_set_camera_transform(rt_renderer* r, const float m[16])
{
    return guarded(R(r), [&] { return m ? R(r)->set_camera_transform(m) : RT_EINVAL; });
}
int rt_apply_transformation_to_camera(rt_renderer* r, const float m[16])
{
    return guarded(R(r), [&] { return m ? R(r)->apply_transformation_to_camera(m) : RT_EINVAL; });
}
int rt_set_camera_matrices(rt_renderer* r, const float pos[3], const float proj_inv[16], const float c2w[16])
{
    return guarded(R(r), [&] { return (pos && proj_inv && c2w) ? R(r)->set_camera_matrices(pos, proj_inv, c2w) : RT_EINVAL; });
}
int rt_set_camera_projection(rt_renderer* r, const float proj[16], const float w2c[16])
{
    return guarded(R(r), [&] { return (proj && w2c) ? R(r)->set_camera_projection(proj, w2c) : RT_EINVAL; });
}
int rt_get_ssao_buffers(rt_renderer* r, float* z, float* n4, int32_t* ao)
{
    return guarded(R(r), [&] { return R(r)->get_ssao_buffers(z, n4, ao); });
}
int rt_set_camera_lens(rt_renderer* r, float fov, float aspect)
{
    return guarded(R(r), [&] { return R(r)->set_camera_lens(fov, aspect); });
}
int rt_get_camera_matrices(rt_renderer* r, float pos[3], float proj_inv[16], float c2w[16])
{
    return guarded(R(r), [&] {
        R(r)->get_camera_matrices(pos, proj_inv, c2w);
        return RT_OK;
    });
}
int rt_set_object_transform(rt_renderer* r, const float m[16])
{
    return guarded(R(r), [&] { return m ? R(r)->set_object_transform(m) : RT_EINVAL; });
}
int rt_reset_previous_transform(rt_renderer* r)
{
    return guarded(R(r), [&] { return R(r)->reset_previous_transform(); });
}
int rt_set_texture(rt_renderer* r, int32_t slot, int32_t w, int32_t h, const float* rgba)
{
    return guarded(R(r), [&] { return R(r)->set_texture(slot, w, h, rgba); });
}
int rt_set_skybox(rt_renderer* r, const int32_t w[6], const int32_t h[6], const float* const faces[6])
{
    return guarded(R(r), [&] { return R(r)->set_skybox(w, h, faces); });
}
int rt_reconstruct_bvh_new(rt_renderer* r)
{
    return guarded(R(r), [&] { return R(r)->reconstruct_bvh_new(); });
}
int rt_destroy_bvh(rt_renderer* r)
{
    return guarded(R(r), [&] { return R(r)->destroy_bvh(); });
}
int rt_ray_trace(rt_renderer* r)
{
    return guarded(R(r), [&] { return R(r)->ray_trace(); });
}
int rt_raster_trace(rt_renderer* r)
{
    return guarded(R(r), [&] { return R(r)->raster_trace(); });
}
int rt_post_process(rt_renderer* r)
{
    return guarded(R(r), [&] { return R(r)->post_process(); });
}
// rt_get_image / rt_lock_image / rt_unlock_image may run on a display thread while the owning
// thread renders: they touch only the image state (under the image mutex), never err_
int rt_get_image(rt_renderer* r, uint32_t* argb, int32_t* w, int32_t* h)
{
    if (!r)
        return bad("null renderer handle");
    try {
        int rc = R(r)->get_image(argb, w, h);
        if (rc != RT_OK)
            g_err = R(r)->display_error();
        return rc;
    } catch (const std::exception& e) {
        g_err = e.what();
        return RT_EINVAL;
    }
}
int rt_lock_image(rt_renderer* r)
{
    if (!r)
        return bad("null renderer handle");
    R(r)->lock_image();
    return RT_OK;
}
int rt_unlock_image(rt_renderer* r)
{
    if (!r)
        return bad("null renderer handle");
    R(r)->unlock_image();
    return RT_OK;
}
int rt_render(rt_renderer* r, float* ms)
{
    return guarded(R(r), [&] {
        int rc = RT_OK;
        float t = rt::render(*R(r), &rc);
        if (ms)
            *ms = t;
        return rc;
    });
}
int rt_request_aux(rt_renderer* r, int32_t want_rgba, int32_t want_hit, int32_t want_shadow)
{
    return guarded(R(r), [&] { return R(r)->request_aux(want_rgba != 0, want_hit != 0, want_shadow != 0); });
}
int rt_get_internal(rt_renderer* r, uint32_t* argb, float* rgba, int32_t* hit_id, float* hit_t, uint8_t* shadow)
{
    return guarded(R(r), [&] { return R(r)->get_internal(argb, rgba, hit_id, hit_t, shadow); });
}
int rt_get_stats(rt_renderer* r, rt_stats* out)
{
    return guarded(R(r), [&] { return out ? R(r)->get_stats(out) : RT_EINVAL; });
}
int rt_debug_read(rt_renderer* r, uint64_t* out, int64_t n)
{
    return guarded(R(r), [&] { return out ? R(r)->debug_read(out, n) : RT_EINVAL; });
}
int rt_tile_costs(rt_renderer* r, uint32_t* out, int64_t n, int32_t* tiles_x, int32_t* tiles_y)
{
    return guarded(R(r), [&] { return tiles_x && tiles_y ? R(r)->tile_costs(out, n, tiles_x, tiles_y) : RT_EINVAL; });
}
int rt_ocone_read(rt_renderer* r, uint32_t* out, int64_t n, int32_t dims[3], float lo_ih[4])
{
    return guarded(R(r), [&] { return dims && lo_ih ? R(r)->origin_cones(out, n, dims, lo_ih) : RT_EINVAL; });
}
int rt_local_rows(rt_renderer* r, int32_t band_rows, int32_t rank, int32_t nranks, int32_t* rows_out)
{
    return guarded(R(r), [&] {
        int n = R(r)->local_rows(band_rows, rank, nranks);
        if (n < 0)
            return bad("bad band layout");
        *rows_out = n;
        return RT_OK;
    });
}
int rt_render_bands_device(rt_renderer* r, int32_t band_rows, int32_t rank, int32_t nranks, uint32_t* d_out,
                           void* hip_stream)
{
    return guarded(R(r), [&] {
        return R(r)->render_bands_device(band_rows, rank, nranks, d_out, reinterpret_cast<hipStream_t>(hip_stream));
    });
}

int rt_render_band_list_device(rt_renderer* r, int32_t band_rows, const int32_t* bands, int32_t nbands, uint32_t* d_out,
                               void* hip_stream)
{
    return guarded(R(r), [&] {
        return R(r)->render_band_list_device(band_rows, bands, nbands, d_out, reinterpret_cast<hipStream_t>(hip_stream));
    });
}
int rt_band_costs(rt_renderer* r, void* hip_stream, double* costs, int32_t nbands)
{
    return guarded(R(r), [&] { return R(r)->band_costs(reinterpret_cast<hipStream_t>(hip_stream), costs, nbands); });
}

int rt_trace_rays(rt_renderer* r, const float* orig, const float* dir, int64_t n, int32_t* tri_id, float* t,
                  float* u, float* v, uint8_t* ret)
{
    return guarded(R(r), [&] { return R(r)->trace_rays(orig, dir, n, tri_id, t, u, v, ret); });
}
int rt_wide_query(rt_renderer* r, const float* orig, const float* dir, int64_t n, int32_t kind, float* o_out,
                  float* d_out, int32_t* status, int32_t* tri_id, float* t, float* u, float* v, uint8_t* shadowed)
{
    return guarded(R(r), [&] { return R(r)->wide_query(orig, dir, n, kind, o_out, d_out, status, tri_id, t, u, v, shadowed); });
}
int rt_risk_words(rt_renderer* r, int32_t src, uint64_t* out, int64_t cap, int64_t* count, int64_t* violations)
{
    return guarded(R(r), [&] { return R(r)->risk_words(src, out, cap, count, violations); });
}
int rt_trace_ray(rt_renderer* r, const float* orig, const float* dir, int64_t n, int32_t current_recursion_depth,
                 float* rgba, int32_t* hit_src, float* t, uint8_t* intersection_found, uint8_t* shadowed)
{
    return guarded(R(r), [&] {
        return R(r)->trace_ray_colors(orig, dir, n, current_recursion_depth, rgba, hit_src, t, intersection_found,
                                      shadowed);
    });
}
int rt_kernel_times(rt_renderer* r, float* ms, int32_t n)
{
    return guarded(R(r), [&] { return ms ? R(r)->kernel_times(ms, n) : RT_EINVAL; });
}
int rt_band_counters(rt_renderer* r, int64_t* shadow_rays, int64_t* reflection_rays)
{
    return guarded(R(r), [&] {
        unsigned long long c[2] = {0, 0};
        int rc = R(r)->band_counters(c);
        if (shadow_rays) *shadow_rays = (int64_t)c[0];
        if (reflection_rays) *reflection_rays = (int64_t)c[1];
        return rc;
    });
}

void rt_make_transform(int32_t kind, float x, float y, float z, float out[16])
{
    switch (kind) {
    case 0: rt::mat::translation(x, y, z, out); break;
    case 1: rt::mat::rotation_x(x, out); break;
    case 2: rt::mat::rotation_y(x, out); break;
    case 3: rt::mat::rotation_z(x, out); break;
    case 4: rt::mat::scale(x, y, z, out); break;
    default: rt::mat::identity(out); break;
    }
}
void rt_compose(const float a[16], const float b[16], float out[16]) { rt::mat::compose(a, b, out); }
void rt_inverse(const float m[16], float out[16]) { rt::mat::inverse(m, out); }
void rt_perspective(float fov, float aspect, float znear, float zfar, float out[16])
{
    rt::mat::perspective(fov, aspect, znear, zfar, out);
}
void rt_transform_points(const float m[16], const float* pts, int64_t n, float* out)
{
    rt::mat::transform_points(m, pts, n, out);
}

struct rt_obj {
    rt::ObjData data;
};

rt_obj* rt_obj_open(const char* path, const float xform[16], int32_t mat_offset)
{
    try {
        float ident[16];
        rt::mat::identity(ident);
        rt_obj* o = new rt_obj;
        std::string err;
        if (!rt::load_obj(path, xform ? xform : ident, mat_offset, o->data, err)) {
            g_err = err;
            delete o;
            return nullptr;
        }
        return o;
    } catch (const std::exception& e) {
        g_err = e.what();
        return nullptr;
    }
}

int rt_obj_counts(const rt_obj* o, int64_t* ntri, int32_t* nmat, int32_t* has_uv)
{
    if (!o)
        return bad("null obj");
    if (ntri) *ntri = (int64_t)o->data.mat.size();
    if (nmat) *nmat = (int32_t)o->data.materials.size();
    if (has_uv) *has_uv = o->data.has_uv;
    return RT_OK;
}

int rt_obj_fetch(const rt_obj* o, float* tri9, int32_t* mat, float* uv6, float* mats16)
{
    if (!o)
        return bad("null obj");
    const rt::ObjData& d = o->data;
    if (tri9) std::memcpy(tri9, d.tri.data(), d.tri.size() * 4);
    if (mat) std::memcpy(mat, d.mat.data(), d.mat.size() * 4);
    if (uv6 && d.has_uv) std::memcpy(uv6, d.uv.data(), d.uv.size() * 4);
    if (mats16) {
        for (size_t i = 0; i < d.materials.size(); i++) {
            const rt::ObjMaterial& m = d.materials[i];
            float* f = mats16 + 16 * i;
            for (int c = 0; c < 3; c++) {
                f[0 + c] = m.ambient[c];
                f[3 + c] = m.diffuse[c];
                f[6 + c] = m.specular[c];
                f[9 + c] = m.emission[c];
            }
            f[12] = m.reflection;
            f[13] = m.roughness;
            f[14] = m.ns;
            f[15] = 0.0f;   // specular_threshold: set by the caller (MainWindow::precompute_materials)
        }
    }
    return RT_OK;
}

void rt_obj_close(rt_obj* o) { delete o; }

// For a ray that skips case (b): how many triangles nearly parallel to it (|cos(N, d)| < W_QS_CLOSEST, N
// = ab x ac exact, per-triangle N and |N| in Nn) or degenerate (no finite q) Moller-Trumbore reports a hit
// from (mt_record, the reference's expressions); grazing counts the first kind tested
static int64_t grazing_reports(const std::vector<rt::GTri>& tris, const std::vector<double>& Nn, rt::v3 o, rt::v3 d,
                               int64_t& grazing)
{
    int64_t viol = 0;
    const double dl = std::sqrt((double)d.x * d.x + (double)d.y * d.y + (double)d.z * d.z);
    for (size_t k = 0; k < tris.size(); k++) {
        const double* N = &Nn[4 * k];
        const double q = std::fabs(N[0] * d.x + N[1] * d.y + N[2] * d.z) / (N[3] * dl);
        if (q == q && !(q < W_QS_CLOSEST))
            continue;   // (a)'s
        grazing += q == q;
        float tt, uu, vv;
        if (rt::mt_record(tris[k], o, d, tt, uu, vv))
            ++viol;
    }
    return viol;
}

static std::vector<double> exact_normals(const std::vector<rt::GTri>& tris)
{
    std::vector<double> Nn(tris.size() * 4);
    for (size_t k = 0; k < tris.size(); k++) {
        const rt::GTri& t = tris[k];
        const double x0 = t.ab[0], x1 = t.ab[1], x2 = t.ab[2], y0 = t.ac[0], y1 = t.ac[1], y2 = t.ac[2];
        Nn[4 * k] = x1 * y2 - x2 * y1;
        Nn[4 * k + 1] = x2 * y0 - x0 * y2;
        Nn[4 * k + 2] = x0 * y1 - x1 * y0;
        Nn[4 * k + 3] = std::sqrt(Nn[4 * k] * Nn[4 * k] + Nn[4 * k + 1] * Nn[4 * k + 1] + Nn[4 * k + 2] * Nn[4 * k + 2]);
    }
    return Nn;
}

// The camera's risk cap by brute force (CPU tests): rays from cam; for each that risk_cap_skip lets skip case
// (b) (the cap as renderer.cpp prepare_risk computes it, or cap_override >= 0), every triangle nearly parallel
// to it goes through Moller-Trumbore.  out[4] = {violations, rays skipping, grazing tests, the cap x 1e9}.
int rt_risk_cap_check(const float* tri9, int64_t n, int32_t max_depth, int32_t leaf_max_obj_count, const float* cam,
                      const float* dir, int64_t nrays, float cap_override, int32_t* skip, int64_t out[4])
{
    if (n <= 0 || !tri9 || !cam || nrays < 0 || (nrays > 0 && !dir) || !out)
        return bad("rt_risk_cap_check: bad arguments");
    try {
        rt::FlatOctree f;
        rt::WBvh w;
        rt::build_flat_octree(tri9, n, max_depth, leaf_max_obj_count, f);
        rt::build_wbvh(f, w);
        if (f.nodes.empty())
            return bad("rt_risk_cap_check: no octree");
        float S = 0.0f;
        for (int a = 0; a < 3; a++)
            S = std::max(S, std::max(std::fabs(f.nodes[0].dn[a]), std::fabs(f.nodes[0].df[a])));
        const float lo[3] = {f.nodes[0].dn[0], f.nodes[0].dn[1], f.nodes[0].dn[2]};
        const float hi[3] = {f.nodes[0].df[0], f.nodes[0].df[1], f.nodes[0].df[2]};
        const float zero[3] = {0, 0, 0};
        const rt::WRiskArgs RA = rt::wbvh_risk_args(lo, hi, S, cam, zero, W_QS_CLOSEST, W_QS_SHADOW);
        float cdir[3];
        double v[3], l = 0;
        for (int a = 0; a < 3; a++) {
            v[a] = 0.5 * ((double)lo[a] + (double)hi[a]) - (double)cam[a];
            l += v[a] * v[a];
        }
        l = std::sqrt(l);
        for (int a = 0; a < 3; a++)
            cdir[a] = l > 0 && l < INFINITY ? (float)(v[a] / l) : (a == 0 ? 1.0f : 0.0f);
        const double c[3] = {cdir[0], cdir[1], cdir[2]};
        float cap = INFINITY;
        for (const rt::GTri& t : w.tris)
            if (rt::wbvh_risk_key(t, RA.p[0][0], RA.p[0][1], RA.p[0][2], RA.G[0], RA.nu[0], RA.slack[0], RA.QS[0]) < INFINITY)
                cap = std::min(cap, rt::risk_cap_tri(t, c));
        if (cap_override >= 0.0f)
            cap = cap_override;
        const std::vector<double> Nn = exact_normals(w.tris);
        std::atomic<int64_t> nskip{0}, nviol{0}, ngraze{0};
        const rt::v3 o = rt::mk(cam[0], cam[1], cam[2]);
        auto body = [&](int64_t b, int64_t e) {
            for (int64_t i = b; i < e; i++) {
                const rt::v3 d = rt::mk(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]);
                const bool sk = RA.on[0] && rt::risk_cap_skip(cap, cdir, d, W_QS_CLOSEST);
                if (skip)
                    skip[i] = sk ? 1 : 0;
                if (!sk)
                    continue;
                ++nskip;
                int64_t g = 0;
                nviol += grazing_reports(w.tris, Nn, o, d, g);
                ngraze += g;
            }
        };
        unsigned hc = std::max(1u, std::min(std::thread::hardware_concurrency(), 16u));
        std::vector<std::thread> th;
        int64_t chunk = (nrays + hc - 1) / hc;
        for (unsigned k = 0; k < hc; k++) {
            int64_t b = (int64_t)k * chunk, e = std::min(nrays, b + chunk);
            if (b < e)
                th.emplace_back(body, b, e);
        }
        for (auto& x : th)
            x.join();
        out[0] = nviol.load();
        out[1] = nskip.load();
        out[2] = ngraze.load();
        out[3] = (int64_t)(cap < INFINITY ? (double)cap * 1e9 : -1);
        return RT_OK;
    } catch (const std::bad_alloc&) {
        g_err = "rt_risk_cap_check: out of host memory";
        return RT_ENOMEM;
    }
}

// The origin cones' soundness by brute force (CPU tests): for each ray (o, d) that ocone_skip lets
// skip case (b), every triangle with q = |cos(N, d)| < W_QS_CLOSEST (N = ab x ac exact) is run through
// Moller-Trumbore (mt_record, the reference's expressions): a reported hit is a violation.
int rt_ocone_check(const float* tri9, int64_t n, int32_t max_depth, int32_t leaf_max_obj_count, int32_t ocone_dim,
                   const float* orig, const float* dir, int64_t nrays, int32_t* skip, int64_t out[6],
                   const uint32_t* cells, const int32_t* dims, const float* lo_ih, uint32_t* cells_out)
{
    if (n <= 0 || !tri9 || nrays < 0 || (nrays > 0 && (!orig || !dir)) || ocone_dim <= 0 || !out)
        return bad("rt_ocone_check: bad arguments");
    try {
        rt::FlatOctree f;
        rt::WBvh w;
        rt::build_flat_octree(tri9, n, max_depth, leaf_max_obj_count, f);
        rt::build_wbvh(f, w);
        float S = 0.0f;
        if (!f.nodes.empty())
            for (int a = 0; a < 3; a++)
                S = std::max(S, std::max(std::fabs(f.nodes[0].dn[a]), std::fabs(f.nodes[0].df[a])));
        rt::OConeGrid g;
        if (cells && dims && lo_ih) {   // a given grid (a renderer's, rt_ocone_read)
            for (int a = 0; a < 3; a++) {
                g.dim[a] = dims[a];
                g.lo[a] = lo_ih[a];
            }
            g.ih = lo_ih[3];
            const size_t nc = (size_t)dims[0] * dims[1] * dims[2];
            g.cells.resize(nc);
            std::memcpy(g.cells.data(), cells, nc * sizeof(uint2));
            g.computed = (int64_t)nc;
            rt::origin_cones_count(g);
        } else {
            rt::build_origin_cones(w, S, W_QS_CLOSEST, 0.0102 + 0x1p-16 * S, ocone_dim, 80.0 * 3.14159265358979 / 180.0, 0, g);
            if (cells_out && !g.cells.empty())
                std::memcpy(cells_out, g.cells.data(), g.cells.size() * sizeof(uint2));
        }
        rt::OConeView v{};
        if (!g.cells.empty()) {
            v.cells = g.cells.data();
            for (int a = 0; a < 3; a++) {
                v.lo[a] = g.lo[a];
                v.dim[a] = g.dim[a];
            }
            v.ih = g.ih;
        }
        const std::vector<double> Nn = exact_normals(w.tris);
        std::atomic<int64_t> nskip{0}, nviol{0}, ngraze{0};
        auto body = [&](int64_t b, int64_t e) {
            for (int64_t i = b; i < e; i++) {
                const rt::v3 o = rt::mk(orig[3 * i], orig[3 * i + 1], orig[3 * i + 2]);
                const rt::v3 d = rt::mk(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]);
                const bool sk = rt::ocone_skip(v, o, d, W_QS_CLOSEST);
                if (skip)
                    skip[i] = sk ? 1 : 0;
                if (!sk)
                    continue;
                ++nskip;
                int64_t g = 0;
                nviol += grazing_reports(w.tris, Nn, o, d, g);
                ngraze += g;
            }
        };
        unsigned hc = std::max(1u, std::min(std::thread::hardware_concurrency(), 16u));
        std::vector<std::thread> th;
        int64_t chunk = (nrays + hc - 1) / hc;
        for (unsigned k = 0; k < hc; k++) {
            int64_t b = (int64_t)k * chunk, e = std::min(nrays, b + chunk);
            if (b < e)
                th.emplace_back(body, b, e);
        }
        for (auto& x : th)
            x.join();
        out[0] = nviol.load();
        out[1] = nskip.load();
        out[2] = ngraze.load();
        out[3] = g.computed;
        out[4] = g.empty;
        out[5] = g.noskip;
        return RT_OK;
    } catch (const std::bad_alloc&) {
        g_err = "rt_ocone_check: out of host memory";
        return RT_ENOMEM;
    }
}

int rt_octree_digest(const float* tri9, int64_t n, int32_t max_depth, int32_t leaf_max_obj_count, int32_t builder,
                     uint64_t* digest, int64_t stats[7], float* ms)
{
    if (n < 0 || (n > 0 && !tri9) || !digest)
        return bad("rt_octree_digest: bad arguments");
    try {
        rt::FlatOctree f;
        auto t0 = std::chrono::steady_clock::now();
        if (builder == 1)
            rt::build_flat_octree_serial(tri9, n, max_depth, leaf_max_obj_count, f);
        else
            rt::build_flat_octree(tri9, n, max_depth, leaf_max_obj_count, f);
        if (ms)
            *ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
        uint64_t h = 1469598103934665603ull;
        auto mix = [&h](const void* p, size_t len) {
            const unsigned char* b = static_cast<const unsigned char*>(p);
            for (size_t i = 0; i < len; i++) {
                h ^= b[i];
                h *= 1099511628211ull;
            }
        };
        mix(f.nodes.data(), f.nodes.size() * sizeof(rt::GNode));
        mix(f.tris.data(), f.tris.size() * sizeof(rt::GTri));
        mix(f.tri_id.data(), f.tri_id.size() * sizeof(int32_t));
        mix(&f.levels, sizeof(f.levels));
        *digest = h;
        if (stats) {
            stats[0] = f.stats.inner;
            stats[1] = f.stats.leaves;
            stats[2] = f.stats.empty_leaves;
            stats[3] = f.stats.max_leaf;
            stats[4] = f.stats.max_depth;
            stats[5] = f.stats.nodes;
            stats[6] = f.levels;
        }
        return RT_OK;
    } catch (const std::bad_alloc&) {
        g_err = "rt_octree_digest: out of host memory";
        return RT_ENOMEM;
    }
}

#if defined(W_DIAG) && !defined(__HIP_DEVICE_COMPILE__)
// host diagnostic counters of wbvh_closest (W_DIAG builds): read and reset
__attribute__((visibility("default"))) void rt_diag_read(long long* out)
{
    for (int i = 0; i < 8; i++)
        out[i] = rt::g_wdiag[i].exchange(0);
}
#endif

int rt_wbvh_query(const float* tri9, int64_t n, int32_t max_depth, int32_t leaf_max_obj_count, const float* orig,
                  const float* dir, int64_t nrays, int32_t* status, int32_t* id, float* t, float* u, float* v,
                  int64_t stats[8], float* ms)
{
    return rt_wbvh_query_ex(tri9, n, max_depth, leaf_max_obj_count, orig, dir, nrays, nullptr, nullptr, 0, nullptr,
                            nullptr, status, id, t, u, v, stats, ms, nullptr, 0, nullptr);
}

int rt_wbvh_query_ex(const float* tri9, int64_t n, int32_t max_depth, int32_t leaf_max_obj_count, const float* orig,
                     const float* dir, int64_t nrays, const float* cam, const float* light, int32_t shadow_rays,
                     float* o_out, float* d_out, int32_t* status, int32_t* id, float* t, float* u, float* v,
                     int64_t stats[8], float* ms, int32_t* ray_nodes, int32_t ocone_dim, int64_t oc_stats[5])
{
    if (n < 0 || (n > 0 && !tri9) || nrays < 0 || (nrays > 0 && (!orig || !dir || !status || !id || !t || !u || !v)) ||
        (shadow_rays && !light))
        return bad("rt_wbvh_query: bad arguments");
    try {
        rt::FlatOctree f;
        rt::WBvh w;
        auto t0 = std::chrono::steady_clock::now();
        rt::build_flat_octree(tri9, n, max_depth, leaf_max_obj_count, f);
        auto t1 = std::chrono::steady_clock::now();
        rt::build_wbvh(f, w);
        if (ms) {
            ms[0] = std::chrono::duration<float, std::milli>(t1 - t0).count();
            ms[1] = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t1).count();
        }
        float S = 0.0f;
        if (!f.nodes.empty())
            for (int a = 0; a < 3; a++)
                S = std::max(S, std::max(std::fabs(f.nodes[0].dn[a]), std::fabs(f.nodes[0].df[a])));
        const bool usable = !w.nodes.empty() && S > 0x1p-20f && S < 0x1p20f;
        // the risk bits of the camera / light (renderer.cpp prepare_risk, kernels.hip wide_risk_kernel)
        std::vector<uint64_t> risk;
        rt::WRiskArgs RA{};
        float cap[2] = {-1.0f, -1.0f};   // (no cap: never skips)
        float cap_dir[2][3] = {};
        if (usable && (cam || light)) {
            const float lo[3] = {f.nodes[0].dn[0], f.nodes[0].dn[1], f.nodes[0].dn[2]};
            const float hi[3] = {f.nodes[0].df[0], f.nodes[0].df[1], f.nodes[0].df[2]};
            const float zero[3] = {0, 0, 0};
            RA = rt::wbvh_risk_args(lo, hi, S, cam ? cam : zero, light ? light : zero, W_QS_CLOSEST, W_QS_SHADOW);
            risk.assign(w.nodes.size() * 8, rt::wrisk_pack(INFINITY, 0));
            std::vector<float> lbox(6 * w.tris.size());
            for (size_t k = 0; k < w.tris.size(); k++) {
                const rt::GNode& L = f.nodes[w.leaf_of_k[k]];
                for (int a = 0; a < 3; a++) {
                    lbox[6 * k + a] = L.dn[a];
                    lbox[6 * k + 3 + a] = L.df[a];
                }
            }
            if (cam)
                rt::wbvh_risk_host(w, lbox, RA, 0, risk);
            if (light)
                rt::wbvh_risk_host(w, lbox, RA, 1, risk);
            // the risk caps (renderer.cpp prepare_risk, kernels.hip wide_risk_kernel): towards the scene's centre
            if (std::getenv("RT_RISK_CAP") == nullptr || std::atoi(std::getenv("RT_RISK_CAP")) != 0)
                for (int sel = 0; sel < 2; sel++) {
                    if (!RA.on[sel] || (sel == 0 ? !cam : !light))
                        continue;
                    const float* X = sel == 0 ? cam : light;
                    double v[3], l = 0;
                    for (int a = 0; a < 3; a++) {
                        v[a] = 0.5 * ((double)lo[a] + (double)hi[a]) - (double)X[a];
                        l += v[a] * v[a];
                    }
                    l = std::sqrt(l);
                    for (int a = 0; a < 3; a++)
                        cap_dir[sel][a] = l > 0 && l < INFINITY ? (float)(v[a] / l) : (a == 0 ? 1.0f : 0.0f);
                    const double c[3] = {cap_dir[sel][0], cap_dir[sel][1], cap_dir[sel][2]};
                    float sm = INFINITY;
                    for (const rt::GTri& t : w.tris)
                        if (rt::wbvh_risk_key(t, RA.p[sel][0], RA.p[sel][1], RA.p[sel][2], RA.G[sel], RA.nu[sel],
                                              RA.slack[sel], RA.QS[sel]) < INFINITY)
                            sm = std::min(sm, rt::risk_cap_tri(t, c));
                    cap[sel] = sm;
                }
        }
        // the origin cones (ocone.hpp) for the rays neither from the camera nor shadow rays (renderer.cpp
        // start_accel's build)
        rt::OConeGrid ocg;
        rt::OConeView ocv{};
        if (usable && ocone_dim > 0) {
            rt::build_origin_cones(w, S, W_QS_CLOSEST, 0.0102 + 0x1p-16 * S, ocone_dim, 80.0 * 3.14159265358979 / 180.0, 0, ocg);
            if (!ocg.cells.empty()) {
                ocv.cells = ocg.cells.data();
                for (int a = 0; a < 3; a++) {
                    ocv.lo[a] = ocg.lo[a];
                    ocv.dim[a] = ocg.dim[a];
                }
                ocv.ih = ocg.ih;
            }
        }
        std::atomic<int64_t> work_n{0}, work_t{0}, n_nob{0};
        const bool probe_hi = std::getenv("RT_WQ_PROBE_HI") != nullptr;
        auto body = [&](int64_t b, int64_t e) {
            rt::WStackLocal stk;
            uint32_t wk[4] = {0, 0, 0, 0};
            for (int64_t i = b; i < e; i++) {
                rt::v3 o = rt::mk(orig[3 * i], orig[3 * i + 1], orig[3 * i + 2]);
                rt::v3 d = rt::mk(dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]);
                const uint64_t* rk = nullptr;
                int rsel = 0;
                float rsub = 0.0f;
                if (shadow_rays) {
                    // is_shadowed's ray (kernels.hip): orig = the hit point p, dir = its normal n
                    const rt::v3 p = o, nrm = d, lp = rt::mk(light[0], light[1], light[2]);
                    o = p + nrm * 1.0e-4f;
                    d = rt::normalize(lp - p);
                    const float nl = std::fabs(nrm.x) + std::fabs(nrm.y) + std::fabs(nrm.z);
                    const float hi = (std::sqrt(rt::length2(p - lp)) + 1.0e-4f * nl) * (1.0f + 0x1p-10f);
                    if (!risk.empty() && hi <= RA.ray_G && nl <= RA.ray_nl) {
                        rk = risk.data();
                        rsel = 1;
                        rsub = rt::wrisk_sub(W_QS_SHADOW, hi, RA.ray_nu);
                    }
                } else if (!risk.empty() && cam && o.x == cam[0] && o.y == cam[1] && o.z == cam[2])
                    rk = risk.data();
                if (o_out) {
                    o_out[3 * i] = o.x;
                    o_out[3 * i + 1] = o.y;
                    o_out[3 * i + 2] = o.z;
                }
                if (d_out) {
                    d_out[3 * i] = d.x;
                    d_out[3 * i + 1] = d.y;
                    d_out[3 * i + 2] = d.z;
                }
                bool nan = false;
                for (int p = 0; p < rt::NPLANES; p++) {
                    rt::v3 pn = rt::mk(rt::PLANE_N[p][0], rt::PLANE_N[p][1], rt::PLANE_N[p][2]);
                    float den = rt::dot(pn, d), num = rt::dot(pn, o);
                    nan |= den != den || num != num;
                }
                id[i] = -1;
                t[i] = -1.0f;
                u[i] = 1.0f;
                v[i] = 0.0f;
                if (f.nodes.empty()) {
                    status[i] = rt::W_MISS;
                    continue;
                }
                if (!usable || nan) {
                    status[i] = rt::W_UNCERT;
                    continue;
                }
                float om = std::max(std::fabs(o.x), std::max(std::fabs(o.y), std::fabs(o.z)));
                float m = 0x1p-16f * (om + S);
                rt::WHit h;
                const uint32_t wk0 = wk[0];
                bool nob = !shadow_rays && !rk && rt::ocone_skip(ocv, o, d, W_QS_CLOSEST);
                if (rk && !shadow_rays && cap[0] >= 0.0f)   // a camera ray: the camera's risk cap
                    nob = rt::risk_cap_skip(cap[0], cap_dir[0], d, W_QS_CLOSEST);
                if (rk && shadow_rays && cap[1] >= 0.0f)    // a shadow ray with the light's words: the light's cap
                    nob = rt::risk_cap_skip(cap[1], cap_dir[1], d, W_QS_SHADOW);
                if (nob)
                    ++n_nob;
                int st = rt::wbvh_closest(w.nodes.data(), w.tris.data(), o, d, m, stk, h, wk, INFINITY, true,
                                          shadow_rays ? W_QS_SHADOW : W_QS_CLOSEST, rk, rsel, rsub, 0u,
                                          (rt::WNoFeed*)nullptr, nob);
                if (st == rt::W_DEEP) {   // the kernels' retry with a deeper stack (kernels.hip wide_closest_deep)
                    rt::WStackArr<rt::W_DEEP_STACK> deep;
                    st = rt::wbvh_closest(w.nodes.data(), w.tris.data(), o, d, m, deep, h, wk, INFINITY, true,
                                          shadow_rays ? W_QS_SHADOW : W_QS_CLOSEST, rk, rsel, rsub);
                    if (st == rt::W_DEEP)
                        st = rt::W_UNCERT;
                }
                if (st == rt::W_HIT && probe_hi) {
                    // (diagnostic, RT_WQ_PROBE_HI=1: the same query again with its answer known up front,
                    // hi = t*: the visits a perfect visiting order would leave; ray_nodes reports those)
                    rt::WStackArr<rt::W_DEEP_STACK> deep;
                    rt::WHit h2;
                    wk[0] = wk0;
                    rt::wbvh_closest(w.nodes.data(), w.tris.data(), o, d, m, deep, h2, wk, h.t, true,
                                     shadow_rays ? W_QS_SHADOW : W_QS_CLOSEST, rk, rsel, rsub);
                }
                if (st == rt::W_HIT) {
                    int32_t slot = w.slot[(size_t)h.k];
                    if (rt::kdop_certifies(f.nodes[w.leaf_of_slot[(size_t)slot]], o, d, h.t)) {
                        id[i] = f.tri_id[(size_t)slot];
                        t[i] = h.t;
                        u[i] = h.u;
                        v[i] = h.v;
                    } else
                        st = rt::W_UNCERT;
                }
                status[i] = st;
                if (ray_nodes)
                    ray_nodes[i] = (int32_t)(wk[0] - wk0);
            }
            work_n += wk[0];
            work_t += wk[1];
        };
        unsigned hc = std::max(1u, std::min(std::thread::hardware_concurrency(), 16u));
        std::vector<std::thread> th;
        int64_t chunk = (nrays + hc - 1) / hc;
        for (unsigned k = 0; k < hc; k++) {
            int64_t b = (int64_t)k * chunk, e = std::min(nrays, b + chunk);
            if (b < e)
                th.emplace_back(body, b, e);
        }
        for (auto& x : th)
            x.join();
        if (stats) {
            stats[0] = w.stats.nodes;
            stats[1] = w.stats.leaves;
            stats[2] = w.stats.max_leaf;
            stats[3] = w.stats.depth;
            stats[4] = work_n.load();
            stats[5] = work_t.load();
            stats[6] = rt::check_wbvh(f, w);
            // the risk words the queries read (wbvh_risk_host), checked against the tree
            if (!risk.empty()) {
                if (cam)
                    stats[6] += rt::check_risk_words(f, w, RA, 0, risk.data());
                if (light)
                    stats[6] += rt::check_risk_words(f, w, RA, 1, risk.data());
            }
            stats[7] = (int64_t)(w.stats.sah * 1000.0f);
        }
        if (oc_stats) {
            oc_stats[0] = ocg.computed;
            oc_stats[1] = ocg.empty;
            oc_stats[2] = ocg.noskip;
            oc_stats[3] = n_nob.load();
            oc_stats[4] = (int64_t)ocg.ms;
        }
        return RT_OK;
    } catch (const std::bad_alloc&) {
        g_err = "rt_wbvh_query: out of host memory";
        return RT_ENOMEM;
    }
}

}  // extern "C"
