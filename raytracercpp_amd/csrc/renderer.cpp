// renderer.cpp -- rt::Renderer (see renderer.hpp).
#include "renderer.hpp"
#include "multidev.hpp"

#include <hipcub/hipcub.hpp>

#include <cstdlib>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <thread>

#include "host_scene.hpp"

extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_ray_trace(const rt::KParams* P, hipStream_t stream);
extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_heavy_prep(const rt::KParams* P, uint32_t* cost,
                                                                                 int ntiles, int32_t* list,
                                                                                 uint32_t* bits, int32_t* ctr,
                                                                                 int32_t* ctr_next,
                                                                                 const unsigned long long* stats_prev,
                                                                                 unsigned long long* stats_next,
                                                                                 float split, int group,
                                                                                 hipStream_t stream);

extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_refl_level0(const rt::KParams* P, rt::FrameRec* fr1,
                                                                           unsigned int* nfr1, hipStream_t stream);
extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_refl_stage(int stage, const rt::KParams* P,
                                                                          const rt::ReflArgs* A, hipStream_t stream);
extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_refl_keys(const rt::KParams* P, const rt::FrameRec* fr,
                                                                         int n, uint32_t* keys, int32_t* idx,
                                                                         hipStream_t stream);
extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_risk_box_init(float* B, size_t nentries,
                                                                                    hipStream_t stream);
extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_trace_rays(const rt::KParams* P, const float* o, const float* d, int n, int32_t* id,
                                           float* t, float* u, float* v, uint8_t* ret, hipStream_t stream);
extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_wide_query(const rt::KParams* P, const float* o,
                                                                                 const float* d, int n, int kind,
                                                                                 float* o_out, float* d_out,
                                                                                 int32_t* status, int32_t* id, float* t,
                                                                                 float* u, float* v, uint8_t* sh,
                                                                                 hipStream_t stream);
extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_trace_colors(const rt::KParams* P, bool refl,
                                                                                   const float* o, const float* d,
                                                                                   int n, float4* rgba, int32_t* src,
                                                                                   float* t, uint8_t* found,
                                                                                   uint8_t* shadow, hipStream_t stream);
extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_raster_stage(int stage, const rt::KParams* P,
                                                                            const rt::RasterArgs* A, int npieces,
                                                                            hipStream_t stream);
extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_raster_shade(const rt::KParams* P,
                                                                            const rt::RasterArgs* A,
                                                                            rt::FrameRec* fr1, unsigned int* nfr1,
                                                                            hipStream_t stream);
extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_ssao(const rt::SsaoArgs* A, hipStream_t stream);
extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_ocone(const rt::OConeEnt* E, const rt::GTri* tris,
                                                                     const uint32_t* todo, int n, const float lo[3],
                                                                     const int32_t dim[3], double h, double r, double slack,
                                                                     double QS, double cos_cap, uint2* cells,
                                                                     size_t ncells, hipStream_t stream);
extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_refl_defer_keys(const rt::ReflArgs* A, int n, uint32_t* keys,
                                                                                hipStream_t stream);
extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_refl_dir_keys(const rt::KParams* P, const rt::ReflArgs* A,
                                                                              uint32_t* keys, int32_t* vals, hipStream_t stream);
extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_refl_shadow_keys(const rt::KParams* P, const rt::SampleRec* sm,
                                                                                 const int32_t* list, int n, uint32_t* keys,
                                                                                 hipStream_t stream);
extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_refl_sort_frames(const rt::FrameRec* fr, const int32_t* order,
                                                                                int n, rt::FrameRec* frs, hipStream_t stream);
extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_wide_gather(
    const rt::GTri* tris, const int32_t* slot, const uint32_t* leaf_of_slot, const int32_t* tri_id,
    const int32_t* tri_mat, int n, rt::GTri* wtris, uint4* wmeta, hipStream_t stream);
extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_wide_risk(
    const rt::GTri* wtris, const uint4* wmeta, const rt::GNode* onodes, const rt::WNode* wnodes, const uint32_t* tri_leaf,
    const uint32_t* parent, uint32_t* K, float* B, unsigned long long* risk, int n, int nnodes, const rt::WRiskArgs* A,
    uint32_t* cap, const float* cap_dir, hipStream_t stream);
extern "C" __attribute__((visibility("hidden"))) hipError_t rt_launch_downscale(const uint32_t* in, int w, int h_rows, int f, uint32_t* out,
                                          hipStream_t stream);

namespace rt {

DevBuf::~DevBuf() { release(); }

void DevBuf::release()
{
    if (p) {
        hipSetDevice(device);
        (void)hipFree(p);
    }
    p = nullptr;
    bytes = 0;
}

hipError_t DevBuf::reserve(size_t n)
{
    if (n <= bytes && p)
        return hipSuccess;
    release();
    if (n == 0)
        n = 16;
    hipError_t e = hipMalloc(&p, n);
    if (e != hipSuccess) {
        p = nullptr;
        return e;
    }
    bytes = n;
    return hipSuccess;
}

// each switch is on unless its variable is set to 0 (RT_DEBUG_WAVES: on when set)
Knobs Knobs::from_env()
{
    Knobs k;
    auto on = [](const char* name, bool dflt) {
        const char* v = getenv(name);
        return v ? v[0] != '0' : dflt;
    };
    k.wbvh = on("RT_WBVH", true);   // (exact mode overrides: Renderer::fill_params)
    k.seg = on("RT_SEG", true);
    k.seg_oct = on("RT_SEG_OCTREE", false);
    k.cones = on("RT_CONES", true);
    k.lslab = on("RT_LSLAB", true);
    k.plain = on("RT_PLAIN", true);
    k.plain_octree = on("RT_PLAIN_OCTREE", true);
    k.quick_wbvh = on("RT_WBVH_QUICK_FIRST", true);
    k.fused_ssaa = on("RT_FUSED_SSAA", true);
    k.refl_engine = on("RT_REFL_ENGINE", true);
    k.refl_sort = on("RT_REFL_SORT", true);
    k.refl_fuse = on("RT_REFL_FUSE", true);
    k.debug_waves = getenv("RT_DEBUG_WAVES") != nullptr;
    k.exact = on("RT_EXACT", false);
    k.risk = on("RT_WBVH_RISK", true);
    k.heavy = on("RT_HEAVY_FIRST", true);
    if (const char* v = getenv("RT_HEAVY_GROUP")) {
        const int g = atoi(v);
        k.heavy_group = g > 1 ? SPLIT_G : 0;   // (the split's group size is the build's, kparams.hpp RT_SPLIT_G)
    }
    if (const char* v = getenv("RT_HEAVY_SPLIT"))
        k.heavy_split = std::max(0.0f, (float)atof(v));
    if (const char* v = getenv("RT_HEAVY_SPLIT_EXP"))
        k.heavy_split_exp = std::max(0.0f, (float)atof(v));
    if (const char* v = getenv("RT_HEAVY_SPLIT_EXP_OVERLAP"))
        k.heavy_split_exp_overlap = std::max(0.0f, (float)atof(v));
    if (const char* v = getenv("RT_SPLIT_PARTS"))
        k.split_parts = atoi(v) == 2 * SPLIT_G ? 2 * SPLIT_G : SPLIT_G;
    if (const char* v = getenv("RT_REFL_DEFER"))   // loop iterations before a reflection query is deferred
        k.refl_defer = std::max(0, atoi(v));
    if (const char* v = getenv("RT_REFL_FEED"))    // lane refill of the reflection queries at this many waiting lanes
        k.refl_feed = std::min(64, std::max(0, atoi(v)));
    if (const char* v = getenv("RT_REFL_FEED_FRAME_ORDER"))
        k.refl_feed_frame_order = atoi(v) != 0;
    if (const char* v = getenv("RT_REFL_SAMPLE_MAJOR"))
        k.refl_sample_major = atoi(v) != 0;
    if (const char* v = getenv("RT_REFL_DIR_SORT"))
        k.refl_dir_sort = atoi(v) != 0;
    if (const char* v = getenv("RT_REFL_FEED_XCD"))
        k.refl_feed_xcd = atoi(v) != 0;
    if (const char* v = getenv("RT_REFL_DEFER_SORT"))
        k.refl_defer_sort = atoi(v) != 0;
    if (const char* v = getenv("RT_REFL_SHADOW_SORT"))
        k.refl_shadow_sort = atoi(v) != 0;
    if (const char* v = getenv("RT_REFL_SORTED_FRAMES"))
        k.refl_sorted_frames = atoi(v) != 0;
    if (const char* v = getenv("RT_RISK_CAP"))
        k.risk_cap = atoi(v) != 0;
    if (const char* v = getenv("RT_OCONE"))
        k.ocone = atoi(v) != 0;
    if (const char* v = getenv("RT_OCONE_DIM"))
        k.ocone_dim = std::min(1024, std::max(1, atoi(v)));
    if (const char* v = getenv("RT_REFL_SHADOW_FEED"))
        k.refl_shadow_feed = std::min(64, std::max(0, atoi(v)));
    {
        const char* v = getenv("RT_INJECT_FRAME_FAIL");   // tests: the k-th ray_trace fails after its image start
        k.inject_fail = v ? std::atoi(v) : 0;
    }
    k.async_accel = on("RT_ASYNC_ACCEL", true);
    if (const char* ce = getenv("RT_REFL_CHUNK_LOG2")) {
        const int v = atoi(ce);
        if (v >= 10 && v <= 27)   // small values (tests): many chunks per level
            k.refl_chunk_log2 = v;
    }
    return k;
}

Renderer::Renderer(int device) : knobs_(Knobs::from_env()), device_(device)
{
    rt_default_settings(&s_);
    mat::identity(c2w_);
    mat::identity(w2c_);
    mat::identity(prev_object_);
    int rw, rh;
    render_size(rw, rh);
    img_w_ = rw;
    img_h_ = rh;
    aspect_ = (float)rw / rh;   // Renderer ctor: _camera.set_aspect_ratio(render_w / render_h), renderer.cpp:93
    update_camera_projection();
}

int Renderer::init(std::string& err)
{
    hipError_t e = hipSetDevice(device_);
    if (e == hipSuccess)
        e = hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking);
    if (e == hipSuccess)
        e = hipStreamCreateWithFlags(&accel_stream_, hipStreamNonBlocking);
    if (e == hipSuccess)
        e = hipStreamCreateWithFlags(&fence_stream_, hipStreamNonBlocking);
    if (e == hipSuccess)
        e = hipDeviceGetAttribute(&num_cus_, hipDeviceAttributeMultiprocessorCount, device_);
    for (int i = 0; i < 4 && e == hipSuccess; i++)
        e = hipEventCreate(&ev_[i]);
    if (e == hipSuccess)
        e = hipEventCreateWithFlags(&risk_ev_, hipEventDisableTiming);
    if (e == hipSuccess)
        e = hipEventCreateWithFlags(&risk_mark_, hipEventDisableTiming);
    if (e != hipSuccess) {
        err = std::string("HIP init failed: ") + hipGetErrorString(e);
        return RT_EHIP;
    }
    DevBuf* all[] = {&d_nodes_, &d_tris_,  &d_tri_id_, &d_tri_mat_, &d_tri_uv_, &d_mats_,   &d_internal_,
                     &d_image_, &d_rgba_,  &d_hit_id_, &d_hit_t_,   &d_shadow_, &d_counters_,
                     &d_tri9_,  &d_rcount_, &d_roff_,  &d_pieces_,  &d_piece_uv_, &d_zkey_, &d_big_, &d_scan_tmp_,
                     &d_zbuf_,  &d_nbuf_,   &d_ao_,     &d_cones_, &d_lslab_, &d_lsin_, &d_wnodes_, &d_wtris_, &d_wmeta_, &d_wtmp_,
                     &d_wlinks_, &d_wrisk_, &d_dbg_, &d_wnodes2_, &d_wtris2_, &d_wmeta2_, &d_wtmp2_, &d_wlinks2_,
                     &d_ocone_, &d_ocone2_, &d_oc_ent_, &d_oc_todo_};
    for (DevBuf* b : all) b->device = device_;
    for (auto& b : d_tex_) b.device = device_;
    for (auto& b : d_sky_) b.device = device_;
    return RT_OK;
}

Renderer::~Renderer()
{
    if (accel_thread_.joinable())
        accel_thread_.join();
    hipSetDevice(device_);
    if (accel_stream_) hipStreamDestroy(accel_stream_);
    for (auto& e : ev_)
        if (e) hipEventDestroy(e);
    if (risk_ev_) hipEventDestroy(risk_ev_);
    if (risk_mark_) hipEventDestroy(risk_mark_);
    for (auto& e : ring_)
        if (e) hipEventDestroy(e);
    for (auto& b : band_slot_) {
        if (b.done) hipEventDestroy(b.done);
        if (b.mark) hipEventDestroy(b.mark);
    }
    if (fence_stream_) hipStreamDestroy(fence_stream_);
    if (stream_) hipStreamDestroy(stream_);
    for (hipEvent_t ev : display_ev_)
        if (ev) hipEventDestroy(ev);
    if (display_stream_) hipStreamDestroy(display_stream_);
    if (display_host_) hipHostFree(display_host_);
    for (void* q : display_old_)
        hipHostFree(q);
}

int Renderer::fail(int code, const std::string& msg)
{
    err_ = msg;
    return code;
}

int Renderer::hip_fail(hipError_t e, const char* what)
{
    err_ = std::string(what) + ": " + hipGetErrorString(e);
    return RT_EHIP;
}

// Renderer::get_render_width_height, renderer.cpp:116-120
void Renderer::render_size(int& w, int& h) const
{
    w = s_.enable_ssaa ? s_.image_width * s_.ssaa_factor : s_.image_width;
    h = s_.enable_ssaa ? s_.image_height * s_.ssaa_factor : s_.image_height;
}

// Camera::set_aspect_ratio / set_fov (camera.cpp:5-19)
void Renderer::update_camera_projection()
{
    mat::perspective(fov_, aspect_, near_, far_, proj_);
    mat::inverse(proj_, proj_inv_);
}

int Renderer::set_settings(const rt_settings& s)
{
    if (s.image_width <= 0 || s.image_height <= 0 || (s.enable_ssaa && s.ssaa_factor <= 0))
        return fail(RT_EINVAL, "invalid image size / ssaa_factor");
    if (s.bvh_max_depth > 30)
        return fail(RT_EUNSUPPORTED, "bvh_max_depth > 30");
    bool bvh_changed = s.enable_bvh != s_.enable_bvh || s.bvh_max_depth != s_.bvh_max_depth ||
                       s.bvh_leaf_object_count != s_.bvh_leaf_object_count;
    s_ = s;
    if (bvh_changed)
        geom_dirty_ = true, ++geom_ver_;
    return RT_OK;
}

// renderer.cpp:250-261
int Renderer::change_render_size(int w, int h)
{
    if (w <= 0 || h <= 0)
        return fail(RT_EINVAL, "invalid render size");
    s_.image_width = w;
    s_.image_height = h;
    int rw, rh;
    render_size(rw, rh);
    {
        std::lock_guard<std::recursive_mutex> g(image_mu_);
        img_w_ = rw;
        img_h_ = rh;
        rendered_ = false;
    }
    aspect_ = (float)rw / rh;
    update_camera_projection();
    return RT_OK;
}

// renderer.cpp:137-144
int Renderer::set_triangles(const float* tri9, const int32_t* mat, const float* uv6, int64_t n)
{
    if (n < 0 || (n > 0 && (!tri9 || !mat)))
        return fail(RT_EINVAL, "set_triangles: null arrays");
    if (n >= (int64_t)1 << 30)
        return fail(RT_EUNSUPPORTED, "set_triangles: more than 2^30 triangles");
    tri_.assign(tri9, tri9 + 9 * n);
    tri_mat_.assign(mat, mat + n);
    // the material range, checked by validate() before every launch without re-reading
    // the per-triangle indices (a 1M-triangle scan per frame cost ~0.2 ms of host time)
    tri_mat_lo_ = INT32_MAX;
    tri_mat_hi_ = INT32_MIN;
    for (int32_t m : tri_mat_) {
        tri_mat_lo_ = std::min(tri_mat_lo_, m);
        tri_mat_hi_ = std::max(tri_mat_hi_, m);
    }
    if (uv6)
        tri_uv_.assign(uv6, uv6 + 6 * n);
    else
        tri_uv_.clear();
    has_bvh_ = s_.enable_bvh;
    geom_dirty_ = true, ++geom_ver_;
    return RT_OK;
}

int Renderer::add_sphere(float cx, float cy, float cz, float r, int mat)
{
    if ((int)shape_kind_.size() >= MAX_SHAPES)
        return fail(RT_EUNSUPPORTED, "too many analytic shapes");
    shape_kind_.push_back(0);
    float p[6] = {cx, cy, cz, r, 0, 0};
    shape_.insert(shape_.end(), p, p + 6);
    shape_mat_.push_back(mat);
    return RT_OK;
}

int Renderer::add_plane(float px, float py, float pz, float nx, float ny, float nz, int mat)
{
    if ((int)shape_kind_.size() >= MAX_SHAPES)
        return fail(RT_EUNSUPPORTED, "too many analytic shapes");
    shape_kind_.push_back(1);
    float p[6] = {px, py, pz, nx, ny, nz};
    shape_.insert(shape_.end(), p, p + 6);
    shape_mat_.push_back(mat);
    return RT_OK;
}

// renderer.cpp:182-186
int Renderer::clear_geometry()
{
    tri_.clear();
    tri_mat_.clear();
    tri_mat_lo_ = INT32_MAX;
    tri_mat_hi_ = INT32_MIN;
    tri_uv_.clear();
    shape_kind_.clear();
    shape_.clear();
    shape_mat_.clear();
    geom_dirty_ = true, ++geom_ver_;
    return RT_OK;
}

int Renderer::set_materials(const float* mats16, int n)
{
    if (n < 0 || (n > 0 && !mats16))
        return fail(RT_EINVAL, "set_materials: null array");
    mats_.assign(mats16, mats16 + (size_t)MAT_STRIDE * n);
    mats_dirty_ = true, ++mats_ver_;
    return RT_OK;
}

int Renderer::change_camera_fov(float fov)
{
    fov_ = fov;
    update_camera_projection();
    return RT_OK;
}

int Renderer::change_camera_aspect_ratio(float aspect)
{
    aspect_ = aspect;
    update_camera_projection();
    return RT_OK;
}

int Renderer::set_light_position(float x, float y, float z)
{
    light_[0] = x;
    light_[1] = y;
    light_[2] = z;
    return RT_OK;
}

// renderer.cpp:226-233
// Exact mode: every query walks the octree over the whole line, the
// reference's own traversal; leaving it rebuilds the wide BVH if it was never built.
int Renderer::set_exact(bool on)
{
    poll_accel(true);   // (reads wb_)
    if (knobs_.exact && !on && knobs_.wbvh && wb_.nodes.empty() && s_.enable_bvh)
        geom_dirty_ = true, ++geom_ver_;
    knobs_.exact = on;
    return RT_OK;
}

int Renderer::set_camera_transform(const float m[16])
{
    std::memcpy(c2w_, m, sizeof(c2w_));
    mat::inverse(c2w_, w2c_);
    v3 p = xform_point(c2w_, mk(0, 0, 0));
    cam_pos_[0] = p.x;
    cam_pos_[1] = p.y;
    cam_pos_[2] = p.z;
    return RT_OK;
}

// renderer.cpp:235-241
int Renderer::apply_transformation_to_camera(const float m[16])
{
    mat::compose(m, c2w_, c2w_);
    mat::inverse(c2w_, w2c_);
    v3 p = xform_point(m, mk(cam_pos_[0], cam_pos_[1], cam_pos_[2]));
    cam_pos_[0] = p.x;
    cam_pos_[1] = p.y;
    cam_pos_[2] = p.z;
    return RT_OK;
}

int Renderer::set_camera_matrices(const float pos[3], const float proj_inv[16], const float c2w[16])
{
    std::memcpy(cam_pos_, pos, sizeof(cam_pos_));
    std::memcpy(proj_inv_, proj_inv, sizeof(proj_inv_));
    std::memcpy(c2w_, c2w, sizeof(c2w_));
    mat::inverse(c2w_, w2c_);
    return RT_OK;
}

int Renderer::set_camera_lens(float fov, float aspect)
{
    fov_ = fov;
    aspect_ = aspect;
    return RT_OK;
}

int Renderer::set_camera_projection(const float proj[16], const float w2c[16])
{
    std::memcpy(proj_, proj, sizeof(proj_));
    std::memcpy(w2c_, w2c, sizeof(w2c_));
    return RT_OK;
}

void Renderer::get_camera_matrices(float pos[3], float proj_inv[16], float c2w[16]) const
{
    std::memcpy(pos, cam_pos_, sizeof(cam_pos_));
    std::memcpy(proj_inv, proj_inv_, sizeof(proj_inv_));
    std::memcpy(c2w, c2w_, sizeof(c2w_));
}

// renderer.cpp:214-224: every triangle goes through object_transform * previous^-1,
// then the BVH is rebuilt.
int Renderer::set_object_transform(const float m[16])
{
    float inv[16], t[16];
    mat::inverse(prev_object_, inv);
    std::memcpy(prev_object_, inv, sizeof(inv));
    mat::compose(m, prev_object_, t);
    size_t n = tri_.size() / 3;
    std::vector<float> out(tri_.size());
    mat::transform_points(t, tri_.data(), (int64_t)n, out.data());
    tri_.swap(out);
    has_bvh_ = true;
    geom_dirty_ = true, ++geom_ver_;
    std::memcpy(prev_object_, m, sizeof(prev_object_));
    return RT_OK;
}

int Renderer::reset_previous_transform()
{
    mat::identity(prev_object_);
    return RT_OK;
}

int Renderer::set_texture(int slot, int w, int h, const float* rgba)
{
    if (slot < 0 || slot >= TEX_SLOTS)
        return fail(RT_EINVAL, "set_texture: bad slot");
    if (!rgba) {
        tex_[slot] = HostTex();
    } else {
        if (w <= 0 || h <= 0)
            return fail(RT_EINVAL, "set_texture: bad size");
        tex_[slot].w = w;
        tex_[slot].h = h;
        tex_[slot].rgba.assign(rgba, rgba + (size_t)w * h * 4);
    }
    tex_dirty_ = true, ++tex_ver_;
    return RT_OK;
}

int Renderer::set_skybox(const int32_t w[6], const int32_t h[6], const float* const faces[6])
{
    for (int i = 0; i < 6; i++) {
        if (!faces || !faces[i]) {
            sky_[i] = HostTex();
            continue;
        }
        if (w[i] <= 0 || h[i] <= 0)
            return fail(RT_EINVAL, "set_skybox: bad face size");
        sky_[i].w = w[i];
        sky_[i].h = h[i];
        sky_[i].rgba.assign(faces[i], faces[i] + (size_t)w[i] * h[i] * 4);
    }
    tex_dirty_ = true, ++tex_ver_;
    return RT_OK;
}

int Renderer::reconstruct_bvh_new()
{
    has_bvh_ = true;
    geom_dirty_ = true, ++geom_ver_;
    return RT_OK;
}

int Renderer::destroy_bvh()
{
    has_bvh_ = false;
    geom_dirty_ = true, ++geom_ver_;
    return RT_OK;
}

// Leaf slabs (kernels.hip leaf_missed): the box of the leaf's
// triangles a, a + ab, a + ac (rounded outward) and, once the cone axis is known, the range of
// their projections on it (rounded outward; the kernel adds its own margin).  Without an
// axis the slab is [-inf, +inf] (no constraint).
static void leaf_slab(const FlatOctree& o, uint32_t a, uint32_t cnt, float* out)
{
    double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (uint32_t k = a; k < a + cnt; k++) {
        const GTri& t = o.tris[k];
        for (int c = 0; c < 3; c++) {
            double p0 = t.a[c], p1 = p0 + t.ab[c], p2 = p0 + t.ac[c];
            mn[c] = std::min(mn[c], std::min(p0, std::min(p1, p2)));
            mx[c] = std::max(mx[c], std::max(p0, std::max(p1, p2)));
        }
    }
    for (int c = 0; c < 3; c++) {
        out[c] = std::nextafter((float)mn[c], -INFINITY);
        out[4 + c] = std::nextafter((float)mx[c], INFINITY);
    }
    out[3] = -INFINITY;
    out[7] = INFINITY;
}

static void leaf_slab_axis(const FlatOctree& o, uint32_t a, uint32_t cnt, double ax, double ay, double az, float* out)
{
    // the projections use the float axis the kernel reads
    const double fx = (float)ax, fy = (float)ay, fz = (float)az;
    double smin = INFINITY, smax = -INFINITY;
    for (uint32_t k = a; k < a + cnt; k++) {
        const GTri& t = o.tris[k];
        for (int v = 0; v < 3; v++) {
            double p[3];
            for (int c = 0; c < 3; c++)
                p[c] = (double)t.a[c] + (v == 1 ? (double)t.ab[c] : v == 2 ? (double)t.ac[c] : 0.0);
            double d = fx * p[0] + fy * p[1] + fz * p[2];
            smin = std::min(smin, d);
            smax = std::max(smax, d);
        }
    }
    out[3] = std::nextafter((float)smin, -INFINITY);
    out[7] = std::nextafter((float)smax, INFINITY);
}

// Leaf normal cones (kernels.hip leaf_backfacing): per leaf, the
// normalised mean of its triangles' stored normals (triangle.cpp:9-10) and the smallest
// cosine between it and any of them, less 1e-6.  Triangles with n == 0 never hit (Mdet ==
// 0) and are left out; a leaf with a normal too small or too large for the kernel's
// rounding argument, or a cone of 90 degrees or more, gets no cone (cos = -2).
static void leaf_cones(const FlatOctree& o, std::vector<float>& out, std::vector<float>& slab, std::vector<float>& lsin)
{
    out.assign(4 * o.tris.size(), 0.0f);
    slab.assign(8 * o.tris.size(), 0.0f);
    lsin.assign(o.tris.size(), 0.0f);
    for (const GNode& g : o.nodes) {
        if (!(g.b & LEAF_BIT))
            continue;
        const uint32_t a = g.a, cnt = g.b & ~LEAF_BIT;
        float* c = &out[4 * (size_t)a];
        c[3] = -2.0f;
        if (cnt > 0) {
            float sm = 1.0f;
            for (uint32_t k = a; k < a + cnt; k++)
                sm = std::min(sm, sin_at_a_f(o.tris[k]));
            lsin[a] = sm;   // leaf_missed's grazing margin
        }
        leaf_slab(o, a, cnt, &slab[8 * (size_t)a]);
        double sx = 0, sy = 0, sz = 0;
        bool ok = cnt > 0;
        for (uint32_t k = a; k < a + cnt && ok; k++) {
            const float* n = o.tris[k].n;
            double len = std::sqrt((double)n[0] * n[0] + (double)n[1] * n[1] + (double)n[2] * n[2]);
            if (len == 0.0)
                continue;
            if (!(len > 1e-30 && len < 1e27)) {
                ok = false;
                break;
            }
            sx += n[0] / len;
            sy += n[1] / len;
            sz += n[2] / len;
        }
        double sl = std::sqrt(sx * sx + sy * sy + sz * sz);
        if (!ok || !(sl > 1e-9))
            continue;
        sx /= sl;
        sy /= sl;
        sz /= sl;
        leaf_slab_axis(o, a, cnt, sx, sy, sz, &slab[8 * (size_t)a]);
        double cmin = 1.0;
        for (uint32_t k = a; k < a + cnt; k++) {
            const float* n = o.tris[k].n;
            double len = std::sqrt((double)n[0] * n[0] + (double)n[1] * n[1] + (double)n[2] * n[2]);
            if (len == 0.0)
                continue;
            cmin = std::min(cmin, (n[0] * sx + n[1] * sy + n[2] * sz) / len);
        }
        cmin -= 1e-6;
        c[0] = (float)sx;   // the axis is kept for leaf_missed's slab even without a cone
        c[1] = (float)sy;
        c[2] = (float)sz;
        if (!(cmin > 0.0))
            continue;
        c[3] = std::nextafter((float)cmin, 0.0f);   // rounded toward 0: never narrower than computed
    }
}

// The leaf cones / slabs and the wide BVH of the current octree, on accel_thread_ (DESIGN.md
// 5.8).  Reads oct_ and the uploaded triangle tables; writes only cones_, lslab_, lsin_, wb_, their
// device buffers and accel_ms_, none of which a frame reads before poll_accel adopts them.
hipError_t Renderer::upload_wide(const WBvh& w, DevBuf& nodes, DevBuf& tris, DevBuf& meta, DevBuf& tmp, DevBuf& links,
                                 hipStream_t stream)
{
    // the nodes, and the permutation from which the device gathers the wide BVH's triangle records
    // and, per triangle, everything a certified hit needs in one 16-B load: the octree slot (the
    // record's triangle), the leaf of its certificate, the caller's triangle index and its material
    // (kernels.hip wide_gather_kernel)
    hipError_t e;
    const size_t nk = w.slot.size(), wn = w.nodes.size() * sizeof(WNode);
    const size_t nl = w.tri_leaf.size() + w.parent.size();
    if ((e = nodes.reserve(wn)) != hipSuccess || (e = tris.reserve(nk * sizeof(GTri))) != hipSuccess ||
        (e = meta.reserve(nk * 16)) != hipSuccess || (e = tmp.reserve(nk * 8)) != hipSuccess ||
        (e = links.reserve(nl * 4)) != hipSuccess)
        return e;
    hipSetDevice(device_);
    int32_t* d_slot = tmp.as<int32_t>();
    uint32_t* d_leaf = reinterpret_cast<uint32_t*>(d_slot + nk);
    if ((e = hipMemcpyAsync(links.p, w.tri_leaf.data(), w.tri_leaf.size() * 4, hipMemcpyHostToDevice, stream)) != hipSuccess ||
        (e = hipMemcpyAsync(links.as<uint32_t>() + w.tri_leaf.size(), w.parent.data(), w.parent.size() * 4,
                            hipMemcpyHostToDevice, stream)) != hipSuccess ||
        (e = hipMemcpyAsync(nodes.p, w.nodes.data(), wn, hipMemcpyHostToDevice, stream)) != hipSuccess ||
        (e = hipMemcpyAsync(d_slot, w.slot.data(), nk * 4, hipMemcpyHostToDevice, stream)) != hipSuccess ||
        (e = hipMemcpyAsync(d_leaf, w.leaf_of_slot.data(), nk * 4, hipMemcpyHostToDevice, stream)) != hipSuccess)
        return e;
    return rt_launch_wide_gather(d_tris_.as<GTri>(), d_slot, d_leaf, d_tri_id_.as<int32_t>(), d_tri_mat_.as<int32_t>(),
                                 (int)nk, tris.as<GTri>(), meta.as<uint4>(), stream);
}

// The risk words' buffer for the resident tree (8 x 8 B words, 8 x 4 B keys and 8 x 24 B boxes per
// node); growing it replaces the buffer, so launches in flight that read it are waited for first.
int Renderer::reserve_risk(size_t nodes)
{
    if (d_wrisk_.bytes >= nodes * 288 + 64)
        return RT_OK;
    if (d_wrisk_.p && (sync_slots() != RT_OK || hipStreamSynchronize(stream_) != hipSuccess))
        return RT_EHIP;
    hipError_t e = d_wrisk_.reserve(nodes * 288 + 64);   // (+ the risk caps)
    return e == hipSuccess ? RT_OK : hip_fail(e, "hipMalloc (risk words)");
}

void Renderer::start_accel()
{
    accel_state_.store(1);
    oc_done_.store(false);
    tree_pending_ = true;
    accel_err_.clear();
    // the origin cones serve the shadow and reflection queries (ocone.hpp)
    const bool want_oc = knobs_.ocone && knobs_.wbvh && !knobs_.exact;
    float S = 0.0f;
    if (oct_nn_ > 0)
        for (int c = 0; c < 3; c++)
            S = std::max(S, std::max(std::fabs(oct_root_.dn[c]), std::fabs(oct_root_.df[c])));
    accel_thread_ = std::thread([this, want_oc, S] {
        using clk = std::chrono::steady_clock;
        auto ms_since = [](clk::time_point t) { return std::chrono::duration<float, std::milli>(clk::now() - t).count(); };
        hipError_t e = hipSetDevice(device_);
        auto t0 = clk::now();
        leaf_cones(oct_, cones_, lslab_, lsin_);
        if (e == hipSuccess && !lslab_.empty()) {
            if ((e = d_lslab_.reserve(lslab_.size() * 4)) == hipSuccess)
                e = hipMemcpyAsync(d_lslab_.p, lslab_.data(), lslab_.size() * 4, hipMemcpyHostToDevice, accel_stream_);
            if (e == hipSuccess && (e = d_lsin_.reserve(lsin_.size() * 4)) == hipSuccess)
                e = hipMemcpyAsync(d_lsin_.p, lsin_.data(), lsin_.size() * 4, hipMemcpyHostToDevice, accel_stream_);
        }
        if (e == hipSuccess && !cones_.empty() && (e = d_cones_.reserve(cones_.size() * 4)) == hipSuccess)
            e = hipMemcpyAsync(d_cones_.p, cones_.data(), cones_.size() * 4, hipMemcpyHostToDevice, accel_stream_);
        accel_ms_[0] = ms_since(t0);
        auto t1 = clk::now();
        if (knobs_.wbvh && !knobs_.exact)
            build_wbvh(oct_, wb_next_);
        else
            wb_next_ = WBvh();
        accel_ms_[1] = ms_since(t1);
        auto t2 = clk::now();
        hipSetDevice(device_);
        if (e == hipSuccess && !wb_next_.nodes.empty())
            e = upload_wide(wb_next_, d_wnodes2_, d_wtris2_, d_wmeta2_, d_wtmp2_, d_wlinks2_, accel_stream_);
        if (e == hipSuccess)
            e = hipStreamSynchronize(accel_stream_);
        accel_ms_[2] = ms_since(t2);
        if (e != hipSuccess)
            accel_err_ = std::string("acceleration structures (upload): ") + hipGetErrorString(e);
        // the origin cones after the tree, which frames may adopt meanwhile (poll_accel): their search
        // reads the tree's nodes and records, copied here, and its device records (resident or not, they
        // live until the next geometry change, which joins this thread first).  Reflection origins lie
        // 0.01 |n| off their hit points (make_frame), shadow origins 1e-4 |n|: the cells within 0.0102 of a
        // triangle.  The host plans, the device searches (ocone_kernel).
        OConeGrid g;
        WBvh w;
        const GTri* wtris = d_wtris2_.as<GTri>();
        if (e == hipSuccess && want_oc && !wb_next_.nodes.empty()) {
            w.nodes = wb_next_.nodes;
            w.tris = wb_next_.tris;
        }
        accel_state_.store(e == hipSuccess ? 2 : 3);
        auto t3 = clk::now();
        OConeJob job;
        if (!w.nodes.empty())
            origin_cones_plan(w, S, W_QS_CLOSEST, 0.0102 + 0x1p-16 * S, knobs_.ocone_dim, 80.0 * 3.14159265358979 / 180.0,
                              g, job);
        w = WBvh();
        if (!job.todo.empty()) {
            // (a failure here only leaves the queries without the cones)
            const size_t ncell = (size_t)g.dim[0] * g.dim[1] * g.dim[2];
            hipError_t eo;
            if ((eo = d_ocone2_.reserve(ncell * sizeof(uint2))) == hipSuccess &&
                (eo = d_oc_ent_.reserve(job.ent.size() * sizeof(OConeEnt))) == hipSuccess &&
                (eo = d_oc_todo_.reserve(job.todo.size() * 4)) == hipSuccess &&
                (eo = hipMemcpyAsync(d_oc_ent_.p, job.ent.data(), job.ent.size() * sizeof(OConeEnt), hipMemcpyHostToDevice,
                                     accel_stream_)) == hipSuccess &&
                (eo = hipMemcpyAsync(d_oc_todo_.p, job.todo.data(), job.todo.size() * 4, hipMemcpyHostToDevice,
                                     accel_stream_)) == hipSuccess &&
                (eo = rt_launch_ocone(d_oc_ent_.as<OConeEnt>(), wtris, d_oc_todo_.as<uint32_t>(), (int)job.todo.size(),
                                      g.lo, g.dim, job.h, job.r, job.slack, job.QS, job.cos_cap, d_ocone2_.as<uint2>(),
                                      ncell, accel_stream_)) == hipSuccess)
                eo = hipStreamSynchronize(accel_stream_);
            if (eo != hipSuccess) {
                g = OConeGrid();
                (void)hipGetLastError();
            }
        }
        ocg_next_ = g;
        oc_ms_ = ms_since(t3);
        oc_done_.store(true);
    });
}

// Adopts a finished background build (wait: blocks until it is, the origin cones included): the SAH
// tree as soon as it is resident, the origin cones when the thread is done.
int Renderer::poll_accel(bool wait)
{
    if (!accel_thread_.joinable())
        return RT_OK;
    if (!wait && accel_state_.load() == 1)
        return RT_OK;
    if (wait || accel_state_.load() == 3 || oc_done_.load()) {
        accel_thread_.join();
        hipSetDevice(device_);
    }
    if (tree_pending_) {
        tree_pending_ = false;
        if (accel_state_.load() == 3) {
            // the SAH tree was not built or uploaded: the resident tree (the quick one, if any) keeps serving
            // frames for this geometry, and rt_stats.wide_tree says so until the next geometry change
            if (accel_thread_.joinable())
                accel_thread_.join();
            accel_state_.store(0);
            wb_next_ = WBvh();
            wide_tree_ = wide_ready_ ? -1 : 0;
            return fail(RT_EHIP, accel_err_);
        }
        cones_ready_ = !cones_.empty();
        lslab_ready_ = !lslab_.empty();
        if (!wb_next_.nodes.empty() || !knobs_.wbvh || knobs_.exact) {
            // the background's tree replaces the resident one (the quick tree, if any): launches in flight
            // keep reading the old buffers, which the next geometry change rewrites only after waiting for them
            std::swap(wb_, wb_next_);
            wb_next_ = WBvh();
            d_wnodes_.swap(d_wnodes2_);
            d_wtris_.swap(d_wtris2_);
            d_wmeta_.swap(d_wmeta2_);
            d_wtmp_.swap(d_wtmp2_);
            d_wlinks_.swap(d_wlinks2_);
        }
        wide_ready_ = !wb_.nodes.empty();
        wide_tree_ = wide_ready_ ? 2 : 0;
        if (wide_ready_ && reserve_risk(wb_.nodes.size()) != RT_OK)
            return RT_EHIP;
        risk_valid_ = false;
        risk_nodes_ = (int64_t)wb_.nodes.size();
        risk_tris_ = (int64_t)wb_.tri_leaf.size();
        ++accel_ver_;
        build_split_ms_[1] = accel_ms_[0];
        build_split_ms_[2] = accel_ms_[1] + accel_ms_[2];
    }
    if (!accel_thread_.joinable()) {   // (joined: the origin cones are done)
        accel_state_.store(0);
        // (the cones describe the geometry, not the tree)
        std::swap(ocg_, ocg_next_);
        ocg_next_ = OConeGrid();
        d_ocone_.swap(d_ocone2_);
        ocone_ready_ = ocg_.computed > 0;
    }
    return RT_OK;
}

int Renderer::finish_accel()
{
    hipError_t e = hipSetDevice(device_);
    if (e != hipSuccess)
        return hip_fail(e, "hipSetDevice");
    return poll_accel(true);
}

// A multi-device helper's scene (rt_set_devices): the lead has built and uploaded the octree
// (render_multi ensures its scene first); the helper copies the lead's device tables to its own
// device instead of building them again, and later the lead's leaf cones / slabs and wide BVH
// once the lead has adopted them.  One host build per geometry change for any number of devices
// (the reference rebuilds once, renderer.cpp:214-224).
int Renderer::adopt_from_lead()
{
    const Renderer& L = *lead_;
    hipError_t e = hipSuccess;
    auto copy = [&](DevBuf& dst, const DevBuf& src, size_t n) {
        if (e != hipSuccess || n == 0)
            return;
        if ((e = dst.reserve(n)) == hipSuccess)
            e = hipMemcpyPeerAsync(dst.p, device_, src.p, L.device_, n, stream_);
    };
    if (geom_dirty_) {
        poll_accel(true);
        cones_ready_ = wide_ready_ = lslab_ready_ = ocone_ready_ = false;
        auto t0 = std::chrono::steady_clock::now();
        oct_ = FlatOctree();   // (never built here)
        oct_nn_ = L.oct_nn_;
        oct_nt_ = L.oct_nt_;
        oct_levels_ = L.oct_levels_;
        oct_root_ = L.oct_root_;
        oct_stats_ = L.oct_stats_;
        has_uv_dev_ = L.has_uv_dev_;
        copy(d_nodes_, L.d_nodes_, (size_t)L.oct_nn_ * sizeof(GNode));
        copy(d_tris_, L.d_tris_, (size_t)L.oct_nt_ * sizeof(GTri));
        copy(d_tri_id_, L.d_tri_id_, (size_t)L.oct_nt_ * 4);
        copy(d_tri_mat_, L.d_tri_mat_, tri_mat_.size() * 4);
        copy(d_tri_uv_, L.d_tri_uv_, L.has_uv_dev_ ? tri_uv_.size() * 4 : 0);
        if (e == hipSuccess)
            e = hipStreamSynchronize(stream_);
        if (e != hipSuccess)
            return hip_fail(e, "rt_set_devices: scene copy from the lead device");
        geom_dirty_ = false;
        tri9_dirty_ = true;
        mir_accel_ = ~0ull;
        build_ms_ = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
        build_split_ms_[0] = build_split_ms_[1] = build_split_ms_[2] = 0.0f;
        build_split_ms_[3] = build_ms_;
    }
    if (mir_accel_ != L.accel_ver_ && mir_geom_ == L.geom_ver_ && !L.geom_dirty_ && (L.cones_ready_ || L.wide_ready_)) {
        const size_t ns = (size_t)L.oct_nt_;
        if (L.cones_ready_) {
            copy(d_cones_, L.d_cones_, 4 * ns * 4);
            if (L.lslab_ready_) {
                copy(d_lslab_, L.d_lslab_, 8 * ns * 4);
                copy(d_lsin_, L.d_lsin_, ns * 4);
            }
        }
        if (L.wide_ready_) {
            copy(d_wnodes_, L.d_wnodes_, L.wb_.nodes.size() * sizeof(WNode));
            copy(d_wtris_, L.d_wtris_, L.wb_.slot.size() * sizeof(GTri));
            copy(d_wmeta_, L.d_wmeta_, L.wb_.slot.size() * 16);
            copy(d_wlinks_, L.d_wlinks_, (L.wb_.tri_leaf.size() + L.wb_.parent.size()) * 4);
            if (e == hipSuccess)
                e = d_wrisk_.reserve(L.wb_.nodes.size() * 288 + 64);
        }
        if (e == hipSuccess)
            e = hipStreamSynchronize(stream_);
        if (e != hipSuccess)
            return hip_fail(e, "rt_set_devices: acceleration structures from the lead device");
        cones_ready_ = L.cones_ready_;
        lslab_ready_ = L.cones_ready_ && L.lslab_ready_;
        wide_ready_ = L.wide_ready_;
        risk_valid_ = false;
        risk_nodes_ = L.risk_nodes_;
        risk_tris_ = L.risk_tris_;
        mir_accel_ = L.accel_ver_;
    }
    return RT_OK;
}

int Renderer::ensure_device_scene()
{
    hipError_t e = hipSetDevice(device_);
    if (e != hipSuccess)
        return hip_fail(e, "hipSetDevice");
    // frames still in flight on other streams read the buffers replaced below
    if ((geom_dirty_ || mats_dirty_ || tex_dirty_) && sync_slots() != RT_OK)
        return RT_EHIP;
    if (lead_) {
        int rc = adopt_from_lead();
        if (rc != RT_OK)
            return rc;
    } else if (geom_dirty_) {
        // a build of the previous geometry reads oct_: let it finish (its result is dropped)
        poll_accel(true);
        cones_ready_ = wide_ready_ = lslab_ready_ = ocone_ready_ = false;
        using clk = std::chrono::steady_clock;
        auto ms_since = [](clk::time_point t) { return std::chrono::duration<float, std::milli>(clk::now() - t).count(); };
        auto t0 = clk::now();
        int64_t n = (int64_t)tri_mat_.size();
        for (float c : tri_)
            if (!std::isfinite(c))
                return fail(RT_EINVAL, "triangle with a non-finite vertex coordinate");
        if (s_.enable_bvh) {
            build_flat_octree(tri_.data(), n, s_.bvh_max_depth, s_.bvh_leaf_object_count, oct_);
            if (oct_.levels > 31)
                return fail(RT_EUNSUPPORTED, "octree deeper than 31 levels");
            if (!oct_.ordered_slabs)
                return fail(RT_EINVAL, "octree volume with d_near > d_far");
        } else {
            // brute-force mode (renderer.cpp:1021-1027): triangles in caller order, no nodes
            oct_ = FlatOctree();
            oct_.tris.resize((size_t)n);
            oct_.tri_id.resize((size_t)n);
            for (int64_t i = 0; i < n; i++) {
                const float* p = tri_.data() + 9 * i;
                v3 a = mk(p[0], p[1], p[2]), b = mk(p[3], p[4], p[5]), c = mk(p[6], p[7], p[8]);
                v3 ab = b - a, ac = c - a, nn = cross(b - a, c - a);
                GTri& g = oct_.tris[(size_t)i];
                g.a[0] = a.x; g.a[1] = a.y; g.a[2] = a.z;
                g.ab[0] = ab.x; g.ab[1] = ab.y; g.ab[2] = ab.z;
                g.ac[0] = ac.x; g.ac[1] = ac.y; g.ac[2] = ac.z;
                g.n[0] = nn.x; g.n[1] = nn.y; g.n[2] = nn.z;
                oct_.tri_id[(size_t)i] = (int32_t)i;
            }
        }
        build_split_ms_[0] = ms_since(t0);
        ++host_builds_;
        oct_nn_ = (int64_t)oct_.nodes.size();
        oct_nt_ = (int64_t)oct_.tris.size();
        oct_levels_ = oct_.levels;
        oct_root_ = oct_nn_ > 0 ? oct_.nodes[0] : GNode{};
        oct_stats_ = oct_.stats;
        has_uv_dev_ = !tri_uv_.empty();
        // the octree and the triangle tables (everything the exact path reads), synchronously
        auto t1 = clk::now();
        size_t nb = oct_.nodes.size() * sizeof(GNode), tb = oct_.tris.size() * sizeof(GTri);
        if ((e = d_nodes_.reserve(nb)) != hipSuccess || (e = d_tris_.reserve(tb)) != hipSuccess ||
            (e = d_tri_id_.reserve(oct_.tri_id.size() * 4)) != hipSuccess ||
            (e = d_tri_mat_.reserve(tri_mat_.size() * 4)) != hipSuccess ||
            (e = d_tri_uv_.reserve(tri_uv_.size() * 4)) != hipSuccess)
            return hip_fail(e, "hipMalloc (scene)");
        hipSetDevice(device_);
        if (nb) e = hipMemcpyAsync(d_nodes_.p, oct_.nodes.data(), nb, hipMemcpyHostToDevice, stream_);
        if (e == hipSuccess && tb) e = hipMemcpyAsync(d_tris_.p, oct_.tris.data(), tb, hipMemcpyHostToDevice, stream_);
        if (e == hipSuccess && !oct_.tri_id.empty())
            e = hipMemcpyAsync(d_tri_id_.p, oct_.tri_id.data(), oct_.tri_id.size() * 4, hipMemcpyHostToDevice, stream_);
        if (e == hipSuccess && !tri_mat_.empty())
            e = hipMemcpyAsync(d_tri_mat_.p, tri_mat_.data(), tri_mat_.size() * 4, hipMemcpyHostToDevice, stream_);
        if (e == hipSuccess && !tri_uv_.empty())
            e = hipMemcpyAsync(d_tri_uv_.p, tri_uv_.data(), tri_uv_.size() * 4, hipMemcpyHostToDevice, stream_);
        // the quick wide BVH (the octree's own hierarchy, O(n): wbvh.hpp build_wbvh_quick) while the octree
        // uploads, resident for the next frames until the SAH tree replaces it
        const bool quick = e == hipSuccess && s_.enable_bvh && knobs_.quick_wbvh && knobs_.wbvh && !knobs_.exact &&
                           oct_nn_ > 0;
        wb_ = WBvh();
        if (quick) {   // (its time counts in build_ms, the blocking part; build_split_ms[2] is the SAH tree's)
            build_wbvh_quick(oct_, wb_, false);   // (records gathered on the device)
            if (!wb_.nodes.empty())
                e = upload_wide(wb_, d_wnodes_, d_wtris_, d_wmeta_, d_wtmp_, d_wlinks_, stream_);
        }
        if (e == hipSuccess)
            e = hipStreamSynchronize(stream_);
        if (e != hipSuccess)
            return hip_fail(e, "upload (scene)");
        build_split_ms_[3] = ms_since(t1);
        geom_dirty_ = false;
        tri9_dirty_ = true;
        build_ms_ = ms_since(t0);
        build_split_ms_[1] = 0.0f;
        wide_tree_ = 0;
        if (!wb_.nodes.empty()) {
            wide_ready_ = true;
            wide_tree_ = 1;
            int rc = reserve_risk(wb_.nodes.size());
            if (rc != RT_OK)
                return rc;
            risk_valid_ = false;
            risk_nodes_ = (int64_t)wb_.nodes.size();
            risk_tris_ = (int64_t)wb_.tri_leaf.size();
            ++accel_ver_;
        }
        build_split_ms_[2] = 0.0f;
        // the leaf cones / slabs and the wide BVH: beside the next frames (RT_ASYNC_ACCEL=0: now)
        if (s_.enable_bvh) {
            start_accel();
            if (!knobs_.async_accel) {
                int rc = poll_accel(true);
                if (rc != RT_OK)
                    return rc;
            }
        } else {
            cones_.clear();
            lslab_.clear();
            lsin_.clear();
            wb_ = WBvh();
        }
    } else {
        int rc = poll_accel(false);
        if (rc != RT_OK)
            return rc;
    }
    if (mats_dirty_) {
        if ((e = d_mats_.reserve(mats_.size() * 4)) != hipSuccess)
            return hip_fail(e, "hipMalloc (materials)");
        if (!mats_.empty() &&
            (e = hipMemcpy(d_mats_.p, mats_.data(), mats_.size() * 4, hipMemcpyHostToDevice)) != hipSuccess)
            return hip_fail(e, "upload (materials)");
        mats_dirty_ = false;
    }
    if (tex_dirty_) {
        for (int i = 0; i < TEX_SLOTS + 6; i++) {
            HostTex& t = i < TEX_SLOTS ? tex_[i] : sky_[i - TEX_SLOTS];
            DevBuf& d = i < TEX_SLOTS ? d_tex_[i] : d_sky_[i - TEX_SLOTS];
            if (t.rgba.empty())
                continue;
            if ((e = d.reserve(t.rgba.size() * 4)) != hipSuccess)
                return hip_fail(e, "hipMalloc (texture)");
            if ((e = hipMemcpy(d.p, t.rgba.data(), t.rgba.size() * 4, hipMemcpyHostToDevice)) != hipSuccess)
                return hip_fail(e, "upload (texture)");
        }
        tex_dirty_ = false;
    }
    return RT_OK;
}

int Renderer::validate() const
{
    // the kernels use the PLANE_N literals: they must be the reference's computed normals
    v3 pn[NPLANES];
    plane_normals(pn);
    for (int i = 0; i < NPLANES; i++)
        if (std::memcmp(&pn[i].x, &PLANE_N[i][0], 4) || std::memcmp(&pn[i].y, &PLANE_N[i][1], 4) ||
            std::memcmp(&pn[i].z, &PLANE_N[i][2], 4))
            return RT_EUNSUPPORTED;
    int nmat = material_count();
    if (s_.shading_method == RT_SHADING) {
        if (!tri_mat_.empty() && (tri_mat_lo_ < 0 || tri_mat_hi_ >= nmat))
            return RT_EINVAL;
        for (int32_t m : shape_mat_)
            if (m < 0 || m >= nmat)
                return RT_EINVAL;
    }
    if (s_.shading_method < 0 || s_.shading_method > 4)
        return RT_EINVAL;
    if ((s_.enable_ao_mapping || s_.shading_method == VISUALIZE_AO) && s_.enable_ao_mapping && tex_[TEX_AO].rgba.empty())
        return RT_EINVAL;
    if (s_.shading_method == RT_SHADING) {
        if (s_.enable_diffuse_mapping && tex_[TEX_DIFFUSE].rgba.empty()) return RT_EINVAL;
        if (s_.enable_normal_mapping && tex_[TEX_NORMAL].rgba.empty()) return RT_EINVAL;
        if (s_.enable_displacement_mapping && (tex_[TEX_DISPLACEMENT].rgba.empty() || s_.parallax_mapping_steps <= 0))
            return RT_EINVAL;
        if (s_.enable_roughness_mapping && tex_[TEX_ROUGHNESS].rgba.empty()) return RT_EINVAL;
    }
    if (s_.enable_skysphere && tex_[TEX_SKYSPHERE].rgba.empty())
        return RT_EINVAL;
    if (!s_.enable_skysphere && s_.enable_skybox)
        for (int i = 0; i < 6; i++)
            if (sky_[i].rgba.empty())
                return RT_EINVAL;
    return RT_OK;
}

static bool any_reflection(const std::vector<float>& mats)
{
    for (size_t i = 0; i + MAT_STRIDE <= mats.size(); i += MAT_STRIDE)
        if (mats[i + 12] > 0.0f)
            return true;
    return false;
}

void Renderer::fill_params(KParams& P) const
{
    std::memset(&P, 0, sizeof(P));
    P.nodes = d_nodes_.as<GNode>();
    P.tris = d_tris_.as<GTri>();
    P.tri_id = d_tri_id_.as<int32_t>();
    P.tri_mat = d_tri_mat_.as<int32_t>();
    P.tri_uv = has_uv_dev_ ? d_tri_uv_.as<float>() : nullptr;
    P.cones = (!cones_ready_ || !knobs_.cones) ? nullptr : d_cones_.as<float>();
    // (the leaf slabs read the cone axis)
    P.lslab = (!P.cones || !lslab_ready_ || !knobs_.lslab) ? nullptr : d_lslab_.as<float>();
    P.lsin = P.lslab ? d_lsin_.as<float>() : nullptr;
    P.scene_scale = 0.0f;
    if (oct_nn_ > 0)
        for (int c = 0; c < 3; c++)
            P.scene_scale = std::max(P.scene_scale, std::max(std::fabs(oct_root_.dn[c]), std::fabs(oct_root_.df[c])));
    // wide BVH: closest-hit queries certified against the octree, when it
    // was built, the scene's scale keeps the certificate's rounding margins (as for the
    // segment queries), and RT_WBVH is not 0
    if (wide_ready_ && knobs_.wbvh && !knobs_.exact && P.scene_scale > 0x1p-20f && P.scene_scale < 0x1p20f) {
        P.wnodes = d_wnodes_.as<WNode>();
        P.wtris = d_wtris_.as<GTri>();
        P.wmeta = d_wmeta_.as<uint4>();
        if (ocone_ready_ && knobs_.ocone) {
            P.ocone.cells = d_ocone_.as<uint2>();
            for (int a = 0; a < 3; a++) {
                P.ocone.lo[a] = ocg_.lo[a];
                P.ocone.dim[a] = ocg_.dim[a];
            }
            P.ocone.ih = ocg_.ih;
        }
    }
    P.nnodes = (int32_t)oct_nn_;
    P.ntri_slots = (int32_t)oct_nt_;
    P.levels = oct_levels_ > 0 ? oct_levels_ : 1;
    P.nshape = (int32_t)shape_kind_.size();
    for (int k = 0; k < P.nshape; k++) {
        P.shape_kind[k] = shape_kind_[k];
        for (int j = 0; j < 6; j++) P.shape[k][j] = shape_[6 * k + j];
        P.shape_mat[k] = shape_mat_[k];
    }
    P.mats = d_mats_.as<float>();
    P.nmat = material_count();
    std::memcpy(P.cam_pos, cam_pos_, sizeof(P.cam_pos));
    std::memcpy(P.proj_inv, proj_inv_, sizeof(P.proj_inv));
    std::memcpy(P.cam_to_world, c2w_, sizeof(P.cam_to_world));
    std::memcpy(P.light, light_, sizeof(P.light));
    {
        // ray generation shortcuts (kparams.hpp): for an image-plane point (x, y, -1) with finite x, y
        // the w row evaluates ((m12 x + m13 y) + m14 (-1)) + m15; with m12 = m13 = 0 that is the
        // constant (-m14) + m15 (the two signed zeros add to a zero that leaves -m14 unchanged when
        // it is nonzero; a zero or non-finite constant keeps the per-pixel path)
        const float* m = proj_inv_;
        bool fin = true;
        for (int i = 0; i < 16; i++) fin = fin && std::isfinite(m[i]);
        P.proj_mode = 0;
        P.proj_w = 1.0f;
        if (fin && m[12] == 0.0f && m[13] == 0.0f && m[14] != 0.0f) {
            volatile float mz = m[14] * -1.0f;   // (volatile: evaluated as the kernel does, in float)
            const float wt = mz + m[15];
            if (std::isfinite(wt) && wt != 0.0f) {
                P.proj_mode = wt == 1.0f ? 1 : 2;
                P.proj_w = 1.0f / wt;
            }
        }
        const float* c = c2w_;
        P.c2w_affine = c[12] == 0.0f && c[13] == 0.0f && c[14] == 0.0f && c[15] == 1.0f;
    }
    for (int i = 0; i < TEX_SLOTS; i++) {
        P.tex[i].px = tex_[i].rgba.empty() ? nullptr : d_tex_[i].as<float4>();
        P.tex[i].w = tex_[i].w;
        P.tex[i].h = tex_[i].h;
    }
    for (int i = 0; i < 6; i++) {
        P.sky[i].px = sky_[i].rgba.empty() ? nullptr : d_sky_[i].as<float4>();
        P.sky[i].w = sky_[i].w;
        P.sky[i].h = sky_[i].h;
    }
    P.shading_method = s_.shading_method;
    P.compute_shadows = s_.compute_shadows;
    P.max_recursion_depth = s_.max_recursion_depth;
    P.enable_bvh = s_.enable_bvh;
    P.enable_ambient = s_.enable_ambient;
    P.enable_diffuse = s_.enable_diffuse;
    P.enable_specular = s_.enable_specular;
    P.enable_emissive = s_.enable_emissive;
    P.rough_reflections_sample_count = s_.rough_reflections_sample_count;
    P.enable_ao_mapping = s_.enable_ao_mapping;
    P.enable_diffuse_mapping = s_.enable_diffuse_mapping;
    P.enable_normal_mapping = s_.enable_normal_mapping;
    P.enable_displacement_mapping = s_.enable_displacement_mapping;
    P.displacement_mapping_strength = s_.displacement_mapping_strength;
    P.parallax_mapping_steps = s_.parallax_mapping_steps;
    P.enable_roughness_mapping = s_.enable_roughness_mapping;
    P.enable_skysphere = s_.enable_skysphere;
    P.enable_skybox = s_.enable_skybox;
    P.rng_seed = s_.rng_seed;
    P.has_reflection = s_.shading_method == RT_SHADING && any_reflection(mats_);
    // segment queries (RT_SEG=0 turns them off): only when the
    // queries' results depend on the triangles alone (analytic shapes read the stale
    // record) and the scene's scale keeps Moller-Trumbore's products far from overflow
    // and underflow, so that the rounding bound of seg_margin holds
    P.seg_scale = 0.0f;
    P.seg_oct = knobs_.seg_oct ? 1 : 0;
    if (knobs_.seg && !knobs_.exact && P.nshape == 0 && oct_nn_ > 0) {
        const GNode& root = oct_root_;
        float S = 0.0f;
        for (int a = 0; a < 3; a++)   // the axis slabs are the vertices' coordinate range
            S = std::max(S, std::max(std::fabs(root.dn[a]), std::fabs(root.df[a])));
        if (S > 0x1p-20f && S < 0x1p20f)
            P.seg_scale = S;
    }
    P.max_blocks = num_cus_ * 8;   // persistent grids: 8 blocks per CU (the plain kernel: its residency)
    // the plain specialisation (RT_PLAIN=0 turns it off); SSAO (zbuf) is checked at launch
    P.plain = knobs_.plain && P.enable_bvh && (P.wnodes || knobs_.plain_octree) && P.shading_method == RT_SHADING && P.nshape == 0 &&
              !P.enable_ao_mapping && !P.enable_diffuse_mapping && !P.enable_normal_mapping &&
              !P.enable_displacement_mapping && !P.enable_skysphere && !P.enable_skybox && !P.has_reflection;
    render_size(P.rw, P.rh);
}


// The trace of one launch (ray_trace / render_bands_device).  Reflective scenes
// with the BVH run the reflection engine (kernels.hip, "Reflections as frames"):
// level 0 shades every primary hit and turns the reflective ones into frames; each
// level then traces its frames' samples in chunks, depth-first over chunks.
// RT_REFL_ENGINE=0 selects the one-lane-per-pixel recursive kernel instead.
int Renderer::launch_trace(const KParams& P, hipStream_t stream)
{
    hipError_t e;
    const bool engine = P.has_reflection && P.enable_bvh && knobs_.refl_engine;
    if (!engine) {
        if ((e = rt_launch_ray_trace(&P, stream)) != hipSuccess)
            return hip_fail(e, "ray_trace_kernel launch");
        return RT_OK;
    }
    for (auto& L : refl_)
        L.fr.device = L.ret.device = L.sm.device = L.hit.device = L.cnt.device = L.list.device = L.sort.device =
            L.sort_tmp.device = L.res.device = L.sdefer.device = L.frs.device = L.slist.device = device_;
    size_t npx = (size_t)P.rw * P.local_rows;
    ReflLevel& L1 = refl_[1];
    if ((e = L1.fr.reserve(npx * sizeof(FrameRec))) != hipSuccess || (e = L1.cnt.reserve(64)) != hipSuccess)
        return hip_fail(e, "hipMalloc (reflection frames)");
    if ((e = hipMemsetAsync(L1.cnt.p, 0, 4, stream)) != hipSuccess)
        return hip_fail(e, "hipMemsetAsync");
    if ((e = rt_launch_refl_level0(&P, L1.fr.as<FrameRec>(), L1.cnt.as<unsigned int>(), stream)) != hipSuccess)
        return hip_fail(e, "refl_level0_kernel launch");
    unsigned n1 = 0;
    if ((e = hipMemcpyAsync(&n1, L1.cnt.p, 4, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
        (e = hipStreamSynchronize(stream)) != hipSuccess)
        return hip_fail(e, "refl_level0_kernel");
    return refl_level(P, 1, (int)n1, stream);
}

// Frames [0, nframes) of 'level' (their samples trace at depth 'level'), in chunks;
// each chunk's child frames are resolved (recursively) before its own resolve.
int Renderer::refl_level(const KParams& P, int level, int nframes, hipStream_t stream)
{
    const int N = P.rough_reflections_sample_count;
    const int stride = N > 0 ? N : 1;
    if (level + 1 >= REFL_LEVELS)
        return fail(RT_EUNSUPPORTED, "reflection recursion deeper than the engine's levels");
    ReflLevel& L = refl_[level];
    ReflLevel& C = refl_[level + 1];
    hipError_t e;
    // about 2^RT_REFL_CHUNK_LOG2 sample slots per chunk (default 2^27: C5 1,757 / 1,841 / 1,902 / 1,927
    // Mrays/s at 2^24 / 2^25 / 2^26 / 2^27, r05; r02: 0.765 / 0.714 / 0.695 / 0.679 s at 2^21 / 2^23 /
    // 2^24 / 2^25): one host round trip per chunk, ~204 B of records per
    // slot (72-B SampleRec, 32-B RawHit, 16-B result, list entry, child frame and its colour).
    // A level may take at most a quarter of the memory still free (what it already holds
    // counts as free), so that the deeper levels, each bounded the same way, fit behind it;
    // an allocation that fails anyway halves the chunk and retries.
    constexpr size_t SLOT_BYTES = sizeof(SampleRec) + sizeof(RawHit) + 4 + 4 + 16 + sizeof(FrameRec) + 12 + 16;
    size_t chunk = (size_t)std::max(1024, (1 << knobs_.refl_chunk_log2) / stride);
    {
        size_t freeb = 0, totalb = 0;
        if (hipMemGetInfo(&freeb, &totalb) == hipSuccess) {
            const size_t held =
                L.sm.bytes + L.hit.bytes + L.list.bytes + L.sdefer.bytes + L.res.bytes + L.frs.bytes + L.slist.bytes + C.fr.bytes +
                C.ret.bytes;
            const size_t cap = (freeb + held) / 4 / (SLOT_BYTES * (size_t)stride);
            chunk = std::max<size_t>(1024, std::min(chunk, cap));
        }
    }
    if ((e = L.ret.reserve((size_t)nframes * 12)) != hipSuccess || (e = L.cnt.reserve(64)) != hipSuccess)
        return hip_fail(e, "hipMalloc (reflection level)");
    for (;;) {
        const size_t slots = std::min((size_t)nframes, chunk) * stride;
        if ((e = L.sm.reserve(slots * sizeof(SampleRec))) == hipSuccess &&
            (e = L.hit.reserve(slots * sizeof(RawHit))) == hipSuccess && (e = L.list.reserve(slots * 4)) == hipSuccess &&
            (e = L.sdefer.reserve(slots * 4)) == hipSuccess && (e = L.res.reserve(slots * 16)) == hipSuccess &&
            (e = C.fr.reserve(slots * sizeof(FrameRec))) == hipSuccess &&
            (e = C.ret.reserve(slots * 12)) == hipSuccess &&
            (!(knobs_.refl_shadow_sort || knobs_.refl_dir_sort || knobs_.refl_defer_sort) || (e = L.slist.reserve(slots * 16)) == hipSuccess))
            break;
        if (e != hipErrorOutOfMemory || chunk <= 1024)
            return hip_fail(e, "hipMalloc (reflection level)");
        (void)hipGetLastError();   // clear the sticky out-of-memory status
        chunk /= 2;
    }
    // the level's frames in Morton order of their origins (coherent sample and shadow rays)
    if ((e = L.sort.reserve((size_t)nframes * 16)) != hipSuccess)
        return hip_fail(e, "hipMalloc (frame sort)");
    uint32_t* keys_in = L.sort.as<uint32_t>();
    uint32_t* keys_out = keys_in + nframes;
    int32_t* idx_in = reinterpret_cast<int32_t*>(keys_out + nframes);
    int32_t* idx_out = idx_in + nframes;
    if ((e = rt_launch_refl_keys(&P, L.fr.as<FrameRec>(), nframes, keys_in, idx_in, stream)) != hipSuccess)
        return hip_fail(e, "refl_keys_kernel launch");
    const int32_t* order = idx_in;
    if (knobs_.refl_sort) {
        size_t tb = 0;
        if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, keys_in, keys_out, idx_in, idx_out, nframes, 0, 30,
                                                    stream)) != hipSuccess ||
            (e = L.sort_tmp.reserve(tb)) != hipSuccess ||
            (e = hipcub::DeviceRadixSort::SortPairs(L.sort_tmp.p, tb, keys_in, keys_out, idx_in, idx_out, nframes, 0,
                                                    30, stream)) != hipSuccess)
            return hip_fail(e, "frame sort");
        order = idx_out;
    }
    // the frames in sorted order, copied once per level (the passes below walk the sorted positions)
    const FrameRec* frs = nullptr;
    if (knobs_.refl_sorted_frames) {
        if ((e = L.frs.reserve((size_t)nframes * sizeof(FrameRec))) != hipSuccess ||
            (e = rt_launch_refl_sort_frames(L.fr.as<FrameRec>(), order, nframes, L.frs.as<FrameRec>(), stream)) != hipSuccess)
            return hip_fail(e, "refl_sort_frames_kernel");
        frs = L.frs.as<FrameRec>();
    }
    for (int c0 = 0; c0 < nframes; c0 += (int)chunk) {
        ReflArgs A;
        A.order = order;
        A.frs = frs;
        A.perm = nullptr;
        A.feed_parts = knobs_.refl_feed_xcd ? L.cnt.as<unsigned int>() + 8 : nullptr;
        A.fr = L.fr.as<FrameRec>();
        A.sm = L.sm.as<SampleRec>();
        A.hit = L.hit.as<RawHit>();
        A.ret = L.ret.as<float>();
        A.child_ret = C.ret.as<float>();
        A.child_fr = C.fr.as<FrameRec>();
        A.child_count = L.cnt.as<unsigned int>();
        A.list = L.list.as<int32_t>();
        A.res = L.res.as<float4>();
        A.list_count = L.cnt.as<unsigned int>() + 1;
        A.c0 = c0;
        A.c1 = (int)std::min<size_t>((size_t)nframes, (size_t)c0 + chunk);
        A.level = level;
        A.stride = stride;
        A.sample_major = knobs_.refl_sample_major ? 1 : 0;
        A.feed_frame_order = knobs_.refl_feed_frame_order ? 1 : 0;
        // long queries (more than max_steps loop iterations) leave the trace kernel's waves and are
        // traced again by stage 7 in waves of their own (the shadow list's buffer, free until pass1;
        // RT_REFL_DEFER=0: off)
        A.defer = L.list.as<int32_t>();
        A.defer_count = L.cnt.as<unsigned int>() + 2;
        A.max_steps = knobs_.refl_defer;
        // lane refill (kernels.hip refl_trace_feed_kernel; RT_REFL_FEED=k: refill at k waiting lanes, 0: off)
        A.feed = knobs_.refl_feed;
        A.feed_ticket = L.cnt.as<unsigned int>() + 4;
        // the shadow pass's lane refill (refl_shadow_feed_kernel; RT_REFL_SHADOW_FEED=k, 0: off)
        A.shadow_feed = knobs_.refl_shadow_feed;
        A.shadow_ticket = L.cnt.as<unsigned int>() + 5;
        A.sdefer = L.sdefer.as<int32_t>();
        A.sdefer_count = L.cnt.as<unsigned int>() + 6;
        if ((e = hipMemsetAsync(L.cnt.p, 0, 64, stream)) != hipSuccess)   // (+ the long kernel's and the feeds' counters)
            return hip_fail(e, "hipMemsetAsync");
        // fused (default): trace, pass1 (+ shadow list), shadow (+ spawn); RT_REFL_FUSE=0: trace,
        // pass1, list, shadow, spawn
        A.fused = knobs_.refl_fuse;
        static const int fused_stages[] = {1, 7, 2, 3}, split_stages[] = {1, 7, 2, 6, 3, 4};
        const int* st = A.fused ? fused_stages : split_stages;
        const int nst = A.fused ? 4 : 6;
        if (knobs_.refl_dir_sort && A.fused && A.feed > 0) {
            // the feed's tickets over the slots grouped by direction bin (a stable sort: the frames' order
            // inside each bin); the buffer is free again once the feed is done (the shadow sort reuses it)
            const int n = (A.c1 - A.c0) * A.stride;
            uint32_t* kin = L.slist.as<uint32_t>();
            uint32_t* kout = kin + n;
            int32_t* vin = reinterpret_cast<int32_t*>(kout + n);
            int32_t* vout = vin + n;
            size_t tb = 0;
            if ((e = rt_launch_refl_dir_keys(&P, &A, kin, vin, stream)) != hipSuccess ||
                (e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kin, kout, vin, vout, n, 0, 7, stream)) != hipSuccess ||
                (e = L.sort_tmp.reserve(tb)) != hipSuccess ||
                (e = hipcub::DeviceRadixSort::SortPairs(L.sort_tmp.p, tb, kin, kout, vin, vout, n, 0, 7, stream)) !=
                    hipSuccess)
                return hip_fail(e, "feed direction sort");
            A.perm = vout;
        }
        for (int k = 0; k < nst; k++) {
            if (st[k] == 7 && knobs_.refl_defer_sort) {
                // the deferred queries in their frames' (Morton) order: a wave's lane groups start from nearby
                // origins (each query's result does not depend on its place in the list)
                unsigned n = 0;
                if ((e = hipMemcpyAsync(&n, A.defer_count, 4, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
                    (e = hipStreamSynchronize(stream)) != hipSuccess)
                    return hip_fail(e, "deferred query count");
                if (n > 1) {
                    int bits = 1;
                    while (bits < 31 && (1u << bits) < (unsigned)(A.c1 - A.c0))
                        bits++;
                    uint32_t* kin = L.slist.as<uint32_t>();
                    uint32_t* kout = kin + n;
                    int32_t* vout = reinterpret_cast<int32_t*>(kout + n);
                    size_t tb = 0;
                    if ((e = rt_launch_refl_defer_keys(&A, (int)n, kin, stream)) != hipSuccess ||
                        (e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kin, kout, A.defer, vout, (int)n, 0, bits,
                                                                stream)) != hipSuccess ||
                        (e = L.sort_tmp.reserve(tb)) != hipSuccess ||
                        (e = hipcub::DeviceRadixSort::SortPairs(L.sort_tmp.p, tb, kin, kout, A.defer, vout, (int)n, 0, bits,
                                                                stream)) != hipSuccess)
                        return hip_fail(e, "deferred query sort");
                    A.defer = vout;
                }
            }
            if (st[k] == 3 && A.fused && knobs_.refl_shadow_sort && P.compute_shadows) {
                // the shadow list sorted by hit point (Morton order): the shadow pass's adjacent lanes start
                // from nearby points (its entries' results do not depend on their order)
                unsigned n = 0;
                if ((e = hipMemcpyAsync(&n, A.list_count, 4, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
                    (e = hipStreamSynchronize(stream)) != hipSuccess)
                    return hip_fail(e, "shadow list count");
                if (n > 1) {
                    uint32_t* kin = L.slist.as<uint32_t>();
                    uint32_t* kout = kin + n;
                    int32_t* vout = reinterpret_cast<int32_t*>(kout + n);
                    size_t tb = 0;
                    if ((e = rt_launch_refl_shadow_keys(&P, A.sm, A.list, (int)n, kin, stream)) != hipSuccess ||
                        (e = hipcub::DeviceRadixSort::SortPairs(nullptr, tb, kin, kout, A.list, vout, (int)n, 0, 30,
                                                                stream)) != hipSuccess ||
                        (e = L.sort_tmp.reserve(tb)) != hipSuccess ||
                        (e = hipcub::DeviceRadixSort::SortPairs(L.sort_tmp.p, tb, kin, kout, A.list, vout, (int)n, 0, 30,
                                                                stream)) != hipSuccess)
                        return hip_fail(e, "shadow list sort");
                    A.list = vout;
                }
            }
            if ((e = rt_launch_refl_stage(st[k], &P, &A, stream)) != hipSuccess)
                return hip_fail(e, "reflection stage launch");
        }
        unsigned nchild = 0;
        if ((e = hipMemcpyAsync(&nchild, L.cnt.p, 4, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
            (e = hipStreamSynchronize(stream)) != hipSuccess)
            return hip_fail(e, "reflection stages");
        if (nchild > 0) {
            int rc = refl_level(P, level + 1, (int)nchild, stream);
            if (rc != RT_OK)
                return rc;
        }
        if ((e = rt_launch_refl_stage(5, &P, &A, stream)) != hipSuccess)
            return hip_fail(e, "refl_resolve_kernel launch");
    }
    return RT_OK;
}

// The raster path: raster_trace (renderer.cpp:869-1006) for one launch (whole frame or
// this rank's bands).  Every triangle is clipped (clip_triangle, :833-854) into pieces
// numbered in (triangle, piece) order; the pieces' covered samples race for each pixel
// through a 64-bit atomicMin of (order-preserving z, piece index), which is the
// sequential z-test's winner (strict <: the first of equal z wins); then every pixel is
// shaded from its winning piece, and reflective hits go through the frame engine.
int Renderer::launch_raster(const KParams& P, hipStream_t stream)
{
    hipError_t e;
    const int64_t n = (int64_t)tri_mat_.size();
    if (tri9_dirty_) {
        if ((e = d_tri9_.reserve(tri_.size() * 4)) != hipSuccess) return hip_fail(e, "hipMalloc (raster triangles)");
        if (!tri_.empty() &&
            (e = hipMemcpyAsync(d_tri9_.p, tri_.data(), tri_.size() * 4, hipMemcpyHostToDevice, stream)) != hipSuccess)
            return hip_fail(e, "upload (raster triangles)");
        tri9_dirty_ = false;
    }
    RasterArgs A;
    std::memset(&A, 0, sizeof(A));
    A.tri9 = d_tri9_.as<float>();
    A.ntri = n;
    std::memcpy(A.proj, proj_, sizeof(A.proj));
    std::memcpy(A.w2c, w2c_, sizeof(A.w2c));
    A.clipping = s_.enable_clipping;
    if ((e = d_rcount_.reserve((size_t)(n + 1) * 4)) != hipSuccess || (e = d_roff_.reserve((size_t)(n + 1) * 4)) != hipSuccess)
        return hip_fail(e, "hipMalloc (raster counts)");
    A.count = d_rcount_.as<int32_t>();
    A.offset = d_roff_.as<int32_t>();
    if ((e = hipMemsetAsync(A.count, 0, (size_t)(n + 1) * 4, stream)) != hipSuccess) return hip_fail(e, "hipMemsetAsync");
    if ((e = rt_launch_raster_stage(0, &P, &A, 0, stream)) != hipSuccess) return hip_fail(e, "raster_count_kernel launch");
    size_t tb = 0;
    if ((e = hipcub::DeviceScan::ExclusiveSum(nullptr, tb, A.count, d_roff_.as<int32_t>(), (int)(n + 1), stream)) !=
            hipSuccess ||
        (e = d_scan_tmp_.reserve(tb)) != hipSuccess ||
        (e = hipcub::DeviceScan::ExclusiveSum(d_scan_tmp_.p, tb, A.count, d_roff_.as<int32_t>(), (int)(n + 1),
                                              stream)) != hipSuccess)
        return hip_fail(e, "piece scan");
    int32_t npieces = 0;
    if ((e = hipMemcpyAsync(&npieces, d_roff_.as<int32_t>() + n, 4, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
        (e = hipStreamSynchronize(stream)) != hipSuccess)
        return hip_fail(e, "raster_count_kernel");
    size_t npx = (size_t)P.rw * P.local_rows;
    if ((e = d_pieces_.reserve((size_t)npieces * sizeof(RasterPiece))) != hipSuccess ||
        (e = d_piece_uv_.reserve((size_t)npieces * 24)) != hipSuccess ||
        (e = d_big_.reserve((size_t)npieces * 4 + 64)) != hipSuccess || (e = d_zkey_.reserve(npx * 8)) != hipSuccess)
        return hip_fail(e, "hipMalloc (raster pieces)");
    A.pieces = d_pieces_.as<RasterPiece>();
    A.piece_uv = d_piece_uv_.as<float>();
    A.zkey = d_zkey_.as<unsigned long long>();
    A.nbig = d_big_.as<unsigned int>();
    A.big = d_big_.as<int32_t>() + 16;
    if ((e = hipMemsetAsync(A.zkey, 0xff, npx * 8, stream)) != hipSuccess ||
        (e = hipMemsetAsync(A.nbig, 0, 4, stream)) != hipSuccess)
        return hip_fail(e, "hipMemsetAsync");
    for (int stage = 1; stage <= 3; stage++)
        if ((e = rt_launch_raster_stage(stage, &P, &A, npieces, stream)) != hipSuccess)
            return hip_fail(e, "raster kernel launch");
    // shading reads texcoords through Rec::tri = piece index: the piece table stands in
    // for tri_uv (trace_triangle's temporary Triangle carries the clipped texcoords)
    KParams PS = P;
    PS.tri_uv = A.piece_uv;
    for (auto& L : refl_)
        L.fr.device = L.ret.device = L.sm.device = L.hit.device = L.cnt.device = L.list.device = L.sort.device =
            L.sort_tmp.device = L.res.device = L.sdefer.device = L.frs.device = L.slist.device = device_;
    ReflLevel& L1 = refl_[1];
    const bool frames = P.has_reflection;
    if (frames) {
        if ((e = L1.fr.reserve(npx * sizeof(FrameRec))) != hipSuccess || (e = L1.cnt.reserve(64)) != hipSuccess)
            return hip_fail(e, "hipMalloc (reflection frames)");
        if ((e = hipMemsetAsync(L1.cnt.p, 0, 4, stream)) != hipSuccess) return hip_fail(e, "hipMemsetAsync");
    }
    if ((e = rt_launch_raster_shade(&PS, &A, frames ? L1.fr.as<FrameRec>() : nullptr,
                                    frames ? L1.cnt.as<unsigned int>() : nullptr, stream)) != hipSuccess)
        return hip_fail(e, "raster_shade_kernel launch");
    if (!frames)
        return RT_OK;
    unsigned n1 = 0;
    if ((e = hipMemcpyAsync(&n1, L1.cnt.p, 4, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
        (e = hipStreamSynchronize(stream)) != hipSuccess)
        return hip_fail(e, "raster_shade_kernel");
    return n1 ? refl_level(P, 1, (int)n1, stream) : RT_OK;
}

// the checks ray_trace / raster_trace / render_bands_device make before a launch
int Renderer::check_frame() const
{
    if (s_.shading_method == RT_SHADING && any_reflection(mats_) && s_.max_recursion_depth > 15)
        return RT_EUNSUPPORTED;
    if (s_.hybrid_rasterization_tracing) {
        if (tri_mat_.size() >= ((size_t)1 << 27))
            return RT_EUNSUPPORTED;   // 12 pieces per triangle must index in 31 bits
        if (s_.shading_method == RT_SHADING && any_reflection(mats_) && !s_.enable_bvh)
            return RT_EUNSUPPORTED;   // the frame engine traces through the octree
    }
    return RT_OK;
}

// Renderer::ray_trace, renderer.cpp:1068-1116
int Renderer::ray_trace()
{
    rt_settings keep = s_;
    s_.hybrid_rasterization_tracing = 0;
    int rc = trace_frame();
    s_.hybrid_rasterization_tracing = keep.hybrid_rasterization_tracing;
    return rc;
}

int Renderer::raster_trace()
{
    rt_settings keep = s_;
    s_.hybrid_rasterization_tracing = 1;
    int rc = trace_frame();
    s_.hybrid_rasterization_tracing = keep.hybrid_rasterization_tracing;
    return rc;
}

int Renderer::trace_frame()
{
    if (validate() != RT_OK)
        return fail(RT_EINVAL, "invalid scene: material index out of range or enabled texture map missing");
    if (check_frame() != RT_OK)
        return fail(RT_EUNSUPPORTED, "reflective materials with max_recursion_depth > 15, a raster frame with "
                                     "reflections and no BVH, or more than 2^27 triangles to rasterise");
    int rc = ensure_device_scene();
    if (rc != RT_OK)
        return rc;
    KParams P;
    fill_params(P);
    last_seg_ = P.seg_scale;
    size_t npx = (size_t)P.rw * P.rh;
    hipError_t e;
    if ((e = d_counters_.reserve(NCOUNTER_WORDS * 8)) != hipSuccess)
        return hip_fail(e, "hipMalloc (counters)");
    // the image state before this frame: restored if the frame fails after the image became its
    // internal buffer (a partly written frame is never presented; when the previous image was that
    // same buffer, its content is gone and the image reads as not rendered)
    const int prev_w = img_w_, prev_h = img_h_;
    const bool prev_internal = img_is_internal_, prev_rendered = rendered_;
    if ((rc = begin_internal_image(P.rw, P.rh)) != RT_OK)
        return rc;
    struct Restore {
        Renderer* r;
        int w, h;
        bool internal, rendered, armed = true;
        ~Restore()
        {
            if (!armed)
                return;
            std::lock_guard<std::recursive_mutex> g(r->image_mu_);
            r->img_w_ = w;
            r->img_h_ = h;
            r->img_is_internal_ = internal;
            r->rendered_ = rendered && !internal;
        }
    } restore{this, prev_w, prev_h, prev_internal, prev_rendered};
    if (knobs_.inject_fail > 0 && ++frames_started_ == knobs_.inject_fail)
        return fail(RT_EHIP, "injected frame failure (RT_INJECT_FRAME_FAIL)");
    if (want_rgba_ && (e = d_rgba_.reserve(npx * 16)) != hipSuccess) return hip_fail(e, "hipMalloc (rgba)");
    if (want_hit_ && ((e = d_hit_id_.reserve(npx * 4)) != hipSuccess || (e = d_hit_t_.reserve(npx * 4)) != hipSuccess))
        return hip_fail(e, "hipMalloc (hit)");
    if (want_shadow_ && (e = d_shadow_.reserve(npx)) != hipSuccess) return hip_fail(e, "hipMalloc (shadow)");
    if (s_.enable_ssao && ((e = d_zbuf_.reserve(npx * 4)) != hipSuccess || (e = d_nbuf_.reserve(npx * 16)) != hipSuccess))
        return hip_fail(e, "hipMalloc (z / normal buffers)");
    P.zbuf = s_.enable_ssao ? d_zbuf_.as<float>() : nullptr;
    P.nbuf = s_.enable_ssao ? d_nbuf_.as<float4>() : nullptr;
    P.band_rows = P.rh;
    P.nranks = 1;
    P.rank = 0;
    P.local_rows = P.rh;
    P.tiles_x = (P.rw + 7) / 8;
    P.tiles_y = (P.rh + 7) / 8;
    P.argb = d_internal_.as<uint32_t>();
    P.rgba = want_rgba_ ? d_rgba_.as<float4>() : nullptr;
    P.hit_id = want_hit_ ? d_hit_id_.as<int32_t>() : nullptr;
    P.hit_t = want_hit_ ? d_hit_t_.as<float>() : nullptr;
    P.shadow = want_shadow_ ? d_shadow_.as<uint8_t>() : nullptr;
    P.counters = d_counters_.as<unsigned long long>();
    if (knobs_.debug_waves) {   // diagnostic builds: per-wave records (rt_debug_read)
        if ((e = d_dbg_.reserve((size_t)DBG_WAVES * DBG_WORDS * 8)) != hipSuccess ||
            (e = hipMemsetAsync(d_dbg_.p, 0, (size_t)DBG_WAVES * DBG_WORDS * 8, stream_)) != hipSuccess)
            return hip_fail(e, "debug buffer");
        P.dbg = d_dbg_.as<unsigned long long>();
    }
    if (wait_slots(stream_) != RT_OK)   // band launches in flight share the engine / raster buffers
        return RT_EHIP;
    if ((rc = prepare_risk(P, stream_)) != RT_OK)
        return rc;
    bool zeroed = false;   // heavy_prep_kernel clears the counter words itself
    if ((rc = prepare_heavy(P, tc_main_, stream_, 0, &zeroed)) != RT_OK)
        return rc;
    if (!zeroed && (e = hipMemsetAsync(d_counters_.p, 0, NCOUNTER_WORDS * 8, stream_)) != hipSuccess)
        return hip_fail(e, "hipMemsetAsync");
    hipEventRecord(ev_[0], stream_);
    if ((rc = launch_frame(P, stream_)) != RT_OK) return rc;
    hipEventRecord(ev_[1], stream_);
    unsigned long long cnt[NCOUNTERS] = {};
    if ((e = hipMemcpyAsync(cnt, d_counters_.p, sizeof(cnt), hipMemcpyDeviceToHost, stream_)) != hipSuccess)
        return hip_fail(e, "counters");
    if ((e = hipStreamSynchronize(stream_)) != hipSuccess) return hip_fail(e, "ray_trace_kernel");
    hipEventElapsedTime(&kernel_ms_, ev_[0], ev_[1]);
    last_primary_ = (int64_t)npx;
    take_counters(cnt);
    aux_valid_ = true;
    ssao_ready_ = s_.enable_ssao;
    post_ms_ = 0;
    restore.armed = false;
    return RT_OK;
}

// Renderer::post_process / apply_ssaa, renderer.cpp:1118-1135
int Renderer::post_process()
{
    if (!rendered_)
        return fail(RT_ESTATE, "post_process before ray_trace");
    if (!img_is_internal_)
        return RT_OK;
    hipError_t e = hipSetDevice(device_);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    post_ms_ = 0;
    if (s_.enable_ssao) {
        if (!ssao_ready_)
            return fail(RT_ESTATE, "post_process: enable_ssao but the last frame was rendered without it");
        int rc = launch_ssao();
        if (rc != RT_OK)
            return rc;
    }
    if (!s_.enable_ssaa)
        return RT_OK;
    int f = s_.ssaa_factor;
    if (img_w_ % f != 0 || img_h_ % f != 0)
        return RT_OK;   // downscale_image_qt_ARGB32 prints and leaves the output untouched
    int dw = img_w_ / f, dh = img_h_ / f;
    {
        std::lock_guard<std::recursive_mutex> g(image_mu_);
        if ((e = d_image_.reserve((size_t)dw * dh * 4)) != hipSuccess) return hip_fail(e, "hipMalloc (ssaa)");
    }
    hipEventRecord(ev_[2], stream_);
    if ((e = rt_launch_downscale(d_internal_.as<uint32_t>(), img_w_, img_h_, f, d_image_.as<uint32_t>(), stream_)) !=
        hipSuccess)
        return hip_fail(e, "downscale launch");
    hipEventRecord(ev_[3], stream_);
    if ((e = hipStreamSynchronize(stream_)) != hipSuccess) return hip_fail(e, "downscale");
    float ms = 0;
    hipEventElapsedTime(&ms, ev_[2], ev_[3]);
    post_ms_ += ms;
    std::lock_guard<std::recursive_mutex> g(image_mu_);   // apply_ssaa's swap under _image_mutex (:1132-1134)
    img_w_ = dw;
    img_h_ = dh;
    img_is_internal_ = false;
    return RT_OK;
}

// Renderer::post_process_ssao_SIMD (renderer.cpp:1229-1434) on the internal image,
// from the z / normal buffers of the last frame.  The two tangents come from the
// host libm exactly as the reference evaluates them: the SIMD loop's double tan
// (renderer.cpp:1245) and the scalar tail's tanf(radians(fov / 2)) (:1379).
int Renderer::launch_ssao()
{
    hipError_t e;
    size_t npx = (size_t)img_w_ * img_h_;
    if ((e = d_ao_.reserve(npx * 4)) != hipSuccess) return hip_fail(e, "hipMalloc (ssao)");
    SsaoArgs A;
    std::memset(&A, 0, sizeof(A));
    A.z = d_zbuf_.as<float>();
    A.n = d_nbuf_.as<float4>();
    A.ao = d_ao_.as<int32_t>();
    A.argb = d_internal_.as<uint32_t>();
    A.w = img_w_;
    A.h = img_h_;
    A.simd_w = img_w_ - img_w_ % 8;
    A.count = s_.ssao_sample_count;
    A.radius = s_.ssao_radius;
    A.amount = s_.ssao_amount;
    const double pi = 3.14159265358979323846;
    A.fovm = (float)std::tan(fov_ / 2 / 180 * pi);
    A.tanv = std::tan(((float)pi / 180) * (fov_ / 2));
    A.aspect = aspect_;
    A.seed = s_.rng_seed;
    std::memcpy(A.proj, proj_, sizeof(A.proj));
    hipEventRecord(ev_[2], stream_);
    if ((e = rt_launch_ssao(&A, stream_)) != hipSuccess) return hip_fail(e, "ssao launch");
    hipEventRecord(ev_[3], stream_);
    if ((e = hipStreamSynchronize(stream_)) != hipSuccess) return hip_fail(e, "ssao");
    float ms = 0;
    hipEventElapsedTime(&ms, ev_[2], ev_[3]);
    post_ms_ += ms;
    return RT_OK;
}

int Renderer::get_ssao_buffers(float* z, float* n4, int32_t* ao)
{
    if (!ssao_ready_)
        return fail(RT_ESTATE, "get_ssao_buffers: the last frame was rendered without enable_ssao");
    hipSetDevice(device_);
    int rw, rh;
    render_size(rw, rh);
    size_t n = (size_t)rw * rh;
    hipError_t e = hipSuccess;
    if (z) e = hipMemcpy(z, d_zbuf_.p, n * 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess && n4) e = hipMemcpy(n4, d_nbuf_.p, n * 16, hipMemcpyDeviceToHost);
    if (e == hipSuccess && ao) {
        if (d_ao_.bytes < n * 4) return fail(RT_ESTATE, "get_ssao_buffers: no SSAO pass yet (post_process)");
        e = hipMemcpy(ao, d_ao_.p, n * 4, hipMemcpyDeviceToHost);
    }
    if (e != hipSuccess) return hip_fail(e, "get_ssao_buffers");
    return RT_OK;
}

int Renderer::get_image(uint32_t* argb, int32_t* w, int32_t* h)
{
    std::lock_guard<std::recursive_mutex> g(image_mu_);
    if (w) *w = img_w_;
    if (h) *h = img_h_;
    if (!argb)
        return RT_OK;
    const size_t n = (size_t)img_w_ * img_h_;
    if (!rendered_) {
        // init_buffers / clear_image fill with BACKGROUND_COLOR (renderer.cpp:131-134)
        uint32_t bg = color_to_argb(col(135.0f / 255.0f, 206.0f / 255.0f, 235.0f / 255.0f));
        for (size_t i = 0; i < n; i++) argb[i] = bg;
        return RT_OK;
    }
    // the image as it stands in HBM: a frame still rendering on stream_ (another thread) is
    // neither waited for nor blocked -- the copy runs on a non-blocking stream of its own
    hipError_t e = hipSetDevice(device_);
    if (e == hipSuccess && !display_stream_)
        e = hipStreamCreateWithFlags(&display_stream_, hipStreamNonBlocking);
    if (e == hipSuccess && display_bytes_ < n * 4) {
        // a larger staging buffer: the old one is freed only when the renderer is destroyed
        // (hipHostFree synchronises the device, i.e. it would wait for the frame in flight)
        void* q = nullptr;
        e = hipHostMalloc(&q, n * 4, hipHostMallocDefault);
        if (e == hipSuccess) {
            if (display_host_)
                display_old_.push_back(display_host_);
            display_host_ = q;
            display_bytes_ = n * 4;
        }
    }
    const DevBuf& src = img_is_internal_ ? d_internal_ : d_image_;
    // in chunks: the DMA of chunk i + 1 runs while the host copies chunk i out of the pinned staging
    // buffer (8.3 MB at 1080p: the two serialised took ~0.7 ms)
    constexpr int NCH = 8;
    const size_t bytes = n * 4, step = ((bytes + NCH - 1) / NCH + 4095) / 4096 * 4096;
    if (e == hipSuccess && !display_ev_[0])
        for (int i = 0; i < NCH && e == hipSuccess; i++)
            e = hipEventCreateWithFlags(&display_ev_[i], hipEventDisableTiming);
    int nch = 0;
    for (size_t off = 0; e == hipSuccess && off < bytes; off += step, nch++) {
        const size_t len = std::min(step, bytes - off);
        e = hipMemcpyAsync(static_cast<char*>(display_host_) + off, static_cast<const char*>(src.p) + off, len,
                           hipMemcpyDeviceToHost, display_stream_);
        if (e == hipSuccess)
            e = hipEventRecord(display_ev_[nch], display_stream_);
    }
    for (int i = 0; e == hipSuccess && i < nch; i++) {
        e = hipEventSynchronize(display_ev_[i]);
        if (e == hipSuccess) {
            const size_t off = (size_t)i * step;
            std::memcpy(reinterpret_cast<char*>(argb) + off, static_cast<const char*>(display_host_) + off,
                        std::min(step, bytes - off));
        }
    }
    if (e != hipSuccess) {
        hipStreamSynchronize(display_stream_);
        // (not err_: the owning thread may be writing it)
        display_err_ = std::string("get_image: ") + hipGetErrorString(e);
        return RT_EHIP;
    }
    return RT_OK;
}

// The frame about to launch renders into the internal buffer, which becomes the image
// (Renderer::_image, written pixel by pixel by ray_trace, renderer.cpp:1080-1112).  The
// reference re-creates _image (uninitialised) each SSAA frame (:1079-1080) and keeps the
// previous one otherwise; here a fresh or re-created image starts as BACKGROUND_COLOR
// (init_buffers, :131-134), so a display sees the frame's finished tiles over a defined fill.
int Renderer::begin_internal_image(int rw, int rh)
{
    std::lock_guard<std::recursive_mutex> g(image_mu_);
    const size_t n = (size_t)rw * rh;
    const bool grown = d_internal_.bytes < n * 4 || !d_internal_.p;
    hipError_t e = d_internal_.reserve(n * 4);
    if (e != hipSuccess) return hip_fail(e, "hipMalloc (image)");
    if (grown || s_.enable_ssaa || !img_is_internal_ || !rendered_ || img_w_ != rw || img_h_ != rh) {
        const uint32_t bg = color_to_argb(col(135.0f / 255.0f, 206.0f / 255.0f, 235.0f / 255.0f));
        if ((e = hipMemsetD32Async((hipDeviceptr_t)d_internal_.p, (int)bg, n, stream_)) != hipSuccess)
            return hip_fail(e, "hipMemsetD32Async (image)");
    }
    img_w_ = rw;
    img_h_ = rh;
    img_is_internal_ = true;
    rendered_ = true;
    return RT_OK;
}

int Renderer::request_aux(bool rgba, bool hit, bool shadow)
{
    want_rgba_ = rgba;
    want_hit_ = hit;
    want_shadow_ = shadow;
    aux_valid_ = false;
    return RT_OK;
}

int Renderer::get_internal(uint32_t* argb, float* rgba, int32_t* hit_id, float* hit_t, uint8_t* shadow)
{
    if (!aux_valid_)
        return fail(RT_ESTATE, "get_internal: no ray_trace since the last request_aux");
    hipSetDevice(device_);
    int rw, rh;
    render_size(rw, rh);
    size_t n = (size_t)rw * rh;
    hipError_t e = hipSuccess;
    if (argb) e = hipMemcpy(argb, d_internal_.p, n * 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess && rgba) {
        if (!want_rgba_) return fail(RT_ESTATE, "rgba not requested");
        e = hipMemcpy(rgba, d_rgba_.p, n * 16, hipMemcpyDeviceToHost);
    }
    if (e == hipSuccess && (hit_id || hit_t)) {
        if (!want_hit_) return fail(RT_ESTATE, "hit buffers not requested");
        if (hit_id) e = hipMemcpy(hit_id, d_hit_id_.p, n * 4, hipMemcpyDeviceToHost);
        if (e == hipSuccess && hit_t) e = hipMemcpy(hit_t, d_hit_t_.p, n * 4, hipMemcpyDeviceToHost);
    }
    if (e == hipSuccess && shadow) {
        if (!want_shadow_) return fail(RT_ESTATE, "shadow buffer not requested");
        e = hipMemcpy(shadow, d_shadow_.p, n, hipMemcpyDeviceToHost);
    }
    if (e != hipSuccess) return hip_fail(e, "get_internal");
    return RT_OK;
}

int Renderer::debug_read(uint64_t* out, int64_t n)
{
    if (!d_dbg_.p || n < 0 || n > (int64_t)DBG_WAVES * DBG_WORDS)
        return fail(RT_EINVAL, "debug_read: no debug buffer (RT_DEBUG_WAVES) or bad size");
    hipError_t e = hipMemcpy(out, d_dbg_.p, (size_t)n * 8, hipMemcpyDeviceToHost);
    return e == hipSuccess ? RT_OK : hip_fail(e, "debug_read");
}

// The shader cycles (s_memtime) of each tile of trace_frame's last launch, tile = ty * tiles_x + tx
// (the heavy-first ordering's input; tools/tile_costs.py).  Zero for tiles off the image.
int Renderer::tile_costs(uint32_t* out, int64_t n, int32_t* tiles_x, int32_t* tiles_y)
{
    const TileCost& T = last_tc_ ? *last_tc_ : tc_main_;   // the last launch's (a band launch's slot, or trace_frame's)
    if (!T.cost.p || T.ntiles <= 0)
        return fail(RT_EINVAL, "tile_costs: no launch with tile costs yet (RT_HEAVY_FIRST=0, reflections or raster?)");
    *tiles_x = T.tiles_x;
    *tiles_y = T.tiles_y;
    if (!out)
        return RT_OK;
    if (n < T.ntiles)
        return fail(RT_EINVAL, "tile_costs: buffer smaller than tiles_x * tiles_y");
    hipError_t e = hipStreamSynchronize(stream_);
    if (e == hipSuccess && sync_slots() != RT_OK)
        return RT_EHIP;
    if (e == hipSuccess)
        e = hipMemcpy(out, T.cost.p, (size_t)T.ntiles * 4, hipMemcpyDeviceToHost);
    return e == hipSuccess ? RT_OK : hip_fail(e, "tile_costs");
}

int Renderer::origin_cones(uint32_t* out, int64_t n, int32_t dims[3], float lo_ih[4])
{
    if (!ocone_ready_)
        return fail(RT_EINVAL, "origin_cones: none resident (no reflective material at the last geometry change, "
                               "RT_OCONE=0, or the SAH tree not adopted yet)");
    const int64_t ncell = (int64_t)ocg_.dim[0] * ocg_.dim[1] * ocg_.dim[2];
    for (int a = 0; a < 3; a++) {
        dims[a] = ocg_.dim[a];
        lo_ih[a] = ocg_.lo[a];
    }
    lo_ih[3] = ocg_.ih;
    if (!out)
        return RT_OK;
    if (n < 2 * ncell)
        return fail(RT_EINVAL, "origin_cones: buffer smaller than 2 words per cell");
    hipError_t e = hipMemcpy(out, d_ocone_.p, (size_t)ncell * sizeof(uint2), hipMemcpyDeviceToHost);
    return e == hipSuccess ? RT_OK : hip_fail(e, "origin_cones");
}

// Per global output band, the cycles of its tiles in the slot's last launch (a tile is charged to the
// band of its first internal row; the heavy-first order's tile costs, a split tile the sum of its parts).
int Renderer::band_costs(hipStream_t stream, double* costs, int nbands)
{
    if (!stream)
        stream = stream_;
    const int H = s_.image_height;
    const BandSlot* S = nullptr;
    for (int i = 0; i < band_nslots_; i++)
        if (band_slot_[i].stream == stream) S = &band_slot_[i];
    if (!S || !S->live || !S->tc.cost.p || S->tc.ntiles <= 0 || S->tc.band_rows <= 0)
        return fail(RT_EINVAL, "band_costs: no band launch with tile costs on this stream");
    const TileCost& T = S->tc;
    if (!costs || nbands < (H + T.band_rows - 1) / T.band_rows)
        return fail(RT_EINVAL, "band_costs: buffer smaller than the image's bands");
    hipError_t e = hipEventSynchronize(S->done);
    std::vector<uint32_t> c((size_t)T.ntiles);
    if (e == hipSuccess)
        e = hipMemcpy(c.data(), T.cost.p, c.size() * 4, hipMemcpyDeviceToHost);
    if (e != hipSuccess)
        return hip_fail(e, "band_costs");
    const int rows_per_band = T.band_rows * T.ssaa;   // internal rows
    std::vector<double> local(T.bands.size(), 0.0);
    for (int ty = 0; ty < T.tiles_y; ty++) {
        const int lb = (8 * ty) / rows_per_band;
        if (lb >= (int)local.size())
            continue;
        double s = 0.0;
        for (int tx = 0; tx < T.tiles_x; tx++)
            s += c[(size_t)ty * T.tiles_x + tx];
        local[lb] += s;
    }
    for (size_t i = 0; i < local.size(); i++)
        if (T.bands[i] < nbands)
            costs[T.bands[i]] = local[i];
    return RT_OK;
}

int Renderer::get_stats(rt_stats* out) const
{
    std::memset(out, 0, sizeof(*out));
    out->primary_rays = last_primary_;
    out->shadow_rays = last_shadow_;
    out->reflection_rays = last_refl_;
    out->kernel_ms = kernel_ms_;
    out->post_ms = post_ms_;
    out->build_ms = build_ms_;
    out->octree_inner = oct_stats_.inner;
    out->octree_leaves = oct_stats_.leaves;
    out->octree_empty_leaves = oct_stats_.empty_leaves;
    out->octree_max_leaf = oct_stats_.max_leaf;
    out->octree_max_depth = oct_stats_.max_depth;
    out->gpu_nodes = oct_nn_;
    out->gpu_tris = oct_nt_;
    out->host_builds = host_builds_;
    if (multi_)
        for (const auto& h : multi_->helpers)
            out->host_builds += h->host_builds_;
    render_size(out->render_width, out->render_height);
    out->seg_scale = last_seg_;
    for (int i = 0; i < 4; i++) out->work[i] = last_work_[i];
    for (int i = 0; i < 4; i++) out->work_wide[i] = last_work_[4 + i];
    for (int i = 0; i < 6; i++) out->uncertified[i] = last_uncert_[i];
    for (int i = 0; i < 6; i++) out->wave_steps[i] = last_wave_[i];
    for (int i = 0; i < 4; i++) out->build_split_ms[i] = build_split_ms_[i];
    out->wide_tree = wide_tree_;
    return RT_OK;
}

int Renderer::local_rows(int band_rows, int rank, int nranks) const
{
    if (band_rows <= 0 || nranks <= 0 || rank < 0 || rank >= nranks)
        return -1;
    int nb = (s_.image_height + band_rows - 1) / band_rows;
    int per = (nb + nranks - 1) / nranks;
    return per * band_rows;
}

int Renderer::render_bands_device(int band_rows, int rank, int nranks, uint32_t* d_out, hipStream_t stream)
{
    return render_bands_impl(band_rows, rank, nranks, nullptr, 0, d_out, stream);
}

int Renderer::render_band_list_device(int band_rows, const int32_t* bands, int nbands, uint32_t* d_out,
                                      hipStream_t stream)
{
    if (band_rows <= 0 || nbands <= 0 || !bands)
        return fail(RT_EINVAL, "render_band_list_device: empty band list");
    const int nb = (s_.image_height + band_rows - 1) / band_rows;
    std::vector<char> seen(nb, 0);
    for (int i = 0; i < nbands; i++) {
        if (bands[i] < 0 || bands[i] >= nb || seen[bands[i]])
            return fail(RT_EINVAL, "render_band_list_device: band out of range or listed twice");
        seen[bands[i]] = 1;
    }
    return render_bands_impl(band_rows, 0, 2, bands, nbands, d_out, stream);
}

// One launch of interleaved bands (bands == nullptr: band b % nranks == rank) or of a band list.
int Renderer::render_bands_impl(int band_rows, int rank, int nranks, const int32_t* bands, int nbands,
                                uint32_t* d_out, hipStream_t stream)
{
    int lrows = bands ? nbands * band_rows : local_rows(band_rows, rank, nranks);
    if (lrows < 0 || !d_out)
        return fail(RT_EINVAL, "render_bands_device: bad band layout");
    if (s_.enable_ssao)   // its samples and 7x7 blur read across bands
        return fail(RT_EUNSUPPORTED, "render_bands_device: SSAO needs the whole frame (use rt_render)");
    if (validate() != RT_OK)
        return fail(RT_EINVAL, "invalid scene: material index out of range or enabled texture map missing");
    if (check_frame() != RT_OK)
        return fail(RT_EUNSUPPORTED, "reflective materials with max_recursion_depth > 15, a raster frame with "
                                     "reflections and no BVH, or more than 2^27 triangles to rasterise");
    int rc = ensure_device_scene();
    if (rc != RT_OK)
        return rc;
    if (!stream)
        stream = stream_;
    KParams P;
    fill_params(P);
    last_seg_ = P.seg_scale;
    hipError_t e;
    // The stream's slot: its own tile-queue counters and SSAA band buffer, so that frames
    // launched on different streams may run concurrently (the tail of one frame overlaps
    // the next; same-stream launches are ordered by the stream).  Only the default trace
    // path keeps all of its per-launch state in the slot: the reflection engine, the raster
    // path and the opt-in modes (octree deferral, split / lean frames, tile order) share
    // buffers across launches, so a launch on another stream first waits for the last one.
    int si = -1;
    for (int i = 0; i < band_nslots_; i++)
        if (band_slot_[i].stream == stream) si = i;
    if (si < 0) {
        if (band_nslots_ < BAND_SLOTS) {
            si = band_nslots_++;
            band_slot_[si].counters.device = band_slot_[si].tmp.device = device_;
            if ((e = hipEventCreateWithFlags(&band_slot_[si].done, hipEventDisableTiming)) != hipSuccess ||
                (e = hipEventCreateWithFlags(&band_slot_[si].mark, hipEventDisableTiming)) != hipSuccess)
                return hip_fail(e, "hipEventCreate");
        } else {
            // a ninth stream: the least recently used slot is recycled once its last launch is
            // done (its own event; the stream it ran on may no longer exist)
            si = 0;
            for (int i = 1; i < BAND_SLOTS; i++)
                if (band_slot_[i].used < band_slot_[si].used) si = i;
            if (band_slot_[si].live && (e = hipEventSynchronize(band_slot_[si].done)) != hipSuccess)
                return hip_fail(e, "render_bands_device: recycling a stream slot");
        }
        band_slot_[si].stream = stream;
    }
    band_slot_[si].used = ++band_uses_;
    // Only the default trace path keeps all of its per-launch state in the slot; the
    // reflection engine and the raster path use buffers shared across launches, so such a
    // launch first waits for every launch still in flight on any stream.
    const bool slot_only = !P.has_reflection && !s_.hybrid_rasterization_tracing;
    if (!slot_only && wait_slots(stream) != RT_OK)
        return RT_EHIP;
    BandSlot& S = band_slot_[si];
    band_last_ = si;
    int f = s_.enable_ssaa ? s_.ssaa_factor : 1;
    P.band_rows = band_rows * f;
    P.nranks = nranks;
    P.rank = rank;
    P.local_rows = lrows * f;
    uint64_t layout_key = 0;
    if (bands) {
        // the list and its inverse in the slot's device buffer; a new list waits for the slot's last
        // launch (which may still read the old one) and is copied synchronously: lists change rarely
        const int nb = (s_.image_height + band_rows - 1) / band_rows;
        std::vector<int32_t> host(bands, bands + nbands);
        host.resize((size_t)nbands + nb, -1);
        for (int i = 0; i < nbands; i++)
            host[(size_t)nbands + bands[i]] = i;
        if (host != S.map_host || nb != S.map_nb) {
            if (S.live && (e = hipEventSynchronize(S.done)) != hipSuccess)
                return hip_fail(e, "render_band_list_device: waiting for the slot's last launch");
            S.map.device = device_;
            if ((e = S.map.reserve(host.size() * 4)) != hipSuccess ||
                (e = hipMemcpy(S.map.p, host.data(), host.size() * 4, hipMemcpyHostToDevice)) != hipSuccess)
                return hip_fail(e, "band list upload");
            S.map_host.swap(host);
            S.map_nb = nb;
        }
        P.band_map = S.map.as<int32_t>();
        P.band_inv = P.band_map + nbands;
        layout_key = 1469598103934665603ull;
        for (int32_t b : S.map_host)
            layout_key = (layout_key ^ (uint64_t)(uint32_t)b) * 1099511628211ull;
    }
    P.tiles_x = (P.rw + 7) / 8;
    P.tiles_y = (P.local_rows + 7) / 8;
    if ((e = S.counters.reserve(NCOUNTER_WORDS * 8)) != hipSuccess) return hip_fail(e, "hipMalloc (counters)");
    // SSAA fused into the trace kernel's tiles (kernels.hip downscale_tile) when every lane
    // of every tile holds a pixel (no padding) and f divides the 8x8
    // tile; otherwise the band is rendered at full size and downscale_kernel filters it.
    // RT_FUSED_SSAA=0 keeps the separate pass.
    const bool fused = (f == 2 || f == 4 || f == 8) && slot_only && knobs_.fused_ssaa && P.rw % 8 == 0 &&
                       P.local_rows % 8 == 0;
    uint32_t* target = d_out;
    if (f > 1 && !fused) {
        if ((e = S.tmp.reserve((size_t)P.rw * P.local_rows * 4)) != hipSuccess)
            return hip_fail(e, "hipMalloc (band)");
        target = S.tmp.as<uint32_t>();
    }
    P.argb = fused ? nullptr : target;
    if (fused) {
        P.ds_out = d_out;
        P.ds_shift = f == 2 ? 1 : (f == 4 ? 2 : 3);
    }
    P.counters = S.counters.as<unsigned long long>();
    if (ring_.empty()) {
        ring_.resize(2 * EV_RING, nullptr);
        for (auto& ev : ring_)
            if ((e = hipEventCreate(&ev)) != hipSuccess) return hip_fail(e, "hipEventCreate");
    }
    if ((rc = prepare_risk(P, stream)) != RT_OK)
        return rc;
    bool zeroed = false;   // heavy_prep_kernel clears the counter words itself (one dispatch fewer)
    bool overlapped = false;   // another band launch still in flight (frames in flight)
    for (int i = 0; i < band_nslots_ && !overlapped; i++)
        overlapped = i != si && band_slot_[i].live && hipEventQuery(band_slot_[i].done) == hipErrorNotReady;
    if ((rc = prepare_heavy(P, S.tc, stream, layout_key, &zeroed, overlapped)) != RT_OK)
        return rc;
    if (!zeroed && (e = hipMemsetAsync(S.counters.p, 0, NCOUNTER_WORDS * 8, stream)) != hipSuccess)
        return hip_fail(e, "hipMemsetAsync");
    S.tc.band_rows = band_rows;
    S.tc.ssaa = f;
    S.tc.bands.resize(lrows / band_rows);
    for (int i = 0; i < (int)S.tc.bands.size(); i++)
        S.tc.bands[i] = bands ? bands[i] : i * nranks + rank;
    hipEventRecord(ring_[2 * ring_next_], stream);
    if ((rc = launch_frame(P, stream)) != RT_OK) return rc;
    hipEventRecord(ring_[2 * ring_next_ + 1], stream);
    ring_next_ = (ring_next_ + 1) % EV_RING;
    if (ring_count_ < EV_RING) ring_count_++;
    if (f > 1 && !fused && (e = rt_launch_downscale(target, P.rw, P.local_rows, f, d_out, stream)) != hipSuccess)
        return hip_fail(e, "downscale launch");
    // 'done' is recorded on the renderer's own fence stream behind the caller's: later waits on it
    // never touch the caller's stream, which may be destroyed by then (an event recorded on a
    // destroyed stream made hipEventSynchronize fail with a capture-state error)
    if ((e = hipEventRecord(S.mark, stream)) != hipSuccess || (e = hipStreamWaitEvent(fence_stream_, S.mark, 0)) != hipSuccess ||
        (e = hipEventRecord(S.done, fence_stream_)) != hipSuccess)
        return hip_fail(e, "hipEventRecord");
    S.live = true;
    return RT_OK;
}

// The frame's grazing-risk keys (KParams::wrisk, wbvh.hpp WRiskArgs): computed on
// 'stream' when the camera, the light or the resident wide BVH changed since the last computation
// (launches in flight on other streams read the keys: the stream first waits for them); every
// launch waits for the computation (risk_ev_).  RT_WBVH_RISK=0: none (every child runs case (b)).
int Renderer::prepare_risk(KParams& P, hipStream_t stream)
{
    P.wrisk = nullptr;
    P.risk_G = 0.0f;
    P.risk_nl = 0.0f;
    P.risk_nu = 0.0f;
    P.risk_cap = nullptr;
    if (!P.wnodes || !knobs_.risk || risk_nodes_ <= 0 || !d_wrisk_.p || !d_wlinks_.p)
        return RT_OK;
    // the risk caps' directions: from the camera / the light towards the scene's centre (any direction is
    // sound; this one makes a convex object's silhouette interior skip case (b), wbvh.hpp risk_cap_skip)
    float cap_dir[2][3];
    for (int sel = 0; sel < 2; sel++) {
        const float* X = sel == 0 ? P.cam_pos : P.light;
        double v[3], l = 0;
        for (int a = 0; a < 3; a++) {
            v[a] = 0.5 * ((double)oct_root_.dn[a] + (double)oct_root_.df[a]) - (double)X[a];
            l += v[a] * v[a];
        }
        l = std::sqrt(l);
        for (int a = 0; a < 3; a++)
            cap_dir[sel][a] = l > 0 && l < INFINITY ? (float)(v[a] / l) : (a == 0 ? 1.0f : 0.0f);
    }
    hipError_t e;
    if (!risk_valid_ || std::memcmp(risk_cam_, P.cam_pos, sizeof risk_cam_) ||
        std::memcmp(risk_light_, P.light, sizeof risk_light_)) {
        if (wait_slots(stream) != RT_OK)
            return RT_EHIP;
        const float lo[3] = {oct_root_.dn[0], oct_root_.dn[1], oct_root_.dn[2]};
        const float hi[3] = {oct_root_.df[0], oct_root_.df[1], oct_root_.df[2]};
        const WRiskArgs A = wbvh_risk_args(lo, hi, P.scene_scale, P.cam_pos, P.light, W_QS_CLOSEST, W_QS_SHADOW);
        risk_valid_ = false;
        const uint32_t* links = d_wlinks_.as<uint32_t>();
        // d_wrisk_: the packed words (8 x 8 B per node), then the walk's keys (8 x 4 B) and boxes (8 x 24 B)
        const size_t ne = (size_t)risk_nodes_ * 8;
        unsigned long long* words = d_wrisk_.as<unsigned long long>();
        uint32_t* K = reinterpret_cast<uint32_t*>(words + ne);
        float* B = reinterpret_cast<float*>(K + ne);
        uint32_t* cap = reinterpret_cast<uint32_t*>(B + 6 * ne);   // (the 2 caps, past the boxes)
        std::memcpy(risk_cap_dir_, cap_dir, sizeof risk_cap_dir_);
        if ((e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(K), 0x7F800000, ne, stream)) != hipSuccess ||
            (e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(cap), 0x7F800000, 2, stream)) != hipSuccess ||
            (e = rt_launch_risk_box_init(B, ne, stream)) != hipSuccess ||
            (e = rt_launch_wide_risk(P.wtris, P.wmeta, P.nodes, P.wnodes, links, links + risk_tris_, K, B, words,
                                     (int)risk_tris_, (int)risk_nodes_, &A, cap, &risk_cap_dir_[0][0], stream)) != hipSuccess ||
            // risk_ev_ is recorded on the renderer's own fence stream behind 'stream' (as a band slot's
            // 'done'): later launches wait on it after the caller may have destroyed 'stream'
            (e = hipEventRecord(risk_mark_, stream)) != hipSuccess ||
            (e = hipStreamWaitEvent(fence_stream_, risk_mark_, 0)) != hipSuccess ||
            (e = hipEventRecord(risk_ev_, fence_stream_)) != hipSuccess)
            return hip_fail(e, "wide_risk_kernel");
        risk_ev_live_ = true;
        risk_valid_ = true;
        std::memcpy(risk_cam_, P.cam_pos, sizeof risk_cam_);
        std::memcpy(risk_light_, P.light, sizeof risk_light_);
        risk_G_ = A.ray_G;
        risk_nl_ = A.ray_nl;
        risk_nu_ = A.ray_nu;
    } else if (risk_ev_live_ && (e = hipStreamWaitEvent(stream, risk_ev_, 0)) != hipSuccess)
        return hip_fail(e, "hipStreamWaitEvent (risk bits)");
    P.wrisk = d_wrisk_.as<uint64_t>();
    P.risk_G = risk_G_;
    P.risk_nl = risk_nl_;
    P.risk_nu = risk_nu_;
    if (knobs_.risk_cap) {
        P.risk_cap = reinterpret_cast<const float*>(d_wrisk_.as<uint8_t>() + (size_t)risk_nodes_ * 288);
        std::memcpy(P.cap_dir, risk_cap_dir_, sizeof P.cap_dir);
    }
    return RT_OK;
}

// Heavy tiles first (KParams::tile_cost, kernels.hip heavy_prep_kernel): the launch's tiles that cost
// the most in the previous launch of the same tile layout on this slot are dequeued first, so that a
// few very long tiles (grazing silhouette rays) start with the frame instead of ending
// it.  Only the order changes; every tile is traced once.  Off for the reflection engine and the raster
// path (their own kernels) and with RT_HEAVY_FIRST=0.
int Renderer::prepare_heavy(KParams& P, TileCost& T, hipStream_t stream, uint64_t layout_key, bool* zeroed,
                            bool overlapped)
{
    if (zeroed)
        *zeroed = false;
    P.tile_cost = nullptr;
    P.heavy_list = nullptr;
    P.heavy_bits = nullptr;
    P.heavy_ctr = nullptr;
    P.heavy_group = 0;
    if (!knobs_.heavy || P.has_reflection || s_.hybrid_rasterization_tracing)
        return RT_OK;
    const int ntiles = P.tiles_x * P.tiles_y;
    if (ntiles <= 0)
        return RT_OK;
    T.cost.device = T.heavy.device = device_;
    const size_t nb = ((size_t)ntiles + 31) / 32;
    hipError_t e;
    // T.heavy: the list (ntiles), the bits (nb words), then two {sum, max} pairs of the launches' tile
    // costs (KParams::tile_stats, alternating: a launch accumulates one, the next heavy_prep reads it)
    // ... and two sets of the list counts and tickets (int32 x 4 each, alternating the same way)
    const size_t stats_off = ((size_t)ntiles * 4 + nb * 4 + 7) / 8 * 8;
    if ((e = T.cost.reserve((size_t)ntiles * 4)) != hipSuccess ||
        (e = T.heavy.reserve(stats_off + 4 * 8 + 2 * 16)) != hipSuccess)
        return hip_fail(e, "hipMalloc (tile costs)");
    unsigned long long* stats = reinterpret_cast<unsigned long long*>(static_cast<char*>(T.heavy.p) + stats_off);
    int32_t* ctrs = reinterpret_cast<int32_t*>(stats + 4);
    uint64_t key = 1469598103934665603ull;
    for (int64_t v : {(int64_t)P.rw, (int64_t)P.rh, (int64_t)P.local_rows, (int64_t)P.tiles_x, (int64_t)P.tiles_y,
                      (int64_t)P.band_rows, (int64_t)P.rank, (int64_t)P.nranks, (int64_t)T.cost.bytes,
                      (int64_t)layout_key})
        key = (key ^ (uint64_t)v) * 1099511628211ull;
    if (key != T.key && ((e = hipMemsetAsync(T.cost.p, 0, (size_t)ntiles * 4, stream)) != hipSuccess ||
                         (e = hipMemsetAsync(stats, 0, 4 * 8 + 2 * 16, stream)) != hipSuccess))
        return hip_fail(e, "hipMemsetAsync (tile costs)");
    T.key = key;
    T.parity ^= 1u;
    T.ntiles = ntiles;
    T.tiles_x = P.tiles_x;
    T.tiles_y = P.tiles_y;
    int32_t* list = T.heavy.as<int32_t>();
    uint32_t* bits = reinterpret_cast<uint32_t*>(list + ntiles);
    // the list counts and tickets of this launch (cleared by the slot's previous heavy_prep, or above)
    int32_t* ctr = ctrs + 4 * T.parity;
    // tiles are split (kernels.hip trace_split_part) only by the plain kernel over the wide BVH, with a
    // fused SSAA block within a part's 8 / G rows
    const int G = knobs_.heavy_group;
    const bool split = G > 1 && !P.has_reflection && P.plain && !P.zbuf && !P.nbuf && P.wnodes && P.nnodes > 0 &&
                       (!P.ds_out || ((1 << P.ds_shift) <= SPLIT_ROWS && (1 << P.ds_shift) <= SPLIT_COLS));
    unsigned long long* stats_next = stats + 2 * T.parity;
    // The split bar (x the launch's mean cycles per wave): a band launch of 1 / N of the frame has ~N times
    // cheaper mean waves on the same grid, and splitting at the full frame's bar there splits tiles that
    // would not outlast the launch (their parts cost ~1.8x their cycles): the bar grows as the launch's
    // share shrinks, by N^0.5 alone and N^0.7 while other band launches are in flight, whose work hides
    // this one's tail (strips N = 8: 0.318 -> 0.227-0.260 ms per step at three in flight with bars
    // 1 / 1.5 / 2 against 0.5, one in flight best at 1-1.5; profiles/r06/strips_split_sweep.log)
    const double share = (double)ntiles / (double)((int64_t)((P.rw + 7) / 8) * ((P.rh + 7) / 8));
    const float split_bar = knobs_.heavy_split *
                            (float)std::pow(std::min(1.0, std::max(share, 1e-6)),
                                            -(double)(overlapped ? knobs_.heavy_split_exp_overlap : knobs_.heavy_split_exp));
    if ((e = rt_launch_heavy_prep(&P, T.cost.as<uint32_t>(), ntiles, list, bits, ctr, ctrs + 4 * (T.parity ^ 1u),
                                  stats + 2 * (T.parity ^ 1u), stats_next, split_bar, split ? G : 0, stream)) != hipSuccess)
        return hip_fail(e, "heavy_prep_kernel");
    P.tile_cost = T.cost.as<uint32_t>();
    P.tile_stats = stats_next;
    last_tc_ = &T;
    P.heavy_list = list;
    P.heavy_bits = bits;
    P.heavy_ctr = ctr;
    P.heavy_group = split ? G : 0;
    P.split_parts = knobs_.split_parts > 0 ? knobs_.split_parts : G;
    if (zeroed)
        *zeroed = true;   // (heavy_prep_kernel cleared P.counters)
    return RT_OK;
}

int Renderer::wait_slots(hipStream_t stream)
{
    for (int i = 0; i < band_nslots_; i++) {
        BandSlot& b = band_slot_[i];
        if (!b.live || b.stream == stream)
            continue;
        hipError_t e = hipStreamWaitEvent(stream, b.done, 0);
        if (e != hipSuccess)
            return hip_fail(e, "hipStreamWaitEvent (frames in flight)");
    }
    return RT_OK;
}

int Renderer::sync_slots()
{
    for (int i = 0; i < band_nslots_; i++) {
        BandSlot& b = band_slot_[i];
        if (!b.live)
            continue;
        hipError_t e = hipEventSynchronize(b.done);
        if (e != hipSuccess)
            return hip_fail(e, "hipEventSynchronize (frames in flight)");
    }
    return RT_OK;
}

int Renderer::trace_rays(const float* orig, const float* dir, int64_t n, int32_t* id, float* t, float* u, float* v,
                         uint8_t* ret)
{
    if (n < 0 || n > (1 << 30) || (n > 0 && (!orig || !dir || !id || !t || !u || !v || !ret)))
        return fail(RT_EINVAL, "trace_rays: bad arguments");
    int rc = ensure_device_scene();
    if (rc != RT_OK)
        return rc;
    if (n == 0)
        return RT_OK;
    KParams P;
    fill_params(P);
    DevBuf din, dout;
    din.device = dout.device = device_;
    size_t nb = (size_t)n;
    hipError_t e;
    if ((e = din.reserve(nb * 24)) != hipSuccess || (e = dout.reserve(nb * 17)) != hipSuccess)
        return hip_fail(e, "hipMalloc (rays)");
    float* d_o = din.as<float>();
    float* d_d = d_o + 3 * nb;
    int32_t* d_id = dout.as<int32_t>();
    float* d_t = reinterpret_cast<float*>(d_id + nb);
    float* d_u = d_t + nb;
    float* d_v = d_u + nb;
    uint8_t* d_r = reinterpret_cast<uint8_t*>(d_v + nb);
    if ((e = hipMemcpyAsync(d_o, orig, nb * 12, hipMemcpyHostToDevice, stream_)) != hipSuccess ||
        (e = hipMemcpyAsync(d_d, dir, nb * 12, hipMemcpyHostToDevice, stream_)) != hipSuccess)
        return hip_fail(e, "upload (rays)");
    if ((e = rt_launch_trace_rays(&P, d_o, d_d, (int)n, d_id, d_t, d_u, d_v, d_r, stream_)) != hipSuccess)
        return hip_fail(e, "trace_rays_kernel launch");
    if ((e = hipMemcpyAsync(id, d_id, nb * 4, hipMemcpyDeviceToHost, stream_)) != hipSuccess ||
        (e = hipMemcpyAsync(t, d_t, nb * 4, hipMemcpyDeviceToHost, stream_)) != hipSuccess ||
        (e = hipMemcpyAsync(u, d_u, nb * 4, hipMemcpyDeviceToHost, stream_)) != hipSuccess ||
        (e = hipMemcpyAsync(v, d_v, nb * 4, hipMemcpyDeviceToHost, stream_)) != hipSuccess ||
        (e = hipMemcpyAsync(ret, d_r, nb, hipMemcpyDeviceToHost, stream_)) != hipSuccess)
        return hip_fail(e, "download (rays)");
    if ((e = hipStreamSynchronize(stream_)) != hipSuccess)
        return hip_fail(e, "trace_rays_kernel");
    return RT_OK;
}

// The frames' wide-BVH query with its status over n host rays (kernels.hip wide_query_kernel): the
// device build of rt_wbvh_query_ex, reading the risk words prepare_risk computes on the GPU
int Renderer::wide_query(const float* orig, const float* dir, int64_t n, int kind, float* o_out, float* d_out,
                         int32_t* status, int32_t* id, float* t, float* u, float* v, uint8_t* shadow)
{
    if (n < 0 || n > (1 << 28) || kind < 0 || kind > 2 ||
        (n > 0 && (!orig || !dir || !o_out || !d_out || !status || !id || !t || !u || !v || !shadow)))
        return fail(RT_EINVAL, "wide_query: bad arguments");
    int rc = ensure_device_scene();
    if (rc == RT_OK)
        rc = poll_accel(true);   // the wide BVH the frames use once it is resident
    if (rc != RT_OK)
        return rc;
    if (n == 0)
        return RT_OK;
    KParams P;
    fill_params(P);
    DevBuf din, dout;
    din.device = dout.device = device_;
    const size_t nb = (size_t)n;
    hipError_t e;
    // outputs: o, d (12 B each), status, id, t, u, v (4 B each), shadowed (1 B) per ray
    constexpr size_t OUT_BYTES = 2 * 12 + 5 * 4 + 1;
    if ((e = din.reserve(nb * 24)) != hipSuccess || (e = dout.reserve(nb * OUT_BYTES)) != hipSuccess)
        return hip_fail(e, "hipMalloc (rays)");
    float* d_o = din.as<float>();
    float* d_d = d_o + 3 * nb;
    float* d_oo = dout.as<float>();
    float* d_do = d_oo + 3 * nb;
    int32_t* d_st = reinterpret_cast<int32_t*>(d_do + 3 * nb);
    int32_t* d_id = d_st + nb;
    float* d_t = reinterpret_cast<float*>(d_id + nb);
    float* d_u = d_t + nb;
    float* d_v = d_u + nb;
    uint8_t* d_sh = reinterpret_cast<uint8_t*>(d_v + nb);
    if ((size_t)(d_sh + nb - dout.as<uint8_t>()) > dout.bytes)
        return fail(RT_EINVAL, "wide_query: output layout exceeds its buffer");
    if (wait_slots(stream_) != RT_OK)
        return RT_EHIP;
    if ((rc = prepare_risk(P, stream_)) != RT_OK)
        return rc;
    if ((e = hipMemcpyAsync(d_o, orig, nb * 12, hipMemcpyHostToDevice, stream_)) != hipSuccess ||
        (e = hipMemcpyAsync(d_d, dir, nb * 12, hipMemcpyHostToDevice, stream_)) != hipSuccess)
        return hip_fail(e, "upload (rays)");
    if ((e = rt_launch_wide_query(&P, d_o, d_d, (int)n, kind, d_oo, d_do, d_st, d_id, d_t, d_u, d_v, d_sh, stream_)) !=
        hipSuccess)
        return hip_fail(e, "wide_query_kernel launch");
    if ((e = hipMemcpyAsync(o_out, d_oo, nb * 12, hipMemcpyDeviceToHost, stream_)) != hipSuccess ||
        (e = hipMemcpyAsync(d_out, d_do, nb * 12, hipMemcpyDeviceToHost, stream_)) != hipSuccess ||
        (e = hipMemcpyAsync(status, d_st, nb * 4, hipMemcpyDeviceToHost, stream_)) != hipSuccess ||
        (e = hipMemcpyAsync(id, d_id, nb * 4, hipMemcpyDeviceToHost, stream_)) != hipSuccess ||
        (e = hipMemcpyAsync(t, d_t, nb * 4, hipMemcpyDeviceToHost, stream_)) != hipSuccess ||
        (e = hipMemcpyAsync(u, d_u, nb * 4, hipMemcpyDeviceToHost, stream_)) != hipSuccess ||
        (e = hipMemcpyAsync(v, d_v, nb * 4, hipMemcpyDeviceToHost, stream_)) != hipSuccess ||
        (e = hipMemcpyAsync(shadow, d_sh, nb, hipMemcpyDeviceToHost, stream_)) != hipSuccess)
        return hip_fail(e, "download (rays)");
    if ((e = hipStreamSynchronize(stream_)) != hipSuccess)
        return hip_fail(e, "wide_query_kernel");
    return RT_OK;
}

// The frame's grazing-risk words for the current camera and light (8 per wide-BVH node, wrisk_pack):
// src 0 as prepare_risk computes them on the GPU (wide_risk_kernel), src 1 by the host walk
// wbvh_risk_host over the resident wide BVH with the same WRiskArgs.  *count = the number of words
// (out may be null to query it).  RT_ESTATE when no wide BVH is resident or the risk words are off.
int Renderer::risk_words(int src, uint64_t* out, int64_t cap, int64_t* count, int64_t* violations)
{
    if (src < 0 || src > 1 || !count)
        return fail(RT_EINVAL, "risk_words: bad arguments");
    int rc = ensure_device_scene();
    if (rc == RT_OK)
        rc = poll_accel(true);
    if (rc != RT_OK)
        return rc;
    KParams P;
    fill_params(P);
    if (!P.wnodes || !knobs_.risk || risk_nodes_ <= 0)
        return fail(RT_ESTATE, "risk_words: no wide BVH with risk words (exact mode, RT_WBVH=0 or RT_WBVH_RISK=0)");
    const int64_t ne = risk_nodes_ * 8;
    *count = ne;
    if (!out)
        return RT_OK;
    if (cap < ne)
        return fail(RT_EINVAL, "risk_words: output too small");
    if (src == 0) {
        if (wait_slots(stream_) != RT_OK)
            return RT_EHIP;
        if ((rc = prepare_risk(P, stream_)) != RT_OK)
            return rc;
        hipError_t e;
        if ((e = hipMemcpyAsync(out, P.wrisk, (size_t)ne * 8, hipMemcpyDeviceToHost, stream_)) != hipSuccess ||
            (e = hipStreamSynchronize(stream_)) != hipSuccess)
            return hip_fail(e, "download (risk words)");
    }
    if (wb_.tris.size() != wb_.slot.size())
        wbvh_fill_tris(oct_, wb_);   // (the quick tree keeps no host copy of the records)
    const float lo[3] = {oct_root_.dn[0], oct_root_.dn[1], oct_root_.dn[2]};
    const float hi[3] = {oct_root_.df[0], oct_root_.df[1], oct_root_.df[2]};
    const WRiskArgs A = wbvh_risk_args(lo, hi, P.scene_scale, P.cam_pos, P.light, W_QS_CLOSEST, W_QS_SHADOW);
    if (violations)
        *violations = 0;
    if (src == 0) {
        if (violations)
            *violations = check_risk_words(oct_, wb_, A, 0, out) + check_risk_words(oct_, wb_, A, 1, out);
        return RT_OK;
    }
    std::vector<float> lbox(6 * wb_.tris.size());
    for (size_t k = 0; k < wb_.tris.size(); k++) {
        const GNode& L = oct_.nodes[wb_.leaf_of_k[k]];
        for (int a = 0; a < 3; a++) {
            lbox[6 * k + a] = L.dn[a];
            lbox[6 * k + 3 + a] = L.df[a];
        }
    }
    std::vector<uint64_t> risk;
    wbvh_risk_host(wb_, lbox, A, 0, risk);
    wbvh_risk_host(wb_, lbox, A, 1, risk);
    std::memcpy(out, risk.data(), (size_t)ne * 8);
    if (violations)
        *violations = check_risk_words(oct_, wb_, A, 0, out) + check_risk_words(oct_, wb_, A, 1, out);
    return RT_OK;
}

// Renderer::trace_ray (renderer.cpp:1008-1066) over n host rays at current_recursion_depth
// 'depth', each with a fresh HitInfo (trace_colors_kernel)
int Renderer::trace_ray_colors(const float* orig, const float* dir, int64_t n, int depth, float* rgba, int32_t* src,
                               float* t, uint8_t* found, uint8_t* shadow)
{
    if (n < 0 || n > (1 << 30) || depth < 0 ||
        (n > 0 && (!orig || !dir || !rgba || !src || !t || !found || !shadow)))
        return fail(RT_EINVAL, "trace_ray: bad arguments");
    if (validate() != RT_OK)
        return fail(RT_EINVAL, "invalid scene: material index out of range or enabled texture map missing");
    if (check_frame() != RT_OK)
        return fail(RT_EUNSUPPORTED, "reflective materials with max_recursion_depth > 15");
    int rc = ensure_device_scene();
    if (rc != RT_OK)
        return rc;
    if (n == 0)
        return RT_OK;
    if (depth > s_.max_recursion_depth) {
        // renderer.cpp:1012-1013: Color(0.0f), the record untouched, intersection_found false
        for (int64_t i = 0; i < n; i++) {
            rgba[4 * i] = rgba[4 * i + 1] = rgba[4 * i + 2] = 0.0f;
            rgba[4 * i + 3] = 1.0f;
            src[i] = -1;
            t[i] = -1.0f;
            found[i] = shadow[i] = 0;
        }
        last_shadow_ = last_refl_ = 0;
        return RT_OK;
    }
    KParams P;
    fill_params(P);
    P.max_recursion_depth = s_.max_recursion_depth - depth;   // only the difference is read
    DevBuf din, dout;
    din.device = dout.device = device_;
    size_t nb = (size_t)n;
    hipError_t e;
    if ((e = din.reserve(nb * 24)) != hipSuccess || (e = dout.reserve(nb * 26)) != hipSuccess ||
        (e = d_counters_.reserve(NCOUNTER_WORDS * 8)) != hipSuccess)
        return hip_fail(e, "hipMalloc (rays)");
    float* d_o = din.as<float>();
    float* d_d = d_o + 3 * nb;
    float4* d_rgba = dout.as<float4>();
    int32_t* d_src = reinterpret_cast<int32_t*>(d_rgba + nb);
    float* d_t = reinterpret_cast<float*>(d_src + nb);
    uint8_t* d_found = reinterpret_cast<uint8_t*>(d_t + nb);
    uint8_t* d_sh = d_found + nb;
    P.counters = d_counters_.as<unsigned long long>();
    if (wait_slots(stream_) != RT_OK)   // band launches in flight share the counters' buffer
        return RT_EHIP;
    if ((rc = prepare_risk(P, stream_)) != RT_OK)
        return rc;
    if ((e = hipMemsetAsync(d_counters_.p, 0, NCOUNTER_WORDS * 8, stream_)) != hipSuccess ||
        (e = hipMemcpyAsync(d_o, orig, nb * 12, hipMemcpyHostToDevice, stream_)) != hipSuccess ||
        (e = hipMemcpyAsync(d_d, dir, nb * 12, hipMemcpyHostToDevice, stream_)) != hipSuccess)
        return hip_fail(e, "upload (rays)");
    if ((e = rt_launch_trace_colors(&P, P.has_reflection, d_o, d_d, (int)n, d_rgba, d_src, d_t, d_found, d_sh,
                                    stream_)) != hipSuccess)
        return hip_fail(e, "trace_colors_kernel launch");
    unsigned long long cnt[NCOUNTERS] = {};
    if ((e = hipMemcpyAsync(rgba, d_rgba, nb * 16, hipMemcpyDeviceToHost, stream_)) != hipSuccess ||
        (e = hipMemcpyAsync(src, d_src, nb * 4, hipMemcpyDeviceToHost, stream_)) != hipSuccess ||
        (e = hipMemcpyAsync(t, d_t, nb * 4, hipMemcpyDeviceToHost, stream_)) != hipSuccess ||
        (e = hipMemcpyAsync(found, d_found, nb, hipMemcpyDeviceToHost, stream_)) != hipSuccess ||
        (e = hipMemcpyAsync(shadow, d_sh, nb, hipMemcpyDeviceToHost, stream_)) != hipSuccess ||
        (e = hipMemcpyAsync(cnt, d_counters_.p, sizeof(cnt), hipMemcpyDeviceToHost, stream_)) != hipSuccess)
        return hip_fail(e, "download (rays)");
    if ((e = hipStreamSynchronize(stream_)) != hipSuccess)
        return hip_fail(e, "trace_colors_kernel");
    last_shadow_ = (int64_t)cnt[0];
    last_refl_ = (int64_t)cnt[1];
    return RT_OK;
}

int Renderer::kernel_times(float* ms, int n)
{
    if (n > ring_count_)
        return fail(RT_EINVAL, "kernel_times: fewer launches recorded");
    hipSetDevice(device_);
    for (int i = 0; i < n; i++) {
        int slot = ((ring_next_ - n + i) % EV_RING + EV_RING) % EV_RING;
        hipError_t e = hipEventSynchronize(ring_[2 * slot + 1]);
        if (e == hipSuccess) e = hipEventElapsedTime(&ms[i], ring_[2 * slot], ring_[2 * slot + 1]);
        if (e != hipSuccess) return hip_fail(e, "kernel_times");
    }
    return RT_OK;
}

// the counters of the last band launch; they also become the stats of the last frame
// (RT_COUNT work), as after ray_trace
int Renderer::band_counters(unsigned long long out[2])
{
    hipSetDevice(device_);
    unsigned long long cnt[NCOUNTERS] = {};
    if (band_last_ < 0)
        return fail(RT_ESTATE, "band_counters: no render_bands_device launch yet");
    hipError_t e = hipEventSynchronize(band_slot_[band_last_].done);
    if (e == hipSuccess)
        e = hipMemcpy(cnt, band_slot_[band_last_].counters.p, sizeof(cnt), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return hip_fail(e, "band_counters");
    out[0] = cnt[0];
    out[1] = cnt[1];
    take_counters(cnt);
    return RT_OK;
}

void Renderer::take_counters(const unsigned long long* cnt)
{
    last_shadow_ = (int64_t)cnt[0];
    last_refl_ = (int64_t)cnt[1];
    for (int i = 0; i < 4; i++) last_work_[i] = (int64_t)cnt[4 + i];
    for (int i = 0; i < 3; i++) last_work_[4 + i] = (int64_t)cnt[10 + i];
    last_work_[7] = (int64_t)cnt[14];
    for (int i = 0; i < 6; i++) last_uncert_[i] = (int64_t)cnt[16 + i];
    for (int i = 0; i < 6; i++) last_wave_[i] = (int64_t)cnt[22 + i];
}

float render(Renderer& renderer, int* rc)
{
    auto t0 = std::chrono::steady_clock::now();
    int r;
    if (renderer.multi_active() && !renderer.render_settings().enable_ssao) {
        // rt_set_devices: bands on every device, gathered to the lead (SSAO frames stay whole)
        r = renderer.render_multi();
    } else {
        // mainUtils.cpp:10-13: raster_trace or ray_trace by the settings
        r = renderer.render_settings().hybrid_rasterization_tracing ? renderer.raster_trace() : renderer.ray_trace();
        if (r == RT_OK)
            r = renderer.post_process();
    }
    if (rc)
        *rc = r;
    return std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace rt
