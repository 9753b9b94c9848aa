// renderer.hpp -- rt::Renderer, the host-side mirror of the reference's
// Renderer class (tp2/projets/renderer/renderer.h:20-355) for the ray-trace hot
// path.  Scene state lives on the host (as in the reference); the octree is
// built on the host and flattened, then nodes, triangles, materials and
// textures are kept resident in HBM, and ray_trace() runs the gfx950 kernels.
#pragma once

#include <stdint.h>

#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rt_mi355x.h"
#include "kparams.hpp"
#include "ocone.hpp"
#include "octree.hpp"
#include "wbvh.hpp"

namespace rt {

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    int device = 0;
    ~DevBuf();
    hipError_t reserve(size_t n);   // grows (never shrinks); contents undefined after growth
    void release();
    template <class T> T* as() const { return static_cast<T*>(p); }
    // exchanges the allocations (a copy would free one buffer twice)
    void swap(DevBuf& o)
    {
        std::swap(p, o.p);
        std::swap(bytes, o.bytes);
        std::swap(device, o.device);
    }
};

struct HostTex {
    int w = 0, h = 0;
    std::vector<float> rgba;
};

// Diagnostic switches, read once from the environment when the renderer is created
// (rt_create); each selects an equivalent path (same framebuffer) for A/B runs and tests.
struct Knobs {
    bool wbvh = true;         // RT_WBVH=0: no wide BVH, every query walks the octree
    bool seg = true;          // RT_SEG=0: shadow queries have no segment end (5.2)
    bool seg_oct = false;     // RT_SEG_OCTREE=1: the octree walks only a shadow / reflection query's segment
                              // (5.2; off by default: it assumes no grazing report falls outside its volumes)
    bool cones = true;        // RT_CONES=0: no leaf normal cones (5.3; also turns the leaf slabs off)
    bool lslab = true;        // RT_LSLAB=0: no leaf slabs (5.4)
    bool plain = true;        // RT_PLAIN=0: no plain specialisation of ray_trace_kernel (5.6)
    bool quick_wbvh = true;   // RT_WBVH_QUICK_FIRST=0: no quick wide BVH after a geometry change (the frames
                              // before the SAH tree is resident walk the octree; 5.9)
    bool plain_octree = true; // RT_PLAIN_OCTREE=0: frames on the octree path (before the wide BVH is resident,
                              // exact mode) take the general kernel, not the plain one (5.8)
    bool fused_ssaa = true;   // RT_FUSED_SSAA=0: band launches downscale in a separate pass (7)
    bool refl_engine = true;  // RT_REFL_ENGINE=0: the one-lane-per-pixel recursive kernel (9)
    bool refl_sort = true;    // RT_REFL_SORT=0: reflection frames in spawn order, not Morton order
    bool refl_fuse = true;    // RT_REFL_FUSE=0: the engine's separate list / spawn passes
    int refl_chunk_log2 = 27; // RT_REFL_CHUNK_LOG2 (10..27): sample slots per engine chunk
    bool debug_waves = false; // RT_DEBUG_WAVES: per-wave records of diagnostic builds (rt_debug_read)
    bool exact = false;       // RT_EXACT=1 / rt_set_exact: wbvh and seg off
    bool risk = true;         // RT_WBVH_RISK=0: no per-frame grazing-risk bits (every child runs case (b), 5.6)
    bool heavy = true;        // RT_HEAVY_FIRST=0: tiles in queue order only (no heavy-first list, 5.6)
    int heavy_group = SPLIT_G; // RT_HEAVY_GROUP=0: no split tiles (else: the build's RT_SPLIT_G parts of a tile,
                              // each with that many lanes per pixel, kernels.hip trace_split_part)
    int split_parts = 0;      // RT_SPLIT_PARTS=n (G or 2 G): parts per split tile (0: G)
    float heavy_split_exp = 0.5f;  // RT_HEAVY_SPLIT_EXP=e: the bar below grows as (frame tiles / launch tiles)^e
    float heavy_split_exp_overlap = 0.7f;  // RT_HEAVY_SPLIT_EXP_OVERLAP: the same while other band launches are
                                           // in flight (the launch's tail overlaps them: fewer splits pay)
    float heavy_split = 0.5f; // RT_HEAVY_SPLIT=c: split the heavy tiles costing >= c x the launch's mean
                              // cycles per wave (heavy_prep_kernel)
    int refl_defer = 32;      // RT_REFL_DEFER=k (refl_feed = 0): reflection queries past k loop iterations
                              // finish in a pass of their own
    int refl_feed = 24;       // RT_REFL_FEED=k: the reflection queries by refl_trace_feed_kernel (lane refill at k
                              // waiting lanes of a wave; C5 16 / 24 / 32 / 48: 1,128 / 1,101 / 1,103 / 1,155 ms per
                              // frame, 1,195 without); 0: refl_trace_kernel with its deferral (RT_REFL_DEFER)
    bool refl_sample_major = true;  // RT_REFL_SAMPLE_MAJOR=0: the engine's slots frame-major (a frame's samples
                              // side by side) instead of sample-major (kernels.hip slot_of)
    bool refl_feed_frame_order = false; // RT_REFL_FEED_FRAME_ORDER=1: the feed hands out a frame's samples together
                              // over the sample-major slots (C5 977 vs 965 ms per frame: not faster)
    bool refl_dir_sort = false;  // RT_REFL_DIR_SORT=1: the feed takes its slots grouped by direction bin
                              // (kernels.hip refl_dir_keys_kernel, ReflArgs::perm)
    bool refl_feed_xcd = true;  // RT_REFL_FEED_XCD=0: one ticket over all the feed's slots instead of eighths, a wave
                              // starting on its XCD's (kernels.hip ReflFeed::fetch, ReflArgs::feed_parts)
    bool refl_defer_sort = false;  // RT_REFL_DEFER_SORT=1: the long kernel takes the deferred queries in their
                              // frames' order (refl_defer_keys_kernel; measured slower)
    bool refl_shadow_sort = true;  // RT_REFL_SHADOW_SORT=0: the engine's shadow pass takes its list in the order
                              // pass1 appended it, not sorted by hit point (kernels.hip refl_shadow_keys_kernel)
    bool refl_sorted_frames = true;  // RT_REFL_SORTED_FRAMES=0: the engine reads frames through the sort order
                              // instead of a sorted copy (kernels.hip refl_sort_frames_kernel)
    bool risk_cap = true;     // RT_RISK_CAP=0: no risk caps (camera / shadow rays into a silhouette's interior skip
                              // case (b), wbvh.hpp risk_cap_skip)
    bool ocone = true;        // RT_OCONE=0: no origin cones (reflection queries always run case (b), ocone.hpp)
    int ocone_dim = 128;      // RT_OCONE_DIM=n: the origin-cone grid's cells along the scene's longest axis
    int refl_shadow_feed = 0; // RT_REFL_SHADOW_FEED=k: the engine's shadow pass by refl_shadow_feed_kernel (lane
                              // refill at k waiting lanes; fused engine only; C5 16 / 24 / 32 / 48: 1,154 / 1,118 /
                              // 1,094 / 1,078 ms per frame, 1,079 without); 0: refl_shadow_kernel per entry
    int inject_fail = 0;      // RT_INJECT_FRAME_FAIL=k (tests): the k-th ray_trace fails after its image start
    bool async_accel = true;  // RT_ASYNC_ACCEL=0: the leaf cones / slabs and the wide BVH are built
                              // before the first frame instead of beside it
    static Knobs from_env();
};

class Renderer {
public:
    explicit Renderer(int device);
    ~Renderer();
    int init(std::string& err);

    // ---- reference API (renderer.h) ----
    const rt_settings& render_settings() const { return s_; }
    int set_settings(const rt_settings& s);
    int set_exact(bool on);
    // waits for the background build of the leaf cones / slabs and the wide BVH
    int finish_accel();
    bool exact() const { return knobs_.exact; }
    int change_render_size(int w, int h);
    int set_triangles(const float* tri9, const int32_t* mat, const float* uv6, int64_t n);
    int add_sphere(float cx, float cy, float cz, float r, int mat);
    int add_plane(float px, float py, float pz, float nx, float ny, float nz, int mat);
    int clear_geometry();
    int set_materials(const float* mats16, int n);
    int material_count() const { return (int)(mats_.size() / MAT_STRIDE); }
    int change_camera_fov(float fov);
    int change_camera_aspect_ratio(float aspect);
    int set_light_position(float x, float y, float z);
    int set_camera_transform(const float m[16]);
    int apply_transformation_to_camera(const float m[16]);
    int set_camera_matrices(const float pos[3], const float proj_inv[16], const float c2w[16]);
    void get_camera_matrices(float pos[3], float proj_inv[16], float c2w[16]) const;
    // Camera::_perspective_proj_mat / _world_to_camera_mat as the caller computed them (raster path)
    int set_camera_projection(const float proj[16], const float w2c[16]);
    // Camera::_fov / _aspect_ratio as the caller holds them (read by SSAO), matrices untouched
    int set_camera_lens(float fov, float aspect);
    int set_object_transform(const float m[16]);
    int reset_previous_transform();
    int set_texture(int slot, int w, int h, const float* rgba);
    int set_skybox(const int32_t w[6], const int32_t h[6], const float* const faces[6]);
    int reconstruct_bvh_new();
    int destroy_bvh();
    int ray_trace();
    // Renderer::raster_trace (renderer.cpp:869-1006): rasterised primary visibility,
    // trace_triangle shading (shadows / reflections through the octree)
    int raster_trace();
    int post_process();
    // Renderer::get_image (renderer.cpp:106-109); callable from another thread while this
    // handle renders (the display thread, QT/mainWindowThreads.cpp:6-23): it copies the image as
    // it stands in HBM on its own stream, so a frame in progress shows its finished tiles
    int get_image(uint32_t* argb, int32_t* w, int32_t* h);
    // Renderer::lock_image_mutex / unlock_image_mutex (renderer.h:41-42, renderer.cpp:96-104):
    // while held, no frame switches or reallocates the image (get_image takes it too)
    void lock_image() { image_mu_.lock(); }
    void unlock_image() { image_mu_.unlock(); }
    std::string display_error()
    {
        std::lock_guard<std::recursive_mutex> g(image_mu_);
        return display_err_;
    }
    // diagnostics: _z_buffer, _normal_buffer (xyz + pad) and the last SSAO pass's counts
    int get_ssao_buffers(float* z, float* n4, int32_t* ao);
    int request_aux(bool rgba, bool hit, bool shadow);
    int get_internal(uint32_t* argb, float* rgba, int32_t* hit_id, float* hit_t, uint8_t* shadow);
    int get_stats(rt_stats* out) const;

    // ---- multi-GPU strips ----
    int local_rows(int band_rows, int rank, int nranks) const;
    int render_bands_device(int band_rows, int rank, int nranks, uint32_t* d_out, hipStream_t stream);
    // the listed OUTPUT bands into consecutive local bands of d_out (cost-balanced strips, strips.py
    // assign_bands); render_bands_device is the list rank, rank + nranks, ...
    int render_band_list_device(int band_rows, const int32_t* bands, int nbands, uint32_t* d_out, hipStream_t stream);
    // per global output band, the shader cycles of its tiles in the last band launch on 'stream' (the
    // bands that launch did not render are left as they are)
    int band_costs(hipStream_t stream, double* costs, int nbands);
    // durations (ms) of the last n ray_trace_kernel launches of render_bands_device,
    // bracketed by HIP events on the launch stream (synchronises on them)
    int kernel_times(float* ms, int n);
    int band_counters(unsigned long long out[2]);
    int debug_read(uint64_t* out, int64_t n);   // diagnostic builds: the per-wave records of the last frame
    int tile_costs(uint32_t* out, int64_t n, int32_t* tiles_x, int32_t* tiles_y);   // trace_frame's last tile costs
    // the resident origin-cone grid (ocone.hpp; rt_ocone_read): its frame, and its words when out holds them
    int origin_cones(uint32_t* out, int64_t n, int32_t dims[3], float lo_ih[4]);
    // single-process multi-device rendering (rt_set_devices, multidev.hpp): render(Renderer&)
    // renders interleaved bands on every device and gathers them here with RCCL
    int set_devices(const int* ids, int n);
    bool multi_active() const { return multi_ != nullptr; }
    int render_multi();

    // BVH::intersect over n host rays (closest hit, reference semantics)
    int trace_rays(const float* orig, const float* dir, int64_t n, int32_t* id, float* t, float* u, float* v,
                   uint8_t* ret);
    // the frames' wide-BVH query and its status over n host rays (rt_wide_query)
    int wide_query(const float* orig, const float* dir, int64_t n, int kind, float* o_out, float* d_out,
                   int32_t* status, int32_t* id, float* t, float* u, float* v, uint8_t* shadow);
    // the risk words for the current camera / light: src 0 the GPU's, 1 the host walk's (rt_risk_words)
    int risk_words(int src, uint64_t* out, int64_t cap, int64_t* count, int64_t* violations);
    // Renderer::trace_ray (shaded) over n host rays at current_recursion_depth 'depth'
    int trace_ray_colors(const float* orig, const float* dir, int64_t n, int depth, float* rgba, int32_t* src,
                         float* t, uint8_t* found, uint8_t* shadow);

    const std::string& error() const { return err_; }

private:
    int fail(int code, const std::string& msg);
    int hip_fail(hipError_t e, const char* what);
    void render_size(int& w, int& h) const;
    void update_camera_projection();
    int ensure_device_scene();
    int validate() const;
    void fill_params(KParams& P) const;
    // the trace of one launch: the ray-trace kernel, or the reflection engine (frames by level)
    int launch_trace(const KParams& P, hipStream_t stream);
    // the raster path of one launch: clip + piece table, z-keys, shading, then the
    // reflection engine for the reflective pixels
    int launch_raster(const KParams& P, hipStream_t stream);
    int launch_frame(const KParams& P, hipStream_t stream)
    {
        return s_.hybrid_rasterization_tracing ? launch_raster(P, stream) : launch_trace(P, stream);
    }
    int check_frame() const;
    int launch_ssao();
    int trace_frame();
    int refl_level(const KParams& P, int level, int nframes, hipStream_t stream);
    // frames in flight (render_bands_device): make 'stream' wait for every live slot's last
    // launch, or the host for all of them (before buffers that launches read are replaced)
    int wait_slots(hipStream_t stream);
    int sync_slots();

    Knobs knobs_;
    int device_;
    // scene versions (bumped with the dirty flags): what a multi-device helper has mirrored
    uint64_t geom_ver_ = 0, mats_ver_ = 0, tex_ver_ = 0;
    uint64_t mir_geom_ = ~0ull, mir_mats_ = ~0ull, mir_tex_ = ~0ull;   // a helper: the lead's versions copied
    // The acceleration structures beside the octree: built on accel_thread_ after
    // the octree is uploaded, adopted by the first frame that starts after they are resident;
    // until then frames take the exact octree path (same results).
    std::thread accel_thread_;
    std::atomic<int> accel_state_{0};   // 0 idle, 1 building, 2 the tree built (the origin cones may follow), 3 failed
    std::atomic<bool> oc_done_{false};  // the background thread has finished (the origin cones included)
    bool tree_pending_ = false;         // the background's tree not adopted yet
    float oc_ms_ = 0.0f;                // the origin cones' build (background, after the tree)
    std::string accel_err_;
    hipStream_t accel_stream_ = nullptr;
    hipStream_t fence_stream_ = nullptr;   // the band slots' 'done' events (render_bands_device)
    float accel_ms_[3] = {};            // cones + slabs, wide BVH, wide-BVH upload (background)
    bool cones_ready_ = false, wide_ready_ = false, lslab_ready_ = false;
    int wide_tree_ = 0;   // rt_stats.wide_tree: 0 none, 1 the quick tree, 2 the SAH tree, -1 its build failed
    uint64_t accel_ver_ = 0;   // bumped when poll_accel adopts a build
    void start_accel();
    int poll_accel(bool wait);
    void mirror_from(const Renderer& lead);
    // a multi-device helper (rt_set_devices): the lead builds the octree, the leaf cones / slabs
    // and the wide BVH once; a helper copies the lead's device buffers to its own device
    const Renderer* lead_ = nullptr;
    uint64_t mir_accel_ = ~0ull;   // the lead's accel_ver_ copied
    int adopt_from_lead();
    int64_t host_builds_ = 0;      // host octree builds (rt_stats host_builds, helpers included)
    struct MultiDev;
    std::unique_ptr<MultiDev> multi_;
    int num_cus_ = 256;
    hipStream_t stream_ = nullptr;
    hipEvent_t ev_[4] = {nullptr, nullptr, nullptr, nullptr};
    std::string err_;

    rt_settings s_;

    // scene (host copies; the reference Renderer copies its inputs too)
    std::vector<float> tri_;
    std::vector<int32_t> tri_mat_;
    int32_t tri_mat_lo_ = INT32_MAX, tri_mat_hi_ = INT32_MIN;   // range of tri_mat_
    std::vector<float> tri_uv_;
    std::vector<int32_t> shape_kind_;
    std::vector<float> shape_;
    std::vector<int32_t> shape_mat_;
    std::vector<float> mats_;
    float cam_pos_[3] = {0, 0, 0};
    float fov_ = 45.0f, near_ = 0.1f, far_ = 1000.0f, aspect_ = 1.0f;
    float proj_[16], proj_inv_[16], c2w_[16], w2c_[16];
    float light_[3] = {3, 3, 2};
    float prev_object_[16];
    HostTex tex_[TEX_SLOTS];
    HostTex sky_[6];
    bool has_bvh_ = false;   // Renderer::_bvh holds a built tree

    // device state
    FlatOctree oct_;
    // what the frames read of the octree on the host (a helper gets the lead's)
    int64_t oct_nn_ = 0, oct_nt_ = 0;
    int oct_levels_ = 0;
    GNode oct_root_{};
    OctreeStats oct_stats_{};
    bool has_uv_dev_ = false;   // d_tri_uv_ holds texcoords
    bool geom_dirty_ = true, mats_dirty_ = true, tex_dirty_ = true;
    DevBuf d_nodes_, d_tris_, d_tri_id_, d_tri_mat_, d_tri_uv_, d_mats_;
    DevBuf d_tex_[TEX_SLOTS], d_sky_[6];
    DevBuf d_internal_, d_image_, d_rgba_, d_hit_id_, d_hit_t_, d_shadow_, d_counters_;
    // SSAO: _z_buffer, _normal_buffer (float4) and the occlusion counts of the internal image
    DevBuf d_zbuf_, d_nbuf_, d_ao_;
    // leaf normal cones, [4] per GTri slot (renderer.cpp leaf_cones)
    std::vector<float> cones_;
    DevBuf d_cones_;
    // leaf slabs, [8] per GTri slot (renderer.cpp leaf_slab)
    std::vector<float> lslab_;
    DevBuf d_lslab_;
    std::vector<float> lsin_;   // per leaf (at its first slot): <= sin(angle at a) of its triangles
    DevBuf d_lsin_;
    // the wide BVH (wbvh.hpp): nodes, triangle records in its leaf order, slot maps
    WBvh wb_;
    DevBuf d_wnodes_, d_wtris_, d_wmeta_;
    DevBuf d_wtmp_;   // the wide BVH's slot map and the octree's slot -> leaf map, for wide_gather_kernel
    // the background build's tree and buffers (start_accel), swapped in at adoption (poll_accel): the
    // resident tree may be the quick one (wbvh.hpp build_wbvh_quick) that frames in flight still read
    WBvh wb_next_;
    DevBuf d_wnodes2_, d_wtris2_, d_wmeta2_, d_wtmp2_, d_wlinks2_;
    // the origin cones (ocone.hpp) of the resident SAH tree's triangles and the background build's
    OConeGrid ocg_, ocg_next_;
    DevBuf d_ocone_, d_ocone2_, d_oc_ent_, d_oc_todo_;
    bool ocone_ready_ = false;
    float risk_cap_dir_[2][3] = {};   // the risk caps' directions of the resident words (camera, light)
    // a wide BVH's upload into the given buffers on 'stream' (the gather of its triangle records and
    // metadata from the resident octree tables on the device)
    hipError_t upload_wide(const WBvh& w, DevBuf& nodes, DevBuf& tris, DevBuf& meta, DevBuf& tmp, DevBuf& links,
                           hipStream_t stream);
    int reserve_risk(size_t nodes);
    // the grazing-risk keys (KParams::wrisk): the walk's links (WBvh::tri_leaf then parent), the keys,
    // and the camera / light / structure they were computed for; risk_ev_ follows their launch
    DevBuf d_wlinks_, d_wrisk_;
    bool risk_valid_ = false;
    int64_t risk_nodes_ = 0, risk_tris_ = 0;   // the resident wide BVH's node and triangle counts
    float risk_cam_[3] = {0, 0, 0}, risk_light_[3] = {0, 0, 0};
    float risk_G_ = 0.0f, risk_nl_ = 0.0f, risk_nu_ = 0.0f;
    hipEvent_t risk_ev_ = nullptr;     // recorded on fence_stream_ behind the computation
    hipEvent_t risk_mark_ = nullptr;   // recorded on the computing stream (fence_stream_ waits on it)
    bool risk_ev_live_ = false;
    // sets P.wrisk (and risk_G / risk_nl) for the frame's camera and light, recomputing the bits on
    // 'stream' when they changed; every launch that reads them waits for their computation
    int prepare_risk(KParams& P, hipStream_t stream);
    DevBuf d_dbg_;                           // diagnostic per-wave records (RT_DEBUG_WAVES)
    bool ssao_ready_ = false;   // the buffers hold the last frame's z / normals
    // raster path: caller-order triangles, per-triangle piece counts / offsets, the piece
    // table and its texcoords, the z-key buffer, the big-piece list, scan scratch
    DevBuf d_tri9_, d_rcount_, d_roff_, d_pieces_, d_piece_uv_, d_zkey_, d_big_, d_scan_tmp_;
    bool tri9_dirty_ = true;
    bool want_rgba_ = false, want_hit_ = false, want_shadow_ = false;
    bool aux_valid_ = false;
    // current image (Renderer::_image): internal from the start of ray_trace, downscaled after
    // post_process.  image_mu_ (Renderer::_image_mutex) guards these fields and the image
    // buffers' (re)allocation against get_image on a display thread, which copies on its own
    // non-blocking stream through a pinned staging buffer.
    std::recursive_mutex image_mu_;
    hipStream_t display_stream_ = nullptr;
    hipEvent_t display_ev_[8] = {};   // get_image's chunks (renderer.cpp get_image)
    void* display_host_ = nullptr;
    size_t display_bytes_ = 0;
    std::vector<void*> display_old_;   // outgrown staging buffers (freed with the renderer)
    int frames_started_ = 0;           // (RT_INJECT_FRAME_FAIL)
    std::string display_err_;   // get_image's last failure (err_ belongs to the owning thread)
    // the image becomes the internal buffer of a frame about to launch (trace_frame)
    int begin_internal_image(int rw, int rh);
    int img_w_ = 0, img_h_ = 0;
    bool img_is_internal_ = false;
    bool rendered_ = false;

    // reflection engine buffers, per level (frames, results, chunk samples / hits, child counter)
    struct ReflLevel {
        DevBuf fr, ret, sm, hit, cnt, list, sort, sort_tmp, res, sdefer, frs, slist;
    };
    static constexpr int REFL_LEVELS = 18;   // max_recursion_depth <= 15: frames at levels 1..16, +1 child slot
    ReflLevel refl_[REFL_LEVELS];

    // render_bands_device: per-stream tile-queue counters and SSAA band buffers, so that
    // frames launched on different streams can be in flight together.  Each
    // slot owns an event recorded after its last launch: launches that use buffers shared
    // across launches (reflection engine, raster path) and scene uploads wait on every live
    // slot's event, never on a stored stream handle (the caller may have destroyed it).
    // heavy tiles first (KParams::tile_cost / heavy_list): the last launch's tile costs of a layout
    struct TileCost {
        DevBuf cost, heavy;
        uint64_t key = 0;
        int ntiles = 0, tiles_x = 0, tiles_y = 0;   // the last launch's layout
        uint32_t parity = 0;   // which of the two tile-cost sums the last launch accumulated
        // its bands (band_costs): output rows per band, the SSAA factor, and the global band of each
        // local band
        int band_rows = 0, ssaa = 1;
        std::vector<int32_t> bands;
    };
    int prepare_heavy(KParams& P, TileCost& T, hipStream_t stream, uint64_t layout_key = 0, bool* zeroed = nullptr,
                      bool overlapped = false);
    int render_bands_impl(int band_rows, int rank, int nranks, const int32_t* bands, int nbands, uint32_t* d_out,
                          hipStream_t stream);
    const TileCost* last_tc_ = nullptr;   // the last launch's (rt_tile_costs)
    TileCost tc_main_;   // trace_frame's launches (stream_)
    struct BandSlot {
        hipStream_t stream = nullptr;
        DevBuf counters, tmp;
        TileCost tc;
        hipEvent_t done = nullptr;   // recorded on fence_stream_ behind the slot's last launch
        hipEvent_t mark = nullptr;   // recorded on 'stream' after that launch (fence_stream_ waits on it)
        bool live = false;           // 'done' has been recorded
        DevBuf map;                  // the band list of the slot's last list launch: map, then inverse
        std::vector<int32_t> map_host;
        int map_nb = 0;              // global bands of that list's image
        uint64_t used = 0;   // band_uses_ at the slot's last launch (least recently used is recycled)
    };
    static constexpr int BAND_SLOTS = 8;
    BandSlot band_slot_[BAND_SLOTS];
    int band_nslots_ = 0, band_last_ = -1;
    uint64_t band_uses_ = 0;
    // event ring for render_bands_device kernel timing
    static constexpr int EV_RING = 256;
    std::vector<hipEvent_t> ring_;
    int ring_next_ = 0, ring_count_ = 0;

    // stats
    int64_t last_primary_ = 0, last_shadow_ = 0, last_refl_ = 0;
    float last_seg_ = 0;   // KParams::seg_scale of the last frame
    int64_t last_work_[8] = {};   // RT_COUNT builds: counters[4..7], [10..12], [14] of the last frame (executed
                                  // k-DOP / MT tests: whole-line, segment; wide-BVH nodes, triangles, uncertified,
                                  // certificates)
    int64_t last_wave_[6] = {};     // RT_COUNT builds: counters[22..27], wide-BVH loop iterations (rt_stats)
    int64_t last_uncert_[6] = {};   // RT_COUNT builds: uncertified wide-BVH queries by reason
    void take_counters(const unsigned long long* cnt);
    float kernel_ms_ = 0, post_ms_ = 0, build_ms_ = 0;
    float build_split_ms_[4] = {};   // octree, leaf cones + slabs, wide BVH, upload
};

// render(Renderer&) (tp2/projets/utils/mainUtils.cpp:6-21): ray_trace then post_process;
// returns the elapsed milliseconds (*rc gets the status; on an error the remaining
// steps are skipped); raster_trace instead of ray_trace when hybrid_rasterization_tracing.
float render(Renderer& renderer, int* rc = nullptr);

}  // namespace rt
