// multidev.cpp -- rt_set_devices: one process, N devices, interleaved bands gathered to the
// lead device with RCCL (multidev.hpp).
#include "multidev.hpp"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <set>

namespace rt {

static_assert(ncclSuccess == 0 && ncclUint8 == 1, "RCCL enum values");

RcclApi* RcclApi::get(std::string* err)
{
    static RcclApi api;
    static std::string load_err;
    static std::once_flag once;
    std::call_once(once, [] {
        for (const char* name : {"librccl.so", "librccl.so.1", "/opt/rocm/lib/librccl.so"}) {
            api.so = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (api.so)
                break;
        }
        if (!api.so) {
            load_err = std::string("librccl not found: ") + dlerror();
            return;
        }
        api.comm_init_all = (CommInitAll)dlsym(api.so, "ncclCommInitAll");
        api.comm_destroy = (CommDestroy)dlsym(api.so, "ncclCommDestroy");
        api.group_start = (Group)dlsym(api.so, "ncclGroupStart");
        api.group_end = (Group)dlsym(api.so, "ncclGroupEnd");
        api.send = (P2P)dlsym(api.so, "ncclSend");
        api.recv = (P2P)dlsym(api.so, "ncclRecv");
        api.error_string = (ErrStr)dlsym(api.so, "ncclGetErrorString");
        if (!api.comm_init_all || !api.comm_destroy || !api.group_start || !api.group_end || !api.send || !api.recv ||
            !api.error_string)
            load_err = "librccl: missing entry points";
    });
    if (!load_err.empty()) {
        if (err)
            *err = load_err;
        return nullptr;
    }
    return &api;
}

Renderer::MultiDev::~MultiDev()
{
    if (!comms.empty())
        if (RcclApi* api = RcclApi::get(nullptr))
            for (void* c : comms)
                if (c)
                    api->comm_destroy(c);
}

int Renderer::set_devices(const int* ids, int n)
{
    if (n == 0 || !ids) {
        multi_.reset();
        return RT_OK;
    }
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess)
        return hip_fail(e, "hipGetDeviceCount");
    if (n < 0 || n > 64)
        return fail(RT_EINVAL, "rt_set_devices: n out of range");
    if (ids[0] != device_)
        return fail(RT_EINVAL, "rt_set_devices: ids[0] must be the handle's device");
    // distinct devices, or the lead's device repeated (several renderers on one device: the
    // band path without RCCL, for tests on a one-device machine)
    bool one_device = true;
    for (int i = 0; i < n; i++)
        one_device = one_device && ids[i] == device_;
    if (!one_device && n > ndev)
        return fail(RT_EINVAL, "rt_set_devices: more devices than the machine has");
    if (!one_device) {
        const char* v = getenv("RT_MULTIDEV_RCCL");
        if (!v || v[0] == '0')
            return fail(RT_EUNSUPPORTED, "rt_set_devices: distinct devices (RCCL) are experimental, not yet run on a "
                                         "multi-GPU machine; set RT_MULTIDEV_RCCL=1 to use them");
    }
    std::set<int> seen;
    for (int i = 0; i < n && !one_device; i++)
        if (ids[i] < 0 || ids[i] >= ndev || !seen.insert(ids[i]).second)
            return fail(RT_EINVAL, "rt_set_devices: device ids must be distinct and in range");
    auto M = std::make_unique<MultiDev>();
    M->one_device = one_device;
    M->ids.assign(ids, ids + n);
    M->gather.device = device_;
    for (int i = 1; i < n; i++) {
        auto h = std::make_unique<Renderer>(ids[i]);
        std::string err;
        if (h->init(err) != RT_OK)
            return fail(RT_EHIP, "rt_set_devices: device " + std::to_string(ids[i]) + ": " + err);
        h->lead_ = this;   // its scene comes from this renderer's build (adopt_from_lead)
        M->helpers.push_back(std::move(h));
        auto b = std::make_unique<DevBuf>();
        b->device = ids[i];
        M->bands.push_back(std::move(b));
    }
    if (n > 1 && !one_device) {
        std::string err;
        RcclApi* api = RcclApi::get(&err);
        if (!api)
            return fail(RT_EUNSUPPORTED, "rt_set_devices: " + err);
        M->comms.assign(n, nullptr);
        int r = api->comm_init_all(M->comms.data(), n, M->ids.data());
        if (r != 0) {
            M->comms.clear();
            return fail(RT_EHIP, std::string("ncclCommInitAll: ") + api->error_string(r));
        }
    }
    multi_ = std::move(M);
    hipSetDevice(device_);
    return RT_OK;
}

// The helpers' copy of the lead's scene: the small state every frame, geometry / materials /
// textures when the lead's versions moved (each change there bumps one).
void Renderer::mirror_from(const Renderer& L)
{
    if (knobs_.exact != L.knobs_.exact)
        set_exact(L.knobs_.exact);
    set_settings(L.s_);   // flags the geometry when the BVH parameters changed
    std::memcpy(cam_pos_, L.cam_pos_, sizeof(cam_pos_));
    fov_ = L.fov_;
    near_ = L.near_;
    far_ = L.far_;
    aspect_ = L.aspect_;
    std::memcpy(proj_, L.proj_, sizeof(proj_));
    std::memcpy(proj_inv_, L.proj_inv_, sizeof(proj_inv_));
    std::memcpy(c2w_, L.c2w_, sizeof(c2w_));
    std::memcpy(w2c_, L.w2c_, sizeof(w2c_));
    std::memcpy(light_, L.light_, sizeof(light_));
    shape_kind_ = L.shape_kind_;
    shape_ = L.shape_;
    shape_mat_ = L.shape_mat_;
    if (mir_geom_ != L.geom_ver_) {
        tri_ = L.tri_;
        tri_mat_ = L.tri_mat_;
        tri_mat_lo_ = L.tri_mat_lo_;
        tri_mat_hi_ = L.tri_mat_hi_;
        tri_uv_ = L.tri_uv_;
        std::memcpy(prev_object_, L.prev_object_, sizeof(prev_object_));
        has_bvh_ = L.has_bvh_;
        geom_dirty_ = true;
        tri9_dirty_ = true;
        mir_geom_ = L.geom_ver_;
    }
    if (mir_mats_ != L.mats_ver_) {
        mats_ = L.mats_;
        mats_dirty_ = true;
        mir_mats_ = L.mats_ver_;
    }
    if (mir_tex_ != L.tex_ver_) {
        for (int i = 0; i < TEX_SLOTS; i++)
            tex_[i] = L.tex_[i];
        for (int i = 0; i < 6; i++)
            sky_[i] = L.sky_[i];
        tex_dirty_ = true;
        mir_tex_ = L.tex_ver_;
    }
}

// render(Renderer&) over the devices of rt_set_devices: every rank renders its bands
// (final resolution, SSAA applied), the helpers' bands go to the lead over RCCL, and the lead
// re-assembles them into its image (what rt_get_image returns).
int Renderer::render_multi()
{
    MultiDev& M = *multi_;
    const int n = (int)M.ids.size(), band = MultiDev::BAND_ROWS;
    const int W = s_.image_width, H = s_.image_height;
    const int lrows = local_rows(band, 0, n);
    if (lrows < 0)
        return fail(RT_EINVAL, "render_multi: bad band layout");
    const size_t chunk = (size_t)lrows * W * 4;
    auto t0 = std::chrono::steady_clock::now();
    hipError_t e = hipSetDevice(device_);
    if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
    // the lead's scene first: the helpers copy its build (one host build per geometry change)
    {
        int rc0 = ensure_device_scene();
        if (rc0 != RT_OK)
            return rc0;
    }
    if ((e = M.gather.reserve(chunk * n)) != hipSuccess) return hip_fail(e, "hipMalloc (gather)");
    for (int i = 1; i < n; i++) {
        Renderer& h = *M.helpers[i - 1];
        h.mirror_from(*this);
        if ((e = hipSetDevice(M.ids[i])) != hipSuccess || (e = M.bands[i - 1]->reserve(chunk)) != hipSuccess)
            return hip_fail(e, "hipMalloc (band buffer)");
    }
    // rank 0 renders straight into its gather slot, the others into their band buffers
    hipSetDevice(device_);
    int rc = render_bands_device(band, 0, n, M.gather.as<uint32_t>(), stream_);
    if (rc != RT_OK)
        return rc;
    for (int i = 1; i < n && rc == RT_OK; i++) {
        Renderer& h = *M.helpers[i - 1];
        hipSetDevice(M.ids[i]);
        rc = h.render_bands_device(band, i, n, M.bands[i - 1]->as<uint32_t>(), nullptr);
        if (rc != RT_OK)
            err_ = "device " + std::to_string(M.ids[i]) + ": " + h.err_;
    }
    hipSetDevice(device_);
    if (rc != RT_OK)
        return rc;
    if (n > 1 && M.one_device) {
        for (int i = 1; i < n && e == hipSuccess; i++) {
            e = hipStreamSynchronize(M.helpers[i - 1]->stream_);
            if (e == hipSuccess)
                e = hipMemcpyAsync(M.gather.as<uint8_t>() + (size_t)i * chunk, M.bands[i - 1]->p, chunk,
                                   hipMemcpyDeviceToDevice, stream_);
        }
        if (e != hipSuccess)
            return hip_fail(e, "band copy");
    } else if (n > 1) {
        RcclApi* api = RcclApi::get(nullptr);
        int r = api->group_start();
        for (int i = 1; i < n && r == 0; i++) {
            r = api->send(M.bands[i - 1]->p, chunk, ncclUint8, 0, M.comms[i], M.helpers[i - 1]->stream_);
            if (r == 0)
                r = api->recv(M.gather.as<uint8_t>() + (size_t)i * chunk, chunk, ncclUint8, i, M.comms[0], stream_);
        }
        int r2 = api->group_end();
        if (r != 0 || r2 != 0)
            return fail(RT_EHIP, std::string("RCCL band gather: ") + api->error_string(r != 0 ? r : r2));
    }
    // band b is local band b / n of rank b % n
    {
        std::lock_guard<std::recursive_mutex> g(image_mu_);
        if ((e = d_image_.reserve((size_t)W * H * 4)) != hipSuccess) return hip_fail(e, "hipMalloc (image)");
    }
    const int nb = (H + band - 1) / band;
    for (int b = 0; b < nb && e == hipSuccess; b++) {
        const int rows = std::min(band, H - b * band);
        const uint8_t* src = M.gather.as<uint8_t>() + (size_t)(b % n) * chunk + (size_t)(b / n) * band * W * 4;
        e = hipMemcpyAsync(d_image_.as<uint8_t>() + (size_t)b * band * W * 4, src, (size_t)rows * W * 4,
                           hipMemcpyDeviceToDevice, stream_);
    }
    if (e == hipSuccess)
        e = hipStreamSynchronize(stream_);
    for (int i = 1; i < n && e == hipSuccess; i++) {
        hipSetDevice(M.ids[i]);
        e = hipStreamSynchronize(M.helpers[i - 1]->stream_);
    }
    hipSetDevice(device_);
    if (e != hipSuccess)
        return hip_fail(e, "render_multi");
    std::lock_guard<std::recursive_mutex> g(image_mu_);
    img_w_ = W;
    img_h_ = H;
    img_is_internal_ = false;
    rendered_ = true;
    aux_valid_ = false;
    ssao_ready_ = false;
    post_ms_ = 0;
    kernel_ms_ = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return RT_OK;
}

}  // namespace rt
