// multidev.hpp -- single-process multi-device rendering (rt_set_devices).
//
// The reference renders a frame on one host (RenderThread::run, tp2/projets/QT/
// mainWindowThreads.cpp:39-65: render(renderer) then the display copy).  With N devices the
// lead renderer (the handle, on ids[0]) keeps the scene; one helper Renderer per other device
// mirrors it before each frame (Renderer::mirror_from: small state every frame, geometry /
// materials / textures when their version changed).  Every device renders the interleaved
// bands of BAND_ROWS output rows with band % N == its rank (render_bands_device, the same
// kernels as one process per GPU), the helpers' band buffers are sent to ids[0] with RCCL
// point-to-point (librccl loaded with dlopen at the first N > 1 call: the library keeps no
// link-time dependency on it), and the lead re-assembles the bands into its image.
#pragma once

#include <stdint.h>

#include <memory>
#include <string>
#include <vector>

#include "renderer.hpp"

namespace rt {

// the RCCL entry points used (rccl.h signatures, resolved from librccl.so at run time)
struct RcclApi {
    typedef int (*CommInitAll)(void** comms, int ndev, const int* devlist);
    typedef int (*CommDestroy)(void* comm);
    typedef int (*Group)();
    typedef int (*P2P)(const void* buf, size_t count, int dtype, int peer, void* comm, hipStream_t stream);
    typedef const char* (*ErrStr)(int);
    void* so = nullptr;
    CommInitAll comm_init_all = nullptr;
    CommDestroy comm_destroy = nullptr;
    Group group_start = nullptr, group_end = nullptr;
    P2P send = nullptr;
    P2P recv = nullptr;
    ErrStr error_string = nullptr;
    // loads librccl once per process; false with *err set when it cannot
    static RcclApi* get(std::string* err);
};

struct Renderer::MultiDev {
    static constexpr int BAND_ROWS = 8;   // output rows per band
    std::vector<int> ids;                 // ids[0] = the lead's device
    std::vector<std::unique_ptr<Renderer>> helpers;   // helpers[i - 1] renders rank i on ids[i]
    std::vector<void*> comms;             // ncclComm_t per rank (N > 1)
    std::vector<std::unique_ptr<DevBuf>> bands;   // bands[i]: rank i's band buffer on ids[i] (i >= 1)
    DevBuf gather;                        // on ids[0]: N slots of local_rows x width ARGB32
    bool one_device = false;              // every id is the lead's device: copies, no RCCL (tests)
    ~MultiDev();
};

}  // namespace rt
