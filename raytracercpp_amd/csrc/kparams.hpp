// kparams.hpp -- plain-old-data launch parameters shared by the host library
// and the kernels (passed by value as the kernel argument).
#pragma once

#include <stdint.h>

#include "octree.hpp"
#include "ocone.hpp"
#include "wbvh.hpp"

namespace rt {

// The split tiles' lane-group size G (kernels.hip trace_split_part; one instantiation in the plain
// kernel): a part is SPLIT_COLS x SPLIT_ROWS = 64 / G pixels of its 8 x 8 tile
#ifndef RT_SPLIT_G
#define RT_SPLIT_G 4
#endif
constexpr int SPLIT_G = RT_SPLIT_G;
constexpr int SPLIT_COLS = SPLIT_G == 8 ? 4 : 8;
constexpr int SPLIT_ROWS = 64 / SPLIT_G / SPLIT_COLS;
static_assert(SPLIT_G == 2 || SPLIT_G == 4 || SPLIT_G == 8, "2, 4 or 8 lanes per pixel");

constexpr int TEX_SLOTS = 6;   // ao, diffuse, normal, displacement, roughness, skysphere (renderer.h:77-84)
constexpr int MAT_STRIDE = 16; // see include/rt_mi355x.h
constexpr int MAX_SHAPES = 64;
constexpr int NCOUNTERS = 32;  // KParams::counters entries (u64) before the tile-queue heads
constexpr int TILE_SHARDS = 8;  // tile-queue shards (blockIdx % TILE_SHARDS; a power of 2; r02: 16 was slower)
constexpr int NCOUNTER_WORDS = NCOUNTERS + 16 * TILE_SHARDS;  // one 128-B line per shard head
constexpr int DBG_WAVES = 16384;   // per-wave diagnostic records (RT_PHASE_TIME builds)
constexpr int DBG_WORDS = 8;       // u64 words per record

enum TexSlot { TEX_AO = 0, TEX_DIFFUSE = 1, TEX_NORMAL = 2, TEX_DISPLACEMENT = 3, TEX_ROUGHNESS = 4, TEX_SKYSPHERE = 5 };
enum Shading { RT_SHADING = 0, ABS_NORMALS = 1, PASTEL_NORMALS = 2, BARYCENTRIC = 3, VISUALIZE_AO = 4 };

struct KTex {
    const float4* px;   // row-major texels (Image, tp2/src/image.h:20-135), nullptr when absent
    int w, h;
};

struct KParams {
    // geometry (flattened octree, octree.hpp)
    const GNode* nodes;
    const GTri* tris;
    const int32_t* tri_id;    // GTri slot -> caller triangle index
    const int32_t* tri_mat;   // caller index -> material
    const float* tri_uv;      // caller index -> u0 u1 u2 v0 v1 v2 (nullptr: (-1,-1,-1))
    const float* cones;       // [4] per GTri slot, set at each leaf's first slot: normal cone (axis, cos);
                              // nullptr: no cones (kernels.hip leaf_backfacing)
    const float* lslab;       // [8] per GTri slot, at each leaf's first slot: box lo xyz, smin, hi xyz, smax
                              // along the cone axis; nullptr: none (kernels.hip leaf_missed)
    float scene_scale;        // largest |vertex coordinate| (leaf_missed's margin)
    const float* lsin;        // per GTri slot, at each leaf's first slot: <= sin(angle at a) of its triangles
    // the wide BVH (wbvh.hpp; nullptr: off) -- closest-hit queries certified against the octree
    const WNode* wnodes;
    const GTri* wtris;           // octree records in wide-BVH leaf order
    const uint4* wmeta;          // wide-BVH triangle k -> {octree GTri slot, flattened octree leaf node (its
                                 // certificate's k-DOP), caller triangle index, material}
    // the frame's grazing-risk words (wbvh.hpp wrisk_pack; nullptr: every child runs the full case (b)):
    // wrisk[(2 node + sel) 4 + j], sel 0 for rays from cam_pos, 1 for shadow rays towards light whose
    // segment bound hi <= risk_G and normal |n|_1 <= risk_nl (kernels.hip is_shadowed); risk_nu: the
    // light's nu (WRiskArgs::ray_nu)
    const uint64_t* wrisk;
    float risk_G, risk_nl, risk_nu;
    // the risk caps (wbvh.hpp risk_cap_skip; with wrisk): risk_cap[sel] >= |cos(N, cap_dir[sel])| of every
    // triangle at risk for the camera (sel 0) / the light (sel 1), computed with the words
    const float* risk_cap;
    float cap_dir[2][3];
    // the origin cones (ocone.hpp; cells nullptr: none resident): the rays without risk words whose
    // ocone_skip holds skip case (b) (the reflection queries, ReflFeed)
    OConeView ocone;
    int32_t nnodes;
    int32_t ntri_slots;       // GTri count (brute-force loop bound when enable_bvh == 0)
    int32_t levels;           // flattened tree depth + 1 (LDS level-stack entries per lane)

    int32_t nshape;
    int32_t shape_kind[MAX_SHAPES];
    float shape[MAX_SHAPES][6];
    int32_t shape_mat[MAX_SHAPES];

    const float* mats;        // [nmat][16]
    int32_t nmat;

    float cam_pos[3];
    float proj_inv[16];
    float cam_to_world[16];
    float light[3];
    // Ray generation shortcuts (kernels.hip camera_dir), set on the host when they give the same
    // bits as Transform::operator()(Point) (mat.cpp:83-100) for every pixel:
    //   proj_mode 1: proj_inv's w row makes w == 1 for every image-plane point; 2: w is the same
    //   value 1 / proj_w_den for every one (row 3 = (0, 0, c, d)), proj_w = that reciprocal;
    //   0: per pixel.  c2w_affine: cam_to_world's row 3 is (0, 0, 0, 1) (w == 1 for finite points).
    int32_t proj_mode;
    float proj_w;
    int32_t c2w_affine;

    KTex tex[TEX_SLOTS];
    KTex sky[6];

    // RenderSettings (rendererSettings.h:6-105)
    int32_t shading_method;
    int32_t compute_shadows;
    int32_t max_recursion_depth;
    int32_t enable_bvh;
    int32_t enable_ambient, enable_diffuse, enable_specular, enable_emissive;
    int32_t rough_reflections_sample_count;
    int32_t enable_ao_mapping, enable_diffuse_mapping, enable_normal_mapping, enable_displacement_mapping;
    float displacement_mapping_strength;
    int32_t parallax_mapping_steps;
    int32_t enable_roughness_mapping, enable_skysphere, enable_skybox;
    uint32_t rng_seed;
    int32_t has_reflection;   // RT_SHADING with a material whose reflection > 0: the reflection engine
    float seg_scale;          // > 0: shadow queries end at the light (kernels.hip is_shadowed's hi, with
                              // seg_margin's rounding bound), the scene's largest |coordinate|; 0: none
    int32_t seg_oct;          // 1: the octree walks only the volumes overlapping a shadow / reflection
                              // query's segment (assumes no grazing report falls outside its
                              // volumes, RT_SEG_OCTREE=1); 0 (default): the octree walks the whole line

    // image: render size (internal, after the SSAA factor) and this launch's rows
    int32_t rw, rh;
    int32_t band_rows;        // internal rows per band
    int32_t nranks, rank;     // bands b with b % nranks == rank are rendered (band_map == nullptr)
    // a band list (rt_render_band_list_device, cost-balanced strips): local band i is the global band
    // band_map[i]; band_inv[b] = the local band of global band b, or -1 (nullptr: the interleaved layout)
    const int32_t* band_map;
    const int32_t* band_inv;
    int32_t local_rows;       // rows in this launch's (padded) local buffers
    int32_t tiles_x, tiles_y; // 8x8 tiles over (rw, local_rows)
    int32_t max_blocks;       // persistent grid size (CUs x resident blocks per CU)
    int32_t plain;            // 1: no texture map, sky, analytic shape, debug shading or SSAO buffers
                              // (ray_trace_kernel's plain specialisation)
    // heavy tiles first (ray_trace_kernel, kernels.hip heavy_prep_kernel; nullptr: off): tile_cost
    // receives each tile's shader cycles; the launch's heavy_list[0 .. heavy_ctr[0]) (the previous
    // launch's slowest tiles of the same layout, flagged in heavy_bits) are dequeued first, by the
    // ticket heavy_ctr[1]; a list entry is the tile | its wave priority level << 28
    uint32_t* tile_cost;
    unsigned long long* tile_stats;   // this launch's sum and max of the tile costs (the next heavy_prep's input)
    const int32_t* heavy_list;
    const uint32_t* heavy_bits;
    int32_t* heavy_ctr;
    // 0: no split tiles; RT_SPLIT_G: heavy_prep_kernel's split tiles are traced first, each as G parts of
    // 64 / G pixels with G lanes per pixel (kernels.hip trace_split_part, by the ticket heavy_ctr[2]; the
    // parts add their cycles to tile_cost)
    int32_t heavy_group;
    int32_t split_parts;      // parts per split tile: G (64 / G pixels each, every lane busy) or 2 G (half)

    // outputs, indexed by local_row * rw + px (nullptr = not requested)
    uint32_t* argb;
    float4* rgba;
    int32_t* hit_id;
    float* hit_t;
    uint8_t* shadow;
    unsigned long long* counters;   // [NCOUNTERS]: [0] shadow rays, [1] reflection rays, [2] tile queue head
                                    // (reflection / raster kernels), [4..7] executed k-DOP / MT tests of
                                    // whole-line / segment queries, [10..11] wide-BVH node visits / triangle
                                    // tests, [12] uncertified queries, [14] certificate k-DOP tests, [16..21]
                                    // uncertified queries by reason (overflow, NaN, overflowed-only, tie, t
                                    // outside (0, inf), certificate failed), [22..27] wide-BVH loop iterations
                                    // (all but [0..2]: RT_COUNT builds only); then the tile-queue heads,
                                    // shard s at counters[NCOUNTERS + 16 s]
    unsigned long long* dbg;        // diagnostic builds (RT_PHASE_TIME): per wave [DBG_WAVES][DBG_WORDS], else nullptr
    // SSAO inputs (enable_ssao): Renderer::_z_buffer / _normal_buffer, renderer.cpp:1107-1110, 975-979
    float* zbuf;
    float4* nbuf;
    // fused SSAA downscale (band launches, ssaa_factor 2 / 4 / 8): each wave box-filters its
    // 8x8 tile's ARGB values across lanes and writes the (8 / f)^2 output pixels to ds_out
    // (local output row lr / f, width rw / f); argb is then nullptr.  nullptr: off.
    uint32_t* ds_out;
    int32_t ds_shift;         // log2(ssaa_factor)
};

// ---- SSAO (kernels.hip "Renderer::post_process_ssao_SIMD") ----
struct SsaoArgs {
    const float* z;          // _z_buffer, INFINITY where nothing was hit
    const float4* n;         // _normal_buffer (xyz)
    int32_t* ao;             // per-pixel occlusion counts
    uint32_t* argb;          // the internal image, blurred occlusion applied in place
    int32_t w, h;            // render size
    int32_t simd_w;          // w - w % 8: columns of the 8-lane loop; the rest take the scalar tail
    int32_t count;           // ssao_sample_count
    float radius, amount;    // ssao_radius, ssao_amount
    float fovm;              // (float)tan(fov / 2 / 180 * M_PI), renderer.cpp:1245 (double tan)
    float tanv;              // tanf(radians(fov / 2)), renderer.cpp:1379
    float aspect;            // Camera::_aspect_ratio
    uint32_t seed;
    float proj[16];          // Camera::_perspective_proj_mat
};

// ---- reflection engine (kernels.hip, "Reflections as frames") ----
// One Renderer::compute_reflection call (renderer.cpp:283-338) of one pixel.
struct FrameRec {
    float ro[3];        // hit point + n * 0.01
    float perfect[3];   // perfect reflection direction
    float n[3];         // (normal-mapped) normal of the hit that reflects
    float fc[3];        // shade_direct colour of that hit (shadow and emission applied)
    float rough;
    int32_t mat;
    uint32_t key;       // RNG key (path-keyed streams)
    int32_t nsamp;      // samples it traces: N (rough > 0), 1 (rough <= 0), 0 (N == 0)
    int32_t parent;     // launch-local pixel (level 1 frames)
};

// One sample of a frame: trace_ray(depth + 1) into the frame's shared HitInfo.
struct SampleRec {
    float d[3];         // direction
    int32_t kind;       // 0: colour final in fc (miss / depth limit), 1: shaded hit, 2: no sample
    float fc[3];        // shade_lit colour (kind 1) or the returned colour (kind 0)
    float ip[3];        // hit point
    float nrm[3];       // shading normal after normal mapping
    int32_t mat;
    float crough;       // roughness of the frame this hit spawns (reflective material)
    int32_t sh;         // is_shadowed
    int32_t child;      // frame index at the next level
    int32_t ray;        // 1: closest-hit query to trace
};

struct RawHit {
    float t, u, v;
    int32_t k;          // GTri slot, -1 none
    float d[3];         // the sample's direction (ReflArgs::fused; else in SampleRec::d)
    int32_t r;          // bit 0: the query's return value; bit 1 (fused): the sample traced a ray
};

struct ReflArgs {
    FrameRec* fr;            // this level's frames
    SampleRec* sm;           // the chunk's samples, (p - c0) * stride + i for sorted position p
    RawHit* hit;             // per sample
    float* ret;              // per frame of this level: colour returned to the parent sample (3 floats)
    const float* child_ret;  // the next level's ret
    FrameRec* child_fr;      // the next level's frames
    unsigned int* child_count;
    const int32_t* order;    // frame at sorted position p is order[p] (spatially sorted)
    const FrameRec* frs;     // (optional) the frames copied in sorted order: frs[p] = fr[order[p]]
    const int32_t* perm;     // (optional) the feed's ticket t takes slot perm[t] (slots grouped by direction)
    unsigned int* feed_parts;   // (optional) 8 tickets, one per eighth of the slots: a wave takes its XCD's
                                // eighth first, then the next ones (RT_REFL_FEED_XCD)
    int32_t* list;           // compacted sample slots with a shadow query
    unsigned int* list_count;
    int32_t c0, c1;          // sorted positions [c0, c1) of this level
    int32_t level;           // samples trace at depth = level
    int32_t stride;          // max(N, 1)
    int32_t sample_major;    // the slots' order (kernels.hip slot_of): 1 sample-major, 0 frame-major
    int32_t feed_frame_order;   // (sample-major) the feed hands out a frame's samples together
    int32_t fused;           // 1: pass1 builds the shadow list and the shadow pass spawns (no list /
                             // spawn kernels), and every sample's result is in res; 0: the separate
                             // passes (RT_REFL_FUSE=0), resolve reads the records
    float4* res;             // fused: per sample slot, the colour it returns (xyz) or, in w as int bits,
                             // the index of the child frame whose colour it returns (-1: xyz)
    int32_t* defer;          // sample slots whose query ran past max_steps in refl_trace_kernel (traced
    unsigned int* defer_count;   // again by refl_trace_long_kernel, whole waves of long queries); 0: off
    int32_t max_steps;
    // > 0: refl_trace_feed_kernel instead of refl_trace_kernel (persistent waves, lane refill when this
    // many lanes wait; the queries the wide BVH does not certify go to the defer list); feed_ticket: its
    // next slot
    int32_t feed;
    unsigned int* feed_ticket;
    // > 0 (fused only): the shadow pass by refl_shadow_feed_kernel (lane refill at this many waiting lanes;
    // shadow_ticket its next list entry), then refl_shadow_kernel over the entries it deferred (sdefer)
    int32_t shadow_feed;
    unsigned int* shadow_ticket;
    int32_t* sdefer;
    unsigned int* sdefer_count;
};

// ---- hybrid rasterisation (kernels.hip "Renderer::raster_trace") ----
// One clipped piece of a triangle, as raster_trace (renderer.cpp:869-1006) derives it.
struct RasterPiece {
    float na[3], nb[3], nc[3];   // Triangle(Triangle4): NDC vertices
    float wa[3], wb[3], wc[3];   // _camera_to_world_mat(proj_inv(NDC triangle)): trace_triangle's triangle
    float inv_area;
    float za, zb, zc;            // matrix_transform_z(cam_to_world, proj_inv(vertex))
    int32_t x0, y0, x1, y1;      // pixel bounding box (clamped)
    int32_t tri;                 // caller triangle index
    int32_t pad;
};

struct RasterArgs {
    const float* tri9;                 // caller triangles (world space), caller order
    int64_t ntri;
    float proj[16];                    // Camera::_perspective_proj_mat
    float w2c[16];                     // Camera::_world_to_camera_mat
    int32_t clipping;                  // RenderSettings::enable_clipping
    int32_t* count;                    // pieces per triangle
    const int32_t* offset;             // exclusive scan of count: first piece of each triangle
    RasterPiece* pieces;               // in (triangle, piece) order
    float* piece_uv;                   // [6] per piece: u0 u1 u2 v0 v1 v2 (the piece's texcoords)
    unsigned long long* zkey;          // per launch-local pixel: (ordered z << 32) | piece, min wins
    int32_t* big;                      // pieces whose bounding box is rasterised by a whole workgroup
    unsigned int* nbig;
};

}  // namespace rt
