"""Frame-engine invariants on the GPU: the risk words' event survives the caller's
stream; the heavy-tiles-first order and the split tiles (4 parts, lane groups) trace every tile exactly
once, C4 included; hair1m frames; the reflection engine's long-query deferral on and off; camera and
light moves after the SAH tree is resident.  Every frame is compared with the oracle.  Reference path:
Renderer::ray_trace (renderer.cpp:1068-1116), whose rows and tiles are independent."""
import ctypes

import numpy as np
import pytest

from oracle.bindings import Oracle

pytestmark = pytest.mark.gpu


@pytest.fixture
def make_renderer():
    import os
    from raytracercpp_amd.renderer import Renderer
    made = []

    def make(**env):
        old = {k: os.environ.get(k) for k in env}
        os.environ.update({k: str(v) for k, v in env.items()})
        try:
            r = Renderer(0)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        made.append(r)
        return r
    yield make
    for r in made:
        r.close()


def test_risk_words_after_the_band_stream_is_destroyed(make_renderer):
    """The frame's risk words are computed on the first band launch's stream; that stream is then
    destroyed, and the next launches (same camera and light: they only wait for the words' event)
    run on new streams.  Every frame equals the one-call render."""
    import torch
    from raytracercpp_amd import scenes
    from raytracercpp_amd.strips import assemble
    R = make_renderer()
    sc, st = scenes.bumpy70k(width=160, height=96)
    R.load_scene(sc, st)
    R.ray_trace()
    R.finish_accel()
    hip = ctypes.CDLL("libamdhip64.so")
    band, nranks = 8, 2
    full = None
    for rep in range(3):
        if rep == 1:
            R.set_light_position((2.0, 4.0, 1.0))   # new words, computed on this round's first stream
        R.ray_trace()
        R.post_process()
        full = R.get_image()
        parts = []
        for rank in range(nranks):
            h = ctypes.c_void_p()
            assert hip.hipStreamCreate(ctypes.byref(h)) == 0
            b = torch.zeros((R.local_rows(band, rank, nranks), st.image_width), dtype=torch.int32, device="cuda:0")
            torch.cuda.synchronize()
            R.render_bands_device(band, rank, nranks, b.data_ptr(), h.value)
            assert hip.hipStreamSynchronize(h) == 0
            assert hip.hipStreamDestroy(h) == 0   # the stream the risk words were computed on is gone
            parts.append(b.cpu().numpy().view(np.uint32))
        assert np.array_equal(assemble(parts, st.image_height, band), full), rep


def _heavy_tiles(cost, nwaves=None, split=0.5):
    """heavy_prep_kernel's rule (kernels.hip): tiles costing >= max(4 x mean, max / 8), at most
    ntiles / 16 of them; with nwaves (the plain kernel's waves), the number of those split into parts
    (cost >= split x the sum / nwaves)."""
    c = cost.ravel().astype(np.uint64)
    thr = max(4 * int(c.sum() // c.size), int(c.max()) // 8)
    heavy = (c >= thr) & (c > 0)
    if nwaves is None:
        return min(int(heavy.sum()), c.size // 16)
    return min(int((heavy & (c >= max(thr, int(split * float(c.sum()) / nwaves)))).sum()), c.size // 16)


@pytest.mark.parametrize("ssaa,group", [(False, 4), (True, 4), (False, 0), (True, 0)])
def test_heavy_first_frames_trace_every_tile_once(make_renderer, ssaa, group):
    """Heavy tiles first (Renderer::prepare_heavy): each frame takes the previous frame's costliest
    tiles first; the costliest of them split into parts traced with a lane group per pixel
    (trace_split_part; RT_HEAVY_GROUP=0: none split).  The light moves between frames, so a tile that was skipped would keep the
    previous frame's pixels and one traced twice would show no difference only if both traces agree:
    every frame must equal the oracle's for its own light, and the heavy list must not be empty."""
    from raytracercpp_amd import scenes
    R = make_renderer(RT_HEAVY_GROUP=group)
    sc, st = scenes.bumpy70k(width=160, height=96, enable_ssaa=ssaa, ssaa_factor=2)
    R.load_scene(sc, st)
    R.ray_trace()
    R.finish_accel()
    R.request_aux(hit=True, shadow=True)
    lights = [(3.0, 3.0, 2.0), (-2.0, 3.5, 1.0), (0.5, -3.0, 2.5), (3.0, 0.5, -1.0)]
    heavy = []
    for L in lights:
        R.set_light_position(L)
        c = R.tile_costs()
        # (the plain kernel's grid at this size: one wave per tile)
        heavy.append((_heavy_tiles(c), _heavy_tiles(c, nwaves=c.size) if group > 1 else 0))
        R.ray_trace()
        g = R.get_internal(argb=True, hit=True, shadow=True)
        sc.light = np.asarray(L, np.float32)
        o = Oracle(sc, st).render_rows()
        assert np.array_equal(g["hit_id"], o.hit_id), L
        assert np.array_equal(g["shadow"], o.shadow), L
        assert np.array_equal(g["argb"], o.argb), L
        R.post_process()
        rw, rh = st.render_size()
        exp = Oracle.downscale(o.argb, rw, rh, 2) if ssaa else o.argb
        assert np.array_equal(R.get_image().ravel(), exp), L
        assert R.stats()["shadow_rays"] == o.counters["shadow_rays"], L   # each pixel's shadow ray counted once
    print("heavy tiles (all, split) per frame:", heavy)
    assert min(h[0] for h in heavy) > 0
    if group > 1:
        assert min(h[1] for h in heavy) > 0   # tiles were split into parts


@pytest.mark.parametrize("group,quick", [(4, 1), (4, 0)])
def test_c4_heavy_parts_match_oracle(make_renderer, group, quick):
    """The benchmark workload (C4) with its heavy tiles split into parts (trace_split_part: G lanes per
    pixel walking one pixel's wide-BVH query together, wbvh_closest<.., G>).  Frame 0 runs right after
    the scene load: on the quick wide BVH (quick = 1, the default), or with
    RT_WBVH_QUICK_FIRST=0 on the octree-only plain kernel ray_trace_kernel<false, true, true>.  Then two
    frames on the SAH tree (heavy lists from the previous frames' tile costs), every internal pixel bit
    for bit; then the band path with the SSAA box filter fused into the tiles and the split parts."""
    import torch
    from raytracercpp_amd import scenes
    from raytracercpp_amd.strips import assemble
    R = make_renderer(RT_HEAVY_GROUP=group, RT_WBVH_QUICK_FIRST=quick)
    sc, st = scenes.sphere1m()
    o = Oracle(sc, st).render_rows()
    R.load_scene(sc, st)
    R.request_aux(hit=True, shadow=True)
    rw, rh = st.render_size()
    exp = Oracle.downscale(o.argb, rw, rh, 2)
    heavy = []
    for frame in range(3):
        if frame:
            heavy.append(_heavy_tiles(R.tile_costs()))
        R.ray_trace()
        g = R.get_internal(argb=True, hit=True, shadow=True)
        assert np.array_equal(g["hit_id"], o.hit_id), f"frame {frame}: {int((g['hit_id'] != o.hit_id).sum())} hit-ID mismatches"
        assert np.array_equal(g["hit_t"].view(np.uint32), o.hit_t.view(np.uint32)), frame
        assert np.array_equal(g["shadow"], o.shadow), frame
        assert np.array_equal(g["argb"], o.argb), frame
        assert R.stats()["shadow_rays"] == o.counters["shadow_rays"], frame
        if frame == 0:
            assert R.stats()["wide_tree"] in ((1, 2) if quick else (0, 2))   # (the SAH tree may be adopted already)
            R.finish_accel()
            assert R.stats()["wide_tree"] == 2   # the SAH tree adopted
    assert min(heavy) > 0, heavy
    band, nranks = 8, 2   # output rows per band (16 internal rows)
    for rep in range(3):   # the first launch per slot has no tile costs yet: no heavy list
        parts = []
        for rank in range(nranks):
            b = torch.zeros((R.local_rows(band, rank, nranks), st.image_width), dtype=torch.int32, device="cuda:0")
            torch.cuda.synchronize()
            R.render_bands_device(band, rank, nranks, b.data_ptr(), 0)
            torch.cuda.synchronize()
            parts.append(b.cpu().numpy().view(np.uint32))
        assert np.array_equal(assemble(parts, st.image_height, band).ravel(), exp), rep
    print(f"C4 heavy tiles per frame (G = {group}):", heavy)


@pytest.mark.parametrize("camera", ["default", "grazing"])
def test_hair1m_frame_matches_oracle(make_renderer, camera):
    """SURVEY.md 8(d)'s hair1m stress scene (1M crossing ribbon triangles, BASELINE configs[3]'s hair /
    mesh scene) at reduced resolution, first frame on the octree path and the next ones on the wide BVH
    (its sound query and the camera / light risk words): every internal pixel's hit ID, t, shadow flag
    and ARGB bit for bit, the SSAA frame too.  'grazing': the camera moved to the hair's silhouette."""
    from raytracercpp_amd import scenes
    R = make_renderer()
    sc, st = scenes.hair1m(width=240, height=136)
    if camera == "grazing":
        sc.cam_pos = np.array([0.0, 1.62, -0.2], np.float32)
        sc.cam_to_world = np.array([1, 0, 0, 0.0, 0, 1, 0, 1.62, 0, 0, 1, -0.2, 0, 0, 0, 1], np.float32)
    o = Oracle(sc, st).render_rows()
    R.load_scene(sc, st)
    R.request_aux(hit=True, shadow=True)
    for frame in ("octree", "wide BVH"):
        R.ray_trace()
        g = R.get_internal(argb=True, hit=True, shadow=True)
        assert np.array_equal(g["hit_id"], o.hit_id), f"{frame}: {int((g['hit_id'] != o.hit_id).sum())} hit-ID mismatches"
        assert np.array_equal(g["hit_t"].view(np.uint32), o.hit_t.view(np.uint32)), frame
        assert np.array_equal(g["shadow"], o.shadow), frame
        assert np.array_equal(g["argb"], o.argb), frame
        R.post_process()
        rw, rh = st.render_size()
        assert np.array_equal(R.get_image().ravel(), Oracle.downscale(o.argb, rw, rh, 2)), frame
        R.finish_accel()
    print(f"hair1m {camera}: {int((o.hit_id >= 0).sum())} of {o.hit_id.size} pixels hit, "
          f"{o.counters['shadow_rays']} shadow rays")


@pytest.mark.parametrize("defer,feed,sfeed", [("48", "0", "0"), ("0", "0", "0"), ("6", "0", "24"), ("32", "16", "1"),
                                               ("32", "1", "64"), ("32", "64", "16"), ("32", "24", "0")])
def test_reflection_deferral_matches_oracle(make_renderer, defer, feed, sfeed):
    """The reflection engine's long-query deferral (RT_REFL_DEFER=k: queries past k loop iterations of
    refl_trace_kernel finish in refl_trace_long_kernel; 0: never deferred) and its lane refill
    (RT_REFL_FEED=k: refl_trace_feed_kernel's persistent waves take new queries when k lanes wait, the
    uncertified ones deferred; RT_REFL_SHADOW_FEED=k: the same for the shadow pass,
    refl_shadow_feed_kernel) change only where a query runs: C5's features at a reduced size, first on
    the quick wide BVH (the frame right after the scene load), then on the SAH tree, equal
    the oracle bit for bit."""
    from raytracercpp_amd import scenes
    sc, st = scenes.sphere1m_refl(width=64, height=36, samples=4)
    st = st.copy(max_recursion_depth=3)
    o = Oracle(sc, st).render_rows()
    R = make_renderer(RT_REFL_DEFER=defer, RT_REFL_FEED=feed, RT_REFL_SHADOW_FEED=sfeed)
    R.load_scene(sc, st)
    R.request_aux(hit=True, shadow=True)
    for frame in ("quick tree", "SAH tree"):
        R.ray_trace()
        g = R.get_internal(argb=True, hit=True, shadow=True)
        assert np.array_equal(g["hit_id"], o.hit_id), frame
        assert np.array_equal(g["shadow"], o.shadow), frame
        assert np.array_equal(g["argb"], o.argb), f"{frame}: {int((g['argb'] != o.argb).sum())} ARGB mismatches"
        assert R.stats()["reflection_rays"] == o.counters["reflection_rays"], frame
        R.finish_accel()


@pytest.mark.parametrize("major,sorted_frames,frame_order,shadow_sort", [
    ("1", "1", "0", "1"), ("1", "0", "0", "1"), ("0", "1", "0", "1"), ("0", "0", "0", "0"), ("1", "1", "1", "1"),
    ("1", "1", "0", "0"), ("1", "1", "0", "1+dir"), ("0", "0", "0", "0+dir"), ("1", "1", "0", "1+defer"), ("1", "1", "0", "1-xcd"), ("0", "1", "1", "1-xcd")])
def test_reflection_engine_layouts_match_oracle(make_renderer, major, sorted_frames, frame_order, shadow_sort):
    """The reflection engine's storage layouts change only where its records live: sample-major or
    frame-major slots (RT_REFL_SAMPLE_MAJOR, kernels.hip slot_of), the frames read from their sorted
    copy or through the sort order (RT_REFL_SORTED_FRAMES, refl_sort_frames_kernel), the feed's tickets
    in slot or frame order (RT_REFL_FEED_FRAME_ORDER), the shadow list sorted by hit point or in append
    order (RT_REFL_SHADOW_SORT, refl_shadow_keys_kernel), the feed's tickets over the slots grouped by
    direction bin (RT_REFL_DIR_SORT, refl_dir_keys_kernel; "+dir"), the deferred queries in their frames'
    order or in the order deferred (RT_REFL_DEFER_SORT, refl_defer_keys_kernel; "+defer"), the feed's
    tickets in eighths per XCD or one ticket (RT_REFL_FEED_XCD; "-xcd": one ticket).  C5's features at a reduced size, on the quick
    tree and then the SAH tree, equal the oracle bit for bit in every combination."""
    from raytracercpp_amd import scenes
    sc, st = scenes.sphere1m_refl(width=64, height=36, samples=4)
    st = st.copy(max_recursion_depth=3)
    o = Oracle(sc, st).render_rows()
    R = make_renderer(RT_REFL_SAMPLE_MAJOR=major, RT_REFL_SORTED_FRAMES=sorted_frames,
                      RT_REFL_FEED_FRAME_ORDER=frame_order, RT_REFL_SHADOW_SORT=shadow_sort[0],
                      RT_REFL_DIR_SORT=int(shadow_sort.endswith("+dir")),
                      RT_REFL_DEFER_SORT=int(shadow_sort.endswith("+defer")),
                      RT_REFL_FEED_XCD=int(not shadow_sort.endswith("-xcd")))
    R.load_scene(sc, st)
    R.request_aux(hit=True, shadow=True)
    for frame in ("quick tree", "SAH tree"):
        R.ray_trace()
        g = R.get_internal(argb=True, hit=True, shadow=True)
        assert np.array_equal(g["hit_id"], o.hit_id), frame
        assert np.array_equal(g["shadow"], o.shadow), frame
        assert np.array_equal(g["argb"], o.argb), f"{frame}: {int((g['argb'] != o.argb).sum())} ARGB mismatches"
        assert R.stats()["reflection_rays"] == o.counters["reflection_rays"], frame
        R.finish_accel()


def test_camera_and_light_moves_after_finish_accel(make_renderer):
    """After the SAH tree is resident (rt_finish_accel), the camera and the light move between frames
    (new camera / light risk words each time, Renderer::prepare_risk): every frame equals the oracle's
    for its own camera and light."""
    from raytracercpp_amd import _lib, scenes
    from raytracercpp_amd.scene import SceneData
    sc, st = scenes.bumpy70k(width=160, height=96)
    R = make_renderer()
    R.load_scene(sc, st)
    R.ray_trace()
    R.finish_accel()
    R.request_aux(hit=True, shadow=True)
    moves = [(None, (2.0, 4.0, 1.0)), (_lib.make_transform("ry", 12), None), (_lib.make_transform("rx", -8), (-3.0, 2.0, 2.0)),
             (_lib.compose(_lib.make_transform("translation", 0.3, -0.2, 0.4), _lib.make_transform("rz", 5)), None)]
    light = np.asarray(sc.light, np.float32)
    for k, (cam, L) in enumerate(moves):
        if cam is not None:
            R.set_camera_transform(cam)
        if L is not None:
            R.set_light_position(L)
            light = np.asarray(L, np.float32)
        R.ray_trace()
        g = R.get_internal(argb=True, hit=True, shadow=True)
        sc2 = SceneData(**vars(sc))
        sc2.cam_pos, sc2.proj_inv, sc2.cam_to_world = R.get_camera_matrices()
        sc2.light = light
        o = Oracle(sc2, st).render_rows()
        assert np.array_equal(g["hit_id"], o.hit_id), k
        assert np.array_equal(g["shadow"], o.shadow), k
        assert np.array_equal(g["argb"], o.argb), k


def test_origin_cones_device_grid(make_renderer):
    """The origin cones (ocone.hpp) the renderer builds on the device once the SAH tree is
    adopted (ocone_kernel): every cell's word equals the host builder's (ocone_cell on the CPU) up to one
    step of the rounded-up half-angle, and the device grid passes the brute-force soundness check
    (rt_ocone_check: no triangle nearly parallel to a ray that skips case (b) reports a hit) on
    reflection-like, grazing and random rays; RT_OCONE=0 builds none."""
    from raytracercpp_amd import _lib, scenes
    from test_ocone import _rays
    sc, st = scenes.uv_sphere_scene(200, 100, 1.5, 0.0, 160, 96)
    sc.materials[0, 12] = 0.5
    R = make_renderer(RT_OCONE_DIM=64)
    R.load_scene(sc, st)
    R.ray_trace()
    R.finish_accel()
    cells, dims, lo_ih = R.ocone_read()
    tri9 = np.asarray(sc.tri, np.float32).reshape(-1, 9)
    o, d = _rays(tri9, 2000, seed=9)
    skip, stats, host = _lib.ocone_check(tri9, o, d, st.bvh_max_depth, st.bvh_leaf_object_count, ocone_dim=64,
                                         want_cells=True)
    host = host[: len(cells)]
    assert stats["violations"] == 0, stats
    code_d, code_h = cells[:, 1] >> 16, host[:, 1] >> 16
    same = np.all(cells == host, axis=1)
    special = (code_d >= 0x7FFE) | (code_h >= 0x7FFE)
    assert np.array_equal(code_d[special], code_h[special])
    assert np.array_equal(cells[:, 0], host[:, 0]) and np.array_equal(cells[:, 1] & 0xFFFF, host[:, 1] & 0xFFFF)
    assert np.abs(code_d.astype(np.int64) - code_h.astype(np.int64)).max() <= 1
    skip_d, sd = _lib.ocone_check(tri9, o, d, st.bvh_max_depth, st.bvh_leaf_object_count, ocone_dim=64,
                                  grid=(cells, dims, lo_ih))
    assert sd["violations"] == 0 and sd["skipping"] > 0, sd
    print(f"device grid {dims.tolist()}: {int(same.sum())} of {len(cells)} words equal the host's; "
          f"rays skipping (b) {sd['skipping']} of {len(o)}")
    # RT_OCONE=0: no grid
    R2 = make_renderer(RT_OCONE=0)
    R2.load_scene(sc, st)
    R2.ray_trace()
    R2.finish_accel()
    with pytest.raises(_lib.RtError):
        R2.ocone_read()
