"""Parity of the HIP path (librt_mi355x.so on cuda:0, through the C ABI) with the
reference-generated golden fixtures and with the oracle.  Bar: bit-exact hit IDs,
hit t, shadow flags and ARGB32; float RGBA within 1e-4 per channel (north_star)."""
import numpy as np
import pytest

from golden_cases import Case, case_names, manifest
from oracle.bindings import Oracle

pytestmark = pytest.mark.gpu

RGBA_TOL = 1e-4
CASES = case_names()


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


@pytest.fixture(scope="module")
def R():
    from raytracercpp_amd.renderer import Renderer
    r = Renderer(0)
    yield r
    r.close()


@pytest.fixture
def make_renderer():
    """A renderer created with diagnostic switches set in the environment (librt_mi355x reads
    them once, at rt_create: renderer.hpp Knobs); the environment is restored afterwards."""
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


def gpu_render(r, sc, st, aux=True):
    r.load_scene(sc, st)
    r.request_aux(rgba=aux, hit=aux, shadow=aux)
    if st.hybrid_rasterization_tracing:
        r.raster_trace()   # what render() runs for these settings (mainUtils.cpp:10-13)
    else:
        r.ray_trace()
    return r.get_internal(argb=True, rgba=aux, hit=aux, shadow=aux)


@pytest.mark.parametrize("name", CASES)
def test_gpu_matches_reference_golden(R, name):
    c = Case(name)
    exp = c.expected()
    g = gpu_render(R, c.scene, c.settings)
    assert np.array_equal(g["hit_id"], exp["hit_id"]), f"{int((g['hit_id'] != exp['hit_id']).sum())} hit-ID mismatches"
    assert np.array_equal(bits(g["hit_t"]), bits(exp["hit_t"]))
    assert np.array_equal(g["shadow"], exp["shadow"])
    assert np.array_equal(g["argb"], exp["argb"]), f"{int((g['argb'] != exp['argb']).sum())} ARGB mismatches"
    assert float(np.abs(g["rgba"] - exp["rgba"]).max()) <= RGBA_TOL
    st = R.stats()
    assert st["shadow_rays"] == c.meta["counters"]["shadow_rays"]
    assert st["reflection_rays"] == c.meta["counters"]["reflection_rays"]
    if c.settings.enable_ssao:
        z, n, _ = R.get_ssao_buffers(ao=False)
        assert np.array_equal(bits(z), bits(exp["zbuf"]))
        assert np.array_equal(bits(n), bits(exp["nbuf"]))
    R.post_process()
    img = R.get_image().ravel()
    if c.settings.enable_ssao:
        _, _, ao = R.get_ssao_buffers()
        assert np.array_equal(ao, exp["ao"]), f"{int((ao != exp['ao']).sum())} occlusion-count mismatches"
    if c.settings.enable_ssaa:
        assert np.array_equal(img, exp["final"])
    else:
        assert np.array_equal(img, exp["ssao"] if c.settings.enable_ssao else exp["argb"])


@pytest.mark.parametrize("name", [n for n in CASES if manifest()[n]["row_samples"]])
def test_gpu_full_resolution_rows_match_reference(R, name):
    c = Case(name)
    for sc, st, rows in c.row_samples():
        g = gpu_render(R, sc, st)
        rw, _ = st.render_size()
        for row, exp in rows.items():
            sl = slice(row * rw, (row + 1) * rw)
            assert np.array_equal(g["hit_id"][sl], exp["hit_id"]), row
            assert np.array_equal(bits(g["hit_t"][sl]), bits(exp["hit_t"])), row
            assert np.array_equal(g["argb"][sl], exp["argb"]), row
            assert float(np.abs(g["rgba"][sl] - exp["rgba"]).max()) <= RGBA_TOL


def test_c4_full_frame_matches_oracle(R):
    """The benchmark workload at full size: every internal pixel and the SSAA frame."""
    from raytracercpp_amd import scenes
    sc, st = scenes.sphere1m()
    g = gpu_render(R, sc, st)
    o = Oracle(sc, st).render_rows()
    assert np.array_equal(g["hit_id"], o.hit_id)
    assert np.array_equal(bits(g["hit_t"]), bits(o.hit_t))
    assert np.array_equal(g["shadow"], o.shadow)
    assert np.array_equal(g["argb"], o.argb)
    R.post_process()
    rw, rh = st.render_size()
    assert np.array_equal(R.get_image().ravel(), Oracle.downscale(o.argb, rw, rh, 2))
    assert R.stats()["shadow_rays"] == o.counters["shadow_rays"]
    assert R.stats()["seg_scale"] > 0   # the shadow queries ran as segment queries


def _random_rays(rng, n, center, spread):
    o = (center + rng.uniform(-spread, spread, size=(n, 3))).astype(np.float32)
    d = rng.standard_normal((n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return o, d.astype(np.float32)


def _voxel_scene(n=8, size=0.2, gap=0.05):
    """Axis-aligned cubes on a grid: many k-DOP slabs coincide, so pending children tie on
    t_near and the libstdc++ heap order (not a sort) decides the visit order."""
    from raytracercpp_amd import scenes
    base, _ = scenes.sphere256()
    cube = np.array([[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0], [0, 0, 1], [1, 0, 1], [1, 1, 1], [0, 1, 1]], np.float32)
    faces = [(0, 2, 1), (0, 3, 2), (4, 5, 6), (4, 6, 7), (0, 1, 5), (0, 5, 4), (3, 6, 2), (3, 7, 6), (0, 4, 7),
             (0, 7, 3), (1, 2, 6), (1, 6, 5)]
    tris = []
    for i in range(n):
        for j in range(n):
            for k in range(n):
                off = np.array([i, j, k], np.float32) * (size + gap) - n * (size + gap) / 2
                v = cube * size + off
                for f in faces:
                    tris.append(np.concatenate([v[f[0]], v[f[1]], v[f[2]]]))
    base.tri = np.array(tris, np.float32)
    base.tri_mat = np.zeros(len(tris), np.int32)
    base.tri_uv = None
    return base


@pytest.mark.parametrize("scene_name", ["robot", "voxels", "sphere1m_surface", "grazing", "tiny", "huge",
                                        "grazing_plane"])
def test_trace_rays_match_oracle(R, scene_name):
    """BVH::intersect on arbitrary rays (rt_trace_rays) vs the oracle: ids, t, u, v, return value."""
    from raytracercpp_amd import scenes
    from raytracercpp_amd.scene import RenderSettings
    rng = np.random.default_rng(5)
    if scene_name == "robot":
        sc, st = scenes.robot1080(width=64, height=36)
        o, d = _random_rays(rng, 50000, np.array([0, 0, -4], np.float32), 3.0)
    elif scene_name == "voxels":
        sc = _voxel_scene()
        st = RenderSettings(bvh_max_depth=12, bvh_leaf_object_count=8)
        o, d = _random_rays(rng, 50000, np.zeros(3, np.float32), 2.5)
        # axis-aligned directions too (zero denominators are skipped planes)
        d[:10000] = np.eye(3, dtype=np.float32)[rng.integers(0, 3, 10000)] * rng.choice([-1, 1], (10000, 1))
    elif scene_name == "grazing":
        # plane denominators below 2^-40 (incl. denormal and zero): vol_test's exact-division path
        sc, st = scenes.robot1080(width=64, height=36)
        o, d = _random_rays(rng, 50000, np.array([0, 0, -4], np.float32), 3.0)
        tiny = rng.choice(np.array([0.0, 1e-13, -1e-13, 1e-30, -1e-41], np.float32), (50000,))
        axis = rng.integers(0, 3, 50000)
        d[np.arange(50000), axis] = tiny
    elif scene_name == "grazing_plane":
        # rays meeting a rotated tessellated plane at sin 1e-7..1e-3: Moller-Trumbore reports
        # hits outside the triangles' boxes; the octree walk tests what the
        # reference tests and returns its record
        import dataclasses
        from test_wbvh import grazing_plane_case
        tri, o, d = grazing_plane_case()
        sc, st = scenes.robot1080(width=64, height=36)
        sc = dataclasses.replace(sc, tri=tri, tri_mat=np.zeros(len(tri), np.int32), tri_uv=None)
    elif scene_name in ("tiny", "huge"):
        # every slab value outside [2^-38, 2^39): the whole scene takes the exact-division path
        f = np.float32(1e-13 if scene_name == "tiny" else 1e13)
        sc, st = scenes.robot1080(width=64, height=36)
        sc.tri = (sc.tri * f).astype(np.float32)
        o, d = _random_rays(rng, 50000, np.array([0, 0, -4], np.float32) * f, 3.0 * f)
    else:
        sc, st = scenes.sphere1m(width=64, height=36)
        idx = rng.integers(0, sc.ntri, 20000)
        t9 = sc.tri[idx].reshape(-1, 3, 3).astype(np.float64)
        p = t9.mean(axis=1)
        n = np.cross(t9[:, 1] - t9[:, 0], t9[:, 2] - t9[:, 0])
        n /= np.maximum(np.linalg.norm(n, axis=1, keepdims=True), 1e-30)
        o = (p + 1e-4 * n).astype(np.float32)
        d = np.array([3, 3, 2]) - p
        d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    R.load_scene(sc, st)
    gi, gt, gu, gv, gr = R.trace_rays(o, d)
    oi, ot, ou, ov, orr, _ = Oracle(sc, st).bvh_query(o, d)
    assert np.array_equal(gi, oi)
    assert np.array_equal(gr, orr)
    assert np.array_equal(bits(gt), bits(ot))
    assert np.array_equal(bits(gu), bits(ou)) and np.array_equal(bits(gv), bits(ov))


@pytest.mark.parametrize("scene_name", ["bumpy70k", "c5_small"])
def test_bands_reassemble_to_full_frame(R, scene_name):
    """Image strips (multi-GPU layout) rendered on one GPU and re-assembled == the full render
    (also through the reflection engine: pixel seeds use global rows, frames write local rows)."""
    import torch
    from raytracercpp_amd import scenes
    from raytracercpp_amd.strips import assemble
    if scene_name == "bumpy70k":
        sc, st = scenes.bumpy70k(width=320, height=180, enable_ssaa=True, ssaa_factor=2)
    else:
        sc, st = scenes.sphere1m_refl(width=80, height=45, samples=4)
        st = st.copy(max_recursion_depth=2)
    R.load_scene(sc, st)
    R.ray_trace()
    R.post_process()
    full = R.get_image()
    for nranks, band in ((1, 8), (2, 8), (3, 5), (8, 8)):
        parts = []
        for rank in range(nranks):
            n = R.local_rows(band, rank, nranks)
            buf = torch.zeros((n, st.image_width), dtype=torch.int32, device="cuda:0")
            R.render_bands_device(band, rank, nranks, buf.data_ptr(), 0)
            torch.cuda.synchronize()
            parts.append(buf.cpu().numpy().view(np.uint32))
        assert np.array_equal(assemble(parts, st.image_height, band), full), (nranks, band)


@pytest.mark.parametrize("f", [2, 3, 4, 8])
@pytest.mark.parametrize("fused", ["1", "0"])
def test_band_streams_fused_ssaa(make_renderer, f, fused):
    """Band launches in flight on two streams (per-stream tile queues and band buffers), with
    the SSAA box filter fused into the trace kernel's tiles (f = 2, 4, 8; f = 3 and
    RT_FUSED_SSAA=0 take the separate downscale pass): re-assembled == the full render."""
    import torch
    from raytracercpp_amd import scenes
    from raytracercpp_amd.strips import assemble
    R = make_renderer(RT_FUSED_SSAA=fused)
    sc, st = scenes.bumpy70k(width=160, height=96, enable_ssaa=True, ssaa_factor=f)
    R.load_scene(sc, st)
    R.ray_trace()
    R.post_process()
    full = R.get_image()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for nranks, band in ((1, 8), (4, 8), (3, 4)):
        bufs = [torch.zeros((R.local_rows(band, rank, nranks), st.image_width), dtype=torch.int32, device="cuda:0")
                for rank in range(nranks)]
        torch.cuda.synchronize()   # the fills ran on the default stream
        for rank in range(nranks):
            R.render_bands_device(band, rank, nranks, bufs[rank].data_ptr(), streams[rank % 2].cuda_stream)
        torch.cuda.synchronize()
        parts = [b.cpu().numpy().view(np.uint32) for b in bufs]
        assert np.array_equal(assemble(parts, st.image_height, band), full), (nranks, band)


@pytest.mark.parametrize("f", [2, 3])
def test_band_lists_cost_balanced(make_renderer, f):
    """Cost-balanced strips (rt_render_band_list_device + rt_band_costs, strips.assign_bands): each
    "rank" renders the interleaved layout, the band costs of its launches are summed into one vector,
    then every rank renders its balanced list on its own stream, a few frames in flight (heavy lists
    and split tiles learnt per list); the re-assembled frame equals the full render (f = 2 fused SSAA,
    f = 3 the separate pass), the costs cover every band, and bad lists are refused."""
    import torch
    from raytracercpp_amd import scenes
    from raytracercpp_amd._lib import RtError
    from raytracercpp_amd.strips import assemble, assign_bands, num_bands
    R = make_renderer()
    sc, st = scenes.bumpy70k(width=320, height=184, enable_ssaa=True, ssaa_factor=f)
    R.load_scene(sc, st)
    R.ray_trace()
    R.finish_accel()
    R.ray_trace()
    R.post_process()
    full = R.get_image()
    band, nranks = 8, 3
    nb = num_bands(st.image_height, band)
    streams = [torch.cuda.Stream() for _ in range(nranks)]
    costs = np.zeros(nb)
    for rank in range(nranks):
        b = torch.zeros((R.local_rows(band, rank, nranks), st.image_width), dtype=torch.int32, device="cuda:0")
        torch.cuda.synchronize()
        for _ in range(2):
            R.render_bands_device(band, rank, nranks, b.data_ptr(), streams[rank].cuda_stream)
        costs = R.band_costs(nb, streams[rank].cuda_stream, costs)
    assert (costs > 0).all(), costs
    lists = assign_bands(costs, nranks)
    assert sorted(np.concatenate(lists).tolist()) == list(range(nb))
    per = len(lists[0])
    bufs = [torch.zeros((per * band, st.image_width), dtype=torch.int32, device="cuda:0") for _ in range(nranks)]
    torch.cuda.synchronize()
    for rep in range(3):
        for rank in range(nranks):
            R.render_band_list_device(band, lists[rank], bufs[rank].data_ptr(), streams[rank].cuda_stream)
        torch.cuda.synchronize()
        parts = [x.cpu().numpy().view(np.uint32) for x in bufs]
        assert np.array_equal(assemble(parts, st.image_height, band, lists), full), rep
    # the list launches' own costs cover exactly their bands
    c2 = np.zeros(nb)
    for rank in range(nranks):
        c2 = R.band_costs(nb, streams[rank].cuda_stream, c2)
    assert (c2 > 0).all()
    for bad in ([0, 0], [nb], [-1]):
        with pytest.raises(RtError):
            R.render_band_list_device(band, bad, bufs[0].data_ptr(), streams[0].cuda_stream)


def test_render_api_and_errors(R):
    from raytracercpp_amd import scenes
    from raytracercpp_amd._lib import RtError
    from raytracercpp_amd.renderer import render
    sc, st = scenes.cube1080(width=64, height=40, enable_ssaa=True, ssaa_factor=2)
    R.load_scene(sc, st)
    ms = render(R)
    assert ms >= 0
    assert R.get_image().shape == (40, 64)
    R.ray_trace()   # without post_process the image stays at render size (renderer.cpp:1079-1080)
    assert R.get_image().shape == (80, 128)
    bad = sc.tri_mat.copy()
    bad[0] = 7
    R.set_triangles(sc.tri, bad, sc.tri_uv)
    with pytest.raises(RtError):
        R.ray_trace()
    R.set_triangles(sc.tri, sc.tri_mat, sc.tri_uv)
    st2 = st.copy(enable_normal_mapping=True)
    R.set_render_settings(st2)
    with pytest.raises(RtError):
        R.ray_trace()   # normal map enabled but not set
    R.set_render_settings(st)
    R.ray_trace()
    nonfinite = sc.tri.copy()
    nonfinite[3, 4] = np.nan
    R.set_triangles(nonfinite, sc.tri_mat, sc.tri_uv)
    with pytest.raises(RtError, match="non-finite"):
        R.ray_trace()   # NaN / inf vertices are rejected (slab test)
    R.set_triangles(sc.tri, sc.tri_mat, sc.tri_uv)
    R.ray_trace()


def test_object_and_camera_transforms_match_oracle(R):
    """Renderer::set_object_transform / set_camera_transform (renderer.cpp:214-233) then render."""
    from raytracercpp_amd import _lib, scenes
    sc, st = scenes.robot1080(width=96, height=54)
    R.load_scene(sc, st)
    m1 = _lib.compose(_lib.make_transform("translation", 0.2, -1.0, 0.5), _lib.make_transform("rz", 15))
    m2 = _lib.make_transform("ry", -20)
    R.set_object_transform(m1)
    R.set_object_transform(m2)   # second call undoes m1 through previous^-1
    cam = _lib.compose(_lib.make_transform("translation", 0.0, 1.0, 1.5), _lib.make_transform("rx", -10))
    R.set_camera_transform(cam)
    R.request_aux(hit=True)
    R.ray_trace()
    g = R.get_internal(argb=True, hit=True)
    # expected: host transforms replayed on the triangle soup, same camera
    t = _lib.compose(m2, _lib.inverse(m1))
    tri = _lib.transform_points(t, _lib.transform_points(m1, sc.tri.reshape(-1, 3))).reshape(-1, 9)
    sc2 = scenes.SceneData(**{**vars(sc), "tri": tri}) if hasattr(scenes, "SceneData") else None
    from raytracercpp_amd.scene import SceneData
    sc2 = SceneData(**{**vars(sc), "tri": tri})
    pos, pinv, c2w = R.get_camera_matrices()
    sc2.cam_pos, sc2.proj_inv, sc2.cam_to_world = pos, pinv, c2w
    o = Oracle(sc2, st).render_rows()
    assert np.array_equal(g["hit_id"], o.hit_id)
    assert np.array_equal(g["argb"], o.argb)


def test_reflection_engine_matches_oracle_c5_small(make_renderer):
    """C5 features (1M tris, rough reflections, normal + parallax maps) at a reduced size: the
    frame-level reflection engine (default) and the recursive kernel (RT_REFL_ENGINE=0)
    against the oracle, bit for bit, with the same shadow / reflection ray counts."""
    from raytracercpp_amd import scenes
    sc, st = scenes.sphere1m_refl(width=64, height=36, samples=4)
    st = st.copy(max_recursion_depth=3)
    o = Oracle(sc, st).render_rows()
    # (engine, fused passes, chunk log2): the default engine, its separate list / spawn passes,
    # many small chunks per level (depth-first over chunks), and the recursive kernel
    for engine, fuse, clog in (("1", "1", "24"), ("1", "0", "24"), ("1", "1", "10"), ("0", "1", "24")):
        R = make_renderer(RT_REFL_ENGINE=engine, RT_REFL_FUSE=fuse, RT_REFL_CHUNK_LOG2=clog)
        engine = f"engine {engine} fuse {fuse} chunk 2^{clog}"
        g = gpu_render(R, sc, st)
        assert np.array_equal(g["hit_id"], o.hit_id), engine
        assert np.array_equal(bits(g["hit_t"]), bits(o.hit_t)), engine
        assert np.array_equal(g["shadow"], o.shadow), engine
        assert np.array_equal(g["argb"], o.argb), f"{engine}: {int((g['argb'] != o.argb).sum())} ARGB mismatches"
        assert float(np.abs(g["rgba"] - o.rgba).max()) <= RGBA_TOL
        stt = R.stats()
        assert stt["shadow_rays"] == o.counters["shadow_rays"], engine
        assert stt["reflection_rays"] == o.counters["reflection_rays"], engine


# C5 at its own configuration: 1920x1080, SSAA 2, 16 rough samples, depth 5,
# normal + parallax maps.  Output rows whose internal row pairs are checked (scenes.c5_check_rows,
# the same rows as bench.py's C5 check): the r03 rows plus 12 seeded ones in the top silhouette,
# pole and bottom silhouette bands (internal rows ~337 .. 1823).
from raytracercpp_amd.scenes import C5_CHECK_ROWS as C5_OUTPUT_ROWS  # noqa: E402


def test_c5_full_config_matches_oracle(R):
    """The whole C5 frame on the GPU (frame engine, 2^27-slot chunks, multi-level Morton sorts,
    ~2.2G reflection rays) against the oracle on 32 internal rows (16 output rows): hit ID, hit t bits, shadow
    flags and ARGB exact, float RGBA within 1e-4, the SSAA output rows exact, and the shadow /
    reflection ray counts of each row pair (a one-output-row band launch, rt_band_counters)."""
    import torch
    from raytracercpp_amd import scenes
    sc, st = scenes.sphere1m_refl()
    assert (st.image_width, st.image_height, st.ssaa_factor, st.rough_reflections_sample_count,
            st.max_recursion_depth) == (1920, 1080, 2, 16, 5)
    assert st.enable_normal_mapping and st.enable_displacement_mapping
    rows = [2 * r + k for r in C5_OUTPUT_ROWS for k in (0, 1)]
    orc = Oracle(sc, st)
    pairs = [orc.render_row_set([2 * r, 2 * r + 1]) for r in C5_OUTPUT_ROWS]

    class _Rows:   # the pairs' outputs in row order
        pass
    o = _Rows()
    for k in ("hit_id", "hit_t", "shadow", "argb", "rgba"):
        setattr(o, k, np.concatenate([getattr(p, k) for p in pairs]))
    g = gpu_render(R, sc, st)
    rw, rh = st.render_size()
    assert R.stats()["reflection_rays"] > 2_000_000_000   # the whole frame ran
    for i, row in enumerate(rows):
        sl, ol = slice(row * rw, (row + 1) * rw), slice(i * rw, (i + 1) * rw)
        assert np.array_equal(g["hit_id"][sl], o.hit_id[ol]), row
        assert np.array_equal(bits(g["hit_t"][sl]), bits(o.hit_t[ol])), row
        assert np.array_equal(g["shadow"][sl], o.shadow[ol]), row
        assert np.array_equal(g["argb"][sl], o.argb[ol]), f"row {row}: {int((g['argb'][sl] != o.argb[ol]).sum())} ARGB mismatches"
        assert float(np.abs(g["rgba"][sl] - o.rgba[ol]).max()) <= RGBA_TOL, row
    assert int(o.shadow.sum()) > 0 and len(set(o.hit_id.tolist())) > 100
    R.post_process()
    img = R.get_image()
    ds = Oracle.downscale(o.argb, rw, len(rows), 2).reshape(len(C5_OUTPUT_ROWS), st.image_width)
    for i, r in enumerate(C5_OUTPUT_ROWS):
        assert np.array_equal(img[r], ds[i]), r
    # per row pair: one output row as a band (band_rows 1, rank r of image_height ranks)
    H = st.image_height
    for i, r in enumerate(C5_OUTPUT_ROWS):
        buf = torch.zeros((R.local_rows(1, r, H), st.image_width), dtype=torch.int32, device="cuda:0")
        torch.cuda.synchronize()
        R.render_bands_device(1, r, H, buf.data_ptr(), 0)
        torch.cuda.synchronize()
        shadow, refl = R.band_counters()
        assert (shadow, refl) == (pairs[i].counters["shadow_rays"], pairs[i].counters["reflection_rays"]), r
        assert np.array_equal(buf.cpu().numpy().view(np.uint32)[0], ds[i]), r


def _check_vs_oracle(g, o, label, counters=True, R=None):
    assert np.array_equal(g["hit_id"], o.hit_id), f"{label}: {int((g['hit_id'] != o.hit_id).sum())} hit-ID mismatches"
    assert np.array_equal(bits(g["hit_t"]), bits(o.hit_t)), label
    assert np.array_equal(g["shadow"], o.shadow), label
    assert np.array_equal(g["argb"], o.argb), f"{label}: {int((g['argb'] != o.argb).sum())} ARGB mismatches"
    assert float(np.abs(g["rgba"] - o.rgba).max()) <= RGBA_TOL, label
    if counters:
        stt = R.stats()
        assert stt["shadow_rays"] == o.counters["shadow_rays"], label
        assert stt["reflection_rays"] == o.counters["reflection_rays"], label


@pytest.mark.parametrize("scene_name", ["bumpy70k", "robot_clip", "robot_noclip", "c5_small", "sphere1m"])
def test_raster_trace_matches_oracle(R, scene_name):
    """raster_trace (renderer.cpp:869-1006) against the oracle's sequential raster: the
    z-buffer winner (first of equal z), its depth, and trace_triangle's shading, including
    big pieces (workgroup rasterised), frustum clipping, and reflective hits through the
    frame engine."""
    from raytracercpp_amd import scenes
    if scene_name == "bumpy70k":
        sc, st = scenes.bumpy70k(width=320, height=180)
    elif scene_name in ("robot_clip", "robot_noclip"):
        from raytracercpp_amd import _lib
        sc, st = scenes.robot1080(width=200, height=120)
        st = st.copy(enable_clipping=scene_name == "robot_clip")
        # camera inside the scene: many triangles cross the near plane / the frustum sides
        R.load_scene(sc, st)
        R.set_camera_transform(_lib.compose(_lib.make_transform("translation", 0.3, 0.2, 1.2),
                                            _lib.make_transform("ry", 25)))
        pos, pinv, c2w = R.get_camera_matrices()
        from raytracercpp_amd.scene import SceneData
        sc = SceneData(**{**vars(sc), "cam_pos": pos, "proj_inv": pinv, "cam_to_world": c2w,
                          "world_to_cam": _lib.inverse(c2w)})
    elif scene_name == "c5_small":
        sc, st = scenes.sphere1m_refl(width=64, height=36, samples=4)
        st = st.copy(max_recursion_depth=2)
    else:
        sc, st = scenes.sphere1m(width=160, height=90)
    st = st.copy(hybrid_rasterization_tracing=True)
    o = Oracle(sc, st).raster()
    g = gpu_render(R, sc, st)
    _check_vs_oracle(g, o, scene_name, R=R)


def test_raster_bands_reassemble_to_full_frame(R):
    """raster_trace through render_bands_device (each rank keeps its own bands' z-keys)."""
    import torch
    from raytracercpp_amd import scenes
    from raytracercpp_amd.renderer import render
    from raytracercpp_amd.strips import assemble
    sc, st = scenes.sphere1m_refl(width=80, height=45, samples=2)
    st = st.copy(max_recursion_depth=2, hybrid_rasterization_tracing=True)
    R.load_scene(sc, st)
    render(R)
    full = R.get_image()
    for nranks, band in ((1, 8), (2, 8), (3, 5)):
        parts = []
        for rank in range(nranks):
            n = R.local_rows(band, rank, nranks)
            buf = torch.zeros((n, st.image_width), dtype=torch.int32, device="cuda:0")
            R.render_bands_device(band, rank, nranks, buf.data_ptr(), 0)
            torch.cuda.synchronize()
            parts.append(buf.cpu().numpy().view(np.uint32))
        assert np.array_equal(assemble(parts, st.image_height, band), full), (nranks, band)


def test_raster_errors_and_dispatch(R):
    """render() picks raster_trace by the settings; reflections without the BVH are refused."""
    from raytracercpp_amd import scenes
    from raytracercpp_amd._lib import RtError
    from raytracercpp_amd.renderer import render
    sc, st = scenes.cube1080(width=64, height=40)
    st = st.copy(hybrid_rasterization_tracing=True)
    R.load_scene(sc, st)
    R.request_aux(hit=True)
    render(R)
    g = R.get_internal(argb=True, hit=True)
    o = Oracle(sc, st).raster()
    assert np.array_equal(g["argb"], o.argb) and np.array_equal(g["hit_id"], o.hit_id)
    R.ray_trace()   # ray_trace stays ray_trace whatever the settings say
    g2 = R.get_internal(argb=True, hit=True)
    assert np.array_equal(g2["argb"], Oracle(sc, st).render_rows().argb)
    sc, st = scenes.sphere1m_refl(width=32, height=18, samples=2)
    st = st.copy(hybrid_rasterization_tracing=True, enable_bvh=False)
    R.load_scene(sc, st)
    with pytest.raises(RtError):
        R.raster_trace()


@pytest.mark.parametrize("raster,w,h,kw", [
    (False, 331, 187, dict(ssao_sample_count=32, ssao_radius=0.4)),
    (False, 160, 90, dict(ssao_sample_count=16, ssao_radius=0.7, enable_ssaa=True, ssaa_factor=2,
                          enable_normal_mapping=True)),
    (True, 245, 131, dict(ssao_sample_count=24, ssao_radius=0.5, ssao_amount=0.8)),
])
def test_ssao_matches_oracle(R, raster, w, h, kw):
    """post_process_ssao_SIMD on the GPU (occlusion kernel + LDS blur) against the oracle,
    bit-exact: z / normal buffers, per-pixel counts, the internal and the final image."""
    from raytracercpp_amd import scenes
    if kw.get("enable_normal_mapping"):
        # C5 features: normal-mapped buffers, reflective hits through the frame engine's level 0
        sc, st = scenes.sphere1m_refl(width=w, height=h, samples=2)
        st = st.copy(enable_ssao=True, max_recursion_depth=3, **kw)
    else:
        sc, st = scenes.bumpy70k(width=w, height=h, enable_ssao=True, hybrid_rasterization_tracing=raster, **kw)
    o = Oracle(sc, st)
    ref = o.raster() if raster else o.render_rows()
    ref_img, ref_ao = o.ssao(ref)
    g = gpu_render(R, sc, st, aux=False)
    assert np.array_equal(g["argb"], ref.argb)
    z, n, _ = R.get_ssao_buffers(ao=False)
    assert np.array_equal(bits(z), bits(ref.zbuf))
    assert np.array_equal(bits(n), bits(ref.nbuf))
    R.post_process()
    _, _, ao = R.get_ssao_buffers()
    assert ref_ao.max() > 0
    assert np.array_equal(ao, ref_ao), f"{int((ao != ref_ao).sum())} occlusion-count mismatches"
    img = R.get_image().ravel()
    if st.enable_ssaa:
        rw, rh = st.render_size()
        ref_img = Oracle.downscale(ref_img, rw, rh, st.ssaa_factor)
    assert np.array_equal(img, ref_img)


def test_ssao_errors(R):
    """SSAO needs the whole frame: band rendering refuses it; post_process refuses stale buffers."""
    import torch
    from raytracercpp_amd import scenes
    from raytracercpp_amd._lib import RtError
    sc, st = scenes.bumpy70k(width=64, height=40)
    R.load_scene(sc, st)
    R.ray_trace()
    R.set_render_settings(st.copy(enable_ssao=True))
    with pytest.raises(RtError):
        R.post_process()   # the frame was traced without z / normal buffers
    out = torch.empty((R.local_rows(8, 0, 1), 64), dtype=torch.int32, device="cuda")
    with pytest.raises(RtError):
        R.render_bands_device(8, 0, 1, out.data_ptr())


@pytest.mark.parametrize("name", ["c2_cube", "robot", "c3_bumpy70k", "mirror", "rough", "textured", "raster_rough"])
def test_whole_line_queries_match_reference_golden(make_renderer, name):
    """RT_SEG=0 RT_CONES=0: every query walks the whole line and tests every triangle of
    every leaf it enters, as the reference does (no segment culling, DESIGN.md 5.2, no leaf
    normal cones, 5.3); the framebuffer is the same."""
    if name not in CASES:
        pytest.skip(f"no golden case {name}")
    c = Case(name)
    exp = c.expected()
    R = make_renderer(RT_SEG=0, RT_CONES=0)
    g = gpu_render(R, c.scene, c.settings)
    assert R.stats()["seg_scale"] == 0
    assert np.array_equal(g["hit_id"], exp["hit_id"])
    assert np.array_equal(bits(g["hit_t"]), bits(exp["hit_t"]))
    assert np.array_equal(g["shadow"], exp["shadow"])
    assert np.array_equal(g["argb"], exp["argb"])
    assert float(np.abs(g["rgba"] - exp["rgba"]).max()) <= RGBA_TOL


def _soup_scene(rng, n=4000):
    """Random triangles in front of the camera -- a third of them slivers (nearly collinear
    vertices), some degenerate (a repeated vertex) -- over a tessellated ground plane y = -1.5."""
    from raytracercpp_amd import scenes
    from raytracercpp_amd.scene import SceneData, empty_shapes
    base, st = scenes.bumpy70k(width=8, height=8)
    c = rng.uniform([-2.0, -1.4, -7.0], [2.0, 1.5, -2.5], (n, 3))
    e1 = rng.normal(size=(n, 3)) * 0.25
    e2 = rng.normal(size=(n, 3)) * 0.25
    sl = rng.random(n) < 0.33
    e2[sl] = e1[sl] * rng.uniform(0.5, 2.0, (int(sl.sum()), 1)) + rng.normal(size=(int(sl.sum()), 3)) * 1e-6
    dg = rng.random(n) < 0.05
    e2[dg] = e1[dg]
    soup = np.concatenate([c, c + e1, c + e2], axis=1)
    g = np.linspace(-6.0, 6.0, 25)
    ground = []
    for i in range(24):
        for k in range(24):
            a, b = (g[i], -1.5, g[k] - 6), (g[i + 1], -1.5, g[k] - 6)
            cc, d = (g[i + 1], -1.5, g[k + 1] - 6), (g[i], -1.5, g[k + 1] - 6)
            ground += [a + d + cc, a + cc + b]   # facing +y
    tri = np.concatenate([soup, np.array(ground)], axis=0).astype(np.float32)
    sc = SceneData(**{**vars(base), "tri": tri, "tri_mat": np.zeros(len(tri), np.int32), "tri_uv": None})
    sc.shape_kind, sc.shape, sc.shape_mat = empty_shapes()
    return sc, st


@pytest.mark.parametrize("scene_name,light", [
    ("soup", (3.0, 3.0, 2.0)), ("soup", (0.0, 0.0, -4.5)), ("soup", (60.0, -1.4999, -4.0)),
    ("soup", (30.0, -1.5, -4.0)), ("voxels", (3.0, 3.0, 2.0)), ("voxels", (0.01, 0.02, 0.03)),
    ("voxels", (0.3, 0.0, 0.0)),
])
def test_segment_queries_match_oracle(R, scene_name, light):
    """Segment-culled shadow queries against the oracle's whole-line traversal
    on scenes built to stress the culling margins: slivers and degenerate triangles, lights
    inside the geometry, a light grazing (and one exactly in) a tessellated ground plane,
    axis-aligned voxels whose k-DOP slabs coincide."""
    from raytracercpp_amd.scene import empty_shapes
    rng = np.random.default_rng(11)
    if scene_name == "soup":
        sc, st = _soup_scene(rng)
        st = st.copy(image_width=240, image_height=160)
    else:
        sc = _voxel_scene(n=6)
        sc.shape_kind, sc.shape, sc.shape_mat = empty_shapes()
        from raytracercpp_amd import scenes
        _, st = scenes.bumpy70k(width=240, height=160)
        st = st.copy(bvh_leaf_object_count=8)
    sc.light = np.asarray(light, np.float32)
    o = Oracle(sc, st).render_rows()
    g = gpu_render(R, sc, st)
    assert R.stats()["seg_scale"] > 0
    assert int(o.shadow.sum()) > 0
    _check_vs_oracle(g, o, f"{scene_name} {light}", R=R)


FRAME_MODES = {
    "generic": {"RT_PLAIN": "0"},   # the kernel without the plain specialisation
    "octree": {"RT_WBVH": "0"},     # no wide BVH: every query walks the octree
    "exact": {"RT_EXACT": "1"},     # exact mode: the octree over the whole line
}


@pytest.mark.parametrize("mode", sorted(FRAME_MODES))
@pytest.mark.parametrize("scene_name", ["soup", "voxels", "bumpy_ssaa"])
def test_frame_modes_match_oracle(make_renderer, mode, scene_name):
    """The frame's equivalent paths on the segment-query stress scenes and an SSAA frame:
    the same framebuffers as the oracle."""
    from raytracercpp_amd import scenes
    from raytracercpp_amd.scene import empty_shapes
    R = make_renderer(**FRAME_MODES[mode])
    rng = np.random.default_rng(5)
    if scene_name == "soup":
        sc, st = _soup_scene(rng)
        st = st.copy(image_width=200, image_height=120)
        sc.light = np.asarray((60.0, -1.4999, -4.0), np.float32)
    elif scene_name == "voxels":
        sc = _voxel_scene(n=6)
        sc.shape_kind, sc.shape, sc.shape_mat = empty_shapes()
        _, st = scenes.bumpy70k(width=200, height=120)
        st = st.copy(bvh_leaf_object_count=8)
        sc.light = np.asarray((0.3, 0.0, 0.0), np.float32)
    else:
        sc, st = scenes.bumpy70k(width=160, height=90, enable_ssaa=True, ssaa_factor=2)
    o = Oracle(sc, st).render_rows()
    g = gpu_render(R, sc, st)
    _check_vs_oracle(g, o, f"{scene_name} {mode}", R=R)


@pytest.mark.parametrize("case", ["huge", "ssao", "bands", "golden"])
def test_octree_path_matches_oracle(make_renderer, case):
    """The exact octree traversal on its own (RT_WBVH=0; the wide BVH's fallback)
    on the paths the stress scenes above do not reach: a scene scaled by 1e13 whose
    Moller-Trumbore products overflow (NaN hits), the SSAO z / normal writes, band rendering
    re-assembled into the full frame, and every ray-traced golden case."""
    import torch
    from raytracercpp_amd import scenes
    from raytracercpp_amd.strips import assemble
    R = make_renderer(RT_WBVH=0)
    if case == "golden":
        ran = 0
        for name in CASES:
            c = Case(name)
            st = c.settings
            if st.hybrid_rasterization_tracing:
                continue
            exp = c.expected()
            g = gpu_render(R, c.scene, st)
            assert np.array_equal(g["hit_id"], exp["hit_id"]), name
            assert np.array_equal(bits(g["hit_t"]), bits(exp["hit_t"])), name
            assert np.array_equal(g["shadow"], exp["shadow"]), name
            assert np.array_equal(g["argb"], exp["argb"]), name
            assert R.stats()["shadow_rays"] == c.meta["counters"]["shadow_rays"], name
            ran += 1
        assert ran > 0
        return
    if case == "huge":
        f = np.float32(1e13)
        sc, st = scenes.robot1080(width=96, height=54)
        sc.tri = (sc.tri * f).astype(np.float32)
        sc.light = (np.asarray(sc.light, np.float32) * f).astype(np.float32)
    elif case == "ssao":
        sc, st = scenes.bumpy70k(width=131, height=77, enable_ssao=True, ssao_sample_count=16, ssao_radius=0.5)
    else:
        sc, st = scenes.bumpy70k(width=160, height=90, enable_ssaa=True, ssaa_factor=2)
    if case == "bands":
        R.load_scene(sc, st)
        R.ray_trace()
        R.post_process()
        full = R.get_image()
        o = Oracle(sc, st).render_rows()
        rw, rh = st.render_size()
        assert np.array_equal(full.ravel(), Oracle.downscale(o.argb, rw, rh, 2))
        for nranks, band in ((2, 8), (3, 5)):
            parts = []
            for rank in range(nranks):
                n = R.local_rows(band, rank, nranks)
                buf = torch.zeros((n, st.image_width), dtype=torch.int32, device="cuda:0")
                R.render_bands_device(band, rank, nranks, buf.data_ptr(), 0)
                torch.cuda.synchronize()
                parts.append(buf.cpu().numpy().view(np.uint32))
            assert np.array_equal(assemble(parts, st.image_height, band), full), (nranks, band)
        return
    o = Oracle(sc, st)
    ref = o.render_rows()
    g = gpu_render(R, sc, st, aux=case != "ssao")
    if case == "ssao":
        assert np.array_equal(g["argb"], ref.argb)
        z, n, _ = R.get_ssao_buffers(ao=False)
        assert np.array_equal(bits(z), bits(ref.zbuf))
        assert np.array_equal(bits(n), bits(ref.nbuf))
        ref_img, ref_ao = o.ssao(ref)
        R.post_process()
        _, _, ao = R.get_ssao_buffers()
        assert np.array_equal(ao, ref_ao)
        assert np.array_equal(R.get_image().ravel(), ref_img)
        return
    _check_vs_oracle(g, ref, case, R=R)


def test_band_slots_recycle_and_shared_buffers(R):
    """Frames in flight across more streams than the renderer has band slots (8): the least
    recently used slot is recycled once its own last launch is done, even when its stream was
    destroyed; a reflection-engine band launch (buffers shared across launches) after launches
    on other streams waits for them.  Every re-assembled frame equals the full render."""
    import ctypes
    import torch
    from raytracercpp_amd import scenes
    from raytracercpp_amd.strips import assemble
    sc, st = scenes.bumpy70k(width=160, height=96, enable_ssaa=True, ssaa_factor=2)
    R.load_scene(sc, st)
    R.ray_trace()
    R.post_process()
    full = R.get_image()
    band, nranks = 8, 3
    hip = ctypes.CDLL("libamdhip64.so")
    for rep_ in range(2):
        # raw HIP streams, destroyed after each round: the slots keep stale handles
        streams = []
        for _ in range(11):
            h = ctypes.c_void_p()
            assert hip.hipStreamCreate(ctypes.byref(h)) == 0
            streams.append(h)
        bufs = []
        for i, s in enumerate(streams):
            rank = i % nranks
            b = torch.zeros((R.local_rows(band, rank, nranks), st.image_width), dtype=torch.int32, device="cuda:0")
            torch.cuda.synchronize()
            R.render_bands_device(band, rank, nranks, b.data_ptr(), s.value)
            bufs.append(b)
        for s in streams:
            assert hip.hipStreamSynchronize(s) == 0
        for k in range(0, 9, nranks):
            parts = [bufs[k + r].cpu().numpy().view(np.uint32) for r in range(nranks)]
            assert np.array_equal(assemble(parts, st.image_height, band), full), (rep_, k)
        for s in streams:
            assert hip.hipStreamDestroy(s) == 0
    sc2, st2 = scenes.sphere1m_refl(width=80, height=45, samples=2)
    st2 = st2.copy(max_recursion_depth=2)
    R.load_scene(sc2, st2)
    R.ray_trace()
    R.post_process()
    full2 = R.get_image()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    parts = []
    for rank, s in ((0, s1), (1, s2)):
        b = torch.zeros((R.local_rows(band, rank, 2), st2.image_width), dtype=torch.int32, device="cuda:0")
        torch.cuda.synchronize()
        R.render_bands_device(band, rank, 2, b.data_ptr(), s.cuda_stream)
        parts.append(b)
    torch.cuda.synchronize()
    assert np.array_equal(assemble([p.cpu().numpy().view(np.uint32) for p in parts], st2.image_height, band), full2)


def test_rccl_frame_pipeline_world1():
    """bench.py's N>1 path on one GPU: an RCCL process group (world size 1, torchrun) on a
    high-priority stream, three frames in flight (the bench's default) with asynchronous all-gathers
    (strips.FramePipeline, gather forced on): every gathered frame equals the rendered strips
    (tools/nccl_check.py).  Runs in its own process: the rendezvous and RCCL state stay out of
    this one."""
    import os
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "1",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), "tools/nccl_check.py"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0 and "nccl pipeline ok" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])


def _telephoto_plane_scene(h0=1e-3, roll=0.2, yaw=17.0, fov=0.5, size=20.0, n=400, width=320, height=180):
    """A 40 x 40 plane of 320,000 triangles, h0 below a telephoto camera (fov 0.5 degrees): the
    lower part of the frame meets it at grazing angles between 5e-5 and 5e-3."""
    import dataclasses
    from raytracercpp_amd import scenes
    from test_wbvh import _grid

    def rot(ax, deg):
        a = np.deg2rad(deg)
        c, s_ = np.cos(a), np.sin(a)
        return np.array([[c, -s_, 0], [s_, c, 0], [0, 0, 1]]) if ax == "z" else np.array([[c, 0, s_], [0, 1, 0], [-s_, 0, c]])
    sc, st = scenes.robot1080(width=width, height=height)
    T = scenes.default_transforms()
    rw, rh = st.render_size()
    proj, pinv = T.camera_matrices(fov, np.float32(rw) / np.float32(rh))
    Rm = rot("z", roll) @ rot("y", yaw)
    g = _grid(n, size).reshape(-1, 3, 3) + np.array([0, 0, -size - 0.5])
    tri = (g @ Rm.T + np.array([0, -h0, 0])).reshape(-1, 9).astype(np.float32)
    sc = dataclasses.replace(sc, tri=tri, tri_mat=np.zeros(len(tri), np.int32), tri_uv=None, proj_inv=pinv, proj=proj,
                             cam_fov=fov)
    return sc, st


@pytest.mark.parametrize("mode", ["exact", "default"])
def test_grazing_plane_frame_matches_oracle(make_renderer, mode):
    """A frame whose rays graze a tessellated plane: exact mode (rt_set_exact)
    walks the octree as the reference does; the default certificate is exact here too (the
    adversarial rays of tests/test_wbvh.py are steeper than a frame's pixels reach)."""
    R = make_renderer()
    R.set_exact(mode == "exact")
    sc, st = _telephoto_plane_scene()
    o = Oracle(sc, st).render_rows()
    g = gpu_render(R, sc, st)
    assert int((o.hit_id >= 0).sum()) > 10000
    _check_vs_oracle(g, o, f"grazing plane {mode}", R=R)


@pytest.mark.parametrize("n", [1, 2, 3])
def test_set_devices_bands_match_one_device(make_renderer, n):
    """rt_set_devices with the device repeated n times (n renderers on one device; the band
    copy replaces the RCCL send): every frame equals the one-device frame and the oracle, also
    after light, material and geometry changes that the helpers must mirror."""
    from raytracercpp_amd import scenes
    from raytracercpp_amd.renderer import render
    R = make_renderer()
    sc, st = scenes.bumpy70k(width=200, height=117, enable_ssaa=True, ssaa_factor=2)
    R.load_scene(sc, st)
    R.set_devices([0] * n)
    rw, rh = st.render_size()
    for step in range(4):
        if step == 1:
            R.set_light_position((1.0, 4.0, 3.0))
            sc.light = np.asarray((1.0, 4.0, 3.0), np.float32)
        if step == 2:
            sc.tri = (sc.tri * np.float32(0.9)).astype(np.float32)
            sc.materials = sc.materials.copy()
            sc.materials[0, 0] = 0.2
            R.set_materials(sc.materials)
            R.set_triangles(sc.tri, sc.tri_mat, sc.tri_uv)
        if step == 3:
            R.finish_accel()   # the helpers then copy the lead's cones / slabs and wide BVH
        render(R)
        multi = R.get_image().ravel().copy()
        o = Oracle(sc, st).render_rows()
        assert np.array_equal(multi, Oracle.downscale(o.argb, rw, rh, 2)), f"step {step}"
        # one host octree build per geometry change for all n devices (the helpers copy the
        # lead's device tables; reference renderer.cpp:214-224 rebuilds once)
        assert R.stats()["host_builds"] == (1 if step < 2 else 2), (step, R.stats()["host_builds"])
    R.set_devices([])
    render(R)
    assert np.array_equal(R.get_image().ravel(), multi)


@pytest.mark.gpu
def test_set_devices_first_frame_after_geometry_change(make_renderer):
    """rt_set_devices with 3 renderers: the frame right after set_triangles costs about the
    one-device first frame (one build; the helpers copy the lead's tables), not three builds."""
    import time
    from raytracercpp_amd import scenes
    from raytracercpp_amd.renderer import render
    sc, st = scenes.sphere1m(width=320, height=180)
    times = {}
    for n in (1, 3):
        R = make_renderer()
        R.load_scene(sc, st)
        if n > 1:
            R.set_devices([0] * n)
        render(R)
        R.finish_accel()
        render(R)
        tri = (sc.tri * np.float32(1.01)).astype(np.float32)
        R.set_triangles(tri, sc.tri_mat, sc.tri_uv)
        t0 = time.perf_counter()
        render(R)
        times[n] = time.perf_counter() - t0
        assert R.stats()["host_builds"] == 2
    print("first frame after a geometry change:", times)
    assert times[3] < 1.6 * times[1] + 0.02, times


def test_async_accel_frames(make_renderer):
    """The product default: the first frame after a geometry change runs on the
    quick wide BVH (the octree's own hierarchy) while the leaf cones / slabs and the SAH tree are still
    building, later frames on them; every frame equals the oracle, also when the geometry changes again
    mid-build."""
    from raytracercpp_amd import scenes
    R = make_renderer(RT_ASYNC_ACCEL="1")
    sc, st = scenes.sphere1m(width=160, height=90)
    o = Oracle(sc, st).render_rows()
    for step in range(4):
        if step == 2:   # a new geometry while the previous build may still run
            sc.tri = (sc.tri * np.float32(1.01)).astype(np.float32)
            R.set_triangles(sc.tri, sc.tri_mat, sc.tri_uv)
            o = Oracle(sc, st).render_rows()
        g = gpu_render(R, sc, st) if step == 0 else None
        if g is None:
            R.request_aux(rgba=True, hit=True, shadow=True)
            R.ray_trace()
            g = R.get_internal(argb=True, rgba=True, hit=True, shadow=True)
        _check_vs_oracle(g, o, f"async step {step}", R=R)
        if step == 0:
            assert R.stats()["build_split_ms"][2] == 0.0   # the SAH tree was not adopted yet
        if step == 1:
            R.finish_accel()
    R.finish_accel()
    assert R.stats()["build_split_ms"][2] > 0.0


@pytest.mark.parametrize("cam", ["constant_w", "projective_proj", "projective_c2w", "w_one"])
def test_camera_matrix_forms_match_oracle(R, cam):
    """Ray generation (renderer.cpp:1086-1098) for every form of the caller's camera matrices: the
    kernel skips Transform::operator()(Point)'s division when w is the same for every pixel
    (KParams::proj_mode, c2w_affine); projective rows take the per-pixel path.  Bit-exact vs the
    oracle's per-pixel evaluation."""
    import dataclasses
    from raytracercpp_amd import scenes
    sc, st = scenes.bumpy70k(width=96, height=64)
    pinv = np.asarray(sc.proj_inv, np.float32).copy()
    c2w = np.asarray(sc.cam_to_world, np.float32).copy()
    if cam == "projective_proj":
        pinv[12], pinv[13] = np.float32(0.0123), np.float32(-0.0071)   # w varies with the pixel
    elif cam == "projective_c2w":
        c2w[12:16] = np.float32([0.002, -0.001, 0.003, 1.0])
    elif cam == "w_one":
        # (-m14) + m15 == 1: w == 1 for every pixel, the point is not scaled (proj_mode 1)
        pinv[15] = np.float32(1.0) + pinv[14]
        assert np.float32(-pinv[14]) + pinv[15] == np.float32(1.0)
    sc = dataclasses.replace(sc, proj_inv=pinv, cam_to_world=c2w)
    o = Oracle(sc, st).render_rows()
    g = gpu_render(R, sc, st)
    assert int((o.hit_id >= 0).sum()) > 500, cam
    _check_vs_oracle(g, o, cam, R=R)


def test_band_counters_across_repeated_launches(R):
    """Band launches of the default trace path each clear their stream slot's counters
    (render_bands_device's hipMemsetAsync on the slot's stream before the launch): repeated
    launches on one stream and on alternating streams each report the frame's shadow-ray count
    and produce the same strips."""
    import torch
    from raytracercpp_amd import scenes
    sc, st = scenes.bumpy70k(width=160, height=96, enable_ssaa=True, ssaa_factor=2)
    R.load_scene(sc, st)
    R.ray_trace()
    full_shadow = R.stats()["shadow_rays"]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    nloc = R.local_rows(8, 0, 1)
    outs = [torch.zeros((nloc, st.image_width), dtype=torch.int32, device="cuda:0") for _ in range(2)]
    torch.cuda.synchronize()
    first = None
    for i in range(6):
        s = streams[0] if i < 3 else streams[i % 2]
        R.render_bands_device(8, 0, 1, outs[i % 2].data_ptr(), s.cuda_stream)
        sh, rf = R.band_counters()
        assert (sh, rf) == (full_shadow, 0), (i, sh, full_shadow)
        img = outs[i % 2].cpu().numpy()
        if first is None:
            first = img.copy()
        assert np.array_equal(img, first), i


@pytest.mark.parametrize("ssaa", [False, True])
def test_failed_frame_keeps_the_previous_image(make_renderer, ssaa):
    """A frame that fails after its image became the internal buffer (RT_INJECT_FRAME_FAIL: the
    2nd ray_trace) is never presented: with SSAA the previous (downscaled) image stays; without,
    the internal buffer was reused, so the image reads as not rendered (background)."""
    from raytracercpp_amd import scenes
    from raytracercpp_amd._lib import RtError
    R = make_renderer(RT_INJECT_FRAME_FAIL="2")
    sc, st = scenes.bumpy70k(width=96, height=54, enable_ssaa=ssaa, ssaa_factor=2)
    R.load_scene(sc, st)
    R.ray_trace()
    R.post_process()
    first = R.get_image().copy()
    with pytest.raises(RtError):
        R.ray_trace()
    after = R.get_image()
    if ssaa:
        assert after.shape == first.shape and np.array_equal(after, first)
    else:
        bg = np.uint32(0xFF87CEEB)
        assert (after.ravel().view(np.uint32) == bg).all()
    R.ray_trace()   # the next frame renders normally
    R.post_process()
    assert np.array_equal(R.get_image(), first)


def test_set_devices_distinct_rccl(make_renderer):
    """The RCCL send / receive path of rt_set_devices (distinct devices, RT_MULTIDEV_RCCL=1):
    frames equal the one-device frame.  Needs two or more devices (skipped on one-GPU boxes);
    without the switch distinct devices are refused (experimental, include/rt_mi355x.h)."""
    import os
    import torch
    from raytracercpp_amd import scenes
    from raytracercpp_amd.renderer import render
    from raytracercpp_amd._lib import RtError
    n = torch.cuda.device_count()
    sc, st = scenes.bumpy70k(width=200, height=117, enable_ssaa=True, ssaa_factor=2)
    if n < 2:
        R = make_renderer()
        R.load_scene(sc, st)
        with pytest.raises(RtError):
            R.set_devices([0, 0, 0][:1] + [1])   # a second device id that does not exist here
        pytest.skip("one device: the RCCL path needs two or more")
    R1 = make_renderer()
    R1.load_scene(sc, st)
    render(R1)
    one = R1.get_image().copy()
    R = make_renderer(RT_MULTIDEV_RCCL="1")
    R.load_scene(sc, st)
    R.set_devices(list(range(min(n, 4))))
    render(R)
    assert np.array_equal(R.get_image(), one)


@pytest.mark.gpu
def test_tile_costs_and_heavy_order_keep_the_frame(R):
    """rt_tile_costs: after a frame, one cost per 8x8 tile of the render (zero only off the image);
    the next frames dequeue the costliest tiles first at raised wave priority (heavy_prep_kernel,
    set_wave_prio) and must produce the same image (only the order changes)."""
    from raytracercpp_amd import scenes
    sc, st = scenes.bumpy70k(width=160, height=96)
    R.load_scene(sc, st)
    R.ray_trace()
    first = R.get_image().copy()
    c = R.tile_costs()
    rw, rh = st.render_size()
    assert c.shape == ((rh + 7) // 8, (rw + 7) // 8)
    assert (c > 0).all()
    for _ in range(3):
        R.ray_trace()
        assert np.array_equal(R.get_image(), first)
    assert R.tile_costs().shape == c.shape
