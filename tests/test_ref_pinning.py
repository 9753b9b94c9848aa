"""Pins the oracle and the product's host code against the reference's own compiled
translation units (oracle/_ref/libref_harness.so).  Skipped where the reference
harness was not built (it needs /root/reference at build time).  CPU only."""
import os

import numpy as np
import pytest

from oracle.bindings import Oracle, RefHarness
from raytracercpp_amd import _lib, scenes
from raytracercpp_amd.scene import RenderSettings

pytestmark = pytest.mark.skipif(not RefHarness.available(), reason="reference harness not built")

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "data")


def u32(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def random_rays(rng, n, center, spread):
    o = (center + rng.uniform(-spread, spread, size=(n, 3))).astype(np.float32)
    d = rng.standard_normal((n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return o, d.astype(np.float32)


@pytest.mark.parametrize("obj,depth,leaf", [("Robot/robot.obj", 12, 40), ("Robot/robot.obj", 6, 8),
                                            ("Geometry/geometry.obj", 12, 4)])
def test_oracle_bvh_query_random_rays(obj, depth, leaf):
    m = _lib.make_transform("translation", 0, 0, -4)
    tri, mat, uv, mats = RefHarness.load_obj(os.path.join(DATA, obj), m)
    rng = np.random.default_rng(7)
    o, d = random_rays(rng, 20000, np.array([0, 0, -4], np.float32), 3.0)
    sc, _ = scenes.sphere256()
    sc.tri, sc.tri_mat, sc.tri_uv = tri, mat, uv
    st = RenderSettings(bvh_max_depth=depth, bvh_leaf_object_count=leaf)
    ids, t, u, v, ret, _ = Oracle(sc, st).bvh_query(o, d)
    rids, rt_, ru, rv, rret = RefHarness.bvh_query(tri, depth, leaf, o, d)
    assert np.array_equal(ids, rids)
    assert np.array_equal(ret, rret)
    assert np.array_equal(u32(t), u32(rt_))
    assert np.array_equal(u32(u), u32(ru)) and np.array_equal(u32(v), u32(rv))
    assert (ret == 1).sum() > 1000   # the rays do hit the mesh


def test_oracle_bvh_query_sphere1m_surface_rays():
    """Shadow-like rays leaving the 1M-tri surface (deep traversal, big max-depth leaves)."""
    sc, st = scenes.sphere1m(width=64, height=36)
    rng = np.random.default_rng(3)
    idx = rng.integers(0, sc.ntri, 3000)
    t9 = sc.tri[idx].reshape(-1, 3, 3).astype(np.float64)
    p = t9.mean(axis=1)
    n = np.cross(t9[:, 1] - t9[:, 0], t9[:, 2] - t9[:, 0])
    n /= np.maximum(np.linalg.norm(n, axis=1, keepdims=True), 1e-30)
    o = (p + 1e-4 * n).astype(np.float32)
    d = np.array([3, 3, 2], np.float64) - p
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    ids, t, u, v, ret, _ = Oracle(sc, st).bvh_query(o, d.astype(np.float32))
    rids, rt_, ru, rv, rret = RefHarness.bvh_query(sc.tri, 12, 40, o, d.astype(np.float32))
    assert np.array_equal(ids, rids) and np.array_equal(ret, rret) and np.array_equal(u32(t), u32(rt_))


def test_heap_order_matches_reference_queue_type():
    rng = np.random.default_rng(11)
    for _ in range(3000):
        n = int(rng.integers(1, 9))
        keys = rng.integers(-2, 3, size=n).astype(np.float32)
        if rng.random() < 0.2:
            keys[rng.integers(0, n)] = -0.0
        assert np.array_equal(Oracle.heap_order(keys), RefHarness.heap_order(keys))


def test_product_transforms_match_reference():
    for kind, args in (("translation", (0, 0, -5)), ("rx", (20,)), ("ry", (30,)), ("rz", (-45,)),
                       ("scale", (1.5, 1.5, 1.5)), ("identity", ())):
        assert np.array_equal(u32(_lib.make_transform(kind, *args)), u32(RefHarness.transform(kind, *args)))
    a = _lib.compose(_lib.make_transform("translation", 0, 0, -3), _lib.make_transform("ry", 30))
    b = RefHarness.compose(RefHarness.transform("translation", 0, 0, -3), RefHarness.transform("ry", 30))
    assert np.array_equal(u32(a), u32(b))
    assert np.array_equal(u32(_lib.inverse(a)), u32(RefHarness.inverse(b)))
    for fov, aspect in ((80, 1.0), (80, 16 / 9), (45, 1.0), (90, 0.5)):
        p, pi = _lib.camera_matrices(fov, np.float32(aspect))
        rp, rpi = RefHarness.camera_matrices(fov, np.float32(aspect))
        assert np.array_equal(u32(p), u32(rp)) and np.array_equal(u32(pi), u32(rpi))
    pts = np.random.default_rng(0).uniform(-5, 5, (1000, 3)).astype(np.float32)
    assert np.array_equal(u32(_lib.transform_points(a, pts)), u32(RefHarness.transform_points(a, pts)))
    assert np.array_equal(u32(scenes.transform_points_f32(a, pts)), u32(RefHarness.transform_points(a, pts)))


@pytest.mark.parametrize("obj", ["cube.obj", "Robot/robot.obj", "Geometry/geometry.obj"])
def test_product_obj_loader_matches_reference(obj):
    m = _lib.compose(_lib.make_transform("translation", 0, 0, -4), _lib.make_transform("ry", 30))
    a = _lib.load_obj(os.path.join(DATA, obj), m, mat_offset=2)
    b = RefHarness.load_obj(os.path.join(DATA, obj), m, mat_offset=2)
    for x, y in zip(a, b):
        if x is None:
            assert y is None
            continue
        assert x.shape == y.shape and np.array_equal(u32(x), u32(y))


def test_specular_threshold_formula_matches_reference():
    for spec, ns in (((0.5, 0.5, 0.5), 250.0), ((0.5, 0.5, 0.5), 5.0), ((0.2, 0.3, 0.9), 20.0)):
        assert np.float32(scenes.specular_threshold(spec, ns)) == np.float32(RefHarness.specular_threshold(spec, ns))


def test_reference_row_sample_equals_full_render_rows():
    """bench.py's CPU baseline times ref_render_row_sample: it renders exactly the strided rows."""
    sc, st = scenes.bumpy70k(width=96, height=54)
    full = RefHarness.render_rows(sc, st)
    rw, rh = st.render_size()
    samp = RefHarness.render_row_sample(sc, st, 1, rh // 4, 4)
    rows = 1 + 4 * np.arange(rh // 4)
    assert np.array_equal(samp.argb.reshape(-1, rw), full.argb.reshape(rh, rw)[rows])
    assert np.array_equal(samp.hit_id.reshape(-1, rw), full.hit_id.reshape(rh, rw)[rows])
    assert samp.seconds > 0


@pytest.mark.parametrize("raster,w,h,kw", [
    (False, 211, 101, dict(ssao_sample_count=24, ssao_radius=0.3, rng_seed=99)),
    (False, 96, 56, dict(ssao_sample_count=12, ssao_radius=0.9, ssao_amount=0.6, enable_ssaa=True, ssaa_factor=2)),
    (True, 165, 93, dict(ssao_sample_count=20, ssao_radius=0.6)),
])
def test_oracle_ssao_matches_reference_simd_helpers(raster, w, h, kw):
    """post_process_ssao_SIMD (renderer.cpp:1229-1434): the oracle's scalar restatement of
    the AVX2 lanes and scalar tail against the reference's own __m256 helpers."""
    sc, st = scenes.bumpy70k(width=w, height=h, enable_ssao=True, hybrid_rasterization_tracing=raster, **kw)
    o = Oracle(sc, st)
    res = o.raster() if raster else o.render_rows()
    ref = RefHarness.raster(sc, st) if raster else RefHarness.render_rows(sc, st)
    assert np.array_equal(u32(res.zbuf), u32(ref.zbuf))
    assert np.array_equal(u32(res.nbuf), u32(ref.nbuf))
    a1, ao1 = o.ssao(res)
    a2, ao2 = RefHarness.ssao(sc, st, ref)
    assert ao1.max() > 0
    assert np.array_equal(ao1, ao2)
    assert np.array_equal(a1, a2)
