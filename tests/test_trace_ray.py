"""Renderer::trace_ray for arbitrary rays (renderer.h:144, renderer.cpp:1008-1066): the shaded
counterpart of BVH::intersect's ray API.

CPU: the oracle's orc_trace_rays_shaded, fed every pixel's camera ray in pixel order (ray i =
pixel i, so rough reflections draw pixel i's stream), reproduces the reference-generated golden
frames -- it is the per-pixel body of ray_trace (renderer.cpp:1086-1113) with the ray built here.
GPU: rt_trace_ray equals the golden frames the same way, and the oracle on random rays at
current_recursion_depth 0, 1 and past max_recursion_depth: bit-exact sources, t and flags, float
RGBA within 1e-4 (north_star)."""
import numpy as np
import pytest

from golden_cases import Case, case_names, manifest
from oracle.bindings import Oracle

RGBA_TOL = 1e-4
# ray-traced golden frames (the raster cases shade through trace_triangle, SSAO post-processes)
TRACE_CASES = [n for n in case_names() if not manifest()[n]["settings"].get("hybrid_rasterization_tracing")
               and not manifest()[n]["settings"].get("enable_ssao")]
SMALL_CASES = ["textured", "diffuse_map_skysphere", "mirror", "rough", "brute_force", "shading_3", "c1_sphere256"]


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def _xform_point(m, x, y, z):
    """Transform::operator()(Point) (mat.cpp:83-100) in float32, the reference's operation order."""
    m = np.asarray(m, np.float32)
    xt = m[0] * x + m[1] * y + m[2] * z + m[3]
    yt = m[4] * x + m[5] * y + m[6] * z + m[7]
    zt = m[8] * x + m[9] * y + m[10] * z + m[11]
    wt = m[12] * x + m[13] * y + m[14] * z + m[15]
    w = np.float32(1) / wt
    keep = wt == np.float32(1)
    return (np.where(keep, xt, xt * w), np.where(keep, yt, yt * w), np.where(keep, zt, zt * w))


def camera_rays(sc, st):
    """Every pixel's primary ray of Renderer::ray_trace (renderer.cpp:1086-1098), pixel order."""
    rw, rh = st.render_size()
    py, px = np.meshgrid(np.arange(rh, dtype=np.float32), np.arange(rw, dtype=np.float32), indexing="ij")
    f32 = np.float32
    y_world = (py + f32(0.5)) / f32(rh) * f32(2) - f32(1)
    x_world = (px + f32(0.5)) / f32(rw) * f32(2) - f32(1)
    vs = _xform_point(sc.proj_inv, x_world, y_world, np.full_like(x_world, -1))
    ws = _xform_point(sc.cam_to_world, *vs)
    cam = np.asarray(sc.cam_pos, np.float32)
    d = np.stack([ws[0] - cam[0], ws[1] - cam[1], ws[2] - cam[2]], axis=-1).reshape(-1, 3)
    # Vector::normalize (vec.cpp:150-154): 1 / sqrt(length2), then a scale
    l2 = d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1] + d[:, 2] * d[:, 2]
    k = f32(1) / np.sqrt(l2)
    d = d * k[:, None]
    o = np.broadcast_to(cam, d.shape).copy()
    return o.astype(np.float32), d.astype(np.float32)


def _check_against_golden(rgba, src, t, found, shadow, exp):
    assert np.array_equal(np.where(found == 1, src, -1), exp["hit_id"])
    assert np.array_equal(bits(t), bits(exp["hit_t"]))
    assert np.array_equal(shadow, exp["shadow"])
    assert float(np.abs(rgba.reshape(-1, 4) - exp["rgba"].reshape(-1, 4)).max()) <= RGBA_TOL


@pytest.mark.parametrize("name", SMALL_CASES)
def test_oracle_trace_ray_reproduces_golden_frames(name):
    c = Case(name)
    o, d = camera_rays(c.scene, c.settings)
    rgba, src, t, found, shadow, cnt = Oracle(c.scene, c.settings).trace_ray(o, d, 0)
    _check_against_golden(rgba, src, t, found, shadow, c.expected())
    assert cnt["shadow_rays"] == c.meta["counters"]["shadow_rays"]
    assert cnt["reflection_rays"] == c.meta["counters"]["reflection_rays"]


def test_oracle_trace_ray_past_max_depth_is_black():
    c = Case("mirror")
    o, d = camera_rays(c.scene, c.settings)
    rgba, src, t, found, shadow, _ = Oracle(c.scene, c.settings).trace_ray(o[:100], d[:100],
                                                                          c.settings.max_recursion_depth + 1)
    assert np.all(rgba == np.array([0, 0, 0, 1], np.float32)) and np.all(found == 0) and np.all(src == -1)
    assert np.all(t == -1)


@pytest.fixture(scope="module")
def R():
    from raytracercpp_amd.renderer import Renderer
    r = Renderer(0)
    yield r
    r.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", TRACE_CASES)
def test_gpu_trace_ray_reproduces_golden_frames(R, name):
    c = Case(name)
    R.load_scene(c.scene, c.settings)
    o, d = camera_rays(c.scene, c.settings)
    rgba, src, t, found, shadow = R.trace_ray(o, d, 0)
    _check_against_golden(rgba, src, t, found, shadow, c.expected())
    st = R.stats()
    assert st["shadow_rays"] == c.meta["counters"]["shadow_rays"]
    assert st["reflection_rays"] == c.meta["counters"]["reflection_rays"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", SMALL_CASES)
def test_gpu_trace_ray_random_rays_match_oracle(R, name):
    """Rays from random origins around the scene at depths 0, 1 and max + 1 (black)."""
    c = Case(name)
    R.load_scene(c.scene, c.settings)
    orc = Oracle(c.scene, c.settings)
    rng = np.random.default_rng(17)
    n = 20000
    cam = np.asarray(c.scene.cam_pos, np.float32)
    o = (cam + rng.uniform(-1.5, 1.5, (n, 3))).astype(np.float32)
    d = rng.standard_normal((n, 3))
    d[: n // 2, 2] = -np.abs(d[: n // 2, 2]) * 3   # half of them roughly down the view axis
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    for depth in (0, 1, c.settings.max_recursion_depth + 1):
        g = R.trace_ray(o, d, depth)
        e = orc.trace_ray(o, d, depth)
        assert np.array_equal(g[1], e[1]), (depth, int((g[1] != e[1]).sum()))
        assert np.array_equal(bits(g[2]), bits(e[2])), depth
        assert np.array_equal(g[3], e[3]) and np.array_equal(g[4], e[4]), depth
        assert float(np.abs(g[0] - e[0]).max()) <= RGBA_TOL, depth
        st = R.stats()
        assert st["shadow_rays"] == e[5]["shadow_rays"] and st["reflection_rays"] == e[5]["reflection_rays"], depth


@pytest.mark.gpu
def test_gpu_trace_ray_errors(R):
    from raytracercpp_amd._lib import RtError
    c = Case("mirror")
    R.load_scene(c.scene, c.settings)
    o = np.zeros((4, 3), np.float32)
    with pytest.raises(RtError):
        R.trace_ray(o, o, -1)
    rgba, src, t, found, shadow = R.trace_ray(o[:0], o[:0], 0)
    assert rgba.shape == (0, 4)
