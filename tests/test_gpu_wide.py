"""The sound wide-BVH query on the GPU build itself (rt_wide_query / rt_risk_words).

tests/test_wbvh.py proves on the HOST build (correctly rounded reciprocal and square root, the
host risk walk wbvh_risk_host) that every certified answer of the wide query is the reference's
BVH::intersect record (bvh.h:212-287, Moller-Trumbore triangle.cpp:25-91) on adversarial grazing
rays.  The frames run the DEVICE build: the hardware reciprocal / square root of wbvh.hpp and the
risk words wide_risk_kernel computes with atomics.  Here every one of those grazing cases runs
through the device query (kernels.hip wide_query_kernel, the frames' wbvh_closest + kdop_certifies),
the device risk words are compared with the host walk's, and the camera-plane scenes are rendered
as frames and compared with the oracle.  Bar: 0 certified answers differing from the oracle."""
import dataclasses

import numpy as np
import pytest

import test_wbvh as tw
from oracle.bindings import Oracle
from raytracercpp_amd import scenes
from raytracercpp_amd.scene import RenderSettings

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


@pytest.fixture(scope="module")
def R():
    from raytracercpp_amd.renderer import Renderer
    r = Renderer(0)
    yield r
    r.close()


def _scene(tri, cam=None, light=None, width=64, height=36):
    sc, st = scenes.robot1080(width=width, height=height)
    sc = dataclasses.replace(sc, tri=np.ascontiguousarray(tri, np.float32), tri_mat=np.zeros(len(tri), np.int32),
                             tri_uv=None)
    if cam is not None:
        sc.cam_pos = np.asarray(cam, np.float32)
    if light is not None:
        sc.light = np.asarray(light, np.float32)
    return sc, st


def _oracle_for(sc):
    return Oracle(sc, RenderSettings(bvh_max_depth=12, bvh_leaf_object_count=40))


def _device_differences(R, tri, o, d, kind, cam=None, light=None):
    """Runs the rays through the device query; returns (certified fraction, differing certified
    answers, the device's output).  The oracle answers the rays the device built.  Every input is
    finite: a NaN ray is a miss on both sides and would inflate the certified fraction."""
    assert np.isfinite(o).all() and np.isfinite(d).all(), "non-finite ray inputs"
    sc, st = _scene(tri, cam, light)
    R.load_scene(sc, st)
    g = R.wide_query(o, d, kind)
    oi, ot, ou, ov, orr, _ = _oracle_for(sc).bvh_query(g["o"], g["d"])
    status = g["status"]
    cert = status != 2
    bad = cert & ((status == 1) != (orr != 0))
    hit = (status == 1) & (orr != 0)
    bad |= hit & ((g["id"] != oi) | (bits(g["t"]) != bits(ot)) | (bits(g["u"]) != bits(ou)) | (bits(g["v"]) != bits(ov)))
    g["oracle"] = (oi, ot, orr)
    return float(cert.mean()), int(bad.sum()), g


def _shadow_decisions(g, p, light):
    """is_shadowed's decision (renderer.cpp:340-402) from the oracle's record of each ray, against the
    frame's own decision through the device's segment query (out 'shadowed': 2 = not decided)."""
    oi, ot, orr = g["oracle"]
    o, d = g["o"], g["d"]
    q = o + d * ot[:, None]
    pq = p - q
    pl = p - np.asarray(light, np.float32)[None]
    l2 = lambda v: (v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1]) + v[:, 2] * v[:, 2]
    ref = (orr != 0) & (l2(pq) < l2(pl))
    dec = g["shadowed"] != 2
    return float(dec.mean()), int((dec & ((g["shadowed"] == 1) != ref)).sum())


@pytest.mark.parametrize("seed,sin_lo,sin_hi", [(99, 1e-7, 1e-3), (5, 1e-9, 1e-5), (17, 1e-5, 1e-1)])
def test_device_grazing_plane(R, seed, sin_lo, sin_hi):
    """tests/test_wbvh.py::test_grazing_plane_certified_answers_match_oracle on the device build."""
    tri, o, d = tw.grazing_plane_case(seed=seed, sin_lo=sin_lo, sin_hi=sin_hi)
    cert, bad, _ = _device_differences(R, tri, o, d, kind=0)
    print(f"device grazing plane seed {seed}: {cert:.4f} certified, {bad} certified answers differ")
    assert bad == 0
    assert cert > 0.5


def test_device_grazing_sphere(R):
    tri, o, d = tw.grazing_sphere_case()
    cert, bad, _ = _device_differences(R, tri, o, d, kind=0)
    print(f"device grazing sphere: {cert:.4f} certified, {bad} certified answers differ")
    assert bad == 0
    assert cert > 0.5


def test_device_grazing_slivers(R):
    rng = np.random.default_rng(11)
    tri = tw._soup(rng)
    T = tri.reshape(-1, 3, 3).astype(np.float64)
    k = rng.integers(0, len(T), 20000)
    n = np.cross(T[k, 1] - T[k, 0], T[k, 2] - T[k, 0])
    ok = np.linalg.norm(n, axis=1) > 1e-12
    k, n = k[ok], n[ok] / np.linalg.norm(n[ok], axis=1, keepdims=True)
    e = T[k, 1] - T[k, 0]
    e /= np.maximum(np.linalg.norm(e, axis=1, keepdims=True), 1e-30)
    eps = np.exp(rng.uniform(np.log(1e-7), np.log(1e-3), len(k)))
    d = e + n * eps[:, None]
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = T[k].mean(1) - d * rng.uniform(0.2, 2.0, len(k))[:, None] + n * (eps * rng.uniform(-1, 1, len(k)))[:, None]
    cert, bad, _ = _device_differences(R, tri, o.astype(np.float32), d.astype(np.float32), kind=0)
    print(f"device grazing slivers: {cert:.4f} certified, {bad} certified answers differ")
    assert bad == 0


@pytest.mark.parametrize("h", [0.0, 1e-7, 1e-4, 1e-1])
def test_device_camera_grazing_plane(R, h):
    """Camera rays from a camera at height h above the tessellated plane (the camera's risk words)."""
    tri, o, d, cam = tw._plane_frame(23, h)
    cert, bad, _ = _device_differences(R, tri, o, d, kind=1, cam=cam, light=cam + np.float32(7.0))
    print(f"device camera at {h} from the plane: {cert:.4f} certified, {bad} differ")
    assert bad == 0


def test_device_camera_sphere_silhouette(R):
    rng = np.random.default_rng(4)
    sc, _ = scenes.bumpy70k(width=8, height=8)
    tri = sc.tri
    T = tri.reshape(-1, 3, 3).astype(np.float64)
    cam = np.array([0.3, 0.2, 6.0])
    k = rng.integers(0, len(T), 20000)
    p = T[k].mean(1) + (T[k, 1] - T[k, 0]) * rng.uniform(-0.3, 0.3, (20000, 1))
    d = p - cam
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = np.repeat(cam[None].astype(np.float32), 20000, 0)
    cert, bad, _ = _device_differences(R, tri, o, d.astype(np.float32), kind=1, cam=cam)
    print(f"device sphere silhouette from the camera: {cert:.4f} certified, {bad} differ")
    assert bad == 0


def _light_plane(h, n=20000):
    rng = np.random.default_rng(31)
    Rm = tw._rotation(rng)
    off = rng.uniform(-5, 5, 3)
    tri = (tw._grid(400, 4.0).reshape(-1, 3, 3) @ Rm.T + off).reshape(-1, 9).astype(np.float32)
    L = (np.array([rng.uniform(-6, 6), h, rng.uniform(-6, 6)]) @ Rm.T + off).astype(np.float32)
    hp = np.zeros(n)
    hp[n // 2:] = rng.choice([-1, 1], n - n // 2) * np.exp(rng.uniform(np.log(1e-9), np.log(1e-3), n - n // 2))
    p = (np.stack([rng.uniform(-4, 4, n), hp, rng.uniform(-4, 4, n)], 1) @ Rm.T + off).astype(np.float32)
    az = rng.uniform(0, 2 * np.pi, n)
    nl = np.stack([np.cos(az), np.zeros(n), np.sin(az)], 1)
    nl[: n // 2] = [0.0, 1.0, 0.0]
    nrm = (nl @ Rm.T).astype(np.float32)
    return tri, p, nrm, L


@pytest.mark.parametrize("h", [0.0, 1e-6, 1e-3])
def test_device_light_grazing_plane(R, h):
    """Shadow rays from the plane (and from surfaces standing on it) to a light at height h: every ray
    grazes the plane (the light's risk words); the frame's shadow decisions too."""
    tri, p, nrm, L = _light_plane(h)
    cert, bad, g = _device_differences(R, tri, p, nrm, kind=2, light=L, cam=np.array([0.0, 30.0, 0.0], np.float32))
    dec, dbad = _shadow_decisions(g, p, L)
    print(f"device light at {h} from the plane: {cert:.4f} certified, {bad} differ; "
          f"{dec:.4f} shadow decisions by the wide query, {dbad} differ")
    assert bad == 0 and dbad == 0


def test_device_light_sphere_terminator(R):
    rng = np.random.default_rng(8)
    sc, _ = scenes.bumpy70k(width=8, height=8)
    tri = sc.tri
    T = tri.reshape(-1, 3, 3).astype(np.float64)
    L = np.array([5.0, 0.5, 1.0], np.float32)
    nn = np.cross(T[:, 1] - T[:, 0], T[:, 2] - T[:, 0])
    area = np.linalg.norm(nn, axis=1)
    nn /= np.maximum(area, 1e-30)[:, None]
    toL = L - T.mean(1)
    toL /= np.linalg.norm(toL, axis=1, keepdims=True)
    # the terminator: the triangles most nearly edge-on to the light (zero-area pole triangles have no
    # normal and are left out, or their zero directions would sort first)
    key = np.where(area > 1e-12, np.abs((nn * toL).sum(1)), np.inf)
    k = np.argsort(key)[:20000]
    uv = rng.uniform(0, 1, (len(k), 2))
    uv[uv.sum(1) > 1] = 1 - uv[uv.sum(1) > 1]
    p = (T[k, 0] + (T[k, 1] - T[k, 0]) * uv[:, :1] + (T[k, 2] - T[k, 0]) * uv[:, 1:]).astype(np.float32)
    cert, bad, g = _device_differences(R, tri, p, nn[k].astype(np.float32), kind=2, light=L,
                                       cam=np.array([0.0, 0.0, 6.0], np.float32))
    dec, dbad = _shadow_decisions(g, p, L)
    print(f"device sphere terminator: {cert:.4f} certified, {bad} differ; {dec:.4f} decided, {dbad} differ")
    assert bad == 0 and dbad == 0


def _words_agree(gw, hw):
    """GPU risk words vs the host walk's: equal, or each GPU key <= the host key and each GPU box
    holding the host box (a sound over-approximation)."""
    if np.array_equal(gw, hw):
        return True
    gk = (gw >> np.uint64(48)).astype(np.uint32) << 16
    hk = (hw >> np.uint64(48)).astype(np.uint32) << 16
    gkf, hkf = gk.view(np.float32), hk.view(np.float32)
    ok = gkf <= hkf
    has = hkf < np.inf
    for a in range(3):
        glo = (gw >> np.uint64(8 * a)) & np.uint64(255)
        ghi = (gw >> np.uint64(8 * (a + 3))) & np.uint64(255)
        hlo = (hw >> np.uint64(8 * a)) & np.uint64(255)
        hhi = (hw >> np.uint64(8 * (a + 3))) & np.uint64(255)
        ok &= ~has | ((glo <= hlo) & (ghi >= hhi))
    return bool(ok.all())


@pytest.mark.parametrize("scene_name", ["plane_camera", "plane_light", "terminator", "sphere1m"])
def test_device_risk_words_match_host_walk(R, scene_name):
    """wide_risk_kernel's words (GPU atomics over the wide BVH's triangles) against wbvh_risk_host's
    walk over the same resident tree, for the camera and the light of the frame."""
    if scene_name == "plane_camera":
        tri, _, _, cam = tw._plane_frame(23, 1e-7)
        sc, st = _scene(tri, cam=cam, light=cam + np.float32(3.0))
    elif scene_name == "plane_light":
        tri, _, _, L = _light_plane(1e-6)
        sc, st = _scene(tri, cam=np.array([0.0, 30.0, 0.0], np.float32), light=L)
    elif scene_name == "terminator":
        sc0, _ = scenes.bumpy70k(width=8, height=8)
        sc, st = _scene(sc0.tri, cam=np.array([0.0, 0.0, 6.0], np.float32), light=np.array([5.0, 0.5, 1.0], np.float32))
    else:
        sc, st = scenes.sphere1m(width=64, height=36)
    R.load_scene(sc, st)
    gw, gbad = R.risk_words(0)
    hw, hbad = R.risk_words(1)
    assert gbad == 0 and hbad == 0, (gbad, hbad)
    assert gw.shape == hw.shape and gw.size > 0
    at_risk = int(((hw >> np.uint64(48)) != np.uint64(0x7F80)).sum())
    same = int((gw == hw).sum())
    print(f"{scene_name}: {gw.size} words, {at_risk} at risk on the host, {same} bitwise equal")
    assert at_risk > 0
    assert _words_agree(gw, hw)


def _camera_plane_scene(h, width=160, height=90, seed=23):
    """The tessellated plane of tests/test_wbvh.py::_plane_frame under a camera at height h that looks
    along it, horizontally: the rows below the horizon meet it at grazing angles.  The camera sits at
    the world origin (the plane is placed around it), so that its rays resolve directions far finer
    than the float spacing of a distant position would allow, and the vertical field of view scales
    with h (half-angle ~20 h, at most 30 degrees) so that the band of hits at t > 0.1 (trace_ray's
    minimum, renderer.cpp:1039-1040) fills a quarter of the frame.  At h = 0 the camera is in the plane:
    every ray either leaves it or meets it within rounding of t = 0 (a frame of misses, each certified
    against spurious grazing reports)."""
    rng = np.random.default_rng(seed)
    Rm = tw._rotation(rng)
    C = np.array([rng.uniform(-3, 3), h, rng.uniform(-3, 3)])
    tri = ((tw._grid(400, 4.0).reshape(-1, 3, 3) - C) @ Rm.T).reshape(-1, 9).astype(np.float32)
    az = rng.uniform(0, 2 * np.pi)
    fwd = np.array([np.cos(az), 0.0, np.sin(az)])
    right = np.cross(fwd, [0.0, 1.0, 0.0])
    right /= np.linalg.norm(right)
    up = np.cross(right, fwd)
    c2w = np.eye(4)
    c2w[:3, :3] = Rm @ np.column_stack([right, up, -fwd])   # camera x right, y up, looking down -z
    sc, st = scenes.robot1080(width=width, height=height)
    T = scenes.default_transforms()
    rw, rh = st.render_size()
    fov = float(min(60.0, np.degrees(2.0 * np.arctan(20.0 * max(h, 1e-7)))))
    proj, pinv = T.camera_matrices(fov, np.float32(rw) / np.float32(rh))
    sc = dataclasses.replace(sc, tri=tri, tri_mat=np.zeros(len(tri), np.int32), tri_uv=None, proj_inv=pinv, proj=proj,
                             cam_fov=fov, cam_pos=np.zeros(3, np.float32),
                             cam_to_world=c2w.astype(np.float32).ravel(), world_to_cam=None,
                             light=((np.array([0.5, 3.0, -0.7]) - C) @ Rm.T).astype(np.float32))
    return sc, st


@pytest.mark.parametrize("h", [0.0, 1e-7, 1e-4, 1e-1])
def test_camera_plane_frames_match_oracle(R, h):
    """The camera-at-h plane scenes rendered as frames (ray_trace with the wide BVH resident and the
    GPU's risk words) against the oracle's frame: hit IDs, t, shadow flags and ARGB bit for bit."""
    sc, st = _camera_plane_scene(h)
    R.load_scene(sc, st)
    R.ray_trace()
    R.finish_accel()
    R.request_aux(rgba=True, hit=True, shadow=True)
    R.ray_trace()
    g = R.get_internal(argb=True, rgba=True, hit=True, shadow=True)
    o = Oracle(sc, st).render_rows()
    hits = int((o.hit_id >= 0).sum())
    print(f"camera at {h}: {hits} of {o.hit_id.size} pixels hit the plane")
    if h > 0:
        assert hits > 500
    assert np.array_equal(g["hit_id"], o.hit_id), f"{int((g['hit_id'] != o.hit_id).sum())} hit-ID mismatches"
    assert np.array_equal(bits(g["hit_t"]), bits(o.hit_t))
    assert np.array_equal(g["shadow"], o.shadow)
    assert np.array_equal(g["argb"], o.argb)
    assert float(np.abs(g["rgba"] - o.rgba).max()) <= 1e-4


def _group_case(name):
    """(tri, o, d, kind, cam, light) of one grazing case above."""
    if name == "plane":
        tri, o, d = tw.grazing_plane_case(seed=99, sin_lo=1e-7, sin_hi=1e-3)
        return tri, o, d, 0, None, None
    if name == "sphere":
        tri, o, d = tw.grazing_sphere_case()
        return tri, o, d, 0, None, None
    if name == "camera_plane":
        tri, o, d, cam = tw._plane_frame(23, 1e-7)
        return tri, o, d, 1, cam, cam + np.float32(7.0)
    if name == "light_plane":
        tri, p, nrm, L = _light_plane(0.0)
        return tri, p, nrm, 2, np.array([0.0, 30.0, 0.0], np.float32), L
    raise KeyError(name)


@pytest.mark.parametrize("G", [2, 4, 8])
@pytest.mark.parametrize("name", ["plane", "sphere", "camera_plane", "light_plane"])
def test_device_lane_groups_match_one_lane(R, monkeypatch, name, G):
    """wbvh_closest<.., G> (G lanes walking one ray's tree together: work taken from each other's stacks,
    the best hit shared, kernels.hip trace_split_part) returns the one-lane query's answers bit for
    bit -- status, triangle, t, u, v and the shadow decision -- on the grazing cases above, and 0 of its
    certified answers differ from the oracle."""
    tri, o, d, kind, cam, light = _group_case(name)
    monkeypatch.delenv("RT_WIDE_QUERY_GROUP", raising=False)
    cert1, bad1, g1 = _device_differences(R, tri, o, d, kind, cam=cam, light=light)
    monkeypatch.setenv("RT_WIDE_QUERY_GROUP", str(G))
    certG, badG, gG = _device_differences(R, tri, o, d, kind, cam=cam, light=light)
    for k in ("status", "id", "shadowed"):
        assert np.array_equal(gG[k], g1[k]), (k, int((gG[k] != g1[k]).sum()))
    for k in ("t", "u", "v"):
        assert np.array_equal(bits(gG[k]), bits(g1[k])), k
    print(f"{name}, {G} lanes per ray: {certG:.4f} certified, {badG} differ (one lane: {cert1:.4f}, {bad1})")
    assert badG == 0
