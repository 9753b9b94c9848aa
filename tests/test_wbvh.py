"""The wide-BVH certified closest hit (raytracercpp_amd/csrc/wbvh.hpp), run on
the host through rt_wbvh_query (the same traversal and certificate code the primary-ray
kernel compiles), against the oracle's BVH::intersect (bvh.h:212-287): every CERTIFIED
query must return the reference's record and boolean bit for bit; queries it cannot
certify go to the exact octree traversal on the GPU.  CPU only (no GPU call)."""
import numpy as np
import pytest

from oracle.bindings import Oracle
from raytracercpp_amd import _lib, scenes
from raytracercpp_amd.scene import RenderSettings


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def _rays(rng, n, center, spread):
    o = (center + rng.uniform(-spread, spread, size=(n, 3))).astype(np.float32)
    d = rng.standard_normal((n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return o, d.astype(np.float32)


def _voxels(n=8, size=0.2, gap=0.05):
    cube = np.array([[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0], [0, 0, 1], [1, 0, 1], [1, 1, 1], [0, 1, 1]], np.float32)
    faces = [(0, 2, 1), (0, 3, 2), (4, 5, 6), (4, 6, 7), (0, 1, 5), (0, 5, 4), (3, 6, 2), (3, 7, 6), (0, 4, 7),
             (0, 7, 3), (1, 2, 6), (1, 6, 5)]
    tris = []
    for i in range(n):
        for j in range(n):
            for k in range(n):
                v = cube * size + np.array([i, j, k], np.float32) * (size + gap) - n * (size + gap) / 2
                tris += [np.concatenate([v[f[0]], v[f[1]], v[f[2]]]) for f in faces]
    return np.array(tris, np.float32)


def _soup(rng, n=4000):
    c = rng.uniform([-2.0, -1.4, -7.0], [2.0, 1.5, -2.5], (n, 3))
    e1 = rng.normal(size=(n, 3)) * 0.25
    e2 = rng.normal(size=(n, 3)) * 0.25
    sl = rng.random(n) < 0.33
    e2[sl] = e1[sl] * rng.uniform(0.5, 2.0, (int(sl.sum()), 1)) + rng.normal(size=(int(sl.sum()), 3)) * 1e-6
    dg = rng.random(n) < 0.05
    e2[dg] = e1[dg]
    return np.concatenate([c, c + e1, c + e2], axis=1).astype(np.float32)


def _check(tri, o, d, depth=12, leaf=40, max_uncert=0.01):
    status, ids, t, u, v, stats, _ = _lib.wbvh_query(tri, o, d, depth, leaf)
    assert stats["violations"] == 0
    base, _ = scenes.robot1080(width=8, height=8)
    import dataclasses
    sc = dataclasses.replace(base, tri=np.ascontiguousarray(tri, np.float32), tri_mat=np.zeros(len(tri), np.int32),
                             tri_uv=None)
    oi, ot, ou, ov, orr, _ = Oracle(sc, RenderSettings(bvh_max_depth=depth, bvh_leaf_object_count=leaf)).bvh_query(o, d)
    cert = status != 2
    hit = status == 1
    assert np.array_equal((orr != 0)[cert], hit[cert]), "return value"
    assert np.array_equal(ids[hit], oi[hit]), f"{int((ids[hit] != oi[hit]).sum())} hit-ID mismatches"
    for a, b in ((t, ot), (u, ou), (v, ov)):
        assert np.array_equal(bits(a[hit]), bits(b[hit]))
    assert (status == 2).mean() <= max_uncert, f"{(status == 2).mean():.4f} not certified"
    return status, stats


@pytest.mark.parametrize("scene_name", ["robot", "voxels", "sphere1m_surface", "grazing", "soup", "bumpy_camera",
                                        "bumpy_shadow", "robot_shadow"])
def test_certified_queries_match_oracle(scene_name):
    rng = np.random.default_rng(7)
    max_uncert = 0.01
    if scene_name == "robot":
        tri = scenes.robot1080()[0].tri
        o, d = _rays(rng, 50000, np.array([0, 0, -4], np.float32), 3.0)
    elif scene_name == "voxels":
        # coinciding slabs and exactly tied hits (shared cube edges and faces): ties are not certified
        tri = _voxels()
        o, d = _rays(rng, 50000, np.zeros(3, np.float32), 2.5)
        d[:10000] = np.eye(3, dtype=np.float32)[rng.integers(0, 3, 10000)] * rng.choice([-1, 1], (10000, 1))
        max_uncert = 0.2
    elif scene_name == "grazing":
        # tiny / zero / denormal direction components: zero slab denominators in both structures
        tri = scenes.robot1080()[0].tri
        o, d = _rays(rng, 50000, np.array([0, 0, -4], np.float32), 3.0)
        tiny = rng.choice(np.array([0.0, 1e-13, -1e-13, 1e-30, -1e-41], np.float32), (50000,))
        d[np.arange(50000), rng.integers(0, 3, 50000)] = tiny
    elif scene_name == "soup":
        # slivers (nearly collinear vertices) and degenerate triangles
        tri = _soup(rng)
        o, d = _rays(rng, 50000, np.array([0, 0, -1], np.float32), 1.0)
    elif scene_name in ("bumpy_shadow", "robot_shadow"):
        # is_shadowed's rays from the camera's hits toward the light: the backface cones
        # (wbvh.hpp RT_W_CONE) skip most of the patches around each origin
        import tools.shadow_probe as sp
        sc, st = (scenes.bumpy70k if scene_name == "bumpy_shadow" else scenes.robot1080)(width=320, height=180)
        o, d = sp.shadow_rays(sc, st, 1)
        tri = sc.tri
    elif scene_name == "bumpy_camera":
        sc, st = scenes.bumpy70k(width=480, height=270)
        import tools.wbvh_probe as wp
        o, d = wp.camera_rays(sc, st, 1)
        tri = sc.tri
    else:
        # shadow-ray-like queries leaving the 1M-triangle sphere's surface
        sc, _ = scenes.sphere1m(width=64, height=36)
        tri = sc.tri
        idx = rng.integers(0, sc.ntri, 20000)
        t9 = tri[idx].reshape(-1, 3, 3).astype(np.float64)
        p = t9.mean(axis=1)
        n = np.cross(t9[:, 1] - t9[:, 0], t9[:, 2] - t9[:, 0])
        n /= np.maximum(np.linalg.norm(n, axis=1, keepdims=True), 1e-30)
        o = (p + 1e-4 * n).astype(np.float32)
        dd = rng.standard_normal((20000, 3))
        d = (dd / np.linalg.norm(dd, axis=1, keepdims=True)).astype(np.float32)
    status, _ = _check(tri, o, d, max_uncert=max_uncert)
    assert (status == 1).sum() > 0


def test_scaled_scenes_are_not_certified():
    """Outside 2^-20 < scale < 2^20 the certificate's rounding margins are not claimed:
    every query goes to the exact traversal."""
    rng = np.random.default_rng(3)
    tri = scenes.robot1080()[0].tri
    for f in (np.float32(1e-13), np.float32(1e13)):
        o, d = _rays(rng, 2000, np.array([0, 0, -4], np.float32) * f, 3.0 * f)
        status, *_ = _lib.wbvh_query(tri * f, o, d)
        assert (status == 2).all()


def test_structure_on_degenerate_inputs():
    """All-equal centroids, duplicated and zero-area triangles, a single triangle."""
    rng = np.random.default_rng(5)
    t = rng.uniform(-1, 1, (3000, 9)).astype(np.float32)
    t[:500] = t[0]                    # 500 copies of one triangle
    t[500:800, 3:6] = t[500:800, 0:3]   # degenerate
    for tri in (t, t[:1], np.repeat(t[:1], 40, axis=0)):
        o, d = _rays(rng, 5000, np.zeros(3, np.float32), 1.5)
        _check(tri, o, d, max_uncert=1.0)


def _grid(n, size):
    g = np.linspace(-size, size, n + 1)
    X, Z = np.meshgrid(g, g, indexing="ij")
    P = np.stack([X, np.zeros_like(X), Z], -1)
    a, b, c, d = P[:-1, :-1].reshape(-1, 3), P[1:, :-1].reshape(-1, 3), P[1:, 1:].reshape(-1, 3), P[:-1, 1:].reshape(-1, 3)
    return np.concatenate([np.concatenate([a, d, c], 1), np.concatenate([a, c, b], 1)], 0)


def _rotation(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def grazing_plane_case(seed=99, n_rays=20000, sin_lo=1e-7, sin_hi=1e-3):
    """A tessellated 400 x 400 plane in a random orientation and rays that meet it at grazing
    angles (sin in [sin_lo, sin_hi]): the adversarial input of DESIGN.md 5.6."""
    rng = np.random.default_rng(seed)
    R = _rotation(rng)
    off = rng.uniform(-5, 5, 3)
    tri = (_grid(400, 4.0).reshape(-1, 3, 3) @ R.T + off).reshape(-1, 9).astype(np.float32)
    s = np.exp(rng.uniform(np.log(sin_lo), np.log(sin_hi), n_rays))
    az = rng.uniform(0, 2 * np.pi, n_rays)
    cs = np.sqrt(1 - s * s)
    d = np.stack([cs * np.cos(az), -s, cs * np.sin(az)], 1)
    L = rng.uniform(0.5, 6.0, n_rays)
    p = np.stack([rng.uniform(-3, 3, n_rays), np.zeros(n_rays), rng.uniform(-3, 3, n_rays)], 1)
    o = ((p - d * L[:, None]) @ R.T + off).astype(np.float32)
    return tri, o, (d @ R.T).astype(np.float32)


def grazing_q(tri, ids, d):
    """Q = sin(angle at a) |cos(n, d)| of triangle ids[i] for ray i (the conditioning of its
    Moller-Trumbore test)."""
    T = tri[ids].astype(np.float64).reshape(-1, 3, 3)
    ab, ac = T[:, 1] - T[:, 0], T[:, 2] - T[:, 0]
    n = np.cross(ab, ac)
    dd = d.astype(np.float64)
    return np.abs((n * dd).sum(1)) / (np.linalg.norm(ab, axis=1) * np.linalg.norm(ac, axis=1) * np.linalg.norm(dd, axis=1))


def _grazing_differences(tri, o, d, **risk):
    """(certified fraction, number of certified answers that differ from the oracle's BVH::intersect);
    risk: the frame's risk points (cam / light / shadow_rays, _lib.wbvh_query), the oracle answering
    the rays the query built"""
    import dataclasses
    status, ids, t, u, v, stats, _, o, d = _lib.wbvh_query(tri, o, d, 12, 40, rays_out=True, **risk)
    assert stats["violations"] == 0
    base, _ = scenes.robot1080(width=8, height=8)
    sc = dataclasses.replace(base, tri=np.ascontiguousarray(tri, np.float32), tri_mat=np.zeros(len(tri), np.int32),
                             tri_uv=None)
    oi, ot, ou, ov, orr, _ = Oracle(sc, RenderSettings(bvh_max_depth=12, bvh_leaf_object_count=40)).bvh_query(o, d)
    cert = status != 2
    bad = cert & ((status == 1) != (orr != 0))
    hit = (status == 1) & (orr != 0)
    bad |= hit & ((ids != oi) | (bits(t) != bits(ot)) | (bits(u) != bits(ou)) | (bits(v) != bits(ov)))
    return float(cert.mean()), int(bad.sum())


@pytest.mark.parametrize("seed,sin_lo,sin_hi", [(99, 1e-7, 1e-3), (5, 1e-9, 1e-5), (17, 1e-5, 1e-1)])
def test_grazing_plane_certified_answers_match_oracle(seed, sin_lo, sin_hi):
    """The adversarial input of DESIGN.md 5.6: a tessellated plane and rays that meet it at
    grazing angles, where Moller-Trumbore reports hits far outside a triangle's box (r03 measured
    131 of 20,000 certified answers differing with the r02 query).  The query's child test bounds
    every point Moller-Trumbore can report (wbvh.hpp wbvh_closest), so every certified answer is
    the reference's; what it cannot bound it leaves uncertified (the exact octree traversal)."""
    tri, o, d = grazing_plane_case(seed=seed, sin_lo=sin_lo, sin_hi=sin_hi)
    cert, bad = _grazing_differences(tri, o, d)
    print(f"grazing plane seed {seed}: {cert:.4f} certified, {bad} certified answers differ")
    assert bad == 0


def grazing_sphere_case(seed=3, n_rays=20000):
    """Rays nearly tangent to a 1M-triangle-class tessellated sphere (a smaller UV sphere here):
    silhouette rays at 1e-8 .. 1e-2 of the radius from tangency, from inside and outside the
    scene box."""
    rng = np.random.default_rng(seed)
    sc, _ = scenes.bumpy70k(width=8, height=8)
    tri = sc.tri
    T = tri.reshape(-1, 3, 3).astype(np.float64)
    c = T.reshape(-1, 3).mean(0)
    # tangent planes of triangles with an area only: the UV sphere's zero-area pole triangles have
    # no normal (their rays would be NaN and check nothing)
    area = np.linalg.norm(np.cross(T[:, 1] - T[:, 0], T[:, 2] - T[:, 0]), axis=1)
    ok = np.flatnonzero(area > 1e-12)
    k = ok[rng.integers(0, len(ok), n_rays)]
    p = T[k].mean(1)
    n = np.cross(T[k, 1] - T[k, 0], T[k, 2] - T[k, 0])
    n /= np.linalg.norm(n, axis=1, keepdims=True)
    t1 = np.cross(n, rng.standard_normal((n_rays, 3)))
    t1 /= np.linalg.norm(t1, axis=1, keepdims=True)
    eps = np.exp(rng.uniform(np.log(1e-8), np.log(1e-2), n_rays))
    d = t1 + n * (eps * rng.choice([-1, 1], n_rays))[:, None]
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = p - d * rng.uniform(0.5, 4.0, n_rays)[:, None] + n * (eps * rng.uniform(0, 1, n_rays))[:, None]
    o, d = o.astype(np.float32), d.astype(np.float32)
    assert np.isfinite(o).all() and np.isfinite(d).all()
    return tri, o, d


def test_grazing_sphere_certified_answers_match_oracle():
    tri, o, d = grazing_sphere_case()
    cert, bad = _grazing_differences(tri, o, d)
    print(f"grazing sphere: {cert:.4f} certified, {bad} certified answers differ")
    assert bad == 0
    assert cert > 0.5


def test_grazing_sliver_soup_certified_answers_match_oracle():
    """Slivers and degenerate triangles (the soup scene) hit at grazing angles: rays in the plane
    of a random sliver, offset by 1e-7 .. 1e-3."""
    rng = np.random.default_rng(11)
    tri = _soup(rng)
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
    cert, bad = _grazing_differences(tri, o.astype(np.float32), d.astype(np.float32))
    print(f"grazing slivers: {cert:.4f} certified, {bad} certified answers differ")
    assert bad == 0


# ---- the frame's grazing-risk bits (wbvh.hpp wbvh_risk_tri) ----
# Rays from the camera position read the camera's bits, shadow rays the light's: a child whose bit
# is clear skips case (b).  Adversarial placements: the camera / light at 0 .. 1e-1 from the plane of
# a tessellated plane (every ray grazes it), on a tangent of the sphere.

def _plane_frame(seed, h, n_rays=20000):
    """The grazing plane of grazing_plane_case and a camera at height h above it, looking at points
    of the plane (ray sines ~ h / distance) and along it (a third of the rays just above / below)."""
    rng = np.random.default_rng(seed)
    R = _rotation(rng)
    off = rng.uniform(-5, 5, 3)
    tri = (_grid(400, 4.0).reshape(-1, 3, 3) @ R.T + off).reshape(-1, 9).astype(np.float32)
    C = np.array([rng.uniform(-5, 5), h, rng.uniform(-5, 5)])
    p = np.stack([rng.uniform(-4, 4, n_rays), np.zeros(n_rays), rng.uniform(-4, 4, n_rays)], 1)
    d = p - C
    k = n_rays // 3
    d[:k, 1] = rng.choice([-1, 1], k) * np.exp(rng.uniform(np.log(1e-9), np.log(1e-3), k)) * np.linalg.norm(d[:k], axis=1)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    cam = (C @ R.T + off).astype(np.float32)
    return tri, np.repeat(cam[None], n_rays, 0), (d @ R.T).astype(np.float32), cam


@pytest.mark.parametrize("h", [0.0, 1e-7, 1e-4, 1e-1])
def test_risk_bits_camera_grazing_plane(h):
    tri, o, d, cam = _plane_frame(23, h)
    cert, bad = _grazing_differences(tri, o, d, cam=cam)
    print(f"camera at {h} from the plane: {cert:.4f} certified, {bad} differ")
    assert bad == 0


def test_risk_bits_camera_sphere_silhouette():
    """Camera rays tangent to the bumpy sphere from one camera point (its silhouette)."""
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
    cert, bad = _grazing_differences(tri, o, d.astype(np.float32), cam=cam.astype(np.float32))
    print(f"sphere silhouette from the camera: {cert:.4f} certified, {bad} differ")
    assert bad == 0


@pytest.mark.parametrize("h", [0.0, 1e-6, 1e-3])
def test_risk_bits_light_grazing_plane(h):
    """Shadow rays from hit points on the plane towards a light at height h above it: every ray
    grazes the plane."""
    rng = np.random.default_rng(31)
    R = _rotation(rng)
    off = rng.uniform(-5, 5, 3)
    tri = (_grid(400, 4.0).reshape(-1, 3, 3) @ R.T + off).reshape(-1, 9).astype(np.float32)
    L = (np.array([rng.uniform(-6, 6), h, rng.uniform(-6, 6)]) @ R.T + off).astype(np.float32)
    n = 20000
    # hit points on the plane (normal up) and, for half the rays, on surfaces standing on it (normals
    # in the plane) at heights up to +-1e-3: their rays start next to the plane
    hp = np.zeros(n)
    hp[n // 2:] = rng.choice([-1, 1], n - n // 2) * np.exp(rng.uniform(np.log(1e-9), np.log(1e-3), n - n // 2))
    p = (np.stack([rng.uniform(-4, 4, n), hp, rng.uniform(-4, 4, n)], 1) @ R.T + off).astype(np.float32)
    az = rng.uniform(0, 2 * np.pi, n)
    nl = np.stack([np.cos(az), np.zeros(n), np.sin(az)], 1)
    nl[: n // 2] = [0.0, 1.0, 0.0]
    nrm = (nl @ R.T).astype(np.float32)
    cert, bad = _grazing_differences(tri, p, nrm, light=L, shadow_rays=True)
    print(f"light at {h} from the plane: {cert:.4f} certified, {bad} differ")
    assert bad == 0


def test_risk_bits_light_sphere_terminator():
    """Shadow rays from points on the bumpy sphere near its terminator (normal nearly perpendicular
    to the light) and a camera in the same frame."""
    rng = np.random.default_rng(8)
    sc, _ = scenes.bumpy70k(width=8, height=8)
    tri = sc.tri
    T = tri.reshape(-1, 3, 3).astype(np.float64)
    L = np.array([5.0, 0.5, 1.0], np.float32)
    nn = np.cross(T[:, 1] - T[:, 0], T[:, 2] - T[:, 0])
    nn /= np.maximum(np.linalg.norm(nn, axis=1, keepdims=True), 1e-30)
    c = T.mean(1)
    toL = L - c
    toL /= np.linalg.norm(toL, axis=1, keepdims=True)
    cosl = np.abs((nn * toL).sum(1))
    k = np.argsort(cosl)[:20000]   # the triangles closest to grazing the light
    uv = rng.uniform(0, 1, (len(k), 2))
    uv[uv.sum(1) > 1] = 1 - uv[uv.sum(1) > 1]
    p = T[k, 0] + (T[k, 1] - T[k, 0]) * uv[:, :1] + (T[k, 2] - T[k, 0]) * uv[:, 1:]
    cert, bad = _grazing_differences(tri, p.astype(np.float32), nn[k].astype(np.float32), light=L,
                                     cam=np.array([0.0, 0.0, 6.0], np.float32), shadow_rays=True)
    print(f"sphere terminator: {cert:.4f} certified, {bad} differ")
    assert bad == 0
