"""Origin cones (ocone.hpp): the reflection queries skip case (b) of the wide query when
no triangle nearly parallel to the ray can report a hit.  CPU tests (no GPU):
  * soundness by brute force (rt_ocone_check): for every ray the grid lets skip case (b), every triangle
    with |cos(N, d)| < the query's split (or degenerate) goes through Moller-Trumbore
    (triangle.cpp:25-91) and must report nothing -- on spheres, a bumpy sphere, a sphere on a floor,
    fur, a cube and a triangle soup with slivers and degenerate records, with reflection-like rays,
    rays grazing the triangles near their origin and random rays;
  * the host wide query answers the same with and without the cones, and visits fewer nodes with them."""
import numpy as np
import pytest

from raytracercpp_amd import _lib, scenes


def _sphere(nu, nv, bump=0.0, scale=1.5):
    # scaled and moved in float32 as the scenes' object transform does: the pole quads' coincident vertices
    # (sin(pi) ~ 1e-16 apart in object space) become equal, so their records have a zero normal (never hit)
    tri, _ = scenes.uv_sphere_triangles(nu, nv, bump=bump, texcoords=False)
    off = np.array([0.125, 0.25, -0.5] * 3, np.float32)
    return (tri.reshape(-1, 9) * np.float32(scale) + off).astype(np.float32)


def _floor(n=20, y=-1.5, half=3.0):
    xs = np.linspace(-half, half, n + 1, dtype=np.float64)
    out = []
    for i in range(n):
        for j in range(n):
            a = (xs[i], y, xs[j]); b = (xs[i], y, xs[j + 1]); c = (xs[i + 1], y, xs[j + 1]); d = (xs[i + 1], y, xs[j])
            out += [a + b + c, a + c + d]   # facing +y
    return np.array(out, np.float32)


def _soup(n=600, seed=5, bad=True):
    rng = np.random.default_rng(seed)
    c = rng.uniform(-1, 1, (n, 1, 3))
    t = c + rng.normal(0, 0.08, (n, 3, 3))
    if bad:
        t[: n // 6, 2] = t[: n // 6, 0] + 1e-4 * (t[: n // 6, 1] - t[: n // 6, 0])   # slivers
        t[n // 6: n // 5, 2] = t[n // 6: n // 5, 1]                                  # degenerate (two equal vertices)
    return t.reshape(-1, 9).astype(np.float32)


def _cube():
    tri, _, _, _ = _lib.load_obj(scenes.data_path("cube.obj"), np.eye(4, dtype=np.float32))
    return np.asarray(tri, np.float32).reshape(-1, 9)


MESHES = {
    "sphere": lambda: _sphere(120, 60),
    "bumpy": lambda: _sphere(100, 50, bump=0.08, scale=1.2),
    "sphere_floor": lambda: np.concatenate([_sphere(80, 40), _floor()]),
    "fur": lambda: scenes.hair_triangles(nstrands=300, nseg=6).reshape(-1, 9),
    "cube": _cube,
    "soup": _soup,
    "soup_clean": lambda: _soup(bad=False),
}


def _rays(tri9, n, seed):
    """Reflection-like rays (hit point + 0.01 n, outgoing hemisphere), rays from points of a triangle's
    plane grazing it or its neighbours, random rays through the scene box, and rays from the reflection-like
    origins back into the surface."""
    rng = np.random.default_rng(seed)
    T = tri9.reshape(-1, 3, 3).astype(np.float64)
    nrm = np.cross(T[:, 1] - T[:, 0], T[:, 2] - T[:, 0])
    ln = np.linalg.norm(nrm, axis=1)
    ok = ln > 1e-12
    idx = rng.choice(np.flatnonzero(ok), n)
    w = rng.dirichlet([1, 1, 1], n)
    p = (T[idx] * w[:, :, None]).sum(1)
    nn = nrm[idx] / ln[idx][:, None]
    # 1. reflection-like
    d1 = rng.normal(size=(n, 3))
    d1 /= np.linalg.norm(d1, axis=1, keepdims=True)
    d1 = np.where(((d1 * nn).sum(1) < 0)[:, None], -d1, d1)
    o1 = p + 0.01 * nn
    # 2. grazing: from a point of the plane (offset by up to 1e-4 either side) towards a point of a nearby
    #    triangle, tilted by up to ~1e-3 out of the plane
    j = np.clip(idx + rng.integers(-3, 4, n), 0, len(T) - 1)
    q = (T[j] * rng.dirichlet([1, 1, 1], n)[:, :, None]).sum(1)
    o2 = p + nn * rng.uniform(-1e-4, 1e-4, (n, 1)) - (q - p) * rng.uniform(0.2, 2.0, (n, 1))
    d2 = q - o2
    d2 /= np.linalg.norm(d2, axis=1, keepdims=True) + 1e-30
    d2 = d2 + nn * rng.uniform(-1e-3, 1e-3, (n, 1))
    # 3. random
    lo, hi = tri9.reshape(-1, 3).min(0), tri9.reshape(-1, 3).max(0)
    o3 = rng.uniform(lo - 0.05, hi + 0.05, (n, 3))
    d3 = rng.normal(size=(n, 3))
    # 4. into the surface from above it (a rough sample turning back: the front route)
    d4 = -d1 + nn * rng.uniform(-0.3, 0.3, (n, 1))
    o = np.concatenate([o1, o2, o3, o1]).astype(np.float32)
    d = np.concatenate([d1, d2, d3, d4]).astype(np.float32)
    keep = np.isfinite(o).all(1) & np.isfinite(d).all(1) & (np.abs(d).sum(1) > 0)
    return o[keep], d[keep]


@pytest.mark.parametrize("name", sorted(MESHES))
def test_origin_cones_sound_by_brute_force(name):
    tri9 = MESHES[name]()
    o, d = _rays(tri9, 1500, seed=len(name))
    skip, st = _lib.ocone_check(tri9, o, d, ocone_dim=48)
    assert st["violations"] == 0, st
    assert st["grazing_tests"] > 0 or st["skipping"] == 0, st
    # the reflection-like third of the rays mostly skips case (b) on smooth surfaces (a sliver or degenerate
    # record with a non-zero normal is at risk from everywhere: the soup's cells have no bound)
    if name in ("sphere", "sphere_floor", "cube"):
        assert skip[: len(skip) // 3].mean() > 0.3, (name, skip[: len(skip) // 3].mean(), st)
    if name == "soup":
        assert st["skipping"] == 0, st
    print(name, st, "skip fraction", skip.mean())


def test_brute_force_check_catches_a_wrong_grid():
    """The checker has teeth: a grid claiming no triangle is at risk anywhere (every ray skips case (b))
    lets grazing rays through, and Moller-Trumbore reports hits from nearly parallel triangles."""
    tri9 = MESHES["sphere"]()
    o, d = _rays(tri9, 1500, seed=6)
    _, st, cells = _lib.ocone_check(tri9, o, d, ocone_dim=32, want_cells=True)
    assert st["violations"] == 0
    lo = tri9.reshape(-1, 3).min(0) - 0.5
    wrong = np.zeros((8, 2), np.uint32)
    wrong[:, 1] = 0x7FFE << 16   # OC_EMPTY
    span = float((tri9.reshape(-1, 3).max(0) - lo).max() + 1.0)
    _, bad = _lib.ocone_check(tri9, o, d, ocone_dim=32, grid=(wrong, np.array([2, 2, 2], np.int32),
                                                                 np.array([*lo, 2.0 / span], np.float32)))
    assert bad["skipping"] > 0.9 * len(o) and bad["violations"] > 0, bad


def test_origin_cones_same_answers_fewer_visits():
    tri9 = _sphere(200, 100)
    o, d = _rays(tri9, 3000, seed=11)
    o, d = o[:3000], d[:3000]   # the reflection-like rays
    n0 = np.zeros(len(o), np.int32)
    n1 = np.zeros(len(o), np.int32)
    oc = np.zeros(5, np.int64)
    a = _lib.wbvh_query(tri9, o, d, 12, 40, ray_nodes=n0)
    b = _lib.wbvh_query(tri9, o, d, 12, 40, ray_nodes=n1, ocone_dim=64, oc_stats=oc)
    for x, y in zip(a[:5], b[:5]):
        assert np.array_equal(x, y)
    assert a[5]["violations"] == 0 and b[5]["violations"] == 0
    assert oc[3] > len(o) // 2, oc            # most skip case (b)
    assert n1.sum() < 0.7 * n0.sum(), (n0.mean(), n1.mean())
    print(f"visits per ray {n0.mean():.2f} -> {n1.mean():.2f}; rays skipping (b) {oc[3]} of {len(o)}; cells {oc[0]}")


def _camera_rays(tri9, n, seed):
    """A camera off the scene's box; rays towards random points of random triangles, towards points of the
    triangles most nearly edge-on to the camera (the silhouette), and in random directions."""
    rng = np.random.default_rng(seed)
    T = tri9.reshape(-1, 3, 3).astype(np.float64)
    lo, hi = T.reshape(-1, 3).min(0), T.reshape(-1, 3).max(0)
    cam = (lo + hi) / 2 + np.array([0.3, 0.45, 1.0]) * 1.6 * (hi - lo).max()
    nrm = np.cross(T[:, 1] - T[:, 0], T[:, 2] - T[:, 0])
    ln = np.linalg.norm(nrm, axis=1)
    ok = np.flatnonzero(ln > 1e-12)
    ctr = T.mean(1)
    w = ctr - cam
    edge = np.abs((nrm * w).sum(1)) / (ln * np.linalg.norm(w, axis=1) + 1e-30)
    sil = ok[np.argsort(edge[ok])[: max(50, len(ok) // 50)]]
    pick = np.concatenate([rng.choice(ok, n), rng.choice(sil, n)])
    p = (T[pick] * rng.dirichlet([1, 1, 1], len(pick))[:, :, None]).sum(1)
    d = np.concatenate([p - cam, rng.normal(size=(n // 2, 3))])
    return cam.astype(np.float32), d.astype(np.float32)


@pytest.mark.parametrize("name", ["sphere", "bumpy", "sphere_floor", "cube", "soup_clean"])
def test_risk_cap_sound_by_brute_force(name):
    """The camera's risk cap (wbvh.hpp risk_cap_skip): for every camera ray it lets skip case (b), no triangle
    nearly parallel to the ray (or degenerate) reports a hit in Moller-Trumbore; on the smooth sphere most rays
    at the object skip."""
    tri9 = MESHES[name]()
    cam, d = _camera_rays(tri9, 1500, seed=len(name) + 1)
    skip, st = _lib.risk_cap_check(tri9, cam, d)
    assert st["violations"] == 0, st
    if name == "sphere":
        assert skip[:1500].mean() > 0.5 and st["grazing_tests"] > 0, (skip[:1500].mean(), st)
    print(name, st, "skip fraction", skip.mean())


def test_risk_cap_check_catches_a_wrong_cap():
    """The checker has teeth: a cap of 1 (every at-risk normal claimed parallel to the centre's direction)
    lets the silhouette's grazing rays skip, and Moller-Trumbore reports hits from the nearly parallel
    triangles they graze."""
    tri9 = MESHES["sphere"]()
    cam, d = _camera_rays(tri9, 1500, seed=3)
    _, good = _lib.risk_cap_check(tri9, cam, d)
    _, bad = _lib.risk_cap_check(tri9, cam, d, cap_override=1.0)
    assert good["violations"] == 0 and bad["violations"] > 0, (good, bad)
