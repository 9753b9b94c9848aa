"""Host check of the wide BVH on shadow rays (rt_wbvh_query, no GPU): camera rays are traced
by the oracle, and from every hit p a ray o = p + n 1e-4 toward the light (n = the hit
triangle's unit normal, as is_shadowed builds it up to the shading normal) is queried through
the wide BVH and the oracle; certified answers must agree.  Prints the work per ray.
    python tools/shadow_probe.py [config] [row_stride]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np

from oracle.bindings import Oracle
from raytracercpp_amd import _lib, scenes
from tools.wbvh_probe import camera_rays


def shadow_rays(sc, st, stride):
    o, d = camera_rays(sc, st, stride)
    oi, ot, _, _, orr, _ = Oracle(sc, st).bvh_query(o, d)
    hit = (orr != 0) & (ot > 0.1)
    p = (o[hit] + d[hit] * ot[hit, None]).astype(np.float32)
    T = np.asarray(sc.tri, np.float32).reshape(-1, 3, 3)[oi[hit]]
    n = np.cross(T[:, 1] - T[:, 0], T[:, 2] - T[:, 0])
    n = (n / np.maximum(np.linalg.norm(n, axis=1, keepdims=True), 1e-30)).astype(np.float32)
    o2 = (p + n * np.float32(1e-4)).astype(np.float32)
    L = np.asarray(sc.light, np.float32)
    d2 = (L - p)
    d2 = (d2 / np.linalg.norm(d2, axis=1, keepdims=True)).astype(np.float32)
    return o2, d2


def check(sc, st, o, d):
    status, ids, t, u, v, stats, _ = _lib.wbvh_query(sc.tri, o, d, st.bvh_max_depth, st.bvh_leaf_object_count)
    oi, ot, ou, ov, orr, _ = Oracle(sc, st).bvh_query(o, d)
    cert = status != 2
    bad = cert & ((ids != oi) | (t.view(np.uint32) != ot.view(np.uint32)) | (u.view(np.uint32) != ou.view(np.uint32)) |
                  (v.view(np.uint32) != ov.view(np.uint32)) | ((status == 1) != (orr != 0)))
    return status, stats, int(bad.sum())


if __name__ == "__main__":
    name = sys.argv[1] if len(sys.argv) > 1 else "sphere1m"
    stride = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    sc, st = scenes.CONFIGS[name]()
    o, d = shadow_rays(sc, st, stride)
    status, stats, bad = check(sc, st, o, d)
    n = len(status)
    print(f"{name}: {n} shadow rays  certified miss {int((status == 0).sum())}  hit {int((status == 1).sum())}  "
          f"not certified {int((status == 2).sum())}  MISMATCHES {bad}")
    print(f"  per ray: {stats['node_visits'] / n:.2f} node visits, {stats['tri_tests'] / n:.2f} triangle tests")
    sys.exit(1 if bad else 0)
