"""Host check of the wide-BVH certified closest hit (rt_wbvh_query, no GPU) against the
oracle's BVH::intersect on camera rays of a scene: agreement of every certified query,
fraction not certified, work per ray and build times.
    python tools/wbvh_probe.py [config] [row_stride]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np

from oracle.bindings import Oracle
from raytracercpp_amd import _lib, scenes


def camera_rays(sc, st, stride):
    rw, rh = st.render_size()
    ys = np.arange(0, rh, stride, dtype=np.float32)
    xs = np.arange(rw, dtype=np.float32)
    X, Y = np.meshgrid(xs, ys)
    xw = ((X + np.float32(0.5)) / np.float32(rw) * np.float32(2) - np.float32(1)).astype(np.float32)
    yw = ((Y + np.float32(0.5)) / np.float32(rh) * np.float32(2) - np.float32(1)).astype(np.float32)
    P = np.stack([xw.ravel(), yw.ravel(), -np.ones(xw.size, np.float32), np.ones(xw.size, np.float32)], 1)
    vs = P @ np.asarray(sc.proj_inv, np.float32).reshape(4, 4).T
    vs = vs[:, :3] / vs[:, 3:4]
    ws = np.concatenate([vs, np.ones((vs.shape[0], 1), np.float32)], 1) @ np.asarray(sc.cam_to_world, np.float32).reshape(4, 4).T
    d = ws[:, :3] - np.asarray(sc.cam_pos, np.float32)
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    o = np.broadcast_to(np.asarray(sc.cam_pos, np.float32), d.shape).copy()
    return o, d


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "sphere1m"
    stride = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    sc, st = scenes.CONFIGS[name]()
    o, d = camera_rays(sc, st, stride)
    t0 = time.time()
    status, ids, t, u, v, stats, ms = _lib.wbvh_query(sc.tri, o, d, st.bvh_max_depth, st.bvh_leaf_object_count)
    t1 = time.time()
    oi, ot, ou, ov, orr, _ = Oracle(sc, st).bvh_query(o, d)
    t2 = time.time()
    n = len(status)
    cert = status != 2
    bad = cert & ((ids != oi) | (t.view(np.uint32) != ot.view(np.uint32)) | (u.view(np.uint32) != ou.view(np.uint32)) |
                  (v.view(np.uint32) != ov.view(np.uint32)) | ((status == 1) != (orr != 0)))
    print(f"{name}: {n} rays  certified miss {int((status == 0).sum())}  hit {int((status == 1).sum())}  "
          f"not certified {int((status == 2).sum())} ({(status == 2).mean() * 100:.3f}%)  MISMATCHES {int(bad.sum())}")
    print(f"  wide BVH {stats}  octree build {ms[0]:.1f} ms  wide build {ms[1]:.1f} ms")
    print(f"  per ray: {stats['node_visits'] / n:.2f} node visits, {stats['tri_tests'] / n:.2f} triangle tests;"
          f" host query {t1 - t0:.2f} s, oracle {t2 - t1:.2f} s")
    return int(bad.sum())


if __name__ == "__main__":
    sys.exit(1 if main() else 0)
