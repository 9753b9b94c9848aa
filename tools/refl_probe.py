"""Host probe of C5-like reflection rays (rt_wbvh_query_ex, no GPU): wide-node visits per reflection ray
and how they split by the ray's angle to the surface normal at its origin.  The rays: certified camera
hits of sphere1m_refl (every `stride`-th internal row), origin p + 0.01 n (make_frame), directions the
perfect reflection tilted at random by up to `spread` radians (a stand-in for the rough samples).
    python tools/refl_probe.py make <rays.npz> [stride] [samples] [spread]
    python tools/refl_probe.py run <rays.npz> <visits.npy>       (RT_LIB_PATH: the build to price)
    python tools/refl_probe.py report <rays.npz> <visits.npy> [<visits2.npy> ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np

from raytracercpp_amd import _lib, scenes
from tools.wbvh_probe import camera_rays


def make(path, stride=32, samples=4, spread=0.3):
    sc, st = scenes.sphere1m_refl()
    o, d = camera_rays(sc, st, stride)
    stt, ids, t, u, v, stats, ms = _lib.wbvh_query(sc.tri, o, d, st.bvh_max_depth, st.bvh_leaf_object_count,
                                                   cam=sc.cam_pos)
    hit = stt == 1
    T = sc.tri[ids[hit]].reshape(-1, 3, 3).astype(np.float64)
    p = o[hit] + d[hit] * t[hit][:, None]
    n = np.cross(T[:, 1] - T[:, 0], T[:, 2] - T[:, 0])
    n /= np.linalg.norm(n, axis=1, keepdims=True)
    dd = d[hit].astype(np.float64)
    r = dd - 2 * (dd * n).sum(1, keepdims=True) * n
    rng = np.random.default_rng(7)
    ro, rd, cosn = [], [], []
    for _ in range(samples):
        x = r + spread * rng.standard_normal(r.shape)
        x /= np.linalg.norm(x, axis=1, keepdims=True)
        x = np.where(((x * n).sum(1) > 0)[:, None], x, r)   # into the outer hemisphere
        ro.append(p + 0.01 * n)
        rd.append(x)
        cosn.append((x * n).sum(1))
    np.savez(path, o=np.concatenate(ro).astype(np.float32), d=np.concatenate(rd).astype(np.float32),
             cosn=np.concatenate(cosn))
    print(f"{len(np.concatenate(cosn))} reflection rays from {int(hit.sum())} camera hits")


def run(path, out):
    sc, st = scenes.sphere1m_refl()
    z = np.load(path)
    nodes = np.zeros(len(z["o"]), np.int32)
    oc = np.zeros(5, np.int64)
    dim = int(os.environ.get("OCONE_DIM", "0"))
    stt, ids, t, u, v, stats, ms = _lib.wbvh_query(sc.tri, z["o"], z["d"], st.bvh_max_depth, st.bvh_leaf_object_count,
                                                   cam=sc.cam_pos, ray_nodes=nodes, ocone_dim=dim, oc_stats=oc)
    np.save(out, nodes)
    np.save(out.replace(".npy", "_ans.npy"), np.stack([stt, ids, t.view(np.int32)], 1))
    print(f"{os.environ.get('RT_LIB_PATH', 'default')} ocone {dim}: {nodes.mean():.3f} visits/ray, hits "
          f"{int((stt == 1).sum())}, uncertified {int((stt == 2).sum())}, violations {stats['violations']}; cells "
          f"{oc[0]} (empty {oc[1]}, no bound {oc[2]}), rays skipping (b) {oc[3]}, grid {oc[4]} ms")


def report(path, outs):
    z = np.load(path)
    ang = np.degrees(np.arccos(np.clip(z["cosn"], -1, 1)))
    vs = [np.load(f) for f in outs]
    edges = [0, 30, 45, 60, 70, 75, 80, 85, 90.01]
    print("angle to n    rays   " + "  ".join(os.path.basename(f) for f in outs))
    for a, b in zip(edges[:-1], edges[1:]):
        m = (ang >= a) & (ang < b)
        print(f"{a:4.0f}-{b:3.0f}  {int(m.sum()):8d}  " + "  ".join(f"{v[m].mean() if m.any() else 0:9.3f}" for v in vs))
    print(f"all        {len(ang):8d}  " + "  ".join(f"{v.mean():9.3f}" for v in vs))


if __name__ == "__main__":
    cmd = sys.argv[1]
    if cmd == "make":
        make(sys.argv[2], *[float(x) if "." in x else int(x) for x in sys.argv[3:]])
    elif cmd == "run":
        run(sys.argv[2], sys.argv[3])
    else:
        report(sys.argv[2], sys.argv[3:])
