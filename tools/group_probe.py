"""How long one heavy tile's rays take through the wide query with G lanes per ray (rt_wide_query,
RT_WIDE_QUERY_GROUP=G: wbvh_closest<.., G>), and whether the answers are the same for every G.
GPU box:   python tools/group_probe.py [config] [tiles]
For the `tiles` costliest 8x8 tiles of a C4-style frame (rt_tile_costs), their 64 camera rays: the
time of one rt_wide_query call (best of 15, host clock around the call: launch + copies included, so
compare the differences) for the costliest tile alone and for all of them, then the shadow rays of
their hits (kind 2)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np

from raytracercpp_amd import scenes
from tools.wbvh_probe import camera_rays


def timed(r, o, d, kind, reps=15):
    best = 1e30
    out = None
    for _ in range(reps):
        t0 = time.perf_counter()
        out = r.wide_query(o, d, kind)
        best = min(best, time.perf_counter() - t0)
    return best * 1e3, out


def main():
    from raytracercpp_amd.renderer import Renderer
    name = sys.argv[1] if len(sys.argv) > 1 else "sphere1m"
    ntop = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    sc, st = scenes.CONFIGS[name]()
    r = Renderer(0)
    r.load_scene(sc, st)
    r.ray_trace()
    r.finish_accel()
    r.ray_trace()
    r.ray_trace()
    c = r.tile_costs()
    rw, rh = st.render_size()
    top = np.argsort(c.ravel())[::-1][:ntop]
    o_all, d_all = camera_rays(sc, st, 1)
    sel = []
    for i in top:
        ty, tx = divmod(int(i), c.shape[1])
        ys, xs = np.meshgrid(np.arange(ty * 8, ty * 8 + 8), np.arange(tx * 8, tx * 8 + 8), indexing="ij")
        sel.append((ys * rw + xs).ravel())
    sel = np.concatenate(sel)
    o, d = o_all[sel], d_all[sel]
    print(f"{name}: top {ntop} tiles, costs {c.ravel()[top[:4]].tolist()} ...", flush=True)
    ref = None
    for G in (1, 2, 4, 8):
        os.environ["RT_WIDE_QUERY_GROUP"] = str(G)
        t1, _ = timed(r, o[:64], d[:64], 1)
        tn, out = timed(r, o, d, 1)
        hit = out["status"] == 1
        T = sc.tri[out["id"][hit]].reshape(-1, 3, 3) if hit.any() else np.zeros((0, 3, 3), np.float32)
        p = (o[hit] + d[hit] * out["t"][hit][:, None]).astype(np.float32)
        n = np.cross(T[:, 1] - T[:, 0], T[:, 2] - T[:, 0])
        n = (n / np.maximum(np.linalg.norm(n, axis=1, keepdims=True), 1e-30)).astype(np.float32)
        ts, sh = timed(r, p, n, 2) if len(p) else (0.0, None)
        key = (out["status"].copy(), out["id"].copy(), out["t"].view(np.uint32).copy(),
               None if sh is None else sh["shadowed"].copy())
        same = ref is None or all(np.array_equal(a, b) for a, b in zip(key, ref) if a is not None)
        ref = ref or key
        print(f"  G={G}: costliest tile {t1:.3f} ms, {len(o)} rays {tn:.3f} ms, {len(p)} shadow rays {ts:.3f} ms; "
              f"certified {int((out['status'] <= 1).sum())}/{len(o)}; same answers as G=1: {same}", flush=True)


if __name__ == "__main__":
    main()
