"""Per-tile cost of a frame (rt_tile_costs): where the C4 kernel's critical path sits.

GPU box:   python tools/tile_costs.py gpu [config] [frames] [out.npy]
    renders the config `frames` times (trace_frame: the heavy-first order of each launch uses the
    previous one's costs) and prints the tile-cost distribution of the last launch: quantiles,
    the top tiles (tx, ty, cycles, multiple of the median) and how much of the kernel's time the
    costliest tile alone spans; saves the (tiles_y, tiles_x) array.
Container: python tools/tile_costs.py host [config] costs.npy [top]
    for the `top` costliest tiles, the wide-node visits of each of the tile's 64 primary rays and
    their shadow rays on the host (rt_wbvh_query_ex, ray_nodes): is the tile long because one ray
    walks far, or because many do?
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np

from raytracercpp_amd import scenes


def gpu(name, frames, out):
    import torch
    from raytracercpp_amd.renderer import Renderer
    sc, st = scenes.CONFIGS[name]()
    r = Renderer(0)
    r.load_scene(sc, st)
    r.ray_trace()
    r.finish_accel()
    for _ in range(frames):
        r.ray_trace()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r.ray_trace()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3
    c = r.tile_costs().astype(np.float64)
    np.save(out, c.astype(np.uint32))
    v = np.sort(c[c > 0].ravel())
    med = float(np.median(v))
    print(f"{name}: tiles {c.shape[1]} x {c.shape[0]} ({v.size} on the image), last frame {ms:.3f} ms wall")
    qs = [0.5, 0.9, 0.99, 0.999, 0.9999, 1.0]
    print("  cycles per tile: " + "  ".join(f"q{q:g} {v[min(v.size - 1, int(q * v.size))]:.0f}" for q in qs))
    print(f"  sum {v.sum():.4g} cycles; the costliest tile = {v[-1] / med:.1f} x median, "
          f"{v[-1] / (v.sum() / 3072):.2f} x the mean cycles per wave (3072 waves)")
    mean = v.mean()
    thr = max(4 * mean, v[-1] / 8)
    print(f"  heavy list threshold {thr:.0f}: {(v >= thr).sum()} tiles, {v[v >= thr].sum() / v.sum() * 100:.1f}% of the cycles")
    idx = np.argsort(c.ravel())[::-1][:30]
    print("  top tiles (tx, ty, cycles, x median):")
    for i in idx:
        ty, tx = divmod(int(i), c.shape[1])
        print(f"    {tx:4d} {ty:4d} {c.ravel()[i]:10.0f} {c.ravel()[i] / med:7.1f}")


def host(name, path, top):
    from raytracercpp_amd import _lib
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from wbvh_probe import camera_rays
    sc, st = scenes.CONFIGS[name]()
    c = np.load(path).astype(np.float64)
    med = float(np.median(c[c > 0]))
    rw, rh = st.render_size()
    o_all, d_all = camera_rays(sc, st, 1)
    cam = np.asarray(sc.cam_pos, np.float32)
    light = np.asarray(sc.light, np.float32)
    idx = np.argsort(c.ravel())[::-1][:top]
    print(f"{name}: per tile: cycles/median | primary node visits max, mean | shadow rays, visits max, mean")
    for i in list(idx) + list(np.argsort(np.abs(c.ravel() - med))[:3]):
        ty, tx = divmod(int(i), c.shape[1])
        ys, xs = np.mgrid[ty * 8:ty * 8 + 8, tx * 8:tx * 8 + 8]
        ok = (ys < rh) & (xs < rw)
        pix = (ys[ok] * rw + xs[ok]).ravel()
        o, d = o_all[pix], d_all[pix]
        nodes = np.zeros(len(pix), np.int32)
        st_, ids, t, u, v, _, _ = _lib.wbvh_query(sc.tri, o, d, st.bvh_max_depth, st.bvh_leaf_object_count,
                                                  cam=cam, light=light, ray_nodes=nodes)
        hit = st_ == 1
        p = (o + d * t[:, None])[hit].astype(np.float32)
        msg = f"  tile ({tx:3d},{ty:3d}) {c.ravel()[i] / med:6.1f} | {nodes.max():5d} {nodes.mean():7.1f}"
        if hit.any():
            # the shadow ray's origin/normal as is_shadowed takes them: hit point and the geometric normal
            tri = sc.tri.reshape(-1, 9)[ids[hit]]
            n = np.cross(tri[:, 3:6] - tri[:, 0:3], tri[:, 6:9] - tri[:, 0:3])
            n = n / np.linalg.norm(n, axis=1, keepdims=True)
            n = np.where((n * d[hit]).sum(1, keepdims=True) > 0, -n, n).astype(np.float32)
            sn = np.zeros(len(p), np.int32)
            _lib.wbvh_query(sc.tri, p, n, st.bvh_max_depth, st.bvh_leaf_object_count, cam=cam, light=light,
                            shadow_rays=True, ray_nodes=sn)
            msg += f" | {len(p):3d} {sn.max():5d} {sn.mean():7.1f}"
        print(msg, flush=True)


if __name__ == "__main__":
    mode = sys.argv[1] if len(sys.argv) > 1 else "gpu"
    name = sys.argv[2] if len(sys.argv) > 2 else "sphere1m"
    if mode == "gpu":
        gpu(name, int(sys.argv[3]) if len(sys.argv) > 3 else 5,
            sys.argv[4] if len(sys.argv) > 4 else os.path.join(ROOT, "gpurun_out", "tile_costs.npy"))
    else:
        host(name, sys.argv[3], int(sys.argv[4]) if len(sys.argv) > 4 else 10)
