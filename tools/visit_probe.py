"""Host probe of the wide query's work on a frame's rays (rt_wbvh_query_ex, no GPU): wide-node visits
per primary ray (the camera's risk words) and per shadow ray (the light's), their tail, and the
costliest 8x8 tiles' longest rays.  With RT_LIB_PATH pointing at a variant build (tools/variants.py
build ...) the same rays price a variant of the child test.
    python tools/visit_probe.py [config] [tile_row_stride]
Rays: every tile_row_stride-th row of 8x8 tiles (all 8 rows of each), so tile maxima are exact."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np

from raytracercpp_amd import _lib, scenes
from tools.wbvh_probe import camera_rays


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "sphere1m"
    tstride = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    sc, st = scenes.CONFIGS[name]()
    rw, rh = st.render_size()
    o, d = camera_rays(sc, st, 1)
    rows = np.concatenate([np.arange(ty * 8, min(ty * 8 + 8, rh)) for ty in range(0, (rh + 7) // 8, tstride)])
    sel = (rows[:, None] * rw + np.arange(rw)[None, :]).ravel()
    o, d = o[sel], d[sel]
    nodes = np.zeros(len(o), np.int32)
    st_, ids, t, u, v, stats, ms, oo, do = _lib.wbvh_query(sc.tri, o, d, st.bvh_max_depth, st.bvh_leaf_object_count,
                                                            cam=sc.cam_pos, rays_out=True, ray_nodes=nodes)
    assert stats["violations"] == 0, stats
    # shadow rays of the certified hits (is_shadowed: hit point, geometric normal)
    hit = st_ == 1
    T = sc.tri[ids[hit]].reshape(-1, 3, 3)
    p = (o[hit] + d[hit] * t[hit][:, None]).astype(np.float32)
    n = np.cross(T[:, 1] - T[:, 0], T[:, 2] - T[:, 0])
    n = (n / np.linalg.norm(n, axis=1, keepdims=True)).astype(np.float32)
    lit = ((sc.light[None] - p) * n).sum(1) > 0
    snodes = np.zeros(int(lit.sum()), np.int32)
    _lib.wbvh_query(sc.tri, p[lit], n[lit], st.bvh_max_depth, st.bvh_leaf_object_count, cam=sc.cam_pos,
                    light=sc.light, shadow_rays=True, ray_nodes=snodes)
    q = np.percentile(nodes, [50, 90, 99, 99.9, 100])
    print(f"{name}: {len(o)} primary rays ({len(rows)} rows): {nodes.mean():.3f} node visits/ray; "
          f"p50/p90/p99/p99.9/max {q[0]:.0f}/{q[1]:.0f}/{q[2]:.0f}/{q[3]:.0f}/{q[4]:.0f}; "
          f"not certified {int((st_ == 2).sum())}")
    qs = np.percentile(snodes, [50, 90, 99, 99.9, 100]) if len(snodes) else [0] * 5
    print(f"  {len(snodes)} shadow rays: {snodes.mean() if len(snodes) else 0:.3f} node visits/ray; "
          f"p50/p90/p99/p99.9/max {qs[0]:.0f}/{qs[1]:.0f}/{qs[2]:.0f}/{qs[3]:.0f}/{qs[4]:.0f}")
    # per tile: the longest primary ray (the wave's iterations are at least that)
    tx = rw // 8
    tile = (np.repeat(np.arange(len(rows)) // 8, rw) * tx + np.tile(np.arange(rw) // 8, len(rows)))
    tmax = np.zeros(tile.max() + 1, np.int64)
    np.maximum.at(tmax, tile, nodes)
    top = np.sort(tmax)[::-1]
    print(f"  tiles: {len(tmax)}; longest-ray visits, top 10: {top[:10].tolist()}; tiles over 100: {int((tmax > 100).sum())},"
          f" over 200: {int((tmax > 200).sum())}")
    print(f"  hit rays {nodes[hit].mean():.3f} visits/ray, misses {nodes[~hit].mean():.3f}; mean over tiles of the "
          f"longest ray {tmax.mean():.3f} (the waves' iterations: {tmax.mean() / max(nodes.mean(), 1e-9):.2f}x the mean ray)")


if __name__ == "__main__":
    main()
