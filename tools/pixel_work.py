"""Per-pixel traversal work of the C4 frame (diagnostic build -DRT_COUNT=2: hit_t = the pixel's
k-DOP tests, argb = its Moller-Trumbore tests, primary + shadow queries as executed).
    python tools/variants.py build pc="-DRT_COUNT=2"               (here)
    RT_LIB_PATH=_variants/librt_pc.so python tools/pixel_work.py   (GPU box)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np

from raytracercpp_amd import scenes
from raytracercpp_amd.renderer import Renderer

# the deferred pass writes real hit t / colours, not the diagnostic values: keep every
# pixel in the main pass (ray_trace_defer_kernel has no RT_COUNT==2 / RT_TILE_TIME writes)
os.environ["RT_DEFER_BUDGET"] = "0"
sc, st = scenes.sphere1m()
r = Renderer(0)
r.load_scene(sc, st)
r.request_aux(hit=True, shadow=True)
r.ray_trace()
g = r.get_internal(argb=True, hit=True, shadow=True)
rw, rh = st.render_size()
vol = g["hit_t"].reshape(rh, rw)
tri = g["argb"].reshape(rh, rw).view(np.uint32).astype(np.float64)
hit = g["hit_id"].reshape(rh, rw) >= 0
for name, a in (("k-DOP", vol), ("MT", tri)):
    f = np.sort(a.ravel())[::-1]
    print(f"{name}: max {f[0]:.0f}  p99.99 {f[int(f.size * 1e-4)]:.0f}  p99.9 {f[int(f.size * 1e-3)]:.0f}  "
          f"p99 {f[int(f.size * 0.01)]:.0f}  mean {f.mean():.1f}  mean(hit) {a[hit].mean():.1f}  mean(miss) {a[~hit].mean():.1f}")
for (py, px) in ((992, 1176), (995, 1180), (912, 1192), (430, 1560)):
    blk = slice(py, py + 8), slice(px, px + 8)
    print(f"tile at y {py} x {px}: k-DOP max {vol[blk].max():.0f}  MT max {tri[blk].max():.0f}  hits {int(hit[blk].sum())}/64")
for (py, px) in ((440, 1528), (992, 1176)):
    blk = slice(py, py + 8), slice(px, px + 8)
    print(f"tile y {py} x {px} k-DOP per pixel:\n{vol[blk].astype(np.int64)}\nMT per pixel:\n{tri[blk].astype(np.int64)}")
# heaviest tiles by the largest per-pixel node work, and the tiles named on the command line
tv = vol[: rh // 8 * 8, : rw // 8 * 8].reshape(rh // 8, 8, rw // 8, 8).max(axis=(1, 3))
tt = tri[: rh // 8 * 8, : rw // 8 * 8].reshape(rh // 8, 8, rw // 8, 8).max(axis=(1, 3))
ty, tx = np.unravel_index(np.argsort(tv.ravel())[::-1][:8], tv.shape)
for a, b in zip(ty, tx):
    print(f"  heavy tile row {a} col {b}: max node/k-DOP {tv[a, b]:.0f}  max MT {tt[a, b]:.0f}")
for arg in sys.argv[1:]:
    a, b = map(int, arg.split(","))
    blk = slice(a * 8, a * 8 + 8), slice(b * 8, b * 8 + 8)
    print(f"tile row {a} col {b} node/k-DOP per pixel:\n{vol[blk].astype(np.int64)}\nMT per pixel:\n{tri[blk].astype(np.int64)}")
