"""Where the C4 frame's time goes, tile by tile (diagnostic build -DRT_TILE_TIME=1: the
kernel writes each pixel's trace time, in wall-clock ticks, into the hit_t buffer).
    python tools/variants.py build tt="-DRT_TILE_TIME=1"                 (here)
    RT_LIB_PATH=_variants/librt_tt.so python tools/tile_times.py      (GPU box)"""
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
r.request_aux(hit=True)
r.ray_trace()
r.ray_trace()
g = r.get_internal(argb=False, hit=True)
hid = g["hit_id"].reshape(st.render_size()[1], st.render_size()[0])
rw, rh = st.render_size()
t = g["hit_t"].reshape(rh, rw).astype(np.float64) / 100.0   # wall clock at 100 MHz -> us
tiles = t[: rh // 8 * 8, : rw // 8 * 8].reshape(rh // 8, 8, rw // 8, 8).max(axis=(1, 3))
flat = np.sort(tiles.ravel())[::-1]
print("kernel ms", r.stats()["kernel_ms"], " tiles", flat.size)
print("tile time us: max %.1f  p99.9 %.1f  p99 %.1f  p90 %.1f  median %.1f  mean %.1f" % (
    flat[0], flat[int(flat.size * 0.001)], flat[int(flat.size * 0.01)], flat[int(flat.size * 0.1)],
    np.median(flat), flat.mean()))
print("sum of tile times / 5120 waves: %.3f ms" % (flat.sum() / 1e3 / (256 * 4 * 5)))
ty, tx = np.unravel_index(np.argsort(tiles.ravel())[::-1][:12], tiles.shape)
for a, b in zip(ty, tx):
    print(f"  tile row {a:4d} col {b:4d}  {tiles[a, b]:9.1f} us  (pixel y {a * 8}, x {b * 8})")
np.save(os.path.join(ROOT, "gpurun_out", "tile_times.npy"), tiles.astype(np.float32))
a, b = ty[0], tx[0]
print("heaviest tile, per-pixel us (hit id < 0: miss):")
for yy in range(8):
    print("  " + " ".join(f"{t[a * 8 + yy, b * 8 + xx]:7.0f}{'*' if hid[a * 8 + yy, b * 8 + xx] >= 0 else ' '}" for xx in range(8)))
