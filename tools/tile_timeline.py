"""Timeline of the C4 frame's tiles (diagnostic build -DRT_TILE_TIME=1: hit_t = a pixel's
trace ticks, rgba.w = its start tick, 100 MHz wall clock): when the heaviest tiles start
and end, how many tiles are in flight over time, and what the last microseconds run.
    python tools/variants.py build tt="-DRT_TILE_TIME=1"                (here)
    RT_LIB_PATH=_variants/librt_tt.so python tools/tile_timeline.py  (GPU box)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np

from raytracercpp_amd import scenes
from raytracercpp_amd.renderer import Renderer

sc, st = scenes.sphere1m()
r = Renderer(0)
r.load_scene(sc, st)
r.request_aux(rgba=True, hit=True)
for _ in range(3):
    r.ray_trace()
g = r.get_internal(argb=False, rgba=True, hit=True)
rw, rh = st.render_size()
dur = g["hit_t"].reshape(rh, rw).astype(np.float64) / 100.0
start = np.ascontiguousarray(g["rgba"][:, 3]).view(np.uint32).reshape(rh, rw).astype(np.int64)
T = lambda a: a[: rh // 8 * 8, : rw // 8 * 8].reshape(rh // 8, 8, rw // 8, 8)
tdur = T(dur).max(axis=(1, 3))
tst = T(start).min(axis=(1, 3))
t0 = tst.min()
ts = (tst - t0) / 100.0
te = ts + tdur
print("kernel ms", r.stats()["kernel_ms"], " last tile end us %.1f" % te.max())
order = np.argsort(tdur.ravel())[::-1]
for i in order[:10]:
    a, b = np.unravel_index(i, tdur.shape)
    print(f"  heavy tile ({a},{b}): start {ts[a, b]:8.1f} us  dur {tdur[a, b]:7.1f}  end {te[a, b]:8.1f}")
last = np.argsort(te.ravel())[::-1]
print("last tiles to end:")
for i in last[:10]:
    a, b = np.unravel_index(i, tdur.shape)
    print(f"  tile ({a},{b}): start {ts[a, b]:8.1f} us  dur {tdur[a, b]:7.1f}  end {te[a, b]:8.1f}")
for q in (0.5, 0.9, 0.99, 0.999, 1.0):
    print(f"  {q * 100:5.1f}% of tiles started by {np.quantile(ts, q):8.1f} us, ended by {np.quantile(te, q):8.1f} us")
hist = np.zeros(int(te.max()) // 50 + 1)
for a, b in zip(ts.ravel(), te.ravel()):
    hist[int(a) // 50: int(b) // 50 + 1] += 1
print("tiles in flight per 50 us:", " ".join(str(int(x)) for x in hist))
