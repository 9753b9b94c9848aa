"""Per-wave accounting of the C4 frame (diagnostic build -DRT_WAVE_STATS=1, RT_DEBUG_WAVES=1):
when each persistent wave starts and exits, how many tiles it ran, and how much of its life
it spent inside tiles (the rest: dequeues and the time before it became resident).
    python tools/variants.py build ws="-DRT_WAVE_STATS=1"                      (here)
    RT_DEBUG_WAVES=1 RT_LIB_PATH=_variants/librt_ws.so python tools/wave_stats.py  (GPU box)"""
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
for _ in range(3):
    r.ray_trace()
d = r.debug_read(16384 * 8).reshape(-1, 8)[:, :4].astype(np.int64)
d = d[d[:, 1] > 0]
t0 = d[:, 0].min()
b, e, n, busy = (d[:, 0] - t0) / 100.0, (d[:, 1] - t0) / 100.0, d[:, 2], d[:, 3] / 100.0
print(f"kernel ms {r.stats()['kernel_ms']:.3f}  waves recorded {len(d)}  (with tiles: {(n > 0).sum()})")
for name, a in (("start us", b), ("exit us", e), ("tiles", n), ("busy us", busy), ("life us", e - b),
                ("idle us (life - busy)", e - b - busy)):
    q = np.quantile(a, [0, 0.1, 0.5, 0.9, 1.0])
    print(f"  {name:22s} min {q[0]:9.1f}  p10 {q[1]:9.1f}  median {q[2]:9.1f}  p90 {q[3]:9.1f}  max {q[4]:9.1f}")
print(f"  sum busy / sum life {busy.sum() / max(1e-9, (e - b).sum()):.3f};  mean idle per tile {((e - b - busy) / np.maximum(n, 1)).mean():.2f} us")
# concurrency over time
grid = np.arange(0, e.max() + 10, 10.0)
live = [(b <= g).sum() - (e <= g).sum() for g in grid]
print("  waves alive per 10 us:", " ".join(str(int(x)) for x in live[::5]))
