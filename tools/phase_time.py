"""Where a wave's time goes in the C4 frame (plain kernel), from the diagnostic build
-DRT_PHASE_TIME=1: shader cycles per phase summed over the waves, and per unit of work.
    python tools/variants.py build ph="-DRT_PHASE_TIME=1"                         (here)
    RT_DEBUG_WAVES=1 RT_LIB_PATH=_variants/librt_ph.so python tools/phase_time.py [--miss]  (GPU box)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np

os.environ.setdefault("RT_ASYNC_ACCEL", "0")   # every frame on the wide BVH

from raytracercpp_amd import scenes
from raytracercpp_amd.renderer import Renderer

NAMES = ["tile setup", "ray generation", "primary query", "shading", "shadow query", "framebuffer", "dequeue"]
sc, st = scenes.sphere1m()
if "--miss" in sys.argv:   # every primary ray misses (the sphere moved behind the camera)
    import dataclasses
    sc = dataclasses.replace(sc, tri=(sc.tri + np.tile(np.float32([0, 0, 100]), 3)).astype(np.float32))
r = Renderer(0)
r.load_scene(sc, st)
for _ in range(3):
    r.ray_trace()
s = r.stats()
d = r.debug_read(16384 * 8).reshape(-1, 8)[:, :7].astype(np.float64)
d = d[d.sum(1) > 0]
tot = d.sum()
print(f"kernel ms {s['kernel_ms']:.3f}  waves {len(d)}  mean cycles per wave {d.sum(1).mean():.0f}")
for k, n in enumerate(NAMES):
    print(f"  {n:16s} {d[:, k].sum() / tot * 100:6.1f} %   mean per wave {d[:, k].mean():10.0f} cycles")
w = d.sum(1)
q = np.quantile(w, [0.5, 0.9, 0.99, 1.0])
print(f"  cycles per wave: median {q[0]:.0f}  p90 {q[1]:.0f}  p99 {q[2]:.0f}  max {q[3]:.0f}")
top = d[w >= np.quantile(w, 0.99)]
print("  slowest 1% of waves, mean cycles per phase: " +
      "  ".join(f"{n} {top[:, k].mean():.0f}" for k, n in enumerate(NAMES)))
