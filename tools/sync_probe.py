"""Where the synchronous call surface's time goes (bench.py's sync leg: rt_ray_trace + rt_post_process +
rt_get_image, one frame at a time, utils/mainUtils.cpp:6-21): host wall time of each call, averaged.
GPU box:  python tools/sync_probe.py [config] [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np

from raytracercpp_amd import scenes


def main():
    from raytracercpp_amd.renderer import Renderer
    name = sys.argv[1] if len(sys.argv) > 1 else "sphere1m"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    sc, st = scenes.CONFIGS[name]()
    r = Renderer(0)
    r.load_scene(sc, st)
    r.ray_trace()
    r.finish_accel()
    img = None
    for _ in range(5):
        r.ray_trace()
        r.post_process()
        img = r.get_image(img)
    t = np.zeros((steps, 4))
    for i in range(steps):
        t0 = time.perf_counter()
        r.ray_trace()
        t1 = time.perf_counter()
        r.post_process()
        t2 = time.perf_counter()
        img = r.get_image(img)
        t3 = time.perf_counter()
        t[i] = (t1 - t0, t2 - t1, t3 - t2, r.stats()["kernel_ms"] * 1e-3)
    m = t.mean(0) * 1e3
    print(f"{name}: ray_trace {m[0]:.3f} ms (kernel {m[3]:.3f}), post_process {m[1]:.3f} ms, get_image {m[2]:.3f} ms, "
          f"total {m[:3].sum():.3f} ms per frame", flush=True)


if __name__ == "__main__":
    main()
