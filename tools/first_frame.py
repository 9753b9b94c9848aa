"""The first frame after a geometry change (renderer.cpp:137-144 / 214-224 rebuild
unconditionally): Renderer::set_object_transform, then the next ray_trace runs before the wide BVH is
resident.  Prints per transform: the host time of set_object_transform (octree build +
upload), the first frame's kernel time (HIP events) and wall time, the frame after rt_finish_accel, and
whether the two images are the same bits.
    GPU box: python tools/first_frame.py [config] [transforms]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np

from raytracercpp_amd import scenes


def rot_y(deg, centre):
    a = np.radians(deg)
    c, s = np.cos(a), np.sin(a)
    R = np.array([[c, 0, s, 0], [0, 1, 0, 0], [-s, 0, c, 0], [0, 0, 0, 1]])
    T = np.eye(4)
    T[:3, 3] = centre
    Ti = np.eye(4)
    Ti[:3, 3] = -np.asarray(centre)
    return (T @ R @ Ti).astype(np.float32).ravel()


def main():
    import torch
    from raytracercpp_amd.renderer import Renderer
    name = sys.argv[1] if len(sys.argv) > 1 else "sphere1m"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    sc, st = scenes.CONFIGS[name]()
    r = Renderer(0)
    r.load_scene(sc, st)
    r.ray_trace()
    r.finish_accel()
    r.ray_trace()
    steady = r.stats()["kernel_ms"]
    centre = sc.tri.reshape(-1, 3).mean(0)
    for k in range(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r.set_object_transform(rot_y(7.0 * (k + 1), centre))
        t1 = time.perf_counter()
        r.ray_trace()
        t2 = time.perf_counter()
        s = r.stats()
        first = r.get_image().copy()
        r.finish_accel()
        r.ray_trace()
        wide = r.stats()["kernel_ms"]
        same = bool(np.array_equal(first, r.get_image()))
        print(json.dumps({"config": name, "transform": k, "set_object_transform_ms": round((t1 - t0) * 1e3, 2),
                          "first_frame_kernel_ms": round(s["kernel_ms"], 3), "first_frame_wall_ms": round((t2 - t1) * 1e3, 2),
                          "wide_frame_kernel_ms": round(wide, 3), "steady_kernel_ms": round(steady, 3),
                          "same_image": same, "plain_octree": os.environ.get("RT_PLAIN_OCTREE", "1")}), flush=True)


if __name__ == "__main__":
    main()
