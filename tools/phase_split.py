"""Kernel time of the C4 frame with and without shadow rays (RenderSettings::compute_shadows),
and with the literal whole-line traversal, to split the frame between primary and shadow work."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
from raytracercpp_amd import scenes
from raytracercpp_amd.renderer import Renderer

sc, st = scenes.sphere1m()
r = Renderer(0)
for label, kw, env in (("primary+shadow", {}, {}), ("primary only", {"compute_shadows": False}, {}),
                       ("primary+shadow, RT_CONES=0", {}, {"RT_CONES": "0"}),
                       ("primary+shadow, RT_SEG=0 RT_CONES=0", {}, {"RT_SEG": "0", "RT_CONES": "0"})):
    for k in ("RT_SEG", "RT_CONES"):
        os.environ.pop(k, None)
    os.environ.update(env)
    r.load_scene(sc, st.copy(**kw))
    ts = []
    for i in range(8):
        r.ray_trace()
        ts.append(r.stats()["kernel_ms"])
    s = r.stats()
    print(f"{label:40s} kernel {np.median(ts[2:]):7.3f} ms  shadow rays {s['shadow_rays']}", flush=True)
