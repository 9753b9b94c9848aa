"""Kernel time of the C4 frame split by phase and path: with and without shadow rays
(RenderSettings::compute_shadows), wide BVH on / off (RT_WBVH), deferral on / off
(RT_DEFER_BUDGET), the literal whole-line traversal; with an RT_COUNT build, the
wide-BVH work and uncertified queries too.
    python tools/phase_split.py [label ...]      (GPU box; all variants by default)"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
from raytracercpp_amd import scenes
from raytracercpp_amd.renderer import Renderer

VARIANTS = [
    ("primary+shadow", {}, {}),
    ("primary only", {"compute_shadows": False}, {}),
    ("primary+shadow, RT_WBVH=0", {}, {"RT_WBVH": "0"}),
    ("primary only, RT_WBVH=0", {"compute_shadows": False}, {"RT_WBVH": "0"}),
    ("primary+shadow, no deferral", {}, {"RT_DEFER_BUDGET": "0"}),
    ("primary only, no deferral", {"compute_shadows": False}, {"RT_DEFER_BUDGET": "0"}),
    ("primary+shadow, RT_WBVH=0 RT_SEG=0 RT_CONES=0", {}, {"RT_WBVH": "0", "RT_SEG": "0", "RT_CONES": "0"}),
    ("primary only, barycentric shading", {"compute_shadows": False, "shading_method": 3}, {}),
    ("all rays miss (sphere behind the camera)", {"compute_shadows": False}, {"_behind": "1"}),
]
want = sys.argv[1:]
sc, st = scenes.sphere1m()
r = Renderer(0)
for label, kw, env in VARIANTS:
    if want and label not in want:
        continue
    for k in ("RT_SEG", "RT_CONES", "RT_WBVH", "RT_DEFER_BUDGET"):
        os.environ.pop(k, None)
    behind = env.pop("_behind", None) if "_behind" in env else None
    os.environ.update(env)
    if behind:
        import dataclasses
        sc2 = dataclasses.replace(sc, tri=(sc.tri + np.tile(np.float32([0, 0, 100]), 3)).astype(np.float32))
        r.load_scene(sc2, st.copy(**kw))
    else:
        r.load_scene(sc, st.copy(**kw))
    ts = []
    for i in range(8):
        r.ray_trace()
        ts.append(r.stats()["kernel_ms"])
    s = r.stats()
    w = s["work"]
    extra = f"  deferred {s['deferred_pixels']}"
    if any(w) or any(s.get("work_wide", [0])):
        extra += f"  work {w} abandoned {s['work_abandoned']} wide {s.get('work_wide')}"
    print(f"{label:48s} kernel {np.median(ts[2:]):7.3f} ms  shadow rays {s['shadow_rays']}{extra}", flush=True)
