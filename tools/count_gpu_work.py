"""Traversal work the GPU kernels actually do (k-DOP tests, Moller-Trumbore tests) on a
benchmark workload, from the diagnostic build (-DRT_COUNT=1):
    python tools/variants.py build count="-DRT_COUNT=1"        (here)
    RT_LIB_PATH=_variants/librt_count.so python tools/count_gpu_work.py [config]   (GPU box)
Prints one JSON line per mode: the default (wide BVH + segment queries) and the octree's
literal whole-line traversal (RT_WBVH=0 RT_SEG=0; the switches are read when a renderer is
created, so each mode gets its own)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from raytracercpp_amd import scenes
from raytracercpp_amd.renderer import Renderer

name = sys.argv[1] if len(sys.argv) > 1 else "sphere1m"
modes = sys.argv[2:] or ["seg", "whole_line"]
sc, st = scenes.CONFIGS[name]()
import ctypes
from raytracercpp_amd import _lib
_diag = getattr(_lib.lib(), "rt_diag_wave_steps", None) if hasattr(_lib, "lib") else None
for mode in modes:
    if mode == "whole_line":
        os.environ["RT_SEG"] = "0"
        os.environ["RT_WBVH"] = "0"
    r = Renderer(0)
    r.load_scene(sc, st)
    r.ray_trace()        # builds the octree; the wide BVH and leaf cones build beside it
    r.finish_accel()     # counted frame on the adopted structures
    steps = (ctypes.c_ulonglong * 8)()
    if _diag:
        _diag(steps)   # clear
    r.ray_trace()
    s = r.stats()
    if _diag:
        _diag(steps)
    st8 = list(steps)
    w = s["work"]
    print(json.dumps({"config": name, "mode": mode, "seg_scale": s["seg_scale"], "primary_rays": s["primary_rays"],
                      "shadow_rays": s["shadow_rays"], "reflection_rays": s["reflection_rays"],
                      "vol_tests_whole_line": w[0], "tri_tests_whole_line": w[1],
                      "vol_tests_segment": w[2], "tri_tests_segment": w[3],
                      "wide_node_visits": s["work_wide"][0], "wide_tri_tests": s["work_wide"][1],
                      "wide_uncertified": s["work_wide"][2], "wide_certificates": s["work_wide"][3],
                      "uncertified_by_reason": s["uncertified"], "kernel_ms": s["kernel_ms"],
                      "wave_steps_primary": s["wave_steps"][:3], "wave_steps_shadow": s["wave_steps"][3:],
                      "wave_node_steps": st8[0], "uniform_node_steps": st8[1], "wave_leaf_steps": st8[2],
                      "uniform_leaf_steps": st8[3], "node_step_lanes": st8[4], "leaf_step_lanes": st8[5],
                      "distinct_nodes": st8[6], "distinct_leaves": st8[7],
                      "simd_efficiency": [round(s["wave_steps"][i + 1] / max(1, 64 * s["wave_steps"][i]), 4)
                                          for i in (0, 3)]}), flush=True)
