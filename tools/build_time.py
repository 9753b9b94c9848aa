"""Host build time of the C4 scene's acceleration structures (no GPU): the octree (bvh.h restated,
parallel) and the wide BVH, phase by phase (RT_BUILD_PROFILE=1 prints them), through
rt_wbvh_query.  Usage: RT_BUILD_PROFILE=1 python tools/build_time.py [repeats]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raytracercpp_amd import _lib, scenes

sc, st = scenes.sphere1m()
o = np.zeros((1, 3), np.float32)
d = np.array([[0, 0, -1]], np.float32)
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    r = _lib.wbvh_query(sc.tri, o, d)
    print("octree %.1f ms, wide BVH %.1f ms" % r[6], r[5], flush=True)
