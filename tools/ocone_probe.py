"""The renderer's origin-cone grid on C5's scene (GPU box): code histogram of the computed cells, and how
many of tools/refl_probe.py's reflection-like rays skip case (b) on it (host evaluation of ocone_skip).
    python tools/ocone_probe.py [rays.npz]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

from raytracercpp_amd import _lib, scenes
from raytracercpp_amd.renderer import Renderer

sc, st = scenes.sphere1m_refl(width=64, height=36, samples=2)
R = Renderer(0)
R.load_scene(sc, st)
t0 = time.time()
R.ray_trace()
R.finish_accel()
print(f"accel {time.time() - t0:.2f} s", flush=True)
cells, dims, lo_ih = R.ocone_read()
code = cells[:, 1] >> 16
print("dims", dims.tolist(), "lo_ih", lo_ih.tolist(), "cells", len(code), flush=True)
for name, m in (("noskip", code == 0x7FFF), ("empty", code == 0x7FFE), ("cone", code < 0x7FFE)):
    print(name, int(m.sum()))
beta = code[code < 0x7FFE] * (90.0 / 0x7FFD)
if len(beta):
    print("half-angle deg percentiles 10/50/90/99:", np.percentile(beta, [10, 50, 90, 99]).round(2).tolist())
if len(sys.argv) > 1:
    z = np.load(sys.argv[1])
    o, d = z["o"][:400], z["d"][:400]
    skip, stt = _lib.ocone_check(sc.tri, o, d, st.bvh_max_depth, st.bvh_leaf_object_count, ocone_dim=int(dims.max()),
                                 grid=(cells, dims, lo_ih))
    print("rays skipping (b):", stt["skipping"], "of", len(o), "violations", stt["violations"], flush=True)
