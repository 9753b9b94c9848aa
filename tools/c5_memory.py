import sys, os
sys.path.insert(0, os.getcwd())
import torch
from raytracercpp_amd import scenes
from raytracercpp_amd.renderer import Renderer
f0, tot = torch.cuda.mem_get_info()
sc, st = scenes.sphere1m_refl()
r = Renderer(0); r.load_scene(sc, st); r.ray_trace(); r.finish_accel(); r.ray_trace()
torch.cuda.synchronize()
f1, _ = torch.cuda.mem_get_info()
print("device memory held after a C5 frame: %.1f GB of %.1f GB" % ((f0 - f1) / 1e9, tot / 1e9))
