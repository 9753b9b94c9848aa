"""Quick GPU-vs-oracle mismatch report (debug tool)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from raytracercpp_amd import scenes
from raytracercpp_amd.renderer import Renderer
from oracle.bindings import Oracle

def run(name, sc, st, r):
    r.load_scene(sc, st)
    r.request_aux(rgba=True, hit=True, shadow=True)
    t0 = time.time(); r.ray_trace(); t1 = time.time()
    g = r.get_internal(argb=True, rgba=True, hit=True, shadow=True)
    s = r.stats()
    o = Oracle(sc, st).render_rows()
    print(f"{name:10s} ntri={sc.ntri:8d} {s['render_width']}x{s['render_height']} kernel {s['kernel_ms']:.3f} ms wall {1e3*(t1-t0):.1f} ms build {s['build_ms']:.1f} ms "
          f"| argb!= {int((g['argb']!=o.argb).sum())} hit!= {int((g['hit_id']!=o.hit_id).sum())} "
          f"t!= {int((g['hit_t'].view(np.uint32)!=o.hit_t.view(np.uint32)).sum())} shadow!= {int((g['shadow']!=o.shadow).sum())} "
          f"rgba maxdiff {float(np.abs(g['rgba']-o.rgba).max()):.3g} | shadow rays gpu {s['shadow_rays']} oracle {o.counters['shadow_rays']} | oracle {o.seconds*1e3:.1f} ms", flush=True)

r = Renderer(0)
W, H = int(sys.argv[1]) if len(sys.argv) > 1 else 320, int(sys.argv[2]) if len(sys.argv) > 2 else 180
run("sphere256", *scenes.sphere256(), r)
run("cube", *scenes.cube1080(width=W, height=H), r)
run("robot", *scenes.robot1080(width=W, height=H), r)
run("bumpy70k", *scenes.bumpy70k(width=W, height=H), r)
run("sphere1m", *scenes.sphere1m(width=W, height=H), r)
