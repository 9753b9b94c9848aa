"""One rank's band launch at N ranks: where its critical path sits (rt_tile_costs of the band launch).
GPU box:  python tools/band_tile_costs.py [config] [nranks] [rank ...]
For each rank: the launch-local tile cost distribution after a few launches (heavy-first and split
tiles from the previous launch's costs), the costliest tiles, and the costliest against the mean
cycles per wave of the launch's grid (3072 waves at one frame in flight)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np

from raytracercpp_amd import scenes


def main():
    import torch
    from raytracercpp_amd.renderer import Renderer
    name = sys.argv[1] if len(sys.argv) > 1 else "sphere1m"
    nranks = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    ranks = [int(x) for x in sys.argv[3:]] or list(range(nranks))
    # several layouts in one process: "8:0,1:0" style lists through BAND_LAYOUTS
    layouts = [tuple(map(int, x.split(":"))) for x in os.environ.get("BAND_LAYOUTS", "").split(",") if x]
    sc, st = scenes.CONFIGS[name]()
    r = Renderer(0)
    r.load_scene(sc, st)
    r.ray_trace()
    r.finish_accel()
    band = 8
    for nranks, rank in (layouts or [(nranks, rk) for rk in ranks]):
        out = torch.zeros((r.local_rows(band, rank, nranks), st.image_width), dtype=torch.int32, device="cuda:0")
        for _ in range(6):
            r.render_bands_device(band, rank, nranks, out.data_ptr(), 0)
        torch.cuda.synchronize()
        for _ in range(20):   # one frame in flight: the launch's duration (HIP events)
            r.render_bands_device(band, rank, nranks, out.data_ptr(), 0)
        torch.cuda.synchronize()
        kms = r.kernel_times(20)
        c = r.tile_costs().astype(np.float64).ravel()
        v = np.sort(c[c > 0])
        mean_wave = v.sum() / 3072
        top = np.argsort(c)[::-1][:6]
        print(f"{name} N={nranks} rank {rank}: {v.size} tiles, sum {v.sum():.3g} cycles, mean per wave {mean_wave:.3g}; "
              f"costliest {v[-1]:.3g} ({v[-1] / mean_wave:.2f} x the mean wave), q0.99 {v[int(0.99 * v.size)]:.3g}; "
              f"top {[int(c[i]) for i in top]}; kernel {np.mean(kms):.4f} ms (min {np.min(kms):.4f}); "
              f"env {os.environ.get('RT_HEAVY_SPLIT', '-')}/{os.environ.get('RT_HEAVY_GROUP', '-')}", flush=True)


if __name__ == "__main__":
    main()
