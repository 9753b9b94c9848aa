"""Per-rank cost of one image-strip step at N = 1, 2, 4, 8 (rank 0's bands rendered on one GPU,
no collective): wall time per step (host launch included) and the kernel time, to see what the
multi-GPU bench can scale to before the all-gather."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch
from raytracercpp_amd import scenes
from raytracercpp_amd.renderer import Renderer

sc, st = scenes.sphere1m()
r = Renderer(0)
r.load_scene(sc, st)
stream = torch.cuda.current_stream()
for n in (1, 2, 4, 8):
    worst = 0.0
    for rank in range(n):
        rows = r.local_rows(8, rank, n)
        out = torch.empty((rows, st.image_width), dtype=torch.int32, device="cuda")
        for _ in range(3):
            r.render_bands_device(8, rank, n, out.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize()
        K = 20
        t0 = time.perf_counter()
        for _ in range(K):
            r.render_bands_device(8, rank, n, out.data_ptr(), stream.cuda_stream)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / K * 1e3
        kern = float(np.mean(r.kernel_times(K)))
        worst = max(worst, wall)
        print(f"N={n} rank {rank}: wall {wall:6.3f} ms/step  kernel {kern:6.3f} ms", flush=True)
    print(f"N={n}: slowest rank {worst:.3f} ms/step -> ideal-gather scaling {6.45 / worst if n > 1 else 1:.2f}x", flush=True)
