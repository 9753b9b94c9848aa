"""Fused SSAA (RT_FUSED_SSAA) vs the separate downscale pass, band by band (diagnostic)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from raytracercpp_amd import scenes
from raytracercpp_amd.renderer import Renderer
from raytracercpp_amd.strips import rank_rows

r = Renderer(0)
for f, nranks, band, two in ((4, 3, 4, True), (4, 3, 4, False), (4, 1, 4, False), (2, 3, 4, False), (4, 2, 4, False)):
    sc, st = scenes.bumpy70k(width=160, height=96, enable_ssaa=True, ssaa_factor=f)
    r.load_scene(sc, st)
    res = {}
    for fz in ("1", "0"):
        os.environ["RT_FUSED_SSAA"] = fz
        streams = [torch.cuda.Stream(), torch.cuda.Stream()] if two else [torch.cuda.current_stream()] * 2
        bufs = []
        for rank in range(nranks):
            n = r.local_rows(band, rank, nranks)
            buf = torch.zeros((n, st.image_width), dtype=torch.int32, device="cuda:0")
            r.render_bands_device(band, rank, nranks, buf.data_ptr(), streams[rank % 2].cuda_stream)
            bufs.append(buf)
        torch.cuda.synchronize()
        res[fz] = [b.cpu().numpy().view(np.uint32) for b in bufs]
    for rank in range(nranks):
        d = np.argwhere(res["1"][rank] != res["0"][rank])
        rows = sorted(set(d[:, 0].tolist()))
        print(f"f={f} nranks={nranks} band={band} two={two} rank={rank}: {len(d)} px differ, local rows {rows[:20]}",
              flush=True)
