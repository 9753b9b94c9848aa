"""RCCL path of bench.py on one GPU (world size 1, torchrun): high-priority process group, three
frames in flight with async all-gathers into one flat buffer (strips.FramePipeline with the gather
forced on) and the re-assembly on the slot's stream; every gathered and re-assembled frame must equal
the rendered strips.  Usage (GPU box):
  python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \\
      --master-port 29511 tools/nccl_check.py"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.distributed as dist
from raytracercpp_amd import scenes
from raytracercpp_amd.renderer import Renderer
from raytracercpp_amd.strips import FramePipeline, gather_index

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
opts = dist.ProcessGroupNCCL.Options()
opts.is_high_priority_stream = True
dist.init_process_group("nccl", device_id=dev, pg_options=opts)
sc, st = scenes.bumpy70k(width=320, height=184, enable_ssaa=True, ssaa_factor=2)
r = Renderer(0)
r.load_scene(sc, st)
band = 8
n = r.local_rows(band, 0, 1)
q = 3   # frames in flight: bench.py's default (--inflight)
streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(q - 1)]
outs = [torch.zeros((n, st.image_width), dtype=torch.int32, device=dev) for _ in range(q)]
torch.cuda.synchronize()
# the gather forced on with one rank, and rank 0's in-step re-assembly (bench.py) through gather_index
idx = torch.as_tensor(gather_index(st.image_height, band, 1, n), device=dev)
frames = [torch.zeros((st.image_height, st.image_width), dtype=torch.int32, device=dev) for _ in range(q)]
pipe = FramePipeline(lambda o, s: r.render_bands_device(band, 0, 1, o.data_ptr(), s.cuda_stream), outs, 1, streams, dist,
                     assemble=lambda i, flat: torch.index_select(flat, 0, idx, out=frames[i]), gather=True)
ok = True
for k in range(12):
    pipe.step()
pipe.drain()
ref = outs[0].clone()
for i in range(q):
    ok &= bool(torch.equal(pipe.parts[i][0], outs[i])) and bool(torch.equal(outs[i], ref))
    ok &= bool(torch.equal(frames[i], ref[:st.image_height]))
print("nccl pipeline ok" if ok else "nccl pipeline MISMATCH", flush=True)
dist.destroy_process_group()
sys.exit(0 if ok else 1)
