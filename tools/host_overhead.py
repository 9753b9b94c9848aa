"""Host cost of one bench step, on ONE GPU: wall time per call when the GPU work is tiny.
    python -m torch.distributed.run --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 \
        tools/host_overhead.py        (GPU box)
Reports microseconds per call of (a) rt_render_bands_device on a 64x64 frame, (b) the same through
strips.FramePipeline with two frames in flight, (c) an asynchronous RCCL all-gather of a 1-MB
buffer (world size 1, high-priority stream, as bench.py enqueues it), (d) (b) + (c) together."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def per_call(fn, n=2000, warm=50):
    import torch
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e6


def main():
    import torch
    import torch.distributed as dist
    from raytracercpp_amd import scenes
    from raytracercpp_amd.renderer import Renderer
    from raytracercpp_amd.strips import FramePipeline
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    opts = dist.ProcessGroupNCCL.Options()
    opts.is_high_priority_stream = True
    dist.init_process_group("nccl", device_id=dev, pg_options=opts)
    sc, st = scenes.bumpy70k(width=64, height=64)
    r = Renderer(0)
    r.load_scene(sc, st)
    r.ray_trace()
    r.finish_accel()
    W = st.image_width
    nloc = r.local_rows(8, 0, 1)
    streams = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)]
    outs = [torch.empty((nloc, W), dtype=torch.int32, device=dev) for _ in range(2)]
    k = [0]

    def bands():
        k[0] += 1
        r.render_bands_device(8, 0, 1, outs[k[0] % 2].data_ptr(), streams[k[0] % 2].cuda_stream)

    a = per_call(bands)
    pipe = FramePipeline(lambda o, s: r.render_bands_device(8, 0, 1, o.data_ptr(), s.cuda_stream), outs, 1, streams,
                         dist)
    b = per_call(pipe.step)
    big = torch.zeros(262144, dtype=torch.int32, device=dev)   # 1 MB, a rank's strips at N = 8
    parts = [torch.empty_like(big)]
    works = []

    def gather():
        works.append(dist.all_gather(parts, big, async_op=True))
        if len(works) > 4:
            works.pop(0).wait()

    c = per_call(gather)
    for w in works:
        w.wait()
    pipe2 = FramePipeline(lambda o, s: r.render_bands_device(8, 0, 1, o.data_ptr(), s.cuda_stream), outs, 2, streams,
                          None)

    class _D:   # a 2-rank pipeline's gather, issued on the world-1 group
        @staticmethod
        def all_gather(p, o, async_op=True):
            return dist.all_gather(p[:1], o, async_op=async_op)

    pipe2.dist = _D
    d = per_call(pipe2.step)
    pipe2.drain()
    print(f"host us per call: render_bands_device {a:.1f}, FramePipeline step {b:.1f}, "
          f"async all_gather {c:.1f}, pipeline step with gather {d:.1f}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
