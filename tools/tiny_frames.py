"""Per-frame fixed cost on ONE GPU: many band launches of a tiny frame (64x64, bumpy70k) on two
alternating streams, as bench.py's frames in flight issue them; run under rocprofv3 --kernel-trace
to see each launch's kernels and the gaps between them.
    rocprofv3 --kernel-trace --stats -d gpurun_out/tiny -o run -- python3 tools/tiny_frames.py (GPU box)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("RT_ASYNC_ACCEL", "0")


def main():
    import torch
    from raytracercpp_amd import scenes
    from raytracercpp_amd.renderer import Renderer
    w = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    sc, st = scenes.bumpy70k(width=w, height=w)
    r = Renderer(0)
    r.load_scene(sc, st)
    r.ray_trace()
    nloc = r.local_rows(8, 0, 1)
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    outs = [torch.empty((nloc, st.image_width), dtype=torch.int32, device="cuda") for _ in range(2)]
    for i in range(20):
        r.render_bands_device(8, 0, 1, outs[i % 2].data_ptr(), streams[i % 2].cuda_stream)
    torch.cuda.synchronize()
    n = 500
    t0 = time.perf_counter()
    for i in range(n):
        r.render_bands_device(8, 0, 1, outs[i % 2].data_ptr(), streams[i % 2].cuda_stream)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n * 1e6
    k = r.kernel_times(64)
    print(f"{w}x{w}: {dt:.1f} us per frame, ray_trace_kernel {1e3 * float(k.mean()):.1f} us (HIP events)", flush=True)


if __name__ == "__main__":
    main()
