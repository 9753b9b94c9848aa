"""Strip-scaling probe on ONE GPU: per-step time of one rank's share of the C4 frame.

For each N in --ranks, renders rank r's bands (render_bands_device(band, r, N)) K times
back to back on one stream and reports the step time (wall clock over K async steps),
the mean ray_trace_kernel time (HIP events) and the implied N-GPU throughput bound
(frame rays / slowest rank's step time), i.e. the strip path without the gather.
Usage (GPU box): python tools/strip_scaling.py [--ranks 1 2 4 8] [--steps 50]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ranks", type=int, nargs="+", default=[1, 2, 4, 8])
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--band-rows", type=int, default=8)
    ap.add_argument("--config", default="sphere1m")
    ap.add_argument("--all-ranks", action="store_true", help="time every rank of each N (default: rank 0 and N-1)")
    ap.add_argument("--inflight", type=int, nargs="+", default=[1],
                    help="frames in flight: consecutive steps alternate over this many streams")
    ap.add_argument("--balance", action="store_true",
                    help="cost-balanced band lists (strips.assign_bands over the interleaved layout's band costs)")
    args = ap.parse_args()
    import torch
    from raytracercpp_amd import scenes
    from raytracercpp_amd.renderer import Renderer

    sc, st = scenes.CONFIGS[args.config]()
    r = Renderer(0)
    r.load_scene(sc, st)
    r.ray_trace()
    r.finish_accel()   # every timed step on the wide BVH
    W = st.image_width
    rw, rh = st.render_size()
    band = args.band_rows
    res = []
    from raytracercpp_amd.strips import assign_bands, num_bands
    nb = num_bands(st.image_height, band)
    lists = {}
    if args.balance:
        # every rank's band costs under the interleaved layout (each rank's share alone on the GPU, as
        # on its own GPU), summed into one vector, then the balanced lists
        for n in args.ranks:
            costs = np.zeros(nb)
            for rank in range(n):
                nloc = r.local_rows(band, rank, n)
                o = torch.empty((nloc, W), dtype=torch.int32, device="cuda")
                for _ in range(args.warmup + 2):
                    r.render_bands_device(band, rank, n, o.data_ptr(), 0)
                costs = r.band_costs(nb, 0, costs)
            lists[n] = assign_bands(costs, n)
            loads = [float(costs[lst].sum()) for lst in lists[n]]
            print(json.dumps({"N": n, "balanced_loads_rel": [round(x / max(loads), 3) for x in loads]}), flush=True)
    for q in args.inflight:
        streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(q - 1)]
        for n in args.ranks:
            ranks = range(n) if args.all_ranks else sorted({0, n - 1})
            for rank in ranks:
                lst = lists[n][rank] if n in lists else None
                nloc = (len(lists[n][0]) * band) if lst is not None else r.local_rows(band, rank, n)
                outs = [torch.empty((nloc, W), dtype=torch.int32, device="cuda") for _ in range(q)]

                def step(i):
                    if lst is not None:
                        r.render_band_list_device(band, lst, outs[i % q].data_ptr(), streams[i % q].cuda_stream)
                    else:
                        r.render_bands_device(band, rank, n, outs[i % q].data_ptr(), streams[i % q].cuda_stream)

                for i in range(args.warmup):
                    step(i)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for i in range(args.steps):
                    step(i)
                th = (time.perf_counter() - t0) / args.steps   # host time per enqueued step
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / args.steps
                k = float(np.mean(r.kernel_times(args.steps)))
                shadow, _ = r.band_counters()
                rec = {"inflight": q, "N": n, "rank": rank, "balanced": lst is not None, "step_ms": round(dt * 1e3, 4), "kernel_ms": round(k, 4),
                       "overhead_ms": round(dt * 1e3 - k, 4), "host_ms": round(th * 1e3, 4), "local_rows": nloc,
                       "shadow_rays": shadow}
                res.append(rec)
                print(json.dumps(rec), flush=True)
    for q in args.inflight:
        base = [x for x in res if x["N"] == 1 and x["inflight"] == 1]
        if base:
            b = base[0]["step_ms"]
            for n in args.ranks:
                worst = max(x["step_ms"] for x in res if x["N"] == n and x["inflight"] == q)
                print(json.dumps({"inflight": q, "N": n, "bound_speedup_no_gather": round(b / worst, 3)}), flush=True)

if __name__ == "__main__":
    main()
