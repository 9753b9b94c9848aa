#!/usr/bin/env python
"""Headline benchmark: Mrays/s (primary + shadow) at 1920x1080 on the 1M-triangle scene.

Workload (BASELINE.json configs[3]): 1,000,000-triangle UV
sphere, 1920x1080 with 2x2 SSAA (ssaa_factor 2 -> 3840x2160 internal rays), primary
rays + one shadow ray per shaded hit, octree BVH depth 12 / leaf 40.  One "step"
renders the whole frame: ray generation, octree traversal, Moller-Trumbore,
shadow rays, RT shading, quantisation and the SSAA downscale, as image strips on
N GPUs (one process per GPU) followed by the RCCL all-gather of the strips.

Run: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* from the env).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0        # MI355X HBM3E peak (MI355X_MICROARCH.md)
NODE_BYTES = 56              # one octree k-DOP test reads 14 floats
TRI_BYTES = 48               # one Moller-Trumbore test reads a, b-a, c-a, n
WIDE_NODE_BYTES = 96         # one wide-BVH node visit reads the 96-B node (6 x 16-B loads)
CERT_BYTES = 72              # one certificate: the octree leaf's 64-B node + two 4-B slot maps
PIXEL_BYTES = 4              # ARGB32 write per internal pixel
COUNTS_FILE = os.path.join(ROOT, "profiles", "work_counts.json")
# rocprofv3 PMC summary of this kernel on the same command (tools/profile_gpu.sh + profile_summary.py)
PROFILE_SUMMARY = os.path.join(ROOT, "profiles", "r02d", "summary.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)   # a step is ~0.55 ms: 50 keep the pipeline fill / drain small
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="sphere1m")
    ap.add_argument("--band-rows", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--inflight", type=int, default=2,
                    help="frames in flight: consecutive steps alternate over this many streams (DESIGN.md 7)")
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    from raytracercpp_amd import scenes
    from raytracercpp_amd.renderer import Renderer
    from raytracercpp_amd.strips import FramePipeline, assemble_torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        # RCCL on a high-priority stream: with frames in flight the gather's blocks are
        # dispatched ahead of the next frame's persistent grid instead of waiting for its tail
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        dist.init_process_group("nccl", device_id=dev, pg_options=opts)

    sc, st = scenes.CONFIGS[args.config]()
    r = Renderer(local)
    r.load_scene(sc, st)
    W, H = st.image_width, st.image_height
    rw, rh = st.render_size()
    band = args.band_rows
    nloc = r.local_rows(band, rank, world)
    # Frames in flight: step i renders on stream i % q into its own output
    # buffer, and its all-gather is enqueued asynchronously behind it, so the next frame's
    # kernel fills the CUs that this frame's tail leaves idle and the gather overlaps it.
    # Before a slot is reused its previous gather has finished reading the buffer (wait).
    q = max(1, args.inflight)
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(q - 1)]
    outs = [torch.empty((nloc, W), dtype=torch.int32, device=dev) for _ in range(q)]
    pipe = FramePipeline(lambda o, s: r.render_bands_device(band, rank, world, o.data_ptr(), s.cuda_stream),
                         outs, world, streams, dist)
    step, drain = pipe.step, pipe.drain

    t_build0 = time.perf_counter()
    step()   # first call builds + uploads the octree
    drain()
    t_first = time.perf_counter() - t_build0
    shadow_local, refl_local = r.band_counters()
    for _ in range(args.warmup):
        step()
    drain()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    last = 0
    for _ in range(args.steps):
        last = step()
    drain()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ktimes = r.kernel_times(args.steps)
    k_mean = float(np.mean(ktimes))

    t = torch.tensor([elapsed, float(shadow_local), k_mean, float(refl_local)], dtype=torch.float64, device=dev)
    if world > 1:
        tm = t.clone()
        dist.all_reduce(tm, op=dist.ReduceOp.MAX)
        ts = t.clone()
        dist.all_reduce(ts, op=dist.ReduceOp.SUM)
        elapsed_max = float(tm[0])
        shadow_total = int(ts[1])
        k_mean_max = float(tm[2])
        refl_total = int(ts[3])
    else:
        elapsed_max, shadow_total, k_mean_max, refl_total = elapsed, int(shadow_local), k_mean, int(refl_local)
    c5 = args.config == "sphere1m_refl"
    frame = assemble_torch(pipe.parts[last], H, band) if rank == 0 else None

    if rank == 0:
        primary = rw * rh
        rays = primary + shadow_total + (refl_total if c5 else 0)
        ms_per_step = 1e3 * elapsed_max / args.steps
        value = rays * args.steps / elapsed_max / 1e6
        img = frame.cpu().numpy().view(np.uint32)
        metric = ("Mrays/sec (primary+shadow+reflection) at 1920x1080, 1M-tri scene + rough reflections (C5)" if c5
                  else "Mrays/sec (primary+shadow) at 1920x1080, 1M-tri scene; max |dpixel|")
        res = {
            "metric": metric,
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (deterministic 1M-tri UV sphere, SURVEY.md 8(d) C4)",
            "config": {"workload": ("C5 sphere1m_refl: C4 + reflection 0.5 / roughness 0.3, 16 samples, depth 5, "
                                    "normal + parallax maps" if c5 else
                                    "C4 sphere1m: 1,000,000 tris, 1920x1080, ssaa_factor 2 (3840x2160 rays), "
                                    "primary + shadow, octree 12/40"), "image": [W, H], "render": [rw, rh],
                       "rays_per_frame": rays, "primary_rays": primary, "shadow_rays": shadow_total,
                       "reflection_rays": refl_total, "band_rows": band, "parallelism": f"image strips x{world}",
                       "frames_in_flight": q},
            "kernel_ms": round(k_mean_max, 4),
            "first_call_s": round(t_first, 3),
        }
        counts = None
        if os.path.exists(COUNTS_FILE):
            with open(COUNTS_FILE) as f:
                counts = json.load(f).get(args.config)
        share = 1.0 / world
        # Roofline: the bytes the launch's traversal reads, per the counted units of
        # the RT_COUNT build (tools/count_gpu_work.py -> profiles/work_counts.json "gpu_executed"):
        # WIDE_NODE_BYTES per wide-BVH node visit, TRI_BYTES per Moller-Trumbore test, CERT_BYTES per
        # certificate, NODE_BYTES per octree k-DOP test (uncertified queries), PIXEL_BYTES per pixel,
        # over the mean kernel time; "traffic" is the measured HBM bytes per launch (PMC, 2 x
        # FETCH_SIZE + WRITE_SIZE) -- the ~90 MB scene lives in L2 / Infinity Cache.
        ex = counts.get("gpu_executed") if counts else None
        ms_per_step_local = 1e3 * elapsed_max / args.steps
        default_path = all(os.environ.get(k, "1") != "0" for k in ("RT_WBVH", "RT_SEG", "RT_CONES"))
        if ex and default_path:
            xb = (WIDE_NODE_BYTES * ex.get("wide_node_visits", 0) + TRI_BYTES * ex.get("wide_tri_tests", 0) +
                  CERT_BYTES * ex.get("wide_certificates", 0) +
                  NODE_BYTES * (ex["vol_tests_whole_line"] + ex["vol_tests_segment"]) +
                  TRI_BYTES * (ex["tri_tests_whole_line"] + ex["tri_tests_segment"]) + PIXEL_BYTES * primary)
            xa = xb * share / (k_mean_max * 1e-3) / 1e9
            traffic = None
            if world == 1 and args.config == "sphere1m" and os.path.exists(PROFILE_SUMMARY):
                with open(PROFILE_SUMMARY) as f:
                    traffic = json.load(f).get("hbm_traffic_bytes_per_launch")
            res["roofline"] = {"bound": "hbm", "achieved": round(xa, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                               "frac": round(xa / PEAK_HBM_GBS, 4), "traffic": int(traffic) if traffic else None,
                               "algorithmic_bytes_per_frame": xb,
                               "basis": "bytes read by the executed traversal (wide-BVH nodes 96 B, triangles 48 B, "
                                        "certificates 72 B, octree k-DOPs 56 B) + 4 B/pixel; RT_COUNT counts",
                               # with frames in flight a launch shares the GPU with the next frame's, so
                               # its duration (above) is longer than the step; the same bytes over the
                               # step interval (whole-job rate)
                               "per_step": {"achieved": round(xb * share / (ms_per_step_local * 1e-3) / 1e9, 1),
                                            "frac": round(xb * share / (ms_per_step_local * 1e-3) / 1e9 / PEAK_HBM_GBS, 4)}}
            if counts and "child_tests_primary" in counts:
                # SURVEY.md 8(d)'s model priced on the REFERENCE's traversal (oracle count mode): the work
                # the reference's octree walk would read, per second of this kernel
                tests = counts["child_tests_primary"] + counts["child_tests_shadow"]
                tris = counts["tri_tests_primary"] + counts["tri_tests_shadow"]
                nbytes = NODE_BYTES * tests + TRI_BYTES * tris + PIXEL_BYTES * primary
                res["roofline"]["reference_traversal_equivalent"] = {
                    "bytes_per_frame": nbytes, "achieved": round(nbytes * share / (k_mean_max * 1e-3) / 1e9, 1)}
        if world == 1 and not args.no_cpu_baseline:
            if c5:
                res["cpu_baseline"] = cpu_baseline_c5(sc, st, args.cpu_threads)
            else:
                res["cpu_baseline"], res["max_abs_dpixel"] = cpu_baseline(sc, st, img, args.cpu_threads)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(sc, st, gpu_img, threads):
    """CPU baseline on the box's host cores, and max |dpixel| of the GPU frame.
    * the reference itself (oracle/_ref/libref_harness.so: the reference's own compiled
      BVH / triangle / vector code driven by the harness's restated pixel loop, OpenMP
      schedule(dynamic) over rows as renderer.cpp:1082) timed on a bounded sample of row
      bands spread over the frame (octree build excluded), when that library was built;
    * the oracle's C restatement (oracle/liboracle.so, OpenMP) on the full frame, which
      also gives the pixel comparison (and the baseline when the reference is absent)."""
    from oracle.bindings import Oracle, RefHarness
    threads = threads or int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    o = Oracle(sc, st)
    res = o.render_rows(nthreads=threads)
    rw, rh = st.render_size()
    ref = Oracle.downscale(res.argb, rw, rh, st.ssaa_factor) if st.enable_ssaa else res.argb
    g = gpu_img.ravel()
    d = 0
    for sh in (16, 8, 0):
        d = max(d, int(np.max(np.abs(((g >> sh) & 0xFF).astype(np.int32) - ((ref >> sh) & 0xFF).astype(np.int32)))))
    port_rays = res.counters["primary_rays"] + res.counters["shadow_rays"]
    port = {"value": round(port_rays / res.seconds / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"full C4 frame ({rw}x{rh} primary + {res.counters['shadow_rays']} shadow rays) "
                      f"in {res.seconds:.2f} s, oracle.c OpenMP x{threads}"}
    if not RefHarness.available():
        return port, d
    os.environ.setdefault("OMP_NUM_THREADS", str(threads))
    stride = 2
    rr = RefHarness.render_row_sample(sc, st, stride // 2, rh // stride, stride)
    rays = rr.counters["primary_rays"] + rr.counters["shadow_rays"]
    base = {"value": round(rays / rr.seconds / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "reference",
            "sample": f"every {stride}th internal row of the C4 frame ({rh // stride} rows x {rw}: {rr.counters['primary_rays']}"
                      f" primary + {rr.counters['shadow_rays']} shadow rays in {rr.seconds:.2f} s, octree build "
                      f"excluded), reference TUs + OpenMP x{threads}",
            "port_value": port["value"]}
    return base, d


def cpu_baseline_c5(sc, st, threads):
    """C5: the reference harness on every 128th internal row (primary + shadow + reflection rays)."""
    from oracle.bindings import RefHarness
    threads = threads or int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    if not RefHarness.available():
        return None
    os.environ.setdefault("OMP_NUM_THREADS", str(threads))
    rw, rh = st.render_size()
    stride = 128
    rr = RefHarness.render_row_sample(sc, st, stride // 2, rh // stride, stride)
    c = rr.counters
    rays = c["primary_rays"] + c["shadow_rays"] + c["reflection_rays"]
    return {"value": round(rays / rr.seconds / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "reference",
            "sample": f"every {stride}th internal row ({rh // stride} rows x {rw}: {c['primary_rays']} primary + "
                      f"{c['shadow_rays']} shadow + {c['reflection_rays']} reflection rays in {rr.seconds:.2f} s), "
                      f"reference TUs + OpenMP x{threads}"}


if __name__ == "__main__":
    main()
