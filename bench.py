#!/usr/bin/env python
"""Headline benchmark: Mrays/s (primary + shadow) at 1920x1080 on the 1M-triangle scene.

Workload (BASELINE.json configs[3]): 1,000,000-triangle UV
sphere, 1920x1080 with 2x2 SSAA (ssaa_factor 2 -> 3840x2160 internal rays), primary
rays + one shadow ray per shaded hit, octree BVH depth 12 / leaf 40.  One "step"
renders the whole frame: ray generation, octree traversal, Moller-Trumbore,
shadow rays, RT shading, quantisation and the SSAA downscale, as image strips on
N GPUs (one process per GPU) followed by the RCCL all-gather of the strips.

Run: python bench.py [--gpus N --steps K --warmup W].  For N > 1 the driver launches it
under torch.distributed.run (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* from the env); when
WORLD_SIZE is unset and N > 1, bench.py starts that launcher itself as a child process
before anything touches a GPU.  --dry-run exercises the launch / strip / gather / check
plumbing on CPU ranks over gloo with synthetic pattern strips (no GPU, no renderer).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Roofline.  The kernel is bound by dependent gathers through L1 / L2, not by
# HBM: its ~130 MB working set stays in L2 and the Infinity Cache (profiles/r03g: 41 MB of
# HBM traffic per launch against 4.2 GB read by the traversal).  The executed bytes are
# priced against the L2 ceiling; the HBM rate and the guide's random-row gather rate are
# reported beside it.  Peaks: /opt/skills/guides/MI355X_MICROARCH.md.
PEAK_L2_GBS = 34500.0        # L2 aggregate, 8 XCDs (MI355X_MICROARCH.md, L2 per XCD)
PEAK_HBM_GBS = 8000.0        # HBM3E spec peak
GATHER_151MB_GBS = 7650.0    # uniformly random 1,152-B rows of a 151 MB table (Indexed rows: 7.4-7.9 TB/s)
NODE_BYTES = 56              # one octree k-DOP test reads 14 floats
TRI_BYTES = 48               # one Moller-Trumbore test reads a, b-a, c-a, n
WIDE_NODE_BYTES = 160        # one wide-BVH node visit reads the 128-B node and the ray kind's 32 B of risk words
                             # (8 + 2 x 16-B loads)
CERT_BYTES = 72              # one certificate: the octree leaf's 64-B node + two 4-B slot maps
PIXEL_BYTES = 4              # ARGB32 write per internal pixel
COUNTS_FILE = os.path.join(ROOT, "profiles", "work_counts.json")
# configs whose oracle frame takes minutes on the host (hair1m: ~100 s on 8 threads): bench checks
# every CHECK_STRIDE-th output row (its f internal rows) instead of the whole frame
SAMPLED_CHECK = ("hair1m",)
CHECK_STRIDE = 8
# rocprofv3 PMC summary of the benched kernel (tools/profile_gpu.sh + profile_summary.py, copied from the
# round's profile directory): kept outside the per-round directories so that it ships to the GPU box
PROFILE_SUMMARY = os.path.join(ROOT, "profiles", "c4_summary.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)   # a step is ~0.55 ms: 50 keep the pipeline fill / drain small
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="sphere1m")
    ap.add_argument("--band-rows", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-check", action="store_true", help="skip max_abs_dpixel (the oracle frame)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--inflight", type=int, default=3,
                    help="frames in flight: consecutive steps alternate over this many streams (DESIGN.md 7)")
    ap.add_argument("--no-balance", dest="balance", action="store_false",
                    help="N > 1: keep the interleaved bands (default: cost-balanced band lists after the warm-up)")
    ap.add_argument("--no-legs", action="store_true", help="N = 1: skip the sync and moving-camera legs")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU ranks over gloo, synthetic pattern strips: the launch / gather / check plumbing only")
    return ap.parse_args()


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n: int) -> int:
    """--gpus N > 1 without a launcher: run N ranks under torch.distributed.run as a child
    process (this process has not touched a GPU) and return its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.run(cmd, env=env).returncode


def pattern_strip(rows: np.ndarray, width: int) -> np.ndarray:
    """Dry run: a deterministic ARGB value per (global row, column); padding rows stay 0."""
    col = np.arange(width, dtype=np.uint64)
    v = (rows.astype(np.int64)[:, None].astype(np.uint64) * np.uint64(0x9E3779B1) + col[None, :] * np.uint64(0x85EBCA77))
    v = (v ^ (v >> np.uint64(15))) & np.uint64(0x00FFFFFF)
    out = (v | np.uint64(0xFF000000)).astype(np.uint32)
    out[rows < 0] = 0
    return out.view(np.int32)


def max_abs_dpixel(a: np.ndarray, b: np.ndarray) -> int:
    a = np.asarray(a).ravel().view(np.uint32)
    b = np.asarray(b).ravel().view(np.uint32)
    d = 0
    for sh in (16, 8, 0):
        d = max(d, int(np.max(np.abs(((a >> sh) & 0xFF).astype(np.int32) - ((b >> sh) & 0xFF).astype(np.int32)))))
    return d


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "0"))
    if world == 0 and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = max(world, 1)
    if args.dry_run:
        return dry_run(args, world)
    import torch
    import torch.distributed as dist
    from raytracercpp_amd import scenes
    from raytracercpp_amd.renderer import Renderer
    from raytracercpp_amd.strips import FramePipeline, assign_bands, gather_index, num_bands

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        # RCCL on a high-priority stream: with frames in flight the gather's blocks are
        # dispatched ahead of the next frame's persistent grid instead of waiting for its tail
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        dist.init_process_group("nccl", device_id=dev, pg_options=opts)
        world = dist.get_world_size()

    sc, st = scenes.CONFIGS[args.config]()
    r = Renderer(local)
    r.load_scene(sc, st)
    W, H = st.image_width, st.image_height
    rw, rh = st.render_size()
    band = args.band_rows
    nb = num_bands(H, band)
    c5 = args.config == "sphere1m_refl"
    # Frames in flight: step i renders on stream i % q into its own output
    # buffer, and its all-gather is enqueued asynchronously behind it, so the next frame's
    # kernel fills the CUs that this frame's tail leaves idle and the gather overlaps it.
    # Before a slot is reused its previous gather has finished reading the buffer (wait).
    q = max(1, args.inflight)
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(q - 1)]

    def make_pipe(lists):
        """The strips pipeline of this rank: the interleaved bands (lists None) or a band list per
        rank; rank 0 re-assembles every gathered frame on the slot's stream inside the step."""
        nloc = len(lists[0]) * band if lists is not None else r.local_rows(band, rank, world)
        outs = [torch.empty((nloc, W), dtype=torch.int32, device=dev) for _ in range(q)]
        if lists is None:
            render = lambda o, s_: r.render_bands_device(band, rank, world, o.data_ptr(), s_.cuda_stream)  # noqa: E731
        else:
            mine = lists[rank]
            render = lambda o, s_: r.render_band_list_device(band, mine, o.data_ptr(), s_.cuda_stream)  # noqa: E731
        frames, asm = None, None
        if world > 1 and rank == 0:
            idx = torch.as_tensor(gather_index(H, band, world, nloc, lists), device=dev)
            frames = [torch.empty((H, W), dtype=torch.int32, device=dev) for _ in range(q)]
            asm = lambda i, flat: torch.index_select(flat, 0, idx, out=frames[i])  # noqa: E731
        pipe = FramePipeline(render, outs, world, streams, dist, assemble=asm)
        return pipe, (frames if frames is not None else outs)

    pipe, frames = make_pipe(None)
    t_build0 = time.perf_counter()
    pipe.step()   # first call: builds + uploads the octree; the wide BVH and leaf cones build beside it
    pipe.drain()
    t_first = time.perf_counter() - t_build0
    r.finish_accel()   # the timed frames run on the wide BVH
    t_accel = time.perf_counter() - t_build0
    build = r.stats()
    shadow_local, refl_local = r.band_counters()
    for _ in range(args.warmup):
        pipe.step()
    pipe.drain()
    balance = None
    if world > 1 and args.balance and not c5:
        # cost-balanced strips (strips.assign_bands): the warm-up frames' band costs of every rank,
        # summed (each band was rendered by one rank), give every rank the same balanced lists
        costs = r.band_costs(nb, streams[(args.warmup - 1) % q].cuda_stream if args.warmup else 0)
        ct = torch.as_tensor(costs, device=dev)
        dist.all_reduce(ct)
        costs = ct.cpu().numpy()
        lists = assign_bands(costs, world)
        loads = [float(costs[lst].sum()) for lst in lists]
        balance = {"interleaved_max_over_mean": round(max(float(costs[b::world].sum()) for b in range(world)) /
                                                      (sum(loads) / world), 4),
                   "balanced_max_over_mean": round(max(loads) / (sum(loads) / world), 4),
                   "bands_per_rank": [len(x) for x in lists]}
        pipe, frames = make_pipe(lists)
        for _ in range(args.warmup):   # (each stream's heavy lists learn the new layout)
            pipe.step()
        pipe.drain()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    last = 0
    for _ in range(args.steps):
        last = pipe.step()
    pipe.drain()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    ktimes = r.kernel_times(args.steps)
    k_mean = float(np.mean(ktimes))

    t = torch.tensor([elapsed, float(shadow_local), k_mean, float(refl_local)], dtype=torch.float64, device=dev)
    if world > 1:
        allt = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(allt, t)
        per_rank = torch.stack(allt).cpu().numpy()
    else:
        per_rank = t.cpu().numpy()[None, :]
    elapsed_max = float(per_rank[:, 0].max())
    shadow_total = int(per_rank[:, 1].sum())
    k_max, k_min = float(per_rank[:, 2].max()), float(per_rank[:, 2].min())
    refl_total = int(per_rank[:, 3].sum())
    frame = frames[last] if rank == 0 else None

    if rank == 0:
        primary = rw * rh
        rays = primary + shadow_total + (refl_total if c5 else 0)
        ms_per_step = 1e3 * elapsed_max / args.steps
        value = rays * args.steps / elapsed_max / 1e6
        img = frame.cpu().numpy().view(np.uint32)
        metric = ("Mrays/sec (primary+shadow+reflection) at 1920x1080, 1M-tri scene + rough reflections (C5)" if c5
                  else "Mrays/sec (primary+shadow) at 1920x1080, 1M-tri scene; max |dpixel|")
        workloads = {"sphere1m_refl": "C5 sphere1m_refl: C4 + reflection 0.5 / roughness 0.3, 16 samples, depth 5, "
                                      "normal + parallax maps",
                     "sphere1m": "C4 sphere1m: 1,000,000 tris, 1920x1080, ssaa_factor 2 (3840x2160 rays), "
                                 "primary + shadow, octree 12/40",
                     "hair1m": "hair1m: 50k ribbon strands (1,000,000 tris), 1920x1080, ssaa_factor 2, "
                               "primary + shadow, octree 12/40 (BASELINE configs[3]'s hair scene)"}
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
            "data": f"synthetic (deterministic {args.config} scene, SURVEY.md 8(d))",
            "config": {"workload": workloads.get(args.config, args.config), "image": [W, H], "render": [rw, rh],
                       "rays_per_frame": rays, "primary_rays": primary, "shadow_rays": shadow_total,
                       "reflection_rays": refl_total, "band_rows": band, "parallelism": f"image strips x{world}",
                       "frames_in_flight": q, "world_size": world,
                       "bands": "cost-balanced lists" if balance else "interleaved b % N"},
            "kernel_ms": round(k_max, 4),
            "kernel_ms_per_rank": {"max": round(k_max, 4), "min": round(k_min, 4)},
            "first_call_s": round(t_first, 3),
            "accel_ready_s": round(t_accel, 3),
            "build_ms": {"total": round(build["build_ms"], 1),
                         **{k: round(v, 1) for k, v in zip(("octree", "cones_slabs_background", "wide_bvh_background",
                                                             "octree_upload"), build["build_split_ms"])}},
        }
        if balance:
            res["balance"] = balance
        legs = {}
        if world == 1 and not c5 and not args.no_legs:
            legs["sync"], sync_img = sync_leg(r, args, rays)
            legs["moving_camera"], mv_img, mv_scene = moving_camera_leg(r, args, pipe, frames, sc, primary)
        rl = roofline(args.config, world, (legs.get("sync") or {}).get("kernel_ms"), k_max, ms_per_step, primary)
        if rl:
            res["roofline"] = rl
        res.update(legs)
        if not args.no_check or (world == 1 and not args.no_cpu_baseline):
            base, dpx, check = cpu_leg(sc, st, img, args.cpu_threads, c5, check=not args.no_check,
                                       baseline=world == 1 and not args.no_cpu_baseline, name=args.config,
                                       extra={"sync": (sc, sync_img), "moving_camera": (mv_scene, mv_img)} if legs else None)
            if base:
                res["cpu_baseline"] = base
            if dpx is not None:
                res["max_abs_dpixel"] = dpx.pop("main")
                res["dpixel_check"] = check
                for k, v in dpx.items():
                    res[k]["max_abs_dpixel"] = v
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def sync_leg(r, args, rays):
    """The reference's synchronous call surface (utils/mainUtils.cpp:6-21, QT/mainWindowThreads.cpp:39-65):
    rt_ray_trace + rt_post_process + rt_get_image to host, one frame at a time.  Its kernel time (HIP
    events around the one launch, rt_stats.kernel_ms) is the non-overlapped per-launch duration that
    the roofline prices."""
    img = None   # the caller's image buffer, kept across frames (as a display keeps its QImage)
    for _ in range(args.warmup):
        r.ray_trace()
        r.post_process()
        img = r.get_image(img)
    kms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r.ray_trace()
        kms.append(r.stats()["kernel_ms"])
        r.post_process()
        img = r.get_image(img)
    el = time.perf_counter() - t0
    return ({"value": round(rays * args.steps / el / 1e6, 3), "unit": "Mrays/s", "ms_per_step": round(1e3 * el / args.steps, 4),
             "kernel_ms": round(float(np.mean(kms)), 4), "frames_in_flight": 1,
             "what": "rt_ray_trace + rt_post_process + rt_get_image into the caller's host buffer, one frame at a "
                     "time"}, img.ravel().copy())


def moving_camera_leg(r, args, pipe, frames, sc, primary):
    """set_camera_transform before every step (a small yaw sweep, renderer.cpp:235-241's camera
    transform): the per-camera work -- the camera's risk words (wide_risk_kernel + pack) and the heavy
    list from the previous, slightly different view -- runs inside the timed loop; frames in flight as
    the headline.  Returns the leg, the last frame and that frame's scene (camera) for the check."""
    import dataclasses
    import torch
    from raytracercpp_amd import _lib
    angles = [0.25 * (k % 8) for k in range(args.steps + args.warmup)]

    def step(k):
        r.set_camera_transform(_lib.make_transform("ry", angles[k]))
        return pipe.step()
    for k in range(args.warmup):
        step(k)
    pipe.drain()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    last = 0
    for k in range(args.warmup, args.warmup + args.steps):
        last = step(k)
    pipe.drain()
    el = time.perf_counter() - t0
    shadow, _ = r.band_counters()   # (the last frame's; the sweep changes it little)
    img = frames[last].cpu().numpy().view(np.uint32).ravel()
    sc2 = dataclasses.replace(sc)
    sc2.cam_pos, sc2.proj_inv, sc2.cam_to_world = r.get_camera_matrices()
    r.set_camera_matrices(sc.cam_pos, sc.proj_inv, sc.cam_to_world)
    rays = primary + shadow
    return ({"value": round(rays * args.steps / el / 1e6, 3), "unit": "Mrays/s", "ms_per_step": round(1e3 * el / args.steps, 4),
             "frames_in_flight": len(pipe.outs), "camera": "set_camera_transform(ry(0.25 * (k % 8) deg)) every step",
             "rays_per_frame_last": rays}, img, sc2)


def roofline(config, world, sync_kernel_ms, overlapped_kernel_ms, ms_per_step, primary):
    """The roofline object, recomputable from the files it names: unit counts of
    the RT_COUNT build (profiles/work_counts.json "gpu_executed") times bytes per unit, per
    launch (this rank's share of the frame), over the launch's HIP-event duration with no other
    frame in flight (the sync leg's rt_ray_trace launch; at N > 1, where there is no sync leg, the
    step interval).  The frames-in-flight launches overlap each other, so their duration
    (overlapped_kernel_ms) is reported beside it, not priced."""
    kernel_ms = sync_kernel_ms if sync_kernel_ms else ms_per_step
    if not os.path.exists(COUNTS_FILE):
        return None
    with open(COUNTS_FILE) as f:
        counts = json.load(f).get(config)
    ex = counts.get("gpu_executed") if counts else None
    if not ex:
        return None
    units = {"wide_node_visits": ex.get("wide_node_visits", 0), "wide_tri_tests": ex.get("wide_tri_tests", 0),
             "certificates": ex.get("wide_certificates", 0),
             "octree_kdop_tests": ex["vol_tests_whole_line"] + ex["vol_tests_segment"],
             "octree_tri_tests": ex["tri_tests_whole_line"] + ex["tri_tests_segment"], "pixels": primary}
    per = {"wide_node_visits": WIDE_NODE_BYTES, "wide_tri_tests": TRI_BYTES, "certificates": CERT_BYTES,
           "octree_kdop_tests": NODE_BYTES, "octree_tri_tests": TRI_BYTES, "pixels": PIXEL_BYTES}
    frame_bytes = sum(units[k] * per[k] for k in units)
    share = 1.0 / world
    launch_bytes = frame_bytes * share
    achieved = launch_bytes / (kernel_ms * 1e-3) / 1e9
    out = {"bound": "l1_l2_gather", "achieved": round(achieved, 1), "peak": PEAK_L2_GBS, "unit": "GB/s",
           "frac": round(achieved / PEAK_L2_GBS, 4), "traffic": None,
           "basis": "bytes the launch's traversal reads (units x bytes_per_unit, RT_COUNT build counts for the "
                    "whole frame, x 1/world) / kernel_ms: " + ("the sync leg's launch (HIP events on its stream, one "
                    "frame in flight)" if sync_kernel_ms else "the step interval") + "; peak = L2 aggregate",
           "units_per_frame": units, "bytes_per_unit": per, "bytes_per_launch": int(launch_bytes),
           "kernel_ms": round(kernel_ms, 4), "overlapped_launch_ms": round(overlapped_kernel_ms, 4),
           "counts_source": "profiles/work_counts.json [%s].gpu_executed" % config,
           "gather_ceiling": {"peak": GATHER_151MB_GBS, "unit": "GB/s", "frac": round(achieved / GATHER_151MB_GBS, 4),
                              "what": "uniformly random 1,152-B rows of a 151 MB table (MI355X_MICROARCH.md, "
                                      "Indexed rows), the guide's rate for a working set like this one's ~130 MB"},
           "per_step": {"achieved": round(launch_bytes / (ms_per_step * 1e-3) / 1e9, 1),
                        "frac": round(launch_bytes / (ms_per_step * 1e-3) / 1e9 / PEAK_L2_GBS, 4)}}
    if world == 1 and config == "sphere1m" and os.path.exists(PROFILE_SUMMARY):
        with open(PROFILE_SUMMARY) as f:
            traffic = json.load(f).get("hbm_traffic_bytes_per_launch")
        if traffic:
            out["traffic"] = int(traffic)
            hbm = traffic / (kernel_ms * 1e-3) / 1e9
            with open(PROFILE_SUMMARY) as f:
                src = json.load(f).get("source", "")
            out["hbm"] = {"bytes_per_launch": int(traffic), "achieved": round(hbm, 1), "peak": PEAK_HBM_GBS,
                          "frac": round(hbm / PEAK_HBM_GBS, 4),
                          "source": os.path.relpath(PROFILE_SUMMARY, ROOT) + " (2 x FETCH_SIZE + WRITE_SIZE) " + src}
    if "child_tests_primary" in counts:
        # SURVEY.md 8(d)'s model priced on the REFERENCE's traversal (oracle count mode): the work
        # the reference's octree walk would read, per second of this kernel -- a rate of retiring
        # the reference's work, not a bandwidth
        tests = counts["child_tests_primary"] + counts["child_tests_shadow"]
        tris = counts["tri_tests_primary"] + counts["tri_tests_shadow"]
        nbytes = NODE_BYTES * tests + TRI_BYTES * tris + PIXEL_BYTES * primary
        out["reference_traversal_equivalent"] = {
            "bytes_per_frame": nbytes, "rate_GBs": round(nbytes * share / (kernel_ms * 1e-3) / 1e9, 1)}
    return out


def cgroup_cpus():
    """CPUs the job's cgroup may use (cpu.max quota / period, cgroup v2; v1 cfs files), or None."""
    for q, per in (("/sys/fs/cgroup/cpu.max", None), ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us",
                                                         "/sys/fs/cgroup/cpu/cpu.cfs_period_us")):
        try:
            with open(q) as f:
                txt = f.read().split()
            if per is None:
                if txt[0] == "max":
                    return None
                return max(1, int(int(txt[0]) / int(txt[1])))
            quota = int(txt[0])
            if quota <= 0:
                return None
            with open(per) as f:
                return max(1, int(quota / int(f.read().split()[0])))
        except (OSError, ValueError, IndexError, ZeroDivisionError):
            continue
    return None


def all_cores():
    """Every core this process may run on (OMP_NUM_THREADS=$(nproc), as the
    reference's OpenMP loop forks, renderer.cpp:1082): the affinity mask, capped by the cgroup's
    CPU quota when one is set (threads beyond it only time-share the quota)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    q = cgroup_cpus()
    return min(aff, q) if q else aff


def cpu_info(threads):
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = None
    return {"cpu_model": model, "os_cpu_count": os.cpu_count(), "affinity_cpus": affinity,
            "cgroup_cpu_quota": cgroup_cpus(), "threads": threads}


def cpu_leg(sc, st, gpu_img, threads, c5, check=True, baseline=True, name="sphere1m", extra=None):
    """The CPU leg (rank 0, outside the timed region): the only place bench.py uses oracle/.
    * check: max |dpixel| of the GPU frame against the oracle's C restatement -- the full C4
      frame, or for C5 the row pairs of C5_CHECK_ROWS (oracle.render_row_set, downscaled);
    * baseline (N = 1): the reference itself (oracle/_ref/libref_harness.so: the reference's
      own compiled BVH / triangle / vector code under the harness's OpenMP schedule(dynamic)
      row loop, renderer.cpp:1082) on a bounded row sample, one warm-up pass then the median of
      5; the port's rate (oracle.c) beside it, or as the baseline when the
      reference library was not built."""
    from oracle.bindings import Oracle, RefHarness, RefHarnessShipped
    from raytracercpp_amd.scenes import C5_CHECK_ROWS   # the 16 output rows of test_c5_full_config_matches_oracle
    if not threads:
        threads = all_cores()
    env_threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    rw, rh = st.render_size()
    W = st.image_width
    dpx, check_desc, port = None, None, None
    o = Oracle(sc, st)
    if check or baseline:
        out_rows = (list(C5_CHECK_ROWS) if c5 else
                    list(range(CHECK_STRIDE // 2, st.image_height, CHECK_STRIDE)) if name in SAMPLED_CHECK else None)
        f = st.ssaa_factor if st.enable_ssaa else 1
        rows = None if out_rows is None else [f * r + k for r in out_rows for k in range(f)]

        def oracle_frame(orc):
            """(the oracle's output rows to compare: the whole frame or the sampled rows, its run)"""
            if rows is None:
                rr = orc.render_rows(nthreads=threads)
                return (Oracle.downscale(rr.argb, rw, rh, f) if f > 1 else rr.argb), rr
            rr = orc.render_row_set(rows, nthreads=threads)
            return (Oracle.downscale(rr.argb, rw, len(rows), f) if f > 1 else rr.argb).reshape(len(out_rows), W), rr

        def gpu_rows(img):
            return np.asarray(img) if out_rows is None else np.asarray(img).reshape(-1, W)[out_rows]
        ref, res = oracle_frame(o)
        if out_rows is not None:
            check_desc = (f"output rows {out_rows} (internal rows {rows})" if c5 else
                          f"every {CHECK_STRIDE}th output row ({len(out_rows)} rows from {out_rows[0]}, their "
                          f"{len(rows)} internal rows)") + " vs oracle.c, SSAA applied"
        else:
            check_desc = "whole frame vs oracle.c (the C restatement), SSAA applied"
        port_rays = res.counters["primary_rays"] + res.counters["shadow_rays"] + res.counters["reflection_rays"]
        if check:
            dpx = {"main": max_abs_dpixel(gpu_rows(gpu_img), ref)}
            for k, (sck, imgk) in (extra or {}).items():
                # the legs' last frames: the same scene (sync) against the same oracle frame, or the
                # moved camera's own oracle frame
                dpx[k] = max_abs_dpixel(gpu_rows(imgk), ref if sck is sc else oracle_frame(Oracle(sck, st))[0])
        port = {"value": round(port_rays / res.seconds / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
                "sample": ("the check rows" if out_rows is not None else f"full frame ({rw}x{rh} primary + "
                           f"{res.counters['shadow_rays']} shadow rays)") + f" in {res.seconds:.2f} s, oracle.c OpenMP x{threads}"}
    if not baseline:
        return None, dpx, check_desc
    if not RefHarness.available():
        port.update(cpu_info(threads))
        return port, dpx, check_desc
    stride = 128 if c5 else 2

    def ref_rate(nthr, H=RefHarness):
        H.set_threads(nthr)
        passes = []
        rr = None
        for i in range(6):   # one warm-up pass, then 5 timed
            rr = H.render_row_sample(sc, st, stride // 2, rh // stride, stride)
            if i:
                passes.append(rr.seconds)
        sec = float(np.median(passes))
        c = rr.counters
        rays = c["primary_rays"] + c["shadow_rays"] + (c["reflection_rays"] if c5 else 0)
        return rays / sec / 1e6, passes, c

    rate, passes, c = ref_rate(threads)
    # the box's default team (OMP_NUM_THREADS, 16 on the GPU pool) beside it, when it differs
    alt = None
    if env_threads and env_threads != threads:
        alt = {"threads": env_threads, "value": round(ref_rate(env_threads)[0], 3)}
    RefHarness.set_threads(threads)
    base = {"value": round(rate, 3), "unit": "Mrays/s", "cores": threads, "kind": "reference",
            "sample": f"every {stride}th internal row of the {'C5' if c5 else 'C4'} frame ({rh // stride} rows x {rw}: "
                      f"{c['primary_rays']} primary + {c['shadow_rays']} shadow"
                      + (f" + {c['reflection_rays']} reflection" if c5 else "") +
                      f" rays, octree build excluded), reference TUs + OpenMP x{threads}; median of 5 passes "
                      f"after one warm-up ({', '.join(f'{p:.3f}' for p in passes)} s)",
            "port_value": port["value"] if port else None}
    base["flags"] = "g++ -O3 -ffp-contract=off -fopenmp (oracle/Makefile REF_CXXFLAGS: the parity build)"
    if RefHarnessShipped.available():
        # the same TUs at the reference's shipped optimisation flags (tp2/CMakeLists.txt:105-117, made
        # portable): the baseline a user of the reference would time
        srate, spasses, _ = ref_rate(threads, RefHarnessShipped)
        base["shipped_flags"] = {"value": round(srate, 3), "unit": "Mrays/s", "cores": threads,
                                 "flags": "g++ -O3 -march=x86-64-v3 -mfma -fopenmp, default FP contraction "
                                          "(oracle/Makefile ref_v3)",
                                 "passes_s": [round(p, 3) for p in spasses]}
    if alt:
        base["omp_num_threads_env"] = alt
    base.update(cpu_info(threads))
    return base, dpx, check_desc


def dry_run(args, world):
    """--dry-run: gloo ranks, each 'renders' its bands as a pattern keyed by the global row, frames in
    flight through strips.FramePipeline, the same flat all-gather and in-step re-assembly on rank 0 as
    the GPU path; after the warm-up, the cost-balanced band lists from synthetic band costs (a costly
    cluster of bands, as the sphere's silhouette), summed over the ranks with the same all-reduce; rank
    0 checks the last frame against the pattern computed whole."""
    import torch
    import torch.distributed as dist
    from raytracercpp_amd import scenes
    from raytracercpp_amd.strips import FramePipeline, assign_bands, gather_index, list_rows, num_bands, rank_rows
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
        world = dist.get_world_size()
    _, st = scenes.CONFIGS[args.config]()
    W, H = st.image_width, st.image_height
    band = args.band_rows
    nb = num_bands(H, band)
    q = max(1, args.inflight)

    def make_pipe(lists):
        nloc = len(lists[0]) * band if lists is not None else len(rank_rows(H, band, rank, world))
        rows = list_rows(lists[rank], H, band, nloc // band) if lists is not None else rank_rows(H, band, rank, world)
        outs = [torch.zeros((nloc, W), dtype=torch.int32) for _ in range(q)]
        frames = [torch.zeros((H, W), dtype=torch.int32) for _ in range(q)]
        idx = torch.as_tensor(gather_index(H, band, world, nloc, lists))

        def render(o, _stream):
            o.copy_(torch.from_numpy(pattern_strip(rows, W)))
        if world == 1:
            return FramePipeline(render, outs, 1), [o[:H] for o in outs], rows
        asm = (lambda i, flat: torch.index_select(flat, 0, idx, out=frames[i])) if rank == 0 else None
        return FramePipeline(render, outs, world, None, dist, assemble=asm), frames, rows
    pipe, frames, rows = make_pipe(None)
    for _ in range(args.warmup):
        pipe.step()
    pipe.drain()
    balanced = False
    if world > 1 and args.balance:
        mine = np.zeros(nb)
        b = np.unique(rows[rows >= 0] // band)
        mine[b] = 1.0 + 40.0 * ((b > 0.45 * nb) & (b < 0.55 * nb))
        ct = torch.as_tensor(mine)
        dist.all_reduce(ct)
        pipe, frames, rows = make_pipe(assign_bands(ct.numpy(), world))
        balanced = True
        for _ in range(args.warmup):
            pipe.step()
        pipe.drain()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    last = 0
    for _ in range(args.steps):
        last = pipe.step()
    pipe.drain()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if rank == 0:
        frame = frames[last].numpy()
        expect = pattern_strip(np.arange(H), W)
        ms = 1e3 * elapsed / max(1, args.steps)
        print(json.dumps({"metric": "dry run: strip layout + gloo all-gather + re-assembly (no rendering)",
                          "value": 0.0, "unit": "Mrays/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True,
                          "scaling": "strong", "vs_baseline": None, "dtype": "u32", "data": "synthetic pattern strips",
                          "config": {"workload": "dry run", "image": [W, H], "band_rows": band,
                                     "parallelism": f"image strips x{world}", "world_size": world,
                                     "bands": "cost-balanced lists" if balanced else "interleaved b % N"},
                          "dry_run": True, "max_abs_dpixel": max_abs_dpixel(frame, expect)}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
