"""Summarise a tools/profile_gpu.sh run into profiles/<tag>/: kernel stats csv +
summary.json (per-launch PMC averages of the ray-trace kernel, HBM traffic per
MI355X_MICROARCH.md: bytes = 2 x FETCH_SIZE[KB] x 1024 + WRITE_SIZE[KB] x 1024).
   python tools/profile_summary.py gpurun_out/prof_r01 profiles/r01"""
import collections, csv, glob, json, os, shutil, sys

src, dst = sys.argv[1], sys.argv[2]
os.makedirs(dst, exist_ok=True)
out = {"kernels": {}, "pmc_ray_trace_kernel": {}}
stats = glob.glob(f"{src}/trace/**/run_kernel_stats.csv", recursive=True)
if stats:
    shutil.copy(stats[0], os.path.join(dst, "kernel_stats.csv"))
    for r in csv.DictReader(open(stats[0])):
        out["kernels"][r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                     "total_ns": float(r["TotalDurationNs"]), "pct": float(r["Percentage"])}
for f in sorted(glob.glob(f"{src}/pmc_*/**/run_counter_collection.csv", recursive=True)):
    # per dispatch: the sum over the rows of one dispatch (instances / dimensions), then
    # the mean over the dispatches of the ray_trace_kernel instance launched most often (the
    # steady-state frame; the first frame of a scene may take the exact octree instance while
    # the wide BVH is built in the background)
    agg = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    for r in csv.DictReader(open(f)):
        if "ray_trace_kernel" in r["Kernel_Name"]:
            agg[r["Kernel_Name"]][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    if agg:
        main = max(agg, key=lambda n: max(len(v) for v in agg[n].values()))
        out["pmc_kernel_name"] = main
        for k, v in agg[main].items():
            out["pmc_ray_trace_kernel"][k] = sum(v.values()) / len(v)
    name = f.split(os.sep)[-3] if "pmc_" in f.split(os.sep)[-3] else os.path.basename(os.path.dirname(f))
    shutil.copy(f, os.path.join(dst, f"{name}_counters.csv"))
p = out["pmc_ray_trace_kernel"]
if "FETCH_SIZE" in p and "WRITE_SIZE" in p:
    out["hbm_read_bytes_per_launch"] = 2 * p["FETCH_SIZE"] * 1024
    out["hbm_write_bytes_per_launch"] = p["WRITE_SIZE"] * 1024
    out["hbm_traffic_bytes_per_launch"] = out["hbm_read_bytes_per_launch"] + out["hbm_write_bytes_per_launch"]
if "TCC_HIT_sum" in p:
    out["l2_hit_rate"] = p["TCC_HIT_sum"] / max(1.0, p["TCC_HIT_sum"] + p["TCC_MISS_sum"])
if "SQ_THREAD_CYCLES_VALU" in p and "SQ_ACTIVE_INST_VALU" in p:
    out["valu_lane_utilisation"] = p["SQ_THREAD_CYCLES_VALU"] / (64.0 * p["SQ_ACTIVE_INST_VALU"])
if "SQ_INSTS_VALU" in p and "GRBM_GUI_ACTIVE" in p:
    # VALU issue: a wave64 VALU instruction occupies its SIMD's issue for 2 cycles
    # (MI355X_MICROARCH.md); 1024 SIMDs over the kernel's GPU-busy cycles.  GRBM_GUI_ACTIVE
    # comes summed over the 8 XCDs (8x the kernel's duration in cycles)
    out["grbm_cycles_per_xcd"] = p["GRBM_GUI_ACTIVE"] / 8.0
    out["valu_issue_fraction"] = 2.0 * p["SQ_INSTS_VALU"] / (1024.0 * out["grbm_cycles_per_xcd"])
if "TD_TD_BUSY_sum" in p and "GRBM_GUI_ACTIVE" in p:
    # 256 TD / TA instances (one per CU)
    out["td_busy_fraction"] = p["TD_TD_BUSY_sum"] / 256.0 / (p["GRBM_GUI_ACTIVE"] / 8.0)
    out["td_stall_on_l1_fraction"] = p.get("TD_TC_STALL_sum", 0.0) / 256.0 / (p["GRBM_GUI_ACTIVE"] / 8.0)
if "TA_BUSY_avr" in p and "GRBM_GUI_ACTIVE" in p:
    out["ta_busy_fraction"] = p["TA_BUSY_avr"] / (p["GRBM_GUI_ACTIVE"] / 8.0)
if "SQ_WAIT_ANY" in p and "SQ_WAVE_CYCLES" in p:
    out["wave_wait_fraction"] = p["SQ_WAIT_ANY"] / p["SQ_WAVE_CYCLES"]
traces = glob.glob(f"{src}/trace/**/run_kernel_trace.csv", recursive=True)
if traces:
    # per-instance resources as dispatched (scratch bytes per lane, VGPRs)
    res = {}
    for r in csv.DictReader(open(traces[0])):
        if "ray_trace_kernel" in r["Kernel_Name"] and r["Kernel_Name"] not in res:
            res[r["Kernel_Name"]] = {"scratch_bytes_per_lane": int(r["Scratch_Size"]), "vgprs": int(r["VGPR_Count"]),
                                     "sgprs": int(r["SGPR_Count"]), "grid": int(r["Grid_Size_X"])}
    out["ray_trace_resources"] = res
json.dump(out, open(os.path.join(dst, "summary.json"), "w"), indent=1, sort_keys=True)
print(json.dumps({k: v for k, v in out.items() if k != "kernels"}, indent=1))
