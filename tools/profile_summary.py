"""Summarise a tools/profile_gpu.sh run into profiles/<tag>/: kernel stats csv + summary.json.

For every kernel whose name contains one of the given substrings (default: ray_trace_kernel), the
per-launch PMC averages and the derived fields: HBM traffic per MI355X_MICROARCH.md (bytes = 2 x
FETCH_SIZE[KB] x 1024 + WRITE_SIZE[KB] x 1024), L2 hit rate, VALU issue and lane utilisation, TA /
TD busy, the waves' waiting fraction; plus the dispatch resources (scratch, VGPRs) from the kernel
trace.  The ray-trace kernel's fields stay at the top level (pmc_ray_trace_kernel, hbm_*, ...).
   python tools/profile_summary.py gpurun_out/prof_r05 profiles/r05 [substring ...]"""
import collections, csv, glob, json, os, shutil, sys

src, dst = sys.argv[1], sys.argv[2]
subs = sys.argv[3:] or ["ray_trace_kernel"]
os.makedirs(dst, exist_ok=True)
out = {"kernels": {}, "pmc_ray_trace_kernel": {}, "pmc_per_kernel": {}}
stats = glob.glob(f"{src}/trace/**/run_kernel_stats.csv", recursive=True)
if stats:
    shutil.copy(stats[0], os.path.join(dst, "kernel_stats.csv"))
    for r in csv.DictReader(open(stats[0])):
        out["kernels"][r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                     "total_ns": float(r["TotalDurationNs"]), "pct": float(r["Percentage"])}


def derive(p):
    d = {}
    if "FETCH_SIZE" in p and "WRITE_SIZE" in p:
        d["hbm_read_bytes_per_launch"] = 2 * p["FETCH_SIZE"] * 1024
        d["hbm_write_bytes_per_launch"] = p["WRITE_SIZE"] * 1024
        d["hbm_traffic_bytes_per_launch"] = d["hbm_read_bytes_per_launch"] + d["hbm_write_bytes_per_launch"]
    if "TCC_HIT_sum" in p:
        d["l2_hit_rate"] = p["TCC_HIT_sum"] / max(1.0, p["TCC_HIT_sum"] + p["TCC_MISS_sum"])
    if "SQ_THREAD_CYCLES_VALU" in p and "SQ_ACTIVE_INST_VALU" in p:
        d["valu_lane_utilisation"] = p["SQ_THREAD_CYCLES_VALU"] / (64.0 * p["SQ_ACTIVE_INST_VALU"])
    if "GRBM_GUI_ACTIVE" in p:
        # GRBM_GUI_ACTIVE comes summed over the 8 XCDs (8x the kernel's duration in cycles)
        d["grbm_cycles_per_xcd"] = p["GRBM_GUI_ACTIVE"] / 8.0
        if "SQ_INSTS_VALU" in p:
            # a wave64 VALU instruction occupies its SIMD's issue for 2 cycles (MI355X_MICROARCH.md); 1024 SIMDs
            d["valu_issue_fraction"] = 2.0 * p["SQ_INSTS_VALU"] / (1024.0 * d["grbm_cycles_per_xcd"])
        if "TD_TD_BUSY_sum" in p:   # 256 TD / TA instances (one per CU)
            d["td_busy_fraction"] = p["TD_TD_BUSY_sum"] / 256.0 / d["grbm_cycles_per_xcd"]
            d["td_stall_on_l1_fraction"] = p.get("TD_TC_STALL_sum", 0.0) / 256.0 / d["grbm_cycles_per_xcd"]
        if "TA_BUSY_avr" in p:
            d["ta_busy_fraction"] = p["TA_BUSY_avr"] / d["grbm_cycles_per_xcd"]
    if "SQ_WAIT_ANY" in p and "SQ_WAVE_CYCLES" in p:
        d["wave_wait_fraction"] = p["SQ_WAIT_ANY"] / p["SQ_WAVE_CYCLES"]
    if "SQ_INSTS_VALU" in p and "SQ_WAVES" in p and p["SQ_WAVES"] > 0:
        d["valu_insts_per_wave"] = p["SQ_INSTS_VALU"] / p["SQ_WAVES"]
    return d


# per counter file: per dispatch, the sum over the rows of one dispatch (instances / dimensions); per
# kernel, the mean over its dispatches.  For the ray-trace kernel, the instance launched most often (the
# steady-state frame; the first frame of a scene may take the exact octree instance)
per = collections.defaultdict(dict)
for f in sorted(glob.glob(f"{src}/pmc_*/**/run_counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    for r in csv.DictReader(open(f)):
        if any(s in r["Kernel_Name"] for s in subs):
            agg[r["Kernel_Name"]][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for kname, counters in agg.items():
        for k, v in counters.items():
            per[kname][k] = sum(v.values()) / len(v)
    rt = [n for n in agg if "ray_trace_kernel" in n]
    if rt:
        main = max(rt, key=lambda n: max(len(v) for v in agg[n].values()))
        out["pmc_kernel_name"] = main
        for k, v in agg[main].items():
            out["pmc_ray_trace_kernel"][k] = sum(v.values()) / len(v)
    name = f.split(os.sep)[-3] if "pmc_" in f.split(os.sep)[-3] else os.path.basename(os.path.dirname(f))
    if os.path.getsize(f) < (1 << 20):   # (a C5 run's passes hold ~10k dispatches: kept in gpurun_out only)
        shutil.copy(f, os.path.join(dst, f"{name}_counters.csv"))
out.update(derive(out["pmc_ray_trace_kernel"]))
for kname, p in per.items():
    out["pmc_per_kernel"][kname] = dict(counters=p, **derive(p))
traces = glob.glob(f"{src}/trace/**/run_kernel_trace.csv", recursive=True)
if traces:
    # per-instance resources as dispatched (scratch bytes per lane, VGPRs), and each kernel's launches
    res = {}
    durations = collections.defaultdict(list)
    for r in csv.DictReader(open(traces[0])):
        n = r["Kernel_Name"]
        if any(s in n for s in subs):
            durations[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
            if n not in res:
                res[n] = {"scratch_bytes_per_lane": int(r["Scratch_Size"]), "vgprs": int(r["VGPR_Count"]),
                          "sgprs": int(r["SGPR_Count"]), "grid": int(r["Grid_Size_X"])}
    out["ray_trace_resources"] = {k: v for k, v in res.items() if "ray_trace_kernel" in k}
    out["resources"] = res
    out["launch_ms"] = {k: {"n": len(v), "max": round(max(v), 4), "mean": round(sum(v) / len(v), 4),
                            "last": [round(x, 4) for x in v[-6:]]} for k, v in durations.items()}
json.dump(out, open(os.path.join(dst, "summary.json"), "w"), indent=1, sort_keys=True)
print(json.dumps({k: v for k, v in out.items() if k not in ("kernels", "pmc_per_kernel")}, indent=1))
