"""Per-dispatch averages of the PMC counters rocprofv3 collected for one kernel.
    python tools/pmc_kernel.py <dir with run_counter_collection.csv ...> [kernel substring]"""
import collections, csv, glob, os, sys

def collect(d, sub="ray_trace_kernel"):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if sub in r["Kernel_Name"]:
                agg[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in agg.items()}

if __name__ == "__main__":
    for k, v in sorted(collect(sys.argv[1], *(sys.argv[2:3])).items()):
        print(f"{k:40s} {v:16.1f}")
