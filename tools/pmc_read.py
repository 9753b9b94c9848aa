"""Per-dispatch sums of the counters tools/pmc_quick.sh collected for one kernel (default: the plain
ray_trace_kernel): python tools/pmc_read.py <outdir> [kernel substring]"""
import collections
import csv
import glob
import sys

out = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "ray_trace_kernel"
for f in sorted(glob.glob(f"{out}/p*/**/run_counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            agg[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for k, v in sorted(agg.items()):
        vals = list(v.values())
        print(f"{k:24s} {len(vals)} dispatches, last: {vals[-1]:.4g}")
