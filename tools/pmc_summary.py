"""Average PMC counters per ray_trace_kernel dispatch from rocprofv3 csv dirs."""
import csv, collections, glob, sys
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/run_counter_collection.csv", recursive=True):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if "ray_trace_kernel" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in sorted(agg.items()):
            print(f"{k:32s} {sum(v)/len(v):20.1f}   (n={len(v)})")
