"""Per-dispatch values of single-counter rocprofv3 --pmc passes (KB counters shown in MB), the trace kernels
only:  python tools/pmc_dispatch.py gpurun_out/<dir>/pmc_write [more pass dirs]"""
import collections, csv, glob, sys

for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if "ray_trace" in r["Kernel_Name"] or "refl_" in r["Kernel_Name"]:
                agg[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])][r["Dispatch_Id"]] += float(r["Counter_Value"])
        for (k, c), v in sorted(agg.items()):
            print(f"{d}: {k} {c} per dispatch (MB):", [round(x / 1024, 1) for x in v.values()])
