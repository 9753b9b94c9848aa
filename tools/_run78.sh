set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/c5prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5prof/trace -o run -- python3 bench.py --config sphere1m_refl --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/c5prof/bench.log 2>&1 || { tail gpurun_out/c5prof/bench.log; exit 1; }
f=$(find gpurun_out/c5prof/trace -name "run_kernel_stats.csv" | head -1)
cp $f gpurun_out/c5prof/kernel_stats.csv
python3 -c "
import csv
rows=list(csv.DictReader(open('gpurun_out/c5prof/kernel_stats.csv')))
for r in sorted(rows,key=lambda r:-float(r['TotalDurationNs']))[:14]:
    print(r['Name'][:90], r['Calls'], round(float(r['TotalDurationNs'])/1e6,2),'ms', r['Percentage'])
"
grep '^{' gpurun_out/c5prof/bench.log | cut -c1-400
