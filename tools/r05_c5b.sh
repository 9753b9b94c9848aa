#!/bin/bash
# r05: C5 with the reflection trace in line (octree fallback by value) -- parity tests of the reflection
# engine, the C5 bench line
set -e
O=gpurun_out/r05c5c
mkdir -p $O
( while sleep 30; do echo "[tick] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 400 --timeout-method thread -k "refl or c5 or trace_ray" > $O/pytest_refl.log 2>&1
tail -1 $O/pytest_refl.log
timeout -k 10 600 python bench.py --config sphere1m_refl --steps 6 --warmup 2 --no-cpu-baseline > $O/bench_c5.json.log 2>&1
grep -h '^{' $O/bench_c5.json.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('C5', d['value'], d['ms_per_step'], d.get('kernel_ms'), d.get('max_abs_dpixel'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --config sphere1m_refl --steps 3 --warmup 1 --no-cpu-baseline --no-check > $O/trace.log 2>&1
python -c "
import csv,glob
f=glob.glob('$O/trace/**/run_kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:6]: print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us', r['Percentage'])"
