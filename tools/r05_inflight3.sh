#!/bin/bash
# r05: the default bench lines (three frames in flight) for C4 and C5, with their checks
set -e
O=gpurun_out/r05if3
mkdir -p $O
( while sleep 30; do echo "[tick] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python bench.py > $O/bench_c4.json.log 2>&1
grep -h '^{' $O/bench_c4.json.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('C4', d['value'], d['ms_per_step'], d.get('kernel_ms'), d.get('max_abs_dpixel'), d['roofline'].get('achieved'), d['roofline'].get('frac'), d['config'].get('frames_in_flight'))"
timeout -k 10 600 python bench.py --config sphere1m_refl --steps 6 --warmup 2 --no-cpu-baseline > $O/bench_c5.json.log 2>&1
grep -h '^{' $O/bench_c5.json.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('C5', d['value'], d['ms_per_step'], d.get('max_abs_dpixel'), d['config'].get('frames_in_flight'))"
timeout -k 10 300 python bench.py > $O/bench_c4b.json.log 2>&1
grep -h '^{' $O/bench_c4b.json.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('C4', d['value'], d['ms_per_step'], d.get('kernel_ms'), d.get('max_abs_dpixel'))"
