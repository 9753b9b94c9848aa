#!/bin/bash
# r05: C5 by the reflection queries' deferral threshold (RT_REFL_DEFER, loop iterations)
set -e
O=gpurun_out/r05d
mkdir -p $O
( while sleep 30; do echo "[tick] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
for k in 48 24 32 64 16 48; do
  RT_REFL_DEFER=$k timeout -k 10 600 python bench.py --config sphere1m_refl --steps 6 --warmup 2 --no-cpu-baseline --no-check > $O/bench_$k.log 2>&1
  grep -h '^{' $O/bench_$k.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('defer $k', d['value'], d['ms_per_step'])"
done
