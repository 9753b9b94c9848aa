#!/bin/bash
# r05: C4 by frames in flight (bench.py --inflight)
set -e
O=gpurun_out/r05if
mkdir -p $O
for q in 2 3 4 1 2; do
  timeout -k 10 300 python bench.py --inflight $q --no-cpu-baseline --no-check > $O/bench_q$q.log 2>&1
  grep -h '^{' $O/bench_q$q.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('inflight $q', d['value'], d['ms_per_step'], d.get('kernel_ms'))"
done
