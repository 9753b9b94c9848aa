#!/bin/bash
# r05: C5 by the reflection engine's chunk size (RT_REFL_CHUNK_LOG2 sample slots per chunk)
set -e
O=gpurun_out/r05chunk
mkdir -p $O
( while sleep 30; do echo "[tick] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
run() {   # name log2
  RT_REFL_CHUNK_LOG2=$2 timeout -k 10 600 python bench.py --config sphere1m_refl --steps 6 --warmup 2 --no-cpu-baseline --no-check > $O/bench_$1.log 2>&1
  grep -h '^{' $O/bench_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('$1', d['value'], d['ms_per_step'])"
}
run c25 25
run c24 24
run c26 26
run c27 27
run c25b 25
