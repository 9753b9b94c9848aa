#!/bin/bash
# r05: the deferral threshold again at chunks of 2^27 slots
set -e
O=gpurun_out/r05cd
mkdir -p $O
( while sleep 30; do echo "[tick] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
run() {   # name defer
  RT_REFL_DEFER=$2 timeout -k 10 600 python bench.py --config sphere1m_refl --steps 6 --warmup 2 --no-cpu-baseline --no-check > $O/bench_$1.log 2>&1
  grep -h '^{' $O/bench_$1.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('$1', d['value'], d['ms_per_step'])"
}
run d32 32
run d24 24
run d20 20
run d40 40
run d32b 32
