#!/bin/bash
# Runs on the GPU box: kernel-trace stats + PMC passes (one rocprofv3 run per pass,
# counters never combined with sys/runtime traces) of bench.py.
# Usage: bash tools/profile_gpu.sh <tag> [bench args...]   -> gpurun_out/prof_<tag>/...
#   e.g. bash tools/profile_gpu.sh r04c5 --config sphere1m_refl
set -u
TAG=${1:-r01}
shift || true
EXTRA="$*"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-check --no-legs $EXTRA > $OUT/trace.log 2>&1 || exit 1
pass() {   # pass <name> <counters...>
    local name=$1; shift
    timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $OUT/pmc_$name -o run -- \
        python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-check --no-legs $EXTRA > $OUT/pmc_$name.log 2>&1
}
pass fetch FETCH_SIZE || exit 2
pass write WRITE_SIZE || exit 3
pass tcc TCC_HIT_sum TCC_MISS_sum || exit 4
pass sq SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit 5
pass sq2 SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS || exit 6
pass sq3 SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH SQ_INSTS_VALU GRBM_GUI_ACTIVE || exit 7
pass mem TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_LATENCY_sum GRBM_GUI_ACTIVE || exit 8
find $OUT -name "*.csv" | sort
