#!/bin/bash
# Two quick rocprofv3 PMC passes over a short C4 bench (counters only, one run per pass).
# Usage: bash tools/pmc_quick.sh <outdir> [bench args...]   (RT_LIB_PATH selects a variant library)
set -u
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS \
    --output-format csv -d $OUT/p1 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-check "$@" > $OUT/p1.log 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/p2 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-check "$@" > $OUT/p2.log 2>&1 || exit 2
