#!/bin/bash
# One rocprofv3 PMC pass (counters only, kernel-trace not combined with sys/runtime traces) over bench.py.
# Usage: bash tools/pmc.sh <outdir> <counter> [<counter> ...]
set -u
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d $OUT -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/run.log 2>&1
