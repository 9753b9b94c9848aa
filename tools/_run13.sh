set -u
export TMPDIR=/tmp
OUT=gpurun_out/prof_r02b
mkdir -p $OUT
pass() {
    local name=$1; shift
    timeout -k 10 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/pmc_$name -o run -- \
        python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/pmc_$name.log 2>&1
}
pass ta TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES || exit 2
pass tcp TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCP_TA_ADDR_STALL_CYCLES || exit 3
pass sqc SQC_ICACHE_MISSES SQC_ICACHE_REQ SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_LEVEL_WAVES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit 4
pass sq4 SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_WAIT_ANY SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE || exit 5
