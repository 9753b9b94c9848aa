set -u
export TMPDIR=/tmp
O=gpurun_out/p40
mkdir -p $O
M="all rays miss (sphere behind the camera)"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_miss -o run -- python3 tools/phase_split.py "$M" > $O/trace_miss.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $O/pmc_miss -o run -- python3 tools/phase_split.py "$M" > $O/pmc_miss.log 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $O/pmc_hit -o run -- python3 tools/phase_split.py "primary+shadow" > $O/pmc_hit.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_INSTS_SMEM --output-format csv -d $O/pmc2_hit -o run -- python3 tools/phase_split.py "primary+shadow" > $O/pmc2_hit.log 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_LDS SQ_INSTS_SMEM --output-format csv -d $O/pmc2_miss -o run -- python3 tools/phase_split.py "$M" > $O/pmc2_miss.log 2>&1 || exit 5
