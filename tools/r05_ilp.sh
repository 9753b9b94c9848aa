#!/bin/bash
# r05: lane groups with the children's tests interleaved (W_GROUP_ILP=1 variant) against the default
set -e
O=gpurun_out/r05i
mkdir -p $O
RT_LIB_PATH=_variants/librt_ilp.so timeout -k 10 300 python tools/group_probe.py sphere1m 16 > $O/group_probe_ilp.log 2>&1
grep "G=" $O/group_probe_ilp.log
RT_LIB_PATH=_variants/librt_ilp.so RT_HEAVY_GROUP=4 timeout -k 10 240 python bench.py --no-cpu-baseline > $O/bench_ilp.log 2>&1
grep -h '^{' $O/bench_ilp.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('ilp G=4', d['value'], d['ms_per_step'], d.get('kernel_ms'), d.get('max_abs_dpixel'))"
RT_LIB_PATH=_variants/librt_ilp.so RT_HEAVY_GROUP=4 timeout -k 10 300 python tools/strip_scaling.py --ranks 1 8 --steps 30 --all-ranks > $O/strips_ilp.log 2>&1
grep bound $O/strips_ilp.log
