#!/bin/bash
# r05: lane-group device queries (parity + timing of the costliest tiles), the plain kernel's LDS stash
# (bench + WRITE_SIZE)
set -e
O=gpurun_out/r05s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_wide.py -k "lane_groups" > $O/pytest_groups.log 2>&1
tail -1 $O/pytest_groups.log
timeout -k 10 300 python tools/group_probe.py sphere1m 16 > $O/group_probe.log 2>&1
cat $O/group_probe.log
timeout -k 10 240 python bench.py > $O/bench.log 2>&1
grep -h '^{' $O/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d['value'], d['ms_per_step'], d.get('kernel_ms'), d.get('max_abs_dpixel'))"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-check > $O/pmc_write.log 2>&1
python tools/profile_summary.py $O $O/sum > /dev/null
python -c "import json; d=json.load(open('$O/sum/summary.json')); print('write MB/launch', d.get('hbm_write_bytes_per_launch', 0)/1e6)"
RT_PLAIN_OCTREE=0 timeout -k 10 300 python tools/first_frame.py sphere1m 3 > $O/first_frame_general.log 2>&1
RT_PLAIN_OCTREE=1 timeout -k 10 300 python tools/first_frame.py sphere1m 3 > $O/first_frame_plain.log 2>&1
cat $O/first_frame_general.log $O/first_frame_plain.log | grep '^{'
