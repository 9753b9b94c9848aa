#!/bin/bash
# r05: the plain kernel without spills (deep retry's record by value, LDS-held pixel state): the GPU
# suite, bench by heavy group, WRITE_SIZE / FETCH_SIZE, strips
set -e
O=gpurun_out/r05n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1
tail -2 $O/pytest_gpu.log
for g in 0 4 0 4; do
  RT_HEAVY_GROUP=$g timeout -k 10 240 python bench.py --no-cpu-baseline > $O/bench_g$g.log 2>&1
  grep -h '^{' $O/bench_g$g.log | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print('G=$g', d['value'], d['ms_per_step'], d.get('kernel_ms'), d.get('max_abs_dpixel'))"
done
RT_HEAVY_GROUP=4 timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-check > $O/pmc_write.log 2>&1
RT_HEAVY_GROUP=4 timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-check > $O/pmc_fetch.log 2>&1
python tools/pmc_dispatch.py $O/pmc_write $O/pmc_fetch
RT_HEAVY_GROUP=4 timeout -k 10 300 python tools/strip_scaling.py --ranks 1 2 4 8 --steps 30 --all-ranks > $O/strips_g4.log 2>&1
grep bound $O/strips_g4.log
