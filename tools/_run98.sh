set -u
mkdir -p gpurun_out
for b in 8 4 5 8 4 5; do
RT_BLOCKS_PER_CU=$b timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/r02_bench98_$b.log 2>&1 || exit 2
echo $b $(grep -h '^{' gpurun_out/r02_bench98_$b.log | grep -o '"value": [0-9.]*')
done
RT_BLOCKS_PER_CU=4 timeout -k 10 200 python tools/strip_scaling.py --ranks 1 8 --inflight 2 > gpurun_out/r02_strips98.log 2>&1 || exit 3
grep -h '"rank": 0' gpurun_out/r02_strips98.log | cut -c 1-90
