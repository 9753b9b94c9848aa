set -u
mkdir -p gpurun_out
for v in r4 r5 r6; do
RT_LIB_PATH=_variants/librt_$v.so timeout -k 10 300 python bench.py --config sphere1m_refl --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r02_c5_92_$v.log 2>&1 || exit 4
echo $v $(grep -h '^{' gpurun_out/r02_c5_92_$v.log | grep -o '"ms_per_step": [0-9.]*')
done
