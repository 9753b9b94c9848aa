set -u
mkdir -p gpurun_out
for cfg in "r4 24" "r5 24" "r4 25" "r5 25" "r4 24" "r5 25"; do
set -- $cfg
RT_LIB_PATH=_variants/librt_$1.so RT_REFL_CHUNK_LOG2=$2 timeout -k 10 300 python bench.py --config sphere1m_refl --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r02_c5_96_$1_$2.log 2>&1 || exit 4
echo $1 $2 $(grep -h '^{' gpurun_out/r02_c5_96_$1_$2.log | grep -o '"ms_per_step": [0-9.]*')
done
