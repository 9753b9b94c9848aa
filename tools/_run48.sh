set -u
for v in ph phnopf; do
echo "== $v" >> gpurun_out/r02_phase48.log
RT_DEBUG_WAVES=1 RT_LIB_PATH=_variants/librt_$v.so timeout -k 10 200 python tools/phase_time.py >> gpurun_out/r02_phase48.log 2>&1
RT_DEBUG_WAVES=1 RT_LIB_PATH=_variants/librt_$v.so timeout -k 10 200 python tools/phase_time.py --miss >> gpurun_out/r02_phase48.log 2>&1
done
