set -u
for v in base batch4 sh32 base batch4 sh32; do
echo "== $v" >> gpurun_out/r02_phase39.log
RT_LIB_PATH=_variants/librt_$v.so timeout -k 10 200 python tools/phase_split.py "primary+shadow" "all rays miss (sphere behind the camera)" >> gpurun_out/r02_phase39.log 2>&1
done
