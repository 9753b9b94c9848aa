set -u
mkdir -p gpurun_out
for v in w4 bq8 w4 bq8; do
RT_LIB_PATH=_variants/librt_$v.so timeout -k 10 200 python tools/strip_scaling.py --ranks 1 8 --inflight 2 > gpurun_out/r02_strips89_$v.log 2>&1 || exit 3
echo $v; grep -h '"rank": 0' gpurun_out/r02_strips89_$v.log | cut -c 1-90
done
