#!/bin/bash
# The one GPU-box driver (replaces the per-experiment r05_*.sh scripts).
# Usage (on the box, via gpurun):  bash tools/gpu_job.sh <outdir> <step> [<step> ...]
# Each step runs under its own time limit; logs go to gpurun_out/<outdir>/<step>.log and one status
# line per step to gpurun_out/<outdir>/steps.log.  A step that times out, is killed or crashes
# (exit >= 124) ends the job; an ordinary failure (a failing test, exit 1) ends it too unless the
# step name is prefixed with '-' (then the job goes on).  A heartbeat line is printed every 30 s.
# Environment: ENV_<STEP>="VAR=x VAR2=y" adds variables to one step; a step written step@tag runs with
# ENV_<TAG> instead and logs to step@tag.log (the same step under several settings); BENCH_ARGS extra
# bench.py args.
#
# Steps:
#   suite          pytest -m gpu (the whole GPU suite)
#   smoke          __graft_entry__.smoke()
#   bench          bench.py (C4 headline line, CPU baseline and check)
#   bench_fast     bench.py --no-cpu-baseline (C4, check only)
#   bench_c5       bench.py --config sphere1m_refl --steps 6 --warmup 2 --no-cpu-baseline
#   bench_hair     bench.py --config hair1m --no-cpu-baseline
#   strips1        tools/strip_scaling.py, one frame in flight, every rank, N = 1 2 4 8
#   strips3        the same with three frames in flight (and one, for the like-for-like ratio)
#   strips3b       strips3 with cost-balanced band lists (--balance)
#   nccl           tools/nccl_check.py under torch.distributed.run (RCCL pipeline, world size 1)
#   tilecosts      tools/tile_costs.py gpu sphere1m 5
#   bandcosts      tools/band_tile_costs.py: one rank's band launch (N:rank in BAND_LAYOUTS), tile costs + time
#   trace_c4       rocprofv3 kernel trace of bench.py (three frames in flight)
#   trace_c4_1     rocprofv3 kernel trace of bench.py --inflight 1 (per-kernel durations not overlapped)
#   trace_strips8  rocprofv3 kernel trace of the strips probe at N = 8 (ranks 0 and 7, one and three in flight)
#   pmc_c4         PMC passes of bench.py (tools/profile_gpu.sh)
#   trace_c5 / pmc_c5 / trace_hair / pmc_hair   the same for C5 / hair1m
#   count_c4 / count_c5 / count_hair   RT_COUNT=1 work counts (needs _variants/librt_count.so)
#   py:<file>      python <file> (a probe under tools/)
#   pt:<expr>      pytest -m gpu -k <expr> (a subset of the GPU suite)
set -u
OUT=gpurun_out/${1:?outdir}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
( while sleep 30; do echo "[tick] $(date +%T)"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
BA=${BENCH_ARGS:-}

last_json() {   # last_json <log>: the bench line's key fields
    grep -h '^{' "$1" | python3 -c "import json,sys
d=json.loads(sys.stdin.readlines()[-1]); r=d.get('roofline') or {}
print(d['config'].get('workload','')[:24], 'value', d['value'], 'ms/step', d['ms_per_step'], 'kernel', d.get('kernel_ms'),
      'dpx', d.get('max_abs_dpixel'), 'frac', r.get('frac'), 'sync', (d.get('sync') or {}).get('value'),
      'moving', (d.get('moving_camera') or {}).get('value'))" || true
}

trace() {   # trace <name> <secs> <bench args...>
    local name=$1${TAG:+_$TAG} secs=$2; shift 2
    timeout -k 10 "$secs" rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$name" -o run -- \
        python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-check --no-legs "$@"
}

run_step() {
    local step=$1
    case "$step" in
    suite) python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread ;;
    smoke) python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
    bench) python bench.py $BA ;;
    bench_fast) python bench.py --no-cpu-baseline $BA ;;
    bench_q2) python bench.py --no-cpu-baseline --no-legs --inflight 2 $BA ;;
    bench_q4) python bench.py --no-cpu-baseline --no-legs --inflight 4 $BA ;;
    bench_c5) python bench.py --config sphere1m_refl --steps 6 --warmup 2 --no-cpu-baseline $BA ;;
    bench_hair) python bench.py --config hair1m --steps 20 --warmup 3 --no-cpu-baseline $BA ;;
    strips1) python tools/strip_scaling.py --ranks 1 2 4 8 --steps 40 --all-ranks --inflight 1 ;;
    strips3) python tools/strip_scaling.py --ranks 1 2 4 8 --steps 40 --all-ranks --inflight 1 3 ;;
    strips3b) python tools/strip_scaling.py --ranks 1 2 4 8 --steps 40 --all-ranks --inflight 1 3 --balance ;;
    strips4) python tools/strip_scaling.py --ranks 1 2 4 8 --steps 40 --all-ranks --inflight 1 3 4 ;;
    nccl) python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \
              --master-port 29517 tools/nccl_check.py ;;
    tilecosts) python tools/tile_costs.py gpu sphere1m 5 "$OUT/tile_costs.npy" ;;
    tilecosts_hair) python tools/tile_costs.py gpu hair1m 5 "$OUT/tile_costs_hair.npy" ;;
    bandcosts) BAND_LAYOUTS=${BAND_LAYOUTS:-1:0,8:0,8:3,8:5} python tools/band_tile_costs.py sphere1m ;;
    trace_c4) trace trace_c4 300 ;;
    trace_strips8) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_strips8" -o run -- \
                       python3 tools/strip_scaling.py --ranks 8 --steps 40 --inflight 1 3 ;;
    trace_c4_1) trace trace_c4_1 300 --inflight 1 ;;
    trace_c5) trace trace_c5 600 --config sphere1m_refl --steps 4 --warmup 1 ;;
    trace_hair) trace trace_hair 300 --config hair1m ;;
    pmc_c4) bash tools/profile_gpu.sh "${OUT#gpurun_out/}_c4" ;;
    pmc_c5) bash tools/profile_gpu.sh "${OUT#gpurun_out/}_c5" --config sphere1m_refl ;;
    pmc_hair) bash tools/profile_gpu.sh "${OUT#gpurun_out/}_hair" --config hair1m ;;
    count_c4) RT_LIB_PATH=_variants/librt_count.so python tools/count_gpu_work.py sphere1m seg ;;
    count_c5) RT_LIB_PATH=_variants/librt_count.so python tools/count_gpu_work.py sphere1m_refl seg ;;
    count_hair) RT_LIB_PATH=_variants/librt_count.so python tools/count_gpu_work.py hair1m seg ;;
    py:*) python ${step#py:} ;;
    pt:*) python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -k "${step#pt:}" ;;
    *) echo "unknown step $step"; return 2 ;;
    esac
}

limit() {
    case "$1" in
    suite) echo 1200 ;; bench_c5|trace_c5|pmc_c5|pmc_c4|pmc_hair|count_c5) echo 900 ;; *) echo 400 ;;
    esac
}

for spec in "$@"; do
    soft=0
    step=$spec
    if [ "${spec#-}" != "$spec" ]; then soft=1; step=${spec#-}; fi
    tag=
    if [ "${step#*@}" != "$step" ]; then tag=${step#*@}; step=${step%%@*}; fi
    key=$(echo "${tag:-${step%%:*}}" | tr 'a-z' 'A-Z')
    envv=$(eval echo "\${ENV_${key}:-}")
    log="$OUT/$(echo "$step${tag:+@$tag}" | tr '/:' '__').log"
    start=$(date +%s)
    ( [ -n "$envv" ] && export $envv; run_step_limit=$(limit "$step"); \
      timeout -k 10 "$run_step_limit" bash -c "$(declare -f run_step trace); OUT=$OUT BA='$BA' TAG='$tag'; run_step '$step'" ) > "$log" 2>&1
    rc=$?
    echo "$step${tag:+@$tag} rc=$rc $(( $(date +%s) - start ))s" | tee -a "$OUT/steps.log"
    case "$step" in
    bench*) last_json "$log" ;;
    suite) tail -1 "$log" ;;
    strips*) grep bound "$log" || true ;;
    esac
    if [ "$rc" -ge 124 ]; then echo "stopping after $step (rc=$rc)" | tee -a "$OUT/steps.log"; exit "$rc"; fi
    if [ "$rc" -ne 0 ] && [ "$soft" = 0 ]; then echo "stopping after $step (rc=$rc)" | tee -a "$OUT/steps.log"; exit "$rc"; fi
done
