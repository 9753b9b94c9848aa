#!/bin/bash
# Runs on the GPU box: a list of steps, each under its own time limit, logs in
# gpurun_out/<name>.log and one status line per step in gpurun_out/steps.log.
# A step that times out, is killed or crashes (exit >= 124) ends the script;
# an ordinary failure (e.g. a failing test, exit 1) does not.
# Usage: bash tools/gpu_steps.sh "name|seconds|command" ...
set -u
mkdir -p gpurun_out
for spec in "$@"; do
    name=${spec%%|*}
    rest=${spec#*|}
    secs=${rest%%|*}
    cmd=${rest#*|}
    start=$(date +%s)
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "$name rc=$rc $(( $(date +%s) - start ))s" >> gpurun_out/steps.log
    if [ "$rc" -ge 124 ]; then
        echo "stopping after $name (rc=$rc)" >> gpurun_out/steps.log
        exit "$rc"
    fi
done
