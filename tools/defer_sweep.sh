#!/bin/bash
# Deferred-pixel knob sweep (GPU box): RT_DEFER_BUDGET x RT_GROUP_SHIFT on the C4 bench.
# SWEEP="budget:shift ..." overrides the list; the previous commit's build (_variants/librt_head.so) runs first.
line=$(RT_LIB_PATH=_variants/librt_head.so timeout -k 10 120 python bench.py --no-cpu-baseline | grep "^{") || exit 1
echo "previous commit: $(echo "$line" | cut -c1-200)"
for cfg in ${SWEEP:-0:4 750:4 500:4 250:4 250:3 150:4 500:5 750:4}; do
  set -- ${cfg/:/ }
  line=$(RT_DEFER_BUDGET=$1 RT_GROUP_SHIFT=$2 timeout -k 10 120 python bench.py --no-cpu-baseline | grep '^{') || exit 1
  echo "budget $1 shift $2: $(echo "$line" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], "Mrays/s kernel", d["kernel_ms"], "ms dpix", d.get("max_abs_dpixel"))')"
done
