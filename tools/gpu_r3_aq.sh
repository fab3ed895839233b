#!/bin/bash
# Finer CU-budget sweep of the weight-gradient split plan (LJSpeech, BC2013_GST), two repetitions.
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for c in LJSpeech BC2013_GST; do
  for rep in 1 2; do
    for cus in 0 160 192 224; do
      SSAMD_WGRAD_CUS=$cus timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --synth-steps 0 > gpurun_out/aq_${c}_$cus.log 2>&1 || { tail -20 gpurun_out/aq_${c}_$cus.log; exit 1; }
      tail -1 gpurun_out/aq_${c}_$cus.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c cus=$cus', d['value'], d['ms_per_step'])"
    done
  done
done
