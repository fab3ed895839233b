#!/bin/bash
# Same-box synthesis A/B: bench_synth.py with ARGS_A vs ARGS_B, ROUNDS times (JSON lines -> gpurun_out/ab_synth.jsonl)
#   gpurun -- 'ARGS_A="--bucketed" ARGS_B="" bash tools/ab_synth.sh'
set -o pipefail
cd "$(dirname "$0")/.."; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for i in $(seq 1 ${ROUNDS:-2}); do
  for arm in A B; do
    v=ARGS_$arm
    timeout -k 10 300 python bench_synth.py --steps ${STEPS:-10} --b1-runs ${B1:-30} ${!v} > gpurun_out/ab_synth_$arm.log 2>&1 || { tail -30 gpurun_out/ab_synth_$arm.log; exit 1; }
    l=$(tail -1 gpurun_out/ab_synth_$arm.log)
    echo "$l" >> gpurun_out/ab_synth.jsonl
    echo "[$arm ${!v}] $(echo "$l" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["b1_ms"], d["vocoder"])')"
  done
done
