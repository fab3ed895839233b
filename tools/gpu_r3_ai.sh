#!/bin/bash
# A/B: side-stream inputs released at the join (DEFER_RELEASE=0) vs during the next forward (=1); host tail marks on.
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 SSAMD_HOST_TAIL=1
for i in 1 2; do
  for d in 0 1; do
    SSAMD_DEFER_RELEASE=$d timeout -k 10 300 python bench.py --steps 20 --warmup 5 --synth-steps 0 > gpurun_out/ai_${d}_${i}.log 2>&1 || { tail -20 gpurun_out/ai_${d}_${i}.log; exit 1; }
    tail -1 gpurun_out/ai_${d}_${i}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('defer=$d', d['value'], d['ms_per_step'], d.get('host_tail_ms'), d.get('host_enqueue_ms_per_step'))"
  done
done
