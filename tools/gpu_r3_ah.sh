#!/bin/bash
# LJSpeech bench with host step-tail timestamps (SSAMD_HOST_TAIL=1), then plain bench x2.
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
SSAMD_HOST_TAIL=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --synth-steps 0 > gpurun_out/ah_tail.log 2>&1 || { tail -20 gpurun_out/ah_tail.log; exit 1; }
tail -1 gpurun_out/ah_tail.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('tail', d['value'], d['ms_per_step'], d.get('host_tail_ms'), d.get('host_enqueue_ms_per_step'))"
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --synth-steps 0 > gpurun_out/ah_$i.log 2>&1 || { tail -20 gpurun_out/ah_$i.log; exit 1; }
  tail -1 gpurun_out/ah_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('plain', d['value'], d['ms_per_step'], d.get('host_enqueue_ms_per_step'))"
done
bash tools/gpu_r3_af.sh
