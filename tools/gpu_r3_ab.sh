#!/bin/bash
# CU-masked weight-gradient side stream A/B (LJSpeech x2, BC2013 x1).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2; do
for c in LJSpeech BC2013; do
  [ "$c" = BC2013 ] && [ $rep = 2 ] && continue
  for m in "" "--side-cu-mask 0x77777777" "--side-cu-mask 0x55555555" "--side-cu-mask 0x7f7f7f7f"; do
    timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 3 --synth-steps 0 $m > gpurun_out/ab_b.log 2>&1 || { tail -20 gpurun_out/ab_b.log; exit 1; }
    tail -1 gpurun_out/ab_b.log | python -c "import sys,json; r=json.loads(sys.stdin.read()); print('$c', '${m:-allCU}', r['value'], r['ms_per_step'], 'host', r['host_enqueue_ms_per_step'])"
  done
done
done
