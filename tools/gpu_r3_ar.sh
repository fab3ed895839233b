#!/bin/bash
# A/B: weight gradient issued before (SSAMD_WGRAD_FIRST=1) vs after (0) the layer's data gradient;
# GPU numerics tests of the side stream with the new order first.
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
SSAMD_WGRAD_FIRST=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "side_stream or model_step or train" > gpurun_out/ar_tests.log 2>&1 || { tail -30 gpurun_out/ar_tests.log; exit 1; }
tail -1 gpurun_out/ar_tests.log
for c in LJSpeech BC2013 BC2013_GST; do
  for rep in 1 2; do
    for f in 0 1; do
      SSAMD_WGRAD_FIRST=$f timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --synth-steps 0 > gpurun_out/ar_${c}_$f.log 2>&1 || { tail -20 gpurun_out/ar_${c}_$f.log; exit 1; }
      tail -1 gpurun_out/ar_${c}_$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c first=$f', d['value'], d['ms_per_step'])"
    done
  done
done
