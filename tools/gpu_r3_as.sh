#!/bin/bash
# A/B: weight-gradient-first issue order "auto" (below 80k rows) vs off.
# GPU numerics tests of the side stream with the new order first.
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for c in LJSpeech BC2013 BC2013_GST; do
  for rep in 1 2; do
    for f in 0 auto; do
      SSAMD_WGRAD_FIRST=$f timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --synth-steps 0 > gpurun_out/as_${c}_$f.log 2>&1 || { tail -20 gpurun_out/as_${c}_$f.log; exit 1; }
      tail -1 gpurun_out/as_${c}_$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c first=$f', d['value'], d['ms_per_step'])"
    done
  done
done
