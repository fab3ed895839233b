#!/bin/bash
# Per-phase host/device step timing for the training configs (bench.py --phase-times).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for cfg in ${CONFIGS:-LJSpeech BC2013 BC2013_GST}; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config $cfg --synth-steps 0 --phase-times ${BENCHARGS} > gpurun_out/phase_$cfg.log 2>&1 || { tail -20 gpurun_out/phase_$cfg.log; exit 1; }
  tail -1 gpurun_out/phase_$cfg.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["config"]["model"], d["value"], d["ms_per_step"], json.dumps(d.get("phase_ms")))'
done
