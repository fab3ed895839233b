#!/bin/bash
# GPU session: the style-config training benches (BC2013 FiLM reference encoder, BC2013 GST).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for cfg in ${CFGS:-BC2013 BC2013_GST}; do
  timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-6} --warmup 2 > gpurun_out/bench_$cfg.log 2>&1 || { tail -30 gpurun_out/bench_$cfg.log; exit 1; }
  tail -1 gpurun_out/bench_$cfg.log
done
