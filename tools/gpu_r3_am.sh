#!/bin/bash
# GEMM variant sweep at decoder-sized M (LJSpeech batch 200: M = 61k and 113k rows)
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for L in 305 565; do
  L=$L timeout -k 10 240 python tools/exp_small_m.py > gpurun_out/am_L$L.jsonl 2>&1 || { tail -20 gpurun_out/am_L$L.jsonl; exit 1; }
  cat gpurun_out/am_L$L.jsonl
done
