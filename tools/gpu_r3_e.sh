#!/bin/bash
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 150 python tools/exp_wgrad_pp.py > gpurun_out/exp_wgrad_pp.jsonl 2> gpurun_out/exp_wgrad_pp.err || { tail -30 gpurun_out/exp_wgrad_pp.err; cat gpurun_out/exp_wgrad_pp.jsonl; exit 1; }
cat gpurun_out/exp_wgrad_pp.jsonl
