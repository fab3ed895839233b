#!/bin/bash
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python tools/grad_err_budget.py > gpurun_out/grad_budget.txt 2>&1 || { tail -30 gpurun_out/grad_budget.txt; exit 1; }
cat gpurun_out/grad_budget.txt | grep -v Warn
timeout -k 10 400 python -u -m pytest tests/test_train_fidelity_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/fidelity.log 2>&1 || { tail -40 gpurun_out/fidelity.log; exit 1; }
tail -5 gpurun_out/fidelity.log
