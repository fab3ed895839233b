#!/bin/bash
# At-HEAD check after the issue-order default: full GPU suite + default bench line.
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/at_gpu_tests.log 2>&1 || { tail -30 gpurun_out/at_gpu_tests.log; exit 1; }
tail -1 gpurun_out/at_gpu_tests.log
timeout -k 10 240 python bench.py > gpurun_out/at_bench_lj.log 2>&1 || { tail -20 gpurun_out/at_bench_lj.log; exit 1; }
tail -1 gpurun_out/at_bench_lj.log
