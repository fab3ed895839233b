#!/bin/bash
# Whole-ResBlock kernel: numerics test, A/B timing, full GPU suite, bench at HEAD.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 180 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "whole_block or resblock_layer" > gpurun_out/o_rb_test.log 2>&1 || { tail -30 gpurun_out/o_rb_test.log; exit 1; }
tail -2 gpurun_out/o_rb_test.log
timeout -k 10 180 python -u tools/exp_rb_whole.py > gpurun_out/o_rb_whole.jsonl 2>gpurun_out/o_rb_whole.err || { tail -20 gpurun_out/o_rb_whole.err; exit 1; }
cat gpurun_out/o_rb_whole.jsonl
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/o_gpu_tests.log 2>&1 || { tail -30 gpurun_out/o_gpu_tests.log; exit 1; }
tail -2 gpurun_out/o_gpu_tests.log
timeout -k 10 240 python bench.py > gpurun_out/o_bench.log 2>&1 || { tail -20 gpurun_out/o_bench.log; exit 1; }
tail -1 gpurun_out/o_bench.log
