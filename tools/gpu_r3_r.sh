#!/bin/bash
# Whole-ResBlock 2-workgroup K=3 tiles: test + A/B timing; then bench lines (LJSpeech + RTF, BC2013, GST).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 180 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "whole_block" > gpurun_out/r_rb_test.log 2>&1 || { tail -30 gpurun_out/r_rb_test.log; exit 1; }
tail -1 gpurun_out/r_rb_test.log
timeout -k 10 180 python -u tools/exp_rb_whole.py > gpurun_out/r_rb_whole.jsonl 2>gpurun_out/r_rb_whole.err || { tail -20 gpurun_out/r_rb_whole.err; exit 1; }
cat gpurun_out/r_rb_whole.jsonl
bash tools/gpu_r3_q.sh
