#!/bin/bash
# Whole-ResBlock prefetch version: test + A/B timing; LJSpeech at-HEAD kernel profile.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 180 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "whole_block" > gpurun_out/p_rb_test.log 2>&1 || { tail -30 gpurun_out/p_rb_test.log; exit 1; }
tail -1 gpurun_out/p_rb_test.log
timeout -k 10 180 python -u tools/exp_rb_whole.py > gpurun_out/p_rb_whole.jsonl 2>gpurun_out/p_rb_whole.err || { tail -20 gpurun_out/p_rb_whole.err; exit 1; }
cat gpurun_out/p_rb_whole.jsonl
TAG=r3_v3_LJ timeout -k 10 400 bash tools/gpu_prof_head.sh || exit 1
