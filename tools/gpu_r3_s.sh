#!/bin/bash
# C=128 layer kernel at 4 waves / 64x64 wave tiles: test + timing; GST sync scan + host profile.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 180 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "whole_block or resblock_layer" > gpurun_out/s_rb_test.log 2>&1 || { tail -30 gpurun_out/s_rb_test.log; exit 1; }
tail -1 gpurun_out/s_rb_test.log
timeout -k 10 180 python -u tools/exp_rb_whole.py > gpurun_out/s_rb_whole.jsonl 2>gpurun_out/s_rb_whole.err || { tail -20 gpurun_out/s_rb_whole.err; exit 1; }
cat gpurun_out/s_rb_whole.jsonl
timeout -k 10 200 python -u tools/sync_debug.py BC2013_GST > gpurun_out/s_sync_gst.txt 2>&1 || { tail -20 gpurun_out/s_sync_gst.txt; exit 1; }
tail -30 gpurun_out/s_sync_gst.txt
