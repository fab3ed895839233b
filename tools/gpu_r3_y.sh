#!/bin/bash
# (1) whole-ResBlock paired epilogue stores: test + timing + PMC; (2) LN weight-gradient reductions on the
# side stream: GPU tests + A/B; (3) per-stream split detail of LJSpeech / BC2013.
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 180 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "whole_block" > gpurun_out/y_rb_test.log 2>&1 || { tail -30 gpurun_out/y_rb_test.log; exit 1; }
tail -1 gpurun_out/y_rb_test.log
timeout -k 10 180 python -u tools/exp_rb_whole.py > gpurun_out/y_rb_whole.jsonl 2>gpurun_out/y_rb_whole.err || { tail -20 gpurun_out/y_rb_whole.err; exit 1; }
cat gpurun_out/y_rb_whole.jsonl
PMC_TARGET=tools/pmc_rb_whole.py timeout -k 10 300 bash tools/gpu_pmc.sh > gpurun_out/y_pmc_rb.txt 2>&1 || { tail -20 gpurun_out/y_pmc_rb.txt; exit 1; }
grep -A2 "resblock_fused" gpurun_out/y_pmc_rb.txt | grep "lds_conflict" | head
bash tools/gpu_r3_x.sh || exit 1
bash tools/gpu_r3_w.sh || exit 1
