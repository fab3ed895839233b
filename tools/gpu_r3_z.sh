#!/bin/bash
# torch-op census with call sites (LJSpeech, BC2013); whole-ResBlock reverted epilogue re-timed.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for c in LJSpeech BC2013; do
  timeout -k 10 300 python tools/torch_ops_census.py $c > gpurun_out/z_census_$c.txt 2>&1 || { tail -20 gpurun_out/z_census_$c.txt; exit 1; }
  head -80 gpurun_out/z_census_$c.txt
done
timeout -k 10 180 python -u tools/exp_rb_whole.py > gpurun_out/z_rb_whole.jsonl 2>gpurun_out/z_rb_whole.err || { tail -20 gpurun_out/z_rb_whole.err; exit 1; }
cat gpurun_out/z_rb_whole.jsonl
