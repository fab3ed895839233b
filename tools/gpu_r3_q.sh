#!/bin/bash
# bench lines at HEAD: LJSpeech (+ synth RTF), BC2013, BC2013_GST; host profile of the GST step.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 240 python bench.py > gpurun_out/q_bench_lj.log 2>&1 || { tail -20 gpurun_out/q_bench_lj.log; exit 1; }
tail -1 gpurun_out/q_bench_lj.log
timeout -k 10 200 python bench.py --config BC2013 --synth-steps 0 --phase-times > gpurun_out/q_bench_bc.log 2>&1 || { tail -20 gpurun_out/q_bench_bc.log; exit 1; }
tail -1 gpurun_out/q_bench_bc.log
timeout -k 10 200 python bench.py --config BC2013_GST --synth-steps 0 --phase-times > gpurun_out/q_bench_gst.log 2>&1 || { tail -20 gpurun_out/q_bench_gst.log; exit 1; }
tail -1 gpurun_out/q_bench_gst.log
