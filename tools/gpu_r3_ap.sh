#!/bin/bash
# At-HEAD evidence: full GPU suite, bench (LJSpeech + RTF) and BC2013 / GST lines, LJSpeech + synth
# kernel profiles, (PMC summaries: r3_v9).
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/ap_gpu_tests.log 2>&1 || { tail -30 gpurun_out/ap_gpu_tests.log; exit 1; }
tail -2 gpurun_out/ap_gpu_tests.log
timeout -k 10 240 python bench.py > gpurun_out/ap_bench_lj.log 2>&1 || { tail -20 gpurun_out/ap_bench_lj.log; exit 1; }
tail -1 gpurun_out/ap_bench_lj.log
for c in BC2013 BC2013_GST; do
  timeout -k 10 200 python bench.py --config $c --synth-steps 0 > gpurun_out/ap_bench_$c.log 2>&1 || { tail -20 gpurun_out/ap_bench_$c.log; exit 1; }
  tail -1 gpurun_out/ap_bench_$c.log
done
TAG=r3_v10_LJ timeout -k 10 400 bash tools/gpu_prof_head.sh || exit 1
TAG=r3_v10_synth timeout -k 10 300 bash tools/gpu_prof_synth.sh > gpurun_out/ap_prof_synth.log 2>&1 || { tail -20 gpurun_out/ap_prof_synth.log; exit 1; }
tail -5 gpurun_out/ap_prof_synth.log
