#!/bin/bash
# Attention kernel session: GPU numerics tests of the attention paths, attention micro-bench,
# then the headline training bench.  Every GPU step has its own time limit.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/ -x -v -m gpu --timeout 120 --timeout-method thread -k "${TESTK:-attn or attention or packed or parity}" > gpurun_out/pytest_attn.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_attn.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_kernels.py --only-attn --iters 20 > gpurun_out/kbench_attn.log 2>&1 || { tail -20 gpurun_out/kbench_attn.log; exit 1; }
grep '^{' gpurun_out/kbench_attn.log
for cfg in ${CONFIGS:-LJSpeech BC2013}; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config $cfg --synth-steps 0 > gpurun_out/bench_$cfg.log 2>&1 || { tail -30 gpurun_out/bench_$cfg.log; exit 1; }
  tail -1 gpurun_out/bench_$cfg.log | cut -c1-200
done
