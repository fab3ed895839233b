#!/bin/bash
# Weight-gradient session: full GPU tests, split / reduction sweep, headline bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/exp_wgrad_splits.py > gpurun_out/wsplit.jsonl 2> gpurun_out/wsplit.err || { tail -20 gpurun_out/wsplit.err; exit 1; }
timeout -k 10 120 python tools/exp_packed_wgrad.py 2>/dev/null | grep "^{" > gpurun_out/pkwgrad.jsonl || exit 1
cat gpurun_out/pkwgrad.jsonl
cat gpurun_out/wsplit.jsonl
for cfg in ${CONFIGS:-LJSpeech}; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config $cfg --synth-steps 0 > gpurun_out/bench_$cfg.log 2>&1 || { tail -30 gpurun_out/bench_$cfg.log; exit 1; }
  tail -1 gpurun_out/bench_$cfg.log | cut -c1-200
done
