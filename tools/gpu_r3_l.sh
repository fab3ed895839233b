#!/bin/bash
# Round 3: batched-load LayerNorm kernels -- tests + benches (compare with r3_k's kernel-path lines).
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_l.log 2>&1 || { tail -40 gpurun_out/pytest_l.log; exit 1; }
tail -2 gpurun_out/pytest_l.log
for rep in 1 2; do
for c in LJSpeech BC2013 BC2013_GST; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --synth-steps 0 > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
  tail -1 gpurun_out/b.log | python -c "import sys,json; r=json.loads(sys.stdin.read()); print('$c', r['value'], r['ms_per_step'], 'host', r['host_enqueue_ms_per_step'])"
done
done
