#!/bin/bash
# Round 3: generated native launch bindings -- full GPU suite + A/B vs ctypes.
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_m.log 2>&1 || { tail -40 gpurun_out/pytest_m.log; exit 1; }
tail -2 gpurun_out/pytest_m.log
for rep in 1 2; do
for c in BC2013_GST BC2013 LJSpeech; do
  for cb in "" "--ctypes-bindings"; do
    timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --synth-steps 0 $cb > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
    tail -1 gpurun_out/b.log | python -c "import sys,json; r=json.loads(sys.stdin.read()); print('$c', '$cb', r['value'], r['ms_per_step'], 'host', r['host_enqueue_ms_per_step'])"
  done
done
done
