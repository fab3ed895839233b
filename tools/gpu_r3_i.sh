#!/bin/bash
# Round 3: host enqueue time vs wall per step (is the step host-bound?).
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for c in BC2013 BC2013_GST LJSpeech; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --synth-steps 0 > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
  tail -1 gpurun_out/b.log | python -c "import sys,json; r=json.loads(sys.stdin.read()); print('$c', r['value'], r['ms_per_step'], 'host', r['host_enqueue_ms_per_step'])"
done
timeout -k 10 300 python bench.py --config BC2013 --steps 10 --warmup 3 --synth-steps 0 --phase-times > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
tail -1 gpurun_out/b.log
