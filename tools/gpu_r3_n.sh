#!/bin/bash
# Round 3: lean side-stream path (native stream wait, no record_stream) -- tests, GST host profile, benches.
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_ddp_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_n.log 2>&1 || { tail -40 gpurun_out/pytest_n.log; exit 1; }
tail -2 gpurun_out/pytest_n.log
timeout -k 10 300 python tools/host_profile.py BC2013_GST 5 > gpurun_out/hostprof_GST.txt 2>&1 || { tail -20 gpurun_out/hostprof_GST.txt; exit 1; }
head -45 gpurun_out/hostprof_GST.txt
for rep in 1 2; do
for c in BC2013_GST BC2013 LJSpeech; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --synth-steps 0 > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
  tail -1 gpurun_out/b.log | python -c "import sys,json; r=json.loads(sys.stdin.read()); print('$c', r['value'], r['ms_per_step'], 'host', r['host_enqueue_ms_per_step'])"
done
done
