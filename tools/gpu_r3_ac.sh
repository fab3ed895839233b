#!/bin/bash
# Deferred side-stream weight-gradient issue: bitwise / DDP / train GPU tests + A/B (2 reps).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py tests/test_ddp_gpu.py tests/test_train_fidelity_gpu.py -x -q --timeout 300 --timeout-method thread -k "side or bitwise or determin or ddp or bucket or continuation or fidelity or model_step" > gpurun_out/ac_pytest.log 2>&1 || { tail -40 gpurun_out/ac_pytest.log; exit 1; }
tail -2 gpurun_out/ac_pytest.log
for rep in 1 2; do
for c in LJSpeech BC2013; do
  for f in "" "--no-wgrad-defer"; do
    timeout -k 10 200 python bench.py --config $c --steps 10 --warmup 3 --synth-steps 0 $f > gpurun_out/ac_b.log 2>&1 || { tail -20 gpurun_out/ac_b.log; exit 1; }
    tail -1 gpurun_out/ac_b.log | python -c "import sys,json; r=json.loads(sys.stdin.read()); print('$c', '${f:-defer}', r['value'], r['ms_per_step'], 'host', r['host_enqueue_ms_per_step'])"
  done
done
done
