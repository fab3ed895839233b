#!/bin/bash
# BN backward raw-bf16 / 8-row batches: kernel A/B vs the HEAD library, bench A/B; step tail trace.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
OLD=$(ls ab/libssamd_kernels_*.so | head -1)
timeout -k 10 120 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 100 --timeout-method thread -k "bn or postnet or batchnorm" > gpurun_out/ag_pytest.log 2>&1 || { tail -30 gpurun_out/ag_pytest.log; exit 1; }
tail -1 gpurun_out/ag_pytest.log
for rep in 1 2; do
  echo -n "new "; timeout -k 10 120 python tools/exp_bn_bwd.py || exit 1
  echo -n "old "; SSAMD_KERNEL_LIB=$OLD timeout -k 10 120 python tools/exp_bn_bwd.py || exit 1
done
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --synth-steps 0 > gpurun_out/ag_b.log 2>&1 || { tail -20 gpurun_out/ag_b.log; exit 1; }
  tail -1 gpurun_out/ag_b.log | python -c "import sys,json; r=json.loads(sys.stdin.read()); print('new', r['value'], r['ms_per_step'])"
  SSAMD_KERNEL_LIB=$OLD timeout -k 10 200 python bench.py --steps 10 --warmup 3 --synth-steps 0 > gpurun_out/ag_b.log 2>&1 || { tail -20 gpurun_out/ag_b.log; exit 1; }
  tail -1 gpurun_out/ag_b.log | python -c "import sys,json; r=json.loads(sys.stdin.read()); print('old', r['value'], r['ms_per_step'])"
done
bash tools/gpu_r3_af.sh || exit 1
