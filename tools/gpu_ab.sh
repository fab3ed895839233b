#!/bin/bash
# Same-box A/B of the training step: bench with the in-tree kernel library (B) and with
# ab/libssamd_kernels_$BASE.so (A), alternated ROUNDS times.  Optional GPU tests first (TESTK).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -n "$TESTK" ]; then
  timeout -k 10 600 python -u -m pytest tests/ -x -q -m gpu --timeout 120 --timeout-method thread -k "$TESTK" > gpurun_out/pytest_ab.log 2>&1
  rc=$?; tail -2 gpurun_out/pytest_ab.log; [ $rc -ne 0 ] && exit $rc
fi
A=ab/libssamd_kernels_$BASE.so
[ -f "$A" ] || { echo "missing $A"; exit 1; }
for i in $(seq 1 ${ROUNDS:-2}); do
  for cfg in ${CONFIGS:-LJSpeech}; do
    SSAMD_KERNEL_LIB=$A timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config $cfg --synth-steps 0 > gpurun_out/ab_A.log 2>&1 || { tail -20 gpurun_out/ab_A.log; exit 1; }
    echo "A $cfg $(tail -1 gpurun_out/ab_A.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config $cfg --synth-steps 0 > gpurun_out/ab_B.log 2>&1 || { tail -20 gpurun_out/ab_B.log; exit 1; }
    echo "B $cfg $(tail -1 gpurun_out/ab_B.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
