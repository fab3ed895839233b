#!/bin/bash
# One GPU session: build, kernel numerics tests, smoke, bench (hip vs torch reference backend).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
python csrc/build.py > gpurun_out/build.log 2>&1 || { echo "build failed"; cat gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps ${STEPS:-6} --warmup 2 > gpurun_out/bench_hip.log 2>&1 || { tail -30 gpurun_out/bench_hip.log; exit 1; }
tail -3 gpurun_out/bench_hip.log
if [ -n "$REFBENCH" ]; then
timeout -k 10 600 python bench.py --steps 4 --warmup 2 --backend reference > gpurun_out/bench_ref.log 2>&1 || { tail -30 gpurun_out/bench_ref.log; exit 1; }
tail -3 gpurun_out/bench_ref.log
fi
