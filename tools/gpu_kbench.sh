#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
python csrc/build.py > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_kernels.py --iters 10 2>&1 | grep -v amdgpu.ids | tee gpurun_out/kbench.log
timeout -k 10 600 python bench.py --steps 8 --warmup 3 > gpurun_out/bench_hip.log 2>&1 || { tail -30 gpurun_out/bench_hip.log; exit 1; }
tail -1 gpurun_out/bench_hip.log
