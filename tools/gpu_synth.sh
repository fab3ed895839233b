#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
python csrc/build.py > gpurun_out/build.log 2>&1 || { cat gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench_synth.py --batch ${SBATCH:-256} --steps 3 --warmup 1 > gpurun_out/bench_synth.log 2>&1 || { tail -30 gpurun_out/bench_synth.log; exit 1; }
tail -1 gpurun_out/bench_synth.log
