#!/bin/bash
# Data-parallel rehearsal on a 1-GPU box: RCCL bucket path with a single-rank communicator
# (tests/test_ddp_gpu.py) and the 2-rank launcher + collectives over gloo with both ranks on
# the one GPU (bench.py --gpus 2 --dist-backend gloo).  The real 1->8 RCCL run is the driver's.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_ddp_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/t_ddp_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/t_ddp_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --synth-steps 1 --synth-batch 32 > gpurun_out/bench_gloo2.log 2>&1 || { tail -30 gpurun_out/bench_gloo2.log; exit 1; }
tail -1 gpurun_out/bench_gloo2.log
