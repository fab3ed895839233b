#!/bin/bash
# FiLM gradient path check (GPU box): targeted kernel/model tests, determinism, BC2013 census + bench.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_kernels_gpu.py -k "film or model_step or layernorm or packed_vs_padded" > gpurun_out/film_tests.log 2>&1 \
  || { tail -40 gpurun_out/film_tests.log; exit 1; }
tail -3 gpurun_out/film_tests.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_train_gpu.py tests/test_gst_gpu.py > gpurun_out/train_tests.log 2>&1 \
  || { tail -40 gpurun_out/train_tests.log; exit 1; }
tail -3 gpurun_out/train_tests.log
timeout -k 10 240 python tools/copy_census.py BC2013 > gpurun_out/census_BC2013_after.txt 2>&1 || { tail -20 gpurun_out/census_BC2013_after.txt; exit 1; }
head -8 gpurun_out/census_BC2013_after.txt
for c in BC2013 BC2013_GST LJSpeech; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --synth-steps 0 > gpurun_out/bench_$c.log 2>&1 || { tail -20 gpurun_out/bench_$c.log; exit 1; }
  tail -1 gpurun_out/bench_$c.log
done
