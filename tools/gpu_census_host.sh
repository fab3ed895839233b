#!/bin/bash
# Torch-op / slot-copy census and host cProfile of one steady-state step (GPU box), for the configs
# given in CFGS (default: BC2013 LJSpeech).  Each GPU step has its own time limit.
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for c in ${CFGS:-BC2013 LJSpeech}; do
  timeout -k 10 240 python tools/copy_census.py $c > gpurun_out/census_$c.txt 2>&1 || { tail -20 gpurun_out/census_$c.txt; exit 1; }
  timeout -k 10 240 python tools/host_profile.py $c 5 > gpurun_out/hostprof_$c.txt 2>&1 || { tail -20 gpurun_out/hostprof_$c.txt; exit 1; }
done
head -12 gpurun_out/census_*.txt
