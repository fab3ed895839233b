#!/bin/bash
# Host profiles GST vs BC2013; BC2013 at-HEAD kernel profile; ResBlock kernels PMC.
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for c in BC2013_GST BC2013; do
  timeout -k 10 300 python tools/host_profile.py $c 5 > gpurun_out/t_hostprof_$c.txt 2>&1 || { tail -20 gpurun_out/t_hostprof_$c.txt; exit 1; }
  head -12 gpurun_out/t_hostprof_$c.txt
done
TAG=r3_v5_BC BENCHARGS="--config BC2013" timeout -k 10 400 bash tools/gpu_prof_head.sh || exit 1
PMC_TARGET=tools/pmc_rb_whole.py timeout -k 10 300 bash tools/gpu_pmc.sh > gpurun_out/t_pmc_rb.txt 2>&1 || { tail -20 gpurun_out/t_pmc_rb.txt; exit 1; }
grep -A2 "resblock" gpurun_out/t_pmc_rb.txt | head -60
