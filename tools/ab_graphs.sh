#!/bin/bash
# Small-batch training steps: eager vs HIP-graph steps (train/graphs.py), with the side stream as the policy decides
# or forced on (SSAMD_EXPERIMENTAL side_wgrad=1).  gpurun -- 'bash tools/ab_graphs.sh' -> gpurun_out/ab_graphs.txt
set -o pipefail
cd "$(dirname "$0")/.."; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for cfg in ${CONFIGS:-"LibriTTS" "BC2013 --batch 10"}; do
  for arm in "eager|" "graphs|--graphs" "graphs+side|--graphs@side_wgrad=1"; do
    name=${arm%%|*}; rest=${arm#*|}; flags=${rest%%@*}; exp=""; [ "$rest" != "$flags" ] && exp=${rest#*@}
    SSAMD_EXPERIMENTAL="$exp" timeout -k 10 300 python bench.py --config $cfg --steps ${STEPS:-30} --warmup 5 --synth-steps 0 $flags > gpurun_out/ab_graphs_run.log 2>&1 || { tail -30 gpurun_out/ab_graphs_run.log; exit 1; }
    echo "$cfg [$name] $(tail -1 gpurun_out/ab_graphs_run.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["host_enqueue_ms_per_step"], d.get("graphs"))')" | tee -a gpurun_out/ab_graphs.txt
  done
done
