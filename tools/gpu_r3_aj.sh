#!/bin/bash
# Host-lead probe (per step: GPU finish minus host enqueue end) for the three bench configs, and
# backward on the engine's device thread (default) vs the calling thread; then a GST host cProfile.
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 SSAMD_HOST_TAIL=1 SSAMD_HOST_LEAD=1
for c in LJSpeech BC2013_GST BC2013; do
  for st in 0 1; do
    SSAMD_BWD_SAME_THREAD=$st timeout -k 10 300 python bench.py --config $c --steps 12 --warmup 5 --synth-steps 0 > gpurun_out/aj_${c}_$st.log 2>&1 || { tail -20 gpurun_out/aj_${c}_$st.log; exit 1; }
    tail -1 gpurun_out/aj_${c}_$st.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c same_thread=$st', d['value'], d['ms_per_step'], d.get('host_enqueue_ms_per_step'), d.get('host_tail_ms'), 'lead', d.get('host_lead_ms'))"
  done
done
timeout -k 10 240 python tools/host_profile.py BC2013_GST 5 > gpurun_out/aj_hostprof_GST.txt 2>&1 || { tail -20 gpurun_out/aj_hostprof_GST.txt; exit 1; }
head -50 gpurun_out/aj_hostprof_GST.txt
