#!/bin/bash
# Step-tail trace of LJSpeech at HEAD with the host lead printed (is the host ahead under the profiler?)
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out/ak
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp SSAMD_HOST_LEAD=1 SSAMD_HOST_TAIL=1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/ak/1" -o run -- python3 "$R/bench.py" --steps 6 --warmup 3 --synth-steps 0 > "$R/gpurun_out/ak_1.log" 2>&1 || { tail -20 "$R/gpurun_out/ak_1.log"; exit 1; }
cd "$R"
tail -1 gpurun_out/ak_1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('traced', d['value'], d['ms_per_step'], d.get('host_enqueue_ms_per_step'), d.get('host_tail_ms'), 'lead', d.get('host_lead_ms'))"
t=$(find gpurun_out/ak/1 -name "*kernel_trace.csv" | head -1)
python tools/stream_split.py "$t" --last 2 --detail --tail 12 || exit 1
rm -rf gpurun_out/ak/1
