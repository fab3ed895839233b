set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
for args in "--config BC2013" "--config BC2013_GST" "--config LibriTTS" "--config BC2013 --batch 10"; do
  timeout -k 10 300 python bench.py $args --steps 20 --warmup 5 --synth-steps 0 --synth-b1-runs 0 > gpurun_out/cfgb.log 2>&1 || { tail -20 gpurun_out/cfgb.log; exit 1; }
  echo "$args $(tail -1 gpurun_out/cfgb.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("host_enqueue_ms_per_step"))')"
done
