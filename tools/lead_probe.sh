set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
mkdir -p gpurun_out
export SSAMD_EXPERIMENTAL=host_lead=1,host_tail=1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --synth-steps 0 --synth-b1-runs 0 > gpurun_out/lead_lj.log 2>&1 || exit 1
tail -1 gpurun_out/lead_lj.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["host_enqueue_ms_per_step"], d.get("host_lead_ms"), d.get("host_tail_ms"))'
for c in "BC2013 --batch 10" "LibriTTS" "BC2013_GST"; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --synth-steps 0 --synth-b1-runs 0 > gpurun_out/lead_cfg.log 2>&1 || exit 1
  echo "$c: $(tail -1 gpurun_out/lead_cfg.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["host_enqueue_ms_per_step"], d.get("host_lead_ms"), d.get("host_tail_ms"))')"
done
