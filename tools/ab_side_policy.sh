set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {
  SSAMD_EXPERIMENTAL="$3" timeout -k 10 300 python bench.py $2 --steps 30 --warmup 5 --synth-steps 0 --synth-b1-runs 0 > gpurun_out/abp.log 2>&1 || { tail -20 gpurun_out/abp.log; exit 1; }
  echo "$1 $(tail -1 gpurun_out/abp.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["host_enqueue_ms_per_step"], round(d["value"]*d["ms_per_step"]/1000))')"
}
for c in "--config BC2013 --batch 20" "--config BC2013 --batch 30" "--config BC2013 --batch 45" "--config LibriTTS --batch 32" "--config LibriTTS --batch 64" "--config BC2013_GST --batch 30" "--config BC2013_GST --batch 50"; do
  run "$c side=1" "$c" "side_wgrad=1"
  run "$c side=0" "$c" "side_wgrad=0"
done
