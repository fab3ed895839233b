set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # label, env, args
  SSAMD_EXPERIMENTAL="$2" timeout -k 10 300 python bench.py $3 --steps 20 --warmup 5 --synth-steps 0 --synth-b1-runs 0 > gpurun_out/abf.log 2>&1 || { tail -20 gpurun_out/abf.log; exit 1; }
  echo "$1 $(tail -1 gpurun_out/abf.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
for cfg in "--config BC2013" "--config BC2013_GST"; do
  for rep in 1 2; do
    run "$cfg frac=0.75" "" "$cfg"
    run "$cfg frac=0.5" "wgrad_cu_frac=0.5" "$cfg"
    run "$cfg frac=0.625" "wgrad_cu_frac=0.625" "$cfg"
    run "$cfg frac=1.0" "wgrad_cu_frac=1.0" "$cfg"
    run "$cfg no-side" "" "$cfg --no-side-wgrad"
  done
done
