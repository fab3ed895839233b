set -o pipefail
mkdir -p gpurun_out
for wb in 256 384 512 768; do
  SSAMD_WGRAD_BLOCKS=$wb timeout -k 10 200 python bench.py --steps 20 --warmup 5 --synth-steps 0 > gpurun_out/exp_wb$wb.log 2>&1 || exit 1
  echo "wb=$wb $(tail -1 gpurun_out/exp_wb$wb.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
