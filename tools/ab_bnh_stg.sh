set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "bn_act" > gpurun_out/bnt.log 2>&1 || { tail -30 gpurun_out/bnt.log; exit 1; }
tail -1 gpurun_out/bnt.log
for i in 1 2; do
for v in 1 0; do
  SSAMD_EXPERIMENTAL=gemm_bnh_stg=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --synth-steps 0 --synth-b1-runs 0 > gpurun_out/ab.log 2>&1 || { tail -20 gpurun_out/ab.log; exit 1; }
  echo "bnh_stg=$v $(tail -1 gpurun_out/ab.log | cut -c1-200)"
done; done
