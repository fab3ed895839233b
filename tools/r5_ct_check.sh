set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/kt.log 2>&1 || { tail -30 gpurun_out/kt.log; exit 1; }
tail -1 gpurun_out/kt.log
timeout -k 10 600 python tools/gemm_census.py --iters 10 > gpurun_out/census_ct.jsonl 2>/dev/null || exit 1
tail -1 gpurun_out/census_ct.jsonl
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --synth-steps 0 --synth-b1-runs 0 > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 1; }
echo "bench $(tail -1 gpurun_out/b.log | cut -c1-150)"
done
