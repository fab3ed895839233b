# ping-pong weight-gradient reads with DS immediate offsets: tests, per-shape timing vs the A/B base, whole-tree bench
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -x -q --timeout 200 --timeout-method thread -k "wgrad or bitwise or determin" > gpurun_out/wpp_t.log 2>&1 || { tail -30 gpurun_out/wpp_t.log; exit 1; }
tail -1 gpurun_out/wpp_t.log
timeout -k 10 200 python tools/exp_wgrad_stg.py --loops 0 1 > gpurun_out/wpp_B.log 2>&1 || { tail -20 gpurun_out/wpp_B.log; exit 1; }
SSAMD_KERNEL_LIB=$PWD/ab/base/speakingstyle_amd/_lib/libssamd_kernels.so timeout -k 10 200 python tools/exp_wgrad_stg.py --loops 0 1 > gpurun_out/wpp_A.log 2>&1 || { tail -20 gpurun_out/wpp_A.log; exit 1; }
SSAMD_KERNEL_LIB=$PWD/speakingstyle_amd/_lib/libssamd_kernels.so timeout -k 10 200 python tools/exp_wgrad_stg.py --loops 0 1 > gpurun_out/wpp_B.log 2>&1 || { tail -20 gpurun_out/wpp_B.log; exit 1; }
python - <<'PY'
import json
for tag in ("A", "B"):
    for l in open(f"gpurun_out/wpp_{tag}.log"):
        if l.startswith("{"):
            d = json.loads(l)
            print(tag, d["shape"], "pp1", d["pp1_us"], "pp0", d["pp0_us"], "bitwise", d["dW_bitwise"])
PY
ROUNDS=3 bash tools/gpu.sh abtree
