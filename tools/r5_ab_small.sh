# same-box A/B of small main-stream kernel fixes: tests first, then the whole-tree bench (ab/base = HEAD)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_train_gpu.py -x -q --timeout 200 --timeout-method thread -k "${K:-length_regulator or unpack or pack_unpack or bitwise or determin}" > gpurun_out/small_t.log 2>&1 || { tail -30 gpurun_out/small_t.log; exit 1; }
tail -1 gpurun_out/small_t.log
ROUNDS=${ROUNDS:-3} bash tools/gpu.sh abtree
