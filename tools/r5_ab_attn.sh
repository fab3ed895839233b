# attention change: GPU tests, kernel micro-bench (this tree vs ab/base library), whole-tree LJSpeech A/B
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "attention or attn or model_step or packed" > gpurun_out/at_t.log 2>&1 || { tail -30 gpurun_out/at_t.log; exit 1; }
tail -1 gpurun_out/at_t.log
for tag in A B; do
  lib=$PWD/speakingstyle_amd/_lib/libssamd_kernels.so; [ $tag = A ] && lib=$PWD/ab/base/speakingstyle_amd/_lib/libssamd_kernels.so
  SSAMD_KERNEL_LIB=$lib timeout -k 10 300 python tools/bench_kernels.py --only-attn > gpurun_out/at_kb_$tag.log 2>&1 || { tail -20 gpurun_out/at_kb_$tag.log; exit 1; }
  echo "$tag $(grep 'H2 D128' gpurun_out/at_kb_$tag.log | cut -c1-160)"
done
ROUNDS=3 bash tools/gpu.sh abtree
