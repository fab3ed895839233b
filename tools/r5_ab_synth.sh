# same-box A/B of the synthesis RTF: ab/base (A) vs this tree (B), bench_synth.py, ROUNDS rounds; K = pytest filter first
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -n "$K" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$K" > gpurun_out/syn_t.log 2>&1 || { tail -30 gpurun_out/syn_t.log; exit 1; }
  tail -1 gpurun_out/syn_t.log
fi
for i in $(seq 1 ${ROUNDS:-2}); do
  (cd ab/base && timeout -k 10 300 python bench_synth.py --steps ${STEPS:-10} > ../../gpurun_out/syn_A.log 2>&1) || { tail -20 gpurun_out/syn_A.log; exit 1; }
  echo "A $(grep '^{' gpurun_out/syn_A.log | tail -1 | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
  timeout -k 10 300 python bench_synth.py --steps ${STEPS:-10} > gpurun_out/syn_B.log 2>&1 || { tail -20 gpurun_out/syn_B.log; exit 1; }
  echo "B $(grep '^{' gpurun_out/syn_B.log | tail -1 | python -c 'import json,sys; print(json.loads(sys.stdin.read())["value"])')"
done
