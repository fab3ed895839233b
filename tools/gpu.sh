#!/bin/bash
# Parameterised GPU-box harness (replaces the per-experiment gpu_*.sh scripts).  Run through
#   gpurun --timeout S -- 'bash tools/gpu.sh <task> [<task> ...]'
# Tasks run in order; each GPU step has its own time limit and the script stops at the first
# failure (no retries).  Tree must be pre-built on the CPU (python csrc/build.py).
#
# tasks:
#   tests            full `pytest -m gpu` (K=<expr> narrows it)            -> gpurun_out/tests.log
#   smoke            __graft_entry__.smoke()
#   bench            bench.py $BENCHARGS (repeat REP times)                  -> gpurun_out/bench_<i>.log
#   prof             rocprofv3 kernel trace of $BENCHARGS training steps      -> gpurun_out/$TAG_{summary,last_step,grid,split}.txt
#                    (TREE=ab/base profiles the A/B base tree's bench.py instead)
#   synthprof        rocprofv3 kernel trace of bench_synth.py $SYNTHARGS     -> gpurun_out/$TAG_synth_summary.txt
#   pmc              PMC (SQ + HBM passes) of one training step              -> gpurun_out/$TAG_pmc/summary.txt
#   synthpmc         PMC of one synthesis step (bench_synth.py --batch 64)
#   ab               same-box A/B: ab/libssamd_kernels_$BASE.so (A) vs in-tree (B), ROUNDS x CONFIGS
#   abtree           same-box A/B of whole trees: ab/base (git worktree, pre-built) (A) vs this tree (B)
#   abexp            same-box A/B of experiment switches: EXPS="arm1|arm2|..." (arm = name=v,name=v, - = defaults,
#                    base = the ab/base tree)
#   py:<script>      python <script> (a tools/ experiment), output -> gpurun_out/<script>.log
#   pmcpy:<script>   PMC passes (PASSES="ctr ctr ...|ctr ...") of python <script> $PYARGS -> gpurun_out/<script>_pmc.txt
set -o pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
cd "$R"; mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
TAG=${TAG:-run}

jv() { python -c 'import json,sys; d=json.loads([l for l in sys.stdin.read().strip().splitlines() if l.startswith("{")][-1]); print(d["value"], d["ms_per_step"], d.get("synth_rtf"))'; }

prof_py() {  # tag script args...: kernel trace + stats of a python run
  local tag=$1; shift
  mkdir -p "$R/gpurun_out/$tag"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/$tag" -o run -- python3 "$@" > "$R/gpurun_out/$tag.log" 2>&1) || { tail -30 "gpurun_out/$tag.log"; return 1; }
}

pmc_py() {  # tag counters script args...
  local tag=$1 ctr=$2; shift 2
  mkdir -p "$R/gpurun_out/$tag"
  (cd /tmp && timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d "$R/gpurun_out/$tag" -o p -- python3 "$@" > "$R/gpurun_out/$tag.log" 2>&1) || { tail -20 "gpurun_out/$tag.log"; return 1; }
}

SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
MEM="FETCH_SIZE GRBM_GUI_ACTIVE"  # FETCH_SIZE takes 3 of the 4 TCC counters: WRITE_SIZE needs its own pass

for task in "$@"; do
  echo "== $task"
  case "$task" in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ${K:+-k "$K"} > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
      tail -1 gpurun_out/tests.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
      tail -1 gpurun_out/smoke.log ;;
    bench)
      for i in $(seq 1 ${REP:-1}); do
        timeout -k 10 400 python bench.py ${BENCHARGS} > gpurun_out/bench_$i.log 2>&1 || { tail -30 gpurun_out/bench_$i.log; exit 1; }
        echo "bench[$i] $BENCHARGS: $(tail -1 gpurun_out/bench_$i.log | jv)"
        tail -1 gpurun_out/bench_$i.log >> gpurun_out/bench_lines.jsonl
      done ;;
    prof)
      prof_py "$TAG" "$R/${TREE:+$TREE/}bench.py" --steps 3 --warmup 2 --synth-steps 0 ${BENCHARGS} || exit 1
      t=$(find gpurun_out/$TAG -name "*kernel_trace.csv" | head -1)
      f=$(find gpurun_out/$TAG -name "*kernel_stats.csv" | head -1)
      python tools/prof_summary.py "$f" "$t" > gpurun_out/${TAG}_summary.txt
      python tools/last_step.py "$t" 70 > gpurun_out/${TAG}_last_step.txt
      python tools/grid_census.py "$t" --top 60 > gpurun_out/${TAG}_grid.txt
      python tools/stream_split.py "$t" --last 2 --detail --gaps 25 --tail ${TAILN:-0} > gpurun_out/${TAG}_split.txt 2>&1 || true
      rm -f "$t"; rm -rf gpurun_out/$TAG
      head -25 gpurun_out/${TAG}_last_step.txt ;;
    synthprof)
      prof_py "${TAG}_synth" "$R/bench_synth.py" --steps 2 --warmup 1 ${SYNTHARGS} || exit 1
      t=$(find gpurun_out/${TAG}_synth -name "*kernel_trace.csv" | head -1)
      f=$(find gpurun_out/${TAG}_synth -name "*kernel_stats.csv" | head -1)
      python tools/prof_summary.py "$f" "$t" > gpurun_out/${TAG}_synth_summary.txt
      python tools/grid_census.py "$t" --all --top 60 > gpurun_out/${TAG}_synth_grid.txt 2>&1 || true
      rm -rf gpurun_out/${TAG}_synth
      head -30 gpurun_out/${TAG}_synth_summary.txt ;;
    pmc)
      pmc_py ${TAG}_pmc/train_sq "$SQ" "$R/bench.py" --steps 1 --warmup 1 --synth-steps 0 ${BENCHARGS} &&
      pmc_py ${TAG}_pmc/train_mem "$MEM" "$R/bench.py" --steps 1 --warmup 1 --synth-steps 0 ${BENCHARGS} || exit 1
      python tools/pmc_summary.py gpurun_out/${TAG}_pmc > gpurun_out/${TAG}_pmc_summary.txt || exit 1
      find gpurun_out/${TAG}_pmc -name "*.csv" -size +4M -delete
      head -50 gpurun_out/${TAG}_pmc_summary.txt ;;
    synthpmc)
      pmc_py ${TAG}_spmc/synth_sq "$SQ" "$R/bench_synth.py" --steps 1 --warmup 0 --batch 64 ${SYNTHARGS} &&
      pmc_py ${TAG}_spmc/synth_mem "$MEM" "$R/bench_synth.py" --steps 1 --warmup 0 --batch 64 ${SYNTHARGS} || exit 1
      python tools/pmc_summary.py gpurun_out/${TAG}_spmc > gpurun_out/${TAG}_spmc_summary.txt || exit 1
      find gpurun_out/${TAG}_spmc -name "*.csv" -size +4M -delete
      head -40 gpurun_out/${TAG}_spmc_summary.txt ;;
    ab)
      A=ab/libssamd_kernels_$BASE.so
      [ -f "$A" ] || { echo "missing $A"; exit 1; }
      for i in $(seq 1 ${ROUNDS:-2}); do
        for cfg in ${CONFIGS:-LJSpeech}; do
          SSAMD_KERNEL_LIB=$A timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config $cfg --synth-steps 0 ${BENCHARGS} > gpurun_out/ab_A.log 2>&1 || { tail -20 gpurun_out/ab_A.log; exit 1; }
          echo "A $cfg $(jv < gpurun_out/ab_A.log)"
          timeout -k 10 300 python bench.py --steps 10 --warmup 3 --config $cfg --synth-steps 0 ${BENCHARGS} > gpurun_out/ab_B.log 2>&1 || { tail -20 gpurun_out/ab_B.log; exit 1; }
          echo "B $cfg $(jv < gpurun_out/ab_B.log)"
        done
      done ;;
    abtree)
      # same-box A/B of the whole tree: ab/base (a git worktree of BASE, built on the CPU) = A, this tree = B
      [ -f ab/base/bench.py ] || { echo "missing ab/base (git worktree add ab/base <rev> && (cd ab/base && python csrc/build.py))"; exit 1; }
      for i in $(seq 1 ${ROUNDS:-2}); do
        for cfg in ${CONFIGS:-LJSpeech}; do
          (cd ab/base && timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 --config $cfg --synth-steps 0 ${BENCHARGS} > ../../gpurun_out/ab_A.log 2>&1) || { tail -20 gpurun_out/ab_A.log; exit 1; }
          echo "A $cfg $(jv < gpurun_out/ab_A.log)"
          timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 --config $cfg --synth-steps 0 ${BENCHARGS} > gpurun_out/ab_B.log 2>&1 || { tail -20 gpurun_out/ab_B.log; exit 1; }
          echo "B $cfg $(jv < gpurun_out/ab_B.log)"
        done
      done ;;
    abexp)
      # same-box A/B of experiment switches in this tree: EXPS="name=v,name=v|name=v" (| separates arms; "-" = defaults)
      IFS='|' read -ra ARMS <<< "${EXPS:--}"
      for i in $(seq 1 ${ROUNDS:-2}); do
        for cfg in ${CONFIGS:-LJSpeech}; do
          for arm in "${ARMS[@]}"; do
            e=$arm; [ "$e" = "-" ] && e=""
            d=.; [ "$e" = "base" ] && { d=ab/base; e=""; }
            case "$e" in tree:*) d=${e#tree:}; e="";; esac
            (cd $d && SSAMD_EXPERIMENTAL="$e" timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 --config $cfg --synth-steps 0 ${BENCHARGS} > $R/gpurun_out/abexp.log 2>&1) || { tail -20 gpurun_out/abexp.log; exit 1; }
            echo "[$arm] $cfg $(jv < gpurun_out/abexp.log)"
          done
        done
      done ;;
    py:*)
      s=${task#py:}; b=$(basename "$s" .py)
      timeout -k 10 400 python -u "$s" ${PYARGS} > gpurun_out/$b.log 2>&1 || { tail -40 gpurun_out/$b.log; exit 1; }
      tail -${PYTAIL:-25} gpurun_out/$b.log ;;
    pmcpy:*)
      s=${task#pmcpy:}; b=$(basename "$s" .py)
      IFS='|' read -ra PS <<< "${PASSES:-$SQ}"
      rm -rf gpurun_out/${b}_pmc; i=0
      for ctr in "${PS[@]}"; do
        i=$((i + 1))
        pmc_py ${b}_pmc/p$i "$ctr" "$R/$s" ${PYARGS} || exit 1
      done
      python tools/pmc_kernels.py gpurun_out/${b}_pmc "${PMCFILT:-}" > gpurun_out/${b}_pmc.txt || exit 1
      rm -rf gpurun_out/${b}_pmc
      cat gpurun_out/${b}_pmc.txt ;;
    *) echo "unknown task $task"; exit 2 ;;
  esac
done
