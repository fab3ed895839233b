# End-to-end CLI run on the GPU (train.py synthetic -> checkpoint -> resume -> synthesize.py single + batch):
# bash tools/gpu_cli_e2e.sh [config]   (logs + wavs under gpurun_out/cli_e2e; the ~0.4 GB checkpoints go to
# $TMPDIR so the box's gpurun_out stays under the copy-back cap)
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
CFG=${1:-LJSpeech}
OUT=gpurun_out/cli_e2e/$CFG
CK=${TMPDIR:-/tmp}/cli_e2e_ckpt/$CFG
rm -rf "$OUT" "$CK"; mkdir -p "$OUT" "$CK"
python - "$CFG" "$OUT" "$CK" <<'PY'
import sys, yaml
cfg, out, ck = sys.argv[1], sys.argv[2], sys.argv[3]
t = yaml.safe_load(open(f"config/{cfg}/train.yaml"))
t["path"] = {"ckpt_path": ck, "log_path": f"{out}/log", "result_path": f"{out}/result"}
t["step"].update(total_step=40, log_step=10, synth_step=20, val_step=20, save_step=20)
yaml.safe_dump(t, open(f"{out}/train.yaml", "w"))
PY
P=config/$CFG/preprocess.yaml; M=config/$CFG/model.yaml; T=$OUT/train.yaml
timeout -k 10 400 python train.py -p $P -m $M -t $T --synthetic --max_steps 30 > $OUT/train.log 2>&1 || { tail -30 $OUT/train.log; exit 1; }
tail -3 $OUT/train.log
ls $CK
timeout -k 10 400 python train.py -p $P -m $M -t $T --synthetic --restore_step 20 --max_steps 40 > $OUT/resume.log 2>&1 || { tail -30 $OUT/resume.log; exit 1; }
tail -2 $OUT/resume.log
# the resumed run's step-30 losses must equal the uninterrupted run's (weights, Adam, LR, data position)
a=$(grep '^Step 30/' $OUT/train.log | cut -d, -f2-); b=$(grep '^Step 30/' $OUT/resume.log | cut -d, -f2-)
[ -n "$a" ] && [ "$a" = "$b" ] || { echo "RESUME MISMATCH at step 30: [$a] vs [$b]"; exit 1; }
echo "resume exact at step 30:$a"
timeout -k 10 300 python synthesize.py --mode single --text "Printing, in the only sense with which we are at present concerned." --restore_step 40 -p $P -m $M -t $T > $OUT/synth.log 2>&1 || { tail -30 $OUT/synth.log; exit 1; }
tail -2 $OUT/synth.log
find $OUT/result -name "*.wav"
rm -rf "$CK"
