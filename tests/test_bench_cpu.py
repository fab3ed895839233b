"""bench.py launcher on the CPU (gloo): ``--gpus N`` starts N ranks by itself, every
rank sees WORLD_SIZE == N, the JSON reports the world actually seen, the frame
count is the sum over ranks of the timed steps, and a failing rank ends the job
with a non-zero status naming the rank."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    env.update(kw)
    return env


ARGS = ["--steps", "2", "--warmup", "1", "--tiny", "--batch", "3", "--pool", "3"]


def _expected_frames(world, steps=2, warm=1, batch=3, pool=3):
    from speakingstyle_amd.data.synthetic import SyntheticBatches

    total = 0
    for r in range(world):
        gen = SyntheticBatches(batch, seed=1000 + r, max_seq_len=1000)
        ps = []
        for _ in range(pool):
            b = gen.make_batch()
            ps.append((len(b[0]) * b[8], gen.last_valid_frames))
        ps.sort(key=lambda e: -e[0])
        total += sum(ps[(warm + i) % pool][1] for i in range(steps))
    return total


def test_bench_launches_two_ranks():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--synth-batch", "2", "--synth-steps", "2",
                        "--synth-b1-runs", "3"] + ARGS,
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["world_size_seen"] == 2
    assert rec["config"]["parallelism"] == "dp2" and rec["config"]["global_batch"] == 6
    assert rec["bucket_overlap"] is True
    frames = rec["value"] * rec["ms_per_step"] * rec["steps"] / 1000.0
    np.testing.assert_allclose(frames, _expected_frames(2), rtol=2e-3)
    assert rec["synth_rtf"] > 0 and rec["synth"]["batch_per_gpu"] == 2 and rec["synth"]["distinct_batches"] == 2
    b1 = rec["synth"]["b1"]  # batch-1 latency (like-for-like with the reference's 113-frame point)
    assert rec["synth_rtf_b1"] > 0 and b1["runs"] == 3 and b1["mel_frames"] > 0
    assert rec["synth_vs_baseline"] == round(1.33 / rec["synth_rtf_b1"], 1)


def test_bench_single_process_default():
    r = subprocess.run([sys.executable, "bench.py", "--synth-steps", "0"] + ARGS, cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["n_gpus"] == 1 and "synth_rtf" not in rec
    frames = rec["value"] * rec["ms_per_step"] * rec["steps"] / 1000.0
    np.testing.assert_allclose(frames, _expected_frames(1, warm=1), rtol=2e-3)


def test_bench_failing_rank_exits_nonzero():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--synth-steps", "0"] + ARGS, cwd=ROOT,
                       env=_env(SSAMD_EXPERIMENTAL="fail_rank=1", SSAMD_DIST_TIMEOUT_S="60"), capture_output=True, text=True,
                       timeout=900)
    assert r.returncode != 0
    assert "[rank 1] FAILED" in r.stderr and "injected failure on rank 1" in r.stderr


def test_world_size_mismatch_is_an_error():
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "3", "--synth-steps", "0"] + ARGS, cwd=ROOT,
                       env=_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True, timeout=600)
    assert r.returncode != 0 and "3 ranks were requested" in r.stderr


def test_slurm_job_script_syntax():
    """scripts/train_job.sh (the reference's scripts/train_job.sh counterpart): valid bash,
    one torchrun rank per GPU, RCCL env set; a full 2-rank CPU run of it is in docs (slow)."""
    import subprocess

    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts", "train_job.sh")
    subprocess.run(["bash", "-n", path], check=True)
    text = open(path).read()
    assert "torch.distributed.run" in text and "--nproc-per-node" in text
    assert "HSA_ENABLE_IPC_MODE_LEGACY=0" in text and "#SBATCH --gres=gpu:8" in text
