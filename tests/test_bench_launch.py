"""bench.py's rank-count contract on the CPU (no GPU call is reached): a launcher's WORLD_SIZE that differs from
--gpus, and --comm rccl with fewer GPUs than ranks, exit non-zero before anything is measured,
so a multi-GPU run can never print a line for the wrong N."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
QUICK = ["--steps", "1", "--warmup", "0", "--other", "0", "--cpu-runs", "0", "--cpu-seconds", "0", "--frontend", "0",
         "--solve-all", "0", "--model-scaling", "0", "--weak", "0"]


def _run(args, **env):
    e = dict(os.environ, **env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args + QUICK, cwd=ROOT, env=e,
                          capture_output=True, text=True, timeout=120)


def test_world_size_mismatch_exits_nonzero():
    r = _run(["--gpus", "1"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0 and "WORLD_SIZE=2 but --gpus 1" in r.stderr
    assert r.stdout.strip() == ""


def test_rccl_needs_one_gpu_per_rank():
    # under a launcher (WORLD_SIZE set) on a box with fewer GPUs than ranks: refused before any rendezvous (64 ranks:
    # more GPUs than any box has, so the refusal does not depend on how HIP reads an empty HIP_VISIBLE_DEVICES)
    r = _run(["--gpus", "64", "--comm", "rccl"], WORLD_SIZE="64", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0 and "one GPU per rank" in r.stderr
    assert r.stdout.strip() == ""
