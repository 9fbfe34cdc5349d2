"""bench.py's rank launcher and DP protocol on the CPU (no GPU needed).

The driver runs ``python bench.py --gpus N`` with no launcher: bench.py must start the N rank
processes itself (before any GPU call), report ``n_gpus == N`` and fail when a rank fails.  The
ranks run the train_image.py step (train_image.py:93-144, the one exchange step being the
gradient all-reduce of :139-144) through the gloo backend on CPU tensors at a small size."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, extra_env=None, timeout=600):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(MHADA_BENCH_BACKEND="gloo", OMP_NUM_THREADS="2")
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, cwd=REPO, env=env,
                          capture_output=True, text=True, timeout=timeout)


def _json_lines(out):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


# two images per rank: each rank's micro-batch is one coupled forward call
SMALL = ["--train", "--device", "cpu", "--train-res", "64", "--train-batch", "2", "--steps", "1", "--warmup", "0"]


def test_gpus_2_self_launches_two_ranks():
    p = _run(["--gpus", "2"] + SMALL)
    assert p.returncode == 0, p.stderr[-4000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout  # rank 0 only
    r = lines[0]
    assert r["n_gpus"] == 2
    assert r["config"]["global_batch"] == 4 and r["config"]["backend"] == "gloo"
    ag = r["rank_agreement"]
    assert ag["identical"] and ag["world"] == 2 and ag["backend"] == "gloo", ag
    assert all(v == v for v in r["last_losses"].values())  # finite (not NaN)


def test_world_size_must_match_gpus():
    p = _run(["--gpus", "2"] + SMALL, extra_env={"WORLD_SIZE": "1", "RANK": "0"})
    assert p.returncode != 0
    assert "WORLD_SIZE=1 but --gpus 2" in p.stderr


def test_failing_rank_fails_the_job():
    # a resolution the ViT rejects (not a multiple of the patch size) makes every rank raise;
    # the parent must exit non-zero instead of printing a line
    p = _run(["--gpus", "2", "--train", "--device", "cpu", "--train-res", "60", "--train-batch", "1",
              "--steps", "1", "--warmup", "0"], timeout=300)
    assert p.returncode != 0
    assert not _json_lines(p.stdout)


@pytest.mark.parametrize("argv", [["--gpus", "2", "--device", "cpu", "--steps", "1"]])
def test_cpu_device_is_training_only(argv):
    p = _run(argv, timeout=120)
    assert p.returncode != 0
