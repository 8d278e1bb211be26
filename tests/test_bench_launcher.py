"""`python bench.py --gpus N` measures N ranks or fails: without WORLD_SIZE the
bench starts the N ranks itself, so with fewer visible GPUs than asked (none in this container) it must
exit non-zero instead of printing a one-GPU line; a WORLD_SIZE that disagrees with --gpus is an error
too. CPU-only: these runs stop before any GPU call."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=180, env=e, cwd=ROOT)


def test_gpus_2_without_gpus_fails():
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"], HIP_VISIBLE_DEVICES="")
    assert r.returncode != 0
    assert r.stdout.strip() == ""  # no JSON line: never a silent smaller run
    assert "visible GPU" in r.stderr


def test_gpus_2_gloo_rehearsal_without_gpu_fails():
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"], DDSHE_DIST_BACKEND="gloo", HIP_VISIBLE_DEVICES="")
    assert r.returncode != 0 and r.stdout.strip() == ""


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "3", "--steps", "1"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr
