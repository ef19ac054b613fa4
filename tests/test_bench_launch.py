"""bench.py's multi-rank launcher and gather protocol on the CPU (gloo).

`python bench.py --gpus N` without a torch.distributed environment starts N
rank processes itself; `--config rehearsal` runs the N > 1 protocol (barrier +
max-over-ranks timing, fixed-capacity record all-gather) on synthetic find
results without touching a GPU.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def _run(args, env, timeout=240):
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=timeout)


def test_launcher_two_ranks():
    p = _run(["--config", "rehearsal", "--gpus", "2", "--steps", "3", "--warmup", "1"], _env())
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3
    assert d["gather_ok"] is True
    assert d["counts"] == [100, 101] and d["gathered_records"] == 201


def test_launcher_three_ranks():
    p = _run(["--config", "rehearsal", "--gpus", "3", "--steps", "2", "--warmup", "0"], _env())
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    assert d["n_gpus"] == 3 and d["gather_ok"] is True


def test_world_mismatch_fails():
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = _run(["--config", "rehearsal", "--gpus", "2", "--steps", "1", "--warmup", "0"], env)
    assert p.returncode != 0
    assert "WORLD_SIZE" in p.stderr
