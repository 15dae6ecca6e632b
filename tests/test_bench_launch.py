"""CPU tests of bench.py's multi-GPU entry: `--gpus N`
runs N ranks itself (torch.distributed.run child, one process per GPU) and
reports the whole-job value (SUM of units over ranks / MAX of time); a box
with fewer devices than N is refused, never measured as one GPU.  --stub
replaces the GPU step with a CPU sleep (gloo), so the launcher, rank setup and
aggregation run here exactly as on the GPU node."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None, timeout=240):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, cwd=REPO, env=e,
                          capture_output=True, text=True, timeout=timeout)


def _line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_two_ranks_sum_and_max():
    r = _run(["--gpus", "2", "--stub", "--steps", "5", "--warmup", "1", "--batch", "1000"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2 and d["steps"] == 5 and d["stub"] is True
    assert d["units_total"] == 2 * 1000 * 5                      # SUM over both ranks
    assert d["seconds_max"] >= 5 * 0.004                         # rank 1 sleeps 4 ms per step: MAX over ranks
    assert abs(d["value"] - d["units_total"] / d["seconds_max"]) < 1e-6 * d["value"]


def test_four_ranks():
    r = _run(["--gpus", "4", "--stub", "--steps", "2", "--warmup", "0", "--batch", "10"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 4 and d["units_total"] == 4 * 10 * 2
    assert d["seconds_max"] >= 2 * 0.008


def test_single_rank_stub():
    r = _run(["--gpus", "1", "--stub", "--steps", "3", "--warmup", "0", "--batch", "7"])
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 1 and d["units_total"] == 21


def test_too_few_gpus_refused():
    # this container has no GPU: --gpus 2 must fail loudly, not report one GPU
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu"], timeout=120)
    assert r.returncode == 2
    assert "refusing" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_world_size_mismatch_refused():
    r = _run(["--gpus", "2", "--stub", "--steps", "1"], env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE=1" in r.stderr
