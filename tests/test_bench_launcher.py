"""bench.py --gpus N starts its own N rank processes when no launcher is around it
(VERDICT r2 #1): GPU-free stub ranks check the rank environment, the gloo rendezvous
on 127.0.0.1, the single JSON line, and that a failing rank fails the job."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(n, extra_env=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n), "--stub"],
                          cwd=REPO, env=env, capture_output=True, text=True, timeout=300)


def test_launcher_starts_n_ranks_and_prints_one_line():
    out = _run(2)
    assert out.returncode == 0, out.stderr
    # gloo's own connection notice also goes to stdout; the bench line is the one JSON line
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    rec = json.loads(lines[0])
    assert rec["stub"] and rec["n_ranks"] == 2
    ranks = rec["ranks"]
    assert [r["RANK"] for r in ranks] == ["0", "1"]
    assert [r["LOCAL_RANK"] for r in ranks] == ["0", "1"]
    assert all(r["WORLD_SIZE"] == "2" and r["MASTER_ADDR"] == "127.0.0.1" for r in ranks)
    assert len({r["pid"] for r in ranks}) == 2 and os.getpid() not in {r["pid"] for r in ranks}


def test_launcher_fails_when_a_rank_fails():
    out = _run(2, {"RYD_BENCH_STUB_FAIL_RANK": "1"})
    assert out.returncode != 0


def test_single_gpu_runs_in_process():
    out = _run(1)
    assert out.returncode == 0, out.stderr
    rec = json.loads(out.stdout.strip().splitlines()[-1])
    assert rec["n_ranks"] == 1 and rec["ranks"][0]["pid"] != os.getpid()
