"""bench.py --gpus N on CPU: the launch logic and the cross-rank reduction.

tests/bench_stub_rank.py runs bench.main() with the GPU engine replaced by the
CPU restatement (test-only stub).  `--gpus 2` without WORLD_SIZE makes bench
start two rank processes itself (no exec, fresh children); they join a gloo
group, and rank 0 prints one JSON line whose n_gpus is 2, whose value is the
requests of BOTH ranks over the max of their times, and whose replica count
is the job's.  A --gpus that disagrees with WORLD_SIZE is refused.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB = os.path.join(ROOT, "tests", "bench_stub_rank.py")


def _run(args, tmp_path, extra_env=None):
    env = dict(os.environ, PU_STUB_OUT=str(tmp_path), PU_STUB_REQS="1200")
    env.pop("WORLD_SIZE", None)
    env.update(extra_env or {})
    return subprocess.run([sys.executable, STUB, *args], capture_output=True, text=True, timeout=600, env=env,
                          cwd=ROOT)


def test_two_ranks_launched_by_bench_reduce_over_ranks(tmp_path):
    r = _run(["--gpus", "2", "--dist-backend", "gloo", "--no-cpu", "--steps", "3", "--warmup", "1"], tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout            # rank 0 only
    b = json.loads(lines[0])
    per_rank = [tuple(map(int, (tmp_path / f"rank{k}.txt").read_text().split())) for k in range(2)]
    total = sum(p for p, _ in per_rank)
    assert b["n_gpus"] == 2
    assert total == 2 * 2 * 1200
    assert b["value"] == total / 1.5             # both ranks' requests over the slowest rank's 0.5 + 1 s
    assert b["ms_per_step"] == 1.5 / 3 * 1e3
    assert b["config"]["replicas_total"] == 4
    assert b["per_simulation_accesses_per_s"] == b["value"] / 4
    assert per_rank[0][1] != per_rank[1][1]      # the ranks simulated disjoint replicas (seeds)
    assert b["parity"] is None and b["cpu_baseline"] is None   # the CPU baseline is an N=1 line only


def test_gpus_must_match_world_size(tmp_path):
    r = _run(["--gpus", "2", "--dist-backend", "gloo", "--no-cpu"], tmp_path,
             {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "refusing" in r.stderr
