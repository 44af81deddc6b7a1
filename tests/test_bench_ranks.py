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
    assert b["rank_parity"] is None                              # --no-cpu: no reference processes
    job = b["roofline"]["job"]
    assert job["peak"] == 2 * bench_peak() and len(job["per_rank_frac"]) == 2
    assert job["avg_launch_ms_max_over_ranks"] == 1.0


def bench_peak():
    sys.path.insert(0, ROOT)
    import bench
    return bench.HBM_PEAK_GBS


# the stub's ranks run 1,200 requests per replica: the reference processes
# fill 600 (the "warmup") and replay the next 600 (the "timed window")
PARITY_ARGS = ["--gpus", "2", "--dist-backend", "gloo", "--steps", "1", "--warmup", "1", "--chunk", "600",
               "--ensemble-seconds", "2"]


def test_two_ranks_check_their_replicas_against_the_reference(tmp_path):
    """N>1: each rank forks reference processes for two of its replicas,
    compares their delays with its own and the results are gathered: the line
    carries parity true, one entry per rank, and the job-level roofline."""
    r = _run(PARITY_ARGS, tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    b = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    rp = b["rank_parity"]
    assert b["parity"] is True and rp["bit_identical"] is True
    assert [p["rank"] for p in rp["per_rank"]] == [0, 1]
    for p in rp["per_rank"]:
        assert p["replicas"] == [0, 1] and p["bit_identical"]
        assert p["requests_compared"] == 2 * 1200
    assert b["cpu_baseline_ensemble"] is None and b["replica_parity"] is None


def test_a_mismatch_on_one_rank_fails_the_job(tmp_path):
    r = _run(PARITY_ARGS, tmp_path, {"PU_STUB_CORRUPT_RANK": "1"})
    assert r.returncode == 1, r.stderr[-3000:]
    b = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    rp = b["rank_parity"]
    assert b["parity"] is False and rp["bit_identical"] is False
    assert [p["bit_identical"] for p in rp["per_rank"]] == [True, False]
    assert "PARITY FAILURE" in r.stderr


def test_gpus_must_match_world_size(tmp_path):
    r = _run(["--gpus", "2", "--dist-backend", "gloo", "--no-cpu"], tmp_path,
             {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "refusing" in r.stderr


def test_other_configurations_keep_the_contract(tmp_path):
    """--config C3: the same line for the 256-core three-level shape (its own
    stream and metric), with the per-rank reference parity."""
    r = _run([*PARITY_ARGS, "--config", "C3"], tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    b = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert "256 cores (C3)" in b["metric"] and b["config"]["workload"].startswith("C3:")
    assert b["parity"] is True and len(b["rank_parity"]["per_rank"]) == 2
