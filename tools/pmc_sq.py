"""Wave-state PMC counters of the engine kernel (run on the GPU box).

Where a wave's cycles go: SQ_WAIT_ANY (parked on s_waitcnt / barrier: memory
latency), SQ_WAIT_INST_ANY (issue stalls), SQ_ACTIVE_INST_* (issuing), plus
instruction mixes and L2 hit/miss — each pass a separate rocprofv3 run of
bench.py (counter-block limits: MI355X_MICROARCH.md; no --pmc pass is combined
with a trace domain).  Sums over the timed launches (the last `steps`).

    python tools/pmc_sq.py --out gpurun_out/sq.json -- --steps 3 --warmup 5 --no-cpu --no-extras
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the timed (throughput) launches of bench.py: time-sliced or replica-pool, the
# compiled configuration's kernel or the ahead-of-time one
KERNEL = "uncore_kernel<1, 1, false>|uncore_kernel<1, 2, false>|pu_jit_uncore_s1_h0|pu_jit_uncore_s2_h0"
PASSES = [
    ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"],
    ["SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS", "SQ_INSTS_VALU",
     "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"],
    ["TCC_HIT_sum", "TCC_MISS_sum", "TCC_EA0_RDREQ_sum", "TCC_EA0_WRREQ_sum"],
    ["SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_INSTS_LDS"],
    ["SQ_THREAD_CYCLES_VALU", "SQ_ACTIVE_INST_VALU"],
    ["SQ_INSTS_SMEM", "SQ_INSTS_BRANCH", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_MISC", "SQ_INSTS_SENDMSG"],
    ["SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_TRANS_F64"],
]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--work", default=os.path.join(ROOT, "gpurun_out", "pmc_sq"))
    ap.add_argument("--kernel", default=KERNEL, help="kernel name substrings to sum over, '|'-separated")
    ap.add_argument("bench_args", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    bargs = [x for x in a.bench_args if x != "--"]
    steps = int(bargs[bargs.index("--steps") + 1]) if "--steps" in bargs else 10
    os.makedirs(a.work, exist_ok=True)
    os.environ.setdefault("TMPDIR", "/tmp")
    out = {"bench_args": bargs, "passes": PASSES, "per_launch": {}}
    for i, counters in enumerate(PASSES):
        d = os.path.join(a.work, f"p{i}")
        shutil.rmtree(d, ignore_errors=True)
        cmd = ["rocprofv3", "--pmc", *counters, "--output-format", "csv", "-d", d, "-o", "run", "--",
               sys.executable, os.path.join(ROOT, "bench.py"), *bargs]
        print("+", " ".join(cmd), flush=True)
        with open(os.path.join(a.work, f"p{i}.log"), "w") as f:
            r = subprocess.run(cmd, cwd=ROOT, stdout=f, stderr=subprocess.STDOUT, timeout=300)
        if r.returncode != 0:
            out[f"pass{i}_error"] = r.returncode
            continue
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        vals: dict = {}
        for fn in files:
            with open(fn) as fh:
                for row in csv.DictReader(fh):
                    if not any(k in row.get("Kernel_Name", "") for k in a.kernel.split("|")):
                        continue
                    did = int(row["Dispatch_Id"])
                    vals.setdefault(row["Counter_Name"], {}).setdefault(did, 0.0)
                    vals[row["Counter_Name"]][did] += float(row["Counter_Value"])
        for name, per in vals.items():
            ids = sorted(per)[-steps:]
            out["per_launch"][name] = sum(per[k] for k in ids) / len(ids)
    # accesses per launch of these runs (the bench line each pass printed)
    acc = []
    for i in range(len(PASSES)):
        try:
            with open(os.path.join(a.work, f"p{i}.log")) as f:
                line = [ln for ln in f if ln.startswith("{")][-1]
            b = json.loads(line)
            acc.append(b["config"]["replicas_per_gpu"] * b["config"]["mean_requests_per_replica_per_step"])
        except (OSError, IndexError, ValueError, KeyError):
            pass
    pl = out["per_launch"]
    if acc:
        out["accesses_per_launch"] = sum(acc) / len(acc)
        out["per_access"] = {k: v / out["accesses_per_launch"] for k, v in pl.items() if k.startswith("SQ_INSTS")}
    if pl.get("SQ_LDS_IDX_ACTIVE"):
        out["lds_bank_conflict_share"] = pl.get("SQ_LDS_BANK_CONFLICT", 0.0) / pl["SQ_LDS_IDX_ACTIVE"]
    if pl.get("SQ_ACTIVE_INST_VALU") and "SQ_THREAD_CYCLES_VALU" in pl:
        # rocprof's VALUUtilization: active lanes per VALU issue cycle / 64
        out["valu_lane_utilization"] = pl["SQ_THREAD_CYCLES_VALU"] / (pl["SQ_ACTIVE_INST_VALU"] * 64.0)
    sys.path.insert(0, ROOT)
    from primesim_amd import uncore
    out["src_hash"] = uncore.library_source_hash()
    if "SQ_WAVE_CYCLES" in pl and pl["SQ_WAVE_CYCLES"]:
        wc = pl["SQ_WAVE_CYCLES"]
        out["share_of_wave_cycles"] = {k: pl[k] / wc for k in pl if k.startswith(("SQ_WAIT", "SQ_ACTIVE"))}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
