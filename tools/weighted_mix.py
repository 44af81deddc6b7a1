"""Executed instruction mix of the headline kernel by region: the static
instructions of each region (line tables: every instruction's inline chain
from llvm-symbolizer) times how often the region runs per access.  Answers
"which source region issues the SALU / VALU work per access" with executed
counts, not static ones (round-4 verdict item 3).

Regions follow the engine's structure (engine.hip): the request loop, the
L1 walk (mesi + set probes), the home slice (access_home_impl), the probe
loop, the downward share/inval (down_impl), a transmit's setup and tail
(net_transmit outside the hop window), the route window (per window), the
M/G/1 wait (per window), the tree operation (per tree hop).  A region inlined
at several call sites is one copy per site; every copy is the same code, so a
region's executed count is its static count per copy times the region's
visits per access.  Visits per access come from the PU_PROF region profile
(windows, tree hops: --regions) and the CPU restatement's counters on the
same stream (transmits, home accesses, down calls).  Code outside every
region (kernel prologue, counter flush, replica pool) runs once per launch
or per replica and is listed with weight 0.

    python tools/weighted_mix.py [--regions profiles/r4n_regions_ens.txt] [--kernel pu_jit_uncore_s2_h0]
"""
from __future__ import annotations

import argparse
import collections
import glob
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
LLVM = "/opt/rocm/lib/llvm/bin"
from salu_lines import klass  # noqa: E402

ENGINE = os.path.join(ROOT, "primesim_amd", "csrc", "engine.hip")


def build_hsaco(preset: str, d: str, extra: str = "", kernel: str = "pu_jit_uncore_s2_h0") -> str:
    env = dict(os.environ, PRIMEUNCORE_JIT_CACHE=d, PRIMEUNCORE_JIT_EXTRA=("-gline-tables-only " + extra).strip())
    code = ("import ctypes as C, sys; sys.path.insert(0, %r); import primesim_amd as P; "
            "from primesim_amd import config as CF, uncore; cfg = P.config_from_dict(CF.preset(%r)); "
            "rc = uncore.lib().pu_config_jit_warm(C.byref(cfg)); sys.exit(0 if rc >= 0 else 1)") % (ROOT, preset)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True)
    if r.returncode != 0:
        raise SystemExit(r.stderr[-3000:])
    # two code objects per configuration (jit.cpp): the one holding the kernel
    (hsaco,) = [f for f in glob.glob(os.path.join(d, "*.hsaco")) if kernel.encode() in open(f, "rb").read()]
    return hsaco


def instructions(hsaco: str, kernel: str) -> list:
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", hsaco], capture_output=True,
                         text=True).stdout
    out, inside = [], False
    for ln in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <([^>]+)>:", ln)
        if m:
            inside = m.group(1) == kernel
            continue
        if not inside:
            continue
        m = re.match(r"^\s+(\S+).*//\s*([0-9A-F]+):", ln)
        if m:
            out.append((int(m.group(2), 16), m.group(1)))
    return out


def chains(hsaco: str, addrs: list) -> list:
    inp = "".join(f"0x{a:x}\n" for a in addrs)
    r = subprocess.run([f"{LLVM}/llvm-symbolizer", "--inlining", f"--obj={hsaco}", "--functions=short"],
                       input=inp, capture_output=True, text=True)
    res, cur, lines = [], [], r.stdout.splitlines()
    i = 0
    while i < len(lines):
        if not lines[i].strip():
            res.append(cur)
            cur = []
            i += 1
            continue
        fn = lines[i].strip()
        loc = lines[i + 1].strip() if i + 1 < len(lines) else ""
        m = re.search(r"([\w.]+):(\d+)", loc)
        cur.append((re.sub(r"<.*", "", fn), m.group(1) if m else "?", int(m.group(2)) if m else 0))
        i += 2
    if cur:
        res.append(cur)
    return res


def marker_lines() -> dict:
    """Line numbers in engine.hip that bound net_transmit's window and tree sections."""
    src = open(ENGINE).read().splitlines()

    def find(pat, start=0):
        for k in range(start, len(src)):
            if pat in src[k]:
                return k + 1
        raise SystemExit(f"marker not found: {pat}")
    nt = find("__device__ __forceinline__ uint64_t net_transmit(")
    win0 = find("for (int b0 = 0; b0 < hops; b0 += 64)", nt)
    post = find("PROF_T(p_post);", win0)
    trees = []
    k = win0
    while True:
        try:
            a = find("PROF_T(p_tree);", k)
        except SystemExit:
            break
        if a > post:
            break
        b = find("PROF_ADD(PF_NTREE, p_tree);", a)
        trees.append((a, b))
        k = b
    return {"win": (win0, post), "trees": trees}


TREE_FNS = {"tree_op", "tree_case", "ring_load", "ring_dma", "vm_wait_dma", "ring_from_lds", "ring_shift",
            "dpp_next", "dpp_prev"}


def region_of(chain: list, mk: dict) -> tuple:
    """(region, copy key) for an instruction's inline chain (innermost first)."""
    names = [f for f, _, _ in chain]
    # net_transmit frame: the line inside net_transmit is the location of the
    # frame inlined into it (or the instruction itself)
    for i, (fn, _, line) in enumerate(chain):
        if fn == "net_transmit":
            copy = tuple(l for _, _, l in chain[i + 1:])
            inner = names[:i]
            if "mg1_wait" in inner or any(n in ("rcp_nr", "div_nr") for n in inner):
                return "window: M/G/1 wait", copy
            if any(n in TREE_FNS for n in inner) or any(a <= line <= b for a, b in mk["trees"]):
                return "tree operation", copy
            w0, w1 = mk["win"]
            if w0 <= line < w1:
                return "route window", copy
            return "transmit setup/tail", copy
    for i, (fn, _, line) in enumerate(chain):
        if fn in ("down_impl", "children"):
            return "down (share/inval)", tuple(l for _, _, l in chain[i + 1:])
        if fn == "probe":
            return "probe loop", tuple(l for _, _, l in chain[i + 1:])
        if fn == "access_home_impl" or fn == "dir_stage":
            return "home slice", tuple(l for _, _, l in chain[i + 1:])
        if fn in ("mesi", "mesi_bus", "access", "tlb_translate"):
            return "L1 walk", tuple(l for _, _, l in chain[i + 1:])
        if fn == "replica_loop":
            return "request loop", tuple(l for _, _, l in chain[i + 1:])
    return "once per launch/replica", ()


def oracle_rates(requests: int) -> dict:
    """Per-access counters of the CPU restatement on bench's replica-0 stream over the bench window."""
    import bench
    import oracle as O
    import primesim_amd as P
    from primesim_amd import config as CF
    from primesim_amd.dist import replica_seed
    cfg = P.config_from_dict(CF.preset("C4"))
    n_w = 5 * 40960
    reqs = P.generate_stream(bench.stream_spec(replica_seed(bench.SEED_BASE, 0, 0), n_w + requests))
    ref = O.CpuRef(cfg)
    for prog, th in P.stream_threads(bench.stream_spec(bench.SEED_BASE)):
        ref.alloc_core(prog, th)
    ref.run(reqs[:n_w])
    a = ref.stats().as_dict()
    ref.run(reqs[n_w:])
    b = ref.stats().as_dict()
    d = {k: b[k] - a[k] for k in b if isinstance(b[k], int)}
    n = max(1, d["requests"])
    return {"transmits": d["net_accesses"] / n, "home": d["directory_ins"] / n,
            "down": d["lockdown_calls"] / n, "link_visits": d["net_distance"] / n}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("preset", nargs="?", default="C4")
    ap.add_argument("--kernel", default="pu_jit_uncore_s2_h0")
    ap.add_argument("--regions", default=os.path.join(ROOT, "profiles", "r4n_regions_ens.txt"),
                    help="PU_PROF region profile (tools/prof_regions.py output) for windows and tree hops")
    ap.add_argument("--requests", type=int, default=100000, help="oracle requests for the other rates")
    ap.add_argument("--sq", default=os.path.join(ROOT, "profiles", "r4n_sq.json"),
                    help="SQ counters of the same kernel: measured VALU/SALU per access to compare with")
    ap.add_argument("--json", default="")
    ap.add_argument("--extra", default="", help="more compile options for the compiled configuration")
    a = ap.parse_args()

    with tempfile.TemporaryDirectory(prefix="pu_wmix_") as d:
        hsaco = build_hsaco(a.preset, d, a.extra, a.kernel)
        ins = instructions(hsaco, a.kernel)
        ch = chains(hsaco, [x for x, _ in ins])
    assert len(ch) == len(ins), (len(ch), len(ins))
    mk = marker_lines()

    # visits per access
    txt = open(a.regions).read()
    prof = json.loads(txt[txt.index("{\n"):])
    rates = oracle_rates(a.requests)
    acc = None
    m1 = re.search(r'"mean_requests_per_replica_per_step": ([\d.]+)', txt)
    m2 = re.search(r'"replicas_per_gpu": (\d+)', txt)
    m3 = re.search(r'"steps": (\d+)', txt)
    if m1 and m2 and m3:
        acc = float(m1.group(1)) * int(m2.group(1)) * int(m3.group(1))
    windows = prof["windows"] / acc if acc else rates["transmits"]
    tree = prof["tree_hops"] / acc if acc else 0.0
    weight = {"request loop": 1.0, "L1 walk": 1.0, "home slice": rates["home"], "probe loop": rates["down"],
              "down (share/inval)": rates["down"], "transmit setup/tail": rates["transmits"],
              "route window": windows, "window: M/G/1 wait": windows, "tree operation": tree,
              "once per launch/replica": 0.0}

    static = collections.defaultdict(collections.Counter)
    copies = collections.defaultdict(set)
    for (addr, op), c in zip(ins, ch):
        reg, key = region_of(c, mk)
        static[reg][klass(op)] += 1
        if op.startswith(("v_readlane", "v_writelane", "v_readfirstlane")):
            static[reg]["lane"] += 1      # VALU lane moves: readlanes of wave values and SGPR spill traffic
        copies[reg].add(key)
    cls = ("valu", "salu", "branch", "vmem", "lds", "smem", "lane")
    rows, tot = [], collections.Counter()
    for reg, c in static.items():
        nc = max(1, len(copies[reg]))
        per = {k: c[k] / nc for k in cls}
        dyn = {k: per[k] * weight[reg] for k in cls}
        tot.update(dyn)
        rows.append((reg, nc, weight[reg], per, dyn))
    rows.sort(key=lambda r: -(r[4]["valu"] + r[4]["salu"]))
    out = []
    out.append(f"{a.kernel} ({a.preset}): executed instructions per access by region = static per inlined copy x "
               f"visits per access")
    out.append(f"visits per access: windows {windows:.2f}, tree hops {tree:.2f} ({os.path.relpath(a.regions, ROOT)}); "
               f"transmits {rates['transmits']:.2f}, home accesses {rates['home']:.2f}, down calls {rates['down']:.2f} "
               f"(CPU restatement, replica 0's stream, {a.requests} requests after the bench warmup)")
    out.append(f"{'region':26s} {'copies':>6s} {'visits':>7s} | {'VALU':>7s} {'(lane)':>7s} {'SALU':>7s} {'branch':>7s} "
               f"{'VMEM':>6s} | static/copy VALU SALU")
    for reg, nc, w, per, dyn in rows:
        out.append(f"{reg:26s} {nc:6d} {w:7.2f} | {dyn['valu']:7.0f} {dyn['lane']:7.0f} {dyn['salu']:7.0f} "
                   f"{dyn['branch']:7.0f} {dyn['vmem']:6.1f} | {per['valu']:8.0f} {per['salu']:5.0f}")
    out.append(f"{'total (weighted)':26s} {'':6s} {'':7s} | {tot['valu']:7.0f} {tot['lane']:7.0f} {tot['salu']:7.0f} "
               f"{tot['branch']:7.0f} {tot['vmem']:6.1f}")
    if os.path.exists(a.sq):
        sq = json.load(open(a.sq))
        pl = sq.get("per_launch", {})
        pa = sq.get("per_access", {})
        v, s_ = pa.get("SQ_INSTS_VALU"), pa.get("SQ_INSTS_SALU")
        if v and s_:
            out.append(f"measured ({os.path.relpath(a.sq, ROOT)}): VALU {v:.0f}, SALU {s_:.0f} per access (the static "
                       f"x visits estimate counts both sides of every branch, so it runs high)")
    print("\n".join(out))
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"rows": [{"region": r, "copies": nc, "visits_per_access": w, "static_per_copy": per,
                                 "per_access": dyn} for r, nc, w, per, dyn in rows],
                       "total_per_access": dict(tot)}, f, indent=1)


if __name__ == "__main__":
    main()
