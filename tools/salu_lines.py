"""Static instruction mix of one compiled-configuration kernel, by source
function and line: the preset's kernels compiled by jit.cpp's hipRTC path with
line tables (PRIMEUNCORE_JIT_EXTRA=-gline-tables-only; the options are part of
the cache key, so the product's cache is untouched), disassembled with
llvm-objdump -l, every instruction charged to the innermost (inlined) source
line.  Static counts: how many instructions of each class the code holds for
a function, not how often they run; tools/prof_regions.py's visit counts
(windows, tree hops, accesses) give the weights.  No GPU.

    python tools/salu_lines.py [C4] [--kernel pu_jit_uncore_s1_h0] [--top 40]
"""
from __future__ import annotations

import argparse
import collections
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "primesim_amd", "csrc")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"

# SQ_INSTS_SALU counts scalar ALU ops; waits, nops, branches and scalar memory
# have their own counters (or none)
NOT_SALU = re.compile(r"^s_(waitcnt|nop|branch|cbranch|load|buffer|store|memtime|memrealtime|sleep|setprio|"
                      r"barrier|endpgm|dcache|sendmsg|trap|icache|getpc|setpc|swappc|call|set_gpr_idx|"
                      r"ttracedata|inst_prefetch|clause)")


def klass(op: str) -> str:
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("s_branch", "s_cbranch", "s_setpc", "s_swappc")):
        return "branch"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_"):
        return "other_s" if NOT_SALU.match(op) else "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def functions(path: str) -> list[tuple[int, str]]:
    """(first line, name) of every function definition starting at column 0."""
    out = []
    pat = re.compile(r"^(?:template\s*<.*>\s*)?(?:static\s+)?(?:__device__|__global__|__host__|inline|"
                     r"extern|[A-Za-z_][\w:<>, *&]*\s)[^;=(]*?\b([A-Za-z_]\w*)\s*\(")
    meth = re.compile(r"^    (?:static\s+)?__device__\s.*?\b([A-Za-z_]\w*)\s*\(")   # Engine's methods
    with open(path) as f:
        for i, ln in enumerate(f, 1):
            m = meth.match(ln)
            if m:
                out.append((i, "Engine::" + m.group(1)))
                continue
            if ln[:1].isspace() or ln.startswith(("#", "//", "}")):
                continue
            m = pat.match(ln)
            if m and m.group(1) not in ("if", "for", "while", "switch", "return", "sizeof"):
                out.append((i, m.group(1)))
    return out


def compile_lines(preset: str) -> str:
    with tempfile.TemporaryDirectory(prefix="pu_salu_") as d:
        env = dict(os.environ, PRIMEUNCORE_JIT_CACHE=d, PRIMEUNCORE_JIT_EXTRA="-gline-tables-only")
        code = ("import ctypes as C, sys; sys.path.insert(0, %r); import primesim_amd as P; "
                "from primesim_amd import config as CF, uncore; cfg = P.config_from_dict(CF.preset(%r)); "
                "rc = uncore.lib().pu_config_jit_warm(C.byref(cfg)); sys.exit(0 if rc >= 0 else 1)") % (ROOT, preset)
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True)
        if r.returncode != 0:
            raise SystemExit(r.stderr[-3000:])
        # two code objects per configuration (jit.cpp: throughput and latency kernels)
        return "".join(subprocess.run([OBJDUMP, "-d", "-l", "--no-show-raw-insn", hsaco], capture_output=True,
                                      text=True).stdout for hsaco in sorted(glob.glob(os.path.join(d, "*.hsaco"))))


def tally(dis: str, kernel: str):
    per_line: dict = collections.defaultdict(collections.Counter)
    cur = ("?", 0)
    inside = False
    for ln in dis.splitlines():
        m = re.match(r"^[0-9a-f]+ <([^>]+)>:", ln)
        if m:
            inside = m.group(1) == kernel
            continue
        if not inside:
            continue
        m = re.match(r"^; .*/([\w.]+):(\d+)", ln)
        if m:
            cur = (m.group(1), int(m.group(2)))
            continue
        s = ln.strip()
        if not s or s.startswith(";"):
            continue
        op = s.split()[0]
        if re.match(r"^[sv]_|^ds_|^global_|^buffer_|^flat_|^scratch_", op):
            per_line[cur][klass(op)] += 1
            if klass(op) == "salu":
                per_line[cur]["op:" + op] += 1
    return per_line


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("preset", nargs="?", default="C4")
    ap.add_argument("--kernel", default="pu_jit_uncore_s1_h0")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    per_line = tally(compile_lines(a.preset), a.kernel)
    fn_cache: dict = {}

    def fn_of(file: str, line: int) -> str:
        if file not in fn_cache:
            p = os.path.join(CSRC, file)
            fn_cache[file] = functions(p) if os.path.exists(p) else []
        name = "?"
        for first, n in fn_cache[file]:
            if first > line:
                break
            name = n
        return f"{file}:{name}"

    per_fn: dict = collections.defaultdict(collections.Counter)
    tot = collections.Counter()
    for (file, line), c in per_line.items():
        per_fn[fn_of(file, line)].update(c)
        tot.update(c)
    cls = ("salu", "valu", "branch", "smem", "lds", "vmem", "other_s")
    print(f"{a.kernel}: " + ", ".join(f"{k} {tot[k]}" for k in cls))
    print("\nby function (static):")
    for fn, c in sorted(per_fn.items(), key=lambda kv: -kv[1]["salu"])[:a.top]:
        ops = sorted(((k[3:], v) for k, v in c.items() if k.startswith("op:")), key=lambda kv: -kv[1])[:4]
        print(f"  {fn:40s} " + " ".join(f"{k} {c[k]:4d}" for k in cls[:3]) + "   " +
              ", ".join(f"{o} {n}" for o, n in ops))
    print("\nby line (static SALU):")
    for (file, line), c in sorted(per_line.items(), key=lambda kv: -kv[1]["salu"])[:a.top]:
        ops = sorted(((k[3:], v) for k, v in c.items() if k.startswith("op:")), key=lambda kv: -kv[1])[:3]
        print(f"  {file}:{line:<6d} {fn_of(file, line):32s} salu {c['salu']:4d} valu {c['valu']:4d}   " +
              ", ".join(f"{o} {n}" for o, n in ops))


if __name__ == "__main__":
    main()
