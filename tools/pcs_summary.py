"""Summarise a rocprofv3 PC-sampling CSV (run on the GPU box): samples per
instruction of one kernel, hottest first, with the instruction text.

    python tools/pcs_summary.py DIR KERNEL_SUBSTRING OUT.txt [TOP]
"""
from __future__ import annotations

import collections
import csv
import glob
import os
import sys


def main() -> None:
    d, kern, out = sys.argv[1], sys.argv[2], sys.argv[3]
    top = int(sys.argv[4]) if len(sys.argv) > 4 else 300
    files = [f for f in glob.glob(os.path.join(d, "**", "*.csv"), recursive=True) if "pc_sampl" in f.lower()]
    lines = [f"files: {files}"]
    cnt: collections.Counter = collections.Counter()
    text: dict = {}
    total = 0
    header = None
    for fn in files:
        with open(fn) as f:
            rd = csv.DictReader(f)
            header = rd.fieldnames
            for row in rd:
                kn = row.get("Kernel_Name") or row.get("Dispatch_Kernel_Name") or ""
                if kern and kern not in kn and kn:
                    continue
                key = row.get("Code_Object_Offset") or row.get("Instruction_Pc") or row.get("PC") or ""
                ins = row.get("Instruction") or ""
                cmt = row.get("Instruction_Comment") or ""
                cnt[key] += 1
                text[key] = (ins, cmt)
                total += 1
    lines.append(f"columns: {header}")
    lines.append(f"samples: {total}")
    for key, n in cnt.most_common(top):
        ins, cmt = text[key]
        lines.append(f"{n:8d} {100.0 * n / max(1, total):6.2f}% {key:>10s}  {ins}  {cmt[:120]}")
    # instruction classes
    cls: collections.Counter = collections.Counter()
    for key, n in cnt.items():
        op = (text[key][0].split() or ["?"])[0]
        cls[op] += n
    lines.append("\nby opcode:")
    for op, n in cls.most_common(60):
        lines.append(f"{n:8d} {100.0 * n / max(1, total):6.2f}% {op}")
    with open(out, "w") as f:
        f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
