"""The golden generator's counting wraps, timed: the reference uncore compiled
in place with -Wl,--wrap counters (oracle/_ref/libprime_ref.so) against the
same objects linked without them (libprime_ref_nowrap.so, bench.py's CPU
baseline), one host core, on bench.py's C4 replica-0 stream after the bench's
warmup fill, interleaved rounds.  Both must produce identical delays.

    python tools/ref_overhead.py [--seconds 5] [--rounds 3] [--replay open|closed]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--replay", choices=("open", "closed"), default="open")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    import bench
    import oracle as O
    import primesim_amd as P
    from primesim_amd import config as CF
    from primesim_amd.dist import replica_seed
    xml = os.path.join("/tmp", f"ref_overhead_{os.getpid()}.xml")
    CF.write_xml(CF.preset("C4"), xml)
    fill = 5 * 40960
    reqs = P.generate_stream(bench.stream_spec(replica_seed(bench.SEED_BASE, 0, 0), fill + 2_000_000))
    threads = P.stream_threads(bench.stream_spec(bench.SEED_BASE))
    mode = O.MODE_CLOSED if a.replay == "closed" else 0
    rates = {"wrapped": [], "plain": []}
    delays = {}
    for rnd in range(a.rounds):
        for kind in ("wrapped", "plain"):
            eng = O.RefUncore(xml, plain=kind == "plain")
            eng.set_mode(mode)
            for prog, th in threads:
                eng.alloc_core(prog, th)
            for s in range(0, fill, 16384):
                eng.run(reqs[s:min(fill, s + 16384)])
            done, out, t0 = fill, [], time.perf_counter()
            while time.perf_counter() - t0 < a.seconds and done < len(reqs):
                d, rc = eng.run(reqs[done:done + 4096])
                out.append(d)
                done += len(d)
                if rc != 0:
                    break
            el = time.perf_counter() - t0
            rates[kind].append((done - fill) / el)
            d = np.concatenate(out)
            prev = delays.get(kind)
            delays[kind] = d if prev is None or len(d) > len(prev) else prev
            eng.close()
            print(f"[ref_overhead] round {rnd} {kind}: {rates[kind][-1]:.0f} accesses/s", flush=True)
    m = min(len(delays["wrapped"]), len(delays["plain"]))
    same = bool(np.array_equal(delays["wrapped"][:m], delays["plain"][:m]))
    res = {"replay": a.replay, "cpu_model": bench.cpu_model(), "seconds_per_run": a.seconds,
           "wrapped_accesses_per_s": rates["wrapped"], "plain_accesses_per_s": rates["plain"],
           "plain_over_wrapped": float(np.median(rates["plain"]) / np.median(rates["wrapped"])),
           "delays_identical": same, "requests_compared": m}
    print(json.dumps(res))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)
    os.remove(xml)
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
