"""Seeded M/G/1 queue states for the arithmetic fuzz (tests/test_units_oracle.py,
tests/test_gpu_mg1.py).  A state is the reference QueueModelMG1's members
(queue_model_m_g_1.h:16-19): _num_arrivals n (UInt64), _sigma_service_time
(Σ packet lengths, a double), _sigma_service_time_square (Σ squares) and
_newest_arrival_time (UInt64).  Families (all integer-valued sums, as the
engine and the reference accumulate integer packet lengths):

  random     n log-uniform up to 2^40, lengths 1..64, Σs² anywhere in
             [Σs²/n, Σs·max] (Cauchy-Schwarz), newest log-uniform up to 2^62
  flat       every packet the same length (variance exactly 0) and ±1 around it
  overload   newest < Σs: arrival rate >= service rate (the 0.999 clamp)
  edge       newest just above Σs: λ just below μ, the largest waits
  integer    variance 0 and newest = n·p + d with d | n·p²/2: the exact wait
             n·p²/(2d) is an integer, so the rounding of every step decides
             whether ceil gives k or k + 1
  small      n 1..16, newest 1..64
"""
import numpy as np


def states(count: int, seed: int = 1):
    rng = np.random.default_rng(seed)
    k = count // 6
    fams = []

    # random
    n = np.exp(rng.uniform(0, np.log(2.0 ** 40), k)).astype(np.uint64) + 1
    P = rng.integers(1, 65, k).astype(np.float64)
    mean = rng.uniform(1.0, 1.0, k) + rng.random(k) * (P - 1.0)
    nf = n.astype(np.float64)
    s = np.clip(np.round(nf * mean), nf, nf * P)
    lo = np.ceil(s * s / nf)
    hi = np.maximum(lo, s * P)
    q = np.floor(lo + rng.random(k) * (hi - lo))
    w = np.exp(rng.uniform(0, np.log(2.0 ** 62), k)).astype(np.uint64) + 1
    fams.append((n, s, q, w))

    # flat (variance 0) and its neighbours
    n = rng.integers(1, 2 ** 36, k).astype(np.uint64)
    p = rng.integers(1, 65, k).astype(np.float64)
    nf = n.astype(np.float64)
    s = nf * p
    q = nf * p * p + rng.integers(-1, 2, k)
    q = np.maximum(q, np.ceil(s * s / nf))
    w = (s * rng.uniform(0.5, 40.0, k)).astype(np.uint64) + 1
    fams.append((n, s, q, w))

    # overload: newest < Σs
    n = rng.integers(1, 2 ** 32, k).astype(np.uint64)
    nf = n.astype(np.float64)
    s = nf * rng.integers(1, 20, k)
    q = s * rng.integers(1, 20, k)
    q = np.maximum(q, np.ceil(s * s / nf))
    w = np.maximum(1, (s * rng.random(k))).astype(np.uint64)
    fams.append((n, s, q, w))

    # edge: newest just above Σs (λ just below μ)
    n = rng.integers(1, 2 ** 30, k).astype(np.uint64)
    nf = n.astype(np.float64)
    s = nf * rng.integers(1, 12, k)
    q = np.maximum(s * rng.integers(1, 12, k), np.ceil(s * s / nf))
    w = s.astype(np.uint64) + rng.integers(1, 64, k).astype(np.uint64)
    fams.append((n, s, q, w))

    # integer: exact waits n p^2 / (2d)
    n = rng.integers(1, 2 ** 24, k).astype(np.uint64) * 2
    p = rng.integers(1, 33, k).astype(np.uint64)
    m = (n * p * p) // 2
    d = np.maximum(1, m // rng.integers(1, 5000, k).astype(np.uint64))
    d = np.gcd(d, m)
    nf = n.astype(np.float64)
    s = nf * p.astype(np.float64)
    q = nf * (p * p).astype(np.float64)
    w = n * p + d
    fams.append((n, s, q, w))

    # small
    r = count - 5 * k
    n = rng.integers(1, 17, r).astype(np.uint64)
    nf = n.astype(np.float64)
    s = nf * rng.integers(1, 9, r)
    q = np.maximum(s * rng.integers(1, 9, r), np.ceil(s * s / nf))
    w = rng.integers(1, 65, r).astype(np.uint64)
    fams.append((n, s, q, w))

    n = np.concatenate([f[0] for f in fams]).astype(np.uint64)
    s = np.concatenate([f[1] for f in fams]).astype(np.float64)
    q = np.concatenate([f[2] for f in fams]).astype(np.float64)
    w = np.concatenate([f[3] for f in fams]).astype(np.uint64)
    return n, s, q, w
