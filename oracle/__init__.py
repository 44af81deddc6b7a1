"""TEST INFRASTRUCTURE ONLY — the parity oracle.

* `CpuRef`: the CPU restatement of the reference uncore (oracle/cpu_ref.cpp,
  built into oracle/libpu_oracle.so).  Checker for the HIP engine and the
  "port" CPU baseline.
* `RefUncore`: the reference's own uncore compiled in place from
  /root/reference/src (oracle/_ref/libprime_ref.so; only where it was built).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package.  The product (primesim_amd) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import tempfile
from typing import Optional

import numpy as np

from primesim_amd import _abi as A

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_LIB = os.path.join(HERE, "libpu_oracle.so")
REF_LIB = os.path.join(HERE, "_ref", "libprime_ref.so")
REF_NOWRAP_LIB = os.path.join(HERE, "_ref", "libprime_ref_nowrap.so")   # no counting wraps: the CPU baseline

_olib: Optional[C.CDLL] = None
_rlib: Optional[C.CDLL] = None
_rlib_plain: Optional[C.CDLL] = None


def oracle_lib() -> C.CDLL:
    global _olib
    if _olib is None:
        if not os.path.exists(ORACLE_LIB):
            raise RuntimeError(f"{ORACLE_LIB} missing: run `make -C oracle`")
        L = C.CDLL(ORACLE_LIB)
        P = C.POINTER
        L.cpuref_create.restype = C.c_void_p
        L.cpuref_create.argtypes = [P(A.SimCfg), C.c_char_p, C.c_size_t]
        L.cpuref_destroy.argtypes = [C.c_void_p]
        L.cpuref_alloc_core.argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.cpuref_run.restype = C.c_long
        L.cpuref_run.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        L.cpuref_stats.argtypes = [C.c_void_p, P(A.Stats)]
        L.cpuref_set_mode.argtypes = [C.c_void_p, C.c_int]
        L.cpuref_completion.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.cpuref_cache_counters.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t]
        L.cpuref_mg1_batch.argtypes = [C.c_void_p] * 4 + [C.c_size_t, C.c_void_p]
        L.cpuref_queue_run.argtypes = [C.c_uint64, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p,
                                       P(C.c_uint64)]
        L.cpuref_network_run.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_uint64, C.c_uint64,
                                         C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p,
                                         P(A.Stats)]
        _olib = L
    return _olib


def ref_available(plain: bool = False) -> bool:
    return os.path.exists(REF_NOWRAP_LIB if plain else REF_LIB)


def ref_lib(plain: bool = False) -> C.CDLL:
    """The reference uncore compiled in place: with the counting wraps (the
    golden generator; every extra counter), or plain (no wraps: the CPU
    baseline's timing; extra counters read 0)."""
    global _rlib, _rlib_plain
    if (_rlib_plain if plain else _rlib) is None:
        path = REF_NOWRAP_LIB if plain else REF_LIB
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make -C oracle ref` where /root/reference exists")
        L = C.CDLL(path)
        P = C.POINTER
        L.ref_create.restype = C.c_void_p
        L.ref_create.argtypes = [C.c_char_p, P(C.c_int)]
        L.ref_get_config.argtypes = [C.c_void_p, P(A.SimCfg)]
        L.ref_alloc_core.argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.ref_get_core_id.argtypes = [C.c_void_p, C.c_int, C.c_int]
        L.ref_run.restype = C.c_long
        L.ref_run.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        L.ref_completion.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
        L.ref_set_mode.argtypes = [C.c_void_p, C.c_int]
        L.ref_report.restype = C.c_long
        L.ref_report.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p, C.c_size_t]
        L.ref_counters.argtypes = [C.c_void_p]
        L.ref_destroy.argtypes = [C.c_void_p]
        L.ref_queue_run.argtypes = [C.c_uint64, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
        L.ref_mg1_batch.argtypes = [C.c_void_p] * 4 + [C.c_size_t, C.c_void_p]
        L.ref_network_run.restype = C.c_long
        L.ref_network_run.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_uint64, C.c_uint64,
                                      C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p,
                                      C.c_char_p, C.c_char_p, C.c_size_t]
        if plain:
            _rlib_plain = L
        else:
            _rlib = L
    return _rlib_plain if plain else _rlib


class CpuRef:
    """CPU restatement of System + the prime.cpp request loop."""

    def __init__(self, cfg: A.SimCfg):
        err = C.create_string_buffer(256)
        self._h = oracle_lib().cpuref_create(C.byref(cfg), err, 256)
        if not self._h:
            raise RuntimeError(f"cpuref_create: {err.value.decode()}")
        self.num_cores = cfg.sys.num_cores
        self.num_levels = cfg.sys.num_levels

    def close(self):
        if self._h:
            oracle_lib().cpuref_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def alloc_core(self, prog: int, thread: int) -> int:
        return oracle_lib().cpuref_alloc_core(self._h, prog, thread)

    def run(self, reqs: np.ndarray) -> tuple[np.ndarray, int]:
        reqs = np.ascontiguousarray(reqs, dtype=A.REQ_DTYPE)
        d = np.zeros(len(reqs), dtype=np.int32)
        rc = oracle_lib().cpuref_run(self._h, reqs.ctypes.data, len(reqs), d.ctypes.data)
        return d, int(rc)

    def set_mode(self, mode: int) -> None:
        """MODE_CLOSED (closed-loop replay) | MODE_NOHALT (System::access semantics)."""
        oracle_lib().cpuref_set_mode(self._h, mode)

    def stats(self) -> A.Stats:
        s = A.Stats()
        oracle_lib().cpuref_stats(self._h, C.byref(s))
        return s

    def completion(self) -> np.ndarray:
        out = np.zeros(self.num_cores, dtype=np.int64)
        oracle_lib().cpuref_completion(self._h, out.ctypes.data, self.num_cores)
        return out

    def cache_counters(self, level: int, ncaches: int) -> np.ndarray:
        out = np.zeros(ncaches * 4, dtype=np.uint64)
        oracle_lib().cpuref_cache_counters(self._h, level, out.ctypes.data, out.size)
        return out.reshape(-1, 4)


def cpuref_queue(min_proc: int, t: np.ndarray, p: np.ndarray) -> tuple[np.ndarray, int]:
    t = np.ascontiguousarray(t, dtype=np.uint64)
    p = np.ascontiguousarray(p, dtype=np.uint64)
    out = np.zeros(len(t), dtype=np.uint64)
    calls = C.c_uint64(0)
    oracle_lib().cpuref_queue_run(min_proc, t.ctypes.data, p.ctypes.data, len(t), out.ctypes.data, C.byref(calls))
    return out, int(calls.value)


def cpuref_network(nodes: int, net_type: int, data_width: int, header_flits: int, router_delay: int,
                   link_delay: int, inject_delay: int, src, dst, ln, timer) -> tuple[np.ndarray, A.Stats]:
    src = np.ascontiguousarray(src, dtype=np.int32)
    dst = np.ascontiguousarray(dst, dtype=np.int32)
    ln = np.ascontiguousarray(ln, dtype=np.int32)
    timer = np.ascontiguousarray(timer, dtype=np.uint64)
    out = np.zeros(len(src), dtype=np.uint64)
    st = A.Stats()
    oracle_lib().cpuref_network_run(nodes, net_type, data_width, header_flits, router_delay, link_delay,
                                    inject_delay, src.ctypes.data, dst.ctypes.data, ln.ctypes.data,
                                    timer.ctypes.data, len(src), out.ctypes.data, C.byref(st))
    return out, st


MODE_CLOSED, MODE_NOHALT, MODE_MSGHALT = 1, 2, 4   # oracle/cpu_ref.h CPUREF_*
MODE_MSGSKIP = 8   # abandon the rest of a message whose running delay goes negative, keep receiving


REF_COUNTER_NAMES = ("link_visits", "link_flits", "mg1_calls", "lockdown_calls", "bus_accesses",
                     "transmits", "dram_accesses")


class RefUncore:
    """The reference's own System (compiled in place) + the prime.cpp loop."""

    def __init__(self, xml_path: str, plain: bool = False):
        err = C.c_int(0)
        self._L = ref_lib(plain)     # plain: the build without the counting wraps (counters() reads 0)
        self._h = self._L.ref_create(xml_path.encode(), C.byref(err))
        if not self._h:
            raise RuntimeError(f"reference XmlParser rejected {xml_path}")
        cfg = A.SimCfg()
        self._L.ref_get_config(self._h, C.byref(cfg))
        self.cfg = cfg
        self.num_cores = cfg.sys.num_cores

    def close(self):
        if self._h:
            self._L.ref_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    def alloc_core(self, prog: int, thread: int) -> int:
        return self._L.ref_alloc_core(self._h, prog, thread)

    def run(self, reqs: np.ndarray) -> tuple[np.ndarray, int]:
        reqs = np.ascontiguousarray(reqs, dtype=A.REQ_DTYPE)
        d = np.zeros(len(reqs), dtype=np.int32)
        rc = self._L.ref_run(self._h, reqs.ctypes.data, len(reqs), d.ctypes.data)
        return d, int(rc)

    def completion(self) -> np.ndarray:
        out = np.zeros(self.num_cores, dtype=np.int64)
        self._L.ref_completion(self._h, out.ctypes.data, self.num_cores)
        return out

    def set_mode(self, mode: int) -> None:
        self._L.ref_set_mode(self._h, mode)

    def report(self) -> str:
        fd, tmp = tempfile.mkstemp(suffix=".report")
        os.close(fd)
        n = self._L.ref_report(self._h, tmp.encode(), None, 0)
        fd, tmp = tempfile.mkstemp(suffix=".report")
        os.close(fd)
        buf = C.create_string_buffer(n + 1)
        self._L.ref_report(self._h, tmp.encode(), buf, n + 1)
        return buf.value.decode()

    @staticmethod
    def counters() -> dict:
        out = (C.c_uint64 * 7)()
        ref_lib().ref_counters(out)     # the wrapped build's counters (golden generation)
        return dict(zip(REF_COUNTER_NAMES, [int(x) for x in out]))


def _mg1_args(n, s, q, w):
    n = np.ascontiguousarray(n, dtype=np.uint64)
    s = np.ascontiguousarray(s, dtype=np.float64)
    q = np.ascontiguousarray(q, dtype=np.float64)
    w = np.ascontiguousarray(w, dtype=np.uint64)
    assert len(n) == len(s) == len(q) == len(w)
    return n, s, q, w


def ref_mg1(n, s, q, w) -> np.ndarray:
    """The reference's QueueModelMG1::computeQueueDelay on the states (n, Σs, Σs², newest)."""
    n, s, q, w = _mg1_args(n, s, q, w)
    out = np.zeros(len(n), dtype=np.uint64)
    ref_lib().ref_mg1_batch(n.ctypes.data, s.ctypes.data, q.ctypes.data, w.ctypes.data, len(n), out.ctypes.data)
    return out


def cpuref_mg1(n, s, q, w) -> np.ndarray:
    """The restatement's mg1_wait on the same states."""
    n, s, q, w = _mg1_args(n, s, q, w)
    out = np.zeros(len(n), dtype=np.uint64)
    oracle_lib().cpuref_mg1_batch(n.ctypes.data, s.ctypes.data, q.ctypes.data, w.ctypes.data, len(n),
                                  out.ctypes.data)
    return out


def ref_queue(min_proc: int, t: np.ndarray, p: np.ndarray) -> np.ndarray:
    t = np.ascontiguousarray(t, dtype=np.uint64)
    p = np.ascontiguousarray(p, dtype=np.uint64)
    out = np.zeros(len(t), dtype=np.uint64)
    ref_lib().ref_queue_run(min_proc, t.ctypes.data, p.ctypes.data, len(t), out.ctypes.data)
    return out
