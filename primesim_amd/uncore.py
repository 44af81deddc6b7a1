"""Python host mirror of the reference's uncore interface, over the C ABI.

`UncoreManager` follows reference src/uncore_manager.h:51-68 (init, allocCore,
deallocCore, getCoreId, uncore_access, report) with the same argument meaning
and error behaviour (uncore_access returns -1 for core_id >= num_cores,
system.cpp:147-150).  It adds the batch paths the engine is built for:
`access_batch` (host arrays, one replica) and `run_device` (device-resident
requests for every replica, the benchmark path).

The HIP library is mandatory: importing works everywhere (stream generation
and config parsing are host code), but creating an engine without a GPU or
without the built library raises — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _abi as A

_HERE = os.path.dirname(os.path.abspath(__file__))
# PRIMEUNCORE_LIB selects another build of the same library (the region-profiling
# build, tools/prof_regions.py); there is no fallback when it is missing.
LIB_PATH = os.environ.get("PRIMEUNCORE_LIB") or os.path.join(_HERE, "libprimeuncore.so")
_lib: Optional[C.CDLL] = None


class UncoreError(RuntimeError):
    pass


def lib() -> C.CDLL:
    """Load libprimeuncore.so (build it with __graft_entry__.build())."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise UncoreError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'`")
    # One HIP runtime per process: PyTorch bundles its own libamdhip64 under the
    # same SONAME (libamdhip64.so.7) but NEEDs it as "libamdhip64.so", so if this
    # library loaded /opt/rocm's copy first, torch would load a second runtime
    # and find no GPU.  Loading torch first makes both share torch's runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    P = C.POINTER
    sig = {
        "pu_config_load_xml": (C.c_int, [C.c_char_p, P(A.SimCfg)]),
        "pu_config_parse_xml": (C.c_int, [C.c_char_p, C.c_size_t, P(A.SimCfg)]),
        "pu_config_write_xml": (C.c_int, [P(A.SimCfg), C.c_char_p, C.c_size_t, P(C.c_size_t)]),
        "pu_create": (C.c_void_p, [P(A.SimCfg), C.c_int, C.c_int]),
        "pu_config_geo_source": (C.c_long, [P(A.SimCfg), C.c_char_p, C.c_size_t]),
        "pu_config_jit_warm": (C.c_int, [P(A.SimCfg)]),
        "pu_compiled_config": (C.c_int, [C.c_void_p]),
        "pu_compiled_compiler": (C.c_int, [C.c_void_p]),
        "pu_jit_source_tag": (C.c_char_p, []),
        "pu_jit_prof_read": (C.c_int, [C.POINTER(C.c_ulonglong), C.c_int, C.c_int]),
        "pu_destroy": (None, [C.c_void_p]),
        "pu_reset": (C.c_int, [C.c_void_p]),
        "pu_num_replicas": (C.c_int, [C.c_void_p]),
        "pu_replica_bytes": (C.c_uint64, [C.c_void_p]),
        "pu_limit_positions": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
        "pu_replica_pool_bytes": (C.c_uint64, [C.c_void_p]),
        "pu_resident_replicas": (C.c_int, [C.c_void_p]),
        "pu_alloc_core": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
        "pu_dealloc_core": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
        "pu_get_core_id": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
        "pu_access": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, P(C.c_uint64), C.c_int64]),
        "pu_access_status": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, P(C.c_uint64), C.c_int64,
                                       P(C.c_int32)]),
        "pu_access_batch": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t, C.c_void_p]),
        "pu_run_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
        "pu_run_device_sliced": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                           C.c_void_p]),
        "pu_pool_slots": (C.c_int, [C.c_void_p]),
        "pu_pool_words": (C.c_long, [C.c_int]),
        "pu_run_device_pool": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                         C.c_int, C.c_uint64, C.c_void_p]),
        "pu_synchronize": (C.c_int, [C.c_void_p]),
        "pu_set_device_req_format": (C.c_int, [C.c_void_p, C.c_int]),
        "pu_pack_req16": (C.c_int, [C.c_void_p, C.c_size_t, C.c_void_p]),
        "pu_core_completion": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t]),
        "pu_stats_get": (C.c_int, [C.c_void_p, C.c_int, P(A.Stats)]),
        "pu_report": (C.c_long, [C.c_void_p, C.c_int, C.c_int, C.c_char_p, C.c_size_t]),
        "pu_last_kernel_ms": (C.c_double, [C.c_void_p]),
        "pu_set_resident": (C.c_int, [C.c_void_p, C.c_int]),
        "pu_resident_info": (C.c_int, [C.c_void_p, P(C.c_uint64), C.c_size_t]),
        "pu_last_error": (C.c_char_p, []),
        "pu_version": (C.c_char_p, []),
        "pu_set_replay_mode": (C.c_int, [C.c_void_p, C.c_int]),
        "pu_sim_start_time": (None, [C.c_void_p]),
        "pu_sim_finish_time": (None, [C.c_void_p]),
        "pu_error_flags": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t]),
        "pu_stream_count": (C.c_int64, [P(A.StreamParams)]),
        "pu_stream_generate": (C.c_int64, [P(A.StreamParams), C.c_void_p, C.c_size_t]),
        "pu_stream_thread_of": (C.c_int, [P(A.StreamParams), C.c_int, P(C.c_int), P(C.c_int)]),
        "pu_stream_open": (C.c_void_p, [P(A.StreamParams)]),
        "pu_stream_close": (None, [C.c_void_p]),
        "pu_stream_next": (C.c_int64, [C.c_void_p, C.c_void_p, C.c_size_t]),
        "pu_stream_position": (C.c_int64, [C.c_void_p]),
        "pu_stream_next_many": (C.c_int64, [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t, C.c_size_t, C.c_int]),
        "pu_msglog_open": (C.c_void_p, [C.c_char_p, C.c_int]),
        "pu_msglog_next": (C.c_int64, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]),
        "pu_msglog_messages": (C.c_int64, [C.c_void_p]),
        "pu_msglog_create": (C.c_void_p, [C.c_char_p]),
        "pu_msglog_append": (C.c_int, [C.c_void_p, C.c_int32, C.c_void_p, C.c_int32]),
        "pu_msglog_close": (C.c_int, [C.c_void_p]),
        "pu_msglog_from_requests": (C.c_int, [C.c_char_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_int,
                                              C.c_void_p, C.c_int]),
        "pu_trace_write": (C.c_int, [C.c_char_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_int]),
        "pu_alloc_core_replica": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int]),
        "pu_dealloc_core_replica": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int]),
        "pu_get_core_id_replica": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int]),
        "pu_server_create": (C.c_void_p, [C.c_void_p, P(A.ServerOpts)]),
        "pu_server_create_exec": (C.c_void_p, [A.EXEC_FN, C.c_void_p, C.c_int, P(A.ServerOpts)]),
        "pu_server_run": (C.c_int, [C.c_void_p]),
        "pu_server_round": (C.c_int, [C.c_void_p, C.c_int]),
        "pu_server_stop": (None, [C.c_void_p]),
        "pu_server_get_stats": (C.c_int, [C.c_void_p, P(A.ServerStats)]),
        "pu_server_destroy": (None, [C.c_void_p]),
        "pu_client_connect": (C.c_void_p, [C.c_char_p, C.c_int, C.c_int]),
        "pu_client_send": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_int]),
        "pu_client_recv": (C.c_int, [C.c_void_p, C.c_int, P(C.c_int32)]),
        "pu_client_close": (None, [C.c_void_p]),
        "pu_unit_mg1_run": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p,
                                      C.c_int]),
        "pu_unit_queue_run": (C.c_int, [C.c_uint64, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p,
                                        P(C.c_uint64), C.c_int]),
        "pu_unit_network_run": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_uint64, C.c_uint64,
                                          C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p,
                                          P(A.Stats), C.c_int]),
    }
    for name, (res, args) in sig.items():
        if name == "pu_jit_prof_read" and not hasattr(L, name):
            continue   # diagnostics only: libraries of older commits (same-box A/B variants) lack it
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def last_error() -> str:
    return lib().pu_last_error().decode()


# PU_E* codes (include/primeuncore.h).  pu_access returns them in-band (a
# wrapped delay may collide with one); the mirror uses pu_access_status.
PU_ERRORS = (-5, -12, -19, -22, -34, -71, -95)
PU_REPLAY_OPEN, PU_REPLAY_CLOSED = 0, 1
PU_REQ_FMT_32, PU_REQ_FMT_16 = 0, 1


def library_source_hash() -> str:
    """The source hash pu_version() was built with (tools/src_hash.py)."""
    v = lib().pu_version().decode()
    return v.rsplit(" src ", 1)[1] if " src " in v else ""


# ---------------------------------------------------------------- config
def load_config(path: str) -> A.SimCfg:
    """XmlParser::parse equivalent (reference xml_parser.cpp:684)."""
    cfg = A.SimCfg()
    rc = lib().pu_config_load_xml(path.encode(), C.byref(cfg))
    if rc != 0:
        raise UncoreError(f"config {path}: {last_error()}")
    return cfg


def parse_config(text: str) -> A.SimCfg:
    cfg = A.SimCfg()
    b = text.encode()
    rc = lib().pu_config_parse_xml(b, len(b), C.byref(cfg))
    if rc != 0:
        raise UncoreError(f"config: {last_error()}")
    return cfg


def config_from_dict(sim: dict) -> A.SimCfg:
    from .config import to_xml
    return parse_config(to_xml(sim))


# ---------------------------------------------------------------- streams
@dataclass
class StreamSpec:
    kind: int
    num_cores: int
    seed: int = 1
    quantum: int = 1000
    num_quanta: int = 1
    max_msg: int = 100
    num_progs: int = 1
    max_requests: int = 0
    write_pct: int = -1

    def params(self) -> A.StreamParams:
        return A.StreamParams(self.kind, self.num_cores, self.seed, self.quantum, self.num_quanta,
                              self.max_msg, self.num_progs, self.max_requests, self.write_pct, 0)


def pack_req16(reqs: np.ndarray) -> np.ndarray:
    """REQ_DTYPE records -> 16-B pu_req16 records (uint64 pairs, primeuncore.h);
    raises UncoreError naming the first record that does not fit."""
    assert reqs.dtype == A.REQ_DTYPE and reqs.flags.c_contiguous
    out = np.empty(reqs.shape + (2,), dtype=np.uint64)
    if lib().pu_pack_req16(reqs.ctypes.data, reqs.size, out.ctypes.data) != 0:
        raise UncoreError(last_error())
    return out


def generate_stream(spec: StreamSpec) -> np.ndarray:
    """Deterministic synthetic request stream in canonical order (REQ_DTYPE)."""
    p = spec.params()
    n = lib().pu_stream_count(C.byref(p))
    if n < 0:
        raise UncoreError(f"stream: {last_error()} ({n})")
    out = np.zeros(n, dtype=A.REQ_DTYPE)
    if n:
        got = lib().pu_stream_generate(C.byref(p), out.ctypes.data, n)
        if got != n:
            raise UncoreError(f"stream generation returned {got}, expected {n}")
    return out


class StreamSet:
    """Resumable generators for several streams (pu_stream_open/next_many):
    `next(n)` returns the next n requests of every stream as an [count, n]
    array; the chunks concatenate to exactly generate_stream's output."""

    def __init__(self, specs: list[StreamSpec]):
        self._h = []
        for sp in specs:
            p = sp.params()
            h = lib().pu_stream_open(C.byref(p))
            if not h:
                self.close()
                raise UncoreError(f"stream: {last_error()}")
            self._h.append(h)
        self._arr = (C.c_void_p * len(self._h))(*self._h)

    def __len__(self) -> int:
        return len(self._h)

    def next_into(self, out: np.ndarray, threads: int = 0) -> int:
        """Fill out[i, :] with stream i's next out.shape[1] requests; returns the
        smallest number produced (short only at the end of a stream)."""
        assert out.dtype == A.REQ_DTYPE and out.ndim == 2 and out.shape[0] == len(self._h)
        assert out.flags.c_contiguous
        got = lib().pu_stream_next_many(self._arr, len(self._h), out.ctypes.data, out.shape[1], out.shape[1],
                                        threads)
        if got < 0:
            raise UncoreError(f"stream: {last_error()}")
        return int(got)

    def next(self, n: int, threads: int = 0) -> np.ndarray:
        out = np.zeros((len(self._h), n), dtype=A.REQ_DTYPE)
        got = self.next_into(out, threads)
        return out[:, :got]

    def position(self, i: int = 0) -> int:
        return int(lib().pu_stream_position(self._h[i]))

    def close(self) -> None:
        for h in self._h:
            lib().pu_stream_close(h)
        self._h = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---------------------------------------------------------------- MsgMem logs
MSGMEM_DTYPE = np.dtype([("mem_type", np.uint8), ("_pad", np.uint8, 3), ("mem_size", np.int32),
                         ("addr_dmem", np.uint64), ("timer", np.int64)])   # reference common.h:49-59
assert MSGMEM_DTYPE.itemsize == 24
MSG_MEM_REQUESTS, MSG_PROCESS_STARTING, MSG_PROCESS_FINISHING = 0, -3, -1
MSG_BARRIER, MSG_NEW_THREAD, MSG_THREAD_FINISHING, MSG_PROGRAM_EXITING = -2, -4, -8, -5


def msglog_from_stream(path: str, reqs: np.ndarray, spec: "StreamSpec") -> None:
    """Write a synthetic stream as the MsgMem message log its cores would have sent."""
    threads = stream_threads(spec)
    tp = np.array([t[0] for t in threads], np.int32)
    ti = np.array([t[1] for t in threads], np.int32)
    ct = np.arange(spec.num_cores, dtype=np.int32)
    reqs = np.ascontiguousarray(reqs, dtype=A.REQ_DTYPE)
    rc = lib().pu_msglog_from_requests(path.encode(), reqs.ctypes.data, len(reqs), tp.ctypes.data, ti.ctypes.data,
                                       len(threads), ct.ctypes.data, spec.num_cores)
    if rc != 0:
        raise UncoreError(f"msglog: {last_error()}")


class MsgLogWriter:
    """Capture side: append messages exactly as prime.cpp:53 receives them."""

    def __init__(self, path: str):
        self._h = lib().pu_msglog_create(path.encode())
        if not self._h:
            raise UncoreError(f"msglog: {last_error()}")

    def append(self, source: int, records: np.ndarray) -> None:
        records = np.ascontiguousarray(records, dtype=MSGMEM_DTYPE)
        if lib().pu_msglog_append(self._h, source, records.ctypes.data, len(records)) != 0:
            raise UncoreError(f"msglog: {last_error()}")

    def close(self) -> None:
        if self._h:
            lib().pu_msglog_close(self._h)
            self._h = None


def msglog_read(path: str, um: "UncoreManager | None" = None, num_cores: int = 0,
                chunk: int = 1 << 16) -> np.ndarray:
    """Replay a MsgMem log into requests (prime.cpp:55-137 semantics), resolving
    core ids through um's ThreadSched (or the log's own over num_cores cores)."""
    L = lib().pu_msglog_open(path.encode(), num_cores)
    if not L:
        raise UncoreError(f"msglog: {last_error()}")
    parts = []
    try:
        h = um._handle() if um is not None else None
        while True:
            buf = np.zeros(chunk, dtype=A.REQ_DTYPE)
            n = lib().pu_msglog_next(L, h, buf.ctypes.data, chunk)
            if n < 0:
                raise UncoreError(f"msglog: {last_error()}")
            if n == 0:
                break
            parts.append(buf[:n])
    finally:
        lib().pu_msglog_close(L)
    return np.concatenate(parts) if parts else np.zeros(0, dtype=A.REQ_DTYPE)


def stream_threads(spec: StreamSpec) -> list[tuple[int, int]]:
    """(prog_id, thread_id) of every core, in allocation order."""
    p = spec.params()
    res = []
    for c in range(spec.num_cores):
        pr, th = C.c_int(), C.c_int()
        if lib().pu_stream_thread_of(C.byref(p), c, C.byref(pr), C.byref(th)) != 0:
            raise UncoreError(last_error())
        res.append((pr.value, th.value))
    return res


# ---------------------------------------------------------------- engine
@dataclass
class InsMem:
    """reference src/cache.h:92-99 (the fields System::access reads)."""
    mem_type: int
    prog_id: int
    addr_dmem: int
    thread_id: int = 0
    rec_thread_id: int = 0


class UncoreManager:
    """reference UncoreManager (uncore_manager.h:51-68) backed by the HIP engine."""

    def __init__(self) -> None:
        self._h: Optional[int] = None
        self.cfg: Optional[A.SimCfg] = None
        self.replicas = 0

    # UncoreManager::init (uncore_manager.cpp:46-50)
    def init(self, cfg: A.SimCfg, replicas: int = 1, device: int = 0) -> None:
        h = lib().pu_create(C.byref(cfg), replicas, device)
        if not h:
            raise UncoreError(f"pu_create: {last_error()}")
        self._h = h
        self.cfg = cfg
        self.replicas = replicas

    def close(self) -> None:
        if self._h:
            lib().pu_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _handle(self) -> int:
        if not self._h:
            raise UncoreError("UncoreManager not initialised")
        return self._h

    def reset(self) -> None:
        if lib().pu_reset(self._handle()) != 0:
            raise UncoreError(last_error())

    @property
    def replica_bytes(self) -> int:
        return int(lib().pu_replica_bytes(self._handle()))

    @property
    def replica_pool_bytes(self) -> int:
        """The sharer-bitmap pool's share of replica_bytes."""
        return int(lib().pu_replica_pool_bytes(self._handle()))

    @property
    def resident_replicas(self) -> int:
        """Replicas the engine kernel holds resident on the device at once."""
        n = lib().pu_resident_replicas(self._handle())
        if n <= 0:
            raise UncoreError(last_error())
        return int(n)

    def allocCore(self, prog_id: int, thread_id: int) -> int:
        return lib().pu_alloc_core(self._handle(), prog_id, thread_id)

    def deallocCore(self, prog_id: int, thread_id: int) -> int:
        return lib().pu_dealloc_core(self._handle(), prog_id, thread_id)

    def getCoreId(self, prog_id: int, thread_id: int) -> int:
        return lib().pu_get_core_id(self._handle(), prog_id, thread_id)

    # UncoreManager::uncore_access (uncore_manager.cpp:82-85)
    def uncore_access(self, core_id: int, ins_mem: InsMem, timer: int) -> int:
        addr = C.c_uint64(ins_mem.addr_dmem)
        d = C.c_int32(0)
        rc = lib().pu_access_status(self._handle(), core_id, ins_mem.prog_id, ins_mem.mem_type, C.byref(addr), timer,
                                    C.byref(d))
        if rc != 0:                       # status out of band: every int delay is a delay
            raise UncoreError(f"uncore_access: {last_error()}")
        ins_mem.addr_dmem = addr.value
        return d.value

    def access_batch(self, reqs: np.ndarray, replica: int = 0) -> np.ndarray:
        """prime.cpp:120-137 for a run of messages; returns per-request delays."""
        reqs = np.ascontiguousarray(reqs, dtype=A.REQ_DTYPE)
        out = np.zeros(len(reqs), dtype=np.int32)
        rc = lib().pu_access_batch(self._handle(), replica, reqs.ctypes.data, len(reqs), out.ctypes.data)
        if rc != 0:
            raise UncoreError(f"access_batch: {last_error()}")
        return out

    # UncoreManager::getSimStartTime / getSimFinishTime (uncore_manager.cpp:52-60)
    def getSimStartTime(self) -> None:
        lib().pu_sim_start_time(self._handle())

    def getSimFinishTime(self) -> None:
        lib().pu_sim_finish_time(self._handle())

    def set_replay_mode(self, mode: int) -> None:
        """PU_REPLAY_OPEN (recorded timers) or PU_REPLAY_CLOSED (timer_i += the
        core's earlier batch delays, core_manager.cpp:265)."""
        if lib().pu_set_replay_mode(self._handle(), mode) != 0:
            raise UncoreError(last_error())

    def set_device_req_format(self, fmt: int) -> None:
        """PU_REQ_FMT_32 (pu_req) or PU_REQ_FMT_16 (pu_req16, pack_req16): the
        record format run_device / run_device_sliced / run_device_pool read."""
        if lib().pu_set_device_req_format(self._handle(), fmt) != 0:
            raise UncoreError(last_error())

    def error_flags(self, n: Optional[int] = None) -> np.ndarray:
        """PU_ERRF_* bits of replicas [0, n)."""
        n = self.replicas if n is None else n
        out = np.zeros(n, dtype=np.uint64)
        if lib().pu_error_flags(self._handle(), out.ctypes.data, n) != 0:
            raise UncoreError(last_error())
        return out

    def limit_positions(self, n: Optional[int] = None) -> np.ndarray:
        """Per replica: index of the first request of the last launch that raised
        a PU_ERRF_LIMITS bit (2^64-1: none)."""
        n = self.replicas if n is None else n
        out = np.zeros(n, dtype=np.uint64)
        if lib().pu_limit_positions(self._handle(), out.ctypes.data, n) != 0:
            raise UncoreError(last_error())
        return out

    def run_device(self, d_reqs_ptr: int, d_off_ptr: int, d_delay_ptr: int, stream_ptr: int = 0) -> None:
        """All replicas at once on device-resident buffers (asynchronous)."""
        rc = lib().pu_run_device(self._handle(), d_reqs_ptr, d_off_ptr, d_delay_ptr, stream_ptr or None)
        if rc != 0:
            raise UncoreError(f"run_device: {last_error()}")

    def run_device_sliced(self, d_reqs_ptr: int, d_off_ptr: int, d_delay_ptr: int, d_pos_ptr: int, budget_us: int,
                          stream_ptr: int = 0) -> None:
        """Time-sliced run: replica r continues from d_pos[r] for at most budget_us
        of wall time (stopping only between requests) and advances d_pos[r]."""
        rc = lib().pu_run_device_sliced(self._handle(), d_reqs_ptr, d_off_ptr, d_delay_ptr, d_pos_ptr, budget_us,
                                        stream_ptr or None)
        if rc != 0:
            raise UncoreError(f"run_device_sliced: {last_error()}")

    def pool_slots(self) -> int:
        """Most wavefronts of a replica-pool launch: min(replicas, resident replicas)."""
        n = lib().pu_pool_slots(self._handle())
        if n < 0:
            raise UncoreError(f"pool_slots: {last_error()}")
        return int(n)

    @staticmethod
    def pool_words(slots: int) -> int:
        """uint32 words of the scheduling array a pool of `slots` wavefronts needs (all 0 to start)."""
        n = lib().pu_pool_words(slots)
        if n < 0:
            raise UncoreError(f"pool_words: {last_error()}")
        return int(n)

    def run_device_pool(self, d_reqs_ptr: int, d_off_ptr: int, d_delay_ptr: int, d_pos_ptr: int, d_sched_ptr: int,
                        slots: int, budget_us: int, stream_ptr: int = 0) -> None:
        """Time-sliced run of more replicas than run at once: each of `slots`
        wavefronts continues its replica and, once that replica's range is done
        (or it halted), takes the next unstarted one (pu_run_device_pool)."""
        rc = lib().pu_run_device_pool(self._handle(), d_reqs_ptr, d_off_ptr, d_delay_ptr, d_pos_ptr, d_sched_ptr,
                                      slots, budget_us, stream_ptr or None)
        if rc != 0:
            raise UncoreError(f"run_device_pool: {last_error()}")

    def synchronize(self) -> None:
        if lib().pu_synchronize(self._handle()) != 0:
            raise UncoreError(last_error())

    def last_kernel_ms(self) -> float:
        return float(lib().pu_last_kernel_ms(self._handle()))

    def set_resident(self, mode: int) -> int:
        """Resident mode for uncore_access / short batches (pu_set_resident):
        1 on, 0 off, -1 query; returns the previous mode."""
        rc = lib().pu_set_resident(self._handle(), mode)
        if rc < 0:
            raise UncoreError(last_error())
        return rc

    def resident_info(self) -> dict:
        """The resident kernel (pu_resident_info): running, commands served,
        kernels launched, eligible, and per command the mean kernel-side phases
        (request copy, message loop, close, mailbox) and host-side call time in µs."""
        out = (C.c_uint64 * 10)()
        if lib().pu_resident_info(self._handle(), out, 10) < 0:
            raise UncoreError(last_error())
        n = max(1, int(out[1]))
        nfull = max(1, int(out[1]) - int(out[9]))
        sums_us = {"request_copy": out[4] / 100, "message_loop": out[5] / 100, "close": out[6] / 100,
                   "mailbox": out[7] / 100, "host_call": out[8] / 1000}
        return {"running": bool(out[0]), "commands": int(out[1]), "launches": int(out[2]), "eligible": bool(out[3]),
                "fast_answers": int(out[9]), "sums_us": sums_us,
                "mean_us": {k: v / (n if k == "host_call" else nfull) for k, v in sums_us.items()}}

    def stats(self, replica: int = 0) -> A.Stats:
        s = A.Stats()
        if lib().pu_stats_get(self._handle(), replica, C.byref(s)) != 0:
            raise UncoreError(last_error())
        return s

    def completion(self, replica: int = 0) -> np.ndarray:
        n = self.cfg.sys.num_cores
        out = np.zeros(n, dtype=np.int64)
        if lib().pu_core_completion(self._handle(), replica, out.ctypes.data, n) != 0:
            raise UncoreError(last_error())
        return out

    # UncoreManager::report (uncore_manager.cpp:87-98)
    def report(self, replica: int = 0, include_time: bool = False) -> str:
        n = lib().pu_report(self._handle(), replica, int(include_time), None, 0)
        if n < 0:
            raise UncoreError(last_error())
        buf = C.create_string_buffer(n + 1)
        lib().pu_report(self._handle(), replica, int(include_time), buf, n + 1)
        return buf.value.decode()


# ---------------------------------------------------------------- unit hooks
def unit_queue(min_proc: int, t: np.ndarray, p: np.ndarray, device: int = 0) -> tuple[np.ndarray, int]:
    """The history-tree queue model alone on the GPU."""
    t = np.ascontiguousarray(t, dtype=np.uint64)
    p = np.ascontiguousarray(p, dtype=np.uint64)
    out = np.zeros(len(t), dtype=np.uint64)
    calls = C.c_uint64(0)
    rc = lib().pu_unit_queue_run(min_proc, t.ctypes.data, p.ctypes.data, len(t), out.ctypes.data, C.byref(calls),
                                 device)
    if rc != 0:
        raise UncoreError(f"unit_queue: {last_error()}")
    return out, int(calls.value)


def unit_network(nodes: int, net_type: int, data_width: int, header_flits: int, router_delay: int,
                 link_delay: int, inject_delay: int, src, dst, ln, timer, device: int = 0):
    """Network::transmit sequence alone on the GPU."""
    src = np.ascontiguousarray(src, dtype=np.int32)
    dst = np.ascontiguousarray(dst, dtype=np.int32)
    ln = np.ascontiguousarray(ln, dtype=np.int32)
    timer = np.ascontiguousarray(timer, dtype=np.uint64)
    out = np.zeros(len(src), dtype=np.uint64)
    st = A.Stats()
    rc = lib().pu_unit_network_run(nodes, net_type, data_width, header_flits, router_delay, link_delay,
                                   inject_delay, src.ctypes.data, dst.ctypes.data, ln.ctypes.data,
                                   timer.ctypes.data, len(src), out.ctypes.data, C.byref(st), device)
    if rc != 0:
        raise UncoreError(f"unit_network: {last_error()}")
    return out, st
