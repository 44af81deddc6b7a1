"""Server front-end: prime.cpp's message loop over a Unix-domain socket.

`PrimeServer` serves an engine (`UncoreManager`, one session per replica) the
way the reference's `prime` process serves its Pin clients over MPI
(src/prime.cpp:35-137); `Client` is what core_manager.cpp's MPI_Send/MPI_Recv
calls become.  `CoreManagerDriver` plays a canonical request
stream through clients in the order core_manager.cpp sends it: PROCESS_STARTING
(core_manager.cpp:86-91), NEW_THREAD + core reply (:296-302), MEM_REQUESTS
batches + delay reply (:251-258), THREAD_FINISHING (:333-337), PROCESS_FINISHING
+ count reply and PROGRAM_EXITING per handler thread (:469-478).

The server executes requests on the HIP engine only; `PrimeServer.with_executor`
takes a host callable instead, for tests of the message protocol on machines
without a GPU (the callable is test scaffolding, not a fallback).
"""
from __future__ import annotations

import ctypes as C
import threading
from typing import Callable, Optional

import numpy as np

from . import _abi as A
from .uncore import (MSG_MEM_REQUESTS, MSG_NEW_THREAD, MSG_PROCESS_FINISHING, MSG_PROCESS_STARTING,
                     MSG_PROGRAM_EXITING, MSG_THREAD_FINISHING, MSGMEM_DTYPE, UncoreError, UncoreManager, last_error,
                     lib)


def _opts(socket_path: str, report_prefix: Optional[str], sessions: int, recv_threads: int, max_msg: int,
          verbose: bool) -> A.ServerOpts:
    o = A.ServerOpts()
    o.socket_path = socket_path.encode()
    o.report_prefix = report_prefix.encode() if report_prefix else None
    o.num_sessions = sessions
    o.num_recv_threads = recv_threads
    o.max_msg_size = max_msg
    o.verbose = int(verbose)
    return o


class PrimeServer:
    """pu_server: sessions 0..sessions-1 on replicas 0..sessions-1 of `um`."""

    def __init__(self, um: UncoreManager, socket_path: str, sessions: int = 1, report_prefix: Optional[str] = None,
                 verbose: bool = False):
        cfg = um.cfg
        self._o = _opts(socket_path, report_prefix, sessions, cfg.num_recv_threads, cfg.max_msg_size, verbose)
        self._keep = (um,)
        self._h = lib().pu_server_create(um._handle(), C.byref(self._o))
        if not self._h:
            raise UncoreError(f"server: {last_error()}")
        self._thread: Optional[threading.Thread] = None
        self.rc: Optional[int] = None

    @classmethod
    def with_executor(cls, fn: Callable[[int, np.ndarray], np.ndarray], num_cores: int, socket_path: str,
                      sessions: int = 1, recv_threads: int = 1, max_msg: int = 100) -> "PrimeServer":
        """Protocol-test server: fn(session, reqs) -> per-request delays (or
        (delays, PU_ERRF_* bits) to report an engine-side error), on the host."""
        self = cls.__new__(cls)

        def tramp(_ctx, session, reqs_p, n, delays_p):
            try:
                reqs = np.frombuffer((C.c_char * (n * A.REQ_DTYPE.itemsize)).from_address(reqs_p),
                                     dtype=A.REQ_DTYPE).copy()
                out = np.frombuffer((C.c_int32 * n).from_address(delays_p), dtype=np.int32)
                res = fn(session, reqs)
                flags = 0
                if isinstance(res, tuple):
                    res, flags = res
                out[:] = np.asarray(res, dtype=np.int32)
                return int(flags)
            except Exception:   # noqa: BLE001 — reported to the C side as an error code
                return -5

        self._cb = A.EXEC_FN(tramp)
        self._o = _opts(socket_path, None, sessions, recv_threads, max_msg, False)
        self._keep = ()
        self._h = lib().pu_server_create_exec(self._cb, None, num_cores, C.byref(self._o))
        if not self._h:
            raise UncoreError(f"server: {last_error()}")
        self._thread = None
        self.rc = None
        return self

    def round(self, timeout_ms: int = 0) -> int:
        n = lib().pu_server_round(self._h, timeout_ms)
        if n < 0:
            raise UncoreError(f"server: {last_error()}")
        return n

    def run(self) -> int:
        return lib().pu_server_run(self._h)

    def start(self) -> None:
        """Serve on a background thread until every session ends (or stop())."""
        def body():
            self.rc = self.run()
        self._thread = threading.Thread(target=body, daemon=True)
        self._thread.start()

    def join(self, timeout: Optional[float] = None) -> int:
        assert self._thread is not None
        self._thread.join(timeout)
        if self._thread.is_alive():
            raise TimeoutError("server still running")
        return int(self.rc)

    def stop(self) -> None:
        lib().pu_server_stop(self._h)

    def stats(self) -> dict:
        s = A.ServerStats()
        lib().pu_server_get_stats(self._h, C.byref(s))
        return {k: getattr(s, k) for k, _ in A.ServerStats._fields_}

    def close(self) -> None:
        if self._h:
            if self._thread is not None and self._thread.is_alive():
                self.stop()
                self._thread.join(10)
            lib().pu_server_destroy(self._h)
            self._h = None


class Client:
    """The MPI endpoint of one Pin thread (core_manager.cpp's MPI_Send / MPI_Recv)."""

    def __init__(self, socket_path: str, session: int, rank: int):
        self.rank = rank
        self._h = lib().pu_client_connect(socket_path.encode(), session, rank)
        if not self._h:
            raise UncoreError(f"client: {last_error()}")

    def send(self, records: np.ndarray, tag: int = 0) -> None:
        r = np.ascontiguousarray(records, dtype=MSGMEM_DTYPE)
        if lib().pu_client_send(self._h, tag, r.ctypes.data, len(r)) != 0:
            raise UncoreError(f"client: {last_error()}")

    def recv(self, tag: int) -> int:
        v = C.c_int32()
        if lib().pu_client_recv(self._h, tag, C.byref(v)) != 0:
            raise UncoreError(f"client: {last_error()}")
        return v.value

    def control(self, message_type: int, mem_size: int = 0, tag: int = 0) -> None:
        r = np.zeros(1, MSGMEM_DTYPE)
        r[0]["timer"] = message_type
        r[0]["mem_size"] = mem_size
        self.send(r, tag)

    def close(self) -> None:
        if self._h:
            lib().pu_client_close(self._h)
            self._h = None


def mem_message(thread_id: int, reqs: np.ndarray) -> np.ndarray:
    """A MEM_REQUESTS buffer as core_manager.cpp:251-256 fills it: header record
    (mem_size = thread id, addr_dmem = record count incl. the header), then one
    record per request (mem_type, addr_dmem, timer)."""
    m = np.zeros(len(reqs) + 1, MSGMEM_DTYPE)
    m[0]["timer"] = MSG_MEM_REQUESTS
    m[0]["mem_size"] = thread_id
    m[0]["addr_dmem"] = len(reqs) + 1
    m[1:]["mem_type"] = reqs["mem_type"]
    m[1:]["addr_dmem"] = reqs["addr"]
    m[1:]["timer"] = reqs["timer"]
    return m


class CoreManagerDriver:
    """Plays a canonical request stream through the server, one client per rank.

    `threads[c]` = (prog_id, thread_id) of core c (uncore.stream_threads); the
    ranks are the prog ids.  Messages go out in canonical order, each answered
    before the next is sent, so the server sees the order the oracle replays.
    Returns the batch delay of every MEM_REQUESTS message."""

    def __init__(self, socket_path: str, session: int, threads: list[tuple[int, int]], recv_threads: int = 1):
        self.threads = threads
        self.recv_threads = recv_threads
        ranks = sorted({p for p, _ in threads})
        self.clients = {r: Client(socket_path, session, r) for r in ranks}
        self.tag_of: dict[tuple[int, int], int] = {}

    def start(self) -> None:
        for r, c in self.clients.items():                       # core_manager.cpp:86-91
            c.control(MSG_PROCESS_STARTING)
        for p, t in self.threads:                               # core_manager.cpp:296-302
            c = self.clients[p]
            c.control(MSG_NEW_THREAD, mem_size=t, tag=0)
            self.tag_of[(p, t)] = c.recv(t)

    def run(self, reqs: np.ndarray, core_thread: Optional[list[tuple[int, int]]] = None) -> np.ndarray:
        """Send every batch of `reqs` (batch_start marks); core ids map to
        (prog, thread) through the allocation order of start()."""
        ct = core_thread or self.threads
        starts = np.nonzero(reqs["batch_start"])[0].tolist() + [len(reqs)]
        out = np.zeros(len(starts) - 1, np.int32)
        for i in range(len(starts) - 1):
            b = reqs[starts[i]:starts[i + 1]]
            p, t = ct[int(b[0]["core"])]
            c = self.clients[p]
            c.send(mem_message(t, b), tag=self.tag_of[(p, t)])
            out[i] = c.recv(t)
        return out

    def finish(self) -> list[int]:
        for p, t in self.threads:                               # core_manager.cpp:333-337
            self.clients[p].control(MSG_THREAD_FINISHING, mem_size=t, tag=self.tag_of[(p, t)])
        left = []
        for r, c in self.clients.items():                       # core_manager.cpp:469-478
            c.control(MSG_PROCESS_FINISHING)
            n = c.recv(0)
            left.append(n)
            if n == 0:
                for i in range(self.recv_threads):
                    c.control(MSG_PROGRAM_EXITING, tag=i)
        return left

    def close(self) -> None:
        for c in self.clients.values():
            c.close()
