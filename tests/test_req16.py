"""The 16-B device request record (pu_req16, include/primeuncore.h) that the
bench's timed window uses:

* CPU: pu_pack_req16 keeps every field the engine reads (decoded here with
  the layout the header states) and refuses a record that does not fit, at
  each field's boundary;
* GPU: the device-run entry points under PU_REQ_FMT_16 give the delays,
  counters and completion cycles of the same requests as 32-B pu_req, and
  those of the CPU restatement (pool, time-sliced and unsliced launches, open
  and closed loop, C2 and the bench's C4 kernel).
"""
import numpy as np
import pytest

import primesim_amd as P
from primesim_amd import _abi as A
from primesim_amd import config as CF
from primesim_amd import uncore as U


def _decode(p: np.ndarray) -> dict:
    a, b = p[..., 0], p[..., 1]
    return {"addr": a, "timer": (b & np.uint64((1 << 40) - 1)).astype(np.int64),
            "core": ((b >> np.uint64(40)) & np.uint64(0xFFFF)).astype(np.int32),
            "prog_id": ((b >> np.uint64(56)) & np.uint64(63)).astype(np.int32),
            "mem_type": ((b >> np.uint64(62)) & np.uint64(1)).astype(np.uint8),
            "batch_start": (b >> np.uint64(63)).astype(np.uint8)}


@pytest.mark.parametrize("kind,cores", [(A.PU_STREAM_UNIFORM_HOTSPOT, 1024), (A.PU_STREAM_MULTIPROGRAM, 256)])
def test_pack_req16_keeps_every_field(kind, cores):
    reqs = P.generate_stream(P.StreamSpec(kind, cores, seed=17, max_requests=20000))
    got = _decode(U.pack_req16(reqs))
    for k, v in got.items():
        np.testing.assert_array_equal(v, reqs[k].astype(v.dtype), err_msg=k)
    assert np.all(reqs["tag"] == 0)


def test_pack_req16_fits_at_the_boundaries():
    r = np.zeros(3, dtype=A.REQ_DTYPE)
    r["addr"] = [0, 2**64 - 1, 12345]
    r["timer"] = [0, 2**40 - 1, 7]
    r["core"] = [0, 65535, 3]
    r["prog_id"] = [0, 63, 1]
    r["mem_type"] = [0, 1, 1]
    r["batch_start"] = [1, 0, 1]
    got = _decode(U.pack_req16(r))
    for k, v in got.items():
        np.testing.assert_array_equal(v, r[k].astype(v.dtype), err_msg=k)


@pytest.mark.parametrize("field,value", [("timer", -1), ("timer", 2**40), ("core", -1), ("core", 65536),
                                         ("prog_id", -1), ("prog_id", 64), ("mem_type", 2), ("batch_start", 2),
                                         ("tag", 1)])
def test_pack_req16_refuses_what_does_not_fit(field, value):
    r = np.zeros(4, dtype=A.REQ_DTYPE)
    r["timer"] = 5
    r[field][2] = value
    with pytest.raises(U.UncoreError, match="request 2 does not fit"):
        U.pack_req16(r)


def test_pack_req16_empty():
    assert U.pack_req16(np.zeros(0, dtype=A.REQ_DTYPE)).shape == (0, 2)


# ---------------------------------------------------------------- GPU parity

def _oracle(cfg, spec, reqs, closed=False):
    import oracle as O
    ref = O.CpuRef(cfg)
    if closed:
        ref.set_mode(O.MODE_CLOSED)
    for prog, th in P.stream_threads(spec):
        ref.alloc_core(prog, th)
    d, rc = ref.run(reqs)
    assert rc == 0
    return d, ref


def _run(cfg, specs, host, fmt, how, slots=4, budget_us=300, closed=False):
    """Every replica's stream through one device-run entry point with the
    records in format `fmt`; returns (delays [R, n], per-replica stats, completions)."""
    import torch
    R, n = host.shape
    dev = torch.device("cuda", 0)
    rec = host if fmt == U.PU_REQ_FMT_32 else U.pack_req16(host)
    um = P.UncoreManager()
    um.init(cfg, replicas=R)
    try:
        if closed:
            um.set_replay_mode(U.PU_REPLAY_CLOSED)
        for prog, th in P.stream_threads(specs[0]):
            um.allocCore(prog, th)
        um.set_device_req_format(fmt)
        off = np.arange(R + 1, dtype=np.uint64) * np.uint64(n)
        d_reqs = torch.from_numpy(np.ascontiguousarray(rec).reshape(-1).view(np.uint8).copy()).to(dev)
        d_off = torch.from_numpy(off.view(np.int64)).to(dev)
        d_pos = torch.from_numpy(off[:-1].copy().view(np.int64)).to(dev)
        d_del = torch.full((R * n,), -7, dtype=torch.int32, device=dev)
        s = torch.cuda.Stream(dev)
        if how == "unsliced":
            um.run_device(d_reqs.data_ptr(), d_off.data_ptr(), d_del.data_ptr(), s.cuda_stream)
            torch.cuda.synchronize(dev)
        else:
            d_sched = torch.zeros(um.pool_words(slots), dtype=torch.int32, device=dev)
            for _ in range(20000):
                if how == "pool":
                    um.run_device_pool(d_reqs.data_ptr(), d_off.data_ptr(), d_del.data_ptr(), d_pos.data_ptr(),
                                       d_sched.data_ptr(), slots, budget_us, s.cuda_stream)
                else:
                    um.run_device_sliced(d_reqs.data_ptr(), d_off.data_ptr(), d_del.data_ptr(), d_pos.data_ptr(),
                                         budget_us, s.cuda_stream)
                torch.cuda.synchronize(dev)
                pos = d_pos.cpu().numpy().view(np.uint64)
                if np.array_equal(pos, off[1:]):
                    break
            else:
                raise AssertionError("the runs did not finish")
        got = d_del.cpu().numpy().reshape(R, n)
        stats = [um.stats(r).as_dict() for r in range(R)]
        comp = [um.completion(r) for r in range(R)]
        return got, stats, comp
    finally:
        um.close()


@pytest.mark.gpu
@pytest.mark.parametrize("preset,kind,cores,R,n,how,closed", [
    ("C2", A.PU_STREAM_SHARED_UNIFORM, 64, 12, 3000, "pool", False),
    ("C2", A.PU_STREAM_SHARED_UNIFORM, 64, 10, 3000, "sliced", True),
    ("C2", A.PU_STREAM_SHARED_UNIFORM, 64, 6, 2000, "unsliced", False),
    ("C4", A.PU_STREAM_UNIFORM_HOTSPOT, 1024, 8, 1500, "pool", False),
])
def test_req16_runs_equal_req32_and_the_restatement(preset, kind, cores, R, n, how, closed):
    cfg = P.config_from_dict(CF.preset(preset))
    specs = [P.StreamSpec(kind, cores, seed=900 + r, max_requests=n) for r in range(R)]
    host = np.stack([P.generate_stream(sp) for sp in specs])
    g16, s16, c16 = _run(cfg, specs, host, U.PU_REQ_FMT_16, how, closed=closed)
    g32, s32, c32 = _run(cfg, specs, host, U.PU_REQ_FMT_32, how, closed=closed)
    np.testing.assert_array_equal(g16, g32)
    assert s16 == s32
    for a, b in zip(c16, c32):
        np.testing.assert_array_equal(a, b)
    for r in (0, R - 1):
        want, ref = _oracle(cfg, specs[r], host[r], closed=closed)
        np.testing.assert_array_equal(g16[r], want, err_msg=f"replica {r}")
        ws = ref.stats().as_dict()
        assert {k: s16[r][k] for k in ws if k != "requests"} == {k: ws[k] for k in ws if k != "requests"}
        np.testing.assert_array_equal(c16[r], ref.completion())
