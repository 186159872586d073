"""The synchronous *_now entries and the resident dispatcher that serves small
stripes (rse_dispatch.hip) against the oracle.

The reference's methods return when done (core.rs:597-695); rse_encode_now /
rse_verify_now / rse_reconstruct(_data)_now do too.  Small stripes run on one
resident workgroup that polls pinned host memory for requests: no launch, no
stream.  These tests check its bytes against the CPU oracle at every size
around its limits (and the launch path it falls back to beyond them), that it
reads fresh inputs and leaves fresh outputs when other kernels rewrite the
same buffers between calls (cross-XCD caches), that it ends by itself when
idle and comes back on the next call, and that concurrent callers are served
correctly.
"""
import ctypes
import threading
import time

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

DISPATCH, IDLE_US, MAX_BYTES, DISPATCHED, LAUNCHES = 39, 40, 41, 42, 43


@pytest.fixture(scope="module")
def R():
    import reed_solomon_erasure as R_
    return R_


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def oracle_stripe(rng, field, k, p, nbytes):
    full = [rng.integers(0, 256, nbytes, dtype=np.uint8) for _ in range(k)] + \
           [np.zeros(nbytes, np.uint8) for _ in range(p)]
    O.Codec(field, k, p).encode(full)
    return full


def shape_of(field, nbytes):
    return (nbytes,) if field == 8 else (nbytes // 2, 2)


@pytest.mark.parametrize("field,k,p", [(8, 10, 4), (8, 4, 4), (8, 16, 16), (8, 32, 32),
                                       (8, 50, 20), (8, 5, 2), (16, 20, 8), (8, 1, 1)])
@pytest.mark.parametrize("nbytes", [16, 1024, 4096, 16384, 32768, 65536, 1000])
def test_now_matches_oracle(R, field, k, p, nbytes):
    """encode_now / verify_now / reconstruct_now / reconstruct_data_now against
    the oracle; the dispatcher serves exactly the calls within its limits
    (16-byte lengths up to RSE_OPT_DISPATCH_MAX_BYTES, k x outputs <= 1024),
    the launch path the rest, with the same bytes."""
    lib = R._lib.load()
    rng = np.random.default_rng(field * 7919 + k * 31 + p * 7 + nbytes)
    full = oracle_stripe(rng, field, k, p, nbytes)
    r = R.core.ReedSolomon(k, p, field)
    shape = shape_of(field, nbytes)
    fits = (lib.rse_get_option(DISPATCH) == 1 and nbytes % 16 == 0 and
            nbytes <= lib.rse_get_option(MAX_BYTES) and k * p <= 1024)
    t = [dev(x).reshape(shape) for x in full[:k]] + \
        [torch.full(shape, 0x5A, dtype=torch.uint8, device="cuda") for _ in range(p)]
    d0 = lib.rse_get_option(DISPATCHED)
    r.encode_now(t)
    for i in range(p):  # no synchronisation: the call returned with the parity written
        assert (t[k + i].cpu().numpy().reshape(-1) == full[k + i]).all(), i
    assert lib.rse_get_option(DISPATCHED) - d0 == (1 if fits else 0)
    assert r.verify_now(t)
    t[k + p - 1].view(-1)[nbytes // 2] ^= 1
    assert not r.verify_now(t)
    t[k + p - 1].view(-1)[nbytes // 2] ^= 1
    t[0].view(-1)[nbytes - 1] ^= 0x80
    assert not r.verify_now(t)
    t[0].view(-1)[nbytes - 1] ^= 0x80
    # reconstruct: up to p random shards lost, every form
    for trial in range(3):
        lost = sorted(rng.choice(k + p, int(rng.integers(1, p + 1)), replace=False).tolist())
        present = [i not in lost for i in range(k + p)]
        tb = [x.clone() for x in t]
        for e in lost:
            tb[e].fill_(0x33)
        r.reconstruct_now(list(zip(tb, present)))
        for i in range(k + p):
            assert (tb[i].cpu().numpy().reshape(-1) == full[i]).all(), (trial, lost, i)
        for e in lost:
            tb[e].fill_(0x33)
        r.reconstruct_data_now(list(zip(tb, present)))
        for i in range(k + p):
            want = full[i] if (i < k or i not in lost) else np.full(nbytes, 0x33, np.uint8)
            assert (tb[i].cpu().numpy().reshape(-1) == want).all(), (trial, lost, i, "data")
        opt = [None if i in lost else x.clone() for i, x in enumerate(t)]
        r.reconstruct_now(opt)  # Option<T>: missing shards allocated
        for i in range(k + p):
            assert (opt[i].cpu().numpy().reshape(-1) == full[i]).all(), (trial, lost, i, "opt")


def test_now_launch_path_when_dispatch_is_off(R):
    """RSE_OPT_DISPATCH 0: every *_now call takes the launch path; same bytes."""
    lib = R._lib.load()
    old = lib.rse_get_option(DISPATCH)
    try:
        lib.rse_set_option(DISPATCH, 0)
        test_now_matches_oracle(R, 8, 10, 4, 4096)  # asserts that nothing was dispatched
    finally:
        lib.rse_set_option(DISPATCH, old)


@pytest.mark.parametrize("n,wgs,calls", [(8192, 0, 200), (65536, 8, 100)])
def test_now_fresh_inputs_and_outputs_across_kernels(R, n, wgs, calls):
    """The same device buffers, rewritten by torch kernels (whose workgroups
    land on every XCD) between calls: every call must read the new inputs and
    leave its outputs where the next torch kernel reads them -- every word
    checked.  The 64 KiB case spreads each request over all 8 resident
    dispatcher workgroups (RSE_OPT_DISPATCH_WORKGROUPS 8, shards up to the
    size limit), so the hand-off is exercised on several XCDs' L2s at sizes
    where an L1-cold test alone could not see a stale line
    (MI355X_MICROARCH.md, the agent-scope acquire each request takes)."""
    lib = R._lib.load()
    WGS = 45
    old = [lib.rse_get_option(x) for x in (WGS, MAX_BYTES)]
    if wgs:
        lib.rse_set_option(WGS, wgs)
        lib.rse_set_option(MAX_BYTES, max(n, old[1]))
        lib.rse_dispatcher_stop()  # relaunched with `wgs` workgroups
    try:
        _fresh_inputs(R, lib, n, calls)
    finally:
        lib.rse_set_option(WGS, old[0])
        lib.rse_set_option(MAX_BYTES, old[1])
        lib.rse_dispatcher_stop()


def _fresh_inputs(R, lib, n, calls):
    k, p = 10, 4
    r = R.galois_8.ReedSolomon(k, p)
    oc = O.Codec(8, k, p)
    t = [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(k + p)]
    d0 = lib.rse_get_option(DISPATCHED)
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    for it in range(calls):
        for x in t[:k]:  # new inputs, written by a kernel
            x.copy_(torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda", generator=g))
        if it % 2:
            for x in t[k:]:
                x.fill_(it & 0xFF)  # stale parity lines in L2s of other XCDs
            _ = [x.sum().item() for x in t[k:]]  # read them there
        r.encode_now(t)
        host = [x.cpu().numpy() for x in t]
        want = [h.copy() for h in host[:k]] + [np.zeros(n, np.uint8) for _ in range(p)]
        oc.encode(want)
        for i in range(p):
            assert (host[k + i] == want[k + i]).all(), (it, i)
        # a torch kernel reads the parity the dispatcher wrote
        assert int(torch.bitwise_xor(t[k], torch.from_numpy(want[k]).cuda()).sum()) == 0, it
    assert lib.rse_get_option(DISPATCHED) - d0 == calls


def test_dispatcher_idles_out_and_comes_back(R):
    """After RSE_OPT_DISPATCH_IDLE_US without a call the resident kernel ends
    (a device synchronisation then returns), and the next call starts it
    again; rse_dispatcher_stop ends it at once."""
    lib = R._lib.load()
    old = lib.rse_get_option(IDLE_US)
    k, p, n = 4, 4, 1024
    rng = np.random.default_rng(5)
    full = oracle_stripe(rng, 8, k, p, n)
    r = R.galois_8.ReedSolomon(k, p)
    t = [dev(x) for x in full[:k]] + [torch.zeros(n, dtype=torch.uint8, device="cuda")
                                       for _ in range(p)]
    try:
        lib.rse_set_option(IDLE_US, 300)
        lib.rse_dispatcher_stop()
        l0 = lib.rse_get_option(LAUNCHES)
        r.encode_now(t)
        r.encode_now(t)  # back to back: the same resident kernel
        assert lib.rse_get_option(LAUNCHES) - l0 == 1
        time.sleep(0.05)  # it ended
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        assert time.perf_counter() - t0 < 0.5
        for x in t[k:]:
            x.zero_()
        r.encode_now(t)
        assert lib.rse_get_option(LAUNCHES) - l0 == 2
        for i in range(p):
            assert (t[k + i].cpu().numpy() == full[k + i]).all()
        lib.rse_set_option(IDLE_US, 1000000)
        lib.rse_dispatcher_stop()
        r.encode_now(t)  # a kernel that would stay for 1 s
        t0 = time.perf_counter()
        lib.rse_dispatcher_stop()  # ends it now
        torch.cuda.synchronize()
        assert time.perf_counter() - t0 < 0.5
        l1 = lib.rse_get_option(LAUNCHES)
        r.encode_now(t)
        assert lib.rse_get_option(LAUNCHES) - l1 == 1
    finally:
        lib.rse_set_option(IDLE_US, old)
        lib.rse_dispatcher_stop()


def test_now_from_many_threads(R):
    """Four threads, each its own codec and shards, 100 calls each: every
    result right (one request in flight per device, callers serialised)."""
    errors = []

    def worker(seed):
        try:
            rng = np.random.default_rng(seed)
            k, p, n = 4 + seed, 2 + seed % 3, 2048
            full = oracle_stripe(rng, 8, k, p, n)
            r = R.galois_8.ReedSolomon(k, p)
            t = [dev(x) for x in full[:k]] + [torch.zeros(n, dtype=torch.uint8, device="cuda")
                                               for _ in range(p)]
            torch.cuda.synchronize()
            for it in range(100):
                for x in t[k:]:
                    x.fill_(it & 0xFF)
                r.encode_now(t)
                for i in range(p):
                    if not (t[k + i].cpu().numpy() == full[k + i]).all():
                        errors.append((seed, it, i))
                        return
        except Exception as e:  # noqa: BLE001 -- reported below
            errors.append((seed, repr(e)))

    ths = [threading.Thread(target=worker, args=(s,)) for s in range(4)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors


def test_now_c_abi_latency(R):
    """One 10+4 x 1 KiB rse_encode_now from C-ABI pointer arrays: well under
    the launch path's ~18 us (a loose bound; the bench reports the figure)."""
    lib = R._lib.load()
    k, p, n = 10, 4, 1024
    r = R.galois_8.ReedSolomon(k, p)
    t = torch.zeros((k + p, n), dtype=torch.uint8, device="cuda")
    ptrs = (ctypes.c_void_p * (k + p))(*[t[i].data_ptr() for i in range(k + p)])
    lens = (ctypes.c_size_t * (k + p))(*([n] * (k + p)))
    torch.cuda.synchronize()
    for _ in range(20):
        assert lib.rse_encode_now(r._h, ptrs, lens, k + p) == 0
    t0 = time.perf_counter()
    for _ in range(200):
        lib.rse_encode_now(r._h, ptrs, lens, k + p)
    us = (time.perf_counter() - t0) / 200 * 1e6
    assert us < 15, us


@pytest.mark.parametrize("wgs,units", [(1, 1), (3, 1), (8, 1), (8, 3), (32, 1), (32, 2)])
def test_now_dispatcher_workgroup_counts(R, wgs, units):
    """RSE_OPT_DISPATCH_WORKGROUPS: the resident kernel's workgroups split a
    request's (vector, output block) items, as many as RSE_OPT_DISPATCH_LANE_UNITS
    gives the request; every count gives the oracle's bytes for encode, verify
    and reconstruct, at sizes that use one and all of them (up to 256 KiB
    shards with the size limit raised)."""
    lib = R._lib.load()
    WGS, UNITS = 45, 49
    old = [lib.rse_get_option(x) for x in (WGS, MAX_BYTES, UNITS)]
    try:
        lib.rse_set_option(UNITS, units)
        lib.rse_set_option(WGS, wgs)
        lib.rse_set_option(MAX_BYTES, 1 << 18)
        lib.rse_dispatcher_stop()  # the next call launches with `wgs` workgroups
        for nbytes in (1024, 16384, 65536, 1 << 18):
            d0 = lib.rse_get_option(DISPATCHED)
            test_now_matches_oracle(R, 8, 10, 4, nbytes)
            assert lib.rse_get_option(DISPATCHED) - d0 >= 1 + 3  # the encode and the verifies
    finally:
        lib.rse_set_option(WGS, old[0])
        lib.rse_set_option(MAX_BYTES, old[1])
        lib.rse_set_option(UNITS, old[2])
        lib.rse_dispatcher_stop()
