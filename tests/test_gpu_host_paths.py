"""Host-memory (end-to-end) paths, the Field-level boundary, and the parity
cases round 1 left open, each compared bit for bit with the CPU oracle
(oracle/rse_oracle.c, pinned by the reference's KATs).

* reconstruct / reconstruct_data / verify / verify_with_buffer on HOST shards
  (the reference API's own form, core.rs:597-695): pinned and pageable,
  Option and (T, bool), single- and multi-chunk pipelines, per-stripe
  patterns (rse_reconstruct_host_batch);
* rse_code_shards_host (the code_some_slices hook), rse_gal_mul(_xor) (the
  simd_c FFI signature, simd_c/reedsolomon.h:30-42) and galois_16 mul_slice
  (lib.rs:99-118);
* encode_single / ShardByShard against the oracle's encode_single(_sep) after
  every step (core.rs:545-592, 101-231);
* GF(2^16) codecs with k + p > 256 (GF(2^16)'s reason to exist);
* more than 254 distinct erasure patterns, so the decode-matrix LRU
  (core.rs:24, 697-731) evicts, with oracle bytes before and after;
* a stream of another device (skipped on a one-GPU box).
"""
import ctypes
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import oracle as O  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def R():
    import reed_solomon_erasure as R
    return R


@pytest.fixture
def small_chunks(R):
    """64 KiB pipeline chunks, so modest shards take many chunks (and a ragged
    last one) through the host pipeline."""
    lib = R._lib.load()
    old = lib.rse_get_option(7)
    lib.rse_set_option(7, 64)
    yield
    lib.rse_set_option(7, old)


def rand_shards(rng, n_shards, n_bytes):
    return [rng.integers(0, 256, n_bytes, dtype=np.uint8) for _ in range(n_shards)]


def oracle_full(field, k, p, n_elems, rng):
    es = field // 8
    oc = O.Codec(field, k, p)
    full = rand_shards(rng, k, n_elems * es) + [np.zeros(n_elems * es, np.uint8) for _ in range(p)]
    oc.encode(full)
    return oc, full


def as_host(a, pin):
    t = torch.from_numpy(a.copy())
    return t.pin_memory() if pin else t


def as_np(x):
    return x.numpy() if isinstance(x, torch.Tensor) else x


# ------------------------------------------------------------ reconstruct
@pytest.mark.parametrize("field,k,p,n", [(8, 10, 4, 300_001), (16, 20, 8, 40_003),
                                         (8, 12, 5, 999), (16, 3, 2, 1)])
def test_reconstruct_host_matches_oracle(R, small_chunks, field, k, p, n):
    rng = np.random.default_rng(100 + k)
    oc, full = oracle_full(field, k, p, n, rng)
    r = R.core.ReedSolomon(k, p, field)
    T = k + p
    for trial in range(8):
        data_only = bool(trial & 1)
        pin = bool(trial & 2)
        flagged = bool(trial & 4)
        e = int(rng.integers(1, p + 1))
        erased = sorted(rng.choice(T, e, replace=False).tolist())
        present = [i not in erased for i in range(T)]
        # the oracle on the same erasure (core.rs:733-923)
        want = [x.copy() if ok else np.zeros_like(x) for x, ok in zip(full, present)]
        oc.reconstruct(want, present, data_only)
        if flagged:  # (T, bool): missing buffers are overwritten in place
            bufs = [as_host(x if ok else np.full_like(x, 7), pin) for x, ok in zip(full, present)]
            r.reconstruct_data_host([(b, ok) for b, ok in zip(bufs, present)]) if data_only \
                else r.reconstruct_host([(b, ok) for b, ok in zip(bufs, present)])
            got = [as_np(b) for b in bufs]
            for i in range(T):
                if present[i] or (data_only and i >= k):
                    want_i = full[i] if present[i] else np.full_like(full[i], 7)
                    assert (got[i] == want_i).all(), (erased, i)  # untouched
                else:
                    assert (got[i] == want[i]).all(), (erased, i, data_only)
        else:  # Option<T>: missing entries are allocated and filled
            shards = [as_host(x, pin) if ok else None for x, ok in zip(full, present)]
            r.reconstruct_data_host(shards) if data_only else r.reconstruct_host(shards)
            for i in range(T):
                if data_only and i >= k and not present[i]:
                    assert shards[i] is None
                else:
                    assert (as_np(shards[i]) == want[i]).all(), (erased, i, data_only)


def test_reconstruct_host_errors_touch_nothing(R):
    rng = np.random.default_rng(7)
    k, p, n = 5, 3, 1000
    _, full = oracle_full(8, k, p, n, rng)
    r = R.galois_8.ReedSolomon(k, p)
    bufs = [x.copy() for x in full]
    present = [False] * 4 + [True] * 4  # 4 present < k
    with pytest.raises(R.RSError) as ei:
        r.reconstruct_host([(b, ok) for b, ok in zip(bufs, present)])
    assert ei.value.error == R.Error.TooFewShardsPresent
    bad = [x.copy() for x in full]
    bad[3] = bad[3][:-1]
    with pytest.raises(R.RSError) as ei:
        r.reconstruct_host([(b, i != 0) for i, b in enumerate(bad)])
    assert ei.value.error == R.Error.IncorrectShardSize
    with pytest.raises(R.RSError) as ei:
        r.reconstruct_host([(b, True) for b in bufs[:-1]])
    assert ei.value.error == R.Error.TooFewShards
    assert all((a == b).all() for a, b in zip(bufs, full))


@pytest.mark.parametrize("field,k,p", [(8, 10, 4), (16, 20, 8), (8, 7, 3)])
def test_reconstruct_host_batch_per_stripe_patterns(R, small_chunks, field, k, p):
    rng = np.random.default_rng(31 + k)
    T, es, n, stripes = k + p, field // 8, 100_003, 6
    oc = O.Codec(field, k, p)
    flat = np.zeros((stripes, T, n * es), np.uint8)
    for s in range(stripes):
        sh = rand_shards(rng, k, n * es) + [np.zeros(n * es, np.uint8) for _ in range(p)]
        oc.encode(sh)
        flat[s] = np.stack(sh)
    for data_only in (False, True):
        pres = np.ones((stripes, T), bool)
        for s in range(1, stripes):  # stripe 0 has nothing missing: no bytes move
            e = int(rng.integers(1, p + 1))
            pres[s, rng.choice(T, e, replace=False)] = False
        want = flat.copy()
        work = flat.copy()
        for s in range(stripes):
            lost = [i for i in range(T) if not pres[s, i]]
            work[s, lost] = 0
            sh = [want[s, i].copy() if pres[s, i] else np.zeros(n * es, np.uint8) for i in range(T)]
            oc.reconstruct(sh, pres[s].tolist(), data_only)
            if data_only:
                for i in range(k, T):
                    if not pres[s, i]:
                        sh[i][:] = 0  # untouched by reconstruct_data
            want[s] = np.stack(sh)
        h = torch.from_numpy(work.reshape(-1).copy()).pin_memory()
        r = R.core.ReedSolomon(k, p, field)
        r.reconstruct_host_batch(h, n, stripes, pres, data_only=data_only)
        assert (h.numpy().reshape(stripes, T, -1) == want).all()


# ----------------------------------------------------------------- verify
@pytest.mark.parametrize("field,k,p,n", [(8, 10, 4, 200_017), (16, 20, 8, 3001)])
def test_verify_host_and_buffer(R, small_chunks, field, k, p, n):
    rng = np.random.default_rng(41)
    oc, full = oracle_full(field, k, p, n, rng)
    r = R.core.ReedSolomon(k, p, field)
    for pin in (True, False):
        hs = [as_host(x, pin) for x in full]
        assert r.verify_host(hs)
        buf = [as_host(np.full_like(full[0], 3), pin) for _ in range(p)]
        assert r.verify_with_buffer_host(hs, buf)
        assert all((as_np(b) == full[k + i]).all() for i, b in enumerate(buf))
        # corrupt one byte of one shard (data or parity): detected, and the
        # buffer still holds the correct parity (core.rs:328-331)
        for victim in (0, k + p - 1):
            x = as_np(hs[victim])
            j = int(rng.integers(0, x.size))
            x[j] ^= 0x5A
            assert not r.verify_host(hs)
            assert not oc.verify([as_np(h) for h in hs])
            buf2 = [as_host(np.zeros_like(full[0]), pin) for _ in range(p)]
            assert not r.verify_with_buffer_host(hs, buf2)
            want = [np.zeros_like(full[0]) for _ in range(p)]
            oc.verify_with_buffer([as_np(h) for h in hs], want)
            assert all((as_np(b) == w).all() for b, w in zip(buf2, want))
            x[j] ^= 0x5A
    with pytest.raises(R.RSError) as ei:
        r.verify_host([as_host(x, False) for x in full[:-1]])
    assert ei.value.error == R.Error.TooFewShards


def test_verify_host_flat_per_stripe(R, small_chunks):
    rng = np.random.default_rng(43)
    k, p, n, stripes = 10, 4, 150_001, 5
    oc = O.Codec(8, k, p)
    flat = np.zeros((stripes, k + p, n), np.uint8)
    for s in range(stripes):
        sh = rand_shards(rng, k, n) + [np.zeros(n, np.uint8) for _ in range(p)]
        oc.encode(sh)
        flat[s] = np.stack(sh)
    flat[2, 11, 12345] ^= 1
    flat[4, 0, n - 1] ^= 0x80
    r = R.galois_8.ReedSolomon(k, p)
    ok = r.verify_host_flat(torch.from_numpy(flat.reshape(-1)).pin_memory(), n, stripes)
    assert ok.tolist() == [True, True, False, True, False]


# ------------------------------------------------- the Field-level boundary
@pytest.mark.parametrize("field", [8, 16])
@pytest.mark.parametrize("accumulate", [False, True])
def test_code_shards_host_matches_oracle(R, small_chunks, field, accumulate):
    rng = np.random.default_rng(47 + field)
    es, n, n_in, n_out = field // 8, 70_001, 7, 3
    rows = rng.integers(0, 256, (n_out, n_in, es) if field == 16 else (n_out, n_in), dtype=np.uint8)
    ins = rand_shards(rng, n_in, n * es)
    outs = rand_shards(rng, n_out, n * es)
    want = [np.zeros(n * es, np.uint8) for _ in range(n_out)]
    O.code_some_slices(field, rows, ins, want)
    if accumulate:
        want = [w ^ o for w, o in zip(want, outs)]
    rows_int = (rows[..., 0].astype(int) << 8 | rows[..., 1]) if field == 16 else rows
    got = [torch.from_numpy(o.copy()).pin_memory() for o in outs]
    R.core.code_shards_host(field, rows_int.tolist(), [torch.from_numpy(x) for x in ins], got,
                            accumulate)
    assert all((g.numpy() == w).all() for g, w in zip(got, want))


def test_gal_mul_ffi_contract(R):
    """rse_gal_mul(_xor): the simd_c signature (simd_c/reedsolomon.h:30-42) --
    coefficient tables in, bytes processed out (the whole length: no tail
    for galois_8.rs:301-304 to finish)."""
    lib = R._lib.load()
    _, _, _, low, high = O.gf8_tables()
    rng = np.random.default_rng(53)
    for n in (1, 34, 4097, 1 << 20):
        x = rng.integers(0, 256, n, dtype=np.uint8)
        d_in = torch.from_numpy(x).cuda()
        d_out = torch.from_numpy(rng.integers(0, 256, n, dtype=np.uint8)).cuda()
        torch.cuda.synchronize()
        for c in (0, 1, 2, 25, 177, 255):
            lo = np.ascontiguousarray(low[c])
            hi = np.ascontiguousarray(high[c])
            u8 = ctypes.POINTER(ctypes.c_uint8)
            before = d_out.cpu().numpy()
            assert lib.rse_gal_mul_xor(lo.ctypes.data_as(u8), hi.ctypes.data_as(u8),
                                       d_in.data_ptr(), d_out.data_ptr(), n) == n
            assert (d_out.cpu().numpy() == before ^ O.gf8_mul_slice(c, x)).all()
            assert lib.rse_gal_mul(lo.ctypes.data_as(u8), hi.ctypes.data_as(u8),
                                   d_in.data_ptr(), d_out.data_ptr(), n) == n
            assert (d_out.cpu().numpy() == O.gf8_mul_slice(c, x)).all()


def _u8p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def _host_buf(a, kind):
    """A host copy of `a`: a numpy (pageable) array, or a pinned CPU tensor
    (its numpy view shares the pinned memory)."""
    if kind == "pageable":
        return a.copy()
    return torch.from_numpy(a.copy()).pin_memory().numpy()


@pytest.mark.parametrize("kind", ["pageable", "pinned"])
def test_gal_mul_ffi_on_host_slices(R, kind):
    """rse_gal_mul(_xor) exactly as galois_8.rs:291-327 calls
    reedsolomon_gal_mul(_xor): HOST slices (simd_c/reedsolomon.h:30-42), the
    coefficient's MUL_TABLE_LOW/HIGH rows, bytes done returned.  Every length
    0..130 (the SIMD kernel's tails), 34, and 1 MiB; out equals the oracle's
    mul_slice(_xor), so the reference's tail loop would have nothing to do."""
    lib = R._lib.load()
    _, _, _, low, high = O.gf8_tables()
    rng = np.random.default_rng(71)
    lens = list(range(0, 131)) + [34, 1 << 20]
    for n in lens:
        cs = (0, 1, 2, 29, 142, 255) if n in (34, 1 << 20) else (int(rng.integers(0, 256)),)
        x = _host_buf(rng.integers(0, 256, n, dtype=np.uint8), kind)
        for c in cs:
            lo, hi = np.ascontiguousarray(low[c]), np.ascontiguousarray(high[c])
            o = _host_buf(rng.integers(0, 256, n, dtype=np.uint8), kind)
            before = o.copy()
            assert lib.rse_gal_mul_xor(_u8p(lo), _u8p(hi), x.ctypes.data, o.ctypes.data, n) == n
            assert (o == before ^ O.gf8_mul_slice(c, x)).all(), (n, c)
            assert lib.rse_gal_mul(_u8p(lo), _u8p(hi), x.ctypes.data, o.ctypes.data, n) == n
            assert (o == O.gf8_mul_slice(c, x)).all(), (n, c)


def test_gal_mul_ffi_mixed_memory(R):
    """One slice in host memory and the other in HBM: routed by where each
    lives (hipPointerGetAttributes), same bytes as the oracle."""
    lib = R._lib.load()
    _, _, _, low, high = O.gf8_tables()
    rng = np.random.default_rng(73)
    for n in (1, 130, 65_537):
        c = int(rng.integers(1, 256))
        lo, hi = np.ascontiguousarray(low[c]), np.ascontiguousarray(high[c])
        x = rng.integers(0, 256, n, dtype=np.uint8)
        o = rng.integers(0, 256, n, dtype=np.uint8)
        d_in = torch.from_numpy(x).cuda()
        host_out = o.copy()
        torch.cuda.synchronize()
        assert lib.rse_gal_mul_xor(_u8p(lo), _u8p(hi), d_in.data_ptr(), host_out.ctypes.data, n) == n
        assert (host_out == o ^ O.gf8_mul_slice(c, x)).all()
        d_out = torch.from_numpy(o).cuda()
        torch.cuda.synchronize()
        assert lib.rse_gal_mul(_u8p(lo), _u8p(hi), x.ctypes.data, d_out.data_ptr(), n) == n
        assert (d_out.cpu().numpy() == O.gf8_mul_slice(c, x)).all()


def test_gal_mul_ordered_after_null_stream_work(R):
    """rse_gal_mul(_xor) on device slices still being written by work the
    caller queued on the null stream (torch's default stream), with no
    synchronisation in between: the library stream is a blocking stream, so
    the hook reads the finished input and xors into the finished output."""
    lib = R._lib.load()
    _, _, _, low, high = O.gf8_tables()
    n = 48 << 20
    c = 0xB7
    lo, hi = np.ascontiguousarray(low[c]), np.ascontiguousarray(high[c])
    torch.cuda.synchronize()
    with torch.cuda.stream(torch.cuda.default_stream()):
        base = torch.arange(n, device="cuda", dtype=torch.int64)
        d_in = ((base * 2654435761) >> 7).remainder(256).to(torch.uint8)
        d_out = ((base * 40503) >> 3).remainder(256).to(torch.uint8)
        for _ in range(4):  # more queued work, so the hook's launch would overtake it
            d_in = d_in ^ ((d_in >> 1) & 0x55)
        assert lib.rse_gal_mul_xor(_u8p(lo), _u8p(hi), d_in.data_ptr(), d_out.data_ptr(), n) == n
    torch.cuda.synchronize()
    x = d_in.cpu().numpy()
    o0 = (((np.arange(n, dtype=np.int64) * 40503) >> 3) % 256).astype(np.uint8)
    assert (d_out.cpu().numpy() == o0 ^ O.gf8_mul_slice(c, x)).all()


def test_verify_with_buffer_read_from_another_stream(R):
    """verify_with_buffer (core.rs:654-669) returns with the correct parity in
    the caller's buffer: read back at once on a different non-blocking
    stream (not ordered after the call's stream), it equals encode's."""
    k, p, L = 10, 4, 16 << 20
    r = R.galois_8.ReedSolomon(k, p)
    from reed_solomon_erasure.core import fill_splitmix
    shards = [torch.empty(L, dtype=torch.uint8, device="cuda") for _ in range(k + p)]
    for i in range(k):
        fill_splitmix(shards[i], 0x5EED, 900 + i)
    r.encode(shards)
    want = torch.stack(shards[k:]).cpu()
    for rep in range(3):
        buf = [torch.full((L,), 0x3C, dtype=torch.uint8, device="cuda") for _ in range(p)]
        torch.cuda.synchronize()
        assert r.verify_with_buffer(shards, buf)
        side = torch.cuda.Stream()  # non-blocking with respect to the null stream
        with torch.cuda.stream(side):
            got = torch.stack(buf).to("cpu", non_blocking=False)
        side.synchronize()
        assert torch.equal(got, want), rep


@pytest.mark.parametrize("kind", ["pageable", "pinned"])
def test_field_mul_slice_on_host_slices(R, kind):
    """galois_8 mul_slice(_xor) and galois_16's Field::mul_slice(_add)
    (lib.rs:99-118) on host slices, through the raw C ABI (as a Rust Field
    impl binds them) and through the Python mirror."""
    from reed_solomon_erasure import galois_8, galois_16
    lib = R._lib.load()
    rng = np.random.default_rng(79)
    for n in (1, 2, 33, 130, 4096 + 3, 1 << 19):
        x = _host_buf(rng.integers(0, 256, (n, 2), dtype=np.uint8), kind)
        o = _host_buf(rng.integers(0, 256, (n, 2), dtype=np.uint8), kind)
        for c in [(0, 1), (1, 0), (0xD2, 0x0F), (255, 255), (0, 0)]:
            for add in (0, 1):
                before = o.copy()
                cb = (ctypes.c_uint8 * 2)(*c)
                assert lib.rse_gf16_mul_slice(cb, x.ctypes.data, o.ctypes.data, n, add, None) == 0
                want = np.zeros(n * 2, np.uint8)
                O.code_some_slices(16, np.array([[c]], np.uint8), [x.reshape(-1)], [want])
                if add:
                    want ^= before.reshape(-1)
                assert (o.reshape(-1) == want).all(), (n, c, add)
        galois_16.mul_slice_add((3, 7), x, o)  # the Python mirror, same routing
        x8 = x.reshape(-1)
        o8 = o.reshape(-1)
        before = o8.copy()
        galois_8.mul_slice_xor(117, x8, o8)
        assert (o8 == before ^ O.gf8_mul_slice(117, x8)).all()
        assert lib.rse_gf8_mul_slice(25, x8.ctypes.data, o8.ctypes.data, x8.size, 0, None) == 0
        assert (o8 == O.gf8_mul_slice(25, x8)).all()


def test_scratch_pool_short_lived_threads(R):
    """Calls lease their streams, events, verdict words and pipeline ring from
    a process-wide pool (at most 4 idle per device): host encodes and verifies
    on 48 short-lived threads leave neither resource sets nor HBM behind."""
    import threading
    lib = R._lib.load()
    r = R.galois_8.ReedSolomon(10, 4)
    rng = np.random.default_rng(83)
    n = 3 << 20
    data = [torch.from_numpy(rng.integers(0, 256, n, dtype=np.uint8)).pin_memory() for _ in range(10)]

    par = [[torch.empty(n, dtype=torch.uint8).pin_memory() for _ in range(4)] for _ in range(4)]

    def work(i):
        shards = data + par[i]
        r.encode_host(shards)
        assert r.verify_host(shards)

    def wave():
        ts = [threading.Thread(target=work, args=(i,)) for i in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        torch.cuda.synchronize()

    wave()  # up to 4 sets in use at once, then kept idle (the cap)
    free1 = torch.cuda.mem_get_info()[0]
    live1 = lib.rse_get_option(24)
    for _ in range(11):  # 44 more threads, each gone after its call
        wave()
    assert lib.rse_get_option(24) <= 4 and lib.rse_get_option(24) <= max(live1, 4)
    assert free1 - torch.cuda.mem_get_info()[0] < (32 << 20)  # nothing piles up per thread


def test_field_mul_slice_both_fields(R):
    from reed_solomon_erasure import galois_8, galois_16
    rng = np.random.default_rng(59)
    n = 33_333
    x8 = rng.integers(0, 256, n, dtype=np.uint8)
    o8 = rng.integers(0, 256, n, dtype=np.uint8)
    d_in, d_out = torch.from_numpy(x8).cuda(), torch.from_numpy(o8.copy()).cuda()
    galois_8.mul_slice_xor(117, d_in, d_out)
    assert (d_out.cpu().numpy() == o8 ^ O.gf8_mul_slice(117, x8)).all()
    galois_8.mul_slice(25, d_in, d_out)
    assert (d_out.cpu().numpy() == O.gf8_mul_slice(25, x8)).all()
    x = rng.integers(0, 256, (n, 2), dtype=np.uint8)
    o = rng.integers(0, 256, (n, 2), dtype=np.uint8)
    for c in [(0, 1), (1, 0), (0xD2, 0x0F), (255, 255), (0, 0)]:
        for add in (False, True):
            d_in = torch.from_numpy(x).cuda()
            d_out = torch.from_numpy(o.copy()).cuda()
            (galois_16.mul_slice_add if add else galois_16.mul_slice)(c, d_in, d_out)
            want = np.zeros(n * 2, np.uint8)
            O.code_some_slices(16, np.array([[c]], np.uint8), [x.reshape(-1)], [want])
            if add:
                want ^= o.reshape(-1)
            assert (d_out.cpu().numpy().reshape(-1) == want).all(), (c, add)
    with pytest.raises(ValueError):
        galois_16.mul_slice((1, 2), d_in, d_out[:-1])


# ------------------------------------------------ encode_single vs oracle
@pytest.mark.parametrize("field,k,p", [(8, 10, 4), (8, 5, 3), (16, 6, 2), (16, 20, 8)])
def test_encode_single_steps_match_oracle(R, field, k, p):
    """encode_single(_sep) and ShardByShard after EVERY step -- the first call
    overwrites parity, later ones accumulate (core.rs:503-507) -- against the
    oracle's encode_single(_sep)."""
    rng = np.random.default_rng(61 + k)
    es, n = field // 8, 20_000 + 3
    oc = O.Codec(field, k, p)
    data = rand_shards(rng, k, n * es)
    ref = data + [rng.integers(0, 256, n * es, dtype=np.uint8) for _ in range(p)]  # stale parity
    shape = (n,) if field == 8 else (n, 2)
    dv = [torch.from_numpy(x.copy()).cuda().reshape(shape) for x in ref]
    ref_sep = [x.copy() for x in ref[k:]]
    par_sep = [torch.from_numpy(x.copy()).cuda().reshape(shape) for x in ref[k:]]
    r = R.core.ReedSolomon(k, p, field)
    sbs = R.ShardByShard(r)
    for i in range(k):
        oc.encode_single(i, ref)
        sbs.encode(dv)
        oc.encode_single_sep(i, ref[i], ref_sep)
        r.encode_single_sep(i, dv[i], par_sep)
        torch.cuda.synchronize()
        for j in range(p):
            assert (dv[k + j].cpu().numpy().reshape(-1) == ref[k + j]).all(), (i, j)
            assert (par_sep[j].cpu().numpy().reshape(-1) == ref_sep[j]).all(), (i, j)
    assert sbs.parity_ready() and oc.verify(ref)


# ------------------------------------------------ GF(2^16) past 256 shards
@pytest.mark.parametrize("k,p,lens", [(300, 60, [1, 7, 1000, 4099]), (1000, 24, [5, 2051])])
def test_gf16_beyond_256_shards(R, k, p, lens):
    rng = np.random.default_rng(k + p)
    oc = O.Codec.shared(16, k, p)
    r = R.galois_16.ReedSolomon(k, p)
    assert (np.array(r.matrix(), np.int64) ==
            (oc.matrix()[..., 0].astype(np.int64) << 8 | oc.matrix()[..., 1])).all()
    for n in lens:
        full = rand_shards(rng, k, 2 * n) + [np.zeros(2 * n, np.uint8) for _ in range(p)]
        oc.encode(full)
        dv = [torch.from_numpy(x).cuda().reshape(n, 2) for x in full[:k]] + \
             [torch.zeros((n, 2), dtype=torch.uint8, device="cuda") for _ in range(p)]
        r.encode(dv)
        torch.cuda.synchronize()
        for j in range(p):
            assert (dv[k + j].cpu().numpy().reshape(-1) == full[k + j]).all(), (n, j)
        assert r.verify(dv)
        if k <= 300:  # reconstruct: e data + parity shards lost
            lost = sorted(rng.choice(k + p, min(p, 12), replace=False).tolist())
            for i in lost:
                dv[i].zero_()
            r.reconstruct([(t, i not in lost) for i, t in enumerate(dv)])
            torch.cuda.synchronize()
            for i in lost:
                assert (dv[i].cpu().numpy().reshape(-1) == full[i]).all(), (n, i)


# ------------------------------------------------ decode-matrix LRU eviction
def test_lru_eviction_keeps_oracle_bytes(R):
    """More than 254 distinct erasure patterns (core.rs:24): early patterns are
    evicted and rebuilt on their next use, with the same bytes."""
    import itertools
    rng = np.random.default_rng(67)
    k, p, n = 10, 4, 1031
    oc, full = oracle_full(8, k, p, n, rng)
    r = R.galois_8.ReedSolomon(k, p)
    pats = [c for e in (2, 3) for c in itertools.combinations(range(k + p), e)][:300]
    dev_full = [torch.from_numpy(x).cuda() for x in full]

    def run(pat):
        bufs = [t.clone() if i not in pat else torch.zeros_like(t) for i, t in enumerate(dev_full)]
        r.reconstruct([(b, i not in pat) for i, b in enumerate(bufs)])
        return bufs

    for rnd in range(2):  # second round: the first 46 patterns were evicted
        for pat in (pats if rnd == 0 else pats[:60]):
            bufs = run(pat)
            torch.cuda.synchronize()
            for i in pat:
                assert (bufs[i].cpu().numpy() == full[i]).all(), (pat, i)


# ------------------------------------------------------------- devices
def test_stream_of_another_device(R):
    """Shards and stream on cuda:1 while cuda:0 is current: the call runs on
    the stream's device and restores the caller's (include/rse_hip.h)."""
    if torch.cuda.device_count() < 2:
        pytest.skip("one GPU on this box")
    rng = np.random.default_rng(71)
    k, p, n = 10, 4, 1 << 20
    _, full = oracle_full(8, k, p, n, rng)
    r = R.galois_8.ReedSolomon(k, p)
    torch.cuda.set_device(0)
    dv = [torch.from_numpy(x).to("cuda:1") for x in full[:k]] + \
         [torch.zeros(n, dtype=torch.uint8, device="cuda:1") for _ in range(p)]
    r.encode(dv)
    assert torch.cuda.current_device() == 0
    assert r.verify(dv)
    for j in range(p):
        assert (dv[k + j].cpu().numpy() == full[k + j]).all()


def test_last_kernel_reports_what_ran(R):
    from reed_solomon_erasure.core import last_kernel
    r = R.galois_8.ReedSolomon(10, 4)
    big = [torch.zeros(1 << 20, dtype=torch.uint8, device="cuda") for _ in range(14)]
    r.encode(big)
    assert last_kernel().startswith("bitslice gf8 10+4"), last_kernel()
    small = [torch.zeros(100, dtype=torch.uint8, device="cuda") for _ in range(14)]
    r.encode(small)
    assert last_kernel().startswith("table gf8 10+4"), last_kernel()
    torch.cuda.synchronize()


# ------------------------------------------------------ JIT disk cache
def test_cached_module_gives_oracle_bytes(tmp_path):
    """A run-time specialised module built by one process and loaded from the
    on-disk cache by another (no compile: RSE_OPT_JIT_MODULES stays 0) codes
    the oracle's bytes, on its bit-sliced kernels."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RSE_JIT_CACHE_DIR=str(tmp_path))
    pre = ("import sys; sys.path.insert(0, 'reed-solomon-erasure_amd'); sys.path.insert(0, '.'); "
           "import reed_solomon_erasure as R; L = R._lib.load(); ")
    build = subprocess.run([sys.executable, "-c", pre +
                            "print(R.galois_16.ReedSolomon(11, 5).kernel_kind(wait=True))"],
                           capture_output=True, text=True, env=env, timeout=600, cwd=root)
    assert build.stdout.split() == ["bitslice-specialised"], build.stderr[-2000:]
    use = pre + """
import numpy as np, torch
from oracle import oracle as O
L.rse_set_option(9, 2)
k, p, n = 11, 5, 3 * 16384 + 4096 + 10
rng = np.random.default_rng(5)
full = [rng.integers(0, 256, 2 * n, dtype=np.uint8) for _ in range(k)] + \\
       [np.zeros(2 * n, np.uint8) for _ in range(p)]
O.Codec(16, k, p).encode(full)
r = R.galois_16.ReedSolomon(k, p)
t = [torch.from_numpy(x).cuda().view(n, 2) for x in full[:k]] + \\
    [torch.zeros((n, 2), dtype=torch.uint8, device='cuda') for _ in range(p)]
b0 = L.rse_get_option(6)
r.encode(t)
torch.cuda.synchronize()
same = all((t[k + i].cpu().numpy().reshape(-1) == full[k + i]).all() for i in range(p))
print(same, L.rse_get_option(6) - b0 > 0, L.rse_get_option(10), L.rse_get_option(16))
"""
    out = subprocess.run([sys.executable, "-c", use], capture_output=True, text=True, env=env,
                         timeout=600, cwd=root)
    assert out.returncode == 0, out.stderr[-3000:]
    same, bitsliced, built, hits = out.stdout.split()
    assert same == "True" and bitsliced == "True" and built == "0" and int(hits) >= 1


@pytest.mark.parametrize("field,k,p", [(8, 10, 4), (16, 6, 3)])
def test_encode_sep_and_single_host_match_oracle(R, small_chunks, field, k, p):
    """encode_sep / encode_single / encode_single_sep on HOST shards
    (core.rs:545-632) against the oracle, step by step."""
    rng = np.random.default_rng(81 + k)
    es, n = field // 8, 90_001
    oc = O.Codec(field, k, p)
    data = rand_shards(rng, k, n * es)
    r = R.core.ReedSolomon(k, p, field)
    par = [torch.zeros(n * es, dtype=torch.uint8).pin_memory() for _ in range(p)]
    r.encode_sep_host([torch.from_numpy(d) for d in data], par)
    want = [np.zeros(n * es, np.uint8) for _ in range(p)]
    oc.encode_sep(data, want)
    assert all((a.numpy() == b).all() for a, b in zip(par, want))
    stale = [rng.integers(0, 256, n * es, dtype=np.uint8) for _ in range(p)]
    ref = data + [x.copy() for x in stale]
    ref_sep = [x.copy() for x in stale]
    hs = [torch.from_numpy(x.copy()) for x in ref]
    hp = [torch.from_numpy(x.copy()).pin_memory() for x in stale]
    for i in range(k):
        oc.encode_single(i, ref)
        r.encode_single_host(i, hs)
        oc.encode_single_sep(i, ref[i], ref_sep)
        r.encode_single_sep_host(i, torch.from_numpy(data[i]), hp)
        for j in range(p):
            assert (hs[k + j].numpy() == ref[k + j]).all(), (i, j)
            assert (hp[j].numpy() == ref_sep[j]).all(), (i, j)
    with pytest.raises(R.RSError) as ei:
        r.encode_single_host(k, hs)
    assert ei.value.error == R.Error.InvalidIndex


# ------------------------------------------ reconstruct_batch, shared patterns
@pytest.mark.parametrize("field,k,p,lost", [(8, 10, 4, (0, 1)), (16, 20, 8, (0, 1, 2, 3, 4, 5, 6, 7)),
                                            (8, 12, 4, (3, 13))])
def test_reconstruct_batch_shared_pattern_runs(R, field, k, p, lost):
    """A lost disk: every stripe of a batch misses the same shards.  Long runs
    of one pattern take the shared-pattern path (one plan; the pattern's own
    kernel under RSE_OPT_JIT 2) and give the oracle's bytes; two runs of
    different patterns too."""
    lib = R._lib.load()
    rng = np.random.default_rng(91 + k)
    T, es, n, stripes = k + p, field // 8, 16384 + 4096 + 64, 32
    oc = O.Codec(field, k, p)
    flat = np.zeros((stripes, T, n * es), np.uint8)
    for s in range(stripes):
        sh = rand_shards(rng, k, n * es) + [np.zeros(n * es, np.uint8) for _ in range(p)]
        oc.encode(sh)
        flat[s] = np.stack(sh)
    second = tuple(i for i in range(T) if i not in lost)[:len(lost)]
    old = lib.rse_get_option(9)
    try:
        lib.rse_set_option(9, 2)
        for runs in ((lost,), (lost, second)):
            pres = np.ones((stripes, T), bool)
            for s in range(stripes):
                pres[s, list(runs[(s * len(runs)) // stripes])] = False
            work = flat.copy()
            work[~pres] = 0
            d = torch.from_numpy(work.reshape(-1)).cuda()
            r = R.core.ReedSolomon(k, p, field)
            p0 = lib.rse_get_option(12)
            r.reconstruct_batch(d, n, stripes, pres, data_only=False)
            torch.cuda.synchronize()
            assert lib.rse_get_option(12) - p0 == len(runs)  # one pattern kernel per run
            assert (d.cpu().numpy().reshape(stripes, T, -1) == flat).all()
    finally:
        lib.rse_set_option(9, old)


@pytest.mark.parametrize("direct", [1, 0])
@pytest.mark.parametrize("field,k,p,n", [(8, 10, 4, 4096 + 7), (16, 20, 8, 1000), (8, 4, 4, 1)])
def test_host_direct_and_pipeline_agree(R, field, k, p, n, direct):
    """RSE_OPT_HOST_DIRECT: a one-stripe host call moving at most 2 MiB takes
    one pinned staging buffer (one DMA each way) instead of the pipeline's
    per-shard copies.  Both give the oracle's bytes for encode, verify (and a
    corrupted shard), verify_with_buffer and reconstruct, on pageable and
    pinned shards."""
    lib = R._lib.load()
    old = lib.rse_get_option(32)
    lib.rse_set_option(32, direct)
    try:
        rng = np.random.default_rng(7000 + n + k)
        oc, full = oracle_full(field, k, p, n, rng)
        r = R.core.ReedSolomon(k, p, field)
        T = k + p
        for pin in (False, True):
            hs = [as_host(x if i < k else np.full_like(x, 0xEE), pin) for i, x in enumerate(full)]
            r.encode_host(hs)
            assert all((as_np(hs[i]) == full[i]).all() for i in range(T))
            assert r.verify_host(hs)
            buf = [as_host(np.zeros_like(full[0]), pin) for _ in range(p)]
            assert r.verify_with_buffer_host(hs, buf)
            assert all((as_np(b) == full[k + i]).all() for i, b in enumerate(buf))
            x = as_np(hs[k - 1])
            x[-1] ^= 0x11
            assert not r.verify_host(hs)
            x[-1] ^= 0x11
            erased = sorted(rng.choice(T, p, replace=False).tolist())
            shards = [as_host(full[i], pin) if i not in erased else None for i in range(T)]
            r.reconstruct_host(shards)
            assert all((as_np(shards[i]) == full[i]).all() for i in range(T)), erased
    finally:
        lib.rse_set_option(32, old)


def test_device_flags_must_sit_with_the_stripes(R):
    """rse_reconstruct_batch reads device-resident flags in place, so they
    must be on the stripes' device: flags in HBM with host stripes (C ABI),
    or on another GPU (Python mirror and C ABI), are refused with
    RSE_ERR_INVALID_ARGUMENT (100) / InvalidShardFlags before anything is
    written."""
    import ctypes
    lib = R._lib.load()
    k, p, n, stripes = 4, 2, 4096, 3
    T = k + p
    r = R.galois_8.ReedSolomon(k, p)
    present = torch.ones((stripes, T), dtype=torch.uint8, device="cuda")
    present[:, 0] = 0
    hostbuf = np.full(stripes * T * n, 0x33, np.uint8)
    rc = lib.rse_reconstruct_batch(r._h, hostbuf.ctypes.data, n, stripes,
                                   ctypes.cast(present.data_ptr(), ctypes.POINTER(ctypes.c_uint8)),
                                   0, torch.cuda.current_stream().cuda_stream)
    assert rc == 100 and (hostbuf == 0x33).all()
    if torch.cuda.device_count() < 2:
        return
    buf = torch.full((stripes * T * n,), 0x33, dtype=torch.uint8, device="cuda:0")
    other = present.to("cuda:1")
    with pytest.raises(R.RSError) as ei:
        r.reconstruct_batch(buf, n, stripes, other)
    assert ei.value.error == R.Error.InvalidShardFlags
    rc = lib.rse_reconstruct_batch(r._h, buf.data_ptr(), n, stripes,
                                   ctypes.cast(other.data_ptr(), ctypes.POINTER(ctypes.c_uint8)),
                                   0, torch.cuda.current_stream().cuda_stream)
    assert rc == 100 and bool((buf == 0x33).all())


@pytest.mark.parametrize("zc", [1, 0])
@pytest.mark.parametrize("field,k,p", [(8, 10, 4), (16, 20, 8)])
def test_pipeline_outputs_in_place(R, small_chunks, field, k, p, zc):
    """RSE_OPT_HOST_ZC_OUT: the shards an encode or reconstruct writes, when
    they are pinned device-mapped host memory, are stored by the kernel in
    place (no D2H copies); 0 keeps the D2H copies.  Both give the oracle's
    bytes for encode_host_flat, reconstruct_host_batch (every stripe its own
    pattern, data only and with parity), per-shard encode_host with one
    pageable parity shard among pinned ones (that stripe falls back to the
    copies), and a verify of the result."""
    lib = R._lib.load()
    old = lib.rse_get_option(53)
    lib.rse_set_option(53, zc)
    try:
        es = field // 8
        n = 3 * 65536 + 4096 + 16  # several 64 KiB chunks and a ragged one
        stripes, T = 3, k + p
        rng = np.random.default_rng(31 * k + zc)
        oc = O.Codec(field, k, p)
        full = np.zeros((stripes, T, n * es), np.uint8)
        for s_ in range(stripes):
            sh = rand_shards(rng, k, n * es) + [np.zeros(n * es, np.uint8) for _ in range(p)]
            oc.encode(sh)
            full[s_] = np.stack(sh)
        r = R.core.ReedSolomon(k, p, field)
        h = torch.from_numpy(full.reshape(-1).copy()).pin_memory()
        hv = h.view(stripes, T, n * es)
        hv[:, k:].fill_(0xC3)
        r.encode_host_flat(h, n, stripes)
        assert (hv.numpy() == full).all()
        assert r.verify_host_flat(h, n, stripes).all()
        pres = np.ones((stripes, T), bool)
        for s_ in range(stripes):
            pres[s_, rng.choice(T, p, replace=False)] = False
        for data_only in (True, False):
            w = hv.numpy()
            w[~pres] = 0x3C
            r.reconstruct_host_batch(h, n, stripes, pres, data_only=data_only)
            got = hv.numpy()
            for s_ in range(stripes):
                for i in range(T):
                    if pres[s_, i] or not data_only or i < k:
                        assert (got[s_, i] == full[s_, i]).all(), (data_only, s_, i)
                    else:
                        assert (got[s_, i] == 0x3C).all(), (data_only, s_, i)  # not rebuilt
            hv.copy_(torch.from_numpy(full))
        # per-shard host stripe: pinned shards, one pageable parity shard
        hs = [torch.from_numpy(full[0, i].copy()).pin_memory() for i in range(k)] + \
             [torch.full((n * es,), 0x77, dtype=torch.uint8).pin_memory() for _ in range(p - 1)] + \
             [torch.full((n * es,), 0x77, dtype=torch.uint8)]
        r.encode_host([x.view(n, 2) if field == 16 else x for x in hs])
        for i in range(T):
            assert (hs[i].numpy() == full[0, i]).all(), i
    finally:
        lib.rse_set_option(53, old)
