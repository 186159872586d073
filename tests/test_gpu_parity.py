"""Parity of the HIP library against the oracle and the reference's fixtures.

Every test runs the product path (librse_hip.so through its C ABI, via the
Python mirror of the reference API) on an MI355X and compares bit-for-bit with
the CPU oracle (oracle/rse_oracle.c) or with golden vectors produced by the
reference's own compiled kernel (tests/golden/).  Integer arithmetic: the bar
is exact equality.
"""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from conftest import kernels_or_skip  # noqa: E402
from oracle import oracle as O  # noqa: E402

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))
KAT, GEN = GOLDEN["reference_kats"], GOLDEN["generated"]
SEED = GEN["seed"]


@pytest.fixture(scope="module")
def R():
    import reed_solomon_erasure as R
    return R


@pytest.fixture(scope="module", autouse=True)
def pattern_budget(R):
    """One process runs every test here, and the library builds at most
    RSE_OPT_JIT_MAX_PATTERNS decode-pattern modules (and blocks) per process:
    lift the caps so the tests that count pattern launches do not depend on
    how many patterns the tests before them used."""
    lib = R._lib.load()
    old = lib.rse_get_option(35), lib.rse_get_option(36)
    lib.rse_set_option(35, 1 << 20)
    lib.rse_set_option(36, 1 << 20)
    yield
    lib.rse_set_option(35, old[0])
    lib.rse_set_option(36, old[1])


@pytest.fixture
def subfield(R, request):
    """RSE_OPT_SUBFIELD for one test (read when a codec is created): 1, the
    default, codes GF(2^16) codecs of at most 256 shards in the GF(2^8)
    subfield; 0 keeps their GF(2^16) kernels, which codecs past 256 shards
    need, so the kernel tests run both.  GF(2^8) cases run once."""
    lib = R._lib.load()
    cs = request.node.callspec.params
    field = cs.get("field", 16)
    if request.param == 0 and (field == 8 or cs.get("k", 0) + cs.get("p", 0) > 256):
        pytest.skip("GF(2^8), or past 256 shards: GF(2^16) kernels either way")
    old = lib.rse_get_option(34)
    lib.rse_set_option(34, request.param)
    yield request.param
    lib.rse_set_option(34, old)


SUBFIELD = pytest.mark.parametrize("subfield", [1, 0], indirect=True, ids=["sub", "gf16"])


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint8)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def rand_shards(rng, n_shards, n_bytes):
    return [rng.integers(0, 256, n_bytes, dtype=np.uint8) for _ in range(n_shards)]


def gf16_view(a):
    return a.reshape(-1, 2)


# ------------------------------------------------------------ kernels
def test_native_library_is_loaded(R):
    lib = R._lib.load()
    assert lib.rse_version().decode().startswith("rse-mi355x")
    assert torch.cuda.is_available()


def test_mul_slice_kats(R):  # galois_8.rs:482-552 through rse_gf8_mul_slice
    lib = R._lib.load()
    inp = dev(KAT["mul_slice_input"])
    out = torch.zeros_like(inp)
    for c, xor, expect in KAT["mul_slice_steps"]:
        assert lib.rse_gf8_mul_slice(c, inp.data_ptr(), out.data_ptr(), inp.numel(), int(xor),
                                     ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
        assert host(out).tolist() == expect


def test_mul_slice_every_coefficient_and_tail(R):
    lib = R._lib.load()
    rng = np.random.default_rng(7)
    _, _, mul, _, _ = O.gf8_tables()
    for n in [1, 5, 15, 16, 17, 33, 100, 4099]:
        x = rng.integers(0, 256, n, dtype=np.uint8)
        base = rng.integers(0, 256, n, dtype=np.uint8)
        dx = dev(x)
        for c in range(256):
            for xor in (0, 1):
                out = dev(base)
                lib.rse_gf8_mul_slice(c, dx.data_ptr(), out.data_ptr(), n, xor,
                                      ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
                want = mul[c][x] ^ (base if xor else 0)
                assert (host(out) == want).all(), (n, c, xor)


def test_fill_matches_host_prng(R):
    from reed_solomon_erasure.core import fill_splitmix
    for n in [1, 7, 8, 9, 1000, 1 << 20]:
        t = torch.empty(n, dtype=torch.uint8, device="cuda")
        fill_splitmix(t, SEED, 3)
        assert (host(t) == O.splitmix_bytes(SEED, 3, n)).all()


# ------------------------------------------------------------ codec KATs
@pytest.mark.parametrize("name", ["one_encode", "readme", "reconstruct_2_2"])
def test_encode_kats(R, name):
    kat = KAT[name]
    r = R.galois_8.ReedSolomon(kat["k"], kat["p"])
    n = len(kat["data"][0])
    shards = [dev(d) for d in kat["data"]] + [torch.full((n,), 77, dtype=torch.uint8,
                                                         device="cuda") for _ in range(kat["p"])]
    r.encode(shards)
    assert [host(s).tolist() for s in shards[kat["k"]:]] == kat["parity"]
    assert r.verify(shards)
    shards[-1][0] += 1
    assert not r.verify(shards)


def test_reconstruct_kat_sequence(R):  # tests/mod.rs:249-353
    r = R.galois_8.ReedSolomon(2, 2)
    s = [dev([0, 1, 2]), dev([3, 4, 5]), dev([200, 201, 203]), dev([100, 101, 102])]
    r.encode(s)
    assert r.verify(s)
    s[0].copy_(dev([101, 102, 103]))
    r.reconstruct(list(zip(s, [False, True, True, True])))
    assert r.verify(s)
    assert [host(x).tolist() for x in s] == [[0, 1, 2], [3, 4, 5], [6, 11, 12], [5, 14, 11]]
    s[0].copy_(dev([201, 202, 203]))
    s[2].copy_(dev([101, 102, 103]))
    r.reconstruct_data(list(zip(s, [False, True, False, True])))
    assert not r.verify(s)
    assert [host(x).tolist() for x in s] == [[0, 1, 2], [3, 4, 5], [101, 102, 103], [5, 14, 11]]
    s[2].copy_(dev([101, 102, 103]))
    s[3].copy_(dev([201, 202, 203]))
    r.reconstruct_data(list(zip(s, [True, True, False, False])))
    assert not r.verify(s)
    assert [host(x).tolist() for x in s] == [[0, 1, 2], [3, 4, 5], [101, 102, 103], [201, 202, 203]]


def test_reconstruct_error_handling(R):  # tests/mod.rs:810-848
    r = R.galois_8.ReedSolomon(2, 2)
    s = [dev([0, 1, 2]), dev([3, 4, 5]), dev([200, 201, 203]), dev([100, 101, 102])]
    r.encode(s)
    s[0].copy_(dev([101, 102, 103]))
    flags = [[x, f] for x, f in zip(s, [True, False, False, False])]
    with pytest.raises(R.RSError) as ei:
        r.reconstruct([tuple(f) for f in flags])
    assert ei.value.error == R.Error.TooFewShardsPresent
    flags[3][1] = True
    r.reconstruct([tuple(f) for f in flags])


# ------------------------------------------------- golden vectors (reference SIMD)
def test_encode_10_4_matches_reference_kernel_vectors(R):
    r = R.galois_8.ReedSolomon(10, 4)
    for n, want in GEN["gf8_10_4_encode"].items():
        n = int(n)
        s = [dev(O.splitmix_bytes(SEED + n, i, n)) for i in range(10)] + \
            [torch.empty(n, dtype=torch.uint8, device="cuda") for _ in range(4)]
        r.encode(s)
        got = [host(x) for x in s[10:]]
        assert [sha(x) for x in got] == want["parity_sha256"], n
        if want["parity_hex"]:
            assert [x.tobytes().hex() for x in got] == want["parity_hex"]


def test_full_size_digests(R):
    """BASELINE configs at full size: 10+2 x 1 MiB, 10+4 x 16 MiB (GF(2^8),
    reference SIMD digests) and 20+8 x 4 MiB (GF(2^16), oracle digests),
    data generated on the device by the same PRNG."""
    from reed_solomon_erasure.core import fill_splitmix
    for key, want in GEN["full_size"].items():
        f, k, p, n = key.split("_")
        field, k, p, n = int(f[2:]), int(k), int(p), int(n)
        r = R.core.ReedSolomon(k, p, field)
        shape = (n,) if field == 8 else (n // 2, 2)
        s = [torch.empty(shape, dtype=torch.uint8, device="cuda") for _ in range(k + p)]
        for i in range(k):
            fill_splitmix(s[i], SEED, i)
        r.encode(s)
        assert [sha(host(x)) for x in s[:k]] == want["data_sha256"]
        assert [sha(host(x)) for x in s[k:]] == want["parity_sha256"], key
        assert r.verify(s)
        # reconstruct with data shards 0 and 1 erased (BASELINE config 3)
        orig = [x.clone() for x in s[:2]]
        s[0].zero_()
        s[1].fill_(0xA5)
        r.reconstruct([(x, i not in (0, 1)) for i, x in enumerate(s)])
        assert all(torch.equal(a, b) for a, b in zip(orig, s[:2]))
        assert [sha(host(x)) for x in s[:2]] == want["data_sha256"][:2]


# ------------------------------------------------------------ vs the oracle
CONFIGS = [(8, 1, 1), (8, 3, 2), (8, 5, 5), (8, 10, 4), (8, 10, 2), (8, 7, 3), (8, 12, 4),
           (8, 17, 9), (8, 33, 17), (8, 40, 20), (8, 100, 30),
           (16, 1, 1), (16, 3, 2), (16, 10, 4), (16, 20, 8), (16, 35, 17), (16, 9, 5)]
LENGTHS = [1, 2, 3, 15, 16, 17, 31, 63, 64, 65, 257, 4097]


@pytest.mark.parametrize("field,k,p", CONFIGS)
def test_encode_matches_oracle(R, field, k, p):
    rng = np.random.default_rng(k * 131 + p + field)
    r = R.core.ReedSolomon(k, p, field)
    oc = O.Codec(field, k, p)
    es = 2 if field == 16 else 1
    for n in LENGTHS:
        nb = n * es
        data = rand_shards(rng, k, nb)
        want = data + [np.zeros(nb, np.uint8) for _ in range(p)]
        oc.encode(want)
        shape = (n,) if field == 8 else (n, 2)
        s = [dev(d).reshape(shape) for d in data] + \
            [torch.full(shape, 0x5A, dtype=torch.uint8, device="cuda") for _ in range(p)]
        r.encode(s)
        for i in range(p):
            assert (host(s[k + i]).reshape(-1) == want[k + i]).all(), (field, k, p, n, i)
        assert r.verify(s)
        # encode_sep gives the same bytes (tests/mod.rs:591-662)
        par = [torch.zeros(shape, dtype=torch.uint8, device="cuda") for _ in range(p)]
        r.encode_sep(s[:k], par)
        assert all(torch.equal(a, b) for a, b in zip(par, s[k:]))


@pytest.mark.parametrize("field", [8, 16])
def test_unaligned_views(R, field):
    """Shards that are not 16-B aligned take the element path; same bytes."""
    rng = np.random.default_rng(11)
    k, p = 6, 3
    r = R.core.ReedSolomon(k, p, field)
    oc = O.Codec(field, k, p)
    es = 2 if field == 16 else 1
    for off in [1, 2, 3, 4, 8, 15]:
        off = off * es
        n = 999
        big = [dev(x) for x in rand_shards(rng, k + p, n * es + 64)]
        views = [b[off:off + n * es] for b in big]
        if field == 16:
            views = [v.view(n, 2) for v in views]
        r.encode(views)
        arr = [host(b)[off:off + n * es].copy() for b in big]
        want = [a.copy() for a in arr]
        oc.encode(want)
        assert all((a == b).all() for a, b in zip(arr, want))


@pytest.mark.parametrize("field,k,p", [(8, 10, 4), (8, 8, 5), (8, 40, 20), (8, 3, 30),
                                       (16, 20, 8), (16, 6, 3), (16, 36, 18)])
def test_reconstruct_matches_oracle(R, field, k, p):
    rng = np.random.default_rng(k * 7 + p + field)
    r = R.core.ReedSolomon(k, p, field)
    oc = O.Codec(field, k, p)
    es = 2 if field == 16 else 1
    n = 1037
    shape = (n,) if field == 8 else (n, 2)
    for trial in range(6):
        full = rand_shards(rng, k, n * es) + [np.zeros(n * es, np.uint8) for _ in range(p)]
        oc.encode(full)
        n_erase = int(rng.integers(1, p + 1))
        erased = sorted(rng.choice(k + p, n_erase, replace=False).tolist())
        present = [i not in erased for i in range(k + p)]
        data_only = bool(trial % 2)
        # oracle ((T, bool) semantics) on garbage-filled missing buffers
        ob = [x.copy() for x in full]
        for e in erased:
            ob[e][:] = 0x33
        oc.reconstruct(ob, present, data_only=data_only)
        # product, (T, bool) form
        tb = [dev(x).reshape(shape) for x in ob]
        for e in erased:
            tb[e].fill_(0x33)
        (r.reconstruct_data if data_only else r.reconstruct)(list(zip(tb, present)))
        for i in range(k + p):
            assert (host(tb[i]).reshape(-1) == ob[i]).all(), (trial, erased, i, data_only)
        for i in range(k):
            assert (ob[i] == full[i]).all()
        # product, Option form: missing = None, allocated and filled in place
        opt = [dev(x).reshape(shape) if pr else None for x, pr in zip(full, present)]
        (r.reconstruct_data if data_only else r.reconstruct)(opt)
        for i in range(k + p):
            if data_only and i >= k and not present[i]:
                assert opt[i] is None
            else:
                assert (host(opt[i]).reshape(-1) == full[i]).all()


def test_reconstruct_cache_hit_same_result(R):  # tests/mod.rs:167-247
    rng = np.random.default_rng(5)
    r = R.galois_8.ReedSolomon(8, 5)
    master = [dev(x) for x in rand_shards(rng, 13, 100_000)]
    r.encode(master)
    for erase in [(0, 2), (0, 2), (0, 2, 12), (0, 1, 9, 10, 11)]:
        s = [None if i in erase else m.clone() for i, m in enumerate(master)]
        r.reconstruct(s)
        assert all(torch.equal(a, b) for a, b in zip(s, master))
        assert r.verify(s)
    s = [None if i in (0, 1, 12) else m.clone() for i, m in enumerate(master)]
    r.reconstruct_data(s)
    assert torch.equal(s[0], master[0]) and torch.equal(s[1], master[1]) and s[12] is None


def test_verify_with_buffer_gives_correct_parity(R):  # tests/mod.rs:966-1056
    rng = np.random.default_rng(9)
    r = R.galois_8.ReedSolomon(10, 3)
    for _ in range(20):
        raw = [dev(x) for x in rand_shards(rng, 13, 100)]
        enc = [x.clone() for x in raw]
        r.encode(enc)
        buf = [dev(x) for x in rand_shards(rng, 3, 100)]
        assert not r.verify_with_buffer(raw, buf)
        assert all(torch.equal(a, b) for a, b in zip(enc[10:], buf))
        buf = [dev(x) for x in rand_shards(rng, 3, 100)]
        assert r.verify_with_buffer(enc, buf)
        assert all(torch.equal(a, b) for a, b in zip(enc[10:], buf))


def test_verify_detects_every_single_byte_corruption(R):  # tests/mod.rs:480-589
    rng = np.random.default_rng(13)
    for field, k, p, n in [(8, 10, 4, 4099), (16, 20, 8, 2051), (8, 40, 20, 777)]:
        r = R.core.ReedSolomon(k, p, field)
        shape = (n,) if field == 8 else (n, 2)
        s = [dev(x).reshape(shape) for x in rand_shards(rng, k + p, n * (field // 8))]
        r.encode(s)
        assert r.verify(s)
        for _ in range(8):
            i = int(rng.integers(0, k + p))
            j = int(rng.integers(0, s[i].numel()))
            flat = s[i].view(-1)
            old = flat[j].item()
            flat[j] = old ^ int(rng.integers(1, 256))
            assert not r.verify(s)
            flat[j] = old
        assert r.verify(s)


@pytest.mark.parametrize("spin", [1, 0])
def test_verify_completion_word(R, spin):
    """RSE_OPT_SPIN_WAIT: a verify that is one compiled check-kernel launch
    (10+4, whole 16 KiB chunks) returns when the kernel's last workgroup stores
    the completion word; the verdicts must match the stream-synchronised ones
    call after call (the workgroup count rezeroes itself), at every grid size,
    with verify_with_buffer's parity written, on shards with a 4 KiB tail (not
    armed), and from threads verifying on their own streams at once."""
    import threading
    lib = R._lib.load()
    rng = np.random.default_rng(31 + spin)
    r = R.galois_8.ReedSolomon(10, 4)
    lib.rse_set_option(31, spin)
    try:
        for n, grid in [(16384, 0), (1 << 20, 0), (3 * 16384, 1), (1 << 20, 7), (16384 + 4096, 0)]:
            lib.rse_set_option(2, grid)
            s = [dev(x) for x in rand_shards(rng, 14, n)]
            r.encode(s)
            for it in range(24):
                i = int(rng.integers(0, 14))
                j = int(rng.choice([0, n - 1, int(rng.integers(0, n))]))
                bad = it % 3 != 0
                old = s[i][j].item()
                if bad:
                    s[i][j] = old ^ int(rng.integers(1, 256))
                assert r.verify(s) == (not bad), (n, grid, it)
                if it % 4 == 1:
                    buf = [torch.zeros(n, dtype=torch.uint8, device="cuda") for _ in range(4)]
                    assert r.verify_with_buffer(s, buf) == (not bad)
                    want = [x.clone() for x in s]
                    r.encode(want)
                    assert all(torch.equal(a, b) for a, b in zip(want[10:], buf)), (n, grid, it)
                s[i][j] = old
            assert r.verify(s)
        lib.rse_set_option(2, 0)
        n = 1 << 20
        stripes = [[dev(x) for x in rand_shards(rng, 14, n)] for _ in range(4)]
        for st in stripes:
            r.encode(st)
        torch.cuda.synchronize()
        stripes[1][12][77] ^= 1
        stripes[3][0][n - 1] ^= 8
        want = [True, False, True, False]
        errors = []

        def worker(t):
            try:
                stream = torch.cuda.Stream()
                with torch.cuda.stream(stream):
                    for _ in range(40):
                        if r.verify(stripes[t]) != want[t]:
                            errors.append(t)
            except Exception as e:  # noqa: BLE001 -- reported below
                errors.append(repr(e))

        th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errors, errors
    finally:
        lib.rse_set_option(31, 1)
        lib.rse_set_option(2, 0)


# ------------------------------------------------------ shard by shard / single
@pytest.mark.parametrize("field,k,p", [(8, 10, 4), (8, 5, 3), (16, 6, 2)])
def test_shard_by_shard_same_as_encode(R, field, k, p):  # tests/mod.rs:1165-1317
    rng = np.random.default_rng(17)
    r = R.core.ReedSolomon(k, p, field)
    n = 3001
    shape = (n,) if field == 8 else (n, 2)
    s = [dev(x).reshape(shape) for x in rand_shards(rng, k + p, n * (field // 8))]
    expect = [x.clone() for x in s]
    r.encode(expect)
    sbs = R.ShardByShard(r)
    for i in range(k):
        assert not sbs.parity_ready()
        assert sbs.cur_input_index() == i
        sbs.encode(s)
    assert sbs.parity_ready()
    assert all(torch.equal(a, b) for a, b in zip(s, expect))
    with pytest.raises(R.SBSError) as ei:
        sbs.encode(s)
    assert ei.value.kind == R.SBSErrorKind.TooManyCalls
    sbs.reset()
    # sep flavour
    par = [torch.full(shape, 9, dtype=torch.uint8, device="cuda") for _ in range(p)]
    for i in range(k):
        sbs.encode_sep(s[:k], par)
    assert all(torch.equal(a, b) for a, b in zip(par, expect[k:]))
    sbs.reset()
    sbs.encode(s)
    with pytest.raises(R.SBSError) as ei:
        sbs.reset()
    assert ei.value.kind == R.SBSErrorKind.LeftoverShards
    sbs.reset_force()
    with pytest.raises(R.SBSError) as ei:
        sbs.encode(s[:-1])
    assert ei.value.kind == R.SBSErrorKind.RSError and ei.value.error == R.Error.TooFewShards


def test_encode_single_sep_and_errors(R):  # tests/mod.rs:2205-2303
    rng = np.random.default_rng(19)
    r = R.galois_8.ReedSolomon(10, 3)
    s = [dev(x) for x in rand_shards(rng, 13, 1000)]
    expect = [x.clone() for x in s]
    r.encode(expect)
    for i in range(10):
        r.encode_single_sep(i, s[i], s[10:])
    assert all(torch.equal(a, b) for a, b in zip(s, expect))
    with pytest.raises(R.RSError) as ei:
        r.encode_single(10, s)
    assert ei.value.error == R.Error.InvalidIndex
    with pytest.raises(R.RSError) as ei:
        r.encode_single_sep(0, s[0][:999], s[10:])
    assert ei.value.error == R.Error.IncorrectShardSize


# ------------------------------------------------------------ many stripes
def test_encode_flat_many_stripes(R):
    k, p, n, stripes = 10, 4, 65536 + 16, 7
    r = R.galois_8.ReedSolomon(k, p)
    buf = torch.empty(stripes * (k + p) * n, dtype=torch.uint8, device="cuda")
    from reed_solomon_erasure.core import fill_splitmix
    fill_splitmix(buf, SEED, 99)
    ref = buf.clone().view(stripes, k + p, n)
    r.encode_flat(buf, n, stripes)
    for s in range(stripes):
        shards = [ref[s, i] for i in range(k + p)]
        r.encode(shards)
    assert torch.equal(buf.view(stripes, k + p, n), ref)
    # all stripes lose the same shards; reconstruct_data_flat restores data
    erased = (1, 4, 11)
    v = buf.view(stripes, k + p, n)
    for e in erased:
        v[:, e].fill_(0)
    r.reconstruct_data_flat(buf, n, stripes, [i not in erased for i in range(k + p)])
    assert torch.equal(v[:, :k], ref[:, :k])


@pytest.mark.parametrize("field,k,p,n,stripes", [
    (8, 10, 4, 1024, 70_000),    # > 65535 stripes in flight: the kernels' stripe loop
    (8, 3, 2, 48, 5_000),        # tiny aligned shards
    (8, 5, 3, 37, 3_000),        # unaligned stride: byte path
    (16, 6, 3, 1024, 3_000),     # GF(2^16) small shards
])
def test_flat_small_shards_many_stripes(R, field, k, p, n, stripes):
    """Flat encode / verify_flat / reconstruct_data_flat over many small
    stripes (all stripes in flight on the table kernels), against the
    oracle's encode of a sample of stripes and against stripe-by-stripe calls."""
    rng = np.random.default_rng(field + k + n + stripes)
    es = field // 8
    T = k + p
    r = R.core.ReedSolomon(k, p, field)
    oc = O.Codec(field, k, p)
    host_buf = rng.integers(0, 256, stripes * T * n * es, dtype=np.uint8)
    d = dev(host_buf)
    r.encode_flat(d, n, stripes)
    got = host(d).reshape(stripes, T, n * es)
    for s_ in list(range(0, stripes, max(1, stripes // 40))) + [stripes - 1]:
        want = [got[s_, i].copy() for i in range(k)] + [np.zeros(n * es, np.uint8) for _ in range(p)]
        oc.encode(want)
        for i in range(p):
            assert (got[s_, k + i] == want[k + i]).all(), (s_, i)
    assert r.verify_flat(d, n, stripes).all()
    erased = [0, k]  # a data and a parity shard of every stripe
    v = d.view(stripes, T, n * es)
    for e in erased:
        v[:, e].fill_(0)
    r.reconstruct_data_flat(d, n, stripes, [i not in erased for i in range(T)])
    back = host(d).reshape(stripes, T, n * es)
    assert (back[:, :k] == got[:, :k]).all()


@pytest.mark.parametrize("field,k,p,n,stripes,bs,hp", [
    (8, 10, 4, 4096 + 16, 33, 1, 0),     # 4 KiB chunks bit-sliced (one per wave) + device planner
    (16, 20, 8, 2048 + 8, 40, 1, 0),     # GF(2^16) 4 KiB shards + 16 bytes: the same
    (8, 12, 4, 3 * 4096, 7, 1, 0),       # run-time specialised codec, 4 KiB chunks only
    (8, 10, 4, 4096 + 1000, 9, 0, 0),    # unaligned stride: device planner only
    (8, 10, 4, 1037, 9, 0, 0),           # device planner, byte path
    (8, 32, 16, 256, 5, 0, 0),           # one descriptor block per stripe
    (8, 1, 1, 64, 3, 0, 0),
    (8, 40, 20, 512, 3, 0, 0),           # k > 32: 2 input x 2 output blocks
    (8, 100, 60, 96, 3, 0, 0),           # 4 x 4 blocks, up to 60 erasures
    (16, 20, 8, 300, 4, 0, 0),           # GF(2^16) device planner
    (16, 300, 60, 64, 3, 0, 0),          # GF(2^16) past 256 shards: 10 x 4 blocks
    (16, 33, 17, 1001, 3, 0, 0),         # GF(2^16), byte path, odd blocks
    (16, 1, 40000, 8, 2, 0, 1),          # past the planner's LDS budget: host planner
    (8, 10, 4, 2 * 16384 + 48, 9, 1, 0),   # bit-sliced syndrome batch + device-planned tail
    (8, 10, 2, 16384, 5, 1, 0),            # bit-sliced only
    (16, 20, 8, 16384 + 8, 5, 1, 0),       # GF(2^16) bit-sliced + device-planned tail
    (8, 12, 4, 2 * 16384, 7, 1, 0),        # run-time specialised codec
    (16, 6, 3, 8192 * 3, 4, 1, 0),         # run-time specialised GF(2^16) codec
])
@pytest.mark.parametrize("dflags", [False, True])
@SUBFIELD
def test_reconstruct_batch_per_stripe_patterns(R, subfield, field, k, p, n, stripes, bs, hp, dflags):
    """rse_reconstruct_batch: every stripe with its own erasure pattern, against
    the oracle's reconstruct of each stripe (core.rs:680/690 semantics).  bs:
    the whole 16 KiB chunks run on the bit-sliced syndrome kernels from
    per-stripe descriptors planned on the device (one launch, counted); the
    rest on the table kernels from descriptors the device planner writes
    (either field, any k and p).  hp: stripes planned on the host per call
    (RSE_OPT_HOST_PLANNED_STRIPES) -- none unless the batch is past the
    device planner's LDS budget.  dflags: the flags handed over in device
    memory (read in place: the device scan, no copy)."""
    rng = np.random.default_rng(field * 1000 + k * 31 + p)
    lib = R._lib.load()
    old_jit = lib.rse_get_option(9)
    lib.rse_set_option(9, 2)  # run-time specialised kernels: wait for the build
    r = R.core.ReedSolomon(k, p, field)
    if bs:
        assert r.kernel_kind(wait=True).startswith("bitslice")
    oc = O.Codec(field, k, p)
    es = field // 8
    T = k + p
    full = []
    for s in range(stripes):
        st = rand_shards(rng, k, n * es) + [np.zeros(n * es, np.uint8) for _ in range(p)]
        oc.encode(st)
        full.append(st)
    for data_only in (False, True):
        present = np.ones((stripes, T), bool)
        for s in range(stripes):
            if s % 4 == 3:
                continue  # nothing missing
            ne = int(rng.integers(1, p + 1))
            present[s, rng.choice(T, ne, replace=False)] = False
        buf = np.concatenate([np.concatenate(st) for st in full]).copy()
        v = buf.reshape(stripes, T, n * es)
        v[~present] = 0x5A
        want = v.copy()
        for s in range(stripes):
            ob = [want[s, i].copy() for i in range(T)]
            oc.reconstruct(ob, present[s].tolist(), data_only=data_only)
            want[s] = np.stack(ob)
        d = dev(buf)
        n0 = lib.rse_get_option(6)
        h0 = lib.rse_get_option(25)
        flags = torch.from_numpy(present).cuda() if dflags else present
        r.reconstruct_batch(d, n, stripes, flags, data_only=data_only)
        got = host(d).reshape(stripes, T, n * es)
        assert lib.rse_get_option(6) - n0 == bs, data_only
        rebuilds = (~present[:, :k]).any() if data_only else (~present).any()
        assert lib.rse_get_option(25) - h0 == (stripes if hp and rebuilds else 0), data_only
        assert (got == want).all(), data_only
        # every data shard is back; parity back unless data_only
        for s in range(stripes):
            for i in range(T):
                if i < k or not data_only:
                    assert (got[s, i] == full[s][i]).all(), (s, i, data_only)
    lib.rse_set_option(9, old_jit)


@pytest.mark.parametrize("field,k,p", [(8, 10, 4), (16, 20, 8)])
@pytest.mark.parametrize("dflags", [False, True])
def test_reconstruct_batch_parity_only_losses(R, field, k, p, dflags):
    """Stripes that lost only parity shards (a scrub that found a bad parity
    disk): no data shard is missing, so no stripe needs the Gauss-Jordan
    (e_cap = 0), and the lost parity is rebuilt from the sigma rows on the
    bit-sliced syndrome kernels (one launch), not the table planner; with
    data_only nothing is written.  Against the oracle's encode."""
    rng = np.random.default_rng(4242 + field + int(dflags))
    lib = R._lib.load()
    r = R.core.ReedSolomon(k, p, field)
    assert r.kernel_kind(wait=True).startswith("bitslice")
    es, T, stripes, n = field // 8, k + p, 9, 16384 + 64
    oc = O.Codec(field, k, p)
    full = []
    for s in range(stripes):
        st = rand_shards(rng, k, n * es) + [np.zeros(n * es, np.uint8) for _ in range(p)]
        oc.encode(st)
        full.append(np.stack(st))
    want = np.stack(full)
    present = np.ones((stripes, T), bool)
    for s in range(stripes):
        lost = rng.choice(p, int(rng.integers(1, p + 1)), replace=False)
        present[s, k + lost] = False
    for data_only in (False, True):
        v = want.copy()
        v[~present] = 0x5A
        d = dev(v.reshape(-1))
        n0 = lib.rse_get_option(6)
        flags = torch.from_numpy(present).cuda() if dflags else present
        r.reconstruct_batch(d, n, stripes, flags, data_only=data_only)
        got = host(d).reshape(stripes, T, n * es)
        if data_only:
            assert (got == v).all()  # nothing lost that data_only rebuilds
        else:
            assert lib.rse_get_option(6) - n0 == 1  # the bit-sliced syndrome launch
            assert (got == want).all()


def test_reconstruct_batch_many_stripes_and_errors(R):
    """> 65535 stripes (grid.y chunking), tiny unaligned shards, all patterns
    drawn at random; errors leave every stripe untouched."""
    k, p, n, stripes = 3, 2, 7, 70_001
    rng = np.random.default_rng(77)
    r = R.galois_8.ReedSolomon(k, p)
    buf = torch.empty(stripes * (k + p) * n, dtype=torch.uint8, device="cuda")
    buf.copy_(torch.from_numpy(rng.integers(0, 256, buf.numel(), dtype=np.uint8)))
    r.encode_flat(buf, n, stripes)
    master = buf.clone()
    present = np.ones((stripes, k + p), bool)
    for s in range(stripes):
        present[s, rng.choice(k + p, int(rng.integers(0, p + 1)), replace=False)] = False
    v = buf.view(stripes, k + p, n)
    v[torch.from_numpy(~present).cuda()] = 0
    r.reconstruct_batch(buf, n, stripes, present)
    assert torch.equal(buf, master)
    # one stripe with too few shards: error, nothing written
    present[12345] = [False, False, False, True, True]
    v[12345, :3] = 0
    v[5, 0] = 0
    present[5] = [False, True, True, True, True]
    snap = buf.clone()
    with pytest.raises(R.RSError) as ei:
        r.reconstruct_batch(buf, n, stripes, present)
    assert ei.value.error == R.Error.TooFewShardsPresent
    assert torch.equal(buf, snap)


@pytest.mark.parametrize("field,k,p", [(16, 20, 8), (8, 10, 4), (8, 10, 2)])
@pytest.mark.parametrize("chunks,extra", [(1, 0), (3, 16), (2, 2), (6, 1717),
                                          (0, 4096), (1, 12336), (2, 8194)])  # 4 KiB chunks
@SUBFIELD
def test_bitslice_matches_table_kernels_and_oracle(R, subfield, field, k, p, chunks, extra):
    """The bit-sliced kernels (compiled-in parity rows) against the table
    kernels and the oracle: encode (whole 16 KiB chunks bit-sliced, the rest
    table-coded), verify (check mode) and multi-stripe flat encode."""
    lib = R._lib.load()
    es = field // 8
    nbytes = chunks * 16384 + extra * es
    n_elems = nbytes // es
    shape = (n_elems,) if field == 8 else (n_elems, 2)
    rng = np.random.default_rng(nbytes + k)
    r = R.core.ReedSolomon(k, p, field)
    oc = O.Codec(field, k, p)
    full = rand_shards(rng, k, nbytes) + [np.zeros(nbytes, np.uint8) for _ in range(p)]
    oc.encode(full)
    outs = {}
    try:
        for bs in (1, 0):
            assert lib.rse_set_option(5, bs) == 0
            t = [dev(x).reshape(shape) for x in full[:k]] + \
                [torch.zeros(shape, dtype=torch.uint8, device="cuda") for _ in range(p)]
            n0 = lib.rse_get_option(6)
            r.encode(t)
            torch.cuda.synchronize()
            assert lib.rse_get_option(6) - n0 == bs
            outs[bs] = [host(x).reshape(-1) for x in t[k:]]
            assert r.verify(t)
            flat = t[k + p - 1].view(-1)
            flat[nbytes - 1] ^= 1
            assert not r.verify(t)
            flat[nbytes - 1] ^= 1
            t[0].view(-1)[0] ^= 0x80
            assert not r.verify(t)
        for i in range(p):
            assert (outs[1][i] == full[k + i]).all(), i
            assert (outs[0][i] == full[k + i]).all(), i
        # flat multi-stripe
        stripes = 3
        buf = np.concatenate([np.concatenate(full)] * stripes)
        for s in range(stripes):
            buf[(s * (k + p) + k) * nbytes:(s + 1) * (k + p) * nbytes] = 0
        d = dev(buf)
        assert lib.rse_set_option(5, 1) == 0
        n0 = lib.rse_get_option(6)
        r.encode_flat(d, n_elems, stripes)
        # a stripe stride that is not a multiple of 16 B cannot be vectorised
        assert lib.rse_get_option(6) - n0 == (1 if nbytes % 16 == 0 else 0)
        got = host(d).reshape(stripes, k + p, nbytes)
        for s in range(stripes):
            for i in range(k + p):
                assert (got[s, i] == full[i]).all(), (s, i)
    finally:
        lib.rse_set_option(5, 1)


@pytest.mark.parametrize("field,k,p", [(16, 20, 8), (8, 10, 4), (8, 10, 2)])
@SUBFIELD
def test_bitslice_kernel_variants(R, subfield, field, k, p):
    """Every compiled bit-sliced encode variant (plain, scheduling barrier,
    cross-chunk prefetch, LDS-DMA rings of 3 and 2 slots) x nt, in store and
    check modes, over several stripes and workgroup counts so that workgroups
    run 0, 1 and many chunks."""
    lib = R._lib.load()
    es = field // 8
    nbytes = 5 * 16384
    rng = np.random.default_rng(field + k + p)
    oc = O.Codec(field, k, p)
    full = rand_shards(rng, k, nbytes) + [np.zeros(nbytes, np.uint8) for _ in range(p)]
    oc.encode(full)
    stripes = 3
    base = np.concatenate([np.concatenate(full)] * stripes)
    r = R.core.ReedSolomon(k, p, field)
    try:
        for var in (0, 1, 2, 3, 4, 5, 6, 7, 8, 9):
            for nt in (0, 1):
                for gx in (1, 7, 4096):
                    lib.rse_set_option(4, var)
                    lib.rse_set_option(1, nt)
                    lib.rse_set_option(2, gx)
                    d = dev(base)
                    d.view(stripes, k + p, nbytes)[:, k:].fill_(0)
                    n0 = lib.rse_get_option(6)
                    r.encode_flat(d, nbytes // es, stripes)
                    torch.cuda.synchronize()
                    assert lib.rse_get_option(6) - n0 == 1
                    assert (host(d) == base).all(), (var, nt, gx)
                    # check mode (verify) on the same variant: clean, then one flipped byte
                    for s_ in range(stripes):
                        sh = [d.view(stripes, k + p, nbytes)[s_, i].view(-1) for i in range(k + p)]
                        if field == 16:
                            sh = [x.view(-1, 2) for x in sh]
                        assert r.verify(sh), (var, nt, gx, s_)
                    d.view(stripes, k + p, nbytes)[1, k + p - 1, 77] ^= 4
                    sh = [d.view(stripes, k + p, nbytes)[1, i].view(-1) for i in range(k + p)]
                    if field == 16:
                        sh = [x.view(-1, 2) for x in sh]
                    assert not r.verify(sh), (var, nt, gx)
    finally:
        lib.rse_set_option(4, -1)
        lib.rse_set_option(1, 1)
        lib.rse_set_option(2, 0)


@pytest.mark.parametrize("field,k,p", [(16, 20, 8), (8, 10, 4), (8, 10, 2)])
@SUBFIELD
def test_bitslice_reconstruct_every_erasure_count(R, subfield, field, k, p):
    """Syndrome reconstruct on the bit-sliced kernels (compiled parity rows,
    runtime erasure pattern) against the oracle: every number of erased
    shards 1..p, data and/or parity, reconstruct and reconstruct_data, a
    length with whole chunks plus a table-coded tail; then the flat
    many-stripe reconstruct_data."""
    lib = R._lib.load()
    es = field // 8
    nbytes = 2 * 16384 + 48 * es
    n_elems = nbytes // es
    shape = (n_elems,) if field == 8 else (n_elems, 2)
    rng = np.random.default_rng(k * 100 + p + field)
    r = R.core.ReedSolomon(k, p, field)
    oc = O.Codec(field, k, p)
    full = rand_shards(rng, k, nbytes) + [np.zeros(nbytes, np.uint8) for _ in range(p)]
    oc.encode(full)
    patterns = []
    for ne in range(1, p + 1):
        patterns.append(sorted(rng.choice(k + p, ne, replace=False).tolist()))
    patterns += [list(range(min(p, k))), list(range(k, k + p)), [0, k + p - 1]]
    for trial, erased in enumerate(patterns):
        present = [i not in erased for i in range(k + p)]
        for data_only in (False, True):
            tb = [dev(x).reshape(shape) for x in full]
            for e in erased:
                tb[e].fill_(0x33)
            n0 = lib.rse_get_option(6)
            (r.reconstruct_data if data_only else r.reconstruct)(list(zip(tb, present)))
            torch.cuda.synchronize()
            only_parity_missing = all(e >= k for e in erased)
            if not (data_only and only_parity_missing):
                assert lib.rse_get_option(6) - n0 == 1, (erased, data_only)
            for i in range(k + p):
                got = host(tb[i]).reshape(-1)
                if data_only and i >= k and i in erased:
                    assert (got == 0x33).all()
                else:
                    assert (got == full[i]).all(), (erased, data_only, i)
    # flat, several stripes, one pattern
    stripes, erased = 3, [1, 4] if p >= 2 else [1]
    buf = np.concatenate([np.concatenate(full)] * stripes)
    d = dev(buf)
    v = d.view(stripes, k + p, nbytes)
    for e in erased:
        v[:, e].fill_(0)
    n0 = lib.rse_get_option(6)
    r.reconstruct_data_flat(d, n_elems, stripes, [i not in erased for i in range(k + p)])
    torch.cuda.synchronize()
    assert lib.rse_get_option(6) - n0 == 1
    got = host(d).reshape(stripes, k + p, nbytes)
    for s_ in range(stripes):
        for i in range(k):
            assert (got[s_, i] == full[i]).all(), (s_, i)


@pytest.mark.parametrize("field,k,p", [(16, 20, 8), (8, 10, 4)])
@SUBFIELD
def test_reconstruct_every_mixing_mode(R, subfield, field, k, p):
    """The three e x e mixings of the syndrome reconstruct (RSE_OPT_RECON_MIX
    0 v_perm tables, 1 doubling chains, 2 Horner's rule -- the default) give
    the oracle's bytes on the same patterns: every syndrome row in use (rows
    4..7 of the Horner masks set bit 31 of their mask words), data plus
    parity lost, single erasures, and random patterns with both methods."""
    from reed_solomon_erasure.core import last_kernel
    lib = R._lib.load()
    es = field // 8
    nbytes = 16384 * 2
    n_elems = nbytes // es
    shape = (n_elems,) if field == 8 else (n_elems, 2)
    rng = np.random.default_rng(77 + field)
    r = R.core.ReedSolomon(k, p, field)
    oc = O.Codec(field, k, p)
    full = rand_shards(rng, k, nbytes) + [np.zeros(nbytes, np.uint8) for _ in range(p)]
    oc.encode(full)
    patterns = [list(range(p)), list(range(p - 1)) + [k], [0], [k - 1],
                list(range(p - 2)) + [k, k + p - 1], [1, k + 1]]
    patterns += [sorted(rng.choice(k + p, int(rng.integers(1, p + 1)), replace=False).tolist())
                 for _ in range(6)]
    names = {0: "mix-tables", 1: "mix-chain", 2: "mix-horner ", 3: "mix-horner4"}
    jp = lib.rse_get_option(11)
    lib.rse_set_option(11, 0)  # no decode-pattern kernels: every use is a first use
    pairs = lib.rse_get_option(28)
    lib.rse_set_option(28, 0)  # 8 sigma rows in one wave too (pairs: test_reconstruct_wave_pairs)
    try:
        for mix in (3, 2, 1, 0):
            assert lib.rse_set_option(17, mix) == 0
            for erased in patterns:
                present = [i not in erased for i in range(k + p)]
                tb = [dev(x).reshape(shape) for x in full]
                for e in erased:
                    tb[e].fill_(0x5A)
                r.reconstruct(list(zip(tb, present)))
                torch.cuda.synchronize()
                if any(e < k for e in erased):
                    assert names[mix] in last_kernel(), (mix, erased, last_kernel())
                for i in erased:
                    assert (host(tb[i]).reshape(-1) == full[i]).all(), (mix, erased, i)
    finally:
        lib.rse_set_option(17, 3)
        lib.rse_set_option(11, jp)
        lib.rse_set_option(28, pairs)


# RSE_OPT_RECON_PAIRS: pairs per workgroup (1, 2); 3 the prefetching variant,
# 6 the compact mixing (one pair per workgroup)
@pytest.mark.parametrize("pairs", [8, 1, 2, 3, 6, 7])
@SUBFIELD
def test_reconstruct_wave_pairs(R, subfield, pairs):
    """GF(2^16) 20+8 syndrome reconstruct at 8 sigma rows on wave pairs
    (RSE_OPT_RECON_PAIRS, the default): each wave of a pair holds 4 syndrome
    rows, data planes are exchanged through LDS and the outputs' partial sums
    combined there.  Against the oracle: 8 data shards lost (the bench's
    pattern), odd output counts (one wave owns one more output), missing
    parity rows on either wave's rows, data shards of only one index parity
    present in a round, patterns whose syndrome rows are all on one wave, and
    random patterns; the shared-pattern kernel (flat stripes, one 16 KiB chunk
    plus a table-kernel tail) and reconstruct_batch (per-stripe patterns, the
    descriptor kernel) alike, each checked to run on the pair kernels."""
    from reed_solomon_erasure.core import last_kernel
    lib = R._lib.load()
    k, p, field = 20, 8, 16
    nbytes = 16384 * 3  # 3 chunks = 6 units of 8 KiB (last_kernel names the pair kernel)
    n_elems = nbytes // 2
    rng = np.random.default_rng(2028)
    r = R.core.ReedSolomon(k, p, field)
    oc = O.Codec(field, k, p)
    full = rand_shards(rng, k, nbytes) + [np.zeros(nbytes, np.uint8) for _ in range(p)]
    oc.encode(full)
    patterns = [list(range(8)), list(range(12, 20)), [1, 3, 5, 7, 9, 11, 13], [0, 2, 4, 6, 8],
                list(range(5)) + [k + 5, k + 6, k + 7], [0, k + 4, k + 5, k + 6, k + 7],
                [19, k + 7], list(range(7)) + [k], [3, 4, 5, 6, 7, 8, 9, 10],
                [0, 1, 2, 3, 4, 5, 6, k + 7]]
    patterns += [sorted(rng.choice(k + p, int(rng.integers(5, p + 1)), replace=False).tolist())
                 for _ in range(8)]
    jp, pp = lib.rse_get_option(11), lib.rse_get_option(28)
    lib.rse_set_option(11, 0)  # no decode-pattern kernels: every use is a first use
    lib.rse_set_option(28, pairs)
    try:
        for erased in patterns:
            present = [i not in erased for i in range(k + p)]
            tb = [dev(x).reshape(n_elems, 2) for x in full]
            for e in erased:
                tb[e].fill_(0x5A)
            r.reconstruct(list(zip(tb, present)))
            torch.cuda.synchronize()
            for i in erased:
                assert (host(tb[i]).reshape(-1) == full[i]).all(), (erased, i)
            # more than 4 data shards lost: syndrome rows past the 4th, NS = 8
            if sum(1 for e in erased if e < k) > 4:
                eff = (2 if subfield else 1) if pairs == 8 else pairs  # 8: by field
                np_, slot = (2, 1) if eff == 2 else (1, eff - 1 if eff >= 3 else 0)
                assert f"ns8 pairs{np_} s{slot}" in last_kernel(), (erased, last_kernel())
        # reconstruct_batch: every stripe its own pattern, all with 8 sigma
        # rows; shards with a 4 KiB remainder (one-wave kernel) and a tail
        nbytes = 16384 * 3 + 4096 + 32
        n_elems = nbytes // 2
        full = rand_shards(rng, k, nbytes) + [np.zeros(nbytes, np.uint8) for _ in range(p)]
        oc.encode(full)
        stripes = 6
        flat = np.concatenate([np.stack(full)] * stripes)
        d = dev(flat.reshape(-1)).reshape(stripes * (k + p), n_elems, 2)
        pres = np.ones((stripes, k + p), bool)
        for s_ in range(stripes):
            pres[s_, patterns[s_]] = False
            for e in patterns[s_]:
                d[s_ * (k + p) + e].fill_(0x33)
        r.reconstruct_batch(d.reshape(-1), n_elems, stripes, pres, data_only=False)
        torch.cuda.synchronize()
        got = host(d).reshape(stripes, k + p, nbytes)
        for s_ in range(stripes):
            for i in range(k + p):
                assert (got[s_, i] == full[i]).all(), (s_, i)
    finally:
        lib.rse_set_option(11, jp)
        lib.rse_set_option(28, pp)


JIT_CODECS = [(8, 12, 4), (8, 6, 3), (8, 4, 2), (8, 32, 8), (8, 1, 1), (8, 17, 5),
              (16, 10, 4), (16, 4, 2), (16, 6, 7)]


@pytest.mark.parametrize("field,k,p", JIT_CODECS)
@SUBFIELD
def test_run_time_specialised_bitslice(R, subfield, field, k, p):
    """Codecs without compiled-in bit-sliced kernels get them specialised at
    run time (hiprtc, rse_jit.cpp).  With RSE_OPT_JIT 2 the first launch waits
    for the build, so every call below runs the specialised kernels (checked
    with the bit-sliced launch counter): encode, verify (clean and corrupted),
    reconstruct / reconstruct_data at every erasure count 1..p, and flat
    multi-stripe encode, all against the oracle."""
    lib = R._lib.load()
    es = field // 8
    nbytes = 2 * 16384 + 48 * es
    n_elems = nbytes // es
    shape = (n_elems,) if field == 8 else (n_elems, 2)
    rng = np.random.default_rng(field * 1000 + k * 10 + p)
    oc = O.Codec(field, k, p)
    full = rand_shards(rng, k, nbytes) + [np.zeros(nbytes, np.uint8) for _ in range(p)]
    oc.encode(full)
    old = lib.rse_get_option(9)
    try:
        assert lib.rse_set_option(9, 2) == 0
        assert lib.rse_set_option(11, 0) == 0  # the syndrome kernels, not decode-pattern ones
        r = R.core.ReedSolomon(k, p, field)
        # GF(2^16) 10+4 in the subfield is the compiled GF(2^8) 10+4
        compiled = field == 16 and subfield and (k, p) in ((10, 4), (10, 2), (20, 8))
        assert r.kernel_kind(wait=True) == ("bitslice-compiled" if compiled
                                            else "bitslice-specialised")
        t = [dev(x).reshape(shape) for x in full[:k]] + \
            [torch.full(shape, 0x5A, dtype=torch.uint8, device="cuda") for _ in range(p)]
        n0 = lib.rse_get_option(6)
        r.encode(t)
        torch.cuda.synchronize()
        assert lib.rse_get_option(6) - n0 == 1
        for i in range(p):
            assert (host(t[k + i]).reshape(-1) == full[k + i]).all(), i
        assert r.verify(t)
        t[k + p - 1].view(-1)[nbytes - 1] ^= 1  # in the table-coded tail
        assert not r.verify(t)
        t[k + p - 1].view(-1)[nbytes - 1] ^= 1
        t[0].view(-1)[100] ^= 0x80  # in a bit-sliced chunk
        assert not r.verify(t)
        t[0].view(-1)[100] ^= 0x80
        patterns = [sorted(rng.choice(k + p, ne, replace=False).tolist()) for ne in range(1, p + 1)]
        patterns += [list(range(min(p, k))), list(range(k, k + p))]
        for erased in patterns:
            present = [i not in erased for i in range(k + p)]
            for data_only in (False, True):
                tb = [dev(x).reshape(shape) for x in full]
                for e in erased:
                    tb[e].fill_(0x33)
                n0 = lib.rse_get_option(6)
                (r.reconstruct_data if data_only else r.reconstruct)(list(zip(tb, present)))
                torch.cuda.synchronize()
                if not (data_only and all(e >= k for e in erased)):
                    assert lib.rse_get_option(6) - n0 == 1, (erased, data_only)
                for i in range(k + p):
                    got = host(tb[i]).reshape(-1)
                    if data_only and i >= k and i in erased:
                        assert (got == 0x33).all()
                    else:
                        assert (got == full[i]).all(), (erased, data_only, i)
        stripes = 3
        buf = np.concatenate([np.concatenate(full)] * stripes)
        d = dev(buf)
        d.view(stripes, k + p, nbytes)[:, k:].fill_(0)
        n0 = lib.rse_get_option(6)
        r.encode_flat(d, n_elems, stripes)
        torch.cuda.synchronize()
        assert lib.rse_get_option(6) - n0 == 1
        assert (host(d) == buf).all()
    finally:
        lib.rse_set_option(9, old)
        lib.rse_set_option(11, 1)


@pytest.mark.parametrize("field,k,p,erasures", [
    (8, 10, 4, [[0, 1], [3], [2, 11], [0, 5, 9, 13], [10, 12]]),
    (16, 20, 8, [[0, 1, 2, 3, 4, 5, 6, 7], [19, 20]]),
    (8, 12, 4, [[1, 2, 3], [0, 15]]),
    (8, 32, 8, [[0, 8, 16, 24, 32, 33, 39]]),
])
@SUBFIELD
def test_decode_pattern_kernels(R, subfield, field, k, p, erasures):
    """Repeated erasure patterns get their composed decode rows specialised
    into a bit-sliced kernel at run time (RSE_OPT_JIT 2: built on first use
    and waited for).  reconstruct, reconstruct_data and the flat many-stripe
    form on the pattern kernels (RSE_OPT_PATTERN_LAUNCHES counts them) must
    give the oracle's bytes; in the default mode a pattern's first use runs
    the syndrome kernel instead."""
    lib = R._lib.load()
    es = field // 8
    nbytes = 2 * 16384 + 40 * es
    n_elems = nbytes // es
    shape = (n_elems,) if field == 8 else (n_elems, 2)
    rng = np.random.default_rng(field + k + p)
    oc = O.Codec(field, k, p)
    full = rand_shards(rng, k, nbytes) + [np.zeros(nbytes, np.uint8) for _ in range(p)]
    oc.encode(full)
    r = R.core.ReedSolomon(k, p, field)
    old = lib.rse_get_option(9)
    try:
        # default mode: a fresh pattern's first use is not a pattern launch
        lib.rse_set_option(9, 1)
        fresh = [i for i in range(k + p) if i not in erasures[0]][:1]
        tb = [dev(x).reshape(shape) for x in full]
        n0 = lib.rse_get_option(12)
        r.reconstruct([(x, i not in fresh) for i, x in enumerate(tb)])
        torch.cuda.synchronize()
        assert lib.rse_get_option(12) == n0
        assert lib.rse_set_option(9, 2) == 0
        for erased in erasures:
            present = [i not in erased for i in range(k + p)]
            for data_only in (False, True):
                if data_only and all(e >= k for e in erased):
                    continue
                tb = [dev(x).reshape(shape) for x in full]
                for e in erased:
                    tb[e].fill_(0x77)
                n0 = lib.rse_get_option(12)
                (r.reconstruct_data if data_only else r.reconstruct)(list(zip(tb, present)))
                torch.cuda.synchronize()
                assert lib.rse_get_option(12) - n0 == 1, (erased, data_only)
                for i in range(k + p):
                    got = host(tb[i]).reshape(-1)
                    if data_only and i >= k and i in erased:
                        assert (got == 0x77).all()
                    else:
                        assert (got == full[i]).all(), (erased, data_only, i)
        # flat: several stripes, first pattern
        erased = erasures[0]
        stripes = 3
        buf = np.concatenate([np.concatenate(full)] * stripes)
        d = dev(buf)
        v = d.view(stripes, k + p, nbytes)
        for e in erased:
            v[:, e].fill_(0)
        n0 = lib.rse_get_option(12)
        r.reconstruct_data_flat(d, n_elems, stripes, [i not in erased for i in range(k + p)])
        torch.cuda.synchronize()
        assert lib.rse_get_option(12) - n0 == 1
        got = host(d).reshape(stripes, k + p, nbytes)
        for s_ in range(stripes):
            for i in range(k):
                assert (got[s_, i] == full[i]).all(), (s_, i)
    finally:
        lib.rse_set_option(9, old)


@pytest.mark.parametrize("field,k,p,n", [
    (8, 10, 4, 2 * 16384 + 48),   # bit-sliced chunks + table tail
    (16, 20, 8, 16384 + 8),       # GF(2^16) bit-sliced + tail
    (8, 12, 4, 16384),            # run-time specialised codec
    (8, 3, 2, 1000),              # table kernels (exact shape)
    (8, 7, 3, 777),               # table kernels, byte path (stride not 16-aligned)
    (8, 40, 20, 300),             # k > 32: sums materialised, then compared per stripe
])
@SUBFIELD
def test_verify_flat_per_stripe(R, subfield, field, k, p, n):
    """rse_verify_flat: one pass over many stripes, one verdict per stripe
    (core.rs:637-651 applied stripe by stripe), with corruptions in data and
    parity shards, in bit-sliced chunks and in tails, and clean stripes."""
    lib = R._lib.load()
    es = field // 8
    nb = n * es
    T = k + p
    stripes = 11
    rng = np.random.default_rng(field * 100 + k + p + n)
    oc = O.Codec(field, k, p)
    buf = []
    for _ in range(stripes):
        st = rand_shards(rng, k, nb) + [np.zeros(nb, np.uint8) for _ in range(p)]
        oc.encode(st)
        buf.append(np.concatenate(st))
    buf = np.concatenate(buf)
    want = np.ones(stripes, bool)
    v = buf.reshape(stripes, T, nb)
    for s_ in (1, 4, 5, 9):
        i = int(rng.integers(0, T))
        pos = int(rng.integers(0, nb)) if s_ != 9 else nb - 1
        v[s_, i, pos] ^= 1 + int(rng.integers(0, 255))
        want[s_] = False
    old = lib.rse_get_option(9)
    try:
        lib.rse_set_option(9, 2)
        r = R.core.ReedSolomon(k, p, field)
        d = dev(buf)
        got = r.verify_flat(d, n, stripes)
        assert (got == want).all(), (got, want)
        # the same verdicts as verify() stripe by stripe
        dv = d.view(stripes, T, nb)
        shape = (n,) if field == 8 else (n, 2)
        for s_ in range(stripes):
            assert r.verify([dv[s_, i].view(*shape) for i in range(T)]) == want[s_]
        # nothing was written
        assert (host(d) == buf).all()
    finally:
        lib.rse_set_option(9, old)


def test_encode_host_matches_device(R):
    rng = np.random.default_rng(23)
    k, p = 10, 4
    r = R.galois_8.ReedSolomon(k, p)
    for n in [100, (8 << 20) + 3, 20 << 20]:
        data = rand_shards(rng, k, n)
        hs = [torch.from_numpy(d).pin_memory() for d in data] + \
             [torch.zeros(n, dtype=torch.uint8).pin_memory() for _ in range(p)]
        r.encode_host(hs)
        ds = [dev(d) for d in data] + [torch.empty(n, dtype=torch.uint8, device="cuda")
                                        for _ in range(p)]
        r.encode(ds)
        for i in range(p):
            assert (hs[k + i].numpy() == host(ds[k + i])).all()
    # flat host stripes through one pipeline, pinned and pageable
    for pin in (True, False):
        n, stripes = (4 << 20) + 100, 3
        rng2 = np.random.default_rng(pin)
        h = torch.from_numpy(rng2.integers(0, 256, stripes * (k + p) * n, dtype=np.uint8))
        if pin:
            h = h.pin_memory()
        d = h.cuda()
        r.encode_host_flat(h, n, stripes)
        r.encode_flat(d, n, stripes)
        assert torch.equal(h, d.cpu())
    # pageable numpy memory works too
    data = rand_shards(rng, k, 5000)
    hs = data + [np.zeros(5000, np.uint8) for _ in range(p)]
    r.encode_host(hs)
    want = data + [np.zeros(5000, np.uint8) for _ in range(p)]
    O.Codec(8, k, p).encode(want)
    assert all((a == b).all() for a, b in zip(hs, want))


# ------------------------------------------------------ device inversion
def test_device_inversion_matches_oracle(R):
    lib = R._lib.load()
    rng = np.random.default_rng(29)
    oc = O.Codec(8, 10, 4)
    m = oc.matrix()
    mats, want = [], []
    for _ in range(64):  # decode submatrices of random erasure patterns
        erased = rng.choice(14, int(rng.integers(1, 5)), replace=False)
        valid = [i for i in range(14) if i not in erased][:10]
        mats.append(m[valid])
        want.append(O.matrix_invert(8, m[valid]))
    for n in [1, 3, 17, 64, 255]:  # random (mostly invertible) matrices
        for _ in range(2):
            a = rng.integers(0, 256, (n, n), dtype=np.uint8)
            try:
                want.append(O.matrix_invert(8, a))
            except ValueError:
                continue
            mats.append(a)
    by_n = {}
    for a, w in zip(mats, want):
        by_n.setdefault(a.shape[0], []).append((a, w))
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for n, items in by_n.items():
        src = dev(np.stack([a for a, _ in items]))
        dst = torch.empty_like(src)
        sing = torch.full((len(items),), 7, dtype=torch.int32, device="cuda")
        assert lib.rse_gf8_invert_batch(src.data_ptr(), dst.data_ptr(), sing.data_ptr(), n,
                                        len(items), stream) == 0
        assert (host(sing) == 0).all()
        assert (host(dst) == np.stack([w for _, w in items])).all(), n
    # singular (matrix.rs:419-423)
    src = dev(np.array(KAT["matrix_singular"], np.uint8)[None])
    dst = torch.empty_like(src)
    sing = torch.zeros(1, dtype=torch.int32, device="cuda")
    lib.rse_gf8_invert_batch(src.data_ptr(), dst.data_ptr(), sing.data_ptr(), 2, 1, stream)
    assert host(sing)[0] == 1


def test_device_inversion_gf16_matches_oracle(R):
    """rse_gf16_invert_batch (matrix.rs:195-261 over galois_16): decode
    submatrices of GF(2^16) codecs (20+8, 300+60 past 256 shards) and random
    matrices, in LDS (n <= 127) and in the device workspace (n = 128, 300),
    against the oracle's matrix_invert(16, ...); singular matrices flagged."""
    lib = R._lib.load()
    rng = np.random.default_rng(37)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    cases = []
    for k, p, count in ((20, 8, 24), (300, 60, 2)):
        m = O.Codec(16, k, p).matrix()
        for _ in range(count):
            erased = rng.choice(k + p, int(rng.integers(1, p + 1)), replace=False)
            valid = [i for i in range(k + p) if i not in erased][:k]
            cases.append(m[valid])
    for n in (1, 2, 7, 64, 127, 128):
        for _ in range(2):
            cases.append(rng.integers(0, 256, (n, n, 2), dtype=np.uint8))
    by_n = {}
    for a in cases:
        try:
            w = O.matrix_invert(16, a)
        except ValueError:
            continue
        by_n.setdefault(a.shape[0], []).append((a, w))
    assert {20, 300, 127, 128} <= set(by_n)
    for n, items in by_n.items():
        src = dev(np.stack([a for a, _ in items]))
        dst = torch.empty_like(src)
        sing = torch.full((len(items),), 7, dtype=torch.int32, device="cuda")
        assert lib.rse_gf16_invert_batch(src.data_ptr(), dst.data_ptr(), sing.data_ptr(), n,
                                         len(items), stream) == 0
        assert (host(sing) == 0).all(), n
        assert (host(dst) == np.stack([w for _, w in items])).all(), n
    # singular: a repeated row, and a zero column, next to an invertible one
    good = by_n[20][0][0]
    bad1 = good.copy()
    bad1[5] = bad1[2]
    bad2 = good.copy()
    bad2[:, 7] = 0
    src = dev(np.stack([bad1, good, bad2]))
    dst = torch.zeros_like(src)
    sing = torch.full((3,), 7, dtype=torch.int32, device="cuda")
    assert lib.rse_gf16_invert_batch(src.data_ptr(), dst.data_ptr(), sing.data_ptr(), 20, 3,
                                     stream) == 0
    assert host(sing).tolist() == [1, 0, 1]
    assert (host(dst)[1] == by_n[20][0][1]).all()


# ------------------------------------------------ quickcheck-style round trips
def test_random_round_trips(R):  # tests/mod.rs:355-478, tests/galois_16.rs:36-140
    rng = np.random.default_rng(31)
    for trial in range(40):
        field = 8 if trial % 3 else 16
        k = int(rng.integers(1, 256))
        p = int(rng.integers(1, 256))
        if k + p > 256:
            p -= k + p - 256
        n = int(rng.integers(1, 3000))
        r = R.core.ReedSolomon(k, p, field)
        shape = (n,) if field == 8 else (n, 2)
        expect = [dev(x).reshape(shape) for x in rand_shards(rng, k + p, n * (field // 8))]
        r.encode(expect)
        assert r.verify(expect)
        corrupt = int(rng.integers(0, p + 1))
        pos = rng.choice(k + p, corrupt, replace=False).tolist()
        s = [x.clone() for x in expect]
        for q in pos:
            s[q].random_(0, 256)
        r.reconstruct([(x, i not in pos) for i, x in enumerate(s)])
        assert all(torch.equal(a, b) for a, b in zip(s, expect)), (field, k, p, n, pos)
        assert r.verify(s)


def test_random_round_trips_bitsliced(R):
    """Quickcheck-style round trips (tests/mod.rs:355-478) at chunk-sized
    lengths, so that the bit-sliced kernels run: random codecs of both fields
    with k <= 32, p <= 8 (compiled in or specialised at run time, waited for),
    random lengths with ragged tails, random erasures rebuilt by the syndrome
    kernels and by decode-pattern kernels; every shard against the oracle."""
    lib = R._lib.load()
    rng = np.random.default_rng(4242)
    old = lib.rse_get_option(9)
    try:
        lib.rse_set_option(9, 2)
        for trial in range(3):  # each codec costs a few seconds of hiprtc
            field = 16 if trial % 2 else 8
            k, p = int(rng.integers(1, 25)), int(rng.integers(1, 9))
            es = field // 8
            n = int(rng.integers(16384, 3 * 16384)) // es  # elements
            shape = (n,) if field == 8 else (n, 2)
            oc = O.Codec(field, k, p)
            full = rand_shards(rng, k, n * es) + [np.zeros(n * es, np.uint8) for _ in range(p)]
            oc.encode(full)
            r = R.core.ReedSolomon(k, p, field)
            assert r.kernel_kind(wait=True).startswith("bitslice"), (field, k, p)
            t = [dev(x).reshape(shape) for x in full[:k]] + \
                [torch.zeros(shape, dtype=torch.uint8, device="cuda") for _ in range(p)]
            r.encode(t)
            for i in range(p):
                assert (host(t[k + i]).reshape(-1) == full[k + i]).all(), (field, k, p, n, i)
            assert r.verify(t)
            for patterns in (0, 1):
                lib.rse_set_option(11, patterns)
                erased = rng.choice(k + p, int(rng.integers(1, p + 1)), replace=False).tolist()
                s_ = [x.clone() for x in t]
                for e in erased:
                    s_[e].random_(0, 256)
                r.reconstruct([(x, i not in erased) for i, x in enumerate(s_)])
                for i in range(k + p):
                    assert torch.equal(s_[i], t[i]), (field, k, p, n, erased, patterns, i)
    finally:
        lib.rse_set_option(9, old)
        lib.rse_set_option(11, 1)


def test_concurrent_threads_and_streams(R):
    """ReedSolomon is Sync (core.rs:349: the decode-matrix cache is behind a
    mutex): one codec shared by 4 host threads, each on its own HIP stream,
    encoding and reconstructing its own stripes (ctypes drops the GIL for the
    calls) -- every result the oracle's, and the run-time build of a codec
    requested by all threads at once happens once."""
    import threading
    lib = R._lib.load()
    k, p, n = 12, 4, 3 * 16384 + 4096 + 7
    oc = O.Codec(8, k, p)
    r = R.galois_8.ReedSolomon(k, p)
    built0 = lib.rse_get_option(10)
    errors = []

    def work(t):
        try:
            rng = np.random.default_rng(100 + t)
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                for it in range(6):
                    data = rand_shards(rng, k, n)
                    want = data + [np.zeros(n, np.uint8) for _ in range(p)]
                    oc.encode(want)
                    sh = [dev(x) for x in data] + [torch.zeros(n, dtype=torch.uint8, device="cuda")
                                                   for _ in range(p)]
                    r.encode(sh)
                    erased = rng.choice(k + p, int(rng.integers(1, p + 1)), replace=False).tolist()
                    for e in erased:
                        sh[e].fill_(0)
                    r.reconstruct([(x, i not in erased) for i, x in enumerate(sh)])
                    st.synchronize()
                    for i in range(k + p):
                        if not (sh[i].cpu().numpy() == want[i]).all():
                            errors.append((t, it, i))
        except Exception as e:  # surfaced below
            errors.append(repr(e))

    ths = [threading.Thread(target=work, args=(t,)) for t in range(4)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    assert not errors, errors[:5]
    r.kernel_kind(wait=True)
    assert lib.rse_get_option(10) - built0 <= 2 + 8  # codec modules once (+ any patterns)


# ------------------------------------------------ every compiled variant
@pytest.mark.parametrize("field,k,p", [(8, 10, 4), (8, 10, 2), (16, 20, 8), (8, 3, 2), (8, 12, 6)])
def test_all_kernel_variants_and_launch_shapes(R, field, k, p):
    """Launch-shape options and alternate kernel variants (tools/tune.py) change
    speed only: every combination must produce the oracle's bytes."""
    lib = R._lib.load()
    rng = np.random.default_rng(37)
    r = R.core.ReedSolomon(k, p, field)
    oc = O.Codec(field, k, p)
    es = field // 8
    stripes, n = 3, 512 * 16 * 3 + 16 * 7 + 5  # full VPL=2 spans, leftovers, byte tail
    shape = (n,) if field == 8 else (n, 2)
    saved = [lib.rse_get_option(i) for i in (1, 2, 3, 4)]
    data = [rand_shards(rng, k, n * es) for _ in range(stripes)]
    want = []
    for s in range(stripes):
        w = data[s] + [np.zeros(n * es, np.uint8) for _ in range(p)]
        oc.encode(w)
        want.append(np.concatenate(w))
    try:
        for variant in range(5):
            for nt in (0, 1):
                for gx, gy in [(0, 1), (3, 1), (1, 0), (2, 2), (4096, 1)]:
                    for key, val in ((1, nt), (2, gx), (3, gy), (4, variant)):
                        lib.rse_set_option(key, val)
                    buf = torch.empty(stripes * (k + p) * n * es, dtype=torch.uint8, device="cuda")
                    v = buf.view(stripes, k + p, n * es)
                    for s in range(stripes):
                        for i in range(k):
                            v[s, i].copy_(dev(data[s][i]))
                    r.encode_flat(buf, n, stripes)
                    got = host(buf).reshape(stripes, -1)
                    for s in range(stripes):
                        assert (got[s] == want[s]).all(), (variant, nt, gx, gy, s)
                    shards = [v[0, i].view(*shape) for i in range(k + p)]
                    assert r.verify(shards)
    finally:
        for key, val in zip((1, 2, 3, 4), saved):
            lib.rse_set_option(key, val)


# ------------------------------------------------------------ bench, N > 1
@pytest.mark.parametrize("ranks,extras", [(2, False), (4, True)])
def test_bench_ranks_rehearsal(ranks, extras, tmp_path):
    """bench.py's multi-rank path (torch.distributed.run, barrier, max-over-
    ranks timing, whole-job value) with `ranks` ranks sharing the one GPU over
    gloo.  Every rank checks its own first and last stripe against the
    reference digests and the verdicts are combined (BASELINE config 4's
    self-check, rehearsed at 4 stripes per rank); with extras, every rank also
    runs the host-memory leg at once."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RSE_BENCH_REHEARSAL="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={ranks}", "--master-addr", "127.0.0.1", "--master-port",
           str(29533 + ranks), os.path.join(root, "bench.py"), "--gpus", str(ranks), "--steps",
           "2", "--warmup", "1", "--stripes", "4", "--no-cpu",
           "--full-out", str(tmp_path / "full.json")] + ([] if extras else ["--no-extras"])
    out = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=600, cwd=root)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == ranks and d["config"]["global_stripes_per_step"] == 4 * ranks
    assert d["config"]["parity_check_vs_reference"] is True
    assert d["config"]["parity_check_per_rank"] == [1] * ranks
    assert d["config"]["parity_checked_stripes_rank0"] == [0, 3]
    assert len(d["roofline"]["kernel_ms_per_launch_per_rank"]) == ranks
    lo, hi = d["roofline"]["kernel_ms_per_launch_min_max"]
    assert 0 < lo <= hi
    # what the collective saw: the rehearsal's gloo group of `ranks` ranks, each
    # rank's device gathered (all on the one GPU here, so not distinct)
    coll = d["collective"]
    assert coll["backend"] == "gloo" and coll["world_size"] == ranks and coll["rehearsal"]
    coll = json.load(open(tmp_path / "full.json"))["collective"]  # with every rank's device
    assert len(coll["rank_devices"]) == ranks
    assert all(x["device"] == "cuda:0" and x["pci"] for x in coll["rank_devices"])
    assert coll["distinct_gpus"] is False
    assert d["value"] > 0 and d["roofline"]["achieved"] > 0
    assert len(json.dumps(d)) < 4096  # the printed line stays compact at N ranks
    full = json.load(open(tmp_path / "full.json"))  # every leg
    assert full["config"] == d["config"] and full["value"] == d["value"]
    if extras:
        h = full["end_to_end_host_all_ranks"]
        assert h["ranks"] == ranks and h["parity_matches_device_all_ranks"] is True


# (field, k, p, modules): one wide module (p <= 64, k + 2p <= 480), or past
# 64 outputs one module per output group of <= 64 (round 6; 8 x 32 blocks
# before).  Waves per workgroup
# (rse_jit.cpp wide_waves): 1 for p < 4, else 4 (p <= 32), 8 (10+40: shares
# of 5; 4+17: 5/4/4/4), or 16 for GF(2^8) past 48 outputs (64+64: 4 each).
WIDE_CODECS = [(8, 40, 2, 1), (8, 6, 10, 1), (16, 36, 3, 1), (8, 33, 9, 1), (16, 20, 12, 1),
               (8, 10, 40, 1), (16, 4, 17, 1), (8, 4, 66, 2),  # 66 outputs: two groups of 33
               (8, 32, 32, 1), (8, 64, 64, 1)]  # benches/bandwidth.rs:94-95's widest (half chunks)


def test_wide_sixteen_waves(R):
    """RSE_OPT_WIDE_SPLIT 4: 4 outputs per wave, so a 60+60 codec's module is
    16 waves (1024 lanes, half chunks, paired networks, ~115 VGPRs); the same
    bytes as the oracle for encode, verify and flat stripes.  A codec no other
    test builds (modules are keyed by rows, not options)."""
    from reed_solomon_erasure.core import last_kernel
    lib = R._lib.load()
    old = lib.rse_get_option(18)
    try:
        assert lib.rse_set_option(18, 4) == 0
        test_wide_codec_kernels(R, 1, 8, 60, 60, 1)
        assert last_kernel().startswith("bitslice-wide gf8 60+60 w16 half"), last_kernel()
    finally:
        lib.rse_set_option(18, old)


def test_wide_full_chunks_option(R):
    """RSE_OPT_WIDE_HALF 0: a GF(2^8) paired wide module on 4 KiB chunks per
    wave (two plane groups per lane, wide_body_lds_deep) instead of the
    default 2 KiB ones (wide_body_half); the same bytes.  A codec no other
    test builds (modules are keyed by rows, not options)."""
    from reed_solomon_erasure.core import last_kernel
    lib = R._lib.load()
    old = lib.rse_get_option(38)
    try:
        assert lib.rse_set_option(38, 0) == 0
        test_wide_codec_kernels(R, 1, 8, 34, 10, 1)
        assert "half" not in last_kernel(), last_kernel()
    finally:
        lib.rse_set_option(38, old)
    test_wide_codec_kernels(R, 1, 8, 35, 10, 1)  # the default: half chunks
    assert last_kernel().startswith("bitslice-wide gf8 35+10 w4 half"), last_kernel()


def test_wide_codec_unbalanced_waves(R):
    """RSE_OPT_WIDE_BALANCE 0: W = ceil(p / 8) waves (2 for 7+11, shares 6/5)
    instead of 4; same bytes.  A codec no other test builds (modules are keyed
    by rows, not options)."""
    lib = R._lib.load()
    old = lib.rse_get_option(19)
    try:
        assert lib.rse_set_option(19, 0) == 0
        test_wide_codec_kernels(R, 1, 8, 7, 11, 1)
        from reed_solomon_erasure.core import last_kernel
        assert last_kernel().startswith("bitslice-wide gf8 7+11 w2"), last_kernel()
    finally:
        lib.rse_set_option(19, old)


@pytest.mark.parametrize("field,k,p,modules", WIDE_CODECS)
@SUBFIELD
def test_wide_codec_kernels(R, subfield, field, k, p, modules):
    """Wide codecs (k > 32 or p > 8) on their run-time specialised kernels:
    one module whose workgroup's waves each code <= 8 outputs over all k
    inputs of the same 4 KiB chunk (every input read once, every output
    written once: ONE launch), or -- past 64 outputs -- blocks of 8 outputs x
    32 inputs launched output block by output block, later input blocks
    accumulating.  Encode, verify (compare fused into the wide kernel) and flat
    multi-stripe encode match the oracle over whole 4 KiB chunks and a
    table-coded tail."""
    lib = R._lib.load()
    es = field // 8
    nbytes = 2 * 16384 + 4096 + 48 * es
    n_elems = nbytes // es
    shape = (n_elems,) if field == 8 else (n_elems, 2)
    rng = np.random.default_rng(field * 1000 + k * 10 + p)
    oc = O.Codec(field, k, p)
    full = rand_shards(rng, k, nbytes) + [np.zeros(nbytes, np.uint8) for _ in range(p)]
    oc.encode(full)
    blocks = modules
    old, old51 = lib.rse_get_option(9), lib.rse_get_option(51)
    try:
        assert lib.rse_set_option(9, 2) == 0
        # k = p = 16 / 32 / 64 default to the FFT kernels (tests/test_gpu_fft.py):
        # the wide modules here are their RSE_OPT_FFT 0 path
        assert lib.rse_set_option(51, 0) == 0
        r = R.core.ReedSolomon(k, p, field)
        assert r.kernel_kind(wait=True) == "bitslice-specialised"
        t = [dev(x).reshape(shape) for x in full[:k]] + \
            [torch.full(shape, 0x5A, dtype=torch.uint8, device="cuda") for _ in range(p)]
        n0 = lib.rse_get_option(6)
        r.encode(t)
        torch.cuda.synchronize()
        assert lib.rse_get_option(6) - n0 == blocks
        from reed_solomon_erasure.core import last_kernel
        if modules == 1:
            kf = 8 if field == 8 or subfield else 16  # every codec here has <= 256 shards
            assert last_kernel().startswith(f"bitslice-wide gf{kf} {k}+{p}"), last_kernel()
            if kf == 8 and p > 48:  # RSE_OPT_WIDE_SPLIT auto: 4 outputs per wave
                assert " w16 " in last_kernel(), last_kernel()
        for i in range(p):
            assert (host(t[k + i]).reshape(-1) == full[k + i]).all(), i
        assert r.verify(t)
        t[k + p - 1].view(-1)[20000] ^= 1  # in a bit-sliced chunk
        assert not r.verify(t)
        t[k + p - 1].view(-1)[20000] ^= 1
        t[k - 1].view(-1)[nbytes - 1] ^= 0x80  # in the table-coded tail
        assert not r.verify(t)
        t[k - 1].view(-1)[nbytes - 1] ^= 0x80
        stripes = 3
        flat = torch.full((stripes, k + p, nbytes), 0xA5, dtype=torch.uint8, device="cuda")
        for s_ in range(stripes):
            for i in range(k):
                flat[s_, i] = dev(np.roll(full[i], s_))
        r.encode_flat(flat, n_elems, stripes)
        torch.cuda.synchronize()
        got = host(flat)
        for s_ in range(stripes):
            sh = [np.roll(full[i], s_) for i in range(k)] + \
                 [np.zeros(nbytes, np.uint8) for _ in range(p)]
            oc.encode(sh)
            for i in range(p):
                assert (got[s_, k + i] == sh[k + i]).all(), (s_, i)
    finally:
        lib.rse_set_option(9, old)
        lib.rse_set_option(51, old51)


@pytest.mark.parametrize("k,p,lim,modules", [(20, 70, 128, 2), (40, 70, 16, 6), (128, 128, 128, 2)])
def test_wide_output_groups(R, k, p, lim, modules):
    """Past one wide module's 64 outputs (round 6): the outputs split into
    balanced groups of <= 64, each coded over every input by one wide module
    (20+70: two of 20 x 35; GF(2^8)'s widest, 128+128: two of 128 x 64), or --
    past RSE_OPT_WIDE_BLOCK_INPUTS inputs (here 16) -- by a chain over input
    blocks writing the group's outputs at their offset (40+70: two chains of
    three).  Encode (one launch per module), verify, a 3-stripe encode_flat,
    and a first-use reconstruct of more than 64 lost shards, against the
    oracle."""
    lib = R._lib.load()
    field, nbytes = 8, 16384 + 4096 + 48
    rng = np.random.default_rng(k * 1000 + p)
    oc = O.Codec(field, k, p)
    full = rand_shards(rng, k, nbytes) + [np.zeros(nbytes, np.uint8) for _ in range(p)]
    oc.encode(full)
    old = [lib.rse_get_option(x) for x in (9, 46)]
    try:
        assert lib.rse_set_option(9, 2) == 0
        assert lib.rse_set_option(46, lim) == 0
        r = R.core.ReedSolomon(k, p, field)
        assert r.kernel_kind(wait=True) == "bitslice-specialised"
        t = [dev(x) for x in full[:k]] + [torch.full((nbytes,), 0x5A, dtype=torch.uint8,
                                                     device="cuda") for _ in range(p)]
        n0 = lib.rse_get_option(6)
        r.encode(t)
        torch.cuda.synchronize()
        from reed_solomon_erasure.core import last_kernel
        assert lib.rse_get_option(6) - n0 == modules, last_kernel()
        assert last_kernel().startswith(f"bitslice-wide-groups gf8 {k}+{p} g2"), last_kernel()
        for i in range(p):
            assert (host(t[k + i]) == full[k + i]).all(), i
        assert r.verify(t)
        t[k + p - 1][9000] ^= 1
        assert not r.verify(t)
        t[k + p - 1][9000] ^= 1
        stripes = 3
        flat = torch.full((stripes, k + p, nbytes), 0xA5, dtype=torch.uint8, device="cuda")
        for s_ in range(stripes):
            for i in range(k):
                flat[s_, i] = dev(np.roll(full[i], s_))
        r.encode_flat(flat, nbytes, stripes)
        got = host(flat)
        for s_ in range(stripes):
            sh = [np.roll(full[i], s_) for i in range(k)] + [np.zeros(nbytes, np.uint8)
                                                              for _ in range(p)]
            oc.encode(sh)
            for i in range(p):
                assert (got[s_, k + i] == sh[k + i]).all(), (s_, i)
        # more than 64 shards lost, first use of the pattern (RSE_OPT_JIT 1:
        # syndrome / table kernels, no decode-pattern build)
        assert lib.rse_set_option(9, 1) == 0
        lost = sorted(rng.choice(k + p, p, replace=False).tolist())
        for i in lost:
            t[i].fill_(0)
        r.reconstruct([(x, i not in lost) for i, x in enumerate(t)])
        for i in range(k + p):
            assert (host(t[i]) == full[i]).all(), (i, i in lost)
    finally:
        lib.rse_set_option(9, old[0])
        lib.rse_set_option(46, old[1])


@pytest.mark.parametrize("lim,label", [(128, "x8 (125+24"), (400, "x3 (334+24")])
def test_wide_block_chain_gf16_past_256(R, lim, label):
    """GF(2^16) 1000+24 (k + 2p > 480: too wide for one wide module's pointer
    block) on a chain of wide modules over input blocks (rse_jit.cpp;
    RSE_OPT_WIDE_BLOCK_INPUTS 128: 8 blocks of 125 data shards), each coding
    all 24 outputs, the blocks after the first reading the sums so far as 24
    more inputs.  Encode (whole 4 KiB chunks on the chain, a table-coded tail),
    verify (sums materialised through the chain, then compared) and a
    2-stripe encode_flat against the oracle; also on 3 blocks of 333-334
    inputs (RSE_OPT_WIDE_BLOCK_INPUTS 400).  The modules come from the tree's
    jitcache (tools/prebuild_all.sh builds the default chain's; the 400-input
    ones, ~145 minutes of hiprtc, were built by hand: without them that case
    skips)."""
    lib = R._lib.load()
    k, p = 1000, 24
    nbytes = 2 * 4096 + 96
    n_elems = nbytes // 2
    rng = np.random.default_rng(1024)
    oc = O.Codec.shared(16, k, p)
    full = rand_shards(rng, k, nbytes) + [np.zeros(nbytes, np.uint8) for _ in range(p)]
    oc.encode(full)
    old = lib.rse_get_option(9)
    old46 = lib.rse_get_option(46)
    try:
        assert lib.rse_set_option(9, 2) == 0
        assert lib.rse_set_option(46, lim) == 0  # data inputs per chain block
        r = R.core.ReedSolomon(k, p, 16)
        assert kernels_or_skip(r, f"GF(2^16) 1000+24, blocks of <= {lim}") == \
            "bitslice-specialised"
        t = [dev(x).reshape(n_elems, 2) for x in full[:k]] + \
            [torch.full((n_elems, 2), 0x5A, dtype=torch.uint8, device="cuda") for _ in range(p)]
        n0 = lib.rse_get_option(6)
        r.encode(t)
        torch.cuda.synchronize()
        assert lib.rse_get_option(6) - n0 == int(label[1])
        from reed_solomon_erasure.core import last_kernel
        assert last_kernel().startswith(f"bitslice-wide-blocks gf16 1000+24 {label}"), last_kernel()
        for i in range(p):
            assert (host(t[k + i]).reshape(-1) == full[k + i]).all(), i
        assert r.verify(t)
        t[k + p - 1].view(-1)[5000] ^= 1  # in a chain-coded chunk
        assert not r.verify(t)
        t[k + p - 1].view(-1)[5000] ^= 1
        t[k - 1].view(-1)[nbytes - 1] ^= 0x80  # in the table-coded tail
        assert not r.verify(t)
        t[k - 1].view(-1)[nbytes - 1] ^= 0x80
        stripes = 2
        flat = torch.full((stripes, k + p, nbytes), 0xA5, dtype=torch.uint8, device="cuda")
        for s_ in range(stripes):
            flat[s_, :k] = dev(np.stack([np.roll(full[i], 7 * s_) for i in range(k)]))
        r.encode_flat(flat, n_elems, stripes)
        torch.cuda.synchronize()
        got = host(flat)
        for s_ in range(stripes):
            sh = [np.roll(full[i], 7 * s_) for i in range(k)] + \
                 [np.zeros(nbytes, np.uint8) for _ in range(p)]
            oc.encode(sh)
            for i in range(p):
                assert (got[s_, k + i] == sh[k + i]).all(), (s_, i)
    finally:
        lib.rse_set_option(9, old)
        lib.rse_set_option(46, old46)


@pytest.mark.parametrize("nbytes,stripes", [(1024, 5), (1024, 8), (2048, 3)])
def test_wide_block_chain_gf16_short_shards(R, nbytes, stripes):
    """The 1000+24 chain on 1 and 2 KiB shards: a wave's chunk
    then takes 4 (2) consecutive stripes, and the blocks after the first read
    and rewrite the running sums of every stripe of the chunk in place -- over
    stripe counts that are (not) a multiple of the stripes per chunk, every
    stripe against the oracle, and a guard stripe after the batch untouched."""
    lib = R._lib.load()
    k, p = 1000, 24
    n_elems = nbytes // 2
    T = k + p
    rng = np.random.default_rng(nbytes + stripes)
    oc = O.Codec.shared(16, k, p)
    old = lib.rse_get_option(9)
    try:
        assert lib.rse_set_option(9, 2) == 0
        r = R.core.ReedSolomon(k, p, 16)
        assert kernels_or_skip(r, "GF(2^16) 1000+24, blocks of <= 128") == \
            "bitslice-specialised"
        buf = rng.integers(0, 256, (stripes + 1) * T * nbytes, dtype=np.uint8)
        d = dev(buf)
        n0 = lib.rse_get_option(6)
        r.encode_flat(d, n_elems, stripes)
        torch.cuda.synchronize()
        from reed_solomon_erasure.core import last_kernel
        assert lib.rse_get_option(6) - n0 == 8, last_kernel()
        assert last_kernel().startswith("bitslice-wide-blocks gf16 1000+24 x8"), last_kernel()
        got = host(d).reshape(stripes + 1, T, nbytes)
        ref = buf.reshape(stripes + 1, T, nbytes)
        assert (got[stripes] == ref[stripes]).all()  # guard stripe
        assert (got[:stripes, :k] == ref[:stripes, :k]).all()
        for s_ in range(stripes):
            sh = [ref[s_, i].copy() for i in range(k)] + [np.zeros(nbytes, np.uint8)
                                                          for _ in range(p)]
            oc.encode(sh)
            for i in range(p):
                assert (got[s_, k + i] == sh[k + i]).all(), (s_, i)
        ok = r.verify_flat(d, n_elems, stripes)
        assert ok.all()
        v = got.copy()
        v[stripes - 1, k + 3, nbytes // 2] ^= 0x10
        want = np.arange(stripes) != stripes - 1
        assert (r.verify_flat(dev(v.reshape(-1)), n_elems, stripes) == want).all()
    finally:
        lib.rse_set_option(9, old)


@pytest.mark.parametrize("field,k,p,erased", [(8, 40, 2, [3, 39]), (8, 6, 10, [0, 1, 2, 5, 6, 8, 9, 12, 15]),
                                              (16, 36, 3, [0, 35, 37])])
def test_wide_reconstruct_pattern_blocks(R, field, k, p, erased):
    """A wide codec's repeated erasure pattern (RSE_OPT_JIT 2: the first use)
    gets block kernels for its composed decode rows; reconstruct and
    reconstruct_data_flat then run them (pattern-launch counter) and match the
    oracle."""
    lib = R._lib.load()
    es = field // 8
    nbytes = 16384 + 4096 + 32 * es
    n_elems = nbytes // es
    shape = (n_elems,) if field == 8 else (n_elems, 2)
    rng = np.random.default_rng(field * 7 + k * 3 + p)
    oc = O.Codec(field, k, p)
    full = rand_shards(rng, k, nbytes) + [np.zeros(nbytes, np.uint8) for _ in range(p)]
    oc.encode(full)
    present = [i not in erased for i in range(k + p)]
    old = lib.rse_get_option(9)
    try:
        assert lib.rse_set_option(9, 2) == 0
        r = R.core.ReedSolomon(k, p, field)
        tb = [dev(x).reshape(shape) for x in full]
        for e in erased:
            tb[e].fill_(0x33)
        n0 = lib.rse_get_option(12)
        r.reconstruct(list(zip(tb, present)))
        torch.cuda.synchronize()
        assert lib.rse_get_option(12) - n0 == 1
        for i in range(k + p):
            assert (host(tb[i]).reshape(-1) == full[i]).all(), i
        stripes = 2
        flat = torch.empty((stripes, k + p, nbytes), dtype=torch.uint8, device="cuda")
        for s_ in range(stripes):
            for i in range(k + p):
                flat[s_, i] = dev(full[i]) if present[i] else 0x77
        n0 = lib.rse_get_option(12)
        r.reconstruct_data_flat(flat, n_elems, stripes, present)
        torch.cuda.synchronize()
        if any(e < k for e in erased):
            assert lib.rse_get_option(12) - n0 == 1
        got = host(flat)
        for s_ in range(stripes):
            for i in range(k):
                assert (got[s_, i] == full[i]).all(), (s_, i)
    finally:
        lib.rse_set_option(9, old)


@pytest.mark.parametrize("k,p", [(12, 4), (6, 3)])
def test_jit_verify_completion_word(R, k, p):
    """verify() of a run-time specialised codec (rse_jit.cpp rse_jit_check)
    returns through the kernel's completion word like the compiled codecs':
    whole 16 KiB chunks only, so one check launch is the whole call.  Clean
    stripes verify, and a byte flipped anywhere -- first or last chunk, data
    or parity -- is caught (a kernel that signalled before every verdict store
    landed would miss some)."""
    from reed_solomon_erasure.core import last_kernel
    lib = R._lib.load()
    old = lib.rse_get_option(9)
    lib.rse_set_option(9, 2)  # wait for the codec's module
    try:
        rng = np.random.default_rng(4242 + k)
        n = 16384 * 37
        full = rand_shards(rng, k, n) + [np.zeros(n, np.uint8) for _ in range(p)]
        O.Codec(8, k, p).encode(full)
        r = R.galois_8.ReedSolomon(k, p)
        shards = [dev(x) for x in full]
        for _ in range(3):
            assert r.verify(shards)
        assert last_kernel().startswith(f"bitslice-jit gf8 {k}+{p}"), last_kernel()
        for shard, off in [(0, 0), (k - 1, n - 1), (k, 5), (k + p - 1, n - 16384), (k // 2, n // 2)]:
            t = shards[shard]
            t[off] ^= 0x81
            assert not r.verify(shards), (shard, off)
            t[off] ^= 0x81
            assert r.verify(shards)
    finally:
        lib.rse_set_option(9, old)


@pytest.mark.parametrize("depth,field,k,p", [(1, 8, 7, 3), (2, 8, 6, 5), (3, 16, 9, 2)])
def test_sub_chunk_depth_option(R, depth, field, k, p):
    """RSE_OPT_SUB_DEPTH: the narrow modules' 1 / 2 KiB kernels with 1 input in
    flight per wave (bitslice_body, round 4's kernels) or 2 / 3 (rse_sub_ext.hpp;
    the default 4 runs in test_sub_chunk_shards): the same checks.  Codecs no
    other test builds (modules are keyed by rows, not options)."""
    lib = R._lib.load()
    old = lib.rse_get_option(50)
    try:
        assert lib.rse_set_option(50, depth) == 0
        for kib in (1, 2):
            test_sub_chunk_shards(R, field, k, p, kib)
    finally:
        lib.rse_set_option(50, old)


@pytest.mark.parametrize("field,k,p", [
    (8, 10, 4), (8, 10, 2), (16, 20, 8),   # compiled codecs
    (8, 4, 4), (8, 8, 8), (8, 5, 2), (16, 6, 3),  # run-time specialised
    (8, 50, 20), (8, 16, 16), (16, 40, 12),  # wide codecs (one module, LDS bodies)
    (8, 32, 32), (8, 64, 64),                # wide, half chunks, 8 outputs per wave
    (8, 40, 2),                              # wide, one wave (plain body)
])
@pytest.mark.parametrize("kib", [1, 2])
def test_sub_chunk_shards(R, field, k, p, kib):
    """RSE_OPT_SUB_CHUNKS: shards of exactly 1 or 2 KiB (benches/bandwidth.rs:
    88-190's blocks) on the bit-sliced kernels, 4 or 2 stripes per 4 KiB chunk.
    Ragged stripe counts (the last chunk's lanes past the last stripe load and
    store nothing: a guard stripe after the batch stays as it was), parity
    against the oracle stripe by stripe and against the table kernels
    (option 33 = 0), verify_flat's per-stripe verdicts from the lanes of
    shared chunks, and reconstruct_data_flat."""
    from reed_solomon_erasure.core import last_kernel
    lib = R._lib.load()
    es = field // 8
    nb = kib * 1024
    n = nb // es
    T = k + p
    oc = O.Codec(field, k, p)
    old9, old33, old51 = lib.rse_get_option(9), lib.rse_get_option(33), lib.rse_get_option(51)
    try:
        lib.rse_set_option(9, 2)  # run-time builds waited for
        lib.rse_set_option(51, 0)  # 16+16 .. 64+64: the wide modules, not the FFT kernels
        r = R.core.ReedSolomon(k, p, field)
        assert r.kernel_kind(wait=True).startswith("bitslice")
        for stripes in (1, 3, 6, 1001):
            rng = np.random.default_rng(stripes * 7 + k + p + kib + field)
            buf = rng.integers(0, 256, (stripes + 1) * T * nb, dtype=np.uint8)
            d = dev(buf)
            r.encode_flat(d, n, stripes)
            kern = last_kernel()
            assert f"sub{kib}" in kern and kern.startswith("bitslice"), kern
            got = host(d).reshape(stripes + 1, T, nb)
            assert (got[stripes] == buf.reshape(stripes + 1, T, nb)[stripes]).all()  # guard
            assert (got[:, :k] == buf.reshape(stripes + 1, T, nb)[:, :k]).all()
            for s_ in sorted(x for x in {0, 1, stripes // 2, stripes - 2, stripes - 1}
                             if 0 <= x < stripes):
                want = [got[s_, i].copy() for i in range(k)] + [np.zeros(nb, np.uint8)
                                                               for _ in range(p)]
                oc.encode(want)
                for i in range(p):
                    assert (got[s_, k + i] == want[k + i]).all(), (stripes, s_, i, kern)
            # the table kernels write the same bytes
            lib.rse_set_option(33, 0)
            d2 = dev(buf)
            r.encode_flat(d2, n, stripes)
            assert "sub" not in last_kernel(), last_kernel()
            assert (host(d2) == host(d)).all()
            lib.rse_set_option(33, 1)
            # per-stripe verdicts from lanes that share chunks
            good = host(d)
            v = good.reshape(stripes + 1, T, nb).copy()
            want_ok = np.ones(stripes, bool)
            for s_ in sorted({stripes - 1, stripes // 3}):
                v[s_, int(rng.integers(0, T)), int(rng.integers(0, nb))] ^= 0x5A
                want_ok[s_] = False
            dv = dev(v.reshape(-1))
            assert (r.verify_flat(dv, n, stripes) == want_ok).all()
            assert r.verify_flat(d, n, stripes).all()
            # rebuild two lost data shards of every stripe
            lost = [1, k - 1] if k > 2 else [0]
            dd = d.view(stripes + 1, T, nb)
            for e in lost:
                dd[:stripes, e].fill_(0)
            r.reconstruct_data_flat(d, n, stripes, [i not in lost for i in range(T)])
            assert (host(d) == good).all()
    finally:
        lib.rse_set_option(9, old9)
        lib.rse_set_option(33, old33)
        lib.rse_set_option(51, old51)


def test_wide_launch_follows_the_module_not_the_options(R):
    """A wide module's workgroup shape is fixed when it is generated
    (RSE_OPT_WIDE_SPLIT: outputs per wave); changing the option afterwards
    must not change the launch (a 512-lane launch of a 256-lane module fails
    to launch).  GF(2^8) 3+30: 4 waves by default, 8 at 4 outputs per wave."""
    from reed_solomon_erasure.core import last_kernel
    lib = R._lib.load()
    k, p, n = 3, 30, 3 * 4096 + 16
    rng = np.random.default_rng(330)
    oc = O.Codec(8, k, p)
    full = rand_shards(rng, k, n) + [np.zeros(n, np.uint8) for _ in range(p)]
    oc.encode(full)
    old9, old18 = lib.rse_get_option(9), lib.rse_get_option(18)
    try:
        lib.rse_set_option(9, 2)
        r = R.core.ReedSolomon(k, p, 8)
        assert r.kernel_kind(wait=True) == "bitslice-specialised"
        lib.rse_set_option(18, 4)
        t = [dev(x) for x in full[:k]] + [torch.zeros(n, dtype=torch.uint8, device="cuda")
                                          for _ in range(p)]
        r.encode(t)
        torch.cuda.synchronize()
        assert last_kernel().startswith("bitslice-wide gf8 3+30 w4"), last_kernel()
        for i in range(p):
            assert (host(t[k + i]) == full[k + i]).all(), i
    finally:
        lib.rse_set_option(9, old9)
        lib.rse_set_option(18, old18)


@pytest.mark.parametrize("field,k,p", [(8, 10, 4), (16, 20, 8), (8, 6, 3)])
@pytest.mark.parametrize("nbytes", [4096, 8192 + 32, 12288])
def test_pattern_kernels_below_16_kib(R, field, k, p, nbytes):
    """Shards of 4 to 16 KiB: the syndrome kernels take 16 KiB chunks only, so
    a repeated pattern gets its own kernel (4 KiB chunks, one per wave) here
    too (RSE_OPT_JIT 2: built on first use); reconstruct, reconstruct_data
    and the flat form against the oracle, each a pattern launch."""
    lib = R._lib.load()
    es = field // 8
    n_elems = nbytes // es
    shape = (n_elems,) if field == 8 else (n_elems, 2)
    rng = np.random.default_rng(nbytes + k + field)
    oc = O.Codec(field, k, p)
    full = rand_shards(rng, k, nbytes) + [np.zeros(nbytes, np.uint8) for _ in range(p)]
    oc.encode(full)
    erased = [0, k - 1] + ([k] if p > 2 else [])
    present = [i not in erased for i in range(k + p)]
    old = lib.rse_get_option(9)
    try:
        lib.rse_set_option(9, 2)
        r = R.core.ReedSolomon(k, p, field)
        for data_only in (False, True):
            tb = [dev(x).reshape(shape) for x in full]
            for e in erased:
                tb[e].fill_(0x6B)
            n0 = lib.rse_get_option(12)
            (r.reconstruct_data if data_only else r.reconstruct)(list(zip(tb, present)))
            torch.cuda.synchronize()
            assert lib.rse_get_option(12) - n0 == 1, data_only
            for i in range(k + p):
                got = host(tb[i]).reshape(-1)
                if data_only and i >= k and i in erased:
                    assert (got == 0x6B).all()
                else:
                    assert (got == full[i]).all(), (data_only, i)
        stripes = 5
        buf = np.concatenate([np.concatenate(full)] * stripes)
        d = dev(buf)
        v = d.view(stripes, k + p, nbytes)
        for e in erased:
            v[:, e].fill_(0)
        n0 = lib.rse_get_option(12)
        r.reconstruct_data_flat(d, n_elems, stripes, present)
        torch.cuda.synchronize()
        assert lib.rse_get_option(12) - n0 == 1
        got = host(d).reshape(stripes, k + p, nbytes)
        for s_ in range(stripes):
            for i in range(k):
                assert (got[s_, i] == full[i]).all(), (s_, i)
    finally:
        lib.rse_set_option(9, old)


@pytest.mark.parametrize("field,k,p", [(8, 10, 4), (16, 20, 8), (8, 6, 3)])
@pytest.mark.parametrize("nbytes", [4096, 8192 + 32, 16384 + 4096 + 48, 2 * 16384 + 3 * 4096])
@SUBFIELD
def test_syndrome_reconstruct_4k_chunks(R, subfield, field, k, p, nbytes):
    """First use of a pattern (no decode-pattern kernels) on shards with whole
    4 KiB chunks past their 16 KiB ones, or shorter than 16 KiB: the syndrome
    reconstruct codes those chunks too (one wave each, Horner mixing), the
    table kernels only the sub-4 KiB tail.  Every erasure count, data and
    parity, reconstruct and reconstruct_data, one stripe and flat stripes,
    against the oracle."""
    from reed_solomon_erasure.core import last_kernel
    lib = R._lib.load()
    es = field // 8
    n_elems = nbytes // es
    shape = (n_elems,) if field == 8 else (n_elems, 2)
    rng = np.random.default_rng(nbytes * 3 + k + p + field)
    oc = O.Codec(field, k, p)
    full = rand_shards(rng, k, nbytes) + [np.zeros(nbytes, np.uint8) for _ in range(p)]
    oc.encode(full)
    patterns = [sorted(rng.choice(k + p, ne, replace=False).tolist()) for ne in range(1, p + 1)]
    patterns += [list(range(min(p, k)))]
    old9, old11, old37 = lib.rse_get_option(9), lib.rse_get_option(11), lib.rse_get_option(37)
    try:
        lib.rse_set_option(9, 2)   # run-time codecs built before the first call
        lib.rse_set_option(11, 0)  # no decode-pattern kernels: the syndrome path
        lib.rse_set_option(37, 0)  # 4 KiB syndrome chunks at any size of pattern
        r = R.core.ReedSolomon(k, p, field)
        r.kernel_kind(wait=True)
        for erased in patterns:
            present = [i not in erased for i in range(k + p)]
            for data_only in (False, True):
                if data_only and all(e >= k for e in erased):
                    continue
                tb = [dev(x).reshape(shape) for x in full]
                for e in erased:
                    tb[e].fill_(0x3C)
                n0 = lib.rse_get_option(6)
                (r.reconstruct_data if data_only else r.reconstruct)(list(zip(tb, present)))
                torch.cuda.synchronize()
                assert lib.rse_get_option(6) - n0 == 1, (erased, data_only)
                if nbytes < 16384 and nbytes % 4096 == 0:  # (a tail: the table kernel's name)
                    assert "w4" in last_kernel(), last_kernel()
                for i in range(k + p):
                    got = host(tb[i]).reshape(-1)
                    if data_only and i >= k and i in erased:
                        assert (got == 0x3C).all()
                    else:
                        assert (got == full[i]).all(), (erased, data_only, i)
        stripes = 3
        erased = patterns[min(2, len(patterns) - 1)]
        buf = np.concatenate([np.concatenate(full)] * stripes)
        d = dev(buf)
        v = d.view(stripes, k + p, nbytes)
        for e in erased:
            v[:, e].fill_(0)
        r.reconstruct_data_flat(d, n_elems, stripes, [i not in erased for i in range(k + p)])
        got = host(d).reshape(stripes, k + p, nbytes)
        for s_ in range(stripes):
            for i in range(k):
                assert (got[s_, i] == full[i]).all(), (s_, i)
        # the default threshold: a small pattern of a short shard stays on the
        # table kernels (k x outputs < 64), a large one takes the 4 KiB chunks
        lib.rse_set_option(37, old37)
        if nbytes == 4096 and (field == 8 or subfield):
            for erased, w4 in (([0], k * 1 >= 64), (list(range(p)), k * p >= 64)):
                tb = [dev(x).reshape(shape) for x in full]
                r.reconstruct(list(zip(tb, [i not in erased for i in range(k + p)])))
                torch.cuda.synchronize()
                # (not the launch count: another test's decode-pattern module for
                # the same rows may serve the table-kernel route bit-sliced)
                assert ("-recon " in last_kernel()) == w4, (erased, last_kernel())
    finally:
        lib.rse_set_option(9, old9)
        lib.rse_set_option(11, old11)
        lib.rse_set_option(37, old37)
