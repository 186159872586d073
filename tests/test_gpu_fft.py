"""The additive-FFT kernels (rse_fft.hip) of GF(2^8) codecs with k = p = 16, 32
and 64 -- the reference bench's 16+16 .. 64+64 (benches/bandwidth.rs:88-190)
-- against the oracle's coefficient-matrix encode and reconstruct
(core.rs:481-509, 680-923), and against the library's own coefficient-network
path (RSE_OPT_FFT 0) on the same bytes.

Covered: encode of 1 KiB shards (two stripes per 2 KiB column, odd stripe
counts, a guard stripe after the batch), whole 2 KiB columns, shards with a
tail past the last column (coded by the other kernels), per-shard encode,
verify and verify_flat (a corrupted byte in a data or a parity shard, per
stripe), and every data shard rebuilt from the parity shards
(reconstruct_data_flat / reconstruct / reconstruct_data)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import oracle as O  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def R():
    import reed_solomon_erasure as R
    return R


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint8)).cuda()


def host(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


LENS = [1024, 2048, 4096, 6144, 2048 + 48, 10240 + 16]


@pytest.mark.parametrize("k", [16, 32, 64])
@pytest.mark.parametrize("nb", LENS)
def test_fft_encode_verify_rebuild(R, k, nb):
    from reed_solomon_erasure.core import last_kernel
    lib = R._lib.load()
    p, T = k, 2 * k
    oc = O.Codec(8, k, p)
    r = R.galois_8.ReedSolomon(k, p)
    stripes_list = (1, 3) if nb > 2048 else (1, 3, 7)
    for stripes in stripes_list:
        rng = np.random.default_rng(k * 1000 + nb + stripes)
        buf = rng.integers(0, 256, (stripes + 1) * T * nb, dtype=np.uint8)
        d = dev(buf)
        r.encode_flat(d, nb, stripes)
        kern = last_kernel()
        assert kern.startswith(f"fft gf8 {k}+{k} code"), kern
        got = host(d).reshape(stripes + 1, T, nb)
        ref = buf.reshape(stripes + 1, T, nb)
        assert (got[stripes] == ref[stripes]).all()  # guard stripe untouched
        assert (got[:, :k] == ref[:, :k]).all()
        for s_ in sorted({0, stripes // 2, stripes - 1}):
            want = [got[s_, i].copy() for i in range(k)] + [np.zeros(nb, np.uint8)
                                                           for _ in range(p)]
            oc.encode(want)
            for i in range(p):
                assert (got[s_, k + i] == want[k + i]).all(), (stripes, s_, i)
        # the coefficient-network path writes the same bytes
        old = lib.rse_get_option(51)
        lib.rse_set_option(51, 0)
        try:
            d2 = dev(buf)
            r.encode_flat(d2, nb, stripes)
            assert not last_kernel().startswith("fft"), last_kernel()
            assert (host(d2) == host(d)).all()
        finally:
            lib.rse_set_option(51, old)
        # per-stripe verdicts
        good = host(d)
        v = good.reshape(stripes + 1, T, nb).copy()
        want_ok = np.ones(stripes, bool)
        bad = {stripes - 1: k + int(rng.integers(0, p))}  # a parity byte
        if stripes > 1:
            bad[0] = int(rng.integers(0, k))  # a data byte
        for s_, i in bad.items():
            v[s_, i, int(rng.integers(0, nb))] ^= 0x5A
            want_ok[s_] = False
        dv = dev(v.reshape(-1))
        assert (r.verify_flat(dv, nb, stripes) == want_ok).all()
        assert last_kernel().startswith(f"fft gf8 {k}+{k} check"), last_kernel()
        assert r.verify_flat(d, nb, stripes).all()
        # every data shard rebuilt from the parity shards
        dd = d.view(stripes + 1, T, nb)
        dd[:stripes, :k].fill_(0xA5)
        r.reconstruct_data_flat(d, nb, stripes, [i >= k for i in range(T)])
        assert last_kernel().startswith(f"fft gf8 {k}+{k} code"), last_kernel()
        assert (host(d) == good).all()


@pytest.mark.parametrize("k", [16, 32, 64])
def test_fft_per_shard_calls(R, k):
    """The per-shard API (separate allocations): encode, verify, and
    reconstruct / reconstruct_data with every data shard lost, against the
    oracle."""
    from reed_solomon_erasure.core import last_kernel
    p, nb = k, 4096 + 2048
    rng = np.random.default_rng(k)
    data = [rng.integers(0, 256, nb, dtype=np.uint8) for _ in range(k)]
    want = [x.copy() for x in data] + [np.zeros(nb, np.uint8) for _ in range(p)]
    O.Codec(8, k, p).encode(want)
    r = R.galois_8.ReedSolomon(k, p)
    sh = [dev(x) for x in data] + [torch.zeros(nb, dtype=torch.uint8, device="cuda")
                                   for _ in range(p)]
    r.encode(sh)
    assert last_kernel().startswith("fft"), last_kernel()
    for i in range(k + p):
        assert (host(sh[i]) == want[i]).all(), i
    assert r.verify(sh)
    sh[k + 3][77] ^= 1
    assert not r.verify(sh)
    sh[k + 3][77] ^= 1
    for data_only in (True, False):
        for i in range(k):
            sh[i].fill_(0)
        pairs = [(s, i >= k) for i, s in enumerate(sh)]
        if data_only:
            r.reconstruct_data(pairs)
        else:
            r.reconstruct(pairs)
        assert last_kernel().startswith("fft"), last_kernel()
        for i in range(k + p):
            assert (host(sh[i]) == want[i]).all(), (data_only, i)


def test_fft_not_for_other_shapes(R):
    """Codecs that are not k = p = 16 / 32 / 64, and other decode patterns,
    keep their kernels (one data shard lost on 32+32)."""
    from reed_solomon_erasure.core import last_kernel
    k, nb, stripes = 32, 2048, 5
    T = 2 * k
    rng = np.random.default_rng(5)
    buf = rng.integers(0, 256, stripes * T * nb, dtype=np.uint8)
    r = R.galois_8.ReedSolomon(k, k)
    d = dev(buf)
    r.encode_flat(d, nb, stripes)
    good = host(d)
    dd = d.view(stripes, T, nb)
    dd[:, 7].fill_(0)
    r.reconstruct_data_flat(d, nb, stripes, [i != 7 for i in range(T)])
    assert not last_kernel().startswith("fft"), last_kernel()
    assert (host(d) == good).all()
    r2 = R.galois_8.ReedSolomon(32, 16)
    s2 = [torch.zeros(nb, dtype=torch.uint8, device="cuda") for _ in range(48)]
    r2.encode(s2)
    assert not last_kernel().startswith("fft"), last_kernel()


@pytest.mark.parametrize("k", [16, 32, 64])
def test_fft_gf16_subfield_codecs(R, k):
    """GF(2^16) codecs of at most 256 shards code in the GF(2^8) subfield
    (DESIGN §4), so GF(2^16) 16+16 .. 64+64 take the same FFT kernels: encode
    of 2 KiB columns and a ragged tail, verify, and every data shard rebuilt,
    against the GF(2^16) oracle."""
    from reed_solomon_erasure.core import last_kernel
    p, n_elems, stripes = k, 2048 + 24, 3
    nb, T = 2 * n_elems, 2 * k
    oc = O.Codec(16, k, p)
    rng = np.random.default_rng(160 + k)
    full = np.zeros((stripes, T, nb), np.uint8)
    for s_ in range(stripes):
        sh = [rng.integers(0, 256, nb, dtype=np.uint8) for _ in range(k)] + \
             [np.zeros(nb, np.uint8) for _ in range(p)]
        oc.encode(sh)
        full[s_] = np.stack(sh)
    r = R.galois_16.ReedSolomon(k, p)
    assert r.kernel_kind() == "fft-compiled"
    buf = full.copy()
    buf[:, k:] = 0x69
    d = dev(buf.reshape(-1))
    r.encode_flat(d, n_elems, stripes)
    assert last_kernel().startswith(f"fft gf8 {k}+{k} code") or \
        not last_kernel().startswith("fft"), last_kernel()  # the tail ran last
    assert (host(d).reshape(stripes, T, nb) == full).all()
    assert r.verify_flat(d, n_elems, stripes).all()
    d.view(stripes, T, nb)[:, :k].fill_(0)
    r.reconstruct_data_flat(d, n_elems, stripes, [i >= k for i in range(T)])
    assert (host(d).reshape(stripes, T, nb) == full).all()
