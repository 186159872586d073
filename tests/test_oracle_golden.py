"""Pin the CPU oracle (oracle/rse_oracle.c) before trusting it as the checker.

Every known answer the reference's own tests hold for the hot path is checked
here (file:line in tests/golden/make_golden.py), plus agreement with the
reference's own compiled SIMD kernel (oracle/_ref, built from
/root/reference/simd_c/reedsolomon.c) on every tail length.  CPU only.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))
KAT = GOLDEN["reference_kats"]
GEN = GOLDEN["generated"]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def u8(x):
    return np.array(x, dtype=np.uint8)


# ------------------------------------------------------------ GF(2^8)
def test_log_table_same_as_backblaze():  # galois_8.rs:339-363
    log, exp, mul, low, high = O.gf8_tables()
    assert log.tolist() == KAT["log_table"]


def test_galois_kats():  # galois_8.rs:482-552
    for a, b, r in KAT["mul"]:
        assert O.gf8_mul(a, b) == r
    for a, n, r in KAT["exp"]:
        assert O.gf8_exp(a, n) == r
    inp = u8(KAT["mul_slice_input"])
    out = np.zeros_like(inp)
    for c, xor, expect in KAT["mul_slice_steps"]:
        O.gf8_mul_slice(c, inp, out, xor=xor)
        assert out.tolist() == expect


def test_mul_table_is_field_multiplication_mod_0x11d():
    """The LOG/EXP tables (build.rs:13-94) tabulate polynomial multiplication
    modulo 0x11D -- the algebra the device kernels evaluate with xtime chains."""
    _, _, mul, low, high = O.gf8_tables()

    def pmul(a, b):
        r = 0
        for i in range(8):
            if b >> i & 1:
                r ^= a << i
        for i in range(15, 7, -1):
            if r >> i & 1:
                r ^= 0x11D << (i - 8)
        return r

    a = np.arange(256)
    for b in range(256):
        assert mul[:, b].tolist() == [pmul(int(x), b) for x in a]
    for c in range(256):  # gen_mul_table_half (build.rs:71-94)
        assert low[c].tolist() == [mul[c, n] for n in range(16)]
        assert high[c].tolist() == [mul[c, n << 4] for n in range(16)]


def test_gf8_field_identities():  # galois_8.rs:392-424 test_identity, :466-479 test_exp
    for a in range(1, 256):
        assert O.gf8_mul(a, O.gf8_div(1, a)) == 1
    for a in range(256):
        power = 1
        for j in range(256):
            assert O.gf8_exp(a, j) == power
            power = O.gf8_mul(power, a)


# ------------------------------------------------------------ GF(2^16)
def test_gf16_sage_vectors():  # sage/galois_ext_test.sage:10-26
    s = KAT["gf16_sage"]
    e1, e2 = tuple(s["e1"]), tuple(s["e2"])
    assert O.gf16_add(e1, e2) == tuple(s["sum"])
    assert O.gf16_mul(e1, e2) == tuple(s["product"])
    assert O.gf16_div(e1, e2) == tuple(s["quotient"])
    assert O.gf16_inverse((1, 0)) == tuple(s["inv_b"])


def test_gf16_inverse_is_field_inverse_for_every_element():
    """galois_16.rs:285-315's extended Euclid agrees with the unique field
    inverse on all 65535 nonzero elements, so any correct inversion (the
    product's a^(2^16-2)) reproduces the reference byte for byte."""
    for a in range(1, 65536):
        e = (a >> 8, a & 0xFF)
        assert O.gf16_mul(e, O.gf16_inverse(e)) == (0, 1)


def test_gf16_exp_zero_is_one():  # galois_16.rs:405-409
    assert O.gf16_exp((0, 0), 0) == (0, 1)
    assert O.gf16_exp((0, 0), 3) == (0, 0)


# ------------------------------------------------------------ matrices
def test_matrix_kats():  # matrix.rs:372-411, 419-423
    a, b, expect = KAT["matrix_multiply"]
    assert O.matrix_multiply(8, u8(a), u8(b)).tolist() == expect
    for m, inv in KAT["matrix_inverse"]:
        assert O.matrix_invert(8, u8(m)).tolist() == inv
    with pytest.raises(ValueError):
        O.matrix_invert(8, u8(KAT["matrix_singular"]))


def test_encoding_matrices_match_golden():
    for name, hexstr in GEN["encoding_matrices"].items():
        field, k, p = (int(x) for x in name[2:].split("_"))
        assert O.Codec(field, k, p).matrix().tobytes().hex() == hexstr
        m = O.Codec(field, k, p).matrix()
        if field == 8:
            assert (m[:k] == np.eye(k, dtype=np.uint8)).all()  # systematic


def test_survey_10_4_parity_rows():  # SURVEY.md §8 a8 (verified restatement)
    m = O.Codec(8, 10, 4).matrix()[10:].tolist()
    assert m[0] == [129, 150, 175, 184, 210, 196, 254, 232, 3, 2]
    assert m[3] == [214, 191, 10, 98, 111, 6, 183, 223, 4, 5]


# ------------------------------------------------------------ codec KATs
@pytest.mark.parametrize("name", ["one_encode", "readme", "reconstruct_2_2"])
def test_encode_kats(name):  # tests/mod.rs:851-893, README, tests/mod.rs:249-353
    kat = KAT[name]
    c = O.Codec(8, kat["k"], kat["p"])
    n = len(kat["data"][0])
    shards = [u8(d) for d in kat["data"]] + [np.zeros(n, np.uint8) for _ in range(kat["p"])]
    c.encode(shards)
    assert [s.tolist() for s in shards[kat["k"]:]] == kat["parity"]
    assert c.verify(shards)
    shards[-1][0] ^= 1
    assert not c.verify(shards)


def test_reconstruct_kat_sequence():  # tests/mod.rs:249-353 step by step
    c = O.Codec(8, 2, 2)
    s = [u8([0, 1, 2]), u8([3, 4, 5]), u8([200, 201, 203]), u8([100, 101, 102])]
    c.encode(s)
    assert c.verify(s)
    s[0][:] = [101, 102, 103]
    c.reconstruct(s, [False, True, True, True])
    assert [x.tolist() for x in s] == [[0, 1, 2], [3, 4, 5], [6, 11, 12], [5, 14, 11]]
    s[0][:] = [201, 202, 203]
    s[2][:] = [101, 102, 103]
    c.reconstruct(s, [False, True, False, True], data_only=True)
    assert not c.verify(s)
    assert [x.tolist() for x in s] == [[0, 1, 2], [3, 4, 5], [101, 102, 103], [5, 14, 11]]
    s[2][:] = [101, 102, 103]
    s[3][:] = [201, 202, 203]
    c.reconstruct(s, [True, True, False, False], data_only=True)
    assert [x.tolist() for x in s] == [[0, 1, 2], [3, 4, 5], [101, 102, 103], [201, 202, 203]]


def test_decode_matrices_match_golden():
    c = O.Codec(8, 10, 4)
    m = c.matrix()
    for key, hexstr in GEN["gf8_10_4_decode"].items():
        erased = [int(x) for x in key.split(",")]
        valid = [i for i in range(14) if i not in erased][:10]
        assert O.matrix_invert(8, m[valid]).tobytes().hex() == hexstr


# ---------------------------------------------------- vs the reference kernel
@pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref not built (no /root/reference)")
def test_oracle_mul_slice_matches_reference_simd_every_tail():
    ref = O.ref()
    rng = np.random.default_rng(1)
    for n in list(range(0, 131)) + [1000, 4099]:
        inp = rng.integers(0, 256, n, dtype=np.uint8)
        base = rng.integers(0, 256, n, dtype=np.uint8)
        for c in (0, 1, 2, 25, 52, 177, 255):
            for xor in (False, True):
                a = base.copy()
                b = base.copy()
                O.gf8_mul_slice(c, inp, a, xor=xor)
                f = ref.ref_gf8_mul_slice_xor if xor else ref.ref_gf8_mul_slice
                f(c, O._p(inp) if n else None, O._p(b) if n else None, n)
                assert (a == b).all(), (n, c, xor)


@pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref not built (no /root/reference)")
def test_reference_simd_kats():  # test_galois through the reference's own kernel
    ref = O.ref()
    inp = u8(KAT["mul_slice_input"])
    out = np.zeros_like(inp)
    for c, xor, expect in KAT["mul_slice_steps"]:
        (ref.ref_gf8_mul_slice_xor if xor else ref.ref_gf8_mul_slice)(c, O._p(inp), O._p(out),
                                                                       inp.size)
        assert out.tolist() == expect


def test_oracle_encode_matches_reference_vectors():
    c = O.Codec(8, 10, 4)
    seed = GEN["seed"]
    for n, want in GEN["gf8_10_4_encode"].items():
        n = int(n)
        s = [O.splitmix_bytes(seed + n, i, n) for i in range(10)] + \
            [np.zeros(n, np.uint8) for _ in range(4)]
        c.encode(s)
        assert [sha(x) for x in s[10:]] == want["parity_sha256"]


def test_oracle_full_size_10_2_digest():
    want = GEN["full_size"][f"gf8_10_2_{1 << 20}"]
    c = O.Codec(8, 10, 2)
    n = 1 << 20
    s = [O.splitmix_bytes(GEN["seed"], i, n) for i in range(10)] + \
        [np.zeros(n, np.uint8) for _ in range(2)]
    assert [sha(x) for x in s[:10]] == want["data_sha256"]
    c.encode(s)
    assert [sha(x) for x in s[10:]] == want["parity_sha256"]


# ------------------------------------------------------------ error semantics
def E(code):
    return pytest.raises(O.OracleError, match=f"^{code}$")


def test_oracle_error_precedence():  # tests/mod.rs:97-116, 1058-1163, macros.rs:142-245
    with E(3):
        O.Codec(8, 0, 1)
    with E(5):
        O.Codec(8, 1, 0)
    with E(2):
        O.Codec(8, 129, 128)
    c = O.Codec(8, 3, 2)
    s4 = [np.zeros(10, np.uint8) for _ in range(4)]
    with E(1):
        c.encode(s4)
    with E(2):
        c.encode(s4 + s4[:2])
    c2 = O.Codec(8, 2, 2)
    for shards, code in [([[0, 0, 0], [0, 1], [1, 2, 3], [0, 0, 0]], 9),
                         ([[0, 1], [0, 1], [1, 2, 3], [0, 0, 0]], 9),
                         ([[], [0, 1, 3], [1, 2, 3], [0, 0, 0]], 11)]:
        arr = [u8(x) for x in shards]
        with E(code):
            c2.encode(arr)
        with E(code):
            c2.verify(arr)
        with E(code):
            c2.reconstruct(arr, [True] * 4)
    with E(10):
        c2.reconstruct([np.zeros(3, np.uint8)] * 4, [False] * 4)
    # verify_with_buffer counts (tests/mod.rs:905-964)
    c3 = O.Codec(8, 3, 2)
    sh = [np.zeros(100, np.uint8) for _ in range(5)]
    with E(7):
        c3.verify_with_buffer(sh, [np.zeros(100, np.uint8)])
    with E(8):
        c3.verify_with_buffer(sh, [np.zeros(100, np.uint8)] * 3)
    with E(11):
        c3.verify_with_buffer(sh, [np.zeros(0, np.uint8), np.zeros(100, np.uint8)])
    with E(9):
        c3.verify_with_buffer(sh, [np.zeros(100, np.uint8), np.zeros(99, np.uint8)])
    # encode_single / sep (tests/mod.rs:2304-2619)
    with E(13):
        c3.encode_single(3, sh)
    with E(13):
        c3.encode_single_sep(3, sh[0], sh[3:])
    with E(3):
        c3.encode_sep(sh[:2], sh[3:])
    with E(6):
        c3.encode_sep(sh[:3], sh[2:])


@pytest.mark.parametrize("k,p", [(3, 2), (20, 8), (40, 12), (100, 30), (200, 56)])
def test_gf16_codecs_of_256_shards_code_in_the_gf8_subfield(k, p):
    """rse_codec.cpp kfield / RSE_OPT_SUBFIELD: a GF(2^16) codec of at most
    256 shards has every encoding-matrix entry in the GF(2^8) subfield (its
    Vandermonde points 0..k+p-1 are, galois_16.rs:97-107), equal to the
    GF(2^8) codec's matrix; a subfield constant multiplies each byte of an
    element on its own (galois_16.rs:20-52), so encode and every decode
    pattern give the GF(2^8) codec's bytes.  Checked on the oracle (the
    restatement of the reference): matrices, multiplication by every subfield
    constant, encode and a reconstruct."""
    m16, m8 = O.Codec(16, k, p).matrix(), O.Codec(8, k, p).matrix()
    assert (m16[..., 0] == 0).all() and (m16[..., 1] == m8).all()
    rng = np.random.default_rng(k * 7 + p)
    for c in range(256):
        a = tuple(int(x) for x in rng.integers(0, 256, 2))
        assert O.gf16_mul((0, c), a) == (O.gf8_mul(c, a[0]), O.gf8_mul(c, a[1]))
    n = 64
    s16 = [rng.integers(0, 256, 2 * n, dtype=np.uint8) for _ in range(k)] + \
          [np.zeros(2 * n, np.uint8) for _ in range(p)]
    s8 = [x.copy() for x in s16]
    O.Codec(16, k, p).encode(s16)
    O.Codec(8, k, p).encode(s8)
    for i in range(k, k + p):
        assert (s16[i] == s8[i]).all(), i
    lost = sorted(rng.choice(k + p, p, replace=False).tolist())
    r16 = [np.zeros(2 * n, np.uint8) if i in lost else s16[i].copy() for i in range(k + p)]
    O.Codec(16, k, p).reconstruct(r16, [i not in lost for i in range(k + p)])
    for i in lost:
        assert (r16[i] == s8[i]).all(), i


def test_gf16_codecs_past_256_shards_leave_the_subfield():
    """Past 256 shards the Vandermonde points leave GF(2^8): GF(2^16) proper."""
    m = O.Codec(16, 250, 7).matrix()
    assert (m[..., 0] != 0).any()
