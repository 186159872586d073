"""CPU check of the algebra behind rse_fft.hip: for GF(2^8) codecs with
k = p = 2^m, encode is the inverse additive FFT (Lin-Chung-Han novel basis) on
the subspace {0 .. k-1} followed by the forward transform on the coset
{k .. 2k-1}, and rebuilding every data shard from the parity shards is the
same pair with the cosets swapped.  Both are compared with the oracle's
restatement of the reference's matrix encode and reconstruct (core.rs:430-436,
481-509, 680-923) byte for byte.  The butterflies and twiddles here are the
ones the kernels are generated from (level i, block offset j: twiddle
s^_i(beta ^ j)); this is a pure-Python restatement, test infrastructure."""
import functools

import numpy as np
import pytest

from oracle import oracle as O


def gmul(a, b):  # GF(2^8) modulo 0x11D (build.rs:11)
    r = 0
    while b:
        if b & 1:
            r ^= a
        b >>= 1
        a <<= 1
        if a & 0x100:
            a ^= 0x11D
    return r


@functools.lru_cache(maxsize=None)
def ginv(a):
    return next(x for x in range(1, 256) if gmul(a, x) == 1)


@functools.lru_cache(maxsize=None)
def vanish(i, x):  # s_i(x) = prod over a in span(1, 2, .. 2^(i-1)) of (x + a)
    r = 1
    for a in range(1 << i):
        r = gmul(r, x ^ a)
    return r


@functools.lru_cache(maxsize=None)
def skew(i, x):  # s^_i(x) = s_i(x) / s_i(2^i)
    return gmul(vanish(i, x), ginv(vanish(i, 1 << i)))


def fft(d, beta):  # novel-basis coefficients -> values at beta ^ j
    d = list(d)
    n = len(d)
    for i in reversed(range(n.bit_length() - 1)):
        h = 1 << i
        for j in range(0, n, 2 * h):
            s = skew(i, beta ^ j)
            for t in range(j, j + h):
                d[t] ^= gmul(s, d[t + h])
                d[t + h] ^= d[t]
    return d


def ifft(v, beta):  # values at beta ^ j -> novel-basis coefficients
    d = list(v)
    n = len(d)
    for i in range(n.bit_length() - 1):
        h = 1 << i
        for j in range(0, n, 2 * h):
            s = skew(i, beta ^ j)
            for t in range(j, j + h):
                d[t + h] ^= d[t]
                d[t] ^= gmul(s, d[t + h])
    return d


@pytest.mark.parametrize("k", [2, 4, 8, 16, 32, 64, 128])
def test_fft_encode_and_rebuild_match_the_matrix_codec(k):
    p, n = k, 5
    rng = np.random.default_rng(k)
    data = [rng.integers(0, 256, n, dtype=np.uint8) for _ in range(k)]
    sh = [x.copy() for x in data] + [np.zeros(n, np.uint8) for _ in range(p)]
    oc = O.Codec(8, k, p)
    oc.encode(sh)
    for b in range(n):
        par = fft(ifft([int(x[b]) for x in data], 0), k)
        assert par == [int(sh[k + j][b]) for j in range(p)], (k, b)
        back = fft(ifft(par, k), 0)
        assert back == [int(x[b]) for x in data], (k, b)
    # the oracle's reconstruct with every data shard lost gives the same bytes
    lost = [x.copy() for x in sh]
    for i in range(k):
        lost[i][:] = 0
    oc.reconstruct(lost, [False] * k + [True] * p, data_only=True)
    for i in range(k):
        assert (lost[i] == data[i]).all(), i


def test_fft_twiddles_of_the_transform_on_the_subspace():
    """The first block of every level of the transform on {0 .. k-1} has a
    zero twiddle (s_i vanishes on span(1 .. 2^(i-1)), which holds 0) and no
    other twiddle is zero: the kernels' free butterflies."""
    for m in range(1, 7):
        k = 1 << m
        for i in range(m):
            for j in range(0, k, 2 << i):
                assert (skew(i, j) == 0) == (j == 0)
                assert skew(i, k ^ j) != 0


@pytest.mark.parametrize("k", [2, 4, 8, 16, 32, 64, 128])
def test_parity_block_is_its_own_inverse(k):
    """The k x k parity block of the k+k codec (core.rs:430-436) equals its
    inverse -- the decode rows of every data shard from the parity shards
    (core.rs:697-731) -- so rse_fft.hip's one kernel serves encode and the
    rebuild: Q(x) = P(x ^ k) swaps the cosets {0..k-1} and {k..2k-1}."""
    m = np.asarray(O.Codec(8, k, k).matrix(), np.uint8)
    par = m[k:]
    assert (np.asarray(O.matrix_invert(8, par), np.uint8) == par).all()
