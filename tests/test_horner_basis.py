"""The Horner-mixing basis of the syndrome reconstruct (rse_kernels.hpp,
DESIGN.md section 4) against the oracle's GF(2^16) arithmetic (galois_16.rs
restated in oracle/rse_oracle.c), on the CPU: z is a root of
z^16 + z^6 + z^2 + z + 1, from_b / to_b are inverse bit matrices mapping
z-coordinates to elements, and Horner's rule over the coordinates of any c
multiplies by c.  The GPU parity tests check the kernels built on it."""
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from oracle import oracle as O  # noqa: E402

CSRC = os.path.join(HERE, "..", "reed-solomon-erasure_amd", "csrc")


def mul(a, b):  # uint16 elements, (x-coefficient << 8) | constant
    h, l = O.gf16_mul((a >> 8, a & 0xFF), (b >> 8, b & 0xFF))
    return (h << 8) | l


def parity(x):
    return bin(x).count("1") & 1


def test_horner_basis_against_the_oracle(tmp_path):
    exe = tmp_path / "horner_basis"
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", CSRC,
                    os.path.join(HERE, "native", "horner_basis.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split("\n")
    head = out[0].split()
    z, taps = int(head[1]), int(head[3])
    to_b = [int(x) for x in out[1].split()[1:]]
    from_b = [int(x) for x in out[2].split()[1:]]
    coords = dict(tuple(int(v) for v in x.split(":")) for x in out[3].split()[1:])
    # z is a root of the pentanomial; its powers are the basis columns
    zp = [1]
    for _ in range(16):
        zp.append(mul(zp[-1], z))
    rel = zp[16] ^ 1
    for i in range(1, 16):
        if (taps >> i) & 1:
            rel ^= zp[i]
    assert rel == 0 and taps == (1 << 6) | (1 << 2) | (1 << 1)
    for j in range(16):
        assert from_b[j] == sum(((zp[i] >> j) & 1) << i for i in range(16))
    rng = np.random.default_rng(16)
    for _ in range(200):
        e = int(rng.integers(0, 65536))
        co = sum(parity(e & to_b[i]) << i for i in range(16))
        assert sum(parity(co & from_b[j]) << j for j in range(16)) == e  # inverse matrices
        v = 0  # the coordinates are e's expansion in the powers of z
        for i in range(16):
            if (co >> i) & 1:
                v ^= zp[i]
        assert v == e
    # horner_coords (host and device planner) and Horner's rule multiply by c
    for c, co in coords.items():
        assert co == sum(parity(c & to_b[i]) << i for i in range(16))
        for _ in range(20):
            s = int(rng.integers(0, 65536))
            v = 0
            for i in range(15, -1, -1):
                v = mul(v, z)
                if (co >> i) & 1:
                    v ^= s
            assert v == mul(c, s), (c, s)
