"""Generate tests/golden/golden.json -- run in the build container:

    python tests/golden/make_golden.py

Two kinds of fixtures:

* ``reference_kats``: known-answer data transcribed from the reference's own
  tests (file:line cited per entry).  Pure data, no reference code.
* ``generated``: vectors produced by the reference's OWN compiled SIMD kernel
  (simd_c/reedsolomon.c, built from /root/reference by oracle/Makefile into
  oracle/_ref/librse_ref.so and driven in core.rs:481-509 loop order) for
  GF(2^8), and by the C restatement (oracle/rse_oracle.c) for matrices and
  GF(2^16) (the reference has no native GF(2^16) path).  Shard bytes come from
  oracle.splitmix_bytes(seed, shard_id, n), so the tests can regenerate the
  inputs on either side (numpy on the host, rse_fill_splitmix on the GPU).
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

SEED = 0x5EED


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def reference_kats():
    return {
        # galois_8.rs:339-363 BACKBLAZE_LOG_TABLE (first entry changed to 0)
        "log_table": [
            0, 0, 1, 25, 2, 50, 26, 198, 3, 223, 51, 238, 27, 104, 199, 75, 4, 100, 224, 14, 52, 141,
            239, 129, 28, 193, 105, 248, 200, 8, 76, 113, 5, 138, 101, 47, 225, 36, 15, 33, 53, 147,
            142, 218, 240, 18, 130, 69, 29, 181, 194, 125, 106, 39, 249, 185, 201, 154, 9, 120, 77,
            228, 114, 166, 6, 191, 139, 98, 102, 221, 48, 253, 226, 152, 37, 179, 16, 145, 34, 136, 54,
            208, 148, 206, 143, 150, 219, 189, 241, 210, 19, 92, 131, 56, 70, 64, 30, 66, 182, 163,
            195, 72, 126, 110, 107, 58, 40, 84, 250, 133, 186, 61, 202, 94, 155, 159, 10, 21, 121, 43,
            78, 212, 229, 172, 115, 243, 167, 87, 7, 112, 192, 247, 140, 128, 99, 13, 103, 74, 222,
            237, 49, 197, 254, 24, 227, 165, 153, 119, 38, 184, 180, 124, 17, 68, 146, 217, 35, 32,
            137, 46, 55, 63, 209, 91, 149, 188, 207, 205, 144, 135, 151, 178, 220, 252, 190, 97, 242,
            86, 211, 171, 20, 42, 93, 158, 132, 60, 57, 83, 71, 109, 65, 162, 31, 45, 67, 216, 183,
            123, 164, 118, 196, 23, 73, 236, 127, 12, 111, 246, 108, 161, 59, 82, 41, 157, 85, 170,
            251, 96, 134, 177, 187, 204, 62, 90, 203, 89, 95, 176, 156, 169, 160, 81, 11, 245, 22, 235,
            122, 117, 44, 215, 79, 174, 213, 233, 230, 231, 173, 232, 116, 214, 244, 234, 168, 80, 88,
            175,
        ],
        # galois_8.rs:482-552 test_galois
        "mul": [[3, 4, 12], [7, 7, 21], [23, 45, 41]],
        "exp": [[2, 2, 4], [5, 20, 235], [13, 7, 43]],
        "mul_slice_input": [0, 1, 2, 3, 4, 5, 6, 10, 50, 100, 150, 174, 201, 255, 99, 32, 67, 85,
                            200, 199, 198, 197, 196, 195, 194, 193, 192, 191, 190, 189, 188, 187,
                            186, 185],
        # (coefficient, xor_into, expected) applied in sequence to ONE output buffer
        "mul_slice_steps": [
            [25, False, [0x0, 0x19, 0x32, 0x2b, 0x64, 0x7d, 0x56, 0xfa, 0xb8, 0x6d, 0xc7, 0x85, 0xc3,
                         0x1f, 0x22, 0x7, 0x25, 0xfe, 0xda, 0x5d, 0x44, 0x6f, 0x76, 0x39, 0x20, 0xb,
                         0x12, 0x11, 0x8, 0x23, 0x3a, 0x75, 0x6c, 0x47]],
            [52, True, [0x0, 0x2d, 0x5a, 0x77, 0xb4, 0x99, 0xee, 0x2f, 0x79, 0xf2, 0x7, 0x51, 0xd4,
                        0x19, 0x31, 0xc9, 0xf8, 0xfc, 0xf9, 0x4f, 0x62, 0x15, 0x38, 0xfb, 0xd6, 0xa1,
                        0x8c, 0x96, 0xbb, 0xcc, 0xe1, 0x22, 0xf, 0x78]],
            [177, False, [0x0, 0xb1, 0x7f, 0xce, 0xfe, 0x4f, 0x81, 0x9e, 0x3, 0x6, 0xe8, 0x75, 0xbd,
                          0x40, 0x36, 0xa3, 0x95, 0xcb, 0xc, 0xdd, 0x6c, 0xa2, 0x13, 0x23, 0x92, 0x5c,
                          0xed, 0x1b, 0xaa, 0x64, 0xd5, 0xe5, 0x54, 0x9a]],
            [117, True, [0x0, 0xc4, 0x95, 0x51, 0x37, 0xf3, 0xa2, 0xfb, 0xec, 0xc5, 0xd0, 0xc7, 0x53,
                         0x88, 0xa3, 0xa5, 0x6, 0x78, 0x97, 0x9f, 0x5b, 0xa, 0xce, 0xa8, 0x6c, 0x3d,
                         0xf9, 0xdf, 0x1b, 0x4a, 0x8e, 0xe8, 0x2c, 0x7d]],
        ],
        # matrix.rs:372-379 test_matrix_multiply
        "matrix_multiply": [[[1, 2], [3, 4]], [[5, 6], [7, 8]], [[11, 22], [19, 42]]],
        # matrix.rs:381-411 test_matrix_inverse_pass_cases (+ singular case :419-423)
        "matrix_inverse": [
            [[[56, 23, 98], [3, 100, 200], [45, 201, 123]],
             [[175, 133, 33], [130, 13, 245], [112, 35, 126]]],
            [[[1, 0, 0, 0, 0], [0, 1, 0, 0, 0], [0, 0, 0, 1, 0], [0, 0, 0, 0, 1], [7, 7, 6, 6, 1]],
             [[1, 0, 0, 0, 0], [0, 1, 0, 0, 0], [123, 123, 1, 122, 122], [0, 0, 1, 0, 0],
              [0, 0, 0, 1, 0]]],
        ],
        "matrix_singular": [[4, 2], [12, 6]],
        # tests/mod.rs:851-893 test_one_encode (5+5)
        "one_encode": {"k": 5, "p": 5,
                       "data": [[0, 1], [4, 5], [2, 3], [6, 7], [8, 9]],
                       "parity": [[12, 13], [10, 11], [14, 15], [90, 91], [94, 95]]},
        # README.md (3+2 x 4-byte example)
        "readme": {"k": 3, "p": 2,
                   "data": [[0, 1, 2, 3], [4, 5, 6, 7], [8, 9, 10, 11]],
                   "parity": [[12, 13, 14, 15], [16, 17, 18, 19]]},
        # tests/mod.rs:249-353 test_reconstruct (2+2)
        "reconstruct_2_2": {"k": 2, "p": 2,
                            "data": [[0, 1, 2], [3, 4, 5]],
                            "parity": [[6, 11, 12], [5, 14, 11]]},
        # sage/galois_ext_test.sage:10-26 -- GF(2^8) 'a' is 0x02 (Conway
        # polynomial x^8+x^4+x^3+x^2+1 = 0x11D, the generator of build.rs:11);
        # elements written [coefficient of b, constant].
        "gf16_sage": {
            "e1": [0b11010010, 0b00001111], "e2": [0b10100100, 0b10011010],
            "sum": [0b01110110, 0b10010101], "product": [0b00010111, 0b10101010],
            "quotient": [0b11111101, 0b01001010], "inv_b": [0b00011011, 0b00110110],
        },
    }


def generated():
    ref = O.ref()
    out = {"seed": SEED, "prng": "oracle.splitmix_bytes(seed, shard_id, nbytes)"}

    mats = {}
    for field, k, p in [(8, 3, 2), (8, 10, 2), (8, 10, 4), (8, 5, 5), (8, 2, 2), (8, 20, 4),
                        (16, 20, 8), (16, 10, 4), (16, 3, 2)]:
        c = O.Codec(field, k, p)
        mats[f"gf{field}_{k}_{p}"] = c.matrix().tobytes().hex()
    out["encoding_matrices"] = mats

    # 10+4 GF(2^8) encodes through the reference's own SIMD kernel at lengths
    # that exercise every vector/tail split of both the reference and ours.
    c = O.Codec(8, 10, 4)
    rows = np.ascontiguousarray(c.matrix()[10:])
    enc = {}
    for n in [1, 2, 15, 16, 17, 31, 32, 33, 34, 63, 64, 65, 100, 1000, 4097, 10003]:
        data = [O.splitmix_bytes(SEED + n, s, n) for s in range(10)]
        par = [np.zeros(n, np.uint8) for _ in range(4)]
        ref.ref_gf8_code_some_slices(rows.ctypes.data_as(O._u8p), 4, 10, O._ptrs(data),
                                     O._ptrs(par), n)
        enc[str(n)] = {"parity_sha256": [sha(p) for p in par],
                       "parity_hex": [p.tobytes().hex() for p in par] if n <= 64 else None}
    out["gf8_10_4_encode"] = enc

    # decode matrices (k x k inverse of the valid rows, core.rs:711-722)
    dec = {}
    m = c.matrix()
    for erased in [(0, 1), (0, 12), (9, 10, 11, 13), (3,), (10, 11, 12, 13)]:
        valid = [i for i in range(14) if i not in erased][:10]
        inv = O.matrix_invert(8, m[valid])
        dec[",".join(map(str, erased))] = inv.tobytes().hex()
    out["gf8_10_4_decode"] = dec

    # Full-size configurations (BASELINE.json configs): parity digests.
    full = {}
    # 50+20: the widest configuration of the reference's own bench
    # (benches/bandwidth.rs:128), at the 1 MiB shards of the README table
    for (k, p, n) in [(10, 2, 1 << 20), (10, 4, 16 << 20), (50, 20, 1 << 20)]:
        cc = O.Codec(8, k, p)
        rr = np.ascontiguousarray(cc.matrix()[k:])
        data = [O.splitmix_bytes(SEED, s, n) for s in range(k)]
        par = [np.zeros(n, np.uint8) for _ in range(p)]
        ref.ref_gf8_code_some_slices(rr.ctypes.data_as(O._u8p), p, k, O._ptrs(data),
                                     O._ptrs(par), n)
        full[f"gf8_{k}_{p}_{n}"] = {"data_sha256": [sha(d) for d in data],
                                    "parity_sha256": [sha(x) for x in par]}
    # GF(2^16) 20+8 x 4 MiB through the C restatement of lib.rs:99-118.
    k, p, nbytes = 20, 8, 4 << 20
    cc = O.Codec(16, k, p)
    rr = np.ascontiguousarray(cc.matrix()[k:])
    data = [O.splitmix_bytes(SEED, s, nbytes) for s in range(k)]
    par = [np.zeros(nbytes, np.uint8) for _ in range(p)]
    O.code_some_slices(16, rr, data, par)
    full[f"gf16_{k}_{p}_{nbytes}"] = {"data_sha256": [sha(d) for d in data],
                                      "parity_sha256": [sha(x) for x in par]}
    # GF(2^16) 40+12 x 1 MiB: a wide GF(2^16) codec (k > 32, p > 8) on its
    # one-module kernel in bench.py's other_configs
    k, p, nbytes = 40, 12, 1 << 20
    cc = O.Codec(16, k, p)
    rr = np.ascontiguousarray(cc.matrix()[k:])
    data = [O.splitmix_bytes(SEED, s, nbytes) for s in range(k)]
    par = [np.zeros(nbytes, np.uint8) for _ in range(p)]
    O.code_some_slices(16, rr, data, par)
    full[f"gf16_{k}_{p}_{nbytes}"] = {"data_sha256": [sha(d) for d in data],
                                      "parity_sha256": [sha(x) for x in par]}
    out["full_size"] = full
    out["gf8_10_4_stripe_parity"] = stripe_parity(ref)
    return out


def bench_stripes():
    """Global stripes whose parity bench.py checks at N ranks: every rank's
    first and last stripe at 512 stripes per rank (N = 1..8, BASELINE config
    4's 4096 stripes), and at 4 stripes per rank for the one-GPU rehearsals of
    the N > 1 path (2 and 4 ranks)."""
    ids = set()
    for per in (512, 4):
        for r in range(8):
            ids |= {per * r, per * r + per - 1}
    return sorted(ids)


def stripe_parity(ref):
    """Parity digests of 10+4 x 16 MiB global stripe g, whose shard i holds
    oracle.splitmix_bytes(SEED, (g << 8) | i, 16 MiB) (bench.py shard_id)."""
    k, p, n = 10, 4, 16 << 20
    rr = np.ascontiguousarray(O.Codec(8, k, p).matrix()[k:])
    res = {}
    for g in bench_stripes():
        data = [O.splitmix_bytes(SEED, (g << 8) | i, n) for i in range(k)]
        par = [np.zeros(n, np.uint8) for _ in range(p)]
        ref.ref_gf8_code_some_slices(rr.ctypes.data_as(O._u8p), p, k, O._ptrs(data),
                                     O._ptrs(par), n)
        res[str(g)] = [sha(x) for x in par]
    return res


def main():
    O.build()
    g = {"reference_kats": reference_kats(), "generated": generated()}
    path = os.path.join(HERE, "golden.json")
    with open(path, "w") as f:
        json.dump(g, f, indent=1, sort_keys=True)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
