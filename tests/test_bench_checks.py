"""The bench's correctness flags can fail.

bench.py's reconstruct legs poison the erased shards before their timed calls
and compare every rebuilt shard with its synthetic bytes afterwards; its verify
legs corrupt two stripes that must come back false.  On CPU the codec is
stubbed: a reconstruct that writes nothing, or writes wrong bytes, and a verify
that always answers true, must turn the flags false, while a correct stand-in
(the oracle, test infrastructure) turns them true.  The `gpu` test runs the
same legs through the HIP library and asserts the flags are true.
"""
import hashlib
import time

import numpy as np
import pytest
import torch

import bench
from oracle import oracle as O

K, P, L, N = 4, 2, 4096, 4


def _cpu_fill(t, seed, shard):
    t.copy_(torch.from_numpy(O.splitmix_bytes(seed, shard, t.numel())))


def _cpu_timed_ms(fn, reps, stream=None):
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return max((time.perf_counter() - t0) / reps * 1e3, 1e-6)


@pytest.fixture
def cpu_bench(monkeypatch):
    monkeypatch.setattr(bench, "timed_ms", _cpu_timed_ms)
    monkeypatch.setattr(bench, "_sync", lambda: None)


def _stripes():
    """N encoded stripes (oracle) of K+P shards of L bytes: v[stripe, shard, byte]."""
    c = O.Codec(8, K, P)
    v = torch.zeros((N, K + P, L), dtype=torch.uint8)
    for s in range(N):
        sh = [O.splitmix_bytes(bench.SEED, bench.shard_id(s, i), L) for i in range(K)]
        sh += [np.zeros(L, np.uint8) for _ in range(P)]
        c.encode(sh)
        v[s] = torch.from_numpy(np.stack(sh))
    return v


class _NoOp:
    """Writes nothing and accepts everything."""

    def reconstruct_data_flat(self, flat, elems, n, present):
        pass

    def verify(self, shards):
        return True

    def verify_flat(self, flat, L_, n):
        return np.ones(n, bool)


class _Zeros(_NoOp):
    """Writes the wrong bytes (zeros) into the erased shards."""

    def reconstruct_data_flat(self, flat, elems, n, present):
        v = flat.view(n, len(present), -1)
        for i, ok in enumerate(present):
            if not ok:
                v[:, i].zero_()


class _Oracle:
    """A correct stand-in: the CPU restatement of core.rs."""

    def __init__(self):
        self.c = O.Codec(8, K, P)

    def reconstruct_data_flat(self, flat, elems, n, present):
        v = flat.view(n, len(present), -1)
        for s in range(n):
            sh = [v[s, i].numpy() for i in range(len(present))]
            self.c.reconstruct(sh, present, data_only=True)

    def verify(self, shards):
        return self.c.verify([x.numpy() for x in shards])

    def verify_flat(self, flat, L_, n):
        v = flat.view(n, K + P, L_)
        return np.array([self.verify([v[s, i] for i in range(K + P)]) for s in range(n)])


def _recon(codec, v, erased=(0, 1)):
    want = [hashlib.sha256(O.splitmix_bytes(bench.SEED, bench.shard_id(0, i), L).tobytes())
            .hexdigest() for i in erased]
    return bench.reconstruct_leg(codec, v, K, list(erased), L, N, None, _cpu_fill,
                                 list(range(N)), want, reps=2)


def test_reconstruct_flags_false_for_a_kernel_that_writes_nothing(cpu_bench):
    v = _stripes()
    leg = _recon(_NoOp(), v)
    assert leg["rebuilt_ok_all_stripes"] is False
    assert leg["rebuilt_stripe0_vs_digests"] is False
    assert bench.rebuilt_ok(v, N, [0, 1], list(range(N)), _cpu_fill) is False
    assert (v[:, 0] == bench.POISON).all()  # the poison is what it left


def test_reconstruct_flags_false_for_wrong_bytes(cpu_bench):
    assert _recon(_Zeros(), _stripes())["rebuilt_ok_all_stripes"] is False


def test_reconstruct_flags_true_for_a_correct_rebuild(cpu_bench):
    v = _stripes()
    leg = _recon(_Oracle(), v, (0, 2))
    assert leg["rebuilt_ok_all_stripes"] is True
    assert leg["rebuilt_stripe0_vs_digests"] is True
    assert (v == _stripes()).all()


def test_reconstruct_digest_flag():
    """Stripe 0 against fixture digests: true for the right bytes, false
    after a flipped byte."""
    v = _stripes()
    want = [hashlib.sha256(v[0, i].numpy().tobytes()).hexdigest() for i in (0, 1)]
    assert bench.digests_ok(v, [0, 1], want)
    v[0, 1, 7] ^= 1
    assert not bench.digests_ok(v, [0, 1], want)


def test_verify_flags_false_for_a_verify_that_accepts_everything(cpu_bench):
    v = _stripes()
    before = v.clone()
    per_call, flat = bench.verify_leg(_NoOp(), v, K, P, L, N, reps=2)
    assert per_call["verdicts_ok"] is False and flat["verdicts_ok"] is False
    assert len(per_call["corrupted_stripes"]) == 2
    assert (v == before).all()  # the corrupted bytes are restored


def test_verify_flags_true_for_a_correct_verify(cpu_bench):
    per_call, flat = bench.verify_leg(_Oracle(), _stripes(), K, P, L, N, reps=2)
    assert per_call["verdicts_ok"] is True and flat["verdicts_ok"] is True


@pytest.mark.gpu
def test_bench_legs_on_the_gpu():
    """The same legs through the HIP library: every flag true, on GF(2^8)
    10+4 (syndrome kernel and repeated pattern) and GF(2^16) 20+8 at 8 lost;
    and false for a stubbed codec on the same device buffers."""
    import reed_solomon_erasure as R
    from reed_solomon_erasure.core import fill_splitmix
    stream = torch.cuda.current_stream()
    for field, k, p, nb, n, erased in ((8, 10, 4, 64 << 10, 6, [0, 1]),
                                       (16, 20, 8, 64 << 10, 4, list(range(8)))):
        v = torch.empty((n, k + p, nb), dtype=torch.uint8, device="cuda")
        for s in range(n):
            for i in range(k):
                fill_splitmix(v[s, i], bench.SEED, bench.shard_id(s, i))
        r = R.core.ReedSolomon(k, p, field)
        elems = nb // (field // 8)
        r.encode_flat(v.view(-1), elems, n)
        leg = bench.reconstruct_leg(r, v, k, erased, elems, n, stream, fill_splitmix,
                                    list(range(n)), reps=2)
        assert leg["rebuilt_ok_all_stripes"] is True, (field, leg)
        if field == 8:
            a, b = bench.verify_leg(r, v, k, p, nb, n, reps=2)
            assert a["verdicts_ok"] is True and b["verdicts_ok"] is True
            assert a["c_abi"]["verdicts_ok"] is True and a["c_abi"]["us_per_call"] > 0
            assert r.verify_flat(v.view(-1), nb, n).all()  # restored
            a, b = bench.verify_leg(_NoOp(), v, k, p, nb, n, reps=2)
            assert a["verdicts_ok"] is False and b["verdicts_ok"] is False
        leg = bench.reconstruct_leg(_NoOp(), v, k, erased, elems, n, stream, fill_splitmix,
                                    list(range(n)), reps=2)
        assert leg["rebuilt_ok_all_stripes"] is False


def test_reference_rows_and_cpu_call():
    """The CPU side of the reference bench matrix: encode codes the parity
    rows, reconstruct the decode rows of the first k present shards (core.rs:
    801-861), and the reference kernel's per-call time is measured in C."""
    rows, ins = bench._ref_rows(4, 4, None)
    assert rows.shape == (4, 4) and ins == [0, 1, 2, 3]
    rows, ins = bench._ref_rows(4, 4, [0, 1])
    assert rows.shape == (2, 4) and ins == [2, 3, 4, 5]
    # the decode rows rebuild the erased shards from the valid ones
    c = O.Codec(8, 4, 4)
    sh = [O.splitmix_bytes(1, i, 1000) for i in range(4)] + [np.zeros(1000, np.uint8)] * 4
    sh = [np.array(x) for x in sh]
    c.encode(sh)
    out = [np.zeros(1000, np.uint8) for _ in range(2)]
    O.code_some_slices(8, rows, [sh[i] for i in ins], out)
    assert all(np.array_equal(out[j], sh[j]) for j in range(2))
    if O.ref_available():
        us = bench.cpu_reference_call_us(10, 4, 1024, None, budget_s=0.005)
        assert us is not None and 0 < us < 1e4


@pytest.mark.gpu
def test_reference_bench_matrix_on_the_gpu():
    """bench.py's reference bench matrix at a reduced set of shapes: every
    column measured, parity and rebuilt shards checked, the crossover sweep
    filled in."""
    out = bench.reference_bench_matrix(torch.cuda.current_stream(),
                                       shapes=[(1024, 4, 4), (4096, 10, 4)],
                                       crossover_sizes=(1024, 65536))
    ops = {(e["shape"], e["op"]) for e in out["entries"]}
    assert ("4+4 x 1 KiB", "reconstruct_all") in ops and ("10+4 x 4 KiB", "encode") in ops
    for e in out["entries"]:
        assert e["gpu_call_device_us"] > 0 and e["gpu_call_host_us"] > 0
        if e["op"] == "encode":
            assert e["parity_stripe0_vs_oracle"] is True and e["gpu_flat"]["GB_per_s"] > 0
        elif e["op"] != "reconstruct_none":
            assert e["rebuilt_ok_all_stripes"] is True
    assert len(out["crossover_10_4"]["rows"]) == 2


# ------------------------------------------------------ the printed line
_LINE_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "collective", "roofline", "cpu_baseline", "library")


def _split_full(full):
    """A full results dict -> (line, cpu, extras) as bench.main holds them."""
    line = {key: full[key] for key in _LINE_KEYS}
    cpu = {key: full[key] for key in ("cpu_baseline_legs", "cpu_host") if key in full}
    extras = {key: x for key, x in full.items() if key not in _LINE_KEYS and key not in cpu}
    return line, cpu, extras


def test_printed_line_is_last_compact_and_complete(tmp_path, capsys):
    """Round 4's full bench results (28.7 KB, tests/golden/bench_full_r04s17.json,
    the last line of profiles/r04/s17/bench.log) through bench.emit_results:
    the LAST stdout line parses, is < 4096 bytes, and carries the contract keys,
    roofline.frac and cpu_baseline.value; every leg is in the full file."""
    import json
    import os
    full = json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                       "bench_full_r04s17.json")))
    assert len(json.dumps(full)) > 8192  # the line the driver could not read
    line, cpu, extras = _split_full(full)
    out_path = tmp_path / "full.json"
    bench.emit_results(line, cpu, extras, str(out_path))
    stdout = capsys.readouterr().out
    last = stdout.rstrip("\n").split("\n")[-1]
    assert len(last.encode()) < 4096
    got = json.loads(last)
    for key in _LINE_KEYS[:-1]:
        assert key in got, key
    assert got["value"] == full["value"] and got["ms_per_step"] == full["ms_per_step"]
    assert 0 < got["roofline"]["frac"] < 1 and got["roofline"]["peak"] == 8000.0
    assert got["roofline"]["algorithmic_bytes_per_launch"] > 0
    assert got["cpu_baseline"]["value"] > 0 and got["cpu_baseline"]["kind"] == "reference"
    assert got["config"]["workload"] == full["config"]["workload"]
    assert got["checks"]["all_true"] is True and got["checks"]["flags"] > 50
    legs = got["legs"]
    assert legs["reconstruct_10_4_lost_0_1_GBps"] == full["reconstruct"]["algorithmic_GB_per_s"]
    assert legs["ref_bench_encode_GBps"]["64+64x1K"] > 0
    assert json.load(open(out_path)) == full  # nothing lost: every leg in the file


def test_printed_line_reports_a_false_flag_and_still_fits(tmp_path, capsys):
    import json
    import os
    full = json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                       "bench_full_r04s17.json")))
    full["reference_bench_matrix"]["entries"][3]["rebuilt_ok_all_stripes"] = False
    full["reference_bench_matrix"]["entries"] *= 8  # a much longer matrix
    line, cpu, extras = _split_full(full)
    got = bench.emit_results(line, cpu, extras, str(tmp_path / "f.json"))
    last = capsys.readouterr().out.rstrip("\n").split("\n")[-1]
    assert len(last.encode()) < 4096 and json.loads(last) == got
    assert got["checks"]["all_true"] is False
    assert got["checks"]["false"][0].startswith("reference_bench_matrix.entries[3]")


def test_host_agreement_flag():
    """The two pinned-host flat encode legs must agree within 10 % (VERDICT r05
    §4): the flag is true for 66.0 k / 65.7 k MB/s, false for round 5's
    39.6 k / 72.6 k, and the ratio to plain duplex copies is a number, not a
    correctness flag.  Nothing is added when a leg did not run or the job had
    several ranks."""
    def extras(flat, ranks_mb, ranks=1):
        return {"end_to_end_host_all_ranks": {"MB_per_s_all_ranks": ranks_mb, "ranks": ranks},
                "end_to_end_pinned_host_flat": {"MB_per_s": flat,
                                                "raw_pinned_duplex_MB_per_s": 76000.0}}
    e = extras(66000.0, 65700.0)
    bench.host_agreement(e)
    f = e["end_to_end_pinned_host_flat"]
    assert f["host_flat_legs_agree_within_10pct"] is True
    assert f["vs_raw_duplex"] == round(66000.0 / 76000.0, 3)
    assert ("end_to_end_pinned_host_flat.host_flat_legs_agree_within_10pct", True) in \
        bench.correctness_flags(e)
    assert not [x for x in bench.correctness_flags(e) if "duplex" in x[0]]
    e = extras(39600.0, 72600.0)
    bench.host_agreement(e)
    assert e["end_to_end_pinned_host_flat"]["host_flat_legs_agree_within_10pct"] is False
    e = extras(39600.0, 72600.0, ranks=2)
    bench.host_agreement(e)
    assert "host_flat_legs_agree_within_10pct" not in e["end_to_end_pinned_host_flat"]
    e = {"end_to_end_pinned_host_flat": {"MB_per_s": 1.0}}
    bench.host_agreement(e)
    assert e == {"end_to_end_pinned_host_flat": {"MB_per_s": 1.0}}


def test_warm_calls_runs_for_the_time_given():
    n = []
    t0 = time.perf_counter()
    bench.warm_calls(lambda: n.append(1), seconds=0.05)
    assert time.perf_counter() - t0 >= 0.05 and len(n) >= 2
