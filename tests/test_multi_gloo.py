"""The multi-GPU path of bench.py, rehearsed on CPU with 2 gloo ranks.

Each rank encodes its own block of global stripes (bench.stripes_for_rank) with
the CPU checker standing in for the GPU kernel, the slowest rank's time is
all-reduced (bench.reduce_timing) and the job throughput aggregated
(bench.job_throughput).  Checks: the partition is disjoint and complete, the
aggregate equals the single-process computation, and every stripe's parity is
identical whichever rank encoded it (stripes are independent, so placement
cannot change results).
"""
import hashlib
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import bench
from oracle import oracle as O

K, P, L, STRIPES_PER_RANK = 4, 2, 4096, 5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _stripe_digest(g):
    c = O.Codec(8, K, P)
    shards = [O.splitmix_bytes(bench.SEED, bench.shard_id(g, i), L) for i in range(K)]
    shards += [np.zeros(L, np.uint8) for _ in range(P)]
    c.encode(shards)
    return hashlib.sha256(b"".join(x.tobytes() for x in shards[K:])).hexdigest()


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    assert bench.init_collective(world, rank, 0, rehearsal=False) == "gloo"  # no GPU here
    coll = bench.collective_info(world, 0, False)
    mine = bench.stripes_for_rank(STRIPES_PER_RANK * world, rank, world)
    digests = {g: _stripe_digest(g) for g in mine}
    elapsed = 0.5 + rank  # deterministic stand-in for the timed region
    t = bench.reduce_timing(elapsed, world)
    gathered = [None] * world
    dist.all_gather_object(gathered, digests)
    verdicts = bench.gather(1 if rank else -1, world, rank, None)  # per-rank verdicts
    if rank == 0:
        q.put((t, gathered, [list(bench.stripes_for_rank(STRIPES_PER_RANK * world, r, world))
                             for r in range(world)], verdicts, coll))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_stripe_split_and_reduction():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    t, gathered, parts, verdicts, coll = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    # partition: disjoint, complete, equal sizes (weak scaling)
    flat = [g for part in parts for g in part]
    assert sorted(flat) == list(range(STRIPES_PER_RANK * world))
    assert all(len(part) == STRIPES_PER_RANK for part in parts)
    # timing reduction is the max over ranks; throughput counts every rank's bytes
    assert t == 1.5
    assert verdicts == [-1.0, 1.0]  # every rank's verdict, in rank order, on rank 0
    stripe_bytes = (K + P) * L
    v = bench.job_throughput(3, STRIPES_PER_RANK, world, stripe_bytes, t)
    assert v == pytest.approx(3 * STRIPES_PER_RANK * world * stripe_bytes / 1.5 / (1 << 20))
    # what the collective saw: the backend, both ranks, each rank's device
    assert coll["backend"] == "gloo" and coll["world_size"] == world
    assert [d["pid"] for d in coll["rank_devices"]] == sorted({d["pid"] for d in coll["rank_devices"]})
    assert len(coll["rank_devices"]) == world and coll["distinct_gpus"] is False  # CPU ranks
    # placement-independent results
    merged = {}
    for d in gathered:
        merged.update(d)
    for g in range(STRIPES_PER_RANK * world):
        assert merged[g] == _stripe_digest(g)


def test_uneven_partition():
    parts = [bench.stripes_for_rank(10, r, 4) for r in range(4)]
    assert [len(p) for p in parts] == [3, 3, 2, 2]
    assert sorted(g for p in parts for g in p) == list(range(10))


def test_golden_covers_every_rank_first_and_last_stripe():
    """BASELINE config 4 (4096 stripes over 8 GPUs, 512 each) and the 2/4-rank
    rehearsals (4 stripes each): every rank's first and last stripe has a
    reference digest, so no rank's output goes unchecked."""
    gold = bench.golden_stripes()
    for per, ranks in ((512, 8), (512, 4), (512, 2), (512, 1), (4, 4), (4, 2)):
        for r in range(ranks):
            part = bench.stripes_for_rank(per * ranks, r, ranks)
            assert str(part.start) in gold and str(part.stop - 1) in gold


def test_check_stripes_detects_a_flipped_byte():
    import torch
    k, p, n = 10, 4, 16 << 20
    v = torch.zeros((1, k + p, n), dtype=torch.uint8)
    shards = [O.splitmix_bytes(bench.SEED, bench.shard_id(0, i), n) for i in range(k)]
    shards += [np.zeros(n, np.uint8) for _ in range(p)]
    O.Codec(8, k, p).encode(shards)
    v[0] = torch.from_numpy(np.stack(shards))
    assert bench.check_stripes(v, range(0, 1), 1, k, p) == (1, [0])
    v[0, k + 2, 12345] ^= 1
    assert bench.check_stripes(v, range(0, 1), 1, k, p) == (0, [0])
    assert bench.check_stripes(v, range(5, 6), 1, k, p) == (-1, [])  # no digest: unchecked


def test_missing_peer_fails_fast():
    """A rank whose peer never joins exits non-zero within the collective
    deadline instead of hanging (bench.init_collective)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()), RSE_BENCH_COLLECTIVE_TIMEOUT="5")
    code = "import bench; bench.init_collective(2, 0, 0, False); print('joined')"
    out = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True,
                         text=True, timeout=120)
    assert out.returncode in (4, 5), (out.returncode, out.stderr[-2000:])
    assert "joined" not in out.stdout
    assert "rank 0/2" in out.stderr
