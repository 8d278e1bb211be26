"""World-size-2 gloo test (CPU) of the multi-GPU fold orchestration: row sharding,
the all-gather of per-rank partials and the partial algebra used by
dds_combine_partials. Each rank's partial is computed with the oracle's Montgomery
restatement (radix 2^27, R = 2^(27*S)), exactly the value dds_col_fold_partial returns."""
import os
import random

import pytest
import torch.multiprocessing as mp

from oracle import homo

S = 152  # r27 limbs of a 4096-bit modulus
R = 1 << (27 * S)


def r27(x):
    return [(x >> (27 * i)) & ((1 << 27) - 1) for i in range(S)]


def from_r27(ws):
    return sum(int(w) << (27 * i) for i, w in enumerate(ws))


def partial(xs, N):
    Rinv = pow(R, -1, N)
    v = R % N
    for x in xs:
        v = v * x * Rinv % N
    return v


def _worker(rank, world, port, N, xs, out_q):
    import numpy as np
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import ddshe.dist as dd
    row0, cnt = dd.shard_range(len(xs), world, rank)
    v = partial(xs[row0:row0 + cnt], N)
    parts, rows = dd.gather_partials(np.array(r27(v), dtype=np.uint32), cnt)
    if rank == 0:
        # dds_combine_partials: fold the partials like rows, then multiply by R^k
        Rinv = pow(R, -1, N)
        acc = from_r27(parts[0])
        for p in parts[1:]:
            acc = acc * from_r27(p) * Rinv % N
        k = int(rows.sum())
        out_q.put((acc * pow(R, k, N) * Rinv % N, k))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_two_rank_gather_combine(world, keys):
    N = keys["paillier2048_committed"]["nsquare"]
    rng = random.Random(4)
    xs = [rng.randrange(N) for _ in range(37)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + rng.randrange(1000)
    procs = [ctx.Process(target=_worker, args=(r, world, port, N, xs, q)) for r in range(world)]
    for p in procs:
        p.start()
    res, k = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert k == len(xs)
    assert res == homo.modmul_fold(xs, N)


def test_shard_range_covers_rows():
    import ddshe.dist as dd
    for total in (0, 1, 7, 10, 1000):
        for world in (1, 2, 3, 8):
            got = [dd.shard_range(total, world, r) for r in range(world)]
            assert sum(c for _, c in got) == total
            nxt = 0
            for r0, c in got:
                if c:
                    assert r0 == nxt
                    nxt += c
