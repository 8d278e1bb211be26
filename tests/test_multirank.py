"""World-size-2 gloo test (CPU) of the multi-GPU fold orchestration: row sharding,
the all-gather of per-rank partials and the partial algebra used by
dds_combine_partials. Each rank's partial is restated from the engine's definition
(dds_col_fold_partial): S2 = 160 radix-2^28 limbs holding the canonical prod * 2^E mod N plus the
signed exponent E in two words, where a fold with G first-level groups and the reduction tree
(ddshe_tree.hip: 162 limbs of 26 bits) gives E = 28*148*(G - rows) - 26*162*(G - 1)."""
import os
import random

import pytest
import torch.multiprocessing as mp

from oracle import homo

W, S, S2 = 28, 148, 160  # throughput / partial limb counts for a 4095-bit modulus
WS, WS2 = W * S, 26 * 162  # level-1 and reduction-tree Montgomery exponents


def limbs(x):
    return [(x >> (W * i)) & ((1 << W) - 1) for i in range(S2)]


def from_limbs(ws):
    return sum(int(w) << (W * i) for i, w in enumerate(ws[:S2]))


def pow2(e, N):
    return pow(2, e, N) if e >= 0 else pow((N + 1) // 2, -e, N)


def partial(xs, N, G):
    """What dds_col_fold_partial returns for rows xs folded by G first-level groups."""
    import numpy as np
    E = WS * (G - len(xs)) - WS2 * (G - 1)
    prod = 1
    for x in xs:
        prod = prod * x % N
    v = prod * pow2(E, N) % N
    words = limbs(v) + [E & 0xFFFFFFFF, (E >> 32) & 0xFFFFFFFF]
    return np.array(words, dtype=np.uint32)


def combine(parts, N):
    """dds_combine_partials: tail-shape tree over the partials, then finalize."""
    n = len(parts)
    E = -WS2 * (n - 1)
    acc = None
    for p in parts:
        e = int(p[S2]) | (int(p[S2 + 1]) << 32)
        if e >= 1 << 63:
            e -= 1 << 64
        E += e
        v = from_limbs(p)
        acc = v if acc is None else acc * v * pow2(-WS2, N) % N
    return acc * pow2(WS2 - E, N) * pow2(-WS2, N) % N


def _worker(rank, world, port, N, xs, out_q):
    import numpy as np
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import ddshe.dist as dd
    row0, cnt = dd.shard_range(len(xs), world, rank)
    part = partial(xs[row0:row0 + cnt], N, G=max(1, cnt // 2) if rank == 0 else 3)
    parts, rows = dd.gather_partials(part, cnt)
    if rank == 0:
        out_q.put((combine(list(parts), N), int(rows.sum())))
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
