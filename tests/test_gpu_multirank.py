"""Multi-process fold on the GPU: two ranks share cuda:0, each folds its
contiguous key range to a partial with dds_col_fold_partial, the partials travel through
one all-gather (gloo here: RCCL refuses two ranks on one device; the driver's multi-GPU
bench uses RCCL over xGMI) and rank 0 combines them with dds_combine_partials. The result
must equal the single-rank fold bit for bit (modular product: any partition, same residue)."""
import os
import random

import pytest
import torch.multiprocessing as mp

from oracle import homo

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dependable-data-storage-csd2017_amd")


def _worker(rank, world, port, N, xs, out_q):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import ddshe
    import ddshe.dist as dd
    eng = ddshe.Engine(0)
    row0, cnt = dd.shard_range(len(xs), world, rank)
    col = eng.column(N, max(1, cnt))
    col.append(xs[row0:row0 + cnt])
    part, rows = col.fold_partial(0, cnt)
    parts, rows_all = dd.gather_partials(part, rows)
    if rank == 0:
        out_q.put((eng.combine_partials(N, parts, rows_all), int(rows_all.sum())))
    col.close()
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("name,k,world", [("paillier2048_committed", 1001, 2),
                                          ("paillier1024_seed1", 4099, 3),
                                          ("rsa2048_seed3", 513, 2)])
def test_multirank_fold_matches_single(keys, name, k, world):
    key = keys[name]
    N = key["nsquare"] if "nsquare" in key else key["n"]
    rng = random.Random(k)
    xs = [rng.randrange(N) for _ in range(k)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30500 + rng.randrange(1000)
    procs = [ctx.Process(target=_worker, args=(r, world, port, N, xs, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res, rows = q.get(timeout=100)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert rows == k
    assert res == homo.modmul_fold(xs, N)


def _worker_fill(rank, world, port, N, total, seed, out_q):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import ddshe
    import ddshe.dist as dd
    eng = ddshe.Engine(0)
    row0, cnt = dd.shard_range(total, world, rank)
    col = eng.column(N, max(1, cnt))
    col.fill_random(2040, seed, row0, cnt)  # rows depend on their global index: shards = slices of one column
    part, rows = col.fold_partial(0, cnt)
    parts, rows_all = dd.gather_partials(part, rows)
    if rank == 0:
        out_q.put((eng.combine_partials(N, parts, rows_all), int(rows_all.sum())))
    col.close()
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


def test_multirank_partials_from_lane_folds(eng, keys):
    """Ranks whose shards take the one-bignum-per-lane MultAll fold (k_fold1: >= ~1M rows each, 74-limb
    partial exponent): the combined result equals the single-process fold of the whole column."""
    N = keys["rsa2048_seed3"]["n"]
    total, seed = 2_400_000, 44
    col = eng.column(N, total)
    col.fill_random(2040, seed, 0, total)
    want = col.fold()
    col.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31600 + random.Random(seed).randrange(1000)
    procs = [ctx.Process(target=_worker_fill, args=(r, 2, port, N, total, seed, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res, rows = q.get(timeout=100)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert rows == total
    assert res == want
