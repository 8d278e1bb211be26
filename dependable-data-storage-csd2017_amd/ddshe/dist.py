"""Multi-GPU orchestration of the fold: rows sharded by contiguous key range, one
partial per rank, partials gathered to rank 0 and combined there.
(One process driving all GPUs uses the C-ABI's dds_mctx instead: ddshe.MultiEngine.)

Each rank's partial is the un-finalised Montgomery fold of its shard,
v(S) = prod(S) * R^(1-|S|) mod N (S r27 words), plus its row count. Modular product
is not an RCCL reduction op, so the only collective is one all-gather of
(S + 2) 32-bit words per rank (608 B + 8 B at a 2048-bit Paillier key); the G
partials are then folded on rank 0's GPU by dds_combine_partials.
"""
from __future__ import annotations

import numpy as np


def shard_range(total: int, world: int, rank: int):
    """Contiguous row range [row0, row0+count) owned by `rank`."""
    per = (total + world - 1) // world
    row0 = min(total, rank * per)
    return row0, max(0, min(per, total - row0))


def pack_partial(part: np.ndarray, rows: int) -> np.ndarray:
    part = np.ascontiguousarray(part, dtype=np.uint32)
    return np.concatenate([part, np.array([rows & 0xFFFFFFFF, rows >> 32], dtype=np.uint32)])


def unpack_partials(mat: np.ndarray):
    mat = np.ascontiguousarray(mat).view(np.uint32)
    rows = mat[:, -2].astype(np.uint64) | (mat[:, -1].astype(np.uint64) << np.uint64(32))
    return np.ascontiguousarray(mat[:, :-2]), rows


def gather_partials(part: np.ndarray, rows: int, device=None, group=None):
    """All-gather every rank's (partial, rows). Returns (partials[world, S], rows[world])
    on every rank. `device` is the tensor device of the backend (cuda for RCCL, cpu for gloo)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    t = torch.from_numpy(pack_partial(part, rows).view(np.int32))
    if device is not None:
        t = t.to(device)
    bufs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(bufs, t, group=group)
    mat = torch.stack(bufs).cpu().numpy()
    return unpack_partials(mat)


def gather_partials_device(col, first: int, count: int, coll_dev, group=None):
    """Device-to-device form: this rank's partial is folded straight into a device tensor
    (dds_col_fold_partial_device), all-gathered (RCCL over xGMI when coll_dev is a GPU; the gloo
    rehearsal stages through host memory) and returned as one device tensor of world x partial_words
    words on this rank's GPU, ready for Engine.combine_partials_device. No host staging of the limbs
    on the RCCL path."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    pw = col.partial_words
    part = torch.empty(pw, dtype=torch.int32, device="cuda")
    col.fold_partial_device(part.data_ptr(), first, count)
    src = part if coll_dev.type == "cuda" else part.cpu()
    out = torch.empty(world * pw, dtype=torch.int32, device=src.device)
    dist.all_gather_into_tensor(out, src, group=group)
    return out if out.is_cuda else out.to("cuda")
