#!/usr/bin/env python3
"""Headline benchmark: Paillier homomorphic adds/sec (2048-bit key, mod n^2) — BASELINE.json.

A "step" is one SumAll HomoAdd fold (DDSRestServer.scala:412-430) over the whole
device-resident ciphertext column: k = --rows synthetic Paillier ciphertexts under the
reference's committed 2048-bit key (client.conf:85; n^2 = 4095 bits), sharded by row
range over the ranks. Each rank folds its shard to one partial on its GPU; for N > 1
the partials (608 B each) are gathered over RCCL and combined on rank 0's GPU.
value = (k - 1) HomoAdd operations per step * steps / (max-over-ranks wall time).

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under
torch.distributed.run (one process per GPU).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "dependable-data-storage-csd2017_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

S_32 = 128                      # 32-bit limbs of the 4096-bit modulus
MAC_PER_MODMUL = 2 * S_32 * S_32 + S_32   # algorithmic 32x32->64 MACs per modmul (CIOS)
# integer-VALU peak: v_mad_u64_u32 issues at half rate (measured: same rate as v_fma_f64,
# tools/microbench/ubench.hip) = 64 lane-ops/clk/CU x 256 CU x 2.4 GHz
PEAK_TMAC = 64 * 256 * 2.4e9 / 1e12


def load_key():
    raw = json.load(open(os.path.join(ROOT, "tests", "golden", "keys.json")))
    return {k: int(v, 16) for k, v in raw["paillier2048_committed"].items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows", type=int, default=10_000_000,
                    help="ciphertexts per rank per step (weak scaling); whole job with --strong")
    ap.add_argument("--strong", action="store_true", help="split --rows over the ranks instead")
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--pool", type=int, default=1024)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (rank 0, N=1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify", type=int, default=1, help="check Dec(result) == sum(m) on rank 0")
    args = ap.parse_args()

    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)

    import ddshe
    import ddshe.dist as ddist

    key = load_key()
    nsq = key["nsquare"]
    eng = ddshe.Engine(local)
    stream = torch.cuda.current_stream()
    eng.set_stream(stream.cuda_stream)

    # shard rows by contiguous key range; weak scaling: each rank owns --rows rows
    total = args.rows if args.strong else args.rows * world
    row0, mine = ddist.shard_range(total, world, rank)
    per = (total + world - 1) // world
    col = eng.column(nsq, max(1, mine))
    t_fill = time.time()
    if mine:
        col.fill_paillier_synth(key["n"], key["g"], args.seed, row0, mine, args.pool)
    torch.cuda.synchronize()
    t_fill = time.time() - t_fill

    mb = (nsq.bit_length() + 7) // 8

    def step():
        if world == 1:
            return col.fold()
        part, rows = col.fold_partial()
        parts, rows_all = ddist.gather_partials(part, rows, device=torch.device("cuda", local))
        if rank != 0:
            return None
        return eng.combine_partials(nsq, parts, rows_all)

    for _ in range(args.warmup):
        res = step()
    eng.set_timing(True)
    eng.reset_timing()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    eng.set_timing(False)
    fold_ms, fold_launches, _, fold_modmuls = eng.timing()
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    out = None
    if rank == 0:
        ok = None
        if args.verify:
            from oracle import homo  # checker only
            ms = ddshe.synth_plaintexts(args.seed, 0, total)
            ok = homo.paillier_decrypt(res, key) == int(ms.astype(np.int64).sum()) % key["n"]
            if not ok:
                print("VERIFY FAILED: Dec(fold) != sum(m)", file=sys.stderr)
        adds = (total - 1) * args.steps
        value = adds / elapsed
        avg_launch_s = fold_ms / max(1, fold_launches) / 1e3
        per_launch_mac = fold_modmuls / max(1, fold_launches) * MAC_PER_MODMUL
        achieved = per_launch_mac / avg_launch_s / 1e12 if fold_launches else None
        traffic = None
        tf = os.path.join(ROOT, "profiles", "r01_pmc_traffic.json")
        if os.path.exists(tf):  # HBM bytes per launch from the committed rocprofv3 PMC passes, per row
            pm = json.load(open(tf))
            traffic = pm["hbm_bytes_per_launch"] / pm["rows_per_launch"] * mine  # the launch reads every row once
        roofline = {
            "bound": "valu-int",
            "kernel": "k_fold<152,4> (first fold level over the rows)",
            "achieved": achieved, "peak": PEAK_TMAC, "unit": "TMAC/s",
            "frac": (achieved / PEAK_TMAC) if achieved else None,
            "traffic": traffic, "traffic_unit": "bytes/launch (PMC, profiles/r01_pmc_traffic.json)",
            "avg_launch_ms": avg_launch_s * 1e3,
            "modmuls_per_launch": fold_modmuls / max(1, fold_launches),
            "mac_per_modmul": MAC_PER_MODMUL,
        }
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(col, nsq, mb, args.cpu_seconds)
        out = {
            "metric": "Paillier homomorphic adds/sec (2048-bit key, mod n^2)",
            "value": value, "unit": "HomoAdd/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None, "dtype": "u32", "data": "synthetic (seeded Paillier ciphertexts, committed key)",
            "config": {"workload": "paillier_sumall_fold_10M_2048bit", "rows": total, "rows_per_gpu": per, "key_bits": key["n"].bit_length(),
                       "modulus_bits": nsq.bit_length(), "parallelism": f"rows-sharded x{world}",
                       "global_batch": total, "seq_len": None, "model": None},
            "roofline": roofline, "cpu_baseline": cpu, "verified": ok, "fill_s": t_fill,
        }
        print(json.dumps(out))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    col.close()
    eng.close()
    return out


def cpu_baseline(col, nsq, mb, seconds):
    """Reference fold restated in C (oracle/csrc/fold_ref.c: BigInteger multiply+mod),
    1 thread, on a bounded prefix of the same column; also checks the GPU on that prefix."""
    from oracle import cref
    calib = min(len(col), 2000)
    ops = b"".join(x.to_bytes(mb, "big") for x in col.read(0, calib))
    mod_be = nsq.to_bytes(mb, "big")
    t = time.perf_counter()
    cref.fold_be(mod_be, ops, mb, calib)
    rate = (calib - 1) / (time.perf_counter() - t)
    sample = int(min(len(col), max(calib, rate * seconds)))
    ops = b"".join(x.to_bytes(mb, "big") for x in col.read(0, sample))
    t = time.perf_counter()
    ref = cref.fold_be(mod_be, ops, mb, sample)
    dt = time.perf_counter() - t
    gpu = col.fold(0, sample)
    return {"value": (sample - 1) / dt, "unit": "HomoAdd/s", "cores": 1, "kind": "port",
            "sample": f"first {sample} rows of the same column, acc=acc*x mod n^2 (schoolbook+Knuth D), {dt:.1f}s",
            "gpu_matches_sample": gpu == int.from_bytes(ref, "big")}


if __name__ == "__main__":
    main()
