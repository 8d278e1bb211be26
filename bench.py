#!/usr/bin/env python3
"""Headline benchmark: Paillier homomorphic adds/sec (2048-bit key, mod n^2) — BASELINE.json.

A "step" is one SumAll HomoAdd fold (DDSRestServer.scala:412-430) over the whole
device-resident ciphertext column: k = --rows synthetic Paillier ciphertexts under the
reference's committed 2048-bit key (client.conf:85; n^2 = 4095 bits), sharded by row
range over the ranks. Each rank folds its shard to one partial on its GPU; for N > 1
the partials (608 B each) are gathered over RCCL and combined on rank 0's GPU.
value = (k - 1) HomoAdd operations per step * steps / (max-over-ranks wall time).

Launch: python bench.py [--gpus N --steps K --warmup W]. For N > 1 either under
torch.distributed.run (one process per GPU, WORLD_SIZE = N), or directly: without WORLD_SIZE the
process starts N ranks itself (a torch.distributed.run child, before any GPU call), relays rank
0's JSON line and exits with the child's status. Fewer than N visible devices is an error
(exit 2), never a silent one-GPU line; DDSHE_DIST_BACKEND=gloo rehearses N ranks on one device.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
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


def window_counts(e: int):
    """(squarings, multiplies, table products) of the engine's sliding-window schedule for a
    uniform exponent e (mirror of window_schedule in ddshe_capi.cpp)."""
    nb = e.bit_length()
    if nb == 0:
        return 0, 0, 0
    w = 1 if nb <= 24 else 3 if nb <= 80 else 4 if nb <= 240 else 5
    i, sq, mul = nb - 1, 0, 0
    first = True
    while i >= 0:
        if not (e >> i) & 1:
            sq, i = sq + 1, i - 1
            continue
        j = max(i - w + 1, 0)
        while not (e >> j) & 1:
            j += 1
        if not first:
            sq, mul = sq + i - j + 1, mul + 1
        first, i = False, j - 1
    table = 1 + (1 if w > 1 else 0) + (2 ** (w - 1) - 1)  # x*R, x^2, odd powers
    return sq, mul, table


def binary_ladder_modmuls(e: int, m_bits: int = 14) -> int:
    """SURVEY.md §8d work unit of one encryption: left-to-right binary modexp of r^n and g^m."""
    return (e.bit_length() - 1) + (m_bits - 1) + (bin(e).count("1") - 1) + (m_bits // 2 - 1) + 1


def visible_devices() -> int:
    """GPUs this process can see. torch.cuda.device_count() counts them without initialising HIP on
    this image, so the launcher may call it before it starts the ranks."""
    import torch
    return torch.cuda.device_count()


def launch_ranks(n: int, backend: str) -> int:
    """`python bench.py --gpus N` without WORLD_SIZE: run the N ranks as one torch.distributed.run
    child (127.0.0.1 rendezvous on a free port, the same command line otherwise), relay rank 0's JSON
    line after checking it reports n_gpus == N, and return the child's exit status (non-zero when any
    rank failed). The parent makes no GPU call and never exec()s."""
    import socket
    import subprocess
    have = visible_devices()
    need = n if backend == "nccl" else 1
    if have < need:
        print(f"bench.py: --gpus {n} needs {need} visible GPU(s) for the {backend} backend, found {have}; "
              "refusing to report a smaller run", file=sys.stderr)
        return 2
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this pool (RCCL peer buffers)
    env.setdefault("OMP_NUM_THREADS", "1")
    child = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    lines = []
    for line in child.stdout:  # ranks' other output passes through to stderr as it comes
        if line.lstrip().startswith("{"):
            lines.append(line.strip())
        else:
            sys.stderr.write(line)
            sys.stderr.flush()
    rc = child.wait()
    if rc != 0:
        print(f"bench.py: ranks exited with status {rc}", file=sys.stderr)
        return rc
    if len(lines) != 1:
        print(f"bench.py: expected one JSON line from rank 0, got {len(lines)}", file=sys.stderr)
        return 3
    if json.loads(lines[0]).get("n_gpus") != n:
        print(f"bench.py: rank 0 reported n_gpus != {n}", file=sys.stderr)
        return 3
    print(lines[0], flush=True)
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); default WORLD_SIZE under torch.distributed.run, else 1")
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--workload", choices=("sum", "product_filter", "encrypt_sum", "order", "entry_search"),
                    default="sum",
                    help="sum: BASELINE.json config 2 (headline); product_filter: config 3; encrypt_sum: config 4; "
                         "order: OrderLS over the config-3 OPE column (SURVEY.md §8f rank 2); "
                         "entry_search: SearchEntryOR + SearchEq over a string table (§8f rank 3)")
    ap.add_argument("--rows", type=int, default=None,
                    help="rows per rank per step (weak scaling); whole job with --strong")
    ap.add_argument("--strong", action="store_true", help="split --rows over the ranks instead")
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--pool", type=int, default=1024)
    ap.add_argument("--public", action="store_true", help="encrypt_sum: public-key path (no CRT)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (rank 0, N=1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="sum: skip the host-boundary (PCIe/decimal) rates")
    ap.add_argument("--e2e-dec-rows", type=int, default=1_000_000, help="sum: decimal-route sample rows")
    ap.add_argument("--verify", type=int, default=1, help="check the result on rank 0")
    ap.add_argument("--no-extras", action="store_true",
                    help="sum: skip the extra lines (configs 3 and 4, latency, strong scaling, one-process multi-GPU)")
    ap.add_argument("--strong-rows", type=int, default=10_000_000,
                    help="rows of the strong-scaling and one-process multi-GPU lines (the north-star config)")
    args = ap.parse_args()
    dflt = {"sum": (10_000_000, 20, 3, 2), "product_filter": (10_000_000, 10, 5, 3),
            "encrypt_sum": (1_000_000, 2, 1, 4), "order": (10_000_000, 10, 2, 3),
            "entry_search": (10_000_000, 10, 2, 5)}[args.workload]
    args.rows = dflt[0] if args.rows is None else args.rows
    args.steps = dflt[1] if args.steps is None else args.steps
    args.warmup = dflt[2] if args.warmup is None else args.warmup
    args.seed = dflt[3] if args.seed is None else args.seed
    # DDSHE_DIST_BACKEND=gloo rehearses the N > 1 flow with every rank on one GPU (the partial
    # gather then goes through host memory); the driver's multi-GPU runs use RCCL ("nccl").
    backend = os.environ.get("DDSHE_DIST_BACKEND", "nccl")
    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus is None:
        args.gpus = int(env_world) if env_world else 1
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if env_world is None and args.gpus > 1:
        return launch_ranks(args.gpus, backend)
    if env_world is not None and int(env_world) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}", file=sys.stderr)
        return 2

    import torch
    import torch.distributed as dist

    world = args.gpus
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    devices = visible_devices()
    if backend == "gloo":
        if devices < 1:
            print("bench.py: no visible GPU", file=sys.stderr)
            return 2
        local = local % devices
    elif devices <= local:
        print(f"bench.py: rank {rank} needs device {local}, {devices} visible", file=sys.stderr)
        return 2
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(local)
    coll_dev = torch.device("cuda", local) if backend == "nccl" else torch.device("cpu")

    import ddshe
    import ddshe.dist as ddist

    eng = ddshe.Engine(local)
    stream = torch.cuda.current_stream()
    eng.set_stream(stream.cuda_stream)

    # shard rows by contiguous key range; weak scaling: each rank owns --rows rows
    total = args.rows if args.strong else args.rows * world
    row0, mine = ddist.shard_range(total, world, rank)
    ctx = dict(args=args, coll_dev=coll_dev, eng=eng, world=world, rank=rank, local=local, total=total, row0=row0, mine=mine,
               per=(total + world - 1) // world, torch=torch, ddshe=ddshe, ddist=ddist)
    wl = {"sum": SumWorkload, "product_filter": ProductFilterWorkload, "encrypt_sum": EncryptSumWorkload,
          "order": OrderWorkload, "entry_search": EntrySearchWorkload}[args.workload](ctx)
    t_fill = time.time()
    wl.setup()
    torch.cuda.synchronize()
    t_fill = time.time() - t_fill

    for _ in range(args.warmup):
        res = wl.step()
    eng.set_timing(True)
    eng.reset_timing()
    wl.reset_timers()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = wl.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    eng.set_timing(False)
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    # every rank's own check of its shard (N > 1, whatever --no-extras says), then the extra lines
    # measured by every rank together (collectives inside), before rank 0 reports
    wl.last_res = res
    ranks_ok = wl.verify_distributed() if world > 1 and args.verify else None
    extra = wl.extra_distributed() if not args.no_extras else {}
    out = None
    if rank == 0:
        out = wl.report(res, elapsed)
        out["fill_s"] = t_fill
        if ranks_ok is not None:
            out["verified"] = ranks_ok if out.get("verified") is None else bool(out["verified"] and ranks_ok)
        out["config"]["distinct_devices"] = min(world, devices)
        if backend == "gloo" and world > 1:
            out["config"]["note"] = f"gloo rehearsal: {world} ranks on {min(world, devices)} device(s)"
        out.update(extra)
    wl.close()
    if not args.no_extras:
        if rank == 0:
            try:  # extra lines never cost the headline line (nor leave the other ranks in the barrier)
                out.update(wl.extra_rank0())
            except Exception as e:  # noqa: BLE001
                import traceback
                out["extras_error"] = f"{type(e).__name__}: {e}"
                out["extras_traceback"] = traceback.format_exc()[-1500:]
        if world > 1:
            dist.barrier()
    if rank == 0:
        assert out["n_gpus"] == args.gpus, (out["n_gpus"], args.gpus)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    eng.close()
    return 0


class _Workload:
    def __init__(self, ctx):
        self.__dict__.update(ctx)

    def reset_timers(self):
        pass

    def strong_split_line(self, full, parts=8):
        """The 8-GPU strong split stated on one GPU: one rank's share (rows/8) folded to a device partial
        (dds_col_fold_partial_device) and the combine of 8 such partials (dds_combine_partials_device) timed
        separately; the 8 partials cover all rows, so the combine must equal the full fold."""
        torch = self.torch
        pw = self.col.partial_words
        cnt = self.mine // parts
        buf = torch.empty(parts * pw, dtype=torch.int32, device="cuda")

        def fold_share(i):
            self.col.fold_partial_device(buf.data_ptr() + 4 * i * pw, i * cnt, cnt)
            torch.cuda.synchronize()

        def med(fn, reps=9):
            ts = []
            for _ in range(reps):
                t = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t)
            return sorted(ts)[reps // 2] * 1e3
        for i in range(parts):
            fold_share(i)
        share_ms = med(lambda: fold_share(0))
        # the share's first level alone (HIP events around its k_fold launch): the rest of share_ms is
        # its tail (reduction of the level-1 partials to one device partial) plus the host call
        self.eng.set_timing(True)
        self.eng.reset_timing()
        for _ in range(5):
            fold_share(0)
        lvl_ms, lvl_n, _, _ = self.eng.timing()
        self.eng.set_timing(False)
        level1_ms = lvl_ms / lvl_n if lvl_n else None
        rows = [cnt] * parts
        got = self.eng.combine_partials_device(self.nsq, buf.data_ptr(), rows)
        comb_ms = med(lambda: self.eng.combine_partials_device(self.nsq, buf.data_ptr(), rows))
        tail_ms = share_ms - level1_ms if level1_ms else None
        return {"rows_per_share": cnt, "shares": parts, "share_fold_partial_ms": share_ms,
                "share_level1_ms": level1_ms, "share_fold_tail_ms": tail_ms,
                "combine_ms": comb_ms, "combined_equals_full_fold": got == full if cnt * parts == self.mine else None,
                "tail_plus_combine_share": (tail_ms + comb_ms) / (share_ms + comb_ms) if tail_ms else None,
                "note": "an 8-GPU strong-split step is about share_fold_partial_ms + one all-gather of "
                        f"{parts}x{4 * pw} B + combine_ms (host wall clock, each call synchronised)"}

    def verify_distributed(self):
        """N > 1 and --verify: each rank's check of its own shard, min over ranks (collective: every
        rank calls it); None where rank 0's report verifies the combined result instead."""
        return None

    def extra_distributed(self):
        return {}

    def extra_rank0(self):
        return {}

    def all_ranks_ok(self, ok):
        """N > 1: every rank's own check (its shard's result against its host restatement), min over ranks."""
        import torch.distributed as dist
        t = self.torch.tensor([1 if ok else 0], dtype=self.torch.int32, device=self.coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    def fold_or_combine(self, col, modulus, count=None, rows_all=None):
        """One SumAll/MultAll fold over this rank's rows [0, count); N > 1: the partial is folded into a
        device tensor, all-gathered device-to-device (RCCL over xGMI) and combined on rank 0's GPU."""
        count = len(col) if count is None else count
        if self.world == 1:
            return col.fold(0, count)
        gathered = self.ddist.gather_partials_device(col, 0, count, self.coll_dev)
        if self.rank != 0:
            return None
        rows_all = rows_all if rows_all is not None else [self.per] * self.world
        return self.eng.combine_partials_device(modulus, gathered.data_ptr(), rows_all)

    def timed(self, step, steps, warmup):
        """warmup + `steps` timed calls of step() bracketed by barrier + sync; max over ranks."""
        torch = self.torch
        import torch.distributed as dist
        for _ in range(warmup):
            res = step()
        if self.world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            res = step()
        torch.cuda.synchronize()
        if self.world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if self.world > 1:
            tt = torch.tensor([el], dtype=torch.float64, device=self.coll_dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = float(tt.item())
        return res, el

    def fold_roofline(self, s32):
        """Dominant kernel (first fold level) from HIP events on its launch stream."""
        fold_ms, fold_launches, _, fold_modmuls = self.eng.timing()
        mac = 2 * s32 * s32 + s32
        avg_launch_s = fold_ms / max(1, fold_launches) / 1e3
        per_launch_mac = fold_modmuls / max(1, fold_launches) * mac
        achieved = per_launch_mac / avg_launch_s / 1e12 if fold_launches else None
        return {"bound": "valu-int", "achieved": achieved, "peak": PEAK_TMAC, "unit": "TMAC/s",
                "frac": (achieved / PEAK_TMAC) if achieved else None, "avg_launch_ms": avg_launch_s * 1e3,
                "modmuls_per_launch": fold_modmuls / max(1, fold_launches), "mac_per_modmul": mac}

    def common(self, metric, value, unit, elapsed, workload, extra_cfg):
        a = self.args
        return {
            "metric": metric, "value": value, "unit": unit, "n_gpus": self.world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": elapsed / a.steps * 1e3, "higher_is_better": True,
            "scaling": "strong" if a.strong else "weak", "vs_baseline": None, "dtype": "u32",
            "config": dict({"workload": workload, "rows": self.total, "rows_per_gpu": self.per,
                            "parallelism": f"rows-sharded x{self.world}", "global_batch": self.total,
                            "seq_len": None, "model": None}, **extra_cfg),
        }

    def close(self):
        pass


class SumWorkload(_Workload):
    """BASELINE.json config 2 (headline): SumAll HomoAdd fold over 10M ciphertexts, committed 2048-bit key."""

    def setup(self):
        self.key = load_key()
        self.nsq = self.key["nsquare"]
        self.col = self.eng.column(self.nsq, max(1, self.mine))
        if self.mine:
            self.col.fill_paillier_synth(self.key["n"], self.key["g"], self.args.seed, self.row0, self.mine,
                                         self.args.pool)
        self.col_sample = self.col.read(0, min(self.mine, 256)) if self.mine else []

    def step(self):
        return self.fold_or_combine(self.col, self.nsq)

    def report(self, res, elapsed):
        a, key, nsq = self.args, self.key, self.nsq
        ok = None
        if a.verify:
            from oracle import homo  # checker only
            ms = self.ddshe.synth_plaintexts(a.seed, 0, self.total)
            ok = homo.paillier_decrypt(res, key) == int(ms.astype("int64").sum()) % key["n"]
            if not ok:
                print("VERIFY FAILED: Dec(fold) != sum(m)", file=sys.stderr)
        roof = self.fold_roofline(S_32)
        roof["kernel"] = "k_fold<148,4,28> (first fold level over the rows)"
        # HBM bytes per launch from the committed rocprofv3 PMC passes of this kernel (10M rows, each read once)
        traffic = pmc_traffic("sum", ("k_fold<148, 4, 28, true, false, false>",), largest=True)
        if traffic is not None:
            traffic *= self.mine / 1e7
        roof.update(traffic=traffic, traffic_unit=f"HBM bytes per launch (PMC, profiles/{PMC_FILE})")
        vp = valu_pmc(("r06_pmc_valu_fold.json", "r04_pmc_valu_fold.json", "r03_pmc_valu_fold.json"))
        if vp:  # rocprofv3 VALU counters of the same kernel (north star: VALU-roofline fraction)
            roof["valu_pmc"] = vp
        cpu = None
        if self.world == 1 and not a.no_cpu_baseline:
            cpu = cpu_baseline(self.col, nsq, (nsq.bit_length() + 7) // 8, a.cpu_seconds)
        e2e = None
        if self.world == 1 and not a.no_e2e:
            e2e = self.end_to_end(res)
        split = self.strong_split_line(res) if self.world == 1 and not a.no_extras else None
        out = self.common("Paillier homomorphic adds/sec (2048-bit key, mod n^2)",
                          (self.total - 1) * a.steps / elapsed, "HomoAdd/s", elapsed,
                          "paillier_sumall_fold_10M_2048bit",
                          {"key_bits": key["n"].bit_length(), "modulus_bits": nsq.bit_length()})
        out.update(data="synthetic (seeded Paillier ciphertexts, committed key)", roofline=roof, cpu_baseline=cpu,
                   end_to_end=e2e, verified=ok, strong_split_1gpu=split,
                   fold_tail_ms=elapsed / a.steps * 1e3 - roof["avg_launch_ms"] if roof["achieved"] else None)
        return out

    def extra_distributed(self):
        """N > 1: the strong-scaling line of the north-star config — args.strong_rows rows over all
        ranks (each folds the first shard_range rows of its resident column), partials moved
        device-to-device and combined on rank 0's GPU."""
        if self.world == 1:
            return {}
        a = self.args
        cnts = [self.ddist.shard_range(a.strong_rows, self.world, r)[1] for r in range(self.world)]
        if max(cnts) > self.mine:
            return {"strong": {"skipped": "fewer resident rows per rank than the strong shard"}}
        res, el = self.timed(lambda: self.fold_or_combine(self.col, self.nsq, cnts[self.rank], cnts), a.steps,
                             a.warmup)
        if self.rank != 0:
            return {}
        ok = None
        if a.verify:
            from oracle import homo  # checker only
            ms = sum(int(self.ddshe.synth_plaintexts(a.seed, r * self.per, c).astype("int64").sum())
                     for r, c in enumerate(cnts))
            ok = homo.paillier_decrypt(res, self.key) == ms % self.key["n"]
        return {"strong": {"metric": "Paillier homomorphic adds/sec (2048-bit key, mod n^2), strong scaling",
                           "value": (a.strong_rows - 1) * a.steps / el, "unit": "HomoAdd/s", "n_gpus": self.world,
                           "rows": a.strong_rows, "steps": a.steps, "ms_per_step": el / a.steps * 1e3,
                           "scaling": "strong", "verified": ok,
                           "partials": "dds_col_fold_partial_device -> all_gather_into_tensor ("
                                       + ("RCCL, device to device" if self.coll_dev.type == "cuda" else
                                          "gloo rehearsal, staged through host memory")
                                       + ") -> dds_combine_partials_device"}}

    def extra_rank0(self):
        out = {"single_process_multi_gpu": self.single_process_line()}
        if self.world == 1:
            out["latency"] = self.latency_lines()
            out["configs"] = run_extra_configs(self)
        return out

    def single_process_line(self):
        """One process drives all N GPUs through the C-ABI's multi-device context (dds_mctx: the form
        a JNA caller uses): args.strong_rows rows sharded in 64-row blocks, every shard folded on its
        own GPU, partials copied device-to-device (xGMI peer copies) and combined on GPU 0."""
        a, torch = self.args, self.torch
        if torch.cuda.device_count() < a.gpus:
            return {"skipped": f"{torch.cuda.device_count()} visible devices < {a.gpus}"}
        k, rows = self.key, a.strong_rows
        m = self.ddshe.MultiEngine(list(range(a.gpus)))
        col = m.column(self.nsq, rows)
        col.fill_paillier_synth(k["n"], k["g"], a.seed, rows, a.pool)
        for _ in range(a.warmup):
            res = col.fold()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            res = col.fold()
        el = time.perf_counter() - t0
        ok = None
        if a.verify:
            from oracle import homo  # checker only
            ms = self.ddshe.synth_plaintexts(a.seed, 0, rows)
            ok = homo.paillier_decrypt(res, k) == int(ms.astype("int64").sum()) % k["n"]
        col.close()
        m.close()
        return {"metric": "Paillier homomorphic adds/sec (2048-bit key, mod n^2), one process, all GPUs",
                "value": (rows - 1) * a.steps / el, "unit": "HomoAdd/s", "n_gpus": a.gpus, "rows": rows,
                "steps": a.steps, "ms_per_step": el / a.steps * 1e3, "scaling": "strong", "verified": ok,
                "path": "dds_mcol_fold: shard folds on their GPUs, hipMemcpyPeerAsync of the partials, combine on GPU 0"}

    def latency_lines(self):
        """Request latency (host wall clock per call, inputs resident / as the route holds them):
        BASELINE.json config 1 (SumAll over 10k ciphertexts, 1024-bit key) through the resident column
        and the decimal route entry point, the reference path (OpenSSL BN_mod_mul fold, 1 core) on the
        same rows, and the pairwise /Sum route (DDSRestServer.scala:355-395) on the committed key."""
        import numpy as np
        from oracle import cref  # CPU reference timing only
        eng = self.eng
        k1 = load_keyset("paillier1024_seed1")
        nsq1 = k1["nsquare"]
        col = eng.column(nsq1, 10000)
        col.fill_paillier_synth(k1["n"], k1["g"], 1, 0, 10000, 64)

        def med(fn, reps):
            ts = []
            for _ in range(reps):
                t = time.perf_counter()
                r = fn()
                ts.append(time.perf_counter() - t)
            ts.sort()
            return r, ts[len(ts) // 2] * 1e3, ts[int(len(ts) * 0.99)] * 1e3

        eng.set_stream(None)  # latency of the engine's own streams (no torch stream sync in the call)
        col.fold()
        gpu, fold_ms, fold_p99 = med(col.fold, 50)
        # the same call at the C-ABI with its arguments built once (what a JNA binding does per request)
        import ctypes as C
        fout = (C.c_uint8 * (col.mb + 4096))()
        flen = C.c_size_t()
        fold_c = self.ddshe._lib.dds_col_fold

        def c_fold():
            st = fold_c(col._h, 0, 10000, fout, len(fout), C.byref(flen))
            assert st == 0, st
            return flen.value
        _, fold_c_ms, fold_c_p99 = med(c_fold, 50)
        assert int.from_bytes(bytes(fout[: flen.value]), "big") == gpu

        def cpu_per_fold(c, count, reps):
            """host CPU of the calling thread (thread clock) and wall time per dds_col_fold, timing off"""
            out, ln = (C.c_uint8 * (c.mb + 4096))(), C.c_size_t()
            st = fold_c(c._h, 0, count, out, len(out), C.byref(ln))
            assert st == 0, (count, st, self.ddshe._lib.dds_last_error())
            cs, ws = [], []
            for _ in range(reps):
                c0, w0 = time.thread_time(), time.perf_counter()
                st = fold_c(c._h, 0, count, out, len(out), C.byref(ln))
                assert st == 0, (count, st)
                cs.append(time.thread_time() - c0)
                ws.append(time.perf_counter() - w0)
            cs.sort()
            ws.sort()
            return {"rows": count, "host_cpu_ms": cs[len(cs) // 2] * 1e3, "wall_ms": ws[len(ws) // 2] * 1e3}
        host_cpu = [cpu_per_fold(col, 10000, 50)]
        big_rows = min(self.args.rows, 10_000_000)  # the headline column is closed by now: a fresh one
        big = eng.column(self.nsq, big_rows)
        big.fill_paillier_synth(self.key["n"], self.key["g"], self.args.seed, 0, big_rows, self.args.pool)
        for cnt, reps in ((1_000_000, 10), (10_000_000, 5)):
            if big_rows >= cnt:
                host_cpu.append(cpu_per_fold(big, cnt, reps))
        big.close()
        rows = [str(x) for x in col.read(0, 10000)]
        # the C entry point a JNA binding calls with its String[] (marshalling of the Python strings done once,
        # outside the timed call: the JVM hands over its strings as they are)
        arr = (C.c_char_p * len(rows))(*[r.encode() for r in rows])
        cap = sum(len(r) for r in rows) * 2 + 64
        obuf, olen, modb = C.create_string_buffer(cap), C.c_size_t(), str(nsq1).encode()

        def dec_call():
            st = self.ddshe._lib.dds_sum_all_dec(eng._h, arr, len(rows), modb, obuf, cap, C.byref(olen))
            assert st == 0, st
            return obuf.value.decode()
        dec, dec_ms, _ = med(dec_call, 20)
        dec_py, dec_py_ms, _ = med(lambda: eng.sum_all_dec(rows, str(nsq1)), 5)
        assert dec_py == dec
        mb = (nsq1.bit_length() + 7) // 8
        buf = col.read_buffer(0, 10000).tobytes()
        t = time.perf_counter()
        ref = int.from_bytes(cref.bn_fold_be(nsq1.to_bytes(mb, "big"), buf, mb, 10000), "big")
        cpu_ms = (time.perf_counter() - t) * 1e3
        col.close()
        k2 = self.key
        a, b = (str(x) for x in (self.col_sample[0], self.col_sample[1]))
        pair, pair_ms, pair_p99 = med(lambda: eng.pair_modmul_dec(a, b, str(k2["nsquare"])), 200)
        conc = self.concurrent_pairs(k2["nsquare"], threads=64, per_thread=32)
        native = self.native_pairs(k2["nsquare"], threads=64, per_thread=200)  # engine default (host products)
        native_gpu = self.native_pairs(k2["nsquare"], threads=64, per_thread=200, policy=0)  # GPU batches only
        rng = np.random.default_rng(5)
        n_pairs = 65536
        xa = [self.col_sample[i % len(self.col_sample)] for i in range(n_pairs)]
        xb = [self.col_sample[(i * 7 + 3) % len(self.col_sample)] for i in range(n_pairs)]
        eng.modmul_pairs(k2["nsquare"], xa[:64], xb[:64])
        t = time.perf_counter()
        pr = eng.modmul_pairs(k2["nsquare"], xa, xb)
        pairs_s = n_pairs / (time.perf_counter() - t)
        # the C entry point on big-endian buffers as a JNA caller holds them (Python int <-> bytes outside)
        import ctypes as C
        nsq2 = k2["nsquare"]
        mb = (nsq2.bit_length() + 7) // 8
        ba = b"".join(x.to_bytes(mb, "big") for x in xa)
        bb = b"".join(x.to_bytes(mb, "big") for x in xb)
        ob = (C.c_uint8 * (mb * n_pairs))()
        lib = self.ddshe._lib
        modb = nsq2.to_bytes(mb, "big")
        ts = []
        for _ in range(3):
            t = time.perf_counter()
            assert lib.dds_modmul_pairs(eng._h, modb, mb, ba, bb, mb, n_pairs, ob) == 0
            ts.append(time.perf_counter() - t)
        pairs_c_s = n_pairs / min(ts)
        ok_c = int.from_bytes(bytes(ob[:mb]), "big") == xa[0] * xb[0] % nsq2
        del rng
        eng.set_stream(self.torch.cuda.current_stream().cuda_stream)
        return {"config1_sumall_10k_1024bit": {
                    "resident_fold_ms": fold_ms, "resident_fold_p99_ms": fold_p99,
                    "resident_fold_c_abi_ms": fold_c_ms, "resident_fold_c_abi_p99_ms": fold_c_p99,
                    "decimal_route_ms": dec_ms,
                    "decimal_route_path": "dds_sum_all_dec (String[] of 10k BigInteger.toString rows -> decimal reply)",
                    "decimal_route_with_python_marshalling_ms": dec_py_ms,
                    "cpu_reference_ms": cpu_ms, "cpu_kind": "OpenSSL BN_mod_mul fold, 1 core (oracle/csrc/bn_baseline.c)",
                    "speedup_resident_vs_cpu": cpu_ms / fold_ms,
                    "matches": gpu == ref and dec == str(ref)},
                "host_cpu_per_fold": {
                    "folds": host_cpu,
                    "how": "time.thread_time of the calling thread around dds_col_fold (timing off): the finalize "
                           "spins on the root's sequence word up to DDSHE_FOLD_SPIN_ROWS (100k) rows and polls it "
                           "between 50 us sleeps above; 10k rows on the config-1 column, 1M / 10M rows on a fresh "
                           "column of the headline's rows"},
                "pair_sum_route_2048bit": {"median_ms": pair_ms, "p99_ms": pair_p99,
                                           "path": "dds_pair_modmul_dec, one caller (the /Sum route body)",
                                           "matches": pair == str(int(a) * int(b) % k2["nsquare"])},
                "pair_sum_route_concurrent_2048bit": conc,
                "pair_sum_route_native_threads_2048bit": native,
                "pair_sum_route_native_threads_gpu_batches_2048bit": native_gpu,
                "pairs_batched_2048bit": {"pairs": n_pairs, "pairs_per_s": pairs_c_s,
                                          "path": "dds_modmul_pairs (k_pairs + k_egress_be), big-endian host buffers in and out",
                                          "pairs_per_s_with_python_int_marshalling": pairs_s,
                                          "matches": ok_c and pr[:4] == [x * y % nsq2 for x, y in zip(xa[:4], xb[:4])]}}

    def concurrent_pairs(self, m, threads, per_thread):
        """/Sum requests from `threads` concurrent callers (the proxy's route pool), each a blocking
        dds_pair_modmul_dec call: throughput, per-call latency and calls per k_pairs launch."""
        import threading
        eng = self.eng
        samp = [str(x) for x in self.col_sample]
        want = {}
        lat, bad = [], []
        c0, l0 = eng.pair_stats()
        start = threading.Barrier(threads + 1)

        def worker(t):
            mine = []
            start.wait()
            for i in range(per_thread):
                a, b = samp[(t * 131 + i) % len(samp)], samp[(t * 17 + 7 * i + 1) % len(samp)]
                t0 = time.perf_counter()
                r = eng.pair_modmul_dec(a, b, str(m))
                mine.append(time.perf_counter() - t0)
                if (t + i) % 16 == 0 and r != str(int(a) * int(b) % m):
                    bad.append((t, i))
            lat.extend(mine)

        th = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
        for x in th:
            x.start()
        start.wait()
        t0 = time.perf_counter()
        for x in th:
            x.join()
        wall = time.perf_counter() - t0
        c1, l1 = eng.pair_stats()
        lat.sort()
        del want
        return {"threads": threads, "calls": threads * per_thread, "pairs_per_s": threads * per_thread / wall,
                "median_ms": lat[len(lat) // 2] * 1e3, "p99_ms": lat[int(len(lat) * 0.99)] * 1e3,
                "calls_per_launch": (c1 - c0) / max(1, l1 - l0),
                "path": "dds_pair_modmul_dec from concurrent threads (engine default policy: host products; "
                        "DDS_PAIR_GPU: one k_pairs launch per burst)",
                "matches": not bad}

    def native_pairs(self, m, threads, per_thread, policy=None):
        """The same /Sum load from native threads (tools/native/pair_bench: C++ std::threads calling
        dds_pair_modmul_dec, no interpreter lock), as the JVM's ForkJoin pool would (DDSRestServer.scala:21).
        Runs as a child process on the same GPU; its samples are checked here with Python ints. policy:
        the context's serving policy (DDSHE_PAIR_POLICY; None: the engine default)."""
        exe = os.path.join(ROOT, "tools", "native", "pair_bench")
        if not os.path.exists(exe):
            return {"skipped": "tools/native/pair_bench not built"}
        import subprocess
        env = dict(os.environ)
        if policy is not None:
            env["DDSHE_PAIR_POLICY"] = str(policy)
        pr = subprocess.run([exe, str(m), str(threads), str(per_thread)], capture_output=True, text=True, timeout=300,
                            env=env)
        if pr.returncode != 0:
            return {"error": pr.stderr[-400:]}
        res = json.loads(pr.stdout.strip().splitlines()[-1])
        samples = res.pop("samples")
        res["matches"] = bool(samples) and all(int(r) == int(a) * int(b) % m for a, b, r in samples)
        res["checked_samples"] = len(samples)
        res["path"] = "tools/native/pair_bench: %d C++ threads x %d dds_pair_modmul_dec calls" % (threads, per_thread)
        return res

    def end_to_end(self, res):
        """Host-boundary rates, outside the timed region (never `value`): (1) the binary boundary
        (dds_paillier_sum on a host buffer of 512-byte big-endian rows: H2D + ingest + fold), all rows;
        (2) the decimal route (BigInteger.toString rows, DDSRestServer.scala:417-422: host chars ->
        GPU parse -> resident column -> fold -> decimal result) on a bounded sample."""
        import numpy as np
        nsq = self.nsq
        out = {}
        buf = self.col.read_buffer(0, self.mine)
        for rep in range(2):  # first call sizes the context's device buffers
            t = time.perf_counter()
            got = self.eng.fold_buffer(nsq, buf)
            dt = time.perf_counter() - t
        out["binary"] = {"rows": self.mine, "seconds": dt, "rows_per_s": self.mine / dt,
                         "host_GBps": buf.nbytes / dt / 1e9, "matches": got == res,
                         "path": "dds_paillier_sum (pageable host buffer -> H2D -> k_ingest_be -> fold)"}
        del buf
        # u distinct decimal rows (Python str() costs ~30 us per 4096-bit row), tiled `rep` times
        u = min(self.mine, 100_000, self.args.e2e_dec_rows)
        rep = max(1, self.args.e2e_dec_rows // u)
        k = u * rep
        rows = [str(x) for x in self.col.read(0, u)]
        chars = "".join(rows).encode() * rep  # Arrow-style (chars, offsets): how a JNA shim passes String[]
        lens = np.tile(np.array([len(r) for r in rows], dtype=np.uint64), rep)
        offs = np.zeros(k + 1, dtype=np.uint64)
        np.cumsum(lens, out=offs[1:])
        # median of 5 calls after one that sizes the buffers (2 calls left the second one 26-46 ms box to box)
        ts = []
        for _ in range(6):
            t = time.perf_counter()
            dcol = self.eng.column(nsq, k)
            dcol.append_dec((chars, offs))
            dec = dcol.fold()
            dec_s = str(dec)
            ts.append(time.perf_counter() - t)
            dcol.close()
        dt = sorted(ts[1:])[2]
        out["decimal"] = {"rows": k, "distinct_rows": u, "seconds": dt, "min_seconds": min(ts[1:]),
                          "rows_per_s": k / dt, "chars": len(chars),
                          "host_GBps": len(chars) / dt / 1e9,
                          "matches_resident_fold": dec == pow(self.col.fold(0, u), rep, nsq),
                          "path": "dds_col_append_dec (k_dec_parse on the GPU) + dds_col_fold, decimal result"}
        # CPU side of the same decimal boundary: what the reference route does per row before the
        # modmul (BigInteger(String) parse, :417,419), restated as Python int() on the sample
        t = time.perf_counter()
        _ = [int(r) for r in rows[: min(k, 20000)]]
        out["decimal"]["cpu_parse_rows_per_s_1core"] = min(k, 20000) / (time.perf_counter() - t)
        # (3) the route entry point a JNA binding calls with the String[] it holds (dds_sum_all_dec:
        # NUL-terminated rows -> GPU parse -> fold -> decimal text), same rows
        import ctypes as C
        enc = [r.encode() for r in rows]
        arr = (C.c_char_p * k)(*(enc * rep))
        cap = 4 * len(str(nsq)) + 64
        res_buf = C.create_string_buffer(cap)
        olen = C.c_size_t()
        ts = []
        for _ in range(6):
            t = time.perf_counter()
            st = self.ddshe._lib.dds_sum_all_dec(self.eng._h, arr, k, str(nsq).encode(), res_buf, cap, C.byref(olen))
            ts.append(time.perf_counter() - t)
        dt = sorted(ts[1:])[2]
        out["strings"] = {"rows": k, "seconds": dt, "min_seconds": min(ts[1:]), "rows_per_s": k / dt,
                          "host_GBps": len(chars) / dt / 1e9,
                          "matches": st == 0 and res_buf.value.decode() == str(dec),
                          "path": "dds_sum_all_dec (String[] rows, the route-level JNA entry point)"}
        return out

    def close(self):
        self.col.close()


def run_extra_configs(main_wl):
    """BASELINE.json configs 3 and 4 in the default run (rank 0, N = 1): each workload with its own
    defaults, its own warmup and timed steps, roofline and CPU baseline, reported as an extra key of the
    headline line so the driver's BENCH record carries them."""
    import copy
    out = {}
    # config 3 warms up 5 steps: its first k_fold1 launches run while the clock ramps (profiles/r06_pf_fold1_dispatches.json)
    for name, cls, rows, steps, warmup, seed in (("config3_product_filter", ProductFilterWorkload, 10_000_000, 10, 5, 3),
                                                 ("config4_encrypt_sum", EncryptSumWorkload, 1_000_000, 2, 1, 4)):
        a = copy.copy(main_wl.args)
        a.rows, a.steps, a.warmup, a.seed, a.strong = rows, steps, warmup, seed, False
        ctx = {k: getattr(main_wl, k) for k in ("coll_dev", "eng", "world", "rank", "local", "torch", "ddshe", "ddist")}
        ctx.update(args=a, total=rows, row0=0, mine=rows, per=rows)
        wl = cls(ctx)
        wl.setup()
        main_wl.torch.cuda.synchronize()
        for _ in range(warmup):
            res = wl.step()
        main_wl.eng.set_timing(True)
        main_wl.eng.reset_timing()
        wl.reset_timers()
        main_wl.torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            res = wl.step()
        main_wl.torch.cuda.synchronize()
        el = time.perf_counter() - t0
        main_wl.eng.set_timing(False)
        out[name] = wl.report(res, el)
        wl.close()
    return out


# tools/gpurun/profile_all.sh passes, summarised by tools/pmc_summary.py (newest round first)
PMC_FILE = next((f for f in ("r06_pmc.json", "r05_pmc.json", "r04_pmc.json", "r03_pmc.json", "r02_pmc_filter_order.json")
                 if os.path.exists(os.path.join(ROOT, "profiles", f))), "r02_pmc_filter_order.json")


def pmc_traffic(workload, kernels, per_step=False, largest=False):
    """HBM bytes per call from the committed rocprofv3 PMC passes (10M rows): the sum over `kernels`
    of bytes per dispatch (times dispatches per call when per_step: the PMC run did one call; the
    largest dispatch when `largest`: the 10M-row launch among the extra lines' smaller ones)."""
    tf = os.path.join(ROOT, "profiles", PMC_FILE)
    if not os.path.exists(tf):
        return None
    ks = json.load(open(tf))["kernels"]
    tot = 0.0
    for k in kernels:
        d = ks.get(f"{workload}:{k}")
        if d is None:  # a template that gained trailing parameters since the name was written here
            d = next((v for n, v in ks.items() if n.startswith(f"{workload}:{k[:-1]},")), None)
        if d is None:
            return None
        if largest and "hbm_bytes_max_dispatch" in d:
            tot += d["hbm_bytes_max_dispatch"]
        else:
            tot += d["hbm_bytes_per_dispatch"] * (d["dispatches"] if per_step else 1)
    return tot


def order_pmc_traffic():
    """HBM bytes of one OrderLS call on raw arrays: the last raw call (the carried plan: no min / max pass)
    of the per-call PMC split (tools/order_call_traffic.py -> profiles/r06_order_call_traffic.json; the
    order bench's FETCH_SIZE / WRITE_SIZE passes with one warmup and two steps); older rounds: one raw call
    with k_rs_prep + k_rs_red and the resident line's calls averaged."""
    cf = os.path.join(ROOT, "profiles", "r06_order_call_traffic.json")
    if os.path.exists(cf):
        raw = [c for c in json.load(open(cf))["calls"] if "__amd_rocclr_copyBuffer" not in c["kernels"]]
        if raw:
            return raw[-1]["hbm_bytes"]
    once = pmc_traffic("order", ("k_rs_prep", "k_rs_red"), per_step=True)
    rest = pmc_traffic("order", ("k_rs_hist<256>", "k_rs_scan_tiles", "k_rs_scan_chunks", "k_rs_scatter<256>", "k_msd_local", "k_msd_big"),
                       per_step=True)
    calls = (pmc_entry(["order"], "k_msd_local") or (None, 0))[1]
    if once is None or rest is None or not calls:
        return None
    return once + rest / calls


def pmc_entry(workloads, kernel):
    """(bytes per dispatch, dispatches) of `kernel` under the first of `workloads` that has it"""
    tf = os.path.join(ROOT, "profiles", PMC_FILE)
    if not os.path.exists(tf):
        return None
    ks = json.load(open(tf))["kernels"]
    for w in workloads:
        d = ks.get(f"{w}:{kernel}")
        if d is not None:
            return d["hbm_bytes_per_dispatch"], d["dispatches"]
    return None


def valu_pmc(names):
    """The first committed rocprofv3 SQ/GRBM pass summary (tools/pmc_valu_summary.py) among `names`: the
    kernel's 64-bit VALU issue rate against the half-rate v_mad_u64_u32 peak at the clock measured in that
    run, and its 64-bit instructions per expected lane mad (1.0 = nothing but the Montgomery mads)."""
    for vname in names:
        vf = os.path.join(ROOT, "profiles", vname)
        if os.path.exists(vf):
            dv = json.load(open(vf))["derived"]
            out = {"mad_issue_frac_at_measured_clock": dv["mad_issue_frac_of_half_rate_peak_at_measured_clock"],
                   "int64_share_of_valu": dv.get("valu_int64_share_of_valu", dv.get("mad_share_of_valu")),
                   "clock_GHz": dv["clock_GHz_est"], "source": "profiles/" + vname}
            for k in ("int64_instr_per_expected_mad", "issue_stall_share", "waitcnt_share"):
                if k in dv:
                    out[k] = dv[k]
            return out
    return None


def engine_shape(bits: int):
    """(S, W) of the engine's lane-group shape for a modulus of `bits` bits (kShapes, ddshe_shapes.hpp:
    the first with S*W >= bits + 2)."""
    for S, W in ((40, 28), (76, 28), (112, 28), (148, 28), (232, 27), (320, 27), (640, 27)):
        if S * W >= bits + 2:
            return S, W
    raise ValueError(bits)


def load_keyset(name):
    raw = json.load(open(os.path.join(ROOT, "tests", "golden", "keys.json")))
    return {k: (int(v, 16) if k != "x509_hex" else v) for k, v in raw[name].items()}


class ProductFilterWorkload(_Workload):
    """BASELINE.json config 3: RSA HomoMult product (MultAll, DDSRestServer.scala:491-539) + OPE range
    filter (SearchGt/GtEq/Lt/LtEq, :682-830) over 10M rows, synthetic 2048-bit RSA key (e = 65537).
    Rows: c_i = (j_i+1)^e mod n with j_i = splitmix64(seed ^ splitmix64(i)) % 9999; OPE column =
    a seeded strictly increasing int64 map of the same plaintexts; bound = the map at m = 5000."""

    def setup(self):
        import numpy as np
        torch = self.torch
        self.key = load_keyset("rsa2048_seed3")
        n, e = self.key["n"], self.key["e"]
        self.table = self.eng.modexp_batch(n, e, list(range(1, 10000)))  # HomoMult.encrypt on the GPU
        self.col = self.eng.column(n, max(1, self.mine))
        if self.mine:
            self.col.fill_table_synth(self.table, self.args.seed, self.row0, self.mine)
        rng = np.random.default_rng(self.args.seed)
        self.ope_map = np.cumsum(rng.integers(1, 1 << 40, size=10001, dtype=np.int64)) - (1 << 52)
        j = self.ddshe.synth_indices(self.args.seed, self.row0, self.mine, 9999)
        self.ope_host = self.ope_map[j.astype(np.int64) + 1]
        self.d_ope = torch.from_numpy(self.ope_host).to("cuda")
        self.d_valid = torch.ones(max(1, self.mine), dtype=torch.uint8, device="cuda")
        self.d_out = torch.empty(max(1, self.mine), dtype=torch.int32, device="cuda")
        self.bound = int(self.ope_map[5000])
        # the same OPE values as a resident column behind the C-ABI (dds_opecol: what a JNA caller holds)
        self.opecol = self.eng.opecol(max(1, self.mine))
        if self.mine:
            self.opecol.append(self.ope_host)
        self.ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        self.fold_ms = self.filter_ms = 0.0

    def reset_timers(self):
        self.fold_ms = self.filter_ms = 0.0

    def step(self):
        self.ev[0].record()
        res = self.fold_or_combine(self.col, self.key["n"])
        self.ev[1].record()
        counts = {op: self.eng.ope_filter_device(self.d_ope.data_ptr(), self.d_valid.data_ptr(), self.mine,
                                                 self.bound, op, self.d_out.data_ptr())
                  for op in ("gt", "ge", "lt", "le")}
        self.ev[2].record()
        self.ev[2].synchronize()
        self.fold_ms += self.ev[0].elapsed_time(self.ev[1])
        self.filter_ms += self.ev[1].elapsed_time(self.ev[2])
        return res, counts

    def report(self, res, elapsed):
        import numpy as np
        a, key = self.args, self.key
        prod, counts = res
        ok = None
        if a.verify:
            j = self.ddshe.synth_indices(a.seed, 0, self.total, 9999)
            cnt = np.bincount(j, minlength=9999)
            want = 1
            for t, c in zip(self.table, cnt.tolist()):
                if c:
                    want = want * pow(t, c, key["n"]) % key["n"]
            ok = prod == want
            if self.world == 1:
                for op, f in (("gt", np.greater), ("ge", np.greater_equal), ("lt", np.less), ("le", np.less_equal)):
                    ok = ok and counts[op] == int(f(self.ope_host, self.bound).sum())
            if not ok:
                print("VERIFY FAILED", file=sys.stderr)
        roof = self.fold_roofline(64)
        if os.environ.get("DDSHE_FOLD1", "1") != "0":  # >= 1M rows: one bignum per lane (ddshe_fold.hpp)
            s1 = 76 if os.environ.get("DDSHE_FOLD1_74", "1") == "0" else 74
            roof["kernel"] = f"k_fold1<{s1},28> (first MultAll fold level, 2048-bit n, one bignum per lane)"
            kname = f"k_fold1<{s1}, 28, {'true' if s1 == 76 else 'false'}, false>"
        else:
            roof["kernel"] = "k_fold<76,2,28,QP> (first MultAll fold level, 2048-bit n)"
            kname = "k_fold<76, 2, 28, true>"
        roof["traffic"] = pmc_traffic("product_filter", (kname,))
        roof["traffic_unit"] = f"HBM bytes per launch (PMC, profiles/{PMC_FILE})"
        if kname.startswith("k_fold1<74"):  # VALU counters of the same kernel
            vp = valu_pmc(("r06_pmc_valu_fold1.json", "r02_pmc_valu_fold1.json"))
            if vp:
                roof["valu_pmc"] = vp
        _, _, filt_dev_ms, _ = self.eng.timing()  # HIP events around the filter launches (device time)
        filt_s = filt_dev_ms / 1e3 / (4 * a.steps)
        matches = sum(counts.values()) / 4
        filt_bytes = 9 * self.mine + 4 * matches  # int64 OPE value + valid byte per row, u32 id per match
        filt = {"bound": "hbm", "achieved": filt_bytes / filt_s / 1e9, "peak": 8000.0, "unit": "GB/s",
                "frac": filt_bytes / filt_s / 1e9 / 8000.0, "avg_filter_ms": filt_s * 1e3,
                "kernel": "k_ope_count + k_ope_scatter (device time, HIP events on the launch stream)",
                "avg_filter_call_ms": self.filter_ms / (4 * a.steps),
                "algorithmic_bytes": filt_bytes, "traffic": pmc_traffic("product_filter", ("k_ope_count<true>", "k_ope_scatter")),
                "traffic_unit": "HBM bytes per filter call (PMC, profiles/" + PMC_FILE + ")"}
        cpu = None
        if self.world == 1 and not a.no_cpu_baseline:
            n = key["n"]
            mb = (n.bit_length() + 7) // 8
            cpu = cpu_baseline(self.col, n, mb, a.cpu_seconds)
            cpu["unit"] = "HomoMult/s"
        out = self.common("RSA HomoMult product + OPE range filter rows/sec (2048-bit key)",
                          self.total * a.steps / elapsed, "rows/s", elapsed, "rsa_multall_plus_ope_filter_10M_2048bit",
                          {"key_bits": key["n"].bit_length(), "filters_per_step": 4})
        # Search through the resident OPE column with host output (the JNA-shaped call: bound as text, row
        # ids back in host memory), outside the timed region
        # into the reply buffer a caller reuses (engine-allocated, dds_host_alloc: one DMA), and into a fresh
        # numpy array per call (pageable, first-touched by the copy: what a caller allocating per request pays)
        res_ms, fresh_ms, res_ok = [], [], True
        ids_buf = self.eng.host_alloc(max(1, self.mine), np.uint32)
        for op, f in (("gt", np.greater), ("ge", np.greater_equal), ("lt", np.less), ("le", np.less_equal)):
            for _ in range(3):
                t = time.perf_counter()
                ids = self.opecol.search(str(self.bound), op, out=ids_buf)
                res_ms.append((time.perf_counter() - t) * 1e3)
            if self.world == 1:
                res_ok = res_ok and len(ids) == counts[op] and (len(ids) == 0 or bool(f(self.ope_host[ids], self.bound).all()))
            t = time.perf_counter()
            fresh = self.opecol.search(str(self.bound), op)
            fresh_ms.append((time.perf_counter() - t) * 1e3)
            res_ok = res_ok and bool(np.array_equal(fresh, ids))
        res_ms.sort()
        fresh_ms.sort()
        filt["resident_opecol_search"] = {"median_ms": res_ms[len(res_ms) // 2], "matches": res_ok,
                                          "fresh_array_median_ms": fresh_ms[len(fresh_ms) // 2],
                                          "path": "dds_opecol_search (device filter + D2H of the matching row ids "
                                                  "into a dds_host_alloc reply buffer; fresh_array: a new numpy "
                                                  "array per call)"}
        del ids
        self.eng.host_free(ids_buf)
        # the route-shaped answer as a row bitmask (dds_opecol_search_mask): 1 bit per row crosses PCIe,
        # written by the count kernel straight into a device-mapped reply buffer the caller reuses:
        # an engine-allocated one (dds_host_alloc, placed by the HIP runtime for the device) and a caller
        # array page-locked once (dds_host_register)
        nwords = max(1, (self.mine + 63) // 64)
        route_bytes = 9 * self.mine  # what the route reads per call (int64 + class byte per row)

        def mask_route(mbuf):
            ms, ok = [], True
            for op, f in (("gt", np.greater), ("ge", np.greater_equal), ("lt", np.less), ("le", np.less_equal)):
                for _ in range(5):
                    t = time.perf_counter()
                    words, cnt = self.opecol.search_mask(str(self.bound), op, out=mbuf)
                    ms.append((time.perf_counter() - t) * 1e3)
                if self.world == 1:
                    bits = np.unpackbits(words.view(np.uint8), bitorder="little")[: self.mine].astype(bool)
                    ok = ok and cnt == counts[op] and bool(np.array_equal(bits, f(self.ope_host, self.bound)))
            ms.sort()
            return ms[len(ms) // 2], ok

        abuf = self.eng.host_alloc(nwords, np.uint64)
        med, mk_ok = mask_route(abuf)
        self.eng.host_free(abuf)
        rbuf = np.zeros(nwords, dtype=np.uint64)
        self.eng.host_register(rbuf)
        reg_med, reg_ok = mask_route(rbuf)
        self.eng.host_unregister(rbuf)
        zc = os.environ.get("DDSHE_MASK_ZEROCOPY", "1") != "0"
        native = self.native_search() if self.world == 1 else None
        filt["resident_opecol_search_mask"] = {
            "median_ms": med, "matches": mk_ok and reg_ok, "rows": self.mine,
            "registered_caller_array_ms": reg_med,
            "route_roofline": {"bound": "hbm", "achieved": route_bytes / (med / 1e3) / 1e9, "peak": 8000.0,
                               "unit": "GB/s", "frac": route_bytes / (med / 1e3) / 1e9 / 8000.0,
                               "note": "column bytes / whole call time (host clock), mask read-back included"},
            "native_call": native,
            "path": "dds_opecol_search_mask into a dds_host_alloc reply buffer (median_ms) and into a "
                    "dds_host_register'ed caller array (registered_caller_array_ms): one k_ope_count launch "
                    "stores the mask words through the buffer's device mapping and the per-tile counts into a "
                    "mapped host array the host adds up" + (": no copies" if zc else
                                                              "; DDSHE_MASK_ZEROCOPY=0: one D2H of n/8 bytes + the count")}
        out.update(data="synthetic (seeded RSA ciphertexts of U[1,10^4) plaintexts, seeded OPE map)",
                   roofline=roof, filter_roofline=filt, cpu_baseline=cpu, verified=ok,
                   fold_ms_per_step=self.fold_ms / a.steps, filter_ms_per_step=self.filter_ms / a.steps,
                   homomult_per_s=(self.total - 1) * a.steps / elapsed, matches=counts)
        return out

    def native_search(self):
        """The same route from C++ (tools/native/search_bench: the call a JNA binding makes, without the
        Python binding's marshalling) over its own seeded 10M-row OPE column, every reply checked in the
        child against a host count of the predicate."""
        exe = os.path.join(ROOT, "tools", "native", "search_bench")
        if not os.path.exists(exe):
            return {"skipped": "tools/native/search_bench not built"}
        import subprocess
        pr = subprocess.run([exe, str(self.mine)], capture_output=True, text=True, timeout=300)
        if pr.returncode != 0:
            return {"error": pr.stderr[-400:]}
        return json.loads(pr.stdout.strip().splitlines()[-1])

    def close(self):
        self.col.close()
        self.opecol.close()


class EncryptSumWorkload(_Workload):
    """BASELINE.json config 4: batched Paillier encryption (g^m r^n mod n^2, HomoAdd.encrypt,
    SJHomoLibProvider.scala:58) + SumAll over the fresh ciphertexts, synthetic 3072-bit key
    (n^2 6144-bit). Sub-batch: 1M rows per GPU per step (SURVEY.md §8d allows 1M). r_i from a
    seeded device stream (dds_col_fill_random), m_i as in config 2. CRT halves unless --public."""

    def setup(self):
        torch = self.torch
        self.key = load_keyset("paillier3072_seed4")
        k = self.key
        self.rcol = self.eng.column(k["nsquare"], max(1, self.mine))
        self.out = self.eng.column(k["nsquare"], max(1, self.mine))
        if self.mine:
            self.rcol.fill_random(k["n"].bit_length() - 1, self.args.seed, self.row0, self.mine)
        self.ms = self.ddshe.synth_plaintexts(self.args.seed, self.row0, self.mine)
        self.d_m = torch.from_numpy(self.ms.astype("int32")).to("cuda")
        self.ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        self.enc_ms = 0.0

    def reset_timers(self):
        self.enc_ms = 0.0

    def step(self):
        k = self.key
        self.out.truncate(0)
        self.ev[0].record()
        pq = (None, None) if self.args.public else (k["p"], k["q"])
        self.out.encrypt_paillier(self.rcol, 0, self.d_m.data_ptr(), self.mine, k["n"], k["g"], *pq)
        self.ev[1].record()
        res = self.fold_or_combine(self.out, k["nsquare"])
        self.ev[1].synchronize()
        self.enc_ms += self.ev[0].elapsed_time(self.ev[1])
        return res

    def report(self, res, elapsed):
        a, k = self.args, self.key
        ok = None
        if a.verify:
            from oracle import homo  # checker only
            ms_all = self.ddshe.synth_plaintexts(a.seed, 0, self.total)
            ok = homo.paillier_decrypt(res, k) == int(ms_all.astype("int64").sum()) % k["n"]
            if self.world == 1:
                idx = [0, self.mine // 2, self.mine - 1]
                rs = self.rcol.read(0, self.mine) if self.mine <= 4096 else None
                for i in idx:
                    r = rs[i] if rs else self.rcol.read(i, 1)[0]
                    ok = ok and self.out.read(i, 1)[0] == homo.paillier_encrypt(int(self.ms[i]), r, k)
            if not ok:
                print("VERIFY FAILED", file=sys.stderr)
        enc_s = self.enc_ms / 1e3 / a.steps
        # work actually issued per encryption: per CRT half (or the n^2 modulus with --public)
        n = k["n"]
        sq, mul, tab = window_counts(n)
        m_ops = 2 * 14  # g^m_i ladder (<= 14 bits, both products issued per bit) + 1 merge
        if a.public:
            s32 = (k["nsquare"].bit_length() + 31) // 32
            per_enc = [(sq + mul + tab + m_ops + 2, s32)]
        else:
            s32 = (k["p"].bit_length() * 2 + 31) // 32
            per_enc = [(sq + mul + tab + m_ops + 3, s32)] * 2
        mac_issued = sum(cnt * (2 * s * s + s) for cnt, s in per_enc)
        achieved = mac_issued * self.mine / enc_s / 1e12
        # the same products in the engine's own limbs (28- or 27-bit: what the VALU actually issues)
        mod_bits = k["nsquare"].bit_length() if a.public else 2 * k["p"].bit_length()
        S_eng, W_eng = engine_shape(mod_bits)
        lane_mads = sum(cnt for cnt, _ in per_enc) * (2 * S_eng * S_eng + S_eng)
        s_full = (k["nsquare"].bit_length() + 31) // 32
        binary_mac = binary_ladder_modmuls(n) * (2 * s_full * s_full + s_full)
        roof = {"bound": "valu-int", "kernel": "k_modexp_ladder (encrypt phase: pre + ladder + CRT kernels)",
                "achieved": achieved, "peak": PEAK_TMAC, "unit": "TMAC/s", "frac": achieved / PEAK_TMAC,
                "mac_per_encrypt_issued": mac_issued,
                "mac_unit": "32x32-bit MACs of the products the ladder issues, 2s^2+s with s = 32-bit limbs of the modulus",
                "lane_mads_per_encrypt": lane_mads, "engine_shape": [S_eng, W_eng],
                "lane_mad_frac": lane_mads * self.mine / enc_s / 1e12 / PEAK_TMAC,
                "mac_per_encrypt_binary_ladder_n2": binary_mac,
                "effective_vs_binary_ladder_n2": binary_mac * self.mine / enc_s / 1e12,
                "avg_encrypt_ms": enc_s * 1e3, "traffic": None}
        if not a.public:  # the ladder's HBM bytes (PMC), per dispatch: one dispatch per CRT half and 1M-row chunk
            lad = pmc_entry(("encrypt_sum", "sum"), "k_modexp_ladder<112, 4, 28, true>")
            if lad is not None:
                roof["traffic"] = lad[0]
                roof["traffic_unit"] = (f"HBM bytes per k_modexp_ladder<112,4,28> dispatch (PMC, profiles/{PMC_FILE});"
                                        " the per-row window tables are streamed from HBM")
                roof["traffic_rows_per_dispatch"] = self.mine
            vp = valu_pmc(("r06_pmc_valu_ladder.json",))
            if vp:  # the ladder's own SQ/GRBM pass: 64-bit VALU issue rate, waits
                roof["valu_pmc"] = vp
        cpu = None
        if self.world == 1 and not a.no_cpu_baseline:
            cpu = cpu_encrypt_baseline(k, self.rcol, self.ms, a.cpu_seconds, self.out)
        out = self.common("Paillier encryptions + HomoAdd sum /sec (3072-bit key, mod n^2)",
                          self.total * a.steps / elapsed, "encrypt/s", elapsed,
                          "paillier_encrypt_sum_3072bit_1M_per_gpu",
                          {"key_bits": n.bit_length(), "modulus_bits": k["nsquare"].bit_length(),
                           "path": "public (n, g)" if a.public else "CRT (p^2, q^2 halves)"})
        out.update(data="synthetic (seeded r stream on device, m ~ U[0,10^4))", roofline=roof, cpu_baseline=cpu,
                   verified=ok, encrypt_ms_per_step=self.enc_ms / a.steps)
        return out

    def close(self):
        self.rcol.close()
        self.out.close()


class OrderWorkload(_Workload):
    """OrderLS (DDSRestServer.scala:541-573) over a 10M-row OPE column: int64 values of a seeded
    increasing map of U[1,10^4) plaintexts (many ties, as the generator's), 5 % of rows lacking
    the position. Each rank orders its own shard (the route's result is per shard; a k-way merge
    of shard orders is not part of this measurement)."""

    def setup(self):
        import numpy as np
        torch = self.torch
        rng = np.random.default_rng(self.args.seed)
        ope_map = np.cumsum(rng.integers(1, 1 << 40, size=10001, dtype=np.int64)) - (1 << 52)
        j = self.ddshe.synth_indices(self.args.seed, self.row0, self.mine, 9999)
        self.col = ope_map[j.astype(np.int64) + 1]
        self.valid = (rng.random(self.mine) > 0.05).astype(np.uint8)
        self.d_col = torch.from_numpy(self.col).to("cuda")
        self.d_valid = torch.from_numpy(self.valid).to("cuda")
        self.d_out = torch.empty(max(1, self.mine), dtype=torch.int32, device="cuda")

    def step(self):
        self.eng.ope_order_device(self.d_col.data_ptr(), self.d_valid.data_ptr(), self.mine, True,
                                  self.d_out.data_ptr())
        return None

    def local_ok(self):
        """This rank's OrderLS permutation against numpy's stable argsort of its shard."""
        import numpy as np
        idx = np.arange(self.mine)
        hold, rest = idx[self.valid != 0], idx[self.valid == 0]
        want = np.concatenate([hold[np.argsort(~self.col[hold], kind="stable")], rest])
        return bool(np.array_equal(self.d_out.cpu().numpy().view(np.uint32), want))

    def verify_distributed(self):
        return self.all_ranks_ok(self.local_ok())

    def report(self, res, elapsed):
        import numpy as np
        a = self.args
        ok = None
        if a.verify and self.world == 1:
            ok = self.local_ok()
            if not ok:
                print("VERIFY FAILED", file=sys.stderr)
        step_s = elapsed / a.steps
        alg = 13 * self.mine  # read key + valid byte, write one row id
        roof = {"bound": "hbm", "kernel": "2 LSD passes over the top 16 bits of the key span (k_rs_hist/k_rs_scan_tiles/k_rs_scan_chunks/"
                "k_rs_scatter; the last scatter also fills the bucket table) + k_msd_local/k_msd_big (in-bucket order "
                "of the buckets holding two distinct keys); the previous call's plan carried (its first histogram also takes "
                "the bounds, k_rs_red checks the plan: no k_rs_prep pass)",
                "achieved": alg / step_s / 1e9, "peak": 8000.0, "unit": "GB/s", "frac": alg / step_s / 1e9 / 8000.0,
                "algorithmic_bytes": alg,
                # pass 1 (hist 9 + scatter 9 + 12) + pass 2 (hist 4 + scatter 12 + 12) (+ the multi-key
                # buckets' copies and rounds)
                "issued_bytes_est": self.mine * (30 + 28),
                "traffic": order_pmc_traffic(),
                "traffic_unit": "HBM bytes per raw OrderLS call (PMC, profiles/r06_order_call_traffic.json)"}
        roof["issued_GBps"] = roof["issued_bytes_est"] / step_s / 1e9  # what the MSD-split design moves
        roof["issued_frac"] = roof["issued_GBps"] / 8000.0
        cpu = None
        if self.world == 1 and not a.no_cpu_baseline:
            t = time.perf_counter()
            idx = np.arange(self.mine)
            hold = idx[self.valid != 0]
            _ = np.concatenate([hold[np.argsort(~self.col[hold], kind="stable")], idx[self.valid == 0]])
            dt = time.perf_counter() - t
            cpu = {"value": self.mine / dt, "unit": "rows/s", "cores": 1, "kind": "port",
                   "sample": f"all {self.mine} rows, numpy stable argsort (the reference sorts with sortWith), {dt:.2f}s"}
        out = self.common("OPE OrderLS rows/sec (int64 keys, stable)", self.total * a.steps / elapsed, "rows/s",
                          elapsed, "ope_orderls_10M", {})
        out.update(data="synthetic (seeded OPE map of U[1,10^4) plaintexts, 5% rows lacking the position)",
                   dtype="int64", roofline=roof, cpu_baseline=cpu, verified=ok)
        if self.world == 1:
            try:
                out["resident_opecol_order"] = self.resident_order()
            except Exception as e:  # noqa: BLE001
                out["resident_opecol_order"] = {"error": repr(e)}
        return out

    def resident_order(self):
        """The serving form: OrderLS on the same rows as a resident OPE column (dds_opecol_order: the
        column's value bounds are kept on its writes, so no min/max pass; ids back in host memory)."""
        import numpy as np
        oc = self.eng.opecol(max(1, self.mine))
        try:
            oc.append(self.col, np.where(self.valid != 0, 2, 0).astype(np.uint8))
            # the reply buffer a caller reuses, engine-allocated (dds_host_alloc): the ids are DMA'd into it
            out_buf = self.eng.host_alloc(max(1, self.mine), np.uint32)
            ts = []
            self.eng.set_timing(True)
            self.eng.reset_timing()
            for _ in range(7):
                t = time.perf_counter()
                perm = oc.order(True, out=out_buf)
                ts.append((time.perf_counter() - t) * 1e3)
            _, _, dev_ms, _ = self.eng.timing()
            self.eng.set_timing(False)
            ts.sort()
            ok = bool(np.array_equal(perm, self.d_out.cpu().numpy().view(np.uint32))) if self.args.verify else None
            del perm
            self.eng.host_free(out_buf)
            med = ts[len(ts) // 2]
            return {"median_ms": med, "device_ms": dev_ms / 7, "matches_raw_array_order": ok,
                    "route_roofline": {"bound": "hbm", "achieved": 13 * self.mine / (med / 1e3) / 1e9, "peak": 8000.0,
                                       "unit": "GB/s", "frac": 13 * self.mine / (med / 1e3) / 1e9 / 8000.0,
                                       "note": "13 B/row / whole call time (host clock), the 40 MB id read-back included"},
                    "path": "dds_opecol_order (no k_rs_prep: bounds kept on writes; device_ms = HIP events around "
                            "the ordering) + D2H of the permutation into a dds_host_alloc reply buffer"}
        finally:
            oc.close()


class EntrySearchWorkload(_Workload):
    """SearchEntryOR (DDSRestServer.scala:879-903) + SearchEq at position 3 (:607-643) over a
    device-resident string table: 10M rows x 8 elements, each a 32-hex-char deterministic
    ciphertext drawn from a seeded vocabulary of 100k (HomoDet.compare = string equality).
    The table (chars, offsets, 32-bit fingerprints) is built once in setup, as a resident index."""

    ELEMS, WIDTH, VOCAB = 8, 32, 100_000

    def setup(self):
        import numpy as np
        rng = np.random.default_rng(self.args.seed)
        vocab = rng.integers(0, 16, size=(self.VOCAB, self.WIDTH), dtype=np.uint8)
        self.vocab = np.where(vocab < 10, vocab + 48, vocab + 87).astype(np.uint8)  # '0'-'9','a'-'f'
        nel = self.mine * self.ELEMS
        self.pick = rng.integers(0, self.VOCAB, size=nel, dtype=np.int64)
        chars = self.vocab[self.pick].tobytes()
        elem_off = np.arange(nel + 1, dtype=np.uint64) * self.WIDTH
        row_off = np.arange(self.mine + 1, dtype=np.uint64) * self.ELEMS
        t = time.perf_counter()
        self.tab = self.ddshe.StrTable(self.eng, chars=chars, elem_off=elem_off, row_off=row_off)
        self.build_s = time.perf_counter() - t
        del chars
        self.needles = [self.vocab[j].tobytes().decode() for j in (11, 222, 3333)]

    def _batch(self, picks):
        """(chars, elem_off, row_off) of rows given as vocabulary indices (rows x ELEMS)"""
        import numpy as np
        n = picks.shape[0]
        return (self.vocab[picks.reshape(-1)].tobytes(), np.arange(n * self.ELEMS + 1, dtype=np.uint64) * self.WIDTH,
                np.arange(n + 1, dtype=np.uint64) * self.ELEMS)

    def mutations(self):
        """The table under the write routes (outside the timed region): the per-request build the parity
        form pays without a resident table, then row rewrites / removals / appends on the resident table
        (C calls on batches already in the table layout), then the scans again, verified."""
        import numpy as np
        rng = np.random.default_rng(self.args.seed + 1)
        out = {"table_build_ms": self.build_s * 1e3,
               "table_build_note": "dds_strtab_create of the whole table from host buffers (upload + fingerprints): "
                                   "what a request pays without the resident table (routes.search_* parity form)"}
        p = self.pick.reshape(self.mine, self.ELEMS)
        live = np.ones(self.mine, dtype=bool)

        def timed(fn, reps=5):
            ts = []
            for _ in range(reps):
                t = time.perf_counter()
                fn()
                ts.append((time.perf_counter() - t) * 1e3)
            ts.sort()
            return ts[len(ts) // 2]

        for nrow in (1, 1000, 100_000):
            ids = rng.choice(self.mine, nrow, replace=False).astype(np.uint64)
            picks = rng.integers(0, self.VOCAB, size=(nrow, self.ELEMS))
            batch = self._batch(picks)
            out[f"write_rows_{nrow}_ms"] = timed(lambda: self.tab.write_rows_flat(ids, *batch))
            p[ids.astype(np.int64)] = picks
        ids = rng.choice(self.mine, 1000, replace=False).astype(np.uint64)
        out["set_live_1000_ms"] = timed(lambda: self.tab.set_live(ids, 0))
        live[ids.astype(np.int64)] = False
        out["search_after_writes_ms"] = timed(lambda: self.tab.search_entry(self.needles, False), 3)
        got_or = self.tab.search_entry(self.needles, False)
        got_eq = self.tab.search_eq(3, self.needles[0])
        want_or = np.nonzero(np.isin(p, [11, 222, 3333]).any(axis=1) & live)[0]
        want_eq = np.nonzero((p[:, 3] == 11) & live)[0]
        out["verified_after_writes"] = bool(np.array_equal(got_or, want_or) and np.array_equal(got_eq, want_eq))
        out["stats"] = self.tab.stats()
        return out

    def step(self):
        a = self.tab.search_entry(self.needles, False)
        b = self.tab.search_eq(3, self.needles[0])
        return a, b

    def local_ok(self, res):
        """This rank's SearchEntryOR / SearchEq rows against numpy over its own table."""
        import numpy as np
        p = self.pick.reshape(self.mine, self.ELEMS)
        want_or = np.nonzero(np.isin(p, [11, 222, 3333]).any(axis=1))[0]
        want_eq = np.nonzero(p[:, 3] == 11)[0]
        return bool(np.array_equal(res[0], want_or) and np.array_equal(res[1], want_eq))

    def verify_distributed(self):
        return self.all_ranks_ok(self.local_ok(self.last_res))

    def report(self, res, elapsed):
        import numpy as np
        a = self.args
        ok = None
        if a.verify and self.world == 1:
            ok = self.local_ok(res)
            if not ok:
                print("VERIFY FAILED", file=sys.stderr)
        _, _, dev_ms, _ = self.eng.timing()
        scan_s = dev_ms / 1e3 / (2 * a.steps)
        # per scan: the 2-byte fingerprints of the elements it must look at (OR: all; Eq: the element at
        # the position, through the position index, + its present bit) + one 4-byte id per match
        alg_or = self.mine * 2 * self.ELEMS + 4 * len(res[0])
        alg_eq = self.mine * (2 + 1 / 8) + 4 * len(res[1])
        alg = (alg_or + alg_eq) / 2
        roof = {"bound": "hbm", "kernel": "k_str_any + k_byte_count/k_ope_scatter (OR), k_str_eq_count + k_ope_scatter (Eq); device time",
                "achieved": alg / scan_s / 1e9, "peak": 8000.0, "unit": "GB/s", "frac": alg / scan_s / 1e9 / 8000.0,
                "avg_scan_ms": scan_s * 1e3, "algorithmic_bytes": alg,
                # HBM bytes per scan from the PMC pass (per dispatch): OR = k_str_any + k_byte_count +
                # k_ope_scatter, Eq = k_str_eq_count + k_ope_scatter, averaged over the two scans like alg
                "traffic": None, "traffic_unit": "HBM bytes per scan (PMC, profiles/" + PMC_FILE + ")"}
        t_or = pmc_traffic("entry_search", ("k_str_any", "k_byte_count", "k_ope_scatter"))
        t_eq = pmc_traffic("entry_search", ("k_str_eq_count", "k_ope_scatter"))
        if t_or is not None and t_eq is not None:
            roof["traffic"] = (t_or + t_eq) / 2
        mut = None
        if self.world == 1:  # before the CPU baseline (its 1.6M Python strings slow every later Python call)
            try:
                mut = self.mutations()
            except Exception as e:  # noqa: BLE001  (reported in the line, not lost)
                mut = {"error": repr(e)}
        cpu = None
        if self.world == 1 and not a.no_cpu_baseline:
            from oracle import homo
            sample = 200_000
            rows = [[self.vocab[j].tobytes().decode() for j in r] for r in
                    self.pick[: sample * self.ELEMS].reshape(sample, self.ELEMS)]
            keyed = list(enumerate(rows))
            t = time.perf_counter()
            homo.search_entry("SearchEntryOR", keyed, self.needles)
            dt = time.perf_counter() - t
            cpu = {"value": sample / dt, "unit": "rows/s", "cores": 1, "kind": "port",
                   "sample": f"first {sample} rows, SearchEntryOR restated in Python (oracle/homo.py), {dt:.2f}s"}
        out = self.common("Deterministic-equality scan rows/sec (SearchEntryOR + SearchEq)",
                          self.total * 2 * a.steps / elapsed, "rows/s", elapsed, "det_entry_search_10Mx8",
                          {"elements_per_row": self.ELEMS, "element_bytes": self.WIDTH})
        out.update(data="synthetic (seeded 32-hex-char ciphertext vocabulary)", dtype="u64 digest + u8",
                   roofline=roof, cpu_baseline=cpu, verified=ok, matches={"or": len(res[0]), "eq": len(res[1])})
        if mut is not None:
            out["resident_mutations"] = mut
        if self.world == 1:
            out["native_call"] = self.native_scan()
        return out

    def native_scan(self):
        """The same two routes from C++ (tools/native/scan_bench: the calls a JNA binding makes, without the
        Python binding's marshalling) over its own seeded table of the same shape, every reply checked in
        the child against a host scan."""
        exe = os.path.join(ROOT, "tools", "native", "scan_bench")
        if not os.path.exists(exe):
            return {"skipped": "tools/native/scan_bench not built"}
        import subprocess
        try:
            pr = subprocess.run([exe, str(self.mine)], capture_output=True, text=True, timeout=300)
        except subprocess.TimeoutExpired:
            return {"error": "timeout"}
        if pr.returncode != 0:
            return {"error": pr.stderr[-400:]}
        return json.loads(pr.stdout.strip().splitlines()[-1])

    def close(self):
        self.tab.close()


def cpu_encrypt_baseline(k, rcol, ms, seconds, out_col=None):
    """Paillier encryption g^m r^n mod n^2 with OpenSSL BN_mod_exp (Montgomery + sliding window,
    oracle/csrc/bn_baseline.c), public key, 1 thread and cpu_threads() threads, on the first rows of
    the same r column; the GPU ciphertexts of those rows are compared."""
    from oracle import cref
    rs = rcol.read(0, min(len(rcol), 64))
    t = time.perf_counter()
    cref.bn_paillier_encrypt(k["n"], k["g"], ms[:8], rs[:8], 1)
    rate = 8 / (time.perf_counter() - t)
    sample = int(min(len(rcol), max(16, rate * seconds), 4096))
    rs = rcol.read(0, sample)
    t = time.perf_counter()
    ref = cref.bn_paillier_encrypt(k["n"], k["g"], ms[:sample], rs, 1)
    dt = time.perf_counter() - t
    th = cpu_threads()
    sample_mt = min(len(rcol), sample * th)
    rs_mt = rcol.read(0, sample_mt)
    t = time.perf_counter()
    cref.bn_paillier_encrypt(k["n"], k["g"], ms[:sample_mt], rs_mt, th)
    dt_mt = time.perf_counter() - t
    res = {"value": sample / dt, "unit": "encrypt/s", "cores": 1, "kind": "port",
           "sample": f"first {sample} rows, g^m r^n mod n^2 with OpenSSL BN_mod_exp (public key), {dt:.1f}s",
           "multi_thread": {"value": sample_mt / dt_mt, "cores": th, "sample": f"first {sample_mt} rows"}}
    if out_col is not None:
        res["gpu_matches_sample"] = out_col.read(0, sample) == ref
    return res


def cpu_threads():
    """Host threads for the multi-threaded baseline: the box's CPU share for one GPU (16), not
    os.cpu_count(), which reports the whole machine there."""
    return max(1, min(16, os.cpu_count() or 1))


def cpu_baseline(col, nsq, mb, seconds):
    """Reference fold restated with OpenSSL (oracle/csrc/bn_baseline.c: acc = acc*x mod N with
    BN_mod_mul, the BigInteger multiply+mod analogue), 1 thread as the reference's single
    onComplete loop, on a bounded prefix of the same column; the GPU fold of that prefix is compared.
    Also: the same prefix sliced over cpu_threads() threads, and the schoolbook C restatement."""
    from oracle import cref
    calib = min(len(col), 4000)
    ops = col.read_buffer(0, calib).tobytes()  # canonical big-endian rows, mb bytes each
    mod_be = nsq.to_bytes(mb, "big")
    t = time.perf_counter()
    cref.bn_fold_be(mod_be, ops, mb, calib)
    rate = (calib - 1) / (time.perf_counter() - t)
    sample = int(min(len(col), max(calib, rate * seconds)))
    ops = col.read_buffer(0, sample).tobytes()
    t = time.perf_counter()
    ref = cref.bn_fold_be(mod_be, ops, mb, sample)
    dt = time.perf_counter() - t
    th = cpu_threads()
    t = time.perf_counter()
    ref_mt = cref.bn_fold_be(mod_be, ops, mb, sample, th)
    dt_mt = time.perf_counter() - t
    small = min(sample, 20000)
    t = time.perf_counter()
    ref_sb = cref.fold_be(mod_be, ops[: small * mb], mb, small)
    dt_sb = time.perf_counter() - t
    gpu = col.fold(0, sample)
    return {"value": (sample - 1) / dt, "unit": "HomoAdd/s", "cores": 1, "kind": "port",
            "sample": f"first {sample} rows of the same column, acc=acc*x mod N with OpenSSL BN_mod_mul, {dt:.1f}s",
            "gpu_matches_sample": gpu == int.from_bytes(ref, "big") == int.from_bytes(ref_mt, "big"),
            "multi_thread": {"value": (sample - 1) / dt_mt, "cores": th,
                             "sample": "same prefix in contiguous slices, partials combined"},
            "schoolbook_port": {"value": (small - 1) / dt_sb, "cores": 1,
                                "sample": f"first {small} rows, oracle/csrc/fold_ref.c (schoolbook + Knuth D)",
                                "matches": int.from_bytes(ref_sb, "big") == col.fold(0, small)},
            # a JVM BigInteger harness when `java` exists on the box (it does not in this image)
            "jvm": shutil.which("java")}


if __name__ == "__main__":
    sys.exit(main())
