"""The device-to-device partial gather through RCCL itself: an `nccl` process group
at world size 1 on cuda:0 (RCCL refuses two ranks on one device, and this box has one GPU), a 100k-row
column under the committed 2048-bit key folded to a device partial (dds_col_fold_partial_device), moved
by all_gather_into_tensor (RCCL kernels on the GPU) and combined by dds_combine_partials_device — the
exact sequence bench.py's N > 1 ranks run (DDSRestServer.scala:412-430 folded by key range). The result
must equal the resident fold and, on a prefix, the oracle's fold; the worker also reports that librccl
is mapped into it, so the test cannot pass on gloo by accident."""
import os
import socket

import pytest
import torch.multiprocessing as mp

from oracle import homo

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "dependable-data-storage-csd2017_amd")


def _worker(port, key, rows, prefix, out_q):
    import sys
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    try:
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                device_id=torch.device("cuda", 0))
        import ddshe
        import ddshe.dist as dd
        eng = ddshe.Engine(0)
        eng.set_stream(torch.cuda.current_stream().cuda_stream)
        nsq = key["nsquare"]
        col = eng.column(nsq, rows)
        col.fill_paillier_synth(key["n"], key["g"], 2, 0, rows, 1024)
        dev = torch.device("cuda", 0)
        got = []
        for cnt in (rows, prefix):
            g = dd.gather_partials_device(col, 0, cnt, dev)
            assert g.is_cuda and g.numel() == col.partial_words
            got.append(eng.combine_partials_device(nsq, g.data_ptr(), [cnt]))
        torch.cuda.synchronize()
        full = col.fold(0, rows)
        pre_rows = col.read(0, prefix)
        maps = open("/proc/self/maps").read()
        out_q.put({"got": got, "full": full, "prefix_rows": pre_rows, "backend": dist.get_backend(),
                   "rccl_mapped": "librccl" in maps})
        col.close()
        eng.close()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001 (reported to the test, not lost in the child)
        import traceback
        out_q.put({"error": f"{type(e).__name__}: {e}", "tb": traceback.format_exc()[-2000:]})


def test_rccl_device_gather_combine(keys):
    key = keys["paillier2048_committed"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:  # a free port for the TCP store
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    p = ctx.Process(target=_worker, args=(port, key, 100_000, 1500, q))
    p.start()
    try:
        r = q.get(timeout=100)
    finally:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert "error" not in r, r
    assert p.exitcode == 0
    assert r["backend"] == "nccl" and r["rccl_mapped"]
    assert r["got"][0] == r["full"]
    assert r["got"][1] == homo.modmul_fold(r["prefix_rows"], key["nsquare"])
