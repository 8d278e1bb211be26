"""A/B probe of the 8-GPU strong-split share on one GPU: one share of the
10M-row headline (1.25M rows, committed 2048-bit key) folded to a device partial
(dds_col_fold_partial_device); prints the share's wall time, its level-1 launch (HIP events) and the
tail. Run under DDSHE_PARTIAL_GROUPS=<cap> to cap level 1's lane groups (0: the engine's plan)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dependable-data-storage-csd2017_amd")]

import torch  # noqa: E402

import ddshe  # noqa: E402
from tests.conftest import _load_keys  # noqa: E402

k = _load_keys()["paillier2048_committed"]
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1_250_000
eng = ddshe.Engine(0)
col = eng.column(k["nsquare"], rows)
col.fill_paillier_synth(k["n"], k["g"], 2, 0, rows, 1024)
pw = col.partial_words
buf = torch.empty(pw, dtype=torch.int32, device="cuda")


def share():
    col.fold_partial_device(buf.data_ptr(), 0, rows)
    torch.cuda.synchronize()


for _ in range(3):
    share()
ts = []
for _ in range(15):
    t = time.perf_counter()
    share()
    ts.append((time.perf_counter() - t) * 1e3)
ts.sort()
eng.set_timing(True)
eng.reset_timing()
for _ in range(5):
    share()
lvl_ms, lvl_n, _, _ = eng.timing()
eng.set_timing(False)
first = buf.cpu().numpy().tobytes()
ok = eng.combine_partials_device(k["nsquare"], buf.data_ptr(), [rows]) == col.fold(0, rows)
lvl = lvl_ms / lvl_n if lvl_n else None
print(json.dumps({"groups_cap": int(os.environ.get("DDSHE_PARTIAL_GROUPS", "0")), "rows": rows,
                  "share_ms": ts[len(ts) // 2], "share_min_ms": ts[0], "level1_ms": lvl,
                  "tail_ms": ts[len(ts) // 2] - lvl if lvl else None, "partial_matches_fold": ok}))
