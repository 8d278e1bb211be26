"""String-table probe (tool, not product): scan time before and after row writes / removals, per call,
to locate where a post-write scan spends its time (run under rocprofv3 --kernel-trace for kernel times)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "dependable-data-storage-csd2017_amd")]
import ddshe  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
E, Wd, V = 8, 32, 100_000
rng = np.random.default_rng(1)
vocab = rng.integers(0, 16, size=(V, Wd), dtype=np.uint8)
vocab = np.where(vocab < 10, vocab + 48, vocab + 87).astype(np.uint8)
pick = rng.integers(0, V, size=rows * E)
eng = ddshe.Engine(0)
tab = ddshe.StrTable(eng, chars=vocab[pick].tobytes(), elem_off=np.arange(rows * E + 1, dtype=np.uint64) * Wd,
                     row_off=np.arange(rows + 1, dtype=np.uint64) * E)
needles = [vocab[j].tobytes().decode() for j in (11, 222, 3333)]


def t(label, fn, reps=3):
    ts = []
    for _ in range(reps):
        a = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - a) * 1e3)
    print(f"{label}: " + " ".join(f"{x:.3f}" for x in ts) + " ms", flush=True)


t("search_entry before", lambda: tab.search_entry(needles))
t("search_eq before", lambda: tab.search_eq(3, needles[0]))
ids = rng.choice(rows, 1000, replace=False).astype(np.uint64)
p = rng.integers(0, V, size=(1000, E))
batch = (vocab[p.reshape(-1)].tobytes(), np.arange(1000 * E + 1, dtype=np.uint64) * Wd,
         np.arange(1001, dtype=np.uint64) * E)
t("write_rows 1000", lambda: tab.write_rows_flat(ids, *batch), 1)
t("search_entry after write", lambda: tab.search_entry(needles))
t("search_eq after write", lambda: tab.search_eq(3, needles[0]))
t("set_live 1000", lambda: tab.set_live(ids, 0), 1)
t("search_entry after set_live", lambda: tab.search_entry(needles))
t("search_eq after set_live", lambda: tab.search_eq(3, needles[0]))
print(tab.stats())
tab.close()
eng.close()
