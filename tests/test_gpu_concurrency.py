"""Concurrent calls on one context (include/ddshe.h: "Calls may run concurrently on one ctx"; the
reference's routes run on the global ForkJoin pool, DDSRestServer.scala:21, with no locking).
Several host threads mix folds under two moduli, chunked host-buffer folds (the shared host copy
pool), decimal ingest and OPE filters on one Engine; every result must be bit-exact."""
import random
import threading

import numpy as np
import pytest

from oracle import homo

pytestmark = pytest.mark.gpu


def test_concurrent_mixed_calls(eng, keys):
    pk = keys["paillier2048_committed"]
    rsa = keys["rsa2048_seed3"]
    nsq, n = pk["nsquare"], rsa["n"]
    rng = random.Random(99)
    xs = [rng.randrange(nsq) for _ in range(257)]
    ys = [rng.randrange(n) for _ in range(301)]
    want_x, want_y = homo.modmul_fold(xs, nsq), homo.modmul_fold(ys, n)
    big = eng.column(nsq, 140_000)  # > one 64 MiB ingest chunk of 512-byte rows
    big.fill_paillier_synth(pk["n"], pk["g"], 5, 0, 140_000)
    buf = big.read_buffer(0, 140_000)
    want_big = big.fold()
    ope = np.random.default_rng(3).integers(-(1 << 62), 1 << 62, size=50_000, dtype=np.int64)
    bound = int(ope[17])
    want_gt = np.flatnonzero(ope > bound).astype(np.uint32)
    errors = []

    def worker(t):
        try:
            for it in range(4):
                k = (t + it) % 4
                if k == 0:
                    assert eng.paillier_sum(nsq, xs) == want_x
                elif k == 1:
                    assert eng.rsa_product(n, ys) == want_y
                elif k == 2:
                    assert eng.fold_buffer(nsq, buf) == want_big
                else:
                    col = eng.column(nsq, len(xs))
                    col.append_dec([str(x) for x in xs])
                    assert col.fold() == want_x
                    col.close()
                    assert np.array_equal(eng.ope_filter(ope, None, bound, "gt"), want_gt)
        except Exception as e:  # reported on the main thread
            errors.append((t, repr(e)))

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(6)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=100)
    big.close()
    assert not any(th.is_alive() for th in threads)
    assert not errors, errors


def test_concurrent_lane_fold_and_small_pairs(eng, keys):
    """Round-2 paths under concurrency: a MultAll fold large enough for the one-bignum-per-lane kernel
    (k_fold1, >= ~1M rows), small pair batches (the latency path) and their batched form, from
    several threads on one context; every result equals the one computed alone."""
    rsa = keys["rsa2048_seed3"]
    n = rsa["n"]
    rows = 1_200_000
    col = eng.column(n, rows)
    col.fill_random(2040, 21, 0, rows)
    want_fold = col.fold()
    sub = list(range(0, rows, 3))
    want_sub = col.fold_rows(sub)
    rng = random.Random(5)
    pa = [[rng.randrange(n) for _ in range(k)] for k in (1, 2, 8, 40)]
    pb = [[rng.randrange(n) for _ in range(k)] for k in (1, 2, 8, 40)]
    want_p = [[x * y % n for x, y in zip(a, b)] for a, b in zip(pa, pb)]
    errors = []

    def worker(t):
        try:
            for it in range(3):
                k = (t + it) % 3
                if k == 0:
                    assert col.fold() == want_fold
                elif k == 1:
                    assert col.fold_rows(sub) == want_sub
                else:
                    for a, b, w in zip(pa, pb, want_p):
                        assert eng.modmul_pairs(n, a, b) == w
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    col.close()
    assert not errors, errors[:3]
