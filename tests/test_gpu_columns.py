"""Resident columns on the GPU: row-subset folds, the one-operand fold returning the appended operand,
decimal replies, the resident OPE column, device-resident partial exchange, partial validation, the
row limit, and concurrent folds with many distinct exponents. All checked against the oracle.
References: DDSRestServer.scala:401-446 (SumAll), :491-539 (MultAll), :541-606 (Order*), :682-830
(Search*)."""
import random
import threading

import numpy as np
import pytest

from oracle import homo

pytestmark = pytest.mark.gpu


def test_fold_rows_vs_oracle(eng, keys):
    N = keys["paillier2048_committed"]["nsquare"]
    rng = random.Random(41)
    xs = [rng.randrange(N) for _ in range(3000)]
    col = eng.column(N, len(xs))
    col.append(xs)
    for ids in ([5, 7], list(range(0, 3000, 3)), sorted(rng.sample(range(3000), 1777)), [9, 9, 9],
                [2999, 0, 1500, 17], list(range(3000))):
        assert col.fold_rows(ids) == homo.modmul_fold([xs[i] for i in ids], N), len(ids)
        assert col.fold_dec(ids) == str(homo.modmul_fold([xs[i] for i in ids], N))
    assert col.fold_rows([42]) == xs[42]
    import ddshe
    with pytest.raises(ddshe.NotFound):
        col.fold_rows([])
    with pytest.raises(ddshe.DDSError):
        col.fold_rows([3000])
    col.close()


def test_fold_rows_rsa_shape(eng, keys):
    n = keys["rsa2048_seed3"]["n"]
    rng = random.Random(43)
    xs = [rng.randrange(n) for _ in range(5000)]
    col = eng.column(n, len(xs))
    col.append(xs)
    ids = sorted(rng.sample(range(5000), 4321))
    assert col.fold_rows(ids) == homo.modmul_fold([xs[i] for i in ids], n)
    col.close()


def test_single_operand_is_the_appended_value(eng, keys):
    """A one-row fold returns the operand unreduced (:416-417), also for rows the column had to store
    as residues: >= 2N binary rows, negative or signed decimal rows."""
    N = keys["paillier1024_seed1"]["nsquare"]
    col = eng.column(N, 16)
    big = 3 * N + 12345                    # >= 2N: reduced on ingest
    mid = N + 77                           # in [N, 2N): stored verbatim
    col.append([big, mid, 5])
    assert col.fold(0, 1) == big and col.fold_rows([0]) == big
    assert col.fold(1, 1) == mid and col.fold_rows([1]) == mid
    assert col.fold(0, 3) == homo.modmul_fold([big, mid, 5], N)
    col.append_dec(["-12345", "+0007", str(5 * N + 3)])
    assert col.fold_dec([3]) == "-12345"
    assert col.fold_dec([4]) == "7"
    assert col.fold_dec([5]) == str(5 * N + 3)
    assert col.fold_rows([5]) == 5 * N + 3
    import ddshe
    with pytest.raises(ddshe.DDSError):
        col.fold_rows([3])                 # a negative operand has no magnitude form
    want = homo.modmul_fold([big, mid, 5, -12345, 7, 5 * N + 3], N)
    assert col.fold_dec(None, 6) == str(want)
    col.truncate(3)
    col.append([11])
    assert col.fold_rows([3]) == 11        # the remembered original of the dropped row is gone
    col.close()


def test_opecol_search_and_order_vs_oracle(eng):
    """dds_opecol against the oracle's route restatement on rows with every class: lacking the
    position, last element, inner; values at the int64 edges and beyond; Int elements."""
    rng = random.Random(7)
    rows = []
    for i in range(4000):
        kind = rng.random()
        if kind < 0.05:
            rows.append((f"k{i}", ["x"] if rng.random() < 0.5 else []))          # lacks position 1
        elif kind < 0.1:
            rows.append((f"k{i}", ["x", str(rng.randrange(-10**6, 10**6))]))    # position 1 is last
        elif kind < 0.12:
            rows.append((f"k{i}", ["x", str(rng.choice([2**63 - 1, -2**63, 2**70, -2**70, 2**63])), "t"]))
        elif kind < 0.14:
            rows.append((f"k{i}", ["x", rng.randrange(-50, 50), "t"]))           # Int element
        else:
            rows.append((f"k{i}", ["x", str(rng.randrange(-10**6, 10**6)), "t"]))
    from ddshe import routes
    for route in ("SearchGt", "SearchGtEq", "SearchLt", "SearchLtEq"):
        for bound in ("0", "999999", str(2**63), str(-2**63), str(2**70), "-5"):
            got = routes.search(eng, route, rows, 1, bound)
            assert sorted(got) == sorted(homo.search(route, rows, 1, bound)), (route, bound)
    # Order: the Int elements make it a 500 (ClassCastException, two or more holders) ...
    with pytest.raises(routes.ServerError):
        routes.order(eng, "OrderLS", rows, 1)
    # ... and so do values outside Long; without them it matches the oracle's stable order
    clean = [(k, r) for k, r in rows if len(r) < 2 or (isinstance(r[1], str) and -2**63 <= int(r[1]) < 2**63)]
    for route in ("OrderLS", "OrderSL"):
        assert routes.order(eng, route, clean, 1) == homo.order(route, clean, 1)


def test_opecol_search_into_reply_buffers(eng):
    """dds_opecol_search into the caller's reusable reply buffer: an engine-allocated one (one DMA), a
    registered numpy array, and a plain array, each equal to the fresh-array answer, with wide (beyond
    int64) matches merged in row order and a buffer reused across calls of different match counts."""
    import numpy as np
    rng = np.random.default_rng(5)
    n = 300_001
    vals = [str(int(v)) for v in rng.integers(-10**9, 10**9, size=n)]
    vals[17] = str(2**70)
    vals[250_000] = str(-2**70)
    col = eng.opecol(n)
    col.append_dec(vals, cls=[2] * n)
    ebuf = eng.host_alloc(n, np.uint32)
    rbuf = np.empty(n, dtype=np.uint32)
    eng.host_register(rbuf)
    pbuf = np.empty(n, dtype=np.uint32)
    try:
        for op in ("gt", "ge", "lt", "le"):
            for bound in ("0", "999999999", "-1000000000", str(2**64)):
                want = col.search(bound, op)
                for buf in (ebuf, rbuf, pbuf):
                    got = col.search(bound, op, out=buf)
                    assert np.array_equal(got, want), (op, bound)
        with pytest.raises(ValueError):
            col.search("0", "gt", out=np.empty(10, dtype=np.uint32))
    finally:
        eng.host_unregister(rbuf)
        eng.host_free(ebuf)


def test_opecol_resident_api(eng):
    """The resident column across requests: appends, truncate, int64 appends, lazy bound parse."""
    import ddshe
    col = eng.opecol(100)
    assert len(col.search("junk", "gt")) == 0                       # no row: bound never parsed
    col.append_dec(["5", None, "7"], cls=[1, 0, 2])
    with pytest.raises(ddshe.DDSError):
        col.search("junk", "gt")                                      # row 2 qualifies -> 500
    assert list(col.search("6", "gt")) == [2]
    assert list(col.search("8", "lt")) == [2]                          # row 0 is not searchable (last)
    col.append(np.array([1, 100, -4], dtype=np.int64))
    assert list(col.search("1", "ge")) == [2, 3, 4]
    assert list(col.order(True)) == [4, 2, 0, 3, 5, 1]                # holders desc, then row 1
    assert list(col.order(False)) == [1, 5, 3, 0, 2, 4]
    col.truncate(3)
    assert len(col) == 3 and list(col.search("0", "gt")) == [2]
    col.append_dec(["zz"], cls=[2])
    with pytest.raises(ddshe.DDSError):
        col.search("0", "gt")
    col.truncate(3)
    assert list(col.search("0", "gt")) == [2]
    col.close()


def test_partial_device_roundtrip(eng, keys):
    """dds_col_fold_partial_device + dds_combine_partials_device (the multi-process D2D exchange)."""
    import torch
    N = keys["paillier2048_committed"]["nsquare"]
    rng = random.Random(51)
    xs = [rng.randrange(N) for _ in range(2500)]
    col = eng.column(N, len(xs))
    col.append(xs)
    pw = col.partial_words
    cuts = [(0, 1000), (1000, 1), (1001, 0), (1001, 1499)]
    buf = torch.zeros(len(cuts) * pw, dtype=torch.int32, device="cuda")
    for j, (a, c) in enumerate(cuts):
        col.fold_partial_device(buf.data_ptr() + 4 * j * pw, a, c)
    torch.cuda.synchronize()
    rows = [c for _, c in cuts]
    assert eng.combine_partials_device(N, buf.data_ptr(), rows) == homo.modmul_fold(xs, N)
    host = buf.cpu().numpy().view(np.uint32).reshape(len(cuts), pw)
    assert eng.combine_partials(N, host, rows) == homo.modmul_fold(xs, N)
    col.close()


def test_combine_rejects_malformed_partials(eng, keys):
    import ddshe
    N = keys["paillier2048_committed"]["nsquare"]
    col = eng.column(N, 100)
    col.append(list(range(2, 102)))
    p, r = col.fold_partial()
    bad = p.copy()
    bad[3] = 1 << 29                                  # limb not normalised
    with pytest.raises(ddshe.DDSError) as ei:
        eng.combine_partials(N, np.stack([p, bad]), [r, r])
    assert ei.value.status == ddshe.DDS_E_RANGE
    bad = p.copy()
    bad[: col.partial_words - 2] = (1 << 28) - 1      # value far above the bound
    with pytest.raises(ddshe.DDSError) as ei:
        eng.combine_partials(N, np.stack([p, bad]), [r, r])
    assert ei.value.status == ddshe.DDS_E_RANGE
    assert eng.combine_partials(N, np.stack([p, p]), [r, r]) == homo.modmul_fold(list(range(2, 102)) * 2, N)
    col.close()


def test_row_limit_is_enforced(eng, keys):
    """Columns beyond the kernels' 32-bit buffer addressing (max_stride) are refused, not wrapped."""
    import ddshe
    N = keys["paillier2048_committed"]["nsquare"]
    with pytest.raises(ddshe.DDSError) as ei:
        eng.column(N, (1 << 28) + 1)
    assert ei.value.status == ddshe.DDS_E_UNSUPPORTED


def test_concurrent_folds_many_exponents(eng, keys):
    """> 64 distinct (count, groups) exponents from 8 threads at once: the finalize multipliers are
    looked up while other threads evict the cache (use-after-free in y_for)."""
    N = keys["paillier1024_seed1"]["nsquare"]
    rng = random.Random(61)
    xs = [rng.randrange(N) for _ in range(400)]
    col = eng.column(N, len(xs))
    col.append(xs)
    prefix = [xs[0]]
    for x in xs[1:]:
        prefix.append(prefix[-1] * x % N)
    errors = []

    def worker(t):
        for k in range(2 + t, 400, 8):
            if col.fold(0, k) != prefix[k - 1]:
                errors.append((t, k))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:5]
    col.close()
