"""The resident string table under the write routes (VERDICT r03 "next" 2 and 4).

SearchEq/NEq (DDSRestServer.scala:607-681), SearchEntry/OR/AND (:831-938) and IsElement (:322-353)
read the stored sets that PutSet (:170-205), AddElement (:220-255), WriteElement (:281-321) and
RemoveSet (:207-218) change. dds_strtab follows them in place (dds_strtab_append / write_rows /
set_live / truncate); checked here against the oracle's restatements after every batch of writes,
through heap compactions and SearchEq position-index patches, and with scans and writes from 16
threads on one table (and on one resident OPE column) at once.
"""
import random
import threading

import numpy as np
import pytest

from oracle import homo

pytestmark = pytest.mark.gpu


def _words(rng, k, tag):
    return [f"{tag}{rng.getrandbits(40):x}" for _ in range(k)] + ["", "7"]


def _rand_row(rng, words):
    return [rng.choice(words) for _ in range(rng.randrange(0, 9))]


def _check_all(tab, rows, live, words, rng, label):
    keyed = [(i, r if lv else None) for i, (r, lv) in enumerate(zip(rows, live))]
    for _ in range(3):
        value = rng.choice(words)
        for position in (0, 1, 3):
            for negate in (False, True):
                route = "SearchNEq" if negate else "SearchEq"
                want = sorted(homo.search_eq(route, keyed, position, value))
                got = tab.search_eq(position, value, negate).tolist()
                assert got == want, (label, route, position, value)
    v = [rng.choice(words) for _ in range(3)]
    assert tab.search_entry(v[:1]).tolist() == sorted(homo.search_entry("SearchEntryOR", keyed, v[:1])), label
    assert tab.search_entry(v).tolist() == sorted(homo.search_entry("SearchEntryOR", keyed, v)), label
    assert tab.search_entry(v, True).tolist() == sorted(homo.search_entry("SearchEntryAND", keyed, v)), label
    from ddshe import NotFound
    for r in rng.sample(range(len(rows)), min(6, len(rows))):
        value = rng.choice(rows[r]) if rows[r] and rng.random() < 0.6 else rng.choice(words)
        if live[r]:
            assert tab.is_element(r, value) == homo.is_element(rows[r], value), (label, r)
        else:
            with pytest.raises(NotFound):
                tab.is_element(r, value)


def test_strtab_writes_vs_oracle(eng):
    """appends, row rewrites (duplicated ids in a batch: the last wins), removals and revivals,
    truncation; SearchEq indexes cached before the writes are patched, not rebuilt; the heap is
    compacted when it fills (stats), every scan exact after every batch."""
    rng = random.Random(404)
    words = _words(rng, 30, "w")
    rows = [_rand_row(rng, words) for _ in range(3000)]
    live = [True] * len(rows)
    tab = eng.strtab(rows)
    try:
        _check_all(tab, rows, live, words, rng, "initial")
        for it in range(24):
            ids = [rng.randrange(len(rows)) for _ in range(60)]
            ids += ids[:5]  # repeated ids: the batch's last row wins
            new = [_rand_row(rng, words) for _ in ids]
            tab.write_rows(ids, new)
            for i, r in zip(ids, new):
                rows[i] = r
                live[i] = True
            app = [_rand_row(rng, words) for _ in range(rng.randrange(0, 40))]
            tab.append(app)
            rows += app
            live += [True] * len(app)
            d = rng.sample(range(len(rows)), 80)
            flags = [rng.random() < 0.75 for _ in d]  # mostly removals, some revivals
            tab.set_live(d, [0 if f else 1 for f in flags])
            for i, f in zip(d, flags):
                live[i] = not f
            if it % 8 == 7:
                keep = len(rows) - 17
                tab.truncate(keep)
                del rows[keep:]
                del live[keep:]
            st = tab.stats()
            assert st["rows"] == len(rows) and st["live"] == sum(live), (it, st)
            assert st["elems"] == sum(len(r) for r in rows), (it, st)
            assert st["heap_elems"] <= 2 * st["elems"] + 2048, (it, st)
            _check_all(tab, rows, live, words, rng, f"iteration {it}")
        st = tab.stats()
        assert st["compactions"] >= 2, st  # the creation's own + at least one from the writes
        assert st["pos_indexes"] >= 2, st
        # writes of rows past the end and bad batches are rejected and change nothing
        from ddshe import DDSError
        with pytest.raises(DDSError):
            tab.write_rows([len(rows)], [["x"]])
        _check_all(tab, rows, live, words, rng, "after rejected writes")
    finally:
        tab.close()


def test_strtab_empty_and_growth(eng):
    """A table created empty (the resident store's start) grows by appends from zero rows and zero
    elements; empty rows and empty strings are rows / elements like any other."""
    rng = random.Random(7)
    words = _words(rng, 5, "e")
    tab = eng.strtab([])
    rows, live = [], []
    try:
        assert tab.nrows == 0 and tab.search_entry(["x"]).tolist() == []
        for it in range(40):
            app = [[] if rng.random() < 0.2 else _rand_row(rng, words) for _ in range(rng.randrange(1, 300))]
            tab.append(app)
            rows += app
            live += [True] * len(app)
            if it % 5 == 4:
                _check_all(tab, rows, live, words, rng, f"growth {it}")
        assert tab.stats()["rows"] == len(rows)
    finally:
        tab.close()


def test_strtab_concurrent_scans_and_writes(eng):
    """16 threads on one table: 12 scan (SearchEq / SearchEntry / IsElement on stable rows and values,
    whose answers no write may change), 4 write the volatile rows (rewrites, removals, revivals) with
    values from their own vocabulary. Every scan answer on the stable vocabulary must be
    exact at every moment; the final state is checked against the oracle."""
    rng = random.Random(99)
    stable_words = _words(rng, 20, "s")[:-2]
    vol_words = _words(rng, 20, "v")[:-2]
    ns, nv = 4000, 2000
    rows = [_rand_row(rng, stable_words) for _ in range(ns)] + [_rand_row(rng, vol_words) for _ in range(nv)]
    live = [True] * len(rows)
    tab = eng.strtab(rows)
    want_eq = {}
    for value in stable_words[:6]:
        for position in (0, 2):
            want_eq[(value, position)] = [i for i in range(ns) if len(rows[i]) - 1 > position and rows[i][position] == value]
    want_any = {v: [i for i in range(ns) if v in rows[i]] for v in stable_words[:6]}
    errors = []
    lock = threading.Lock()
    stop = threading.Event()

    def reader(seed):
        r = random.Random(seed)
        try:
            while not stop.is_set():
                v = r.choice(stable_words[:6])
                if r.random() < 0.5:
                    p = r.choice((0, 2))
                    got = tab.search_eq(p, v).tolist()
                    if got != want_eq[(v, p)]:
                        errors.append(("eq", v, p, len(got), len(want_eq[(v, p)])))
                else:
                    got = tab.search_entry([v]).tolist()
                    if got != want_any[v]:
                        errors.append(("any", v, len(got), len(want_any[v])))
                i = r.randrange(ns)
                if rows[i] and not tab.is_element(i, rows[i][0]):
                    errors.append(("iselem", i))
        except Exception as e:  # noqa: BLE001
            errors.append(("reader", repr(e)))

    def writer(seed):
        r = random.Random(seed)
        try:
            for _ in range(60):
                with lock:  # the host mirror only; the table calls run concurrently with the readers
                    ids = [ns + r.randrange(nv) for _ in range(20)]
                    new = [_rand_row(r, vol_words) for _ in ids]
                    tab.write_rows(ids, new)
                    for i, x in zip(ids, new):
                        rows[i] = x
                        live[i] = True
                    d = [ns + r.randrange(nv) for _ in range(10)]
                    fl = [r.random() < 0.5 for _ in d]
                    tab.set_live(d, [0 if f else 1 for f in fl])
                    for i, f in zip(d, fl):
                        live[i] = not f
        except Exception as e:  # noqa: BLE001
            errors.append(("writer", repr(e)))

    readers = [threading.Thread(target=reader, args=(s,)) for s in range(12)]
    writers = [threading.Thread(target=writer, args=(100 + s,)) for s in range(4)]
    for t in readers + writers:
        t.start()
    for t in writers:
        t.join()
    stop.set()
    for t in readers:
        t.join()
    try:
        assert not errors, errors[:5]
        _check_all(tab, rows, live, vol_words + stable_words, rng, "final")
    finally:
        tab.close()


def test_opecol_concurrent_search_order_writes(eng):
    """16 threads on one resident OPE column (shared lock for Search / Order, exclusive for writes): 12
    run search_mask / search / order and check the stable rows' answers, 4 rewrite the volatile rows
    with values below every stable value; the final state is checked against numpy."""
    rng = np.random.default_rng(5)
    ns, nv = 60_000, 20_000
    vals = np.concatenate([rng.integers(1_000_000, 2_000_000, ns), rng.integers(-1_000, 0, nv)]).astype(np.int64)
    col = eng.opecol(ns + nv)
    col.append(vals)
    bound = 1_500_000
    want_gt = np.flatnonzero(vals[:ns] > bound)
    stable_order = np.argsort(-vals[:ns], kind="stable")
    errors = []

    def reader(seed):
        r = random.Random(seed)
        try:
            for _ in range(25):
                k = r.randrange(3)
                if k == 0:
                    words, cnt = col.search_mask(str(bound), "gt")
                    bits = np.unpackbits(words.view(np.uint8), bitorder="little")[: ns + nv].astype(bool)
                    if not np.array_equal(np.flatnonzero(bits), want_gt) or cnt != len(want_gt):
                        errors.append(("mask", cnt))
                elif k == 1:
                    ids = col.search(str(bound), "gt")
                    if not np.array_equal(ids, want_gt):
                        errors.append(("ids", len(ids)))
                else:
                    perm = col.order(True)  # OrderLS: the stable rows (all above the volatile ones) first
                    if not np.array_equal(perm[:ns], stable_order):
                        errors.append(("order",))
        except Exception as e:  # noqa: BLE001
            errors.append(("reader", repr(e)))

    final = vals.copy()
    flock = threading.Lock()

    def writer(seed):
        r = np.random.default_rng(seed)
        try:
            for _ in range(20):
                ids = ns + r.choice(nv, 200, replace=False)
                v = r.integers(-5_000, 0, 200).astype(np.int64)
                with flock:
                    col.write_rows(ids, v)
                    final[ids] = v
        except Exception as e:  # noqa: BLE001
            errors.append(("writer", repr(e)))

    ts = [threading.Thread(target=reader, args=(s,)) for s in range(12)]
    ts += [threading.Thread(target=writer, args=(200 + s,)) for s in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    try:
        assert not errors, errors[:5]
        assert np.array_equal(col.search(str(-2_000), "lt"), np.flatnonzero(final < -2_000))
        assert np.array_equal(col.order(False), np.argsort(final, kind="stable"))
    finally:
        col.close()


def test_search_mask_registered_buffer(eng):
    """dds_host_register: the Search bitmask DMA'd straight into a registered caller buffer equals the
    staged path's; overlapping registrations are refused; unregistering restores the staged path."""
    from ddshe import DDSError
    rng = np.random.default_rng(11)
    n = 1_000_003
    vals = rng.integers(-(1 << 40), 1 << 40, n).astype(np.int64)
    col = eng.opecol(n)
    col.append(vals)
    buf = np.zeros((n + 63) // 64, dtype=np.uint64)
    eng.host_register(buf)
    try:
        with pytest.raises(DDSError):
            eng.host_register(buf[10:])
        # the count kernel writes the registered buffer through its device mapping (no copy): every reply
        # must be complete when the call returns, whatever the previous contents
        rng2 = np.random.default_rng(12)
        for it in range(60):
            op, f = (("gt", np.greater), ("le", np.less_equal), ("ge", np.greater_equal), ("lt", np.less))[it % 4]
            bound = int(rng2.integers(-(1 << 40), 1 << 40)) if it % 7 else 12345
            buf[:] = np.uint64(0xFFFFFFFFFFFFFFFF) if it % 2 else np.uint64(0)
            words, cnt = col.search_mask(str(bound), op, out=buf)
            assert words is buf
            bits = np.unpackbits(buf.view(np.uint8), bitorder="little")
            want = f(vals, bound)
            assert np.array_equal(bits[:n].astype(bool), want) and not bits[n:].any(), (it, op, bound)
            assert cnt == int(want.sum())
            if it < 4:
                staged, cnt2 = col.search_mask(str(bound), op)
                assert np.array_equal(staged, buf) and cnt2 == cnt
    finally:
        eng.host_unregister(buf)
        col.close()


def test_search_mask_engine_allocated_buffer(eng):
    """dds_host_alloc: an engine-allocated, device-mapped reply buffer takes the Search bitmask like a
    registered one; dds_host_unregister refuses it and dds_host_free releases it once."""
    from ddshe import DDSError
    rng = np.random.default_rng(13)
    n = 300_017
    vals = rng.integers(-(1 << 40), 1 << 40, n).astype(np.int64)
    col = eng.opecol(n)
    col.append(vals)
    buf = eng.host_alloc((n + 63) // 64, np.uint64)
    try:
        with pytest.raises(DDSError):
            eng.host_unregister(buf)
        for it, (op, f) in enumerate((("gt", np.greater), ("le", np.less_equal), ("ge", np.greater_equal),
                                      ("lt", np.less)) * 3):
            bound = int(rng.integers(-(1 << 40), 1 << 40))
            buf[:] = np.uint64(0xFFFFFFFFFFFFFFFF) if it % 2 else np.uint64(0)
            words, cnt = col.search_mask(str(bound), op, out=buf)
            bits = np.unpackbits(buf.view(np.uint8), bitorder="little")
            want = f(vals, bound)
            assert np.array_equal(bits[:n].astype(bool), want) and not bits[n:].any(), (it, op, bound)
            assert cnt == int(want.sum())
    finally:
        eng.host_free(buf)
        col.close()
    with pytest.raises(DDSError):
        eng.host_free(buf)


def test_scan_needles_inline_and_uploaded(eng):
    """Needles of up to 128 bytes in all ride in the kernel arguments; longer ones are uploaded: both
    forms, at the 128-byte edge and past it, answer SearchEntryOR / AND / SearchEq / IsElement as the
    oracle does (long and short elements, fingerprint hits confirmed on the bytes)."""
    rng = random.Random(77)
    longs = [("L%x" % rng.getrandbits(64)) * 20 for _ in range(4)]      # ~340-byte elements
    shorts = [f"s{rng.getrandbits(24):x}" for _ in range(30)]
    edge = ["e" * 42, "f" * 43, "g" * 43]                                   # 128 bytes in all
    words = longs + shorts + edge
    rows = [[rng.choice(words) for _ in range(rng.randrange(0, 7))] for _ in range(3000)]
    tab = eng.strtab(rows)
    keyed = list(enumerate(rows))
    cases = [shorts[:3], edge, edge[:2] + ["h"], longs[:1], longs[:2] + shorts[:1], [longs[3]]]
    for v in cases:
        for route, req in (("SearchEntryOR", False), ("SearchEntryAND", True)):
            if route == "SearchEntryAND" and len(set(v)) < 3:
                continue
            assert tab.search_entry(v, req).tolist() == sorted(homo.search_entry(route, keyed, v)), (route, v)
    for value in (longs[0], edge[1], shorts[5]):
        for position in (0, 2):
            assert tab.search_eq(position, value).tolist() == sorted(homo.search_eq("SearchEq", keyed, position,
                                                                                   value)), (position, value)
    r = next(i for i, row in enumerate(rows) if longs[1] in row)
    assert tab.is_element(r, longs[1])
    tab.close()
