"""Resident columns under the reference's write routes (VERDICT r02 "next" 1).

WriteElement (DDSRestServer.scala:281-321), AddElement (:220-255), RemoveSet (:207-218) and PutSet
(:170-205) change stored sets in place; the read routes re-fetch them. The engine keeps the sets in
resident columns and follows each write with dds_col_write_rows_dec / dds_col_set_live /
dds_opecol_write_rows_dec / dds_opecol_set_live. Checked here:
  * the golden write-route sequences (tests/golden/mutations.json, oracle/make_fixtures.py) replayed
    through ddshe.store.ResidentStore, every read route compared after every step;
  * the C-ABI mutations directly against the oracle on seeded rows (dds_col, dds_mcol over repeated
    devices, dds_opecol), incl. the one-operand / empty rules over live rows and bad writes;
  * a 1M-row synthetic column with 10 % removed rows and rewritten rows: Dec(fold) = sum of the live
    rows' plaintexts (size-independent property).
"""
import json
import os
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _outcome(fn, *a, **kw):
    from ddshe.routes import NotFound, ServerError
    try:
        return fn(*a, **kw)
    except NotFound:
        return {"status": 404}
    except ServerError:
        return {"status": 500}


def test_mutation_sequences_golden(eng):
    from ddshe.store import ResidentStore
    from ddshe.routes import NotFound, ServerError
    fx = json.load(open(os.path.join(HERE, "golden", "mutations.json")))
    pos = fx["positions"]
    nsq, n = int(fx["nsquare"]), int(fx["n"])
    st = ResidentStore(eng, paillier={pos["sum"]: nsq}, rsa={pos["mult"]: n}, ope=[pos["ope"]], capacity=4096)
    bad = []
    try:
        for i, step in enumerate(fx["steps"]):
            op = step["op"]
            status = 200
            try:
                if op == "put":
                    k = st.put_set(step["set"])
                    assert k == step["key"], (i, "key derivation")
                elif op == "put_empty":
                    st.put_empty(step["key"])
                elif op == "remove":
                    st.remove_set(step["key"])
                elif op == "add":
                    st.add_element(step["key"], step["value"])
                elif op == "write":
                    st.write_element(step["key"], step["position"], step["value"])
            except NotFound:
                status = 404
            except ServerError:
                status = 500
            if status != step["status"]:
                bad.append((i, op, "status", step["status"], status))
            idx = {k: j for j, k in enumerate(st.keys)}
            want = step["reads"]
            got = {
                "SumAll": _outcome(st.sum_all, pos["sum"], fx["nsquare"]),
                "MultAll": _outcome(st.mult_all, pos["mult"], fx["pubkey"]),
                "SumAllPlain": _outcome(st.sum_all, pos["sum"], None),
            }
            for route in ("SearchGt", "SearchLtEq"):
                r = _outcome(st.search, route, pos["ope"], fx["bound"])
                got[route] = r if isinstance(r, dict) else sorted(idx[k] for k in r)
            for route in ("OrderLS", "OrderSL"):
                r = _outcome(st.order, route, pos["ope"])
                got[route] = r if isinstance(r, dict) else [idx[k] for k in r]
            # the resident string table under the same writes (SearchEq/NEq, SearchEntry/OR/AND, IsElement)
            for name in want:
                if name.startswith("SearchEq@") or name.startswith("SearchNEq@"):
                    route, rest = name.split("@")
                    p, value = rest.split(":", 1)
                    r = _outcome(st.search_eq, route, int(p), value)
                elif name.startswith("SearchEntry"):
                    route, values = name.split(":", 1)
                    r = _outcome(st.search_entry, route, values.split(","))
                else:
                    continue
                got[name] = r if isinstance(r, dict) else sorted(idx[k] for k in r)
            got["IsElement"] = [[ki, value, _outcome(st.is_element, st.keys[ki] if ki >= 0 else "F" * 128, value)]
                                for ki, value, _ in want["IsElement"]]
            for route, w in want.items():
                if got[route] != w:
                    bad.append((i, op, route, str(w)[:80], str(got[route])[:80]))
    finally:
        st.close()
    assert not bad, bad[:10]


def _dec_list(xs):
    return [str(x) for x in xs]


def test_col_write_and_live_vs_oracle(eng, keys):
    """dds_col_write_rows[_dec] + dds_col_set_live against the oracle fold of the live rows: whole
    range, sub-ranges, row lists, partials; one live row (its operand unreduced), none (404)."""
    from ddshe import NotFound, DDSError
    from oracle import homo
    rng = random.Random(31)
    for kname, rows in (("paillier2048_committed", 700), ("paillier1024_seed1", 3000), ("rsa2048_seed3", 2500)):
        key = keys[kname]
        N = key.get("nsquare", key["n"])
        vals = [rng.randrange(N) for _ in range(rows)]
        col = eng.column(N, rows + 64)
        col.append_dec(_dec_list(vals))
        live = np.ones(rows, dtype=bool)
        for it in range(4):
            w = rng.sample(range(rows), 40)
            nv = [rng.randrange(N) for _ in w]
            nv[0] = N + 3 + rng.randrange(1000)       # stored reduced, kept for a one-row fold
            nv[1] = -(rng.randrange(N))               # negative decimal
            col.write_rows_dec(w, _dec_list(nv))
            for r, v in zip(w, nv):
                vals[r] = v
            d = rng.sample(range(rows), rows // 5)
            flags = [rng.random() < 0.8 for _ in d]   # mostly removals, some revivals
            col.set_live(d, [0 if f else 1 for f in flags])
            for r, f in zip(d, flags):
                live[r] = not f
            assert col.live_count == int(live.sum())
            ids = [i for i in range(rows) if live[i]]
            assert col.fold() == homo.modmul_fold([vals[i] % N for i in ids], N), (kname, it)
            a, b = sorted(rng.sample(range(rows), 2))
            sub = [i for i in range(a, b) if live[i]]
            if len(sub) >= 2:
                assert col.fold(a, b - a) == homo.modmul_fold([vals[i] % N for i in sub], N)
            pick = rng.sample(range(rows), 300)
            kept = [i for i in pick if live[i]]
            assert col.fold_rows(pick) == homo.modmul_fold([vals[i] % N for i in kept], N)
            part, nrows = col.fold_partial(a, b - a)
            assert nrows == len(sub)
        # one live row in a range: returned as written (unreduced, sign kept); none: 404
        r0 = next(i for i in range(rows) if live[i])
        col.write_rows_dec([r0], [str(N + 99)])
        others = [i for i in range(rows) if live[i] and i != r0]
        col.set_live(others, 0)
        assert col.fold_dec() == str(N + 99)
        col.write_rows_dec([r0], [str(-12345)])
        assert col.fold_dec() == "-12345"
        col.set_live([r0], 0)
        with pytest.raises(NotFound):
            col.fold()
        # a bad write changes nothing
        col.set_live(list(range(rows)), 1)
        before = col.fold()
        with pytest.raises(DDSError):
            col.write_rows_dec([3, 5], ["17", "1x"])
        with pytest.raises(DDSError):
            col.write_rows_dec([rows + 5], ["17"])
        assert col.fold() == before
        col.close()


def test_col_write_binary_and_duplicates(eng, keys):
    from oracle import homo
    rng = random.Random(5)
    N = keys["paillier2048_committed"]["nsquare"]
    vals = [rng.randrange(N) for _ in range(300)]
    col = eng.column(N, 512)
    col.append(vals)
    col.write_rows([7, 9, 7], [11, 13, 17])      # repeated id: the last value wins
    vals[7], vals[9] = 17, 13
    assert col.fold() == homo.modmul_fold(vals, N)
    col.truncate(200)                           # rows past the count come back live
    col.set_live(list(range(150, 200)), 0)
    assert col.fold() == homo.modmul_fold(vals[:150], N)
    col.truncate(160)
    col.append(vals[160:300])
    assert col.live_count == 150 + 140
    assert col.fold() == homo.modmul_fold(vals[:150] + vals[160:300], N)
    col.close()


def test_mcol_write_and_live(keys):
    """dds_mcol_* mutations on three shards of one GPU (global row ids across 64-row blocks)."""
    import ddshe
    from oracle import homo
    rng = random.Random(8)
    N = keys["paillier2048_committed"]["nsquare"]
    m = ddshe.MultiEngine(devices=[0, 0, 0])
    col = m.column(N, 5000)
    vals = [rng.randrange(N) for _ in range(4000)]
    col.append_dec(_dec_list(vals))
    live = np.ones(4000, dtype=bool)
    w = rng.sample(range(4000), 120)
    nv = [rng.randrange(N) for _ in w]
    col.write_rows_dec(w, _dec_list(nv))
    for r, v in zip(w, nv):
        vals[r] = v
    d = rng.sample(range(4000), 900)
    col.set_live(d, 0)
    live[d] = False
    assert col.live_count == int(live.sum())
    ids = [i for i in range(4000) if live[i]]
    assert col.fold() == homo.modmul_fold([vals[i] for i in ids], N)
    pick = rng.sample(range(4000), 500)
    assert col.fold_rows(pick) == homo.modmul_fold([vals[i] for i in pick if live[i]], N)
    with pytest.raises(ddshe.DDSError):        # one bad row: nothing written on any shard
        col.write_rows_dec([1, 70, 140], ["5", "7", "x"])
    assert col.fold() == homo.modmul_fold([vals[i] for i in ids], N)
    keep = ids[17]
    col.set_live([i for i in ids if i != keep], 0)
    assert col.fold_dec() == str(vals[keep])  # one live row on one shard
    col.close()
    m.close()


def test_opecol_write_live_search_order(eng):
    """dds_opecol_write_rows[_dec] / set_live against numpy: Search as ids and as a bitmask, Order
    over the live rows (removed sets vanish, others keep their class), 4 ops, ties."""
    rng = np.random.default_rng(12)
    n = 20000
    vals = rng.integers(-1000, 1000, n)
    cls = rng.choice([0, 1, 2, 2, 2], n).astype(np.uint8)
    oc = eng.opecol(n + 100)
    oc.append(vals, cls)
    live = np.ones(n, dtype=bool)
    for it in range(3):
        w = rng.choice(n, 500, replace=False)
        nv = rng.integers(-1000, 1000, 500)
        nc = rng.choice([0, 1, 2], 500).astype(np.uint8)
        if it == 1:
            oc.write_rows_dec(w, [str(x) for x in nv], nc, np.ones(500, np.uint8))
        else:
            oc.write_rows(w, nv, nc)
        vals[w], cls[w] = nv, nc
        d = rng.choice(n, 2000, replace=False)
        f = rng.random(2000) < 0.7
        oc.set_live(d, (~f).astype(np.uint8))
        live[d] = ~f
        assert oc.live_count == int(live.sum())
        for op, fn in (("gt", np.greater), ("ge", np.greater_equal), ("lt", np.less), ("le", np.less_equal)):
            b = int(rng.integers(-1000, 1000))
            want = np.flatnonzero(live & (cls == 2) & fn(vals, b))
            assert np.array_equal(oc.search(b, op), want), (it, op)
            words, cnt = oc.search_mask(b, op)
            bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:n]
            assert cnt == len(want) and np.array_equal(np.flatnonzero(bits), want), (it, op)
        hold = live & (cls != 0)
        lack = live & (cls == 0)
        for desc in (True, False):
            key = -vals if desc else vals
            hi = np.flatnonzero(hold)
            sorted_h = hi[np.argsort(key[hi], kind="stable")]
            rest = np.flatnonzero(lack)
            want = np.concatenate([sorted_h, rest]) if desc else np.concatenate([rest, sorted_h])
            assert np.array_equal(oc.order(desc), want), (it, desc)
    oc.close()


def test_opecol_search_mask_wide_and_edges(eng):
    """search_mask: rows outside Long (host-merged bits), bound outside Long, no qualifying row, and a
    column whose length is not a multiple of 64."""
    oc = eng.opecol(200)
    big = 2 ** 70
    texts = [str(v) for v in range(-60, 70)] + [str(big), str(-big)]
    oc.append_dec(texts, [2] * len(texts), [1] * len(texts))
    n = len(texts)
    num = np.array([int(t) for t in texts], dtype=object)
    for bound in ("5", str(2 ** 80), str(-2 ** 80), str(big)):
        for op, fn in (("gt", lambda a, b: a > b), ("le", lambda a, b: a <= b)):
            want = [i for i in range(n) if fn(int(num[i]), int(bound))]
            words, cnt = oc.search_mask(bound, op)
            bits = np.unpackbits(words.view(np.uint8), bitorder="little")
            assert list(np.flatnonzero(bits)) == want and cnt == len(want), (bound, op)
    oc.set_live(list(range(n)), 0)
    words, cnt = oc.search_mask("bad bound: never parsed", "gt")
    assert cnt == 0 and not words.any()
    oc.close()


def test_removed_rows_at_scale(eng, keys):
    """1M synthetic committed-key rows (BASELINE config 2 generator), 10 % removed, 1000 rewritten with
    fresh encryptions: Dec(fold) = sum of the live rows' plaintexts mod n."""
    import ddshe
    from oracle import homo
    key = keys["paillier2048_committed"]
    n, nsq = key["n"], key["nsquare"]
    rows = 1_000_000
    col = eng.column(nsq, rows)
    col.fill_paillier_synth(n, key["g"], seed=2, row0=0, count=rows)
    ms = ddshe.synth_plaintexts(2, 0, rows).astype(np.int64)
    rng = np.random.default_rng(3)
    dead = rng.choice(rows, rows // 10, replace=False)
    col.set_live(dead, 0)
    live = np.ones(rows, dtype=bool)
    live[dead] = False
    pr = random.Random(4)
    w = [int(x) for x in rng.choice(np.flatnonzero(live), 1000, replace=False)]
    newm = [pr.randrange(10000) for _ in w]
    cs = eng.paillier_encrypt_batch(n, key["g"], newm, [pr.randrange(1, n) for _ in w])
    col.write_rows(w, cs)
    ms[w] = newm
    got = col.fold()
    assert homo.paillier_decrypt(got, key) == int(ms[live].sum()) % n
    col.close()
