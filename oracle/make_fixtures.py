#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ (TEST INFRASTRUCTURE ONLY).

    python oracle/make_fixtures.py            # needs /root/reference for keys.json

* keys.json    — key material decoded from the reference's committed client.conf
                 (src/main/resources/client.conf:81-88) + seeded synthetic keys for
                 the other BASELINE.json configs (1024/3072-bit Paillier, 2048-bit RSA).
* vectors.json — known-answer vectors produced by oracle/homo.py (Python ints):
                 encryptions with fixed (m, r), fold products, decryptions, pairwise
                 products, route-level SumAll/MultAll/Search cases incl. edge cases.

There are no reference-produced vectors to copy (the reference has no tests and its
hlib jar is absent); see oracle/homo.py for how these are pinned.
"""
from __future__ import annotations

import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

from oracle import homo  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")
REF_CONF = "/root/reference/src/main/resources/client.conf"


def hx(x: int) -> str:
    return format(int(x), "x")


def make_keys() -> dict:
    from oracle.javaser import decode_client_conf
    ref = decode_client_conf(open(REF_CONF).read())
    keys = {
        "source": "decoded from reference src/main/resources/client.conf:81-88 (committed key) + seeded synthetic keys",
        "ope_key": ref["ope_key"],
        "paillier2048_committed": {k: hx(v) for k, v in ref["paillier"].items()},
        "rsa1024_committed": {k: (hx(v) if isinstance(v, int) else v) for k, v in ref["rsa"].items()},
        "paillier1024_seed1": {k: hx(v) for k, v in homo.gen_paillier_key(1024, seed=1).items()},
        "rsa2048_seed3": {k: hx(v) for k, v in homo.gen_rsa_key(2048, seed=3).items()},
        "paillier3072_seed4": {k: hx(v) for k, v in homo.gen_paillier_key(3072, seed=4).items()},
    }
    return keys


def load_key(keys, name):
    return {k: (int(v, 16) if k != "x509_hex" else v) for k, v in keys[name].items()}


def paillier_vectors(key, rng, n_rows):
    n, nsq = key["n"], key["nsquare"]
    rows = []
    for _ in range(n_rows):
        m = rng.randrange(0, 10000)  # DDSDataGenerator.scala:274
        r = rng.randrange(1, n)
        rows.append((m, r, homo.paillier_encrypt(m, r, key)))
    cs = [c for _, _, c in rows]
    prod = homo.modmul_fold(cs, nsq)
    dec = homo.paillier_decrypt(prod, key)
    assert dec == sum(m for m, _, _ in rows) % n
    pairs = [(cs[i], cs[(i + 1) % len(cs)], homo.homo_add_sum(cs[i], cs[(i + 1) % len(cs)], nsq)) for i in range(8)]
    return {
        "rows": [{"m": m, "r": hx(r), "c": hx(c)} for m, r, c in rows],
        "fold": hx(prod), "dec_sum": dec,
        "pairs": [{"a": hx(a), "b": hx(b), "c": hx(c)} for a, b, c in pairs],
    }


def rsa_vectors(key, rng, n_rows):
    n = key["n"]
    ms = [rng.randrange(1, 10000) for _ in range(n_rows)]
    cs = [homo.rsa_encrypt(m, key) for m in ms]
    prod = homo.modmul_fold(cs, n)
    pm = 1
    for m in ms:
        pm = pm * m % n
    assert homo.rsa_decrypt(prod, key) == pm
    return {"rows": [{"m": m, "c": hx(c)} for m, c in zip(ms, cs)], "fold": hx(prod), "dec_prod": pm}


def edge_vectors(N, rng):
    """Fold edge cases (SURVEY.md §8c iii) for modulus N."""
    cases = []

    def add(name, ops):
        try:
            res = hx(homo.modmul_fold(ops, N))
        except homo.NotFound:
            res = None
        cases.append({"name": name, "ops": [hx(x) for x in ops], "result": res})

    add("k0_notfound", [])
    add("k1_unreduced_below", [N - 5])
    add("k1_unreduced_above", [N + 12345])       # first operand is NOT reduced (DDSRestServer.scala:416-417)
    add("k2", [rng.randrange(N), rng.randrange(N)])
    add("zero_operand", [rng.randrange(N), 0, rng.randrange(N)])
    add("n_minus_1", [N - 1, N - 1, N - 1])
    add("one", [1, 1, 1, 1])
    add("operand_ge_n", [N + 7, rng.randrange(N), 2 * N - 1])
    add("operand_ge_2n", [2 * N + 3, rng.randrange(N)])
    add("duplicates", [12345678901234567890] * 5)
    add("random_64", [rng.randrange(N) for _ in range(64)])
    return cases


def route_vectors(pk, rsa, rng):
    nsq, n = pk["nsquare"], rsa["n"]
    cs = [homo.paillier_encrypt(rng.randrange(10000), rng.randrange(1, pk["n"]), pk) for _ in range(6)]
    rc = [homo.rsa_encrypt(rng.randrange(1, 10000), rsa) for _ in range(6)]
    ope = [rng.randrange(-2**63, 2**63) for _ in range(6)]
    # rows mirror client.conf:55,60 column schema [OPE, CHE, PSSE, MSE, CHE, CHE, CHE, None]
    rows = []
    for i in range(6):
        rows.append([str(ope[i]), f"che{i}", str(cs[i]), str(rc[i]), "x", "y", "z", "blob"])
    rows.append([str(ope[0]), "short"])            # too short for positions >= 1
    rows.append(list(rows[0]))                     # duplicate row: collapses (Set semantics)
    rows.append([str(ope[3]), "c", str(cs[3])])    # length == position+1 for PSSE: strict guard skips it
    out = {"rows": rows, "cases": []}
    for pos, nsqr in ((2, str(nsq)), (2, None)):
        out["cases"].append({"route": "SumAll", "position": pos, "nsqr": nsqr,
                             "result": homo.sum_all(rows, pos, nsqr)})
    for pos, mod in ((3, n), (3, None)):
        out["cases"].append({"route": "MultAll", "position": pos, "n": None if mod is None else str(mod),
                             "result": homo.mult_all(rows, pos, mod)})
    keyed = [(f"k{i}", r) for i, r in enumerate(rows)]
    for route in ("SearchGt", "SearchGtEq", "SearchLt", "SearchLtEq"):
        for val in (ope[2], -2**63, 2**63 - 1, 0):
            out["cases"].append({"route": route, "position": 0, "value": str(val),
                                 "result": sorted(homo.search(route, keyed, 0, val))})
    try:
        homo.sum_all(rows, 7, str(nsq))
        raise AssertionError("expected 404")
    except homo.NotFound:
        out["cases"].append({"route": "SumAll", "position": 7, "nsqr": str(nsq), "result": None})
    return out


def _outcome(fn, *args, **kw):
    """Route result as a fixture: the reply text / key list, or {"status": 404 | 500}."""
    try:
        r = fn(*args, **kw)
    except homo.NotFound:
        return {"status": 404}
    except homo.ServerError:
        return {"status": 500}
    return sorted(r) if isinstance(r, set) else r


def route_edge_vectors(pk, rsa):
    """Route-level edge cases (VERDICT r01 "What's weak" 1): lazy nsqr / pubkey / bound parsing, out-of-
    Long OPE rows, typed dedup, pairwise guards, even and tiny moduli, Unicode digits, Order's lazy
    parse. Each case names its route and arguments; expected = the oracle's reply or status."""
    nsq, n, xh = pk["nsquare"], rsa["n"], rsa["x509_hex"]
    c = [homo.paillier_encrypt(m, r, pk) for m, r in ((5, 11), (7, 13), (9, 17))]
    rc = [homo.rsa_encrypt(m, rsa) for m in (3, 5, 7)]
    cases = []

    def add(rname, args, fn, **kw):
        cases.append({"route": rname, "args": args, "expected": _outcome(fn, **kw)})

    one = [["0", str(c[0]), "z"]]
    two = [["0", str(c[0]), "z"], ["1", str(c[1]), "z"]]
    for rows, nsqr in ((one, "12x"), (two, "12x"), (two, "1"), (two, "0"), (two, "-77"), (two, "+" + str(nsq)),
                       (two, str(nsq * 4)), (two, str(2 ** 128 * 3)), (two, "1" + "0" * 40)):
        add("SumAll", {"rows": rows, "position": 1, "nsqr": nsqr}, homo.sum_all, rows=rows, position=1, nsqr=nsqr)
    typed = [["a", 5, "z"], ["a", "5", "z"], ["a", 5, "z"], [True, "3", "z"], [1, "3", "z"]]
    for pos in (1, 0):
        add("SumAll", {"rows": typed, "position": pos, "nsqr": None}, homo.sum_all, rows=typed, position=pos, nsqr=None)
        add("MultAll", {"rows": typed, "position": pos, "pubkey": None}, homo.mult_all, rows=typed, position=pos)
    uni = [["x", "\u0663\u0661", "z"], ["y", "+\u0664", "z"], ["w", "-\uff15", "z"]]  # Arabic-Indic 31, 4; fullwidth 5
    add("SumAll", {"rows": uni, "position": 1, "nsqr": None}, homo.sum_all, rows=uni, position=1, nsqr=None)
    add("SumAll", {"rows": uni, "position": 1, "nsqr": "1000"}, homo.sum_all, rows=uni, position=1, nsqr="1000")
    add("SumAll", {"rows": [["x", "\u00b2", "z"]], "position": 1, "nsqr": None}, homo.sum_all,
        rows=[["x", "\u00b2", "z"]], position=1, nsqr=None)  # superscript two: isdigit, not a decimal digit
    mrows1 = [["0", str(rc[0]), "z"]]
    mrows = [["0", str(rc[0]), "z"], ["1", str(rc[1]), "z"], ["2", str(rc[2]), "z"]]
    for rows, key in ((mrows, xh), (mrows1, "zz"), (mrows, "zz"), (mrows, xh[:-2]), (mrows, xh.upper()), (mrows1, None)):
        add("MultAll", {"rows": rows, "position": 1, "pubkey": key}, homo.mult_all, rows=rows, position=1, pubkey=key)
    s1, s2, s3 = ["0", str(c[0])], ["1", str(c[1]), "q"], ["2"]
    for a_, b_, pos, nsqr in ((s1, s2, 1, str(nsq)), (s1, s2, 1, None), (s1, s3, 1, str(nsq)), (None, s2, 1, None),
                              (s1, s1, 1, str(nsq)), (s2, s2, 2, None), (s1, s2, 1, "0")):
        add("Sum", {"set1": a_, "set2": b_, "position": pos, "nsqr": nsqr}, homo.pair_sum, set1=a_, set2=b_,
            position=pos, nsqr=nsqr)
    r1, r2 = ["0", str(rc[0])], ["1", str(rc[1]), "q"]
    for a_, b_, key in ((r1, r2, xh), (r1, r2, None), (r1, r2, "0g"), (r1, ["1"], xh)):
        add("Mult", {"set1": a_, "set2": b_, "position": 1, "pubkey": key}, homo.pair_mult, set1=a_, set2=b_,
            position=1, pubkey=key)
    big = 2 ** 70 + 12345
    srows = [("k0", [str(-big), "x"]), ("k1", [str(big), "x"]), ("k2", ["17", "x"]), ("k3", ["-17", "x"]),
             ("k4", [str(2 ** 63 - 1), "x"]), ("k5", [str(-2 ** 63), "x"]), ("k6", ["5"]), ("k7", [42, "x"]),
             ("k8", ["+0017", "x"]), ("k9", None)]
    for route in ("SearchGt", "SearchGtEq", "SearchLt", "SearchLtEq"):
        for bound in ("17", str(big), str(-big), str(2 ** 80), str(-2 ** 80), str(2 ** 63), str(-2 ** 63 - 1), "0"):
            add(route, {"rows": srows, "position": 0, "value": bound}, homo.search, route=route, keyed_rows=srows,
                position=0, value=bound)
    lone = [("a", ["zz"]), ("b", [])]
    bad = [("a", ["zz", "q"]), ("b", ["1", "q"])]
    for route in ("SearchGt", "SearchLtEq"):
        for rows, bound in ((lone, "bad"), (lone, "3"), (bad, "3"), ([("a", ["1", "q"])], "bad"), ([], "bad")):
            add(route, {"rows": rows, "position": 0, "value": bound}, homo.search, route=route, keyed_rows=rows,
                position=0, value=bound)
    orows = [("a", ["5"]), ("b", []), ("c", ["-3"]), ("d", ["5"]), ("e", None), ("g", ["+7"])]
    for route in ("OrderLS", "OrderSL"):
        for rows, pos in ((orows, 0), ([("a", ["x"]), ("b", [])], 0), ([("a", [5]), ("b", ["6"])], 0),
                          ([("a", [5]), ("b", [])], 0), ([("a", [str(2 ** 64)]), ("b", ["1"])], 0),
                          ([("a", ["1", "2"]), ("b", ["3"])], 1)):
            add(route, {"rows": rows, "position": pos}, homo.order, route=route, keyed_rows=rows, position=pos)
    return cases


def main():
    os.makedirs(GOLDEN, exist_ok=True)
    kpath = os.path.join(GOLDEN, "keys.json")
    if os.path.exists(REF_CONF):
        keys = make_keys()
        json.dump(keys, open(kpath, "w"), indent=1)
    keys = json.load(open(kpath))
    rng = random.Random(2017)
    pk2048 = load_key(keys, "paillier2048_committed")
    pk1024 = load_key(keys, "paillier1024_seed1")
    pk3072 = load_key(keys, "paillier3072_seed4")
    rsa1024 = load_key(keys, "rsa1024_committed")
    rsa2048 = load_key(keys, "rsa2048_seed3")
    vec = {
        "paillier2048_committed": paillier_vectors(pk2048, rng, 24),
        "paillier1024_seed1": paillier_vectors(pk1024, rng, 48),
        "paillier3072_seed4": paillier_vectors(pk3072, rng, 12),
        "rsa1024_committed": rsa_vectors(rsa1024, rng, 48),
        "rsa2048_seed3": rsa_vectors(rsa2048, rng, 48),
        "edges_nsq2048": edge_vectors(pk2048["nsquare"], rng),
        "edges_n1024": edge_vectors(rsa1024["n"], rng),
        "edges_nsq3072": edge_vectors(pk3072["nsquare"], rng),
        "routes": route_vectors(pk2048, rsa1024, rng),
        "route_edges": route_edge_vectors(pk2048, rsa1024),
    }
    json.dump(vec, open(os.path.join(GOLDEN, "vectors.json"), "w"), indent=1)
    print("wrote", kpath, os.path.join(GOLDEN, "vectors.json"))


if __name__ == "__main__":
    main()
