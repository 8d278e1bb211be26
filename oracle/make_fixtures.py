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
    }
    json.dump(vec, open(os.path.join(GOLDEN, "vectors.json"), "w"), indent=1)
    print("wrote", kpath, os.path.join(GOLDEN, "vectors.json"))


if __name__ == "__main__":
    main()
