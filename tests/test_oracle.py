"""CPU tests of the oracle (tests/ infrastructure) against the reference's committed key
material and the golden vectors — no GPU. The oracle is pinned here; see oracle/homo.py."""
import ctypes
import ctypes.util
import math
import os
import random

import pytest

from oracle import homo

REF_CONF = "/root/reference/src/main/resources/client.conf"


def test_keys_json_matches_reference_conf(keys):
    if not os.path.exists(REF_CONF):
        pytest.skip("reference tree not present (GPU box)")
    from oracle.javaser import decode_client_conf
    ref = decode_client_conf(open(REF_CONF).read())
    for k, v in ref["paillier"].items():
        assert keys["paillier2048_committed"][k] == v
    assert keys["rsa1024_committed"]["n"] == ref["rsa"]["n"]
    assert keys["ope_key"] == ref["ope_key"]


@pytest.mark.parametrize("name", ["paillier2048_committed", "paillier1024_seed1", "paillier3072_seed4"])
def test_paillier_key_identities(keys, name):
    k = keys[name]
    n, nsq = k["n"], k["nsquare"]
    assert k["p"] * k["q"] == n and n * n == nsq
    lam = (k["p"] - 1) * (k["q"] - 1) // math.gcd(k["p"] - 1, k["q"] - 1)
    assert lam == k["lambda"]
    L = (pow(k["g"], lam, nsq) - 1) // n
    assert L * k["mu"] % n == 1


def test_committed_key_sizes(keys):
    assert keys["paillier2048_committed"]["n"].bit_length() == 2048
    assert keys["paillier2048_committed"]["nsquare"].bit_length() == 4095   # 128 x 32-bit limbs
    assert keys["rsa1024_committed"]["n"].bit_length() == 1024
    assert keys["rsa1024_committed"]["e"] == 65537


@pytest.mark.parametrize("name", ["rsa1024_committed", "rsa2048_seed3"])
def test_rsa_roundtrip(keys, name):
    k = keys[name]
    for m in (1, 2, 9999, 123456789):
        assert homo.rsa_decrypt(homo.rsa_encrypt(m, k), k) == m


def test_paillier_vectors_recompute(keys, vectors):
    for name in ("paillier2048_committed", "paillier1024_seed1", "paillier3072_seed4"):
        k, v = keys[name], vectors[name]
        rows = v["rows"]
        for row in rows[:4]:
            assert homo.paillier_encrypt(row["m"], int(row["r"], 16), k) == int(row["c"], 16)
        cs = [int(r["c"], 16) for r in rows]
        assert homo.modmul_fold(cs, k["nsquare"]) == int(v["fold"], 16)
        assert homo.paillier_decrypt(int(v["fold"], 16), k) == sum(r["m"] for r in rows) % k["n"] == v["dec_sum"]


def test_edge_vectors_recompute(keys, vectors):
    for name in ("edges_nsq2048", "edges_n1024", "edges_nsq3072"):
        N = {"edges_nsq2048": keys["paillier2048_committed"]["nsquare"],
             "edges_n1024": keys["rsa1024_committed"]["n"],
             "edges_nsq3072": keys["paillier3072_seed4"]["nsquare"]}[name]
        for case in vectors[name]:
            ops = [int(x, 16) for x in case["ops"]]
            if case["result"] is None:
                with pytest.raises(homo.NotFound):
                    homo.modmul_fold(ops, N)
            else:
                assert homo.modmul_fold(ops, N) == int(case["result"], 16), case["name"]


def test_route_vectors_recompute(vectors):
    rv = vectors["routes"]
    rows = rv["rows"]
    keyed = [(f"k{i}", r) for i, r in enumerate(rows)]
    for c in rv["cases"]:
        if c["route"] == "SumAll":
            if c["result"] is None:
                with pytest.raises(homo.NotFound):
                    homo.sum_all(rows, c["position"], c["nsqr"])
            else:
                assert homo.sum_all(rows, c["position"], c["nsqr"]) == c["result"]
        elif c["route"] == "MultAll":
            n = int(c["n"]) if c["n"] else None
            assert homo.mult_all(rows, c["position"], n) == c["result"]
        else:
            assert sorted(homo.search(c["route"], keyed, c["position"], c["value"])) == c["result"]


def test_route_semantics_unit():
    # strict guard (DDSRestServer.scala:415): a row whose last index == position is skipped
    assert homo.sum_all([["1", "7"], ["2", "5", "x"]], 1, "1000") == "5"
    # first operand unreduced when alone (:416-417)
    assert homo.sum_all([["0", "12345", "z"]], 1, "100") == "12345"
    # plain add without nsqr (:425)
    assert homo.sum_all([["0", "3", "z"], ["0", "4", "z"]], 1, None) == "7"
    # duplicates collapse (Set semantics of storedKeys.map, :401-403)
    assert homo.sum_all([["0", "3", "z"], ["0", "3", "z"]], 1, None) == "3"
    with pytest.raises(homo.NotFound):
        homo.sum_all([], 1, None)
    with pytest.raises(homo.ServerError):
        homo.sum_all([["0", "abc", "z"]], 1, None)
    assert homo.pair_sum(["1", "9"], ["1", "8"], 1, "10") == "2"
    with pytest.raises(homo.NotFound):
        homo.pair_sum(["1"], ["1", "8"], 1, "10")


def _openssl():
    path = ctypes.util.find_library("crypto")
    if not path:
        pytest.skip("libcrypto not available")
    lib = ctypes.CDLL(path)
    lib.BN_new.restype = ctypes.c_void_p
    lib.BN_CTX_new.restype = ctypes.c_void_p
    lib.BN_bin2bn.restype = ctypes.c_void_p
    lib.BN_bin2bn.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_void_p]
    lib.BN_bn2bin.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
    lib.BN_num_bits.argtypes = [ctypes.c_void_p]
    lib.BN_mod_mul.argtypes = [ctypes.c_void_p] * 5
    lib.BN_free.argtypes = [ctypes.c_void_p]
    lib.BN_CTX_free.argtypes = [ctypes.c_void_p]
    return lib


def test_oracle_vs_openssl_bn_mod_mul(keys):
    """Independent cross-check of the fold arithmetic with OpenSSL BN_mod_mul."""
    lib = _openssl()
    ctx = lib.BN_CTX_new()

    def bn(x):
        b = x.to_bytes(max(1, (x.bit_length() + 7) // 8), "big")
        return lib.BN_bin2bn(b, len(b), None)

    def toint(p):
        nb = (lib.BN_num_bits(p) + 7) // 8
        buf = ctypes.create_string_buffer(max(1, nb))
        lib.BN_bn2bin(p, buf)
        return int.from_bytes(buf.raw[:nb], "big") if nb else 0

    rng = random.Random(5)
    for N in (keys["paillier2048_committed"]["nsquare"], keys["rsa2048_seed3"]["n"],
              keys["paillier3072_seed4"]["nsquare"]):
        xs = [rng.randrange(N) for _ in range(50)]
        acc, m = bn(xs[0]), bn(N)
        for x in xs[1:]:
            b = bn(x)
            r = lib.BN_new()
            assert lib.BN_mod_mul(r, acc, b, m, ctx) == 1
            lib.BN_free(acc)
            lib.BN_free(b)
            acc = r
        assert toint(acc) == homo.modmul_fold(xs, N)
    lib.BN_CTX_free(ctx)


def test_partial_algebra():
    """Montgomery partial algebra used by the multi-GPU combine: v(S) = prod(S) * R^(1-|S|)."""
    rng = random.Random(9)
    N = rng.randrange(2**300, 2**301) | 1
    R = 2 ** (27 * 12)
    Rinv = pow(R, -1, N)

    def monpro(a, b):
        return a * b * Rinv % N

    xs = [rng.randrange(N) for _ in range(37)]
    parts = []
    for i in range(0, 37, 10):
        v = R % N
        for x in xs[i:i + 10]:
            v = monpro(v, x)
        parts.append(v)
    v = R % N
    for p in parts:
        v = monpro(v, p)
    # v(all) = prod * R^(1-k) * R^(1-#parts)... combine folds partials as rows: R^(1 - k) overall
    v_all = parts[0]
    for p in parts[1:]:
        v_all = monpro(v_all, p)
    assert monpro(v_all, pow(R, len(xs), N)) == homo.modmul_fold(xs, N)


def test_c_restatement_matches_python_oracle(keys):
    from oracle import cref
    rng = random.Random(77)
    for N in (keys["paillier2048_committed"]["nsquare"], keys["rsa1024_committed"]["n"],
              keys["paillier3072_seed4"]["nsquare"], (1 << 127) - 1):
        for k in (2, 3, 50):
            xs = [rng.randrange(N) for _ in range(k)]
            assert cref.fold(N, xs) == homo.modmul_fold(xs, N)
        xs = [N + 5, 3 * N + 1, rng.randrange(N)]        # unreduced inputs
        assert cref.fold(N, xs) == homo.modmul_fold(xs, N)
        assert cref.fold(N, [N + 5]) == N + 5              # k == 1 verbatim


def test_order_route_semantics():
    """OrderLS / OrderSL restatement (DDSRestServer.scala:541-606) on a hand-checked case."""
    rows = [("a", ["5"]), ("b", []), ("c", ["-3"]), ("d", ["5"]), ("e", None), ("f", ["x", "9"]), ("g", ["+7"])]
    assert homo.order("OrderLS", [r for r in rows if r[0] != "f"], 0) == ["g", "a", "d", "c", "b"]
    assert homo.order("OrderSL", [r for r in rows if r[0] != "f"], 0) == ["b", "c", "a", "d", "g"]
    assert homo.order("OrderSL", rows, 1) == ["a", "b", "c", "d", "g", "f"]  # only f holds position 1
    with pytest.raises(homo.ServerError):
        homo.order("OrderLS", rows, 0)                                   # "x".toLong
    assert homo.order("OrderLS", [("a", ["x"]), ("b", [])], 0) == ["a", "b"]  # lone holder: never parsed
    with pytest.raises(homo.ServerError):
        homo.order("OrderSL", [("a", [5]), ("b", ["6"])], 0)             # Int element: ClassCastException


def test_openssl_baselines_match_oracle(keys):
    """The OpenSSL CPU baselines (bench.py cpu_baseline) compute what the oracle computes."""
    from oracle import cref
    if not os.path.exists(cref.BNLIB) and not os.path.exists("/usr/include/openssl/bn.h"):
        pytest.skip("OpenSSL headers absent")
    k = keys["paillier1024_seed1"]
    rng = random.Random(5)
    N = k["nsquare"]
    xs = [rng.randrange(N) for _ in range(101)]
    mb = (N.bit_length() + 7) // 8
    ops = b"".join(x.to_bytes(mb, "big") for x in xs)
    want = homo.modmul_fold(xs, N)
    for threads in (1, 4):
        assert int.from_bytes(cref.bn_fold_be(N.to_bytes(mb, "big"), ops, mb, len(xs), threads), "big") == want
    ms = [rng.randrange(10000) for _ in range(6)]
    rs = [rng.randrange(1, k["n"]) for _ in ms]
    assert cref.bn_paillier_encrypt(k["n"], k["g"], ms, rs, 2) == [homo.paillier_encrypt(m, r, k) for m, r in zip(ms, rs)]


def _oracle_outcome(c):
    a, r = c["args"], c["route"]
    try:
        if r == "SumAll":
            out = homo.sum_all(a["rows"], a["position"], a["nsqr"])
        elif r == "MultAll":
            out = homo.mult_all(a["rows"], a["position"], pubkey=a["pubkey"])
        elif r == "Sum":
            out = homo.pair_sum(a["set1"], a["set2"], a["position"], a["nsqr"])
        elif r == "Mult":
            out = homo.pair_mult(a["set1"], a["set2"], a["position"], pubkey=a["pubkey"])
        elif r.startswith("Search"):
            out = sorted(homo.search(r, [(k, row) for k, row in a["rows"]], a["position"], a["value"]))
        else:
            out = homo.order(r, [(k, row) for k, row in a["rows"]], a["position"])
    except homo.NotFound:
        return {"status": 404}
    except homo.ServerError:
        return {"status": 500}
    return out


def test_route_edge_vectors_recompute(vectors):
    """The route edge fixtures are what the oracle answers (guards against fixture/oracle drift)."""
    for c in vectors["route_edges"]:
        assert _oracle_outcome(c) == c["expected"], (c["route"], str(c["args"])[:120])


def test_route_edge_semantics_unit(keys):
    """Hand-checked reference behaviours behind the fixtures (DDSRestServer.scala line cited)."""
    # nsqr parsed only for the second and later operands (:416-422)
    assert homo.sum_all([["0", "77", "z"]], 1, "not-a-number") == "77"
    with pytest.raises(homo.ServerError):
        homo.sum_all([["0", "77", "z"], ["1", "5", "z"]], 1, "not-a-number")
    # any positive modulus: BigInteger.mod (:423); m <= 0 -> ArithmeticException (500)
    assert homo.sum_all([["0", "77", "z"], ["1", "5", "z"]], 1, "64") == str(77 * 5 % 64)
    assert homo.sum_all([["0", "77", "z"], ["1", "5", "z"]], 1, "1") == "0"
    with pytest.raises(homo.ServerError):
        homo.sum_all([["0", "77", "z"], ["1", "5", "z"]], 1, "0")
    # the Search bound is parsed only for a row that passes the strict guard (:702-704)
    assert homo.search("SearchGt", [("a", ["5"])], 0, "junk") == set()
    with pytest.raises(homo.ServerError):
        homo.search("SearchGt", [("a", ["5", "x"])], 0, "junk")
    # rows outside Long compare as BigIntegers (:704)
    assert homo.search("SearchGt", [("a", [str(2 ** 80), "x"]), ("b", ["3", "x"])], 0, "4") == {"a"}
    # typed dedup: Int 5 and String "5" are different DDSSets (:401-403, DDSJsonProtocol.scala:22-28)
    assert homo.sum_all([["a", 5, "z"], ["a", "5", "z"]], 1, None) == "10"
    assert homo.sum_all([["a", "5", "z"], ["a", "5", "z"]], 1, None) == "5"
    # Unicode decimal digits (Character.digit); a superscript two is not one
    assert homo.java_biginteger("\u0664\u0662") == 42
    with pytest.raises(homo.ServerError):
        homo.java_biginteger("\u00b2")
    # pubkey decoded only when a second operand exists (:515-517)
    assert homo.mult_all([["0", "9", "z"]], 1, pubkey="zz") == "9"
    n = keys["rsa1024_committed"]["n"]
    assert homo.rsa_modulus_from_pubkey_hex(keys["rsa1024_committed"]["x509_hex"]) == n


def test_x509_product_decoder_matches_oracle(keys):
    """ddshe.x509 (product) and the oracle decode the same pubkeys and reject the same junk."""
    from ddshe import x509
    xh = keys["rsa1024_committed"]["x509_hex"]
    assert x509.rsa_modulus(xh) == homo.rsa_modulus_from_pubkey_hex(xh) == keys["rsa1024_committed"]["n"]
    assert x509.rsa_modulus(xh.upper()) == keys["rsa1024_committed"]["n"]
    for junk in ("", "0", "zz", xh[:-2], xh[:40], "3000", xh[:2] + "ff" + xh[4:]):
        with pytest.raises(ValueError):
            x509.rsa_modulus(junk)
        with pytest.raises(homo.ServerError):
            homo.rsa_modulus_from_pubkey_hex(junk)


def test_store_write_routes():
    """oracle Store: the write routes' effects (DDSRestServer.scala:170-321) on what the read routes see."""
    st = homo.Store()
    a = st.put_set(["1", "x", "7", "z"])
    assert a == homo.key_from_set(["1", "x", "7", "z"]) and len(a) == 128 and a == a.upper()
    b = st.put_set(["2", "y", "7"])                          # PSSE is its last element: skipped by SumAll
    assert homo.sum_all(st.rows(), 2, "1000") == "7"
    st.add_element(b, "t")                                   # crosses the strict guard
    assert homo.sum_all(st.rows(), 2, "1000") == "49"
    st.write_element(b, 9, "u")                              # past the end: appended
    assert st.val[b] == ["2", "y", "7", "t", "u"]
    st.remove_set(a)
    assert homo.sum_all(st.rows(), 2, "1000") == "7"
    with pytest.raises(homo.NotFound):
        st.add_element(a, "q")                               # removed: 404
    with pytest.raises(homo.NotFound):
        st.write_element("nope", 0, "q")                     # unknown key: 404
    with pytest.raises(homo.ServerError):
        st.write_element(b, -1, "q")                         # IndexOutOfBounds: 500, unchanged
    assert st.val[b] == ["2", "y", "7", "t", "u"]
    assert st.put_set(["1", "x", "7", "z"]) == a             # same contents, same key: revived
    c = st.put_set(list(st.val[b]))                          # equal to b's current contents: collapses
    assert c != b and homo.sum_all(st.rows(), 2, "1000") == "49"
    st.put_empty("K" * 128)
    assert st.val["K" * 128] is None and "K" * 128 in st.keys
    assert homo.set_to_string(["a", 5, True, None]) == "DDSSet(List(a, 5, true, None))"


def test_mutation_vectors_recompute():
    """tests/golden/mutations.json is what the oracle Store answers (guards fixture / oracle drift)."""
    import json
    from oracle import make_fixtures as mf
    fx = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mutations.json")))
    nsq = int(fx["nsquare"])
    st = homo.Store()
    for i, step in enumerate(fx["steps"]):
        try:
            if step["op"] == "put":
                assert st.put_set(step["set"]) == step["key"]
            elif step["op"] == "put_empty":
                st.put_empty(step["key"])
            elif step["op"] == "remove":
                st.remove_set(step["key"])
            elif step["op"] == "add":
                st.add_element(step["key"], step["value"])
            else:
                st.write_element(step["key"], step["position"], step["value"])
            status = 200
        except homo.NotFound:
            status = 404
        except homo.ServerError:
            status = 500
        assert status == step["status"], i
        assert mf._reads(st, nsq, fx["pubkey"], fx["bound"]) == step["reads"], i


def test_store_key_derivation_product_matches_oracle():
    from ddshe.store import key_from_set
    for s in (["1"], [], ["a", 5, True, None], ["٤", "x" * 300]):
        assert key_from_set(s) == homo.key_from_set(s)


def _spki(n: int, e: int) -> str:
    def der(tag, body):
        ln = len(body)
        enc = bytes([ln]) if ln < 0x80 else bytes([0x80 | ((ln.bit_length() + 7) // 8)]) + ln.to_bytes(
            (ln.bit_length() + 7) // 8, "big")
        return bytes([tag]) + enc + body

    def integer(x):
        return der(0x02, x.to_bytes(x.bit_length() // 8 + 1, "big"))
    alg = der(0x30, der(0x06, bytes.fromhex("2a864886f70d010101")) + der(0x05, b""))
    key = der(0x30, integer(n) + integer(e))
    return der(0x30, alg + der(0x03, b"\0" + key)).hex()


def test_x509_jdk_key_length_check():
    """RSAKeyFactory.checkRSAProviderKeyLengths: length rounded up to a multiple of 8 (505..511-bit
    moduli pass), at most 16384, exponent <= 64 bits above 3072 bits; product and oracle agree."""
    from ddshe import x509
    cases = [((1 << 504) + 1, 65537, True), ((1 << 503) + 1, 65537, False), ((1 << 4095) + 1, (1 << 64) + 1, False),
             ((1 << 4095) + 1, (1 << 63) + 1, True), ((1 << 3071) + 1, (1 << 100) + 1, True),
             ((1 << 16383) + 1, 3, True), ((1 << 16384) + 1, 3, False)]
    for n, e, ok in cases:
        h = _spki(n, e)
        if ok:
            assert x509.rsa_modulus(h) == homo.rsa_modulus_from_pubkey_hex(h) == n
        else:
            with pytest.raises(ValueError):
                x509.rsa_modulus(h)
            with pytest.raises(homo.ServerError):
                homo.rsa_modulus_from_pubkey_hex(h)


def test_equality_scan_semantics():
    """HomoDet.compare on AnyJsonFormat texts (DDSJsonProtocol.scala:22-28) and SearchEntry's needle:
    item.toString of the DDSItem case class (DDSRestServer.scala:845), unlike SearchEntryOR/AND."""
    from oracle import homo
    assert homo.homo_det_compare(True, "true") and homo.homo_det_compare(None, "None")
    assert not homo.homo_det_compare(True, "True")
    assert homo.entry_needle("x") == "DDSItem(x)" and homo.entry_needle(7) == "DDSItem(7)"
    rows = [("a", ["x", "y"]), ("b", ["DDSItem(x)"]), ("c", None), ("d", [True, "z"])]
    assert homo.search_entry("SearchEntry", rows, ["x"]) == {"b"}
    assert homo.search_entry("SearchEntryOR", rows, ["x", "q", "true"]) == {"a", "d"}
    assert homo.search_entry("SearchEntryAND", rows, ["x", "y", "q"]) == set()
    assert homo.search_eq("SearchEq", rows, 0, "x") == {"a"}  # strict guard: length - 1 > position
    assert homo.search_eq("SearchNEq", rows, 0, "x") == {"d"}
    assert homo.is_element(["x", True], "true") and not homo.is_element(["x"], "y")
