"""GPU parity tests: the HIP path (through the C-ABI) against the oracle and the golden
fixtures, bit-exact. Route references: DDSRestServer.scala:355-539 (Sum/SumAll/Mult/MultAll),
:682-830 (Search*), SJHomoLibProvider.scala:58 (encrypt)."""
import random

import numpy as np
import pytest

from oracle import homo

pytestmark = pytest.mark.gpu


def H(x):
    return int(x, 16)


# ---------------------------------------------------------------------------
# golden fixtures
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["paillier2048_committed", "paillier1024_seed1", "paillier3072_seed4"])
def test_paillier_fold_golden(eng, keys, vectors, name):
    k, v = keys[name], vectors[name]
    cs = [H(r["c"]) for r in v["rows"]]
    assert eng.paillier_sum(k["nsquare"], cs) == H(v["fold"])
    assert homo.paillier_decrypt(H(v["fold"]), k) == v["dec_sum"]


@pytest.mark.parametrize("name", ["rsa1024_committed", "rsa2048_seed3"])
def test_rsa_fold_golden(eng, keys, vectors, name):
    k, v = keys[name], vectors[name]
    assert eng.rsa_product(k["n"], [H(r["c"]) for r in v["rows"]]) == H(v["fold"])


@pytest.mark.parametrize("name,key,field", [("edges_nsq2048", "paillier2048_committed", "nsquare"),
                                            ("edges_n1024", "rsa1024_committed", "n"),
                                            ("edges_nsq3072", "paillier3072_seed4", "nsquare")])
def test_fold_edge_cases_golden(eng, keys, vectors, name, key, field):
    import ddshe
    N = keys[key][field]
    for case in vectors[name]:
        ops = [H(x) for x in case["ops"]]
        if case["result"] is None:
            with pytest.raises(ddshe.NotFound):
                eng.modmul_fold(N, ops)
        else:
            assert eng.modmul_fold(N, ops) == H(case["result"]), case["name"]


@pytest.mark.parametrize("name", ["paillier2048_committed", "paillier1024_seed1"])
def test_pairs_golden(eng, keys, vectors, name):
    k, v = keys[name], vectors[name]
    a = [H(p["a"]) for p in v["pairs"]]
    b = [H(p["b"]) for p in v["pairs"]]
    assert eng.modmul_pairs(k["nsquare"], a, b) == [H(p["c"]) for p in v["pairs"]]


def test_routes_golden(eng, vectors):
    """Route-level SumAll / MultAll / Search* through the decimal C-ABI entry points."""
    from ddshe import routes
    rv = vectors["routes"]
    rows = rv["rows"]
    keyed = [(f"k{i}", r) for i, r in enumerate(rows)]
    for c in rv["cases"]:
        if c["route"] == "SumAll":
            if c["result"] is None:
                with pytest.raises(routes.NotFound):
                    routes.sum_all(eng, rows, c["position"], c["nsqr"])
            else:
                assert routes.sum_all(eng, rows, c["position"], c["nsqr"]) == c["result"]
        elif c["route"] == "MultAll":
            assert routes.mult_all(eng, rows, c["position"], c["n"]) == c["result"]
        else:
            assert sorted(routes.search(eng, c["route"], keyed, c["position"], c["value"])) == c["result"]


# ---------------------------------------------------------------------------
# randomized parity at sizes the oracle finishes in seconds
# ---------------------------------------------------------------------------
SIZES = [2, 3, 7, 64, 65, 127, 1000, 4099]


@pytest.mark.parametrize("bits", [512, 1024, 2048, 2050, 3072, 4095, 4096, 6144])
def test_fold_random_moduli(eng, bits):
    rng = random.Random(bits)
    N = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
    for k in (2, 5, 333):
        xs = [rng.randrange(N) for _ in range(k)]
        assert eng.modmul_fold(N, xs) == homo.modmul_fold(xs, N), (bits, k)


# Moduli on either side of the QP limit of each shape (Mont QP reduces against N~ = N·n0, which
# needs W·S >= bits(N) + W + 2; above it the shape keeps n0), with worst-case operands (N-1 and
# near it). k = 5000 runs the tree through 16-lane (> 2048 groups) and 32-lane (QP) levels.
QP_EDGE_BITS = [1090, 1118, 2042, 2070, 2098, 2126, 3106, 3134, 4114, 4142, 6235, 6262]


@pytest.mark.parametrize("bits", QP_EDGE_BITS)
def test_fold_qp_shape_edges(eng, bits):
    rng = random.Random(bits * 7)
    N = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
    for k in (2, 3, 5000):
        xs = [N - 1 - rng.randrange(4) for _ in range(k)]
        assert eng.modmul_fold(N, xs) == homo.modmul_fold(xs, N), (bits, k)
    xs = [rng.randrange(N) for _ in range(777)]
    assert eng.modmul_fold(N, xs) == homo.modmul_fold(xs, N), bits


@pytest.mark.parametrize("bits", [1090, 1118, 3106, 3134])
def test_modexp_qp_shape_edges(eng, bits):
    rng = random.Random(bits * 11)
    N = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
    e = rng.getrandbits(bits) | 1
    xs = [N - 1, N - 2, 1, 0] + [rng.randrange(N) for _ in range(60)]
    assert eng.modexp_batch(N, e, xs) == [pow(x, e, N) for x in xs], bits


@pytest.mark.parametrize("k", SIZES)
def test_fold_sizes_committed_nsq(eng, keys, k):
    N = keys["paillier2048_committed"]["nsquare"]
    rng = random.Random(k)
    xs = [rng.randrange(N) for _ in range(k)]
    assert eng.paillier_sum(N, xs) == homo.modmul_fold(xs, N)


def test_fold_small_modulus_and_wide_operands(eng):
    N = 0xFFFFFFFFFFFFFFC5  # 64-bit prime
    rng = random.Random(3)
    xs = [rng.randrange(N) for _ in range(100)]
    assert eng.modmul_fold(N, xs) == homo.modmul_fold(xs, N)
    # operands >= 2N but within the limb width are reduced on the GPU (k_reduce_rows)
    xs2 = [N * 3 + 5, N * 7 + 11, 2**70 + 3]
    assert eng.modmul_fold(N, xs2) == homo.modmul_fold(xs2, N)


def test_fold_operand_too_wide_is_range_error(eng):
    import ddshe
    N = (1 << 61) - 1      # smallest shape: 40 limbs of 28 bits = 1120 bits of operand width
    with pytest.raises(ddshe.DDSError) as ei:
        eng.modmul_fold(N, [1 << 1500, 3])
    assert ei.value.status == ddshe.DDS_E_RANGE


def test_ingest_lds_path_wide_rows(eng, keys):
    """Rows of a 16-byte multiple width take the LDS-staged ingest (k_ingest_be_lds): rows >= 2N are
    classified and reduced, rows wider than the shape's limbs are a range error, rows just below 2^(W*S)
    pass."""
    import ddshe
    N = keys["rsa2048_seed3"]["n"]
    rng = random.Random(17)
    xs = [rng.randrange(N) for _ in range(200)] + [2 * N, 2 * N - 1, 3 * N + 7, 5 * N + 1, (1 << 2127) + 9]
    rng.shuffle(xs)
    for w in (272, 288):
        assert eng.modmul_fold(N, xs, width=w) == homo.modmul_fold(xs, N)
    with pytest.raises(ddshe.DDSError) as ei:
        eng.modmul_fold(N, xs + [1 << 2200], width=288)
    assert ei.value.status == ddshe.DDS_E_RANGE


def test_even_modulus_folds_like_biginteger(eng):
    """Round 1 refused even moduli; BigInteger.mod takes any positive modulus (see test_gpu_moduli.py)."""
    assert eng.modmul_fold(1 << 100, [3, 5]) == 15
    assert eng.modmul_fold(1 << 100, [1 << 99, 6]) == 0


def test_pairs_random(eng, keys):
    N = keys["rsa2048_seed3"]["n"]
    rng = random.Random(11)
    a = [rng.randrange(N) for _ in range(300)]
    b = [rng.randrange(N) for _ in range(300)]
    assert eng.modmul_pairs(N, a, b) == [x * y % N for x, y in zip(a, b)]


@pytest.mark.parametrize("bits", [61, 512, 1024, 2047, 2048, 3072, 4095, 6144, 8192, 16000])
def test_small_pair_batches_tail_shape(eng, bits):
    """n <= 8 pairs take the latency path (host limb split, k_pairs in the tail shape, one sync):
    every shape, operands >= 2N reduced like BigInteger, wider ones a range error as on the batch path."""
    import ddshe
    rng = random.Random(bits)
    N = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
    for n in (1, 2, 3, 8):
        a = [rng.randrange(N) for _ in range(n)]
        b = [rng.randrange(N) for _ in range(n)]
        if n == 8:
            a[0], b[1], a[2], b[2] = N - 1, N - 1, 2 * N + 3, 3 * N
        assert eng.modmul_pairs(N, a, b) == [x * y % N for x, y in zip(a, b)], n
    with pytest.raises(ddshe.DDSError) as ei:
        eng.modmul_pairs(N, [1 << (2 * bits + 2000)], [3])
    assert ei.value.status == ddshe.DDS_E_RANGE
    m = (1 << bits) - 1
    x = [m - 1, m - 2]
    assert eng.modmul_pairs(m, x, x[::-1]) == [(m - 1) * (m - 2) % m] * 2


def test_bigint_sum(eng):
    rng = random.Random(12)
    xs = [rng.getrandbits(4096) for _ in range(5000)]
    assert eng.bigint_sum(xs) == sum(xs)
    assert eng.bigint_sum([5]) == 5


@pytest.mark.parametrize("count,bits", [(2, 64), (3, 2048), (17, 4096), (1000, 2048), (257, 31)])
def test_bigint_product_tree(eng, count, bits):
    rng = random.Random(count * bits)
    xs = [rng.getrandbits(bits) for _ in range(count)]
    exp = 1
    for x in xs:
        exp *= x
    assert eng.bigint_product(xs) == exp
    assert eng.bigint_product(xs[:1] + [0] + xs[1:]) == 0
    assert eng.mult_all_dec(["-3", "5", "-7"], None) == "105"
    assert eng.mult_all_dec(["-3", "5"], None) == "-15"


def test_decimal_routes_signs_and_formats(eng, keys):
    N = keys["paillier1024_seed1"]["nsquare"]
    vals = ["-12345", "+777", "0000042", str(N + 99)]
    got = eng.sum_all_dec(vals, str(N))
    acc = int(vals[0])
    for v in vals[1:]:
        acc = acc * int(v) % N
    assert got == str(acc)
    assert eng.sum_all_dec(["0007"], str(N)) == "7"      # single operand: BigInteger(str).toString
    assert eng.sum_all_dec(["-5", "3", "10"], None) == "8"
    with pytest.raises(Exception):
        eng.sum_all_dec(["12a"], str(N))


# ---------------------------------------------------------------------------
# encryption
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("name,count", [("paillier1024_seed1", 40), ("paillier2048_committed", 24),
                                        ("paillier3072_seed4", 6)])
def test_encrypt_batch(eng, keys, vectors, name, count):
    k = keys[name]
    rows = vectors[name]["rows"][:count]
    ms = [r["m"] for r in rows]
    rs = [H(r["r"]) for r in rows]
    got = eng.paillier_encrypt_batch(k["n"], k["g"], ms, rs)
    assert got == [H(r["c"]) for r in rows]


def test_encrypt_then_sum_decrypts(eng, keys):
    k = keys["paillier1024_seed1"]
    rng = random.Random(21)
    ms = [rng.randrange(10000) for _ in range(256)] + [0, 2**31 - 1]
    rs = [rng.randrange(1, k["n"]) for _ in ms]
    cs = eng.paillier_encrypt_batch(k["n"], k["g"], ms, rs)
    assert homo.paillier_decrypt(eng.paillier_sum(k["nsquare"], cs), k) == sum(ms) % k["n"]


# ---------------------------------------------------------------------------
# device columns, synthetic rows, partial combination (multi-GPU algebra)
# ---------------------------------------------------------------------------
def test_column_append_fold_read(eng, keys):
    N = keys["paillier2048_committed"]["nsquare"]
    rng = random.Random(31)
    xs = [rng.randrange(N) for _ in range(777)]
    col = eng.column(N, 1000)
    col.append(xs[:500])
    col.append(xs[500:])
    assert len(col) == 777
    assert col.read(10, 5) == xs[10:15]
    assert col.fold() == homo.modmul_fold(xs, N)
    assert col.fold(100, 1) == xs[100]
    assert col.fold(3, 200) == homo.modmul_fold(xs[3:203], N)
    parts, rows = [], []
    for a, b in ((0, 100), (100, 377), (377, 777)):
        p, r = col.fold_partial(a, b - a)
        parts.append(p)
        rows.append(r)
    assert eng.combine_partials(N, np.stack(parts), rows) == homo.modmul_fold(xs, N)


@pytest.mark.parametrize("name", ["paillier2048_committed", "paillier1024_seed1"])
def test_synthetic_rows_decrypt(eng, keys, name):
    import ddshe
    k = keys[name]
    count = 20000
    col = eng.column(k["nsquare"], count)
    col.fill_paillier_synth(k["n"], k["g"], seed=2, row0=0, count=count, pool=64)
    ms = ddshe.synth_plaintexts(2, 0, count)
    sample = col.read(0, 300)
    for i in (0, 1, 299):
        assert homo.paillier_decrypt(sample[i], k) == ms[i]
    assert col.fold(0, 300) == homo.modmul_fold(sample, k["nsquare"])
    assert homo.paillier_decrypt(col.fold(), k) == int(ms.astype(np.int64).sum()) % k["n"]


def test_large_fold_property(eng, keys):
    """Full-size-style property check: Dec(fold of 1M synthetic rows) == sum(m_i)."""
    import ddshe
    k = keys["paillier2048_committed"]
    count = 1_000_003
    col = eng.column(k["nsquare"], count)
    col.fill_paillier_synth(k["n"], k["g"], seed=5, row0=0, count=count, pool=256)
    ms = ddshe.synth_plaintexts(5, 0, count)
    assert homo.paillier_decrypt(col.fold(), k) == int(ms.astype(np.int64).sum()) % k["n"]


# ---------------------------------------------------------------------------
# OPE range filter
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("n", [1, 63, 4096, 4097, 8192, 8193, 100_000, 3_000_001])
def test_ope_filter_vs_numpy(eng, n):
    rng = np.random.default_rng(n)
    col = rng.integers(-2**63, 2**63 - 1, size=n, dtype=np.int64)
    col[: min(n, 10)] = np.array([-2**63, 2**63 - 1, 0, -1, 1, 5, 5, 5, 7, -7], dtype=np.int64)[: min(n, 10)]
    valid = (rng.random(n) > 0.1).astype(np.uint8)
    for bound in (int(col[n // 2]), -2**63, 2**63 - 1, 5):
        for op, f in (("gt", np.greater), ("ge", np.greater_equal), ("lt", np.less), ("le", np.less_equal)):
            exp = np.nonzero(f(col, bound) & (valid != 0))[0].astype(np.uint32)
            got = eng.ope_filter(col, valid, bound, op)
            assert np.array_equal(got, exp), (n, bound, op)
    got = eng.ope_filter(col, None, 0, "ge")
    assert np.array_equal(got, np.nonzero(col >= 0)[0].astype(np.uint32))


def test_ope_filter_long_lookback(eng):
    """> 256 x 8192-row tiles: the single-pass compaction's look-back crosses several probe
    windows; matches are dense (all rows) and sparse (every 1000th row) so tile counts vary."""
    n = 12_000_017
    col = np.arange(n, dtype=np.int64)
    valid = np.ones(n, dtype=np.uint8)
    got = eng.ope_filter(col, valid, -1, "gt")
    assert len(got) == n and np.array_equal(got, np.arange(n, dtype=np.uint32))
    sparse = (col % 1000 == 0).astype(np.int64)
    got = eng.ope_filter(sparse, valid, 0, "gt")
    assert np.array_equal(got, np.nonzero(sparse)[0].astype(np.uint32))


def test_fold_host_buffer_chunked(eng, keys):
    """dds_paillier_sum on a host buffer larger than one pinned ingest chunk (64 MiB): rows cross
    chunk boundaries, and an operand in [N, 2N) in a later chunk still folds as its residue."""
    import ddshe
    key = keys["paillier2048_committed"]
    N = key["nsquare"]
    k = 300_001  # 512-byte rows: 3 chunks of 131072 rows
    col = eng.column(N, k)
    col.fill_paillier_synth(key["n"], key["g"], 7, 0, k)
    buf = col.read_buffer(0, k)
    assert buf.shape == (k, 512)
    want = col.fold()
    assert eng.fold_buffer(N, buf) == want
    r = 250_000
    x = int.from_bytes(bytes(buf[r]), "big")
    buf[r] = np.frombuffer((x + N).to_bytes(512, "big"), dtype=np.uint8)
    assert eng.fold_buffer(N, buf) == want
    ms = ddshe.synth_plaintexts(7, 0, k)
    assert homo.paillier_decrypt(want, key) == int(ms.astype("int64").sum()) % key["n"]
    col.close()


@pytest.mark.parametrize("bits", [61, 1100, 2047, 2048, 4095, 4136])
def test_gpu_egress_pairs_and_column_read(eng, bits):
    """k_egress_be (rW rows -> big-endian bytes on the GPU): batched pairs and column reads at byte widths
    that are not multiples of 4, rows in [N, 2N) read back as their residue (the column keeps rows
    below 2N), rows >= 2N reduced at ingest, the largest shape it serves (S = 160 limbs)."""
    rng = random.Random(bits * 7)
    N = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
    a = [rng.randrange(N) for _ in range(300)] + [N - 1, 0, 1]
    b = [rng.randrange(N) for _ in range(300)] + [N - 1, 5, N - 1]
    assert eng.modmul_pairs(N, a, b) == [x * y % N for x, y in zip(a, b)]
    rows = a[:50] + [N + 3, 2 * N - 1, N, 3 * N + 11]
    col = eng.column(N, len(rows))
    col.append(rows)
    assert col.read(0, len(rows)) == [x % N for x in rows]
    assert col.read(7, 5) == [x % N for x in rows[7:12]]
    col.close()


@pytest.mark.parametrize("key_name", ["paillier1024_seed1", "paillier2048_committed"])
def test_tree_handoff_repeated_folds(eng, keys, key_name):
    """The tree's last levels run in ONE launch with in-kernel hand-offs (sc1 node words, the last
    arriver continues). Repeated folds over every tree shape of the launch plan (256-thread wide
    levels, then the hand-off launch from <= 256 blocks; odd leaf counts leave unpaired nodes) must
    all agree and decrypt to the sum of the plaintexts: a stale sibling read would break either."""
    import ddshe
    k = keys[key_name]
    rows = 70_001
    col = eng.column(k["nsquare"], rows)
    col.fill_paillier_synth(k["n"], k["g"], seed=9, row0=0, count=rows, pool=128)
    ms = ddshe.synth_plaintexts(9, 0, rows).astype(np.int64)
    for count in (3, 257, 513, 1025, 2049, 4097, 8193, 20_000, 70_001):
        want = int(ms[:count].sum()) % k["n"]
        first = col.fold(0, count)
        assert homo.paillier_decrypt(first, k) == want, count
        for _ in range(12):
            assert col.fold(0, count) == first, count
    col.close()


def test_config2_full_size_fold(eng, keys):
    """BASELINE.json config 2 at its full size inside the test suite (not only in bench.py): 10M
    synthetic Paillier ciphertexts under the committed 2048-bit key, resident on the GPU (5.9 GB), one
    SumAll fold; Dec(fold) == sum of the plaintexts, and a 300-row prefix fold equals the oracle's."""
    import ddshe
    k = keys["paillier2048_committed"]
    count = 10_000_000
    col = eng.column(k["nsquare"], count)
    col.fill_paillier_synth(k["n"], k["g"], seed=1, row0=0, count=count, pool=1024)
    ms = ddshe.synth_plaintexts(1, 0, count)
    assert homo.paillier_decrypt(col.fold(), k) == int(ms.astype(np.int64).sum()) % k["n"]
    sample = col.read(0, 300)
    assert col.fold(0, 300) == homo.modmul_fold(sample, k["nsquare"])
    col.close()
