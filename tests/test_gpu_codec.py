"""GPU decimal codec: BigInteger.toString rows -> device column, parsed by
k_dec_parse / k_dec_fix, bit-exact against Python's int(str) (the same radix-10 grammar as
java.math.BigInteger(String) for ASCII input). Reference parse sites:
DDSRestServer.scala:417,419,422,513; row format DDSSet.scala:3, DDSJsonProtocol.scala:14-29."""
import random
import sys

import numpy as np
import pytest

import ddshe
from oracle import homo

pytestmark = pytest.mark.gpu

if hasattr(sys, "set_int_max_str_digits"):  # rows here exceed CPython's default 4300-digit str->int cap
    sys.set_int_max_str_digits(0)


def residue(x, N):
    """dds_col_read returns canonical residues (BigInteger.mod)."""
    return x % N


def fmt(x, rng):
    """BigInteger-valid spellings of x: optional '+', leading zeros."""
    s = str(abs(x))
    if rng.random() < 0.2:
        s = "0" * rng.randrange(1, 20) + s
    if x < 0:
        return "-" + s
    return ("+" + s) if rng.random() < 0.1 else s


@pytest.mark.parametrize("bits", [61, 1000, 2048, 4095, 6140])
def test_append_dec_random_rows(eng, bits):
    rng = random.Random(bits)
    N = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
    xs = []
    for i in range(3000):
        k = rng.randrange(10)
        if k < 6:
            x = rng.randrange(N)
        elif k < 7:
            x = rng.randrange(N, 2 * N)
        elif k < 8:
            x = rng.randrange(2 * N, 1 << (bits + 1))   # below the column capacity, >= 2N
        elif k < 9:
            x = -rng.randrange(1 << (bits + 1))
        else:
            x = rng.randrange(10 ** rng.randrange(1, 30))  # short rows
        xs.append(x)
    col = eng.column(N, len(xs) + 10)
    col.append_dec([fmt(x, rng) for x in xs])
    got = col.read(0, len(xs))
    for i, (x, g) in enumerate(zip(xs, got)):
        assert g == residue(x, N), (i, x)
    assert col.fold() == homo.modmul_fold([g for g in got], N)


def test_append_dec_digit_chunk_boundaries(eng, keys):
    N = keys["paillier2048_committed"]["nsquare"]
    rows = ["0", "-0", "+0", "00000000", "000000000", "1", "-1", "99999999", "100000000", "999999999",
            "1000000000", "12345678" * 2, "12345678" * 2 + "9", "9" * 64, "1" + "0" * 1000,
            str(N - 1), str(N), str(N + 1), str(2 * N - 1), str(2 * N), "-" + str(N), "-" + str(N + 1),
            "0" * 5000 + "42"]
    col = eng.column(N, len(rows))
    col.append_dec(rows)
    got = col.read(0, len(rows))
    for s, g in zip(rows, got):
        assert g == residue(int(s), N), s


def test_append_dec_arrow_layout(eng, keys):
    N = keys["rsa1024_committed"]["n"]
    rng = random.Random(7)
    xs = [rng.randrange(N) for _ in range(500)]
    enc = [str(x).encode() for x in xs]
    chars = b"xx" + b"".join(enc)          # offsets need not start at 0
    offs = np.zeros(len(enc) + 1, dtype=np.uint64)
    offs[0] = 2
    np.cumsum([len(e) for e in enc], out=offs[1:])
    offs[1:] += 2
    col = eng.column(N, len(xs))
    col.append_dec((chars, offs))
    assert col.read(0, len(xs)) == xs


@pytest.mark.parametrize("bad", ["", "-", "+", "12a3", " 12", "12 ", "1 2", "--1", "+-1", "0x10", "1.0",
                                 "١٢", "1e5", "9" * 40 + "/"])
def test_append_dec_format_errors(eng, keys, bad):
    N = keys["paillier1024_seed1"]["nsquare"]
    col = eng.column(N, 8)
    col.append_dec(["5"])
    with pytest.raises(ddshe.DDSError) as ei:
        col.append_dec(["7", bad, "9"])
    assert ei.value.status == ddshe.DDS_E_FORMAT
    assert len(col) == 1 and col.read(0, 1) == [5]


def test_append_dec_too_wide_is_range_error(eng, keys):
    N = keys["paillier1024_seed1"]["nsquare"]
    col = eng.column(N, 8)
    with pytest.raises(ddshe.DDSError) as ei:
        col.append_dec(["3", str(N << 200)])
    assert ei.value.status == ddshe.DDS_E_RANGE
    assert len(col) == 0


def test_sum_all_dec_gpu_codec_matches_column_fold(eng, keys):
    """SumAll over decimal rows (the route's own input format) == fold of the binary column."""
    k = keys["paillier2048_committed"]
    count = 20_000
    col = eng.column(k["nsquare"], count)
    col.fill_paillier_synth(k["n"], k["g"], seed=5, row0=0, count=count, pool=64)
    cs = col.read(0, count)
    got = eng.sum_all_dec([str(c) for c in cs], str(k["nsquare"]))
    assert got == str(col.fold())
    m = ddshe.synth_plaintexts(5, 0, count).astype(np.int64).sum()
    assert homo.paillier_decrypt(int(got), k) == int(m) % k["n"]


def test_mult_all_dec_wide_and_negative_rows(eng, keys):
    """Rows wider than the column (garbage, never a ciphertext) are reduced at the boundary;
    negative rows fold as their residues (BigInteger.mod), DDSRestServer.scala:506-524."""
    n = keys["rsa1024_committed"]["n"]
    rng = random.Random(11)
    xs = [rng.randrange(n) for _ in range(300)]
    xs[5] = n * (1 << 300) + 12345
    xs[17] = -rng.randrange(n * 5)
    xs[200] = -(n << 400) - 7
    got = eng.mult_all_dec([str(x) for x in xs], str(n))
    acc = xs[0]
    for x in xs[1:]:
        acc = acc * x % n
    assert got == str(acc)


def test_sum_all_dec_long_zero_padded_row(eng, keys):
    """A row longer than one staging chunk (64 MiB) still parses (boundary path)."""
    N = keys["paillier1024_seed1"]["nsquare"]
    rows = ["3", "0" * (65 << 20) + "5", "7"]
    assert eng.sum_all_dec(rows, str(N)) == str(3 * 5 * 7 % N)


def test_sum_all_dec_string_rows_parallel_chunks(eng, keys):
    """NUL-terminated rows (the JNA String[] of the route) over several 64 MiB staging chunks, with
    BigInteger spellings ('+', leading zeros, negatives), a row >= N and one row longer than a chunk:
    the host pool's lengths/copies and the chunk cut keep every row intact."""
    k = keys["paillier1024_seed1"]
    N = k["nsquare"]
    rng = random.Random(21)
    xs = [rng.randrange(N) for _ in range(120_000)]
    xs[7] = N + 12345
    xs[60_001] = -rng.randrange(N)
    rows = [fmt(x, rng) for x in xs]
    rows[90_000] = "0" * (65 << 20) + "9"  # longer than one chunk: parsed on the boundary path
    xs[90_000] = 9
    want = 1
    for x in xs:
        want = want * x % N
    assert eng.sum_all_dec(rows, str(N)) == str(want)


def test_sum_all_dec_string_rows_growing_lengths(eng, keys):
    """String[] rows are measured and copied by the host pool into per-thread regions of the pinned
    chunk, with rows per chunk sized by the longest row seen so far: rows that suddenly grow (short
    rows, then ~4.6 KB rows, then rows wider than one thread's region but narrower than a chunk) make
    regions run out of room mid-chunk; the chunk is cut at the first row that did not fit and the rest
    is redone, so every row still folds exactly once, in order."""
    k = keys["paillier1024_seed1"]
    N = k["nsquare"]
    rng = random.Random(33)
    xs = [rng.randrange(N) for _ in range(40_000)]
    rows = [str(x) for x in xs]              # 24 MB: the fused fill (requests of >= 16 MiB)
    for i in range(30_000, 40_000):          # 4 KB of leading zeros each: regions overflow mid-chunk
        rows[i] = "0" * 4_000 + rows[i]
    for i in (33_000, 36_789):               # wider than a region (64 MiB / pool threads), < a chunk
        rows[i] = "0" * (9 << 20) + rows[i]
    xs[77] = -xs[77]
    rows[77] = "-" + rows[77]
    want = 1
    for x in xs:
        want = want * (x % N) % N
    assert eng.sum_all_dec(rows, str(N)) == str(want)
    bad = list(rows)
    bad[35_000] = bad[35_000][:-3] + "x12"
    with pytest.raises(ddshe.DDSError) as ei:
        eng.sum_all_dec(bad, str(N))
    assert ei.value.status == ddshe.DDS_E_FORMAT
    assert "35000" in str(ei.value)


def test_sum_all_dec_two_chunks(eng, keys):
    """dds_sum_all_dec splits a request of fewer than 2^19 rows into two chunks (the second one's
    copies overlap the first one's parse, 4 lanes per row for these small batches): the fold over
    12,001 rows equals the oracle's, and a malformed row or a negative / >= 2N row in the second chunk
    is handled as in the first (NumberFormatException names the row; BigInteger.mod semantics)."""
    from oracle import homo
    N = keys["paillier1024_seed1"]["nsquare"]
    rng = np.random.default_rng(12)
    n = 12_001
    xs = [int(rng.integers(1, 2**62)) * int(rng.integers(1, 2**62)) % N for _ in range(n)]
    xs[8000] = -xs[8000]            # negative row in the second chunk
    xs[9000] = xs[9000] + 3 * N     # row >= 2N in the second chunk
    xs[11] = N - 1
    rows = [str(x) for x in xs]
    want = 1
    for x in xs:
        want = want * (x % N) % N
    assert int(eng.sum_all_dec(rows, str(N))) == want == homo.modmul_fold([x % N for x in xs], N)
    bad = list(rows)
    bad[9500] = "12x4"
    with pytest.raises(ddshe.DDSError) as ei:
        eng.sum_all_dec(bad, str(N))
    assert ei.value.status == ddshe.DDS_E_FORMAT
    assert "9500" in str(ei.value)
