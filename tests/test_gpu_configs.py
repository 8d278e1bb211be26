"""GPU parity for the BASELINE.json configurations (the non-headline ones are parity
cases, not bench lines). Each check is bit-exact against the oracle or a
size-independent property (decrypt of the fold)."""
import random

import numpy as np
import pytest

from oracle import homo

pytestmark = pytest.mark.gpu


def test_config1_paillier1024_10k_vs_c_restatement(eng, keys):
    """Config 1: Paillier HomoAdd sum over 10k encrypted ints, 1024-bit key; the reference
    BigInteger path restated in C (oracle/csrc/fold_ref.c) is the comparison."""
    from oracle import cref
    k = keys["paillier1024_seed1"]
    count = 10_000
    col = eng.column(k["nsquare"], count)
    col.fill_paillier_synth(k["n"], k["g"], seed=1, row0=0, count=count, pool=128)
    cs = col.read(0, count)
    got = eng.paillier_sum(k["nsquare"], cs)          # host-buffer path (ingest + fold)
    assert got == cref.fold(k["nsquare"], cs)
    assert col.fold() == got                           # device-resident path
    import ddshe
    assert homo.paillier_decrypt(got, k) == int(ddshe.synth_plaintexts(1, 0, count).astype(np.int64).sum()) % k["n"]


def test_config3_rsa2048_product_and_ope_filter(eng, keys):
    """Config 3: RSA HomoMult product + OPE range filter, 2048-bit key (scaled to 200k rows
    for the product; the filter runs at the full 10M rows)."""
    k = keys["rsa2048_seed3"]
    n = k["n"]
    rng = np.random.default_rng(3)
    count = 200_000
    ms = rng.integers(1, 10_000, size=count)
    cs = eng.modexp_batch(n, k["e"], ms.tolist())      # HomoMult.encrypt on the GPU
    for i in (0, 1, count - 1):
        assert cs[i] == homo.rsa_encrypt(int(ms[i]), k)
    col = eng.column(n, count)
    col.append(cs)
    prod = col.fold()
    exp = 1
    for m in ms.tolist():
        exp = exp * m % n
    assert homo.rsa_decrypt(prod, k) == exp
    assert col.fold(0, 5000) == homo.modmul_fold(cs[:5000], n)
    # OPE: seeded strictly increasing map of m (order preserving), bound at the median
    rows = 10_000_000
    m_all = rng.integers(0, 10_000, size=rows)
    ope_map = np.cumsum(rng.integers(1, 1 << 40, size=10_000)).astype(np.int64) - (1 << 50)
    col64 = ope_map[m_all]
    valid = np.ones(rows, dtype=np.uint8)
    bound = int(np.sort(col64)[rows // 2])
    for op, f in (("gt", np.greater), ("ge", np.greater_equal), ("lt", np.less), ("le", np.less_equal)):
        got = eng.ope_filter(col64, valid, bound, op)
        assert np.array_equal(got, np.nonzero(f(col64, bound))[0].astype(np.uint32)), op


def test_config4_paillier3072_encrypt_then_sum(eng, keys):
    """Config 4: batched Paillier encrypt (g^m r^n mod n^2) + sum, 3072-bit key (6144-bit n^2),
    scaled to 512 rows per test run; caller-supplied r for bit-exactness."""
    k = keys["paillier3072_seed4"]
    rng = random.Random(4)
    ms = [rng.randrange(10_000) for _ in range(512)]
    rs = [rng.randrange(1, k["n"]) for _ in ms]
    cs = eng.paillier_encrypt_batch(k["n"], k["g"], ms, rs)
    for i in (0, 255, 511):
        assert cs[i] == homo.paillier_encrypt(ms[i], rs[i], k)
    s = eng.paillier_sum(k["nsquare"], cs)
    assert s == homo.modmul_fold(cs, k["nsquare"])
    assert homo.paillier_decrypt(s, k) == sum(ms) % k["n"]


def test_modexp_edge_exponents(eng, keys):
    n = keys["rsa1024_committed"]["n"]
    xs = [0, 1, 2, n - 1, 12345]
    assert eng.modexp_batch(n, 0, xs) == [1 % n] * len(xs)
    assert eng.modexp_batch(n, 1, xs) == [x % n for x in xs]
    assert eng.modexp_batch(n, 65537, xs) == [pow(x, 65537, n) for x in xs]


def test_config3_full_size_product(eng, keys):
    """Config 3's product at its BASELINE size inside the test suite: 10M RSA-2048 ciphertexts
    (rows table[h_i], table = Enc(1..9999) on the GPU, as the bench's column), one MultAll fold through
    the natural dispatch (k_fold1 first level, then the tail shapes over its partials); checked against
    prod_j table[j]^count[j] mod n, and a 5k-row prefix against the oracle (DDSRestServer.scala:506-524)."""
    import ddshe
    k = keys["rsa2048_seed3"]
    n, rows = k["n"], 10_000_000
    table = eng.modexp_batch(n, k["e"], list(range(1, 10000)))
    col = eng.column(n, rows)
    col.fill_table_synth(table, 3, 0, rows)
    prod = col.fold()
    cnt = np.bincount(ddshe.synth_indices(3, 0, rows, 9999), minlength=9999)
    want = 1
    for t, c in zip(table, cnt.tolist()):
        if c:
            want = want * pow(t, c, n) % n
    assert prod == want
    assert col.fold(0, 5000) == homo.modmul_fold(col.read(0, 5000), n)
    col.close()


def test_config4_full_size_encrypt_then_sum(eng, keys):
    """Config 4 at the bench's 1M-row sub-batch inside the test suite: 1M Paillier
    encryptions under the 3072-bit key (CRT halves; r from the seeded device stream, m as config 2),
    then SumAll over the fresh ciphertexts: Dec(sum) == sum(m), and 32 rows spread over the batch equal
    the oracle's g^m r^n mod n^2 (SJHomoLibProvider.scala:58)."""
    import torch

    import ddshe
    k = keys["paillier3072_seed4"]
    rows = 1_000_000
    ms = ddshe.synth_plaintexts(4, 0, rows)
    d_m = torch.from_numpy(ms.astype(np.int32)).to("cuda")
    rcol = eng.column(k["nsquare"], rows)
    rcol.fill_random(k["n"].bit_length() - 1, 4, 0, rows)
    out = eng.column(k["nsquare"], rows)
    out.encrypt_paillier(rcol, 0, d_m.data_ptr(), rows, k["n"], k["g"], k["p"], k["q"])
    torch.cuda.synchronize()
    s = out.fold()
    assert homo.paillier_decrypt(s, k) == int(ms.astype(np.int64).sum()) % k["n"]
    for i in np.linspace(0, rows - 1, 32).astype(int).tolist():
        assert out.read(i, 1)[0] == homo.paillier_encrypt(int(ms[i]), rcol.read(i, 1)[0], k), i
    out.close()
    rcol.close()


def test_fold_buffer_pipelined_pieces(eng, keys):
    """dds_modmul_fold over >= 2^21 host rows folds them in pieces as they cross PCIe (copy stream: DMA +
    k_ingest_be per 64 MiB chunk; compute stream: each piece's fold to a partial, then one tree over the
    pieces): equal to the resident column's fold, also with rows >= 2N in the first and the last piece
    (reduced on the device by k_reduce_rows gated on the ingest flags) and zero-padded wider rows; a row
    wider than the limb width still fails the call."""
    import ddshe
    k = keys["paillier1024_seed1"]
    N = k["nsquare"]
    n = (1 << 21) + 12_345
    col = eng.column(N, n)
    col.fill_paillier_synth(k["n"], k["g"], seed=5, row0=0, count=n, pool=64)
    buf = col.read_buffer(0, n)
    want = col.fold()
    col.close()
    assert eng.fold_buffer(N, buf) == want
    width = buf.shape[1] + 64  # 512 more bits than n^2: past the column's limbs too
    wide = np.zeros((n, width), dtype=np.uint8)
    wide[:, 64:] = buf
    del buf
    for i, mult in ((3, 2), (17, 3), (n - 2, 2), (n // 2, 5)):
        x = int.from_bytes(wide[i].tobytes(), "big") + mult * N
        wide[i] = np.frombuffer(x.to_bytes(width, "big"), dtype=np.uint8)
    assert eng.fold_buffer(N, wide) == want
    wide[n - 7, 0] = 0x80  # >= 2^(8 width - 1): wider than the column's limbs
    with pytest.raises(ddshe.DDSError) as ei:
        eng.fold_buffer(N, wide)
    assert ei.value.status == ddshe.DDS_E_RANGE


def test_fold_buffer_pipelined_rsa_product(eng, keys):
    """The pieced host-row fold on the RSA MultAll shape (2048-bit n, one bignum per lane for long
    pieces): 2^21 + 3 random rows < n folded from a host buffer equal the resident column's fold."""
    k = keys["rsa2048_seed3"]
    n = k["n"]
    rows = (1 << 21) + 3
    col = eng.column(n, rows)
    col.fill_random(2047, seed=9, row0=0, count=rows)
    buf = col.read_buffer(0, rows)
    want = col.fold()
    col.close()
    assert eng.fold_buffer(n, buf) == want
    # and a prefix of the same buffer (one piece, ingest then fold) against the oracle
    prefix = [int.from_bytes(buf[i].tobytes(), "big") for i in range(4000)]
    assert eng.fold_buffer(n, buf[:4000]) == homo.modmul_fold(prefix, n)
