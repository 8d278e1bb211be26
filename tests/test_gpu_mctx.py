"""One caller, several GPU shards (dds_mctx / dds_mcol, SURVEY.md §8b device_mask), checked against
the oracle. On a one-GPU box the shards share device 0 (dds_mctx_create_devices with a repeated
device): the same code path as distinct GPUs except that the partial copies stay on one device."""
import random

import numpy as np
import pytest

from oracle import homo

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]])
def test_mcol_fold_vs_oracle(keys, devices):
    import ddshe
    N = keys["paillier2048_committed"]["nsquare"]
    m = ddshe.MultiEngine(devices)
    assert m.shards == len(devices)
    rng = random.Random(len(devices))
    xs = [rng.randrange(N) for _ in range(1000)]
    col = m.column(N, 5000)
    col.append(xs[:300])                  # appends land on shards in 64-row blocks
    col.append(xs[300:1000])
    assert len(col) == 1000
    assert col.fold() == homo.modmul_fold(xs, N)
    ids = sorted(rng.sample(range(1000), 555))
    assert col.fold_rows(ids) == homo.modmul_fold([xs[i] for i in ids], N)
    assert col.fold_rows([64, 65]) == xs[64] * xs[65] % N             # both on one shard
    assert col.fold_rows([63, 64]) == xs[63] * xs[64] % N             # across a block boundary
    assert col.fold_rows([777]) == xs[777]
    assert col.fold_dec(ids) == str(homo.modmul_fold([xs[i] for i in ids], N))
    col.append_dec(["-5", str(3 * N + 1)])
    assert col.fold_dec([1000]) == "-5"
    assert col.fold_rows([1001]) == 3 * N + 1
    assert col.fold_dec() == str(homo.modmul_fold(xs + [-5, 3 * N + 1], N))
    with pytest.raises(ddshe.NotFound):
        col.fold_rows([])
    col.close()
    m.close()


def test_mcol_mask_and_synth_decrypts(keys):
    """device_mask form + synthetic rows: the sharded column holds the same global rows as one column
    (k_synth_rows maps local rows back to global ones), so Dec(fold) = sum(m_i) and the product equals
    the single-column fold."""
    import ddshe
    k = keys["paillier2048_committed"]
    eng = ddshe.Engine(0)
    one = eng.column(k["nsquare"], 20000)
    one.fill_paillier_synth(k["n"], k["g"], seed=9, row0=0, count=20000, pool=64)
    want = one.fold()
    for m in (ddshe.MultiEngine(mask=1), ddshe.MultiEngine([0, 0, 0, 0])):
        col = m.column(k["nsquare"], 20000)
        col.fill_paillier_synth(k["n"], k["g"], seed=9, count=12345, pool=64)
        col.fill_paillier_synth(k["n"], k["g"], seed=9, count=20000 - 12345, pool=64)
        assert col.fold() == want
        ms = ddshe.synth_plaintexts(9, 0, 20000)
        assert homo.paillier_decrypt(col.fold(), k) == int(ms.astype(np.int64).sum()) % k["n"]
        col.close()
        m.close()
    one.close()
    eng.close()


def test_mcol_append_failure_leaves_column_unchanged(keys):
    import ddshe
    N = keys["rsa1024_committed"]["n"]
    m = ddshe.MultiEngine([0, 0])
    col = m.column(N, 1000)
    col.append(list(range(2, 202)))
    with pytest.raises(ddshe.DDSError):
        col.append_dec(["1"] * 100 + ["12x"] + ["2"] * 100)   # NumberFormatException in one shard
    assert len(col) == 200
    assert col.fold() == homo.modmul_fold(list(range(2, 202)), N)
    col.close()
    m.close()


def test_mcol_rsa_shards_on_the_lane_fold(keys):
    """Shards big enough for the one-bignum-per-lane MultAll fold (k_fold1, >= ~1M rows per shard):
    the same product as one column, and as the oracle on a sampled subset."""
    import ddshe
    n = keys["rsa2048_seed3"]["n"]
    rows = 2_400_000
    one = ddshe.Engine(0)
    col1 = one.column(n, rows)
    col1.fill_random(2040, 33, 0, rows)
    buf = col1.read_buffer(0, rows)
    want = col1.fold()
    m = ddshe.MultiEngine([0, 0])
    mc = m.column(n, rows)
    mc.append_buffer(buf)
    assert len(mc) == rows
    assert mc.fold() == want
    ids = list(range(5, rows, 4099))
    xs = [int.from_bytes(bytes(buf[i]), "big") for i in ids]
    assert mc.fold_rows(ids) == homo.modmul_fold(xs, n)
    mc.close()
    m.close()
    col1.close()
    one.close()
