"""GPU parity of batched encryption (HomoAdd.encrypt, SJHomoLibProvider.scala:58; HomoMult.encrypt, :59):
windowed modexp schedules, the CRT path (p^2 / q^2 halves + Garner) and the device-resident
column path, bit-exact against the oracle (oracle/homo.py) and the golden vectors."""
import random

import numpy as np
import pytest

from oracle import homo

pytestmark = pytest.mark.gpu

PAILLIER = ("paillier1024_seed1", "paillier2048_committed", "paillier3072_seed4")


def H(x):
    return int(x, 16)


@pytest.mark.parametrize("name,count", [("paillier1024_seed1", 40), ("paillier2048_committed", 24),
                                        ("paillier3072_seed4", 6)])
def test_encrypt_crt_golden(eng, keys, vectors, name, count):
    k = keys[name]
    rows = vectors[name]["rows"][:count]
    rs = [H(r["r"]) for r in rows]
    if any(r >= k["n"] for r in rs):
        pytest.skip("golden r outside [1, n)")
    got = eng.paillier_encrypt_batch_crt(k["p"], k["q"], k["g"], [r["m"] for r in rows], rs)
    assert got == [H(r["c"]) for r in rows]


@pytest.mark.parametrize("name", PAILLIER)
def test_encrypt_crt_equals_public_path(eng, keys, name):
    k = keys[name]
    rng = random.Random(5)
    ms = [0, 1, 9999, 2**31 - 1] + [rng.randrange(10000) for _ in range(60)]
    rs = [1, k["n"] - 1, 2, k["n"] // 2] + [rng.randrange(1, k["n"]) for _ in range(60)]
    crt = eng.paillier_encrypt_batch_crt(k["p"], k["q"], k["g"], ms, rs)
    pub = eng.paillier_encrypt_batch(k["n"], k["g"], ms, rs)
    assert crt == pub
    for i in (0, 1, 2, 3, 63):
        assert crt[i] == homo.paillier_encrypt(ms[i], rs[i], k)
    # the factors may come in either order
    assert eng.paillier_encrypt_batch_crt(k["q"], k["p"], k["g"], ms[:8], rs[:8]) == crt[:8]


def test_encrypt_crt_errors(eng, keys):
    import ddshe
    k = keys["paillier1024_seed1"]
    with pytest.raises(ddshe.DDSError) as ei:
        eng.paillier_encrypt_batch_crt(k["p"], k["q"], k["g"], [1], [k["n"]])  # r >= n
    assert ei.value.status == ddshe.DDS_E_RANGE
    with pytest.raises(ddshe.DDSError) as ei:
        eng.paillier_encrypt_batch_crt(k["p"], k["p"], k["g"], [1], [2])  # p == q
    assert ei.value.status == ddshe.DDS_E_ARG
    with pytest.raises(ddshe.DDSError) as ei:
        eng.paillier_encrypt_batch_crt(k["p"], k["q"] + 1, k["g"], [1], [2])  # q + 1 is even
    assert ei.value.status == ddshe.DDS_E_ARG


@pytest.mark.parametrize("name", PAILLIER)
def test_column_encrypt_then_sum(eng, keys, name):
    """Device-resident path of config 4: seeded r column, device m, both paths, then the fold."""
    import torch
    k = keys[name]
    count = 300
    rng = np.random.default_rng(7)
    ms = rng.integers(0, 10000, size=count, dtype=np.uint32)
    d_m = torch.from_numpy(ms.astype(np.int32)).to("cuda")
    rcol = eng.column(k["nsquare"], count)
    rcol.fill_random(k["n"].bit_length() - 1, 11, 0, count)
    rs = rcol.read(0, count)
    assert all(1 <= r < k["n"] and r & 1 for r in rs)
    outs = []
    for p, q in ((None, None), (k["p"], k["q"])):
        out = eng.column(k["nsquare"], count)
        out.encrypt_paillier(rcol, 0, d_m.data_ptr(), count, k["n"], k["g"], p, q)
        torch.cuda.synchronize()
        outs.append(out)
    a, b = outs[0].read(0, count), outs[1].read(0, count)
    assert a == b
    for i in (0, count // 2, count - 1):
        assert a[i] == homo.paillier_encrypt(int(ms[i]), rs[i], k)
    s = outs[1].fold()
    assert homo.paillier_decrypt(s, k) == int(ms.astype(np.int64).sum()) % k["n"]


def test_modexp_window_schedules(eng, keys):
    """Exponents that exercise every window shape: single bits, long zero runs, all-ones runs,
    widths that switch the window size (1, 3, 4, 5)."""
    n = keys["rsa2048_seed3"]["n"] if "rsa2048_seed3" in keys else keys["rsa1024_committed"]["n"]
    rng = random.Random(9)
    xs = [rng.randrange(n) for _ in range(70)] + [0, 1, n - 1]
    exps = [2, 3, 7, 8, 2**24 - 1, 2**25, 2**80 + 1, (2**81 - 1) ^ (1 << 40), 2**240 - 1, 2**241 + 2**3,
            rng.getrandbits(700) | 1, rng.getrandbits(3072), 2**3000]
    for e in exps:
        assert eng.modexp_batch(n, e, xs) == [pow(x, e, n) for x in xs], hex(e)[:20]
