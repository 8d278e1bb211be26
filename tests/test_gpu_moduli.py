"""Every modulus a route can receive (DDSRestServer.scala:422 sends any nsqr, :515-517 any X.509
modulus): even moduli and 1 (BigInteger.mod semantics, CRT split of the engine), and moduli wider than
round 1's 6262-bit limit — the 8192-bit n^2 of a 4096-bit Paillier key and RSA moduli up to the JDK's
16384 bits. Checked against Python ints (the oracle)."""
import random

import pytest

from oracle import homo

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M", [2, 4, 1 << 64, (1 << 100) * 3, (1 << 4000) * 7, 10 ** 40, (2 ** 4095) - 2,
                               6 * ((1 << 2047) + 9), 1])
def test_fold_even_and_unit_moduli(eng, M):
    rng = random.Random(M.bit_length())
    for k in (2, 3, 257):
        xs = [rng.randrange(max(2, M)) for _ in range(k)]
        assert eng.modmul_fold(M, xs) == homo.modmul_fold(xs, M), (M.bit_length(), k)
    xs = [M + 5, 3 * M + 7, rng.getrandbits(M.bit_length() + 40)]    # operands above the modulus
    assert eng.modmul_fold(M, xs) == homo.modmul_fold(xs, M)


def test_decimal_routes_even_modulus(eng):
    M = (1 << 300) * 3 * 5
    vals = ["-12345", "+777", "0000042", str(M * 9 + 99), "-" + str(M + 1)]
    want = 1
    for v in vals:
        want = want * int(v)
    assert eng.sum_all_dec(vals, str(M)) == str(want % M)
    assert eng.mult_all_dec(vals, str(M)) == str(want % M)
    assert eng.sum_all_dec(vals, "1") == "0"
    assert eng.sum_all_dec(["-5"], "4") == "-5"                      # one operand: unreduced


@pytest.mark.parametrize("bits", [6263, 7000, 8190, 8192, 8194, 10000, 16384, 17000])
def test_fold_wide_moduli(eng, bits):
    rng = random.Random(bits)
    N = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
    for k in (2, 3, 300):
        xs = [rng.randrange(N) for _ in range(k)]
        assert eng.modmul_fold(N, xs) == homo.modmul_fold(xs, N), (bits, k)
    xs = [N - 1 - rng.randrange(3) for _ in range(5000)]
    assert eng.modmul_fold(N, xs) == homo.modmul_fold(xs, N), bits


def test_paillier_4096_key_fold_and_encrypt(eng):
    """An 8192-bit n^2: encrypt (public key) + SumAll fold + decrypt on a seeded 4096-bit key."""
    key = homo.gen_paillier_key(4096, seed=12)
    rng = random.Random(13)
    ms = [rng.randrange(10000) for _ in range(24)]
    rs = [rng.randrange(1, key["n"]) for _ in ms]
    cs = eng.paillier_encrypt_batch(key["n"], key["g"], ms, rs)
    assert cs[:3] == [homo.paillier_encrypt(m, r, key) for m, r in zip(ms[:3], rs[:3])]
    s = eng.paillier_sum(key["nsquare"], cs)
    assert s == homo.modmul_fold(cs, key["nsquare"])
    assert homo.paillier_decrypt(s, key) == sum(ms) % key["n"]


def test_wide_modulus_pairs_and_column(eng):
    rng = random.Random(99)
    N = rng.getrandbits(16000) | (1 << 15999) | 1
    a = [rng.randrange(N) for _ in range(40)]
    b = [rng.randrange(N) for _ in range(40)]
    assert eng.modmul_pairs(N, a, b) == [x * y % N for x, y in zip(a, b)]
    col = eng.column(N, 100)
    col.append(a + b)
    assert col.fold() == homo.modmul_fold(a + b, N)
    assert col.fold_rows([3, 50, 79]) == a[3] * b[10] * b[39] % N
    col.close()
