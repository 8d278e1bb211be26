"""GPU parity of the one-bignum-per-lane fold (k_fold1: the narrow shapes S = 40 and 76, i.e. the
2048-bit RSA n of MultAll, DDSRestServer.scala:518, and the n² of a 1024-bit Paillier key, :423).

The library picks k_fold1 only for folds of >= ~1M rows; DDSHE_FOLD1_MIN=0 (read once per process)
forces it at every size, so these checks run in a child process with that setting and compare
against the oracle (homo.modmul_fold, Python ints) bit for bit, plus Dec(fold) = sum(m) at 2M rows
under the default threshold."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, random, sys
ROOT = os.environ["DDS_TEST_ROOT"]
sys.path[:0] = [ROOT, ROOT + "/dependable-data-storage-csd2017_amd"]
import numpy as np
import ddshe
from oracle import homo
keys = json.load(open(ROOT + "/tests/golden/keys.json"))
K = {k: {f: int(x, 16) for f, x in v.items() if f != "x509_hex"} for k, v in keys.items() if isinstance(v, dict)}
eng = ddshe.Engine(0)
res = {}
rng = random.Random(11)

def check(name, mod, rows, subsets=()):
    col = eng.column(mod, len(rows))
    col.append(rows)
    for count in sorted({2, 3, 63, 64, 65, 257, min(len(rows), 4099), len(rows)}):
        if count > len(rows):
            continue
        got = col.fold(0, count)
        res[f"{name}/{count}"] = got == homo.modmul_fold(rows[:count], mod)
    for i, ids in enumerate(subsets):
        res[f"{name}/rows{i}"] = col.fold_rows(ids) == homo.modmul_fold([rows[j] for j in ids], mod)
    col.close()

# 2048-bit RSA n (S = 76, QP modulus): random residues, and the worst case N - 1 everywhere
n = K["rsa2048_seed3"]["n"]
rows = [rng.randrange(n) for _ in range(30000)]
check("rsa2048", n, rows, subsets=[sorted(rng.sample(range(30000), 5000)), list(range(29999, -1, -7))])
check("rsa2048_nm1", n, [n - 1] * 5000)
# n^2 of a 1024-bit Paillier key (S = 76)
nsq = K["paillier1024_seed1"]["nsquare"]
check("paillier1024", nsq, [rng.randrange(nsq) for _ in range(20000)])
# 1024-bit RSA n (S = 40)
n1 = K["rsa1024_committed"]["n"]
check("rsa1024", n1, [rng.randrange(n1) for _ in range(20000)])
# moduli too wide for the QP modulus in their shape (plain CIOS quotient in k_fold1)
for bits, tag in ((2110, "s76_noqp"), (1100, "s40_noqp")):
    m = rng.getrandbits(bits) | (1 << (bits - 1)) | 1
    check(tag, m, [rng.randrange(m) for _ in range(6000)])
# all-ones modulus (every limb at its maximum)
m = (1 << 2047) - 1
check("ones2047", m, [m - 1 - rng.randrange(1000) for _ in range(3000)])
# Dec(fold) = sum(m) at 2M rows of synthetic Paillier ciphertexts
k = K["paillier1024_seed1"]
col = eng.column(k["nsquare"], 2_000_000)
col.fill_paillier_synth(k["n"], k["g"], seed=5, row0=0, count=2_000_000, pool=256)
s = col.fold()
res["dec2M"] = homo.paillier_decrypt(s, k) == int(ddshe.synth_plaintexts(5, 0, 2_000_000).astype(np.int64).sum()) % k["n"]
print(json.dumps(res))
"""


def _run(env_extra):
    env = dict(os.environ, DDS_TEST_ROOT=ROOT, **env_extra)
    p = subprocess.run([sys.executable, "-c", CHILD], capture_output=True, text=True, timeout=110, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


def test_fold1_forced_every_size():
    res = _run({"DDSHE_FOLD1_MIN": "0"})
    bad = [k for k, v in res.items() if not v]
    assert not bad, bad
    assert len(res) > 40


def test_fold1_off_matches_too():
    """The lane-group kernel on the same cases (DDSHE_FOLD1=0): both paths agree with the oracle."""
    res = _run({"DDSHE_FOLD1": "0"})
    bad = [k for k, v in res.items() if not v]
    assert not bad, bad


def test_fold1_76_limbs_qp():
    """k_fold1 at the column's own 76 limbs against N~ = N·n0 (DDSHE_FOLD1_74=0), every size."""
    res = _run({"DDSHE_FOLD1_MIN": "0", "DDSHE_FOLD1_74": "0"})
    bad = [k for k, v in res.items() if not v]
    assert not bad, bad
