"""The reduction tree's hand-off modes: the default in-kernel hand-off (measured-valid
sc1 form, DDSHE_TREE_FENCE=2) and its two fallbacks, agent-scope release/acquire fences
(DDSHE_TREE_FENCE=0) and one level per launch (DDSHE_TREE_LEVELS=1), must give the same SumAll
results (DDSRestServer.scala:412-430). The modes are read once per process, so each runs in its own
child process (one at a time) over the same synthetic rows; every fold is checked by Dec = sum of the
plaintexts and against the default mode's bytes."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys
sys.path[:0] = [os.environ["DDS_ROOT"], os.path.join(os.environ["DDS_ROOT"], "dependable-data-storage-csd2017_amd")]
import ddshe
from tests.conftest import _load_keys
from oracle import homo
k = _load_keys()["paillier2048_committed"]
eng = ddshe.Engine(0)
rows = 20_001
col = eng.column(k["nsquare"], rows)
col.fill_paillier_synth(k["n"], k["g"], seed=13, row0=0, count=rows, pool=64)
ms = ddshe.synth_plaintexts(13, 0, rows)
out = {}
for count in (3, 513, 2049, 4097, 20_001):
    v = col.fold(0, count)
    assert homo.paillier_decrypt(v, k) == int(ms[:count].sum()) % k["n"], count
    for _ in range(4):
        assert col.fold(0, count) == v, count
    out[count] = str(v)
col.close()
eng.close()
print("RESULT " + json.dumps(out))
"""


def _run(env_extra):
    env = dict(os.environ, DDS_ROOT=ROOT, **env_extra)
    p = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, (env_extra, p.stdout[-2000:], p.stderr[-2000:])
    line = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")][-1]
    return json.loads(line[len("RESULT "):])


def test_tree_fallback_modes_agree():
    base = _run({})
    assert _run({"DDSHE_TREE_FENCE": "0"}) == base
    assert _run({"DDSHE_TREE_LEVELS": "1"}) == base
