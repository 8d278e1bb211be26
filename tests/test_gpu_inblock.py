"""Fold sizes around the switch from the tail launches to the reduction tree (level 1 with more than the
tree's 4096 leaves' worth of lane groups: 4160 / 4480 groups, the full group count with two rows per
group, the strong-split share size). SumAll (DDSRestServer.scala:412-430) must stay bit-exact against the
oracle's fold, or Dec(fold) = Σm on synthetic Paillier rows under the committed key, and the device-partial
path must equal the fold. tools/gpurun/inblock_ab.sh also runs this file with DDSHE_FOLD_INBLOCK=1 (level
1 folding each block's partials through LDS, k_fold InBlock: an A/B option, slower, off by default)."""
import random

import numpy as np
import pytest

from oracle import homo

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("k", [8_320, 9_001, 65_539])
def test_inblock_fold_vs_oracle(eng, keys, k):
    key = keys["paillier2048_committed"]
    N = key["nsquare"]
    rng = random.Random(k)
    xs = [rng.randrange(N) for _ in range(k)]
    col = eng.column(N, k)
    col.append(xs)
    try:
        assert col.fold() == homo.modmul_fold(xs, N)
        assert col.fold(17, k - 17 - 5) == homo.modmul_fold(xs[17:k - 5], N)
    finally:
        col.close()


@pytest.mark.parametrize("rows", [300_007, 1_250_000])
def test_inblock_fold_decrypts_and_partial_matches(eng, keys, rows):
    import torch
    key = keys["paillier2048_committed"]
    N = key["nsquare"]
    import ddshe
    col = eng.column(N, rows)
    col.fill_paillier_synth(key["n"], key["g"], 2, 0, rows, 1024)
    try:
        got = col.fold()
        ms = ddshe.synth_plaintexts(2, 0, rows)
        assert homo.paillier_decrypt(got, key) == int(ms.astype(np.int64).sum()) % key["n"]
        # the device partial of the same rows (dds_col_fold_partial_device) combined alone = the fold
        part = torch.empty(col.partial_words, dtype=torch.int32, device="cuda")
        col.fold_partial_device(part.data_ptr(), 0, rows)
        torch.cuda.synchronize()
        assert eng.combine_partials_device(N, part.data_ptr(), [rows]) == got
    finally:
        col.close()
