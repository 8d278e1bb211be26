"""GPU parity of the deterministic-equality scans (SearchEq/NEq, SearchEntry/OR/AND, IsElement;
DDSRestServer.scala:322-353, 607-681, 831-938) against the route restatements in oracle/homo.py.
HomoDet.compare is taken as string equality (hlib absent: unpinned beyond that assumption)."""
import random

import numpy as np
import pytest

from oracle import homo

pytestmark = pytest.mark.gpu


def make_rows(n, seed, vocab=40):
    rng = random.Random(seed)
    words = [format(rng.getrandbits(64), "x") for _ in range(vocab)] + ["", "0", "00", "-7", "7"]
    rows = []
    for i in range(n):
        length = rng.randrange(0, 9)
        rows.append([rng.choice(words) for _ in range(length)])
    return rows, words


@pytest.mark.parametrize("n", [1, 5, 300, 5000])
def test_search_eq_routes(eng, n):
    from ddshe import routes
    rows, words = make_rows(n, n)
    keyed = [(f"k{i}", r if i % 17 else None) for i, r in enumerate(rows)]
    rng = random.Random(1)
    for _ in range(6):
        value = rng.choice(words)
        for position in (0, 2, 7, 9):
            for route in ("SearchEq", "SearchNEq"):
                got = routes.search_eq(eng, route, keyed, position, value)
                assert set(got) == homo.search_eq(route, keyed, position, value), (route, position, value)
                assert len(got) == len(set(got))


@pytest.mark.parametrize("n", [1, 300, 5000])
def test_search_entry_routes(eng, n):
    from ddshe import routes
    rows, words = make_rows(n, n + 1, vocab=12)
    keyed = [(f"k{i}", r if i % 13 else None) for i, r in enumerate(rows)]
    rng = random.Random(2)
    for _ in range(8):
        v = [rng.choice(words) for _ in range(3)]
        assert set(routes.search_entry(eng, "SearchEntry", keyed, v[:1])) == homo.search_entry("SearchEntry", keyed, v[:1])
        for route in ("SearchEntryOR", "SearchEntryAND"):
            assert set(routes.search_entry(eng, route, keyed, v)) == homo.search_entry(route, keyed, v), (route, v)
    # duplicated values can never reach three distinct matches
    w = words[0]
    assert routes.search_entry(eng, "SearchEntryAND", keyed, [w, w, words[1]]) == []


def test_is_element(eng):
    from ddshe import routes
    rows, words = make_rows(50, 9)
    for r in rows:
        for v in words[:10] + [""]:
            assert routes.is_element(eng, r, v) == homo.is_element(r, v)
    with pytest.raises(routes.NotFound):
        routes.is_element(eng, None, "x")


def test_search_large_table(eng):
    """200k rows x up to 8 elements: row ids ascending, exact (digest hits are byte-verified)."""
    rng = np.random.default_rng(4)
    n = 200_000
    vocab = np.array([format(int(x), "032x") for x in rng.integers(0, 2**62, size=1000)])
    lens = rng.integers(1, 9, size=n)
    picks = rng.integers(0, len(vocab), size=int(lens.sum()))
    rows, p = [], 0
    for L in lens:
        rows.append(list(vocab[picks[p:p + L]]))
        p += L
    tab = eng.strtab(rows)
    target = vocab[7]
    want = np.array([i for i, r in enumerate(rows) if target in r], dtype=np.uint32)
    assert np.array_equal(tab.search_entry([target]), want)
    want_eq = np.array([i for i, r in enumerate(rows) if len(r) - 1 > 0 and r[0] == target], dtype=np.uint32)
    assert np.array_equal(tab.search_eq(0, target), want_eq)
    tab.close()


def test_search_eq_position_index_resident(eng):
    """SearchEq / NEq on a resident table read a position-major fingerprint index built on the first
    query at each position (at most 8 kept): 11 positions queried twice (evictions and rebuilds),
    rows shorter than the position (the strict guard length - 1 > position) never match."""
    rng = random.Random(21)
    words = [format(rng.getrandbits(40), "x") for _ in range(6)] + ["", "7"]
    rows = [[rng.choice(words) for _ in range(rng.randrange(0, 13))] for _ in range(20_003)]
    tab = eng.strtab(rows)
    for rep in range(2):
        for position in range(11):
            value = words[(position + rep) % len(words)]
            for negate in (False, True):
                want = np.array([i for i, r in enumerate(rows)
                                 if len(r) - 1 > position and (r[position] == value) != negate], dtype=np.uint32)
                assert np.array_equal(tab.search_eq(position, value, negate), want), (rep, position, negate)
    tab.close()
