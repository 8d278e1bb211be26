"""Host-side mirror of the reference REST proxy routes whose fold/filter loops the
engine replaces (``src/main/scala/dds/http/DDSRestServer.scala``).

Each function takes what the route body holds after its ABD fetches — the fetched
rows (``DDSSet.contents`` lists, ``None`` for a missing set) — applies the route's
own guard/dedup logic exactly as the Scala code does, and hands the whole loop to
ONE batched C-ABI call. Errors follow the route: :class:`NotFound` is the 404
branch, :class:`ServerError` the 500 branch.
"""
from __future__ import annotations

import numpy as np

from . import DDSError, Engine
from . import NotFound as _EngineNotFound

INT64_MIN, INT64_MAX = -(1 << 63), (1 << 63) - 1


class NotFound(Exception):
    """complete(StatusCodes.NotFound)"""


class ServerError(Exception):
    """complete(StatusCodes.InternalServerError)"""


def _dedup(rows):
    # storedKeys.map(fetchSet) + Future.sequence over a Set collapses equal DDSSets
    # (DDSRestServer.scala:401-403); filter(nonEmpty) drops missing ones (:408).
    seen, out = set(), []
    for r in rows:
        if r is None:
            continue
        key = tuple(str(v) for v in r)
        if key not in seen:
            seen.add(key)
            out.append(r)
    return out


def _column(rows, position):
    # guard `contents.length-1 > position` (DDSRestServer.scala:415 / :509)
    return [str(r[position]) for r in rows if len(r) - 1 > position]


def _call(fn, *args):
    try:
        return fn(*args)
    except _EngineNotFound as e:
        raise NotFound() from e
    except DDSError as e:
        raise ServerError(str(e)) from e


def sum_all(eng: Engine, rows, position: int, nsqr: str | None = None) -> str:
    """GET /SumAll?position&nsqr — DDSRestServer.scala:397-446."""
    rows = _dedup(rows)
    if not rows:
        raise NotFound()
    vals = _column(rows, position)
    if not vals:
        raise NotFound()
    return _call(eng.sum_all_dec, vals, nsqr)


def mult_all(eng: Engine, rows, position: int, n: str | None = None) -> str:
    """GET /MultAll?position&pubkey — DDSRestServer.scala:491-539. ``n`` is the
    modulus of the X.509 pubkey (decoded by the caller, :515-517)."""
    rows = _dedup(rows)
    if not rows:
        raise NotFound()
    vals = _column(rows, position)
    if not vals:
        raise NotFound()
    return _call(eng.mult_all_dec, vals, n)


def _pair(rows, position):
    set1, set2 = rows
    if set1 is None or set2 is None:
        raise NotFound()
    if len(set1) - 1 < position or len(set2) - 1 < position:  # :376 / :468
        raise NotFound()
    return [str(set1[position]), str(set2[position])]


def pair_sum(eng: Engine, set1, set2, position: int, nsqr: str | None = None) -> str:
    """GET /Sum?key1&key2&position&nsqr — DDSRestServer.scala:355-395 (HomoAdd.sum, :385)."""
    return _call(eng.sum_all_dec, _pair((set1, set2), position), nsqr)


def pair_mult(eng: Engine, set1, set2, position: int, n: str | None = None) -> str:
    """GET /Mult?key1&key2&position&pubkey — DDSRestServer.scala:447-490 (HomoMult.multiply, :479)."""
    return _call(eng.mult_all_dec, _pair((set1, set2), position), n)


_ROUTE_OP = {"SearchGt": "gt", "SearchGtEq": "ge", "SearchLt": "lt", "SearchLtEq": "le"}


def _parse_int(s) -> int:
    s = str(s)
    body = s[1:] if s[:1] in "+-" else s
    if not body or not body.isascii() or not body.isdigit():
        raise ServerError(f"NumberFormatException: {s!r}")
    return int(s)


def _clamp_bound(op: str, item: int):
    """Map a BigInteger bound outside int64 to an equivalent int64 predicate."""
    if INT64_MIN <= item <= INT64_MAX:
        return op, item
    if item > INT64_MAX:   # col > item / col >= item never; col < item / col <= item always
        return ("gt", INT64_MAX) if op in ("gt", "ge") else ("le", INT64_MAX)
    return ("ge", INT64_MIN) if op in ("gt", "ge") else ("lt", INT64_MIN)


def search(eng: Engine, route: str, keyed_rows, position: int, value) -> list:
    """POST /Search{Gt,GtEq,Lt,LtEq}?position — DDSRestServer.scala:682-830.
    Returns the matching keys (the reference's key order is unspecified: it
    prepends, :705; the engine returns them in row order)."""
    op = _ROUTE_OP[route]
    item = _parse_int(value)
    keys, col, valid, seen = [], [], [], set()
    for key, row in keyed_rows:
        if row is None or key in seen:
            continue
        seen.add(key)
        ok = len(row) - 1 > position
        v = _parse_int(row[position]) if ok else 0
        if ok and not (INT64_MIN <= v <= INT64_MAX):
            raise ServerError("OPE value outside int64 (OPE ciphertexts are Java Long)")
        keys.append(key)
        col.append(v)
        valid.append(1 if ok else 0)
    if not keys:
        return []
    op, bound = _clamp_bound(op, item)
    idx = _call(eng.ope_filter, np.array(col, dtype=np.int64), np.array(valid, dtype=np.uint8), bound, op)
    return [keys[i] for i in idx]


def order(eng: Engine, route: str, keyed_rows, position: int) -> list:
    """GET /OrderLS|/OrderSL?position — DDSRestServer.scala:541-606: keys of the non-empty
    rows, holders of the position (length-1 >= position) by contents(position).toLong
    descending (OrderLS, others last) or ascending (OrderSL, others first); stable for ties."""
    if route not in ("OrderLS", "OrderSL"):
        raise ValueError(route)
    keys, col, valid = [], [], []
    for key, row in keyed_rows:
        if row is None:
            continue
        ok = len(row) - 1 >= position
        v = _parse_int(row[position]) if ok else 0
        if ok and not (INT64_MIN <= v <= INT64_MAX):
            raise ServerError("NumberFormatException: value outside Long (String.toLong)")
        keys.append(key)
        col.append(v)
        valid.append(1 if ok else 0)
    if not keys:
        return []
    idx = _call(eng.ope_order, np.array(col, dtype=np.int64), np.array(valid, dtype=np.uint8), route == "OrderLS")
    return [keys[i] for i in idx]


def _live(keyed_rows):
    keys, rows, seen = [], [], set()
    for key, row in keyed_rows:
        if row is None or key in seen:
            continue
        seen.add(key)
        keys.append(key)
        rows.append(row)
    return keys, rows


def search_eq(eng: Engine, route: str, keyed_rows, position: int, value) -> list:
    """POST /SearchEq|/SearchNEq?position — DDSRestServer.scala:607-681 (HomoDet.compare as
    string equality). Keys in row order (the reference's prepend order is unspecified)."""
    if route not in ("SearchEq", "SearchNEq"):
        raise ValueError(route)
    keys, rows = _live(keyed_rows)
    if not keys:
        return []
    tab = eng.strtab(rows)
    try:
        idx = _call(tab.search_eq, position, value, route == "SearchNEq")
    finally:
        tab.close()
    return [keys[i] for i in idx]


def search_entry(eng: Engine, route: str, keyed_rows, values) -> list:
    """POST /SearchEntry (one value) | /SearchEntryOR | /SearchEntryAND (three) —
    DDSRestServer.scala:831-938."""
    if route not in ("SearchEntry", "SearchEntryOR", "SearchEntryAND"):
        raise ValueError(route)
    keys, rows = _live(keyed_rows)
    if not keys:
        return []
    tab = eng.strtab(rows)
    try:
        idx = _call(tab.search_entry, list(values), route == "SearchEntryAND")
    finally:
        tab.close()
    return [keys[i] for i in idx]


def is_element(eng: Engine, row, value) -> bool:
    """POST /IsElement/{key} — DDSRestServer.scala:322-353: 404 for a missing row."""
    if row is None:
        raise NotFound("no such key")
    tab = eng.strtab([row])
    try:
        return _call(tab.is_element, 0, value)
    finally:
        tab.close()
