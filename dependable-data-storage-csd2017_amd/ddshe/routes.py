"""Host-side mirror of the reference REST proxy routes whose fold/filter loops the
engine replaces (``src/main/scala/dds/http/DDSRestServer.scala``).

Each function takes what the route body holds after its ABD fetches — the fetched
rows (``DDSSet.contents`` lists, ``None`` for a missing set) — applies the route's
own guard/dedup logic exactly as the Scala code does, and hands the whole loop to
ONE batched C-ABI call. Errors follow the route: :class:`NotFound` is the 404
branch, :class:`ServerError` the 500 branch.

Element values are Python objects standing for what ``AnyJsonFormat`` reads
(``DDSJsonProtocol.scala:22-28``): ``str`` (JsString), ``int`` (JsNumber → Int), ``bool``,
``None`` (JsNull). A route that parses an element uses its ``toString``.

These functions take the fetched rows of ONE request, as the reference route does, and are the
parity form of each route: ``search`` / ``order`` / ``search_eq`` build a device table for the
request and free it afterwards. The serving form keeps the columns resident across requests and
follows the write routes: ``ddshe.store.ResidentStore``.
"""
from __future__ import annotations

from . import DDSError, Engine, element_text
from . import NotFound as _EngineNotFound
from . import OPE_CLS_INNER, OPE_CLS_LACKS, OPE_CLS_LAST
from .x509 import rsa_modulus


class NotFound(Exception):
    """complete(StatusCodes.NotFound)"""


class ServerError(Exception):
    """complete(StatusCodes.InternalServerError)"""


def _value_key(v):
    # Scala equality of a contents element: runtime type + value (Int 5 != String "5", true != 1)
    if v is None:
        return ("None",)
    if isinstance(v, bool):
        return ("Boolean", v)
    if isinstance(v, int):
        return ("Int", v)
    return ("String", str(v))


def _dedup(rows):
    # storedKeys.map(fetchSet) + Future.sequence over a Set collapses equal DDSSets
    # (DDSRestServer.scala:401-403; DDSSet(contents: List[Any]) case-class equality, DDSSet.scala:3);
    # filter(nonEmpty) drops missing ones (:408).
    seen, out = set(), []
    for r in rows:
        if r is None:
            continue
        key = tuple(_value_key(v) for v in r)
        if key not in seen:
            seen.add(key)
            out.append(r)
    return out


def _to_string(v) -> str:
    """``toString`` of a contents element, as the text the engine parses. Scala prints booleans in
    lower case and JsNull reads as ``None``; neither parses as an integer, like here."""
    if isinstance(v, bool):
        return "true" if v else "false"
    return str(v)


def _dec_text(v) -> str:
    """The element text for the engine's ASCII decimal parser. ``new BigInteger(String)`` and
    ``Long.parseLong`` map digits with ``Character.digit`` (any Unicode Nd digit); non-ASCII text
    that is such a number is rewritten as its ASCII decimal, anything else is passed through for the
    engine to reject."""
    s = _to_string(v)
    if s.isascii():
        return s
    body = s[1:] if s[:1] in "+-" else s
    if body and body.isdecimal():
        return ("-" if s[:1] == "-" else "") + str(int(body))
    return s


def _column(rows, position):
    # guard `contents.length-1 > position` (DDSRestServer.scala:415 / :509)
    return [_dec_text(r[position]) for r in rows if len(r) - 1 > position]


def _call(fn, *args):
    try:
        return fn(*args)
    except _EngineNotFound as e:
        raise NotFound() from e
    except DDSError as e:
        raise ServerError(str(e)) from e


def sum_all(eng: Engine, rows, position: int, nsqr: str | None = None) -> str:
    """GET /SumAll?position&nsqr — DDSRestServer.scala:397-446. nsqr is parsed only in the
    later-operand branch (:422): the engine ignores it when one operand qualifies."""
    rows = _dedup(rows)
    if not rows:
        raise NotFound()
    vals = _column(rows, position)
    if not vals:
        raise NotFound()
    return _call(eng.sum_all_dec, vals, None if nsqr is None else _dec_text(nsqr))


def _pubkey_modulus(pubkey: str) -> str:
    try:
        return str(rsa_modulus(pubkey))
    except ValueError as e:
        raise ServerError(f"InvalidKeySpecException: {e}") from e


def mult_all(eng: Engine, rows, position: int, n: str | None = None, pubkey: str | None = None) -> str:
    """GET /MultAll?position&pubkey — DDSRestServer.scala:491-539. ``pubkey`` (hex X.509) is decoded
    only in the later-operand branch (:515-517), i.e. when two or more operands qualify; ``n`` may
    be given instead (the modulus, already decoded). Neither: the plain product (:520)."""
    rows = _dedup(rows)
    if not rows:
        raise NotFound()
    vals = _column(rows, position)
    if not vals:
        raise NotFound()
    if pubkey is not None and len(vals) >= 2:
        n = _pubkey_modulus(pubkey)
    return _call(eng.mult_all_dec, vals, None if n is None else _dec_text(n))


def _pair(set1, set2, position):
    if set1 is None or set2 is None:
        raise NotFound()
    if len(set1) - 1 < position or len(set2) - 1 < position:  # :376 / :468 (not strict)
        raise NotFound()
    return [_dec_text(set1[position]), _dec_text(set2[position])]


def pair_sum(eng: Engine, set1, set2, position: int, nsqr: str | None = None) -> str:
    """GET /Sum?key1&key2&position&nsqr — DDSRestServer.scala:355-395 (HomoAdd.sum, :385).
    Two keys, two operands: no dedup (the same set twice is folded twice)."""
    vals = _pair(set1, set2, position)
    if nsqr is None:
        return _call(eng.sum_all_dec, vals, None)  # operand1.add(operand2) (:387)
    return _call(eng.pair_modmul_dec, vals[0], vals[1], _dec_text(nsqr))


def pair_mult(eng: Engine, set1, set2, position: int, n: str | None = None, pubkey: str | None = None) -> str:
    """GET /Mult?key1&key2&position&pubkey — DDSRestServer.scala:447-490 (HomoMult.multiply, :479)."""
    vals = _pair(set1, set2, position)
    if pubkey is not None:
        n = _pubkey_modulus(pubkey)
    if n is None:
        return _call(eng.mult_all_dec, vals, None)  # operand1.multiply(operand2)
    return _call(eng.pair_modmul_dec, vals[0], vals[1], _dec_text(n))


_ROUTE_OP = {"SearchGt": "gt", "SearchGtEq": "ge", "SearchLt": "lt", "SearchLtEq": "le"}


def _ope_rows(keyed_rows, position: int, dedup_keys: bool):
    """keys, element texts, row classes and String flags of the live rows for a dds_opecol."""
    keys, vals, cls, isstr, seen = [], [], [], [], set()
    for key, row in keyed_rows:
        if row is None or (dedup_keys and key in seen):
            continue
        seen.add(key)
        last = len(row) - 1
        c = OPE_CLS_INNER if last > position else OPE_CLS_LAST if last == position else OPE_CLS_LACKS
        keys.append(key)
        cls.append(c)
        if c == OPE_CLS_LACKS:
            vals.append(None)
            isstr.append(0)
        else:
            v = row[position]
            vals.append(_dec_text(v))
            isstr.append(1 if isinstance(v, str) else 0)
    return keys, vals, cls, isstr


def search(eng: Engine, route: str, keyed_rows, position: int, value) -> list:
    """POST /Search{Gt,GtEq,Lt,LtEq}?position — DDSRestServer.scala:682-830 over a resident OPE
    column (dds_opecol). The bound (``item.value.toString``) is parsed only when a row passes the
    strict guard (:702-704); rows and bound compare as BigIntegers (values outside Long included).
    Returns the matching keys in row order (the reference prepends, :705: order unspecified)."""
    op = _ROUTE_OP[route]
    keys, vals, cls, isstr = _ope_rows(keyed_rows, position, True)
    if not keys:
        return []
    col = eng.opecol(len(keys))
    try:
        _call(col.append_dec, vals, cls, isstr)
        idx = _call(col.search, _dec_text(value), op)
    finally:
        col.close()
    return [keys[i] for i in idx]


def order(eng: Engine, route: str, keyed_rows, position: int) -> list:
    """GET /OrderLS|/OrderSL?position — DDSRestServer.scala:541-606 over a resident OPE column: keys
    of the non-empty rows, holders of the position (length-1 >= position) by
    contents(position).asInstanceOf[String].toLong descending (OrderLS, others last) or ascending
    (OrderSL, others first); stable for ties. With two or more holders every holder is parsed (a
    non-String or non-Long holder → 500); a lone holder is never parsed."""
    if route not in ("OrderLS", "OrderSL"):
        raise ValueError(route)
    keys, vals, cls, isstr = _ope_rows(keyed_rows, position, False)
    if not keys:
        return []
    col = eng.opecol(len(keys))
    try:
        _call(col.append_dec, vals, cls, isstr)
        idx = _call(col.order, route == "OrderLS")
    finally:
        col.close()
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


def entry_needle(value) -> str:
    """SearchEntry compares ``item.toString`` (DDSRestServer.scala:845), the DDSItem case class's text
    ``DDSItem(<value>)`` (DDSJsonProtocol.scala:7); OR / AND / IsElement compare the values themselves."""
    return "DDSItem(" + element_text(value) + ")"


def search_entry(eng: Engine, route: str, keyed_rows, values) -> list:
    """POST /SearchEntry (one value) | /SearchEntryOR | /SearchEntryAND (three) —
    DDSRestServer.scala:831-938."""
    if route not in ("SearchEntry", "SearchEntryOR", "SearchEntryAND"):
        raise ValueError(route)
    keys, rows = _live(keyed_rows)
    if not keys:
        return []
    values = [entry_needle(values[0])] if route == "SearchEntry" else list(values)
    tab = eng.strtab(rows)
    try:
        idx = _call(tab.search_entry, values, route == "SearchEntryAND")
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
