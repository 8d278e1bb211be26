"""Resident store: the proxy's view of its stored sets kept on the GPU across requests.

The reference re-fetches every stored set on every aggregation request (``storedKeys.map(fetchSet)``,
``src/main/scala/dds/http/DDSRestServer.scala:401-403``) and folds / filters them on one core. Here
the proxy keeps one resident column per aggregated position instead — the Paillier column of SumAll,
the RSA column of MultAll, the OPE column of Search / Order — and updates it on each successful write
route, so every read route is one GPU call over rows already in HBM:

  PutSet      (:170-205)  a new key appends a row; known contents rewrite their key's row
  AddElement  (:220-255)  the set grows: the row's element at a position may appear, its guard class
                          may change (``length-1 > position`` is strict for SumAll/MultAll/Search)
  WriteElement(:281-321)  the element at a position changes (or the set grows)
  RemoveSet   (:207-218)  the set becomes None: the row leaves every fold, Search and Order

A row stands for one stored key. Per ciphertext column the row is LIVE when the route's loop would
fold it: the set is present, passes the strict guard, parses as an integer, and is the first row of
its content (SumAll/MultAll collapse equal sets: ``Future.sequence`` over a Set, ``:401-403``). The
C-ABI keeps the live mask on the device (``dds_col_set_live``) and folds only live rows; row values
change by ``dds_col_write_rows_dec``. The OPE column carries each row's class (lacks the position /
last element / elements follow) and a live flag (set present), ``dds_opecol_write_rows_dec`` /
``dds_opecol_set_live``. The string table (``dds_strtab``) holds every row's contents for the
deterministic-equality scans (SearchEq/NEq :607-681, SearchEntry/OR/AND :831-938, IsElement
:322-353): a write gives the row new contents (``dds_strtab_write_rows``), RemoveSet clears its live
byte (``dds_strtab_set_live``). Requests the resident columns cannot answer bit for bit (another
modulus than the column's, the plain add / multiply branch without ``nsqr`` / ``pubkey``, a position
without a column) go through ``ddshe.routes`` over the mirrored rows, which is the same batched engine
path the route would take without a resident column.
"""
from __future__ import annotations

import hashlib

import numpy as np

from . import DDSError, Engine, OPE_CLS_INNER, OPE_CLS_LACKS, OPE_CLS_LAST, StrTable
from . import NotFound as _EngineNotFound
from . import routes
from .routes import NotFound, ServerError, _dec_text, _value_key, entry_needle
from .x509 import rsa_modulus


def _elem_str(v) -> str:
    # toString of an AnyJsonFormat element (DDSJsonProtocol.scala:22-28)
    if v is None:
        return "None"
    if isinstance(v, bool):
        return "true" if v else "false"
    return str(v)


def key_from_set(contents) -> str:
    """Utils.getKeyFromSet (Utils.scala:15-18, SHA-512 per dds-system.conf:99): upper-case hex digest of
    ``DDSSet(contents).toString`` = ``DDSSet(List(e1, e2, ...))``."""
    text = "DDSSet(List(" + ", ".join(_elem_str(v) for v in contents) + "))"
    return hashlib.sha512(text.encode("utf-8")).hexdigest().upper()


def _bigint(v):
    """new BigInteger(v.toString) (any Unicode decimal digits, optional sign), or None if it throws."""
    s = _dec_text(v)
    body = s[1:] if s[:1] in "+-" else s
    if not body or not body.isascii() or not body.isdigit():
        return None
    x = int(body)
    return -x if s[:1] == "-" else x


class _CipherColumn:
    """One resident Paillier (SumAll) or RSA (MultAll) column at `position` under `modulus`."""

    def __init__(self, eng: Engine, position: int, modulus: int, capacity: int):
        self.position, self.modulus = position, int(modulus)
        self.col = eng.column(self.modulus, capacity)
        # limb capacity of the resident format: wider operands are stored reduced (the fold's result
        # is the same; a one-operand reply is answered from the host's copy)
        self.cap_bits = self.modulus.bit_length() + 2
        self.live = np.zeros(capacity, dtype=bool)  # per row: folds it (the engine's live mask)
        self.nlive = 0
        self.bad = set()    # rows that qualify but do not parse: the route answers 500

    def mark(self, r, live: bool, bad: bool):
        self.nlive += int(live) - int(self.live[r])
        self.live[r] = live
        (self.bad.add if bad else self.bad.discard)(r)

    def encode(self, value) -> tuple[str, bool]:
        """(engine text, parses) of an element"""
        x = _bigint(value)
        if x is None:
            return "1", False
        if x.bit_length() >= self.cap_bits:
            x %= self.modulus
        return str(x), True


class ResidentStore:
    """Host mirror of the proxy's stored sets with resident GPU columns (see the module docstring).

    paillier: {position: n^2} — SumAll columns (the client's ``nsqr``, DDSHttpClient.scala:228-240)
    rsa:      {position: n}   — MultAll columns (the modulus of the client's ``pubkey``)
    ope:      positions of OPE columns (Search{Gt,GtEq,Lt,LtEq}, OrderLS/OrderSL)
    strings:  keep a resident string table (SearchEq/NEq, SearchEntry/OR/AND, IsElement)
    Keys are derived as the reference derives them (SHA-512 of the set's text); the mirror's row order
    is insertion order.
    """

    def __init__(self, eng: Engine, paillier=None, rsa=None, ope=(), capacity: int = 1 << 16, strings: bool = True):
        self.eng, self.capacity = eng, capacity
        self.keys: list[str] = []
        self.row: dict[str, int] = {}
        self.val: list = []
        self.groups: dict[tuple, list[int]] = {}  # content signature -> rows holding it (ascending)
        self.cols = [_CipherColumn(eng, p, m, capacity) for p, m in (paillier or {}).items()]
        self.cols += [_CipherColumn(eng, p, m, capacity) for p, m in (rsa or {}).items()]
        self.by_pos_sum = {c.position: c for c in self.cols[:len(paillier or {})]}
        self.by_pos_mult = {c.position: c for c in self.cols[len(paillier or {}):]}
        self.ope = {p: eng.opecol(capacity) for p in ope}
        self.tab = StrTable(eng, []) if strings else None

    def close(self):
        for c in self.cols:
            c.col.close()
        for oc in self.ope.values():
            oc.close()
        if self.tab is not None:
            self.tab.close()

    # ---- row state ----
    @staticmethod
    def _sig(contents):
        return None if contents is None else tuple(_value_key(v) for v in contents)

    def _canonical(self, r) -> bool:
        s = self._sig(self.val[r])
        return s is not None and self.groups[s][0] == r

    def _cipher_state(self, c: _CipherColumn, r):
        """(engine text, live, bad) of row r in column c"""
        row = self.val[r]
        if row is None or len(row) <= c.position:
            return "1", False, False
        text, ok = c.encode(row[c.position])
        qualifies = len(row) - 1 > c.position and self._canonical(r)  # DDSRestServer.scala:415 / :509
        return text, qualifies and ok, qualifies and not ok

    def _ope_state(self, p, r):
        """(text, class, is_string, live) of row r in the OPE column at p"""
        row = self.val[r]
        if row is None:
            return None, OPE_CLS_LACKS, 0, False
        last = len(row) - 1
        cls = OPE_CLS_INNER if last > p else OPE_CLS_LAST if last == p else OPE_CLS_LACKS
        if cls == OPE_CLS_LACKS:
            return None, cls, 0, True
        v = row[p]
        return _dec_text(v), cls, 1 if isinstance(v, str) else 0, True

    def _regroup(self, r, old, new):
        """move row r between content groups; rows whose canonical status may have changed"""
        touched = {r}
        so, sn = self._sig(old), self._sig(new)
        if so == sn:
            return touched
        if so is not None:
            g = self.groups[so]
            if g[0] == r and len(g) > 1:
                touched.add(g[1])
            g.remove(r)
            if not g:
                del self.groups[so]
        if sn is not None:
            g = self.groups.setdefault(sn, [])
            if g and r < g[0]:
                touched.add(g[0])
            g.append(r)
            g.sort()
        return touched

    def _apply(self, rows):
        """push the current state of `rows` (existing rows) into every resident column"""
        rows = sorted(rows)
        ids = np.asarray(rows, dtype=np.uint64)
        for c in self.cols:
            st = [self._cipher_state(c, r) for r in rows]
            c.col.write_rows_dec(ids, [t for t, _, _ in st])
            c.col.set_live(ids, [1 if lv else 0 for _, lv, _ in st])
            for r, (_, lv, bad) in zip(rows, st):
                c.mark(r, lv, bad)
        for p, oc in self.ope.items():
            st = [self._ope_state(p, r) for r in rows]
            oc.write_rows_dec(ids, [t for t, _, _, _ in st], [k for _, k, _, _ in st], [s for _, _, s, _ in st])
            oc.set_live(ids, [1 if lv else 0 for _, _, _, lv in st])

    def _append(self, keys, contents):
        """new rows for new keys (one batched append per column); a failed append leaves the store and
        every column as they were"""
        r0 = len(self.keys)
        if r0 + len(keys) > self.capacity:
            raise ServerError("resident store capacity exceeded")
        for k, cont in zip(keys, contents):
            self.row[k] = len(self.keys)
            self.keys.append(k)
            self.val.append(None if cont is None else list(cont))
        touched = set()
        for i, cont in enumerate(contents):
            touched |= self._regroup(r0 + i, None, self.val[r0 + i])
        new = range(r0, r0 + len(keys))
        try:
            for c in self.cols:
                st = [self._cipher_state(c, r) for r in new]
                c.col.append_dec([t for t, _, _ in st])
                for r, (_, lv, bad) in zip(new, st):
                    c.mark(r, lv, bad)
                dead = [r for r, (_, lv, _) in zip(new, st) if not lv]
                if dead:
                    c.col.set_live(np.asarray(dead, dtype=np.uint64), 0)
            for p, oc in self.ope.items():
                st = [self._ope_state(p, r) for r in new]
                oc.append_dec([t for t, _, _, _ in st], [k for _, k, _, _ in st], [s for _, _, s, _ in st])
                dead = [r for r, (_, _, _, lv) in zip(new, st) if not lv]
                if dead:
                    oc.set_live(np.asarray(dead, dtype=np.uint64), 0)
            if self.tab is not None:
                self.tab.append([self.val[r] or [] for r in new])
                dead = [r for r in new if self.val[r] is None]
                if dead:
                    self.tab.set_live(np.asarray(dead, dtype=np.uint64), 0)
        except Exception:
            self._rollback(r0)
            raise
        old = touched - set(new)  # (a new row never displaces an earlier group member; kept general)
        if old:
            self._apply(old)

    def _rollback(self, r0):
        """drop rows r0.. from the mirror and from every device column (an append that raised)"""
        for r in range(len(self.keys) - 1, r0 - 1, -1):
            s = self._sig(self.val[r])
            if s is not None:
                g = self.groups[s]
                g.remove(r)
                if not g:
                    del self.groups[s]
            del self.row[self.keys[r]]
            for c in self.cols:
                if r < len(c.live):
                    c.mark(r, False, False)
        del self.keys[r0:]
        del self.val[r0:]
        for c in self.cols:
            c.col.truncate(r0)
        for oc in self.ope.values():
            oc.truncate(r0)
        if self.tab is not None:
            self.tab.truncate(r0)

    def _set(self, r, contents):
        old = self.val[r]
        self.val[r] = None if contents is None else list(contents)
        self._apply(self._regroup(r, old, self.val[r]))
        if self.tab is not None:
            ids = np.asarray([r], dtype=np.uint64)
            if self.val[r] is None:
                self.tab.set_live(ids, 0)  # RemoveSet: the register holds None
            else:
                self.tab.write_rows(ids, [self.val[r]])

    # ---- write routes ----
    def put_sets(self, sets) -> list[str]:
        """POST /PutSet for each set (DDSRestServer.scala:170-188); new keys are appended in one batch."""
        keys = [key_from_set(s) for s in sets]
        fresh, seen = [], {}
        for k, s in zip(keys, sets):
            if k in self.row:
                self._set(self.row[k], s)
            elif k in seen:
                fresh[seen[k]] = (k, s)
            else:
                seen[k] = len(fresh)
                fresh.append((k, s))
        if fresh:
            self._append([k for k, _ in fresh], [s for _, s in fresh])
        return keys

    def put_set(self, contents) -> str:
        return self.put_sets([contents])[0]

    def put_empty(self, key: str) -> str:
        """POST /PutSet without a body (:190-205): the key (random in the reference) holds None."""
        if key in self.row:
            self._set(self.row[key], None)
        else:
            self._append([key], [None])
        return key

    def remove_set(self, key: str):
        """DELETE /RemoveSet/{key} (:207-218)"""
        if key in self.row and self.val[self.row[key]] is not None:
            self._set(self.row[key], None)

    def add_element(self, key: str, value):
        """PUT /AddElement/{key} (:220-255): 404 for a missing / removed set"""
        r = self.row.get(key)
        if r is None or self.val[r] is None:
            raise NotFound()
        self._set(r, self.val[r] + [value])

    def write_element(self, key: str, position: int, value):
        """PUT /WriteElement/{key}?position (:281-321): replace, or append past the end; 404 for a
        missing / removed set, 500 for a negative position (IndexOutOfBoundsException)"""
        r = self.row.get(key)
        if r is None or self.val[r] is None:
            raise NotFound()
        cur = self.val[r]
        if position > len(cur) - 1:
            self._set(r, cur + [value])
        elif position < 0:
            raise ServerError("IndexOutOfBoundsException")
        else:
            nxt = list(cur)
            nxt[position] = value
            self._set(r, nxt)

    # ---- read routes ----
    def rows(self):
        return list(self.val)

    def keyed_rows(self):
        return list(zip(self.keys, self.val))

    def _fold(self, c: _CipherColumn, modulus_text, modulus_of):
        """the resident fold of column c: 404 / 500 / one-operand reply / GPU fold of the live rows.
        modulus_of(text) parses the request's modulus (raising ServerError), only when >= 2 rows
        qualify, as the route does (:422, :515-517)."""
        if c.bad:
            raise ServerError("NumberFormatException: a qualifying element is not an integer")
        n = c.nlive
        if n == 0:
            raise NotFound()
        if n == 1:  # the first operand, unreduced (:416-417 / :510-511), no modulus parse
            r = int(np.flatnonzero(c.live)[0])
            return str(_bigint(self.val[r][c.position]))
        if modulus_text is None or modulus_of(modulus_text) != c.modulus:
            return None  # not this column's modulus: the caller takes the per-request path
        try:
            return c.col.fold_dec()
        except _EngineNotFound as e:
            raise NotFound() from e
        except DDSError as e:
            raise ServerError(str(e)) from e

    def sum_all(self, position: int, nsqr: str | None = None) -> str:
        """GET /SumAll?position&nsqr (DDSRestServer.scala:397-446)"""
        c = self.by_pos_sum.get(position)
        if c is not None and nsqr is not None:
            def parse(t):
                x = _bigint(t)
                if x is None:
                    raise ServerError("NumberFormatException: nsqr")
                return x
            got = self._fold(c, nsqr, parse)
            if got is not None:
                return got
        return routes.sum_all(self.eng, self.rows(), position, nsqr)

    def mult_all(self, position: int, pubkey: str | None = None) -> str:
        """GET /MultAll?position&pubkey (DDSRestServer.scala:491-539)"""
        c = self.by_pos_mult.get(position)
        if c is not None and pubkey is not None:
            def parse(t):
                try:
                    return rsa_modulus(t)
                except ValueError as e:
                    raise ServerError(f"InvalidKeySpecException: {e}") from e
            got = self._fold(c, pubkey, parse)
            if got is not None:
                return got
        return routes.mult_all(self.eng, self.rows(), position, pubkey=pubkey)

    def search(self, route: str, position: int, value) -> list[str]:
        """POST /Search{Gt,GtEq,Lt,LtEq}?position (:682-830): matching keys in row order (the
        reference's order is unspecified). The match set comes back as a row bitmask."""
        oc = self.ope.get(position)
        if oc is None:
            return routes.search(self.eng, route, self.keyed_rows(), position, value)
        try:
            words, _ = oc.search_mask(_dec_text(value), routes._ROUTE_OP[route])
        except DDSError as e:
            raise ServerError(str(e)) from e
        bits = np.unpackbits(words.view(np.uint8), bitorder="little")[: len(self.keys)]
        return [self.keys[i] for i in np.flatnonzero(bits)]

    def order(self, route: str, position: int) -> list[str]:
        """GET /OrderLS|/OrderSL?position (:541-606)"""
        if route not in ("OrderLS", "OrderSL"):
            raise ValueError(route)
        oc = self.ope.get(position)
        if oc is None:
            return routes.order(self.eng, route, self.keyed_rows(), position)
        try:
            idx = oc.order(route == "OrderLS")
        except DDSError as e:
            raise ServerError(str(e)) from e
        return [self.keys[i] for i in idx]

    def search_eq(self, route: str, position: int, value) -> list[str]:
        """POST /SearchEq|/SearchNEq?position (:607-681): keys in row order (the reference's order is
        unspecified)"""
        if route not in ("SearchEq", "SearchNEq"):
            raise ValueError(route)
        if self.tab is None:
            return routes.search_eq(self.eng, route, self.keyed_rows(), position, value)
        try:
            idx = self.tab.search_eq(position, value, route == "SearchNEq")
        except DDSError as e:
            raise ServerError(str(e)) from e
        return [self.keys[i] for i in idx]

    def search_entry(self, route: str, values) -> list[str]:
        """POST /SearchEntry (one value, compared as ``DDSItem(value)``, :845) | /SearchEntryOR |
        /SearchEntryAND (three, :831-938)"""
        if route not in ("SearchEntry", "SearchEntryOR", "SearchEntryAND"):
            raise ValueError(route)
        if self.tab is None:
            return routes.search_entry(self.eng, route, self.keyed_rows(), values)
        needles = [entry_needle(values[0])] if route == "SearchEntry" else list(values)
        try:
            idx = self.tab.search_entry(needles, route == "SearchEntryAND")
        except DDSError as e:
            raise ServerError(str(e)) from e
        return [self.keys[i] for i in idx]

    def is_element(self, key: str, value) -> bool:
        """POST /IsElement/{key} (:322-353): 404 for an unknown key or a removed set"""
        r = self.row.get(key)
        if r is None or self.val[r] is None:
            raise NotFound()
        if self.tab is None:
            return routes.is_element(self.eng, self.val[r], value)
        try:
            return self.tab.is_element(r, value)
        except _EngineNotFound as e:
            raise NotFound() from e
        except DDSError as e:
            raise ServerError(str(e)) from e
