"""CPU restatement (Python ints) of the reference's homomorphic aggregation path.

TEST INFRASTRUCTURE ONLY — the checker, never the product. Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
anything under ``oracle/``.

Parity status: the arithmetic lives in hlib (``hlib.hj.mlib``, a proprietary jar
that is ABSENT from the reference: ``/root/reference/lib/README.txt:1``; version
unknown/unpinned) and the reference has no tests, fixtures or golden vectors
(SURVEY.md §4, §8c). There is no JVM in this image, so the reference cannot be
run. This oracle is pinned instead by
  (1) the committed key material (``client.conf:85-86``), which satisfies the
      standard Paillier / RSA identities checked in ``tests/test_oracle.py``;
  (2) the published algorithms hlib implements (Paillier 1999, textbook RSA), with
      ``HomoAdd.sum(c1,c2,nsq) = c1·c2 mod nsq`` and
      ``HomoMult.multiply(c1,c2,pk) = c1·c2 mod n`` as the assumed definitions;
  (3) the route semantics of ``DDSRestServer.scala`` restated line by line below;
  (4) an independent cross-check against OpenSSL ``BN_mod_mul`` (tests).
It is therefore "partially pinned": no reference-produced output exists.
"""
from __future__ import annotations

import math
import random

# ---------------------------------------------------------------------------
# hlib primitives (absent jar; call sites cited)
# ---------------------------------------------------------------------------


def homo_add_sum(c1: int, c2: int, nsquare: int) -> int:
    """``HomoAdd.sum(c1, c2, nsquare)`` — Paillier homomorphic addition.
    Call sites: ``DDSRestServer.scala:385`` (Sum) and ``:423`` (SumAll)."""
    return (c1 * c2) % nsquare


def homo_mult_multiply(c1: int, c2: int, n: int) -> int:
    """``HomoMult.multiply(c1, c2, RSAPublicKey)`` — RSA multiplicative homomorphism.
    Call sites: ``DDSRestServer.scala:479`` (Mult) and ``:518`` (MultAll)."""
    return (c1 * c2) % n


def paillier_encrypt(m: int, r: int, key: dict) -> int:
    """``HomoAdd.encrypt(BigInteger m, PaillierKey)`` (``SJHomoLibProvider.scala:58``):
    c = g^m · r^n mod n² with caller-supplied r (hlib draws r at random)."""
    n, nsq = key["n"], key["nsquare"]
    return (pow(key["g"], m, nsq) * pow(r, n, nsq)) % nsq


def paillier_decrypt(c: int, key: dict) -> int:
    """``HomoAdd.decrypt`` (``SJHomoLibProvider.scala:68``): m = L(c^λ mod n²)·μ mod n."""
    n, nsq = key["n"], key["nsquare"]
    u = pow(c, key["lambda"], nsq)
    return ((u - 1) // n) * key["mu"] % n


def rsa_encrypt(m: int, key: dict) -> int:
    """``HomoMult.encrypt(pk, m)`` (``SJHomoLibProvider.scala:59``): textbook RSA."""
    return pow(m, key["e"], key["n"])


def rsa_decrypt(c: int, key: dict) -> int:
    """``HomoMult.decrypt(sk, c)`` (``SJHomoLibProvider.scala:69``)."""
    return pow(c, key["d"], key["n"])


# ---------------------------------------------------------------------------
# Route semantics (DDSRestServer.scala)
# ---------------------------------------------------------------------------


class NotFound(Exception):
    """HTTP 404 from a route (``complete(StatusCodes.NotFound)``)."""


class ServerError(Exception):
    """HTTP 500 from a route (``case Failure(ex) => InternalServerError``)."""


def java_biginteger(s) -> int:
    """``new BigInteger(String)`` (radix 10): an optional '+' or '-', then one or more digits,
    each mapped by ``Character.digit(c, 10)`` — any Unicode decimal digit (category Nd), not only
    ASCII; nothing else (no blanks, no '_'). Anything else is a NumberFormatException (→ 500)."""
    s = str(s)
    body = s[1:] if s[:1] in "+-" else s
    if not body or not body.isdecimal():
        raise ServerError(f"NumberFormatException: {s!r}")
    v = int(body)
    return -v if s[:1] == "-" else v


def java_mod(x: int, m: int) -> int:
    """``BigInteger.mod(m)``: the non-negative residue; ``ArithmeticException`` (→ 500) for m <= 0."""
    if m <= 0:
        raise ServerError("ArithmeticException: BigInteger: modulus not positive")
    return x % m


def value_key(v):
    """Equality of one ``DDSSet.contents`` element as Scala sees it: values of different runtime
    types never compare equal (``AnyJsonFormat`` reads JSON numbers as Int, strings as String,
    booleans as Boolean, null as None — ``DDSJsonProtocol.scala:22-28``), so Int 5 != String "5" and
    true != 1 (Python's ``True == 1`` must not merge them)."""
    if v is None:
        return ("None",)
    if isinstance(v, bool):
        return ("Boolean", v)
    if isinstance(v, int):
        return ("Int", v)
    return ("String", str(v))


def dedup_rows(rows):
    """``storedKeys.map(fetchSet)`` + ``Future.sequence`` over a Set collapses equal
    DDSSets (``DDSRestServer.scala:401-403``; case-class equality of ``contents: List[Any]``,
    element by element with its runtime type, ``DDSSet.scala:3``) and ``filter(nonEmpty)`` drops
    missing ones (``:408``). Rows are lists of column values; None = missing."""
    seen, out = set(), []
    for r in rows:
        if r is None:
            continue
        key = tuple(value_key(v) for v in r)
        if key in seen:
            continue
        seen.add(key)
        out.append(r)
    return out


def sum_all(rows, position: int, nsqr=None) -> str:
    """``GET /SumAll?position&nsqr`` — ``DDSRestServer.scala:397-446``.
    Strict guard ``contents.length-1 > position`` (``:415``); first operand is
    taken unreduced (``:416-417``); each later one is folded with HomoAdd.sum
    (``:422-423``) or plain ``add`` when nsqr is absent (``:425``). ``nsqr`` is parsed only
    inside that later-operand branch (``:422``), i.e. never when one operand qualifies."""
    rows = dedup_rows(rows)
    if not rows:
        raise NotFound()
    acc = None
    for r in rows:
        if len(r) - 1 > position:
            x = java_biginteger(r[position])
            if acc is None:
                acc = x
            elif nsqr is not None:
                acc = homo_add_sum_checked(acc, x, java_biginteger(nsqr))
            else:
                acc = acc + x
    if acc is None:
        raise NotFound()
    return str(acc)


def rsa_modulus_from_pubkey_hex(pubkey: str) -> int:
    """``KeyFactory.getInstance("RSA").generatePublic(new X509EncodedKeySpec(
    DatatypeConverter.parseHexBinary(pubkey)))`` (``DDSRestServer.scala:476-478,515-517``) → its
    modulus. parseHexBinary needs an even number of hex digits; the DER must be an X.509
    SubjectPublicKeyInfo of rsaEncryption; the JDK's RSA key factory (``RSAKeyFactory.
    checkRSAProviderKeyLengths``, JDK 8 source; unpinned against a running JVM) rounds the modulus
    length up to a multiple of 8 and refuses it outside [512, 16384] bits, and refuses exponents wider
    than 64 bits for moduli above 3072 bits. Failures → 500."""
    h = str(pubkey)
    if len(h) % 2 or any(c not in "0123456789abcdefABCDEF" for c in h):
        raise ServerError("IllegalArgumentException: parseHexBinary")
    der = bytes.fromhex(h)

    def tlv(buf, i):  # (tag, value, next) with the declared length fully present
        if i + 2 > len(buf):
            raise ServerError("InvalidKeySpecException: truncated DER")
        tag, ln, i = buf[i], buf[i + 1], i + 2
        if ln & 0x80:
            nb = ln & 0x7F
            ln, i = int.from_bytes(buf[i:i + nb], "big"), i + nb
        if i + ln > len(buf):
            raise ServerError("InvalidKeySpecException: truncated DER")
        return tag, buf[i:i + ln], i + ln

    tag, spki, end = tlv(der, 0)
    if tag != 0x30 or end != len(der):
        raise ServerError("InvalidKeySpecException: not one SubjectPublicKeyInfo")
    tag, alg, i = tlv(spki, 0)
    tag2, oid, _ = tlv(alg, 0)
    if tag != 0x30 or tag2 != 0x06 or oid != bytes.fromhex("2a864886f70d010101"):
        raise ServerError("InvalidKeySpecException: not rsaEncryption")
    tag, bits, i = tlv(spki, i)
    if tag != 0x03 or i != len(spki) or bits[:1] != b"\0":
        raise ServerError("InvalidKeySpecException: bad subjectPublicKey")
    tag, key, j = tlv(bits, 1)
    if tag != 0x30 or j != len(bits):
        raise ServerError("InvalidKeySpecException: bad RSAPublicKey")
    tag, nb, j = tlv(key, 0)
    tag2, eb, j = tlv(key, j)
    if tag != 0x02 or tag2 != 0x02 or j != len(key):
        raise ServerError("InvalidKeySpecException: bad RSAPublicKey")
    n = int.from_bytes(nb, "big", signed=True)
    e = int.from_bytes(eb, "big", signed=True)
    mlen = (n.bit_length() + 7) // 8 * 8
    if n <= 0 or not 512 <= mlen <= 16384:
        raise ServerError("InvalidKeyException: RSA modulus length")
    if mlen > 3072 and e.bit_length() > 64:
        raise ServerError("InvalidKeyException: RSA exponent length")
    return n


def mult_all(rows, position: int, n=None, pubkey=None) -> str:
    """``GET /MultAll?position&pubkey`` — ``DDSRestServer.scala:491-539``.
    ``pubkey`` is the hex X.509 key, decoded only inside the later-operand branch (``:515-517``);
    ``n`` may be given instead (its modulus, already decoded). Neither = plain product (``:520``)."""
    rows = dedup_rows(rows)
    if not rows:
        raise NotFound()
    acc = None
    for r in rows:
        if len(r) - 1 > position:
            x = java_biginteger(r[position])
            if acc is None:
                acc = x
            elif pubkey is not None:
                acc = homo_mult_multiply(acc, x, rsa_modulus_from_pubkey_hex(pubkey))
            elif n is not None:
                acc = homo_mult_multiply(acc, x, n)
            else:
                acc = acc * x
    if acc is None:
        raise NotFound()
    return str(acc)


def homo_add_sum_checked(c1: int, c2: int, nsquare: int) -> int:
    """HomoAdd.sum with BigInteger.mod's exception on a non-positive modulus (→ 500)."""
    return java_mod(c1 * c2, nsquare)


def pair_sum(set1, set2, position: int, nsqr=None) -> str:
    """``GET /Sum?key1&key2&position&nsqr`` — ``DDSRestServer.scala:355-395``
    (guard ``length-1 < position`` → 404 at ``:376``; no dedup: two keys, two operands)."""
    if set1 is None or set2 is None:
        raise NotFound()
    if len(set1) - 1 < position or len(set2) - 1 < position:
        raise NotFound()
    a, b = java_biginteger(set1[position]), java_biginteger(set2[position])
    if nsqr is not None:
        return str(homo_add_sum_checked(a, b, java_biginteger(nsqr)))
    return str(a + b)


def pair_mult(set1, set2, position: int, n=None, pubkey=None) -> str:
    """``GET /Mult?key1&key2&position&pubkey`` — ``DDSRestServer.scala:447-490``."""
    if set1 is None or set2 is None:
        raise NotFound()
    if len(set1) - 1 < position or len(set2) - 1 < position:
        raise NotFound()
    a, b = java_biginteger(set1[position]), java_biginteger(set2[position])
    if pubkey is not None:
        return str(homo_mult_multiply(a, b, rsa_modulus_from_pubkey_hex(pubkey)))
    if n is not None:
        return str(homo_mult_multiply(a, b, n))
    return str(a * b)


OPS = {
    # route -> predicate on (col, item); DDSRestServer.scala compares
    # item.compareTo(col) {<0, <=0, >0, >=0}
    "SearchGt": lambda col, item: item < col,     # :704
    "SearchGtEq": lambda col, item: item <= col,  # :742
    "SearchLt": lambda col, item: item > col,     # :779
    "SearchLtEq": lambda col, item: item >= col,  # :816
}


def search(route: str, keyed_rows, position: int, value) -> set:
    """``POST /Search{Gt,GtEq,Lt,LtEq}?position`` — ``DDSRestServer.scala:682-830``.
    ``keyed_rows`` = list of (key, row). Returns the matching key SET (the
    reference prepends into a list, so order is unspecified: ``:705``). The bound is parsed with
    ``new BigInteger(item.value.toString)`` inside the per-row condition, after the strict guard
    (``:702-704``): only when some row qualifies. Both sides are arbitrary-size BigIntegers."""
    pred = OPS[route]
    out = set()
    seen = set()
    for key, row in keyed_rows:
        if row is None or key in seen:
            continue
        seen.add(key)
        if len(row) - 1 > position:
            item = java_biginteger(value)
            if pred(java_biginteger(row[position]), item):
                out.add(key)
    return out


def java_long(s) -> int:
    """``contents(position).asInstanceOf[String].toLong`` (``DDSRestServer.scala:562,595``): the
    element must be a String (an Int element is a ClassCastException), then
    ``java.lang.Long.parseLong``: optional sign, ``Character.digit`` decimal digits, int64 range.
    Failures → 500."""
    if not isinstance(s, str):
        raise ServerError(f"ClassCastException: {type(s).__name__} is not a String")
    body = s[1:] if s[:1] in "+-" else s
    if not body or not body.isdecimal():
        raise ServerError(f"NumberFormatException: {s!r}")
    v = int(body)
    v = -v if s[:1] == "-" else v
    if not -(1 << 63) <= v < (1 << 63):
        raise ServerError(f"NumberFormatException: {s!r} (out of Long range)")
    return v


def order(route: str, keyed_rows, position: int) -> list:
    """``GET /OrderLS|/OrderSL?position`` — ``DDSRestServer.scala:541-606``.
    Keys of the non-empty rows (``:553``, ``:586``) sorted with the route's comparator
    (``:555-563``, ``:588-596``): a row holds the position iff ``length-1 >= position``;
    OrderLS puts holders first, by ``contents(position).toLong`` descending; OrderSL puts the
    others first, then holders ascending. ``sortWith`` is stable, so equal keys keep the input
    order. (OrderSL's comparator is not strict between two non-holders — ``lt`` is true both
    ways — so the JVM's order among them is an artefact of TimSort; unpinned, kept stable here.)
    The comparator parses only when both operands hold the position, and a sort compares every
    pair of holders that end up adjacent: with two or more holders every holder's element is
    parsed (one bad element → 500); a lone holder is never parsed."""
    rows = [(k, r) for k, r in keyed_rows if r is not None]
    holders = [(k, r) for k, r in rows if len(r) - 1 >= position]
    if len(holders) >= 2:
        hold = [(k, java_long(r[position])) for k, r in holders]
    else:
        hold = [(k, 0) for k, _ in holders]
    rest = [k for k, r in rows if len(r) - 1 < position]
    if route == "OrderLS":
        return [k for k, _ in sorted(hold, key=lambda kv: -kv[1])] + rest
    if route == "OrderSL":
        return rest + [k for k, _ in sorted(hold, key=lambda kv: kv[1])]
    raise ValueError(route)


# Deterministic-equality scans. hlib's HomoDet.compare(a, b) is absent (lib/README.txt:1); a
# deterministic scheme compares ciphertexts by equality, so compare(a, b) := a == b on the
# strings (unpinned beyond that assumption).
def homo_det_compare(a, b) -> bool:
    """HomoDet.compare(a.toString, b.toString) as string equality (both sides as AnyJsonFormat reads
    them, ``DDSJsonProtocol.scala:22-28``)."""
    return element_to_string(a) == element_to_string(b)


def entry_needle(value) -> str:
    """The text SearchEntry compares (``DDSRestServer.scala:845``): ``item.toString`` of the DDSItem case
    class (``DDSJsonProtocol.scala:7``), i.e. ``DDSItem(<value>)`` -- not ``item.value.toString`` as
    SearchEntryOR/AND (``:881-883``, ``:918-920``) and IsElement (``:338``) use."""
    return "DDSItem(" + element_to_string(value) + ")"


def search_eq(route: str, keyed_rows, position: int, value) -> set:
    """``POST /SearchEq|/SearchNEq?position`` — ``DDSRestServer.scala:607-681``: keys of the
    non-empty rows with ``length-1 > position`` (strict, ``:629``) whose ``contents(position)``
    does (Eq) / does not (NEq, ``:667``) compare equal to the item. Key set (prepended list)."""
    out = set()
    for key, row in keyed_rows:
        if row is None or not len(row) - 1 > position:
            continue
        eq = homo_det_compare(row[position], value)
        if eq == (route == "SearchEq"):
            out.add(key)
    return out


def search_entry(route: str, keyed_rows, values) -> set:
    """``POST /SearchEntry`` (one value), ``/SearchEntryOR`` and ``/SearchEntryAND`` (three) —
    ``DDSRestServer.scala:831-938``: a row qualifies when some element equals the value (Entry),
    any of the three (OR, ``:881-883``), or when the set of its elements equal to one of the three
    reaches size 3 (AND, ``:918-927``: all three present and pairwise distinct). SearchEntry's single
    value is compared as ``item.toString`` (``entry_needle``). The per-row ``break``
    (``:851,886,926``) is read as "stop scanning this row" (literally it throws Breaks'
    BreakControl outside any ``breakable``)."""
    if route == "SearchEntry":
        values = [entry_needle(values[0])]
    else:
        values = [element_to_string(v) for v in values]
    out = set()
    for key, row in keyed_rows:
        if row is None:
            continue
        if route == "SearchEntryAND":
            found = {element_to_string(e) for e in row if element_to_string(e) in values}
            if len(found) == 3:
                out.add(key)
        elif any(element_to_string(e) in values for e in row):
            out.add(key)
    return out


def is_element(row, value) -> bool:
    """``POST /IsElement/{key}`` — ``DDSRestServer.scala:322-353``: some element of the row
    compares equal; a missing row is 404 (``:348``)."""
    if row is None:
        raise NotFound()
    return any(homo_det_compare(e, value) for e in row)


# ---------------------------------------------------------------------------
# The store the routes read: storedKeys + the replicated registers (write routes)
# ---------------------------------------------------------------------------


def element_to_string(v) -> str:
    """``toString`` of a contents element as ``AnyJsonFormat`` reads it (``DDSJsonProtocol.scala:22-28``):
    String as is, Int in decimal, Boolean ``true``/``false``, JsNull -> ``None``."""
    if v is None:
        return "None"
    if isinstance(v, bool):
        return "true" if v else "false"
    return str(v)


def set_to_string(contents) -> str:
    """``DDSSet(contents: List[Any]).toString`` (case class around a List, ``DDSSet.scala:3``)."""
    return "DDSSet(List(" + ", ".join(element_to_string(v) for v in contents) + "))"


def key_from_set(contents) -> str:
    """``Utils.getKeyFromSet(set, "SHA-512")`` (``Utils.scala:15-18``, digest from
    ``dds-system.conf:99``): upper-case hex of SHA-512 over ``set.toString.getBytes`` (UTF-8)."""
    import hashlib
    return hashlib.sha512(set_to_string(contents).encode("utf-8")).hexdigest().upper()


class Store:
    """The proxy's ``storedKeys`` (``DDSRestServer.scala:70``) and the value of each key's replicated
    register, as the write routes leave them (the BFT-ABD write/read pair is assumed to succeed: it
    returns the last value written, ``BFTABDNode.scala:103-363``). ``keyed_rows()`` is what the read
    routes fetch (``storedKeys.map(fetchSet)``, ``:401-403``). Key order = insertion order (the
    reference iterates an immutable HashSet: its order is unpinned; it matters only for Order's ties)."""

    def __init__(self):
        self.keys = []
        self.val = {}

    def _store(self, key):
        if key not in self.val:
            self.keys.append(key)

    def put_set(self, contents) -> str:
        """``POST /PutSet`` with a body (``:170-188``): key = SHA-512 of the set's text; the register is
        (re)written, ``storedKeys += key``."""
        key = key_from_set(contents)
        self._store(key)
        self.val[key] = list(contents)
        return key

    def put_empty(self, key: str) -> str:
        """``POST /PutSet`` without a body (``:190-205``): a random key holding None (the key is the
        caller's here, the reference draws it from SecureRandom)."""
        self._store(key)
        self.val[key] = None
        return key

    def remove_set(self, key: str):
        """``DELETE /RemoveSet/{key}`` (``:207-218``): writes None; the key stays in storedKeys, and every
        read route drops it (``filter(nonEmpty)``). 200 for any key."""
        if key in self.val:
            self.val[key] = None

    def add_element(self, key: str, value):
        """``PUT /AddElement/{key}`` (``:220-255``): append the item; 404 when the set is None."""
        cur = self.val.get(key)
        if cur is None:
            raise NotFound()
        self.val[key] = cur + [value]

    def write_element(self, key: str, position: int, value):
        """``PUT /WriteElement/{key}?position`` (``:281-321``): replace ``contents(position)``, or append
        when ``position > size-1``; 404 when the set is None. A negative position throws
        IndexOutOfBoundsException inside the callback (500) and writes nothing."""
        cur = self.val.get(key)
        if cur is None:
            raise NotFound()
        if position > len(cur) - 1:
            self.val[key] = cur + [value]
        elif position < 0:
            raise ServerError("IndexOutOfBoundsException")
        else:
            nxt = list(cur)
            nxt[position] = value
            self.val[key] = nxt

    def rows(self):
        return [self.val[k] for k in self.keys]

    def keyed_rows(self):
        return [(k, self.val[k]) for k in self.keys]


# ---------------------------------------------------------------------------
# Fold primitives used by the tests at sizes beyond route-level vectors
# ---------------------------------------------------------------------------


def modmul_fold(xs, N: int) -> int:
    """SumAll/MultAll fold over k≥1 operands: x0 unreduced when k == 1, else ∏ mod N."""
    if not xs:
        raise NotFound()
    if len(xs) == 1:
        return xs[0]
    acc = xs[0]
    for x in xs[1:]:
        acc = (acc * x) % N
    return acc


def ope_filter(col, valid, bound: int, op: str):
    """Indices i with valid[i] and col[i] <op> bound (ascending)."""
    f = {"gt": lambda c: c > bound, "ge": lambda c: c >= bound,
         "lt": lambda c: c < bound, "le": lambda c: c <= bound}[op]
    return [i for i, (c, v) in enumerate(zip(col, valid)) if v and f(int(c))]


# ---------------------------------------------------------------------------
# Synthetic keys (deterministic, seeded)
# ---------------------------------------------------------------------------

_SMALL_PRIMES = [p for p in range(3, 2000, 2) if all(p % q for q in range(3, int(p ** 0.5) + 1, 2))]


def is_probable_prime(n: int, rng: random.Random, rounds: int = 40) -> bool:
    if n < 2:
        return False
    for p in _SMALL_PRIMES:
        if n % p == 0:
            return n == p
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for _ in range(rounds):
        a = rng.randrange(2, n - 1)
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def gen_prime(bits: int, rng: random.Random) -> int:
    while True:
        c = rng.getrandbits(bits) | (1 << (bits - 1)) | (1 << (bits - 2)) | 1
        if is_probable_prime(c, rng):
            return c


def gen_paillier_key(bits: int, seed: int) -> dict:
    """Paillier key with an n of exactly ``bits`` bits and a random g ∈ Z*_{n²}
    (like the committed key, whose g is random: SURVEY.md F6)."""
    rng = random.Random(seed)
    while True:
        p = gen_prime(bits // 2, rng)
        q = gen_prime(bits // 2, rng)
        n = p * q
        if p != q and n.bit_length() == bits and math.gcd(n, (p - 1) * (q - 1)) == 1:
            break
    nsq = n * n
    lam = (p - 1) * (q - 1) // math.gcd(p - 1, q - 1)
    while True:
        g = rng.randrange(2, nsq)
        if math.gcd(g, n) != 1:
            continue
        L = (pow(g, lam, nsq) - 1) // n
        if math.gcd(L, n) == 1:
            mu = pow(L, -1, n)
            break
    return {"g": g, "lambda": lam, "mu": mu, "n": n, "nsquare": nsq, "p": p, "q": q}


def gen_rsa_key(bits: int, seed: int, e: int = 65537) -> dict:
    rng = random.Random(seed)
    while True:
        p = gen_prime(bits // 2, rng)
        q = gen_prime(bits // 2, rng)
        n = p * q
        phi = (p - 1) * (q - 1)
        if p != q and n.bit_length() == bits and math.gcd(e, phi) == 1:
            return {"n": n, "e": e, "d": pow(e, -1, phi), "p": p, "q": q}
