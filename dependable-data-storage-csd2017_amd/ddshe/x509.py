"""The RSA modulus of the ``pubkey`` parameter of /Mult and /MultAll.

The route decodes it per use with ``KeyFactory.getInstance("RSA").generatePublic(new
X509EncodedKeySpec(DatatypeConverter.parseHexBinary(pubkey)))`` (``DDSRestServer.scala:476-478,
515-517``). This restates what that JDK chain accepts: an even-length hex string, a DER
SubjectPublicKeyInfo { AlgorithmIdentifier { rsaEncryption, NULL }, BIT STRING { RSAPublicKey {
modulus, publicExponent } } } with exact lengths and no trailing bytes, and the JDK RSA key factory's
length check (``RSAKeyFactory.checkRSAProviderKeyLengths``, called by the RSAPublicKeyImpl constructor):
the modulus length rounded up to a multiple of 8 must be 512 to 16384 bits, and a modulus above 3072
bits may not carry an exponent wider than 64 bits. Anything else raises :class:`ValueError`, which the
routes answer with 500 as the reference does. (No JVM here: the check is restated from the JDK 8
source, and the fixtures cover its edges; parity with a particular JDK build is unpinned.)
"""
from __future__ import annotations

_RSA_OID = bytes.fromhex("2a864886f70d010101")  # 1.2.840.113549.1.1.1
_HEX = set("0123456789abcdefABCDEF")


def _tlv(buf: bytes, i: int, tag: int):
    if i + 2 > len(buf) or buf[i] != tag:
        raise ValueError("DER: unexpected tag")
    ln, i = buf[i + 1], i + 2
    if ln & 0x80:
        nb = ln & 0x7F
        if nb == 0 or nb > 4 or i + nb > len(buf) or buf[i] == 0:
            raise ValueError("DER: bad length")
        ln, i = int.from_bytes(buf[i:i + nb], "big"), i + nb
        if ln < 0x80:
            raise ValueError("DER: non-minimal length")
    if i + ln > len(buf):
        raise ValueError("DER: truncated")
    return buf[i:i + ln], i + ln


def _integer(buf: bytes, i: int):
    v, i = _tlv(buf, i, 0x02)
    if not v or (len(v) > 1 and v[0] == 0 and v[1] < 0x80):
        raise ValueError("DER: bad INTEGER")
    return int.from_bytes(v, "big", signed=True), i


def rsa_modulus(pubkey_hex: str) -> int:
    h = str(pubkey_hex)
    if len(h) % 2 or not set(h) <= _HEX:
        raise ValueError("parseHexBinary: not an even-length hex string")
    der = bytes.fromhex(h)
    spki, end = _tlv(der, 0, 0x30)
    if end != len(der):
        raise ValueError("DER: trailing bytes")
    alg, i = _tlv(spki, 0, 0x30)
    oid, j = _tlv(alg, 0, 0x06)
    if oid != _RSA_OID:
        raise ValueError("not an RSA key")
    if j < len(alg):
        _, j = _tlv(alg, j, 0x05)
        if j != len(alg):
            raise ValueError("DER: bad AlgorithmIdentifier")
    bits, i = _tlv(spki, i, 0x03)
    if i != len(spki) or not bits or bits[0] != 0:
        raise ValueError("DER: bad BIT STRING")
    key, k = _tlv(bits, 1, 0x30)
    if k != len(bits):
        raise ValueError("DER: trailing bytes in BIT STRING")
    n, k = _integer(key, 0)
    e, k = _integer(key, k)
    if k != len(key) or n <= 0 or e <= 0:
        raise ValueError("DER: bad RSAPublicKey")
    check_key_lengths(n, e)
    return n


def check_key_lengths(n: int, e: int):
    """RSAKeyFactory.checkRSAProviderKeyLengths(n.bitLength(), e)"""
    mlen = (n.bit_length() + 7) & ~7
    if mlen < 512:
        raise ValueError("RSA keys must be at least 512 bits long")
    if mlen > 16384:
        raise ValueError("RSA keys must be no longer than 16384 bits")
    if mlen > 3072 and e.bit_length() > 64:
        raise ValueError("RSA exponents can be no more than 64 bits if modulus is greater than 3072 bits")
