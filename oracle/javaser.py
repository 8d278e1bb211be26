"""Decoder for the key material committed in the reference's ``client.conf``.

TEST INFRASTRUCTURE ONLY (oracle/): used to produce ``tests/golden/keys.json``.
Nothing on the product path imports this module.

The reference stores its homomorphic keys as base64 Java-serialized objects
(``/root/reference/src/main/resources/client.conf:81-88``) and deserializes them
with hlib's ``keyFromString`` (``src/main/scala/utils/SJHomoLibProvider.scala:43-50``).
This module is a *data-only* parser of the Java Object Serialization Stream
grammar (magic 0xACED, TC_OBJECT / TC_CLASSDESC / TC_REFERENCE / TC_STRING /
TC_ARRAY / TC_ENUM / TC_BLOCKDATA): it never executes anything from the stream.
BigInteger fields are rebuilt from their ``signum`` + big-endian ``magnitude``;
RSA keys inside ``java.security.KeyRep`` are decoded from their X.509 /
PKCS#8 DER encodings.
"""
from __future__ import annotations

import base64
import re
import struct

TC_NULL, TC_REFERENCE, TC_CLASSDESC, TC_OBJECT, TC_STRING = 0x70, 0x71, 0x72, 0x73, 0x74
TC_ARRAY, TC_CLASS, TC_BLOCKDATA, TC_ENDBLOCKDATA, TC_RESET = 0x75, 0x76, 0x77, 0x78, 0x79
TC_BLOCKDATALONG, TC_LONGSTRING, TC_ENUM = 0x7A, 0x7C, 0x7E
BASE_HANDLE = 0x7E0000
SC_WRITE_METHOD, SC_SERIALIZABLE = 0x01, 0x02


class _ClassDesc:
    def __init__(self, name, flags, fields, parent):
        self.name, self.flags, self.fields, self.parent = name, flags, fields, parent


class _Obj:
    def __init__(self, cls):
        self.cls = cls
        self.fields = {}
        self.annotations = []

    def __repr__(self):
        return f"<{self.cls.name} {sorted(self.fields)}>"


class JavaStream:
    def __init__(self, data: bytes):
        self.d = data
        self.i = 0
        self.handles = []
        if self._u16() != 0xACED or self._u16() != 5:
            raise ValueError("not a Java serialization stream")

    # primitive readers -------------------------------------------------
    def _take(self, n):
        if self.i + n > len(self.d):
            raise ValueError("truncated stream")
        b = self.d[self.i:self.i + n]
        self.i += n
        return b

    def _u8(self):
        return self._take(1)[0]

    def _u16(self):
        return struct.unpack(">H", self._take(2))[0]

    def _i32(self):
        return struct.unpack(">i", self._take(4))[0]

    def _utf(self):
        return self._take(self._u16()).decode("utf-8", "replace")

    def _new_handle(self, obj):
        self.handles.append(obj)
        return len(self.handles) - 1

    # grammar -------------------------------------------------------------
    def read(self):
        tc = self._u8()
        return self._content(tc)

    def _content(self, tc):
        if tc == TC_NULL:
            return None
        if tc == TC_REFERENCE:
            return self.handles[self._i32() - BASE_HANDLE]
        if tc == TC_STRING:
            s = self._utf()
            self._new_handle(s)
            return s
        if tc == TC_LONGSTRING:
            n = struct.unpack(">q", self._take(8))[0]
            s = self._take(n).decode("utf-8", "replace")
            self._new_handle(s)
            return s
        if tc == TC_CLASSDESC:
            return self._classdesc_body()
        if tc == TC_OBJECT:
            return self._object()
        if tc == TC_ARRAY:
            return self._array()
        if tc == TC_ENUM:
            cls = self._classdesc()
            h = self._new_handle(None)
            name = self.read()
            self.handles[h] = (cls.name, name)
            return (cls.name, name)
        if tc == TC_BLOCKDATA:
            return self._take(self._u8())
        if tc == TC_BLOCKDATALONG:
            return self._take(self._i32())
        raise ValueError(f"unsupported type code 0x{tc:02x} at {self.i - 1}")

    def _classdesc(self):
        tc = self._u8()
        if tc == TC_NULL:
            return None
        if tc == TC_REFERENCE:
            return self.handles[self._i32() - BASE_HANDLE]
        if tc != TC_CLASSDESC:
            raise ValueError(f"expected class desc, got 0x{tc:02x}")
        return self._classdesc_body()

    def _classdesc_body(self):
        name = self._utf()
        self._take(8)  # serialVersionUID
        h = self._new_handle(None)
        flags = self._u8()
        fields = []
        for _ in range(self._u16()):
            code = chr(self._u8())
            fname = self._utf()
            if code in "L[":
                self.read()  # class name string (or reference)
            fields.append((code, fname))
        # classAnnotation
        while True:
            tc = self._u8()
            if tc == TC_ENDBLOCKDATA:
                break
            self._content(tc)
        parent = self._classdesc()
        cd = _ClassDesc(name, flags, fields, parent)
        self.handles[h] = cd
        return cd

    def _value(self, code):
        if code == "B":
            return struct.unpack(">b", self._take(1))[0]
        if code == "C":
            return self._u16()
        if code == "D":
            return struct.unpack(">d", self._take(8))[0]
        if code == "F":
            return struct.unpack(">f", self._take(4))[0]
        if code == "I":
            return self._i32()
        if code == "J":
            return struct.unpack(">q", self._take(8))[0]
        if code == "S":
            return struct.unpack(">h", self._take(2))[0]
        if code == "Z":
            return self._u8() != 0
        return self.read()

    def _object(self):
        cls = self._classdesc()
        obj = _Obj(cls)
        self._new_handle(obj)
        chain = []
        c = cls
        while c is not None:
            chain.append(c)
            c = c.parent
        for c in reversed(chain):  # superclass data first
            for code, fname in c.fields:
                obj.fields[fname] = self._value(code)
            if c.flags & SC_WRITE_METHOD:
                while True:
                    tc = self._u8()
                    if tc == TC_ENDBLOCKDATA:
                        break
                    obj.annotations.append(self._content(tc))
        return obj

    def _array(self):
        cls = self._classdesc()
        h = self._new_handle(None)
        n = self._i32()
        code = cls.name[1]
        if code == "B":
            arr = self._take(n)
        else:
            arr = [self._value(code) for _ in range(n)]
        self.handles[h] = arr
        return arr


def bigint_from_obj(o: _Obj) -> int:
    """java.math.BigInteger from its serialized (signum, magnitude) fields."""
    mag = int.from_bytes(bytes(o.fields["magnitude"]), "big")
    return -mag if o.fields["signum"] < 0 else mag


# DER --------------------------------------------------------------------
def _der(buf, i=0):
    tag = buf[i]
    ln = buf[i + 1]
    i += 2
    if ln & 0x80:
        nb = ln & 0x7F
        ln = int.from_bytes(buf[i:i + nb], "big")
        i += nb
    return tag, buf[i:i + ln], i + ln


def _der_seq(buf):
    out, i = [], 0
    while i < len(buf):
        tag, val, i = _der(buf, i)
        out.append((tag, val))
    return out


def rsa_public_from_x509(der: bytes):
    _, spki, _ = _der(der)
    items = _der_seq(spki)
    bitstr = items[1][1][1:]  # skip unused-bits byte
    _, rsakey, _ = _der(bitstr)
    n, e = [int.from_bytes(v, "big") for _, v in _der_seq(rsakey)]
    return n, e


def rsa_private_from_pkcs8(der: bytes):
    _, pk, _ = _der(der)
    items = _der_seq(pk)
    _, rsakey, _ = _der(items[2][1])
    vals = [int.from_bytes(v, "big") for _, v in _der_seq(rsakey)]
    keys = ["version", "n", "e", "d", "p", "q", "dp", "dq", "qinv"]
    return dict(zip(keys, vals))


def decode_client_conf(text: str) -> dict:
    """Decode OPE / PSSE (Paillier) / MSE (RSA) keys from client.conf text
    (reference ``src/main/resources/client.conf:81-88``)."""
    def blob(name):
        m = re.search(r"\b" + name + r"\s*=\s*\"([^\"]+)\"", text)
        return base64.b64decode(m.group(1))

    out = {}
    ope = JavaStream(blob("OPE")).read()
    out["ope_key"] = ope.fields["value"]

    pk = JavaStream(blob("PSSE")).read()
    assert pk.cls.name == "hlib.hj.mlib.PaillierKey", pk.cls.name
    out["paillier"] = {k: bigint_from_obj(v) for k, v in pk.fields.items()}

    kp = JavaStream(blob("MSE")).read()
    priv, pub = kp.fields["privateKey"], kp.fields["publicKey"]
    n, e = rsa_public_from_x509(bytes(pub.fields["encoded"]))
    prv = rsa_private_from_pkcs8(bytes(priv.fields["encoded"]))
    assert prv["n"] == n and prv["e"] == e
    out["rsa"] = {"n": n, "e": e, "d": prv["d"], "p": prv["p"], "q": prv["q"],
                  "x509_hex": bytes(pub.fields["encoded"]).hex()}
    return out
