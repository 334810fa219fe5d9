"""Reader of R's serialized data files (.rda / .RData, XDR format, version 2 or 3,
gzip / bzip2 / xz compressed) into plain Python values, and the fixture writer
for the tables the reference ships as data:

    python tools/read_rda.py            # writes tests/golden/rda_fixtures.json

The reference's own data files (read as data, nothing executed):
  data/permittedValues.rda   R/presets.R:22-79     argument ranges of soundgen()
  R/sysdata.rda              data-raw/noiseThresholdsDict.R:1-19   q1/q2 thresholds
  data/presets.rda           R/presets.R:156-410   preset calls and vowel formants
  data/defaults.rda          the soundgen() defaults list (if present)

Mapping: NULL -> None; logical/integer/double/character vectors -> lists (NA ->
None), length-1 vectors stay lists; a list with names -> {"__names__": [...],
"values": [...]}; attributes (dim, dimnames, names, class) are kept under
"__attr__" for atomic vectors.
"""
import bz2
import gzip
import json
import lzma
import os
import struct
import sys

NA_INT = -2147483648


class _Reader:
    def __init__(self, data):
        self.b = data
        self.p = 0
        self.refs = []

    def raw(self, n):
        v = self.b[self.p:self.p + n]
        self.p += n
        return v

    def i32(self):
        return struct.unpack(">i", self.raw(4))[0]

    def f64s(self, n):
        return list(struct.unpack(">%dd" % n, self.raw(8 * n)))

    def length(self):
        n = self.i32()
        if n == -1:
            hi, lo = self.i32(), self.i32()
            n = (hi << 32) + lo
        return n

    def item(self):
        flags = self.i32()
        t = flags & 0xFF
        has_attr = bool(flags & (1 << 9))
        has_tag = bool(flags & (1 << 10))
        if t == 254:  # NILVALUE_SXP
            return None
        if t in (253, 242, 241, 252, 251, 250):  # global/empty/base env, unbound, missing, base namespace
            return {"__special__": t}
        if t == 255:  # REFSXP
            idx = flags >> 8
            if idx == 0:
                idx = self.i32()
            return self.refs[idx - 1]
        if t in (249, 248):  # NAMESPACESXP / PACKAGESXP: a STRSXP-like info vector
            self.i32()  # 0
            n = self.i32()
            info = [self.item() for _ in range(n)]
            v = {"__namespace__": info}
            self.refs.append(v)
            return v
        if t == 1:  # SYMSXP
            name = self.item()
            self.refs.append(name)
            return name
        if t in (2, 6, 17, 239, 240):  # pairlist-like (LISTSXP, LANGSXP, DOTSXP, ATTRLISTSXP, ATTRLANGSXP)
            out = []
            while True:
                attr = self.item() if has_attr else None
                tag = self.item() if has_tag else None
                car = self.item()
                out.append((tag, car))
                flags = self.i32()
                t = flags & 0xFF
                has_attr = bool(flags & (1 << 9))
                has_tag = bool(flags & (1 << 10))
                if t not in (2, 6, 17, 239, 240):
                    self.p -= 4
                    self.item()  # the terminating CDR (NILVALUE)
                    break
            return {"__pairlist__": out}
        if t == 9:  # CHARSXP
            n = self.i32()
            return None if n == -1 else self.raw(n).decode("utf-8", "replace")
        if t in (10, 13):  # LGLSXP, INTSXP
            n = self.length()
            v = list(struct.unpack(">%di" % n, self.raw(4 * n)))
            v = [None if x == NA_INT else x for x in v]
            if t == 10:
                v = [None if x is None else bool(x) for x in v]
            return self._attrs(v, has_attr)
        if t == 14:  # REALSXP
            n = self.length()
            return self._attrs(self.f64s(n), has_attr)
        if t == 15:  # CPLXSXP: n (re, im) pairs
            n = self.length()
            f = self.f64s(2 * n)
            return self._attrs([complex(f[2 * i], f[2 * i + 1]) for i in range(n)], has_attr)
        if t == 24:  # RAWSXP
            n = self.length()
            return self._attrs(list(self.raw(n)), has_attr)
        if t == 16:  # STRSXP
            n = self.length()
            return self._attrs([self.item() for _ in range(n)], has_attr)
        if t in (19, 20):  # VECSXP, EXPRSXP
            n = self.length()
            v = [self.item() for _ in range(n)]
            attr = self._attr_dict() if has_attr else {}
            names = attr.get("names")
            if names is not None:
                return {"__names__": names, "values": v, "__attr__": {k: a for k, a in attr.items() if k != "names"}}
            return v if not attr else {"values": v, "__attr__": attr}
        raise ValueError("unsupported SEXP type %d at byte %d" % (t, self.p))

    def _attr_dict(self):
        pl = self.item()
        return {tag: val for tag, val in pl["__pairlist__"]} if pl else {}

    def _attrs(self, v, has_attr):
        if not has_attr:
            return v
        return {"values": v, "__attr__": self._attr_dict()}


def read_rda(path):
    data = open(path, "rb").read()
    if data[:2] == b"\x1f\x8b":
        data = gzip.decompress(data)
    elif data[:3] == b"BZh":
        data = bz2.decompress(data)
    elif data[:6] == b"\xfd7zXZ\x00":
        data = lzma.decompress(data)
    if data[:5] not in (b"RDX2\n", b"RDX3\n"):
        raise ValueError("not an R save file: %r" % data[:5])
    r = _Reader(data[5:])
    if r.raw(2) != b"X\n":
        raise ValueError("only the XDR serialization format is supported")
    version = r.i32()
    r.i32()  # writer R version
    r.i32()  # minimal reader version
    if version == 3:
        r.raw(r.i32())  # native encoding
    top = r.item()
    return {tag: val for tag, val in top["__pairlist__"]}


def _plain(v):
    """Named lists -> dicts (names kept in order), attributes dropped except dim/dimnames."""
    if isinstance(v, dict) and "__names__" in v:
        return {n: _plain(x) for n, x in zip(v["__names__"], v["values"])}
    if isinstance(v, dict) and "values" in v:
        a = v.get("__attr__", {})
        out = {"values": _plain(v["values"])}
        for k in ("dim", "dimnames", "names", "row.names", "class"):
            if k in a:
                out[k] = _plain(a[k])
        return out
    if isinstance(v, list):
        return [_plain(x) for x in v]
    return v


def main(ref="/root/reference", out=None):
    out = out or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                              "rda_fixtures.json")
    res = {"source": "decoded by tools/read_rda.py from the reference's data files (R XDR serialization)"}
    for rel in ("data/permittedValues.rda", "R/sysdata.rda", "data/presets.rda", "data/defaults.rda"):
        p = os.path.join(ref, rel)
        if os.path.exists(p):
            res[rel] = {k: _plain(v) for k, v in read_rda(p).items()}
    with open(out, "w") as f:
        json.dump(res, f, indent=0, sort_keys=False)
    print(out)


if __name__ == "__main__":
    main(*sys.argv[1:])
