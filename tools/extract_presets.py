"""Extract the soundgen() argument sets of presets$<speaker>$<name>
(R/presets.R:156-410 of the reference) into soundgen_beta_amd/presets.json.

Each preset is an R call string such as
    'soundgen(sylLen = 250, pitchAnchors = list(time = c(0, 1), value = c(147, 150)), ...)'
This script evaluates the small R subset those strings use (soundgen(), list(),
c(), numbers, strings, NA/TRUE/FALSE/NULL) into JSON data: the parameter
values are inputs for the C5 workload, not code. Runs in the build container
(where /root/reference exists); the JSON travels with the repo.

    python tools/extract_presets.py [/root/reference/R/presets.R]
"""
import json
import os
import re
import sys

SRC = sys.argv[1] if len(sys.argv) > 1 else "/root/reference/R/presets.R"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "soundgen_beta_amd", "presets.json")

TOKEN = re.compile(r"\s*(?:(?P<num>(?:\d+\.?\d*|\.\d+)(?:[eE][-+]?\d+)?)|(?P<str>'[^']*'|\"[^\"]*\")"
                   r"|(?P<id>[A-Za-z_.][A-Za-z0-9_.]*)|(?P<sym>[(),=\-+]))")


def tokens(s):
    pos, out = 0, []
    while pos < len(s):
        m = TOKEN.match(s, pos)
        if not m or m.end() == pos:
            if s[pos:].strip() == "":
                break
            raise ValueError("cannot tokenize at %r" % s[pos:pos + 30])
        pos = m.end()
        kind = m.lastgroup
        out.append((kind, m.group(kind)))
    return out


class Parser:
    def __init__(self, toks):
        self.t, self.i = toks, 0

    def peek(self, k=0):
        return self.t[self.i + k] if self.i + k < len(self.t) else (None, None)

    def take(self, val=None):
        tok = self.t[self.i]
        if val is not None and tok[1] != val:
            raise ValueError("expected %r, got %r" % (val, tok))
        self.i += 1
        return tok

    def expr(self):
        kind, val = self.peek()
        if val in ("-", "+"):
            self.take()
            v = self.expr()
            return -v if val == "-" else v
        if kind == "num":
            self.take()
            return float(val)
        if kind == "str":
            self.take()
            return val[1:-1]
        if kind == "id":
            self.take()
            if self.peek()[1] == "(":
                return self.call(val)
            return {"NA": None, "NULL": None, "TRUE": True, "FALSE": False}[val]
        raise ValueError("unexpected %r" % (val,))

    def call(self, fn):
        self.take("(")
        args = []
        while self.peek()[1] != ")":
            name = None
            if self.peek()[0] == "id" and self.peek(1)[1] == "=":
                name = self.take()[1]
                self.take("=")
            args.append((name, self.expr()))
            if self.peek()[1] == ",":
                self.take()
        self.take(")")
        if fn == "c":
            flat = []
            for _, v in args:
                flat.extend(v if isinstance(v, list) else [v])
            return flat
        if fn in ("list", "soundgen"):
            if all(n is not None for n, _ in args):
                d = {}
                for n, v in args:  # a repeated name: R's $ finds the first (F1$Moan formantsNoise$f3)
                    d.setdefault(n, v)
                return d
            return [v for _, v in args]
        raise ValueError("unsupported R function %s()" % fn)


def main():
    text = open(SRC).read()
    start = text.index("presets = list(")
    body = text[start:]
    speakers = [(m.start(), m.group(1)) for m in re.finditer(r"\n  ([A-Za-z0-9]+) = list\(", body)]
    out = {}
    for m in re.finditer(r"\n\s+([A-Za-z0-9_]+) = '(soundgen\((?:[^']*)\))'", body):
        speaker = [s for p, s in speakers if p < m.start()][-1]
        call = " ".join(m.group(2).split())
        args = Parser(tokens(call)).expr()
        out.setdefault(speaker, {})[m.group(1)] = args if isinstance(args, dict) else {}
    n = sum(len(v) for v in out.values())
    json.dump(out, open(OUT, "w"), indent=1, sort_keys=True)
    print("wrote %d presets (%s) to %s" % (n, ", ".join("%s %d" % (k, len(v)) for k, v in out.items()), OUT))


if __name__ == "__main__":
    main()
