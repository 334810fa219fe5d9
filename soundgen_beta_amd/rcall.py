"""R call literals of the subset soundgen's presets and morph() formulas use
(soundgen(...), list(...), c(...), numbers, strings, NA / TRUE / FALSE / NULL)
evaluated into plain Python data: R/presets.R:156-410 stores presets as such
strings, and morph() (R/morph.R:37-56) accepts 'soundgen(...)' strings. Data,
never code: anything outside the subset raises."""
import re

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


def parse_call(text):
    """'soundgen(a = 1, b = list(...))' -> {'a': 1.0, 'b': {...}} (R's list semantics:
    a repeated name keeps the first value, as R's $ finds it)."""
    v = Parser(tokens(" ".join(text.split()))).expr()
    return v if isinstance(v, dict) else {}
