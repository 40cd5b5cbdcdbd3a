"""GaPLAC formula vocabulary and spec parsing — mirror of the reference's Julia surface.

    /root/reference/src/gp_parts.jl        GPCompnent, GPOperation, SqExp, Linear, OU, Cat,
                                           varnames, `+` -> :add, `*` -> :multiply
    /root/reference/src/interface.jl:1-41  Spec, gp_spec, likelihood/response/formula,
                                           make_gp
    /root/reference/src/liklihoods.jl      Gaussian likelihood tag

`Noise` is an extension (the reference names it in README.md:43 but never defines it,
SURVEY.md Q2): bare `Noise` adds 1.0 * delta_ij by observation index, `Noise(v)` adds
v * delta_ij.

The gp part of a formula is Julia expression syntax; the reference `eval`s it inside
the GaPLAC module (interface.jl:31). Here a small recursive-descent parser accepts the
same expressions: calls with positional symbols and keyword arguments (`SqExp(:x; l=2)`,
`SqExp(:x, l=2)`), `+`, `*` (binding tighter than `+`), parentheses and numbers.
"""
from __future__ import annotations

import re
from dataclasses import dataclass
from typing import List, Union


class MethodError(TypeError):
    """Mirror of Julia's MethodError (no method matching the call)."""


class UndefVarError(NameError):
    """Mirror of Julia's UndefVarError."""


class ArgumentError(ValueError):
    """Mirror of Julia's ArgumentError."""


# --------------------------------------------------------------------------- components
class GPCompnent:  # (sic) the reference's spelling, src/gp_parts.jl:3
    def __add__(self, other):
        if not isinstance(other, GPCompnent):
            return NotImplemented
        return GPOperation("add", self, other)

    def __mul__(self, other):
        if not isinstance(other, GPCompnent):
            return NotImplemented
        return GPOperation("multiply", self, other)


@dataclass(eq=True)
class GPOperation(GPCompnent):
    """src/gp_parts.jl:5-9"""
    op: str
    lhs: GPCompnent
    rhs: GPCompnent


@dataclass(eq=True)
class SqExp(GPCompnent):
    """SqExp(x; l=1) — squared exponential, lengthscale l (src/gp_parts.jl:21-27)."""
    varname: str
    lengthscale: float = 1


@dataclass(eq=True)
class Linear(GPCompnent):
    """Linear(x; c=0) — linear kernel with intercept c (src/gp_parts.jl:29-35)."""
    varname: str
    intercept: float = 0


@dataclass(eq=True)
class OU(GPCompnent):
    """OU(x; l=1) — Ornstein-Uhlenbeck / exponential kernel (src/gp_parts.jl:37-43)."""
    varname: str
    lengthscale: float = 1


@dataclass(eq=True)
class Cat(GPCompnent):
    """Cat(x) — categorical (same level -> 1) kernel (src/gp_parts.jl:45-47)."""
    varname: str


@dataclass(eq=True)
class Noise(GPCompnent):
    """Extension: variance * delta_ij by observation index (absent in the reference)."""
    variance: float = 1.0

    @property
    def varname(self):
        return None


def varname(c: GPCompnent):
    return c.varname


def varnames(gpc: GPCompnent) -> List[str]:
    """src/gp_parts.jl:51-53 — one entry per term, left to right (duplicates kept).
    Noise (extension) reads no column and contributes no variable."""
    if isinstance(gpc, GPOperation):
        return varnames(gpc.lhs) + varnames(gpc.rhs)
    if isinstance(gpc, Noise):
        return []
    return [gpc.varname]


# --------------------------------------------------------------------------- likelihood
class AbstractLiklihood:  # (sic) src/liklihoods.jl:1
    pass


class Gaussian(AbstractLiklihood):
    def __eq__(self, other):
        return isinstance(other, Gaussian)

    def __repr__(self):
        return "Gaussian()"


# --------------------------------------------------------------------------- parser
_TOKEN = re.compile(
    r"\s*(?:(?P<num>(?:\d+\.?\d*|\.\d+)(?:[eE][+-]?\d+)?)|(?P<sym>:[A-Za-z_][A-Za-z0-9_!]*)|"
    r"(?P<str>\"[^\"]*\")|(?P<id>[A-Za-z_][A-Za-z0-9_!]*)|(?P<op>[-+*/(),;=]))"
)


def _tokenize(s: str):
    pos, out = 0, []
    s = s.rstrip()
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m or m.end() == pos:
            raise ArgumentError(f"cannot parse formula near {s[pos:]!r}")
        pos = m.end()
        kind = m.lastgroup
        out.append((kind, m.group(kind)))
    return out


_CONSTRUCTORS = {"SqExp": SqExp, "OU": OU, "Linear": Linear, "Cat": Cat, "Noise": Noise}
_KWARGS = {"SqExp": {"l": "lengthscale"}, "OU": {"l": "lengthscale"}, "Linear": {"c": "intercept"}, "Cat": {},
           "Noise": {}}


class _Parser:
    def __init__(self, text: str):
        self.toks = _tokenize(text)
        self.i = 0

    def peek(self):
        return self.toks[self.i] if self.i < len(self.toks) else (None, None)

    def take(self, val=None):
        tok = self.peek()
        if tok[0] is None or (val is not None and tok[1] != val):
            raise ArgumentError(f"expected {val!r}, got {tok[1]!r}")
        self.i += 1
        return tok

    def parse(self):
        e = self.sum()
        if self.i != len(self.toks):
            raise ArgumentError(f"unexpected token {self.peek()[1]!r}")
        return e

    def sum(self):
        e = self.prod()
        while self.peek() == ("op", "+"):
            self.take()
            e = _add(e, self.prod())
        return e

    def prod(self):
        e = self.atom()
        while self.peek() == ("op", "*"):
            self.take()
            e = _mul(e, self.atom())
        return e

    def number(self):
        sign = 1.0
        if self.peek() == ("op", "-"):
            self.take()
            sign = -1.0
        kind, val = self.take()
        if kind != "num":
            raise ArgumentError(f"expected a number, got {val!r}")
        num = float(val) if any(ch in val for ch in ".eE") else int(val)
        if self.peek() == ("op", "/"):  # simple rational literal like 1/2
            self.take()
            kind2, val2 = self.take()
            if kind2 != "num":
                raise ArgumentError("expected a number after '/'")
            return sign * num / float(val2)
        return sign * num

    def atom(self):
        kind, val = self.peek()
        if (kind, val) == ("op", "("):
            self.take()
            e = self.sum()
            self.take(")")
            return e
        if kind == "id":
            self.take()
            if val not in _CONSTRUCTORS:
                raise UndefVarError(f"UndefVarError: {val} not defined")
            if self.peek() != ("op", "("):
                if val == "Noise":
                    return Noise()
                raise MethodError(f"{val} is a type; a call {val}(...) is required")
            self.take("(")
            pos, kw = [], {}
            in_kw = False
            while self.peek() != ("op", ")"):
                if self.peek() == ("op", ";"):
                    self.take()
                    in_kw = True
                    continue
                k2, v2 = self.peek()
                if k2 == "id" and self.i + 1 < len(self.toks) and self.toks[self.i + 1] == ("op", "="):
                    self.take()
                    self.take("=")
                    kw[v2] = self.number()
                elif in_kw:
                    raise ArgumentError("positional argument after ';'")
                elif k2 == "sym":
                    self.take()
                    pos.append(v2[1:])
                elif k2 == "str":
                    self.take()
                    pos.append(v2[1:-1])
                else:
                    pos.append(self.number())
                if self.peek() == ("op", ","):
                    self.take()
            self.take(")")
            return _construct(val, pos, kw)
        raise ArgumentError(f"unexpected token {val!r}")


def _construct(name: str, pos, kw):
    allowed = _KWARGS[name]
    for k in kw:
        if k not in allowed:
            raise MethodError(f"MethodError: no method matching {name}(...; {k}=...)")
    if name == "Noise":
        if len(pos) > 1 or (pos and isinstance(pos[0], str)):
            raise MethodError("MethodError: Noise takes at most one variance")
        return Noise(float(pos[0])) if pos else Noise()
    # inner constructors take exactly one positional (the variable): src/gp_parts.jl:26,34,42,46
    # (the docstring's positional lengthscale, SqExp(x, l), has no method: SURVEY Q12)
    if len(pos) != 1 or not isinstance(pos[0], str):
        raise MethodError(f"MethodError: no method matching {name}({', '.join(map(repr, pos))})")
    args = {allowed[k]: v for k, v in kw.items()}
    return _CONSTRUCTORS[name](pos[0], **args)


def _add(a, b):
    return a + b


def _mul(a, b):
    return a * b


def parse_gp(text: str) -> GPCompnent:
    """Evaluate the gp part of a formula (interface.jl:30-31 `GaPLAC.eval(Meta.parse(gp))`)."""
    return _Parser(text).parse()


# --------------------------------------------------------------------------- Spec
@dataclass
class Spec:
    """src/interface.jl:1-5"""
    response: str
    lik: object
    formula: GPCompnent


def likelihood(gps: Spec):
    return gps.lik


def response(gps: Spec):
    return gps.response


def formula(gps: Spec):
    return gps.formula


def gp_spec(text: str) -> Spec:
    """Parse `resp [: lik] ~| gp` exactly as src/interface.jl:12-34 slices it."""
    spl2 = text.find("~")
    if spl2 < 0:
        # the reference calls last(nothing) here, which throws before its own check
        raise ArgumentError("Invalid formula specification")
    barind = spl2 + 1
    if barind >= len(text) or text[barind] != "|":
        raise ArgumentError("Invalid formula specification")
    spl1 = text.find(":")
    if spl1 < 0 or spl1 > spl2:
        lik = Gaussian()
        spl1 = spl2 - 1
    else:
        lik_s = text[spl1 + 1:spl2].strip()
        if not lik_s:
            lik = Gaussian()
        elif lik_s in ("Gaussian", "Gaussian()"):
            lik = Gaussian()
        else:
            raise UndefVarError(f"UndefVarError: {lik_s} not defined")
    resp = text[:max(spl1, 0)].strip()
    gp = parse_gp(text[barind + 1:].strip())
    return Spec(resp, lik, gp)
