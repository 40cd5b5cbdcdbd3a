"""Formula -> kernel lowering — mirror of /root/reference/src/abstractgp_translations.jl.

The reference turns a formula into a KernelFunctions 0.10.38 kernel tree:
    makekernel (:8-15)      SqExp -> SqExponentialKernel [∘ ScaleTransform(1/l) if l != 1]
                            OU    -> ExponentialKernel   [∘ ScaleTransform(1/l) if l != 1]
                            Linear-> LinearKernel(c);  Cat -> CategoricalKernel
    _convert2eq (:31-35)    `+` -> KernelSum (flattening), `*` -> KernelProduct (flattening)
    kernel(::GPOperation)   (:45-69) walks the top-level kernel's `.kernels`, composing
                            each with SelectTransform([position]) and SUMMING them — a
                            top-level product therefore becomes a sum and a nested
                            product errors; this mirror reproduces both.
    kernel(::GPCompnent)    (:71) a single term, no SelectTransform.
    _walk_kernel (:17-19)   flattens sums / strips transforms.

`lower(kernel)` is this build's addition (SURVEY.md §8b "lowering rule"): it walks the
object `kernel()` returned and emits the flat term descriptor the HIP library consumes,
so whatever the reference computes (including Q1) is reproduced by construction.
`lower_formula(..., products=True)` is the documented true-product extension.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Tuple

from . import formula as F
from ._native import CAT, LINEAR, NOISE, OU, SQEXP

# --------------------------------------------------------------------------- KF mirror


class Kernel:
    def __add__(self, other):
        if not isinstance(other, Kernel):
            return NotImplemented
        a = self.kernels if isinstance(self, KernelSum) else (self,)
        b = other.kernels if isinstance(other, KernelSum) else (other,)
        return KernelSum(tuple(a) + tuple(b))

    def __mul__(self, other):
        if not isinstance(other, Kernel):
            return NotImplemented
        a = self.kernels if isinstance(self, KernelProduct) else (self,)
        b = other.kernels if isinstance(other, KernelProduct) else (other,)
        return KernelProduct(tuple(a) + tuple(b))

    def compose(self, t: "Transform") -> "TransformedKernel":
        """k ∘ t (KernelFunctions: TransformedKernel(k, t); on a TransformedKernel the
        transforms chain, the new one applied first)."""
        if isinstance(self, TransformedKernel):
            return TransformedKernel(self.kernel, ChainTransform((t,) + self.transform.chain()))
        return TransformedKernel(self, t)


class SimpleKernel(Kernel):
    pass


@dataclass(frozen=True)
class SqExponentialKernel(SimpleKernel):
    pass


@dataclass(frozen=True)
class ExponentialKernel(SimpleKernel):
    pass


@dataclass(frozen=True)
class LinearKernel(SimpleKernel):
    c: float = 0.0

    def __post_init__(self):
        if not (self.c >= 0):  # KernelFunctions @check_args(LinearKernel, c, c >= 0)
            raise F.ArgumentError("LinearKernel: c >= 0 required")


@dataclass(frozen=True)
class CategoricalKernel(SimpleKernel):
    """src/gp_parts.jl:11-13"""


@dataclass(frozen=True)
class IndexNoiseKernel(SimpleKernel):
    """Extension kernel for `Noise`: variance * delta_ij by observation index."""
    variance: float = 1.0


class Transform:
    def chain(self) -> tuple:
        return (self,)


@dataclass(frozen=True)
class ScaleTransform(Transform):
    s: float
    lengthscale: Optional[float] = None  # the l it came from (with_lengthscale), if known


@dataclass(frozen=True)
class SelectTransform(Transform):
    select: Tuple[int, ...]  # 1-based column positions, as in Julia


@dataclass(frozen=True)
class ChainTransform(Transform):
    transforms: Tuple[Transform, ...]  # applied left to right

    def chain(self):
        return self.transforms


@dataclass(frozen=True)
class TransformedKernel(Kernel):
    kernel: Kernel
    transform: Transform


@dataclass(frozen=True)
class KernelSum(Kernel):
    kernels: Tuple[Kernel, ...]


@dataclass(frozen=True)
class KernelProduct(Kernel):
    kernels: Tuple[Kernel, ...]


@dataclass(frozen=True)
class KernelTensorProduct(Kernel):
    kernels: Tuple[Kernel, ...]


def with_lengthscale(k: Kernel, l: float) -> TransformedKernel:
    if not (l > 0):
        raise F.ArgumentError("lengthscale must be > 0 (ScaleTransform(s) requires s > 0)")
    return TransformedKernel(k, ScaleTransform(1.0 / l, l))


# --------------------------------------------------------------------------- makekernel


def makekernel(c: F.GPCompnent, *hp):
    """src/abstractgp_translations.jl:8-15 (one- and two-argument methods)."""
    if hp:
        (val,) = hp
        if isinstance(c, F.SqExp):
            return SqExponentialKernel() if val == 1 else with_lengthscale(SqExponentialKernel(), val)
        if isinstance(c, F.OU):
            return ExponentialKernel() if val == 1 else with_lengthscale(ExponentialKernel(), val)
        if isinstance(c, F.Linear):
            return LinearKernel(val)
        # makekernel(::Cat, l) has no method
        raise F.MethodError(f"MethodError: no method matching makekernel({type(c).__name__}, {val!r})")
    if isinstance(c, F.SqExp):
        return SqExponentialKernel() if c.lengthscale == 1 else with_lengthscale(SqExponentialKernel(), c.lengthscale)
    if isinstance(c, F.OU):
        return ExponentialKernel() if c.lengthscale == 1 else with_lengthscale(ExponentialKernel(), c.lengthscale)
    if isinstance(c, F.Linear):
        return LinearKernel(c.intercept)
    if isinstance(c, F.Cat):
        return CategoricalKernel()
    if isinstance(c, F.Noise):
        return IndexNoiseKernel(c.variance)
    raise F.MethodError(f"MethodError: no method matching makekernel({type(c).__name__})")


def _convertop(op: str):
    if op == "add":
        return lambda a, b: a + b
    if op == "multiply":
        return lambda a, b: a * b
    raise F.ArgumentError(f"Operation {op} not yet supported")


def _convert2eq(c, hyperparams=None):
    hyperparams = hyperparams or {}
    if isinstance(c, F.GPOperation):
        return _convertop(c.op)(_convert2eq(c.lhs, hyperparams), _convert2eq(c.rhs, hyperparams))
    vn = getattr(c, "varname", None)
    if vn is not None and vn in hyperparams:
        return makekernel(c, hyperparams[vn])
    return makekernel(c)


def _is_leafish(k) -> bool:
    return isinstance(k, (SimpleKernel, TransformedKernel))


def kernel(formula: F.GPCompnent, hyperparams=None):
    """src/abstractgp_translations.jl:45-71 — returns (kernel, vars)."""
    vars_ = F.varnames(formula)
    ks = _convert2eq(formula, hyperparams)
    if not isinstance(formula, F.GPOperation):
        return ks, vars_
    retkernel = None
    counter = 0
    current_k = 1
    kernels = ks.kernels if hasattr(ks, "kernels") else (ks,)
    noise_terms = []
    while current_k <= len(vars_) or counter < len(kernels):
        if counter >= len(kernels):
            raise IndexError("BoundsError: attempt to access kernels")
        k = kernels[counter]
        if isinstance(k, KernelTensorProduct):
            n = len(k.kernels)
            kk = k.compose(SelectTransform(tuple(range(current_k, current_k + n))))
            current_k += n
        elif isinstance(k, IndexNoiseKernel):
            kk = k  # extension: Noise selects no column
            noise_terms.append(k)
        elif _is_leafish(k):
            kk = k.compose(SelectTransform((current_k,)))
            current_k += 1
        else:
            # `@show typeof(k); error()` — nested products / sums of products
            raise RuntimeError(f"kernel(): unsupported kernel in sum: {type(k).__name__}")
        retkernel = kk if retkernel is None else retkernel + kk
        counter += 1
    return retkernel, vars_


def _walk_kernel(ks) -> list:
    """src/abstractgp_translations.jl:17-19"""
    if isinstance(ks, (KernelTensorProduct, KernelSum)):
        out = []
        for k in ks.kernels:
            out.extend(_walk_kernel(k))
        return out
    if isinstance(ks, TransformedKernel):
        return _walk_kernel(ks.kernel)
    if isinstance(ks, SimpleKernel):
        return [ks]
    raise F.MethodError(f"MethodError: no method matching _walk_kernel({type(ks).__name__})")


# --------------------------------------------------------------------------- lowering


@dataclass
class Descriptor:
    """Flat term list for the C-ABI: (kind, col, param, group); col is 0-based into X."""
    terms: List[Tuple[int, int, float, int]] = field(default_factory=list)


def _lower_leaf(k: Kernel, group: int) -> Tuple[int, int, float, int]:
    col = 0
    scale_l = None
    base = k
    if isinstance(k, TransformedKernel):
        base = k.kernel
        for t in k.transform.chain():
            if isinstance(t, SelectTransform):
                if len(t.select) != 1:
                    raise NotImplementedError("multi-column SelectTransform")
                col = t.select[0] - 1
            elif isinstance(t, ScaleTransform):
                scale_l = t.lengthscale if t.lengthscale is not None else 1.0 / t.s
            else:
                raise NotImplementedError(type(t).__name__)
    if isinstance(base, SqExponentialKernel):
        return (SQEXP, col, 1.0 if scale_l is None else float(scale_l), group)
    if isinstance(base, ExponentialKernel):
        return (OU, col, 1.0 if scale_l is None else float(scale_l), group)
    if isinstance(base, LinearKernel):
        if scale_l is not None:
            raise NotImplementedError("scaled LinearKernel")
        return (LINEAR, col, float(base.c), group)
    if isinstance(base, CategoricalKernel):
        return (CAT, col, 0.0, group)
    if isinstance(base, IndexNoiseKernel):
        return (NOISE, -1, float(base.variance), group)
    raise NotImplementedError(type(base).__name__)


def lower(k: Kernel) -> List[Tuple[int, int, float, int]]:
    """Lower the object returned by kernel() to the C-ABI term descriptor."""
    if isinstance(k, KernelSum):
        out = []
        for g, kk in enumerate(k.kernels):
            if isinstance(kk, KernelProduct):
                for f in kk.kernels:
                    out.append(_lower_leaf(f, g))
            else:
                out.append(_lower_leaf(kk, g))
        return out
    if isinstance(k, KernelProduct):
        return [_lower_leaf(f, 0) for f in k.kernels]
    return [_lower_leaf(k, 0)]


def lower_formula(formula: F.GPCompnent, hyperparams=None, products: bool = False):
    """Descriptor + the variables (X columns, one per term, reference order).

    products=False: exactly what the reference computes (kernel() + lower()).
    products=True : extension — `*` is a true (Hadamard) product and nested products
                    are allowed; X columns are still one per term, in varnames order.
    """
    if not products:
        k, vars_ = kernel(formula, hyperparams)
        return lower(k), vars_
    vars_ = F.varnames(formula)
    hyperparams = hyperparams or {}
    groups: List[List[F.GPCompnent]] = []

    def sum_terms(node):
        if isinstance(node, F.GPOperation) and node.op == "add":
            sum_terms(node.lhs)
            sum_terms(node.rhs)
        else:
            groups.append(prod_terms(node))

    def prod_terms(node):
        if isinstance(node, F.GPOperation):
            if node.op == "multiply":
                return prod_terms(node.lhs) + prod_terms(node.rhs)
            raise NotImplementedError("sum nested inside a product: expand it first")
        return [node]

    sum_terms(formula)
    out = []
    pos = 0
    for g, factors in enumerate(groups):
        for c in factors:
            kk = _convert2eq(c, hyperparams)
            if isinstance(c, F.Noise):
                out.append(_lower_leaf(kk, g))
            else:
                out.append(_lower_leaf(kk.compose(SelectTransform((pos + 1,))), g))
                pos += 1
    return out, vars_
