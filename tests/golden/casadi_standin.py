"""A numeric stand-in for the ``casadi`` module, just large enough to run the
reference's own ``control/MPC.py`` (AlexGisi/mpc-racing) in this container.

TEST INFRASTRUCTURE ONLY: used by ``tests/golden/make_nlp_golden.py`` in the
build container to record what the reference's NLP assembly evaluates to.
casadi 3.6.5 (``requirements.txt:8``) is not installed and cannot be installed
offline, so IPOPT itself never runs; instead ``Opti`` here is a *recording*
Opti: its decision variables take the values of a supplied point w, and it
records, in call order,

* every ``subject_to`` row as (canonical expression value, lbg, ubg),
* every ``set_initial`` value (the initial guess of ``MPC.py:109-131``),
* the objective value passed to ``minimize`` (``MPC.py:86-98``),
* the solver options (``MPC.py:152-161``),

and ``solve()`` returns an OptiSol whose ``value()`` reads the supplied point,
so the reference's own ``ret`` assembly (``MPC.py:166-170``) runs unchanged.

Symbolic pieces (``SX.sym``, ``Function``, ``gradient``) are a lazy expression
tree evaluated in fp64 in the order the reference writes the arithmetic;
``gradient`` is forward-mode (dual numbers).  Matrices follow CasADi's
indexing: a single integer is a column-major linear index, Python negative
indices wrap (``U[:, -1]`` is column N-1), ``M[:, j]`` is a column.

Constraint canonicalisation follows CasADi's Opti (``canon_expr``): when one
side of a comparison is a constant, the other side is the row and the constant
becomes its bound; otherwise the row is ``lhs - rhs`` with bound 0; ``bounded(lb,
e, ub)`` is the row ``e`` in [lb, ub].  Rows of a vector comparison are emitted
in element order.  This is the documented behaviour of casadi's Opti; it could
not be executed here (no casadi), so the row-expression convention -- and with
it the sign convention of ``lam_g`` -- is stated, not pinned.
"""
import math
import types

import numpy as np

INF = math.inf


# --------------------------------------------------------------------------------------------
# forward-mode dual numbers (for ``gradient``)
# --------------------------------------------------------------------------------------------
class Dual:
    __array_ufunc__ = None  # numpy scalars defer to our reflected operators

    def __init__(self, v, d):
        self.v, self.d = v, d

    @staticmethod
    def _p(o):
        return o if isinstance(o, Dual) else Dual(o, 0.0)

    def __add__(self, o):
        o = self._p(o)
        return Dual(self.v + o.v, self.d + o.d)

    __radd__ = __add__

    def __sub__(self, o):
        o = self._p(o)
        return Dual(self.v - o.v, self.d - o.d)

    def __rsub__(self, o):
        return self._p(o) - self

    def __mul__(self, o):
        o = self._p(o)
        return Dual(self.v * o.v, self.d * o.v + self.v * o.d)

    __rmul__ = __mul__

    def __truediv__(self, o):
        o = self._p(o)
        return Dual(self.v / o.v, (self.d * o.v - self.v * o.d) / (o.v * o.v))

    def __rtruediv__(self, o):
        return self._p(o) / self

    def __neg__(self):
        return Dual(-self.v, -self.d)

    def __pow__(self, n):
        if isinstance(n, Dual):
            raise TypeError("dual ** dual not needed by the reference")
        if n == 0:
            return Dual(self.v ** 0, 0.0)
        return Dual(self.v ** n, n * self.v ** (n - 1) * self.d)


# --------------------------------------------------------------------------------------------
# lazy expressions (SX)
# --------------------------------------------------------------------------------------------
def _ev(x, env):
    return x.ev(env) if isinstance(x, Expr) else _num(x)


class Expr:
    __array_ufunc__ = None

    def __init__(self, fn, n=1):
        self.fn = fn
        self.n = n  # number of elements (column vector)

    def ev(self, env):
        return self.fn(env)

    def _bin(self, o, f):
        a, b = self, o
        return Expr(lambda env: f(_ev(a, env), _ev(b, env)))

    def _rbin(self, o, f):
        a, b = o, self
        return Expr(lambda env: f(_ev(a, env), _ev(b, env)))

    def __add__(self, o): return self._bin(o, lambda a, b: a + b)
    def __radd__(self, o): return self._rbin(o, lambda a, b: a + b)
    def __sub__(self, o): return self._bin(o, lambda a, b: a - b)
    def __rsub__(self, o): return self._rbin(o, lambda a, b: a - b)
    def __mul__(self, o): return self._bin(o, lambda a, b: a * b)
    def __rmul__(self, o): return self._rbin(o, lambda a, b: a * b)
    def __truediv__(self, o): return self._bin(o, lambda a, b: a / b)
    def __rtruediv__(self, o): return self._rbin(o, lambda a, b: a / b)
    def __pow__(self, o): return self._bin(o, lambda a, b: a ** b)
    def __neg__(self): return Expr(lambda env, a=self: -_ev(a, env))

    def __getitem__(self, k):
        if not isinstance(k, (int, np.integer)):
            raise TypeError("only scalar indexing of symbols is used by the reference")
        a, n = self, self.n
        return Expr(lambda env: np.asarray(_ev(a, env)).reshape(-1)[k % n])


class _Leaf(Expr):
    _next = 0

    def __init__(self, name, n):
        _Leaf._next += 1
        self.key = (_Leaf._next, name)
        key = self.key
        super().__init__(lambda env: env[key], n)


class SX:
    @staticmethod
    def sym(name, r=1, c=1):
        return _Leaf(name, r * c)


def _has_expr(*xs):
    return any(isinstance(x, Expr) for x in xs)


def _unary(npf, dualf):
    def f(x):
        if isinstance(x, Expr):
            return Expr(lambda env: f(_ev(x, env)))
        if isinstance(x, Dual):
            return dualf(x)
        return npf(_num(x))
    return f


def _dual_only(name):
    def f(x):
        raise TypeError(f"{name} of a dual number is not needed by the reference")
    return f


sin = _unary(np.sin, _dual_only("sin"))
cos = _unary(np.cos, _dual_only("cos"))
tan = _unary(np.tan, _dual_only("tan"))
sqrt = _unary(np.sqrt, _dual_only("sqrt"))
exp = _unary(np.exp, _dual_only("exp"))
atan = _unary(np.arctan, _dual_only("atan"))


def atan2(y, x):
    if _has_expr(y, x):
        return Expr(lambda env: atan2(_ev(y, env), _ev(x, env)))
    return np.arctan2(_num(y), _num(x))


def fmin(a, b):
    if _has_expr(a, b):
        return Expr(lambda env: fmin(_ev(a, env), _ev(b, env)))
    return np.fmin(_num(a), _num(b))


def fmax(a, b):
    if _has_expr(a, b):
        return Expr(lambda env: fmax(_ev(a, env), _ev(b, env)))
    return np.fmax(_num(a), _num(b))


def vertcat(*xs):
    if _has_expr(*xs):
        items = list(xs)
        return Expr(lambda env: np.array([float(_ev(x, env)) for x in items]), len(items))
    return DM(np.array([float(_num(x)) for x in xs]).reshape(-1, 1))


def horzcat(*cols):
    return DM(np.stack([np.asarray(_num(c), dtype=np.float64).reshape(-1) for c in cols], axis=1))


def gradient(expr, s):
    """d expr / d s (scalar s) by forward-mode duals at evaluation time."""
    key = s.key

    def fn(env):
        e2 = dict(env)
        e2[key] = Dual(env[key], 1.0)
        r = expr.ev(e2)
        return r.d if isinstance(r, Dual) else 0.0
    return Expr(fn)


class Function:
    def __init__(self, name, args, outs):
        self.name, self.args, self.out = name, list(args), outs[0]

    def __call__(self, *vals):
        if _has_expr(*vals):
            return Expr(lambda env: self(*[_ev(v, env) for v in vals]), getattr(self.out, "n", 1))
        env = {}
        for a, v in zip(self.args, vals):
            x = np.asarray(_num(v), dtype=np.float64).reshape(-1)
            env[a.key] = x if a.n > 1 else (v if isinstance(v, Dual) else float(x[0]))
        r = _ev(self.out, env)
        if isinstance(r, np.ndarray) and r.size > 1:
            # an expression of decision variables stays one in comparisons (not a constant bound)
            return (_Derived if any(isinstance(v, Var) for v in vals) else DM)(r.reshape(-1, 1))
        return float(np.asarray(r).reshape(-1)[0]) if not isinstance(r, Dual) else r


# --------------------------------------------------------------------------------------------
# numeric matrices (DM) and recorded decision variables
# --------------------------------------------------------------------------------------------
def _num(x):
    if isinstance(x, (DM, Var)):
        v = x.value()
        return float(v.reshape(-1)[0]) if v.size == 1 else v
    if isinstance(x, (tuple, list)):
        return np.array(x, dtype=np.float64)
    return x


def _index(shape, key):
    """Column-major flat positions selected by a CasADi-style index on a matrix of ``shape``."""
    r, c = shape
    pos = np.arange(r * c).reshape((r, c), order="F")
    if isinstance(key, tuple):
        i, j = key
        i = i % r if isinstance(i, (int, np.integer)) else i
        j = j % c if isinstance(j, (int, np.integer)) else j
        sub = pos[i, j]
        sub = np.asarray(sub)
        if sub.ndim == 0:
            return sub.reshape(1, 1)
        if isinstance(key[0], slice) and not isinstance(key[1], slice):
            return sub.reshape(-1, 1)  # a column
        if isinstance(key[1], slice) and not isinstance(key[0], slice):
            return sub.reshape(1, -1)  # a row
        return sub
    if isinstance(key, (int, np.integer)):
        return pos.reshape(-1, order="F")[key % (r * c)].reshape(1, 1)
    raise TypeError(key)


class _Arith:
    __array_ufunc__ = None

    def __add__(self, o): return _num(self) + _num(o)
    def __radd__(self, o): return _num(o) + _num(self)
    def __sub__(self, o): return _num(self) - _num(o)
    def __rsub__(self, o): return _num(o) - _num(self)
    def __mul__(self, o): return _num(self) * _num(o)
    def __rmul__(self, o): return _num(o) * _num(self)
    def __truediv__(self, o): return _num(self) / _num(o)
    def __rtruediv__(self, o): return _num(o) / _num(self)
    def __pow__(self, o): return _num(self) ** _num(o)
    def __neg__(self): return -_num(self)
    def __float__(self): return float(_num(self))


class DM(_Arith):
    def __init__(self, a):
        a = np.asarray(a, dtype=np.float64)
        self.a = a.reshape(-1, 1) if a.ndim == 1 else a

    @property
    def shape(self):
        return self.a.shape

    def value(self):
        return self.a

    def __getitem__(self, key):
        sub = _index(self.a.shape, key)
        flat = self.a.reshape(-1, order="F")
        v = flat[sub]
        return float(v[0, 0]) if v.size == 1 else DM(v)


class Var(_Arith):
    """A (view of a) decision variable of the recording Opti: arithmetic uses the point's values,
    comparisons build constraint records."""

    def __init__(self, opti, vid, pos):
        self.opti, self.vid, self.pos = opti, vid, pos

    @property
    def shape(self):
        return self.pos.shape

    def value(self):
        return self.opti.values[self.vid].reshape(-1, order="F")[self.pos]

    def __getitem__(self, key):
        sub = _index(self.pos.shape, key)
        return Var(self.opti, self.vid, self.pos.reshape(-1, order="F")[sub])

    def _cmp(self, other, kind, swapped=False):
        return _Constraint(self, other, kind) if not swapped else _Constraint(other, self, kind)

    def __eq__(self, o): return _Constraint(self, o, "eq")
    def __le__(self, o): return _Constraint(self, o, "le")
    def __lt__(self, o): return _Constraint(self, o, "le")
    def __ge__(self, o): return _Constraint(o, self, "le")
    def __gt__(self, o): return _Constraint(o, self, "le")
    __hash__ = object.__hash__


class _Derived(DM):
    """Numeric value of a Function of decision variables (not a constant for canon_expr)."""


def _is_const(x):
    return not isinstance(x, (Var, _Derived))


class _Constraint:
    def __init__(self, lhs, rhs, kind):
        # Opti canon_expr: a constant side becomes the bound, otherwise lhs - rhs against 0
        if kind == "eq":
            if _is_const(rhs):
                e, lb, ub = _num(lhs), _num(rhs), _num(rhs)
            elif _is_const(lhs):
                e, lb, ub = _num(rhs), _num(lhs), _num(lhs)
            else:
                e, lb, ub = _num(lhs) - _num(rhs), 0.0, 0.0
        else:  # lhs <= rhs
            if _is_const(rhs):
                e, lb, ub = _num(lhs), -INF, _num(rhs)
            elif _is_const(lhs):
                e, lb, ub = _num(rhs), _num(lhs), INF
            else:
                e, lb, ub = _num(lhs) - _num(rhs), -INF, 0.0
        e = np.asarray(e, dtype=np.float64).reshape(-1)
        self.g = e
        self.lb = np.broadcast_to(np.asarray(lb, dtype=np.float64).reshape(-1), e.shape).copy()
        self.ub = np.broadcast_to(np.asarray(ub, dtype=np.float64).reshape(-1), e.shape).copy()


class _LamG:
    pass


class OptiSol:
    def __init__(self, opti):
        self.opti = opti

    def value(self, x):
        if isinstance(x, _LamG):
            return np.arange(len(self.opti.g), dtype=np.float64)  # row indices (ordering only)
        if isinstance(x, Var):
            v = self.opti.values[x.vid].reshape(-1, order="F")[x.pos]
            if v.size == 1:
                return float(v[0, 0])
            if v.shape[0] == 1 or v.shape[1] == 1:
                return v.reshape(-1)
            return v
        v = np.asarray(_num(x), dtype=np.float64)
        return float(v.reshape(-1)[0]) if v.size == 1 else v


class Opti:
    """Recording Opti.  ``Opti.point`` (a list of arrays, one per ``variable`` call in order) must
    be set before the reference constructs its problem."""
    point = None
    last = None

    def __init__(self):
        self.values = []
        self.init = []
        self.g, self.lbg, self.ubg = [], [], []
        self.row_of_call = []
        self.J = None
        self.options = None
        self.lam_g = _LamG()
        self.debug = OptiSol(self)
        Opti.last = self

    def variable(self, r, c=1):
        vid = len(self.values)
        self.values.append(np.asarray(Opti.point[vid], dtype=np.float64).reshape(r, c))
        self.init.append(np.full((r, c), np.nan))
        return Var(self, vid, np.arange(r * c).reshape((r, c), order="F"))

    def subject_to(self, con):
        self.row_of_call.append(len(self.g))
        self.g.extend(con.g.tolist())
        self.lbg.extend(con.lb.tolist())
        self.ubg.extend(con.ub.tolist())

    def bounded(self, lb, e, ub):
        c = _Constraint.__new__(_Constraint)
        c.g = np.asarray(_num(e), dtype=np.float64).reshape(-1)
        c.lb = np.broadcast_to(np.asarray(_num(lb), dtype=np.float64), c.g.shape).copy()
        c.ub = np.broadcast_to(np.asarray(_num(ub), dtype=np.float64), c.g.shape).copy()
        return c

    def set_initial(self, v, val):
        flat = self.init[v.vid].reshape(-1, order="F")
        vals = np.asarray(_num(val), dtype=np.float64).reshape(-1, order="F")
        flat[v.pos.reshape(-1, order="F")] = np.broadcast_to(vals, (v.pos.size,))
        self.init[v.vid] = flat.reshape(self.init[v.vid].shape, order="F")

    def minimize(self, J):
        self.J = float(_num(J))

    def solver(self, name, opts=None):
        self.options = (name, opts)

    def solve(self):
        return OptiSol(self)


def install():
    """Register this module as ``casadi`` (build container only)."""
    import sys
    mod = types.ModuleType("casadi")
    for k in ("SX", "DM", "Function", "Opti", "gradient", "vertcat", "horzcat", "sin", "cos", "tan", "sqrt",
              "exp", "atan", "atan2", "fmin", "fmax"):
        setattr(mod, k, globals()[k])
    sys.modules["casadi"] = mod
    return mod
