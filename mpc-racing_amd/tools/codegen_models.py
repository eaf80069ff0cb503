"""Generate ``csrc/gen_dynamics.h``: the vehicle dynamics of the MPC NLP with
exact analytic first and second derivatives, as CSE'd straight-line C++.

This replaces CasADi's symbolic AD of ``control/MPC.py``'s ``f_vehicle``
(MPC.py:186-229), ``f_vehicle_kinematic`` (:231-260), ``Fx`` (:273-283) and
``steer_cmd_to_angle`` (:262-271, control/util.py:10-11 with pi = 3.14), plus
the build-defined Blended law (models/BlendedBicycleModel.py:22-46) and the
tyre substitution of learning/vehicle.py:155-160.

Per model three entry points are emitted (templated on the scalar type):
  <model>_f    (x, u)            -> f[6]
  <model>_fj   (x, u)            -> f[6], J[6*8]          (J row-major, cols x0..x5,u0,u1)
  <model>_fjh  (x, u, nu)        -> f[6], J[6*8], H[36]   (H = upper triangle of
                                                          sum_i nu_i d2 f_i / d(x,u)^2, packed row-major)
Tyre models (``*_tyre``) take the front/rear lateral-force jets
(value, d/dalpha, d2/dalpha2) of a scalar tyre law evaluated at the current
slip angles; the chain rule through the slip angles is generated here.

Run:  python mpc-racing_amd/tools/codegen_models.py   (sympy is a build-time tool only)
"""
import os

import sympy as sp
from sympy.printing.c import C99CodePrinter

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "csrc", "gen_dynamics.h")

# vehicle parameters (models/VehicleParameters.py) are runtime values in a struct
PNAMES = ["m", "Iz", "lf", "lr", "Cf", "Cr", "T_max", "r_wheel", "C_wheel", "R", "rho", "C_d",
          "A_f", "C_roll", "g", "max_steer", "Vblendmin", "Vblendmax"]
P = {n: sp.Symbol("P_" + n, real=True) for n in PNAMES}
Ts = sp.Symbol("Ts", positive=True)
X, Y, psi, vx, vy, r = sp.symbols("x0 x1 x2 x3 x4 x5", real=True)
thr, steer = sp.symbols("u0 u1", real=True)
INPUTS = [X, Y, psi, vx, vy, r, thr, steer]
NU = sp.symbols("nu0:6", real=True)
# tyre jets: value, first, second derivative at the current slip angle
TJ = {k: sp.Symbol(k, real=True) for k in ["Ff0", "Ff1", "Ff2", "Fr0", "Fr1", "Fr2"]}
A0F, A0R = sp.symbols("a0f a0r", real=True)


def Fx():
    wheel_rpm = (vx / P["C_wheel"]) * 60
    rpm = wheel_rpm * P["R"] * sp.Rational(9, 2)
    eta = sp.Float("-0.00004428225806", 17) * rpm + sp.Float("1.282413306", 17)
    wheel_force = thr * eta * P["T_max"] * P["R"] / P["r_wheel"]
    drag = sp.Rational(1, 2) * P["rho"] * P["C_d"] * P["A_f"] * vx ** 2
    roll = P["C_roll"] * P["m"] * P["g"]
    return wheel_force - drag - roll


def delta():
    vel = sp.sqrt(vx ** 2 + vy ** 2) * sp.Float("3.6", 17)
    gain = sp.Float("-0.001971664699", 17) * vel + sp.Float("0.986547", 17)
    z = steer * gain * P["max_steer"]
    return (z / 360) * 2 * sp.Float("3.14", 17)


def slip_angles():
    d = delta()
    tf = sp.atan2(vy + P["lf"] * r, vx + sp.Float("0.1", 17))
    tr = sp.atan2(vy - P["lr"] * r, vx + sp.Float("0.1", 17))
    return d, d - tf, -tr


def f_dyn(tyre):
    F = Fx()
    d, af, ar = slip_angles()
    if tyre:
        Fyf = TJ["Ff0"] + TJ["Ff1"] * (af - A0F) + TJ["Ff2"] / 2 * (af - A0F) ** 2
        Fyr = TJ["Fr0"] + TJ["Fr1"] * (ar - A0R) + TJ["Fr2"] / 2 * (ar - A0R) ** 2
    else:
        Fyf = P["Cf"] * af
        Fyr = P["Cr"] * ar
    vxd = ((F - Fyf * sp.sin(d)) / P["m"]) + vy * r
    vyd = ((Fyf * sp.cos(d) + Fyr) / P["m"]) - vx * r
    rd = ((Fyf * sp.cos(d) * P["lf"]) - (Fyr * P["lr"])) / P["Iz"]
    return [X + (vx * sp.cos(psi) - vy * sp.sin(psi)) * Ts,
            Y + (vx * sp.sin(psi) + vy * sp.cos(psi)) * Ts,
            psi + r * Ts,
            vx + vxd * Ts,
            vy + vyd * Ts,
            r + rd * Ts]


def f_kin():
    F = Fx()
    d = delta()
    return [X + (vx * sp.cos(psi) - vy * sp.sin(psi)) * Ts,
            Y + (vx * sp.sin(psi) + vy * sp.cos(psi)) * Ts,
            psi + r * Ts,
            vx + (F / P["m"]) * Ts,
            r * P["lr"],
            (vx / (P["lr"] + P["lf"])) * sp.tan(d)]


def f_blend(tyre):
    lam = (sp.sqrt(vx ** 2 + vy ** 2) - P["Vblendmin"]) / (P["Vblendmax"] - P["Vblendmin"])
    fd = f_dyn(tyre)
    fk = f_kin()
    return [lam * a + (1 - lam) * b for a, b in zip(fd, fk)]


class Printer(C99CodePrinter):
    def _print_Symbol(self, expr):
        n = expr.name
        if n.startswith("P_"):
            return "P." + n[2:]
        if n.startswith("x") and n[1:].isdigit():
            return f"x[{n[1:]}]"
        if n.startswith("u") and n[1:].isdigit():
            return f"u[{n[1:]}]"
        if n.startswith("nu") and n[2:].isdigit():
            return f"nu[{n[2:]}]"
        if n in TJ:
            return {"Ff0": "tf.v", "Ff1": "tf.d", "Ff2": "tf.dd", "Fr0": "tr.v", "Fr1": "tr.d", "Fr2": "tr.dd"}[n]
        return n

    def _print_Pow(self, expr):
        b, e = expr.as_base_exp()
        bs = self.parenthesize(b, 1000)
        if e.is_Integer:
            k = int(e)
            if k == 1:
                return bs
            if k == -1:
                return f"(T(1)/{bs})"
            if 2 <= k <= 4:
                return "(" + "*".join([bs] * k) + ")"
            if -4 <= k <= -2:
                return "(T(1)/(" + "*".join([bs] * (-k)) + "))"
        if e == sp.Rational(1, 2):
            return f"mr_sqrt({self._print(b)})"
        if e == sp.Rational(-1, 2):
            return f"(T(1)/mr_sqrt({self._print(b)}))"
        if e == sp.Rational(3, 2):
            return f"({bs}*mr_sqrt({self._print(b)}))"
        if e == sp.Rational(-3, 2):
            return f"(T(1)/({bs}*mr_sqrt({self._print(b)})))"
        raise ValueError(f"unsupported power {expr}")

    def _print_Float(self, expr):
        return f"T({float(expr)!r})"

    def _print_Rational(self, expr):
        return f"T({float(expr.p) / float(expr.q)!r})"

    def _print_Integer(self, expr):
        return f"T({int(expr)})"

    def _print_Function(self, expr):
        name = {"sin": "mr_sin", "cos": "mr_cos", "tan": "mr_tan", "atan2": "mr_atan2",
                "sqrt": "mr_sqrt"}.get(type(expr).__name__)
        if name is None:
            raise ValueError(f"unsupported function {expr}")
        return f"{name}(" + ", ".join(self._print(a) for a in expr.args) + ")"

    def _print_atan2(self, expr):
        return f"mr_atan2({self._print(expr.args[0])}, {self._print(expr.args[1])})"

    def _print_sin(self, expr):
        return f"mr_sin({self._print(expr.args[0])})"

    def _print_cos(self, expr):
        return f"mr_cos({self._print(expr.args[0])})"

    def _print_tan(self, expr):
        return f"mr_tan({self._print(expr.args[0])})"


def emit(name, outputs, tyre, with_nu):
    """outputs: list of (c_lvalue, expr)."""
    pr = Printer()
    exprs = [e for _, e in outputs]
    if tyre:
        d, af, ar = slip_angles()
        exprs = [sp.sympify(e).subs({A0F: af, A0R: ar}) for e in exprs]
    repl, red = sp.cse(exprs, symbols=sp.numbered_symbols("t"), optimizations="basic")
    args = "const VehParams<T>& P, T Ts, const T* __restrict__ x, const T* __restrict__ u"
    if with_nu:
        args += ", const T* __restrict__ nu"
    if tyre:
        args += ", const TyreJet<T>& tf, const TyreJet<T>& tr"
    outs = []
    for lv, _ in outputs:
        o = lv.split("[")[0]
        if o not in outs:
            outs.append(o)
    args += "".join(f", T* __restrict__ {o}" for o in outs)
    lines = [f"template <typename T>\nMR_HD void {name}({args}) {{"]
    for sym, e in repl:
        lines.append(f"  const T {sym} = {pr.doprint(e)};")
    for (lv, _), e in zip(outputs, red):
        lines.append(f"  {lv} = {pr.doprint(e)};")
    lines.append("}\n")
    return "\n".join(lines), len(repl)


def model_variants(tag, fexpr, tyre):
    code = []
    fo = [(f"f[{i}]", fexpr[i]) for i in range(6)]
    c, n = emit(f"{tag}_f", fo, tyre, False)
    code.append(c)
    jo = [(f"J[{i * 8 + j}]", sp.diff(fexpr[i], v)) for i in range(6) for j, v in enumerate(INPUTS)]
    c, n2 = emit(f"{tag}_fj", fo + jo, tyre, False)
    code.append(c)
    Lg = sum(NU[i] * fexpr[i] for i in range(6))
    ho = []
    k = 0
    for a in range(8):
        for b in range(a, 8):
            ho.append((f"H[{k}]", sp.diff(Lg, INPUTS[a], INPUTS[b])))
            k += 1
    c, n3 = emit(f"{tag}_fjh", fo + jo + ho, tyre, True)
    code.append(c)
    print(f"{tag}: cse temps f={n} fj={n2} fjh={n3}")
    return "\n".join(code)


def main():
    parts = [
        "// GENERATED by mpc-racing_amd/tools/codegen_models.py -- do not edit.",
        "// Vehicle dynamics of the MPC NLP (control/MPC.py:186-283, models/BlendedBicycleModel.py:22-46,",
        "// learning/vehicle.py:155-160) with exact first/second derivatives.",
        "#pragma once",
        '#include "mr_common.h"',
        "namespace mr {",
    ]
    parts.append(model_variants("kin", f_kin(), False))
    parts.append(model_variants("dyn_lin", f_dyn(False), False))
    parts.append(model_variants("dyn_tyre", f_dyn(True), True))
    parts.append(model_variants("blend_lin", f_blend(False), False))
    parts.append(model_variants("blend_tyre", f_blend(True), True))
    parts.append("}  // namespace mr")
    with open(OUT, "w") as fh:
        fh.write("\n".join(parts) + "\n")
    print("wrote", OUT)


if __name__ == "__main__":
    main()
