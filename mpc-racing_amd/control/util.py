"""Helpers of the reference's control/util.py:4-11 (numeric, no CasADi)."""


def make_poly(variable, coeffs):
    """Evaluate the polynomial with coefficients ``coeffs`` (highest order first) at ``variable``."""
    acc = 0
    for c in coeffs:  # Horner
        acc = acc * variable + c
    return acc


def deg2rad(z):
    """Degrees to radians with pi approximated by 3.14, as the reference does."""
    return z / 360 * 2 * 3.14
