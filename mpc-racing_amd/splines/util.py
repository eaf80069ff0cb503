"""Drop-in ``splines.util`` (splines/util.py:3-19): planar point helpers used for the
track-closing point (ParameterizedCenterline.from_file, alpha = 0.9)."""
from math import sqrt


def euclidean(p1, p2):
    return sqrt((p1[0] - p2[0]) ** 2 + (p1[1] - p2[1]) ** 2)


def midpoint(p1, p2, alpha=0.5):
    return (p2[0] - p1[0]) * alpha + p1[0], (p2[1] - p1[1]) * alpha + p1[1]


def interpolate(p1, p2, eps):
    """Points from p1 to p2 by recursive halving until neighbours are within eps."""
    if euclidean(p1, p2) <= eps:
        return p1, p2
    mid = midpoint(p1, p2)
    return interpolate(p1, mid, eps)[:-1] + interpolate(mid, p2, eps)
