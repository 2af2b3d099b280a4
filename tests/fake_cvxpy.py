"""A numeric stand-in for the few cvxpy names solver.py's SDP path uses (test infrastructure, not cvxpy).

cvxpy and MOSEK are not installed in this image, so the real solve cannot run here.  This module evaluates every
expression at the variables' values (numpy), records each constraint with the matrix or value it constrains, and
its Problem.solve only records its arguments and reports "optimal" (the variables keep their initial values: no
optimisation happens).  It lets a CPU test drive Solver.solve_fully_consistent end to end and read back exactly
what the SDP would have been given, at the initial point.
"""
import numpy as np

MOSEK = "MOSEK"
OPTIMAL = "optimal"
OPTIMAL_INACCURATE = "optimal_inaccurate"


class Constraint:
    def __init__(self, kind, value):
        self.kind = kind            # "psd" (value >> 0), "ge" (value >= 0), "eq" (value == 0)
        self.value = np.asarray(value, dtype=np.float64)


class Expr(np.ndarray):
    __array_priority__ = 1000

    def __new__(cls, a):
        return np.array(a, dtype=np.float64).view(cls)

    def __array_wrap__(self, arr, context=None, return_scalar=False):
        return np.asarray(arr).view(Expr)

    def __getitem__(self, k):
        return Expr(np.asarray(self)[k])

    @property
    def value(self):
        return np.asarray(self)

    def __rshift__(self, other):
        return Constraint("psd", np.asarray(self) - np.asarray(other))

    def __ge__(self, other):
        return Constraint("ge", np.asarray(self) - np.asarray(other))

    def __eq__(self, other):
        return Constraint("eq", np.asarray(self) - np.asarray(other))

    __hash__ = None


def Variable(n, value=None):
    return Expr(np.zeros(n) if value is None else value)


def Constant(x):
    return Expr(x)


def reshape(x, shape, order="F"):
    return Expr(np.reshape(np.asarray(x), shape, order=order))


def hstack(xs):
    return Expr(np.hstack([np.atleast_1d(np.asarray(x)) for x in xs]))


def vstack(xs):
    return Expr(np.vstack([np.asarray(x) for x in xs]))


def trace(x):
    return Expr(np.trace(np.asarray(x)))


def quad_form(x, M):
    x = np.asarray(x)
    return Expr(x @ np.asarray(M) @ x)


def sum_squares(x):
    x = np.asarray(x)
    return Expr(np.sum(x * x))


def log_det(x):
    sign, ld = np.linalg.slogdet(np.asarray(x))
    return Expr(ld if sign > 0 else -np.inf)


def log(x):
    return Expr(np.log(np.asarray(x)))


class Minimize:
    def __init__(self, expr):
        self.expr = expr
        self.value = float(np.asarray(expr))


class Problem:
    def __init__(self, objective, constraints):
        self.objective = objective
        self.constraints = list(constraints)
        self.status = None
        self.solve_kwargs = None

    def solve(self, **kwargs):
        self.solve_kwargs = kwargs
        self.status = OPTIMAL
        return self.objective.value
