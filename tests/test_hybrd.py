"""sgv_fsolve (csrc/hybrd.cpp, the library's restatement of MINPACK hybrd as
scipy.optimize.fsolve drives it) against scipy 1.15.3's fsolve itself: the same
iterates bit for bit and the same `ier` on smooth, singular and rootless systems,
and on the reference's MLE Lagrangian (src/sgvamp.py:139-160, evaluated here with
NumPy as the reference does).  Host only: no GPU."""
import numpy as np
import pytest
from scipy import optimize

import hip_backend as hb


def rosenbrock(x):
    return np.array([10.0 * (x[1] - x[0] ** 2), 1.0 - x[0]])


def powell_singular(x):   # singular Jacobian at the root: fsolve stops with ier 5
    return np.array([x[0] + 10 * x[1], np.sqrt(5.0) * (x[2] - x[3]), (x[1] - 2 * x[2]) ** 2,
                     np.sqrt(10.0) * (x[0] - x[3]) ** 2])


def trigonometric(x):
    n = x.size
    return n - np.sum(np.cos(x)) + np.arange(1, n + 1) * (1 - np.cos(x)) - np.sin(x)


def mixed(x):
    return np.array([x[0] ** 2 + x[1] ** 2 - 4, x[0] * x[1] - 1, x[2] ** 3 - x[0]])


def rootless(x):
    return np.array([x[0] ** 2 + 1.0, x[1] - 2.0])


def brown_almost_linear(x):
    n = x.size
    f = x + np.sum(x) - (n + 1)
    f[-1] = np.prod(x) - 1.0
    return f


CASES = [(rosenbrock, [-1.2, 1.0]), (rosenbrock, [0.0, 0.0]),
         (powell_singular, [3.0, -1.0, 0.0, 1.0]), (trigonometric, np.full(6, 1 / 6)),
         (trigonometric, np.full(9, 0.5)), (mixed, [1.5, 0.5, 1.0]), (rootless, [0.3, 0.0]),
         (brown_almost_linear, np.full(5, 0.5)), (brown_almost_linear, np.full(8, 0.9))]


@pytest.mark.parametrize("i", range(len(CASES)))
def test_fsolve_matches_scipy_bitwise(i):
    f, x0 = CASES[i]
    xs, info, ier, _ = optimize.fsolve(f, np.array(x0, dtype=np.float64), full_output=True)
    xh, ih, nfev = hb.fsolve(f, x0)
    assert ih == ier, (f.__name__, ih, ier)
    assert np.array_equal(xh, xs), (f.__name__, np.max(np.abs(xh - xs)))
    # scipy's count includes its wrapper's shape probe and one more call
    assert nfev == info["nfev"] - 2


def reference_lagrangian(L, K, M, a, r1s, gam1s, sigma2, omega0):
    """src/sgvamp.py:139-160 verbatim in NumPy (r1s (K, M))."""
    def f(x):
        y = np.zeros(L + 1)
        omega = x[:L]
        gam = x[L]
        prior_vars0 = sigma2.reshape(1, 1, L)
        gam1invs = 1.0 / gam1s.reshape(K, 1, 1)
        r1s_rs = r1s.reshape(K, M, 1)
        omega_rs = omega.reshape(1, 1, L)
        exp_max = (-np.power(r1s_rs, 2).reshape(K, M, 1) / 2 / (prior_vars0 + gam1invs)).max()
        probs = np.exp(-np.power(r1s_rs, 2) / 2 / (prior_vars0 + gam1invs) - exp_max) / \
            np.sqrt(prior_vars0 + gam1invs)
        num = a.reshape(K, 1, 1) * probs
        den = np.sum(probs * omega_rs, axis=2).reshape(K, M, 1)
        y[:L] = np.sum(num / den, axis=(0, 1)) + (omega0 - 1) / omega + gam
        y[L] = sum(omega) - 1.0
        return y
    return f


@pytest.mark.parametrize("seed,K,nslab,lam", [(0, 1, 1, 0.1), (1, 3, 2, 0.3), (2, 2, 3, 0.05),
                                              (3, 4, 1, 0.5)])
def test_fsolve_on_the_reference_lagrangian(seed, K, nslab, lam):
    """The MLE prior update's solve (src/sgvamp.py:173-179) on a mixture-like r1:
    the library's solver takes scipy's steps exactly."""
    rs = np.random.RandomState(seed)
    M = 4000
    L = nslab + 1
    sig = np.sort(rs.uniform(0.5, 3.0, nslab))
    z = rs.rand(K, M) < lam
    r1s = np.where(z, rs.normal(0, 1.5, (K, M)), 0.0) + rs.normal(0, 0.4, (K, M))
    gam1s = rs.uniform(3.0, 8.0, K)
    a = np.full(K, 1.0 / K)
    omegas = rs.dirichlet(np.ones(nslab))
    omega0 = np.concatenate([[1 - lam], lam * omegas])
    sigma2 = np.concatenate([[1e-16], sig])
    x0 = np.concatenate([omega0, [1.0]])
    f = reference_lagrangian(L, K, M, a, r1s, gam1s, sigma2, omega0)
    xs, _, ier, _ = optimize.fsolve(f, x0, full_output=True)
    xh, ih, _ = hb.fsolve(f, x0)
    assert ih == ier
    assert np.array_equal(xh, xs)


def test_fsolve_callback_error_stops_the_solver():
    calls = []

    def f(x):
        calls.append(1)
        if len(calls) > 3:
            raise ValueError("stop")
        return x - 1.0

    with pytest.raises(ValueError):
        hb.fsolve(f, [0.0, 0.0])
