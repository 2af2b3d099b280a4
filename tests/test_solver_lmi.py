"""The SDP mirror's per-link LMI matrices (src/solver.py:42-121) and its cvxpy path, on the CPU.

cvxpy and MOSEK are absent here, so phi parity (the SDP's output) stays "needs cvxpy + MOSEK".  What is checked:
  * every constraint matrix against the reference's formulas, restated here element by element, at the prior and
    at random phi (1e-12), and the float32 Q_full the reference builds (src/solver.py:69);
  * the entropic term (src/solver.py:164-172), the float32 prior's metric, and an unknown reg_type (no regulariser);
  * the whole cvxpy path (every reg_type, stacked and Gram-form data terms) driven through tests/fake_cvxpy.py,
    a numeric stand-in that records each constraint at the initial point (the prior) instead of solving.
"""
import sys

import numpy as np
import pytest

from system_identification_amd import solver as S
from system_identification_amd.sys_identification import skew


def ref_pseudo_inertia(phi):  # src/solver.py:53-63, element by element
    mass, h_x, h_y, h_z, I_xx, I_xy, I_xz, I_yy, I_yz, I_zz = phi
    trace = (1 / 2) * (I_xx + I_yy + I_zz)
    return np.array([[trace - I_xx, -I_xy, -I_xz, h_x],
                     [-I_xy, trace - I_yy, -I_yz, h_y],
                     [-I_xz, -I_yz, trace - I_zz, h_z],
                     [h_x, h_y, h_z, mass]])


def ref_com(phi, semi_axes, center):  # src/solver.py:76-93
    mass, h = phi[0], np.asarray(phi[1:4])
    Qs = np.diag(semi_axes) ** 2
    tr = (h - mass * center).reshape(1, 3)
    return np.block([[np.array([[mass]]), tr], [tr.T, mass * Qs]])


def ref_ellipsoid(semi_axes, center):  # src/solver.py:65-74
    Q_full = np.zeros((4, 4), dtype=np.float32)
    Q = np.linalg.inv(np.diag(semi_axes) ** 2)
    Q_full[:3, :3] = Q
    Q_full[:3, 3] = Q @ center
    Q_full[3, :3] = (Q @ center).T
    Q_full[3, 3] = 1 - (center.T @ Q @ center)
    return Q_full


def links():
    """(phi, semi_axes, center) of four physically consistent synthetic links (solid boxes)."""
    out = []
    rng = np.random.default_rng(7)
    for k in range(4):
        semi = rng.uniform(0.05, 0.4, 3)
        center = rng.uniform(-0.1, 0.1, 3)
        mass = rng.uniform(0.5, 5.0)
        com = rng.uniform(-0.05, 0.05, 3)
        dims = rng.uniform(0.05, 0.3, 3)  # a solid box: its inertia meets the triangle inequalities (J > 0)
        R, _ = np.linalg.qr(rng.normal(size=(3, 3)))
        Ic = R @ np.diag(mass / 12 * np.array([dims[1] ** 2 + dims[2] ** 2, dims[0] ** 2 + dims[2] ** 2,
                                                dims[0] ** 2 + dims[1] ** 2])) @ R.T
        Ib = Ic + mass * skew(com) @ skew(com).T
        phi = np.array([mass, *(mass * com), Ib[0, 0], Ib[0, 1], Ib[0, 2], Ib[1, 1], Ib[1, 2], Ib[2, 2]])
        out.append((phi, semi, center))
    return out


def test_lmi_matrices_match_reference_formulas():
    rng = np.random.default_rng(3)
    for phi, semi, center in links():
        for x in (phi, phi + rng.normal(scale=0.1, size=10), rng.normal(size=10)):
            J = S.pseudo_inertia_matrix(x)
            assert np.max(np.abs(J - ref_pseudo_inertia(x))) <= 1e-12 * max(1.0, np.abs(x).max())
            C = S.com_constraint_matrix(x, semi, center)
            assert np.max(np.abs(C - ref_com(x, semi, center))) <= 1e-12 * max(1.0, np.abs(x).max())
            # linear in phi: the basis the cvxpy path builds from reproduces them
            assert np.allclose(np.tensordot(x, S.lmi_basis(S.pseudo_inertia_matrix), 1), J, rtol=0, atol=1e-13)
            assert np.allclose(np.tensordot(x, S.lmi_basis(S.com_constraint_matrix, semi, center), 1), C,
                               rtol=0, atol=1e-13)
            # spatial body inertia (src/solver.py:42-51) = [[I_bar, skew(h)]; [skew(h)^T, m 1]]
            m, h = x[0], x[1:4]
            Ib = np.array([[x[4], x[5], x[6]], [x[5], x[7], x[8]], [x[6], x[8], x[9]]])
            I6 = np.block([[Ib, skew(h)], [skew(h).T, m * np.eye(3)]])
            assert np.max(np.abs(S.spatial_body_inertia_matrix(x) - I6)) <= 1e-15 * max(1.0, np.abs(x).max())
        Qf = S.ellipsoid_matrix(semi, center)
        assert Qf.dtype == np.float32
        assert np.array_equal(Qf, ref_ellipsoid(semi, center))
        # the float32 storage differs from the float64 formula at the 1e-8 level, as in the reference
        Q64 = np.linalg.inv(np.diag(semi) ** 2)
        assert abs(float(Qf[0, 0]) - Q64[0, 0]) <= 1e-7 * Q64[0, 0]


def test_entropic_and_pullback_terms():
    for phi, _, _ in links():
        # the entropic term at the prior: -log det J + log(det J + 1e-5) + trace(pinv(J) J) - 4 ~ 1e-5 / det J
        J = ref_pseudo_inertia(phi)
        d = np.linalg.det(J)
        expect = -np.log(d) + np.log(d + 1e-5) + np.trace(np.linalg.pinv(J) @ J) - 4
        assert abs(S.entropic_divergence(phi, phi) - expect) <= 1e-10
        X_map, ldp = S.entropic_prior_terms(phi)
        assert np.allclose(X_map @ J, np.eye(4), atol=1e-8)
        assert abs(ldp - np.log(d + 1e-5)) <= 1e-12
        M = S.pullback_metric(phi)
        assert np.allclose(M, M.T) and np.min(np.linalg.eigvalsh(M)) > 0


def test_unknown_reg_type_solves_unregularised(monkeypatch):
    """src/solver.py:161-180 is an if / elif chain: any other reg_type adds no regulariser and the problem is solved
    with the data term alone.  The mirror does the same (and warns)."""
    import tests.fake_cvxpy as fcp
    monkeypatch.setitem(sys.modules, "cvxpy", fcp)
    L = links()
    prior = np.concatenate([p for p, _, _ in L])
    ells = [{"semi_axes": s_, "center": c_} for _, s_, c_ in L]
    rng = np.random.default_rng(5)
    Y, tau = rng.normal(size=(40, 10 * len(L))), rng.normal(size=40)
    s = S.Solver(Y, tau, len(L), prior, float(sum(p[0] for p, _, _ in L)), ells)
    with pytest.warns(RuntimeWarning, match="reg_type"):
        s.solve_fully_consistent(lambda_reg=0.1, reg_type="bregman")
    data = 0.5 * float(np.sum((Y @ prior - tau) ** 2)) / 40
    assert abs(s._objective.value - data) <= 1e-12 * max(1.0, data)


def ref_pullback_metric(phi):  # src/solver.py:95-121 (cvxpy's .value: the float64 image of the entries)
    M = np.zeros((10, 10))
    P = ref_pseudo_inertia(phi).astype(np.float64)
    P_inv = np.linalg.inv(P)
    for i in range(10):
        for j in range(10):
            v_i = np.zeros(10)
            v_j = np.zeros(10)
            v_i[i] = 1
            v_j[j] = 1
            V_i = ref_pseudo_inertia(v_i).astype(np.float64)
            V_j = ref_pseudo_inertia(v_j).astype(np.float64)
            M[i, j] = np.trace(P_inv @ V_i @ P_inv @ V_j)
    M = (M + M.T) / 2
    eigenvalues = np.linalg.eigvals(M)
    if np.any(eigenvalues < 0):
        shift = - np.min(eigenvalues) + 1e-5
        M = M + shift * np.eye(M.shape[0])
    return M


def ref_entropic_constants(phi):  # src/solver.py:164-172: X = VT.T @ Sigma_inv @ U.T @ J, log(det(J_prior) + 1e-5)
    J_prior = ref_pseudo_inertia(phi).astype(np.float64)
    U, Sigma, VT = np.linalg.svd(J_prior, full_matrices=True)
    Sigma_inv = np.linalg.pinv(np.diag(Sigma))
    return VT.T @ Sigma_inv @ U.T, np.log(np.linalg.det(J_prior) + 1e-5)


def test_float32_prior_metric_and_entropic_constants_bitwise():
    """The prior is float32 (src/sys_identification.py:61) and the reference unpacks the float32 slice, so its
    pseudo-inertia trace and diagonal are float32 sums (src/solver.py:55-57): the pull-back metric and the entropic
    constants built from it must match the reference's restatement bitwise, and differ from a float64 build."""
    differs = False
    for phi, _, _ in links():
        p32 = phi.astype(np.float32)
        assert np.array_equal(S.pullback_metric(p32), ref_pullback_metric(p32))
        X_map, ldp = S.entropic_prior_terms(p32)
        rX, rl = ref_entropic_constants(p32)
        assert np.array_equal(X_map, rX) and ldp == rl
        differs |= not np.array_equal(S.pullback_metric(p32), S.pullback_metric(p32.astype(np.float64)))
    assert differs  # the float32 sums are visible (the test would not see a float64 build otherwise)
    # the solver mirror hands the raw float32 slice of the prior to both (not a float64 copy)
    import inspect
    src = inspect.getsource(S._solve_fully_consistent_cvxpy)
    assert "pullback_metric(prior_raw)" in src and "entropic_prior_terms(prior_raw)" in src


@pytest.mark.parametrize("reg_type", ["constant_pullback", "entropic", "euclidean"])
@pytest.mark.parametrize("form", ["stacked", "gram"])
def test_cvxpy_path_through_numeric_standin(monkeypatch, reg_type, form):
    """Solver.solve_fully_consistent end to end on tests/fake_cvxpy.py: the constraints CVXPY would receive,
    evaluated at the initial point (the prior), equal the numpy LMI functions; the objective equals the data
    term + regulariser evaluated in numpy; the stacked and Gram-form data terms agree."""
    import tests.fake_cvxpy as fcp
    monkeypatch.setitem(sys.modules, "cvxpy", fcp)
    L = links()
    nl = len(L)
    prior = np.concatenate([p for p, _, _ in L])
    ells = [{"semi_axes": s_, "center": c_} for _, s_, c_ in L]
    rng = np.random.default_rng(11)
    rows, ndof = 60, 3
    Y = rng.normal(size=(rows, 10 * nl))
    Bv, Bc = rng.normal(size=(rows, ndof)), rng.normal(size=(rows, ndof))
    tau = rng.normal(size=rows)
    total = float(sum(p[0] for p, _, _ in L))
    if form == "stacked":
        s = S.Solver(Y, tau, nl, prior, total, ells, B_v=Bv, B_c=Bc)
    else:
        A = np.hstack([Y, Bv, Bc])
        ne = {"gram": A.T @ A, "Atb": A.T @ tau, "btb": float(tau @ tau), "num_rows": rows}
        s = S.Solver.from_normal_equations(ne, nl, prior, total, ells, friction=True)
    phi = s.solve_fully_consistent(lambda_reg=0.1, reg_type=reg_type)
    assert np.array_equal(np.asarray(phi), prior)  # the stand-in does not optimise
    cons = s._problem.constraints
    # per link: mass >= 0, J + eps I >> 0, com + eps I >> 0, trace(J Q) >= 0
    for i, (p, semi, center) in enumerate(L):
        want = S.link_lmi_values(p, semi, center)
        c_mass, c_J, c_com, c_tr = cons[4 * i:4 * i + 4]
        assert c_mass.kind == "ge" and abs(float(c_mass.value) - want["mass"]) <= 1e-15
        assert c_J.kind == "psd" and np.max(np.abs(c_J.value - want["J_reg"])) <= 1e-13
        assert c_com.kind == "psd" and np.max(np.abs(c_com.value - want["com_reg"])) <= 1e-13
        assert c_tr.kind == "ge" and abs(float(c_tr.value) - want["trace_JQ"]) <= 1e-12 * max(1, abs(want["trace_JQ"]))
    assert cons[4 * nl].kind == "eq" and abs(float(cons[4 * nl].value)) <= 1e-12 * total
    # objective at the prior (friction variables start at 0)
    x = np.concatenate([prior, np.zeros(2 * ndof)])
    A = np.hstack([Y, Bv, Bc])
    data = 0.5 * float(np.sum((A @ x - tau) ** 2)) / rows
    if reg_type == "entropic":
        reg = sum(S.entropic_divergence(p, p) for p, _, _ in L)
    else:
        reg = 0.0
    assert abs(s._objective.value - (data + 0.1 * reg)) <= 1e-9 * max(1.0, abs(data))
    assert s._problem.solve_kwargs["solver"] == "MOSEK"
