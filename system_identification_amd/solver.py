"""``Solver`` — drop-in for src/solver.py:5, plus the Gram-compressed input.

The reference hands CVXPY the stacked N·nv x W matrices (solver.py:186-190).  The engine produces the
normal equations instead (G = AᵀA, g = Aᵀb, bᵀb, num_rows), so this Solver accepts either form:

    Solver(Y_proj, tau_proj, num_links, phi_prior, total_mass, ellipsoids, B_v=..., B_c=...)   # reference
    Solver.from_normal_equations(ne, num_links, phi_prior, total_mass, ellipsoids, friction=True)

With the Gram, ``sum_squares(A x - b)`` becomes ``sum_squares(R x) - 2 gᵀx + bᵀb`` (R = chol(G)ᵀ), so CVXPY
sees W rows instead of N·nv and the 1/(N·nv) scale of solver.py:190 is kept via ``num_rows``.

``solve_llsq_svd`` (solver.py:32-39) is plain numpy.  ``solve_fully_consistent`` (:123-210) needs cvxpy and
the MOSEK licence exactly like the reference; neither is installed in this project's images, so it raises
ImportError there (φ parity is unverifiable without them — SURVEY.md §8c).
"""
from __future__ import annotations

import numpy as np


class Solver():
    def __init__(self, regressor, tau_vec, num_links, phi_prior, total_mass, bounding_ellipsoids, B_v=None, B_c=None,
                 *, normal_equations=None):
        if normal_equations is None:
            self._Y = np.asarray(regressor)
            self._tau = np.asarray(tau_vec)
            self._nx = self._Y.shape[1]
            self._num_samples = self._Y.shape[0]          # rows = N·nv, the objective's divisor
            self._gram = None
        else:
            ne = normal_equations
            self._Y = None
            self._tau = None
            self._gram = ne
            self._nx = int(ne["nx"])
            self._num_samples = int(ne["num_rows"])
        self._num_links = num_links
        self._num_inertial_params = self._nx // self._num_links
        self._phi_prior = phi_prior
        self.total_mass = total_mass
        self._bounding_ellipsoids = bounding_ellipsoids
        self._identify_fric = (B_v is not None and B_c is not None) or (
            normal_equations is not None and normal_equations.get("ndof", 0) > 0)
        if self._identify_fric:
            self._B_v, self._B_c = B_v, B_c
            self.ndof = B_v.shape[1] if B_v is not None else int(normal_equations["ndof"])
        self._objective = None
        self._constraints = []
        self._problem = None

    @classmethod
    def from_normal_equations(cls, ne: dict, num_links, phi_prior, total_mass, bounding_ellipsoids,
                              friction: bool = True, ndof: int | None = None):
        """``ne`` as returned by SystemIdentification.build_normal_equations (gram is W x W with
        W = 10·num_links + 2·ndof when friction columns are present)."""
        W = ne["gram"].shape[0]
        nphi = 10 * num_links
        nd = (W - nphi) // 2 if friction else 0
        if ndof is not None and friction and ndof != nd:
            raise ValueError("ndof does not match the Gram size")
        d = dict(ne)
        d["nx"] = nphi
        d["ndof"] = nd
        d["W"] = W
        return cls(None, None, num_links, phi_prior, total_mass, bounding_ellipsoids, normal_equations=d)

    # -------------- Unconstrained Solver -------------- #
    def solve_llsq_svd(self):
        """solver.py:32-39: minimum-norm least squares of Y phi = tau (friction columns not used)."""
        if self._gram is None:
            U, Sigma, VT = np.linalg.svd(self._Y, full_matrices=False)
            Sigma_inv = np.linalg.pinv(np.diag(Sigma))
            return VT.T @ Sigma_inv @ U.T @ self._tau
        # the minimum-norm solution from the normal equations, x = pinv(G_YY) g_Y.  The eigenvalues of the Gram
        # carry an absolute error of about n eps w_max (the squaring loses what the SVD of Y keeps), so the
        # rank cut is taken at that level (numpy's matrix_rank tolerance for G), not at the 1e-15 sigma_max
        # of the stacked SVD: a smaller cut keeps the noise eigenvalues of the structurally unidentifiable
        # parameter combinations and divides rounding noise of g by rounding noise of w.  The directions cut
        # are those with sigma below sqrt(n eps) sigma_max (~2e-7 for Spot) — the noise floor of this form.
        n = self._nx
        G = self._gram["gram"][:n, :n]
        g = self._gram["Atb"][:n]
        w, V = np.linalg.eigh(0.5 * (G + G.T))
        wmax = float(w.max()) if w.size else 0.0
        keep = w > max(wmax, 0.0) * n * np.finfo(np.float64).eps
        return V[:, keep] @ ((V[:, keep].T @ g) / w[keep])

    # ------------ Constrained Solver (LMI) ------------ #
    def solve_fully_consistent(self, lambda_reg=1e-1, tol=1e-10, max_iters=1000, reg_type="constant_pullback"):
        """solver.py:123-210.  ``reg_type`` is one of REG_TYPES.  Any other name solves without a regulariser, as the
        reference does (its if / elif chain, solver.py:161-180, adds nothing for it); this mirror also warns."""
        if reg_type not in REG_TYPES:
            import warnings
            warnings.warn(f"unknown reg_type {reg_type!r} (expected one of {REG_TYPES}): solving without a "
                          "regulariser, as src/solver.py does", RuntimeWarning, stacklevel=2)
        try:
            import cvxpy as cp  # noqa: F401
        except ImportError as exc:  # pragma: no cover - depends on the host image
            raise ImportError("solve_fully_consistent needs cvxpy and MOSEK (src/solver.py:2,195), which are not "
                              "installed; use solve_llsq_svd or install them on the solving host") from exc
        return _solve_fully_consistent_cvxpy(self, lambda_reg, tol, max_iters, reg_type)


REG_TYPES = ("constant_pullback", "entropic", "euclidean")


# ---- per-link LMI matrices of the SDP (src/solver.py:42-121), numpy -----------------------------------------
# phi = [m, h_x, h_y, h_z, I_xx, I_xy, I_xz, I_yy, I_yz, I_zz] (the order solver.py:44 / :55 unpack).  Every
# matrix below is linear in phi, so the cvxpy path builds it as sum_k phi_k B_k from the basis these functions
# give (lmi_basis): one definition serves the numeric checks and the SDP, and the coefficients CVXPY sees are
# exactly the numbers the reference's hstack / vstack expressions carry.
def spatial_body_inertia_matrix(phi):
    """solver.py:42-51 — the 6x6 spatial body inertia [[I, h x]; [(h x)^T, m 1]] as the reference lays it out."""
    m, hx, hy, hz, Ixx, Ixy, Ixz, Iyy, Iyz, Izz = np.asarray(phi, dtype=np.float64)
    return np.array([[Ixx, Ixy, Ixz, 0.0, -hz, hy],
                     [Ixy, Iyy, Iyz, hz, 0.0, -hx],
                     [Ixz, Iyz, Izz, -hy, hx, 0.0],
                     [0.0, hz, -hy, m, 0.0, 0.0],
                     [-hz, 0.0, hx, 0.0, m, 0.0],
                     [hy, -hx, 0.0, 0.0, 0.0, m]])


def pseudo_inertia_matrix(phi):
    """solver.py:53-63 — J (4x4): [[tr/2 - I_xx, -I_xy, -I_xz, h_x], ..., [h_x, h_y, h_z, m]], tr = I_xx+I_yy+I_zz.
    The entries are formed in phi's own dtype, as the reference's unpacking of a numpy slice does: the prior is
    float32 (src/sys_identification.py:61), so its trace and diagonal are float32 sums (numpy 2 keeps the Python
    scalar 1/2 weak), and only the finished matrix is float64 (cvxpy's `.value`)."""
    phi = np.asarray(phi)
    if phi.dtype not in (np.float32, np.float64):
        phi = phi.astype(np.float64)
    m, hx, hy, hz, Ixx, Ixy, Ixz, Iyy, Iyz, Izz = phi
    tr = (1 / 2) * (Ixx + Iyy + Izz)
    return np.array([[tr - Ixx, -Ixy, -Ixz, hx],
                     [-Ixy, tr - Iyy, -Iyz, hy],
                     [-Ixz, -Iyz, tr - Izz, hz],
                     [hx, hy, hz, m]], dtype=np.float64)


def ellipsoid_matrix(semi_axes, center):
    """solver.py:65-74 — Q_full (4x4) of the bounding ellipsoid, stored in float32 as the reference stores it
    (the products are formed in the inputs' precision, then rounded once into the float32 matrix)."""
    semi_axes, center = np.asarray(semi_axes), np.asarray(center)
    Q_full = np.zeros((4, 4), dtype=np.float32)
    Q = np.linalg.inv(np.diag(semi_axes) ** 2)
    Q_full[:3, :3] = Q
    Q_full[:3, 3] = Q @ center
    Q_full[3, :3] = (Q @ center).T
    Q_full[3, 3] = 1 - (center.T @ Q @ center)
    return Q_full


def com_constraint_matrix(phi, semi_axes, center):
    """solver.py:76-93 — [[m, (h - m c)^T]; [h - m c, m diag(semi_axes)^2]]."""
    phi = np.asarray(phi, dtype=np.float64)
    m, h = phi[0], phi[1:4]
    Qs = np.diag(np.asarray(semi_axes)) ** 2
    top = (h - m * np.asarray(center)).reshape(1, 3)
    return np.block([[np.array([[m]]), top], [top.T, m * Qs]])


def lmi_basis(fn, *args):
    """B[k] = fn(e_k, *args) for the 10 unit vectors: fn(phi, *args) == sum_k phi_k B[k] for a linear fn."""
    return np.stack([fn(np.eye(10)[k], *args) for k in range(10)])


def pullback_metric(phi_prior_link):
    """solver.py:95-121 — constant pull-back approximation of the Riemannian metric at the prior."""
    M = np.zeros((10, 10))
    P_inv = np.linalg.inv(pseudo_inertia_matrix(phi_prior_link))
    for i in range(10):
        for j in range(10):
            vi = np.zeros(10)
            vj = np.zeros(10)
            vi[i] = 1
            vj[j] = 1
            M[i, j] = np.trace(P_inv @ pseudo_inertia_matrix(vi) @ P_inv @ pseudo_inertia_matrix(vj))
    M = (M + M.T) / 2
    ev = np.linalg.eigvals(M)
    if np.any(ev < 0):
        M = M + (-np.min(ev) + 1e-5) * np.eye(10)
    assert np.min(np.linalg.eigvals(M)) > 0
    return M


def entropic_prior_terms(phi_prior_link):
    """solver.py:164-172 — the constants of the entropic (log-det Bregman) term at the prior: X_map with
    X = X_map @ J (the SVD pseudo-inverse of J_prior, VT.T @ pinv(diag(Sigma)) @ U.T) and log(det(J_prior) + 1e-5)."""
    J_prior = pseudo_inertia_matrix(phi_prior_link)
    U, Sigma, VT = np.linalg.svd(J_prior, full_matrices=True)
    Sigma_inv = np.linalg.pinv(np.diag(Sigma))
    return VT.T @ Sigma_inv @ U.T, float(np.log(np.linalg.det(J_prior) + 1e-5))


def entropic_divergence(phi_link, phi_prior_link):
    """The value of the reference's entropic regulariser for one link at a numeric phi (solver.py:172):
    -log det J + log(det J_prior + 1e-5) + trace(X) - 4, X = pinv_svd(J_prior) J."""
    X_map, log_det_prior = entropic_prior_terms(phi_prior_link)
    J = pseudo_inertia_matrix(phi_link)
    sign, logdet = np.linalg.slogdet(J)
    if sign <= 0:
        return np.inf
    return -logdet + log_det_prior + float(np.trace(X_map @ J)) - 4.0


def link_lmi_values(phi_link, semi_axes, center, epsilon=1e-6):
    """The constraint matrices of one link as solve_fully_consistent states them (solver.py:139-157), at a
    numeric phi: J + eps I (>> 0), com + eps I (>> 0), trace(J Q_full) (>= 0), mass (>= 0)."""
    J = pseudo_inertia_matrix(phi_link)
    return {"J_reg": J + epsilon * np.eye(4),
            "com_reg": com_constraint_matrix(phi_link, semi_axes, center) + epsilon * np.eye(4),
            "trace_JQ": float(np.trace(J @ ellipsoid_matrix(semi_axes, center))),
            "mass": float(np.asarray(phi_link)[0])}


def gram_data_term(G, g, btb):
    """The Gram form of the data term of solver.py:186-190: sum_squares(A x - b) == ‖R x‖² - 2 gᵀx + bᵀb for
    G = AᵀA, g = Aᵀb, with R = diag(sqrt(max(w, 0))) Vᵀ from the eigendecomposition G = V diag(w) Vᵀ (the
    clip drops the rounding-level negative eigenvalues of a PSD Gram).  Returns (R, g, btb): the W x W factor
    that CVXPY sees instead of the N·nv x W stacked matrix, and the linear / constant terms."""
    G = np.asarray(G, dtype=np.float64)
    w, V = np.linalg.eigh(0.5 * (G + G.T))
    R = (V * np.sqrt(np.clip(w, 0.0, None))).T
    return R, np.asarray(g, dtype=np.float64), float(btb)


def gram_data_value(R, g, btb, x):
    """The value of the data term for a numeric x (what CVXPY minimises, evaluated with numpy)."""
    Rx = R @ np.asarray(x, dtype=np.float64)
    return float(Rx @ Rx - 2.0 * (g @ x) + btb)


def _affine(cp, p, basis):
    """sum_k p[k] basis[k] as a CVXPY expression (basis: (10, r, c) constants): vec_F of the matrix is
    basis_F @ p, reshaped column-major (CVXPY's default order)."""
    r, c = basis.shape[1:]
    Bf = np.stack([basis[k].reshape(-1, order="F") for k in range(10)], axis=1)  # (r c, 10)
    return cp.reshape(Bf @ p, (r, c), order="F")


def _solve_fully_consistent_cvxpy(s: Solver, lambda_reg, tol, max_iters, reg_type):
    """solver.py:123-210 with the LMI matrices from the numpy functions above (lmi_basis); the data term from the
    stacked arrays (reference form) or from the normal equations (gram_data_term)."""
    import cvxpy as cp
    nx = s._nx
    phi = cp.Variable(nx, value=np.asarray(s._phi_prior, dtype=float))
    cons = []
    reg = 0
    mass_sum = 0
    eps = 1e-6
    PI = lmi_basis(pseudo_inertia_matrix)
    for idx in range(s._num_links):
        j = idx * s._num_inertial_params
        p = phi[j:j + s._num_inertial_params]
        # the prior slice keeps its dtype (float32 from get_phi_prior) for the metric and the entropic constants,
        # whose pseudo-inertia sums the reference forms in that dtype; as a cvxpy constant it is exact in float64
        prior_raw = np.asarray(s._phi_prior[j:j + s._num_inertial_params])
        prior = prior_raw.astype(np.float64)
        ell = s._bounding_ellipsoids[idx]
        semi, center = np.asarray(ell["semi_axes"]), np.asarray(ell["center"])
        cons.append(p[0] >= 0)
        mass_sum += p[0]
        J = _affine(cp, p, PI)
        cons.append(J + eps * cp.Constant(np.eye(4)) >> 0)
        com = _affine(cp, p, lmi_basis(com_constraint_matrix, semi, center))
        cons.append(com + eps * cp.Constant(np.eye(4)) >> 0)
        cons.append(cp.trace(J @ ellipsoid_matrix(semi, center)) >= 0)
        if reg_type == "constant_pullback":
            reg += 0.5 * cp.quad_form(p - prior, pullback_metric(prior_raw))
        elif reg_type == "entropic":
            # solver.py:164-172 (the reference notes that this form may not converge)
            X_map, log_det_prior = entropic_prior_terms(prior_raw)
            reg += -cp.log_det(J) + log_det_prior + cp.trace(X_map @ J) - 4
    if reg_type == "euclidean":
        reg = cp.quad_form(phi - np.asarray(s._phi_prior, dtype=float), np.eye(nx))
    cons.append(mass_sum == s.total_mass)
    if s._gram is None:
        if s._identify_fric:
            bv, bc = cp.Variable(s.ndof), cp.Variable(s.ndof)
            cons += [bv >= 0, bc >= 0]
            err = cp.sum_squares(s._Y @ phi + s._B_v @ bv + s._B_c @ bc - s._tau)
        else:
            err = cp.sum_squares(s._Y @ phi - s._tau)
    else:
        G, g, btb = s._gram["gram"], s._gram["Atb"], s._gram["btb"]
        if s._identify_fric:
            bv, bc = cp.Variable(s.ndof), cp.Variable(s.ndof)
            cons += [bv >= 0, bc >= 0]
            x = cp.hstack([phi, bv, bc])
        else:
            x = phi
            G, g = G[:nx, :nx], g[:nx]
        R, g, btb = gram_data_term(G, g, btb)
        err = cp.sum_squares(R @ x) - 2 * g @ x + btb
    s._constraints = cons
    s._objective = cp.Minimize(0.5 * err / s._num_samples + lambda_reg * reg)
    s._problem = cp.Problem(s._objective, cons)
    try:
        s._problem.solve(solver=cp.MOSEK, mosek_params={"MSK_IPAR_INTPNT_SOLVE_FORM": "MSK_SOLVE_PRIMAL",
                                                         "MSK_DPAR_INTPNT_TOL_REL_GAP": tol,
                                                         "MSK_DPAR_OPTIMIZER_MAX_TIME": 100.0,
                                                         "MSK_IPAR_INTPNT_MAX_ITERATIONS": max_iters}, verbose=True)
    except Exception as e:  # noqa: BLE001 - solver.py:200-201 prints and falls through to the status check
        print(e)
    if s._problem.status in (cp.OPTIMAL, cp.OPTIMAL_INACCURATE):
        return phi.value
    print("The problem did not solve to optimality. Status:", s._problem.status)
    raise ValueError("The problem did not solve to optimality.")


# ---- checkpoint of the normal equations (the Gram is tiny; resume the SDP without the data) --
def save_normal_equations(path, ne: dict) -> None:
    """Write {gram, Atb, btb, num_rows} to an .npz (plain arrays, no pickle)."""
    np.savez(path, gram=np.asarray(ne["gram"], dtype=np.float64), Atb=np.asarray(ne["Atb"], dtype=np.float64),
             btb=np.float64(ne["btb"]), num_rows=np.int64(ne["num_rows"]))


def load_normal_equations(path) -> dict:
    with np.load(path, allow_pickle=False) as z:
        return {"gram": z["gram"].copy(), "Atb": z["Atb"].copy(), "btb": float(z["btb"]),
                "num_rows": int(z["num_rows"])}
