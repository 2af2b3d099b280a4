"""The contact nullspace projector as K1 computes it (modified Gram-Schmidt, tests/alg_mirror.py)
against the reference's ``P = I - pinv(J_c) J_c`` (src/sys_identification.py:131-135, numpy's pinv with its
default rcond 1e-15).

Both are backward stable in the row space: their distance to the exact projector grows like eps·cond(J_c),
so they agree to ~1e-16·cond.  The north_star bar (1e-6) therefore holds up to cond ~1e9, where pinv's own
answer is already uncertain at that level.  The normal-equations inverse the kernel used before
((J_c J_c^T)^-1, eps·cond^2) failed the bar from cond ~1e5 on; the knee sweep below reaches 5e8 on a
physical configuration (a fixed-base robot standing on nearly straight legs)."""
import numpy as np
import pytest

from oracle import ref_numpy as ref
from system_identification_amd.model import load_robot
from system_identification_amd.synthetic import generate
from tests import alg_mirror as am


def pinv_projector(J):
    return np.eye(J.shape[1]) - np.linalg.pinv(J) @ J


def with_singular_values(rng, k, n, sv):
    U, _ = np.linalg.qr(rng.standard_normal((k, k)))
    V, _ = np.linalg.qr(rng.standard_normal((n, k)))
    return U @ np.diag(sv) @ V.T, V


@pytest.mark.parametrize("cond", [1e0, 1e2, 1e4, 1e6, 1e8])
def test_conditioning_sweep_vs_exact_and_pinv(cond):
    rng = np.random.default_rng(int(np.log10(cond)) + 7)
    for _ in range(10):
        J, V = with_singular_values(rng, 12, 18, 3.0 * np.logspace(0, -np.log10(cond), 12))
        exact = np.eye(18) - V @ V.T
        P = am.projector_mgs(J)
        assert np.abs(P - exact).max() <= 50 * np.finfo(float).eps * cond
        assert np.abs(P - pinv_projector(J)).max() <= 1e-6
        assert np.array_equal(P, P.T)  # bitwise: same products, same summation order


@pytest.mark.parametrize("cnt", [[1, 1, 1, 0], [1, 0, 2, 0], [1, 1, 1, 1]])
def test_near_straight_knees_fixed_base(cnt):
    """solo12_fixed with every knee at eps: one leg's 3x3 Jacobian has cond ~5/eps."""
    m = load_robot("solo12_fixed")
    d = generate(m, 2, config_index=3)
    cnt = np.asarray(cnt, dtype=float)
    knees = [i for i, n in enumerate(m.joint_names) if n.endswith("KFE")]
    assert len(knees) == 4
    for eps in (1e-2, 1e-4, 1e-6, 1e-8, 0.0):
        q = d["q"][:, 0].copy()
        for j in knees:
            q[m.idx_q[j]] = eps
        dd = ref.forward_pass(m, q, d["dq"][:, 0], d["ddq"][:, 0])
        J = ref.compute_J_c(m, dd, cnt)
        P_ref = ref.null_space_projector(m, dd, cnt)
        assert np.abs(am.projector_mgs(J) - P_ref).max() < 1e-6, eps


def test_dependent_zero_and_empty_rows():
    rng = np.random.default_rng(3)
    J = rng.standard_normal((9, 18))
    J = np.vstack([J, 2.0 * J[:3] + J[3:6]])  # three exactly dependent rows
    assert np.abs(am.projector_mgs(J) - pinv_projector(J)).max() < 1e-13
    J[4] = 0.0
    assert np.abs(am.projector_mgs(J) - pinv_projector(J)).max() < 1e-13
    assert np.array_equal(am.projector_mgs(np.zeros((0, 18))), np.eye(18))
    assert np.array_equal(am.projector_mgs(np.zeros((6, 18))), np.eye(18))


def test_projector_identities():
    rng = np.random.default_rng(5)
    J, _ = with_singular_values(rng, 6, 35, np.logspace(0, -3, 6))
    P = am.projector_mgs(J)
    assert np.abs(P @ P - P).max() < 1e-13
    assert np.abs(J @ P).max() < 1e-13
    assert abs(np.trace(P) - 29) < 1e-12


@pytest.mark.parametrize("nv,k", [(18, 12), (18, 6), (35, 6), (35, 3), (18, 0)])
def test_nullspace_rows_factor_the_projector(nv, k):
    """Gram-only mode (north_star "batched QR/nullspace"): K1 emits Zᵀ·A, nv - rank(J_c) rows
    instead of P·A's nv, with Zᵀ from the Householder reconstruction of the MGS basis (tests/alg_mirror.py).
    ZᵀZ = P (so Σ (ZᵀA)ᵀ(ZᵀA) = Σ AᵀPA, the same Gram), ZZᵀ = I, and Z ⊥ J_c; also for dependent rows and
    for well- and ill-conditioned J_c, against the reference's pinv projector."""
    rng = np.random.default_rng(nv + k)
    for trial in range(20):
        J = rng.standard_normal((k, nv))
        if trial % 3 == 1 and k >= 6:
            J[k - 3:] = 2.0 * J[:3] - J[3:6]  # three exactly dependent rows: rank k - 3
        if trial % 3 == 2 and k > 0:
            J, _ = with_singular_values(rng, k, nv, 3.0 * np.logspace(0, -6, k))
        # cond(J_c) = 1e6 on the third kind: MGS's Q is orthonormal to ~eps·cond only, and Z inherits that
        # (the same order as P = I - QᵀQ's own distance to the exact projector, test above)
        tol = 1e-9 if trial % 3 == 2 else 1e-13
        Q = am.mgs_rows(J)
        Zt = am.nullspace_rows(Q)
        r = Q.shape[0]
        assert Zt.shape == (nv - r, nv)
        P = am.projector_mgs(J)
        assert np.abs(Zt.T @ Zt - P).max() < tol
        assert np.abs(Zt @ Zt.T - np.eye(nv - r)).max() < tol
        if k:
            assert np.abs(Zt @ Q.T).max() < tol
            assert np.abs(Zt.T @ Zt - pinv_projector(J)).max() < 1e-9
