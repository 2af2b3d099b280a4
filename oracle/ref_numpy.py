"""CPU ORACLE (test infrastructure only) — numpy fp64 restatement of the reference hot path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module, and only as the checker.  The product path (system_identification_amd) never calls it.

What it restates
----------------
* ``SystemIdentification._update_fk / _compute_J_c / _compute_null_space_proj``
  (src/sys_identification.py:113-135): foot Jacobians in LOCAL_WORLD_ALIGNED (linear rows), stacked
  for every foot with a truthy contact value, ``P = I - pinv(J_c) @ J_c`` with numpy's own ``pinv``
  (rcond 1e-15, exactly as the reference calls it).
* ``get_proj_regressor_torque`` (:401-410) and ``get_proj_friction_regressors`` (:412-418).
* The demo loops and stacking (demo/spot_identification.py:37-56, :84-87).
* pinocchio's ``computeJointTorqueRegressor`` (call site src/sys_identification.py:406) — third-party
  C++ that is NOT installed here (version unpinned, README.md:9).  Restated from its documented
  algorithm: forward pass ``liMi = jointPlacement * M_J(q)``, ``v_i = vJ + liMi^-1 v_parent``,
  ``a_gf_i = S a + v_i x vJ + liMi^-1 a_gf_parent`` with ``a_gf_0 = -gravity``; ``bodyRegressor``;
  backward pass ``Y[rows(j), cols(i)] = S_j^T (jX_i)* bodyRegressor_i`` over the ancestors j of i.

Parity status: **unpinned against pinocchio** (no pinocchio, no reference fixtures, no .dat data).
Pinned instead by build-owned identities (tests/test_oracle_identities.py): Y·phi == an independent
world-frame Newton–Euler, a sympy derivation of the body regressor, finite-difference foot
velocities == J_c·v, and the projector identities.
"""
from __future__ import annotations

import numpy as np

JOINT_FREEFLYER = 1
JOINT_REVOLUTE = 2


# ---- small spatial-algebra helpers (pinocchio conventions: motion = [linear; angular]) ------------

def quat_to_matrix(x, y, z, w):
    """Eigen ``Quaternion::toRotationMatrix`` — no normalisation (pinocchio JointModelFreeFlyer)."""
    tx, ty, tz = 2.0 * x, 2.0 * y, 2.0 * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz = tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    return np.array([
        [1.0 - (tyy + tzz), txy - twz, txz + twy],
        [txy + twz, 1.0 - (txx + tzz), tyz - twx],
        [txz - twy, tyz + twx, 1.0 - (txx + tyy)],
    ])


def axis_rotation(axis, angle):
    """Rotation about a unit axis: pinocchio RX/RY/RZ formulas for the aligned axes."""
    s, c = np.sin(angle), np.cos(angle)
    a = np.asarray(axis, dtype=float)
    if a[0] == 1.0 and a[1] == 0.0 and a[2] == 0.0:
        return np.array([[1.0, 0.0, 0.0], [0.0, c, -s], [0.0, s, c]])
    if a[0] == 0.0 and a[1] == 1.0 and a[2] == 0.0:
        return np.array([[c, 0.0, s], [0.0, 1.0, 0.0], [-s, 0.0, c]])
    if a[0] == 0.0 and a[1] == 0.0 and a[2] == 1.0:
        return np.array([[c, -s, 0.0], [s, c, 0.0], [0.0, 0.0, 1.0]])
    K = np.array([[0.0, -a[2], a[1]], [a[2], 0.0, -a[0]], [-a[1], a[0], 0.0]])
    return np.eye(3) + s * K + (1.0 - c) * (K @ K)


def motion_act_inv(R, t, m):
    """``SE3(R, t).actInv(motion)``: express a motion of the parent frame in the child frame."""
    v, w = m[:3], m[3:]
    return np.concatenate([R.T @ (v - np.cross(t, w)), R.T @ w])


def motion_cross(m1, m2):
    v1, w1 = m1[:3], m1[3:]
    v2, w2 = m2[:3], m2[3:]
    return np.concatenate([np.cross(w1, v2) + np.cross(v1, w2), np.cross(w1, w2)])


def force_act(R, t, F):
    """``SE3(R, t).act`` on a 6xK block of forces (columns [f; n]): child -> parent frame."""
    f = R @ F[:3]
    n = R @ F[3:] + np.cross(t, f, axis=0)
    return np.vstack([f, n])


def body_regressor(v, a):
    """6x10 body regressor: force = Y @ [m, mc, Ixx, Ixy, Iyy, Ixz, Iyz, Izz] for ``f = I a + v x* I v``."""
    vl, w = v[:3], v[3:]
    al, dw = a[:3], a[3:]
    ac = al + np.cross(w, vl)  # classical linear acceleration of the frame origin
    Y = np.zeros((6, 10))
    Y[:3, 0] = ac
    Sdw = np.array([[0.0, -dw[2], dw[1]], [dw[2], 0.0, -dw[0]], [-dw[1], dw[0], 0.0]])
    Sw = np.array([[0.0, -w[2], w[1]], [w[2], 0.0, -w[0]], [-w[1], w[0], 0.0]])
    Sac = np.array([[0.0, -ac[2], ac[1]], [ac[2], 0.0, -ac[0]], [-ac[1], ac[0], 0.0]])
    Y[:3, 1:4] = Sdw + Sw @ Sw
    Y[3:, 1:4] = -Sac

    def bracket(x):  # I @ x == bracket(x) @ [Ixx, Ixy, Iyy, Ixz, Iyz, Izz]
        return np.array([[x[0], x[1], 0.0, x[2], 0.0, 0.0],
                         [0.0, x[0], x[1], 0.0, x[2], 0.0],
                         [0.0, 0.0, 0.0, x[0], x[1], x[2]]])
    Y[3:, 4:] = bracket(dw) + Sw @ bracket(w)
    return Y


# ---- kinematics ----------------------------------------------------------------------------------

class Data:
    pass


def forward_pass(model, q, v, a):
    """Forward pass of computeJointTorqueRegressor + world placements (forwardKinematics)."""
    nj = model.njoints
    d = Data()
    d.liR = [np.eye(3)] * nj
    d.lit = [np.zeros(3)] * nj
    d.oR = [np.eye(3)] * nj
    d.ot = [np.zeros(3)] * nj
    d.v = [np.zeros(6)] * nj
    d.a_gf = [np.zeros(6)] * nj
    d.a_gf[0] = np.concatenate([-np.asarray(model.gravity, dtype=float), np.zeros(3)])
    for i in range(1, nj):
        p = model.parents[i]
        iq, iv = model.idx_q[i], model.idx_v[i]
        if model.jtypes[i] == JOINT_FREEFLYER:
            RJ = quat_to_matrix(q[iq + 3], q[iq + 4], q[iq + 5], q[iq + 6])
            tJ = np.array(q[iq:iq + 3], dtype=float)
            vJ = np.array(v[iv:iv + 6], dtype=float)
            Sa = np.array(a[iv:iv + 6], dtype=float)
        else:
            ax = model.axes[i]
            RJ = axis_rotation(ax, q[iq])
            tJ = np.zeros(3)
            vJ = np.concatenate([np.zeros(3), ax * v[iv]])
            Sa = np.concatenate([np.zeros(3), ax * a[iv]])
        P_R, P_t = model.placements_R[i], model.placements_t[i]
        liR = P_R @ RJ
        lit = P_R @ tJ + P_t
        d.liR[i], d.lit[i] = liR, lit
        vi = vJ.copy()
        if p > 0:
            vi = vi + motion_act_inv(liR, lit, d.v[p])
        d.v[i] = vi
        d.a_gf[i] = motion_cross(vi, vJ) + Sa + motion_act_inv(liR, lit, d.a_gf[p])
        d.oR[i] = d.oR[p] @ liR
        d.ot[i] = d.oR[p] @ lit + d.ot[p]
    return d


def joint_torque_regressor(model, q, v, a, data=None):
    """pinocchio ``computeJointTorqueRegressor(model, data, q, v, a)`` -> (nv, 10*nb)."""
    d = forward_pass(model, q, v, a) if data is None else data
    nv, nb = model.nv, model.nb
    Y = np.zeros((nv, 10 * nb))
    for i in range(nb, 0, -1):
        bR = body_regressor(d.v[i], d.a_gf[i])
        j = i
        while j > 0:
            iv = model.idx_v[j]
            if model.jtypes[j] == JOINT_FREEFLYER:
                Y[iv:iv + 6, 10 * (i - 1):10 * i] = bR
            else:
                Y[iv, 10 * (i - 1):10 * i] = model.axes[j] @ bR[3:]
            if model.parents[j] > 0:
                bR = force_act(d.liR[j], d.lit[j], bR)
            j = model.parents[j]
    return Y


def frame_jacobian_lwa_linear(model, d, frame):
    """``pin.getFrameJacobian(model, data, frame_id, LOCAL_WORLD_ALIGNED)[0:3, :]`` after
    computeJointJacobians: linear velocity of the frame origin, world axes."""
    i = frame.parent
    pf = d.oR[i] @ frame.t + d.ot[i]
    J = np.zeros((3, model.nv))
    j = i
    while j > 0:
        iv = model.idx_v[j]
        if model.jtypes[j] == JOINT_FREEFLYER:
            Rb, pb = d.oR[j], d.ot[j]
            J[:, iv:iv + 3] = Rb
            for k in range(3):
                J[:, iv + 3 + k] = np.cross(Rb[:, k], pf - pb)
        else:
            w = d.oR[j] @ model.axes[j]
            J[:, iv] = np.cross(w, pf - d.ot[j])
        j = model.parents[j]
    return J


def selection_matrix(model):
    """``S`` of src/sys_identification.py:29-37."""
    S = np.zeros((model.nj, model.nv))
    S[:, model.base_dof:] = np.eye(model.nj)
    return S


def compute_J_c(model, d, contact):
    """src/sys_identification.py:119-129, including its quirks: ``m = int(sum(cnt))`` rows of three
    are allocated, feet are added for every truthy value (CONTACT_LOST = 2 counts as contact)."""
    m = int(np.sum(contact))
    J_c = np.zeros((3 * m, model.nv))
    frames = model.contact_frames()
    j = 0
    for index in range(len(frames)):
        if contact[index]:
            J_c[0 + j:3 + j, :] = frame_jacobian_lwa_linear(model, d, frames[index])
            j += 3
    return J_c


def null_space_projector(model, d, contact):
    """src/sys_identification.py:131-135 — ``np.eye(nv) - pinv(J_c) @ J_c``."""
    J_c = compute_J_c(model, d, contact)
    return np.eye(model.nv) - np.linalg.pinv(J_c) @ J_c


def get_proj_regressor_torque(model, q, dq, ddq, tau, cnt):
    """src/sys_identification.py:401-410."""
    q, dq, ddq = (np.asarray(x, dtype=np.float64) for x in (q, dq, ddq))
    d = forward_pass(model, q, dq, ddq)
    Y = joint_torque_regressor(model, q, dq, ddq, data=d)
    P = null_space_projector(model, d, cnt)
    return P @ Y, P @ selection_matrix(model).T @ tau


def get_proj_friction_regressors(model, q, dq, ddq, cnt):
    """src/sys_identification.py:412-418."""
    q, dq, ddq = (np.asarray(x, dtype=np.float64) for x in (q, dq, ddq))
    d = forward_pass(model, q, dq, ddq)
    P = null_space_projector(model, d, cnt)
    S = selection_matrix(model)
    bd = model.base_dof
    return P @ S.T @ np.diag(dq[bd:]), P @ S.T @ np.diag(np.sign(dq[bd:]))


def compute_lambda(model, force, cnt):
    """src/sys_identification.py:137-146 (m = int(sum(cnt)) entries, one 3-block per truthy foot)."""
    m = int(np.sum(cnt))
    lam = np.zeros(3 * m)
    j = 0
    for i in range(len(model.contact_frames())):
        if cnt[i]:
            lam[j:j + 3] = force[3 * i:3 * (i + 1)]
            j += 3
    return lam


def get_full_regressor_force(model, q, dq, ddq, tau, ee_force, cnt):
    """src/sys_identification.py:391-399: Y (unprojected) and F = S^T tau + J_c^T lambda."""
    q, dq, ddq = (np.asarray(x, dtype=np.float64) for x in (q, dq, ddq))
    d = forward_pass(model, q, dq, ddq)
    Y = joint_torque_regressor(model, q, dq, ddq, data=d)
    J_c = compute_J_c(model, d, cnt)
    lam = compute_lambda(model, np.asarray(ee_force, dtype=np.float64), cnt)
    F = selection_matrix(model).T @ np.asarray(tau, dtype=np.float64) + J_c.T @ lam
    return Y, F


def get_projected_y_tau(model, q, dq, ddq, torque, cnt):
    """demo/spot_identification.py:37-45 + :84-85 (per-sample loop, vstack/hstack)."""
    Y, T = [], []
    for i in range(q.shape[1]):
        y, t = get_proj_regressor_torque(model, q[:, i], dq[:, i], ddq[:, i], torque[:, i], cnt[:, i])
        Y.append(y)
        T.append(t)
    return np.vstack(Y), np.hstack(T)


def get_projected_friction_regressors(model, q, dq, ddq, cnt):
    """demo/spot_identification.py:47-56 + :86-87."""
    BV, BC = [], []
    for i in range(q.shape[1]):
        bv, bc = get_proj_friction_regressors(model, q[:, i], dq[:, i], ddq[:, i], cnt[:, i])
        BV.append(bv)
        BC.append(bc)
    return np.vstack(BV), np.vstack(BC)


def normal_equations(Y_proj, tau_proj, B_v, B_c):
    """The Gram the Solver's objective implies (solver.py:186-190): with A = [Y | B_v | B_c] and
    b = tau, returns (A^T A, A^T b, b^T b, rows)."""
    A = np.hstack([Y_proj, B_v, B_c])
    return A.T @ A, A.T @ tau_proj, float(tau_proj @ tau_proj), A.shape[0]
