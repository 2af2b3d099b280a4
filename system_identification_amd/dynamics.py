"""Host-side inverse dynamics, vectorised over samples (world-frame classical Newton–Euler).

Used to synthesise physically consistent torque logs (``tau = S · ID(q, dq, ddq)``) in the
``.dat`` channel layout the reference reads (demo/spot_identification.py:9-34), since the
reference ships no data (.gitignore:9-11).  It is deliberately a *different* formulation from the
regressor path (world frame, point accelerations, subtree wrenches) so the test-suite can use it as an
independent check of ``Y(q, dq, ddq) · phi == tau``.

Conventions follow pinocchio (the reference's dynamics library):
* q = [x y z qx qy qz qw, joints] for a free-flyer (README.md:55-57), dq/ddq = [v_local; w_local, joints];
* the base velocity is expressed in the LOCAL base frame and ddq[0:6] is its time derivative;
* the returned generalized force has the base wrench (local frame, force first) in rows 0-5.
"""
from __future__ import annotations

import numpy as np

from .model import JOINT_FREEFLYER, Model


def _quat_to_matrix(q4: np.ndarray) -> np.ndarray:
    """(N, 4) quaternions (x, y, z, w) -> (N, 3, 3), Eigen's non-normalising formula."""
    x, y, z, w = (q4[:, k] for k in range(4))
    tx, ty, tz = 2 * x, 2 * y, 2 * z
    R = np.empty((q4.shape[0], 3, 3))
    R[:, 0, 0] = 1 - (ty * y + tz * z)
    R[:, 0, 1] = ty * x - tz * w
    R[:, 0, 2] = tz * x + ty * w
    R[:, 1, 0] = ty * x + tz * w
    R[:, 1, 1] = 1 - (tx * x + tz * z)
    R[:, 1, 2] = tz * y - tx * w
    R[:, 2, 0] = tz * x - ty * w
    R[:, 2, 1] = tz * y + tx * w
    R[:, 2, 2] = 1 - (tx * x + ty * y)
    return R


def _axis_rotation(axis: np.ndarray, ang: np.ndarray) -> np.ndarray:
    s, c = np.sin(ang), np.cos(ang)
    K = np.array([[0.0, -axis[2], axis[1]], [axis[2], 0.0, -axis[0]], [-axis[1], axis[0], 0.0]])
    return np.eye(3)[None] + s[:, None, None] * K[None] + (1 - c)[:, None, None] * (K @ K)[None]


def _mv(R, x):
    """Batched 3x3 matrix-vector products, written out (np.einsum on 3x3 blocks cost 3/4 of a G1 1M synthesis)."""
    return R[:, :, 0] * x[:, None, 0] + R[:, :, 1] * x[:, None, 1] + R[:, :, 2] * x[:, None, 2]


def _mtv(R, x):
    """Batched R^T x."""
    return R[:, 0, :] * x[:, 0, None] + R[:, 1, :] * x[:, 1, None] + R[:, 2, :] * x[:, 2, None]


def _mm(A, B):
    """Batched 3x3 products A B (either operand may be a single 3x3 matrix)."""
    A = np.asarray(A)
    B = np.asarray(B)
    a = (lambda k: A[:, :, k, None]) if A.ndim == 3 else (lambda k: A[None, :, k, None])
    b = (lambda k: B[:, None, k, :]) if B.ndim == 3 else (lambda k: B[None, None, k, :])
    return a(0) * b(0) + a(1) * b(1) + a(2) * b(2)


def inverse_dynamics(model: Model, q: np.ndarray, dq: np.ndarray, ddq: np.ndarray) -> np.ndarray:
    """Generalized forces (N, nv) for samples given as (N, nq), (N, nv), (N, nv) arrays."""
    q = np.atleast_2d(np.asarray(q, dtype=float))
    dq = np.atleast_2d(np.asarray(dq, dtype=float))
    ddq = np.atleast_2d(np.asarray(ddq, dtype=float))
    N = q.shape[0]
    nj = model.njoints
    g = np.asarray(model.gravity, dtype=float)
    R = [None] * nj
    p = [None] * nj
    w = [None] * nj       # angular velocity (world)
    dw = [None] * nj      # angular acceleration (world)
    vo = [None] * nj      # velocity of the joint-frame origin (world)
    ao = [None] * nj      # acceleration of the joint-frame origin (world)
    axw = [None] * nj     # world joint axis (revolute)
    R[0] = np.broadcast_to(np.eye(3), (N, 3, 3))
    zero = np.zeros((N, 3))
    p[0], w[0], dw[0], vo[0], ao[0] = zero, zero, zero, zero, zero
    for i in range(1, nj):
        par = model.parents[i]
        iq, iv = model.idx_q[i], model.idx_v[i]
        if model.jtypes[i] == JOINT_FREEFLYER:
            if par != 0:
                raise NotImplementedError("free-flyer only as the root joint")
            Rb = _quat_to_matrix(q[:, iq + 3:iq + 7])
            R[i] = _mm(model.placements_R[i], Rb)
            p[i] = q[:, iq:iq + 3] + model.placements_t[i]
            vl, wl = dq[:, iv:iv + 3], dq[:, iv + 3:iv + 6]
            al, dwl = ddq[:, iv:iv + 3], ddq[:, iv + 3:iv + 6]
            w[i] = _mv(R[i], wl)
            dw[i] = _mv(R[i], dwl)
            vo[i] = _mv(R[i], vl)
            ao[i] = _mv(R[i], al + np.cross(wl, vl))
        else:
            ax = model.axes[i]
            Rpl = _mm(R[par], model.placements_R[i])
            R[i] = _mm(Rpl, _axis_rotation(ax, q[:, iq]))
            r = _mv(R[par], np.broadcast_to(model.placements_t[i], (N, 3)))
            p[i] = p[par] + r
            u = _mv(Rpl, np.broadcast_to(ax, (N, 3)))
            axw[i] = u
            w[i] = w[par] + u * dq[:, iv:iv + 1]
            dw[i] = dw[par] + u * ddq[:, iv:iv + 1] + np.cross(w[par], u * dq[:, iv:iv + 1])
            vo[i] = vo[par] + np.cross(w[par], r)
            ao[i] = ao[par] + np.cross(dw[par], r) + np.cross(w[par], np.cross(w[par], r))
    fsub = [None] * nj
    nsub = [None] * nj  # moment about the joint origin
    for i in range(1, nj):
        Y = model.inertias[i]
        c = _mv(R[i], np.broadcast_to(Y.lever, (N, 3)))  # CoM offset from origin, world
        ac = ao[i] + np.cross(dw[i], c) + np.cross(w[i], np.cross(w[i], c))
        F = Y.mass * (ac - g)
        Iw = _mm(_mm(R[i], Y.inertia_c), np.swapaxes(R[i], 1, 2))
        Nc = _mv(Iw, dw[i]) + np.cross(w[i], _mv(Iw, w[i]))
        fsub[i] = F
        nsub[i] = Nc + np.cross(c, F)
    for i in range(nj - 1, 0, -1):
        par = model.parents[i]
        if par > 0:
            fsub[par] = fsub[par] + fsub[i]
            nsub[par] = nsub[par] + nsub[i] + np.cross(p[i] - p[par], fsub[i])
    tau = np.zeros((N, model.nv))
    for i in range(1, nj):
        iv = model.idx_v[i]
        if model.jtypes[i] == JOINT_FREEFLYER:
            tau[:, iv:iv + 3] = _mtv(R[i], fsub[i])
            tau[:, iv + 3:iv + 6] = _mtv(R[i], nsub[i])
        else:
            tau[:, iv] = (axw[i] * nsub[i]).sum(axis=1)
    return tau
