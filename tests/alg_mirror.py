"""numpy mirror of the HIP kernel's formulation (test helper, not product code).

The kernel does not follow pinocchio's backward pass.  It uses, per sample:

* motion axes of every dof in the base (free-flyer) frame: ``w_r`` (direction) and ``p_r`` (a point);
* the contact Jacobian from the same axes; ``P = I - Q^T Q`` with the rows of ``Q`` an orthonormal basis of
  J_c's row space (modified Gram-Schmidt);
* ``H_i = P · M_i · J_w^T`` (nv x 6, world coordinates), built by one rank-1 update per body from its
  parent (``M_i`` = mask of the dofs supporting body i);
* each regressor column of body i as ``H_i · f^w`` with ``f^w`` the body-regressor column moved to world.

This file lets the test-suite check that formulation against the oracle on the CPU.
"""
import numpy as np

from oracle import ref_numpy as ref

JOINT_FREEFLYER = 1


def world_axes(model, d):
    nv = model.nv
    W = np.zeros((nv, 3))
    Pt = np.zeros((nv, 3))
    lin = np.zeros(nv, dtype=bool)
    for i in range(1, model.njoints):
        iv = model.idx_v[i]
        if model.jtypes[i] == JOINT_FREEFLYER:
            for k in range(3):
                W[iv + k] = d.oR[i][:, k]
                lin[iv + k] = True
                W[iv + 3 + k] = d.oR[i][:, k]
                Pt[iv + 3 + k] = d.ot[i]
        else:
            W[iv] = d.oR[i] @ model.axes[i]
            Pt[iv] = d.ot[i]
    return W, Pt, lin


def contact_jacobian(model, d, cnt, W, Pt, lin):
    rows = []
    for k, f in enumerate(model.contact_frames()):
        if not cnt[k]:
            continue
        pf = d.oR[f.parent] @ f.t + d.ot[f.parent]
        J = np.zeros((3, model.nv))
        for r in model.support_dofs(f.parent):
            J[:, r] = W[r] if lin[r] else np.cross(W[r], pf - Pt[r])
        rows.append(J)
    return np.vstack(rows) if rows else np.zeros((0, model.nv))


def projector_mgs(Jc, thr_rel=1e-14):
    """P = I - Q^T Q with the rows of Q an orthonormal basis of J_c's row space by modified Gram-Schmidt in
    row order, as K1 computes it: row p is taken (q = x_p / |x_p|, removed from every later row) when its
    remaining norm is > thr_rel * the largest row norm, dropped otherwise (pinv's rank cut)."""
    X = np.array(Jc, dtype=np.float64)
    k, nv = X.shape
    nrm = np.einsum("ij,ij->i", X, X)
    thr = thr_rel * thr_rel * (nrm.max() if k else 0.0)
    scale = np.zeros(k)  # 1/|x_p| of each taken row; 0 for dropped rows
    for p in range(k):
        best = nrm[p]
        if not best > thr:
            continue
        inv = 1.0 / np.sqrt(best)
        scale[p] = inv
        for j in range(p + 1, k):
            X[j] = X[j] - ((X[p] @ X[j]) * (inv * inv)) * X[p]
            nrm[j] = X[j] @ X[j]
    Q = X * scale[:, None]
    return np.eye(nv) - Q.T @ Q


def mgs_rows(Jc, thr_rel=1e-14):
    """The orthonormal rows Q of J_c's row space that K1's modified Gram-Schmidt takes (in row order)."""
    X = np.array(Jc, dtype=np.float64)
    k, nv = X.shape
    nrm = np.einsum("ij,ij->i", X, X)
    thr = thr_rel * thr_rel * (nrm.max() if k else 0.0)
    taken = []
    for p in range(k):
        if not nrm[p] > thr:
            continue
        inv2 = 1.0 / nrm[p]
        for j in range(p + 1, k):
            X[j] = X[j] - ((X[p] @ X[j]) * inv2) * X[p]
            nrm[j] = X[j] @ X[j]
        taken.append(X[p] / np.sqrt(nrm[p]))
    return np.array(taken).reshape(len(taken), nv)


def nullspace_rows(Q):
    """Zᵀ ((nv - r) x nv, orthonormal rows spanning null(Q)) as K1's Gram-only mode computes it, so that
    ZZᵀ... Zᵀ Z = I - QᵀQ = P: the Householder vectors of Qᵀ's QR reconstructed by an unpivoted LU of
    Qᵀ - diag(s) (s_j = -sign of the pivot, so every pivot has modulus |d_j| + 1 >= 1), tau_j = |d_j| + 1,
    then row t of Zᵀ = (H_1 ... H_r e_{r+t})ᵀ, H_j = I - tau_j v_j v_jᵀ."""
    Q = np.array(Q, dtype=np.float64)
    r, nv = Q.shape
    V = np.zeros((r, nv))
    tau = np.zeros(r)
    for j in range(r):
        d = Q[j, j]
        sg = 1.0 if d >= 0.0 else -1.0
        v = np.zeros(nv)
        v[j] = 1.0
        v[j + 1:] = Q[j, j + 1:] / (d + sg)
        for k in range(j + 1, r):
            Q[k, j + 1:] -= Q[k, j] * v[j + 1:]
        V[j], tau[j] = v, abs(d) + 1.0
    Zt = np.zeros((nv - r, nv))
    for t in range(nv - r):
        y = np.zeros(nv)
        y[r + t] = 1.0
        for j in range(r - 1, -1, -1):
            y -= tau[j] * (V[j] @ y) * V[j]
        Zt[t] = y
    return Zt


def base_relative(model, d):
    """Poses relative to the free-flyer frame (the kernel's reference frame); v, a_gf unchanged."""
    for i in range(1, model.njoints):
        p = model.parents[i]
        if model.jtypes[i] == JOINT_FREEFLYER:
            d.oR[i], d.ot[i] = np.eye(3), np.zeros(3)
        else:
            d.oR[i] = d.oR[p] @ d.liR[i]
            d.ot[i] = d.oR[p] @ d.lit[i] + d.ot[p]
    return d


def sample_panel(model, q, dq, ddq, tau, cnt):
    """[Y_proj | B_v | B_c | tau_proj] for one sample via the kernel formulation."""
    d = base_relative(model, ref.forward_pass(model, q, dq, ddq))
    W, Pt, lin = world_axes(model, d)
    P = projector_mgs(contact_jacobian(model, d, cnt, W, Pt, lin))
    nv, nb = model.nv, model.nb
    Jw = np.zeros((6, nv))  # world spatial axes [linear at origin; angular]
    for r in range(nv):
        Jw[:, r] = np.concatenate([W[r], np.zeros(3)]) if lin[r] else np.concatenate([np.cross(Pt[r], W[r]), W[r]])
    H = [None] * model.njoints
    for i in range(1, model.njoints):
        par = model.parents[i]
        Hi = np.zeros((nv, 6)) if par == 0 else H[par].copy()
        iv = model.idx_v[i]
        for r in range(iv, iv + model.nv_of(i)):
            Hi += np.outer(P[:, r], Jw[:, r])
        H[i] = Hi
    Y = np.zeros((nv, 10 * nb))
    for i in range(1, model.njoints):
        bR = ref.body_regressor(d.v[i], d.a_gf[i])
        Fw = ref.force_act(d.oR[i], d.ot[i], bR)  # local -> world
        Y[:, 10 * (i - 1):10 * i] = H[i] @ Fw
    bd = model.base_dof
    Bv = P[:, bd:] * dq[bd:]
    Bc = P[:, bd:] * np.sign(dq[bd:])
    t = P[:, bd:] @ tau
    return Y, t, Bv, Bc
