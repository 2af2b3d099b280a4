"""Shared parity metric for the projected per-sample blocks (test helper).

north_star's bar is 1e-6 relative.  A block is compared relative to its own largest magnitude, with one
floor: when the sample's contacts pin every dof (a fixed-base robot standing on all feet: J_c square and
invertible), P = I - J_c^T (J_c J_c^T)^-1 J_c is exactly zero, and both the reference path and ours
return rounding noise of size ~eps·cond(J_c)^2 times the unprojected block.  Relative error between two
noises is meaningless, so the denominator never drops below FLOOR times the unprojected block's scale
(the regressor Y, tau, S^T diag(dq), S^T diag(sign dq)).  For every sample that is not fully pinned the
projected block is of the same order as the unprojected one and the floor does not bind.
"""
import numpy as np

from oracle import ref_numpy as ref

FLOOR = 1e-4


def rel(a, b, scale=0.0):
    return np.abs(a - b).max(initial=0.0) / max(np.abs(b).max(initial=0.0), FLOOR * scale, 1e-300)


def unprojected_scales(model, q, dq, ddq, tau):
    """Per sample: (max|Y|, max|tau|, max|dq_joints|, 1) of the unprojected blocks."""
    bd = model.base_dof
    out = []
    for s in range(q.shape[1]):
        Y = ref.joint_torque_regressor(model, q[:, s], dq[:, s], ddq[:, s])
        out.append((np.abs(Y).max(), np.abs(tau[:, s]).max(initial=0.0), np.abs(dq[bd:, s]).max(initial=0.0), 1.0))
    return out
