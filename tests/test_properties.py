"""Hypothesis property tests over random states for the oracle and for the numpy
mirror of the kernel algebra: the identities must hold for any (q, dq, ddq, contact), not just seeds."""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from tests import alg_mirror as am
from tests.parity import rel as rel_floor
from tests.parity import unprojected_scales
from oracle import ref_numpy as ref
from system_identification_amd.dynamics import inverse_dynamics
from system_identification_amd.model import load_robot

MODELS = {r: load_robot(r) for r in ("solo12", "spot", "g1_29dof", "solo12_fixed")}
robots = st.sampled_from(sorted(MODELS))
seeds = st.integers(0, 2**32 - 1)


def state(m, seed, scale=1.0):
    rng = np.random.default_rng(seed)
    q = rng.normal(0, 0.5 * scale, m.nq)
    if m.floating_base:
        quat = rng.normal(0, 0.3, 4)
        quat[3] += 1.0
        q[3:7] = quat / np.linalg.norm(quat)
    cnt = rng.integers(0, 3, m.n_ee).astype(float)  # {0, 1, 2}: LOST = 2 counts as contact
    return q, rng.normal(0, scale, m.nv), rng.normal(0, 2 * scale, m.nv), rng.normal(0, 20, m.nj), cnt


@settings(max_examples=25, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(robot=robots, seed=seeds)
def test_regressor_is_inverse_dynamics(robot, seed):
    m = MODELS[robot]
    q, v, a, _, _ = state(m, seed)
    Y = ref.joint_torque_regressor(m, q, v, a)
    tau = inverse_dynamics(m, q[None], v[None], a[None])[0]
    assert np.abs(Y @ m.phi_pin() - tau).max() <= 1e-10 * max(1.0, np.abs(tau).max())


@settings(max_examples=25, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(robot=robots, seed=seeds)
def test_projector_identities(robot, seed):
    m = MODELS[robot]
    q, v, a, _, cnt = state(m, seed)
    d = ref.forward_pass(m, q, v, a)
    Jc = ref.compute_J_c(m, d, cnt)
    P = ref.null_space_projector(m, d, cnt)
    assert np.abs(P @ Jc.T).max(initial=0.0) < 1e-10
    assert np.abs(P @ P - P).max() < 1e-10
    assert np.abs(P - P.T).max() < 1e-10
    if not cnt.any():
        assert np.array_equal(P, np.eye(m.nv))


@settings(max_examples=20, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(robot=robots, seed=seeds)
def test_kernel_algebra_matches_oracle(robot, seed):
    """The kernel's formulation (base-frame kinematics, J_w-chain columns, exchange-inverse projector)
    reproduces the oracle's projected regressor, torque and friction regressors."""
    m = MODELS[robot]
    q, v, a, tau, cnt = state(m, seed)
    Y, t, Bv, Bc = am.sample_panel(m, q, v, a, tau, cnt)
    Yr, tr = ref.get_proj_regressor_torque(m, q, v, a, tau, cnt)
    Bvr, Bcr = ref.get_proj_friction_regressors(m, q, v, a, cnt)
    sc = unprojected_scales(m, q[:, None], v[:, None], a[:, None], tau[:, None])[0]
    for x, r, c in zip((Y, t, Bv, Bc), (Yr, tr, Bvr, Bcr), sc):
        assert rel_floor(x, r, c) <= 1e-6  # fully pinned samples: see tests/parity.py
