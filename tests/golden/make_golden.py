"""Generate the committed golden fixtures (tests/golden/*.npz) from the numpy oracle.

The reference cannot be imported here (cvxpy/trimesh/pinocchio absent — SURVEY.md §8c) and ships no
fixtures or .dat data, so the vectors come from oracle/ref_numpy.py, itself pinned by the identity tests
(tests/test_oracle_identities.py).  Each fixture holds inputs (channel-major, as read_data returns them)
and the reference-path outputs: stacked Y_proj, tau_proj, B_v, B_c, the unprojected regressor Y, the
stacked contact Jacobians, and the normal equations.

    python tests/golden/make_golden.py [robot ...]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import ref_numpy as ref  # noqa: E402
from system_identification_amd.model import load_robot  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


def contact_patterns(n_ee):
    if n_ee == 4:
        return [[1, 1, 1, 1], [0, 0, 0, 0], [1, 0, 0, 1], [0, 1, 1, 0], [2, 1, 1, 2], [1, 0, 0, 0], [2, 0, 0, 0],
                [1, 1, 1, 0]]
    return [[1, 1], [0, 0], [1, 0], [0, 1], [2, 1], [2, 2], [1, 2], [0, 2]]


def make(robot, seed):
    m = load_robot(robot)
    rng = np.random.default_rng(seed)
    pats = contact_patterns(m.n_ee)
    N = len(pats)
    q = np.zeros((m.nq, N))
    for i in range(1, m.njoints):
        iq = m.idx_q[i]
        if m.jtypes[i] == 1:
            q[iq:iq + 3] = rng.normal(0, 0.1, (3, N)) + np.array([[0], [0], [0.5]])
            quat = rng.normal(0, 0.2, (4, N))
            quat[3] += 1.0
            quat /= np.linalg.norm(quat, axis=0)
            q[iq + 3:iq + 7] = quat.astype(np.float32).astype(np.float64)  # float32 .dat values
        else:
            lo, hi = m.lower[i], m.upper[i]
            q[iq] = rng.uniform(lo, hi, N) if np.isfinite(lo) and np.isfinite(hi) else rng.uniform(-1, 1, N)
    dq = rng.normal(0, 1.0, (m.nv, N))
    ddq = rng.normal(0, 3.0, (m.nv, N))
    dq[m.base_dof + 0, 0] = 0.0  # sign(0) = 0 in the Coulomb column
    tau = rng.normal(0, 5.0, (m.nj, N))
    cnt = np.array(pats, dtype=float).T
    Y, t = ref.get_projected_y_tau(m, q, dq, ddq, tau, cnt)
    Bv, Bc = ref.get_projected_friction_regressors(m, q, dq, ddq, cnt)
    G, g, btb, rows = ref.normal_equations(Y, t, Bv, Bc)
    Yu = np.vstack([ref.joint_torque_regressor(m, q[:, s], dq[:, s], ddq[:, s]) for s in range(N)])
    Jc = [ref.compute_J_c(m, ref.forward_pass(m, q[:, s], dq[:, s], ddq[:, s]), cnt[:, s]) for s in range(N)]
    Jc_rows = np.array([j.shape[0] for j in Jc])
    Jc_all = np.vstack([j for j in Jc if j.size] or [np.zeros((0, m.nv))])
    path = os.path.join(OUT, f"{robot}.npz")
    np.savez_compressed(path, q=q, dq=dq, ddq=ddq, tau=tau, contact=cnt, Y_proj=Y, tau_proj=t, B_v=Bv, B_c=Bc,
                        gram=G, Atb=g, btb=btb, num_rows=rows, Y=Yu, Jc=Jc_all, Jc_rows=Jc_rows)
    print(f"{robot}: {N} samples -> {path} ({os.path.getsize(path)} B)")


ROBOTS = ("solo12", "spot", "g1_29dof", "solo12_fixed")  # seed 1000 + position

if __name__ == "__main__":
    for k, r in enumerate(ROBOTS):
        if len(sys.argv) == 1 or r in sys.argv[1:]:
            make(r, 1000 + k)
