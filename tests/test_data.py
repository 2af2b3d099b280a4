"""Synthetic logs and the .dat reader/writer (reference format, demo/spot_identification.py:9-34)."""
import numpy as np
import pytest

from system_identification_amd.datio import read_data, write_dat
from system_identification_amd.dynamics import inverse_dynamics
from system_identification_amd.model import load_robot
from system_identification_amd.synthetic import generate, channel_block


@pytest.mark.parametrize("robot", ["spot", "g1_29dof"])
def test_synthetic_shapes_and_values(robot):
    m = load_robot(robot)
    d = generate(m, 600, config_index=1)
    assert d["q"].shape == (m.nq, 600) and d["tau"].shape == (m.nj, 600) and d["contact"].shape == (m.n_ee, 600)
    assert set(np.unique(d["contact"])) <= {0.0, 1.0, 2.0}
    assert np.abs(np.linalg.norm(d["q"][3:7], axis=0) - 1).max() < 1e-6
    for i in range(1, m.njoints):
        if m.jtypes[i] == 2 and np.isfinite(m.lower[i]):
            x = d["q"][m.idx_q[i]]
            assert x.min() >= m.lower[i] - 1e-6 and x.max() <= m.upper[i] + 1e-6
    assert channel_block(d).shape == (m.nq + 2 * m.nv + m.nj + m.n_ee, 600)


def test_noise_free_torque_is_inverse_dynamics():
    m = load_robot("solo12")
    d = generate(m, 50, config_index=0, noise=False)
    tau = inverse_dynamics(m, d["q"].T, d["dq"].T, d["ddq"].T)[:, 6:].T
    # q/dq/ddq are float32-rounded after the torques were computed
    assert np.abs(tau - d["tau"]).max() < 1e-3 * np.abs(tau).max()


def test_dat_round_trip_and_filter(tmp_path):
    import scipy.signal as signal
    m = load_robot("spot")
    d = generate(m, 300, config_index=2)
    write_dat(str(tmp_path), "spot", d)
    q, dq, ddq, tau, cnt = read_data(str(tmp_path) + "/", "spot", "butterworth")
    assert q.dtype == np.float32 and cnt.dtype == np.float32 and dq.dtype == np.float64
    assert np.array_equal(q.astype(np.float64), d["q"]) and np.array_equal(cnt.astype(np.float64), d["contact"])
    b, a = signal.butter(5, 0.15, btype="low", analog=False)
    assert np.allclose(dq, signal.filtfilt(b, a, d["dq"].astype(np.float32), axis=1))
    q2, dq2, _, _, _ = read_data(str(tmp_path) + "/", "spot", "none")
    assert np.array_equal(dq2.astype(np.float64), d["dq"])
