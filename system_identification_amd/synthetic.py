"""Synthetic joint-torque logs in the reference's channel layout.

The reference's own data (`data/*.dat`) is gitignored and not shipped (.gitignore:9-11), so every
config is synthesised: seeds ``default_rng(20250629 + k)``, sinusoidal joint trajectories inside the
URDF limits, a wobbling free-flyer base (LOCAL velocity), torques from inverse dynamics plus noise, and a
gait contact schedule with values {0, 1, 2} (utils/read_spot_system_state.py:62: UNKNOWN/MADE/LOST).

Arrays are channel-major (channels x N), exactly what ``read_data`` returns
(demo/spot_identification.py:9-34): q and contact float32 values, dq/ddq/tau float64.
"""
from __future__ import annotations

import os

import numpy as np

from .dynamics import inverse_dynamics
from .model import JOINT_FREEFLYER, JOINT_REVOLUTE, Model, rpy_to_matrix

SEED_BASE = 20250629


def _matrix_to_quat(R: np.ndarray) -> np.ndarray:
    """(N,3,3) rotation matrices -> (N,4) quaternions (x, y, z, w), w >= 0."""
    N = R.shape[0]
    q = np.empty((N, 4))
    tr = R[:, 0, 0] + R[:, 1, 1] + R[:, 2, 2]
    w = 0.5 * np.sqrt(np.maximum(1.0 + tr, 1e-12))
    q[:, 3] = w
    q[:, 0] = (R[:, 2, 1] - R[:, 1, 2]) / (4 * w)
    q[:, 1] = (R[:, 0, 2] - R[:, 2, 0]) / (4 * w)
    q[:, 2] = (R[:, 1, 0] - R[:, 0, 1]) / (4 * w)
    return q / np.linalg.norm(q, axis=1, keepdims=True)


def _rpy_traj(t, amp, freq, phase):
    """sum of harmonics and its first two derivatives, per column."""
    arg = 2 * np.pi * freq[None] * t[:, None] + phase[None]
    x = (amp[None] * np.sin(arg)).sum(-1)
    dx = (amp[None] * 2 * np.pi * freq[None] * np.cos(arg)).sum(-1)
    ddx = (-amp[None] * (2 * np.pi * freq[None]) ** 2 * np.sin(arg)).sum(-1)
    return x, dx, ddx


def _rotations(rpy):
    return np.stack([rpy_to_matrix(*r) for r in rpy]) if len(rpy) < 2048 else _rotations_vec(rpy)


def _rotations_vec(rpy):
    r, p, y = rpy[:, 0], rpy[:, 1], rpy[:, 2]
    cr, sr, cp, sp, cy, sy = np.cos(r), np.sin(r), np.cos(p), np.sin(p), np.cos(y), np.sin(y)
    R = np.empty((len(r), 3, 3))
    R[:, 0, 0] = cy * cp; R[:, 0, 1] = cy * sp * sr - sy * cr; R[:, 0, 2] = cy * sp * cr + sy * sr
    R[:, 1, 0] = sy * cp; R[:, 1, 1] = sy * sp * sr + cy * cr; R[:, 1, 2] = sy * sp * cr - cy * sr
    R[:, 2, 0] = -sp; R[:, 2, 1] = cp * sr; R[:, 2, 2] = cp * cr
    return R


def _vee(S):
    return np.stack([S[:, 2, 1] - S[:, 1, 2], S[:, 0, 2] - S[:, 2, 0], S[:, 1, 0] - S[:, 0, 1]], axis=1) * 0.5


def contact_schedule(model: Model, t: np.ndarray, rng, gait_hz: float = 2.0) -> np.ndarray:
    """(n_ee, N) contact values: trot (4 feet) / walk (2 feet) with standing and flight windows."""
    nee, N = model.n_ee, t.size
    cnt = np.zeros((nee, N))
    phase = (t * gait_hz) % 1.0
    for k in range(nee):
        group = (k in (0, 3)) if nee == 4 else (k % 2 == 0)
        off = 0.0 if group else 0.5
        ph = (phase - off) % 1.0
        cnt[k] = ph < 0.6
    n_stand = max(1, N // 10)
    cnt[:, :n_stand] = 1.0                      # standing / squatting, all feet down
    n_fly = max(1, N // 50)
    cnt[:, n_stand:n_stand + n_fly] = 0.0        # no contact at all
    lost = (rng.random((nee, N)) < 0.05) & (cnt == 1.0)
    cnt[lost] = 2.0                              # CONTACT_LOST, still truthy in the reference
    return cnt


def generate(model: Model, N: int, config_index: int = 0, rate_hz: float = 500.0,
             noise: bool = True, chunk: int = 65536) -> dict:
    """Synthesise N samples.  Returns dict(q, dq, ddq, tau, contact) channel-major, plus 'tau_clean'."""
    rng = np.random.default_rng(SEED_BASE + config_index)
    t = np.arange(N) / rate_hz
    nq, nv = model.nq, model.nv
    q = np.zeros((N, nq))
    dq = np.zeros((N, nv))
    ddq = np.zeros((N, nv))
    for i in range(1, model.njoints):
        iq, iv = model.idx_q[i], model.idx_v[i]
        if model.jtypes[i] == JOINT_REVOLUTE:
            lo, hi = model.lower[i], model.upper[i]
            if not (np.isfinite(lo) and np.isfinite(hi)) or hi - lo > 2 * np.pi:
                lo, hi = -1.0, 1.0
            mid, half = 0.5 * (lo + hi), 0.5 * (hi - lo)
            amp = 0.6 * half / 3 * rng.uniform(0.5, 1.0, 3)
            freq = rng.uniform(0.2, 3.0, 3)
            ph = rng.uniform(0, 2 * np.pi, 3)
            x, dx, ddx = _rpy_traj(t, amp, freq, ph)
            q[:, iq], dq[:, iv], ddq[:, iv] = mid + x, dx, ddx
        elif model.jtypes[i] == JOINT_FREEFLYER:
            pos, vel, acc = np.zeros((N, 3)), np.zeros((N, 3)), np.zeros((N, 3))
            base = np.array([0.0, 0.0, 0.5])
            for k in range(3):
                x, dx, ddx = _rpy_traj(t, 0.05 / 3 * rng.uniform(0.5, 1.0, 3), rng.uniform(0.2, 2.0, 3),
                                       rng.uniform(0, 2 * np.pi, 3))
                pos[:, k], vel[:, k], acc[:, k] = base[k] + x, dx, ddx
            amps = [0.3 / 3, 0.3 / 3, 0.2 / 3]
            params = [(amps[k] * rng.uniform(0.5, 1.0, 3), rng.uniform(0.2, 2.0, 3), rng.uniform(0, 2 * np.pi, 3))
                      for k in range(3)]

            def rpy_at(tt):
                return np.stack([_rpy_traj(tt, *params[k])[0] for k in range(3)], axis=1)

            h = 1e-4
            R = _rotations_vec(rpy_at(t))
            Rp, Rm = _rotations_vec(rpy_at(t + h)), _rotations_vec(rpy_at(t - h))
            Rpp, Rmm = _rotations_vec(rpy_at(t + 2 * h)), _rotations_vec(rpy_at(t - 2 * h))
            wb = _vee(np.einsum("nji,njk->nik", R, (Rp - Rm) / (2 * h)))
            wbp = _vee(np.einsum("nji,njk->nik", Rp, (Rpp - R) / (2 * h)))
            wbm = _vee(np.einsum("nji,njk->nik", Rm, (R - Rmm) / (2 * h)))
            dwb = (wbp - wbm) / (2 * h)
            v_loc = np.einsum("nji,nj->ni", R, vel)
            a_loc = np.einsum("nji,nj->ni", R, acc) - np.cross(wb, v_loc)
            q[:, iq:iq + 3] = pos
            q[:, iq + 3:iq + 7] = _matrix_to_quat(R)
            dq[:, iv:iv + 3], dq[:, iv + 3:iv + 6] = v_loc, wb
            ddq[:, iv:iv + 3], ddq[:, iv + 3:iv + 6] = a_loc, dwb
    tau_full = np.empty((N, nv))

    def _id(s0):
        s1 = min(N, s0 + chunk)
        tau_full[s0:s1] = inverse_dynamics(model, q[s0:s1], dq[s0:s1], ddq[s0:s1])

    starts = list(range(0, N, chunk))
    if len(starts) > 1:
        # numpy releases the GIL in its array loops: chunks on a few threads (G1 1M: ~70 s -> ~15 s)
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(max_workers=min(8, len(starts), os.cpu_count() or 1)) as ex:
            list(ex.map(_id, starts))
    else:
        for s0 in starts:
            _id(s0)
    tau_clean = tau_full[:, model.base_dof:]
    tau = tau_clean.copy()
    if noise:
        dq = dq + rng.normal(0.0, 0.01, dq.shape)
        ddq = ddq + rng.normal(0.0, 0.01, ddq.shape)
        tau = tau + rng.normal(0.0, 0.5, tau.shape)
    cnt = contact_schedule(model, t, rng)
    # .dat values are float32 (demo/spot_identification.py:10-14)
    f32 = lambda a: np.ascontiguousarray(a.T.astype(np.float32).astype(np.float64))  # noqa: E731
    return {"q": f32(q), "dq": f32(dq), "ddq": f32(ddq), "tau": f32(tau),
            "contact": np.ascontiguousarray(cnt.astype(np.float32).astype(np.float64)),
            "tau_clean": np.ascontiguousarray(tau_clean.T)}


def channel_block(data: dict) -> np.ndarray:
    """[q; dq; ddq; tau; contact] stacked channel-major (the d_in layout of sysid_build_device)."""
    return np.ascontiguousarray(np.vstack([data["q"], data["dq"], data["ddq"], data["tau"], data["contact"]]))
