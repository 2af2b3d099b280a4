"""``.dat`` logs in the reference's format (demo/spot_identification.py:9-34, README.md:50-79).

One channel per row, one time sample per column, tab-delimited text, read as float32:
``{robot}_robot_q.dat`` (nq rows: x y z qx qy qz qw, joints), ``_dq`` / ``_ddq`` (nv rows: base velocity in
the LOCAL frame, joints), ``_tau`` (nj rows), ``_contact`` (n_ee rows, CONTACT_UNKNOWN=0 / MADE=1 / LOST=2).
``read_data`` applies the reference's filters to dq, ddq and tau (Butterworth order 5, cutoff 0.15, filtfilt
along time; or Savitzky–Golay 21/5), which turns them into float64; q and contact stay float32.
"""
from __future__ import annotations

import os

import numpy as np

CHANNELS = ("q", "dq", "ddq", "tau", "contact")


def dat_path(path: str, robot_name: str, channel: str) -> str:
    return os.path.join(path, f"{robot_name}_robot_{channel}.dat")


def write_dat(path: str, robot_name: str, data: dict) -> None:
    """Write channel-major arrays with float32 round-trip precision ('%.9g')."""
    os.makedirs(path, exist_ok=True)
    for ch in CHANNELS:
        a = np.asarray(data[ch], dtype=np.float32)
        np.savetxt(dat_path(path, robot_name, ch), np.atleast_2d(a), delimiter="\t", fmt="%.9g")


def read_data(path, robot_name, filter_type):
    """demo/spot_identification.py:9-34 (solo's variant :9-33 is this with robot_name="solo")."""
    import scipy.signal as signal
    from scipy.signal import savgol_filter
    path = str(path)
    q = np.loadtxt(dat_path(path, robot_name, "q"), delimiter="\t", dtype=np.float32)
    dq = np.loadtxt(dat_path(path, robot_name, "dq"), delimiter="\t", dtype=np.float32)
    ddq = np.loadtxt(dat_path(path, robot_name, "ddq"), delimiter="\t", dtype=np.float32)
    tau = np.loadtxt(dat_path(path, robot_name, "tau"), delimiter="\t", dtype=np.float32)
    cnt = np.loadtxt(dat_path(path, robot_name, "contact"), delimiter="\t", dtype=np.float32)
    if filter_type == "butterworth":
        b, a = signal.butter(5, 0.15, btype="low", analog=False)
        dq = signal.filtfilt(b, a, dq, axis=1)
        ddq = signal.filtfilt(b, a, ddq, axis=1)
        tau = signal.filtfilt(b, a, tau, axis=1)
    elif filter_type == "savitzky":
        dq = savgol_filter(dq, 21, 5)
        ddq = savgol_filter(ddq, 21, 5)
        tau = savgol_filter(tau, 21, 5)
    return q, dq, ddq, tau, cnt
