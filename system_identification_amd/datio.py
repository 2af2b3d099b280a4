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


def load_dat(filename: str, nthreads: int = 0) -> np.ndarray:
    """np.loadtxt(filename, delimiter='\\t', dtype=np.float32) through the native parallel parser in libsysid.so
    (bit-identical values; same squeeze of unit dimensions as loadtxt's default ndmin=0)."""
    import ctypes
    from .engine import load_library
    lib = load_library()
    fn = os.fsencode(str(filename))
    rows, cols = ctypes.c_int64(), ctypes.c_int64()
    if lib.sysid_dat_shape(fn, ctypes.byref(rows), ctypes.byref(cols)) != 0:
        raise ValueError(lib.sysid_io_last_error().decode())
    out = np.empty((rows.value, cols.value), dtype=np.float32)
    ptr = out.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    if lib.sysid_dat_read(fn, ptr, rows.value, cols.value, int(nthreads)) != 0:
        raise ValueError(lib.sysid_io_last_error().decode())
    return np.squeeze(out) if 1 in out.shape else out


def read_data(path, robot_name, filter_type):
    """demo/spot_identification.py:9-34 (solo's variant :9-33 is this with robot_name="solo").  The five
    files are parsed natively (load_dat); the filters are the reference's scipy calls, on the host."""
    import scipy.signal as signal
    from scipy.signal import savgol_filter
    path = str(path)
    q = load_dat(dat_path(path, robot_name, "q"))
    dq = load_dat(dat_path(path, robot_name, "dq"))
    ddq = load_dat(dat_path(path, robot_name, "ddq"))
    tau = load_dat(dat_path(path, robot_name, "tau"))
    cnt = load_dat(dat_path(path, robot_name, "contact"))
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
