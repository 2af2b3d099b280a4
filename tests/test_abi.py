"""The C-ABI library builds, loads without a GPU, and exports every entry point include/sysid.h declares."""
import ctypes
import os
import re

import numpy as np
import pytest

from system_identification_amd import engine
from system_identification_amd.model import load_robot, unpack_header, PACK_MAGIC

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sysid.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int32_t|size_t|void|const char\s*\*)\s+(sysid_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_the_boundary():
    fns = declared_functions()
    for f in ("sysid_model_create", "sysid_destroy", "sysid_last_error", "sysid_build", "sysid_build_device",
              "sysid_workspace_bytes", "sysid_dims", "sysid_check_contacts", "sysid_time_stages"):
        assert f in fns


def test_library_exports_every_declared_symbol():
    lib = engine.load_library()
    for f in declared_functions():
        assert hasattr(lib, f), f
    bound = {name for name, _, _ in engine.SIGNATURES}
    stamps_only = {"sysid_debug_stamps"}
    assert set(declared_functions()) - stamps_only <= bound | stamps_only


def test_abi_version_and_errors_without_gpu():
    lib = engine.load_library()
    assert lib.sysid_abi_version() == 8
    out = ctypes.c_void_p()
    rc = lib.sysid_model_create(b"\x00" * 8, 8, 0, ctypes.byref(out))
    assert rc == engine.SYSID_E_MODEL and not out.value
    assert b"small" in lib.sysid_last_error(None)
    blob = bytearray(load_robot("spot").pack())
    blob[0] ^= 0xFF
    buf = ctypes.create_string_buffer(bytes(blob), len(blob))
    assert lib.sysid_model_create(buf, len(blob), 0, ctypes.byref(out)) == engine.SYSID_E_MODEL


def test_packed_model_header():
    m = load_robot("g1_29dof")
    h = unpack_header(m.pack())
    assert h["magic"] == PACK_MAGIC and h["version"] == 1
    assert (h["nq"], h["nv"], h["njoints"], h["n_contact"], h["base_dof"], h["nj"]) == (36, 35, 31, 2, 6, 29)


def test_host_build_of_kernel_body_column():
    """The kernel's branch-free body-regressor column helper, host instantiation, vs the oracle."""
    from oracle import ref_numpy as ref
    from system_identification_amd.model import rpy_to_matrix
    lib = engine.load_library()
    rng = np.random.default_rng(0)
    P = ctypes.POINTER(ctypes.c_double)
    for _ in range(5):
        R = rpy_to_matrix(*rng.normal(size=3))
        t, v, a = rng.normal(size=3), rng.normal(size=6), rng.normal(size=6)
        b = np.concatenate([R.ravel(), t, v, a])
        Fw = ref.force_act(R, t, ref.body_regressor(v, a))
        for p in range(10):
            o = np.zeros(6)
            assert lib.sysid_debug_body_column(b.ctypes.data_as(P), p, o.ctypes.data_as(P)) == 0
            assert np.abs(o - Fw[:, p]).max() < 1e-13


def test_engine_refuses_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(engine.EngineError):
        engine.Engine(load_robot("spot"))
