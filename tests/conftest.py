import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built libsysid.so")
    # the slowest tests' run times at the end of every run (the whole-N oracle parity tests report theirs)
    if getattr(config.option, "durations", None) is None:
        config.option.durations = 12


REFERENCE = os.environ.get("SYSID_REFERENCE", "/root/reference")
HAS_REFERENCE = os.path.isdir(os.path.join(REFERENCE, "files"))
needs_reference = pytest.mark.skipif(not HAS_REFERENCE, reason="reference checkout not present (GPU box)")
