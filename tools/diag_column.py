import sys, os, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from system_identification_amd.engine import load_library
from system_identification_amd.model import rpy_to_matrix
from oracle import ref_numpy as ref
import torch; torch.cuda.init()
lib = load_library()
rng = np.random.default_rng(0)
R = rpy_to_matrix(*rng.normal(size=3)); t = rng.normal(size=3); v = rng.normal(size=6); a = rng.normal(size=6)
b = np.concatenate([R.ravel(), t, v, a]); Fw = ref.force_act(R, t, ref.body_regressor(v, a))
out = np.zeros(64 * 6); P = ctypes.POINTER(ctypes.c_double)
print("rc", lib.sysid_debug_body_column_device(b.ctypes.data_as(P), out.ctypes.data_as(P)))
out = out.reshape(64, 6)
for l in range(12): print(l, l % 10, np.abs(out[l] - Fw[:, l % 10]).max(), out[l], Fw[:, l % 10])
