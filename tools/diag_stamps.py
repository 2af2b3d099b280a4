import sys, os, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from system_identification_amd import engine as E
from system_identification_amd.model import load_robot
from system_identification_amd.synthetic import generate, channel_block
robot = sys.argv[1] if len(sys.argv) > 1 else "spot"; N = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
torch.cuda.init()
lib = E.load_library(os.path.join(os.path.dirname(E.LIB_PATH), "libsysid_stamps.so"))
lib.sysid_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
E._LIB = lib
m = load_robot(robot); d = generate(m, N, 1); eng = E.Engine(m)
din = torch.from_numpy(channel_block(d)).cuda(); bufs = eng.alloc_device(N)
out = np.zeros(16, dtype=np.uint64)
for it in range(2):
    out[:] = 0
    lib.sysid_debug_stamps(eng._h, ctypes.c_void_p(din.data_ptr()), N, din.stride(0), ctypes.c_void_p(bufs["panel"].data_ptr()), bufs["panel"].stride(0), out.ctypes.data)
names = ["in", "fk", "axes", "Jc+norms", "mgs", "P", "H1+tp", "fric", "Ycols"]
tot = out[:9].sum()
for k, n in enumerate(names): print("%6s %10.0f cycles/sample  %5.1f%%" % (n, out[k] / N, 100 * out[k] / tot))
print("total %.0f cycles per sample per workgroup" % (tot / N))
