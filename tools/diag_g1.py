"""Quick G1 parity check for one library build (SYSID_LIB selects it)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from oracle import ref_numpy as ref
from system_identification_amd.engine import EMIT_ALL, Engine
from system_identification_amd.model import load_robot
from system_identification_amd.synthetic import generate
robot = sys.argv[1] if len(sys.argv) > 1 else "g1_29dof"
model = load_robot(robot); d = generate(model, 24, config_index=2 if robot == "g1_29dof" else 1)
out = Engine(model).build(d["q"], d["dq"], d["ddq"], d["tau"], d["contact"], EMIT_ALL)
Y, t = ref.get_projected_y_tau(model, d["q"], d["dq"], d["ddq"], d["tau"], d["contact"])
print(os.environ.get("SYSID_LIB"), robot, "Y err", np.abs(out["Y_proj"] - Y).max() / np.abs(Y).max(),
      "t err", np.abs(out["tau_proj"] - t).max() / np.abs(t).max(), "Y absmax", np.abs(out["Y_proj"]).max())
