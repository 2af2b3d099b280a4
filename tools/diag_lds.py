import sys, os, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from oracle import ref_numpy as ref
from tests import alg_mirror as am
from system_identification_amd.engine import Engine
from system_identification_amd.model import load_robot
from system_identification_amd.synthetic import generate
P = ctypes.POINTER(ctypes.c_double)
for robot in ["spot"]:
    m = load_robot(robot); d = generate(m, 8, 1); eng = Engine(m)
    s = 3
    x = [np.ascontiguousarray(d[k][:, s:s+1]) for k in ("q", "dq", "ddq", "tau", "contact")]
    off = (ctypes.c_int32 * 12)(); eng.lib.sysid_debug_layout(eng._h, off); off = list(off)
    img = np.zeros(off[11])
    rc = eng.lib.sysid_debug_lds(eng._h, *[a.ctypes.data_as(P) for a in x], img.ctypes.data_as(P), img.size)
    print("rc", rc, off)
    q, dq, ddq, tau, cnt = (a[:, 0] for a in x)
    D = ref.forward_pass(m, q, dq, ddq)
    body = img[off[1]:off[2]].reshape(-1, 24)
    for j in range(1, m.njoints):
        e = [np.abs(body[j, :9] - D.oR[j].ravel()).max(), np.abs(body[j, 9:12] - D.ot[j]).max(),
             np.abs(body[j, 12:18] - D.v[j]).max(), np.abs(body[j, 18:24] - D.a_gf[j]).max()]
        print("body", j, ["%.1e" % v for v in e])
    W, Pt, lin = am.world_axes(m, D)
    print("W", np.abs(img[off[2]:off[3]].reshape(-1, 3) - W).max(), "Pt", np.abs(img[off[3]:off[4]].reshape(-1, 3) - Pt).max())
    Pm = am.projector_cholqr(m, D, cnt, W, Pt, lin)
    print("P", np.abs(img[off[9]:off[9] + m.nv * m.nv].reshape(m.nv, m.nv) - Pm).max())
    H = img[off[10]:off[11]].reshape(m.njoints, m.nv, 6)
    Jw = np.zeros((6, m.nv))
    for r in range(m.nv):
        Jw[:, r] = np.concatenate([W[r], np.zeros(3)]) if lin[r] else np.concatenate([np.cross(Pt[r], W[r]), W[r]])
    Hm = [None] * m.njoints
    for i in range(1, m.njoints):
        par = m.parents[i]; Hi = np.zeros((m.nv, 6)) if par == 0 else Hm[par].copy()
        for r in range(m.idx_v[i], m.idx_v[i] + m.nv_of(i)): Hi += np.outer(Pm[:, r], Jw[:, r])
        Hm[i] = Hi
        print("H", i, np.abs(H[i] - Hi).max())
    out = eng.build(*x)
    Y, t = ref.get_projected_y_tau(m, *x)
    Yg = out["Y_proj"]
    print("col3 gpu", Yg[:4, 3], "ref", Y[:4, 3])
    bR = ref.body_regressor(D.v[1], D.a_gf[1]); Fw = ref.force_act(D.oR[1], D.ot[1], bR)
    print("H1@Fw col3", (Hm[1] @ Fw)[:4, 3])
