"""Demo-level functions of the reference (demo/spot_identification.py, demo/solo_identification.py),
batched on the MI355X engine.

``get_projected_y_tau`` and ``get_projected_friction_regressors`` keep their signatures.  They return the
already-stacked arrays, so the reference's ``np.vstack(Y_proj)`` / ``np.hstack(tau_proj)`` at :84-87 are
identities.  One engine pass serves both calls (SystemIdentification caches it).

    python -m system_identification_amd.demo --robot spot --data <dir with spot_robot_*.dat>
"""
from __future__ import annotations

import argparse

import numpy as np

from .datio import read_data
from .solver import Solver
from .sys_identification import SystemIdentification


def get_projected_y_tau(q, dq, ddq, torque, cnt, sys_idnt: SystemIdentification):
    """demo/spot_identification.py:37-45 — (Y_proj stacked (N·nv x 10·nb), tau_proj stacked (N·nv))."""
    out = sys_idnt._stacked_cached(q, dq, ddq, torque, cnt)
    return out["Y_proj"], out["tau_proj"]


def get_projected_friction_regressors(q, dq, ddq, cnt, sys_idnt: SystemIdentification):
    """demo/spot_identification.py:47-56 — (B_v, B_c) stacked (N·nv x nj each)."""
    out = sys_idnt._stacked_cached(q, dq, ddq, None, cnt)
    return out["B_v"], out["B_c"]


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--robot", default="spot", help="robot name (committed model) or a .urdf path")
    ap.add_argument("--config", default=None, help="robot YAML when --robot is a URDF")
    ap.add_argument("--data", required=True, help="directory with <name>_robot_{q,dq,ddq,tau,contact}.dat")
    ap.add_argument("--name", default=None, help="file prefix (default: robot name)")
    ap.add_argument("--filter", default="butterworth", choices=["butterworth", "savitzky", "none"])
    ap.add_argument("--solver", default="llsq", choices=["llsq", "lmi"])
    args = ap.parse_args(argv)
    sys_idnt = SystemIdentification(args.robot, args.config, floating_base=True)
    name = args.name or sys_idnt._robot_name or args.robot
    q, dq, ddq, tau, cnt = read_data(args.data, name, args.filter)
    total_mass = sys_idnt.get_robot_mass()
    num_links = sys_idnt.get_num_links()
    phi_prior = sys_idnt.get_phi_prior()
    ne = sys_idnt.build_normal_equations(q, dq, ddq, tau, cnt)
    if args.solver == "lmi":
        solver = Solver.from_normal_equations(ne, num_links, phi_prior, total_mass, sys_idnt.get_bounding_ellipsoids())
        phi = solver.solve_fully_consistent()
    else:
        solver = Solver.from_normal_equations(ne, num_links, phi_prior, total_mass, None)
        phi = solver.solve_llsq_svd()
    sys_idnt.print_inertial_params(phi_prior, phi)
    sys_idnt.print_tau_prediction_rmse(q, dq, ddq, tau, cnt, phi_prior, "Prior")
    sys_idnt.print_tau_prediction_rmse(q, dq, ddq, tau, cnt, phi, "Identified")
    return phi


if __name__ == "__main__":
    np.set_printoptions(precision=4, suppress=True)
    main()
