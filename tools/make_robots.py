"""Compile the reference's robot descriptions into the committed JSON models.

Run in the build container (it reads /root/reference, which the GPU box does not have):
    python tools/make_robots.py
Inputs: files/{solo_description,spot_description,g1_description}/ URDF + YAML of the reference
(demo/solo_identification.py:62-64, demo/spot_identification.py:65-66); the G1 YAML is authored here
(system_identification_amd/robots/g1_29dof_config.yaml) because the reference's is a copy of Spot's.
Output: system_identification_amd/robots/<robot>.json (kinematic tree, inertias, frames, YAML data).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from system_identification_amd.model import ROBOT_DIR, build_model_from_urdf  # noqa: E402

REF = os.environ.get("SYSID_REFERENCE", "/root/reference")
SOURCES = {  # name: (urdf, yaml, floating_base)
    "solo12": ("files/solo_description/solo12.urdf", "files/solo_description/solo12_config.yaml", True),
    "spot": ("files/spot_description/spot.urdf", "files/spot_description/spot_config.yaml", True),
    "g1_29dof": ("files/g1_description/g1_29dof.urdf", os.path.join(ROBOT_DIR, "g1_29dof_config.yaml"), True),
    # the reference's fixed-base branch (SystemIdentification(..., floating_base=False),
    # src/sys_identification.py:33-36): the same legs welded to the universe, base_dof = 0
    "solo12_fixed": ("files/solo_description/solo12.urdf", "files/solo_description/solo12_config.yaml", False),
}


def main():
    for name, (urdf, cfg, floating) in SOURCES.items():
        cfg_path = cfg if os.path.isabs(cfg) else os.path.join(REF, cfg)
        m = build_model_from_urdf(os.path.join(REF, urdf), cfg_path, floating_base=floating)
        out = os.path.join(ROBOT_DIR, f"{name}.json")
        m.save_json(out)
        print(f"{name}: nq={m.nq} nv={m.nv} nb={m.nb} n_ee={m.n_ee} -> {out}")


if __name__ == "__main__":
    main()
