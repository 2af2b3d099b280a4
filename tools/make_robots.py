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


def _link(name, mass, com, diag):
    ix, iy, iz = diag
    return (f'  <link name="{name}"><inertial><origin xyz="{com[0]} {com[1]} {com[2]}" rpy="0 0 0"/>'
            f'<mass value="{mass}"/><inertia ixx="{ix}" ixy="0.001" ixz="0" iyy="{iy}" iyz="0.0005" izz="{iz}"/>'
            f'</inertial></link>')


def _joint(name, parent, child, xyz, axis, jtype="revolute"):
    lim = '<limit lower="-1.2" upper="1.2" effort="50" velocity="10"/>' if jtype == "revolute" else ""
    ax = f'<axis xyz="{axis}"/>' if jtype == "revolute" else ""
    return (f'  <joint name="{name}" type="{jtype}"><parent link="{parent}"/><child link="{child}"/>'
            f'<origin xyz="{xyz}" rpy="0.1 0 0"/>{ax}{lim}</joint>')


def snake14():
    """An authored test robot (no reference input): a floating trunk on two 3-joint legs with a 14-joint tail,
    so the runtime-nv K1 takes its 16-slot chain instantiations (C16P for f64, C16Q for the f32 / bf16 chunk
    panels) that the reference's robots never select."""
    L = ['<?xml version="1.0"?>', '<robot name="snake14">', _link("trunk", 4.0, (0.01, 0.0, 0.02), (0.05, 0.08, 0.09))]
    for side, y in (("left", 0.12), ("right", -0.12)):
        prev = "trunk"
        for k, (ax, xyz) in enumerate((("0 0 1", f"0.1 {y} 0"), ("0 1 0", "0 0 -0.05"), ("0 1 0", "0 0 -0.2"))):
            ln = f"{side}_leg{k}"
            L.append(_link(ln, 0.6 - 0.1 * k, (0.0, 0.01, -0.08), (0.004, 0.005, 0.002)))
            L.append(_joint(f"{side}_leg{k}_joint", prev, ln, xyz, ax))
            prev = ln
        L.append(_link(f"{side}_foot", 0.05, (0, 0, 0), (1e-5, 1e-5, 1e-5)))
        L.append(_joint(f"{side}_foot_fixed", prev, f"{side}_foot", "0 0 -0.2", "", "fixed"))
    prev = "trunk"
    for k in range(14):
        ln = f"tail{k:02d}"
        L.append(_link(ln, 0.3 - 0.01 * k, (-0.04, 0.0, 0.005), (0.0008, 0.001, 0.0011)))
        L.append(_joint(f"tail{k:02d}_joint", prev, ln, "-0.2 0 0" if k == 0 else "-0.08 0 0",
                        ("0 0 1", "0 1 0", "1 0 0")[k % 3]))
        prev = ln
    L.append("</robot>")
    urdf = os.path.join(ROBOT_DIR, "snake14.urdf")
    with open(urdf, "w") as fh:
        fh.write("\n".join(L) + "\n")
    links = ["trunk"] + [f"{s}_leg{k}" for s in ("left", "right") for k in range(3)] + [f"tail{k:02d}" for k in range(14)]
    cfg = os.path.join(ROBOT_DIR, "snake14_config.yaml")
    with open(cfg, "w") as fh:
        fh.write("# Authored test robot (tools/make_robots.py snake14): contacts are the two feet.\n")
        fh.write('robot:\n  name: "snake14"\n  mass: 9.57\n  end_effectors_frame_names:\n')
        fh.write('    - "left_foot"\n    - "right_foot"\n  link_names:\n')
        for ln in links:
            fh.write(f'    - "{ln}"\n')
    m = build_model_from_urdf(urdf, cfg, floating_base=True)
    out = os.path.join(ROBOT_DIR, "snake14.json")
    m.save_json(out)
    print(f"snake14: nq={m.nq} nv={m.nv} nb={m.nb} n_ee={m.n_ee} -> {out}")


def main():
    snake14()
    if not os.path.isdir(REF):
        return
    for name, (urdf, cfg, floating) in SOURCES.items():
        cfg_path = cfg if os.path.isabs(cfg) else os.path.join(REF, cfg)
        m = build_model_from_urdf(os.path.join(REF, urdf), cfg_path, floating_base=floating)
        out = os.path.join(ROBOT_DIR, f"{name}.json")
        m.save_json(out)
        print(f"{name}: nq={m.nq} nv={m.nv} nb={m.nb} n_ee={m.n_ee} -> {out}")


if __name__ == "__main__":
    main()
