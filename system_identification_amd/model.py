"""Kinematic-tree model compiler: URDF (+ the reference's robot YAML) -> packed engine model.

The reference builds its model with pinocchio:
``pin.buildModelFromUrdf(urdf, pin.JointModelFreeFlyer())`` (src/sys_identification.py:16), sets
gravity to (0, 0, -9.81) (:22), builds the selection matrix ``S = [0 | I]`` (:29-37) and resolves the
end-effector frame ids from the YAML (:40-55).  pinocchio is not available to this project, so this
module restates the URDF -> model rules it applies (documented pinocchio behaviour):

* the root link gets a free-flyer joint (``floating_base=True``) or is welded to the universe;
* revolute joints become one-dof rotations about their (unit) URDF axis;
* fixed joints are merged into the parent body: the child's inertia is appended to the parent joint
  and the child link becomes a frame of the parent joint;
* the tree is walked depth-first with the children of every link visited in joint-name order (urdfdom
  keeps joints in a name-sorted map), which fixes the joint/column order of the regressor;
* joint placements are the accumulated fixed-joint placement composed with ``origin(xyz, rpy)``, with
  ``R = Rz(yaw) Ry(pitch) Rx(roll)``.

Only the kinematics reach the GPU; inertias are carried for phi_prior and for the test oracles.
"""
from __future__ import annotations

import json
import os
import struct
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field

import numpy as np

JOINT_UNIVERSE = 0
JOINT_FREEFLYER = 1
JOINT_REVOLUTE = 2

PACK_MAGIC = 0x44495953  # 'SYID' little endian
PACK_VERSION = 1
GRAVITY = (0.0, 0.0, -9.81)  # src/sys_identification.py:22


def rpy_to_matrix(r: float, p: float, y: float) -> np.ndarray:
    """R = Rz(y) @ Ry(p) @ Rx(r) (URDF fixed-axis roll-pitch-yaw)."""
    cr, sr = np.cos(r), np.sin(r)
    cp, sp = np.cos(p), np.sin(p)
    cy, sy = np.cos(y), np.sin(y)
    return np.array([
        [cy * cp, cy * sp * sr - sy * cr, cy * sp * cr + sy * sr],
        [sy * cp, sy * sp * sr + cy * cr, sy * sp * cr - cy * sr],
        [-sp, cp * sr, cp * cr],
    ])


def skew(v) -> np.ndarray:
    return np.array([[0.0, -v[2], v[1]], [v[2], 0.0, -v[0]], [-v[1], v[0], 0.0]])


@dataclass
class Inertia:
    """Rigid-body inertia: mass, centre of mass ``lever`` and rotational inertia about the CoM."""
    mass: float = 0.0
    lever: np.ndarray = field(default_factory=lambda: np.zeros(3))
    inertia_c: np.ndarray = field(default_factory=lambda: np.zeros((3, 3)))

    def transformed(self, R: np.ndarray, t: np.ndarray) -> "Inertia":
        return Inertia(self.mass, R @ self.lever + t, R @ self.inertia_c @ R.T)

    def __add__(self, other: "Inertia") -> "Inertia":
        m = self.mass + other.mass
        if m <= 0.0:
            return Inertia(0.0, np.zeros(3), self.inertia_c + other.inertia_c)
        c = (self.mass * self.lever + other.mass * other.lever) / m
        d1, d2 = self.lever - c, other.lever - c
        I = (self.inertia_c + other.inertia_c
             - self.mass * skew(d1) @ skew(d1) - other.mass * skew(d2) @ skew(d2))
        return Inertia(m, c, I)

    def dynamic_parameters(self) -> np.ndarray:
        """pinocchio ``Inertia::toDynamicParameters`` order: [m, mc, Ixx, Ixy, Iyy, Ixz, Iyz, Izz]
        with the rotational inertia taken about the body-frame origin."""
        m, c = self.mass, self.lever
        Io = self.inertia_c - m * skew(c) @ skew(c)
        return np.array([m, m * c[0], m * c[1], m * c[2],
                         Io[0, 0], Io[0, 1], Io[1, 1], Io[0, 2], Io[1, 2], Io[2, 2]])


@dataclass
class Frame:
    name: str
    parent: int           # joint index
    R: np.ndarray         # placement relative to the parent joint frame
    t: np.ndarray
    kind: str             # "joint" | "body" | "fixed_joint"


@dataclass
class LinkInertial:
    """A URDF ``<inertial>`` block as written in the file (used by get_phi_prior)."""
    name: str
    mass: float
    xyz: np.ndarray
    rpy: np.ndarray
    I: np.ndarray  # 3x3 about the CoM, in the inertial frame


@dataclass
class LinkVisual:
    link: str
    kind: str             # box | cylinder | sphere | mesh
    params: list
    xyz: np.ndarray
    filename: str = ""


@dataclass
class Model:
    name: str
    floating_base: bool
    joint_names: list
    parents: list
    jtypes: list
    idx_q: list
    idx_v: list
    axes: np.ndarray          # (njoints, 3)
    placements_R: np.ndarray  # (njoints, 3, 3)
    placements_t: np.ndarray  # (njoints, 3)
    inertias: list            # Inertia per joint (index 0 = universe)
    frames: list
    link_inertials: list = field(default_factory=list)
    link_visuals: list = field(default_factory=list)
    lower: list = field(default_factory=list)   # URDF joint limits (nan for universe / free-flyer)
    upper: list = field(default_factory=list)
    # bounding ellipsoids of the listed links' visuals (src/sys_identification.py:235-264), computed when
    # the model is compiled next to its meshes; None entries mark meshes that are not available
    bounding_ellipsoids: list = field(default_factory=list)
    # robot YAML (files/*/<robot>_config.yaml)
    robot_name: str = ""
    robot_mass: float = 0.0
    end_effector_names: list = field(default_factory=list)
    link_names: list = field(default_factory=list)
    gravity: tuple = GRAVITY

    # ---- dimensions ---------------------------------------------------------------------------
    @property
    def njoints(self) -> int:
        return len(self.joint_names)

    @property
    def nb(self) -> int:
        return self.njoints - 1

    @property
    def nq(self) -> int:
        return sum(7 if t == JOINT_FREEFLYER else 1 for t in self.jtypes[1:])

    @property
    def nv(self) -> int:
        return sum(6 if t == JOINT_FREEFLYER else 1 for t in self.jtypes[1:])

    @property
    def base_dof(self) -> int:
        return 6 if self.floating_base else 0

    @property
    def nj(self) -> int:
        return self.nv - self.base_dof

    @property
    def n_ee(self) -> int:
        return len(self.end_effector_names)

    def nv_of(self, i: int) -> int:
        return 6 if self.jtypes[i] == JOINT_FREEFLYER else 1

    def frame_id(self, name: str) -> int:
        for k, f in enumerate(self.frames):
            if f.name == name:
                return k
        raise ValueError(f"frame '{name}' does not exist")

    def contact_frames(self) -> list:
        return [self.frames[self.frame_id(n)] for n in self.end_effector_names]

    def support(self, i: int) -> list:
        """Joint indices on the path universe -> i (root first), excluding the universe."""
        path = []
        while i > 0:
            path.append(i)
            i = self.parents[i]
        return path[::-1]

    def support_dofs(self, i: int) -> list:
        out = []
        for j in self.support(i):
            out.extend(range(self.idx_v[j], self.idx_v[j] + self.nv_of(j)))
        return out

    def depth(self, i: int) -> int:
        return len(self.support(i))

    def phi_pin(self) -> np.ndarray:
        """Concatenated pinocchio dynamic parameters of every body (10*nb), regressor column order."""
        return np.concatenate([self.inertias[i].dynamic_parameters() for i in range(1, self.njoints)])

    # ---- packing for the C ABI ----------------------------------------------------------------
    def pack(self) -> bytes:
        """Binary model consumed by ``sysid_model_create`` (layout documented in include/sysid.h)."""
        nj_ = self.njoints
        cf = self.contact_frames()
        nc = len(cf)
        header = np.zeros(16, dtype="<i4")
        header[:8] = [PACK_MAGIC, PACK_VERSION, self.nq, self.nv, nj_, nc, self.base_dof, self.nj]
        ints = np.concatenate([
            np.asarray(self.parents, dtype="<i4"), np.asarray(self.jtypes, dtype="<i4"),
            np.asarray(self.idx_q, dtype="<i4"), np.asarray(self.idx_v, dtype="<i4"),
            np.asarray([f.parent for f in cf], dtype="<i4"),
        ])
        if ints.size % 2:
            ints = np.concatenate([ints, np.zeros(1, dtype="<i4")])
        dbl = np.concatenate([
            self.axes.reshape(-1), self.placements_R.reshape(-1), self.placements_t.reshape(-1),
            np.array([f.R for f in cf]).reshape(-1) if nc else np.zeros(0),
            np.array([f.t for f in cf]).reshape(-1) if nc else np.zeros(0),
            np.asarray(self.gravity, dtype=float),
        ]).astype("<f8")
        return header.tobytes() + ints.tobytes() + dbl.tobytes()

    # ---- JSON (committed robot descriptions; the GPU box has no /root/reference) --------------
    def to_json(self) -> dict:
        def inert(I: Inertia):
            return {"mass": I.mass, "lever": I.lever.tolist(), "inertia_c": I.inertia_c.tolist()}
        return {
            "format": "sysid-model-1",
            "name": self.name, "floating_base": self.floating_base,
            "joint_names": self.joint_names, "parents": self.parents, "jtypes": self.jtypes,
            "idx_q": self.idx_q, "idx_v": self.idx_v,
            "axes": self.axes.tolist(), "placements_R": self.placements_R.tolist(),
            "placements_t": self.placements_t.tolist(),
            "inertias": [inert(I) for I in self.inertias],
            "frames": [{"name": f.name, "parent": f.parent, "R": f.R.tolist(), "t": f.t.tolist(),
                        "kind": f.kind} for f in self.frames],
            "link_inertials": [{"name": l.name, "mass": l.mass, "xyz": l.xyz.tolist(),
                                "rpy": l.rpy.tolist(), "I": l.I.tolist()} for l in self.link_inertials],
            "link_visuals": [{"link": v.link, "kind": v.kind, "params": list(v.params),
                              "xyz": v.xyz.tolist(), "filename": v.filename} for v in self.link_visuals],
            "robot": {"name": self.robot_name, "mass": self.robot_mass,
                      "end_effectors_frame_names": self.end_effector_names,
                      "link_names": self.link_names},
            "bounding_ellipsoids": [None if e is None else {"link": e["link"], "semi_axes": list(map(float, e["semi_axes"])),
                                                            "center": list(map(float, e["center"]))}
                                    for e in self.bounding_ellipsoids],
            "lower": [None if not np.isfinite(x) else x for x in self.lower],
            "upper": [None if not np.isfinite(x) else x for x in self.upper],
            "gravity": list(self.gravity),
        }

    @staticmethod
    def from_json(d: dict) -> "Model":
        if d.get("format") != "sysid-model-1":
            raise ValueError("not a sysid-model-1 description")
        rob = d.get("robot", {})
        return Model(
            name=d["name"], floating_base=d["floating_base"], joint_names=list(d["joint_names"]),
            parents=list(d["parents"]), jtypes=list(d["jtypes"]), idx_q=list(d["idx_q"]),
            idx_v=list(d["idx_v"]), axes=np.array(d["axes"], dtype=float),
            placements_R=np.array(d["placements_R"], dtype=float),
            placements_t=np.array(d["placements_t"], dtype=float),
            inertias=[Inertia(I["mass"], np.array(I["lever"]), np.array(I["inertia_c"]))
                      for I in d["inertias"]],
            frames=[Frame(f["name"], f["parent"], np.array(f["R"]), np.array(f["t"]), f["kind"])
                    for f in d["frames"]],
            link_inertials=[LinkInertial(l["name"], l["mass"], np.array(l["xyz"]), np.array(l["rpy"]),
                                         np.array(l["I"])) for l in d.get("link_inertials", [])],
            link_visuals=[LinkVisual(v["link"], v["kind"], list(v["params"]), np.array(v["xyz"]),
                                     v.get("filename", "")) for v in d.get("link_visuals", [])],
            robot_name=rob.get("name", ""), robot_mass=rob.get("mass", 0.0),
            end_effector_names=list(rob.get("end_effectors_frame_names", [])),
            link_names=list(rob.get("link_names", [])),
            bounding_ellipsoids=[None if e is None else {"link": e["link"], "semi_axes": np.array(e["semi_axes"]),
                                                         "center": np.array(e["center"])}
                                 for e in d.get("bounding_ellipsoids", [])],
            lower=[np.nan if x is None else x for x in d.get("lower", [])],
            upper=[np.nan if x is None else x for x in d.get("upper", [])],
            gravity=tuple(d.get("gravity", GRAVITY)),
        )

    def save_json(self, path: str) -> None:
        with open(path, "w") as fh:
            json.dump(self.to_json(), fh, indent=1)

    @staticmethod
    def load_json(path: str) -> "Model":
        with open(path) as fh:
            return Model.from_json(json.load(fh))


# ------------------------------------------------------------------------------------------------
# URDF parsing
# ------------------------------------------------------------------------------------------------

def _floats(s: str | None, n: int, default: float = 0.0) -> np.ndarray:
    if s is None:
        return np.full(n, default, dtype=float)
    v = np.array([float(x) for x in s.split()], dtype=float)
    if v.size != n:
        raise ValueError(f"expected {n} numbers, got '{s}'")
    return v


def _origin(el) -> tuple:
    o = el.find("origin") if el is not None else None
    if o is None:
        return np.eye(3), np.zeros(3), np.zeros(3), np.zeros(3)
    xyz = _floats(o.get("xyz"), 3)
    rpy = _floats(o.get("rpy"), 3)
    return rpy_to_matrix(*rpy), xyz, xyz, rpy


def _link_inertia(link) -> tuple:
    """(Inertia in the link frame, LinkInertial as written) for a URDF <link>."""
    inr = link.find("inertial")
    if inr is None:
        return Inertia(), None
    R, t, xyz, rpy = _origin(inr)
    m_el = inr.find("mass")
    mass = float(m_el.get("value")) if m_el is not None else 0.0
    i_el = inr.find("inertia")
    g = (lambda k: float(i_el.get(k, 0.0))) if i_el is not None else (lambda k: 0.0)
    I = np.array([[g("ixx"), g("ixy"), g("ixz")], [g("ixy"), g("iyy"), g("iyz")],
                  [g("ixz"), g("iyz"), g("izz")]])
    return (Inertia(mass, t.copy(), R @ I @ R.T),
            LinkInertial(link.get("name"), mass, xyz, rpy, I))


def _link_visuals(link) -> list:
    out = []
    for vis in link.findall("visual"):
        geo = vis.find("geometry")
        if geo is None:
            continue
        _, _, xyz, _ = _origin(vis)
        name = link.get("name")
        if geo.find("box") is not None:
            out.append(LinkVisual(name, "box", _floats(geo.find("box").get("size"), 3).tolist(), xyz))
        elif geo.find("cylinder") is not None:
            c = geo.find("cylinder")
            out.append(LinkVisual(name, "cylinder", [float(c.get("radius")), float(c.get("length"))], xyz))
        elif geo.find("sphere") is not None:
            out.append(LinkVisual(name, "sphere", [float(geo.find("sphere").get("radius"))], xyz))
        elif geo.find("mesh") is not None:
            out.append(LinkVisual(name, "mesh", [], xyz, geo.find("mesh").get("filename", "")))
    return out


def mesh_aabb(path: str) -> tuple:
    """(min, max) corners of the vertices of an OBJ or STL (ascii/binary) mesh file."""
    with open(path, "rb") as fh:
        raw = fh.read()
    ext = os.path.splitext(path)[1].lower()
    if ext == ".obj":
        pts = [list(map(float, ln.split()[1:4])) for ln in raw.decode(errors="ignore").splitlines()
               if ln.startswith("v ")]
        V = np.array(pts, dtype=float)
    elif ext == ".stl":
        n = struct.unpack_from("<I", raw, 80)[0] if len(raw) >= 84 else -1
        if len(raw) == 84 + 50 * n:
            rec = np.frombuffer(raw, dtype=np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")]),
                                count=n, offset=84)
            V = rec["v"].reshape(-1, 3).astype(float)
        else:
            V = np.array([list(map(float, ln.split()[1:4])) for ln in raw.decode(errors="ignore").splitlines()
                          if ln.strip().startswith("vertex")], dtype=float)
    else:
        raise ValueError(f"unsupported mesh format: {path}")
    if V.size == 0:
        raise ValueError(f"no vertices in {path}")
    return V.min(axis=0), V.max(axis=0)


def bounding_ellipsoids(model: "Model", urdf_file: str, mesh_root: str | None = None) -> list:
    """Restates ``_compute_bounding_ellipsoids`` (src/sys_identification.py:235-264): for every visual of
    every URDF link listed in the robot YAML, in URDF order, an axis-aligned ellipsoid.
    Box: semi-axes size/2; cylinder: (r, r, l/2); sphere: (r, r, r); all centred at the visual origin.
    Mesh: semi-axes = AABB extents / 2, centre = AABB centre + visual origin.  The reference resolves
    ``filename[10:]`` (strips "package://") under ``files/``; here ``mesh_root`` plays that role and
    plain relative paths resolve next to the URDF.  A missing mesh file gives a ``None`` entry."""
    out = []
    root = mesh_root or os.path.dirname(os.path.dirname(os.path.abspath(urdf_file)))
    for v in model.link_visuals:
        if v.link not in model.link_names:
            continue
        if v.kind == "box":
            semi, center = np.asarray(v.params) / 2.0, np.asarray(v.xyz, dtype=float)
        elif v.kind == "cylinder":
            semi, center = np.array([v.params[0], v.params[0], v.params[1] / 2.0]), np.asarray(v.xyz, dtype=float)
        elif v.kind == "sphere":
            semi, center = np.array([v.params[0]] * 3), np.asarray(v.xyz, dtype=float)
        else:
            fn = v.filename
            path = os.path.join(root, fn[len("package://"):]) if fn.startswith("package://") else \
                os.path.join(os.path.dirname(os.path.abspath(urdf_file)), fn)
            if not os.path.exists(path):
                out.append(None)
                continue
            lo, hi = mesh_aabb(path)
            semi, center = (hi - lo) / 2.0, (hi + lo) / 2.0 + np.asarray(v.xyz, dtype=float)
        out.append({"link": v.link, "semi_axes": semi, "center": center})
    return out


def load_robot_config(config_file: str) -> dict:
    """Robot YAML as read at src/sys_identification.py:40-55."""
    import yaml
    with open(config_file) as fh:
        cfg = yaml.safe_load(fh)
    return cfg.get("robot", {})


def build_model_from_urdf(urdf_file: str, config_file: str | None = None,
                          floating_base: bool = True) -> Model:
    """Parse a URDF into a :class:`Model` (see module docstring for the rules)."""
    root = ET.parse(urdf_file).getroot()
    links = {l.get("name"): l for l in root.findall("link")}
    joints = root.findall("joint")
    children: dict = {name: [] for name in links}
    child_links = set()
    for j in joints:
        p = j.find("parent").get("link")
        c = j.find("child").get("link")
        children.setdefault(p, []).append(j)
        child_links.add(c)
    roots = [n for n in links if n not in child_links]
    if len(roots) != 1:
        raise ValueError(f"URDF must have exactly one root link, found {roots}")
    root_link = roots[0]
    for k in children:
        children[k].sort(key=lambda j: j.get("name"))

    names, parents, jtypes, idx_q, idx_v = ["universe"], [0], [JOINT_UNIVERSE], [0], [0]
    axes, PR, Pt, inertias = [np.zeros(3)], [np.eye(3)], [np.zeros(3)], [Inertia()]
    frames = [Frame("universe", 0, np.eye(3), np.zeros(3), "joint")]
    lower, upper = [np.nan], [np.nan]
    counters = {"q": 0, "v": 0}

    def add_joint(name, parent, jtype, axis, R, t, lim=(np.nan, np.nan)):
        lower.append(lim[0])
        upper.append(lim[1])
        names.append(name)
        parents.append(parent)
        jtypes.append(jtype)
        idx_q.append(counters["q"])
        idx_v.append(counters["v"])
        counters["q"] += 7 if jtype == JOINT_FREEFLYER else 1
        counters["v"] += 6 if jtype == JOINT_FREEFLYER else 1
        axes.append(np.asarray(axis, dtype=float))
        PR.append(R)
        Pt.append(t)
        inertias.append(Inertia())
        frames.append(Frame(name, len(names) - 1, np.eye(3), np.zeros(3), "joint"))
        return len(names) - 1

    def visit(link_name, joint_id, R_lj, t_lj):
        """``link_name`` is rigidly attached to joint ``joint_id`` with placement (R_lj, t_lj)."""
        Y, _ = _link_inertia(links[link_name])
        inertias[joint_id] = inertias[joint_id] + Y.transformed(R_lj, t_lj)
        for j in children.get(link_name, []):
            jt = j.get("type")
            R_o, t_o, _, _ = _origin(j)
            R_c = R_lj @ R_o
            t_c = R_lj @ t_o + t_lj
            child = j.find("child").get("link")
            if jt in ("revolute", "continuous"):
                if jt == "continuous":
                    raise NotImplementedError("continuous joints (JointModelRUB*) are not supported")
                ax_el = j.find("axis")
                axis = _floats(ax_el.get("xyz") if ax_el is not None else "1 0 0", 3)
                nrm = np.linalg.norm(axis)
                if nrm == 0.0:
                    raise ValueError(f"joint {j.get('name')} has a zero axis")
                lim_el = j.find("limit")
                lim = (float(lim_el.get("lower", "nan")), float(lim_el.get("upper", "nan"))) \
                    if lim_el is not None else (np.nan, np.nan)
                jid = add_joint(j.get("name"), joint_id, JOINT_REVOLUTE, axis / nrm, R_c, t_c, lim)
                frames.append(Frame(child, jid, np.eye(3), np.zeros(3), "body"))
                visit(child, jid, np.eye(3), np.zeros(3))
            elif jt == "fixed":
                frames.append(Frame(j.get("name"), joint_id, R_c, t_c, "fixed_joint"))
                frames.append(Frame(child, joint_id, R_c, t_c, "body"))
                visit(child, joint_id, R_c, t_c)
            else:
                raise NotImplementedError(f"URDF joint type '{jt}' ({j.get('name')}) is not supported")

    if floating_base:
        jid = add_joint("root_joint", 0, JOINT_FREEFLYER, np.zeros(3), np.eye(3), np.zeros(3))
        frames.append(Frame(root_link, jid, np.eye(3), np.zeros(3), "body"))
        visit(root_link, jid, np.eye(3), np.zeros(3))
    else:
        frames.append(Frame(root_link, 0, np.eye(3), np.zeros(3), "body"))
        visit(root_link, 0, np.eye(3), np.zeros(3))

    link_inertials = []
    link_visuals = []
    for l in root.findall("link"):
        _, li = _link_inertia(l)
        if li is not None:
            link_inertials.append(li)
        link_visuals.extend(_link_visuals(l))

    model = Model(
        name=root.get("name", ""), floating_base=floating_base, joint_names=names,
        parents=parents, jtypes=jtypes, idx_q=idx_q, idx_v=idx_v,
        axes=np.array(axes), placements_R=np.array(PR), placements_t=np.array(Pt),
        inertias=inertias, frames=frames, link_inertials=link_inertials, link_visuals=link_visuals,
        lower=lower, upper=upper,
    )
    if config_file is not None:
        rc = load_robot_config(config_file)
        model.robot_name = rc.get("name") or ""
        model.robot_mass = rc.get("mass") or 0.0
        model.end_effector_names = list(rc.get("end_effectors_frame_names", []) or [])
        model.link_names = list(rc.get("link_names", []) or [])
        for n in model.end_effector_names:
            model.frame_id(n)  # raises like pinocchio's getFrameId on an unknown name
        model.bounding_ellipsoids = bounding_ellipsoids(model, urdf_file)
    return model


# ------------------------------------------------------------------------------------------------
# Committed robot descriptions (derived from the reference's URDF + YAML by tools/make_robots.py)
# ------------------------------------------------------------------------------------------------

ROBOT_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "robots")
ROBOTS = ("solo12", "spot", "g1_29dof", "solo12_fixed")


def load_robot(name: str) -> Model:
    path = os.path.join(ROBOT_DIR, f"{name}.json")
    if not os.path.exists(path):
        raise ValueError(f"unknown robot '{name}' (known: {', '.join(ROBOTS)})")
    return Model.load_json(path)


def unpack_header(blob: bytes) -> dict:
    h = struct.unpack_from("<16i", blob, 0)
    return {"magic": h[0], "version": h[1], "nq": h[2], "nv": h[3], "njoints": h[4],
            "n_contact": h[5], "base_dof": h[6], "nj": h[7]}
