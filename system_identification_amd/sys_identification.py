"""``SystemIdentification`` — drop-in for src/sys_identification.py:10 backed by the MI355X engine.

Same constructor, attributes and method names as the reference class.  The per-sample hot-path methods
(``get_proj_regressor_torque`` :401, ``get_proj_friction_regressors`` :412) run on the GPU as batches of
one; the batched entry points (``build_stacked``, ``build_normal_equations``) are what the demo-level
loops (demo/spot_identification.py:37-56) become.  Host-side bookkeeping (phi_prior, ellipsoids,
printing) is restated in numpy.  There is no CPU fallback for the regressor/projector: a missing
engine or GPU raises.
"""
from __future__ import annotations

import os

import numpy as np

from . import engine as _engine
from .model import Model, build_model_from_urdf, load_robot, rpy_to_matrix, skew
from .solver import ellipsoid_matrix


def _resolve_model(urdf_file, config_file, floating_base) -> Model:
    """A URDF path (parsed here, like pin.buildModelFromUrdf), a committed model JSON, or a robot name."""
    if isinstance(urdf_file, Model):
        return urdf_file
    s = str(urdf_file)
    if s.endswith(".urdf"):
        return build_model_from_urdf(s, config_file, floating_base=floating_base)
    if s.endswith(".json"):
        m = Model.load_json(s)
    else:
        m = load_robot(s)
    if bool(m.floating_base) != bool(floating_base):
        raise ValueError(f"model '{s}' was compiled with floating_base={m.floating_base}")
    return m


class SystemIdentification(object):
    def __init__(self, urdf_file, config_file=None, floating_base=True, device: int = 0):
        self._urdf_path = urdf_file
        self._floating_base = floating_base
        self.model = _resolve_model(urdf_file, config_file, floating_base)
        self.nq = self.model.nq
        self.nv = self.model.nv
        # selection matrix (src/sys_identification.py:29-37)
        self._base_dof = 6 if floating_base else 0
        self.joints_dof = self.nv - self._base_dof
        self._S = np.zeros((self.joints_dof, self.nv))
        self._S[:, self._base_dof:] = np.eye(self.joints_dof)
        # robot YAML (:40-55)
        self._robot_name = self.model.robot_name
        self._robot_mass = self.model.robot_mass
        self._link_names = list(self.model.link_names)
        self._end_eff_frame_names = list(self.model.end_effector_names)
        self._endeff_ids = [self.model.frame_id(n) for n in self._end_eff_frame_names]
        self._nb_ee = len(self._end_eff_frame_names)
        # parameters (:59-66)
        self._num_inertial_params = 10
        self._num_links = len(self._link_names)
        self._phi_prior = np.zeros((self._num_inertial_params * self._num_links), dtype=np.float32)
        self.B_v = np.eye(self.joints_dof)
        self.B_c = np.eye(self.joints_dof)
        self._bounding_ellipsoids = list(self.model.bounding_ellipsoids)
        self._device = device
        self._engine = None
        self._cache_key = None
        self._cache = None

    # ---- engine ---------------------------------------------------------------------------------
    @property
    def engine(self) -> "_engine.Engine":
        if self._engine is None:
            self._engine = _engine.Engine(self.model, device=self._device)
        return self._engine

    @staticmethod
    def _as_channels(a, rows, name):
        a = np.asarray(a, dtype=np.float64)
        if a.ndim == 1:
            a = a.reshape(-1, 1)
        if a.shape[0] != rows:
            raise ValueError(f"{name}: expected {rows} rows (channels), got shape {a.shape}")
        return a

    def build_stacked(self, q, dq, ddq, tau, cnt, flags: int = _engine.EMIT_ALL) -> dict:
        """Batched hot path.  Inputs channel-major (channels x N) as read_data returns them.
        Returns the stacked arrays the reference builds at demo/spot_identification.py:84-87
        (Y_proj, tau_proj, B_v, B_c) and, with EMIT_GRAM, the normal equations."""
        ch = self._channels(q, dq, ddq, tau, cnt)  # shape errors before the device is touched
        return self.engine.build(*ch, flags)

    def _channels(self, q, dq, ddq, tau, cnt):
        m = self.model
        q = self._as_channels(q, m.nq, "q")
        dq = self._as_channels(dq, m.nv, "dq")
        ddq = self._as_channels(ddq, m.nv, "ddq")
        tau = self._as_channels(tau, m.nj, "tau") if m.nj else np.zeros((0, q.shape[1]))
        cnt = self._as_channels(cnt, m.n_ee, "contact") if m.n_ee else np.zeros((0, q.shape[1]))
        return q, dq, ddq, tau, cnt

    def build_normal_equations(self, q, dq, ddq, tau, cnt) -> dict:
        """Gram of the stacked system: {gram: AᵀA, Atb: Aᵀb, btb: bᵀb, num_rows: N·nv} (src/solver.py:186-190)."""
        return self.build_stacked(q, dq, ddq, tau, cnt, _engine.EMIT_GRAM)

    def _stacked_cached(self, q, dq, ddq, tau, cnt):
        """The demo calls get_projected_y_tau and then get_projected_friction_regressors on the same arrays;
        one engine pass produces both, so the second call reuses it.  The cache key holds the dtype, shape and
        a content hash of every input, so an array modified in between (even keeping its sum, e.g. reordered
        samples) is recomputed."""
        import hashlib

        def fp(a):
            a = np.ascontiguousarray(np.asarray(a))
            return (a.dtype.str, a.shape, hashlib.blake2b(a.tobytes(), digest_size=16).hexdigest())
        key = tuple(fp(a) for a in (q, dq, ddq, cnt))
        tkey = fp(tau) if tau is not None else None
        if self._cache is not None and self._cache_key[0] == key and (tau is None or self._cache_key[1] == tkey):
            return self._cache
        if tau is None:
            tau = np.zeros((self.model.nj, self._as_channels(q, self.model.nq, "q").shape[1]))
            tkey = fp(tau)
        out = self.build_stacked(q, dq, ddq, tau, cnt, _engine.EMIT_Y | _engine.EMIT_TAU | _engine.EMIT_FRICTION)
        self._cache_key, self._cache = (key, tkey), out
        return out

    # ---- per-sample reference API (src/sys_identification.py:391-418) ------------------------
    def get_full_regressor_force(self, q, dq, ddq, tau, ee_force, cnt):
        """Y @ phi = F for the floating-base dynamics M ddq + h = Sᵀ tau + J_cᵀ lambda (:391-399); 1-D inputs
        give one sample like the reference, channel-major 2-D inputs a stacked batch."""
        m = self.model
        q = self._as_channels(q, m.nq, "q")
        N = q.shape[1]
        tau = self._as_channels(tau, m.nj, "tau") if m.nj else np.zeros((0, N))
        cnt = self._as_channels(cnt, m.n_ee, "contact") if m.n_ee else np.zeros((0, N))
        f = self._as_channels(ee_force, 3 * m.n_ee, "ee_force") if m.n_ee else np.zeros((0, N))
        dq = self._as_channels(dq, m.nv, "dq")
        ddq = self._as_channels(ddq, m.nv, "ddq")
        return self.engine.build_full(q, dq, ddq, tau, f, cnt)

    def get_proj_regressor_torque(self, q, dq, ddq, tau, cnt):
        out = self.build_stacked(q, dq, ddq, tau, cnt, _engine.EMIT_Y | _engine.EMIT_TAU)
        return out["Y_proj"], out["tau_proj"]

    def get_proj_friction_regressors(self, q, dq, ddq, cnt):
        tau = np.zeros(self.model.nj)
        out = self.build_stacked(q, dq, ddq, tau, cnt, _engine.EMIT_FRICTION)
        return out["B_v"], out["B_c"]

    # ---- reference accessors (:288-322) --------------------------------------------------------
    def get_robot_mass(self):
        return self._robot_mass

    def get_num_links(self):
        return self._num_links

    def get_bounding_ellipsoids(self):
        if any(e is None for e in self._bounding_ellipsoids):
            missing = [i for i, e in enumerate(self._bounding_ellipsoids) if e is None]
            raise ValueError(f"bounding ellipsoid(s) {missing} need mesh files that are not available "
                             "(e.g. Spot's meshes/base/visual/body.obj is not in the reference checkout)")
        return self._bounding_ellipsoids

    def _compute_inertial_params(self):
        """:266-286 — URDF inertials of the listed links, in URDF order."""
        self.inertial_params = []
        for li in self.model.link_inertials:
            if li.name in self._link_names:
                self.inertial_params.append({"mass": li.mass, "com": np.asarray(li.xyz), "rpy": np.asarray(li.rpy),
                                             "I_c": np.asarray(li.I)})

    def get_phi_prior(self):
        """:297-322 — [m, h, I_bar row 0, I_bar[1,1:], I_bar[2,2]] per link, float32, inertia about the
        link frame origin in the order (Ixx, Ixy, Ixz, Iyy, Iyz, Izz)."""
        self._compute_inertial_params()
        for i in range(self._num_links):
            ip = self.inertial_params[i]
            mass, com = ip["mass"], ip["com"]
            h = mass * com
            R = rpy_to_matrix(*ip["rpy"])
            I_rot = R @ ip["I_c"] @ R.T
            I_bar = I_rot + (mass * skew(com) @ skew(com).T)
            j = 10 * i
            self._phi_prior[j] = mass
            self._phi_prior[j + 1:j + 4] = h
            self._phi_prior[j + 4:j + 7] = I_bar[0, :]
            self._phi_prior[j + 7:j + 9] = I_bar[1, 1:]
            self._phi_prior[j + 9] = I_bar[2, 2]
        return self._phi_prior

    def get_physical_consistency(self, phi):
        """:324-389 — minimum eigenvalues of the LMI matrices and trace(J Q) per link."""
        eig_Ibar, eig_I, eig_J, eig_com, trace_JQ = [], [], [], [], []
        ells = self.get_bounding_ellipsoids()
        for idx in range(self._num_links):
            j = idx * 10
            m, hx, hy, hz, Ixx, Ixy, Ixz, Iyy, Iyz, Izz = phi[j:j + 10]
            h = np.array([hx, hy, hz])
            semi, center = np.asarray(ells[idx]["semi_axes"]), np.asarray(ells[idx]["center"])
            I_bar = np.array([[Ixx, Ixy, Ixz], [Ixy, Iyy, Iyz], [Ixz, Iyz, Izz]])
            I6 = np.zeros((6, 6), dtype=np.float32)
            I6[:3, :3] = I_bar
            I6[:3, 3:] = skew(h)
            I6[3:, :3] = skew(h).T
            I6[3:, 3:] = m * np.eye(3)
            J = np.zeros((4, 4), dtype=np.float32)
            J[:3, :3] = 0.5 * np.trace(I_bar) * np.eye(3) - I_bar
            J[:3, 3] = h
            J[3, :3] = h
            J[3, 3] = m
            Qf = ellipsoid_matrix(semi, center)  # float32, as solver.py:65-74 and :360-366 build it
            C = np.zeros((4, 4), dtype=np.float32)
            C[0, 0] = m
            C[0, 1:] = h - m * center
            C[1:, 0] = h - m * center
            C[1:, 1:] = m * np.diag(semi) ** 2
            eig_Ibar.append(np.min(np.linalg.eigvals(I_bar)))
            eig_I.append(np.min(np.linalg.eigvals(I6)))
            eig_J.append(np.min(np.linalg.eigvals(J)))
            eig_com.append(np.min(np.linalg.eigvals(C)))
            trace_JQ.append(np.trace(J @ Qf))
        return eig_Ibar, eig_I, eig_J, eig_com, trace_JQ

    # ---- reporting (:421-490), batched ---------------------------------------------------------
    def tau_prediction_errors(self, q, dq, ddq, torque, cnt, phi):
        """Rows ``6:`` of (Y_proj phi) and tau_proj for every sample (:426-431), from one engine pass."""
        out = self._stacked_cached(q, dq, ddq, torque, cnt)
        nv, bd = self.nv, self._base_dof
        pred = (out["Y_proj"] @ np.asarray(phi, dtype=np.float64)).reshape(-1, nv)[:, bd:]
        meas = out["tau_proj"].reshape(-1, nv)[:, bd:]
        return pred, meas

    def tau_prediction_rmse(self, q, dq, ddq, torque, cnt, phi):
        """(rmse_total, per-joint RMSE) of :432-433 from one device reduction (K4): the stacked panel is
        built on the GPU and never copied back.  rmse_total keeps the reference's definition, the mean over
        samples of the squared error norm."""
        ch = self._channels(q, dq, ddq, torque, cnt)
        N = ch[0].shape[1]
        err = self.engine.tau_error(*ch, np.asarray(phi, dtype=np.float64))
        bd = self._base_dof
        return float(np.sum(err[bd:]) / N), np.sqrt(err[bd:] / N)

    def print_tau_prediction_rmse(self, q, dq, ddq, torque, cnt, phi, param_name):
        rmse_total, joint_tau_rmse = self.tau_prediction_rmse(q, dq, ddq, torque, cnt, phi)
        print("\n--------------------Torque Prediction Errors--------------------")
        print(f'RMSE for joint torques prediction using {param_name} parameters: total= {rmse_total}\n'
              f'per_joints={joint_tau_rmse}')
        return rmse_total, joint_tau_rmse

    def print_inertial_params(self, prior, identified):
        total_m_prior = 0
        total_m_ident = 0
        self._cell_width = 13
        for i in range(self._num_links):
            expression = f'Inertial Parameters of "{self._link_names[i]}"'
            dash_length = (69 - len(expression)) // 2
            print(f'\n{"-" * dash_length} {expression} {"-" * (69 - len(expression) - dash_length)}')
            w = self._cell_width
            print(f'|{"Parameter":<{w}}|{"A priori":<{w}}|{"Identified":<{w}}|{"Change":<{w}}|{"error %":<{w}}|')
            index = 10 * i
            m_prior, m_ident = prior[index], identified[index]
            com_prior = prior[index + 1:index + 4] / m_prior
            com_ident = identified[index + 1:index + 4] / m_ident
            inertia_prior = prior[index + 4:index + 10]
            inertia_ident = identified[index + 4:index + 10]
            self._print_table("mass (kg)", m_prior, m_ident)
            for k, n in enumerate(("c_x (m)", "c_y (m)", "c_z (m)")):
                self._print_table(n, com_prior[k], com_ident[k])
            for k, n in enumerate(("I_xx", "I_xy", "I_xz", "I_yy", "I_yz", "I_zz")):
                self._print_table(f"{n} (kg.m^2)", inertia_prior[k], inertia_ident[k])
            total_m_prior += m_prior
            total_m_ident += m_ident
        print(f'\nRobot total mass: {total_m_prior} ---- Identified total mass: {total_m_ident}')

    def _print_table(self, description, prior, ident):
        precision = 6
        change = ident - prior
        with np.errstate(divide="ignore", invalid="ignore"):
            error = np.divide(change, np.abs(prior), where=prior != 0) * 100
        error = np.where(np.abs(prior) <= 1e-8, np.nan, error)
        w = self._cell_width
        print(f'|{description:<{w}}|{prior:>{w}.{precision}f}|{ident:>{w}.{precision}f}|'
              f'{change:>{w}.{precision}f}|{float(error):>{w}.{1}f}|')


def default_robot_paths(robot: str, reference_root: str = "/root/reference"):
    """(urdf, yaml) of the reference's robots when its checkout is present (build container only)."""
    table = {
        "solo12": ("files/solo_description/solo12.urdf", "files/solo_description/solo12_config.yaml"),
        "spot": ("files/spot_description/spot.urdf", "files/spot_description/spot_config.yaml"),
    }
    u, c = table[robot]
    return os.path.join(reference_root, u), os.path.join(reference_root, c)
