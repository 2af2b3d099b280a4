"""Host-side mirror of the reference API (no GPU needed for these parts)."""
import numpy as np
import pytest

from system_identification_amd.model import load_robot
from system_identification_amd.solver import Solver, pullback_metric
from system_identification_amd.sys_identification import SystemIdentification
from tests.conftest import REFERENCE, needs_reference


def test_construct_from_robot_name_and_reference_attributes():
    s = SystemIdentification("spot", None, floating_base=True)
    assert (s.nq, s.nv, s.joints_dof, s._base_dof) == (19, 18, 12, 6)
    assert s._S.shape == (12, 18) and np.array_equal(s._S[:, 6:], np.eye(12))
    assert s.get_robot_mass() == 34.0 and s.get_num_links() == 13
    assert s._end_eff_frame_names == ["fl_foot", "fr_foot", "rl_foot", "rr_foot"]
    assert s.B_v.shape == (12, 12)


@needs_reference
def test_construct_from_urdf_like_the_reference():
    import os
    s = SystemIdentification(os.path.join(REFERENCE, "files/solo_description/solo12.urdf"),
                             os.path.join(REFERENCE, "files/solo_description/solo12_config.yaml"), floating_base=True)
    assert s.model.to_json() == load_robot("solo12").to_json()


def test_phi_prior_matches_pinocchio_parameters_up_to_inertia_order():
    """get_phi_prior (src/sys_identification.py:297-322) stores (Ixx, Ixy, Ixz, Iyy, Iyz, Izz) about the
    link frame origin; pinocchio's regressor uses (Ixx, Ixy, Iyy, Ixz, Iyz, Izz) (the latent order quirk)."""
    s = SystemIdentification("solo12")
    phi = s.get_phi_prior()
    assert phi.dtype == np.float32 and phi.shape == (130,)
    pin = s.model.phi_pin()
    # solo12: one URDF link per pinocchio body, listed in the same order
    for i in range(13):
        a, b = phi[10 * i:10 * i + 10].astype(float), pin[10 * i:10 * i + 10]
        assert np.allclose(a[:4], b[:4], rtol=1e-6, atol=1e-7)
        assert np.allclose(a[[4, 5, 6, 7, 8, 9]], b[[4, 5, 7, 6, 8, 9]], rtol=1e-5, atol=1e-7)


def test_bounding_ellipsoids_and_missing_mesh():
    s = SystemIdentification("solo12")
    e = s.get_bounding_ellipsoids()
    assert len(e) == 13 and all(np.all(np.asarray(x["semi_axes"]) > 0) for x in e)
    with pytest.raises(ValueError):
        SystemIdentification("spot").get_bounding_ellipsoids()  # body.obj is a missing blob


def test_physical_consistency_of_prior():
    s = SystemIdentification("solo12")
    phi = s.get_phi_prior().astype(float)
    ev_Ibar, ev_I, ev_J, ev_com, tr = s.get_physical_consistency(phi)
    assert min(ev_J) > 0 and min(ev_I) > 0


def test_llsq_from_normal_equations_equals_stacked():
    rng = np.random.default_rng(0)
    R, n, nd = 400, 30, 3
    A = rng.normal(size=(R, n + 2 * nd))
    A[:, 5] = A[:, 6]  # rank deficiency like unidentifiable inertial combinations
    b = rng.normal(size=R)
    Y = A[:, :n]
    s1 = Solver(Y, b, 3, np.zeros(n), 1.0, None)
    ne = {"gram": A.T @ A, "Atb": A.T @ b, "btb": float(b @ b), "num_rows": R}
    s2 = Solver.from_normal_equations(ne, 3, np.zeros(n), 1.0, None, friction=True)
    assert s2._num_samples == R and s2._nx == n and s2.ndof == nd
    x1, x2 = s1.solve_llsq_svd(), s2.solve_llsq_svd()
    assert np.allclose(x1, x2, atol=1e-8)


def test_pullback_metric_is_spd():
    s = SystemIdentification("solo12")
    phi = s.get_phi_prior().astype(float)
    M = pullback_metric(phi[10:20])
    assert np.all(np.linalg.eigvalsh(M) > 0)


def test_fully_consistent_needs_cvxpy():
    try:
        import cvxpy  # noqa: F401
        pytest.skip("cvxpy installed")
    except ImportError:
        pass
    s = Solver(np.eye(20), np.ones(20), 2, np.zeros(20), 1.0, None)
    with pytest.raises(ImportError):
        s.solve_fully_consistent()


def test_shape_errors_are_value_errors():
    s = SystemIdentification("spot")
    with pytest.raises(ValueError):
        s.build_stacked(np.zeros((18, 3)), np.zeros((18, 3)), np.zeros((18, 3)), np.zeros((12, 3)), np.zeros((4, 3)))


def test_normal_equations_checkpoint_round_trip(tmp_path):
    from system_identification_amd.solver import load_normal_equations, save_normal_equations
    rng = np.random.default_rng(0)
    A = rng.standard_normal((40, 7))
    ne = {"gram": A.T @ A, "Atb": A.T @ A[:, 0], "btb": 3.25, "num_rows": 40}
    save_normal_equations(tmp_path / "ne.npz", ne)
    back = load_normal_equations(tmp_path / "ne.npz")
    assert np.array_equal(back["gram"], ne["gram"]) and np.array_equal(back["Atb"], ne["Atb"])
    assert back["btb"] == 3.25 and back["num_rows"] == 40


@pytest.mark.parametrize("robot", ["spot", "solo12"])
def test_llsq_gram_path_on_real_panel(robot):
    """the Gram-form llsq on a real projected regressor (oracle panel, 400 samples), whose columns
    have structural rank deficiency (unidentifiable inertial combinations).  The minimum-norm solutions of the
    stacked SVD (reference solver.py:32-39) and of the Gram must agree where the data identifies phi: the
    predicted torques Y phi, and phi projected onto the right singular vectors with sigma > 1e-6 sigma_max."""
    from oracle.ref_c import COracle
    from system_identification_amd.model import load_robot
    from system_identification_amd.synthetic import generate
    model = load_robot(robot)
    d = generate(model, 400, config_index=2)
    out = COracle(model).build(d["q"], d["dq"], d["ddq"], d["tau"], d["contact"], gram=False)
    Y, t = out["Y_proj"], out["tau_proj"]
    n = Y.shape[1]
    nl = n // 10
    phi_s = Solver(Y, t, nl, np.zeros(n), 1.0, None).solve_llsq_svd()
    ne = {"gram": Y.T @ Y, "Atb": Y.T @ t, "btb": float(t @ t), "num_rows": Y.shape[0]}
    phi_g = Solver.from_normal_equations(ne, nl, np.zeros(n), 1.0, None, friction=False).solve_llsq_svd()
    assert np.all(np.isfinite(phi_g))
    U, sig, VT = np.linalg.svd(Y, full_matrices=False)
    assert sig[-1] < 1e-10 * sig[0]  # the panel really is rank deficient
    ident = VT[sig > 1e-6 * sig[0]]
    a, b = ident @ phi_s, ident @ phi_g
    assert np.linalg.norm(a - b) <= 1e-6 * np.linalg.norm(a)
    ps, pg = Y @ phi_s, Y @ phi_g
    assert np.linalg.norm(ps - pg) <= 1e-6 * np.linalg.norm(ps)
    # the Gram solution does not blow up along the unidentifiable directions
    assert np.linalg.norm(phi_g) <= 1.5 * np.linalg.norm(phi_s)


def test_prior_table_matches_the_reference_printed_output(capsys):
    """The one output the reference ships (demo/RUN_DEMO.md:10-21): the 'A priori' column that
    print_inertial_params (src/sys_identification.py:439-490) prints for Spot's front_left_hip, from
    get_phi_prior (:297-322).  Pins the host prior and the table format, not the hot path."""
    import json
    import os
    from system_identification_amd.sys_identification import SystemIdentification
    fx = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "run_demo_front_left_hip.json")))
    s = SystemIdentification("spot")
    prior = s.get_phi_prior()
    s.print_inertial_params(prior, prior)
    lines = capsys.readouterr().out.splitlines()
    i = next(k for k, ln in enumerate(lines) if f'"{fx["link"]}"' in ln)
    assert lines[i + 1] == fx["header"]
    for k, (label, value) in enumerate(fx["a_priori"]):
        cells = lines[i + 2 + k].split("|")
        assert cells[1].strip() == label and cells[2].strip() == value, (label, cells)
        assert len(cells[2]) == 13  # the reference's 13-wide right-aligned cell


@pytest.mark.parametrize("robot,friction", [("spot", True), ("solo12", False)])
def test_gram_form_data_term_equals_stacked(robot, friction):
    """f1: the data term CVXPY minimises in the Gram form, ‖R x‖² - 2 gᵀx + bᵀb with R from the
    clipped eigendecomposition of G (solver.gram_data_term), equals the reference's sum_squares(A x - b)
    (src/solver.py:186-190) on the oracle's stacked A for random x, scaled by 1/(2 rows) as in :190."""
    from oracle.ref_c import COracle
    from system_identification_amd.model import load_robot
    from system_identification_amd.solver import gram_data_term, gram_data_value
    from system_identification_amd.synthetic import generate
    model = load_robot(robot)
    d = generate(model, 300, config_index=4)
    o = COracle(model).build(d["q"], d["dq"], d["ddq"], d["tau"], d["contact"])
    A = np.hstack([o["Y_proj"], o["B_v"], o["B_c"]]) if friction else o["Y_proj"]
    b = o["tau_proj"]
    W = A.shape[1]
    G, g = (o["gram"], o["Atb"]) if friction else (o["gram"][:W, :W], o["Atb"][:W])
    R, g, btb = gram_data_term(G, g, o["btb"])
    rows = A.shape[0]
    assert rows == 300 * model.nv
    rng = np.random.default_rng(7)
    for scale in (1e-3, 1.0, 1e2):
        x = rng.standard_normal(W) * scale
        ref_val = 0.5 * float(np.sum((A @ x - b) ** 2)) / rows
        val = 0.5 * gram_data_value(R, g, btb, x) / rows
        assert abs(val - ref_val) <= 1e-10 * abs(ref_val), (scale, val, ref_val)


def test_gram_llsq_noise_floor_is_pinned():
    """the Gram-form llsq cuts eigenvalues at n·eps·w_max (directions with sigma below ~sqrt(n eps)
    sigma_max), where the stacked SVD keeps everything above 1e-15 sigma_max (src/solver.py:37).  A direction at
    1e-8 sigma_max is identified by the stacked path and dropped by the Gram path (its eigenvalue 1e-16 w_max is
    below the squaring's rounding floor), while one at 1e-5 sigma_max is identified by both."""
    rng = np.random.default_rng(11)
    m, n = 400, 20
    U, _ = np.linalg.qr(rng.standard_normal((m, n)))
    V, _ = np.linalg.qr(rng.standard_normal((n, n)))
    sig = np.logspace(0, -3, n)
    sig[-2], sig[-1] = 1e-5, 1e-8
    Y = (U * sig) @ V.T
    c = np.ones(n)
    t = (U * sig) @ c  # tau = Y V c: every direction carries a unit coefficient
    phi_s = Solver(Y, t, 2, np.zeros(n), 1.0, None).solve_llsq_svd()
    ne = {"gram": Y.T @ Y, "Atb": Y.T @ t, "btb": float(t @ t), "num_rows": m}
    phi_g = Solver.from_normal_equations(ne, 2, np.zeros(n), 1.0, None, friction=False).solve_llsq_svd()
    cs, cg = V.T @ phi_s, V.T @ phi_g
    assert abs(cs[-2] - 1.0) < 1e-6 and abs(cg[-2] - 1.0) < 1e-3   # sigma = 1e-5 sigma_max: both
    assert abs(cs[-1] - 1.0) < 1e-3 and abs(cg[-1]) < 1e-6          # sigma = 1e-8: stacked only


def test_bench_traffic_source_is_the_newest_profile(tmp_path, monkeypatch):
    """bench.py's roofline `traffic` comes from the newest committed PMC summary of the same workload:
    r01_v10 after r01_v9 (numbers compared as numbers), r03_p after r03_m (same round: the later tag)."""
    import json
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    for name, fetch in [("r01_v9", 1.0), ("r01_v10", 2.0), ("r03_m", 3.0), ("r03_p", 4.0), ("r02_v9", 5.0)]:
        d = tmp_path / "profiles" / name
        d.mkdir(parents=True)
        (d / "pmc_summary.json").write_text(json.dumps({
            "_config": {"robot": "spot", "samples": 20000},
            "k2_gram_syrk": {"FETCH_bytes_corrected_x2": fetch, "WRITE_bytes": 0.0}}))
    other = tmp_path / "profiles" / "r03_q"
    other.mkdir()
    (other / "pmc_summary.json").write_text(json.dumps({"_config": {"robot": "g1_29dof", "samples": 20000},
                                                        "k2_gram_syrk": {"FETCH_bytes_corrected_x2": 9.0,
                                                                         "WRITE_bytes": 0.0}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    traffic, src = bench.pmc_traffic("k2_gram_syrk", "spot", 20000)
    assert src.endswith(os.path.join("r03_p", "pmc_summary.json")) and traffic == 4


def test_bench_traffic_source_mixed_tags(tmp_path, monkeypatch):
    """A tag that starts with a digit (r03_2) sorts against a word tag (r03_j) without a type error: numbers
    before words at the same position, so r03_j is the newer one."""
    import json
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    for name, fetch in [("r03_2", 1.0), ("r03_j", 2.0), ("r02_10", 3.0)]:
        d = tmp_path / "profiles" / name
        d.mkdir(parents=True)
        (d / "pmc_summary.json").write_text(json.dumps({
            "_config": {"robot": "spot", "samples": 20000},
            "k2_gram_syrk": {"FETCH_bytes_corrected_x2": fetch, "WRITE_bytes": 0.0}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    traffic, src = bench.pmc_traffic("k2_gram_syrk", "spot", 20000)
    assert src.endswith(os.path.join("r03_j", "pmc_summary.json")) and traffic == 2
