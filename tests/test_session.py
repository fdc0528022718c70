"""On-disk formats: the session-folder reader (SessionData::load, Matcher), the
session adapter (SingleSessionAdapter) and the output writers (SaveOnlineCalib / SaveDeviceTrajectory),
on CPU.  The reference holds no session fixture, so the folders come from the synthetic generator
(synth.write_session; tests/golden/session_small is one, made by tests/golden/make_session.py) and the
adapter's outputs are checked against what was written and against the oracle (oracle/refcpu)."""
from __future__ import annotations

import json
import math
import os

import numpy as np
import pytest

from oracle.refcpu import rs_row_poses as ref_row_poses
from visual_inertial_bundle_adjustment_amd import adapter, kinds, session, synth

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "session_small")


@pytest.fixture(scope="module")
def generated(tmp_path_factory):
    p = synth.generate(synth.config("miniB", n_kf=60, n_lm=300))
    d = tmp_path_factory.mktemp("sess")
    synth.write_session(p, str(d))
    return p, str(d)


def _perm(n_win, n_sensor):
    """generator variable order (window-major) -> adapter order (sensor-major, InitCalibration.cpp)"""
    return [w * n_sensor + s for s in range(n_sensor) for w in range(n_win)]


def test_folder_roundtrip(generated):
    """write_session -> SessionData.load -> Matcher -> adapter: the rigs, calibrations and observations
    come back as written (through the device-frame changes of SessionData.cpp:142-295)."""
    p, d = generated
    sd = session.SessionData.load(d)
    assert sd.slam_imu_labels == ["imu-right", "imu-left"] and len(sd.slam_camera_serials) == 3
    assert len(sd.observations) == len(p.fivals[0])
    np.testing.assert_array_equal(sd.observations.timestamp_us, p.rs_mid[p.fvars[0][:, 1]])  # us, not ns
    # the reader rounds projections to fp32 (PointObservation.h:22-23: Eigen::Vector2f)
    np.testing.assert_array_equal(sd.observations.uv, p.fconsts[0][:, :2].astype(np.float32).astype(np.float64))
    assert len(sd.imu) == 2 and np.array_equal(sd.imu[0].timestamp_ns, p.imu_t)
    np.testing.assert_array_equal(sd.imu[1].gyro, p.imu_gyro)
    m = session.Matcher.build(sd)
    assert len(m.rig_to_pose_index) == 60 and (m.obs_to_rig >= 0).all()
    q = adapter.build_problem(sd, m, row_poses=ref_row_poses)
    assert np.abs(q.vars[1] - p.gt[1]).max() < 1e-12      # the folder carries the ground-truth trajectory
    assert np.abs(q.vars[2] - p.gt[2]).max() < 1e-12
    assert np.abs(q.vars[3] - p.gt[3]).max() < 1e-12
    nw = 2
    assert q.windows == [0, 50, 60]
    assert np.abs(q.vars[5] - p.vars[5][_perm(nw, 3)]).max() < 1e-12
    assert np.abs(q.vars[6] - p.vars[6][_perm(nw, 2)]).max() < 1e-12
    assert np.abs(q.vars[7] - p.vars[7]).max() < 1e-12
    cams = p.vars[4][_perm(nw, 3)].copy()
    cams[:, 7:9] = 0.0  # InitSettings defaults: readout time / offset not estimated
    assert np.abs(q.vars[4] - cams).max() < 1e-12


def test_csv_readers_by_header(tmp_path):
    """io::CSVReader::read_header(ignore_no_column, ...): columns found by name in any order, extra
    columns ignored, a missing column is an error; IMU temperature 'nan' reads as NaN (ImuDataReader.cpp)."""
    cols = list(session.OBSERVATION_COLUMNS)
    order = cols[::-1] + ["extra"]
    rows = [[7, 1000123, 2, 10.5, 20.25, 0.7, 0.0, 0.0, 0.7], [8, 1000223, 0, 1.0, 2.0, 1.0, 0.1, 0.2, 1.0]]
    f = tmp_path / "obs.csv"
    with open(f, "w") as fh:
        fh.write(",".join(order) + "\n")
        for r in rows:
            v = dict(zip(cols, r))
            fh.write(",".join(str(v[c]) for c in cols[::-1]) + ",zzz\n")
    o = session.read_point_observations(f)
    np.testing.assert_array_equal(o.point_id, [7, 8])
    np.testing.assert_array_equal(o.timestamp_us, [1000123, 1000223])
    np.testing.assert_array_equal(o.camera_index, [2, 0])
    # Eigen::Matrix2f sqrtH_BaseRes (PointObservation.h:23): read as fp32
    np.testing.assert_array_equal(o.sqrt_h[1], np.float32([[1.0, 0.1], [0.2, 1.0]]).astype(np.float64))
    g = tmp_path / "bad.csv"
    g.write_text(",".join(cols[1:]) + "\n" + "1,2,3,4,5,6,7,8\n")
    with pytest.raises(ValueError, match="point_id"):
        session.read_point_observations(g)
    h = tmp_path / "imu.csv"
    h.write_text(",".join(session.IMU_COLUMNS) + "\n1000,nan,1,2,3,4,5,6\n2000,36.5,1,2,3,4,5,6\n")
    s = session.read_imu_samples(h)
    assert math.isnan(s.temperature[0]) and s.temperature[1] == 36.5
    np.testing.assert_array_equal(s.accel[1], [4, 5, 6])
    e = tmp_path / "empty.csv"
    e.write_text(",".join(cols) + "\n")
    assert len(session.read_point_observations(e)) == 0


def test_matcher_rigs_and_missing_frames(generated, tmp_path):
    """Matcher::buildIndices: rigs are the timestamps in BOTH the online calibration and the trajectory;
    observations of other frames are dropped (Matcher.cpp:20-100); reset events map to rigs (:102-121)."""
    p, d = generated
    out = tmp_path / "cut"
    os.makedirs(out)
    for f in os.listdir(d):
        with open(os.path.join(d, f)) as a, open(out / f, "w") as b:
            lines = a.readlines()
            if f == session.ONLINE_CALIBRATION:
                lines = lines[:3] + lines[4:]          # frame 3 without calibration
            if f == session.OPEN_LOOP_TRAJECTORY:
                lines = lines[:1] + lines[1:10] + lines[11:]  # frame 9 without pose
            b.writelines(lines)
    ts = p.rs_mid
    (out / "reset_events.json").write_text(json.dumps({"reset_events": [{"tracking_timestamp_us": int(ts[20])},
                                                                        {"tracking_timestamp_us": int(ts[30]) + 7}]}))
    sd = session.SessionData.load(str(out))
    m = session.Matcher.build(sd)
    assert len(m.rig_to_pose_index) == 58
    assert int(ts[3]) not in m.timestamp_to_rig and int(ts[9]) not in m.timestamp_to_rig
    dropped = np.isin(sd.observations.timestamp_us, [ts[3], ts[9]])
    assert (m.obs_to_rig[dropped] == -1).all() and (m.obs_to_rig[~dropped] >= 0).all()
    assert m.reset_rigs == {m.timestamp_to_rig[int(ts[20])], m.timestamp_to_rig[int(ts[30])]}


def test_online_calibration_writer_roundtrip(generated, tmp_path):
    """saveOnlineCalib (SaveOnlineCalib.cpp:23-64) of the unoptimized problem reproduces the input
    online calibration of every rig (JSON doubles round-trip exactly)."""
    p, d = generated
    sd = session.SessionData.load(d)
    m = session.Matcher.build(sd)
    q = adapter.build_problem(sd, m, row_poses=ref_row_poses)
    nr = len(q.rig_ts_us)
    cams = [[q.vars[4][q.cam_var(r, s)] for s in range(q.n_cam)] for r in range(nr)]
    extr = [[q.vars[5][q.cam_var(r, s)] for s in range(q.n_cam)] for r in range(nr)]
    imus = [[q.vars[6][q.imu_var(r, s)] for s in range(q.n_imu)] for r in range(nr)]
    iext = [[None] + [q.vars[7][q.imu_extr_var(r, s)] for s in range(1, q.n_imu)] for r in range(nr)]
    f = tmp_path / "online_calibration.jsonl"
    session.save_online_calibration(f, sd, q.rig_pose_index, cams, extr, imus, iext)
    back = session.read_online_calibration(f)
    orig = session.read_online_calibration(os.path.join(d, session.ONLINE_CALIBRATION))
    assert len(back) == len(orig) == nr
    for (t1, u1, c1, i1), (t2, u2, c2, i2) in zip(back, orig):
        assert (t1, u1) == (t2, u2)
        for a, b in zip(c1, c2):
            assert a.label == b.label and a.serial == b.serial and a.model == b.model
            assert np.abs(a.params - b.params).max() < 1e-12
            assert np.abs(a.T_device_camera - b.T_device_camera).max() < 1e-12
            assert a.readout_sec == b.readout_sec and a.time_offset_sec == b.time_offset_sec
        for a, b in zip(i1, i2):
            assert a.label == b.label and np.abs(a.model - b.model).max() < 1e-12
            assert np.abs(a.T_device_imu - b.T_device_imu).max() < 1e-12


def test_trajectory_writers(generated, tmp_path):
    """saveOpenLoopTrajectory / saveCloseLoopTrajectory (SaveDeviceTrajectory.cpp): the unoptimized rigs
    give back the input open-loop trajectory to the 6 significant digits of the C++ stream defaults, and
    the closed-loop file carries the same device poses."""
    p, d = generated
    sd = session.SessionData.load(d)
    q = adapter.build_problem(sd, row_poses=ref_row_poses)
    rv = (q.vars[1], q.vars[2], q.vars[3])
    ps = session.InertialPoses(sd.inertial_poses.T_w_imu[q.rig_pose_index], None, None,
                               q.rig_ts_us, sd.inertial_poses.utc_timestamp_ns[q.rig_pose_index],
                               sd.inertial_poses.quality[q.rig_pose_index], [sd.inertial_poses.uid[i] for i in q.rig_pose_index])
    g = q.vars[8][0, :3]
    session.write_open_loop_trajectory(tmp_path / "ol.csv", ps, rv, sd.T_bodyimu_device, g)
    session.write_closed_loop_trajectory(tmp_path / "cl.csv", ps, rv, sd.T_bodyimu_device, g)
    a = session._read_columns(tmp_path / "ol.csv", session.OPEN_LOOP_COLUMNS[3:16], (np.float64,) * 13)
    b = session._read_columns(os.path.join(d, session.OPEN_LOOP_TRAJECTORY), session.OPEN_LOOP_COLUMNS[3:16],
                              (np.float64,) * 13)
    for x, y in zip(a, b):
        np.testing.assert_allclose(x, y, rtol=1e-5, atol=1e-6)
    c = session._read_columns(tmp_path / "cl.csv", session.CLOSED_LOOP_COLUMNS[3:10], (np.float64,) * 7)
    for x, y in zip(c, a[:7]):
        np.testing.assert_allclose(x, y, rtol=1e-5, atol=1e-6)
    uid = session._read_columns(tmp_path / "cl.csv", ("graph_uid",), (str,))[0]
    assert uid[0] == "synthetic"


def test_omega_at_end_matches_oracle(generated):
    """addOmegaPriors' omegaAtEnd (the host restatement in adapter.compensated_gyro_at_end) equals the
    oracle's computePreIntegration omegaAtEnd (PreIntegration.cpp:272) for every rig and IMU."""
    from oracle.refcpu import preint_omega_at_end
    p, d = generated
    q = adapter.build_problem(session.SessionData.load(d), row_poses=ref_row_poses)
    fv, fc, ts = q.fvars[kinds.F_OMEGA_PRIOR], q.fconsts[kinds.F_OMEGA_PRIOR], q.rig_ts_us
    assert len(fv) == 2 * len(ts)
    for j in range(len(fv)):
        r, i = int(fv[j, 0]), j % 2
        t0 = int(ts[r]) - adapter.K_SMALL_INTERVAL_FOR_OMEGA_US if r == 0 else int(ts[r - 1])
        calib = q.vars[6][q.imu_var(r if r == 0 else r - 1, i)]
        s = q.imu_streams[i]
        ref = preint_omega_at_end(s.timestamp_ns, s.gyro, s.accel, calib, t0, int(ts[r]))
        assert np.abs(fc[j, :3] - ref).max() <= 1e-14
        assert fc[j, 3] == adapter.K_MULTI_IMU_OMEGA_PRIOR_STD
        assert fv[j, 1] == (-1 if i == 0 else q.imu_extr_var(r, 1))


def test_triangulation_and_projection(generated):
    """initPointsFromObservations (InitPointTracks.cpp:29-63): unprojection inverts the projection of both
    camera models, and with the ground-truth trajectory the triangulated points land near the truth."""
    import ctypes as C
    from visual_inertial_bundle_adjustment_amd._lib import load_host_lib
    p, d = generated
    lib = load_host_lib()
    rng = np.random.default_rng(3)
    for cam in (p.vars[4][0], p.vars[4][1], synth.generate(synth.config("A", n_lm=10)).vars[4][0]):
        cam = np.ascontiguousarray(cam)
        for _ in range(50):
            pc = np.array([rng.uniform(-0.6, 0.6), rng.uniform(-0.5, 0.5), 1.0]) * rng.uniform(0.5, 5.0)
            uv, ray = np.zeros(2), np.zeros(3)
            assert lib.vbh_project(cam.ctypes.data, pc.ctypes.data, uv.ctypes.data) == 0
            lib.vbh_unproject(cam.ctypes.data, uv.ctypes.data, ray.ctypes.data)
            assert np.abs(ray / ray[2] - pc / pc[2]).max() < 1e-9
    sd = session.SessionData.load(d)
    m = session.Matcher.build(sd)
    q = adapter.build_problem(sd, m, row_poses=ref_row_poses)
    assert q.triangulated >= 0.95 * q.tried_tracks
    # the folder's point ids are the generator's landmark indices; short baselines (2 s tracks at ~1 m/s,
    # landmarks 1-20 m away) and the x0 calibration leave a few cm of depth error
    err = np.linalg.norm(q.vars[0] - p.gt[0][q.point_ids], axis=1)
    assert np.median(err) < 0.1
    # exact data (ground-truth calibration, no pixel noise, no outliers): with the image-row poses
    # (kModelRollingShutter) rolling-shutter tracks come back as close as global-shutter ones, within the
    # fp32 rounding of the stored projections (PointObservation.h:22; <= 0.12 mm for the farthest points
    # on 2 s baselines); the frame-time pose would leave them 3.6 mm off at the median, 6 cm at worst
    e = synth.generate(synth.config("miniB", n_kf=60, n_lm=300, pixel_sigma=0.0, outlier_frac=0.0))
    for k in (4, 5, 6, 7):
        e.vars[k] = e.gt[k].copy()
    d2 = os.path.join(d, "exact")
    synth.write_session(e, d2)
    q2 = adapter.build_problem(session.SessionData.load(d2), row_poses=ref_row_poses)
    err2 = np.linalg.norm(q2.vars[0] - e.gt[0][q2.point_ids], axis=1)
    rs_pt = np.zeros(len(err2), bool)
    rs_pt[q2.fvars[kinds.F_VISUAL][q2.fivals[kinds.F_VISUAL] >= 0, 0]] = True
    assert q2.triangulated == q2.tried_tracks
    assert err2[~rs_pt].max() < 1e-3 and np.median(err2[~rs_pt]) < 1e-5
    assert err2[rs_pt].max() < 1e-3 and np.median(err2[rs_pt]) < 1e-4


def test_triangulation_matches_oracle(generated):
    """initPointsFromObservations with kModelRollingShutter (Triangulation.cpp:100-237, Triangulation.h:43):
    the product's host triangulation (libviba_host vbh_triangulate, fed the image-row poses) against the
    oracle's restatement (oracle/ref_triang.hpp ref_triangulate) on the same inputs, for a folder with
    noisy rolling-shutter tracks and 1 % outliers: same accepted tracks, identical refine-2 inlier sets,
    points within 1e-9.  The row poses themselves differ from the frame-time poses by the rolling shutter
    (checked non-trivial here); the device form of them is checked in tests/test_session_gpu.py."""
    from oracle.refcpu import triangulate as ref_triangulate
    p, d = generated
    sd = session.SessionData.load(d)
    a = adapter.SessionAdapter(sd, session.Matcher.build(sd), None, ref_row_poses)
    q = a.problem()
    t = a.triangulation
    pts, ok, inl = ref_triangulate(*t["inputs"])
    assert ok.sum() >= 0.95 * len(ok) and np.array_equal(ok, t["ok"])
    np.testing.assert_array_equal(inl, t["inliers"])
    assert (inl == 0).any()   # the outliers are dropped
    assert np.abs(pts - t["points"]).max() <= 1e-9 * max(1.0, np.abs(pts).max())
    # the row-time poses of the rolling-shutter observations move by mm-cm against the frame poses
    rig, camvar, row = a.row_pose_inputs
    rows = ref_row_poses(*a._row_pose_args(q, rig, camvar, row))
    rs = np.array([q.vars[4][c][4] != 0 for c in camvar])
    shift = np.linalg.norm(rows[:, 4:] - q.vars[1][rig][:, 4:], axis=1)
    assert rs.any() and (shift[~rs] == 0).all() and np.median(shift[rs]) > 1e-4


def test_adapter_structure(generated):
    """The factor set of SingleSessionAdapter::initAllVariablesAndFactors: one inertial factor per
    consecutive rig pair and IMU (common / split secondary kinds by the extrinsics window), RW factors
    between consecutive windows, factory priors with precision scaled by the rigs referencing each
    variable, rolling-shutter visual factors for the RGB camera only, one RS interval per rig."""
    p, d = generated
    q = adapter.build_problem(session.SessionData.load(d), row_poses=ref_row_poses)
    F = kinds
    assert len(q.fvars[F.F_IMU]) == 59
    assert len(q.fvars[F.F_IMU_SEC_COMMON]) + len(q.fvars[F.F_IMU_SEC_SPLIT]) == 59
    assert len(q.fvars[F.F_IMU_SEC_SPLIT]) == 1                        # the pair straddling the windows
    assert len(q.fvars[F.F_RW_IMU_CALIB]) == 2 and len(q.fvars[F.F_RW_CAM_INTR]) == 3
    assert len(q.fvars[F.F_RW_IMU_EXTR]) == 1 and len(q.fvars[F.F_RW_CAM_EXTR]) == 3
    assert len(q.fvars[F.F_IMU_PRIOR]) == 4 and len(q.fvars[F.F_CAM_INTR_PRIOR]) == 6
    assert len(q.fvars[F.F_POSE_PRIOR]) == 0
    # camera-intrinsics prior precision: count / (turn-on std * inflate)^2 (FactoryCalibPriors.cpp:33-78)
    h = q.fconsts[F.F_CAM_INTR_PRIOR]
    assert abs(h[0, 24] - 50 / 100.0 ** 2) < 1e-15 and abs(h[1, 24] - 10 / 100.0 ** 2) < 1e-15
    assert abs(h[0, 27] - 50 / (1e-3 * 100.0) ** 2) < 1e-6
    # camera-extrinsics prior: the rotation std converted from degrees twice, as the reference does
    he = q.fconsts[F.F_CAM_EXTR_PRIOR][0, 7:13]
    assert abs(he[3] - 50 / (0.2 * math.pi / 180 * math.pi / 180 * 100) ** 2) / he[3] < 1e-12
    # RW on the camera extrinsics: 1 / sqrt(dt * var) with dt the difference of window mean timestamps
    dt = (adapter.average_timestamp(q.rig_ts_us, 50, 60) - adapter.average_timestamp(q.rig_ts_us, 0, 50)) * 1e-6
    assert abs(q.fconsts[F.F_RW_CAM_EXTR][0, 0] - 1 / math.sqrt(dt * adapter.K_CAM_EXTR_RW_POS_VAR)) < 1e-6
    vis_rs = q.fivals[F.F_VISUAL] >= 0
    cam_of = q.fvars[F.F_VISUAL][:, 3] // 2                                   # sensor of the intrinsics var
    assert vis_rs.any() and np.array_equal(vis_rs, cam_of == 0)
    assert np.array_equal(q.fvars[F.F_VISUAL][vis_rs, 4], q.fvars[F.F_VISUAL][vis_rs, 1])
    # initCamIntrinsics' span: readout + 1 ms slack, + 2 (|offset| + 1 ms) for a non-zero time offset
    # (InitCalibration.cpp:267-271); half interval = 2 ms + span / 2 (:307)
    rgb = q.vars[F.VAR_CAM_INTR][[q.cam_var(r, 0) for r in range(60)]]
    span = rgb[:, 5] + 1e-3 + np.where(rgb[:, 6] != 0, 2 * (np.abs(rgb[:, 6]) + 1e-3), 0.0)
    assert len(q.rs_mid) == 60 and np.array_equal(q.rs_half, (2000 + span * 0.5e6).astype(np.int64))


def test_golden_session_oracle():
    """tests/golden/session_small (a committed reference-format folder) through the adapter into the
    oracle reproduces the stored step and optimize (tests/golden/make_session.py)."""
    from oracle.refcpu import RefEngine
    from parity_util import one_step, rel
    from visual_inertial_bundle_adjustment_amd.engine import Settings
    g = np.load(os.path.join(HERE, "golden", "session_small.npz"))
    q = adapter.build_problem(session.SessionData.load(GOLDEN), row_poses=ref_row_poses)
    assert [len(f) for f in q.fivals] == list(g["n_factors"]) and len(q.vars[0]) == int(g["n_points"])
    e = adapter.load_into(RefEngine(reproj_loss=q.reproj_loss, imu_loss=q.imu_loss,
                                    imu_calib_options=q.imu_calib_options), q)
    o = one_step(e)
    assert abs(o["cost0"] - g["cost0"]) <= 1e-9 * abs(g["cost0"])
    assert abs(o["cost1"] - g["cost1"]) <= 1e-8 * abs(g["cost1"])
    assert rel(o["step"][1], g["step_pose"]) < 1e-6
    e2 = adapter.load_into(RefEngine(reproj_loss=q.reproj_loss, imu_loss=q.imu_loss,
                                     imu_calib_options=q.imu_calib_options), q)
    s = e2.optimize(Settings.default(max_num_iterations=8))
    assert s.num_iterations == int(g["opt_iterations"])
    assert abs(s.final_cost - g["opt_final_cost"]) <= 1e-6 * g["opt_final_cost"]
    assert s.final_cost < 1e-3 * s.initial_cost
