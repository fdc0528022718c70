"""The reference's on-disk formats: the 7-file session folder ark_vi_ba reads, and the
calibration / trajectory files it writes.

Input folder (README.md:29-39; SessionData::load, interfaces/ark/session_data/SessionData.cpp:81-359):

    vrs_source_info.json       SLAM camera serials and IMU labels (camera_index / IMU order)  :86-106
    online_calibration.jsonl   per-frame online calibration, one JSON object a line           :108-276
    factory_calibration.json   device calibration (cameras, IMUs)                             :131-225
    open_loop_trajectory.csv   per-frame pose / velocity / angular velocity (MPS open loop)   :278-295
    session_observations.csv   point observations (PointObservationFormat.h:13-23)            :318-324
    imu_samples_{label}.csv    raw IMU samples per SLAM IMU (imu_types/ImuDataFormat.h:14-23) :326-335
    reset_events.json          optional                                                       :337-358

Outputs (main_AriaKit_ViBa.cpp:122-130): online_calibration.jsonl (SaveOnlineCalib.cpp:23-64),
open_loop_framerate_trajectory.csv and closed_loop_framerate_trajectory.csv (SaveDeviceTrajectory.cpp).

The JSON schemas of the calibrations are projectaria_tools' (CameraCalibration / ImuCalibration JSON;
the projectaria_tools submodule is absent from the reference, so they are restated from its published
format and from the keys the reference's own tools read, tools/save_observations/save_observations.py:
172-197).  Poses are kept as (qx, qy, qz, qw, tx, ty, tz) rows, the data layout of the engine's SE3
variables (include/viba_hip.h).

Notes carried from the reference:
  * session_observations.csv's column ``capture_timestamp_ns`` holds MICROseconds
    (save_observations.py:127-130 writes ``capture_timestamp_ns // 1000``; PointObservationReader
    reads it into ``captureTimestampUs``, PointObservationReader.cpp:27-29).
  * The output trajectories are written with C++ stream defaults (6 significant digits); the online
    calibration with JSON's shortest round-trip doubles (nlohmann::json::dump).
"""
from __future__ import annotations

import csv
import io
import json
import math
import os
from dataclasses import dataclass, field

import numpy as np

# ------------------------------------------------------------------ SE3 rows (qx qy qz qw tx ty tz)


def _qmul(a, b):
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by,
                     aw * by - ax * bz + ay * bw + az * bx,
                     aw * bz + ax * by - ay * bx + az * bw,
                     aw * bw - ax * bx - ay * by - az * bz])


def _qrot(q, v):
    x, y, z, w = q
    u = np.array([x, y, z])
    t = 2.0 * np.cross(u, v)
    return np.asarray(v) + w * t + np.cross(u, t)


def se3(q, t) -> np.ndarray:
    q = np.asarray(q, dtype=np.float64)
    q = q / np.linalg.norm(q)
    return np.concatenate([q, np.asarray(t, dtype=np.float64)])


def se3_identity() -> np.ndarray:
    return np.array([0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0])


def se3_mul(a, b) -> np.ndarray:
    return np.concatenate([_qmul(a[:4], b[:4]), _qrot(a[:4], b[4:]) + a[4:]])


def se3_inv(a) -> np.ndarray:
    qi = np.array([-a[0], -a[1], -a[2], a[3]])
    return np.concatenate([qi, -_qrot(qi, a[4:])])


def se3_act(a, p) -> np.ndarray:
    return _qrot(a[:4], p) + a[4:]


def so3_act(a, v) -> np.ndarray:
    return _qrot(a[:4], v)


def _unit_w_positive(q):
    """Eigen's unit_quaternion().coeffs() as Sophus stores it (sign as computed)."""
    return q / np.linalg.norm(q)


def _pose_to_json(T):
    q = _unit_w_positive(T[:4])
    return {"Translation": [float(x) for x in T[4:]],
            "UnitQuaternion": [float(q[3]), [float(q[0]), float(q[1]), float(q[2])]]}


def _pose_from_json(d):
    w, (x, y, z) = d["UnitQuaternion"]
    return se3([x, y, z, w], d["Translation"])


# ------------------------------------------------------------------ calibrations
# projectaria_tools camera model names and the engine's camera record (include/viba_hip.h VB_CAM_DATA)
CAMERA_MODELS = {"Linear": (0, 4), "FisheyeRadTanThinPrism": (1, 15)}
_MODEL_NAMES = {0: "Linear", 1: "FisheyeRadTanThinPrism"}
# image sizes of Aria's SLAM / RGB streams when a calibration carries none (projectaria_tools takes them
# from the device class)
_DEFAULT_IMAGE_SIZE = {"camera-slam": (640, 480), "camera-rgb": (1408, 1408)}


@dataclass
class CameraCalibration:
    """projectaria_tools CameraCalibration, the fields SessionData / CameraModelParam use."""
    label: str
    serial: str
    model: str                      # "Linear" | "FisheyeRadTanThinPrism"
    params: np.ndarray
    T_device_camera: np.ndarray     # SE3 row
    width: int
    height: int
    valid_radius: float = 0.0
    time_offset_sec: float = 0.0    # getTimeOffsetSecDeviceCamera
    readout_sec: float | None = None  # getReadOutTimeSec (optional: global shutter has none)

    @classmethod
    def from_json(cls, d) -> "CameraCalibration":
        label = d.get("Label", "")
        proj = d["Projection"]
        if proj["Name"] not in CAMERA_MODELS:
            raise ValueError(f"camera {label}: unsupported projection model {proj['Name']!r} "
                             "(CameraModelParam.cpp:30-35 supports Linear and Fisheye624)")
        size = d.get("ImageSize")
        if size is not None:
            w, h = int(size["Width"]), int(size["Height"])
        else:
            w, h = next((v for k, v in _DEFAULT_IMAGE_SIZE.items() if label.startswith(k)), (0, 0))
        ro = d.get("ReadoutTimeSec")
        return cls(label=label, serial=d.get("SerialNumber", ""), model=proj["Name"],
                   params=np.asarray(proj["Params"], dtype=np.float64),
                   T_device_camera=_pose_from_json(d["T_Device_Camera"]), width=w, height=h,
                   valid_radius=float(d.get("ValidRadius", 0.0)),
                   time_offset_sec=float(d.get("TimeOffsetSec_Device_Camera", 0.0)),
                   readout_sec=None if ro is None else float(ro))

    def to_json(self) -> dict:
        d = {"Calibrated": True, "Label": self.label,
             "Projection": {"Description": f"see {self.model} in CameraModelType.h", "Name": self.model,
                            "Params": [float(x) for x in self.params]},
             "SerialNumber": self.serial, "T_Device_Camera": _pose_to_json(self.T_device_camera),
             "ImageSize": {"Width": int(self.width), "Height": int(self.height)},
             "ValidRadius": float(self.valid_radius),
             "TimeOffsetSec_Device_Camera": float(self.time_offset_sec)}
        if self.readout_sec is not None:
            d["ReadoutTimeSec"] = float(self.readout_sec)
        return d

    def rescaled(self, width: int, height: int) -> "CameraCalibration":
        """CameraCalibration::rescale(newSize, scale) as SessionData.cpp:166-171 calls it: projection
        and principal point scaled by width ratio (distortion unchanged)."""
        s = width / self.width
        p = self.params.copy()
        if self.model == "Linear":
            p[:4] *= s
        else:
            p[:3] *= s
        return CameraCalibration(self.label, self.serial, self.model, p, self.T_device_camera.copy(), width,
                                 height, self.valid_radius * s, self.time_offset_sec, self.readout_sec)

    def camera_data(self, estimate_readout=False, estimate_offset=False) -> np.ndarray:
        """The engine's camera record of CameraModelParam(calib, estimateReadoutTime, estimateTimeOffset)
        (include/viba_hip.h VB_CAM_DATA; CameraModelParam.h:83-100)."""
        mid, n = CAMERA_MODELS[self.model]
        if len(self.params) != n:
            raise ValueError(f"camera {self.label}: {self.model} takes {n} params, got {len(self.params)}")
        d = np.zeros(24)
        has_ro = self.readout_sec is not None or estimate_readout
        d[:9] = [mid, n, self.width, self.height, 1.0 if has_ro else 0.0,
                 self.readout_sec or 0.0, self.time_offset_sec, float(estimate_readout), float(estimate_offset)]
        d[9:9 + n] = self.params
        return d

    @staticmethod
    def from_camera_data(like: "CameraCalibration", d) -> "CameraCalibration":
        """A calibration carrying the projection / timing values of an engine camera record."""
        n = int(d[1])
        return CameraCalibration(like.label, like.serial, _MODEL_NAMES[int(d[0])], np.asarray(d[9:9 + n]).copy(),
                                 like.T_device_camera.copy(), int(d[2]), int(d[3]), like.valid_radius,
                                 float(d[6]), float(d[5]) if d[4] != 0 else None)


def imu_model_from_rectification(gyro_rect, gyro_bias, accel_rect, accel_bias, dt_accel, dt_gyro) -> np.ndarray:
    """fromProjectAriaCalibration (ImuCalibConversion.cpp:13-22) + setScaleMatrices
    (ImuMeasurementModelParameters.h:103-119) into the 32-double record of ImuCalibParam
    (ImuCalibParam.cpp:214-228): gyroScale 3, accelScale 3, gyroBias 3, accelBias 3, gyroNonorth 9 and
    accelNonorth 9 (column-major), dtReferenceAccel, dtReferenceGyro."""
    G, A = np.asarray(gyro_rect, dtype=np.float64), np.asarray(accel_rect, dtype=np.float64)
    gs, as_ = np.linalg.norm(G, axis=1), np.linalg.norm(A, axis=1)
    gN, aN = G / gs[:, None], A / as_[:, None]
    if abs(aN[1, 0]) > 1e-14 or abs(aN[2, 0]) > 1e-14 or abs(aN[2, 1]) > 1e-14:
        raise ValueError("ImuMeasurementModelParameters::setScaleMatrices: accel should be upper triangular")
    m = np.zeros(32)
    m[0:3], m[3:6], m[6:9], m[9:12] = gs, as_, gyro_bias, accel_bias
    m[12:21], m[21:30] = gN.ravel(order="F"), aN.ravel(order="F")
    m[30], m[31] = dt_accel, dt_gyro
    return m


def imu_scale_mats(m):
    """(getGyroScaleMat, getAccelScaleMat) of a 32-double record (ImuMeasurementModelParameters.h:123-131)."""
    m = np.asarray(m)
    gN, aN = m[12:21].reshape(3, 3, order="F"), m[21:30].reshape(3, 3, order="F")
    return np.diag(m[0:3]) @ gN, np.diag(m[3:6]) @ aN


@dataclass
class ImuCalibration:
    """projectaria_tools ImuCalibration (the fields the conversion uses)."""
    label: str
    model: np.ndarray          # 32-double ImuMeasurementModelParameters record
    T_device_imu: np.ndarray   # SE3 row

    @classmethod
    def from_json(cls, d) -> "ImuCalibration":
        acc, gyr = d["Accelerometer"], d["Gyroscope"]
        m = imu_model_from_rectification(gyr["Model"]["RectificationMatrix"], gyr["Bias"]["Offset"],
                                         acc["Model"]["RectificationMatrix"], acc["Bias"]["Offset"],
                                         float(acc.get("TimeOffsetSec_Device_Accel", 0.0)),
                                         float(gyr.get("TimeOffsetSec_Device_Gyro", 0.0)))
        return cls(label=d.get("Label", ""), model=m, T_device_imu=_pose_from_json(d["T_Device_Imu"]))

    def to_json(self) -> dict:
        """toProjectAriaCalibration (ImuCalibConversion.cpp:24-37) + imuCalibrationToJson."""
        G, A = imu_scale_mats(self.model)
        m = self.model
        return {"Accelerometer": {"Bias": {"Name": "Constant", "Offset": [float(x) for x in m[9:12]]},
                                  "Model": {"Name": "Linear", "RectificationMatrix": A.tolist()},
                                  "TimeOffsetSec_Device_Accel": float(m[30])},
                "Calibrated": True,
                "Gyroscope": {"Bias": {"Name": "Constant", "Offset": [float(x) for x in m[6:9]]},
                              "Model": {"Name": "Linear", "RectificationMatrix": G.tolist()},
                              "TimeOffsetSec_Device_Gyro": float(m[31])},
                "Label": self.label, "SerialNumber": "", "T_Device_Imu": _pose_to_json(self.T_device_imu)}


@dataclass
class ImuNoiseModel:
    """ImuNoiseModelParameters (imu_types/ImuNoiseModelParameters.h:14-111), defaults of reset()."""
    accel_sample_var: np.ndarray = field(default_factory=lambda: np.full(3, 6.6297049e-3))
    gyro_sample_var: np.ndarray = field(default_factory=lambda: np.full(3, 2.7415568e-05))
    accel_bias_turnon_std: float = 0.03
    gyro_bias_turnon_std: float = 0.5 * 3.14159 / 180
    accel_bias_rw_var: float = 1e-8
    gyro_bias_rw_var: float = 1e-10
    accel_scale_turnon_std: float = 1e-3
    gyro_scale_turnon_std: float = 1e-3
    accel_scale_rw_var: float = 1e-10
    gyro_scale_rw_var: float = 1e-10
    accel_nonorth_turnon_std: float = 0.2 * 3.14159 / 180
    gyro_nonorth_turnon_std: float = 0.2 * 3.14159 / 180
    accel_nonorth_rw_var: float = 1e-12
    gyro_nonorth_rw_var: float = 1e-12
    gyro_accel_time_offset_turnon_std: float = 0.001
    ref_imu_time_offset_turnon_std: float = 0.001
    gyro_accel_time_offset_rw_var: float = 1e-10
    ref_imu_time_offset_rw_var: float = 1e-10
    imu_body_imu_turnon_pos_std: float = 0.001
    imu_body_imu_turnon_rot_std: float = 0.2 * 3.14159 / 180
    imu_body_imu_pos_rw_var: float = 1e-10
    imu_body_imu_rot_rw_var: float = 1e-10 * 3.14159 / 180


@dataclass
class CalibrationState:
    """CalibrationState (SessionData.h:37-54)."""
    cameras: list                  # CameraCalibration per camera
    T_cam_bodyimu: list            # SE3 rows
    imu_models: list               # 32-double records
    T_imu_bodyimu: list            # SE3 rows
    timestamp_us: int = 0


# ------------------------------------------------------------------ CSV files
OBSERVATION_COLUMNS = ("point_id", "capture_timestamp_ns", "camera_index", "projection_base_res_x",
                       "projection_base_res_y", "sqrt_h_base_res_00", "sqrt_h_base_res_01",
                       "sqrt_h_base_res_10", "sqrt_h_base_res_11")
IMU_COLUMNS = ("#timestamp [ns]", "temperature [degC]", "w_RS_S_x [rad s^-1]", "w_RS_S_y [rad s^-1]",
               "w_RS_S_z [rad s^-1]", "a_RS_S_x [m s^-2]", "a_RS_S_y [m s^-2]", "a_RS_S_z [m s^-2]")
OPEN_LOOP_COLUMNS = ("tracking_timestamp_us", "utc_timestamp_ns", "session_uid", "tx_odometry_device",
                     "ty_odometry_device", "tz_odometry_device", "qx_odometry_device", "qy_odometry_device",
                     "qz_odometry_device", "qw_odometry_device", "device_linear_velocity_x_odometry",
                     "device_linear_velocity_y_odometry", "device_linear_velocity_z_odometry",
                     "angular_velocity_x_device", "angular_velocity_y_device", "angular_velocity_z_device",
                     "gravity_x_odometry", "gravity_y_odometry", "gravity_z_odometry", "quality_score")
CLOSED_LOOP_COLUMNS = ("graph_uid", "tracking_timestamp_us", "utc_timestamp_ns", "tx_world_device",
                       "ty_world_device", "tz_world_device", "qx_world_device", "qy_world_device",
                       "qz_world_device", "qw_world_device", "device_linear_velocity_x_device",
                       "device_linear_velocity_y_device", "device_linear_velocity_z_device",
                       "angular_velocity_x_device", "angular_velocity_y_device", "angular_velocity_z_device",
                       "gravity_x_world", "gravity_y_world", "gravity_z_world", "quality_score")


def _r(x) -> str:
    """shortest round-trip text of a double"""
    return repr(float(x))


def _read_columns(path, names, dtypes):
    """Columns `names` of a headed CSV by header name, in any order, extra columns ignored
    (io::CSVReader::read_header(ignore_no_column, ...) semantics of the reference readers)."""
    with open(path, newline="") as f:
        header = f.readline().rstrip("\r\n").split(",")
        header = [h.strip() for h in header]
        idx = []
        for n in names:
            if n not in header:
                raise ValueError(f"{path}: missing column {n!r}")
            idx.append(header.index(n))
        text = f.read()
    if not text.strip():
        return [np.zeros(0, dtype=d) for d in dtypes]
    rows = list(csv.reader(io.StringIO(text)))
    rows = [r for r in rows if r]
    out = []
    for i, d in zip(idx, dtypes):
        col = [r[i].strip() for r in rows]
        if d is str:
            out.append(col)
        elif np.dtype(d).kind in "iu":
            out.append(np.array([int(c) for c in col], dtype=d))
        else:
            out.append(np.array([float(c) for c in col], dtype=d))
    return out


@dataclass
class PointObservations:
    """PointObservation rows (point_observation/PointObservation.h), struct of arrays."""
    point_id: np.ndarray
    timestamp_us: np.ndarray
    camera_index: np.ndarray
    uv: np.ndarray        # (n, 2)
    sqrt_h: np.ndarray    # (n, 2, 2)

    def __len__(self):
        return len(self.point_id)


def read_point_observations(path) -> PointObservations:
    """PointObservationReader::read (PointObservationReader.cpp:19-47)."""
    c = _read_columns(path, OBSERVATION_COLUMNS, (np.int64, np.int64, np.int32) + (np.float64,) * 6)
    n = len(c[0])
    # PointObservation holds the projection and its sqrt information as Eigen::Vector2f / Matrix2f
    # (interfaces/ark/point_observation/PointObservation.h:22-23): the reader rounds them to fp32, and
    # every later use casts those values to double (VisualFactors.cpp:35-36, Triangulation.cpp:139-140)
    f32 = [np.asarray(x, np.float64).astype(np.float32).astype(np.float64) for x in c[3:9]]
    return PointObservations(c[0], c[1], c[2], np.stack([f32[0], f32[1]], axis=1).reshape(n, 2),
                             np.stack(f32[2:6], axis=1).reshape(n, 2, 2))


def write_point_observations(path, obs: PointObservations):
    """PointObservationWriter / save_observations.py:96-170 (the timestamp column carries us)."""
    with open(path, "w") as f:
        f.write(",".join(OBSERVATION_COLUMNS) + "\n")
        for i in range(len(obs)):
            h = obs.sqrt_h[i]
            f.write(f"{int(obs.point_id[i])},{int(obs.timestamp_us[i])},{int(obs.camera_index[i])},"
                    + ",".join(_r(x) for x in (obs.uv[i, 0], obs.uv[i, 1], h[0, 0], h[0, 1], h[1, 0], h[1, 1])) + "\n")


@dataclass
class ImuSamples:
    """ImuMeasurement vector (imu_types/ImuMeasurement.h): ns stamps, temperature, gyro, accel."""
    timestamp_ns: np.ndarray
    temperature: np.ndarray
    gyro: np.ndarray      # (n, 3) rad/s
    accel: np.ndarray     # (n, 3) m/s^2

    def __len__(self):
        return len(self.timestamp_ns)


def read_imu_samples(path) -> ImuSamples:
    """ImuDataReader::read (imu_types/ImuDataReader.cpp:19-50): temperature "nan" (or any non-number)
    reads as NaN."""
    c = _read_columns(path, IMU_COLUMNS, (np.int64, str) + (np.float64,) * 6)

    def temp(s):
        try:
            return float(s)
        except ValueError:
            return math.nan
    n = len(c[0])
    return ImuSamples(c[0], np.array([temp(s) for s in c[1]]), np.stack(c[2:5], axis=1).reshape(n, 3),
                      np.stack(c[5:8], axis=1).reshape(n, 3))


def write_imu_samples(path, s: ImuSamples, digits: int | None = None):
    """ImuDataWriter (imu_types/ImuDataWriter.cpp), the ImuDataFormat header; `digits` significant
    digits (None: shortest round-trip)."""
    fmt = _r if digits is None else (lambda x: f"{float(x):.{digits}g}")
    with open(path, "w") as f:
        f.write(",".join(IMU_COLUMNS) + "\n")
        for i in range(len(s)):
            g, a = s.gyro[i], s.accel[i]
            t = "nan" if math.isnan(s.temperature[i]) else fmt(s.temperature[i])
            f.write(f"{int(s.timestamp_ns[i])},{t}," + ",".join(fmt(x) for x in (*g, *a)) + "\n")


@dataclass
class InertialPoses:
    """InertialPoseState per frame (SessionData.h:27-35), struct of arrays."""
    T_w_imu: np.ndarray        # (n, 7) SE3 rows
    v_w: np.ndarray            # (n, 3)
    omega_bodyimu: np.ndarray  # (n, 3)
    timestamp_us: np.ndarray
    utc_timestamp_ns: np.ndarray
    quality: np.ndarray
    uid: list

    def __len__(self):
        return len(self.timestamp_us)


def read_open_loop_trajectory(path, T_bodyimu_device) -> InertialPoses:
    """mps::readOpenLoopTrajectory + SessionData.cpp:278-295 (USE_OPEN_LOOP): the device states become
    body-IMU states."""
    types = (np.int64, np.int64, str) + (np.float64,) * 17
    c = _read_columns(path, OPEN_LOOP_COLUMNS, types)
    T_device_bodyimu = se3_inv(T_bodyimu_device)
    n = len(c[0])
    T = np.zeros((n, 7))
    v = np.zeros((n, 3))
    w = np.zeros((n, 3))
    for i in range(n):
        T_od = se3([c[6][i], c[7][i], c[8][i], c[9][i]], [c[3][i], c[4][i], c[5][i]])
        lin = np.array([c[10][i], c[11][i], c[12][i]])
        ang = np.array([c[13][i], c[14][i], c[15][i]])
        T[i] = se3_mul(T_od, T_device_bodyimu)
        v[i] = lin + so3_act(T_od, np.cross(ang, T_device_bodyimu[4:]))
        w[i] = so3_act(T_bodyimu_device, ang)
    return InertialPoses(T, v, w, c[0], c[1], c[19], list(c[2]))


def _fmt(x) -> str:
    """operator<<(ostream&, double) with the stream defaults (%g, 6 significant digits)."""
    return f"{x:g}"


def write_open_loop_trajectory(path, poses: InertialPoses, rig_vars, T_bodyimu_device, gravity):
    """saveOpenLoopTrajectory (SaveDeviceTrajectory.cpp:39-92). rig_vars: (T_bodyImu_world rows,
    vel_world, omega) of the problem's sorted rigs; poses: the input states of the same rigs."""
    Tbw, vel, om = rig_vars
    with open(path, "w") as f:
        f.write(",".join(OPEN_LOOP_COLUMNS) + "\n")
        for i in range(len(Tbw)):
            T_od = se3_mul(se3_inv(Tbw[i]), T_bodyimu_device)
            q = _unit_w_positive(T_od[:4])
            lin = vel[i] + so3_act(se3_inv(Tbw[i]), np.cross(om[i], T_bodyimu_device[4:]))
            ang = so3_act(se3_inv(T_bodyimu_device), om[i])
            vals = [*T_od[4:], *q, *lin, *ang, *gravity]
            f.write(f"{int(poses.timestamp_us[i])},{int(poses.utc_timestamp_ns[i])},{poses.uid[i]},"
                    + ",".join(_fmt(x) for x in vals) + f",{_fmt(float(poses.quality[i]))}\n")


def write_closed_loop_trajectory(path, poses: InertialPoses, rig_vars, T_bodyimu_device, gravity):
    """saveCloseLoopTrajectory (SaveDeviceTrajectory.cpp:117-170)."""
    Tbw, vel, om = rig_vars
    with open(path, "w") as f:
        f.write(",".join(CLOSED_LOOP_COLUMNS) + "\n")
        for i in range(len(Tbw)):
            T_wd = se3_mul(se3_inv(Tbw[i]), T_bodyimu_device)
            q = _unit_w_positive(T_wd[:4])
            lin = so3_act(se3_inv(T_bodyimu_device), so3_act(Tbw[i], vel[i]) + np.cross(om[i], T_bodyimu_device[4:]))
            ang = so3_act(se3_inv(T_bodyimu_device), om[i])
            vals = [*T_wd[4:], *q, *lin, *ang, *gravity]
            f.write(f"{poses.uid[i]},{int(poses.timestamp_us[i])},{int(poses.utc_timestamp_ns[i])},"
                    + ",".join(_fmt(x) for x in vals) + f",{_fmt(float(poses.quality[i]))}\n")


def write_open_loop_input(path, poses: InertialPoses, T_bodyimu_device):
    """An MPS open_loop_trajectory.csv whose reading (read_open_loop_trajectory) gives back `poses`
    (full precision; the inverse of SessionData.cpp:282-294)."""
    T_device_bodyimu = se3_inv(T_bodyimu_device)
    with open(path, "w") as f:
        f.write(",".join(OPEN_LOOP_COLUMNS) + "\n")
        for i in range(len(poses)):
            T_od = se3_mul(poses.T_w_imu[i], T_bodyimu_device)
            ang = so3_act(se3_inv(T_bodyimu_device), poses.omega_bodyimu[i])
            lin = poses.v_w[i] - so3_act(T_od, np.cross(ang, T_device_bodyimu[4:]))
            vals = [*T_od[4:], *T_od[:4], *lin, *ang, 0.0, 0.0, -9.81]
            f.write(f"{int(poses.timestamp_us[i])},{int(poses.utc_timestamp_ns[i])},{poses.uid[i]},"
                    + ",".join(repr(float(x)) for x in vals) + f",{float(poses.quality[i])!r}\n")


# ------------------------------------------------------------------ online calibration (jsonl)
def read_online_calibration(path):
    """mps::readOnlineCalibration: one JSON object per line, tracking_timestamp_us + camera / IMU
    calibration lists. Returns [(timestamp_us, utc_ns, [CameraCalibration], [ImuCalibration])]."""
    out = []
    with open(path) as f:
        for line in f:
            if not line.strip():
                continue
            d = json.loads(line)
            out.append((int(d["tracking_timestamp_us"]), int(d.get("utc_timestamp_ns", 0)),
                        [CameraCalibration.from_json(c) for c in d["CameraCalibrations"]],
                        [ImuCalibration.from_json(c) for c in d["ImuCalibrations"]]))
    return out


def write_online_calibration_lines(path, entries):
    """entries: (timestamp_us, utc_ns, [CameraCalibration], [ImuCalibration]) -> jsonl."""
    with open(path, "w") as f:
        for ts, utc, cams, imus in entries:
            f.write(json.dumps({"tracking_timestamp_us": int(ts), "utc_timestamp_ns": int(utc),
                                "CameraCalibrations": [c.to_json() for c in cams],
                                "ImuCalibrations": [i.to_json() for i in imus]}, separators=(",", ":")) + "\n")


# ------------------------------------------------------------------ the session folder
VRS_SOURCE_INFO = "vrs_source_info.json"
ONLINE_CALIBRATION = "online_calibration.jsonl"
FACTORY_CALIBRATION = "factory_calibration.json"
POINT_OBSERVATIONS = "session_observations.csv"
IMU_SAMPLES = "imu_samples_{}.csv"
OPEN_LOOP_TRAJECTORY = "open_loop_trajectory.csv"
# hard-coded Aria accel sample variances (SessionData.cpp:210-223)
_ARIA_ACCEL_VAR = {"imu-left": 7.7951241e-3, "imu-right": 6.6297049e-3}


@dataclass
class SessionData:
    """SessionData (interfaces/ark/session_data/SessionData.h:56-98)."""
    slam_camera_serials: list = field(default_factory=list)
    slam_imu_labels: list = field(default_factory=list)
    T_bodyimu_device: np.ndarray = field(default_factory=se3_identity)
    factory_camera_serials: list = field(default_factory=list)
    factory_camera_labels: list = field(default_factory=list)
    factory_imu_labels: list = field(default_factory=list)
    factory_calib: CalibrationState | None = None
    imu_noise_models: list = field(default_factory=list)
    online_camera_serials: list = field(default_factory=list)
    online_camera_labels: list = field(default_factory=list)
    online_imu_labels: list = field(default_factory=list)
    online_calibs: list = field(default_factory=list)       # CalibrationState per entry
    online_utc_ns: list = field(default_factory=list)
    inertial_poses: InertialPoses | None = None
    observations: PointObservations | None = None
    imu: list = field(default_factory=list)                  # ImuSamples per SLAM IMU
    reset_timestamps_us: list = field(default_factory=list)

    @classmethod
    def load(cls, path, load_imu: bool = True) -> "SessionData":
        """SessionData::load (SessionData.cpp:81-359)."""
        sd = cls()
        p = os.fspath(path)

        def need(name):
            f = os.path.join(p, name)
            if not os.path.exists(f):
                raise FileNotFoundError(f"File not found: {f}")
            return f
        with open(need(VRS_SOURCE_INFO)) as f:
            info = json.load(f)
        sd.slam_camera_serials = list(info["camera_ids"])
        sd.slam_imu_labels = list(info["imu_ids"])

        online = read_online_calibration(need(ONLINE_CALIBRATION))
        if not online:
            raise ValueError("Unable to load online calib!")
        online_cam_index = {c.label: i for i, c in enumerate(online[0][2])}

        with open(need(FACTORY_CALIBRATION)) as f:
            fac = json.load(f)
        fcams = [CameraCalibration.from_json(c) for c in fac.get("CameraCalibrations", [])]
        fimus = [ImuCalibration.from_json(c) for c in fac.get("ImuCalibrations", [])]
        fimu_by_label = {i.label: i for i in fimus}
        body = sd.slam_imu_labels[0]
        if body not in fimu_by_label:
            raise ValueError(f"Slam's IMU n.0 = {body} not present in factory calibration")
        T_device_bodyimu = fimu_by_label[body].T_device_imu
        sd.T_bodyimu_device = se3_inv(T_device_bodyimu)
        sd.factory_imu_labels = [i.label for i in fimus]
        sd.factory_camera_labels = [c.label for c in fcams]
        cams, Tcb = [], []
        for c in fcams:
            # adapt to the online running resolution, take radius / readout / time offset from online
            if c.label in online_cam_index:
                o = online[0][2][online_cam_index[c.label]]
                a = c.rescaled(o.width, o.height) if (o.width, o.height) != (c.width, c.height) else c
                c = CameraCalibration(a.label, a.serial, a.model, a.params, a.T_device_camera, a.width, a.height,
                                      o.valid_radius, o.time_offset_sec, o.readout_sec)
            cams.append(c)
            sd.factory_camera_serials.append(c.serial)
            Tcb.append(se3_mul(se3_inv(c.T_device_camera), T_device_bodyimu))
        imu_models, Tib = [], []
        for i in fimus:
            imu_models.append(i.model.copy())
            Tib.append(se3_mul(se3_inv(i.T_device_imu), T_device_bodyimu))
            nm = ImuNoiseModel()
            if i.label in _ARIA_ACCEL_VAR:
                nm.accel_sample_var = np.full(3, _ARIA_ACCEL_VAR[i.label])
            sd.imu_noise_models.append(nm)
        sd.factory_calib = CalibrationState(cams, Tcb, imu_models, Tib)

        for k, (ts, utc, ocams, oimus) in enumerate(online):
            serials = [c.serial for c in ocams]
            labels = [c.label for c in ocams]
            ilabels = [i.label for i in oimus]
            st = CalibrationState(
                cameras=ocams,
                T_cam_bodyimu=[se3_inv(se3_mul(sd.T_bodyimu_device, c.T_device_camera)) for c in ocams],
                imu_models=[i.model.copy() for i in oimus],
                T_imu_bodyimu=[se3_inv(se3_mul(sd.T_bodyimu_device, i.T_device_imu)) for i in oimus],
                timestamp_us=ts)
            if k == 0:
                sd.online_camera_serials, sd.online_camera_labels, sd.online_imu_labels = serials, labels, ilabels
            elif (serials, labels, ilabels) != (sd.online_camera_serials, sd.online_camera_labels,
                                                 sd.online_imu_labels):
                raise ValueError("mismatch in labels/serials")
            sd.online_calibs.append(st)
            sd.online_utc_ns.append(utc)

        sd.inertial_poses = read_open_loop_trajectory(need(OPEN_LOOP_TRAJECTORY), sd.T_bodyimu_device)
        sd.observations = read_point_observations(need(POINT_OBSERVATIONS))
        if len(sd.observations) == 0:
            raise ValueError("unable to load tracking observations")
        if load_imu:
            for label in sd.slam_imu_labels:
                sd.imu.append(read_imu_samples(need(IMU_SAMPLES.format(label))))
        reset = os.path.join(p, "reset_events.json")
        if os.path.exists(reset):
            with open(reset) as f:
                j = json.load(f)
            if not isinstance(j.get("reset_events"), list):
                raise ValueError("reset_events.json: 'reset_events' must be an array")
            for e in j["reset_events"]:
                if not isinstance(e.get("tracking_timestamp_us"), int):
                    raise ValueError("reset_events.json: tracking_timestamp_us must be an integer")
                sd.reset_timestamps_us.append(int(e["tracking_timestamp_us"]))
        return sd


@dataclass
class Matcher:
    """Matcher::buildIndices (viba/single_session/Matcher.cpp:19-177)."""
    timestamp_to_rig: dict = field(default_factory=dict)
    rig_to_pose_index: np.ndarray | None = None
    rig_to_calib_index: np.ndarray | None = None
    obs_to_rig: np.ndarray | None = None
    point_id_to_index: dict = field(default_factory=dict)
    point_obs: list = field(default_factory=list)      # obs indices per point index
    reset_rigs: set = field(default_factory=set)
    slam_cam_to_factory: list = field(default_factory=list)
    slam_cam_to_online: list = field(default_factory=list)
    slam_imu_to_factory: list = field(default_factory=list)
    slam_imu_to_online: list = field(default_factory=list)

    @classmethod
    def build(cls, sd: SessionData) -> "Matcher":
        m = cls()
        pose_ts = {int(t): i for i, t in enumerate(sd.inertial_poses.timestamp_us)}
        calib_ts = {int(c.timestamp_us): i for i, c in enumerate(sd.online_calibs)}
        ts = sorted(t for t in calib_ts if t in pose_ts)
        m.timestamp_to_rig = {t: i for i, t in enumerate(ts)}
        m.rig_to_pose_index = np.array([pose_ts[t] for t in ts], dtype=np.int64)
        m.rig_to_calib_index = np.array([calib_ts[t] for t in ts], dtype=np.int64)
        obs = sd.observations
        m.obs_to_rig = np.array([m.timestamp_to_rig.get(int(t), -1) for t in obs.timestamp_us], dtype=np.int64)
        for i in np.flatnonzero(m.obs_to_rig >= 0):
            pid = int(obs.point_id[i])
            if pid not in m.point_id_to_index:
                m.point_id_to_index[pid] = len(m.point_id_to_index)
                m.point_obs.append([])
            m.point_obs[m.point_id_to_index[pid]].append(int(i))
        for rt in sd.reset_timestamps_us:
            if rt in m.timestamp_to_rig:
                m.reset_rigs.add(m.timestamp_to_rig[rt])
            else:  # the last rig before the reset
                best_ts, best = -1, -1
                for r, ci in enumerate(m.rig_to_calib_index):
                    t = sd.online_calibs[ci].timestamp_us
                    if best_ts < t < rt:
                        best_ts, best = t, r
                if best >= 0:
                    m.reset_rigs.add(best)
        for s in sd.slam_camera_serials:
            if s not in sd.factory_camera_serials:
                raise ValueError(f"Camera serial number not found in factory calibration: {s}")
            if s not in sd.online_camera_serials:
                raise ValueError(f"Camera serial number not found in online calibration: {s}")
            m.slam_cam_to_factory.append(sd.factory_camera_serials.index(s))
            m.slam_cam_to_online.append(sd.online_camera_serials.index(s))
        for lab in sd.slam_imu_labels:
            if lab not in sd.factory_imu_labels:
                raise ValueError(f"Imu label number not found in factory calibration: {lab}")
            if lab not in sd.online_imu_labels:
                raise ValueError(f"Imu label number not found in online calibration: {lab}")
            m.slam_imu_to_factory.append(sd.factory_imu_labels.index(lab))
            m.slam_imu_to_online.append(sd.online_imu_labels.index(lab))
        return m


def save_online_calibration(path, sd: SessionData, rig_pose_index, cam_models, cam_extr, imu_models, imu_extr):
    """saveOnlineCalib (SaveOnlineCalib.cpp:23-64): one line per rig of the problem.  rig_pose_index[i]:
    the rig's index into sd.inertial_poses (the reference indexes inertialPoses by rig index,
    :34, which coincides when every trajectory frame is a rig); cam_models[i][s] / cam_extr[i][s]:
    the engine camera record / T_Cam_BodyImu of rig i's camera s; imu_models[i][s] and imu_extr[i][s]
    (s >= 1) likewise."""
    T_device_bodyimu = se3_inv(sd.T_bodyimu_device)
    ps = sd.inertial_poses
    entries = []
    for i, pi in enumerate(rig_pose_index):
        cams = []
        for s, serial in enumerate(sd.slam_camera_serials):
            like = sd.factory_calib.cameras[sd.factory_camera_serials.index(serial)]
            c = CameraCalibration.from_camera_data(like, cam_models[i][s])
            c.T_device_camera = se3_mul(T_device_bodyimu, se3_inv(cam_extr[i][s]))
            cams.append(c)
        imus = []
        for s, label in enumerate(sd.slam_imu_labels):
            T_ib = se3_identity() if s == 0 else imu_extr[i][s]
            imus.append(ImuCalibration(label, np.asarray(imu_models[i][s]).copy(), se3_mul(T_device_bodyimu, se3_inv(T_ib))))
        entries.append((int(ps.timestamp_us[pi]), int(ps.utc_timestamp_ns[pi]), cams, imus))
    write_online_calibration_lines(path, entries)
