"""Locating and loading the in-tree native libraries (built by build.py into ./lib)."""
from __future__ import annotations

import ctypes as C
import os

LIB_DIR = os.environ.get("VIBA_LIB_DIR", os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib"))
HIP_LIB = os.path.join(LIB_DIR, "libviba_hip.so")
HIP_LIB_MIXED = os.path.join(LIB_DIR, "libviba_hip_mixed.so")  # config E build (VIBA_MIXED=1)
SYNTH_LIB = os.path.join(LIB_DIR, "libviba_synth.so")
HOST_LIB = os.path.join(LIB_DIR, "libviba_host.so")  # session adapter host code (csrc/session.cpp)

_synth = None
_hip = None
_hip_mixed = None


class NativeLibraryMissing(RuntimeError):
    pass


def _load(path: str) -> C.CDLL:
    if not os.path.exists(path):
        raise NativeLibraryMissing(
            f"{path} is missing: run `python -c 'import __graft_entry__ as g; g.build()'` "
            "(no CPU fallback exists for the HIP path)")
    return C.CDLL(path)


def load_synth_lib() -> C.CDLL:
    global _synth
    if _synth is None:
        lib = _load(SYNTH_LIB)
        P = C.c_void_p
        lib.vbs_generate.restype = P
        lib.vbs_generate.argtypes = [P]
        lib.vbs_default_config.argtypes = [P, C.c_int]
        lib.vbs_free.argtypes = [P]
        for name, rt in [("vbs_vars", P), ("vbs_gt_vars", P), ("vbs_var_const", P),
                         ("vbs_factor_vars", P), ("vbs_factor_ivals", P), ("vbs_factor_consts", P)]:
            f = getattr(lib, name)
            f.restype = rt
            f.argtypes = [P, C.c_int]
        for name in ("vbs_num_vars", "vbs_num_factors"):
            f = getattr(lib, name)
            f.restype = C.c_int64
            f.argtypes = [P, C.c_int]
        lib.vbs_num_rs_tables.restype = C.c_int32
        lib.vbs_num_rs_tables.argtypes = [P]
        lib.vbs_num_imu.restype = C.c_int64
        lib.vbs_num_imu.argtypes = [P]
        for name in ("vbs_rs_offsets", "vbs_rs_samples", "vbs_rs_interp", "vbs_rs_gravity", "vbs_imu_t",
                     "vbs_imu_gyro", "vbs_imu_accel", "vbs_rs_mid", "vbs_rs_half", "vbs_rs_calib"):
            f = getattr(lib, name)
            f.restype = P
            f.argtypes = [P]
        _synth = lib
    return _synth


_host = None


def load_host_lib() -> C.CDLL:
    global _host
    if _host is None:
        lib = _load(HOST_LIB)
        P = C.c_void_p
        lib.vbh_triangulate.argtypes = [C.c_int64] + [P] * 10
        lib.vbh_triangulate.restype = C.c_int
        lib.vbh_project.argtypes = [P, P, P]
        lib.vbh_unproject.argtypes = [P, P, P]
        _host = lib
    return _host


def load_hip_lib(mixed: bool = False) -> C.CDLL:
    """Load the HIP product library (fp64, or the config-E mixed-precision build). Raises
    NativeLibraryMissing when it was not built."""
    global _hip, _hip_mixed
    if mixed:
        if _hip_mixed is None:
            _hip_mixed = _load(HIP_LIB_MIXED)
        return _hip_mixed
    if _hip is None:
        _hip = _load(HIP_LIB)
    return _hip


_amdhip = None


def hip_stream_sync(stream) -> None:
    """hipStreamSynchronize on a raw stream handle (libamdhip64)."""
    global _amdhip
    if _amdhip is None:
        _amdhip = C.CDLL("libamdhip64.so")
        _amdhip.hipStreamSynchronize.argtypes = [C.c_void_p]
        _amdhip.hipStreamSynchronize.restype = C.c_int
    rc = _amdhip.hipStreamSynchronize(stream)
    if rc != 0:
        raise RuntimeError(f"hipStreamSynchronize failed: {rc}")
