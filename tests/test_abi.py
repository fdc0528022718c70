"""C-ABI checks that need no GPU: the product library loads, exports every function that
include/viba_hip.h declares, its structs have the layouts the ctypes mirror assumes, and the
product path fails loudly (error code / exception, never a CPU fallback) without a HIP device."""
from __future__ import annotations

import ctypes as C
import os
import re
import subprocess

import pytest

from visual_inertial_bundle_adjustment_amd import _lib
from visual_inertial_bundle_adjustment_amd.engine import HipEngine, PhaseTimes, Settings, Summary

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "viba_hip.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\*]+\s+\**(vb_\w+)\s*\(", text, flags=re.M)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("vb_create", "vb_finalize", "vb_linearize", "vb_damp_factor_solve", "vb_apply_step", "vb_cost",
                 "vb_optimize", "vb_destroy", "vb_last_error", "vb_set_landmark_shard"):
        assert must in names


@pytest.mark.parametrize("mixed", [False, True])
def test_library_exports_every_declared_symbol(mixed):
    lib = _lib.load_hip_lib(mixed=mixed)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, f"{'libviba_hip_mixed.so' if mixed else 'libviba_hip.so'} does not export {missing}"


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", _lib.HIP_LIB],
                         capture_output=True, text=True)
    if out.returncode != 0:
        pytest.skip("llvm-objdump --offloading unavailable")
    assert "gfx950" in out.stdout + out.stderr


def _c_sizes():
    src = f"""
#include <stdio.h>
#include <stddef.h>
#include "{HEADER}"
int main(void) {{
  printf("%zu %zu %zu %zu %zu %zu %zu\\n", sizeof(vb_config), sizeof(vb_settings), sizeof(vb_summary),
         sizeof(vb_cost_stats), sizeof(vb_phase_times), offsetof(vb_settings, damping),
         offsetof(vb_summary, num_iterations));
  return 0;
}}"""
    d = os.path.join(ROOT, "oracle", "_ref")
    os.makedirs(d, exist_ok=True)
    c, exe = os.path.join(d, "abi_sizes.c"), os.path.join(d, "abi_sizes")
    open(c, "w").write(src)
    subprocess.check_call(["gcc", "-std=c11", "-o", exe, c])
    return [int(x) for x in subprocess.check_output([exe]).split()]


def test_struct_layouts_match_ctypes_mirrors():
    cfg, st, summ, cs, pt, off_damp, off_it = _c_sizes()
    assert cfg == C.sizeof(HipEngine.Config)
    assert st == C.sizeof(Settings)
    assert summ == C.sizeof(Summary)
    assert cs == 3 * 8
    assert pt == C.sizeof(PhaseTimes)
    assert off_damp == Settings.damping.offset
    assert off_it == Summary.num_iterations.offset


def test_factor_tables_match_header():
    from visual_inertial_bundle_adjustment_amd.kinds import NUM_FACTOR_KINDS, factor_num_consts, factor_num_vars
    lib = _lib.load_hip_lib()
    for k in range(NUM_FACTOR_KINDS):
        assert lib.vb_factor_num_vars(k) == factor_num_vars(k)
        assert lib.vb_factor_num_consts(k) == factor_num_consts(k)
    assert lib.vb_factor_num_vars(99) == -1


def test_create_fails_loudly_without_device():
    lib = _lib.load_hip_lib()
    h = C.c_void_p()
    lib.vb_create.argtypes = [C.c_void_p, C.POINTER(C.c_void_p)]
    rc = lib.vb_create(None, C.byref(h))
    if rc == 0:  # a HIP device is present (GPU box): nothing to check here
        lib.vb_destroy.argtypes = [C.c_void_p]
        lib.vb_destroy(h)
        pytest.skip("HIP device present")
    lib.vb_last_error.restype = C.c_char_p
    assert rc == -3 and b"device" in lib.vb_last_error()  # VB_E_HIP
    with pytest.raises(Exception):
        HipEngine()


def test_null_handle_arguments_are_errors():
    lib = _lib.load_hip_lib()
    lib.vb_finalize.argtypes = [C.c_void_p]
    assert lib.vb_finalize(None) != 0
    lib.vb_linearize.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_double)]
    assert lib.vb_linearize(None, 1, 0, None) != 0


def test_missing_library_raises(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "_hip", None)
    monkeypatch.setattr(_lib, "HIP_LIB", str(tmp_path / "nope.so"))
    with pytest.raises(_lib.NativeLibraryMissing):
        _lib.load_hip_lib()
