"""In-tree build of the native libraries (no JIT, no cmake):

    lib/libviba_hip.so    HIP kernels + C-ABI, gfx950 code objects (hipcc --offload-arch=gfx950), fp64
    lib/libviba_hip_mixed.so  the same with -DVIBA_MIXED=1 (config E: fp32 Jacobian records / Schur
                          products, fp64 Cholesky; csrc/engine.hpp)
    lib/libviba_synth.so  synthetic problem generator (g++)
    lib/libviba_host.so   host side of the session adapter: initial point triangulation (g++)
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.environ.get("VIBA_LIB_DIR", os.path.join(HERE, "lib"))
HIP_SOURCES = ["factors.hip", "schur.hip", "solver.hip", "rs.hip", "preint.hip", "pcg.hip", "selinv.hip", "lowprec.hip", "api.hip",
               "finalize.hip", "covariances.hip", "multi.hip", "tools.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("VIBA_OFFLOAD_ARCH", "gfx950")
HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
             # MFMA accumulators in VGPRs: the AGPR form made the compiler copy every accumulator
             # VGPR -> AGPR -> VGPR around each fan-in stage (+7 % fan-in throughput measured)
             "-mllvm", "-amdgpu-mfma-vgpr-form=1", "-pthread", "-Wall", "-Wno-unused-function",
             "-Wno-unused-variable", "-Wno-unused-but-set-variable", "-Wno-unused-value",
             *os.environ.get("VIBA_EXTRA_HIPFLAGS", "").split()]


def sources_digest() -> str:
    """sha256 over the HIP library's sources and headers (csrc/*.hip, *.hpp, include/viba_hip.h): ties a
    measurement (profiles/pmc_summary.json) to the code it measured -- bench.py reports the PMC traffic
    only when the running tree's digest equals the recorded one."""
    import hashlib
    names = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".hpp", ".h")))
    h = hashlib.sha256()
    for f in names + ["../../include/viba_hip.h"]:
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(os.path.basename(f).encode() + b"\0" + fh.read())
    return h.hexdigest()


def _newer(target: str, deps: list[str]) -> bool:
    return os.path.exists(target) and all(os.path.getmtime(target) >= os.path.getmtime(d) for d in deps)


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def build(force: bool = False, verbose: bool = False) -> list[str]:
    os.makedirs(LIB, exist_ok=True)
    headers = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hpp", ".h"))]
    headers.append(os.path.join(HERE, "..", "include", "viba_hip.h"))
    out = []
    # synthetic generator
    synth = os.path.join(LIB, "libviba_synth.so")
    src = os.path.join(CSRC, "synth.cpp")
    if force or not _newer(synth, [src] + headers):
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", synth, src])
    out.append(synth)
    # host side of the session adapter
    host = os.path.join(LIB, "libviba_host.so")
    src = os.path.join(CSRC, "session.cpp")
    if force or not _newer(host, [src]):
        _run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-o", host, src])
    out.append(host)
    # HIP libraries (fp64, mixed): compile objects in parallel, then link
    variants = [("libviba_hip.so", LIB, []), ("libviba_hip_mixed.so", os.path.join(LIB, "mixed"), ["-DVIBA_MIXED=1"])]
    objs = {name: [] for name, _, _ in variants}
    jobs = []
    with cf.ThreadPoolExecutor(max_workers=int(os.environ.get("VIBA_BUILD_JOBS", "6"))) as ex:
        for name, odir, defs in variants:
            os.makedirs(odir, exist_ok=True)
            for s in HIP_SOURCES:
                sp = os.path.join(CSRC, s)
                o = os.path.join(odir, s.replace(".hip", ".o"))
                objs[name].append(o)
                if force or not _newer(o, [sp] + headers):
                    jobs.append(ex.submit(_run, [HIPCC, *HIP_FLAGS, *defs, "-c", sp, "-o", o]))
        for j in jobs:
            r = j.result()
            if verbose and r.stderr:
                print(r.stderr)
    for name, _, _ in variants:
        hip = os.path.join(LIB, name)
        if force or not _newer(hip, objs[name]):
            _run([HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-pthread", "-o", hip, *objs[name]])
        out.append(hip)
    return out


if __name__ == "__main__":
    import sys
    print("\n".join(build(force="--force" in sys.argv, verbose=True)))
