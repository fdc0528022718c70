"""Regenerate tests/golden/session_small/: a reference-format ark_vi_ba input folder (README.md:29-39)
emitted by the synthetic generator (visual_inertial_bundle_adjustment_amd.synth.write_session), plus
session_small.npz: the oracle's one LM step and 8-iteration optimize on the problem the session
adapter builds from that folder (the stored reference of tests/test_session.py).

    python tests/golden/make_session.py            (folder + npz)
    python tests/golden/make_session.py --npz-only (npz from the committed folder)

The adapter triangulates with the oracle's image-row poses (oracle.refcpu.rs_row_poses), so the stored
step needs no GPU.

The folder is data only: 55 rigs at 10 Hz (two 5 s calibration windows), 200 landmarks, an Aria-like rig
(rolling-shutter RGB + two global-shutter SLAM cameras, two IMUs), IMU samples at 10 significant digits.
"""
from __future__ import annotations

import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from oracle.refcpu import RefEngine  # noqa: E402
from parity_util import one_step  # noqa: E402
from visual_inertial_bundle_adjustment_amd import adapter, session, synth  # noqa: E402
from visual_inertial_bundle_adjustment_amd.engine import Settings  # noqa: E402
from visual_inertial_bundle_adjustment_amd.kinds import VAR_NAMES  # noqa: E402

FOLDER = os.path.join(HERE, "session_small")
CONFIG = dict(n_kf=55, n_lm=200)


def main():
    from oracle.refcpu import rs_row_poses
    if "--npz-only" not in sys.argv:
        p = synth.generate(synth.config("miniB", **CONFIG))
        if os.path.exists(FOLDER):
            shutil.rmtree(FOLDER)
        synth.write_session(p, FOLDER, imu_digits=10)
    q = adapter.build_problem(session.SessionData.load(FOLDER), row_poses=rs_row_poses)
    e = adapter.load_into(RefEngine(reproj_loss=q.reproj_loss, imu_loss=q.imu_loss,
                                    imu_calib_options=q.imu_calib_options), q)
    o = one_step(e)
    out = {"cost0": o["cost0"], "model_red": o["model_red"], "cost1": o["cost1"], "stats1": np.array(o["stats1"]),
           "n_factors": np.array([len(f) for f in q.fivals]), "n_points": len(q.vars[0])}
    for k, name in enumerate(VAR_NAMES[:-1]):
        out[f"step_{name}"] = o["step"][k]
    e2 = adapter.load_into(RefEngine(reproj_loss=q.reproj_loss, imu_loss=q.imu_loss,
                                     imu_calib_options=q.imu_calib_options), q)
    s = e2.optimize(Settings.default(max_num_iterations=8))
    out["opt_initial_cost"], out["opt_final_cost"], out["opt_iterations"] = s.initial_cost, s.final_cost, s.num_iterations
    for k, name in enumerate(VAR_NAMES[:-1]):
        out[f"opt_{name}"] = e2.get_vars(k)
    np.savez(os.path.join(HERE, "session_small.npz"), **out)
    print(f"session_small: {q.summary()}, oracle optimize {s.initial_cost:.6g} -> {s.final_cost:.6g} "
          f"in {s.num_iterations} iterations")


if __name__ == "__main__":
    main()
