"""MI355X-native Levenberg-Marquardt inner loop for visual-inertial bundle adjustment.

Drop-in for the `small_thing::Optimizer` hot path driven by `viba::problem`.
"""
from .kinds import *  # noqa: F401,F403
