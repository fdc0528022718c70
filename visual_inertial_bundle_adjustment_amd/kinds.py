"""Variable / factor kind tables of the C-ABI (include/viba_hip.h)."""

VAR_POINT, VAR_POSE, VAR_VEL, VAR_OMEGA, VAR_CAM_INTR, VAR_CAM_EXTR, VAR_IMU_CALIB, VAR_IMU_EXTR, \
    VAR_GRAVITY = range(9)
NUM_VAR_KINDS = 9
VAR_DATA = (3, 7, 3, 3, 24, 7, 32, 7, 4)
VAR_MAX_TANGENT = (3, 6, 3, 3, 17, 6, 23, 6, 2)
VAR_NAMES = ("point", "pose", "vel", "omega", "cam_intr", "cam_extr", "imu_calib", "imu_extr",
             "gravity")

(F_VISUAL, F_IMU, F_IMU_SEC_COMMON, F_IMU_SEC_SPLIT, F_OMEGA_PRIOR, F_RW_IMU_CALIB,
 F_RW_CAM_INTR, F_RW_IMU_EXTR, F_RW_CAM_EXTR, F_POSE_PRIOR, F_IMU_PRIOR, F_CAM_INTR_PRIOR,
 F_CAM_EXTR_PRIOR, F_IMU_EXTR_PRIOR) = range(14)
NUM_FACTOR_KINDS = 14
_NUM_VARS = (5, 6, 9, 10, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1)
_NUM_CONSTS = (6, 331, 331, 331, 4, 23, 17, 6, 6, 43, 55, 41, 13, 13)
FACTOR_NAMES = ("visual", "imu", "imu_sec_common", "imu_sec_split", "omega_prior", "rw_imu_calib",
                "rw_cam_intr", "rw_imu_extr", "rw_cam_extr", "pose_prior", "imu_prior",
                "cam_intr_prior", "cam_extr_prior", "imu_extr_prior")
# variable kind of each factor argument (reference functor argument order)
FACTOR_VAR_KINDS = (
    (0, 1, 5, 4, 2), (6, 1, 2, 1, 2, 8), (6, 1, 2, 3, 1, 2, 3, 7, 8),
    (6, 1, 2, 3, 7, 1, 2, 3, 7, 8), (3, 7), (6, 6), (4, 4), (7, 7), (5, 5), (1,), (6,), (4,),
    (5,), (7,))

PREINT_CONSTS = 4 + 3 + 3 + 1 + 9 * 23 + 81 + 32


def factor_num_vars(kind: int) -> int:
    return _NUM_VARS[kind]


def factor_num_consts(kind: int) -> int:
    return _NUM_CONSTS[kind]

# reduced-system solvers (include/viba_hip.h VB_SOLVER_*; Optimizer.h:31-37 SolverType)
SOLVER_DIRECT, SOLVER_PCG_TRIVIAL, SOLVER_PCG_JACOBI, SOLVER_PCG_GAUSS_SEIDEL, SOLVER_PCG_LOWER_PREC = range(5)
