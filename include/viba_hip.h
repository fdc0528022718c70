/*
 * viba_hip.h -- C-ABI drop-in boundary for the MI355X-native Levenberg-Marquardt inner loop
 * of visual-inertial bundle adjustment (VI-BA).
 *
 * The boundary sits where the reference's `viba::problem` builder hands factors to the generic
 * NLLS engine `small_thing::Optimizer`:
 *
 *   reference call                                             replaced by
 *   ---------------------------------------------------------  ---------------------------------
 *   SingleSessionProblem::inertialPose_set / *_addNew          vb_set_vars
 *     (viba/problem/SingleSessionProblem.h:199-364)
 *   Optimizer::addFactor (lib/small_thing/Optimizer.h:115-175)  vb_add_factors
 *     as called from SingleSessionProblem::add{VisualFactor,
 *     InertialFactor, OmegaPriorFactor, *RWFactor, *Prior}
 *     (viba/problem/SingleSessionProblem.h:64-129)
 *   RollingShutterData::compute results                        vb_set_rs_tables
 *     (lib/motion/preintegration/RollingShutterData.cpp:16-65)
 *   SingleSessionAdapter::initRollingShutterData /             vb_set_imu_measurements,
 *     updateRollingShutterData (viba/single_session/             vb_set_rs_rigs,
 *     InitCalibration.cpp:299-325), ark_vi_ba's preStepCallback  vb_update_rs_tables (and every
 *     (interfaces/ark/main_AriaKit_ViBa.cpp:95-101)              vb_optimize iteration)
 *   registerPointVariables + registeredVariablesToElimination  vb_set_elim_points (implicit: the
 *     Range (SingleSessionProblem.cpp:41-45, Optimizer.cpp:31)   point kind is always eliminated)
 *   Optimizer::initSolver (Optimizer.cpp:166-207)              vb_finalize
 *   Optimizer::computeGradHess (Optimizer.cpp:57-71)           vb_linearize
 *   Optimizer::computeCost (Optimizer.cpp:88-97)               vb_cost
 *   addDamping + factor + solve (Optimizer.cpp:826-833)        vb_damp_factor_solve
 *   solveFunc(gradNewX) (Optimizer.cpp:970)                    vb_solve_with_new_gradient
 *   Optimizer::applyStep (Optimizer.cpp:121-134)               vb_apply_step
 *   backupVariables / restoreVariables (Optimizer.cpp:99-119)  vb_backup / vb_restore
 *   Optimizer::optimize (Optimizer.cpp:768-1106)               vb_optimize
 *
 * Conventions
 *   - All values are IEEE fp64 (the reference path is fp64 end to end).
 *   - SE3 data layout = Sophus::SE3d::data(): [qx, qy, qz, qw, tx, ty, tz]; tangent [upsilon, omega].
 *   - Variables are addressed per kind by a 0-based handle (the order of vb_set_vars rows).
 *   - Every function returns 0 on success, a negative VB_E_* code on error, and never throws;
 *     vb_last_error() returns the message of the last error on the calling thread.
 *   - Host buffers are copied; the handle owns device memory. One handle = one HIP stream.
 */
#ifndef VIBA_HIP_H
#define VIBA_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------------- error codes */
#define VB_OK 0
#define VB_E_ARG (-1)        /* invalid argument / shape mismatch */
#define VB_E_STATE (-2)      /* call out of order (e.g. add after finalize) */
#define VB_E_HIP (-3)        /* HIP runtime error (incl. missing device) */
#define VB_E_NUMERIC (-4)    /* Cholesky breakdown / non-finite values */
#define VB_E_RANGE (-5)      /* rolling-shutter lookup out of range (RollingShutterData.cpp:82-91) */
#define VB_E_UNSUPPORTED (-6)

/* ---------------------------------------------------------------- variable kinds */
enum vb_var_kind {
  VB_VAR_POINT = 0,     /* Variable<Vec3> world point; data 3, tangent 3 (SingleSessionProblem.h:42) */
  VB_VAR_POSE = 1,      /* T_bodyImu_world SE3; data 7, tangent 6 (SingleSessionProblem.h:27) */
  VB_VAR_VEL = 2,       /* vel_world; data 3 (SingleSessionProblem.h:28) */
  VB_VAR_OMEGA = 3,     /* omega in body-imu frame; data 3 (SingleSessionProblem.h:29) */
  VB_VAR_CAM_INTR = 4,  /* CameraModelParam; data VB_CAM_DATA, tangent nParams+estRO+estOff */
  VB_VAR_CAM_EXTR = 5,  /* T_Cam_BodyImu SE3 */
  VB_VAR_IMU_CALIB = 6, /* ImuCalibParam; data 32 (ImuCalibParam.cpp:214-228), tangent = error state */
  VB_VAR_IMU_EXTR = 7,  /* T_Imu_BodyImu SE3 */
  VB_VAR_GRAVITY = 8,   /* S2 gravity: data [x, y, z, radius]; only constant gravity is supported */
  VB_NUM_VAR_KINDS = 9
};

/* camera data record (VB_VAR_CAM_INTR rows and camera priors), VB_CAM_DATA doubles:
 *  [0] model (VB_CAM_LINEAR | VB_CAM_FISHEYE624)  [1] number of projection params
 *  [2] image width   [3] image height   [4] has readout time (0/1)  [5] readout time [s]
 *  [6] time offset Dev->Camera [s]      [7] estimate readout (0/1)   [8] estimate time offset (0/1)
 *  [9 ..] projection params (Linear: fx fy cx cy; Fisheye624: f cx cy k0..k5 p0 p1 s0..s3) */
#define VB_CAM_DATA 24
#define VB_CAM_LINEAR 0
#define VB_CAM_FISHEYE624 1
#define VB_CAM_MAX_TANGENT 17 /* kMaxCamParams, CameraModelParam.h:17 */

#define VB_IMU_CALIB_DATA 32
#define VB_IMU_CALIB_MAX_TANGENT 23 /* kMaxCalibrationStateSize, ImuCalibrationJacobianIndices.h:21 */

/* IMU calibration estimation options (ImuCalibrationOptions; default all on, ImuCalibParam.cpp:15-24) */
#define VB_IMU_OPT_GYRO_BIAS (1 << 0)
#define VB_IMU_OPT_ACCEL_BIAS (1 << 1)
#define VB_IMU_OPT_GYRO_SCALE (1 << 2)
#define VB_IMU_OPT_ACCEL_SCALE (1 << 3)
#define VB_IMU_OPT_GYRO_NONORTH (1 << 4)
#define VB_IMU_OPT_ACCEL_NONORTH (1 << 5)
#define VB_IMU_OPT_REF_TIME_OFFSET (1 << 6)
#define VB_IMU_OPT_GYRO_ACCEL_TIME_OFFSET (1 << 7)
#define VB_IMU_OPT_ALL 0xff

/* ---------------------------------------------------------------- factor kinds
 * var handle order per factor row, and constants per row (doubles):              */
enum vb_factor_kind {
  /* VisualFactor / RollingShutterVisualFactor (VisualFactor.cpp:36-214, added at :216-264)
   * vars  [point, pose, cam_extr, cam_intr, vel]  (vel = -1 and rs = -1 for global shutter)
   * ivals [rs_table]  consts [u, v, sqrtH00, sqrtH01, sqrtH10, sqrtH11]; loss = reprojection loss */
  VB_F_VISUAL = 0,
  /* InertialFactor (InertialFactor.cpp:19-127, added at :322-332)
   * vars [imu_calib, prev_pose, prev_vel, next_pose, next_vel, gravity]
   * consts VB_PREINT_CONSTS: [R qx qy qz qw, dV 3, dP 3, dtSec, J 9x23 col-major (207),
   *                           rvpCov 9x9 col-major (81), calibEvalPoint 32]; loss = imu loss */
  VB_F_IMU = 1,
  /* SecondaryImuInertialFactor, common extrinsics (InertialFactor.cpp:256-301, added :339-351)
   * vars [imu_calib, prev_pose, prev_vel, prev_omega, next_pose, next_vel, next_omega,
   *       imu_extr, gravity]; consts VB_PREINT_CONSTS */
  VB_F_IMU_SEC_COMMON = 2,
  /* SecondaryImuInertialFactor, split extrinsics (InertialFactor.cpp:190-254, added :356-369)
   * vars [imu_calib, prev_pose, prev_vel, prev_omega, prev_imu_extr, next_pose, next_vel,
   *       next_omega, next_imu_extr, gravity]; consts VB_PREINT_CONSTS */
  VB_F_IMU_SEC_SPLIT = 3,
  /* addOmegaPriorFactor (OmegaPriorFactor.cpp:16-62): vars [omega, imu_extr or -1]
   * consts [omega_imu 3, sigma] (sigma = kMultiImuOmegaPriorStdRadSec, Constants.h:19) */
  VB_F_OMEGA_PRIOR = 4,
  /* RW factors (RandomWalkFactor.cpp): vars [prev, next]; consts diagSqrtH (tangent dim) */
  VB_F_RW_IMU_CALIB = 5, /* :16-55 (residual zero-padded to 23) */
  VB_F_RW_CAM_INTR = 6,  /* :57-94 (residual zero-padded to 17) */
  VB_F_RW_IMU_EXTR = 7,  /* :96-130 */
  VB_F_RW_CAM_EXTR = 8,  /* :132-166 */
  /* priors (PriorFactor.cpp) */
  VB_F_POSE_PRIOR = 9,      /* :37-55  vars [pose]; consts [prior T_bodyImu_world 7, H 6x6 (36)] */
  VB_F_IMU_PRIOR = 10,      /* :82-109 vars [imu_calib]; consts [prior data 32, diagH (tangent)] */
  VB_F_CAM_INTR_PRIOR = 11, /* :111-136 vars [cam_intr]; consts [prior cam data 24, diagH] */
  VB_F_CAM_EXTR_PRIOR = 12, /* :138-156 vars [cam_extr]; consts [prior SE3 7, diagH 6] */
  VB_F_IMU_EXTR_PRIOR = 13, /* :158-176 vars [imu_extr]; consts [prior SE3 7, diagH 6] */
  VB_NUM_FACTOR_KINDS = 14
};

#define VB_PREINT_CONSTS (4 + 3 + 3 + 1 + 9 * 23 + 81 + 32)

/* number of variable handles per factor row and constants per row for each kind; constants of the
 * RW / prior kinds are padded to their maximum size (diagonals beyond the tangent dim ignored) */
int vb_factor_num_vars(int kind);
int vb_factor_num_consts(int kind);

/* ---------------------------------------------------------------- settings / summary */
typedef struct vb_config {
  double reproj_loss_radius;  /* HuberLossWithCutoff a (kReprojectionErrorHuberLossWidth = 1) */
  double reproj_loss_cutoff;  /* k (kReprojectionErrorHuberLossCutoff = 3) */
  double imu_loss_radius;     /* +inf by default (Constants.h:24) */
  double imu_loss_cutoff;     /* +inf */
  int32_t imu_calib_options;  /* VB_IMU_OPT_* mask */
  int32_t device;             /* HIP device ordinal */
  int32_t tile;               /* reduced-system tile size (0 = default) */
  int32_t reserved;
} vb_config;

/* Optimizer::Settings (lib/small_thing/Optimizer.h:40-91), direct-solver subset */
typedef struct vb_settings {
  int32_t max_num_iterations;          /* 50 */
  int32_t stop_if_no_improvement_for;  /* 3 */
  int32_t distance_from_troubled_iteration; /* 3 */
  int32_t max_step_factor_attempts;    /* 2 */
  int32_t try_sub_step;                /* 1 */
  int32_t verbose;                     /* log through callback */
  double absolute_cost_tolerance;      /* 1e-8 */
  double relative_cost_tolerance;      /* 1e-10 */
  double variables_tolerance;          /* 1e-5 */
  double damping;                      /* 1e-5 */
  double damping_adjust_on_fail;       /* 2.5 */
  double damping_adjust_on_good_step;  /* 0.7 */
  double damping_adjust_on_average_step; /* 1.5 */
  double damping_max;                  /* 1e8 */
  double damping_min;                  /* 1e-9 */
  double min_relative_cost_reduction;  /* 0.3 */
  double step_factor_decrease;         /* 0.3 */
  double min_step_factor_for_good;     /* 0.7 */
} vb_settings;

typedef struct vb_summary { /* Optimizer::Summary (Optimizer.h:93-99) */
  double initial_cost;
  double final_cost;
  int32_t num_troubled_seqs;
  int32_t largest_troubled_seq;
  int32_t num_iterations;
  int32_t num_rescaled; /* iterations whose full step failed the reduction / failure-rate test (step rescaling) */
} vb_summary;

typedef struct vb_cost_stats { /* CostStats (Factor.h:20-30) */
  int64_t num_total;
  int64_t num_invalid;
  int64_t num_prev_invalid;
} vb_cost_stats;

typedef struct vb_phase_times { /* per-phase device time of the last LM iteration [ms]; linearize_ms of an
                                   iteration vb_optimize linearized speculatively excludes the small
                                   factors and the clear, which ran beside the previous cost pass */
  double linearize_ms, schur_ms, factor_ms, solve_ms, step_ms, cost_ms, total_ms;
  double rs_update_ms; /* device rolling-shutter table rebuild (0 with host tables) */
} vb_phase_times;

typedef void (*vb_log_cb)(const char* msg, void* user);
typedef void (*vb_prestep_cb)(int iteration, void* user);

typedef struct vb_handle_s* vb_handle;

/* ---------------------------------------------------------------- lifecycle */
void vb_default_config(vb_config* cfg);
void vb_default_settings(vb_settings* s);
int vb_create(const vb_config* cfg, vb_handle* out);
int vb_destroy(vb_handle h);
const char* vb_last_error(void);

/* set (or replace before finalize) all variables of one kind: n rows of data (row size per kind:
 * 3/7/3/3/VB_CAM_DATA/7/32/7/4), constant[n] = 1 marks a constant variable (setConstant) */
int vb_set_vars(vb_handle h, int kind, int64_t n, const double* data, const uint8_t* constant);
/* append n factors of one kind: var_idx[n * vb_factor_num_vars(kind)],
 * ivals[n] (VB_F_VISUAL: rs table index or -1; ignored/NULL for other kinds),
 * consts[n * vb_factor_num_consts(kind)] */
int vb_add_factors(vb_handle h, int kind, int64_t n, const int32_t* var_idx, const int32_t* ivals,
                   const double* consts);
/* rolling-shutter tables (RollingShutterData::sampledRvp_ / interp_ / gravityWorld_):
 * table t owns samples [offsets[t], offsets[t+1]) with 11 doubles each
 * [R qx qy qz qw, dV 3, dP 3, dtSec] and (count-1) interpolants of 9 doubles each
 * [gyroRadSec 3, accelMSec2 3, deltaVelMSec 3] stored at interp[(offsets[t] - t) * 9 ...];
 * gravity[3 * t] = gravityWorld */
int vb_set_rs_tables(vb_handle h, int32_t n_tables, const int64_t* offsets, const double* samples,
                     const double* interp, const double* gravity);
/* rolling-shutter tables rebuilt on the device instead: the IMU-0 measurement
 * stream (ImuMeasurement, imu_types/ImuMeasurement.h:18-23; timestamps strictly increasing [ns],
 * gyro[3 n] rad/s, accel[3 n] m/s^2, as SingleSessionAdapter::initRollingShutterData's
 * imu0Measurements, InitCalibration.cpp:299-314) ... */
int vb_set_imu_measurements(vb_handle h, int64_t n, const int64_t* timestamp_ns, const double* gyro_rad_sec,
                            const double* accel_m_sec2);
/* ... and per table t (= the rs_table index of the visual factors): the midpoint (the rig's calib-state
 * timestamp) and half length [us] of RollingShutterData's constructor, the VB_VAR_IMU_CALIB handle
 * whose model parameters integrate it (imuCalib(rig, 0), InitCalibration.cpp:321) and the gravity
 * variable.  Replaces vb_set_rs_tables; both precede vb_finalize. */
int vb_set_rs_rigs(vb_handle h, int32_t n_tables, const int64_t* midpoint_us, const int64_t* half_length_us,
                   const int32_t* imu_calib, int32_t gravity_var);
/* RollingShutterData::compute for every table from the current variables (RollingShutterData.cpp:16-65
 * via updateRollingShutterData, InitCalibration.cpp:316-325); vb_optimize does this at the start of
 * every iteration, as ark_vi_ba's preStepCallback.  VB_E_RANGE when the IMU data does not cover an
 * interval (the reference throws in enumIntegrationSteps, PreIntegration.cpp:16-61). */
int vb_update_rs_tables(vb_handle h);
/* SingleSessionProblem::T_bodyImu_world_atImageRow (viba/problem/VisualFactor.cpp:303-327) for a batch of
 * observations, as SingleSessionAdapter::initPointsFromObservations needs it before the problem exists
 * (Triangulation.cpp:122-123,184-185 with kModelRollingShutter, after updateRollingShutterData,
 * SingleSessionAdapter.cpp:59,64).  Stateless (no handle): the tables of n_rs rigs are built on the device
 * from the IMU-0 stream (RollingShutterData::compute with table t's IMU calibration model rs_calib32[32 t..]
 * and gravity4), then observation i (rig obs_rig[i], camera record obs_cam[i] of cams24, image row
 * obs_row[i]) gets T_midImu_imuAtT^-1 T_bodyImu_world of its rig (rig_pose7, rig_vel3, table rig_rs[r] or
 * -1) when its camera is rolling-shutter or time-offset, else the rig pose; out_pose7: 7 doubles each.
 * VB_E_RANGE: IMU data not covering a table, or a row time outside it (the reference throws);
 * VB_E_ARG: a rolling-shutter camera on a rig without a table (findOrDie). */
int vb_rs_row_poses(int64_t n_imu, const int64_t* imu_t_ns, const double* imu_gyro, const double* imu_accel,
                    int32_t n_rs, const int64_t* rs_mid_us, const int64_t* rs_half_us, const double* rs_calib32,
                    const double* gravity4, int64_t n_rigs, const double* rig_pose7, const double* rig_vel3,
                    const int32_t* rig_rs, int64_t n_cams, const double* cams24, int64_t n_obs,
                    const int32_t* obs_rig, const int32_t* obs_cam, const double* obs_row, double* out_pose7);
/* download table t: sample count, samples (11 doubles each, NULL to skip) and interpolants (9 each) */
int vb_get_rs_table(vb_handle h, int32_t t, int32_t* n_samples, double* samples, double* interp);
/* --recompute-preint (viba/single_session/InertialFactors.cpp:19-70,
 * SingleSessionAdapter::regenerateAllPreintegrationsFromImuMeasurements): the preintegration of every
 * inertial factor row is recomputed from raw IMU data by computePreIntegration
 * (lib/motion/preintegration/PreIntegration.cpp:136-275) at the row's current IMU calibration
 * (its imu_calib variable, which also becomes the row's calibEvalPoint), on the device.
 *   vb_set_imu_stream     the measurement stream of IMU `imu` (imu 0 = vb_set_imu_measurements;
 *                         the ImuMeasurement vectors of SessionData, InertialFactors.cpp:26-27)
 *   vb_set_imu_noise      its sample variances (ImuNoiseModelParameters accel/gyroSampleVariance,
 *                         default: ImuNoiseModelParameters::reset, ImuNoiseModelParameters.h:78-80)
 *   vb_set_preint_sources per row of inertial kind `kind` (VB_F_IMU .. VB_F_IMU_SEC_SPLIT, in
 *                         vb_add_factors order): the IMU and the interval [t0, t1] in us (the rig
 *                         timestamps of generatePreintegration, :29-41)
 *   vb_set_recompute_preint  vb_optimize recomputes them at the start of every iteration
 *   vb_update_preintegrations  recompute now (after vb_finalize); VB_E_RANGE when a stream does not
 *                         cover an interval (enumIntegrationSteps throws, PreIntegration.cpp:36-44)
 * Streams and sources precede vb_finalize. */
int vb_set_imu_stream(vb_handle h, int imu, int64_t n, const int64_t* timestamp_ns, const double* gyro_rad_sec,
                      const double* accel_m_sec2);
int vb_set_imu_noise(vb_handle h, int imu, const double* accel_var3, const double* gyro_var3);
int vb_set_preint_sources(vb_handle h, int kind, int64_t n, const int32_t* imu, const int64_t* t0_us,
                          const int64_t* t1_us);
int vb_set_recompute_preint(vb_handle h, int on);
int vb_update_preintegrations(vb_handle h);
/* constants of factor row `row` of `kind` as the engine currently holds them (e.g. a recomputed
 * VB_PREINT_CONSTS row) */
int vb_get_factor_consts(vb_handle h, int kind, int64_t row, double* out);
/* refinePoints (viba/problem/PointRefinement.cpp:160-196, run by ark_vi_ba before optimize,
 * main_AriaKit_ViBa.cpp:69): every point with visual factors takes up to 5 damped Gauss-Newton steps on
 * those factors alone (optimizeOnePoint, :91-158), one wave per point on the device.  After vb_finalize
 * (and vb_update_rs_tables when rebuilt on the device); whole-problem handles only.
 * costs = {total start cost, total end cost}; stats = {failures, successful iterations, points with
 * at least one iteration} (the reference's log line, :183-194); either may be NULL. */
int vb_refine_points(vb_handle h, double* costs, int64_t* stats);
/* build the symbolic structure (≙ Optimizer::initSolver) and upload everything to HBM */
int vb_finalize(vb_handle h);
int64_t vb_reduced_order(vb_handle h);   /* order of the Schur-reduced (non-point) system */
int64_t vb_total_order(vb_handle h);     /* all registered tangent dims (points included) */

/* ---------------------------------------------------------------- LM building blocks */
/* Optimizer::computeGradHess (updateCachedResults, dontRetryFailed semantics of Factor.h:543-661);
 * linearizes at the current variables and keeps J/e on device; returns the cost */
int vb_linearize(vb_handle h, int update_cache, int dont_retry_failed, double* cost);
/* addDamping(lambda) + factor + solve(step = grad) (Optimizer.cpp:826-833): returns
 * model_cost_reduction = 0.5 * step . grad; the step is kept on device (negated, as :857) */
int vb_damp_factor_solve(vb_handle h, double lambda, double* model_cost_reduction);
/* gradient at the current variables (computeGradHess with hess = nullptr, :910-917) and
 * back_red = -0.5 * grad_new . step */
int vb_gradient_dot_step(vb_handle h, int dont_retry_failed, double* back_red);
/* sub-step: solve with the gradient computed by vb_gradient_dot_step using the existing factor,
 * negate, and store as the sub-step (Optimizer.cpp:958-972) */
int vb_solve_with_new_gradient(vb_handle h);
/* Reduced-system solver (Optimizer::Settings solverType / pcgMaxIterations / pcgDesiredResidual,
 * Optimizer.h:31-45; Optimizer.cpp:211-331).  VB_SOLVER_DIRECT is the tile Cholesky.  The PCG types
 * run the reference's PCG (PCG.cpp:15-104) on the Schur-reduced system after the point elimination,
 * with the preconditioners of Preconditioner.h: identity, block Jacobi over the parameter blocks, and
 * block Gauss-Seidel (the pseudo-factor -- diagonal blocks factored, off-diagonal blocks scaled, no
 * updates -- here over the 64 x 64 tiles of this library's reduced ordering, as BaSpaCho's is over
 * its supernodes), and LowerPrecSolvePrecond (Preconditioner.h:166-246: S cast to fp32 and factored by
 * the tile Cholesky's schedule in fp32, the diagonal raised and the factor redone while it holds a
 * non-finite value; applied by fp32 triangular solves).  Single handle only: VB_E_UNSUPPORTED on a
 * landmark shard or a partitioned rank.  Any time after vb_create. */
#define VB_SOLVER_DIRECT 0
#define VB_SOLVER_PCG_TRIVIAL 1
#define VB_SOLVER_PCG_JACOBI 2
#define VB_SOLVER_PCG_GAUSS_SEIDEL 3
#define VB_SOLVER_PCG_LOWER_PREC 4
int vb_set_solver(vb_handle h, int solver_type, int pcg_max_iterations, double pcg_desired_residual);
/* the reduced ordering of this handle (no reference counterpart: BaSpaCho's own ordering is internal):
 * reduced variable i = (kinds[i], handles[i]) occupies rows [offsets[i], offsets[i] + tangent dim) of the
 * padded order of padded_order rows, cut into 64 x 64 tiles; the block Gauss-Seidel preconditioner's
 * blocks are these tiles.  Any pointer may be NULL (n alone queries the count).  After vb_finalize. */
int vb_reduced_layout(vb_handle h, int32_t* kinds, int32_t* handles, int64_t* offsets, int64_t* n,
                      int64_t* padded_order);
/* Optimizer::computeJointCovariances (lib/small_thing/Optimizer.cpp:503-611; computeCovariances :613-697
 * is the one-variable-per-block case): at the current variables, linearize without touching the cost
 * cache, damp by `damping` (addDamping), factor; while the factor breaks down, raise the damping
 * (+1e-9 below 1e-9, else x2, :530-545).  Block q lists variables [block_start[q], block_start[q + 1])
 * of (kinds, handles); its joint covariance (the matching rows and columns of H^-1, H the damped
 * Hessian) is written column-major, sum of tangent dims squared, after the previous block's.  Reduced
 * variables only: landmark points are eliminated by this engine (VB_E_UNSUPPORTED), constant variables
 * have no covariance (VB_E_ARG).  One reduced solve per column on the device.  used_damping (may be
 * NULL) receives the damping of the factor that succeeded.  Invalidates the LM state of the handle. */
int vb_compute_covariances(vb_handle h, double damping, int64_t n_blocks, const int64_t* block_start,
                           const int32_t* kinds, const int32_t* handles, double* out, double* used_damping);
/* test fault injection: in iteration `iteration` (0-based, -1 = off) of the next vb_optimize calls the
 * model cost reduction is negated, which takes the reference's "quadratic model failing numerically"
 * branch (Optimizer.cpp:835-854: damping *= dampingAdjustOnFail, the step is kept) */
int vb_debug_negate_model_reduction(vb_handle h, int iteration);
/* test fault injection: iteration `iteration` (0-based, -1 = off) of the next vb_optimize calls fails as
 * a reduced-system breakdown would (VB_E_NUMERIC after the step and cost pass were queued): the
 * variables must come back to that iteration's linearization point */
int vb_debug_fail_iteration(vb_handle h, int iteration);
/* test support: slot of reduced tile (I, J) in the vb_reduced_buffers tile store (-1: not stored) */
int vb_debug_tile_slot(vb_handle h, int32_t I, int32_t J, int64_t* slot);
/* iterations and relative residual of the last PCG solve (PCG::Result) */
int vb_pcg_stats(vb_handle h, int32_t* iterations, double* relative_residual);
/* step *= factor (in place) */
int vb_scale_step(vb_handle h, double factor);
/* applyStep(step) or applyStep(substep) (which = 0 / 1); ratios = {Linf, L2, L1} */
int vb_apply_step(vb_handle h, int which, double ratios[3]);
/* Optimizer::computeCost(makeComparableWithStored, &stats) (Factor.h:390-417, 664-701) */
int vb_cost(vb_handle h, int comparable, double* cost, vb_cost_stats* stats);
int vb_backup(vb_handle h);
int vb_restore(vb_handle h);
/* download variables of one kind (row layout as vb_set_vars) */
int vb_get_vars(vb_handle h, int kind, double* out);
/* download the last step (negated solution, per variable kind, rows of the kind's tangent size;
 * constant / unregistered variables get zeros); which = 0 step, 1 sub-step */
int vb_get_step(vb_handle h, int which, int kind, double* out);
/* download gradient (as computed by the last vb_linearize) per kind, like vb_get_step */
int vb_get_gradient(vb_handle h, int kind, double* out);

/* ---------------------------------------------------------------- full loop */
/* Optimizer::optimize (Optimizer.cpp:768-1106, direct solver) */
int vb_optimize(vb_handle h, const vb_settings* s, vb_log_cb log, vb_prestep_cb prestep, void* user,
                vb_summary* out);
int vb_last_phase_times(vb_handle h, vb_phase_times* out);

/* applyStep without the normalisation: raw = {max ratio, sum ratio^2, sum ratio} over the variables
 * this handle counts (a shard: its landmarks, + the reduced variables on the root), so that a
 * multi-device caller can reduce them; vb_apply_step = raw normalised by vb_num_params */
int vb_apply_step_raw(vb_handle h, int which, double raw[3]);
int64_t vb_num_params(vb_handle h);   /* registered parameter blocks (Optimizer.cpp:1017 divisor) */

/* ---------------------------------------------------------------- multi-device (landmark shards)
 * each device owns the landmarks [lm_begin, lm_end) (landmark order = earliest
 * observing rig, so shards are time bands), linearizes their visual factors and eliminates them;
 * the root (is_root = 1) also owns the constant-point observations, every small factor (IMU, omega,
 * random walks, priors) and the identity damping term.  Must precede vb_finalize.  The caller sums
 * the partial reduced systems on the root between the calls below (distributed.py: point-to-point
 * tile bands + reduce of the RHS over RCCL), the root factors/solves, and broadcasts x_red. */
int vb_set_landmark_shard(vb_handle h, int64_t lm_begin, int64_t lm_end, int is_root);
/* device pointers + sizes (in doubles) of the reduced matrix (tile store) and the reduced RHS */
int vb_reduced_buffers(vb_handle h, double** matrix, int64_t* matrix_len, double** rhs,
                       int64_t* rhs_len);
/* exact tile set of a non-root shard's partial reduced system (the root's list is empty): tile
 * indices ascending; tiles == NULL queries the count.  Replaces the band of vb_shard_tile_range
 * for the exchange (ND ordering spreads a shard's contributions over its subtree and the separators
 * above it).  Reference: the per-shard partial Hessian of SURVEY 8e (no reference counterpart: the
 * reference is single-process). */
int vb_shard_tiles(vb_handle h, int32_t* tiles, int64_t* n);
/* gather this shard's tiles (vb_shard_tiles order) into an engine-owned device buffer of
 * n * 64 * 64 doubles; synchronous */
int vb_pack_shard_tiles(vb_handle h, double** buf, int64_t* len);
/* root: add n packed tiles (device buffer, vb_pack_shard_tiles layout of the sender) into the tile
 * store at the device-resident tile indices; synchronous */
int vb_add_tiles(vb_handle h, const int32_t* tiles_dev, int64_t n, const double* buf_dev);
/* the contiguous range of the tile store this shard's partial reduced system can touch */
int vb_shard_tile_range(vb_handle h, int64_t* first_double, int64_t* num_doubles);
/* split of vb_damp_factor_solve (Optimizer.cpp:826-833) for sharded use:
 * (1) partial damped Schur-reduced system + RHS of this shard, (2) root: factor + solve (x_red is
 * left in the RHS buffer), (3) every shard: x_red (in the RHS buffer) -> its points' step and the
 * partial model cost reduction (summed by the caller) */
int vb_assemble_reduced(vb_handle h, double lambda);
int vb_factor_solve_reduced(vb_handle h);
int vb_back_substitute(vb_handle h, double* model_cost_reduction_partial);
/* split of vb_solve_with_new_gradient (Optimizer.cpp:958-972) for sharded use, after
 * vb_gradient_dot_step: (1) partial new RHS, (2) root: solve with the existing factor,
 * (3) every shard: sub-step of its points (which = 1) */
int vb_assemble_new_rhs(vb_handle h);
int vb_solve_reduced(vb_handle h);
int vb_back_substitute_which(vb_handle h, int which, double* model_cost_reduction_partial);
/* ---------------------------------------------------------------- multi-device (partitioned factorization)
 * SURVEY.md §8f-1 (no reference counterpart: the reference factors on one host with BaSpaCho).  With
 * vb_set_partition (before vb_finalize; world a power of two) the nested-dissection order gives rank
 * r the subtree r levels below the top log2(world) separators; the separators ("ROOT" columns) are
 * factored on rank 0.  Every landmark goes to the rank whose subtree its observations touch (none
 * touches two), rank 0 for ROOT-only ones; rank r evaluates and eliminates its landmarks and the
 * small factors writing its columns.  Per LM iteration (distributed.py PartitionedOptimizer):
 *   vb_assemble_reduced -> vb_factor_part(0) -> vb_solve_part(0)
 *   -> sum of ROOT tiles / ROOT rhs rows on rank 0 (vb_part_exchange 0 / 1 + reduce)
 *   -> rank 0: vb_factor_part(1), vb_solve_part(1) -> broadcast ROOT rows of x (vb_part_exchange 2)
 *   -> vb_solve_part(2) -> vb_share_x + all-reduce -> vb_back_substitute */
int vb_set_partition(vb_handle h, int rank, int world);
/* which 0: factor this rank's subtree columns (and apply their updates to its partial ROOT tiles);
 * which 1 (rank 0, after the ROOT tiles were summed): factor the ROOT columns */
int vb_factor_part(vb_handle h, int which);
/* phase 0: forward solve over the subtree (rhs -> partial ROOT rows); 1 (rank 0): forward + backward
 * over the ROOT columns; 2: backward over the subtree given the ROOT rows of x */
int vb_solve_part(vb_handle h, int phase);
/* what 0 ROOT tiles, 1 ROOT rows of the forward-solve work vector, 2 ROOT rows of x;
 * dir 0 packs them into an engine-owned device buffer (returned), dir 1 writes that buffer back */
int vb_part_exchange(vb_handle h, int what, int dir, double** buf, int64_t* len);
/* x rows this rank solved (other rows zero) into the RHS buffer (returned) for an all-reduce sum;
 * then vb_back_substitute reads x_red from that buffer */
int vb_share_x(vb_handle h, double** xred, int64_t* len);
/* [this rank's subtree tile columns, ROOT tile columns, fan-in contributions of its subtree schedule,
 *  of the ROOT schedule (rank 0 only), ROOT tiles exchanged per factorization] */
int vb_part_info(vb_handle h, int64_t* out5);

/* ---------------------------------------------------------------- deferred mode (multi-process LM)
 * The multi-process controllers (distributed.py) read the LM scalars once per iteration, as
 * vb_optimize does (Optimizer.cpp:800-1097 reads them phase by phase).  With vb_set_deferred(h, 1) the
 * phase functions above (vb_update_rs_tables, vb_linearize, vb_assemble_reduced, vb_factor_solve_reduced,
 * vb_solve_reduced, vb_factor_part, vb_solve_part, vb_part_exchange, vb_share_x, vb_pack_shard_tiles,
 * vb_add_tiles, vb_back_substitute_which, vb_apply_step_raw, vb_cost) queue their device work and
 * return without waiting; their scalar outputs are NaN, and the values stay in device slots
 * (vb_scalar_slots) that the caller all-reduces in place on the handle's stream (vb_stream, RCCL) and
 * reads once (vb_read_scalars).  Errors stay in the error words and are reported by vb_read_scalars. */
int vb_set_deferred(vb_handle h, int on);
/* device pointers: red[0] linearization cost, [1] cost-pass cost, [2..4] CostStats (numTotal of the
 * visual factors, numInvalid, numPrevInvalid), [8] max step ratio, [9] sum of squared step ratios,
 * [10] sum of step ratios, [16] twice the model cost reduction -- this handle's partials; err[0..2)
 * error bit words (bitwise-or reducible) */
int vb_scalar_slots(vb_handle h, double** red, int32_t** err);
/* what numTotal adds for this handle's non-visual factors in the cost pass (the root's, else 0) */
int vb_small_factor_count(vb_handle h, int64_t* n);
/* record the point after which the slots hold the iteration's scalars (work queued later, e.g. a
 * speculative linearization, does not delay vb_read_scalars); needs vb_spec_prepare */
int vb_mark_scalars(vb_handle h);
/* copy red[0, n) (n <= 24) to the host after the mark (or after all queued work) and return the error
 * the error words encode (0 if none) */
int vb_read_scalars(vb_handle h, double* out, int n);
/* the two error bit words behind the last error check of this handle (vb_read_scalars, or any
 * synchronous call); a multi-process controller ORs them over the ranks */
int vb_error_words(vb_handle h, int32_t* out2);
/* the code (and vb_last_error text) two error bit words encode, checked in causal order as every
 * synchronous call does: after the words are ORed over the ranks, each rank raises the same error with
 * the same message (the reference's XR_CHECK / throw sites, Optimizer.cpp:200-231, RollingShutterData.cpp) */
int vb_error_from_words(vb_handle h, const int32_t* words2);
/* vb_optimize's speculative next-iteration linearization for an external controller: *ok = 1 when its
 * spare buffers (a second tile store, ResultCache, gradient, rolling-shutter tables) are allocated */
int vb_spec_prepare(vb_handle h, int* ok);
/* queue the rolling-shutter rebuild (if device-built) and the linearization at the current variables
 * into the spare buffers (ark_vi_ba's preStepCallback + Optimizer.cpp:807-812 of the next iteration) */
int vb_spec_linearize(vb_handle h, int dont_retry_failed);
/* use = 1 (the step stayed applied at full size): the spare buffers become the handle's and the handle
 * is linearized (cost partial in red[0]); use = 0: dropped */
int vb_spec_commit(vb_handle h, int use);
/* out2 = [rolling-shutter rebuild ms, linearization ms] of the speculative linearization last committed
 * (its device events; complete once the iteration that used it has read its scalars): an external
 * controller's phase clock attributes them to that iteration, as vb_optimize's vb_phase_times does */
int vb_spec_phase_ms(vb_handle h, double* out2);

/* the HIP stream of the handle (hipStream_t), for interop with torch / RCCL */
void* vb_stream(vb_handle h);

/* ---------------------------------------------------------------- measurement
 * time every launch of one kernel family with HIP events on the handle's stream
 * (0 visual linearize, 1 landmark eliminate, 2 Schur assembly, 3 standalone potrf, 4 tile GEMM
 *  update (+ fused next-diagonal potrf), 5 forward solve, 6 backward solve, 7 point
 *  back-substitution, 8 visual cost, 9 small factors, 10 tile trsm; -1 disables); vb_kernel_time returns launches and summed device milliseconds since enabling */
int vb_profile_kernel(vb_handle h, int family);
int vb_kernel_time(vb_handle h, int64_t* launches, double* total_ms);
/* The profiled family's busy time since enabling: the union of its launches' intervals (the factorization
 * launches on several streams, so its launches can overlap and their summed durations count that time
 * more than once).  Equal to vb_kernel_time's total when the launches do not overlap. */
int vb_kernel_busy_time(vb_handle h, double* busy_ms);
/* [nObs, nPoints, nReducedVars, reducedOrder, nTileCols, nTiles, nGemmPairs (per factorization),
 *  nSmallFactors, Schur landmark-pair entries, Schur observation-pair entries,
 *  elimination levels (one fan-in launch each, except a level without contributions), tiles of S
 *  without the symbolic fill] */
int vb_problem_stats(vb_handle h, int64_t* out12);
/* the direct factorization's schedule as it runs: [elimination levels, fan-in tile contributions per
 * factorization, supernodes, two-column supernodes] -- the column schedule (one level per tile column
 * chain step) unless VIBA_SUPERNODE=1 at vb_create built the two-column supernode schedule */
int vb_factor_schedule_stats(vb_handle h, int64_t* out4);
/* tuning aid: average time [us] of one kernel launch: on scratch tiles (which: 0 potrf, 1 trsm, 2 fan-in)
 * or, alone on the handle's own data (its results are not meant to be used afterwards), 10 visual
 * linearization, 12 landmark elimination, 13 observation-group Gram blocks, 14 Schur tile products,
 * 15 visual cost pass, 16 small factors' evaluation, 17 / 18 their assembly (IMU kinds / the rest, from
 * the staging of an earlier 16), 19 the reduced system's clear */
int vb_bench_kernel(vb_handle h, int which, int iters, double* avg_us);

#ifdef __cplusplus
}
#endif
#endif /* VIBA_HIP_H */
