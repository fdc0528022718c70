// Stand-alone entries: the rolling-shutter row poses of the session set-up and the kernel micro-benchmark.
#include "host.hpp"

// ---------------------------------------------------------------- rolling-shutter row poses (session set-up)
// SingleSessionAdapter::initPointsFromObservations triangulates with T_bodyImu_world_atImageRow
// (Triangulation.cpp:122-123,184-185, kModelRollingShutter = true, Triangulation.h:43) after
// updateRollingShutterData (SingleSessionAdapter.cpp:59,64).  Stateless: builds the tables of the given
// rigs on the device (rs_build_kernel, the per-iteration rebuild's kernel) and evaluates every
// observation's row pose (rs_row_pose_kernel), then frees everything.  Errors as the reference's
// throws / aborts: VB_E_RANGE (IMU data do not cover a table, or a row time outside its table),
// VB_E_ARG (a rolling-shutter camera on a rig without a table).
extern "C" int vb_rs_row_poses(int64_t n_imu, const int64_t* imu_t_ns, const double* imu_gyro, const double* imu_accel,
                               int32_t n_rs, const int64_t* rs_mid_us, const int64_t* rs_half_us, const double* rs_calib32,
                               const double* gravity4, int64_t n_rigs, const double* rig_pose7, const double* rig_vel3,
                               const int32_t* rig_rs, int64_t n_cams, const double* cams24, int64_t n_obs,
                               const int32_t* obs_rig, const int32_t* obs_cam, const double* obs_row, double* out_pose7) {
  if (n_imu < 0 || n_rs < 0 || n_rigs < 0 || n_cams < 0 || n_obs < 0 || (n_obs && (!obs_rig || !obs_cam || !obs_row ||
      !out_pose7 || !rig_pose7 || !rig_vel3 || !rig_rs || !cams24)) || (n_rs && (!imu_t_ns || !imu_gyro || !imu_accel ||
      !rs_mid_us || !rs_half_us || !rs_calib32 || !gravity4)))
    return fail(VB_E_ARG, "bad vb_rs_row_poses arguments");
  for (int64_t i = 0; i < n_obs; i++)
    if (obs_rig[i] < 0 || obs_rig[i] >= n_rigs || obs_cam[i] < 0 || obs_cam[i] >= n_cams)
      return fail(VB_E_ARG, "vb_rs_row_poses: observation with an unknown rig or camera");
  for (int64_t r = 0; r < n_rigs; r++)
    if (rig_rs[r] >= n_rs) return fail(VB_E_ARG, "vb_rs_row_poses: unknown rolling-shutter table");
  for (int64_t i = 1; i < n_imu; i++)
    if (imu_t_ns[i] <= imu_t_ns[i - 1]) return fail(VB_E_ARG, "IMU timestamps must increase");
  if (n_obs == 0) return 0;
  std::vector<void*> mem;
  auto freeAll = [&] { for (void* p : mem) (void)hipFree(p); };
  auto up = [&](auto** dst, const auto* src, size_t n) -> bool {
    void* p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(*src)) != hipSuccess) return false;
    mem.push_back(p);
    *dst = (std::remove_cv_t<std::remove_reference_t<decltype(**dst)>>*)p;
    return n == 0 || hipMemcpy(p, src, n * sizeof(*src), hipMemcpyHostToDevice) == hipSuccess;
  };
  auto zero = [&](auto** dst, size_t n) -> bool {
    void* p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(**dst)) != hipSuccess) return false;
    mem.push_back(p);
    *dst = (std::remove_reference_t<decltype(*dst)>)p;
    return hipMemset(p, 0, std::max<size_t>(n, 1) * sizeof(**dst)) == hipSuccess;
  };
  Dev d{};
  // tables: capacity as vb_finalize sizes them (the samples of [mid - half, mid + half] +- 20 ms, + 4)
  std::vector<int64_t> off(n_rs + 1, 0);
  std::vector<double> v((size_t)n_imu * 6);
  for (int64_t i = 0; i < n_imu; i++)
    for (int k = 0; k < 3; k++) v[6 * i + k] = imu_gyro[3 * i + k], v[6 * i + 3 + k] = imu_accel[3 * i + k];
  for (int32_t t = 0; t < n_rs; t++) {
    const int64_t kWidenNs = 20000000;
    const int64_t a = (rs_mid_us[t] - rs_half_us[t]) * 1000 - kWidenNs, b = (rs_mid_us[t] + rs_half_us[t]) * 1000 + kWidenNs;
    off[t + 1] = off[t] + (std::upper_bound(imu_t_ns, imu_t_ns + n_imu, b) - std::lower_bound(imu_t_ns, imu_t_ns + n_imu, a)) + 4;
  }
  std::vector<int32_t> calibIdx(n_rs);
  std::iota(calibIdx.begin(), calibIdx.end(), 0);
  int32_t *oRig = nullptr, *oCam = nullptr, *rRS = nullptr;
  double *oRow = nullptr, *rPose = nullptr, *rVel = nullptr, *cams = nullptr, *out = nullptr;
  bool ok = zero(&d.err, 4) && up(&oRig, obs_rig, n_obs) && up(&oCam, obs_cam, n_obs) && up(&oRow, obs_row, n_obs) &&
            up(&rPose, rig_pose7, n_rigs * 7) && up(&rVel, rig_vel3, n_rigs * 3) && up(&rRS, rig_rs, n_rigs) &&
            up(&cams, cams24, n_cams * 24) && zero(&out, n_obs * 7);
  if (ok && n_rs) {
    d.nRS = n_rs, d.nImu = n_imu, d.rsGravVar = 0;
    ok = up(&d.imuT, imu_t_ns, n_imu) && up(&d.imuV, v.data(), v.size()) && up(&d.rsMid, rs_mid_us, n_rs) &&
         up(&d.rsHalf, rs_half_us, n_rs) && up(&d.rsCalib, calibIdx.data(), n_rs) &&
         up(&d.var[6], rs_calib32, (size_t)n_rs * 32) && up(&d.var[8], gravity4, 4) && up(&d.rsOff, off.data(), off.size()) &&
         zero(&d.rsS, off[n_rs] * 11) && zero(&d.rsI, (off[n_rs] - n_rs) * 9) && zero(&d.rsG, (size_t)n_rs * 3) &&
         zero(&d.rsN, n_rs);
  }
  if (!ok) {
    freeAll();
    return fail(VB_E_HIP, "vb_rs_row_poses: device allocation / copy failed");
  }
  if (n_rs) launch_rs_build(d, nullptr);
  launch_rs_row_poses(d, n_obs, oRig, oCam, oRow, rPose, rVel, rRS, cams, out, nullptr);
  int32_t e[2] = {0, 0};
  const bool okRun = hipDeviceSynchronize() == hipSuccess && hipMemcpy(e, d.err, sizeof(e), hipMemcpyDeviceToHost) == hipSuccess &&
                     hipMemcpy(out_pose7, out, (size_t)n_obs * 7 * sizeof(double), hipMemcpyDeviceToHost) == hipSuccess;
  freeAll();
  if (!okRun) return fail(VB_E_HIP, "vb_rs_row_poses: kernel failed");
  if (e[1] & 1) return fail(VB_E_RANGE, "enumIntegrationSteps: IMU measurements do not cover a rolling-shutter interval");
  if (e[1] & 2) return fail(VB_E_NUMERIC, "RollingShutterData::compute: non-increasing sample times");
  if (e[1] & 4) return fail(VB_E_STATE, "internal: rolling-shutter table capacity exceeded");
  if (e[0] & 2) return fail(VB_E_ARG, "T_bodyImu_world_atImageRow: rolling-shutter camera on a rig without a table");
  if (e[0] & 1) return fail(VB_E_RANGE, "RollingShutterData::getEstimate: image-row time outside the table");
  return 0;
}

// ---------------------------------------------------------------- kernel micro-benchmark (tuning aid)
// Times one launch of a factorization kernel on scratch tiles (random SPD diagonal tile, random
// off-diagonal tiles), averaged over `iters` launches, kernel-exact (hipExtLaunchKernelGGL events).
// which: 0 potrf, 1 trsm (one tile), 2/3 update (one pair)
extern "C" int vb_bench_kernel(vb_handle h, int which, int iters, double* avg_us) {
  if (!h || !h->finalized || iters <= 0) return fail(VB_E_STATE, "vb_bench_kernel needs a finalized handle");
  if (which >= 10) {  // kernels of the linearize / Schur phases alone, on the handle's own data
    Dev& d = h->d;
    hipEvent_t e0, e1, evP;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    HIPCHK(hipEventCreateWithFlags(&evP, hipEventDisableTiming));
    HIPCHK(hipStreamSynchronize(h->st));
    double total = 0;
    for (int it = 0; it < iters + 1; it++) {
      HIPCHK(hipEventRecord(e0, h->st));
      switch (which) {
        case 10:  // visual linearization (records)
          launch_visual_lin(d, 0, 0, d.obB, d.obE, h->st);
          launch_visual_lin(d, 0, 0, d.fB, d.fE, h->st);
          break;
        case 12: launch_landmark(d, 1e-5, 0, d.lmB, d.lmE, h->st); break;  // landmark elimination
        case 13: launch_groups(d, 1e-5, h->st); break;                     // observation-group Gram blocks
        case 14: launch_schur_products(d, 1e-5, h->st); break;             // Schur tile products
        case 15: launch_visual_cost(d, 1, d.obB, d.obE, h->st); break;     // cost pass (visual)
        // the small factors (staging for 17 / 18 from an earlier 16) and the clear; they change the tiles
        case 16: launch_small_eval(d, 0, d.gRed, h->st); break;
        case 17: launch_small_assemble(d, 0, d.gRed, h->st, 1); break;
        case 18: launch_small_assemble(d, 0, d.gRed, h->st, 2); break;
        case 19:
          if (int rc = clearReduced(h, d, h->st)) return rc;
          break;
        // overlap probes (timing only: the products read the previous elimination's Y): landmark elimination
        // and tile products side by side (20) or in sequence (21); 22: elimination + groups side by side
        case 20:
        case 22:
          HIPCHK(hipEventRecord(h->evFork, h->st));
          HIPCHK(hipStreamWaitEvent(h->st2, h->evFork, 0));
          if (which == 20) launch_schur_products(d, 1e-5, h->st2);
          else launch_groups(d, 1e-5, h->st2);
          HIPCHK(hipEventRecord(h->evJoin, h->st2));
          launch_landmark(d, 1e-5, 0, d.lmB, d.lmE, h->st);
          HIPCHK(hipStreamWaitEvent(h->st, h->evJoin, 0));
          break;
        case 21:
          launch_landmark(d, 1e-5, 0, d.lmB, d.lmE, h->st);
          launch_schur_products(d, 1e-5, h->st);
          break;
        // the factorization (its streams) alone (23), and beside the tile products on stF (24); timing only
        // (the tiles are refactored in place, so their values are garbage after the first launch)
        case 23:
          if (int rc = factorReduced(h, 0)) return rc;
          break;
        case 24:
        case 25: {  // 25: the products on stZ instead
          hipStream_t ps = which == 24 ? h->stF : h->stZ;
          HIPCHK(hipEventRecord(h->evFork, h->st));
          HIPCHK(hipStreamWaitEvent(ps, h->evFork, 0));
          launch_schur_products(d, 1e-5, ps);
          HIPCHK(hipEventRecord(evP, ps));
          if (int rc = factorReduced(h, 0)) return rc;
          HIPCHK(hipStreamWaitEvent(h->st, evP, 0));
          break;
        }
        default: return fail(VB_E_ARG, "vb_bench_kernel: unknown kernel");
      }
      HIPCHK(hipEventRecord(e1, h->st));
      HIPCHK(hipStreamSynchronize(h->st));
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, e0, e1));
      if (it > 0) total += ms;
    }
    hipEventDestroy(e0), hipEventDestroy(e1), hipEventDestroy(evP);
    if (avg_us) *avg_us = total * 1e3 / iters;
    // the timed launches left partial sums in the striped reduction slots (no fold_red after them) and
    // overwrote tiles, gradient and staging: clear the slots, and make the handle re-linearize before
    // any solve or cost comparison uses that state
    HIPCHK(hipMemsetAsync(d.redS, 0, 64 * 8 * sizeof(double), h->st));
    HIPCHK(hipStreamSynchronize(h->st));
    h->linearized = h->factored = false;
    return checkErr(h) == VB_E_HIP ? VB_E_HIP : 0;
  }
  Dev d = h->d;  // copy: tiles / err redirected to scratch
  std::vector<double> A(TS * TS), B(TS * TS);
  uint64_t sd = 12345;
  auto rnd = [&] { sd = sd * 6364136223846793005ULL + 1442695040888963407ULL; return ((sd >> 11) * 0x1.0p-53) - 0.5; };
  std::vector<double> M(TS * TS);
  for (auto& v : M) v = rnd();
  for (int i = 0; i < TS; i++)
    for (int j = 0; j < TS; j++) {
      double s = (i == j) ? TS : 0.0;
      for (int k = 0; k < TS; k++) s += M[i * TS + k] * M[j * TS + k];
      A[j * TS + i] = s;
    }
  for (auto& v : B) v = rnd();
  double *tiles = nullptr, *dinv = nullptr;
  int32_t *colT = nullptr, *pairs = nullptr, *targ = nullptr;
  HIPCHK(hipMalloc(&tiles, 4 * TS * TS * sizeof(double)));
  HIPCHK(hipMalloc(&dinv, 2 * 1024 * sizeof(double)));
  HIPCHK(hipMalloc(&colT, 4 * sizeof(int32_t)));
  HIPCHK(hipMalloc(&pairs, 4 * sizeof(int32_t)));
  HIPCHK(hipMalloc(&targ, sizeof(int32_t)));
  // potrf: tile 0 (col 0); trsm: diag 0 -> target 1; fan-in: 4 x (L_IK 1, L_JK 1) -> target 2 (plain)
  const int32_t ct[4] = {0, 0, 1, 0}, pr[4] = {2, 0, 4, 0}, tg[1] = {0};
  const int32_t fp[8] = {1, 1, 1, 1, 1, 1, 1, 1};
  HIPCHK(hipMemcpy(colT, ct, sizeof(ct), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(pairs, pr, sizeof(pr), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(targ, tg, sizeof(tg), hipMemcpyHostToDevice));
  int32_t* fpD = nullptr;
  HIPCHK(hipMalloc(&fpD, sizeof(fp)));
  HIPCHK(hipMemcpy(fpD, fp, sizeof(fp), hipMemcpyHostToDevice));
  d.tiles = tiles;
  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&e1));
  double total = 0;
  const size_t tb = TS * TS * sizeof(double);
  for (int it = 0; it < iters + 1; it++) {
    // tile 0: SPD (factored first for trsm/update), tile 1: off-diagonal, tile 2: SPD target
    HIPCHK(hipMemcpyAsync(tiles, A.data(), tb, hipMemcpyHostToDevice, h->st));
    HIPCHK(hipMemcpyAsync(tiles + TS * TS, B.data(), tb, hipMemcpyHostToDevice, h->st));
    HIPCHK(hipMemcpyAsync(tiles + 2 * TS * TS, A.data(), tb, hipMemcpyHostToDevice, h->st));
    if (which != 0) launch_potrf(d, colT, targ, 1, dinv, h->st);
    g_prof.start = e0, g_prof.stop = e1, g_prof.consumed = false;
    if (which == 0) launch_potrf(d, colT, targ, 1, dinv, h->st);
    else if (which == 1) launch_trsm(d, colT, colT + 2, targ, 1, dinv, h->st);
    else launch_fanin(d, pairs, fpD, 1, h->st);
    g_prof = ProfSlot();
    HIPCHK(hipStreamSynchronize(h->st));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    if (it > 0) total += ms;  // first launch: warm-up
  }
  hipEventDestroy(e0), hipEventDestroy(e1);
  hipFree(tiles), hipFree(dinv), hipFree(colT), hipFree(pairs), hipFree(targ), hipFree(fpD);
  if (avg_us) *avg_us = total * 1e3 / iters;
  return 0;
}

