// Host side of the HIP LM engine: the C-ABI (include/viba_hip.h) numeric phases and the
// Levenberg-Marquardt controller (≙ Optimizer::optimize, Optimizer.cpp:768-1106).  All numeric work runs
// in HIP kernels on the handle's stream; the host only orders launches, reads back scalars and takes LM
// decisions.  vb_finalize's symbolic analysis is finalize.hip, the multi-process entries multi.hip.
#include "host.hpp"

namespace viba {
ProfSlot g_prof;
}

namespace viba_host {

// kernel families for vb_profile_kernel
enum { KF_VISUAL_LIN = 0, KF_LANDMARK, KF_SCHUR, KF_POTRF, KF_GEMM, KF_FWD, KF_BWD, KF_BACKSUB, KF_VISUAL_COST,
       KF_SMALL, KF_TRSM, KF_SYMV, KF_COUNT };

inline void profBegin(vb_handle h, int fam) {
  if (h->profFamily != fam) return;
  if (h->profUsed + 2 > h->profEv.size()) {
    for (int i = 0; i < 256; i++) {
      hipEvent_t e;
      (void)hipEventCreate(&e);
      h->profEv.push_back(e);
    }
  }
  g_prof.start = h->profEv[h->profUsed], g_prof.stop = h->profEv[h->profUsed + 1], g_prof.consumed = false;
}
inline void profEnd(vb_handle h, int fam) {
  if (h->profFamily != fam) return;
  if (g_prof.consumed) h->profUsed += 2;  // the wrapper launched the family's kernel with the events
  g_prof = ProfSlot();
}
// duration of one profiled launch.  The stop event of a hipExtLaunchKernelGGL launch can still report
// hipErrorNotReady after a wait on a later event of the same stream (about a quarter of the pairs read
// right after vb_optimize's scalar read did, and counted 0 ms: the event-timed fan-in average came out
// 26% low against rocprofv3); such a pair is read again after hipEventSynchronize.
float profPairMs(hipEvent_t a, hipEvent_t b) {
  float ms = 0;
  if (hipEventElapsedTime(&ms, a, b) == hipErrorNotReady) {
    (void)hipEventSynchronize(b);
    (void)hipEventSynchronize(a);
    ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
  }
  return ms;
}
// the first n recorded pairs into the totals: the summed launch durations, and the family's busy time, the
// union of the launches' intervals (launches on several streams overlap: the factorization's streams)
void profAccumulate(vb_handle h, size_t n) {
  std::vector<std::pair<double, double>> iv;
  for (size_t i = 0; i < n; i += 2) {
    const float ms = profPairMs(h->profEv[i], h->profEv[i + 1]);
    h->profMs += ms;
    h->profLaunches++;
    // the launch's start against the first one's, with the same not-ready retry as its duration (a
    // not-ready pair read as 0 would place the launch at the origin and shrink the busy union)
    const float t0 = i > 0 ? profPairMs(h->profEv[0], h->profEv[i]) : 0.0f;
    iv.push_back({(double)t0, (double)t0 + ms});
  }
  std::sort(iv.begin(), iv.end());
  double end = -1e300;
  for (const auto& x : iv) {
    if (x.first > end) h->profBusyMs += x.second - x.first, end = x.second;
    else if (x.second > end) h->profBusyMs += x.second - end, end = x.second;
  }
}
// harvest recorded pairs (call after a stream synchronisation)
void profHarvest(vb_handle h) {
  if (h->profFamily < 0 || h->profUsed == 0) return;
  (void)hipStreamSynchronize(h->st);
  profAccumulate(h, h->profUsed);
  h->profUsed = 0, h->profDone = 0;
}
// harvest the first n entries (complete at the last stream sync) after the next iteration's work is
// queued, so the host reads the event times while the device runs instead of between two iterations;
// the entries still pending move to the front
void profHarvestPrefix(vb_handle h, size_t n) {
  if (h->profFamily < 0 || n == 0 || n > h->profUsed) return;
  profAccumulate(h, n);
  std::rotate(h->profEv.begin(), h->profEv.begin() + n, h->profEv.begin() + h->profUsed);
  h->profUsed -= n, h->profDone = 0;
}

int checkRsErr(vb_handle h, int32_t e);
int checkErr(vb_handle h) {
  int32_t ee[2] = {0, 0};
  HIPCHK(hipMemcpyAsync(ee, h->d.err, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  return errFromWords(h, ee);
}
int errFromWords(vb_handle h, const int32_t* ee) {
  h->lastWords[0] = ee[0], h->lastWords[1] = ee[1];
  const int32_t e = ee[0];
  if (int rc = checkRsErr(h, ee[1])) return rc;
  // in causal order within an iteration: the linearization, the elimination and factorization, then the
  // cost pass at the stepped variables (whose lookups a broken step can push out of range)
  if (e & 1) return fail(VB_E_RANGE, "RollingShutterData::getEstimate: out of range");
  if (e & 2) return fail(VB_E_NUMERIC, "landmark 3x3 Cholesky breakdown");
  if (e & 8) return fail(VB_E_NUMERIC, "reduced system Cholesky breakdown (not positive definite)");
  if (e & 4) return fail(VB_E_STATE, "internal: Schur contribution outside the symbolic structure");
  if (e & 16) return fail(VB_E_HIP, "internal: triangular-solve hand-off timed out");
  if (e & 32) return fail(VB_E_RANGE, "RollingShutterData::getEstimate: out of range (cost pass)");
  return 0;
}

// errors of the last device rolling-shutter rebuild (rs.hip): the reference throws there
int checkRsErr(vb_handle h, int32_t e) {
  if (e & 1) return fail(VB_E_RANGE, "enumIntegrationSteps: IMU measurements do not cover the rolling-shutter interval");
  if (e & 2) return fail(VB_E_NUMERIC, "RollingShutterData::compute: non-increasing sample times");
  if (e & 4) return fail(VB_E_STATE, "internal: rolling-shutter table capacity exceeded");
  if (e & 8) return fail(VB_E_RANGE, "enumIntegrationSteps: IMU measurements do not cover a preintegration interval");
  if (e & 16) return fail(VB_E_NUMERIC, "computePreIntegration: covariance not positive definite");
  return 0;
}

int readRed(vb_handle h, double* out, int i0, int n) {
  HIPCHK(hipMemcpyAsync(out, h->d.red + i0, n * sizeof(double), hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  profHarvest(h);
  return 0;
}
// vb_optimize's one read per iteration: the scalars red[0, n) and the error words in one stream sync;
// the profiled events stay for profHarvestPrefix after the next enqueue
int readRedErr(vb_handle h, double* out, int n) {
  int32_t ee[2] = {0, 0};
  HIPCHK(hipMemcpyAsync(out, h->d.red, n * sizeof(double), hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipMemcpyAsync(ee, h->d.err, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  h->profDone = h->profUsed;
  return errFromWords(h, ee);
}

}  // namespace viba_host

namespace viba_host {
// ------------------------------------------------------------------ numeric phases
// small factors (root only) on the side stream; joinSmall makes the main stream wait for them
bool smallHere(vb_handle h, int mode) { return h->isRoot || (h->partSet && mode != 2); }
void forkSmall(vb_handle h, int mode, double* gOut) {
  if (!smallHere(h, mode)) return;
  (void)hipEventRecord(h->evFork, h->st);
  (void)hipStreamWaitEvent(h->st2, h->evFork, 0);
  launch_small(h->d, mode, gOut, h->st2);
  (void)hipEventRecord(h->evJoin, h->st2);
}
void joinSmall(vb_handle h) {
  if (h->isRoot || h->partSet) (void)hipStreamWaitEvent(h->st, h->evJoin, 0);
}

// visual kernels over this shard's observations (+ the root's constant-point observations)
void visualLinShard(vb_handle h, const Dev& d, int updateCache, int dontRetry) {
  profBegin(h, KF_VISUAL_LIN);
  launch_visual_lin(d, updateCache, dontRetry, d.obB, d.obE, h->st);
  launch_visual_lin(d, updateCache, dontRetry, d.fB, d.fE, h->st);
  profEnd(h, KF_VISUAL_LIN);
  launch_fold_red(d, h->st);
}
void visualCostShard(vb_handle h, int comparable) {
  const Dev& d = h->d;
  profBegin(h, KF_VISUAL_COST);
  launch_visual_cost(d, comparable, d.obB, d.obE, h->st);
  launch_visual_cost(d, comparable, d.fB, d.fE, h->st);
  profEnd(h, KF_VISUAL_COST);
  launch_fold_red(d, h->st);
}

// vb_damp_factor_solve's forward solve runs inside the factorization (potrf_forward / trsm_kernel)
bool fwdFused(vb_handle h) { return !h->partSet && !h->sharded; }

void factorSeq(vb_handle h, const Sched& S) {
  Dev& d = h->d;
  // the forward solve of rhsWork into yvec, fused (schedule 0 of a single handle only)
  const bool fwd = fwdFused(h) && &S == &h->sch[0] && !h->factorOnly;
  double* fb = fwd ? h->rhsWork : nullptr;
  double* fy = fwd ? h->yvec : nullptr;
  for (int32_t L = 0; L < S.nLevels; L++) {
    const int64_t p0 = S.lvP[L], t0 = S.lvT[L], u0 = S.lvU[L];
    profBegin(h, KF_GEMM);
    launch_fanin(d, S.updD + 4 * u0, S.fanPairsD, (int)(S.lvU[L + 1] - u0), h->st);
    profEnd(h, KF_GEMM);
    if (S.lvPF[L + 1] > S.lvPF[L]) {  // potrf + trsm in one launch
      profBegin(h, KF_POTRF);
      launch_potrf_trsm(d, S.ptfD + 5 * S.lvPF[L], (int)(S.lvPF[L + 1] - S.lvPF[L]), h->lscr, h->dinv, h->st, fb, fy);
      profEnd(h, KF_POTRF);
      continue;
    }
    profBegin(h, KF_POTRF);
    launch_potrf(d, S.potrfTileD + p0, S.potrfColD + p0, (int)(S.lvP[L + 1] - p0), h->dinv, h->st, fb, fy);
    profEnd(h, KF_POTRF);
    profBegin(h, KF_TRSM);
    launch_trsm(d, S.trsmDiagD + t0, S.trsmTargetD + t0, S.trsmColD + t0, (int)(S.lvT[L + 1] - t0), h->dinv, h->st,
                S.trsmRowD + t0, fy, fb);
    profEnd(h, KF_TRSM);
  }
  if (S.nPtfDiag) launch_copy_diag(d, S.ptfDiagD, (int)S.nPtfDiag, h->lscr, h->st);
  launch_diag_inverse(d, S.potrfColD, S.lvP[S.nLevels], h->linv, h->st);
}

// the two-column supernode schedule (SnSched): per segment (a level of one stream) the fan-in of its
// targets, the supernodes' diagonal blocks, their rows; then the diagonal-tile inverses of the solves
// (every column).  Streams (nGroups > 1): stream g on snStream(g), forked from the main stream and joined
// back at the end; segments queued level by level, a segment after the streams it depends on (segDep)
// record their progress (one event per stream and level: everything they have queued so far is of
// earlier levels).  A profiled factor family runs the same schedule, eagerly (per-launch events).
}  // namespace viba_host
namespace viba_host {
void factorSeqSn(vb_handle h, int which) {
  Dev& d = h->d;
  const SnSched& S = h->sn[which];
  const bool fwd = fwdFused(h) && which == 0 && !h->factorOnly;
  double* fb = fwd ? h->rhsWork : nullptr;
  double* fy = fwd ? h->yvec : nullptr;
  const bool forked = S.nGroups > 1;
  const int G = forked ? S.nGroups : 1;
  auto stOf = [&](int g) -> hipStream_t {
    if (!forked) return h->st;
    return g == 0 ? h->st : g == 1 ? h->st2 : g == 2 ? h->stZ : h->stF;
  };
  if (forked) {
    (void)hipEventRecord(h->evSnFork, h->st);
    for (int g = 1; g < G; g++) (void)hipStreamWaitEvent(stOf(g), h->evSnFork, 0);
  }
  const int nSeg = (int)S.segG.size();
  // the top separators' chain: the trailing run of levels with one segment each
  int chain0 = 0;
  for (int i = 1; i < nSeg; i++)
    if (S.segL[i] == S.segL[i - 1]) chain0 = i + 1;
  // (on a stream the schedule leaves free: stZ at G = 2, stF at G = 3; stZ then waits for it, evClrDone)
  const bool clearHere = h->clearWanted && which == 0 && (S.nGroups == 2 || S.nGroups == 3) && !h->factorOnly;
  hipStream_t cs = S.nGroups == 2 ? h->stZ : h->stF;
  // the diagonal-tile inverses of the columns factored before the chain, on the same free stream while the
  // chain runs (a few latency-bound waves per level: the chip has room), instead of after the join
  const bool invEarly = which == 0 && (S.nGroups == 2 || S.nGroups == 3) && S.nInvEarly > 0 && chain0 > 0;
  bool invQueued = false;
  for (int i0 = 0; i0 < nSeg;) {
    int i1 = i0;
    while (i1 < nSeg && S.segL[i1] == S.segL[i0]) i1++;
    if (invEarly && i0 == chain0) {  // every stream's levels so far are done: the tiles before the chain are final
      for (int q = 0; q < G; q++) {
        (void)hipEventRecord(h->evInvAt[q], stOf(q));
        (void)hipStreamWaitEvent(cs, h->evInvAt[q], 0);
      }
      launch_diag_inverse(d, S.invEarlyD, S.nInvEarly, h->linv, cs);
      (void)hipEventRecord(h->evInvDone, cs);
      invQueued = true;
    }
    if (clearHere && i0 == chain0) {  // vb_optimize's clear of the spare tile store
      (void)hipEventRecord(h->evClr, stOf(S.segG[i0]));
      (void)hipStreamWaitEvent(cs, h->evClr, 0);
      if (clearReduced(h, specDev(h), cs) == 0) h->clearQueued = true;
      // (stF: specEarly makes stZ wait for it -- not here, where stZ is a factor stream the join waits for)
      h->clearOnF = cs != h->stZ;
      if (h->clearOnF) (void)hipEventRecord(h->evClrDone, cs);
      h->clearWanted = false;
    }
    if (forked) {  // the level's cross-stream dependencies, recorded before any of its launches
      uint32_t need = 0;
      for (int i = i0; i < i1; i++) need |= (uint32_t)S.segDep[i];
      for (int q = 0; q < G; q++)
        if (need >> q & 1) (void)hipEventRecord(h->evSnLvl[q], stOf(q));
    }
    for (int i = i0; i < i1; i++) {
      hipStream_t st = stOf(S.segG[i]);
      if (forked)
        for (int q = 0; q < G; q++)
          if ((uint32_t)S.segDep[i] >> q & 1) (void)hipStreamWaitEvent(st, h->evSnLvl[q], 0);
      const int64_t u0 = S.lvU[i], s0 = S.lvS[i], r0 = S.lvR[i];
      profBegin(h, KF_GEMM);
      launch_fanin(d, S.updD + 4 * u0, S.fanPairsD, (int)(S.lvU[i + 1] - u0), st);
      profEnd(h, KF_GEMM);
      profBegin(h, KF_POTRF);
      if (S.lvF[i + 1] > S.lvF[i])
        launch_snpotrf_trsm(d, S.fusD + 8 * S.lvF[i], (int)(S.lvF[i + 1] - S.lvF[i]), h->lscrSn, h->dinv, st, fb, fy);
      launch_snpotrf(d, S.potD + 4 * s0, (int)(S.lvS[i + 1] - s0), h->dinv, st, fb, fy);
      profEnd(h, KF_POTRF);
      profBegin(h, KF_TRSM);
      launch_sntrsm(d, S.rowD + 8 * r0, (int)(S.lvR[i + 1] - r0), h->dinv, st, fy, fb);
      profEnd(h, KF_TRSM);
    }
    i0 = i1;
  }
  if (forked)
    for (int q = 1; q < G; q++) {
      (void)hipEventRecord(h->evSnLvl[q], stOf(q));
      (void)hipStreamWaitEvent(h->st, h->evSnLvl[q], 0);
    }
  if (S.nCopy) launch_copy_diag(d, S.copyD, (int)S.nCopy, h->lscrSn, h->st);
  if (invQueued) {
    launch_diag_inverse(d, S.invLateD, S.nInvLate, h->linv, h->st);
    (void)hipStreamWaitEvent(h->st, h->evInvDone, 0);
    return;
  }
  const Sched& C = h->sch[which];
  launch_diag_inverse(d, C.potrfColD, C.lvP[C.nLevels], h->linv, h->st);
}

// launch sequences are fixed by the symbolic structure: capture them once into HIP graphs
// (unless one of their kernel families is being profiled, which needs per-launch events)
int captureGraph(vb_handle h, const Sched& S, hipGraphExec_t* out, bool sn = false, int which = 0) {
  hipGraph_t g;
  HIPCHK(hipStreamBeginCapture(h->st, hipStreamCaptureModeThreadLocal));
  if (sn) factorSeqSn(h, which);
  else factorSeq(h, S);
  HIPCHK(hipStreamEndCapture(h->st, &g));
  HIPCHK(hipGraphInstantiate(out, g, nullptr, nullptr, 0));
  HIPCHK(hipGraphDestroy(g));
  return 0;
}

// factor the columns of schedule `which` (0: all, or this rank's subtree in partition mode; 1: ROOT)
int factorReduced(vb_handle h, int which) {
  Sched& S = h->sch[which];
  if (!S.built) return fail(VB_E_STATE, "no factorization schedule here (partition root on rank 0 only)");
  const bool prof = h->profFamily == KF_POTRF || h->profFamily == KF_GEMM || h->profFamily == KF_TRSM;
  // (a profiled family runs launch by launch: its per-launch events, recorded as event nodes inside
  // a graph, cost as much as the graph saves -- measured)
  const bool sn = h->sn[which].built;
  if (!h->useGraphs || prof || h->factorOnly || (sn && h->sn[which].nGroups > 1)) {
    if (sn) factorSeqSn(h, which);
    else factorSeq(h, S);
    return 0;
  }
  hipGraphExec_t& g = sn ? h->sn[which].graph[h->tileSet] : S.graph[h->tileSet];
  if (!g)
    if (int rc = captureGraph(h, S, &g, sn, which)) return rc;
  HIPCHK(hipGraphLaunch(g, h->st));
  return 0;
}

// solves with rhsWork as right-hand side, result in xRed (schedule `which`, phases bit 0 forward,
// bit 1 backward; a partitioned backward pass takes the ROOT rows of xRed as given)
int solveReduced(vb_handle h, int which, int phases) {
  Sched& S = h->sch[which];
  if (!S.built) return fail(VB_E_STATE, "no solve schedule here (partition root on rank 0 only)");
  Dev& d = h->d;
  // one persistent workgroup per CU (every launched workgroup must be resident at once)
  profBegin(h, KF_FWD);
  launch_solve_fanout(d, S.tasksFD, S.nF, S.tasksBD, S.nB, S.expFD, S.expBD, h->colTilesD, h->colRowsD, h->rowTilesD,
                      h->rowColD, h->linv, h->rhsWork, h->yvec, d.xRed, h->solveFlags, h->numCUs, h->st, phases,
                      S.preReadyD, S.nPreReady);
  profEnd(h, KF_FWD);
  return 0;
}

// x_red (xRed) -> points of this shard (x_p = L^-T (z - Y x_c)), step = -x (which 0) or sub-step
// (which 1), and the partial model-cost dot into red[16] (x_red . g_red partial + shard points)
void backSubstitute(vb_handle h, int which) {
  Dev& d = h->d;
  const int64_t p0 = d.lmB * 3, np = (d.lmE - d.lmB) * 3;
  profBegin(h, KF_BACKSUB);
  launch_backsub(d, which, d.lmB, d.lmE, d.xRed, d.xp, h->st);
  profEnd(h, KF_BACKSUB);
  if (which == 0) {
    (void)hipMemsetAsync(d.red + 16, 0, 8 * sizeof(double), h->st);
    launch_dot(d.xRed, d.gRed, d.nRed, d.red + 16, h->st);
    launch_dot(d.xp + p0, d.gp + p0, np, d.red + 16, h->st);
  }
  launch_axpby(which ? d.subRed : d.stepRed, d.xRed, -1.0, 0.0, d.nRed, h->st);
  launch_axpby((which ? d.subPt : d.stepPt) + p0, d.xp + p0, -1.0, 0.0, np, h->st);
}

// ---------------------------------------------------------------- iterative reduced solve
// (Optimizer.cpp:232-331; pcg.hip)
bool pcgMode(vb_handle h) { return h->solverType != VB_SOLVER_DIRECT; }

// device buffers of the PCG path, on first use: the tile list of S x, the five vectors, and the
// preconditioner storage of the selected type
int pcgPrepare(vb_handle h) {
  Dev& d = h->d;
  if (h->partSet || h->sharded)
    return fail(VB_E_UNSUPPORTED, "the PCG solvers run on a single handle (no landmark shards, no partition)");
  const int64_t nPad = (int64_t)d.nT * TS;
  if (!h->symvTilesD) {
    std::vector<int32_t> tl, rc;
    for (int32_t J = 0; J < d.nT; J++)
      for (int64_t c = h->colStart[J]; c < h->colStart[J + 1]; c++)
        if (!h->tileFill[h->colTilesH[c]]) tl.push_back(h->colTilesH[c]), rc.push_back(h->colRowsH[c]), rc.push_back(J);
    h->nSymv = (int64_t)tl.size();
    if (upload(&h->symvTilesD, tl) || upload(&h->symvRCD, rc) || alloc0(&h->pcgR, nPad) || alloc0(&h->pcgZ, nPad) ||
        alloc0(&h->pcgP, nPad) || alloc0(&h->pcgAp, nPad) || alloc0(&h->pcgB, nPad))
      return VB_E_HIP;
  }
  if (h->solverType == VB_SOLVER_PCG_JACOBI && !h->jacL && alloc0(&h->jacL, nPad * 32)) return VB_E_HIP;
  if (h->solverType == VB_SOLVER_PCG_GAUSS_SEIDEL && !h->tilesGS && alloc0(&h->tilesGS, d.nTiles * TS * TS))
    return VB_E_HIP;
  if (h->solverType == VB_SOLVER_PCG_LOWER_PREC && !h->lpTiles &&
      (alloc0(&h->lpTiles, d.nTiles * TS * TS) || alloc0(&h->lpLinv, (size_t)d.nT * TS * TS) || alloc0(&h->lpT, nPad)))
    return VB_E_HIP;
  return 0;
}

// LowerPrecSolvePrecond::init (Preconditioner.h:180-218): S cast to fp32 and factored by the direct
// solver's tile schedule in fp32 (lowprec.hip); while the fp32 sum of the factor is not finite (a
// non-finite entry, or finite entries whose sum overflows), redo it from S with the diagonal raised:
// epsilon 0, then 1e-8, then x3 per attempt
int lpInit(vb_handle h) {
  Dev& d = h->d;
  const Sched& S = h->sch[0];
  const int64_t nEl = d.nTiles * TS * TS;
  float eps = 0.0f;
  for (int attempt = 0; attempt < 200; attempt++) {
    launch_lp_cast(d.tiles, h->lpTiles, nEl, h->st);
    if (eps > 0) {
      launch_lp_damp(h->lpTiles, d.tileIdx, d.nT, d.rvOff, d.rvDim, d.nRV, eps, h->st);
      eps *= 3.0f;
    } else {
      eps = 1e-8f;
    }
    for (int32_t L = 0; L < S.nLevels; L++) {
      const int64_t p0 = S.lvP[L], t0 = S.lvT[L], u0 = S.lvU[L];
      launch_lp_factor_level(h->lpTiles, S.updD + 4 * u0, (int)(S.lvU[L + 1] - u0), S.fanPairsD, S.potrfTileD + p0,
                             S.potrfColD + p0, (int)(S.lvP[L + 1] - p0), S.trsmTargetD + t0, S.trsmColD + t0,
                             (int)(S.lvT[L + 1] - t0), h->lpLinv, h->st);
    }
    // err[3]: a non-finite factor entry; err[2] (as fp32): the factor's sum (Preconditioner.h:216-218)
    HIPCHK(hipMemsetAsync(d.err + 2, 0, 2 * sizeof(int32_t), h->st));
    launch_lp_nonfinite(h->lpTiles, nEl, d.err + 3, reinterpret_cast<float*>(d.err + 2), h->st);
    int32_t w[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(w, d.err + 2, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, h->st));
    HIPCHK(hipStreamSynchronize(h->st));
    float sum;
    std::memcpy(&sum, &w[0], sizeof(float));
    if (!w[1] && std::isfinite(sum)) return 0;
  }
  return fail(VB_E_NUMERIC, "LowerPrecSolvePrecond: the fp32 factor keeps breaking down");
}

// LowerPrecSolvePrecond::operator() (Preconditioner.h:215-237): z = (L L^T)^-1 r in fp32
void lpApply(vb_handle h, const double* r, double* z) {
  Dev& d = h->d;
  const Sched& S = h->sch[0];
  const int64_t n = (int64_t)d.nT * TS;
  launch_lp_cast(r, h->lpT, n, h->st);
  for (int32_t L = 0; L < S.nLevels; L++) {
    const int64_t p0 = S.lvP[L], t0 = S.lvT[L];
    launch_lp_fwd_level(h->lpTiles, S.potrfColD + p0, (int)(S.lvP[L + 1] - p0), S.trsmTargetD + t0, S.trsmColD + t0,
                        S.trsmRowD + t0, (int)(S.lvT[L + 1] - t0), h->lpLinv, h->lpT, h->st);
  }
  for (int32_t L = S.nLevels - 1; L >= 0; L--) {
    const int64_t p0 = S.lvP[L];
    launch_lp_bwd_level(h->lpTiles, h->colStartD, h->colTilesD, h->colRowsD, S.potrfColD + p0, (int)(S.lvP[L + 1] - p0),
                        h->lpLinv, h->lpT, h->st);
  }
  launch_lp_uncast(h->lpT, z, n, h->st);
}

// Preconditioner::init on the assembled (damped) S
int precondInit(vb_handle h) {
  Dev& d = h->d;
  if (int rc = pcgPrepare(h)) return rc;
  if (h->solverType == VB_SOLVER_PCG_JACOBI) {
    launch_jacobi_init(d, h->jacL, h->st);
  } else if (h->solverType == VB_SOLVER_PCG_GAUSS_SEIDEL) {
    // pseudo-factor (BaSpaCho pseudoFactorFrom, Preconditioner.h:125-133): every diagonal tile
    // factored, every off-diagonal tile times L_JJ^-T, no Schur updates -- so all columns at once
    HIPCHK(hipMemcpyAsync(h->tilesGS, d.tiles, (size_t)d.nTiles * TS * TS * sizeof(double), hipMemcpyDeviceToDevice,
                          h->st));
    Dev g = d;
    g.tiles = h->tilesGS;
    const Sched& S = h->sch[0];
    launch_potrf(g, S.potrfTileD, S.potrfColD, (int)S.lvP[S.nLevels], h->dinv, h->st);
    launch_trsm(g, S.trsmDiagD, S.trsmTargetD, S.trsmColD, (int)S.lvT[S.nLevels], h->dinv, h->st);
    launch_diag_inverse(g, S.potrfColD, S.lvP[S.nLevels], h->linv, h->st);
  } else if (h->solverType == VB_SOLVER_PCG_LOWER_PREC) {
    return lpInit(h);
  }
  return 0;
}

// z = M^-1 r (Preconditioner::operator())
int precondApply(vb_handle h, const double* r, double* z) {
  Dev& d = h->d;
  const size_t bytes = (size_t)d.nT * TS * sizeof(double);
  if (h->solverType == VB_SOLVER_PCG_GAUSS_SEIDEL) {
    HIPCHK(hipMemcpyAsync(h->pcgB, r, bytes, hipMemcpyDeviceToDevice, h->st));
    Dev g = d;
    g.tiles = h->tilesGS;
    const Sched& S = h->sch[0];
    launch_solve_fanout(g, S.tasksFD, S.nF, S.tasksBD, S.nB, S.expFD, S.expBD, h->colTilesD, h->colRowsD, h->rowTilesD,
                        h->rowColD, h->linv, h->pcgB, h->yvec, z, h->solveFlags, h->numCUs, h->st, 3,
                        nullptr, 0);
    return 0;
  }
  if (h->solverType == VB_SOLVER_PCG_LOWER_PREC) {
    lpApply(h, r, z);
    return 0;
  }
  HIPCHK(hipMemcpyAsync(z, r, bytes, hipMemcpyDeviceToDevice, h->st));
  if (h->solverType == VB_SOLVER_PCG_JACOBI) launch_jacobi_apply(d, h->jacL, r, z, h->st);
  return 0;
}

// PCG::solve (PCG.cpp:15-104): S x = rhsWork -> xRed, x_0 = 0; stops when |r_k+1| / |r_0| is below
// pcgDesiredResidual or after pcgMaxIterations products.  alpha, beta and the stop test live on the
// device (red[32] = p.Ap, red[33] = r.r, red[36 + (k & 1)] = z.r of iteration k, red[40..42] the stop
// slot, pcg.hip); the host queues kPcgBatch iterations between reads of the stop slot.  Iterations
// queued after the stop leave x, r and p alone (their products and dots are skipped or discarded).
// z = M^-1 r of the last iteration is computed before the test, one preconditioner application the
// reference does not make (it changes nothing returned).  The Gauss-Seidel preconditioner (two
// fan-out triangular solves) costs more than a host read, so it reads every iteration.
int pcgSolve(vb_handle h) {
  Dev& d = h->d;
  const int64_t n = (int64_t)d.nT * TS;
  const size_t bytes = (size_t)n * sizeof(double);
  double* x = d.xRed;
  double *r = h->pcgR, *z = h->pcgZ, *p = h->pcgP, *Ap = h->pcgAp;
  const int batch = h->solverType == VB_SOLVER_PCG_GAUSS_SEIDEL ? 1 : 8;
  HIPCHK(hipMemsetAsync(x, 0, bytes, h->st));
  HIPCHK(hipMemsetAsync(Ap, 0, bytes, h->st));
  HIPCHK(hipMemcpyAsync(r, h->rhsWork, bytes, hipMemcpyDeviceToDevice, h->st));
  if (int rc = precondApply(h, r, z)) return rc;
  HIPCHK(hipMemcpyAsync(p, z, bytes, hipMemcpyDeviceToDevice, h->st));
  HIPCHK(hipMemsetAsync(d.red + 32, 0, 12 * sizeof(double), h->st));
  launch_dot(r, r, n, d.red + 33, h->st);
  launch_dot(z, r, n, d.red + 36, h->st);
  double r02 = 0;
  if (int rc = readRed(h, &r02, 33, 1)) return rc;
  const double r0 = std::sqrt(r02);
  HIPCHK(hipMemsetAsync(d.red + 33, 0, sizeof(double), h->st));
  for (int k = 0;; k++) {
    const int zr = 36 + (k & 1), zrNew = 36 + ((k + 1) & 1);
    profBegin(h, KF_SYMV);
    launch_tile_symv(d.tiles, h->symvTilesD, h->symvRCD, h->nSymv, p, Ap, d.red + 40, h->st);
    profEnd(h, KF_SYMV);
    launch_dot(p, Ap, n, d.red + 32, h->st);
    launch_pcg_xr(x, r, p, Ap, d.red, zr, 32, n, d.red + 33, h->st);
    launch_pcg_check(d.red, r0, h->pcgTol, k, h->pcgMaxIt, zrNew, h->st);
    if (int rc = precondApply(h, r, z)) return rc;
    launch_dot(z, r, n, d.red + zrNew, h->st);
    launch_pcg_p(p, Ap, z, d.red, zrNew, zr, n, h->st);
    if ((k + 1) % batch == 0 || k + 1 >= h->pcgMaxIt) {
      double stop[3];
      if (int rc = readRed(h, stop, 40, 3)) return rc;
      if (stop[0] != 0.0) {
        h->pcgIters = (int32_t)stop[1], h->pcgRelRes = stop[2];
        return checkErr(h);
      }
      if (k + 1 >= h->pcgMaxIt) return fail(VB_E_HIP, "PCG: no stop after pcgMaxIterations");
    }
  }
}

double elapsed(hipEvent_t a, hipEvent_t b) { return profPairMs(a, b); }

}  // namespace viba_host

// ====================================================================== C ABI
extern "C" {

const char* vb_last_error(void) { return g_err.c_str(); }
int vb_factor_num_vars(int k) { return (k >= 0 && k < 14) ? kNumVars[k] : -1; }
int vb_factor_num_consts(int k) { return (k >= 0 && k < 14) ? kNumConsts[k] : -1; }

void vb_default_config(vb_config* c) {
  c->reproj_loss_radius = 1.0, c->reproj_loss_cutoff = 3.0;
  c->imu_loss_radius = INFINITY, c->imu_loss_cutoff = INFINITY;
  c->imu_calib_options = VB_IMU_OPT_ALL, c->device = 0, c->tile = 0, c->reserved = 0;
}
void vb_default_settings(vb_settings* s) {
  s->max_num_iterations = 50, s->stop_if_no_improvement_for = 3, s->distance_from_troubled_iteration = 3;
  s->max_step_factor_attempts = 2, s->try_sub_step = 1, s->verbose = 0;
  s->absolute_cost_tolerance = 1e-8, s->relative_cost_tolerance = 1e-10, s->variables_tolerance = 1e-5;
  s->damping = 1e-5, s->damping_adjust_on_fail = 2.5, s->damping_adjust_on_good_step = 0.7;
  s->damping_adjust_on_average_step = 1.5, s->damping_max = 1e8, s->damping_min = 1e-9;
  s->min_relative_cost_reduction = 0.3, s->step_factor_decrease = 0.3, s->min_step_factor_for_good = 0.7;
}

int vb_create(const vb_config* cfg, vb_handle* out) {
  if (!out) return fail(VB_E_ARG, "null output handle");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(VB_E_HIP, "no HIP device available");
  vb_config c;
  if (cfg) c = *cfg;
  else vb_default_config(&c);
  if (c.tile != 0 && c.tile != TS) return fail(VB_E_UNSUPPORTED, "only tile size 64 is built");
  if (c.device < 0 || c.device >= ndev) return fail(VB_E_ARG, "bad device ordinal");
  HIPCHK(hipSetDevice(c.device));
  vb_handle h = new vb_handle_s();
  h->cfg = c;
  if (const char* e = getenv("VIBA_SPEC_EARLY")) h->specEarly = e[0] != '0';
  if (const char* e = getenv("VIBA_COST_FUSE")) h->costFuse = e[0] != '0';
  if (const char* e = getenv("VIBA_CLEAR_IN_FACTOR")) h->clearInFactor = e[0] != '0';
  if (const char* e = getenv("VIBA_DEBUG_SPEC_FAIL")) h->specFailDebug = e[0] == '1';
  if (const char* e = getenv("VIBA_SUPERNODE")) h->useSn = e[0] == '1';
  if (const char* e = getenv("VIBA_SN_STREAMS")) h->snStreams = std::max(1, std::min(4, atoi(e)));
  {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, c.device) == hipSuccess && prop.multiProcessorCount > 0)
      h->numCUs = prop.multiProcessorCount;
  }
  HIPCHK(hipStreamCreateWithFlags(&h->st, hipStreamNonBlocking));
  HIPCHK(hipStreamCreateWithFlags(&h->st2, hipStreamNonBlocking));
  for (auto& e : h->ev) HIPCHK(hipEventCreate(&e));
  HIPCHK(hipEventCreateWithFlags(&h->evFork, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&h->evJoin, hipEventDisableTiming));
  HIPCHK(hipStreamCreateWithFlags(&h->stZ, hipStreamNonBlocking));
  HIPCHK(hipEventCreateWithFlags(&h->evZero, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&h->evSmallE, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&h->evZJoin, hipEventDisableTiming));
  HIPCHK(hipStreamCreateWithFlags(&h->stF, hipStreamNonBlocking));
  HIPCHK(hipEventCreateWithFlags(&h->evSnFork, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&h->evClr, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&h->evClrDone, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&h->evInvDone, hipEventDisableTiming));
  for (auto& e : h->evInvAt) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&h->evStep, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&h->evRs, hipEventDisableTiming));
  for (auto& e : h->evSnLvl) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  *out = h;
  return 0;
}

int vb_destroy(vb_handle h) {
  if (!h) return 0;
  hipSetDevice(h->cfg.device);
  hipStreamSynchronize(h->st);
  Dev& d = h->d;
  void* ptrs[] = {d.rvKind, d.rvHandle, d.rvDim, d.rvOff, d.rvRowEnd, d.obCostOrder, d.obPack, d.obCP, d.obPose, d.obExtr, d.obIntr, d.obVel,
                  d.obRS, d.obPt, d.obRed, d.obCol, d.obC, d.cache, d.Jt, d.lmObs, d.lmY, d.lmBlk, d.blkRed,
                  d.blkCol, d.pcRow, d.pcBlk, d.bxStart, d.bxEnt, d.Vchol, d.gp, d.z, d.xp, d.Y, d.yZero, d.gpNew, d.zNew, d.ptLm, d.oxStart, d.oxObs, d.oxSlot,
                  d.lxStart, d.lxLm, d.lxCol, d.lxChunk, d.tileWorks, d.schurRuns, d.schurTasks, d.tileEnts, d.grpStart, d.grpObs, d.grpRed, d.tileIdx, d.tiles, d.gRed, d.rhs, d.xRed, d.gRedNew, d.stepRed,
                  d.stepPt, d.subRed, d.subPt, d.lmList, d.rsOff, d.rsS, d.rsI, d.rsG, d.rsN, d.imuT, d.imuV, d.rsMid, d.rsHalf,
                  d.rsCalib, d.red, d.redS, d.err, h->colTilesD,
                  h->colRowsD, h->rowTilesD, h->rowColD, h->padRowsD, h->colStartD, h->rowStartD, h->solveFlags, h->rootTilesD, h->rootRowsD, h->rootPack, h->rowPack, h->ownRowsD, h->ownPack, h->shardTilesD, h->shardPack, (void*)h->d.colOwner, h->dinv, h->yvec,
                  h->rhsWork, h->linv, h->lscr, h->lscrSn, h->refStartD, h->refObsD, h->refPtD, h->refBackD, h->refAccD,
                  h->symvTilesD, h->symvRCD, h->pcgR, h->pcgZ, h->pcgP, h->pcgAp, h->pcgB, h->jacL, h->tilesGS, h->lpTiles, h->lpLinv, h->lpT, h->clearTilesD,
                  (void*)h->pi.src, (void*)h->pi.t, (void*)h->pi.v, (void*)h->pi.off, (void*)h->pi.noise,
                  h->tilesAlt, h->cacheAlt, h->gRedAlt, h->rsSAlt, h->rsIAlt, h->rsGAlt, h->rsNAlt};
  for (void* p : ptrs)
    if (p) hipFree(p);
  for (int k = 0; k < 9; k++) {
    if (d.var[k]) hipFree(d.var[k]);
    if (d.varBak[k]) hipFree(d.varBak[k]);
    if (d.redOf[k]) hipFree(d.redOf[k]);
  }
  for (int k = 0; k < 14; k++) {
    if (d.sf[k].vars) hipFree(d.sf[k].vars);
    if (d.sf[k].consts) hipFree(d.sf[k].consts);
  }
  {
    if (d.sJ) hipFree(d.sJ);
    if (d.sE) hipFree(d.sE);
    if (d.sMeta) hipFree(d.sMeta);
  }
  for (auto& e : h->ev) hipEventDestroy(e);
  if (h->evFork) hipEventDestroy(h->evFork);
  if (h->evJoin) hipEventDestroy(h->evJoin);
  if (h->st2) hipStreamSynchronize(h->st2), hipStreamDestroy(h->st2);
  if (h->evZero) hipEventDestroy(h->evZero);
  if (h->evSmallE) hipEventDestroy(h->evSmallE);
  if (h->evZJoin) hipEventDestroy(h->evZJoin);
  if (h->stZ) hipStreamSynchronize(h->stZ), hipStreamDestroy(h->stZ);
  if (h->stF) hipStreamSynchronize(h->stF), hipStreamDestroy(h->stF);
  if (h->evSnFork) hipEventDestroy(h->evSnFork);
  if (h->evClr) hipEventDestroy(h->evClr);
  if (h->evClrDone) hipEventDestroy(h->evClrDone);
  if (h->evInvDone) hipEventDestroy(h->evInvDone);
  for (auto& e : h->evInvAt)
    if (e) hipEventDestroy(e);
  if (h->evStep) hipEventDestroy(h->evStep);
  if (h->evRs) hipEventDestroy(h->evRs);
  for (hipEvent_t e : h->evSnLvl)
    if (e) hipEventDestroy(e);
  for (auto& e : h->profEv) hipEventDestroy(e);
  if (h->evCost) hipEventDestroy(h->evCost);
  for (auto& row : h->evS)
    for (hipEvent_t e : row)
      if (e) hipEventDestroy(e);
  if (h->stR) hipStreamSynchronize(h->stR), hipStreamDestroy(h->stR);
  if (h->hostRed) hipHostFree(h->hostRed);
  for (SnSched& N : h->sn) {
    for (void* p : {(void*)N.updD, (void*)N.fanPairsD, (void*)N.potD, (void*)N.rowD, (void*)N.fusD, (void*)N.copyD,
                    (void*)N.invEarlyD, (void*)N.invLateD})
      if (p) hipFree(p);
    for (hipGraphExec_t g : N.graph)
      if (g) hipGraphExecDestroy(g);
  }
  for (Sched& S : h->sch) {
    void* sp[] = {S.ptfD, S.ptfDiagD, S.potrfTileD, S.potrfColD, S.trsmDiagD, S.trsmTargetD, S.trsmColD, S.trsmRowD, S.updD, S.fanPairsD,
                  S.tasksFD, S.tasksBD, S.expFD, S.expBD, S.preReadyD};
    for (void* p : sp)
      if (p) hipFree(p);
    for (hipGraphExec_t g : S.graph)
      if (g) hipGraphExecDestroy(g);
  }
  hipStreamDestroy(h->st);
  delete h;
  return 0;
}

int vb_set_vars(vb_handle h, int kind, int64_t n, const double* data, const uint8_t* constant) {
  if (!h || kind < 0 || kind >= 9 || n < 0 || (n > 0 && !data)) return fail(VB_E_ARG, "bad vb_set_vars arguments");
  if (h->finalized) return fail(VB_E_STATE, "vb_set_vars after vb_finalize");
  h->data[kind].assign(data, data + n * kVarData[kind]);
  h->cst[kind].assign(n, 0);
  if (constant) std::copy(constant, constant + n, h->cst[kind].begin());
  return 0;
}

int vb_add_factors(vb_handle h, int kind, int64_t n, const int32_t* var_idx, const int32_t* ivals,
                   const double* consts) {
  if (!h || kind < 0 || kind >= 14 || n < 0 || (n > 0 && (!var_idx || !consts)))
    return fail(VB_E_ARG, "bad vb_add_factors arguments");
  if (h->finalized) return fail(VB_E_STATE, "vb_add_factors after vb_finalize");
  h->fvars[kind].insert(h->fvars[kind].end(), var_idx, var_idx + n * kNumVars[kind]);
  for (int64_t i = 0; i < n; i++) h->fint[kind].push_back(ivals ? ivals[i] : -1);
  h->fconst[kind].insert(h->fconst[kind].end(), consts, consts + n * kNumConsts[kind]);
  return 0;
}

int vb_set_rs_tables(vb_handle h, int32_t nt, const int64_t* offsets, const double* samples, const double* interp,
                     const double* gravity) {
  if (!h || nt < 0) return fail(VB_E_ARG, "bad vb_set_rs_tables arguments");
  if (h->finalized) return fail(VB_E_STATE, "vb_set_rs_tables after vb_finalize");
  if (h->rsDevice) return fail(VB_E_STATE, "vb_set_rs_tables after vb_set_rs_rigs (tables are rebuilt on the device)");
  h->nRS = nt;
  h->rsOff.assign(offsets, offsets + nt + 1);
  const int64_t ns = offsets[nt];
  h->rsS.assign(samples, samples + ns * 11);
  h->rsI.assign(interp, interp + (ns - nt) * 9);
  h->rsG.assign(gravity, gravity + nt * 3);
  for (int t = 0; t < nt; t++)
    if (offsets[t + 1] - offsets[t] < 2) return fail(VB_E_ARG, "RS table needs >= 2 samples");
  return 0;
}

int vb_set_imu_measurements(vb_handle h, int64_t n, const int64_t* timestamp_ns, const double* gyro,
                             const double* accel) {
  if (!h || n < 0 || (n && (!timestamp_ns || !gyro || !accel))) return fail(VB_E_ARG, "bad vb_set_imu_measurements arguments");
  if (h->finalized) return fail(VB_E_STATE, "vb_set_imu_measurements after vb_finalize");
  h->imuT.assign(timestamp_ns, timestamp_ns + n);
  h->imuV.resize((size_t)n * 6);
  for (int64_t i = 0; i < n; i++) {
    if (i && timestamp_ns[i] <= timestamp_ns[i - 1]) return fail(VB_E_ARG, "IMU timestamps must increase");
    for (int k = 0; k < 3; k++) h->imuV[6 * i + k] = gyro[3 * i + k], h->imuV[6 * i + 3 + k] = accel[3 * i + k];
  }
  return 0;
}

int vb_set_rs_rigs(vb_handle h, int32_t nt, const int64_t* mid_us, const int64_t* half_us, const int32_t* imu_calib,
                   int32_t gravity_var) {
  if (!h || nt < 0 || (nt && (!mid_us || !half_us || !imu_calib))) return fail(VB_E_ARG, "bad vb_set_rs_rigs arguments");
  if (h->finalized) return fail(VB_E_STATE, "vb_set_rs_rigs after vb_finalize");
  if (h->imuT.empty() && nt) return fail(VB_E_STATE, "vb_set_rs_rigs needs vb_set_imu_measurements first");
  const int64_t nCalib = (int64_t)h->data[6].size() / 32, nGrav = (int64_t)h->data[8].size() / 4;
  if (gravity_var < 0 || gravity_var >= nGrav) return fail(VB_E_ARG, "vb_set_rs_rigs: unknown gravity variable");
  for (int32_t t = 0; t < nt; t++) {
    if (imu_calib[t] < 0 || imu_calib[t] >= nCalib) return fail(VB_E_ARG, "vb_set_rs_rigs: unknown IMU calibration");
    if (half_us[t] <= 0) return fail(VB_E_ARG, "vb_set_rs_rigs: half length must be positive");
  }
  h->nRS = nt;
  h->rsMid.assign(mid_us, mid_us + nt);
  h->rsHalf.assign(half_us, half_us + nt);
  h->rsCalib.assign(imu_calib, imu_calib + nt);
  h->rsGravVar = gravity_var;
  h->rsDevice = true;
  h->rsS.clear(), h->rsI.clear(), h->rsG.clear(), h->rsOff.clear();
  return 0;
}

// enqueue the rebuild; its errors surface at the next synchronising check (checkErr reads err[1])
int rsUpdateAsync(vb_handle h, bool tables, bool preint) {
  HIPCHK(hipMemsetAsync(h->d.err + 1, 0, sizeof(int32_t), h->st));
  HIPCHK(hipEventRecord(h->ev[8], h->st));
  if (tables) launch_rs_build(h->d, h->st);
  if (preint) launch_preint(h->d, h->pi, h->st);
  HIPCHK(hipEventRecord(h->ev[9], h->st));
  h->rsTimed = true;
  return 0;
}

int vb_update_rs_tables(vb_handle h) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "vb_update_rs_tables before vb_finalize");
  if (!h->rsDevice) return fail(VB_E_STATE, "vb_update_rs_tables without vb_set_rs_rigs");
  if (int rc = rsUpdateAsync(h)) return rc;
  if (h->deferred) return 0;
  int32_t e = 0;
  HIPCHK(hipMemcpyAsync(&e, h->d.err + 1, sizeof(int32_t), hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  return checkRsErr(h, e);
}

int vb_set_imu_stream(vb_handle h, int imu, int64_t n, const int64_t* timestamp_ns, const double* gyro,
                      const double* accel) {
  if (!h || imu < 0 || n < 0 || (n && (!timestamp_ns || !gyro || !accel))) return fail(VB_E_ARG, "bad vb_set_imu_stream arguments");
  if (imu == 0) return vb_set_imu_measurements(h, n, timestamp_ns, gyro, accel);
  if (h->finalized) return fail(VB_E_STATE, "vb_set_imu_stream after vb_finalize");
  if ((int)h->piT.size() <= imu) h->piT.resize(imu + 1), h->piV.resize(imu + 1);
  std::vector<int64_t>& t = h->piT[imu];
  std::vector<double>& v = h->piV[imu];
  t.assign(timestamp_ns, timestamp_ns + n);
  v.resize((size_t)n * 6);
  for (int64_t i = 0; i < n; i++) {
    if (i && timestamp_ns[i] <= timestamp_ns[i - 1]) return fail(VB_E_ARG, "IMU timestamps must increase");
    for (int k = 0; k < 3; k++) v[6 * i + k] = gyro[3 * i + k], v[6 * i + 3 + k] = accel[3 * i + k];
  }
  return 0;
}

int vb_set_imu_noise(vb_handle h, int imu, const double* accel_var, const double* gyro_var) {
  if (!h || imu < 0 || !accel_var || !gyro_var) return fail(VB_E_ARG, "bad vb_set_imu_noise arguments");
  if (h->finalized && (h->pi.n == 0 || 6 * imu + 6 > (int)h->piNoise.size()))
    return fail(VB_E_STATE, "vb_set_imu_noise after vb_finalize for an IMU without preintegration sources");
  if ((int)h->piNoise.size() < 6 * imu + 6) {
    const size_t was = h->piNoise.size();
    h->piNoise.resize(6 * imu + 6);
    for (size_t k = was; k < h->piNoise.size(); k++) h->piNoise[k] = kDefaultImuNoise[k % 6];
  }
  for (int k = 0; k < 3; k++) h->piNoise[6 * imu + k] = accel_var[k], h->piNoise[6 * imu + 3 + k] = gyro_var[k];
  if (h->finalized) {
    HIPCHK(hipMemcpyAsync(const_cast<double*>(h->pi.noise) + 6 * imu, &h->piNoise[6 * imu], 6 * sizeof(double),
                          hipMemcpyHostToDevice, h->st));
    HIPCHK(hipStreamSynchronize(h->st));
  }
  return 0;
}

int vb_set_preint_sources(vb_handle h, int kind, int64_t n, const int32_t* imu, const int64_t* t0_us,
                          const int64_t* t1_us) {
  if (!h || kind < VB_F_IMU || kind > VB_F_IMU_SEC_SPLIT || n < 0 || (n && (!imu || !t0_us || !t1_us)))
    return fail(VB_E_ARG, "bad vb_set_preint_sources arguments (inertial kinds only)");
  if (h->finalized) return fail(VB_E_STATE, "vb_set_preint_sources after vb_finalize");
  if (n != (int64_t)h->fint[kind].size()) return fail(VB_E_ARG, "vb_set_preint_sources: one source per factor row of the kind");
  std::vector<PreintSrc> keep;
  for (const PreintSrc& p : h->piSrc)
    if (p.kind != kind) keep.push_back(p);
  for (int64_t r = 0; r < n; r++) {
    if (imu[r] < 0) return fail(VB_E_ARG, "vb_set_preint_sources: bad IMU index");
    if (t1_us[r] <= t0_us[r]) return fail(VB_E_ARG, "vb_set_preint_sources: empty interval");
    keep.push_back(PreintSrc{kind, imu[r], r, t0_us[r], t1_us[r]});
  }
  h->piSrc.swap(keep);
  return 0;
}

int vb_set_recompute_preint(vb_handle h, int on) {
  if (!h) return fail(VB_E_ARG, "null handle");
  h->recomputePreint = on != 0;
  return 0;
}

int vb_update_preintegrations(vb_handle h) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "vb_update_preintegrations before vb_finalize");
  if (h->pi.n == 0) return 0;
  if (int rc = rsUpdateAsync(h, false, true)) return rc;
  int32_t e = 0;
  HIPCHK(hipMemcpyAsync(&e, h->d.err + 1, sizeof(int32_t), hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  return checkRsErr(h, e);
}

int vb_get_factor_consts(vb_handle h, int kind, int64_t row, double* out) {
  if (!h || kind < 0 || kind >= 14 || !out || row < 0 || row >= (int64_t)h->fint[kind].size())
    return fail(VB_E_ARG, "bad vb_get_factor_consts arguments");
  if (!h->finalized || kind == VB_F_VISUAL) {
    std::copy(&h->fconst[kind][row * kNumConsts[kind]], &h->fconst[kind][(row + 1) * kNumConsts[kind]], out);
    return 0;
  }
  const SmallFactors& sf = h->d.sf[kind];
  HIPCHK(hipMemcpyAsync(out, sf.consts + row * sf.nc, kNumConsts[kind] * sizeof(double), hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  return 0;
}

int vb_refine_points(vb_handle h, double* costs, int64_t* stats) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "vb_refine_points before vb_finalize");
  Dev& d = h->d;
  if (h->partSet || d.lmB != 0 || d.lmE != d.nPts || !h->isRoot)
    return fail(VB_E_UNSUPPORTED, "vb_refine_points needs the whole problem on this handle (no shard / partition)");
  if (!h->refStartD) {
    // observations grouped by point variable (refinePoints' perPointTracks, PointRefinement.cpp:20-45),
    // in device observation order
    std::vector<int32_t> obPt(d.nObs);
    if (d.nObs) HIPCHK(hipMemcpy(obPt.data(), d.obPt, d.nObs * sizeof(int32_t), hipMemcpyDeviceToHost));
    const int64_t nP = d.nvar[0];
    std::vector<int64_t> cnt(nP + 1, 0);
    for (int32_t p : obPt) cnt[p + 1]++;
    for (int64_t p = 0; p < nP; p++) cnt[p + 1] += cnt[p];
    std::vector<int32_t> obs(d.nObs);
    std::vector<int64_t> pos(cnt.begin(), cnt.end() - 1);
    for (int64_t o = 0; o < d.nObs; o++) obs[pos[obPt[o]]++] = (int32_t)o;
    std::vector<int64_t> gs(1, 0);
    std::vector<int32_t> gp;
    for (int64_t p = 0; p < nP; p++)
      if (cnt[p + 1] > cnt[p]) gp.push_back((int32_t)p), gs.push_back(cnt[p + 1]);
    h->nRefG = (int64_t)gp.size();
    if (upload(&h->refStartD, gs) || upload(&h->refObsD, obs) || upload(&h->refPtD, gp) ||
        alloc0(&h->refBackD, (size_t)d.nObs) || alloc0(&h->refAccD, 8))
      return VB_E_HIP;
  }
  HIPCHK(hipMemsetAsync(h->refAccD, 0, 8 * sizeof(double), h->st));
  HIPCHK(hipMemsetAsync(d.err, 0, 2 * sizeof(int32_t), h->st));
  launch_refine_points(d, h->refStartD, h->refObsD, h->refPtD, h->nRefG, h->refBackD, h->refAccD, h->st);
  double acc[8];
  HIPCHK(hipMemcpyAsync(acc, h->refAccD, sizeof(acc), hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  if (int rc = checkErr(h)) return rc;
  if (costs) costs[0] = acc[0], costs[1] = acc[1];
  if (stats) stats[0] = (int64_t)acc[2], stats[1] = (int64_t)acc[3], stats[2] = (int64_t)acc[4];
  h->linearized = false, h->factored = false;
  return 0;
}

int vb_get_rs_table(vb_handle h, int32_t t, int32_t* n_samples, double* samples, double* interp) {
  if (!h || !h->finalized || !n_samples) return fail(VB_E_STATE, "vb_get_rs_table before vb_finalize");
  if (t < 0 || t >= h->nRS) return fail(VB_E_ARG, "vb_get_rs_table: bad table index");
  int32_t n = 0;
  HIPCHK(hipMemcpyAsync(&n, h->d.rsN + t, sizeof(int32_t), hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  *n_samples = n;
  const int64_t s0 = h->rsOff[t];
  if (samples && n) HIPCHK(hipMemcpy(samples, h->d.rsS + s0 * 11, (size_t)n * 11 * sizeof(double), hipMemcpyDeviceToHost));
  if (interp && n > 1)
    HIPCHK(hipMemcpy(interp, h->d.rsI + (s0 - t) * 9, (size_t)(n - 1) * 9 * sizeof(double), hipMemcpyDeviceToHost));
  return 0;
}

int vb_finalize(vb_handle h) {
  if (!h) return fail(VB_E_ARG, "null handle");
  if (h->finalized) return fail(VB_E_STATE, "already finalized");
  HIPCHK(hipSetDevice(h->cfg.device));
  return doFinalize(h);
}

int64_t vb_reduced_order(vb_handle h) { return h ? h->nRedReal : -1; }
int64_t vb_total_order(vb_handle h) { return h ? h->order : -1; }

int vb_set_landmark_shard(vb_handle h, int64_t lm_begin, int64_t lm_end, int is_root) {
  if (!h) return fail(VB_E_ARG, "null handle");
  if (h->finalized) return fail(VB_E_STATE, "vb_set_landmark_shard must precede vb_finalize");
  if (lm_begin < 0 || lm_begin > lm_end) return fail(VB_E_ARG, "bad landmark range");
  h->lmBegin = lm_begin, h->lmEnd = lm_end, h->isRoot = is_root != 0, h->sharded = true;
  return 0;
}

// the reduced system's clear on stream zs: the tiles no Schur item stores whole, the gradient, the
// padded diagonal
int clearReduced(vb_handle h, const Dev& d, hipStream_t zs) {
  if (h->clearTilesD) {
    launch_zero_tiles(d.tiles, h->clearTilesD, h->nClear, zs);
  } else if (h->zeroRuns.empty()) {
    HIPCHK(hipMemsetAsync(d.tiles, 0, (size_t)d.nTiles * TS * TS * sizeof(double), zs));
  } else {  // partitioned: colStart runs are tile-store index ranges (tiles stored column by column)
    for (const auto& r : h->zeroRuns)
      HIPCHK(hipMemsetAsync(d.tiles + r.first * TS * TS, 0, (size_t)(r.second - r.first) * TS * TS * sizeof(double), zs));
  }
  HIPCHK(hipMemsetAsync(d.gRed, 0, (size_t)d.nT * TS * sizeof(double), zs));
  if (h->isRoot || h->partSet) launch_pad_diag(d, h->padRowsD, h->nPadRows, zs);
  return 0;
}

// vb_linearize's device work over the buffers of `d` (h->d, or the speculative copy of vb_optimize:
// another tile store, cache write buffer, reduction and error slots), no host read, no reset of the
// reduction / error slots (the caller's); events evA / evB bracket it.  early: the small factors'
// evaluation and the clear were queued on stZ already (specEarly)
int linearizeBody(vb_handle h, const Dev& d, int update_cache, int dont_retry_failed, hipEvent_t evA, hipEvent_t evB,
                  bool early = false) {
  const bool fuseCost = d.costS != nullptr;
  HIPCHK(hipEventRecord(evA, h->st));
  // the reduced system is cleared and the small factors assembled on the side stream while the visual
  // factors linearize on the main stream (they write only their records and the cost)
  const bool side = smallHere(h, 0);
  hipStream_t zs = side ? h->stZ : h->st;
  if (side && !early) {
    HIPCHK(hipEventRecord(h->evFork, h->st));
    HIPCHK(hipStreamWaitEvent(h->st2, h->evFork, 0));
    HIPCHK(hipStreamWaitEvent(h->stZ, h->evFork, 0));
    launch_small_eval(d, 0, d.gRed, h->st2);
  }
  if (!early)
    if (int rc = clearReduced(h, d, zs)) return rc;
  if (side && early) {
    // evaluation and clear done in order on stZ: the IMU kinds' assembly on st2 waits for both
    HIPCHK(hipEventRecord(h->evZero, h->stZ));
    HIPCHK(hipStreamWaitEvent(h->st2, h->evZero, 0));
    launch_small_assemble(d, 0, d.gRed, h->st2, 1);
    launch_small_assemble(d, 0, d.gRed, h->stZ, 2);
    HIPCHK(hipEventRecord(h->evJoin, h->st2));
    HIPCHK(hipEventRecord(h->evZJoin, h->stZ));
  } else if (side) {
    // the IMU kinds' assembly on st2, the other kinds' on stZ after the clear: both wait for the clear
    // and the evaluation
    HIPCHK(hipEventRecord(h->evZero, h->stZ));
    HIPCHK(hipEventRecord(h->evSmallE, h->st2));
    HIPCHK(hipStreamWaitEvent(h->st2, h->evZero, 0));
    HIPCHK(hipStreamWaitEvent(h->stZ, h->evSmallE, 0));
    launch_small_assemble(d, 0, d.gRed, h->st2, 1);
    launch_small_assemble(d, 0, d.gRed, h->stZ, 2);
    HIPCHK(hipEventRecord(h->evJoin, h->st2));
    HIPCHK(hipEventRecord(h->evZJoin, h->stZ));
  }
  visualLinShard(h, d, update_cache, dont_retry_failed);
  if (fuseCost) {  // the rest of vb_optimize's cost pass (costFusedEnqueue): its sums into red[1..4]
    launch_fold_red(h->d, h->st);
    HIPCHK(hipEventRecord(h->ev[7], h->st));
    HIPCHK(hipEventRecord(h->evCost, h->st));
    h->profAtCost = h->profUsed;
  }
  joinSmall(h);
  if (side) HIPCHK(hipStreamWaitEvent(h->st, h->evZJoin, 0));
  HIPCHK(hipEventRecord(evB, h->st));
  return 0;
}
// cost in red[0], errors in err
int linearizeEnqueue(vb_handle h, int update_cache, int dont_retry_failed) {
  Dev& d = h->d;
  HIPCHK(hipMemsetAsync(d.red, 0, 64 * sizeof(double), h->st));
  HIPCHK(hipMemsetAsync(d.err, 0, sizeof(int32_t), h->st));
  return linearizeBody(h, d, update_cache, dont_retry_failed, h->ev[0], h->ev[1]);
}

int vb_linearize(vb_handle h, int update_cache, int dont_retry_failed, double* cost) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "vb_linearize before vb_finalize");
  if (int rc = linearizeEnqueue(h, update_cache, dont_retry_failed)) return rc;
  h->scalarsMarked = false;
  if (h->deferred) {  // cost in red[0]
    if (cost) *cost = std::nan("");
    h->linearized = true, h->factored = false;
    return 0;
  }
  double c = 0;
  if (int rc = readRed(h, &c, 0, 1)) return rc;
  if (int rc = checkErr(h)) return rc;
  h->times.linearize_ms = elapsed(h->ev[0], h->ev[1]);
  if (h->rsTimed) h->times.rs_update_ms = elapsed(h->ev[8], h->ev[9]), h->rsTimed = false;
  if (cost) *cost = c;
  h->linearized = true, h->factored = false;
  return 0;
}

// damp + eliminate the landmarks (of this shard) into the reduced system and its RHS: the observation-
// group Gram blocks on the side stream beside the landmark elimination (both stream records from HBM;
// neither reads what the other writes), joined before the tile products
int assembleEnqueue(vb_handle h, double lambda) {
  Dev& d = h->d;
  const int addId = (h->isRoot || h->partSet) ? 1 : 0;
  launch_damp(d, lambda, addId, h->st);
  HIPCHK(hipEventRecord(h->evFork, h->st));
  HIPCHK(hipStreamWaitEvent(h->st2, h->evFork, 0));
  launch_groups(d, lambda, h->st2);
  HIPCHK(hipEventRecord(h->evJoin, h->st2));
  profBegin(h, KF_LANDMARK);
  launch_landmark(d, lambda, 0, d.lmB, d.lmE, h->st);
  profEnd(h, KF_LANDMARK);
  HIPCHK(hipMemsetAsync(d.rhs, 0, (size_t)d.nT * TS * sizeof(double), h->st));
  HIPCHK(hipStreamWaitEvent(h->st, h->evJoin, 0));
  profBegin(h, KF_SCHUR);
  launch_schur_products(d, lambda, h->st);
  profEnd(h, KF_SCHUR);
  return 0;
}

// vb_damp_factor_solve's device work (model dot in red[16]); clearErr = false keeps the linearization's
// error bits for one check at the end of the iteration (vb_optimize)
int dampFactorSolveEnqueue(vb_handle h, double lambda, bool clearErr) {
  Dev& d = h->d;
  if (clearErr) HIPCHK(hipMemsetAsync(d.err, 0, sizeof(int32_t), h->st));
  HIPCHK(hipEventRecord(h->ev[2], h->st));
  if (int rc = assembleEnqueue(h, lambda)) return rc;
  HIPCHK(hipEventRecord(h->ev[3], h->st));
  const bool fused = !pcgMode(h) && fwdFused(h);
  if (fused)  // the factorization runs the forward solve of rhsWork (into yvec)
    HIPCHK(hipMemcpyAsync(h->rhsWork, d.rhs, (size_t)d.nT * TS * sizeof(double), hipMemcpyDeviceToDevice, h->st));
  if (pcgMode(h)) {
    if (int rc = precondInit(h)) return rc;
  } else if (int rc = factorReduced(h)) {
    return rc;
  }
  HIPCHK(hipEventRecord(h->ev[4], h->st));
  if (!fused)
    HIPCHK(hipMemcpyAsync(h->rhsWork, d.rhs, (size_t)d.nT * TS * sizeof(double), hipMemcpyDeviceToDevice, h->st));
  if (pcgMode(h)) {
    if (int rc = pcgSolve(h)) return rc;
  } else if (int rc = solveReduced(h, 0, fused ? 2 : 3)) {
    return rc;
  }
  backSubstitute(h, 0);
  HIPCHK(hipEventRecord(h->ev[5], h->st));
  return 0;
}

int vb_damp_factor_solve(vb_handle h, double lambda, double* model_cost_reduction) {
  if (!h || !h->linearized) return fail(VB_E_STATE, "vb_damp_factor_solve needs a fresh vb_linearize");
  if (int rc = dampFactorSolveEnqueue(h, lambda, true)) return rc;
  double dotv = 0;
  if (int rc = readRed(h, &dotv, 16, 1)) return rc;
  if (int rc = checkErr(h)) return rc;
  h->times.schur_ms = elapsed(h->ev[2], h->ev[3]);
  h->times.factor_ms = elapsed(h->ev[3], h->ev[4]);
  h->times.solve_ms = elapsed(h->ev[4], h->ev[5]);
  if (model_cost_reduction) *model_cost_reduction = 0.5 * dotv;
  h->linearized = false, h->factored = true;
  return 0;
}

int vb_gradient_dot_step(vb_handle h, int dont_retry_failed, double* back_red) {
  if (!h || !h->factored) return fail(VB_E_STATE, "vb_gradient_dot_step needs a factorization");
  Dev& d = h->d;
  HIPCHK(hipMemsetAsync(d.err, 0, sizeof(int32_t), h->st));
  HIPCHK(hipMemsetAsync(d.gRedNew, 0, (size_t)d.nT * TS * sizeof(double), h->st));
  HIPCHK(hipMemsetAsync(d.red, 0, 1 * sizeof(double), h->st));
  forkSmall(h, 1, d.gRedNew);
  visualLinShard(h, h->d, 0, dont_retry_failed);
  joinSmall(h);
  launch_landmark(d, 0.0, 1, d.lmB, d.lmE, h->st);
  launch_reduced_grad(d, 0, h->st);
  HIPCHK(hipMemsetAsync(d.red + 16, 0, 8 * sizeof(double), h->st));
  launch_dot(d.gRedNew, d.stepRed, d.nRed, d.red + 16, h->st);
  launch_dot(d.gpNew + d.lmB * 3, d.stepPt + d.lmB * 3, (d.lmE - d.lmB) * 3, d.red + 16, h->st);
  double dotv = 0;
  if (int rc = readRed(h, &dotv, 16, 1)) return rc;
  if (int rc = checkErr(h)) return rc;
  if (back_red) *back_red = -0.5 * dotv;
  return 0;
}

int vb_solve_with_new_gradient(vb_handle h) {
  if (!h || !h->factored) return fail(VB_E_STATE, "vb_solve_with_new_gradient needs a factorization");
  Dev& d = h->d;
  launch_landmark(d, 0.0, 2, d.lmB, d.lmE, h->st);
  launch_reduced_grad(d, 1, h->st);
  HIPCHK(hipMemcpyAsync(h->rhsWork, d.rhs, (size_t)d.nT * TS * sizeof(double), hipMemcpyDeviceToDevice, h->st));
  if (pcgMode(h)) {
    if (int rc = pcgSolve(h)) return rc;
  } else if (int rc = solveReduced(h)) {
    return rc;
  }
  backSubstitute(h, 1);
  HIPCHK(hipStreamSynchronize(h->st));
  return checkErr(h);
}

int vb_set_solver(vb_handle h, int solver_type, int pcg_max_iterations, double pcg_desired_residual) {
  if (!h) return fail(VB_E_ARG, "null handle");
  if (solver_type < VB_SOLVER_DIRECT || solver_type > VB_SOLVER_PCG_LOWER_PREC) return fail(VB_E_ARG, "unknown solver type");
  if (solver_type != VB_SOLVER_DIRECT && (h->partSet || h->sharded))
    return fail(VB_E_UNSUPPORTED, "the PCG solvers run on a single handle (no landmark shards, no partition)");
  if (pcg_max_iterations < 1) return fail(VB_E_ARG, "pcg_max_iterations must be >= 1");
  h->solverType = solver_type, h->pcgMaxIt = pcg_max_iterations, h->pcgTol = pcg_desired_residual;
  return 0;
}
int vb_reduced_layout(vb_handle h, int32_t* kinds, int32_t* handles, int64_t* offsets, int64_t* n, int64_t* padded_order) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "vb_reduced_layout before vb_finalize");
  const int64_t nRV = (int64_t)h->rvKind.size();
  if (n) *n = nRV;
  if (padded_order) *padded_order = (int64_t)h->d.nT * TS;
  for (int64_t i = 0; i < nRV; i++) {
    if (kinds) kinds[i] = h->rvKind[i];
    if (handles) handles[i] = h->rvHandle[i];
    if (offsets) offsets[i] = h->rvOff[i];
  }
  return 0;
}
// Selected inversion (selinv.hip) of the factored tiles: afterwards the tile store holds Z = S^-1 on
// the pattern of L (the factor is consumed).  Levels as the factorization's schedule (a column's level
// is one more than those of the columns its row depends on), run from the last to the first.
int vb_debug_negate_model_reduction(vb_handle h, int iteration) {
  if (!h) return fail(VB_E_ARG, "null handle");
  h->faultNegModelRedIt = iteration;
  return 0;
}
int vb_debug_fail_iteration(vb_handle h, int iteration) {
  if (!h) return fail(VB_E_ARG, "null handle");
  h->faultFailIt = iteration;
  return 0;
}
// slot of tile (I, J) of the reduced tile store (vb_reduced_buffers), -1 when it is not stored
int vb_debug_tile_slot(vb_handle h, int32_t I, int32_t J, int64_t* slot) {
  if (!h || !h->finalized || !slot) return fail(VB_E_STATE, "vb_debug_tile_slot before vb_finalize");
  *slot = -1;
  if (I < J || J < 0 || I >= h->d.nT) return 0;
  for (int64_t c = h->colStart[J]; c < h->colStart[J + 1]; c++)
    if (h->colRowsH[c] == I) *slot = h->colTilesH[c];
  return 0;
}
int vb_pcg_stats(vb_handle h, int32_t* iterations, double* relative_residual) {
  if (!h) return fail(VB_E_ARG, "null handle");
  if (iterations) *iterations = h->pcgIters;
  if (relative_residual) *relative_residual = h->pcgRelRes;
  return 0;
}

int vb_scale_step(vb_handle h, double f) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "not finalized");
  launch_axpby(h->d.stepRed, h->d.stepRed, 0.0, f, h->d.nRed, h->st);
  launch_axpby(h->d.stepPt, h->d.stepPt, 0.0, f, h->d.nPts * 3, h->st);
  return 0;
}

// box-plus of the step (red[8..10]: the raw step ratios), bracketed by events e0 / e1
int applyStepEnqueue(vb_handle h, int which, int e0, int e1) {
  Dev& d = h->d;
  HIPCHK(hipEventRecord(h->ev[e0], h->st));
  HIPCHK(hipMemsetAsync(d.red + 8, 0, 3 * sizeof(double), h->st));
  launch_boxplus(d, which ? d.subRed : d.stepRed, which ? d.subPt : d.stepPt, h->st);
  HIPCHK(hipEventRecord(h->ev[e1], h->st));
  return 0;
}
int vb_apply_step_raw(vb_handle h, int which, double raw[3]) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "not finalized");
  if (int rc = applyStepEnqueue(h, which, 10, 11)) return rc;
  if (h->deferred) {  // raw ratios in red[8..10]
    if (raw) raw[0] = raw[1] = raw[2] = std::nan("");
    return 0;
  }
  double r[3];
  if (int rc = readRed(h, r, 8, 3)) return rc;
  h->times.step_ms = elapsed(h->ev[10], h->ev[11]);
  if (raw) raw[0] = r[0], raw[1] = r[1], raw[2] = r[2];
  return 0;
}
int vb_apply_step(vb_handle h, int which, double ratios[3]) {
  double r[3];
  if (int rc = vb_apply_step_raw(h, which, r)) return rc;
  const double n = (double)std::max<int64_t>(1, h->nParams);
  if (ratios) ratios[0] = r[0], ratios[1] = std::sqrt(r[1] / n), ratios[2] = r[2] / n;
  return 0;
}
int64_t vb_num_params(vb_handle h) { return h ? h->nParams : -1; }

// the cost pass (red[1..4]: cost and CostStats), bracketed by ev[6] / ev[7]
int costEnqueue(vb_handle h, int comparable, bool clearErr) {
  Dev& d = h->d;
  HIPCHK(hipEventRecord(h->ev[6], h->st));
  HIPCHK(hipMemsetAsync(d.red + 1, 0, 4 * sizeof(double), h->st));
  if (clearErr) HIPCHK(hipMemsetAsync(d.err, 0, sizeof(int32_t), h->st));
  forkSmall(h, 2, nullptr);
  visualCostShard(h, comparable);
  joinSmall(h);
  HIPCHK(hipEventRecord(h->ev[7], h->st));
  return 0;
}
// vb_optimize's cost pass with the global-shutter observations folded into the speculative
// linearization queued next (specEnqueue with fuseCost: visual_lin_kernel<true>, then the fold and
// ev[7] / evCost): here only the small factors and the rolling-shutter observations, evaluated with the
// iteration's tables while the rebuild for the next one runs on stF
int costFusedEnqueue(vb_handle h) {
  Dev& d = h->d;
  HIPCHK(hipEventRecord(h->ev[6], h->st));
  HIPCHK(hipMemsetAsync(d.red + 1, 0, 4 * sizeof(double), h->st));
  forkSmall(h, 2, nullptr);
  profBegin(h, KF_VISUAL_COST);
  launch_visual_cost(d, 1, h->costRsB[0], d.obE, h->st);
  launch_visual_cost(d, 1, h->costRsB[1], d.fE, h->st);
  profEnd(h, KF_VISUAL_COST);
  joinSmall(h);
  return 0;
}
void costStats(vb_handle h, const double* r, double* cost, vb_cost_stats* stats) {
  int64_t nSmall = 0;
  if (h->isRoot)
    for (int k = 1; k < 14; k++) nSmall += h->d.sf[k].n;
  if (cost) *cost = r[0];
  if (stats) stats->num_total = (int64_t)std::llround(r[1]) + nSmall, stats->num_invalid = std::llround(r[2]),
             stats->num_prev_invalid = std::llround(r[3]);
}
int vb_cost(vb_handle h, int comparable, double* cost, vb_cost_stats* stats) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "not finalized");
  if (int rc = costEnqueue(h, comparable, !h->deferred)) return rc;
  if (h->deferred) {  // cost and CostStats in red[1..4] (vb_small_factor_count: the root's addition)
    if (cost) *cost = std::nan("");
    return 0;
  }
  double r[4];
  if (int rc = readRed(h, r, 1, 4)) return rc;
  if (int rc = checkErr(h)) return rc;
  h->times.cost_ms = elapsed(h->ev[6], h->ev[7]);
  costStats(h, r, cost, stats);
  return 0;
}

int vb_backup(vb_handle h) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "not finalized");
  int64_t len[9];
  for (int k = 0; k < 9; k++) len[k] = (int64_t)h->data[k].size();
  launch_copy_vars(h->d, true, len, h->st);
  return 0;
}
int vb_restore(vb_handle h) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "not finalized");
  int64_t len[9];
  for (int k = 0; k < 9; k++) len[k] = (int64_t)h->data[k].size();
  launch_copy_vars(h->d, false, len, h->st);
  return 0;
}

int vb_get_vars(vb_handle h, int kind, double* out) {
  if (!h || kind < 0 || kind >= 9 || !out) return fail(VB_E_ARG, "bad vb_get_vars arguments");
  if (!h->finalized) {
    std::copy(h->data[kind].begin(), h->data[kind].end(), out);
    return 0;
  }
  HIPCHK(hipMemcpyAsync(out, h->d.var[kind], h->data[kind].size() * sizeof(double), hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  return 0;
}

static int getPerKind(vb_handle h, const double* red, const double* pt, int kind, double* out) {
  Dev& d = h->d;
  const int64_t n = d.nvar[kind];
  const int md = kMaxTan[kind];
  std::fill(out, out + n * md, 0.0);
  if (kind == 0) {
    std::vector<double> v(d.nPts * 3);
    if (!v.empty()) HIPCHK(hipMemcpyAsync(v.data(), pt, v.size() * sizeof(double), hipMemcpyDeviceToHost, h->st));
    HIPCHK(hipStreamSynchronize(h->st));
    for (int64_t p = 0; p < n; p++) {
      const int l = h->lmOfPoint[p];
      if (l >= 0) std::copy(&v[l * 3], &v[l * 3] + 3, out + p * 3);
    }
    return 0;
  }
  std::vector<double> v(d.nRed);
  if (!v.empty()) HIPCHK(hipMemcpyAsync(v.data(), red, v.size() * sizeof(double), hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  for (int i = 0; i < d.nRV; i++)
    if (h->rvKind[i] == kind) std::copy(&v[h->rvOff[i]], &v[h->rvOff[i]] + h->rvDim[i], out + (int64_t)h->rvHandle[i] * md);
  return 0;
}

int vb_get_step(vb_handle h, int which, int kind, double* out) {
  if (!h || !h->finalized || kind < 0 || kind >= 9 || !out) return fail(VB_E_ARG, "bad vb_get_step arguments");
  return getPerKind(h, which ? h->d.subRed : h->d.stepRed, which ? h->d.subPt : h->d.stepPt, kind, out);
}
// The visual part of the gradient is assembled inside the Schur pass (vb_damp_factor_solve); before
// that, assemble it on demand into the gradient-only buffers (same kernels as gradient_dot_step).
int vb_get_gradient(vb_handle h, int kind, double* out) {
  if (!h || !h->finalized || kind < 0 || kind >= 9 || !out) return fail(VB_E_ARG, "bad vb_get_gradient arguments");
  if (h->linearized) {
    Dev& d = h->d;
    HIPCHK(hipMemsetAsync(d.gRedNew, 0, (size_t)d.nT * TS * sizeof(double), h->st));
    if (smallHere(h, 1)) launch_small(d, 1, d.gRedNew, h->st);
    launch_landmark(d, 0.0, 1, d.lmB, d.lmE, h->st);
    launch_reduced_grad(d, 0, h->st);
    return getPerKind(h, d.gRedNew, d.gpNew, kind, out);
  }
  return getPerKind(h, h->d.gRed, h->d.gp, kind, out);
}

int vb_last_phase_times(vb_handle h, vb_phase_times* out) {
  if (!h || !out) return fail(VB_E_ARG, "null argument");
  *out = h->times;
  return 0;
}

void* vb_stream(vb_handle h) { return h ? (void*)h->st : nullptr; }

int vb_profile_kernel(vb_handle h, int family) {
  if (!h || family < -1 || family >= KF_COUNT) return fail(VB_E_ARG, "bad kernel family");
  profHarvest(h);
  h->profFamily = family, h->profLaunches = 0, h->profMs = 0.0, h->profBusyMs = 0.0, h->profUsed = 0, h->profDone = 0;
  return 0;
}
int vb_kernel_time(vb_handle h, int64_t* launches, double* total_ms) {
  if (!h) return fail(VB_E_ARG, "null handle");
  profHarvest(h);
  if (launches) *launches = h->profLaunches;
  if (total_ms) *total_ms = h->profMs;
  return 0;
}
int vb_kernel_busy_time(vb_handle h, double* busy_ms) {
  if (!h || !busy_ms) return fail(VB_E_ARG, "null argument");
  profHarvest(h);
  *busy_ms = h->profBusyMs;
  return 0;
}
int vb_problem_stats(vb_handle h, int64_t* out) {  // 12 entries
  if (!h || !h->finalized || !out) return fail(VB_E_STATE, "not finalized");
  const Dev& d = h->d;
  out[0] = d.nObs, out[1] = d.nPts, out[2] = d.nRV, out[3] = d.nRed, out[4] = d.nT, out[5] = d.nTiles;
  out[6] = h->nPairs;
  int64_t sm = 0;
  for (int k = 1; k < 14; k++) sm += d.sf[k].n;
  out[7] = sm;
  // Schur work-list sizes: landmark-pair entries, observation-pair entries
  out[8] = h->nTileEnt, out[9] = h->nObEnt;
  // levels of the tile Cholesky (fan-in launches per factorization); tiles of S itself (the stored
  // tiles less the symbolic fill: what the PCG product reads)
  int64_t nS = 0;
  for (uint8_t f : h->tileFill) nS += f ? 0 : 1;
  out[10] = h->nLevels, out[11] = nS;
  return 0;
}

// the factorization's schedule as it runs: [levels, fan-in contributions per factorization, supernodes,
// two-column supernodes] (the column schedule: supernodes = columns, no two-column ones)
int vb_factor_schedule_stats(vb_handle h, int64_t* out4) {
  if (!h || !h->finalized || !out4) return fail(VB_E_STATE, "not finalized");
  if (h->sn[0].built) {
    const SnSched& N = h->sn[0];
    out4[0] = N.nLevels, out4[1] = N.nPairs, out4[2] = N.nSuper, out4[3] = N.nTwo;
  } else {
    out4[0] = h->nLevels, out4[1] = h->nPairs, out4[2] = h->d.nT, out4[3] = 0;
  }
  return 0;
}

int vb_reduced_buffers(vb_handle h, double** matrix, int64_t* matrix_len, double** rhs, int64_t* rhs_len) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "not finalized");
  if (matrix) *matrix = h->d.tiles;
  if (matrix_len) *matrix_len = h->d.nTiles * TS * TS;
  if (rhs) *rhs = h->d.rhs;
  if (rhs_len) *rhs_len = (int64_t)h->d.nT * TS;
  return 0;
}

// ---- vb_optimize's speculative linearization of the next iteration (vb_handle_s::tilesAlt ..)
// Frees whatever specPrepare got before a failure (nothing has been swapped into h->d then).
void specRelease(vb_handle h) {
  for (void* p : {(void*)h->tilesAlt, (void*)h->cacheAlt, (void*)h->gRedAlt, (void*)h->rsSAlt, (void*)h->rsIAlt,
                  (void*)h->rsGAlt, (void*)h->rsNAlt})
    if (p) (void)hipFree(p);
  h->tilesAlt = h->cacheAlt = h->gRedAlt = h->rsSAlt = h->rsIAlt = h->rsGAlt = nullptr;
  h->rsNAlt = nullptr;
  for (auto& row : h->evS)
    for (hipEvent_t& e : row)
      if (e) (void)hipEventDestroy(e), e = nullptr;
  if (h->evCost) (void)hipEventDestroy(h->evCost), h->evCost = nullptr;
  if (h->stR) (void)hipStreamDestroy(h->stR), h->stR = nullptr;
  if (h->hostRed) (void)hipHostFree(h->hostRed), h->hostRed = nullptr;
  (void)hipGetLastError();
}
// The spare tile store (nTiles x 32 KB: 2.2 GB at config C), ResultCache, gradient and rolling-shutter
// tables of the speculative linearization, allocated at the first vb_optimize that speculates.  Returns
// false when any of it cannot be had: the caller then runs the plain controller (no speculation), as
// before the speculative path existed, instead of failing a problem that fits without it.
bool specPrepare(vb_handle h) {
  if (h->specReady) return true;
  Dev& d = h->d;
  bool ok = !alloc0(&h->tilesAlt, (size_t)d.nTiles * TS * TS) && !alloc0(&h->cacheAlt, d.nObs) &&
            !alloc0(&h->gRedAlt, (size_t)d.nT * TS) && !h->specFailDebug;
  if (ok && h->rsDevice) {
    const int64_t ns = h->rsOff[h->nRS];
    ok = !alloc0(&h->rsSAlt, ns * 11) && !alloc0(&h->rsIAlt, (ns - h->nRS) * 9) &&
         !alloc0(&h->rsGAlt, (size_t)h->nRS * 3) && !alloc0(&h->rsNAlt, h->nRS);
  }
  for (auto& row : h->evS)
    for (hipEvent_t& e : row) ok = ok && hipEventCreate(&e) == hipSuccess;
  ok = ok && hipEventCreateWithFlags(&h->evCost, hipEventDisableTiming) == hipSuccess;
  ok = ok && hipStreamCreateWithFlags(&h->stR, hipStreamNonBlocking) == hipSuccess;
  ok = ok && hipHostMalloc((void**)&h->hostRed, 32 * sizeof(double), hipHostMallocDefault) == hipSuccess;
  if (!ok) specRelease(h);
  h->specReady = ok;
  return ok;
}
// the buffers the speculative work writes instead of h->d's
Dev specDev(vb_handle h) {
  Dev ds = h->d;
  ds.tiles = h->tilesAlt, ds.cacheW = h->cacheAlt, ds.gRed = h->gRedAlt;
  ds.red = h->d.red + 48, ds.err = h->d.err + 4;
  ds.redS = h->d.redS + 64 * 8;  // own stripes: the fused cost pass adds into the handle's (costS)
  if (h->rsDevice) ds.rsS = h->rsSAlt, ds.rsI = h->rsIAlt, ds.rsG = h->rsGAlt, ds.rsN = h->rsNAlt;
  return ds;
}
// ark_vi_ba's preStepCallback (the rolling-shutter rebuild at the accepted variables) and the
// linearization of the next iteration, queued behind this iteration's cost pass; event set p
// With early set, specEarly queued the small factors' evaluation and the clear beside the cost pass.
// rsDone: vb_optimize already cleared the speculative slots and queued the rebuild on stF (evRs), beside
// the cost pass; the main stream only waits for it.
int specEnqueue(vb_handle h, int dontRetry, int p, bool early, bool rsDone, bool fuseCost) {
  Dev ds = specDev(h);
  if (fuseCost) ds.costS = h->d.redS;
  if (!early && !rsDone) {
    HIPCHK(hipMemsetAsync(ds.red, 0, 16 * sizeof(double), h->st));
    HIPCHK(hipMemsetAsync(ds.err, 0, 2 * sizeof(int32_t), h->st));
  }
  if (rsDone) {
    HIPCHK(hipStreamWaitEvent(h->st, h->evRs, 0));
  } else {
    HIPCHK(hipEventRecord(h->evS[p][0], h->st));
    if (h->rsDevice) launch_rs_build(ds, h->st);
    HIPCHK(hipEventRecord(h->evS[p][1], h->st));
  }
  return linearizeBody(h, ds, 1, dontRetry, h->evS[p][2], h->evS[p][3], early);
}
// The part of the speculative linearization that needs only the stepped variables, queued on stZ after
// the box-plus so it runs beside the cost pass (which leaves the HBM and most CUs idle): the small
// factors' evaluation into the staging slots and the clear of the spare tile store and gradient.  The
// staging slots are free there (the iteration's assembly is joined, and vb_gradient_dot_step's
// evaluation forks from the main stream after the speculative linearization's join).
int specEarly(vb_handle h, bool cleared, bool storeCleared) {
  if (!smallHere(h, 0)) return 0;
  const Dev ds = specDev(h);
  if (!cleared) {
    HIPCHK(hipMemsetAsync(ds.red, 0, 16 * sizeof(double), h->st));
    HIPCHK(hipMemsetAsync(ds.err, 0, 2 * sizeof(int32_t), h->st));
  }
  HIPCHK(hipEventRecord(h->evFork, h->st));
  HIPCHK(hipStreamWaitEvent(h->stZ, h->evFork, 0));
  if (storeCleared && h->clearOnF) HIPCHK(hipStreamWaitEvent(h->stZ, h->evClrDone, 0));
  launch_small_eval(ds, 0, ds.gRed, h->stZ);
  // (storeCleared: the factorization queued the clear on stZ already, factorSeqSn)
  return storeCleared ? 0 : clearReduced(h, ds, h->stZ);
}
// the step was accepted at full size: the speculative buffers become the handle's
void specCommit(vb_handle h) {
  Dev& d = h->d;
  std::swap(d.tiles, h->tilesAlt);
  std::swap(d.cache, h->cacheAlt);
  d.cacheW = d.cache;
  std::swap(d.gRed, h->gRedAlt);
  if (h->rsDevice) {
    std::swap(d.rsS, h->rsSAlt), std::swap(d.rsI, h->rsIAlt);
    std::swap(d.rsG, h->rsGAlt), std::swap(d.rsN, h->rsNAlt);
  }
  h->tileSet ^= 1;
  launch_spec_commit(d, h->st);
}
// the iteration's scalars red[0, n) and error words, read on the readback stream once the cost pass
// (evCost) is done, while whatever was queued behind it runs
int readIterScalars(vb_handle h, double* out, int n) {
  HIPCHK(hipStreamWaitEvent(h->stR, h->evCost, 0));
  HIPCHK(hipMemcpyAsync(h->hostRed, h->d.red, n * sizeof(double), hipMemcpyDeviceToHost, h->stR));
  HIPCHK(hipMemcpyAsync(h->hostRed + 24, h->d.err, 2 * sizeof(int32_t), hipMemcpyDeviceToHost, h->stR));
  HIPCHK(hipStreamSynchronize(h->stR));
  std::copy(h->hostRed, h->hostRed + n, out);
  h->profDone = h->profAtCost;
  int32_t ee[2];
  std::memcpy(ee, h->hostRed + 24, sizeof(ee));
  return errFromWords(h, ee);
}

// Optimizer::optimize (Optimizer.cpp:768-1106).  Per iteration the linearization, damp + eliminate +
// factor + solve, backup, box-plus and cost pass are queued back to back and the host reads their
// scalars once.  Unless a prestep callback or --recompute-preint needs the host between iterations, the
// next iteration's rolling-shutter rebuild and linearization are queued speculatively behind the cost
// pass (into second buffers, specEnqueue), so the device works while the host decides; they are used
// when the step is accepted at full size, the common case.  An error after the backup restores the
// variables of the iteration's linearization point before returning.
int vb_optimize(vb_handle h, const vb_settings* sp, vb_log_cb log, vb_prestep_cb pre, void* user, vb_summary* out) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "vb_optimize before vb_finalize");
  vb_settings s;
  if (sp) s = *sp;
  else vb_default_settings(&s);
  double damping = s.damping;
  int it = 0, lastImpr = 0, lastTroubled = -10;
  double initialCost = 0, finalCost = 0, troubledStartDamping = damping;
  int troubledStart = 0, nTroubled = 0, largestTroubled = 0, nRescaled = 0;
  int dontRetry = 0;
  auto acceptable = [](const vb_cost_stats& st) {
    const double rate = st.num_invalid / (st.num_total + 1.0);
    return rate < 0.03 && (st.num_invalid < st.num_prev_invalid * 2.0 + 50);
  };
  const bool preint = h->recomputePreint && h->pi.n > 0;
  // (no memory for the spare buffers: the plain controller, which needs none)
  const bool speculate = !pre && !preint && !h->sharded && !h->partSet && specPrepare(h);
  bool specQueued = false;  // the current iteration's rebuild + linearization were queued speculatively
  int specSet = 0;
  int rc;
  char buf[512];
  // an error after this iteration's backup: the variables go back to the linearization point
  bool backedUp = false;
  auto bail = [&](int code) {
    if (backedUp && vb_restore(h) == 0) (void)hipStreamSynchronize(h->st);
    (void)hipStreamSynchronize(h->st);
    return code;
  };
  while (true) {
    auto t0 = std::chrono::steady_clock::now();
    backedUp = false;
    if (specQueued) {
      specCommit(h);
    } else {
      // ark_vi_ba's preStepCallback (main_AriaKit_ViBa.cpp:95-101): updateRollingShutterData
      // and, under --recompute-preint, the preintegrations from the IMU streams (InertialFactors.cpp:19-70)
      if ((h->rsDevice || preint) && (rc = rsUpdateAsync(h, h->rsDevice, preint))) return bail(rc);
      if (pre) pre(it, user);
      if ((rc = linearizeEnqueue(h, 1, dontRetry))) return bail(rc);
    }
    // damp + eliminate + factor + solve, backup, box-plus and the cost pass queued back to back; the host
    // reads their scalars (costs, CostStats, model reduction, step ratios) and errors once, after the cost
    // pass: none of them changes what the queued work does
    double prevCost, modelRed, ratios[3], newCost;
    vb_cost_stats st;
    const bool specNext = speculate && it + 1 < s.max_num_iterations;
    const bool early = specNext && smallHere(h, 0) && h->specEarly;
    h->clearWanted = early && h->clearInFactor, h->clearQueued = false;
    rc = dampFactorSolveEnqueue(h, damping, false);
    const bool storeCleared = h->clearQueued;
    h->clearWanted = h->clearQueued = false;
    if (rc) return bail(rc);
    if ((rc = vb_backup(h))) return bail(rc);
    backedUp = true;
    if ((rc = applyStepEnqueue(h, 0, 10, 11))) return bail(rc);
    // the next iteration's rolling-shutter rebuild (a few latency-bound waves) on stF beside the cost pass
    // instead of after it on the main stream: the speculative slots are cleared first (the rebuild sets
    // error bits), and the main stream waits for it (evRs) before the linearization -- and so before
    // anything the host queues after its read, e.g. a restore of the variables the rebuild reads
    bool rsSide = false;
    if (specNext && h->rsDevice) {
      const Dev ds = specDev(h);
      const int p = specSet ^ 1;
      if (hipMemsetAsync(ds.red, 0, 16 * sizeof(double), h->st) != hipSuccess ||
          hipMemsetAsync(ds.err, 0, 2 * sizeof(int32_t), h->st) != hipSuccess ||
          hipEventRecord(h->evStep, h->st) != hipSuccess || hipStreamWaitEvent(h->stF, h->evStep, 0) != hipSuccess ||
          hipEventRecord(h->evS[p][0], h->stF) != hipSuccess)
        return bail(fail(VB_E_HIP, "speculative rebuild fork"));
      launch_rs_build(ds, h->stF);
      if (hipEventRecord(h->evS[p][1], h->stF) != hipSuccess || hipEventRecord(h->evRs, h->stF) != hipSuccess)
        return bail(fail(VB_E_HIP, "speculative rebuild join"));
      rsSide = true;
    }
    if (early && (rc = specEarly(h, rsSide, storeCleared))) return bail(rc);
    // the global-shutter part of the cost pass inside the speculative linearization (every observation
    // evaluated there: not under dontRetry)
    const bool fuseCost = specNext && h->costFuse && !dontRetry;
    if ((rc = fuseCost ? costFusedEnqueue(h) : costEnqueue(h, 1, false))) return bail(rc);
    const bool wasSpec = specQueued;
    const int wasSet = specSet;
    specQueued = false;
    if (speculate) {
      if (!fuseCost) {  // (fused: recorded after the speculative visual linearization)
        if (hipEventRecord(h->evCost, h->st) != hipSuccess) return bail(fail(VB_E_HIP, "hipEventRecord"));
        h->profAtCost = h->profUsed;
      }
      // the next iteration's rebuild + linearization, assuming this step is accepted at full size (not
      // after the last iteration: its work would only be discarded)
      if (it + 1 < s.max_num_iterations) {
        specSet ^= 1;
        if ((rc = specEnqueue(h, dontRetry, specSet, early, rsSide, fuseCost))) return bail(rc);
        specQueued = true;
      }
    }
    profHarvestPrefix(h, h->profDone);  // the previous iteration's event times, read while this one runs
    {
      double r[17];
      if ((rc = speculate ? readIterScalars(h, r, 17) : readRedErr(h, r, 17))) return bail(rc);
      if (it == h->faultFailIt) return bail(fail(VB_E_NUMERIC, "reduced system Cholesky breakdown (injected)"));
      prevCost = r[0], modelRed = 0.5 * r[16];
      const double n = (double)std::max<int64_t>(1, h->nParams);
      ratios[0] = r[8], ratios[1] = std::sqrt(r[9] / n), ratios[2] = r[10] / n;
      costStats(h, r + 1, &newCost, &st);
      if (wasSpec) {
        h->times.linearize_ms = elapsed(h->evS[wasSet][2], h->evS[wasSet][3]);
        if (h->rsDevice) h->times.rs_update_ms = elapsed(h->evS[wasSet][0], h->evS[wasSet][1]);
      } else {
        h->times.linearize_ms = elapsed(h->ev[0], h->ev[1]);
        if (h->rsTimed) h->times.rs_update_ms = elapsed(h->ev[8], h->ev[9]), h->rsTimed = false;
      }
      h->times.schur_ms = elapsed(h->ev[2], h->ev[3]);
      h->times.factor_ms = elapsed(h->ev[3], h->ev[4]);
      h->times.solve_ms = elapsed(h->ev[4], h->ev[5]);
      h->times.step_ms = elapsed(h->ev[10], h->ev[11]);
      h->times.cost_ms = elapsed(h->ev[6], h->ev[7]);
      h->linearized = false, h->factored = true;
    }
    finalCost = prevCost;
    if (it == 0) initialCost = prevCost;
    if (it == h->faultNegModelRedIt) modelRed = -modelRed;  // test fault injection
    if (modelRed < 0) {
      // Optimizer.cpp:835-854: the reference re-linearizes into `hess` at the same point (the caches
      // and the gradient it recomputes are the ones it has) and raises the damping, keeping the old
      // step.  Its re-linearization also overwrites the factor in `hess`, so a later sub-step solve
      // of that iteration runs BaSpaCho's triangular solves on an unfactored matrix; that value is
      // defined by BaSpaCho's storage layout and is not reproduced: here the sub-step uses the
      // factor (tests/test_parity_configs.py forces this branch).
      damping *= s.damping_adjust_on_fail;
    }
    double costRed = prevCost - newCost;
    const double ratioRedToCost = costRed / newCost;
    double ratioRedToExp = costRed / modelRed;
    double applied = 1.0;
    bool okRate = acceptable(st);
    bool rescaled = false;
    if (s.max_step_factor_attempts > 0 && (ratioRedToExp < s.min_relative_cost_reduction || !okRate)) {
      rescaled = true, nRescaled++;
      double backRed;
      if ((rc = vb_gradient_dot_step(h, dontRetry, &backRed))) return bail(rc);
      double sf = backRed > 0 ? modelRed / (modelRed + backRed) : s.step_factor_decrease;
      for (int i = 0; i < s.max_step_factor_attempts; i++) {
        applied *= sf;
        if ((rc = vb_scale_step(h, sf)) || (rc = vb_restore(h))) return bail(rc);
        double rr[3];
        if ((rc = vb_apply_step(h, 0, rr))) return bail(rc);
        vb_cost_stats stF;
        double costF;
        if ((rc = vb_cost(h, 1, &costF, &stF))) return bail(rc);
        const double redF = prevCost - newCost;  // Optimizer.cpp:935 (reference uses the full-step cost)
        const double rF = redF / (modelRed * applied);
        if (rF >= s.min_relative_cost_reduction && acceptable(stF)) {
          newCost = costF, st = stF, costRed = redF, ratioRedToExp = rF, okRate = true;
          break;
        }
        if (s.try_sub_step) {
          double br;
          if ((rc = vb_gradient_dot_step(h, dontRetry, &br))) return bail(rc);
          if ((rc = vb_solve_with_new_gradient(h))) return bail(rc);
          double r2[3];
          if ((rc = vb_apply_step(h, 1, r2))) return bail(rc);
          vb_cost_stats stS;
          double costS;
          if ((rc = vb_cost(h, 1, &costS, &stS))) return bail(rc);
          const double redS = prevCost - costS;
          const double rS = redS / (modelRed * applied);
          if (rS >= s.min_relative_cost_reduction && acceptable(stS)) {
            newCost = costS, st = stS, costRed = redS, ratioRedToExp = rS, okRate = true;
            break;
          }
        }
        dontRetry = 1;
        sf = s.step_factor_decrease;
      }
    }
    const char* tol = ratioRedToCost < s.relative_cost_tolerance     ? "relative cost"
                      : costRed < s.absolute_cost_tolerance          ? "absolute cost"
                      : ratios[1] < s.variables_tolerance            ? "variable"
                                                                     : nullptr;
    const bool rejected = newCost > prevCost || !okRate;
    // the speculative linearization assumed the full step stays applied
    if (rejected || rescaled) specQueued = false;
    if (rejected) {
      if (lastTroubled != it - 1) troubledStartDamping = damping, troubledStart = it;
      damping *= s.damping_adjust_on_fail;
      if ((rc = vb_restore(h))) return bail(rc);
      if (damping > s.damping_max) break;
      lastTroubled = it;
    } else {
      if (lastTroubled == it - 1)
        if (troubledStartDamping < 1e1 && damping > 1e-3) {
          nTroubled++;
          largestTroubled = std::max(largestTroubled, it - troubledStart);
        }
      if (ratioRedToExp >= s.min_relative_cost_reduction && applied > s.min_step_factor_for_good)
        damping = std::max(damping * s.damping_adjust_on_good_step, s.damping_min);
      else
        damping *= s.damping_adjust_on_average_step;
      finalCost = newCost;
    }
    h->times.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    it++;
    if (log && s.verbose) {
      snprintf(buf, sizeof(buf),
               "it %d cost %.12g -> %.12g lambda %.3g (t %.2f ms: lin %.2f schur %.2f factor %.2f solve %.2f)", it,
               prevCost, newCost, damping, h->times.total_ms, h->times.linearize_ms, h->times.schur_ms,
               h->times.factor_ms, h->times.solve_ms);
      log(buf, user);
    }
    if (!tol) lastImpr = it;
    if (it >= lastImpr + s.stop_if_no_improvement_for && it >= lastTroubled + s.distance_from_troubled_iteration) break;
    if (it >= s.max_num_iterations) break;
  }
  // (a speculative linearization left queued by a convergence stop is never committed; its buffers are
  // the spare ones)
  HIPCHK(hipStreamSynchronize(h->st));
  if (out) {
    out->initial_cost = initialCost, out->final_cost = finalCost;
    out->num_troubled_seqs = nTroubled, out->largest_troubled_seq = largestTroubled, out->num_iterations = it;
    out->num_rescaled = nRescaled;
  }
  return 0;
}

}  // extern "C"

