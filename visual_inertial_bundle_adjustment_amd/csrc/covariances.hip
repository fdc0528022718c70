// Covariances (≙ Optimizer::computeJointCovariances / computeCovariances, Optimizer.cpp:503-697): the
// selected inversion of the tile factor (selinv.hip) and the per-column solves of off-pattern blocks.
#include "host.hpp"

extern "C" {
int selectedInversion(vb_handle h) {
  Dev& d = h->d;
  const int32_t nT = d.nT;
  std::vector<int32_t> level(nT, 0);
  int32_t nLev = 0;
  for (int32_t J = 0; J < nT; J++) {
    for (int64_t i = h->rowStart[J]; i < h->rowStart[J + 1]; i++) level[J] = std::max(level[J], level[h->rowColH[i]] + 1);
    nLev = std::max(nLev, level[J] + 1);
  }
  std::vector<std::vector<int32_t>> cols(nLev);
  for (int32_t J = 0; J < nT; J++) cols[level[J]].push_back(J);
  // per level: U items (L slot, J), Z items (target slot, I, J, first U of the column), diagonal items
  // (J, first U); U indices restart at 0 every level (one compact scratch of the largest level)
  std::vector<int32_t> uIt, zIt, dIt;
  std::vector<int64_t> lvU(nLev + 1, 0), lvZ(nLev + 1, 0), lvD(nLev + 1, 0);
  int64_t maxU = 1;
  for (int32_t L = nLev - 1, k = 0; L >= 0; L--, k++) {
    int32_t u = 0;
    for (int32_t J : cols[L]) {
      const int64_t c0 = h->colStart[J], n = h->colStart[J + 1] - c0;
      for (int64_t q = 1; q < n; q++) {
        uIt.insert(uIt.end(), {h->colTilesH[c0 + q], J});
        zIt.insert(zIt.end(), {h->colTilesH[c0 + q], h->colRowsH[c0 + q], J, u});
      }
      dIt.insert(dIt.end(), {J, u});
      u += (int32_t)(n - 1);
    }
    maxU = std::max<int64_t>(maxU, u);
    lvU[k + 1] = (int64_t)uIt.size() / 2, lvZ[k + 1] = (int64_t)zIt.size() / 4, lvD[k + 1] = (int64_t)dIt.size() / 2;
  }
  int32_t *uD = nullptr, *zD = nullptr, *dD = nullptr;
  double* U = nullptr;
  int rc = 0;
  if (upload(&uD, uIt) || upload(&zD, zIt) || upload(&dD, dIt) ||
      hipMalloc((void**)&U, (size_t)maxU * TS * TS * sizeof(double)) != hipSuccess) {
    rc = fail(VB_E_HIP, "selected inversion: device allocation");
  } else {
    for (int32_t k = 0; k < nLev; k++)
      launch_selinv_level(d.tiles, d.tileIdx, nT, h->colStartD, h->colRowsD, h->colTilesD, h->linv, U,
                          uD + 2 * lvU[k], (int)(lvU[k + 1] - lvU[k]), zD + 4 * lvZ[k], (int)(lvZ[k + 1] - lvZ[k]),
                          dD + 2 * lvD[k], (int)(lvD[k + 1] - lvD[k]), h->st);
    if (hipStreamSynchronize(h->st) != hipSuccess) rc = fail(VB_E_HIP, "selected inversion: kernel failure");
  }
  for (void* p : {(void*)uD, (void*)zD, (void*)dD, (void*)U})
    if (p) (void)hipFree(p);
  return rc;
}

int vb_compute_covariances(vb_handle h, double damping, int64_t n_blocks, const int64_t* block_start,
                           const int32_t* kinds, const int32_t* handles, double* out, double* used_damping) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "vb_compute_covariances before vb_finalize");
  if (h->partSet || h->sharded) return fail(VB_E_UNSUPPORTED, "covariances run on a single handle");
  if (n_blocks < 0 || (n_blocks > 0 && (!block_start || !kinds || !handles || !out)))
    return fail(VB_E_ARG, "vb_compute_covariances: null argument");
  if (!h->sch[0].built) return fail(VB_E_STATE, "no factorization schedule");
  // (kind, handle) -> reduced variable
  std::unordered_map<int64_t, int32_t> rvOf;
  for (size_t i = 0; i < h->rvKind.size(); i++) rvOf[((int64_t)h->rvKind[i] << 32) | (uint32_t)h->rvHandle[i]] = (int32_t)i;
  const int64_t nv = n_blocks ? block_start[n_blocks] : 0;
  std::vector<int32_t> rv(nv);
  for (int64_t q = 0; q < n_blocks; q++)
    if (block_start[q + 1] < block_start[q]) return fail(VB_E_ARG, "block_start must be non-decreasing");
  for (int64_t i = 0; i < nv; i++) {
    if (kinds[i] == VB_VAR_POINT) return fail(VB_E_UNSUPPORTED, "covariance of a landmark point (points are eliminated)");
    auto it = rvOf.find(((int64_t)kinds[i] << 32) | (uint32_t)handles[i]);
    if (it == rvOf.end()) return fail(VB_E_ARG, "covariance of a constant or unknown variable");
    rv[i] = it->second;
  }
  Dev& d = h->d;
  // initDirectSolverData + factor, retried with more damping while the factor breaks down
  double lam = damping;
  for (int attempt = 0;; attempt++) {
    if (int rc = vb_linearize(h, 0, 0, nullptr)) return rc;
    HIPCHK(hipMemsetAsync(d.err, 0, sizeof(int32_t), h->st));
    launch_landmark(d, lam, 0, d.lmB, d.lmE, h->st);
    HIPCHK(hipMemsetAsync(d.rhs, 0, (size_t)d.nT * TS * sizeof(double), h->st));
    launch_schur(d, lam, 1, h->st);
    h->factorOnly = true;  // (the fused forward solve would run on a stale right-hand side)
    const int frc = factorReduced(h);
    h->factorOnly = false;
    if (frc) return frc;
    int32_t e = 0;
    HIPCHK(hipMemcpyAsync(&e, d.err, sizeof(int32_t), hipMemcpyDeviceToHost, h->st));
    HIPCHK(hipStreamSynchronize(h->st));
    if (!(e & (2 | 8))) {
      if (int rc = checkErr(h)) return rc;
      break;
    }
    if (attempt > 200) return fail(VB_E_NUMERIC, "covariances: factor keeps breaking down");
    lam = lam < 1e-9 ? lam + 1e-9 : lam * 2.0;
  }
  if (used_damping) *used_damping = lam;
  // Every element (row ra, column rb of the padded reduced order) of a block whose tiles lie on the
  // factor's pattern comes from the selected inversion.  That covers SingleSessionProblem::
  // computeCovariances' request (SingleSessionProblem.cpp:66-118): a rig's pose, velocity and omega
  // couple directly in S, and a calibration variable is one block.  Blocks off the pattern (joint
  // blocks of uncoupled variables) take one reduced solve per column S x = e, before the inversion
  // consumes the factor.  VIBA_COV_SOLVES=1 sends every block that way (test aid).
  const int32_t nT = d.nT;
  std::vector<int32_t> tix((size_t)nT * nT, -1);
  for (int32_t J = 0; J < nT; J++)
    for (int64_t c = h->colStart[J]; c < h->colStart[J + 1]; c++) tix[(size_t)h->colRowsH[c] * nT + J] = h->colTilesH[c];
  auto elem = [&](int64_t ra, int64_t rb) -> int64_t {  // Z(ra, rb) in the tile store, -1 off the pattern
    if (ra / TS < rb / TS) std::swap(ra, rb);
    const int32_t t = tix[(size_t)(ra / TS) * nT + rb / TS];
    return t < 0 ? -1 : (int64_t)t * TS * TS + (rb % TS) * TS + ra % TS;
  };
  const bool forceSolves = getenv("VIBA_COV_SOLVES") && atoi(getenv("VIBA_COV_SOLVES")) == 1;
  std::vector<int64_t> outOff(n_blocks + 1, 0), gidx;
  std::vector<uint8_t> bySolve(n_blocks, forceSolves ? 1 : 0);
  std::vector<std::vector<int64_t>> offs(n_blocks);
  for (int64_t q = 0; q < n_blocks; q++) {
    const int64_t b = block_start[q], e = block_start[q + 1];
    std::vector<int64_t>& off = offs[q];
    off.assign(e - b + 1, 0);
    for (int64_t i = b; i < e; i++) off[i - b + 1] = off[i - b] + h->rvDim[rv[i]];
    const int64_t n = off.back();
    outOff[q + 1] = outOff[q] + n * n;
    for (int64_t i = b; i < e; i++)
      for (int c = 0; c < h->rvDim[rv[i]]; c++)
        for (int64_t j = b; j < e; j++)
          for (int r = 0; r < h->rvDim[rv[j]]; r++) {
            const int64_t at = elem(h->rvOff[rv[j]] + r, h->rvOff[rv[i]] + c);
            gidx.push_back(at);
            if (at < 0) bySolve[q] = 1;
          }
  }
  const int64_t nPad = (int64_t)nT * TS;
  std::vector<double> rhs(nPad, 0.0), x(nPad);
  bool anyInv = false;
  for (int64_t q = 0; q < n_blocks; q++) {
    if (!bySolve[q]) {
      anyInv = true;
      continue;
    }
    const int64_t b = block_start[q], e = block_start[q + 1], n = offs[q].back();
    double* o = out + outOff[q];
    for (int64_t i = b; i < e; i++)
      for (int c = 0; c < h->rvDim[rv[i]]; c++) {
        const int64_t row = h->rvOff[rv[i]] + c;
        rhs[row] = 1.0;
        HIPCHK(hipMemcpyAsync(h->rhsWork, rhs.data(), nPad * sizeof(double), hipMemcpyHostToDevice, h->st));
        rhs[row] = 0.0;
        if (int rc = solveReduced(h)) return rc;
        HIPCHK(hipMemcpyAsync(x.data(), d.xRed, nPad * sizeof(double), hipMemcpyDeviceToHost, h->st));
        HIPCHK(hipStreamSynchronize(h->st));
        const int64_t col = offs[q][i - b] + c;
        for (int64_t j = b; j < e; j++)
          for (int r = 0; r < h->rvDim[rv[j]]; r++) o[col * n + offs[q][j - b] + r] = x[h->rvOff[rv[j]] + r];
      }
  }
  if (anyInv) {
    if (int rc = selectedInversion(h)) return rc;
    for (int64_t q = 0; q < n_blocks; q++)  // solved blocks: gather anything (their slots are overwritten below)
      if (bySolve[q]) std::fill(gidx.begin() + outOff[q], gidx.begin() + outOff[q + 1], 0);
    const int64_t ng = (int64_t)gidx.size();
    int64_t* idxD = nullptr;
    double* valD = nullptr;
    std::vector<double> val(ng);
    int rc = 0;
    if (upload(&idxD, gidx) || hipMalloc((void**)&valD, std::max<int64_t>(1, ng) * sizeof(double)) != hipSuccess) {
      rc = fail(VB_E_HIP, "covariances: device allocation");
    } else {
      launch_gather(d.tiles, idxD, ng, valD, h->st);
      if (hipMemcpyAsync(val.data(), valD, ng * sizeof(double), hipMemcpyDeviceToHost, h->st) != hipSuccess ||
          hipStreamSynchronize(h->st) != hipSuccess)
        rc = fail(VB_E_HIP, "covariances: gather");
    }
    if (idxD) (void)hipFree(idxD);
    if (valD) (void)hipFree(valD);
    if (rc) return rc;
    for (int64_t q = 0; q < n_blocks; q++)
      if (!bySolve[q]) std::copy(val.begin() + outOff[q], val.begin() + outOff[q + 1], out + outOff[q]);
  }
  h->linearized = false, h->factored = false;
  return checkErr(h);
}
}  // extern "C"
