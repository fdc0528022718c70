// vb_finalize: nested-dissection order of the reduced variables, tile pattern and symbolic fill (≙
// Optimizer::initSolver, Optimizer.cpp:166-207), the landmark / observation-group layouts, the Schur work
// lists, the factorization schedules (level-scheduled columns, two-column supernodes on streams) and the
// solve task lists.
#include "host.hpp"

namespace viba_host {
// the two-column supernode schedule (SnSched) of a column schedule from the column patterns: colSel(J)
// columns factored here, tgtSel(J) fan-in targets in column J, srcSel(K) contributions from column K
// (the selectors of the column schedule's build(): all columns on a single handle; a rank's subtree plus
// its ROOT targets, or the ROOT columns, in partition mode)
int buildSupernodes(vb_handle h, SnSched& S, const std::vector<int32_t>& tileIdx, int32_t nT, int64_t nTiles,
                    const std::function<bool(int32_t)>& colSel, const std::function<bool(int32_t)>& tgtSel,
                    const std::function<bool(int32_t)>& srcSel, int nGroups = 1) {
  auto colRows = [&](int32_t J, int64_t& a, int64_t& b) { a = h->colStart[J], b = h->colStart[J + 1]; };
  // pair J with J + 1: J + 1 is J's first off-diagonal row (its parent) and every other row of J is a
  // row of J + 1 (so the pair's rows are J + 1's), both in one nested-dissection part
  std::vector<int8_t> pr(nT, 0);
  for (int32_t J = 0; J + 1 < nT; J++) {
    if (pr[J]) continue;
    int64_t a, b, a2, b2;
    colRows(J, a, b), colRows(J + 1, a2, b2);
    if (b - a < 2 || h->colRowsH[a + 1] != J + 1 || h->colOwner[J] != h->colOwner[J + 1] || !colSel(J) ||
        !colSel(J + 1))
      continue;
    bool sub = true;
    int64_t q = a2 + 1;
    for (int64_t c = a + 2; c < b && sub; c++) {
      while (q < b2 && h->colRowsH[q] < h->colRowsH[c]) q++;
      sub = q < b2 && h->colRowsH[q] == h->colRowsH[c];
    }
    if (sub) pr[J] = 1, pr[J + 1] = 2;
  }
  // supernode levels: one more than the levels of the supernodes of every row tile (pair-internal
  // (J + 1, J) excluded)
  std::vector<int32_t> lev(nT, 0);
  int32_t nLev = 0;
  for (int32_t J = 0; J < nT; J++) {
    if (pr[J] == 2) continue;
    int32_t lv = 0;
    for (int32_t X = J; X <= J + (pr[J] == 1 ? 1 : 0); X++)
      for (int64_t i = h->rowStart[X]; i < h->rowStart[X + 1]; i++) {
        const int32_t K = h->rowColH[i];
        if (X == J + 1 && K == J) continue;
        lv = std::max(lv, lev[K] + 1);
      }
    lev[J] = lv;
    if (pr[J] == 1) lev[J + 1] = lv;
    nLev = std::max(nLev, lv + 1);
  }
  std::vector<std::vector<int32_t>> sup(nLev);  // first column of every supernode, by level
  for (int32_t J = 0; J < nT; J++)
    if (pr[J] != 2) sup[lev[J]].push_back(J);
  // fan-in contributions by target tile, sources in level order, pair-internal ones left out
  std::vector<int64_t> ccnt(nTiles + 1, 0);
  std::vector<int32_t> pairs;
  for (int pass = 0; pass < 2; pass++) {
    std::vector<int64_t> pos;
    if (pass == 1) {
      for (int64_t t = 0; t < nTiles; t++) ccnt[t + 1] += ccnt[t];
      pos.assign(ccnt.begin(), ccnt.end() - 1);
      pairs.assign(2 * (size_t)ccnt[nTiles], 0);
    }
    for (int32_t L = 0; L < nLev; L++)
      for (int32_t J0 : sup[L])
        for (int32_t K = J0; K <= J0 + (pr[J0] == 1 ? 1 : 0); K++) {
          if (!srcSel(K)) continue;
          const int64_t c0 = h->colStart[K], n = h->colStart[K + 1] - c0;
          for (int64_t qi = 1; qi < n; qi++)
            for (int64_t qk = 1; qk <= qi; qk++) {
              if (pr[K] == 1 && qk == 1) continue;  // targets in column K + 1: inside the supernode
              if (!tgtSel(h->colRowsH[c0 + qk])) continue;
              const int32_t t = tileIdx[(size_t)h->colRowsH[c0 + qi] * nT + h->colRowsH[c0 + qk]];
              if (t < 0) return fail(VB_E_STATE, "internal: symbolic fill incomplete");
              if (pass == 0) {
                ccnt[t + 1]++;
              } else {
                const int64_t at = pos[t]++;
                pairs[2 * at] = h->colTilesH[c0 + qi], pairs[2 * at + 1] = h->colTilesH[c0 + qk];
              }
            }
        }
  }
  if (ccnt[nTiles] >= INT32_MAX) return fail(VB_E_STATE, "tile Cholesky too large (contribution count)");
  // Streams (nGroups > 1): the supernodes' elimination tree (parent: the supernode of the first row below
  // it) cut into independent subtrees on separate streams, so one subtree's diagonal blocks and rows
  // (latency-bound, a few workgroups) run beside another's fan-in instead of behind a level barrier of the
  // whole chip.  The tree is split from its roots down, heaviest subtree first, until none outweighs
  // 1/nGroups of the frontier by more than 15%; the frontier's subtrees go to the streams longest first.
  // Their ancestors (the separators above the cut) follow the stream of their heaviest child and wait for
  // the others' (segDep), so sibling separators also run side by side.  Weights: the fan-in contributions
  // into a supernode's columns.
  std::vector<int32_t> grp(nT, 0);
  std::vector<int32_t> snPar(nT, -1);
  int G = std::max(1, nGroups);
  if (G > 1) {
    std::vector<int32_t> snOf(nT);
    std::vector<int32_t>& par = snPar;
    std::vector<double> W(nT, 0.0);
    std::vector<std::vector<int32_t>> kids(nT);
    for (int32_t J = 0; J < nT; J++) snOf[J] = pr[J] == 2 ? J - 1 : J;
    for (int32_t J0 = 0; J0 < nT; J0++) {
      if (pr[J0] == 2) continue;
      const int32_t Jl = pr[J0] == 1 ? J0 + 1 : J0;
      if (h->colStart[Jl + 1] - h->colStart[Jl] > 1) par[J0] = snOf[h->colRowsH[h->colStart[Jl] + 1]];
      for (int32_t J = J0; J <= Jl; J++)
        for (int64_t c = h->colStart[J]; c < h->colStart[J + 1]; c++) W[J0] += (double)(ccnt[h->colTilesH[c] + 1] - ccnt[h->colTilesH[c]]);
    }
    std::vector<double> own(W);
    for (int32_t J0 = 0; J0 < nT; J0++)  // parents come after their children in the elimination order
      if (pr[J0] != 2 && par[J0] >= 0) W[par[J0]] += W[J0], kids[par[J0]].push_back(J0);
    std::vector<int32_t> front;
    for (int32_t J0 = 0; J0 < nT; J0++)
      if (pr[J0] != 2 && par[J0] < 0) front.push_back(J0);
    std::vector<int8_t> top(nT, 0);
    for (int it = 0; it < 4 * nT && front.size() < 256; it++) {
      double tot = 0.0;
      size_t xi = 0;
      for (size_t i = 0; i < front.size(); i++) {
        tot += W[front[i]];
        if (W[front[i]] > W[front[xi]]) xi = i;
      }
      const int32_t X = front[xi];
      if (W[X] <= 1.15 * tot / G || kids[X].empty()) break;
      top[X] = 1;
      front.erase(front.begin() + (ptrdiff_t)xi);
      front.insert(front.end(), kids[X].begin(), kids[X].end());
    }
    std::stable_sort(front.begin(), front.end(), [&](int32_t a, int32_t b) { return W[a] > W[b]; });
    std::vector<double> load(G, 0.0);
    std::vector<int32_t> rootG(nT, -1);
    for (int32_t X : front) {
      const int g = (int)(std::min_element(load.begin(), load.end()) - load.begin());
      load[g] += W[X], rootG[X] = g;
    }
    for (int32_t J0 = nT - 1; J0 >= 0; J0--)  // the frontier subtrees, parents first
      if (pr[J0] != 2 && !top[J0]) grp[J0] = rootG[J0] >= 0 ? rootG[J0] : par[J0] >= 0 ? grp[par[J0]] : 0;
    for (int32_t J0 = 0; J0 < nT; J0++)  // the separators above the cut, children first
      if (pr[J0] != 2 && top[J0]) {
        int32_t best = -1;
        for (int32_t C : kids[J0])
          if (best < 0 || W[C] > W[best]) best = C;
        grp[J0] = best >= 0 ? grp[best] : 0;
      }
    for (int32_t J0 = 0; J0 < nT; J0++)
      if (pr[J0] == 1) grp[J0 + 1] = grp[J0];
    if (getenv("VIBA_STATS")) {
      std::vector<double> gw(G, 0.0), gt(G, 0.0);
      std::vector<int> gs(G, 0);
      for (int32_t J0 = 0; J0 < nT; J0++)
        if (pr[J0] != 2) gw[grp[J0]] += own[J0], gs[grp[J0]]++, gt[grp[J0]] += top[J0] ? own[J0] : 0.0;
      for (int g = 0; g < G; g++)
        fprintf(stderr, "[factor stats] stream %d: supernodes %d, contributions %.0f (%.0f above the cut)\n", g, gs[g], gw[g],
                gt[g]);
    }
  }
  // a stream's segment shares the chip with the other streams' segments of its level: the fan-in workgroup
  // target and the fused-level threshold are divided by their number
  std::vector<int> nAct(nLev, 0);
  for (int32_t L = 0; L < nLev; L++) {
    uint32_t m = 0;
    for (int32_t J0 : sup[L]) m |= 1u << grp[J0];
    nAct[L] = __builtin_popcount(m);
  }
  // levels with at most this many row items run snpotrf_trsm8_kernel (re-swept at two streams, r05an: 128 /
  // 512 the same, 1024 -1.7%)
  const int64_t fuseMax = 256;
  // fan-in workgroups per level launch, divided among the level's active streams (r05ao: 2048 / 4096 the
  // same, 6144 -0.8%)
  const int64_t fanTarget = 3072;
  std::vector<int32_t> fan, pot, rows, fus, copy;
  S.lvU.assign(1, 0), S.lvS.assign(1, 0), S.lvR.assign(1, 0), S.lvF.assign(1, 0);
  S.segG.clear(), S.segL.clear(), S.segDep.clear();

  S.nTwo = 0;
  auto tile = [&](int32_t I, int32_t J) { return tileIdx[(size_t)I * nT + J]; };
  // segments: (stream, level), level-major; segDep: the other streams whose earlier segments this one
  // needs (streams of its supernodes' children)
  for (int32_t L = 0; L < nLev; L++)
  for (int g = 0; g < G; g++) {
    std::vector<int32_t> supL;
    uint32_t dep = 0;
    for (int32_t J0 : sup[L])
      if (grp[J0] == g) supL.push_back(J0);
    if (supL.empty()) continue;
    if (G > 1)
      for (int32_t J0 = 0; J0 < nT; J0++)
        if (pr[J0] != 2 && snPar[J0] >= 0 && grp[snPar[J0]] == g && lev[snPar[J0]] == L && grp[J0] != g) dep |= 1u << grp[J0];
    int64_t total = 0;
    for (int32_t J0 : supL)
      for (int32_t J = J0; J <= J0 + (pr[J0] == 1 ? 1 : 0); J++)
        for (int64_t c = h->colStart[J]; c < h->colStart[J + 1]; c++) total += ccnt[h->colTilesH[c] + 1] - ccnt[h->colTilesH[c]];
    const int share = std::max(1, nAct[L]);
    const int64_t fanWgs = fanTarget / share;
    const int64_t cs = std::min<int64_t>(32, std::max<int64_t>(4, (total + fanWgs - 1) / fanWgs));
    const size_t u0 = fan.size() / 4;
    int64_t nRowsL = 0;
    for (int32_t J0 : supL) {
      if (!colSel(J0)) continue;
      const int32_t Jl = pr[J0] == 1 ? J0 + 1 : J0;
      nRowsL += h->colStart[Jl + 1] - h->colStart[Jl] - 1;
    }
    const bool fused = nRowsL <= fuseMax / share;
    for (int32_t J0 : supL) {
      const bool two = pr[J0] == 1;
      const int32_t J2 = two ? J0 + 1 : -1;
      for (int32_t J = J0; J <= (two ? J2 : J0); J++)
        for (int64_t c = h->colStart[J]; c < h->colStart[J + 1]; c++) {
          if (!tgtSel(J)) continue;
          const int32_t t = h->colTilesH[c];
          const int64_t b = ccnt[t], m = ccnt[t + 1] - b;
          if (m == 0) continue;
          const int64_t nch = (m + cs - 1) / cs;
          for (int64_t k = 0; k < nch; k++) {
            const int64_t s0 = b + m * k / nch, s1 = b + m * (k + 1) / nch;
            fan.insert(fan.end(), {t, (int32_t)s0, (int32_t)(s1 - s0), nch > 1 ? 1 : 0});
          }
        }
      if (!colSel(J0)) continue;
      const int32_t t11 = tile(J0, J0), t21 = two ? tile(J2, J0) : -1, t22 = two ? tile(J2, J2) : -1;
      S.nTwo += two ? 1 : 0;
      // rows below the supernode: those of its last column (a pair's first column has no others)
      const int32_t Jl = two ? J2 : J0;
      if (fused) {
        copy.insert(copy.end(), {t11, J0});
        if (two) copy.insert(copy.end(), {t22, J2, t21, nT + J0});
        if (h->colStart[Jl + 1] - h->colStart[Jl] == 1) fus.insert(fus.end(), {t11, J0, t21, t22, -1, -1, -1, 1});
        for (int64_t c = h->colStart[Jl] + 1; c < h->colStart[Jl + 1]; c++) {
          const int32_t I = h->colRowsH[c];
          fus.insert(fus.end(), {t11, J0, t21, t22, two ? tile(I, J0) : h->colTilesH[c], two ? h->colTilesH[c] : -1, I,
                                 c == h->colStart[Jl] + 1 ? 1 : 0});
        }
        continue;
      }
      pot.insert(pot.end(), {t11, J0, t21, t22});
      for (int64_t c = h->colStart[Jl] + 1; c < h->colStart[Jl + 1]; c++) {
        const int32_t I = h->colRowsH[c];
        rows.insert(rows.end(), {two ? tile(I, J0) : h->colTilesH[c], two ? h->colTilesH[c] : -1, J0, J2, I, t11, t21, t22});
      }
    }
    {  // longest chunks first within each XCD's range (as the column schedule)
      std::vector<std::array<int32_t, 4>> q((fan.size() / 4) - u0);
      for (size_t i = 0; i < q.size(); i++)
        for (int k = 0; k < 4; k++) q[i][k] = fan[4 * (u0 + i) + k];
      const size_t nq = q.size(), qq = nq / 8, rr = nq % 8;
      for (size_t x = 0, b0 = 0; x < 8; x++) {
        const size_t len = qq + (x < rr ? 1 : 0);
        std::stable_sort(q.begin() + b0, q.begin() + b0 + len, [](const auto& a, const auto& b) { return a[2] > b[2]; });
        b0 += len;
      }
      for (size_t i = 0; i < q.size(); i++)
        for (int k = 0; k < 4; k++) fan[4 * (u0 + i) + k] = q[i][k];
    }
    S.lvU.push_back((int64_t)fan.size() / 4), S.lvS.push_back((int64_t)pot.size() / 4), S.lvR.push_back((int64_t)rows.size() / 8);
    S.lvF.push_back((int64_t)fus.size() / 8);
    S.segG.push_back(g), S.segL.push_back(L), S.segDep.push_back((int32_t)dep);
  }
  S.nGroups = G;
  S.nLevels = nLev, S.nPairs = ccnt[nTiles];
  S.nSuper = 0;
  for (int32_t J = 0; J < nT; J++) S.nSuper += (pr[J] != 2 && colSel(J)) ? 1 : 0;
  S.nCopy = (int64_t)copy.size() / 2;
  // diagonal-tile inverses (factorSeqSn): the columns of in-place (not fused) supernodes before the top
  // separators' chain, and the rest; the same rule for the chain as factorSeqSn's
  std::vector<int32_t> invE, invL;
  {
    const int nSeg = (int)S.segG.size();
    int chain0 = 0;
    for (int i = 1; i < nSeg; i++)
      if (S.segL[i] == S.segL[i - 1]) chain0 = i + 1;
    std::vector<uint8_t> early(nT, 0);
    for (int i = 0; i < chain0; i++)
      for (int64_t k = S.lvS[i]; k < S.lvS[i + 1]; k++) {
        early[pot[4 * k + 1]] = 1;
        if (pot[4 * k + 2] >= 0) early[pot[4 * k + 1] + 1] = 1;
      }
    for (int32_t J = 0; J < nT; J++) {
      if (!colSel(J)) continue;
      (early[J] ? invE : invL).push_back(J);
    }
  }
  S.nInvEarly = (int64_t)invE.size(), S.nInvLate = (int64_t)invL.size();
  if (upload(&S.updD, fan) || upload(&S.fanPairsD, pairs) || upload(&S.potD, pot) || upload(&S.rowD, rows) ||
      upload(&S.fusD, fus) || upload(&S.copyD, copy) || upload(&S.invEarlyD, invE) || upload(&S.invLateD, invL))
    return VB_E_HIP;
  if (S.nCopy && !h->lscrSn && alloc0(&h->lscrSn, 2 * (size_t)nT * TS * TS)) return VB_E_HIP;
  S.built = true;
  return 0;
}

int doFinalize(vb_handle h) {
  Dev& d = h->d;
  d.jac = makeJac(h->cfg.imu_calib_options);
  d.reproj = makeLoss(h->cfg.reproj_loss_radius, h->cfg.reproj_loss_cutoff);
  d.imu = makeLoss(h->cfg.imu_loss_radius, h->cfg.imu_loss_cutoff);
  d.T = TS;
  for (int k = 0; k < 9; k++) {
    d.nvar[k] = (int64_t)h->cst[k].size();
    if ((int64_t)h->data[k].size() != d.nvar[k] * kVarData[k]) return fail(VB_E_ARG, "variable data size mismatch");
  }
  // ---------------- registration (registerAllVariables; points = elimination range)
  auto tdimOf = [&](int kind, int hh) -> int {
    switch (kind) {
      case 0: case 2: case 3: return 3;
      case 1: case 5: case 7: return 6;
      case 4: {
        const double* c = &h->data[4][(size_t)hh * 24];
        return (int)c[1] + (c[7] != 0 ? 1 : 0) + (c[8] != 0 ? 1 : 0);
      }
      case 6: return d.jac.size;
      default: return 2;
    }
  };
  std::vector<int32_t> redOf[9];
  for (int k = 0; k < 9; k++) redOf[k].assign(d.nvar[k], -1);
  std::vector<int32_t>& lmOf = h->lmOfPoint;
  lmOf.assign(d.nvar[0], -1);
  int64_t nPts = 0;
  std::vector<std::pair<int, int>> red;  // (kind, handle)
  for (int fk = 0; fk < 14; fk++) {
    const int nv = kNumVars[fk];
    const int64_t n = (int64_t)h->fint[fk].size();
    for (int64_t f = 0; f < n; f++)
      for (int s = 0; s < nv; s++) {
        const int kind = kFK[fk][s], hh = h->fvars[fk][f * nv + s];
        if (hh < 0) continue;
        if (hh >= d.nvar[kind]) return fail(VB_E_ARG, "factor references an unknown variable handle");
        if (h->cst[kind][hh]) continue;
        if (kind == 8) return fail(VB_E_UNSUPPORTED, "non-constant gravity is not supported");
        if (kind == 0) {
          if (lmOf[hh] < 0) lmOf[hh] = -2;  // mark; numbered below in handle order
          continue;
        }
        if (redOf[kind][hh] < 0) {
          redOf[kind][hh] = (int32_t)red.size();
          red.push_back({kind, hh});
        }
      }
  }
  // landmark numbering: by the earliest rig that observes the point (time-banded landmark shards
  // and locality of the Schur lists), ties by handle
  {
    std::vector<int64_t> firstRig(d.nvar[0], INT64_MAX);
    const int64_t nv0 = (int64_t)h->fint[0].size();
    for (int64_t f = 0; f < nv0; f++) {
      const int32_t pt = h->fvars[0][f * 5], pose = h->fvars[0][f * 5 + 1];
      if (lmOf[pt] == -2) firstRig[pt] = std::min<int64_t>(firstRig[pt], pose);
    }
    std::vector<int64_t> pts;
    for (int64_t p = 0; p < d.nvar[0]; p++)
      if (lmOf[p] == -2) pts.push_back(p);
    std::stable_sort(pts.begin(), pts.end(), [&](int64_t a, int64_t b) { return firstRig[a] < firstRig[b]; });
    for (int64_t p : pts) lmOf[p] = (int32_t)nPts++;
  }
  // ---------------- reduced ordering: mean pose ordinal of co-occurring poses
  const int nRV = (int)red.size();
  std::vector<double> ks(nRV, 0.0), kc(nRV, 0.0);
  for (int fk = 0; fk < 14; fk++) {
    const int nv = kNumVars[fk];
    const int64_t n = (int64_t)h->fint[fk].size();
    for (int64_t f = 0; f < n; f++) {
      double ps = 0;
      int pc = 0;
      for (int s = 0; s < nv; s++)
        if (kFK[fk][s] == 1 && h->fvars[fk][f * nv + s] >= 0) ps += h->fvars[fk][f * nv + s], pc++;
      if (!pc) continue;
      for (int s = 0; s < nv; s++) {
        const int kind = kFK[fk][s], hh = h->fvars[fk][f * nv + s];
        if (hh < 0 || kind == 0 || kind == 8 || redOf[kind][hh] < 0) continue;
        ks[redOf[kind][hh]] += ps, kc[redOf[kind][hh]] += pc;
      }
    }
  }
  std::vector<int> ord(nRV);
  std::iota(ord.begin(), ord.end(), 0);
  auto key = [&](int r) { return red[r].first == 1 ? (double)red[r].second : (kc[r] > 0 ? ks[r] / kc[r] : 1e30); };
  std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) {
    const double ka = key(a), kb = key(b);
    if (ka != kb) return ka < kb;
    if (red[a].first != red[b].first) return red[a].first < red[b].first;
    return red[a].second < red[b].second;
  });
  // ---------------- nested dissection over the time order (the ordering is ours)
  // The time-ordered reduced system is a band (landmark tracks span up to ~60 rigs), whose Cholesky
  // is a chain as long as the matrix.  Recursive bisection: cut the time order at half its
  // dimension; the left variables coupled across the cut form the separator, ordered after both
  // halves; each part starts on a tile boundary so that parts stay independent tile columns and the
  // factorization runs level by level (factorSeq).  Any symmetric order is a valid Cholesky order:
  // the separators only need to be sufficient, not minimal.
  std::vector<int> tp(nRV);
  for (int i = 0; i < nRV; i++) tp[ord[i]] = i;
  std::vector<int> hiP(tp), loP(tp);
  {
    auto regPos = [&](int kind, int hh) -> int {
      if (hh < 0 || kind == 0 || kind == 8 || redOf[kind][hh] < 0) return -1;
      return tp[redOf[kind][hh]];
    };
    std::vector<int> lmLo(nPts, INT32_MAX), lmHi(nPts, -1);
    const int64_t nv0 = (int64_t)h->fint[0].size();
    auto obsPos = [&](int64_t f, int* ps) {
      const int32_t* v = &h->fvars[0][f * 5];
      ps[0] = regPos(1, v[1]), ps[1] = regPos(5, v[2]), ps[2] = regPos(4, v[3]);
      ps[3] = h->fint[0][f] >= 0 ? regPos(2, v[4]) : -1;
    };
    for (int64_t f = 0; f < nv0; f++) {
      int ps[4];
      obsPos(f, ps);
      const int l = lmOf[h->fvars[0][f * 5]];
      int lo = INT32_MAX, hi = -1;
      for (int k = 0; k < 4; k++)
        if (ps[k] >= 0) lo = std::min(lo, ps[k]), hi = std::max(hi, ps[k]);
      if (hi < 0) continue;
      if (l >= 0) {
        lmLo[l] = std::min(lmLo[l], lo), lmHi[l] = std::max(lmHi[l], hi);
      } else {
        for (int k = 0; k < 4; k++)
          if (ps[k] >= 0) {
            const int r = ord[ps[k]];
            hiP[r] = std::max(hiP[r], hi), loP[r] = std::min(loP[r], lo);
          }
      }
    }
    for (int64_t f = 0; f < nv0; f++) {
      const int l = lmOf[h->fvars[0][f * 5]];
      if (l < 0 || lmHi[l] < 0) continue;
      int ps[4];
      obsPos(f, ps);
      for (int k = 0; k < 4; k++)
        if (ps[k] >= 0) {
          const int r = ord[ps[k]];
          hiP[r] = std::max(hiP[r], lmHi[l]), loP[r] = std::min(loP[r], lmLo[l]);
        }
    }
    for (int fk = 1; fk < 14; fk++) {
      const int nv = kNumVars[fk];
      const int64_t n = (int64_t)h->fint[fk].size();
      for (int64_t f = 0; f < n; f++) {
        int lo = INT32_MAX, hi = -1;
        for (int sl = 0; sl < nv; sl++) {
          const int q = regPos(kFK[fk][sl], h->fvars[fk][f * nv + sl]);
          if (q >= 0) lo = std::min(lo, q), hi = std::max(hi, q);
        }
        for (int sl = 0; sl < nv; sl++) {
          const int q = regPos(kFK[fk][sl], h->fvars[fk][f * nv + sl]);
          if (q >= 0) hiP[ord[q]] = std::max(hiP[ord[q]], hi), loP[ord[q]] = std::min(loP[ord[q]], lo);
        }
      }
    }
  }
  std::vector<int> tdims(nRV);
  for (int r = 0; r < nRV; r++) tdims[r] = tdimOf(red[r].first, red[r].second);
  int64_t leafDims = 1024;
  // cut: the thinnest separator -- the left variables coupled across the cut, or the right ones --
  // among the cuts within +-cutWin of the part's median (config C: 954k -> 701k tile contributions,
  // 110 -> 89 levels against the median cut with left separators; wider windows unbalance the parts:
  // 0.1: 746k, 0.25: 880k).  VIBA_ND_CUTWIN=0: the round-1 order, the median cut with left separators
  // (tests/test_ordering_gpu.py); an imbalance penalty was tried and dropped
  double cutWin = 0.05;
  if (const char* e = getenv("VIBA_ND_CUTWIN")) cutWin = std::max(0.0, std::min(0.45, atof(e)));
  const bool sepRight = cutWin > 0.0;
  const double cutBal = 0.0;  // imbalance weight
  if (const char* e = getenv("VIBA_ND_LEAF")) leafDims = std::max<int64_t>(64, atoll(e));
  std::vector<int> nord;             // final order (registration indices)
  std::vector<size_t> partBegin;     // parts (tile-aligned) in nord
  // partitioned factorization (vb_set_partition, world = 2^k): the parts below depth k belong to
  // the subtree (= rank) they descend from; the separators above, and any part emitted there, are
  // ROOT parts (factored by rank 0)
  const int world = h->partWorld;
  const bool parted = h->partSet;
  int partK = 0;
  while ((1 << partK) < world) partK++;
  // world 1: the top separator is still the ROOT part, both subtrees below it are rank 0's (so a
  // one-rank partitioned run takes every exchange of the protocol, e.g. over RCCL with one GPU)
  if (parted && partK == 0) partK = 1;
  std::vector<int> partOwner;
  std::function<void(std::vector<int>&, int, int, int)> dissect = [&](std::vector<int>& vs, int depth, int sub,
                                                                      int own) {
    if (own < 0 && depth == partK) own = sub % world;
    int64_t dims = 0;
    for (int r : vs) dims += tdims[r];
    // a separator above depth k is ROOT; an undivided set above depth k is a whole subtree, so it
    // goes to the first rank of the ranks below it
    auto emit = [&](std::vector<int>& part, bool separator) {
      if (part.empty()) return;
      partBegin.push_back(nord.size());
      partOwner.push_back(own >= 0 ? own : separator ? world : (sub << (partK - depth)) % world);
      nord.insert(nord.end(), part.begin(), part.end());
    };
    if (dims <= leafDims || vs.size() < 4) return emit(vs, false);
    int64_t acc = 0;
    size_t k = 0;
    while (k < vs.size() && acc + tdims[vs[k]] <= dims / 2) acc += tdims[vs[k++]];
    if (k == 0 || k >= vs.size()) return emit(vs, false);
    bool right = false;
    if (cutWin > 0.0) {
      const size_t w = (size_t)(cutWin * (double)vs.size());
      const size_t k0 = k > w + 1 ? k - w : 1, k1 = std::min(vs.size() - 1, k + w);
      double best = 1e300;
      size_t bk = k;
      bool br = false;
      // separator widths of every candidate cut c (vs ascends in tp): sl(c) = dims of the i < c with
      // hiP >= tp(c), sr(c) = dims of the i >= c with loP < tp(c); two sweeps over Fenwick trees keyed
      // by time position, O(|vs| log nRV) per part instead of a rescan per candidate
      const size_t nc = k1 - k0 + 1;
      std::vector<int64_t> slC(nc, 0), srC(nc, 0), bit(nRV + 1, 0);
      auto bitAdd = [&](int pos, int64_t v) { for (int x = std::min(pos, nRV - 1) + 1; x <= nRV; x += x & -x) bit[x] += v; };
      auto bitSum = [&](int pos) { int64_t r = 0; for (int x = pos; x > 0; x -= x & -x) r += bit[x]; return r; };  // keys < pos
      {
        int64_t tot = 0;
        for (size_t i = 0; i < k0; i++) bitAdd(hiP[vs[i]], tdims[vs[i]]), tot += tdims[vs[i]];
        for (size_t c = k0; c <= k1; c++) {
          slC[c - k0] = tot - bitSum(tp[vs[c]]);
          bitAdd(hiP[vs[c]], tdims[vs[c]]), tot += tdims[vs[c]];
        }
      }
      if (sepRight) {
        std::fill(bit.begin(), bit.end(), 0);
        for (size_t i = vs.size(); i-- > k1 + 1;) bitAdd(loP[vs[i]], tdims[vs[i]]);
        for (size_t c = k1 + 1; c-- > k0;) {
          bitAdd(loP[vs[c]], tdims[vs[c]]);
          srC[c - k0] = bitSum(tp[vs[c]]);
        }
      }
      int64_t accC = 0;
      for (size_t i = 0; i < k0; i++) accC += tdims[vs[i]];
      for (size_t c = k0; c <= k1; accC += tdims[vs[c]], c++) {
        const int64_t sl = slC[c - k0], sr = srC[c - k0];
        const double pen = cutBal * (double)std::llabs(2 * accC - dims) * 0.5;  // imbalance, in dims
        if (sl + pen < best) best = sl + pen, bk = c, br = false;
        if (sepRight && sr + pen < best) best = sr + pen, bk = c, br = true;
      }
      k = bk, right = br;
    }
    const int cut = tp[vs[k]];
    std::vector<int> L, R, S;
    int64_t sd = 0;
    if (!right) {  // separator: the left variables coupled across the cut
      R.assign(vs.begin() + k, vs.end());
      for (size_t i = 0; i < k; i++) {
        if (hiP[vs[i]] >= cut) S.push_back(vs[i]), sd += tdims[vs[i]];
        else L.push_back(vs[i]);
      }
    } else {  // the right variables coupled across it
      L.assign(vs.begin(), vs.begin() + k);
      for (size_t i = k; i < vs.size(); i++) {
        if (loP[vs[i]] < cut) S.push_back(vs[i]), sd += tdims[vs[i]];
        else R.push_back(vs[i]);
      }
    }
    if (L.empty() || R.empty() || 2 * sd > dims) return emit(vs, false);  // no useful separator
    dissect(L, depth + 1, 2 * sub, own);
    dissect(R, depth + 1, 2 * sub + 1, own);
    emit(S, true);
  };
  {
    std::vector<int> all(ord.begin(), ord.end());
    dissect(all, 0, 0, -1);
  }
  h->rvKind.resize(nRV), h->rvHandle.resize(nRV), h->rvDim.resize(nRV), h->rvOff.resize(nRV + 1);
  std::vector<int64_t> padRows;
  int64_t off = 0, nRedReal = 0;
  {
    size_t pi = 0;
    for (int i = 0; i < nRV; i++) {
      if (pi < partBegin.size() && partBegin[pi] == (size_t)i) {  // parts start on a tile boundary
        const int64_t a = (off + TS - 1) / TS * TS;
        for (int64_t r = off; r < a; r++) padRows.push_back(r);
        off = a, pi++;
      }
      const auto [kind, hh] = red[nord[i]];
      h->rvKind[i] = kind, h->rvHandle[i] = hh, h->rvDim[i] = tdims[nord[i]], h->rvOff[i] = off;
      off += h->rvDim[i], nRedReal += h->rvDim[i];
      redOf[kind][hh] = i;
    }
    const int64_t a = (off + TS - 1) / TS * TS;
    for (int64_t r = off; r < a; r++) padRows.push_back(r);
  }
  h->rvOff[nRV] = off;
  const int64_t nRed = off;
  // the small-factor assembly packs a reduced row with 5 more bits into an int32 (factors.hip)
  if (nRed >= ((int64_t)1 << 26)) return fail(VB_E_ARG, "reduced system order must stay below 2^26");
  // owner of every tile column (parts start on tile boundaries; trailing padding joins the last part)
  {
    const int64_t nTc = (nRed + TS - 1) / TS;
    h->colOwner.assign(nTc, (int8_t)(partOwner.empty() ? 0 : partOwner.back()));
    size_t pi = 0;
    for (int i = 0; i < nRV; i++) {
      while (pi + 1 < partBegin.size() && partBegin[pi + 1] <= (size_t)i) pi++;
      const int64_t t0 = h->rvOff[i] / TS, t1 = (h->rvOff[i] + h->rvDim[i] - 1) / TS;
      for (int64_t t = t0; t <= t1; t++) h->colOwner[t] = (int8_t)partOwner[pi];
    }
    // (parts start on tile boundaries and a part's alignment padding shares a tile with its last
    // rows, so every tile column holds variables of exactly one part)
  }
  // partition mode: landmarks (and constant-point observations) go to the rank whose subtree
  // interior they touch -- never two (a variable coupled across a cut is in that cut's separator);
  // those touching only ROOT columns go to rank 0.  Landmarks are renumbered so every rank's are
  // contiguous (stable: time order within a rank).
  auto redOwner = [&](int kind, int32_t hh) -> int {
    if (hh < 0 || kind == 8 || redOf[kind][hh] < 0) return -1;
    const int i = redOf[kind][hh];
    return h->colOwner[h->rvOff[i] / TS];
  };
  auto obsOwner = [&](int64_t f) {
    const int32_t* v = &h->fvars[0][f * 5];
    const int os[4] = {redOwner(1, v[1]), redOwner(5, v[2]), redOwner(4, v[3]), h->fint[0][f] >= 0 ? redOwner(2, v[4]) : -1};
    for (int o : os)
      if (o >= 0 && o < world) return o;
    return 0;  // ROOT columns only (or none): rank 0
  };
  std::vector<int> lmRank(nPts, 0);
  if (parted) {
    const int64_t nv0 = (int64_t)h->fint[0].size();
    std::vector<int> lmOwn(nPts, -1);
    for (int64_t f = 0; f < nv0; f++) {
      const int l = lmOf[h->fvars[0][f * 5]];
      if (l < 0) continue;
      lmOwn[l] = std::max(lmOwn[l], obsOwner(f));
    }
    std::vector<int32_t> byRank(nPts);
    std::iota(byRank.begin(), byRank.end(), 0);
    for (int64_t l = 0; l < nPts; l++) lmRank[l] = std::max(0, lmOwn[l]);
    std::stable_sort(byRank.begin(), byRank.end(), [&](int32_t a, int32_t b) { return lmRank[a] < lmRank[b]; });
    std::vector<int32_t> newIdx(nPts);
    for (int64_t i = 0; i < nPts; i++) newIdx[byRank[i]] = (int32_t)i;
    for (auto& x : lmOf)
      if (x >= 0) x = newIdx[x];
    std::vector<int> r2(nPts);
    for (int64_t l = 0; l < nPts; l++) r2[newIdx[l]] = lmRank[l];
    lmRank.swap(r2);
  }
  h->nRedReal = nRedReal, h->nParts = (int64_t)partBegin.size();
  d.nRV = nRV, d.nRed = nRed, d.nPts = nPts;
  h->nParams = nPts + nRV;
  h->order = nPts * 3 + nRedReal;
  if (upload(&h->padRowsD, padRows)) return VB_E_HIP;
  h->nPadRows = (int64_t)padRows.size();

  // ---------------- visual observations, sorted by landmark (constant-point obs at the end)
  const int64_t nObs = (int64_t)h->fint[0].size();
  std::vector<int64_t> perm(nObs);
  std::iota(perm.begin(), perm.end(), 0);
  auto lmKey = [&](int64_t f) -> int64_t {
    const int l = lmOf[h->fvars[0][f * 5]];
    return l < 0 ? (parted ? INT64_MAX - world + obsOwner(f) : INT64_MAX) : l;
  };
  std::stable_sort(perm.begin(), perm.end(), [&](int64_t a, int64_t b) { return lmKey(a) < lmKey(b); });
  d.nObs = nObs;
  d.nObsPad = ((nObs + 255) / 256) * 256;
  std::vector<int32_t> obPose(nObs), obExtr(nObs), obIntr(nObs), obVel(nObs), obRS(nObs), obPt(nObs);
  std::vector<int32_t> obRed(nObs * 4, -1), obCol(nObs * 4, -1);
  std::vector<double> obC(nObs * 6);
  std::vector<int64_t> lmObs(nPts + 1, 0);
  for (int64_t i = 0; i < nObs; i++) {
    const int64_t f = perm[i];
    const int32_t* v = &h->fvars[0][f * 5];
    obPt[i] = v[0], obPose[i] = v[1], obExtr[i] = v[2], obIntr[i] = v[3];
    obRS[i] = h->fint[0][f];
    obVel[i] = obRS[i] >= 0 ? v[4] : 0;
    if (obRS[i] >= h->nRS) return fail(VB_E_ARG, "visual factor references an unknown RS table");
    if (obRS[i] >= 0 && (v[4] < 0 || v[4] >= d.nvar[2])) return fail(VB_E_ARG, "RS visual factor needs a velocity");
    obRed[i * 4 + 0] = redOf[1][v[1]];
    obRed[i * 4 + 1] = redOf[5][v[2]];
    obRed[i * 4 + 2] = redOf[4][v[3]];
    obRed[i * 4 + 3] = obRS[i] >= 0 ? redOf[2][v[4]] : -1;
    std::copy(&h->fconst[0][f * 6], &h->fconst[0][f * 6] + 6, &obC[i * 6]);
    const int l = lmOf[v[0]];
    if (l >= 0) lmObs[l + 1]++;
  }
  for (int64_t l = 0; l < nPts; l++) lmObs[l + 1] += lmObs[l];
  h->nLmObs = lmObs[nPts];
  // landmark blocks D(l)
  std::vector<int64_t> lmBlk(nPts + 1, 0), lmY(nPts + 1, 0);
  std::vector<int32_t> blkRed, blkCol;
  std::vector<int32_t> tmp;
  for (int64_t l = 0; l < nPts; l++) {
    tmp.clear();
    for (int64_t o = lmObs[l]; o < lmObs[l + 1]; o++)
      for (int s = 0; s < 4; s++)
        if (obRed[o * 4 + s] >= 0) tmp.push_back(obRed[o * 4 + s]);
    std::sort(tmp.begin(), tmp.end());
    tmp.erase(std::unique(tmp.begin(), tmp.end()), tmp.end());
    int32_t col = 0;
    for (int32_t r : tmp) {
      blkRed.push_back(r);
      blkCol.push_back(col);
      col += h->rvDim[r];
    }
    lmBlk[l + 1] = (int64_t)blkRed.size();
    lmY[l + 1] = lmY[l] + 3 * (int64_t)col;
    for (int64_t o = lmObs[l]; o < lmObs[l + 1]; o++)
      for (int s = 0; s < 4; s++) {
        const int32_t r = obRed[o * 4 + s];
        if (r < 0) continue;
        const int64_t q = std::lower_bound(blkRed.begin() + lmBlk[l], blkRed.begin() + lmBlk[l + 1], r) - blkRed.begin();
        obCol[o * 4 + s] = (blkCol[q] << 5) | h->rvDim[r];  // panel column and width (<= 17) in one word
      }
  }
  // reduced row of every landmark panel column
  std::vector<int32_t> pcRow(lmY[nPts] / 3);
  d.nYcol = lmY[nPts] / 3;
  for (int64_t l = 0; l < nPts; l++)
    for (int64_t b = lmBlk[l]; b < lmBlk[l + 1]; b++) {
      const int32_t r = blkRed[b];
      for (int j = 0; j < h->rvDim[r]; j++) pcRow[lmY[l] / 3 + blkCol[b] + j] = (int32_t)(h->rvOff[r] + j);
    }
  // panel column -> landmark block, landmark block -> its observation slots (landmark_kernel)
  std::vector<int32_t> pcBlk(lmY[nPts] / 3);
  std::vector<int64_t> bxStart(blkRed.size() + 1, 0);
  std::vector<int32_t> bxEnt;
  {
    for (int64_t l = 0; l < nPts; l++)
      for (int64_t b = lmBlk[l]; b < lmBlk[l + 1]; b++)
        for (int j = 0; j < h->rvDim[blkRed[b]]; j++) pcBlk[lmY[l] / 3 + blkCol[b] + j] = (int32_t)b;
    auto blockOf = [&](int64_t l, int64_t o, int s) {
      return std::lower_bound(blkRed.begin() + lmBlk[l], blkRed.begin() + lmBlk[l + 1], obRed[o * 4 + s]) - blkRed.begin();
    };
    for (int64_t l = 0; l < nPts; l++)
      for (int64_t o = lmObs[l]; o < lmObs[l + 1]; o++)
        for (int s = 0; s < 4; s++)
          if (obRed[o * 4 + s] >= 0) bxStart[blockOf(l, o, s) + 1]++;
    for (size_t b = 0; b < blkRed.size(); b++) bxStart[b + 1] += bxStart[b];
    bxEnt.resize(bxStart[blkRed.size()]);
    std::vector<int64_t> fb(bxStart.begin(), bxStart.end() - 1);
    if (nObs >= (int64_t(1) << 29)) return fail(VB_E_ARG, "too many visual observations (2^29)");
    for (int64_t l = 0; l < nPts; l++)
      for (int64_t o = lmObs[l]; o < lmObs[l + 1]; o++)
        for (int s = 0; s < 4; s++)
          if (obRed[o * 4 + s] >= 0) bxEnt[fb[blockOf(l, o, s)]++] = (int32_t)((o << 2) | s);
  }
  // incidence lists O(X), L(X)
  std::vector<int64_t> oxStart(nRV + 1, 0), lxStart(nRV + 1, 0);
  for (int64_t o = 0; o < nObs; o++)
    for (int s = 0; s < 4; s++)
      if (obRed[o * 4 + s] >= 0) oxStart[obRed[o * 4 + s] + 1]++;
  for (int64_t b = 0; b < (int64_t)blkRed.size(); b++) lxStart[blkRed[b] + 1]++;
  for (int i = 0; i < nRV; i++) oxStart[i + 1] += oxStart[i], lxStart[i + 1] += lxStart[i];
  std::vector<int32_t> oxObs(oxStart[nRV]), oxSlot(oxStart[nRV]), lxLm(lxStart[nRV]), lxCol(lxStart[nRV]);
  {
    std::vector<int64_t> fo(oxStart.begin(), oxStart.end() - 1), fl(lxStart.begin(), lxStart.end() - 1);
    for (int64_t o = 0; o < nObs; o++)
      for (int s = 0; s < 4; s++) {
        const int32_t r = obRed[o * 4 + s];
        if (r < 0) continue;
        oxObs[fo[r]] = (int32_t)o, oxSlot[fo[r]] = s, fo[r]++;
      }
    for (int64_t l = 0; l < nPts; l++)
      for (int64_t b = lmBlk[l]; b < lmBlk[l + 1]; b++) {
        const int32_t r = blkRed[b];
        lxLm[fl[r]] = (int32_t)l, lxCol[fl[r]] = blkCol[b], fl[r]++;
      }
  }
  // ---------------- this handle's landmark shard
  if (parted) {  // partition mode: this rank's landmarks and constant-point observations
    const int me = h->partRank;
    int64_t a = 0;
    while (a < nPts && lmRank[a] < me) a++;
    int64_t b = a;
    while (b < nPts && lmRank[b] == me) b++;
    h->lmBegin = a, h->lmEnd = b, h->isRoot = me == 0;
  }
  if (h->lmEnd < 0) h->lmBegin = 0, h->lmEnd = nPts;
  if (h->lmBegin < 0 || h->lmEnd > nPts || h->lmBegin > h->lmEnd) return fail(VB_E_ARG, "bad landmark shard range");
  d.lmB = h->lmBegin, d.lmE = h->lmEnd, d.root = h->isRoot ? 1 : 0;
  {  // landmark lists by panel width (schur.hip landmark_stage_kernel)
    std::vector<int32_t> small, big;
    int64_t bigCols = 0;
    for (int64_t l = h->lmBegin; l < h->lmEnd; l++) {
      const int64_t nc = (lmY[l + 1] - lmY[l]) / 3;
      if (nc <= kLmSmallCols) small.push_back((int32_t)l);
      else big.push_back((int32_t)l), bigCols = std::max(bigCols, nc);
    }
    d.nLmSmall = (int64_t)small.size(), d.nLmBig = (int64_t)big.size(), d.lmBigCols = (int32_t)bigCols;
    small.insert(small.end(), big.begin(), big.end());
    if (upload(&d.lmList, small)) return VB_E_HIP;
  }
  d.obB = lmObs[h->lmBegin], d.obE = lmObs[h->lmEnd], d.obFree = lmObs[nPts];
  // constant-point observations of this handle: [fB, fE) (the root's whole tail unless partitioned)
  d.fB = d.obFree, d.fE = h->isRoot ? nObs : d.obFree;
  if (parted) {
    int64_t a = d.obFree;
    while (a < nObs && obsOwner(perm[a]) < h->partRank) a++;
    int64_t b = a;
    while (b < nObs && obsOwner(perm[b]) == h->partRank) b++;
    d.fB = a, d.fE = b;
  }
  // ---------------- couplings: row ends and the tile pattern
  const int32_t nT = (int32_t)((nRed + TS - 1) / TS);
  d.nT = nT;
  std::vector<int64_t> rowEnd(nRV);
  for (int i = 0; i < nRV; i++) rowEnd[i] = h->rvOff[i] + h->rvDim[i];
  std::vector<uint8_t> pat((size_t)nT * nT, 0);
  auto coupleBlocks = [&](int a, int b) {  // reduced ids; a, b any order
    if (h->rvOff[a] < h->rvOff[b]) std::swap(a, b);
    rowEnd[b] = std::max(rowEnd[b], h->rvOff[a] + h->rvDim[a]);
    const int64_t r0 = h->rvOff[a] / TS, r1 = (h->rvOff[a] + h->rvDim[a] - 1) / TS;
    const int64_t c0 = h->rvOff[b] / TS, c1 = (h->rvOff[b] + h->rvDim[b] - 1) / TS;
    for (int64_t I = r0; I <= r1; I++)
      for (int64_t J = c0; J <= c1; J++)
        if (I >= J) pat[I * nT + J] = 3;  // 3: written by a direct term (damping, visual groups, small factors)
  };
  for (int i = 0; i < nRV; i++) coupleBlocks(i, i);
  for (int64_t o = 0; o < nObs; o++)
    for (int s = 0; s < 4; s++)
      for (int t = 0; t <= s; t++)
        if (obRed[o * 4 + s] >= 0 && obRed[o * 4 + t] >= 0) coupleBlocks(obRed[o * 4 + s], obRed[o * 4 + t]);
  for (int64_t l = 0; l < nPts; l++) {
    const int64_t b0 = lmBlk[l], b1 = lmBlk[l + 1];
    if (b1 == b0) continue;
    // row end: the suffix partner with the largest offset is the last block
    const int last = blkRed[b1 - 1];
    for (int64_t b = b0; b < b1; b++)
      rowEnd[blkRed[b]] = std::max(rowEnd[blkRed[b]], h->rvOff[last] + h->rvDim[last]);
    // tile pattern over the distinct tiles touched
    std::vector<int64_t> tl;
    for (int64_t b = b0; b < b1; b++) {
      const int r = blkRed[b];
      for (int64_t t = h->rvOff[r] / TS; t <= (h->rvOff[r] + h->rvDim[r] - 1) / TS; t++) tl.push_back(t);
    }
    std::sort(tl.begin(), tl.end());
    tl.erase(std::unique(tl.begin(), tl.end()), tl.end());
    for (size_t a = 0; a < tl.size(); a++)
      for (size_t b = 0; b <= a; b++) {
        uint8_t& q = pat[tl[a] * nT + tl[b]];
        q = q ? q : 1;  // 1: landmark (Schur) terms only
      }
  }
  for (int fk = 1; fk < 14; fk++) {
    const int nv = kNumVars[fk];
    const int64_t n = (int64_t)h->fint[fk].size();
    for (int64_t f = 0; f < n; f++)
      for (int s = 0; s < nv; s++)
        for (int t = 0; t <= s; t++) {
          const int ks_ = kFK[fk][s], kt = kFK[fk][t];
          const int hs = h->fvars[fk][f * nv + s], ht = h->fvars[fk][f * nv + t];
          if (hs < 0 || ht < 0 || ks_ == 8 || kt == 8 || ks_ == 0 || kt == 0) continue;
          if (redOf[ks_][hs] < 0 || redOf[kt][ht] < 0) continue;
          coupleBlocks(redOf[ks_][hs], redOf[kt][ht]);
        }
  }
  // symbolic tile Cholesky (fill)
  for (int32_t J = 0; J < nT; J++) {
    std::vector<int32_t> rows;
    for (int32_t I = J + 1; I < nT; I++)
      if (pat[(size_t)I * nT + J]) rows.push_back(I);
    for (size_t a = 0; a < rows.size(); a++)
      for (size_t b = 0; b <= a; b++) {
        uint8_t& q = pat[(size_t)rows[a] * nT + rows[b]];
        q = q ? q : 2;  // 2: fill (zero in S; the PCG product skips it)
      }
  }
  std::vector<int32_t> tileIdx((size_t)nT * nT, -1);
  h->tileFill.clear();
  std::vector<uint8_t> tileDirect;  // per tile: a direct term (not only landmark products) writes it
  h->colStart.assign(nT + 1, 0);
  h->colTilesH.clear(), h->colRowsH.clear();
  int64_t nTiles = 0;
  for (int32_t J = 0; J < nT; J++) {
    for (int32_t I = J; I < nT; I++)
      if (I == J || pat[(size_t)I * nT + J]) {
        tileIdx[(size_t)I * nT + J] = (int32_t)nTiles;
        h->tileFill.push_back(I != J && pat[(size_t)I * nT + J] == 2 ? 1 : 0);
        tileDirect.push_back(I == J || pat[(size_t)I * nT + J] == 3 ? 1 : 0);
        h->colTilesH.push_back((int32_t)nTiles++);
        h->colRowsH.push_back(I);
      }
    h->colStart[J + 1] = (int64_t)h->colTilesH.size();
  }
  d.nTiles = nTiles;
  // ---------------- Schur assembly work by target tile (this shard's landmarks and observations)
  {
    std::vector<TileWork> works;
    // landmark entries
    struct Seg { int64_t t, c0, c1; };
    std::vector<Seg> sg;
    auto segments = [&](int64_t l) {  // panel columns split by the tile their reduced row falls in
      sg.clear();
      const int64_t cb = lmY[l] / 3, nc = (lmY[l + 1] - lmY[l]) / 3;
      for (int64_t c = 0; c < nc; c++) {
        const int64_t t = pcRow[cb + c] / TS;
        if (sg.empty() || sg.back().t != t) sg.push_back({t, c, c + 1});
        else sg.back().c1 = c + 1;
      }
    };
    std::vector<int64_t> tcnt(nTiles + 1, 0);
    for (int64_t l = h->lmBegin; l < h->lmEnd; l++) {
      segments(l);
      for (size_t a = 0; a < sg.size(); a++)
        for (size_t b = 0; b <= a; b++) {
          const int32_t ti = tileIdx[(size_t)sg[a].t * nT + sg[b].t];
          if (ti < 0) return fail(VB_E_STATE, "internal: landmark tile outside the symbolic structure");
          tcnt[ti + 1]++;
        }
    }
    for (int64_t t = 0; t < nTiles; t++) tcnt[t + 1] += tcnt[t];
    std::vector<TileEnt> ents(tcnt[nTiles]);
    {
      std::vector<int64_t> cur(tcnt.begin(), tcnt.end() - 1);
      for (int64_t l = h->lmBegin; l < h->lmEnd; l++) {
        segments(l);
        const int64_t cb = lmY[l] / 3;
        for (size_t a = 0; a < sg.size(); a++)
          for (size_t b = 0; b <= a; b++) {
            const int32_t ti = tileIdx[(size_t)sg[a].t * nT + sg[b].t];
            TileEnt& e = ents[cur[ti]++];
            e.colI = (uint32_t)(cb + sg[a].c0), e.nI = (uint16_t)(sg[a].c1 - sg[a].c0);
            e.colJ = (uint32_t)(cb + sg[b].c0), e.nJ = (uint16_t)(sg[b].c1 - sg[b].c0);
            e.lm = (uint32_t)l;
            e.maskI = e.maskJ = 0;
            for (int64_t c = sg[a].c0; c < sg[a].c1; c++) e.maskI |= 1ull << (pcRow[cb + c] % TS);
            for (int64_t c = sg[b].c0; c < sg[b].c1; c++) e.maskJ |= 1ull << (pcRow[cb + c] % TS);
          }
      }
    }
    // entries of a tile in runs of identical (maskI, maskJ) (solver.hip schur_run4_kernel), by
    // landmark within a run
    for (int64_t t = 0; t < nTiles; t++)
      std::sort(ents.begin() + tcnt[t], ents.begin() + tcnt[t + 1], [](const TileEnt& a, const TileEnt& b) {
        if (a.maskI != b.maskI) return a.maskI < b.maskI;
        if (a.maskJ != b.maskJ) return a.maskJ < b.maskJ;
        return a.lm < b.lm;
      });
    // observation groups: this shard's observations by their 4 reduced blocks (rig, camera)
    std::vector<int32_t> gobs;
    for (int64_t o = 0; o < nObs; o++)
      if ((o >= d.obB && o < d.obE) || (o >= d.fB && o < d.fE)) gobs.push_back((int32_t)o);
    auto gkey = [&](int32_t o, int s) { return obRed[(int64_t)o * 4 + s]; };
    std::stable_sort(gobs.begin(), gobs.end(), [&](int32_t a, int32_t b) {
      for (int s = 0; s < 4; s++)
        if (gkey(a, s) != gkey(b, s)) return gkey(a, s) < gkey(b, s);
      return false;
    });
    std::vector<int64_t> gstart;
    std::vector<int32_t> gred;
    int64_t tlo = INT64_MAX, thi = -1;
    std::vector<uint8_t> touched(nTiles, 0);
    for (size_t i = 0; i < gobs.size(); i++) {
      bool fresh = i == 0;
      for (int s = 0; s < 4 && !fresh; s++) fresh = gkey(gobs[i], s) != gkey(gobs[i - 1], s);
      if (!fresh) continue;
      gstart.push_back((int64_t)i);
      for (int s = 0; s < 4; s++) gred.push_back(gkey(gobs[i], s));
      for (int s = 0; s < 4; s++)  // tiles the group touches (for the shard's tile band)
        for (int t = 0; t <= s; t++) {
          int32_t A = gkey(gobs[i], s), B = gkey(gobs[i], t);
          if (A < 0 || B < 0) continue;
          if (h->rvOff[A] < h->rvOff[B]) std::swap(A, B);
          for (int64_t I = h->rvOff[A] / TS; I <= (h->rvOff[A] + h->rvDim[A] - 1) / TS; I++)
            for (int64_t J = h->rvOff[B] / TS; J <= std::min<int64_t>(I, (h->rvOff[B] + h->rvDim[B] - 1) / TS); J++) {
              const int32_t tt = tileIdx[(size_t)I * nT + J];
              if (tt >= 0) tlo = std::min<int64_t>(tlo, tt), thi = std::max<int64_t>(thi, tt), touched[tt] = 1;
            }
        }
    }
    gstart.push_back((int64_t)gobs.size());
    d.nGroups = (int64_t)gred.size() / 4;
    if (upload(&d.grpStart, gstart) || upload(&d.grpObs, gobs) || upload(&d.grpRed, gred)) return VB_E_HIP;
    // work items: a tile's landmark entries in near-equal chunks of at most kChunkLm; `kind` = 1 when
    // the tile is split over several items (fp64 atomics), else the item owns the tile (plain RMW).
    // Items run in tile-column order (xcd_block hands each XCD a contiguous range of them).
    const int64_t kChunkLm = 256;
    std::vector<int32_t> itemsPerTile(nTiles, 0);
    for (int32_t J = 0; J < nT; J++)
      for (int64_t c = h->colStart[J]; c < h->colStart[J + 1]; c++) {
        const int32_t ti = h->colTilesH[c];
        const int64_t e0 = tcnt[ti], n = tcnt[ti + 1] - e0, nch = (n + kChunkLm - 1) / kChunkLm;
        for (int64_t k = 0; k < nch; k++) {
          TileWork w{};
          const int64_t s0 = n * k / nch, s1 = n * (k + 1) / nch;
          w.tile = ti, w.I = h->colRowsH[c], w.J = J, w.count = (int32_t)(s1 - s0);
          w.start = e0 + s0, w.kind = 0;
          works.push_back(w);
          itemsPerTile[ti]++;
          tlo = std::min<int64_t>(tlo, ti), thi = std::max<int64_t>(thi, ti), touched[ti] = 1;
        }
      }
    for (TileWork& w : works) w.kind = itemsPerTile[w.tile] > 1 ? 1 : 0;
    // (items by the median landmark of their entries instead of by tile column: 52.7 against 52.9 it/s, r05)
    // a tile written by exactly one Schur item and by no direct term is stored whole by that item (kind
    // 2: no read of the tile) and left out of the clear in vb_linearize (single handle; shards and
    // partitions clear their tile ranges and add); the clear covers the rest, by tile list
    if (!h->sharded && !h->partSet) {
      std::vector<int32_t> clr;
      for (TileWork& w : works)
        if (w.kind == 0 && !tileDirect[w.tile]) w.kind = 2;
      std::vector<uint8_t> stored(nTiles, 0);
      for (const TileWork& w : works)
        if (w.kind == 2) stored[w.tile] = 1;
      for (int64_t t = 0; t < nTiles; t++)
        if (!stored[t]) clr.push_back((int32_t)t);
      h->nClear = (int64_t)clr.size();
      if (upload(&h->clearTilesD, clr)) return VB_E_HIP;
    }
    // per item: its runs of identical (maskI, maskJ) and its tasks (run, chunk of <= kSchurCh landmarks,
    // kSchurTR compact block rows), dealt to the 4 waves longest-first by an MFMA + gather cost model and
    // kept in (run, chunk) order per wave, so a wave rebuilds its row maps only when its run changes
    // (schur_run4_kernel: no run scan, no per-run global mask reads, balanced waves)
    std::vector<uint64_t> runsH;
    std::vector<uint32_t> tasksH;
    for (TileWork& w : works) {
      const bool diag = w.I == w.J;
      std::vector<int> rs;
      for (int e = 0; e < w.count; e++) {
        const TileEnt& a = ents[w.start + e];
        if (e == 0 || a.maskI != ents[w.start + e - 1].maskI || a.maskJ != ents[w.start + e - 1].maskJ) rs.push_back(e);
      }
      rs.push_back(w.count);
      w.runFirst = (int32_t)(runsH.size() / 2), w.nRuns = (uint16_t)(rs.size() - 1);
      struct Tk {
        uint32_t code;
        double cost;
      };
      std::vector<Tk> tl;
      for (size_t r = 0; r + 1 < rs.size(); r++) {
        const uint64_t mI = ents[w.start + rs[r]].maskI, mJ = diag ? mI : ents[w.start + rs[r]].maskJ;
        runsH.push_back(mI), runsH.push_back(mJ);
        const int nbI = (__builtin_popcountll(mI) + 15) / 16, nbJ = (__builtin_popcountll(mJ) + 15) / 16;
        for (int c0 = rs[r]; c0 < rs[r + 1]; c0 += kSchurCh)
          for (int a0 = 0; a0 < nbJ; a0 += kSchurTR) {
            const int nl = std::min(kSchurCh, rs[r + 1] - c0), nr = std::min(kSchurTR, nbJ - a0);
            // plane groups of four landmarks (schur_task): three k-steps and two loads per operand block each
            const int ng = (nl + 3) / 4;
            int mf = 0;
            for (int i = 0; i < nr; i++)
              for (int b = 0; b < nbI; b++) mf += (!diag || a0 + i <= b) ? 1 : 0;
            const double cost = ng * (48.0 * mf + 6.0 * (nr + nbI)) + 6.0 * mf + 24.0 + (diag && a0 == 0 ? 6.0 * nl : 0.0);
            tl.push_back({(uint32_t)r | ((uint32_t)c0 << 8) | ((uint32_t)nl << 16) | ((uint32_t)a0 << 22), cost});
          }
      }
      std::stable_sort(tl.begin(), tl.end(), [](const Tk& a, const Tk& b) { return a.cost > b.cost; });
      std::vector<uint32_t> per[4];
      double load[4] = {0, 0, 0, 0};
      for (const Tk& t : tl) {
        const int k = (int)(std::min_element(load, load + 4) - load);
        load[k] += t.cost, per[k].push_back(t.code);
      }
      w.taskFirst = (int32_t)tasksH.size();
      for (int k = 0; k < 4; k++) {
        std::sort(per[k].begin(), per[k].end(), [](uint32_t a, uint32_t b) {
          return (a & 0xffffu) != (b & 0xffffu) ? (a & 0xffffu) < (b & 0xffffu) : a < b;  // run, chunk, row
        });
        w.wOff[k] = (uint16_t)(tasksH.size() - w.taskFirst);
        tasksH.insert(tasksH.end(), per[k].begin(), per[k].end());
      }
      w.wOff[4] = (uint16_t)(tasksH.size() - w.taskFirst);
    }
    if (getenv("VIBA_STATS")) {  // diagnostics: compact widths, MFMA padding, runs, tasks
      int64_t hI[5] = {0}, hJ[5] = {0}, nRun = 0, nTask = 0, runLm = 0;
      double useful = 0, issued = 0, issued4 = 0, gathered = 0, segBytes = 0;
      double nlHist[17] = {0}, kDense = 0, kGroup = 0, gDense = 0, gGroup = 0;
      auto bin = [](int n) { return n <= 4 ? 0 : n <= 8 ? 1 : n <= 16 ? 2 : n <= 32 ? 3 : 4; };
      for (const TileWork& w : works) {
        const bool diag = w.I == w.J;
        std::vector<int> rlen(w.nRuns, 0);
        for (int e = 0, k = -1; e < w.count; e++) {
          const TileEnt& a = ents[w.start + e];
          if (e == 0 || a.maskI != ents[w.start + e - 1].maskI || a.maskJ != ents[w.start + e - 1].maskJ) k++;
          rlen[k]++;
        }
        for (int r = 0; r < w.nRuns; r++) {
          const uint64_t mI = runsH[2 * ((size_t)w.runFirst + r)], mJ = runsH[2 * ((size_t)w.runFirst + r) + 1];
          const int nI = __builtin_popcountll(mI), nJ = __builtin_popcountll(mJ);
          const int nl = rlen[r];
          hI[bin(nI)]++, hJ[bin(nJ)]++, nRun++, runLm += nl;
          const double rows = 3.0 * nl;
          useful += 2.0 * rows * nI * nJ * (diag ? 0.5 : 1.0);
          const int nbI = (nI + 15) / 16, nbJ = (nJ + 15) / 16;
          issued += 2.0 * 4.0 * std::ceil(rows / 4.0) * 256.0 * nbI * nbJ * (diag ? 0.5 : 1.0);
          issued4 += 2.0 * 4.0 * std::ceil(rows / 4.0) * 16.0 * ((nI + 3) / 4) * ((nJ + 3) / 4) * (diag ? 0.5 : 1.0);
        }
        nTask += w.wOff[4];
        for (int t = 0; t < w.wOff[4]; t++) {  // gathered operand bytes: every k-step's NR + NBI 16-wide rows
          const uint32_t code = tasksH[(size_t)w.taskFirst + t];
          const int r = code & 255, nl = (code >> 16) & 63, a0 = (code >> 22) & 3;
          const uint64_t mI = runsH[2 * ((size_t)w.runFirst + r)], mJ = runsH[2 * ((size_t)w.runFirst + r) + 1];
          const int nbI = (__builtin_popcountll(mI) + 15) / 16, nbJ = (__builtin_popcountll(mJ) + 15) / 16;
          const int nr = std::min(kSchurTR, nbJ - a0);
          gathered += 4.0 * ((3 * nl + 3) / 4) * (nr + nbI) * 16 * sizeof(rec_t);
          // k-steps and gather instructions of the dense K mapping (3 rows per landmark, 4 per k-step) against a
          // plane-grouped one (each lane group one landmark's 3 planes over 3 k-steps, the remainder dense)
          int mf = 0;
          for (int i = 0; i < nr; i++)
            for (int b = 0; b < nbI; b++) mf += (!diag || a0 + i <= b) ? 1 : 0;
          const int ksD = (3 * nl + 3) / 4, ksG = 3 * (nl / 4) + (3 * (nl % 4) + 3) / 4;
          nlHist[std::min(nl, 16)] += 1.0, kDense += (double)ksD * mf, kGroup += (double)ksG * mf;
          gDense += (double)ksD * (nr + nbI), gGroup += (double)((nl / 4) * 2 + (3 * (nl % 4) + 3) / 4) * (nr + nbI);
        }
        for (int e = 0; e < w.count; e++) {  // the entries' Y segments once per item
          const TileEnt& a = ents[w.start + e];
          segBytes += 3.0 * (__builtin_popcountll(a.maskI) + (diag ? 0 : __builtin_popcountll(a.maskJ))) * sizeof(rec_t);
        }
      }
      fprintf(stderr,
              "[schur stats] items %zu runs %lld tasks %lld landmarks/run %.2f; nI <=4/8/16/32/64: %lld %lld %lld %lld "
              "%lld; nJ: %lld %lld %lld %lld %lld; GFLOP useful %.2f issued(16x16) %.2f issued(4x4) %.2f; GB gathered %.2f, "
              "entry segments %.2f\n",
              works.size(), (long long)nRun, (long long)nTask, (double)runLm / std::max<int64_t>(1, nRun),
              (long long)hI[0], (long long)hI[1], (long long)hI[2], (long long)hI[3], (long long)hI[4], (long long)hJ[0],
              (long long)hJ[1], (long long)hJ[2], (long long)hJ[3], (long long)hJ[4], useful * 1e-9, issued * 1e-9,
              issued4 * 1e-9, gathered * 1e-9, segBytes * 1e-9);
      fprintf(stderr, "[schur stats] tasks by landmarks:");
      for (int k = 1; k <= 16; k++) fprintf(stderr, " %d:%.0f", k, nlHist[k]);
      fprintf(stderr, "; MFMAs dense K %.3g, plane-grouped K %.3g; gather instructions dense %.3g, plane-grouped %.3g\n",
              kDense, kGroup, gDense, gGroup);
    }
    if (upload(&d.schurRuns, runsH) || upload(&d.schurTasks, tasksH)) return VB_E_HIP;
    // longest-first is unnecessary: chunks are bounded; keep column order (locality of Y / records)
    d.nTileWorks = (int64_t)works.size();
    h->nTileEnt = (int64_t)ents.size(), h->nObEnt = d.nGroups;
    if (upload(&d.tileWorks, works) || upload(&d.tileEnts, ents)) return VB_E_HIP;
    // tiles this shard's partial system can touch: the enclosing range (vb_shard_tile_range) and the
    // exact set (vb_shard_tiles: landmark and observation-group targets; the root, which also holds
    // the small factors and the damping, receives rather than sends)
    if (h->isRoot) h->tileFirst = 0, h->tileCount = nTiles;
    else if (thi < 0) h->tileFirst = 0, h->tileCount = 0;
    else h->tileFirst = tlo, h->tileCount = thi - tlo + 1;
    h->shardTiles.clear();
    if (!h->isRoot)
      for (int64_t t = 0; t < nTiles; t++)
        if (touched[t]) h->shardTiles.push_back((int32_t)t);
    if (!h->shardTiles.empty() &&
        (upload(&h->shardTilesD, h->shardTiles) || alloc0(&h->shardPack, h->shardTiles.size() * (size_t)TS * TS)))
      return VB_E_HIP;
  }
  h->rowStart.assign(nT + 1, 0);
  h->rowTilesH.clear(), h->rowColH.clear();
  for (int32_t J = 0; J < nT; J++) {
    for (int32_t K = 0; K < J; K++)
      if (tileIdx[(size_t)J * nT + K] >= 0) h->rowTilesH.push_back(tileIdx[(size_t)J * nT + K]), h->rowColH.push_back(K);
    h->rowStart[J + 1] = (int64_t)h->rowTilesH.size();
  }
  // ---------------- level schedule of the tile Cholesky: a column's level is one more than the
  // levels of the columns that update it (its row tiles); the columns of one level are independent
  // and are factored by one batched potrf, one batched trsm and one batched update launch
  {
    std::vector<int32_t> level(nT, 0);
    int32_t nLev = 0;
    for (int32_t J = 0; J < nT; J++) {
      for (int64_t i = h->rowStart[J]; i < h->rowStart[J + 1]; i++) level[J] = std::max(level[J], level[h->rowColH[i]] + 1);
      nLev = std::max(nLev, level[J] + 1);
    }
    std::vector<std::vector<int32_t>> cols(nLev);
    for (int32_t J = 0; J < nT; J++) cols[level[J]].push_back(J);
    if (getenv("VIBA_STATS")) {  // diagnostics: 2-column supernodes (J, J + 1) and their levels
      // pairable: J + 1 is J's first off-diagonal row (its parent) and J's other rows are all rows of J + 1
      std::vector<int8_t> pair(nT, 0);
      int64_t nPair = 0;
      for (int32_t J = 0; J + 1 < nT; J++) {
        if (pair[J] || (J > 0 && pair[J - 1] == 1)) continue;
        const int64_t a = h->colStart[J], b = h->colStart[J + 1], a2 = h->colStart[J + 1], b2 = h->colStart[J + 2];
        if (b - a < 2 || h->colRowsH[a + 1] != J + 1) continue;
        bool sub = true;
        int64_t q = a2 + 1;
        for (int64_t c = a + 2; c < b && sub; c++) {
          while (q < b2 && h->colRowsH[q] < h->colRowsH[c]) q++;
          sub = q < b2 && h->colRowsH[q] == h->colRowsH[c];
        }
        if (sub) pair[J] = 1, pair[J + 1] = 2, nPair++;
      }
      std::vector<int32_t> slev(nT, 0);
      int32_t nSl = 0;
      for (int32_t J = 0; J < nT; J++) {
        int32_t lv = 0;
        auto rowsOf = [&](int32_t X) {
          for (int64_t i = h->rowStart[X]; i < h->rowStart[X + 1]; i++) {
            const int32_t K = h->rowColH[i];
            if (pair[X] == 2 && K == X - 1) continue;  // internal to the supernode
            lv = std::max(lv, slev[K] + 1);
          }
        };
        if (pair[J] == 2) continue;
        rowsOf(J);
        if (pair[J] == 1) rowsOf(J + 1);
        slev[J] = lv;
        if (pair[J] == 1) slev[J + 1] = lv;
        nSl = std::max(nSl, lv + 1);
      }
      int64_t contrib = 0, internal = 0;
      for (int32_t K = 0; K < nT; K++) {
        const int64_t n = h->colStart[K + 1] - h->colStart[K];
        contrib += (n - 1) * n / 2;
        if (pair[K] == 1) internal += n - 1;  // targets in column K + 1 from K
      }
      fprintf(stderr, "[factor stats] tile columns %d levels %d; pairable 2-column supernodes %lld (%lld columns), "
                      "supernode levels %d; contributions %lld of which internal to pairs %lld\n",
              nT, nLev, (long long)nPair, (long long)(2 * nPair), nSl, (long long)contrib, (long long)internal);
      for (int32_t L = 0; L < nLev; L++) {
        int64_t c = 0, np = 0;
        for (int32_t J : cols[L]) {
          const int64_t n = h->rowStart[J + 1] - h->rowStart[J];
          c += n, np += pair[J] ? 1 : 0;
        }
        fprintf(stderr, "[factor stats] level %d columns %zu (paired %lld) row tiles %lld\n", L, cols[L].size(),
                (long long)np, (long long)c);
      }
    }
    const int64_t fanWgs = 3072;  // re-tuned for the thin-separator order (2048: -0.5%, 4096-8192: -0.3%)
    // Build one schedule.  colSel(J): columns factored here (potrf, trsm, solve diagonal tasks);
    // tgtSel(J): fan-in targets in column J; srcSel(K): contributions from column K; preSel(J): rows
    // whose x is known before the backward solve (their tile tasks run, they get no diagonal task).
    auto build = [&](Sched& S, auto colSel, auto tgtSel, auto srcSel, auto preSel) -> int {
      // contributions by target: column K's pair (qi >= qk) of off-diagonal tiles updates the target
      // tile (row qi, row qk) with L_{qi,K} L_{qk,K}^T (counting sort by target tile; sources in
      // level order, so every target's list runs from old to new columns)
      std::vector<int64_t> ccnt(nTiles + 1, 0);
      std::vector<int32_t> pairs;
      for (int pass = 0; pass < 2; pass++) {
        std::vector<int64_t> pos;
        if (pass == 1) {
          for (int64_t t = 0; t < nTiles; t++) ccnt[t + 1] += ccnt[t];
          pos.assign(ccnt.begin(), ccnt.end() - 1);
          pairs.assign(2 * (size_t)ccnt[nTiles], 0);
        }
        for (int32_t LK = 0; LK < nLev; LK++)
          for (int32_t K : cols[LK]) {
            if (!srcSel(K)) continue;
            const int64_t c0 = h->colStart[K], n = h->colStart[K + 1] - c0;
            for (int64_t qi = 1; qi < n; qi++)
              for (int64_t qk = 1; qk <= qi; qk++) {
                if (!tgtSel(h->colRowsH[c0 + qk])) continue;
                const int32_t t = tileIdx[(size_t)h->colRowsH[c0 + qi] * nT + h->colRowsH[c0 + qk]];
                if (t < 0) return fail(VB_E_STATE, "internal: symbolic fill incomplete");
                if (pass == 0) {
                  ccnt[t + 1]++;
                } else {
                  const int64_t at = pos[t]++;
                  pairs[2 * at] = h->colTilesH[c0 + qi], pairs[2 * at + 1] = h->colTilesH[c0 + qk];
                }
              }
          }
      }
      if (ccnt[nTiles] >= INT32_MAX) return fail(VB_E_STATE, "tile Cholesky too large (contribution count)");
      // per level: fan-in of the level's target tiles, then potrf of its diagonals, then trsm.  A
      // target's list is cut into near-equal chunks of at most `cs` contributions, cs chosen per
      // level so the launch has ~fanWgs workgroups (>= 4 contributions per chunk: one per wave)
      std::vector<int32_t> pT, pC, tD, tT, tC, tR, fan;
      S.lvP.assign(nLev + 1, 0), S.lvT.assign(nLev + 1, 0), S.lvU.assign(nLev + 1, 0);
      S.lvPF.assign(nLev + 1, 0);
      std::vector<int32_t> ptf, ptfDiag;
      for (int32_t L = 0; L < nLev; L++) {
        int64_t total = 0;
        for (int32_t J : cols[L])
          if (tgtSel(J))
            for (int64_t c = h->colStart[J]; c < h->colStart[J + 1]; c++) total += ccnt[h->colTilesH[c] + 1] - ccnt[h->colTilesH[c]];
        const int64_t cs = std::min<int64_t>(32, std::max<int64_t>(4, (total + fanWgs - 1) / fanWgs));
        for (int32_t J : cols[L]) {
          const int64_t c0 = h->colStart[J], n = h->colStart[J + 1] - c0;
          if (colSel(J)) {
            pT.push_back(h->colTilesH[c0]), pC.push_back(J);
            for (int64_t q = 1; q < n; q++)
              tD.push_back(h->colTilesH[c0]), tT.push_back(h->colTilesH[c0 + q]), tC.push_back(J), tR.push_back(h->colRowsH[c0 + q]);
          }
          if (!tgtSel(J)) continue;
          for (int64_t q = 0; q < n; q++) {
            const int32_t t = h->colTilesH[c0 + q];
            const int64_t b = ccnt[t], m = ccnt[t + 1] - b;
            if (m == 0) continue;
            const int64_t nch = (m + cs - 1) / cs;
            for (int64_t k = 0; k < nch; k++) {
              const int64_t s0 = b + m * k / nch, s1 = b + m * (k + 1) / nch;
              fan.insert(fan.end(), {t, (int32_t)s0, (int32_t)(s1 - s0), nch > 1 ? 1 : 0});
            }
          }
        }
        {  // longest chunks first within each XCD's range (the dispatcher hands them out in order, LPT): +0.9%
          const size_t u0 = (size_t)S.lvU[L];
          std::vector<std::array<int32_t, 4>> q((fan.size() / 4) - u0);
          for (size_t i = 0; i < q.size(); i++)
            for (int k = 0; k < 4; k++) q[i][k] = fan[4 * (u0 + i) + k];
          // within each XCD's contiguous range of the launch (solver.hip xcd_block)
          const size_t nq = q.size(), qq = nq / 8, rr = nq % 8;
          for (size_t x = 0, b0 = 0; x < 8; x++) {
            const size_t len = qq + (x < rr ? 1 : 0);
            std::stable_sort(q.begin() + b0, q.begin() + b0 + len, [](const auto& a, const auto& b) { return a[2] > b[2]; });
            b0 += len;
          }
          for (size_t i = 0; i < q.size(); i++)
            for (int k = 0; k < 4; k++) fan[4 * (u0 + i) + k] = q[i][k];
        }
        S.lvP[L + 1] = (int64_t)pT.size(), S.lvT[L + 1] = (int64_t)tT.size(), S.lvU[L + 1] = (int64_t)fan.size() / 4;
        if (h->ptFuseMax > 0 && S.lvP[L + 1] > S.lvP[L] && S.lvT[L + 1] - S.lvT[L] <= h->ptFuseMax)
          for (int32_t J : cols[L]) {
            if (!colSel(J)) continue;
            const int64_t c0 = h->colStart[J], n = h->colStart[J + 1] - c0;
            const int32_t dt = h->colTilesH[c0];
            if (n == 1) ptf.insert(ptf.end(), {dt, J, -1, -1, 1});
            for (int64_t q = 1; q < n; q++) ptf.insert(ptf.end(), {dt, J, h->colTilesH[c0 + q], h->colRowsH[c0 + q], q == 1 ? 1 : 0});
            ptfDiag.insert(ptfDiag.end(), {dt, J});
          }
        S.lvPF[L + 1] = (int64_t)ptf.size() / 5;
      }
      S.nLevels = nLev, S.nPairs = ccnt[nTiles];
      // fan-out solve task lists, by elimination level: every task of a level only waits on tasks of
      // earlier levels (or the level's own diagonal task listed first), so the waves' in-flight window
      // spans all independent subtrees of the level
      std::vector<int32_t> tf, tb, ef(nT, 0), eb(nT, 0), pre;
      for (int32_t L = 0; L < nLev; L++)
        for (int32_t K : cols[L]) {
          if (!colSel(K)) continue;
          tf.insert(tf.end(), {K, -1});
          for (int64_t c = h->colStart[K] + 1; c < h->colStart[K + 1]; c++) tf.insert(tf.end(), {K, (int32_t)c});
          for (int64_t c = h->rowStart[K]; c < h->rowStart[K + 1]; c++) ef[K] += srcSel(h->rowColH[c]) ? 1 : 0;
          eb[K] = (int32_t)(h->colStart[K + 1] - h->colStart[K] - 1);
        }
      for (int32_t L = nLev - 1; L >= 0; L--)
        for (int32_t J : cols[L]) {
          const bool own = colSel(J), known = preSel(J);
          if (own) tb.insert(tb.end(), {J, -1});
          if (known) pre.push_back(J);
          if (!own && !known) continue;
          for (int64_t c = h->rowStart[J]; c < h->rowStart[J + 1]; c++)
            if (colSel(h->rowColH[c])) tb.insert(tb.end(), {J, (int32_t)c});
        }
      S.nF = (int64_t)tf.size() / 2, S.nB = (int64_t)tb.size() / 2, S.nPreReady = (int64_t)pre.size();
      if (upload(&S.potrfTileD, pT) || upload(&S.potrfColD, pC) || upload(&S.trsmDiagD, tD) ||
          upload(&S.trsmTargetD, tT) || upload(&S.trsmColD, tC) || upload(&S.trsmRowD, tR) || upload(&S.updD, fan) ||
          upload(&S.fanPairsD, pairs) || upload(&S.tasksFD, tf) || upload(&S.tasksBD, tb) ||
          upload(&S.expFD, ef) || upload(&S.expBD, eb) || upload(&S.preReadyD, pre) || upload(&S.ptfD, ptf) ||
          upload(&S.ptfDiagD, ptfDiag))
        return VB_E_HIP;
      S.nPtfDiag = (int64_t)ptfDiag.size() / 2;
      if (S.nPtfDiag && !h->lscr && alloc0(&h->lscr, (size_t)nT * TS * TS)) return VB_E_HIP;
      S.built = true;
      return 0;
    };
    const int W = h->partWorld, me = h->partRank;
    auto any = [](int32_t) { return true; };
    auto none = [](int32_t) { return false; };
    if (!h->partSet) {
      if (int rc = build(h->sch[0], any, any, any, none)) return rc;
    } else {
      auto own = [&](int32_t J) { return h->colOwner[J] == me; };
      auto root = [&](int32_t J) { return h->colOwner[J] == W; };
      auto ownOrRoot = [&](int32_t J) { return h->colOwner[J] == me || h->colOwner[J] == W; };
      if (int rc = build(h->sch[0], own, ownOrRoot, own, root)) return rc;
      if (me == 0)
        if (int rc = build(h->sch[1], root, root, root, none)) return rc;
      for (int32_t J = 0; J < nT; J++)
        if (ownOrRoot(J)) {  // the only tiles this rank writes: cleared per linearize instead of the store
          const int64_t a = h->colStart[J], b = h->colStart[J + 1];
          if (!h->zeroRuns.empty() && h->zeroRuns.back().second == a) h->zeroRuns.back().second = b;
          else h->zeroRuns.push_back({a, b});
        }
      for (int32_t J = 0; J < nT; J++)
        if (root(J)) {
          h->rootRows.push_back(J);
          for (int64_t c = h->colStart[J]; c < h->colStart[J + 1]; c++) h->rootTiles.push_back(h->colTilesH[c]);
        }
      std::vector<int32_t> ownRows;
      for (int32_t J = 0; J < nT; J++)
        if (own(J) || (me == 0 && root(J))) ownRows.push_back(J);
      h->nOwnRows = (int64_t)ownRows.size();
      if (upload(&h->ownRowsD, ownRows) || alloc0(&h->ownPack, ownRows.size() * (size_t)TS + 1)) return VB_E_HIP;
      if (upload(&h->rootTilesD, h->rootTiles) || upload(&h->rootRowsD, h->rootRows) ||
          alloc0(&h->rootPack, h->rootTiles.size() * (size_t)TS * TS + 1) ||
          alloc0(&h->rowPack, h->rootRows.size() * (size_t)TS + 1))
        return VB_E_HIP;
    }
    h->nLevels = nLev;
    h->nPairs = h->sch[0].nPairs + h->sch[1].nPairs;
    if (h->useSn) {
      if (!h->partSet) {
        auto any = [](int32_t) { return true; };
        if (int rc = buildSupernodes(h, h->sn[0], tileIdx, nT, nTiles, any, any, any, h->snStreams)) return rc;
      } else {
        auto own = [&](int32_t J) { return h->colOwner[J] == me; };
        auto root = [&](int32_t J) { return h->colOwner[J] == W; };
        auto ownOrRoot = [&](int32_t J) { return h->colOwner[J] == me || h->colOwner[J] == W; };
        if (int rc = buildSupernodes(h, h->sn[0], tileIdx, nT, nTiles, own, ownOrRoot, own)) return rc;
        if (me == 0)
          if (int rc = buildSupernodes(h, h->sn[1], tileIdx, nT, nTiles, root, root, root)) return rc;
      }
    }
  }
  // ---------------- small factors (+ whitening square roots)
  for (int fk = 1; fk < 14; fk++) {
    SmallFactors& sf = d.sf[fk];
    sf.nv = kNumVars[fk];
    sf.n = (int64_t)h->fint[fk].size();
    const int extra = (fk >= 1 && fk <= 3) ? 81 : fk == 9 ? 36 : 0;
    sf.nc = kNumConsts[fk] + extra;
    std::vector<double> cs((size_t)sf.n * sf.nc);
    for (int64_t f = 0; f < sf.n; f++) {
      const double* src = &h->fconst[fk][f * kNumConsts[fk]];
      double* dst = &cs[f * sf.nc];
      std::copy(src, src + kNumConsts[fk], dst);
      if (fk >= 1 && fk <= 3) {
        if (!precisionChol(src + 11 + 207, 9, dst + 331)) return fail(VB_E_NUMERIC, "preintegration covariance not SPD");
      } else if (fk == 9) {
        psdSqrt(src + 7, 6, dst + 43);
      }
    }
    if (upload(&sf.vars, h->fvars[fk])) return VB_E_HIP;
    if (upload(&sf.consts, cs)) return VB_E_HIP;
    sf.stage = d.nSmallStage;
    d.nSmallStage += sf.n;
  }
  if ((h->isRoot || h->partSet) && d.nSmallStage > 0 &&
      (alloc0(&d.sJ, (size_t)d.nSmallStage * kSmallJ) || alloc0(&d.sE, (size_t)d.nSmallStage * kSmallE) ||
       alloc0(&d.sMeta, (size_t)d.nSmallStage * kSmallMeta)))
    return VB_E_HIP;
  // ---------------- --recompute-preint inputs (preint.hip)
  if (!h->piSrc.empty()) {
    const int nStreams = (int)std::max<size_t>(1, h->piT.size());
    std::vector<int64_t> off(nStreams + 1, 0), tAll;
    std::vector<double> vAll;
    for (int s = 0; s < nStreams; s++) {
      const std::vector<int64_t>& t = s == 0 ? h->imuT : h->piT[s];
      const std::vector<double>& v = s == 0 ? h->imuV : h->piV[s];
      tAll.insert(tAll.end(), t.begin(), t.end());
      vAll.insert(vAll.end(), v.begin(), v.end());
      off[s + 1] = (int64_t)tAll.size();
    }
    for (const PreintSrc& p : h->piSrc)
      if (p.imu < 0 || p.imu >= nStreams || off[p.imu + 1] == off[p.imu])
        return fail(VB_E_ARG, "preintegration source names an IMU without a measurement stream");
    std::vector<double> noise((size_t)nStreams * 6);
    for (int s = 0; s < nStreams; s++)
      for (int k = 0; k < 6; k++)
        noise[s * 6 + k] = 6 * s + k < (int)h->piNoise.size() ? h->piNoise[6 * s + k] : kDefaultImuNoise[k];
    h->piNoise = noise;
    PreintSrc* srcD = nullptr;
    int64_t *tD = nullptr, *offD = nullptr;
    double *vD = nullptr, *nD = nullptr;
    if (upload(&srcD, h->piSrc) || upload(&tD, tAll) || upload(&vD, vAll) || upload(&offD, off) || upload(&nD, noise))
      return VB_E_HIP;
    h->pi.src = srcD, h->pi.t = tD, h->pi.v = vD, h->pi.off = offD, h->pi.noise = nD;
    h->pi.n = (int64_t)h->piSrc.size();
  }
  // ---------------- uploads
  for (int k = 0; k < 9; k++) {
    if (upload(&d.var[k], h->data[k])) return VB_E_HIP;
    if (alloc0(&d.varBak[k], h->data[k].size())) return VB_E_HIP;
    if (upload(&d.redOf[k], redOf[k])) return VB_E_HIP;
  }
  if (upload(&d.rvKind, h->rvKind) || upload(&d.rvHandle, h->rvHandle) || upload(&d.rvDim, h->rvDim) ||
      upload(&d.rvOff, h->rvOff) || upload(&d.rvRowEnd, rowEnd))
    return VB_E_HIP;
  // visual_cost_kernel's order: the observations of each range the kernels run over ([obB, obE),
  // [fB, fE) and the gaps between them), stably partitioned into global-shutter then rolling-shutter,
  // so a wave takes one of the two evaluation paths instead of both
  std::vector<int32_t> costOrder(nObs);
  {
    std::vector<int64_t> cuts = {0, d.obB, d.obE, d.fB, d.fE, nObs};
    std::sort(cuts.begin(), cuts.end());
    for (size_t c = 0; c + 1 < cuts.size(); c++) {
      int64_t w = cuts[c];
      for (int pass = 0; pass < 2; pass++)
        for (int64_t i = cuts[c]; i < cuts[c + 1]; i++)
          if ((obRS[i] >= 0) == (pass == 1)) costOrder[w++] = (int32_t)i;
    }
  }
  if (upload(&d.obCostOrder, costOrder)) return VB_E_HIP;
  {
    auto rsStart = [&](int64_t b, int64_t e) {
      int64_t n = 0;
      for (int64_t i = b; i < e; i++) n += obRS[i] < 0;
      return b + n;
    };
    h->costRsB[0] = rsStart(d.obB, d.obE), h->costRsB[1] = rsStart(d.fB, d.fE);
  }
  {
    std::vector<int32_t> pack((size_t)nObs * 8);
    std::vector<double> cp((size_t)nObs * 6);
    for (int64_t i = 0; i < nObs; i++) {
      const int32_t o = costOrder[i];
      int32_t* q = &pack[(size_t)i * 8];
      q[0] = o, q[1] = obPt[o], q[2] = obPose[o], q[3] = obExtr[o], q[4] = obIntr[o], q[5] = obRS[o], q[6] = obVel[o];
      q[7] = (obRed[(size_t)o * 4 + kSlotIntr] >= 0 ? 1 : 0) | (obRed[(size_t)o * 4 + kSlotVel] >= 0 ? 2 : 0);
      for (int k = 0; k < 6; k++) cp[(size_t)i * 6 + k] = obC[(size_t)o * 6 + k];
    }
    if (upload(&d.obPack, pack) || upload(&d.obCP, cp)) return VB_E_HIP;
  }
  if (upload(&d.obPose, obPose) || upload(&d.obExtr, obExtr) || upload(&d.obIntr, obIntr) ||
      upload(&d.obVel, obVel) || upload(&d.obRS, obRS) || upload(&d.obPt, obPt) || upload(&d.obRed, obRed) ||
      upload(&d.obCol, obCol) || upload(&d.obC, obC))
    return VB_E_HIP;
  if (alloc0(&d.cache, nObs) || alloc0(&d.Jt, (size_t)kJPlanes * d.nObsPad)) return VB_E_HIP;
  if (upload(&d.lmObs, lmObs) || upload(&d.lmY, lmY) || upload(&d.lmBlk, lmBlk) || upload(&d.blkRed, blkRed) ||
      upload(&d.blkCol, blkCol) || upload(&d.ptLm, lmOf) || upload(&d.pcRow, pcRow) || upload(&d.pcBlk, pcBlk) ||
      upload(&d.bxStart, bxStart) || upload(&d.bxEnt, bxEnt))
    return VB_E_HIP;
  if (alloc0(&d.Vchol, nPts * 6) || alloc0(&d.gp, nPts * 3) || alloc0(&d.z, nPts * 3) || alloc0(&d.xp, nPts * 3) ||
      alloc0(&d.Y, lmY[nPts] + 128) || alloc0(&d.yZero, 256) ||  // + the over-read of the Schur gathers
      alloc0(&d.gpNew, nPts * 3) || alloc0(&d.zNew, nPts * 3))
    return VB_E_HIP;
  std::vector<int64_t> lxChunk;
  for (int i = 0; i < nRV; i++)
    for (int64_t b = lxStart[i]; b < lxStart[i + 1]; b += 1024)
      lxChunk.insert(lxChunk.end(), {i, b, std::min<int64_t>(b + 1024, lxStart[i + 1])});
  d.nLxChunk = (int64_t)lxChunk.size() / 3;
  if (upload(&d.oxStart, oxStart) || upload(&d.oxObs, oxObs) || upload(&d.oxSlot, oxSlot) ||
      upload(&d.lxStart, lxStart) || upload(&d.lxLm, lxLm) || upload(&d.lxCol, lxCol) || upload(&d.lxChunk, lxChunk))
    return VB_E_HIP;
  if (upload(&d.tileIdx, tileIdx) || alloc0(&d.tiles, (size_t)nTiles * TS * TS)) return VB_E_HIP;
  {
    int8_t* co = nullptr;
    if (upload(&co, h->colOwner)) return VB_E_HIP;
    d.colOwner = co, d.myRank = h->partRank, d.world = h->partWorld;
  }
  const size_t nPad = (size_t)nT * TS;
  if (alloc0(&d.gRed, nPad) || alloc0(&d.rhs, nPad) || alloc0(&d.xRed, nPad) || alloc0(&d.gRedNew, nPad) ||
      alloc0(&d.stepRed, nPad) || alloc0(&d.stepPt, nPts * 3) || alloc0(&d.subRed, nPad) ||
      alloc0(&d.subPt, nPts * 3) || alloc0(&h->yvec, nPad) || alloc0(&h->rhsWork, nPad))
    return VB_E_HIP;
  if (upload(&h->colStartD, h->colStart) || upload(&h->rowStartD, h->rowStart) ||
      alloc0(&h->solveFlags, 4 * (size_t)nT))
    return VB_E_HIP;
  if (upload(&h->colTilesD, h->colTilesH) || upload(&h->colRowsD, h->colRowsH) ||
      upload(&h->rowTilesD, h->rowTilesH) || upload(&h->rowColD, h->rowColH))
    return VB_E_HIP;
  if (alloc0(&h->dinv, (size_t)(nT + 1) * 1024) || alloc0(&h->linv, (size_t)nT * TS * TS))
    return VB_E_HIP;
  d.nRS = h->nRS;
  if (h->rsDevice) {
    // table capacity: the IMU samples of [mid - half, mid + half] widened by 20 ms on both sides (the
    // reference-time offsets of the calibration move the gyro boundaries by far less), + 4
    const int64_t kWidenNs = 20000000;
    h->rsOff.assign(h->nRS + 1, 0);
    for (int32_t t = 0; t < h->nRS; t++) {
      const int64_t a = (h->rsMid[t] - h->rsHalf[t]) * 1000 - kWidenNs, b = (h->rsMid[t] + h->rsHalf[t]) * 1000 + kWidenNs;
      const int64_t cnt = std::upper_bound(h->imuT.begin(), h->imuT.end(), b) -
                          std::lower_bound(h->imuT.begin(), h->imuT.end(), a);
      h->rsOff[t + 1] = h->rsOff[t] + cnt + 4;
    }
    const int64_t ns = h->rsOff[h->nRS];
    std::vector<int32_t> zeroN(h->nRS, 0);
    if (upload(&d.rsOff, h->rsOff) || alloc0(&d.rsS, ns * 11) || alloc0(&d.rsI, (ns - h->nRS) * 9) ||
        alloc0(&d.rsG, (size_t)h->nRS * 3) || upload(&d.rsN, zeroN) || upload(&d.imuT, h->imuT) ||
        upload(&d.imuV, h->imuV) || upload(&d.rsMid, h->rsMid) || upload(&d.rsHalf, h->rsHalf) ||
        upload(&d.rsCalib, h->rsCalib))
      return VB_E_HIP;
    d.nImu = (int64_t)h->imuT.size();
    d.rsGravVar = h->rsGravVar;
  } else {
    std::vector<int32_t> cnt(h->nRS);
    for (int32_t t = 0; t < h->nRS; t++) cnt[t] = (int32_t)(h->rsOff[t + 1] - h->rsOff[t]);
    if (h->rsOff.empty()) h->rsOff.assign(1, 0);
    if (upload(&d.rsOff, h->rsOff) || upload(&d.rsS, h->rsS) || upload(&d.rsI, h->rsI) || upload(&d.rsG, h->rsG) ||
        upload(&d.rsN, cnt))
      return VB_E_HIP;
  }
  if (alloc0(&d.red, 64) || alloc0(&d.redS, 2 * 64 * 8) || alloc0(&d.err, 8)) return VB_E_HIP;
  d.cacheW = d.cache;
  h->finalized = true;
  return 0;
}

}  // namespace viba_host
