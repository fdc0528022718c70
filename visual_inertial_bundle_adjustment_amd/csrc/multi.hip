// Multi-process building blocks (distributed.py): landmark shards, the partitioned factorization and
// the deferred (one host read per iteration) mode.
#include "host.hpp"

extern "C" {
// sharded building blocks (landmark shards).  The host controller
// (distributed.py) sums the partial reduced systems / right-hand sides of all shards on the root
// between these calls; every rank runs the same LM decisions.
int vb_shard_tiles(vb_handle h, int32_t* tiles, int64_t* n) {
  if (!h || !h->finalized || !n) return fail(VB_E_STATE, "not finalized");
  *n = (int64_t)h->shardTiles.size();
  if (tiles) std::copy(h->shardTiles.begin(), h->shardTiles.end(), tiles);
  return 0;
}
int vb_pack_shard_tiles(vb_handle h, double** buf, int64_t* len) {
  if (!h || !h->finalized || !buf || !len) return fail(VB_E_STATE, "not finalized");
  const int64_t n = (int64_t)h->shardTiles.size();
  if (n) launch_tile_gather(h->d, h->shardTilesD, n, h->shardPack, h->st);
  if (!h->deferred) HIPCHK(hipStreamSynchronize(h->st));
  *buf = h->shardPack, *len = n * TS * TS;
  return 0;
}
int vb_add_tiles(vb_handle h, const int32_t* tiles_dev, int64_t n, const double* buf_dev) {
  if (!h || !h->finalized || n < 0 || (n && (!tiles_dev || !buf_dev))) return fail(VB_E_ARG, "bad vb_add_tiles arguments");
  if (n) launch_tile_scatter_add(h->d, tiles_dev, n, buf_dev, h->st);
  if (!h->deferred) HIPCHK(hipStreamSynchronize(h->st));
  return 0;
}
int vb_shard_tile_range(vb_handle h, int64_t* first_double, int64_t* num_doubles) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "not finalized");
  if (first_double) *first_double = h->tileFirst * TS * TS;
  if (num_doubles) *num_doubles = h->tileCount * TS * TS;
  return 0;
}
// partial S (damped, Schur-reduced over this shard) in the tile store and partial RHS in rhs
int vb_assemble_reduced(vb_handle h, double lambda) {
  if (!h || !h->linearized) return fail(VB_E_STATE, "vb_assemble_reduced needs vb_linearize");
  if (!h->deferred) HIPCHK(hipMemsetAsync(h->d.err, 0, sizeof(int32_t), h->st));
  HIPCHK(hipEventRecord(h->ev[2], h->st));
  if (int rc = assembleEnqueue(h, lambda)) return rc;
  HIPCHK(hipEventRecord(h->ev[3], h->st));
  h->linearized = false;
  if (h->deferred) return 0;
  HIPCHK(hipStreamSynchronize(h->st));
  return checkErr(h);
}
// root: factor the (summed) tile store and solve with the (summed) rhs; x_red is left in rhs
int vb_factor_solve_reduced(vb_handle h) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "not finalized");
  if (!h->deferred) HIPCHK(hipMemsetAsync(h->d.err, 0, sizeof(int32_t), h->st));
  if (int rc = factorReduced(h)) return rc;
  HIPCHK(hipMemcpyAsync(h->rhsWork, h->d.rhs, (size_t)h->d.nT * TS * sizeof(double), hipMemcpyDeviceToDevice, h->st));
  if (int rc = solveReduced(h)) return rc;
  HIPCHK(hipMemcpyAsync(h->d.rhs, h->d.xRed, (size_t)h->d.nT * TS * sizeof(double), hipMemcpyDeviceToDevice, h->st));
  h->factored = true;
  if (h->deferred) return 0;
  HIPCHK(hipStreamSynchronize(h->st));
  return checkErr(h);
}
// root: solve with the existing factor, rhs -> x_red (left in rhs)
int vb_solve_reduced(vb_handle h) {
  if (!h || !h->factored) return fail(VB_E_STATE, "vb_solve_reduced needs a factorization");
  HIPCHK(hipMemcpyAsync(h->rhsWork, h->d.rhs, (size_t)h->d.nT * TS * sizeof(double), hipMemcpyDeviceToDevice, h->st));
  if (int rc = solveReduced(h)) return rc;
  HIPCHK(hipMemcpyAsync(h->d.rhs, h->d.xRed, (size_t)h->d.nT * TS * sizeof(double), hipMemcpyDeviceToDevice, h->st));
  if (!h->deferred) HIPCHK(hipStreamSynchronize(h->st));
  return 0;
}
// x_red (broadcast into rhs) -> step (which 0) / sub-step (which 1) of this shard; which 0 also
// returns the partial model cost reduction 0.5 (x_red . g_red_partial + x_p . g_p over the shard)
int vb_back_substitute_which(vb_handle h, int which, double* mcr) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "not finalized");
  Dev& d = h->d;
  HIPCHK(hipMemcpyAsync(d.xRed, d.rhs, (size_t)d.nT * TS * sizeof(double), hipMemcpyDeviceToDevice, h->st));
  backSubstitute(h, which);
  double v = 0;
  if (h->deferred) {  // partial model dot in red[16]
    v = std::nan("");
  } else if (which == 0) {
    if (int rc = readRed(h, &v, 16, 1)) return rc;
  } else {
    HIPCHK(hipStreamSynchronize(h->st));
  }
  if (mcr) *mcr = 0.5 * v;
  h->factored = true;
  return 0;
}
int vb_back_substitute(vb_handle h, double* mcr) { return vb_back_substitute_which(h, 0, mcr); }
// partial new reduced RHS of this shard (after vb_gradient_dot_step): rhs = gRedNew_part - Y^T zNew
int vb_assemble_new_rhs(vb_handle h) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "not finalized");
  Dev& d = h->d;
  launch_landmark(d, 0.0, 2, d.lmB, d.lmE, h->st);
  launch_reduced_grad(d, 1, h->st);
  HIPCHK(hipStreamSynchronize(h->st));
  return 0;
}


// ---------------- partitioned factorization (nested-dissection subtrees per rank)
int vb_set_partition(vb_handle h, int rank, int world) {
  if (!h) return fail(VB_E_ARG, "null handle");
  if (h->finalized) return fail(VB_E_STATE, "vb_set_partition must precede vb_finalize");
  if (world < 1 || world > 64 || (world & (world - 1)) || rank < 0 || rank >= world)
    return fail(VB_E_ARG, "vb_set_partition: world must be a power of two in [1, 64], 0 <= rank < world");
  h->partRank = rank, h->partWorld = world, h->partSet = true;
  return 0;
}
// which 0: this rank's subtree columns (+ their fan-in into the ROOT tiles); 1 (rank 0): ROOT columns
int vb_factor_part(vb_handle h, int which) {
  if (!h || !h->finalized || which < 0 || which > 1) return fail(VB_E_STATE, "vb_factor_part: bad state / schedule");
  if (!h->deferred) HIPCHK(hipMemsetAsync(h->d.err, 0, sizeof(int32_t), h->st));
  if (int rc = factorReduced(h, which)) return rc;
  h->factored = true;
  if (h->deferred) return 0;
  HIPCHK(hipStreamSynchronize(h->st));
  return checkErr(h);
}
// phase 0: rhsWork = rhs, forward solve over this rank's subtree (partial ROOT rows of rhsWork);
// 1 (rank 0): forward + backward over the ROOT columns (ROOT rows of rhsWork summed);
// 2: backward over this rank's subtree (ROOT rows of xRed given)
int vb_solve_part(vb_handle h, int phase) {
  if (!h || !h->factored || phase < 0 || phase > 2) return fail(VB_E_STATE, "vb_solve_part: bad state / phase");
  if (!h->deferred) HIPCHK(hipMemsetAsync(h->d.err, 0, sizeof(int32_t), h->st));
  if (phase == 0)
    HIPCHK(hipMemcpyAsync(h->rhsWork, h->d.rhs, (size_t)h->d.nT * TS * sizeof(double), hipMemcpyDeviceToDevice, h->st));
  if (int rc = solveReduced(h, phase == 1 ? 1 : 0, phase == 0 ? 1 : phase == 1 ? 3 : 2)) return rc;
  if (h->deferred) return 0;
  HIPCHK(hipStreamSynchronize(h->st));
  return checkErr(h);
}
// what 0: the ROOT-column tiles of the tile store, 1: ROOT rows of rhsWork, 2: ROOT rows of xRed;
// dir 0 packs them into the engine-owned buffer (returned), dir 1 writes the buffer back
int vb_part_exchange(vb_handle h, int what, int dir, double** buf, int64_t* len) {
  if (!h || !h->finalized || what < 0 || what > 2 || dir < 0 || dir > 1 || !buf || !len)
    return fail(VB_E_ARG, "bad vb_part_exchange arguments");
  if (!h->partSet) return fail(VB_E_STATE, "vb_part_exchange needs vb_set_partition");
  const bool tiles = what == 0;
  const int32_t* idx = tiles ? h->rootTilesD : h->rootRowsD;
  const int64_t n = tiles ? (int64_t)h->rootTiles.size() : (int64_t)h->rootRows.size();
  double* base = tiles ? h->d.tiles : what == 1 ? h->rhsWork : h->d.xRed;
  double* pk = tiles ? h->rootPack : h->rowPack;
  launch_chunk_copy(base, idx, n, tiles ? TS * TS : TS, pk, dir == 0 ? 0 : 1, h->st);
  if (!h->deferred) HIPCHK(hipStreamSynchronize(h->st));
  *buf = pk, *len = n * (tiles ? TS * TS : TS);
  return 0;
}
// ---------------- deferred mode: one host read per LM iteration in the multi-process controllers
// (distributed.py).  With it on, the phase functions (vb_update_rs_tables, vb_linearize,
// vb_assemble_reduced, vb_factor_solve_reduced, vb_solve_reduced, vb_factor_part, vb_solve_part,
// vb_part_exchange, vb_share_x, vb_pack_shard_tiles, vb_add_tiles, vb_back_substitute_which,
// vb_apply_step_raw, vb_cost) only queue their work; the scalars they would return stay in the
// reduction slots, which the caller all-reduces in place on the handle's stream (RCCL) and reads once.
int vb_set_deferred(vb_handle h, int on) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "vb_set_deferred before vb_finalize");
  h->deferred = on != 0;
  return 0;
}
// red: [0] linearization cost, [1] cost pass cost, [2] observations evaluated, [3] invalid, [4] invalid
// at the linearization point, [8] max |step| / |x| ratio, [9] sum of squared ratios, [10] sum of ratios,
// [16] 2 x model cost reduction (partials of this handle); err: two error words (bitwise, max-reducible)
int vb_scalar_slots(vb_handle h, double** red, int32_t** err) {
  if (!h || !h->finalized) return fail(VB_E_STATE, "vb_scalar_slots before vb_finalize");
  if (red) *red = h->d.red;
  if (err) *err = h->d.err;
  return 0;
}
// what the cost pass's CostStats.numTotal adds for the non-visual factors this handle evaluates
int vb_small_factor_count(vb_handle h, int64_t* n) {
  if (!h || !h->finalized || !n) return fail(VB_E_STATE, "vb_small_factor_count before vb_finalize");
  *n = 0;
  if (h->isRoot)
    for (int k = 1; k < 14; k++) *n += h->d.sf[k].n;
  return 0;
}
int vb_error_words(vb_handle h, int32_t* out2) {
  if (!h || !out2) return fail(VB_E_ARG, "bad vb_error_words arguments");
  out2[0] = h->lastWords[0], out2[1] = h->lastWords[1];
  return 0;
}
int vb_error_from_words(vb_handle h, const int32_t* words2) {
  if (!h || !words2) return fail(VB_E_ARG, "bad vb_error_from_words arguments");
  return errFromWords(h, words2);
}
// the point on the stream after which the slots hold the iteration's (reduced) scalars: work queued
// later (a speculative linearization) does not delay vb_read_scalars.  Needs vb_spec_prepare.
int vb_mark_scalars(vb_handle h) {
  if (!h || !h->specReady) return fail(VB_E_STATE, "vb_mark_scalars needs vb_spec_prepare");
  if (hipEventRecord(h->evCost, h->st) != hipSuccess) return fail(VB_E_HIP, "hipEventRecord");
  h->profAtCost = h->profUsed;
  h->scalarsMarked = true;
  return 0;
}
// red[0, n) (n <= 24) and the error words, after the mark (or the whole queue without one); the
// return code is the error the words encode
int vb_read_scalars(vb_handle h, double* out, int n) {
  if (!h || !h->finalized || !out || n < 0 || n > 24) return fail(VB_E_ARG, "bad vb_read_scalars arguments");
  const bool marked = h->scalarsMarked;
  h->scalarsMarked = false;
  return marked ? readIterScalars(h, out, n) : readRedErr(h, out, n);
}
// the speculative linearization of vb_optimize for an external controller: *ok = 0 when its spare
// buffers cannot be had (then the controller linearizes every iteration itself)
int vb_spec_prepare(vb_handle h, int* ok) {
  if (!h || !h->finalized || !ok) return fail(VB_E_STATE, "vb_spec_prepare before vb_finalize");
  *ok = specPrepare(h) ? 1 : 0;
  return 0;
}
// queue the rolling-shutter rebuild and the linearization at the current (stepped) variables into the
// spare buffers, behind everything queued so far
int vb_spec_linearize(vb_handle h, int dont_retry_failed) {
  if (!h || !h->specReady) return fail(VB_E_STATE, "vb_spec_linearize needs vb_spec_prepare");
  h->specSet ^= 1;
  h->specPending = true;
  return specEnqueue(h, dont_retry_failed, h->specSet, false);
}
// use = 1: the step stayed applied at full size, the spare buffers become the handle's (the
// linearization cost moves to red[0]); use = 0: drop them (the next vb_linearize overwrites)
int vb_spec_commit(vb_handle h, int use) {
  if (!h || !h->specReady || !h->specPending) return fail(VB_E_STATE, "vb_spec_commit without vb_spec_linearize");
  h->specPending = false;
  if (!use) return 0;
  specCommit(h);
  h->specCommitted = h->specSet;
  h->linearized = true, h->factored = false;
  return 0;
}

// the rolling-shutter rebuild and linearization times (ms) of the speculative linearization last committed
// (its events precede the cost pass of the iteration that used it, so they are complete once that
// iteration's scalars were read)
int vb_spec_phase_ms(vb_handle h, double* out2) {
  if (!h || !out2) return fail(VB_E_ARG, "bad vb_spec_phase_ms arguments");
  out2[0] = out2[1] = 0.0;
  const int p = h->specCommitted;
  if (!h->specReady || p < 0) return 0;
  if (h->rsDevice) out2[0] = elapsed(h->evS[p][0], h->evS[p][1]);
  out2[1] = elapsed(h->evS[p][2], h->evS[p][3]);
  return 0;
}

// [subtree tile columns of this rank, ROOT tile columns, fan-in contributions of the local schedule,
//  of the ROOT schedule (rank 0), ROOT tiles exchanged]
int vb_part_info(vb_handle h, int64_t* out5) {
  if (!h || !h->finalized || !out5) return fail(VB_E_STATE, "not finalized");
  int64_t own = 0, root = 0;
  for (int8_t o : h->colOwner) own += o == h->partRank, root += o == h->partWorld;
  if (!h->partSet) own = (int64_t)h->colOwner.size(), root = 0;
  out5[0] = own, out5[1] = root, out5[2] = h->sch[0].nPairs, out5[3] = h->sch[1].nPairs;
  out5[4] = (int64_t)h->rootTiles.size();
  return 0;
}
// after the backward phase: the rows this rank solved (its subtree; + ROOT on rank 0) of xRed, other
// rows zeroed, into the rhs buffer (returned) -- the caller all-reduces it, then vb_back_substitute
int vb_share_x(vb_handle h, double** xred, int64_t* len) {
  if (!h || !h->finalized || !xred || !len) return fail(VB_E_ARG, "bad vb_share_x arguments");
  Dev& d = h->d;
  HIPCHK(hipMemsetAsync(d.rhs, 0, (size_t)d.nT * TS * sizeof(double), h->st));
  launch_chunk_copy(d.xRed, h->ownRowsD, h->nOwnRows, TS, h->ownPack, 0, h->st);
  launch_chunk_copy(d.rhs, h->ownRowsD, h->nOwnRows, TS, h->ownPack, 1, h->st);
  if (!h->deferred) HIPCHK(hipStreamSynchronize(h->st));
  *xred = d.rhs, *len = (int64_t)d.nT * TS;
  return 0;
}

}  // extern "C"
