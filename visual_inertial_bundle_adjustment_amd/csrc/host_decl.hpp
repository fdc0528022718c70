// Declarations of the host functions the engine's translation units share (host.hpp): api.hip defines
// all but doFinalize / buildSupernodes (finalize.hip).
#pragma once

namespace viba_host {
// kernel-family event timing and error words (api.hip)
float profPairMs(hipEvent_t a, hipEvent_t b);
double elapsed(hipEvent_t a, hipEvent_t b);
void profHarvest(vb_handle h);
int checkErr(vb_handle h);
int errFromWords(vb_handle h, const int32_t* ee);
int readRed(vb_handle h, double* out, int i0, int n);
int readRedErr(vb_handle h, double* out, int n);
// numeric phases (api.hip)
bool smallHere(vb_handle h, int mode);
int factorReduced(vb_handle h, int which = 0);
int solveReduced(vb_handle h, int which = 0, int phases = 3);
void backSubstitute(vb_handle h, int which);
// vb_finalize (finalize.hip)
int doFinalize(vb_handle h);
}  // namespace viba_host

extern "C" {
// queued phases and vb_optimize's speculation (api.hip; C linkage, defined in its C-ABI block)
int clearReduced(vb_handle h, const Dev& d, hipStream_t zs);
Dev specDev(vb_handle h);
int rsUpdateAsync(vb_handle h, bool tables = true, bool preint = false);
int linearizeEnqueue(vb_handle h, int update_cache, int dont_retry_failed);
int assembleEnqueue(vb_handle h, double lambda);
int dampFactorSolveEnqueue(vb_handle h, double lambda, bool clearErr);
int applyStepEnqueue(vb_handle h, int which, int e0, int e1);
int costEnqueue(vb_handle h, int comparable, bool clearErr);
bool specPrepare(vb_handle h);
void specRelease(vb_handle h);
int specEnqueue(vb_handle h, int dontRetry, int p, bool early, bool rsDone = false, bool fuseCost = false);
int specEarly(vb_handle h, bool cleared = false, bool storeCleared = false);
void specCommit(vb_handle h);
int readIterScalars(vb_handle h, double* out, int n);
}
