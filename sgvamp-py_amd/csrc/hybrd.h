// Library-internal entry of the fsolve restatement (hybrd.cpp): not part of
// the C ABI (hidden symbol).
#pragma once
#include "sgvamp_hip.h"

// the forward-difference Jacobian's n evaluations in one call: F row j (n
// values) = fcn(x + h_j e_j); return < 0 to stop the solve
typedef int (*sgv_fsolve_jac_fn)(void* user, int n, const double* x, const double* h, double* F);

// sgv_fsolve with an optional batched Jacobian (jac == nullptr: n calls of fcn)
__attribute__((visibility("hidden"))) int sgv_fsolve_jac(int n, sgv_fsolve_fn fcn,
                                                         sgv_fsolve_jac_fn jac, void* user,
                                                         double* x_io, double* fvec_out,
                                                         int* nfev_out);
