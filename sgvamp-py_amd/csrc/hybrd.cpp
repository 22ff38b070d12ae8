// Powell's hybrid method for F(x) = 0 (MINPACK hybrd, More, Garbow and Hillstrom,
// Argonne 1980), as scipy.optimize.fsolve drives it: forward-difference Jacobian
// (dense), automatic variable scaling (mode 1), no printing.  The reference's MLE
// prior update calls fsolve on the Lagrangian of the spike-and-slab likelihood
// (src/sgvamp.py:179); here the solver runs inside the library so an MLE update
// needs no return to Python between function evaluations (sgv_step,
// SGV_STEP_MLE).  Host-only C++; the function evaluations are the caller's.
//
// The routines below follow MINPACK's hybrd, fdjac1, qrfac (no pivoting),
// qform, dogleg, r1updt, r1mpyq and enorm statement by statement (same operation
// order, column-major work arrays, 1-based loops shifted to 0-based), so the
// iterates and the termination code agree with scipy 1.15.3's fsolve
// (tests/test_hybrd.py).
//
// This file is a derivative of MINPACK, distributed under its license:
//
//   Minpack Copyright Notice (1999) University of Chicago.  All rights reserved
//
//   Redistribution and use in source and binary forms, with or without
//   modification, are permitted provided that the following conditions are met:
//
//   1. Redistributions of source code must retain the above copyright notice,
//   this list of conditions and the following disclaimer.
//
//   2. Redistributions in binary form must reproduce the above copyright
//   notice, this list of conditions and the following disclaimer in the
//   documentation and/or other materials provided with the distribution.
//
//   3. The end-user documentation included with the redistribution, if any,
//   must include the following acknowledgment:
//
//      "This product includes software developed by the University of
//      Chicago, as Operator of Argonne National Laboratory.
//
//   Alternately, this acknowledgment may appear in the software itself, if and
//   wherever such third-party acknowledgments normally appear.
//
//   4. WARRANTY DISCLAIMER. THE SOFTWARE IS SUPPLIED "AS IS" WITHOUT WARRANTY
//   OF ANY KIND. THE COPYRIGHT HOLDER, THE UNITED STATES, THE UNITED STATES
//   DEPARTMENT OF ENERGY, AND THEIR EMPLOYEES: (1) DISCLAIM ANY WARRANTIES,
//   EXPRESS OR IMPLIED, INCLUDING BUT NOT LIMITED TO ANY IMPLIED WARRANTIES OF
//   MERCHANTABILITY, FITNESS FOR A PARTICULAR PURPOSE, TITLE OR
//   NON-INFRINGEMENT, (2) DO NOT ASSUME ANY LEGAL LIABILITY OR RESPONSIBILITY
//   FOR THE ACCURACY, COMPLETENESS, OR USEFULNESS OF THE SOFTWARE, (3) DO NOT
//   REPRESENT THAT USE OF THE SOFTWARE WOULD NOT INFRINGE PRIVATELY OWNED
//   RIGHTS, (4) DO NOT WARRANT THAT THE SOFTWARE WILL FUNCTION UNINTERRUPTED,
//   THAT IT IS ERROR-FREE OR THAT ANY ERRORS WILL BE CORRECTED.
//
//   5. LIMITATION OF LIABILITY. IN NO EVENT WILL THE COPYRIGHT HOLDER, THE
//   UNITED STATES, THE UNITED STATES DEPARTMENT OF ENERGY, OR THEIR EMPLOYEES:
//   BE LIABLE FOR ANY INDIRECT, INCIDENTAL, CONSEQUENTIAL, SPECIAL OR PUNITIVE
//   DAMAGES OF ANY KIND OR NATURE, INCLUDING BUT NOT LIMITED TO LOSS OF PROFITS
//   OR LOSS OF DATA, FOR ANY REASON WHATSOEVER, WHETHER SUCH LIABILITY IS
//   ASSERTED ON THE BASIS OF CONTRACT, TORT (INCLUDING NEGLIGENCE OR STRICT
//   LIABILITY), OR OTHERWISE, EVEN IF ANY OF SAID PARTIES HAS BEEN WARNED OF
//   THE POSSIBILITY OF SUCH LOSS OR DAMAGES.
//
// This product includes software developed by the University of Chicago, as
// Operator of Argonne National Laboratory.
#include <cmath>
#include <cstring>
#include <vector>

#include "hybrd.h"

namespace {

constexpr double EPSMCH = 2.220446049250313e-16;   // dpmpar(1)
constexpr double GIANT = 1.7976931348623157e308;   // dpmpar(3)

// Euclidean norm with MINPACK's overflow/underflow-safe three-sum scheme
double enorm(int n, const double* x) {
  const double rdwarf = 3.834e-20, rgiant = 1.304e19;
  double s1 = 0.0, s2 = 0.0, s3 = 0.0, x1max = 0.0, x3max = 0.0;
  const double agiant = rgiant / (double)n;
  for (int i = 0; i < n; ++i) {
    const double xabs = std::fabs(x[i]);
    if (xabs > rdwarf && xabs < agiant) {
      s2 += xabs * xabs;
    } else if (xabs > rdwarf) {   // large components
      if (xabs > x1max) {
        const double r = x1max / xabs;
        s1 = 1.0 + s1 * (r * r);
        x1max = xabs;
      } else {
        const double r = xabs / x1max;
        s1 += r * r;
      }
    } else {                      // small components
      if (xabs > x3max) {
        const double r = x3max / xabs;
        s3 = 1.0 + s3 * (r * r);
        x3max = xabs;
      } else if (xabs != 0.0) {
        const double r = xabs / x3max;
        s3 += r * r;
      }
    }
  }
  if (s1 != 0.0) return x1max * std::sqrt(s1 + (s2 / x1max) / x1max);
  if (s2 != 0.0) {
    if (s2 >= x3max) return std::sqrt(s2 * (1.0 + (x3max / s2) * (x3max * s3)));
    return std::sqrt(x3max * ((s2 / x3max) + (x3max * s3)));
  }
  return x3max * std::sqrt(s3);
}

// a(i, j) of an n x n column-major array
struct Mat {
  double* p;
  int ld;
  double& operator()(int i, int j) const { return p[(size_t)j * ld + i]; }
};

// Householder QR of the m x n matrix a without pivoting: R's diagonal in rdiag,
// the column norms of a in acnorm, the Householder vectors in a's lower part
void qrfac(int m, int n, Mat a, double* rdiag, double* acnorm, double* wa) {
  for (int j = 0; j < n; ++j) {
    acnorm[j] = enorm(m, &a(0, j));
    rdiag[j] = acnorm[j];
    wa[j] = rdiag[j];
  }
  const int minmn = m < n ? m : n;
  for (int j = 0; j < minmn; ++j) {
    double ajnorm = enorm(m - j, &a(j, j));
    if (ajnorm != 0.0) {
      if (a(j, j) < 0.0) ajnorm = -ajnorm;
      for (int i = j; i < m; ++i) a(i, j) = a(i, j) / ajnorm;
      a(j, j) = a(j, j) + 1.0;
      for (int k = j + 1; k < n; ++k) {
        double sum = 0.0;
        for (int i = j; i < m; ++i) sum = sum + a(i, j) * a(i, k);
        const double temp = sum / a(j, j);
        for (int i = j; i < m; ++i) a(i, k) = a(i, k) - temp * a(i, j);
      }
    }
    rdiag[j] = -ajnorm;
  }
}

// the orthogonal factor Q (m x m) from qrfac's factored form, in place
void qform(int m, int n, Mat q, double* wa) {
  const int minmn = m < n ? m : n;
  for (int j = 1; j < minmn; ++j)
    for (int i = 0; i < j; ++i) q(i, j) = 0.0;
  for (int j = n; j < m; ++j) {
    for (int i = 0; i < m; ++i) q(i, j) = 0.0;
    q(j, j) = 1.0;
  }
  for (int l = 0; l < minmn; ++l) {
    const int k = minmn - 1 - l;
    for (int i = k; i < m; ++i) {
      wa[i] = q(i, k);
      q(i, k) = 0.0;
    }
    q(k, k) = 1.0;
    if (wa[k] == 0.0) continue;
    for (int j = k; j < m; ++j) {
      double sum = 0.0;
      for (int i = k; i < m; ++i) sum = sum + q(i, j) * wa[i];
      const double temp = sum / wa[k];
      for (int i = k; i < m; ++i) q(i, j) = q(i, j) - temp * wa[i];
    }
  }
}

// dogleg step within the trust region: r is the packed upper triangle (by rows)
void dogleg(int n, const double* r, const double* diag, const double* qtb, double delta,
            double* x, double* wa1, double* wa2) {
  // Gauss-Newton direction (1-based jj of the Fortran kept as jj - 1 here)
  int jj = (n * (n + 1)) / 2 + 1;
  for (int k = 1; k <= n; ++k) {
    const int j = n - k + 1;
    jj = jj - k;
    int l = jj + 1;
    double sum = 0.0;
    for (int i = j + 1; i <= n; ++i) {
      sum = sum + r[l - 1] * x[i - 1];
      ++l;
    }
    double temp = r[jj - 1];
    if (temp == 0.0) {
      l = j;
      for (int i = 1; i <= j; ++i) {
        temp = std::fmax(temp, std::fabs(r[l - 1]));
        l = l + n - i;
      }
      temp = EPSMCH * temp;
      if (temp == 0.0) temp = EPSMCH;
    }
    x[j - 1] = (qtb[j - 1] - sum) / temp;
  }
  for (int j = 0; j < n; ++j) {
    wa1[j] = 0.0;
    wa2[j] = diag[j] * x[j];
  }
  const double qnorm = enorm(n, wa2);
  if (qnorm <= delta) return;
  // scaled gradient direction
  int l = 0;
  for (int j = 0; j < n; ++j) {
    const double temp = qtb[j];
    for (int i = j; i < n; ++i) {
      wa1[i] = wa1[i] + r[l] * temp;
      ++l;
    }
    wa1[j] = wa1[j] / diag[j];
  }
  const double gnorm = enorm(n, wa1);
  double sgnorm = 0.0;
  double alpha = delta / qnorm;
  if (gnorm != 0.0) {
    for (int j = 0; j < n; ++j) wa1[j] = (wa1[j] / gnorm) / diag[j];
    l = 0;
    for (int j = 0; j < n; ++j) {
      double sum = 0.0;
      for (int i = j; i < n; ++i) {
        sum = sum + r[l] * wa1[i];
        ++l;
      }
      wa2[j] = sum;
    }
    const double temp = enorm(n, wa2);
    sgnorm = (gnorm / temp) / temp;
    alpha = 0.0;
    if (sgnorm < delta) {
      // the point along the dogleg at which the quadratic is minimized
      const double bnorm = enorm(n, qtb);
      double t = (bnorm / gnorm) * (bnorm / qnorm) * (sgnorm / delta);
      const double dq = delta / qnorm, sd = sgnorm / delta;
      t = t - dq * (sd * sd) + std::sqrt((t - dq) * (t - dq) + (1.0 - dq * dq) * (1.0 - sd * sd));
      alpha = (dq * (1.0 - sd * sd)) / t;
    }
  }
  const double temp = (1.0 - alpha) * std::fmin(sgnorm, delta);
  for (int j = 0; j < n; ++j) x[j] = temp * wa1[j] + alpha * x[j];
}

// rank-one update of the packed (by rows) upper triangle s: s + u v^T = Q s'
// (1-based indices as in MINPACK; the arrays are 0-based)
bool r1updt(int m, int n, double* s, const double* u, double* v, double* w) {
  const double p5 = 0.5, p25 = 0.25;
  int jj = (n * (2 * m - n + 1)) / 2 - (m - n);
  int l = jj;
  for (int i = n; i <= m; ++i) {
    w[i - 1] = s[l - 1];
    ++l;
  }
  const int nm1 = n - 1;
  for (int nmj = 1; nmj <= nm1; ++nmj) {
    const int j = n - nmj;
    jj = jj - (m - j + 1);
    w[j - 1] = 0.0;
    if (v[j - 1] == 0.0) continue;
    double sin, cos, tau;
    if (std::fabs(v[n - 1]) >= std::fabs(v[j - 1])) {
      const double tan = v[j - 1] / v[n - 1];
      cos = p5 / std::sqrt(p25 + p25 * (tan * tan));
      sin = cos * tan;
      tau = sin;
    } else {
      const double cotan = v[n - 1] / v[j - 1];
      sin = p5 / std::sqrt(p25 + p25 * (cotan * cotan));
      cos = sin * cotan;
      tau = 1.0;
      if (std::fabs(cos) * GIANT > 1.0) tau = 1.0 / cos;
    }
    v[n - 1] = sin * v[j - 1] + cos * v[n - 1];
    v[j - 1] = tau;
    l = jj;
    for (int i = j; i <= m; ++i) {
      const double temp = cos * s[l - 1] - sin * w[i - 1];
      w[i - 1] = sin * s[l - 1] + cos * w[i - 1];
      s[l - 1] = temp;
      ++l;
    }
  }
  for (int i = 1; i <= m; ++i) w[i - 1] = w[i - 1] + v[n - 1] * u[i - 1];
  bool sing = false;
  for (int j = 1; j <= nm1; ++j) {
    if (w[j - 1] != 0.0) {
      double sin, cos, tau;
      if (std::fabs(s[jj - 1]) >= std::fabs(w[j - 1])) {
        const double tan = w[j - 1] / s[jj - 1];
        cos = p5 / std::sqrt(p25 + p25 * (tan * tan));
        sin = cos * tan;
        tau = sin;
      } else {
        const double cotan = s[jj - 1] / w[j - 1];
        sin = p5 / std::sqrt(p25 + p25 * (cotan * cotan));
        cos = sin * cotan;
        tau = 1.0;
        if (std::fabs(cos) * GIANT > 1.0) tau = 1.0 / cos;
      }
      l = jj;
      for (int i = j; i <= m; ++i) {
        const double temp = cos * s[l - 1] + sin * w[i - 1];
        w[i - 1] = -sin * s[l - 1] + cos * w[i - 1];
        s[l - 1] = temp;
        ++l;
      }
      w[j - 1] = tau;
    }
    if (s[jj - 1] == 0.0) sing = true;
    jj = jj + (m - j + 1);
  }
  l = jj;
  for (int i = n; i <= m; ++i) {
    s[l - 1] = w[i - 1];
    ++l;
  }
  if (s[jj - 1] == 0.0) sing = true;
  return sing;
}

// a (m x n, leading dimension lda) times the Givens rotations r1updt recorded in v, w
void r1mpyq(int m, int n, double* a, int lda, const double* v, const double* w) {
  Mat A{a, lda};
  const int nm1 = n - 1;
  for (int nmj = 1; nmj <= nm1; ++nmj) {
    const int j = n - nmj;
    double cos, sin;
    if (std::fabs(v[j - 1]) > 1.0) {
      cos = 1.0 / v[j - 1];
      sin = std::sqrt(1.0 - cos * cos);
    } else {
      sin = v[j - 1];
      cos = std::sqrt(1.0 - sin * sin);
    }
    for (int i = 0; i < m; ++i) {
      const double temp = cos * A(i, j - 1) - sin * A(i, n - 1);
      A(i, n - 1) = sin * A(i, j - 1) + cos * A(i, n - 1);
      A(i, j - 1) = temp;
    }
  }
  for (int j = 1; j <= nm1; ++j) {
    double cos, sin;
    if (std::fabs(w[j - 1]) > 1.0) {
      cos = 1.0 / w[j - 1];
      sin = std::sqrt(1.0 - cos * cos);
    } else {
      sin = w[j - 1];
      cos = std::sqrt(1.0 - sin * sin);
    }
    for (int i = 0; i < m; ++i) {
      const double temp = cos * A(i, j - 1) + sin * A(i, n - 1);
      A(i, n - 1) = -sin * A(i, j - 1) + cos * A(i, n - 1);
      A(i, j - 1) = temp;
    }
  }
}

}  // namespace

// scipy.optimize.fsolve(func, x0, full_output=True) with its defaults: xtol
// 1.49012e-08, maxfev 200 (n + 1), epsfcn = machine eps, factor 100, mode 1.
// Returns MINPACK's info (1 = converged; 2 maxfev; 3 xtol too small; 4/5 no
// progress; < 0 the callback's negative status); x_io holds the last iterate.
// jac (may be null): the forward-difference Jacobian's n evaluations in one
// call, F row j = fcn(x + h_j e_j) -- the same points, so the same iterates as
// n calls of fcn; a caller whose evaluations are device passes enqueues them
// back to back and waits once (sgv_mle_update)
int sgv_fsolve_jac(int n, sgv_fsolve_fn fcn, sgv_fsolve_jac_fn jac, void* user, double* x_io,
                   double* fvec_out, int* nfev_out) {
  if (n <= 0 || !fcn || !x_io) return 0;
  const double xtol = 1.49012e-08, factor = 100.0;
  const double epsfcn = EPSMCH;
  const int maxfev = 200 * (n + 1);
  const double p1 = 0.1, p5 = 0.5, p001 = 1e-3, p0001 = 1e-4;
  std::vector<double> fvec(n), diag(n), fjac((size_t)n * n), r((size_t)n * (n + 1) / 2), qtf(n),
      wa1(n), wa2(n), wa3(n), wa4(n), hj(jac ? n : 0), fj(jac ? (size_t)n * n : 0);
  double* x = x_io;
  Mat J{fjac.data(), n};
  int info = 0, nfev = 0;
  int rc = fcn(user, n, x, fvec.data());
  nfev = 1;
  if (rc < 0) {
    info = rc;
  } else {
    double fnorm = enorm(n, fvec.data());
    double xnorm = 0.0, delta = 0.0;
    int iter = 1, ncsuc = 0, ncfail = 0, nslow1 = 0, nslow2 = 0;
    const double eps = std::sqrt(std::fmax(epsfcn, EPSMCH));
    for (;;) {   // outer loop: a fresh forward-difference Jacobian
      bool jeval = true;
      if (jac) {   // fdjac1, the n points in one call
        for (int j = 0; j < n; ++j) {
          hj[j] = eps * std::fabs(x[j]);
          if (hj[j] == 0.0) hj[j] = eps;
        }
        rc = jac(user, n, x, hj.data(), fj.data());
        if (rc >= 0)
          for (int j = 0; j < n; ++j)
            for (int i = 0; i < n; ++i) J(i, j) = (fj[(size_t)j * n + i] - fvec[i]) / hj[j];
      } else {
        for (int j = 0; j < n && rc >= 0; ++j) {   // fdjac1, dense
          const double temp = x[j];
          double h = eps * std::fabs(temp);
          if (h == 0.0) h = eps;
          x[j] = temp + h;
          rc = fcn(user, n, x, wa1.data());
          if (rc < 0) break;
          x[j] = temp;
          for (int i = 0; i < n; ++i) J(i, j) = (wa1[i] - fvec[i]) / h;
        }
      }
      nfev += n;
      if (rc < 0) {
        info = rc;
        break;
      }
      qrfac(n, n, J, wa1.data(), wa2.data(), wa3.data());
      if (iter == 1) {
        for (int j = 0; j < n; ++j) {
          diag[j] = wa2[j];
          if (wa2[j] == 0.0) diag[j] = 1.0;
        }
        for (int j = 0; j < n; ++j) wa3[j] = diag[j] * x[j];
        xnorm = enorm(n, wa3.data());
        delta = factor * xnorm;
        if (delta == 0.0) delta = factor;
      }
      for (int i = 0; i < n; ++i) qtf[i] = fvec[i];
      for (int j = 0; j < n; ++j) {
        if (J(j, j) == 0.0) continue;
        double sum = 0.0;
        for (int i = j; i < n; ++i) sum = sum + J(i, j) * qtf[i];
        const double temp = -sum / J(j, j);
        for (int i = j; i < n; ++i) qtf[i] = qtf[i] + J(i, j) * temp;
      }
      // the triangular factor into r (packed by rows)
      for (int j = 0; j < n; ++j) {
        int l = j;
        for (int i = 0; i < j; ++i) {
          r[l] = J(i, j);
          l = l + n - i - 1;
        }
        r[l] = wa1[j];
      }
      qform(n, n, J, wa1.data());
      for (int j = 0; j < n; ++j) diag[j] = std::fmax(diag[j], wa2[j]);
      bool outer = false;
      for (;;) {   // inner loop: rank-one Jacobian updates
        dogleg(n, r.data(), diag.data(), qtf.data(), delta, wa1.data(), wa2.data(), wa3.data());
        for (int j = 0; j < n; ++j) {
          wa1[j] = -wa1[j];
          wa2[j] = x[j] + wa1[j];
          wa3[j] = diag[j] * wa1[j];
        }
        const double pnorm = enorm(n, wa3.data());
        if (iter == 1) delta = std::fmin(delta, pnorm);
        rc = fcn(user, n, wa2.data(), wa4.data());
        nfev += 1;
        if (rc < 0) {
          info = rc;
          break;
        }
        const double fnorm1 = enorm(n, wa4.data());
        double actred = -1.0;
        if (fnorm1 < fnorm) {
          const double q = fnorm1 / fnorm;
          actred = 1.0 - q * q;
        }
        int l = 0;
        for (int i = 0; i < n; ++i) {
          double sum = 0.0;
          for (int j = i; j < n; ++j) {
            sum = sum + r[l] * wa1[j];
            ++l;
          }
          wa3[i] = qtf[i] + sum;
        }
        const double temp = enorm(n, wa3.data());
        double prered = 0.0;
        if (temp < fnorm) {
          const double q = temp / fnorm;
          prered = 1.0 - q * q;
        }
        double ratio = 0.0;
        if (prered > 0.0) ratio = actred / prered;
        if (ratio < p1) {
          ncsuc = 0;
          ncfail = ncfail + 1;
          delta = p5 * delta;
        } else {
          ncfail = 0;
          ncsuc = ncsuc + 1;
          if (ratio >= p5 || ncsuc > 1) delta = std::fmax(delta, pnorm / p5);
          if (std::fabs(ratio - 1.0) <= p1) delta = pnorm / p5;
        }
        if (ratio >= p0001) {   // successful iteration
          for (int j = 0; j < n; ++j) {
            x[j] = wa2[j];
            wa2[j] = diag[j] * x[j];
            fvec[j] = wa4[j];
          }
          xnorm = enorm(n, wa2.data());
          fnorm = fnorm1;
          iter = iter + 1;
        }
        nslow1 = nslow1 + 1;
        if (actred >= p001) nslow1 = 0;
        if (jeval) nslow2 = nslow2 + 1;
        if (actred >= p1) nslow2 = 0;
        if (delta <= xtol * xnorm || fnorm == 0.0) info = 1;
        if (info != 0) break;
        if (nfev >= maxfev) info = 2;
        if (p1 * std::fmax(p1 * delta, pnorm) <= EPSMCH * xnorm) info = 3;
        if (nslow2 == 5) info = 4;
        if (nslow1 == 10) info = 5;
        if (info != 0) break;
        if (ncfail == 2) {   // recalculate the Jacobian by forward differences
          outer = true;
          break;
        }
        // rank-one modification of the Jacobian; update qtf if necessary
        for (int j = 0; j < n; ++j) {
          double sum = 0.0;
          for (int i = 0; i < n; ++i) sum = sum + J(i, j) * wa4[i];
          wa2[j] = (sum - wa3[j]) / pnorm;
          wa1[j] = diag[j] * ((diag[j] * wa1[j]) / pnorm);
          if (ratio >= p0001) qtf[j] = sum;
        }
        r1updt(n, n, r.data(), wa1.data(), wa2.data(), wa3.data());
        r1mpyq(n, n, fjac.data(), n, wa2.data(), wa3.data());
        r1mpyq(1, n, qtf.data(), 1, wa2.data(), wa3.data());
        jeval = false;
      }
      if (!outer) break;
    }
    if (fvec_out) std::memcpy(fvec_out, fvec.data(), sizeof(double) * n);
  }
  if (nfev_out) *nfev_out = nfev;
  return info;
}

extern "C" int sgv_fsolve(int n, sgv_fsolve_fn fcn, void* user, double* x_io, double* fvec_out,
                          int* nfev_out) {
  return sgv_fsolve_jac(n, fcn, nullptr, user, x_io, fvec_out, nfev_out);
}
