// riptrm_trs_big.hip — Exact_RepMat above RIPTRM_TRS_DIM_MAX.
//
// Reference: compute_direction's Exact_RepMat branch (src/solver/RIPTRM.py:433-444) builds the
// matrix of HwCur in a tangent basis (selfadj_operator2matrix, src/solver/utils.py:565-573) and
// solves TRSgep (RIPTRM.py:218-299); with second_order_stationarity the smallest eigenvalue of
// the same matrix at every trial point is tested (RIPTRM.py:599-617).  No size cap there.
//
// Up to dim 96 the whole subproblem runs inside the state kernel on a matrix held in LDS
// (riptrm_trs.h).  Beyond that the matrix lives in HBM, in caller-owned scratch bound with
// riptrm_trs_bind_workspace, and the library serves the subproblem between lock-step chunks:
//   1. A: NonnegPCA's closed form in the Householder frame of x^perp (the one trs_direction uses:
//      A = (H M H)[1:, 1:] + coef I, M = -S + diag(y / x), O(n^2) work): M densified from S,
//      u = M w by a wave-per-row mat-vec, then the rank-two update in place;
//   2. the interior candidate: SciPy's CG on A p = -a restated loop for loop (oracle
//      trs_oracle.scipy_cg), one mat-vec launch + one single-workgroup update launch per
//      iteration, the convergence flag polled every CG_POLL iterations;
//   3. A = Q diag(lam) Q^T by rocSOLVER dsyevd (loaded with dlopen the first time it is needed);
//   4. g = Q^T a, then the hard case / safeguarded secular Newton / interior choice of
//      riptrm_trs::trs_solve (the same formulas, one workgroup) and x = Q c;
//   5. eta = H [0; x] back in the ambient space, the state machine resumes at PH_TRS_END.
// The trial-point test (second_order_stationarity) builds the matrix at (x_new, y_new) the same
// way and takes dsyevd's smallest eigenvalue (eigenvalues only).
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <math.h>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include "riptrm_ctx.h"
#include "riptrm_wave.h"

using namespace riptrm;

namespace riptrm_big {

#pragma clang fp contract(off)

constexpr int WG = 512;        // single-workgroup kernels
constexpr int GV = 256;        // mat-vec workgroups: 4 waves, one row per wave at a time
constexpr int CG_POLL = 32;    // CG iterations enqueued between flag polls
constexpr int NSC = 32;        // scalar slots per workspace slot

// scalar slots
enum Sc : int {
  SC_TAU = 0, SC_GAM, SC_XX, SC_COEF, SC_WC, SC_AN, SC_ATOL, SC_RHO, SC_RHO_PREV, SC_IT, SC_DONE,
  SC_CG_OK, SC_P1OBJ, SC_KIND, SC_LAM1, SC_MINEIG, SC_INTERIOR, SC_DELTA, SC_XSX, SC_YX
};

__host__ __device__ inline int64_t vpad(int64_t n) { return (n + 63) / 64 * 64; }
constexpr int NVS = 12;        // vectors per slot
enum Vs : int { VS_W = 0, VS_U, VS_A, VS_CGX, VS_R, VS_P, VS_Q, VS_EV, VS_EW, VS_G, VS_PE, VS_X };

// one slot for matrices of order N: [N x N][NVS vectors of vpad(N)][NSC scalars][info]
__host__ __device__ inline int64_t slot_doubles(int64_t N) { return N * N + NVS * vpad(N) + NSC + 8; }

struct Slot {
  double* M;
  double* v[NVS];
  double* sc;
  int32_t* info;
};

inline Slot slot_at(char* base, int64_t N, int s) {
  Slot q;
  double* b = (double*)base + (int64_t)s * slot_doubles(N);
  q.M = b;
  for (int k = 0; k < NVS; ++k) q.v[k] = b + N * N + k * vpad(N);
  q.sc = b + N * N + NVS * vpad(N);
  q.info = (int32_t*)(q.sc + NSC);
  return q;
}

// ---- workgroup reductions (WG threads, fixed order, every thread gets the value) --------------
__device__ __forceinline__ double blk_sum(double v, double* red) {
  v = riptrm_wave::wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = red[0];
#pragma unroll
  for (int i = 1; i < WG / 64; ++i) s += red[i];
  return s;
}
__device__ __forceinline__ double blk_min(double v, double* red) {
  v = riptrm_wave::wave_min(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = red[0];
#pragma unroll
  for (int i = 1; i < WG / 64; ++i) s = fmin(s, red[i]);
  return s;
}
__device__ __forceinline__ double blk_max(double v, double* red) {
  v = riptrm_wave::wave_max(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = red[0];
#pragma unroll
  for (int i = 1; i < WG / 64; ++i) s = fmax(s, red[i]);
  return s;
}

// S_ij of instance b in its layout (MachineT::s_at's arithmetic)
__device__ __forceinline__ double s_at(const DevParams& P, int b, int i, int j) {
  const double* Sb = P.S + (int64_t)b * P.inst_stride;
  if (P.layout == RIPTRM_LAYOUT_SYMTILE) {
    int I = i / TS, J = j / TS;
    if (I > J) {
      const int t = i; i = j; j = t;
      const int u = I; I = J; J = u;
    }
    const int colsT = (J == P.nt - 1) ? P.wl : TS;
    return Sb[sym_off(I, J, P.nt, P.wl) + (int64_t)(i - I * TS) * colsT + (j - J * TS)];
  }
  return Sb[(int64_t)i * P.ld + j];
}

__device__ __forceinline__ const double* vec_of(const DevParams& P, int kind, int b) {
  return P.vec + ((int64_t)kind * P.batch + b) * P.ld;
}

// M = -S + diag(y / x) at (X, Y) = vectors xk, yk of instance b (n x n, row-major, lda n)
__global__ void __launch_bounds__(256) k_dense(DevParams P, int b, int xk, int yk, double* M) {
  const int n = P.n;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)n * n) return;
  const int i = (int)(e / n), j = (int)(e - (int64_t)i * n);
  double m = -s_at(P, b, i, j);
  if (i == j) m += vec_of(P, yk, b)[i] / vec_of(P, xk, b)[i];
  M[e] = m;
}

// w = x + sign(x_0) ||x|| e_0, tau = 2 / w^T w (the Householder reflector of trs_direction);
// xx = x^T x; trial mode (coef < 0 flag): also y^T x for the coefficient
__global__ void __launch_bounds__(WG) k_house(DevParams P, int b, int xk, int yk, double* w, double* sc) {
  __shared__ double red[WG / 64];
  const int n = P.n;
  const double* X = vec_of(P, xk, b);
  const double* Y = vec_of(P, yk, b);
  double xx = 0.0, yx = 0.0;
  for (int i = threadIdx.x; i < n; i += WG) {
    xx += X[i] * X[i];
    yx += Y[i] * X[i];
  }
  xx = blk_sum(xx, red);
  yx = blk_sum(yx, red);
  const double sg = X[0] >= 0.0 ? 1.0 : -1.0;
  double ww = 0.0;
  for (int i = threadIdx.x; i < n; i += WG) {
    const double wi = i == 0 ? X[0] + sg * sqrt(xx) : X[i];
    w[i] = wi;
    ww += wi * wi;
  }
  ww = blk_sum(ww, red);
  if (threadIdx.x == 0) {
    sc[SC_TAU] = 2.0 / ww;
    sc[SC_XX] = xx;
    sc[SC_YX] = yx;
  }
}

// out_i = sum_j A[i lda + j] v_j for i < rows (one wave per row, lanes over j; fixed order:
// lane partial sums in j order, then the wave tree).  skip: if non-null and *skip != 0, nothing.
__global__ void __launch_bounds__(GV) k_gemv(const double* A, int64_t lda, int rows, int cols, const double* v,
                                             double* out, const double* skip) {
  if (skip && *skip != 0.0) return;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (GV / 64) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const double* a = A + (int64_t)row * lda;
  double s = 0.0;
  for (int j = lane; j < cols; j += 64) s += a[j] * v[j];
  s = riptrm_wave::wave_sum(s);
  if (lane == 0) out[row] = s;
}

// out_i = sum_k A[k lda + i] v_k (columns of the row-major view: eigenvectors are rows of it);
// rows split over workgroups, each thread one i, k in order
__global__ void __launch_bounds__(256) k_gemv_t(const double* A, int64_t lda, int rows, int cols, const double* v,
                                                double* out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= cols) return;
  double s = 0.0;
  for (int k = 0; k < rows; ++k) s += A[(int64_t)k * lda + i] * v[k];
  out[i] = s;
}

// gam = w^T u, then (iterate) a_k = c_k - tau w_k (w^T c) for k >= 1 and coef from the state,
// or (trial) coef = (x^T S x + y^T x) x^T x with x^T S x = -x^T (M x) + y^T x (M = -S + diag(y/x))
__global__ void __launch_bounds__(WG) k_repmat_vec(DevParams P, int b, int xk, int ck, const double* w, const double* u,
                                                   const double* mx, double* a, double* sc, int trial) {
  __shared__ double red[WG / 64];
  const int n = P.n;
  double gam = 0.0, wc = 0.0, xmx = 0.0;
  const double* Cv = ck >= 0 ? vec_of(P, ck, b) : nullptr;
  const double* X = vec_of(P, xk, b);
  for (int i = threadIdx.x; i < n; i += WG) {
    gam += w[i] * u[i];
    if (Cv) wc += w[i] * Cv[i];
    if (trial) xmx += X[i] * mx[i];
  }
  gam = blk_sum(gam, red);
  wc = blk_sum(wc, red);
  xmx = blk_sum(xmx, red);
  const double tau = sc[SC_TAU];
  if (Cv)
    for (int k = threadIdx.x + 1; k < n; k += WG) a[k - 1] = Cv[k] - tau * w[k] * wc;
  if (threadIdx.x == 0) {
    sc[SC_GAM] = gam;
    sc[SC_WC] = wc;
    if (trial) {
      const double xSx = -xmx + sc[SC_YX];
      sc[SC_XSX] = xSx;
      sc[SC_COEF] = (xSx + sc[SC_YX]) * sc[SC_XX];
    } else {
      sc[SC_COEF] = P.st[(int64_t)b * ST_N + ST_COEF];
    }
  }
}

// in place, rows / columns 1.. of M: A = M - tau (w u^T + u w^T) + tau^2 gam w w^T + coef I
// (repmat's arithmetic, element for element)
__global__ void __launch_bounds__(256) k_transform(int n, double* M, const double* w, const double* u, const double* sc) {
  const int m = n - 1;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)m * m) return;
  const int i = (int)(e / m) + 1, j = (int)(e - (int64_t)(i - 1) * m) + 1;
  const double tau = sc[SC_TAU];
  const double t2g = (tau * tau) * sc[SC_GAM];
  double v = (M[(int64_t)i * n + j] - tau * (w[i] * u[j] + u[i] * w[j])) + t2g * (w[i] * w[j]);
  if (i == j) v += sc[SC_COEF];
  M[(int64_t)i * n + j] = v;
}

// ---- SciPy CG on A p = -a (trs_oracle.scipy_cg; riptrm_trs::trs_solve's loop) ------------------
__global__ void __launch_bounds__(WG) k_cg_init(int m, const double* a, double* cgx, double* r, double* sc) {
  __shared__ double red[WG / 64];
  double an = 0.0;
  for (int i = threadIdx.x; i < m; i += WG) {
    const double bi = -a[i];
    cgx[i] = 0.0;
    r[i] = bi;
    an += bi * bi;
  }
  an = sqrt(blk_sum(an, red));
  if (threadIdx.x == 0) {
    sc[SC_AN] = an;
    sc[SC_ATOL] = 1e-5 * an;
    sc[SC_IT] = 0.0;
    sc[SC_RHO_PREV] = 1.0;
    sc[SC_DONE] = an == 0.0 ? 2.0 : 0.0;   // b = 0: cg returns b; never eligible
  }
}

// top of a CG iteration: the convergence test, then the direction
__global__ void __launch_bounds__(WG) k_cg_dir(int m, const double* r, double* p, double* sc) {
  __shared__ double red[WG / 64];
  if (sc[SC_DONE] != 0.0) return;
  const double it = sc[SC_IT];
  if (it >= 10.0 * m) {   // maxiter = 10 n
    if (threadIdx.x == 0) sc[SC_DONE] = 3.0;
    return;
  }
  double rr = 0.0;
  for (int i = threadIdx.x; i < m; i += WG) rr += r[i] * r[i];
  rr = blk_sum(rr, red);
  if (sqrt(rr) < sc[SC_ATOL]) {
    if (threadIdx.x == 0) sc[SC_DONE] = 1.0;
    return;
  }
  const double rho = rr;
  const double beta = it > 0.0 ? rho / sc[SC_RHO_PREV] : 0.0;
  for (int i = threadIdx.x; i < m; i += WG) p[i] = it > 0.0 ? p[i] * beta + r[i] : r[i];
  if (threadIdx.x == 0) sc[SC_RHO] = rho;
}

__global__ void __launch_bounds__(WG) k_cg_upd(int m, const double* p, const double* q, double* cgx, double* r,
                                               double* sc) {
  __shared__ double red[WG / 64];
  if (sc[SC_DONE] != 0.0) return;
  double pq = 0.0;
  for (int i = threadIdx.x; i < m; i += WG) pq += p[i] * q[i];
  pq = blk_sum(pq, red);
  const double alpha = sc[SC_RHO] / pq;
  for (int i = threadIdx.x; i < m; i += WG) {
    cgx[i] += alpha * p[i];
    r[i] -= alpha * q[i];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    sc[SC_RHO_PREV] = sc[SC_RHO];
    sc[SC_IT] += 1.0;
  }
}

// ||A p1 + a|| / ||a|| < 1e-5 and p1^T p1 < Delta^2 (RIPTRM.py:246-251); p1's model value
__global__ void __launch_bounds__(WG) k_cg_final(int m, const double* a, const double* cgx, const double* q,
                                                 const double* Delta, double* sc) {
  __shared__ double red[WG / 64];
  double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0;
  for (int i = threadIdx.x; i < m; i += WG) {
    const double res = q[i] + a[i];
    v0 += res * res;
    v1 += cgx[i] * cgx[i];
    v2 += cgx[i] * q[i];
    v3 += a[i] * cgx[i];
  }
  v0 = blk_sum(v0, red);
  v1 = blk_sum(v1, red);
  v2 = blk_sum(v2, red);
  v3 = blk_sum(v3, red);
  if (threadIdx.x == 0) {
    const double an = sc[SC_AN];
    const double D = *Delta;
    sc[SC_CG_OK] = (an != 0.0 && sqrt(v0) / an < 1e-5 && v1 < D * D) ? 1.0 : 0.0;
    sc[SC_P1OBJ] = 0.5 * v2 + v3;
    sc[SC_DELTA] = D;
  }
}

// After dsyevd (ev ascending) and g = Q^T a: the hard case / secular Newton / interior choice of
// riptrm_trs::trs_solve; writes the eigen coordinates pe of the boundary / hard-case candidate and
// the result scalars
__global__ void __launch_bounds__(WG) k_secular(int m, const double* ev, const double* g, double* pe, double tolhc,
                                                double* sc) {
  __shared__ double red[WG / 64];
  const double Delta = sc[SC_DELTA];
  const double D2 = Delta * Delta;
  const double lmin = ev[0];   // ascending: the lowest index of the minimum
  double lmax_abs = 0.0;
  for (int i = threadIdx.x; i < m; i += WG) lmax_abs = fmax(lmax_abs, fabs(ev[i]));
  lmax_abs = blk_max(lmax_abs, red);
  const double hard_tol = 1e-12 * fmax(1.0, lmax_abs);
  double gh = 0.0, gg = 0.0;
  for (int i = threadIdx.x; i < m; i += WG) {
    const double gi = g[i];
    gg += gi * gi;
    if (fabs(ev[i] - lmin) <= hard_tol) gh += gi * gi;
  }
  const double ghard = sqrt(blk_sum(gh, red));
  const double gn = sqrt(blk_sum(gg, red));
  const double lo = -lmin;
  bool have = false;
  double lam1 = 0.0;
  int kind = 0;   // riptrm_trs::K_BOUNDARY
  if (ghard <= tolhc * gn) {
    double x2 = 0.0;
    for (int i = threadIdx.x; i < m; i += WG) {
      const bool hs = fabs(ev[i] - lmin) <= hard_tol;
      const double c = hs ? 0.0 : -g[i] / (ev[i] - lmin);
      pe[i] = c;
      x2 += c * c;
    }
    x2 = blk_sum(x2, red);
    if (x2 < D2) {
      const double alp = sqrt(D2 - x2);
      __syncthreads();
      if (threadIdx.x == 0) pe[0] += alp;
      __syncthreads();
      lam1 = lo;
      kind = 2;   // K_HARDCASE_1
      have = true;
    }
  }
  if (!have) {
    double l1 = lo + gn / Delta;
    for (int itn = 0; itn < 100; ++itn) {
      double s2 = 0.0, s3 = 0.0;
      for (int i = threadIdx.x; i < m; i += WG) {
        const double den = ev[i] + l1;
        const double gi = g[i];
        s2 += (gi / den) * (gi / den);
        s3 += (gi * gi) / (den * den * den);
      }
      s2 = blk_sum(s2, red);
      s3 = blk_sum(s3, red);
      const double xn = sqrt(s2);
      const double f = 1.0 / xn - 1.0 / Delta;
      const double fp = s3 / (xn * xn * xn);
      double nl = l1 - f / fp;
      if (nl <= lo) nl = 0.5 * (lo + l1);
      if (fabs(nl - l1) <= 1e-15 * fmax(1.0, fabs(l1))) {
        l1 = nl;
        break;
      }
      l1 = nl;
    }
    double s2 = 0.0;
    for (int i = threadIdx.x; i < m; i += WG) {
      const double c = -g[i] / (ev[i] + l1);
      pe[i] = c;
      s2 += c * c;
    }
    const double scl = Delta / sqrt(blk_sum(s2, red));
    __syncthreads();
    for (int i = threadIdx.x; i < m; i += WG) pe[i] = pe[i] * scl;
    lam1 = l1;
    kind = 0;
  }
  __syncthreads();
  double o0 = 0.0, o1 = 0.0;
  for (int i = threadIdx.x; i < m; i += WG) {
    const double c = pe[i];
    o0 += ev[i] * c * c;
    o1 += g[i] * c;
  }
  const double xobj = 0.5 * blk_sum(o0, red) + blk_sum(o1, red);
  const bool interior = sc[SC_CG_OK] != 0.0 && sc[SC_P1OBJ] <= xobj;   // RIPTRM.py:294-298
  if (threadIdx.x == 0) {
    sc[SC_INTERIOR] = interior ? 1.0 : 0.0;
    sc[SC_KIND] = interior ? 1.0 : (double)kind;   // riptrm_trs::Kind
    sc[SC_LAM1] = interior ? 0.0 : lam1;
    sc[SC_MINEIG] = lmin;
  }
}

// x <- cgx when the interior candidate won (x = Q pe was computed before)
__global__ void __launch_bounds__(256) k_pick(int m, const double* cgx, double* x, const double* sc) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < m && sc[SC_INTERIOR] != 0.0) x[i] = cgx[i];
}

// eta = H [0; x] (RIPTRM.py:442-444 in the Householder frame), the direction type, j = -1, and the
// instance resumes at PH_TRS_END
__global__ void __launch_bounds__(WG) k_finish_dir(DevParams P, int b, const double* w, const double* x, const double* sc,
                                                   const int32_t* info) {
  __shared__ double red[WG / 64];
  const int n = P.n;
  double wz = 0.0;
  for (int k = threadIdx.x + 1; k < n; k += WG) wz += w[k] * x[k - 1];
  wz = blk_sum(wz, red);
  const double tau = sc[SC_TAU];
  double* E = P.vec + ((int64_t)V_ETA * P.batch + b) * P.ld;
  for (int i = threadIdx.x; i < n; i += WG) E[i] = (i == 0 ? 0.0 : x[i - 1]) - tau * w[i] * wz;
  if (threadIdx.x == 0) {
    double* s = P.st + (int64_t)b * ST_N;
    // dsyevd did not converge (info > 0): scipy.linalg.eig would raise LinAlgError inside
    // outer_step (RIPTRM.py:961-966); the machine stops the instance at PH_TRS_END
    s[ST_TCG_STOP] = *info != 0 ? (double)RIPTRM_TCG_EIGFAIL : RIPTRM_TRS_BOUNDARY + sc[SC_KIND];
    s[ST_J] = -1.0;
    s[ST_PHASE] = PH_TRS_END;
  }
}

__global__ void k_finish_mineig(DevParams P, int b, const double* ev, const int32_t* info) {
  double* s = P.st + (int64_t)b * ST_N;
  s[ST_MINEIG] = *info != 0 ? NAN : ev[0];   // non-converged dsyevd: the machine stops the instance
  s[ST_PHASE] = PH_MINEIG_END;
}

// riptrm_trs_gep outputs for one subproblem
__global__ void __launch_bounds__(256) k_gep_out(int m, const double* x, const double* sc, const double* ev, double* xo,
                                                 double* lam1, int32_t* kind, double* mineig) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < m) xo[i] = x[i];
  if (i == 0) {
    *lam1 = sc[SC_LAM1];
    *kind = RIPTRM_TRS_BOUNDARY + (int32_t)sc[SC_KIND];
    if (mineig) *mineig = ev[0];
  }
}

// copy an m x m block (row-major, lda) into the slot's matrix (lda m) and a into the slot
__global__ void __launch_bounds__(256) k_load(int m, const double* A, int64_t lda, const double* a, double* M, double* av) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < (int64_t)m * m) {
    const int i = (int)(e / m), j = (int)(e - (int64_t)i * m);
    M[e] = A[(int64_t)i * lda + j];
  }
  if (e < m) av[e] = a[e];
}

// ---- rocSOLVER, loaded on first use (no link-time dependency of the library) -----------------------
// (RIPTRM_ROCBLAS_LIB / RIPTRM_ROCSOLVER_LIB in the environment name other libraries: a host whose
// ROCm is elsewhere, or a test that checks the failure path)
typedef int (*fn_create_t)(void**);
typedef int (*fn_set_stream_t)(void*, hipStream_t);
typedef int (*fn_destroy_t)(void*);
typedef int (*fn_syevd_t)(void*, int, int, int, double*, int, double*, double*, int*);
constexpr int EVECT_ORIGINAL = 211, EVECT_NONE = 213, FILL_UPPER = 121;

struct Solver {
  bool tried = false, ok = false;
  std::string why;
  fn_create_t create = nullptr;
  fn_set_stream_t set_stream = nullptr;
  fn_destroy_t destroy = nullptr;
  fn_syevd_t syevd = nullptr;
};

static Solver& solver() {
  static Solver s;
  if (s.tried) return s;
  s.tried = true;
  // dlerror() returns the last message once and clears it: record it right after each failure
  auto open_first = [](const char* a, const char* b) -> void* {
    void* h = dlopen(a, RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen(b, RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      const char* de = dlerror();
      s.why += std::string(s.why.empty() ? "" : "; ") + a + ": " + (de ? de : "not found");
    }
    return h;
  };
  const char* eb = getenv("RIPTRM_ROCBLAS_LIB");
  const char* es = getenv("RIPTRM_ROCSOLVER_LIB");
  void* blas = eb && *eb ? open_first(eb, eb) : open_first("librocblas.so.5", "librocblas.so");
  void* sol = es && *es ? open_first(es, es) : open_first("librocsolver.so.0", "librocsolver.so");
  if (!blas || !sol) {
    s.why = "cannot load rocBLAS / rocSOLVER: " + s.why;
    return s;
  }
  s.create = (fn_create_t)dlsym(blas, "rocblas_create_handle");
  s.set_stream = (fn_set_stream_t)dlsym(blas, "rocblas_set_stream");
  s.destroy = (fn_destroy_t)dlsym(blas, "rocblas_destroy_handle");
  s.syevd = (fn_syevd_t)dlsym(sol, "rocsolver_dsyevd");
  s.ok = s.create && s.set_stream && s.destroy && s.syevd;
  if (!s.ok) s.why = "rocBLAS / rocSOLVER lack rocblas_create_handle / rocblas_set_stream / rocsolver_dsyevd";
  return s;
}

}  // namespace riptrm_big

using namespace riptrm_big;

static unsigned blocks_of(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

static int big_handle(riptrm_ctx* c) {
  Solver& s = solver();
  if (!s.ok) return fail(c, RIPTRM_E_HIP, "Exact_RepMat above dim " + std::to_string(RIPTRM_TRS_DIM_MAX) + ": " + s.why);
  if (!c->big_handle) {
    void* h = nullptr;
    if (s.create(&h) != 0 || !h) return fail(c, RIPTRM_E_HIP, "rocblas_create_handle failed");
    c->big_handle = h;
  }
  if (s.set_stream(c->big_handle, c->stream) != 0) return fail(c, RIPTRM_E_HIP, "rocblas_set_stream failed");
  return RIPTRM_OK;
}

void riptrm_big_release(riptrm_ctx* c) {
  if (c && c->big_handle) {
    Solver& s = solver();
    if (s.ok) (void)s.destroy(c->big_handle);
    c->big_handle = nullptr;
  }
}

// The subproblem min x^T A x / 2 + a^T x s.t. ||x|| <= Delta on the slot: A = q.M + off with leading
// dimension lda (m x m), a = q.v[VS_A].  CG (interior candidate), dsyevd, secular solve; the
// solution lands in q.v[VS_X], the scalars in q.sc.  A is destroyed (eigenvectors).
static int big_solve(riptrm_ctx* c, Slot& q, double* A, int lda, int m, const double* Delta_dev, double tolhc) {
  hipStream_t st = c->stream;
  double* a = q.v[VS_A];
  hipLaunchKernelGGL(k_cg_init, dim3(1), dim3(WG), 0, st, m, a, q.v[VS_CGX], q.v[VS_R], q.sc);
  HIPCHK(c, hipGetLastError());
  double done = 0.0;
  for (int it = 0; it < 10 * m + 1; it += CG_POLL) {
    for (int k = 0; k < CG_POLL; ++k) {
      hipLaunchKernelGGL(k_cg_dir, dim3(1), dim3(WG), 0, st, m, q.v[VS_R], q.v[VS_P], q.sc);
      hipLaunchKernelGGL(k_gemv, dim3(blocks_of(m, GV / 64)), dim3(GV), 0, st, A, (int64_t)lda, m, m, q.v[VS_P],
                         q.v[VS_Q], q.sc + SC_DONE);
      hipLaunchKernelGGL(k_cg_upd, dim3(1), dim3(WG), 0, st, m, q.v[VS_P], q.v[VS_Q], q.v[VS_CGX], q.v[VS_R], q.sc);
    }
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(&done, q.sc + SC_DONE, sizeof(double), hipMemcpyDeviceToHost, st));
    HIPCHK(c, hipStreamSynchronize(st));
    if (done != 0.0) break;
  }
  hipLaunchKernelGGL(k_gemv, dim3(blocks_of(m, GV / 64)), dim3(GV), 0, st, A, (int64_t)lda, m, m, q.v[VS_CGX],
                     q.v[VS_Q], nullptr);
  hipLaunchKernelGGL(k_cg_final, dim3(1), dim3(WG), 0, st, m, a, q.v[VS_CGX], q.v[VS_Q], Delta_dev, q.sc);
  HIPCHK(c, hipGetLastError());
  if (int rc = big_handle(c)) return rc;
  if (solver().syevd(c->big_handle, EVECT_ORIGINAL, FILL_UPPER, m, A, lda, q.v[VS_EV], q.v[VS_EW], q.info) != 0)
    return fail(c, RIPTRM_E_HIP, "rocsolver_dsyevd failed");
  // eigenvector k = row k of the row-major view (column k of dsyevd's column-major output)
  hipLaunchKernelGGL(k_gemv, dim3(blocks_of(m, GV / 64)), dim3(GV), 0, st, A, (int64_t)lda, m, m, a, q.v[VS_G], nullptr);
  hipLaunchKernelGGL(k_secular, dim3(1), dim3(WG), 0, st, m, q.v[VS_EV], q.v[VS_G], q.v[VS_PE], tolhc, q.sc);
  hipLaunchKernelGGL(k_gemv_t, dim3(blocks_of(m, 256)), dim3(256), 0, st, A, (int64_t)lda, m, m, q.v[VS_PE], q.v[VS_X]);
  hipLaunchKernelGGL(k_pick, dim3(blocks_of(m, 256)), dim3(256), 0, st, m, q.v[VS_CGX], q.v[VS_X], q.sc);
  HIPCHK(c, hipGetLastError());
  return RIPTRM_OK;
}

// matrix of HwCur (trial = 0: at (x, y), the subproblem's linear term from cxCur) or of HwNew
// (trial = 1: at (x_new, y_new)) for NonnegPCA instance b, in the slot: A at q.M + n + 1, lda n
static int big_nonnegpca_matrix(riptrm_ctx* c, Slot& q, int b, int trial) {
  hipStream_t st = c->stream;
  const DevParams& P = c->P;
  const int n = P.n;
  const int xk = trial ? V_IN1 : V_X, yk = trial ? V_YNEW : V_Y;
  hipLaunchKernelGGL(k_dense, dim3(blocks_of((int64_t)n * n, 256)), dim3(256), 0, st, P, b, xk, yk, q.M);
  hipLaunchKernelGGL(k_house, dim3(1), dim3(WG), 0, st, P, b, xk, yk, q.v[VS_W], q.sc);
  hipLaunchKernelGGL(k_gemv, dim3(blocks_of(n, GV / 64)), dim3(GV), 0, st, q.M, (int64_t)n, n, n, q.v[VS_W], q.v[VS_U],
                     nullptr);
  const double* Xv = P.vec + ((int64_t)xk * P.batch + b) * P.ld;
  if (trial)   // M x_new for x^T S x
    hipLaunchKernelGGL(k_gemv, dim3(blocks_of(n, GV / 64)), dim3(GV), 0, st, q.M, (int64_t)n, n, n, Xv, q.v[VS_Q],
                       nullptr);
  hipLaunchKernelGGL(k_repmat_vec, dim3(1), dim3(WG), 0, st, P, b, xk, trial ? -1 : (int)V_C, q.v[VS_W], q.v[VS_U],
                     q.v[VS_Q], q.v[VS_A], q.sc, trial);
  hipLaunchKernelGGL(k_transform, dim3(blocks_of((int64_t)(n - 1) * (n - 1), 256)), dim3(256), 0, st, n, q.M, q.v[VS_W],
                     q.v[VS_U], q.sc);
  HIPCHK(c, hipGetLastError());
  return RIPTRM_OK;
}

// Serve every instance parked at PH_TRS_HOST / PH_MINEIG_HOST (one at a time, slot 0).  Returns the
// number of instances resumed in *served.  Synchronises.
int riptrm_big_service(riptrm_ctx* c, int* served) {
  *served = 0;
  const DevParams& P = c->P;
  const int B = P.batch, n = P.n;
  std::vector<double> st((size_t)B * RIPTRM_STAT_NFIELDS);
  HIPCHK(c, hipMemcpyAsync(st.data(), P.stats, st.size() * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (int b = 0; b < B; ++b) {
    const int ph = (int)st[(size_t)b * RIPTRM_STAT_NFIELDS + RIPTRM_STAT_PHASE];
    if (ph != PH_TRS_HOST && ph != PH_MINEIG_HOST) continue;
    if (!c->big_ws || c->big_order < n || c->big_slots < 1)
      return fail(c, RIPTRM_E_STATE, "Exact_RepMat above dim 96 needs riptrm_trs_bind_workspace (order >= n)");
    Slot q = slot_at(c->big_ws, c->big_order, 0);
    const int trial = ph == PH_MINEIG_HOST;
    if (int rc = big_nonnegpca_matrix(c, q, b, trial)) return rc;
    double* A = q.M + n + 1;   // rows / columns 1.. of the n x n buffer
    if (trial) {
      if (int rc = big_handle(c)) return rc;
      if (solver().syevd(c->big_handle, EVECT_NONE, FILL_UPPER, n - 1, A, n, q.v[VS_EV], q.v[VS_EW], q.info) != 0)
        return fail(c, RIPTRM_E_HIP, "rocsolver_dsyevd failed");
      hipLaunchKernelGGL(k_finish_mineig, dim3(1), dim3(1), 0, c->stream, P, b, q.v[VS_EV], q.info);
    } else {
      const double* Delta = P.st + (int64_t)b * ST_N + ST_DELTA;
      if (int rc = big_solve(c, q, A, n, n - 1, Delta, P.opt.trs_tolhardcase)) return rc;
      hipLaunchKernelGGL(k_finish_dir, dim3(1), dim3(WG), 0, c->stream, P, b, q.v[VS_W], q.v[VS_X], q.sc, q.info);
    }
    HIPCHK(c, hipGetLastError());
    ++*served;
  }
  return RIPTRM_OK;
}

// riptrm_trs_gep for dim > RIPTRM_TRS_DIM_MAX: one subproblem at a time through slot 0
int riptrm_big_trs_gep(riptrm_ctx* c, int dim, int batch, const double* A, int64_t lda, int64_t a_stride, const double* a,
                       int64_t ldv, const double* Delta, double tolhc, double* x, double* lam1, int32_t* kind,
                       double* mineig) {
  if (!c->big_ws || c->big_order < dim || c->big_slots < 1)
    return fail(c, RIPTRM_E_STATE, "trs_gep above dim 96 needs riptrm_trs_bind_workspace (order >= dim)");
  Slot q = slot_at(c->big_ws, c->big_order, 0);
  for (int b = 0; b < batch; ++b) {
    hipLaunchKernelGGL(k_load, dim3(blocks_of((int64_t)dim * dim, 256)), dim3(256), 0, c->stream, dim,
                       A + (int64_t)b * a_stride, lda, a + (int64_t)b * ldv, q.M, q.v[VS_A]);
    HIPCHK(c, hipGetLastError());
    if (int rc = big_solve(c, q, q.M, dim, dim, Delta + b, tolhc)) return rc;
    int32_t info = 0;
    HIPCHK(c, hipMemcpyAsync(&info, q.info, sizeof(info), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (info != 0)   // scipy.linalg.eig raises LinAlgError here
      return fail(c, RIPTRM_E_HIP, "trs_gep: rocsolver_dsyevd did not converge (info " + std::to_string(info) +
                                       ") on subproblem " + std::to_string(b));
    hipLaunchKernelGGL(k_gep_out, dim3(blocks_of(dim, 256)), dim3(256), 0, c->stream, dim, q.v[VS_X], q.sc, q.v[VS_EV],
                       x + (int64_t)b * ldv, lam1 + b, kind + b, mineig ? mineig + b : nullptr);
    HIPCHK(c, hipGetLastError());
  }
  return RIPTRM_OK;
}

extern "C" {

int riptrm_trs_backend_status(char* msg, int32_t len) {
  Solver& s = solver();
  if (msg && len > 0) {
    const std::string t = s.ok ? std::string("rocBLAS + rocSOLVER dsyevd loaded") : s.why;
    std::strncpy(msg, t.c_str(), (size_t)len - 1);
    msg[len - 1] = 0;
  }
  return s.ok ? RIPTRM_OK : RIPTRM_E_HIP;
}

int64_t riptrm_trs_workspace_bytes(int32_t order, int32_t slots) {
  if (order < 1 || slots < 1) return 0;
  return slot_doubles(order) * 8 * (int64_t)slots + 256;
}

int riptrm_trs_bind_workspace(riptrm_ctx* ctx, void* ws, int64_t bytes, int32_t order, int32_t slots) {
  if (!ctx) return RIPTRM_E_ARG;
  if (!ws) {   // unbind
    ctx->big_ws = nullptr;
    ctx->big_order = ctx->big_slots = 0;
    return RIPTRM_OK;
  }
  if (order < 1 || slots < 1 || bytes < riptrm_trs_workspace_bytes(order, slots) - 256 || ((uintptr_t)ws % 256) != 0)
    return fail(ctx, RIPTRM_E_ARG, "trs_bind_workspace: need order, slots >= 1, 256-byte alignment and "
                                   "riptrm_trs_workspace_bytes(order, slots) bytes");
  ctx->big_ws = (char*)ws;
  ctx->big_order = order;
  ctx->big_slots = slots;
  return RIPTRM_OK;
}

}  // extern "C"
