// riptrm_trs_big.hip — Exact_RepMat above RIPTRM_TRS_DIM_MAX.
//
// Reference: compute_direction's Exact_RepMat branch (src/solver/RIPTRM.py:433-444) builds the
// matrix of HwCur in a tangent basis (selfadj_operator2matrix, src/solver/utils.py:565-573) and
// solves TRSgep (RIPTRM.py:218-299); with second_order_stationarity the smallest eigenvalue of
// the same matrix at every trial point is tested (RIPTRM.py:599-617).  No size cap there.
//
// Up to dim 96 the whole subproblem runs inside the state kernel on a matrix held in LDS
// (riptrm_trs.h).  Beyond that the matrices live in HBM, in caller-owned scratch bound with
// riptrm_trs_bind_workspace as `slots` slots of order `order`, and the library serves the
// subproblems between lock-step chunks, every parked instance at once (up to `slots` per pass;
// slot k is blockIdx.y of every launch and holds instance ids[k]):
//   1. A: NonnegPCA's closed form in the Householder frame of x^perp (the one trs_direction uses:
//      A = (H M H)[1:, 1:] + coef I, M = -S + diag(y / x), O(n^2) work): M densified from S,
//      u = M w by a wave-per-row mat-vec, then the rank-two update in place;
//   2. the interior candidate: SciPy's CG on A p = -a restated loop for loop (oracle
//      trs_oracle.scipy_cg).  Small orders: the whole CG in ONE launch, one workgroup per slot
//      (k_cg_wg: p and q in LDS, x and r in registers, A streamed from L2 / MALL every iteration).
//      Large orders: one grid-wide mat-vec launch + two single-workgroup launches per iteration for
//      all slots together, the "every slot done" flag polled every CG_POLL iterations;
//   3. A = Q diag(lam) Q^T by rocSOLVER dsyevd_strided_batched over the slots (loaded with dlopen
//      the first time it is needed);
//   4. g = Q^T a, then the hard case / safeguarded secular Newton / interior choice of
//      riptrm_trs::trs_solve (the same formulas, one workgroup per slot) and x = Q c;
//   5. eta = H [0; x] back in the ambient space, the state machine resumes at PH_TRS_END.
// The trial-point test (second_order_stationarity) builds the matrix at (x_new, y_new) the same
// way and takes dsyevd's smallest eigenvalue (eigenvalues only).  Every reduction has a fixed
// order, and a slot's arithmetic does not depend on which other slots share its pass.
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <math.h>
#include <algorithm>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>
#include "riptrm_ctx.h"
#include "riptrm_eig.h"
#include "riptrm_tri.h"
#include "riptrm_wave.h"

using namespace riptrm;

namespace riptrm_big {

#pragma clang fp contract(off)

constexpr int WG = 512;        // single-workgroup kernels
constexpr int GV = 256;        // mat-vec workgroups: 4 waves, one row per wave at a time
constexpr int CG_POLL = 32;    // CG iterations enqueued between flag polls (grid-wide CG)
constexpr int NSC = 32;        // scalar slots per workspace slot
constexpr int CG_WG_MAX = 2048;            // largest order of the one-workgroup CG (LDS p, q)
constexpr int CG_RPT = CG_WG_MAX / WG;     // x / r elements per thread there

// scalar slots
enum Sc : int {
  SC_TAU = 0, SC_GAM, SC_XX, SC_COEF, SC_WC, SC_AN, SC_ATOL, SC_RHO, SC_RHO_PREV, SC_IT, SC_DONE,
  SC_CG_OK, SC_P1OBJ, SC_KIND, SC_LAM1, SC_MINEIG, SC_INTERIOR, SC_DELTA, SC_XSX, SC_YX,
  SC_XOBJ, SC_BKIND, SC_BLAM1,  // the boundary / hard-case candidate, before the interior choice
  SC_TRI_FB                      // the tridiagonal path handed this subproblem to the eigendecomposition path
};

__host__ __device__ inline int64_t vpad(int64_t n) { return (n + 63) / 64 * 64; }
constexpr int NVS = 12;        // vectors per slot
enum Vs : int { VS_W = 0, VS_U, VS_A, VS_CGX, VS_R, VS_P, VS_Q, VS_EV, VS_EW, VS_G, VS_PE, VS_X };

// one slot for matrices of order N: [N x N][NVS vectors of vpad(N)][NSC scalars]; after the slots:
// int32 info[slots], ids[slots], flag[8], sweeps[slots], hits[slots] (+ pad), double residual[slots]
// ... then [the eigensolver's reflectors: riptrm_eig::refl_doubles(N)] (orders it serves)
// (every order m <= N the hand-written eigensolver or the tridiagonal path serves: N <= TRI_MAX)
__host__ __device__ inline int64_t refl_of(int64_t N) {
  return (int64_t)riptrm_eig::refl_doubles((int)(N <= riptrm_tri::TRI_MAX ? N : riptrm_eig::EIG_LDS_MAX));
}
__host__ __device__ inline int64_t slot_doubles(int64_t N) { return N * N + NVS * vpad(N) + NSC + refl_of(N); }
__host__ __device__ inline int64_t off_vec(int64_t N, int k) { return N * N + k * vpad(N); }
__host__ __device__ inline int64_t off_sc(int64_t N) { return N * N + NVS * vpad(N); }
__host__ __device__ inline int64_t off_refl(int64_t N) { return N * N + NVS * vpad(N) + NSC; }
inline int64_t tail_ints(int64_t slots) { return (4 * slots + 8 + 1) / 2 * 2; }   // even: the doubles stay aligned

// the per-instance eigendecomposition cache (riptrm_trs_bind_cache), order N: [Q: N x N][ev][x key]
// [y key][valid] (vectors vpad(N))
__host__ __device__ inline int64_t cache_doubles(int64_t N) { return N * N + 3 * vpad(N) + 8 + refl_of(N); }
inline int64_t tail_bytes(int64_t slots) { return tail_ints(slots) * 4 + slots * 8; }

// the slots of one pass: slot k (blockIdx.y) holds instance / subproblem ids[k]
struct Bat {
  double* base;
  int64_t N, sd;        // order, doubles per slot
  const int32_t* ids;
  int32_t* infos;
};

struct Slot {
  double* M;
  double* v[NVS];
  double* sc;
  int32_t* info;
};

__host__ __device__ inline Slot slot_at(const Bat& B, int k) {
  Slot q;
  double* b = B.base + (int64_t)k * B.sd;
  q.M = b;
  for (int i = 0; i < NVS; ++i) q.v[i] = b + off_vec(B.N, i);
  q.sc = b + off_sc(B.N);
  q.info = B.infos + k;
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

// M = -S + diag(y / x) at (X, Y) = vectors xk, yk of instance ids[k] (n x n, row-major, lda n)
__global__ void __launch_bounds__(256) k_dense(DevParams P, Bat B, int xk, int yk) {
  const int k = blockIdx.y, b = B.ids[k];
  const int n = P.n;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= (int64_t)n * n) return;
  const int i = (int)(e / n), j = (int)(e - (int64_t)i * n);
  double m = -s_at(P, b, i, j);
  if (i == j) m += vec_of(P, yk, b)[i] / vec_of(P, xk, b)[i];
  slot_at(B, k).M[e] = m;
}

// w = x + sign(x_0) ||x|| e_0, tau = 2 / w^T w (the Householder reflector of trs_direction);
// xx = x^T x; y^T x for the trial coefficient
__global__ void __launch_bounds__(WG) k_house(DevParams P, Bat B, int xk, int yk) {
  __shared__ double red[WG / 64];
  const int k = blockIdx.y, b = B.ids[k];
  const Slot q = slot_at(B, k);
  double* w = q.v[VS_W];
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
    q.sc[SC_TAU] = 2.0 / ww;
    q.sc[SC_XX] = xx;
    q.sc[SC_YX] = yx;
  }
}

// out_i = sum_j A[i lda + j] v_j for i < rows, per slot: A, v, out, skip at slot offsets (doubles
// from the slot start; skip < 0: none).  One wave per row, lanes over j; fixed order: lane partial
// sums in j order, then the wave tree.  If *skip != 0 the slot is left alone.
__global__ void __launch_bounds__(GV) k_gemv(Bat B, int64_t aoff, int64_t lda, int rows, int cols, int64_t voff,
                                             int64_t ooff, int64_t skipoff) {
  double* base = B.base + (int64_t)blockIdx.y * B.sd;
  if (skipoff >= 0 && base[skipoff] != 0.0) return;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (GV / 64) + (threadIdx.x >> 6);
  if (row >= rows) return;
  const double* a = base + aoff + (int64_t)row * lda;
  const double* v = base + voff;
  double s = 0.0;
  for (int j = lane; j < cols; j += 64) s += a[j] * v[j];
  s = riptrm_wave::wave_sum(s);
  if (lane == 0) base[ooff + row] = s;
}

// out = M x_new of instance ids[k] (the trial coefficient's x^T S x), the k_gemv arithmetic
__global__ void __launch_bounds__(GV) k_gemv_x(DevParams P, Bat B, int xk) {
  const int k = blockIdx.y, b = B.ids[k];
  const Slot q = slot_at(B, k);
  const int n = P.n;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (GV / 64) + (threadIdx.x >> 6);
  if (row >= n) return;
  const double* a = q.M + (int64_t)row * n;
  const double* v = vec_of(P, xk, b);
  double s = 0.0;
  for (int j = lane; j < n; j += 64) s += a[j] * v[j];
  s = riptrm_wave::wave_sum(s);
  if (lane == 0) q.v[VS_Q][row] = s;
}

// out_i = sum_k A[k lda + i] v_k (columns of the row-major view: eigenvectors are rows of it);
// rows split over workgroups, each thread one i, k in order
__global__ void __launch_bounds__(256) k_gemv_t(Bat B, int64_t aoff, int64_t lda, int rows, int cols, int64_t voff,
                                                int64_t ooff) {
  double* base = B.base + (int64_t)blockIdx.y * B.sd;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= cols) return;
  const double* A = base + aoff;
  const double* v = base + voff;
  double s = 0.0;
  for (int k = 0; k < rows; ++k) s += A[(int64_t)k * lda + i] * v[k];
  base[ooff + i] = s;
}

// gam = w^T u, then (iterate) a_k = c_k - tau w_k (w^T c) for k >= 1; coef = (x^T S x + y^T x) x^T x
// with x^T S x = -x^T (M x) + y^T x (M = -S + diag(y/x)) at the iterate and at the trial point
// alike, so the two matrices of the same (x, y) are the same bits (the trial point's
// eigendecomposition serves the next subproblem there: riptrm_trs_bind_cache)
__global__ void __launch_bounds__(WG) k_repmat_vec(DevParams P, Bat B, int xk, int ck) {
  __shared__ double red[WG / 64];
  const int k = blockIdx.y, b = B.ids[k];
  const Slot q = slot_at(B, k);
  const double *w = q.v[VS_W], *u = q.v[VS_U], *mx = q.v[VS_Q];
  double* a = q.v[VS_A];
  double* sc = q.sc;
  const int n = P.n;
  double gam = 0.0, wc = 0.0, xmx = 0.0;
  const double* Cv = ck >= 0 ? vec_of(P, ck, b) : nullptr;
  const double* X = vec_of(P, xk, b);
  for (int i = threadIdx.x; i < n; i += WG) {
    gam += w[i] * u[i];
    if (Cv) wc += w[i] * Cv[i];
    xmx += X[i] * mx[i];
  }
  gam = blk_sum(gam, red);
  wc = blk_sum(wc, red);
  xmx = blk_sum(xmx, red);
  const double tau = sc[SC_TAU];
  if (Cv)
    for (int i = threadIdx.x + 1; i < n; i += WG) a[i - 1] = Cv[i] - tau * w[i] * wc;
  if (threadIdx.x == 0) {
    sc[SC_GAM] = gam;
    sc[SC_WC] = wc;
    const double xSx = -xmx + sc[SC_YX];
    sc[SC_XSX] = xSx;
    sc[SC_COEF] = (xSx + sc[SC_YX]) * sc[SC_XX];
  }
}

// in place, rows / columns 1.. of M: A = M - tau (w u^T + u w^T) + tau^2 gam w w^T + coef I
// (repmat's arithmetic, element for element)
__global__ void __launch_bounds__(256) k_transform(int n, Bat B) {
  const Slot q = slot_at(B, blockIdx.y);
  const double *w = q.v[VS_W], *u = q.v[VS_U], *sc = q.sc;
  double* M = q.M;
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
// The one-workgroup form and the grid-wide form below do the same arithmetic in the same order
// (sums over i = t, t + WG, ... then the workgroup tree; mat-vec rows as k_gemv).

// ||A p1 + a|| / ||a|| < 1e-5 and p1^T p1 < Delta^2 (RIPTRM.py:246-251); p1's model value.
// Thread t's terms are elements t, t + WG, ...
__device__ __forceinline__ void cg_final_terms(double* red, double* sc, double an, double D, double v0, double v1,
                                               double v2, double v3) {
  v0 = blk_sum(v0, red);
  v1 = blk_sum(v1, red);
  v2 = blk_sum(v2, red);
  v3 = blk_sum(v3, red);
  if (threadIdx.x == 0) {
    sc[SC_CG_OK] = (an != 0.0 && sqrt(v0) / an < 1e-5 && v1 < D * D) ? 1.0 : 0.0;
    sc[SC_P1OBJ] = 0.5 * v2 + v3;
    sc[SC_DELTA] = D;
  }
}

typedef __attribute__((address_space(3))) double lds_f64;

// rows r0 .. r0 + 3 of A (leading dimension lda) . v: each row's own sum in k_gemv's order
template <typename TA>
__device__ __forceinline__ void wg_rows4(const TA* a0, int64_t lda, int r0, int m, const double* v, double* out) {
  const int lane = threadIdx.x & 63;
  double s[4] = {0.0, 0.0, 0.0, 0.0};
  for (int j = lane; j < m; j += 64) {
    const double vj = v[j];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (r0 + u < m) s[u] += a0[(int64_t)u * lda + j] * vj;
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const double t = riptrm_wave::wave_sum(s[u]);
    if (lane == 0 && r0 + u < m) out[r0 + u] = t;
  }
}

// q[row] = A[row] . v over rows m, 8 waves, FOUR rows at a time per wave (independent chains).
// Rows below rl (a multiple of 4) come from their LDS copy Al (leading dimension m): the same
// values, so the same sums.
__device__ __forceinline__ void wg_matvec(const double* __restrict__ A, int64_t lda, int m, const double* v,
                                          double* out, const lds_f64* Al = nullptr, int rl = 0) {
  const int w = threadIdx.x >> 6;
  for (int r0 = 4 * w; r0 < m; r0 += 4 * (WG / 64)) {
    if (r0 < rl) wg_rows4(Al + (int64_t)r0 * m, (int64_t)m, r0, m, v, out);
    else wg_rows4(A + (int64_t)r0 * lda, lda, r0, m, v, out);
  }
}

// rows of A the one-workgroup CG keeps in LDS (dynamic, next to its static p / q / red arrays): all
// of them up to m ~ 120 (SciPy's CG runs to its 10 m iteration cap on indefinite subproblems, so the
// per-iteration mat-vec latency is what counts there)
constexpr int CG_LDS_BYTES = 124 * 1024;
inline int cg_lds_rows(int m) {
  const char* e = getenv("RIPTRM_CG_LDS");   // "0": stream every row (A/B measurements)
  if (e && e[0] == '0') return 0;
  const int r = std::min(m, CG_LDS_BYTES / (8 * m));
  return r >= m ? m : r / 4 * 4;
}

// The whole CG (init, iterations, final test) for slot blockIdx.y, order m <= CG_WG_MAX; A at slot
// offset aoff with leading dimension lda; Delta of the slot at D[ids[k] * dstride]
// Aext (optional): A of slot k at Aext + ids[k] ext_stride instead of the slot (whose copy an
// eigensolve has already overwritten).  skip_indef: the eigenpairs (ev ascending, g = Q^T a) and the
// boundary candidate's model value xobj (k_secular, choose = 0) are known.  The CG is not run, and
// its candidate marked ineligible, only where a bound computed from them shows that no iterate it can
// return passes RIPTRM.py:294-298 (residual < 1e-5 ||a||, ||p1|| < Delta, p1obj <= xobj): with
// A p1 = -a + r, ||r|| <= 1e-5 ||a|| =: e, lam_s = min |lam_i| > 0,
//   ||p1|| >= ||p*|| - e / lam_s            (p* = -A^-1 a: ||p*||^2 = sum g_i^2 / lam_i^2)
//   p1obj = q(p*) + r^T A^-1 r / 2 >= -sum g_i^2 / lam_i / 2 - e^2 / (2 lam_s)
// so the skip needs ||p*|| (1 - 1e-6) - e / lam_s >= Delta, or that lower bound on p1obj above xobj
// by more than a rounding allowance; A not nearly singular (lam_s > 1e-8 max |lam|; definite or
// not: the bounds hold for any iterate with that residual).  Otherwise the CG runs (the same iterate
// as without the skip).
__global__ void __launch_bounds__(WG) k_cg_wg(Bat B, int m, int64_t aoff, int64_t lda, const double* D,
                                              int64_t dstride, int rl, const double* Aext = nullptr,
                                              int64_t ext_stride = 0, int skip_indef = 0) {
  __shared__ double red[WG / 64];
  __shared__ double ps[CG_WG_MAX], qs[CG_WG_MAX];
  extern __shared__ double arows[];   // rows 0 .. rl - 1 of A, leading dimension m
  const int k = blockIdx.y;
  const Slot q = slot_at(B, k);
  const double* A = Aext ? Aext + (int64_t)B.ids[k] * ext_stride : q.M + aoff;
  const double* a = q.v[VS_A];
  const int t = threadIdx.x;
  if (skip_indef) {
    const double *ev = q.v[VS_EV], *g = q.v[VS_G];
    const double lmax = fmax(fabs(ev[0]), fabs(ev[m - 1]));
    double lsm = INFINITY, s1 = 0.0, s2 = 0.0, aa = 0.0;
    for (int i = t; i < m; i += WG) {
      const double l = ev[i], gi = g[i];
      lsm = fmin(lsm, fabs(l));
      s1 += (gi / l) * (gi / l);
      s2 += gi * gi / l;
      aa += a[i] * a[i];
    }
    lsm = -blk_max(-lsm, red);
    s1 = blk_sum(s1, red);
    s2 = blk_sum(s2, red);
    const double e = 1e-5 * sqrt(blk_sum(aa, red));
    const double Dl = D[(int64_t)B.ids[k] * dstride];
    bool skip = *q.info == 0 && lsm > 1e-8 * lmax;
    if (skip) {
      const double xobj = q.sc[SC_XOBJ];
      const bool far = sqrt(s1) * (1.0 - 1e-6) - e / lsm >= Dl;
      const double p1lo = -0.5 * s2 - 0.5 * e * e / lsm;
      const bool worse = p1lo - xobj > 1e-6 * (fabs(s2) + fabs(xobj)) + 1e-10 * (e * 1e5) * Dl;
      skip = far || worse;
    }
    if (skip) {   // uniform over the workgroup
      if (t == 0) {
        q.sc[SC_CG_OK] = 0.0;
        q.sc[SC_P1OBJ] = 0.0;
        q.sc[SC_IT] = 0.0;
        q.sc[SC_DONE] = 4.0;
        q.sc[SC_DELTA] = D[(int64_t)B.ids[k] * dstride];
      }
      return;
    }
  }
  const lds_f64* Al = (const lds_f64*)arows;
  for (int64_t e = t; e < (int64_t)rl * m; e += WG) {
    const int i = (int)(e / m), j = (int)(e - (int64_t)i * m);
    arows[e] = A[(int64_t)i * lda + j];
  }
  __syncthreads();
  double x[CG_RPT], r[CG_RPT];
  double an = 0.0;
#pragma unroll
  for (int u = 0; u < CG_RPT; ++u) {
    const int i = t + u * WG;
    const double bi = i < m ? -a[i] : 0.0;
    x[u] = 0.0;
    r[u] = bi;
    an += bi * bi;
  }
  an = sqrt(blk_sum(an, red));
  const double atol = 1e-5 * an;
  double done = an == 0.0 ? 2.0 : 0.0, it = 0.0, rho_prev = 1.0;
  while (done == 0.0) {   // uniform: every thread holds the same scalars
    if (it >= 10.0 * m) {
      done = 3.0;
      break;
    }
    double rr = 0.0;
#pragma unroll
    for (int u = 0; u < CG_RPT; ++u) rr += r[u] * r[u];   // zero past m
    rr = blk_sum(rr, red);
    if (sqrt(rr) < atol) {
      done = 1.0;
      break;
    }
    const double rho = rr;
    const double beta = it > 0.0 ? rho / rho_prev : 0.0;
#pragma unroll
    for (int u = 0; u < CG_RPT; ++u) {
      const int i = t + u * WG;
      if (i < m) ps[i] = it > 0.0 ? ps[i] * beta + r[u] : r[u];
    }
    __syncthreads();
    wg_matvec(A, lda, m, ps, qs, Al, rl);
    __syncthreads();
    double pq = 0.0;
#pragma unroll
    for (int u = 0; u < CG_RPT; ++u) {
      const int i = t + u * WG;
      if (i < m) pq += ps[i] * qs[i];
    }
    pq = blk_sum(pq, red);
    const double alpha = rho / pq;
#pragma unroll
    for (int u = 0; u < CG_RPT; ++u) {
      const int i = t + u * WG;
      if (i < m) {
        x[u] += alpha * ps[i];
        r[u] -= alpha * qs[i];
      }
    }
    rho_prev = rho;
    it += 1.0;
  }
  // the final test needs A x: x through LDS
  __syncthreads();
#pragma unroll
  for (int u = 0; u < CG_RPT; ++u) {
    const int i = t + u * WG;
    if (i < m) {
      ps[i] = x[u];
      q.v[VS_CGX][i] = x[u];
    }
  }
  __syncthreads();
  wg_matvec(A, lda, m, ps, qs, Al, rl);
  __syncthreads();
  double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0;
#pragma unroll
  for (int u = 0; u < CG_RPT; ++u) {
    const int i = t + u * WG;
    if (i < m) {
      const double res = qs[i] + a[i];
      v0 += res * res;
      v1 += x[u] * x[u];
      v2 += x[u] * qs[i];
      v3 += a[i] * x[u];
    }
  }
  if (t == 0) {
    q.sc[SC_AN] = an;
    q.sc[SC_ATOL] = atol;
    q.sc[SC_IT] = it;
    q.sc[SC_DONE] = done;
  }
  cg_final_terms(red, q.sc, an, D[(int64_t)B.ids[k] * dstride], v0, v1, v2, v3);
}

// The same SciPy CG on ONE wave for orders m <= CGW_MAX (StableIdentification at d = 8: m = 100,
// where ill-conditioned subproblems run the CG to its 10 m iteration cap): A in LDS, two rows per
// lane, p broadcast from LDS, the dot products as wave reductions -- no workgroup barrier in the loop
// (k_cg_wg pays three per iteration).  Rows are zero-padded to a multiple of four and read 16 bytes at
// a time; the row stride cgw_stride(m) = 2 mod 4 doubles puts a 16-lane phase of those reads on
// distinct banks.  Its own fixed summation order (four partial sums per row, j mod 4, then
// (s0 + s1) + (s2 + s3)); skip_indef as k_cg_wg.
constexpr int CGW_MAX = 128;
typedef double cgw_d2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) cgw_d2 lds_d2;
__host__ __device__ inline int cgw_m4(int m) { return (m + 3) / 4 * 4; }
__host__ __device__ inline int cgw_stride(int m) { return cgw_m4(m) + 2; }
inline size_t cg_wave_lds(int m) { return ((size_t)m * cgw_stride(m) + CGW_MAX) * sizeof(double); }
__global__ void __launch_bounds__(64) k_cg_wave(Bat B, int m, int64_t aoff, int64_t lda, const double* D,
                                                int64_t dstride, const double* Aext = nullptr, int64_t ext_stride = 0,
                                                int skip_indef = 0) {
  extern __shared__ double cgs[];
  const int k = blockIdx.y;
  const Slot q = slot_at(B, k);
  const double* A = Aext ? Aext + (int64_t)B.ids[k] * ext_stride : q.M + aoff;
  const double* a = q.v[VS_A];
  const int l = threadIdx.x;
  const double Dl = D[(int64_t)B.ids[k] * dstride];
  if (skip_indef) {   // k_cg_wg's certified skip, with wave reductions
    const double *ev = q.v[VS_EV], *g = q.v[VS_G];
    const double lmax = fmax(fabs(ev[0]), fabs(ev[m - 1]));
    double lsm = INFINITY, s1 = 0.0, s2 = 0.0, aa = 0.0;
    for (int i = l; i < m; i += 64) {
      const double lv = ev[i], gi = g[i];
      lsm = fmin(lsm, fabs(lv));
      s1 += (gi / lv) * (gi / lv);
      s2 += gi * gi / lv;
      aa += a[i] * a[i];
    }
    lsm = riptrm_wave::wave_min(lsm);
    s1 = riptrm_wave::wave_sum(s1);
    s2 = riptrm_wave::wave_sum(s2);
    const double e = 1e-5 * sqrt(riptrm_wave::wave_sum(aa));
    bool skip = *q.info == 0 && lsm > 1e-8 * lmax;
    if (skip) {
      const double xobj = q.sc[SC_XOBJ];
      const bool far = sqrt(s1) * (1.0 - 1e-6) - e / lsm >= Dl;
      const double p1lo = -0.5 * s2 - 0.5 * e * e / lsm;
      const bool worse = p1lo - xobj > 1e-6 * (fabs(s2) + fabs(xobj)) + 1e-10 * (e * 1e5) * Dl;
      skip = far || worse;
    }
    if (skip) {
      if (l == 0) {
        q.sc[SC_CG_OK] = 0.0;
        q.sc[SC_P1OBJ] = 0.0;
        q.sc[SC_IT] = 0.0;
        q.sc[SC_DONE] = 4.0;
        q.sc[SC_DELTA] = Dl;
      }
      return;
    }
  }
  const int ms = cgw_stride(m), m4 = cgw_m4(m);
  lds_f64* Al = (lds_f64*)cgs;
  lds_f64* ps = Al + (int64_t)m * ms;
  for (int64_t e = l; e < (int64_t)m * ms; e += 64) {
    const int i = (int)(e / ms), j = (int)(e - (int64_t)i * ms);
    Al[e] = j < m ? A[(int64_t)i * lda + j] : 0.0;
  }
  for (int j = m + l; j < m4; j += 64) ps[j] = 0.0;
  double x[2] = {0.0, 0.0}, r[2];
  double an = 0.0;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = l + 64 * u;
    const double bi = i < m ? -a[i] : 0.0;
    r[u] = bi;
    an += bi * bi;
  }
  an = sqrt(riptrm_wave::wave_sum(an));
  const double atol = 1e-5 * an;
  double done = an == 0.0 ? 2.0 : 0.0, it = 0.0, rho_prev = 1.0;
  __syncthreads();
  // rows i = l and l + 64 of A . p, each with four partial sums (j mod 4), then (s0 + s1) + (s2 + s3);
  // both rows in one loop (twelve 16-byte loads in flight per step of four)
  auto matvec = [&](double* qv) {
    const int i0 = l < m ? l : m - 1, i1 = l + 64 < m ? l + 64 : m - 1;
    const lds_d2* r0 = (const lds_d2*)(Al + i0 * ms);
    const lds_d2* r1 = (const lds_d2*)(Al + i1 * ms);
    const lds_d2* pv = (const lds_d2*)ps;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0, b0 = 0.0, b1 = 0.0, b2 = 0.0, b3 = 0.0;
#pragma unroll 2
    for (int h = 0; h < m4 / 2; h += 2) {
      const cgw_d2 x0 = r0[h], x1 = r0[h + 1], y0 = r1[h], y1 = r1[h + 1], p0 = pv[h], p1 = pv[h + 1];
      a0 += x0.x * p0.x;
      a1 += x0.y * p0.y;
      a2 += x1.x * p1.x;
      a3 += x1.y * p1.y;
      b0 += y0.x * p0.x;
      b1 += y0.y * p0.y;
      b2 += y1.x * p1.x;
      b3 += y1.y * p1.y;
    }
    qv[0] = l < m ? (a0 + a1) + (a2 + a3) : 0.0;
    qv[1] = l + 64 < m ? (b0 + b1) + (b2 + b3) : 0.0;
  };
  while (done == 0.0) {   // uniform
    if (it >= 10.0 * m) {
      done = 3.0;
      break;
    }
    const double rr = riptrm_wave::wave_sum(r[0] * r[0] + r[1] * r[1]);   // zero past m
    if (sqrt(rr) < atol) {
      done = 1.0;
      break;
    }
    const double rho = rr;
    const double beta = it > 0.0 ? rho / rho_prev : 0.0;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = l + 64 * u;
      if (i < m) ps[i] = it > 0.0 ? ps[i] * beta + r[u] : r[u];
    }
    __syncthreads();
    double qv[2];
    matvec(qv);
    double pq = 0.0;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = l + 64 * u;
      if (i < m) pq += ps[i] * qv[u];
    }
    pq = riptrm_wave::wave_sum(pq);
    const double alpha = rho / pq;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (l + 64 * u < m) {
        x[u] += alpha * ps[l + 64 * u];
        r[u] -= alpha * qv[u];
      }
    }
    rho_prev = rho;
    it += 1.0;
    __syncthreads();
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = l + 64 * u;
    if (i < m) {
      ps[i] = x[u];
      q.v[VS_CGX][i] = x[u];
    }
  }
  __syncthreads();
  double qv[2];
  matvec(qv);
  double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = l + 64 * u;
    if (i < m) {
      const double res = qv[u] + a[i];
      v0 += res * res;
      v1 += x[u] * x[u];
      v2 += x[u] * qv[u];
      v3 += a[i] * x[u];
    }
  }
  v0 = riptrm_wave::wave_sum(v0);
  v1 = riptrm_wave::wave_sum(v1);
  v2 = riptrm_wave::wave_sum(v2);
  v3 = riptrm_wave::wave_sum(v3);
  if (l == 0) {
    q.sc[SC_AN] = an;
    q.sc[SC_ATOL] = atol;
    q.sc[SC_IT] = it;
    q.sc[SC_DONE] = done;
    q.sc[SC_CG_OK] = (an != 0.0 && sqrt(v0) / an < 1e-5 && v1 < Dl * Dl) ? 1.0 : 0.0;   // RIPTRM.py:246-251
    q.sc[SC_P1OBJ] = 0.5 * v2 + v3;
    q.sc[SC_DELTA] = Dl;
  }
}

// grid-wide CG, one launch each step for all slots (grid.y = slot)
__global__ void __launch_bounds__(WG) k_cg_init(Bat B, int m) {
  __shared__ double red[WG / 64];
  const Slot q = slot_at(B, blockIdx.y);
  const double* a = q.v[VS_A];
  double an = 0.0;
  for (int i = threadIdx.x; i < m; i += WG) {
    const double bi = -a[i];
    q.v[VS_CGX][i] = 0.0;
    q.v[VS_R][i] = bi;
    an += bi * bi;
  }
  an = sqrt(blk_sum(an, red));
  if (threadIdx.x == 0) {
    double* sc = q.sc;
    sc[SC_AN] = an;
    sc[SC_ATOL] = 1e-5 * an;
    sc[SC_IT] = 0.0;
    sc[SC_RHO_PREV] = 1.0;
    sc[SC_DONE] = an == 0.0 ? 2.0 : 0.0;   // b = 0: cg returns b; never eligible
  }
}

// top of a CG iteration: the convergence test, then the direction
__global__ void __launch_bounds__(WG) k_cg_dir(Bat B, int m) {
  __shared__ double red[WG / 64];
  const Slot q = slot_at(B, blockIdx.y);
  double* sc = q.sc;
  const double *r = q.v[VS_R];
  double* p = q.v[VS_P];
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

__global__ void __launch_bounds__(WG) k_cg_upd(Bat B, int m) {
  __shared__ double red[WG / 64];
  const Slot q = slot_at(B, blockIdx.y);
  double* sc = q.sc;
  const double *p = q.v[VS_P], *qv = q.v[VS_Q];
  double *cgx = q.v[VS_CGX], *r = q.v[VS_R];
  if (sc[SC_DONE] != 0.0) return;
  double pq = 0.0;
  for (int i = threadIdx.x; i < m; i += WG) pq += p[i] * qv[i];
  pq = blk_sum(pq, red);
  const double alpha = sc[SC_RHO] / pq;
  for (int i = threadIdx.x; i < m; i += WG) {
    cgx[i] += alpha * p[i];
    r[i] -= alpha * qv[i];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    sc[SC_RHO_PREV] = sc[SC_RHO];
    sc[SC_IT] += 1.0;
  }
}

// flag[0] = 1 when every slot of the pass has left the CG loop
__global__ void k_cg_alldone(Bat B, int cnt, int32_t* flag) {
  if (threadIdx.x != 0) return;
  int all = 1;
  for (int k = 0; k < cnt; ++k) all &= slot_at(B, k).sc[SC_DONE] != 0.0;
  flag[0] = all;
}

__global__ void __launch_bounds__(WG) k_cg_final(Bat B, int m, const double* D, int64_t dstride) {
  __shared__ double red[WG / 64];
  const int k = blockIdx.y;
  const Slot q = slot_at(B, k);
  const double *a = q.v[VS_A], *cgx = q.v[VS_CGX], *qv = q.v[VS_Q];
  double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0;
  for (int i = threadIdx.x; i < m; i += WG) {
    const double res = qv[i] + a[i];
    v0 += res * res;
    v1 += cgx[i] * cgx[i];
    v2 += cgx[i] * qv[i];
    v3 += a[i] * cgx[i];
  }
  cg_final_terms(red, q.sc, q.sc[SC_AN], D[(int64_t)B.ids[k] * dstride], v0, v1, v2, v3);
}

// After dsyevd (ev ascending) and g = Q^T a: the hard case / secular Newton / interior choice of
// riptrm_trs::trs_solve; writes the eigen coordinates pe of the boundary / hard-case candidate and
// the result scalars
// choose = 0 (the StableIdentification service's certified CG skip, which needs xobj before it
// decides on the CG): only the candidate and xobj; k_choose makes the interior choice after the CG.
__global__ void __launch_bounds__(WG) k_secular(Bat B, int m, double tolhc, int choose = 1) {
  __shared__ double red[WG / 64];
  const Slot q = slot_at(B, blockIdx.y);
  const double *ev = q.v[VS_EV], *g = q.v[VS_G];
  double* pe = q.v[VS_PE];
  double* sc = q.sc;
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
  if (!choose) {
    if (threadIdx.x == 0) {
      sc[SC_XOBJ] = xobj;
      sc[SC_BKIND] = (double)kind;
      sc[SC_BLAM1] = lam1;
      sc[SC_MINEIG] = lmin;
    }
    return;
  }
  const bool interior = sc[SC_CG_OK] != 0.0 && sc[SC_P1OBJ] <= xobj;   // RIPTRM.py:294-298
  if (threadIdx.x == 0) {
    sc[SC_INTERIOR] = interior ? 1.0 : 0.0;
    sc[SC_KIND] = interior ? 1.0 : (double)kind;   // riptrm_trs::Kind
    sc[SC_LAM1] = interior ? 0.0 : lam1;
    sc[SC_MINEIG] = lmin;
  }
}

// the interior choice of k_secular (RIPTRM.py:294-298) after a deferred (choose = 0) secular solve
__global__ void k_choose(Bat B, int cnt) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= cnt) return;
  double* sc = slot_at(B, k).sc;
  const bool interior = sc[SC_CG_OK] != 0.0 && sc[SC_P1OBJ] <= sc[SC_XOBJ];
  sc[SC_INTERIOR] = interior ? 1.0 : 0.0;
  sc[SC_KIND] = interior ? 1.0 : sc[SC_BKIND];
  sc[SC_LAM1] = interior ? 0.0 : sc[SC_BLAM1];
}

// Delta of slot k -> sc[SC_DELTA] (the CG's final terms write it otherwise; the deferred secular
// solve runs before the CG)
__global__ void k_set_delta(Bat B, int cnt, const double* D, int64_t dstride) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= cnt) return;
  slot_at(B, k).sc[SC_DELTA] = D[(int64_t)B.ids[k] * dstride];
}

// SciPy's CG (RIPTRM.py:240-251; the loop of k_cg_wave, restated from scipy.sparse.linalg.cg) on
// the subproblem's eigen-coordinates.  With A = Q diag(lam) Q^T (lam ascending at VS_EV, g = Q^T a at
// VS_G), the CG on diag(lam) y = -g generates y_k = Q^T x_k of the CG on A x = -a: Krylov subspaces,
// residual norms and step lengths are invariant under the orthogonal change of basis, so it is the
// same iterate up to rounding, at O(m) per iteration instead of an m x m mat-vec.  The stopping test
// uses ||a|| (atol = 1e-5 ||a||) and the final test the true residual diag(lam) y + g = Q^T (A x + a).
// One wave per slot, element i on lane i mod 64 (m <= 256).  The candidate stays in eigen-coordinates
// at VS_CGX (k_pick_eig).  skip_test: k_cg_wg's certified skip first.
__global__ void __launch_bounds__(64) k_cg_diag(Bat B, int m, const double* D, int64_t dstride, int skip_test) {
  const int k = blockIdx.y;
  const Slot q = slot_at(B, k);
  const double *ev = q.v[VS_EV], *g = q.v[VS_G], *a = q.v[VS_A];
  const int l = threadIdx.x;
  const double Dl = D[(int64_t)B.ids[k] * dstride];
  double lam[4], x[4], r[4], p[4];
  double an = 0.0, lsm = INFINITY, s1 = 0.0, s2 = 0.0;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = l + 64 * u;
    const double ai = i < m ? a[i] : 0.0, gi = i < m ? g[i] : 0.0;
    lam[u] = i < m ? ev[i] : 0.0;
    r[u] = -gi;
    x[u] = p[u] = 0.0;
    an += ai * ai;
    if (i < m) {
      lsm = fmin(lsm, fabs(lam[u]));
      s1 += (gi / lam[u]) * (gi / lam[u]);
      s2 += gi * gi / lam[u];
    }
  }
  an = sqrt(riptrm_wave::wave_sum(an));
  if (skip_test) {   // k_cg_wg's certified skip (the bounds there)
    const double lmax = fmax(fabs(ev[0]), fabs(ev[m - 1]));
    lsm = riptrm_wave::wave_min(lsm);
    s1 = riptrm_wave::wave_sum(s1);
    s2 = riptrm_wave::wave_sum(s2);
    const double e = 1e-5 * an;
    bool skip = *q.info == 0 && lsm > 1e-8 * lmax;
    if (skip) {
      const double xobj = q.sc[SC_XOBJ];
      const bool far = sqrt(s1) * (1.0 - 1e-6) - e / lsm >= Dl;
      const double p1lo = -0.5 * s2 - 0.5 * e * e / lsm;
      const bool worse = p1lo - xobj > 1e-6 * (fabs(s2) + fabs(xobj)) + 1e-10 * (e * 1e5) * Dl;
      skip = far || worse;
    }
    if (skip) {
      if (l == 0) {
        q.sc[SC_CG_OK] = 0.0;
        q.sc[SC_P1OBJ] = 0.0;
        q.sc[SC_IT] = 0.0;
        q.sc[SC_DONE] = 4.0;
        q.sc[SC_DELTA] = Dl;
      }
      return;
    }
  }
  const double atol = 1e-5 * an;
  double done = an == 0.0 ? 2.0 : 0.0, it = 0.0, rho_prev = 1.0;
  while (done == 0.0) {   // uniform
    if (it >= 10.0 * m) {
      done = 3.0;
      break;
    }
    const double rr = riptrm_wave::wave_sum((r[0] * r[0] + r[1] * r[1]) + (r[2] * r[2] + r[3] * r[3]));
    if (sqrt(rr) < atol) {
      done = 1.0;
      break;
    }
    const double rho = rr;
    const double beta = it > 0.0 ? rho / rho_prev : 0.0;
    double qv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      p[u] = it > 0.0 ? p[u] * beta + r[u] : r[u];
      qv[u] = lam[u] * p[u];
    }
    const double pq = riptrm_wave::wave_sum((p[0] * qv[0] + p[1] * qv[1]) + (p[2] * qv[2] + p[3] * qv[3]));
    const double alpha = rho / pq;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      x[u] += alpha * p[u];
      r[u] -= alpha * qv[u];
    }
    rho_prev = rho;
    it += 1.0;
  }
  double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = l + 64 * u;
    if (i < m) {
      const double ax = lam[u] * x[u], gi = g[i];
      const double res = ax + gi;
      v0 += res * res;
      v1 += x[u] * x[u];
      v2 += x[u] * ax;
      v3 += gi * x[u];
      q.v[VS_CGX][i] = x[u];
    }
  }
  v0 = riptrm_wave::wave_sum(v0);
  v1 = riptrm_wave::wave_sum(v1);
  v2 = riptrm_wave::wave_sum(v2);
  v3 = riptrm_wave::wave_sum(v3);
  if (l == 0) {
    q.sc[SC_AN] = an;
    q.sc[SC_ATOL] = atol;
    q.sc[SC_IT] = it;
    q.sc[SC_DONE] = done;
    q.sc[SC_CG_OK] = (an != 0.0 && sqrt(v0) / an < 1e-5 && v1 < Dl * Dl) ? 1.0 : 0.0;   // RIPTRM.py:246-251
    q.sc[SC_P1OBJ] = 0.5 * v2 + v3;
    q.sc[SC_DELTA] = Dl;
  }
}

// pe <- the CG's eigen-coordinates when the interior candidate won (then x = Q pe for either)
__global__ void __launch_bounds__(256) k_pick_eig(Bat B, int m) {
  const Slot q = slot_at(B, blockIdx.y);
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < m && q.sc[SC_INTERIOR] != 0.0) q.v[VS_PE][i] = q.v[VS_CGX][i];
}

// x <- cgx when the interior candidate won (x = Q pe was computed before)
__global__ void __launch_bounds__(256) k_pick(Bat B, int m) {
  const Slot q = slot_at(B, blockIdx.y);
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < m && q.sc[SC_INTERIOR] != 0.0) q.v[VS_X][i] = q.v[VS_CGX][i];
}

// eta = H [0; x] (RIPTRM.py:442-444 in the Householder frame), the direction type, j = -1, and the
// instance resumes at PH_TRS_END
__global__ void __launch_bounds__(WG) k_finish_dir(DevParams P, Bat B) {
  __shared__ double red[WG / 64];
  const int k = blockIdx.y, b = B.ids[k];
  const Slot q = slot_at(B, k);
  const double *w = q.v[VS_W], *x = q.v[VS_X];
  const int n = P.n;
  double wz = 0.0;
  for (int i = threadIdx.x + 1; i < n; i += WG) wz += w[i] * x[i - 1];
  wz = blk_sum(wz, red);
  const double tau = q.sc[SC_TAU];
  double* E = P.vec + ((int64_t)V_ETA * P.batch + b) * P.ld;
  for (int i = threadIdx.x; i < n; i += WG) E[i] = (i == 0 ? 0.0 : x[i - 1]) - tau * w[i] * wz;
  if (threadIdx.x == 0) {
    double* s = P.st + (int64_t)b * ST_N;
    // dsyevd did not converge (info > 0): scipy.linalg.eig would raise LinAlgError inside
    // outer_step (RIPTRM.py:961-966); the machine stops the instance at PH_TRS_END
    s[ST_TCG_STOP] = *q.info != 0 ? (double)RIPTRM_TCG_EIGFAIL : RIPTRM_TRS_BOUNDARY + q.sc[SC_KIND];
    s[ST_J] = -1.0;
    s[ST_PHASE] = PH_TRS_END;
  }
}

// the smallest eigenvalue of the trial point's matrix -> the instance, which resumes at PH_MINEIG_END.
// NaN (the machine stops the instance, RIPTRM_ERR_EIGEN) when the eigenvalues are not valid: a
// non-converged rocSOLVER dsyevd (info > 0), non-finite input (1) or a timed-out exchange (3).  The
// hand-written solvers' info 2 (Gram-Schmidt could not orthonormalise the vectors, riptrm_eig.h) leaves
// the bisection's eigenvalues valid: vals_ok2 = 1 there.
__device__ __forceinline__ bool eig_values_ok(int info, int vals_ok2) { return info == 0 || (info == 2 && vals_ok2); }
__global__ void k_finish_mineig(DevParams P, Bat B, int cnt, int vals_ok2) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= cnt) return;
  const Slot q = slot_at(B, k);
  double* s = P.st + (int64_t)B.ids[k] * ST_N;
  s[ST_MINEIG] = eig_values_ok(*q.info, vals_ok2) ? q.v[VS_EV][0] : NAN;
  s[ST_PHASE] = PH_MINEIG_END;
}

// riptrm_trs_gep outputs of slot blockIdx.y (subproblem ids[k])
__global__ void __launch_bounds__(256) k_gep_out(Bat B, int m, int64_t ldv, double* xo, double* lam1, int32_t* kind,
                                                 double* mineig) {
  const int k = blockIdx.y, b = B.ids[k];
  const Slot q = slot_at(B, k);
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < m) xo[(int64_t)b * ldv + i] = q.v[VS_X][i];
  if (i == 0) {
    lam1[b] = q.sc[SC_LAM1];
    kind[b] = RIPTRM_TRS_BOUNDARY + (int32_t)q.sc[SC_KIND];
    if (mineig) mineig[b] = q.v[VS_EV][0];
  }
}

// the smallest eigenvalue of slot k (eigenvalues ascending) -> mineig[ids[k]]; NaN when the
// eigensolve did not converge
__global__ void k_min_out(Bat B, int cnt, double* mineig, int vals_ok2) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= cnt) return;
  const Slot q = slot_at(B, k);
  mineig[B.ids[k]] = eig_values_ok(*q.info, vals_ok2) ? q.v[VS_EV][0] : NAN;
}

// copy subproblem ids[k]'s m x m block (row-major, lda) into slot k's matrix (lda m) and a
__global__ void __launch_bounds__(256) k_load(Bat B, int m, const double* A, int64_t lda, int64_t a_stride,
                                              const double* a, int64_t ldv) {
  const int k = blockIdx.y, b = B.ids[k];
  const Slot q = slot_at(B, k);
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < (int64_t)m * m) {
    const int i = (int)(e / m), j = (int)(e - (int64_t)i * m);
    q.M[e] = A[(int64_t)b * a_stride + (int64_t)i * lda + j];
  }
  if (e < m) q.v[VS_A][e] = a[(int64_t)b * ldv + e];
}

// v <- H^T v = H_{m-2} ... H_0 v (backward = 0) or H v = H_0 ... H_{m-2} v (backward = 1), H the
// tridiagonalisation's reflectors of the slot's matrix (compact eigenvectors: q_k = H z_k, riptrm_eig.h),
// from slot offset voff to ooff (may be the same).  One workgroup per slot: the reflectors and tau are
// staged into LDS by all threads, then one wave runs the m - 1 reflections with v in registers (lane l
// owns elements l, l + 64, l + 128, l + 192; each dot product in lane order, then the wave tree).
static_assert(riptrm_eig::EIG_LDS_MAX <= 256, "k_refl_apply holds four elements per lane");
__global__ void __launch_bounds__(256) k_refl_apply(Bat B, int m, int64_t voff, int64_t ooff, int backward) {
  extern __shared__ double smem[];
  riptrm_eig::lds_t* R = (riptrm_eig::lds_t*)smem;
  double* base = B.base + (int64_t)blockIdx.y * B.sd;
  const double* Rg = base + off_refl(B.N);
  const int nt = riptrm_eig::refl_tau(m), nr = nt + m - 1;
  // staged with sixteen loads in flight per thread (a load-then-store loop waits out one memory
  // latency per element: ~78 of them at m = 199)
  for (int q0 = 0; q0 < nr; q0 += 256 * 16) {
    double v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int q = q0 + u * 256 + (int)threadIdx.x;
      v[u] = Rg[q < nr ? q : nr - 1];
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int q = q0 + u * 256 + (int)threadIdx.x;
      if (q < nr) R[q] = v[u];
    }
  }
  __syncthreads();
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x;
  double v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int j = lane + 64 * q;
    v[q] = j < m ? base[voff + j] : 0.0;
  }
  for (int t = 0; t < m - 1; ++t) {
    const int i = backward ? m - 2 - t : t;
    const double tau = R[nt + i];
    if (tau == 0.0) continue;   // uniform
    const int c = riptrm_eig::refl_col(m, i) - i - 1;   // element j > i of reflector i at c + j
    double u[4], s = 0.0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = lane + 64 * q;
      u[q] = (j > i && j < m) ? R[c + j] : 0.0;
      s += u[q] * v[q];
    }
    const double f = tau * riptrm_wave::wave_sum(s);
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = v[q] - f * u[q];
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int j = lane + 64 * q;
    if (j < m) base[ooff + j] = v[q];
  }
}

// ---- the per-instance eigendecomposition cache (riptrm_trs_bind_cache) ------------------------------
__device__ __forceinline__ double* cache_of(double* cache, int64_t N, int b) { return cache + (int64_t)b * cache_doubles(N); }

// after the trial point's eigensolve: slot k's eigenvectors (the n x n buffer), eigenvalues and the
// trial point (x_new, y_new) -> instance ids[k]'s cache entry; valid iff the eigensolve converged
// tri: the tridiagonal path's T (d, e: the first two rows of the eigenvector area) instead of Q
__global__ void __launch_bounds__(256) k_cache_store(DevParams P, Bat B, double* cache, int64_t N, int tri) {
  const int k = blockIdx.y, b = B.ids[k];
  const Slot q = slot_at(B, k);
  double* C = cache_of(cache, N, b);
  const int n = P.n;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (tri) {
    if (e < n - 1) {
      C[e] = q.v[VS_R][e];
      C[N + e] = q.v[VS_P][e];
    }
  } else if (e < (int64_t)n * n) {
    C[e] = q.M[e];
  }
  if (e < n - 1) C[N * N + e] = q.v[VS_EV][e];
  if (e < n) {
    C[N * N + vpad(N) + e] = vec_of(P, V_IN1, b)[e];
    C[N * N + 2 * vpad(N) + e] = vec_of(P, V_YNEW, b)[e];
  }
  if (e == 0) C[N * N + 3 * vpad(N)] = *q.info == 0 ? 1.0 : 0.0;
  // the reflectors of the compact eigenvectors (riptrm_eig.h) or of T, when the hand-written paths made them
  if ((n - 1 <= riptrm_eig::EIG_LDS_MAX || tri) && e < (int64_t)riptrm_eig::refl_doubles(n - 1))
    C[N * N + 3 * vpad(N) + 8 + e] = B.base[(int64_t)k * B.sd + off_refl(B.N) + e];
}

// hits[k] = 1 iff instance ids[k]'s cache entry is valid and was taken at exactly this (x, y): then
// its matrix is the same bits as the one this subproblem would build (k_repmat_vec)
__global__ void __launch_bounds__(256) k_cache_check(DevParams P, Bat B, const double* cache, int64_t N, int32_t* hits) {
  const int k = blockIdx.y, b = B.ids[k];
  const double* C = cache + (int64_t)b * cache_doubles(N);
  const int n = P.n;
  const double *X = vec_of(P, V_X, b), *Y = vec_of(P, V_Y, b);
  int ok = C[N * N + 3 * vpad(N)] == 1.0;
  for (int i = threadIdx.x; i < n; i += 256)
    ok &= (X[i] == C[N * N + vpad(N) + i]) & (Y[i] == C[N * N + 2 * vpad(N) + i]);
  ok = __syncthreads_and(ok);
  if (threadIdx.x == 0) hits[k] = ok;
}

// a cache hit: the cached eigenvectors / eigenvalues -> slot k (after its CG used the matrix)
__global__ void __launch_bounds__(256) k_cache_load(DevParams P, Bat B, const double* cache, int64_t N, int tri) {
  const int k = blockIdx.y, b = B.ids[k];
  const Slot q = slot_at(B, k);
  const double* C = cache + (int64_t)b * cache_doubles(N);
  const int n = P.n;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (tri) {
    if (e < n - 1) {
      q.v[VS_R][e] = C[e];
      q.v[VS_P][e] = C[N + e];
    }
  } else if (e < (int64_t)n * n) {
    q.M[e] = C[e];
  }
  if (e < n - 1) q.v[VS_EV][e] = C[N * N + e];
  if ((n - 1 <= riptrm_eig::EIG_LDS_MAX || tri) && e < (int64_t)riptrm_eig::refl_doubles(n - 1))
    B.base[(int64_t)k * B.sd + off_refl(B.N) + e] = C[N * N + 3 * vpad(N) + 8 + e];
  if (e == 0) *q.info = 0;
}

// ---- the keyed per-instance cache of the StableIdentification service (KeyedEigCache) ------------
// entry of order m, key length kl: [valid, 7 pad][key: kl to 8][ev: vpad(m)][Z: m x m][reflectors + tau]
__host__ __device__ inline int64_t kc_kpad(int kl) { return (kl + 7) / 8 * 8; }
__host__ __device__ inline int64_t kc_doubles(int m, int kl) {
  return 8 + kc_kpad(kl) + vpad(m) + (int64_t)m * m + (int64_t)riptrm_eig::refl_doubles(m);
}

// hits[k] = 1 iff instance ids[k]'s entry is valid and its key equals the instance's key bit for bit
__global__ void __launch_bounds__(256) k_kc_check(Bat B, const double* keys, int64_t kstride, int kl, const double* cache,
                                                  int64_t cstride, int32_t* hits) {
  const int k = blockIdx.y, b = B.ids[k];
  const double* C = cache + (int64_t)b * cstride;
  const double* K = keys + (int64_t)b * kstride;
  int ok = C[0] == 1.0;
  for (int i = threadIdx.x; i < kl; i += 256) ok &= K[i] == C[8 + i];
  ok = __syncthreads_and(ok);
  if (threadIdx.x == 0) hits[k] = ok;
}

// after an eigensolve with compact vectors: slot k's eigenvalues, Z (the slot's matrix, lda m), the
// reflectors and instance ids[k]'s key -> its entry; valid iff the eigensolve succeeded
__global__ void __launch_bounds__(256) k_kc_store(Bat B, int m, const double* keys, int64_t kstride, int kl, double* cache,
                                                  int64_t cstride) {
  const int k = blockIdx.y, b = B.ids[k];
  const Slot q = slot_at(B, k);
  double* C = cache + (int64_t)b * cstride;
  const int64_t kp = kc_kpad(kl), e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const double* R = B.base + (int64_t)k * B.sd + off_refl(B.N);
  if (e < kl) C[8 + e] = keys[(int64_t)b * kstride + e];
  if (e < m) C[8 + kp + e] = q.v[VS_EV][e];
  if (e < (int64_t)m * m) C[8 + kp + vpad(m) + e] = q.M[e];
  if (e < (int64_t)riptrm_eig::refl_doubles(m)) C[8 + kp + vpad(m) + (int64_t)m * m + e] = R[e];
  if (e == 0) C[0] = *q.info == 0 ? 1.0 : 0.0;
}

// a hit: instance ids[k]'s cached eigenvalues, Z and reflectors -> slot k
__global__ void __launch_bounds__(256) k_kc_load(Bat B, int m, int kl, const double* cache, int64_t cstride) {
  const int k = blockIdx.y, b = B.ids[k];
  const Slot q = slot_at(B, k);
  const double* C = cache + (int64_t)b * cstride;
  const int64_t kp = kc_kpad(kl), e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  double* R = B.base + (int64_t)k * B.sd + off_refl(B.N);
  if (e < m) q.v[VS_EV][e] = C[8 + kp + e];
  if (e < (int64_t)m * m) q.M[e] = C[8 + kp + vpad(m) + e];
  if (e < (int64_t)riptrm_eig::refl_doubles(m)) R[e] = C[8 + kp + vpad(m) + (int64_t)m * m + e];
  if (e == 0) *q.info = 0;
}

__global__ void k_cache_invalidate(double* cache, int64_t N, int batch) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < batch) cache[(int64_t)b * cache_doubles(N) + N * N + 3 * vpad(N)] = 0.0;
}

// ---- rocSOLVER, loaded on first use (no link-time dependency of the library) -----------------------
// (RIPTRM_ROCBLAS_LIB / RIPTRM_ROCSOLVER_LIB in the environment name other libraries: a host whose
// ROCm is elsewhere, or a test that checks the failure path)
typedef int (*fn_create_t)(void**);
typedef int (*fn_set_stream_t)(void*, hipStream_t);
typedef int (*fn_destroy_t)(void*);
typedef int (*fn_syevd_sb_t)(void*, int, int, int, double*, int, int64_t, double*, int64_t, double*, int64_t, int*, int);
typedef int (*fn_syevj_sb_t)(void*, int, int, int, int, double*, int, int64_t, double, double*, int, int*, double*, int64_t,
                             int*, int);
typedef int (*fn_syevdj_sb_t)(void*, int, int, int, double*, int, int64_t, double*, int64_t, int*, int);
typedef int (*fn_syevd_t)(void*, int, int, int, double*, int, double*, double*, int*);
constexpr int EVECT_ORIGINAL = 211, EVECT_NONE = 213, FILL_UPPER = 121, ESORT_ASCENDING = 252;

struct Solver {
  bool tried = false, ok = false;
  std::string why;
  fn_create_t create = nullptr;
  fn_set_stream_t set_stream = nullptr;
  fn_destroy_t destroy = nullptr;
  fn_syevd_sb_t syevd_sb = nullptr;
  fn_syevj_sb_t syevj_sb = nullptr;     // A/B only (RIPTRM_BIG_EIG)
  fn_syevdj_sb_t syevdj_sb = nullptr;
  fn_syevd_t syevd = nullptr;           // one matrix per call (large orders)
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
  s.syevd_sb = (fn_syevd_sb_t)dlsym(sol, "rocsolver_dsyevd_strided_batched");
  s.syevj_sb = (fn_syevj_sb_t)dlsym(sol, "rocsolver_dsyevj_strided_batched");
  s.syevdj_sb = (fn_syevdj_sb_t)dlsym(sol, "rocsolver_dsyevdj_strided_batched");
  s.syevd = (fn_syevd_t)dlsym(sol, "rocsolver_dsyevd");
  s.ok = s.create && s.set_stream && s.destroy && s.syevd_sb;
  if (!s.ok)
    s.why = "rocBLAS / rocSOLVER lack rocblas_create_handle / rocblas_set_stream / rocsolver_dsyevd_strided_batched";
  return s;
}

}  // namespace riptrm_big

using namespace riptrm_big;

static unsigned blocks_of(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }
static bool getenv_is(const char* name, char v) {
  const char* e = getenv(name);
  return e && e[0] == v;
}

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
  if (c && c->tri_grid) {
    (void)hipFree(c->tri_grid);
    c->tri_grid = nullptr;
    c->tri_grid_bytes = 0;
  }
  if (c && c->eig_scratch) {
    (void)hipFree(c->eig_scratch);
    c->eig_scratch = nullptr;
    c->eig_scratch_bytes = 0;
  }
  if (c && c->big_handle) {
    Solver& s = solver();
    if (s.ok) (void)s.destroy(c->big_handle);
    c->big_handle = nullptr;
  }
}

// the workspace's pass descriptor and its id / flag arrays (after the slots)
static Bat bat_of(riptrm_ctx* c) {
  const int64_t N = c->big_order, sd = slot_doubles(N);
  double* base = (double*)c->big_ws;
  int32_t* tail = (int32_t*)(base + sd * c->big_slots);
  return Bat{base, N, sd, tail + c->big_slots, tail};
}
static int32_t* tail_of(riptrm_ctx* c) { return (int32_t*)((double*)c->big_ws + slot_doubles(c->big_order) * c->big_slots); }
static int32_t* flag_of(riptrm_ctx* c) { return tail_of(c) + 2 * c->big_slots; }

// A = Q diag(lam) Q^T for the pass's cnt slots (A at slot offset aoff, lda; eigenvalues ascending into
// VS_EV, eigenvectors over A when vectors): rocSOLVER dsyevd (default) or, for A/B measurements
// (RIPTRM_BIG_EIG=j / dj), its Jacobi dsyevj / dsyevdj
// the hand-written eigensolver serves order m (riptrm_eig.h; RIPTRM_BIG_EIG=r, or j / dj / s, keeps
// rocSOLVER for A/B measurements): its eigenvectors are compact (those of the tridiagonal form over
// the matrix, the reflectors in the slot), applied through k_refl_apply
static bool eig_compact(int m) {
  const char* e = getenv("RIPTRM_BIG_EIG");
  return m <= riptrm_eig::EIG_LDS_MAX && !(e && e[0] != 'h');
}

static int refl_apply(riptrm_ctx* c, const Bat& B, int cnt, int m, int64_t voff, int64_t ooff, int backward) {
  const size_t shm = (size_t)(riptrm_eig::refl_tau(m) + m) * sizeof(double);
  HIPCHK(c, hipFuncSetAttribute((const void*)k_refl_apply, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
  hipLaunchKernelGGL(k_refl_apply, dim3(1, cnt), dim3(256), shm, c->stream, B, m, voff, ooff, backward);
  HIPCHK(c, hipGetLastError());
  return RIPTRM_OK;
}

// the distributed tridiagonalisation (riptrm_tri.h) for the hand-written eigensolver's first phase:
// RIPTRM_EIG_TRI=1 (A/B; orders >= 64)
static int tri_launch(riptrm_ctx* c, const riptrm_tri::TriArgs& a, int cnt, int m);
static bool eig_tri_front(int m) {
  const char* e = getenv("RIPTRM_EIG_TRI");
  return m >= 64 && e && e[0] == '1';
}

// k_eig_lds with 1024 threads per matrix (16 waves: the symv and rank-2 update of the
// tridiagonalisation hide more LDS latency), or 512 (RIPTRM_EIG_THREADS=512, A/B)
static int launch_eig(riptrm_ctx* c, int cnt, int m, double* A, int64_t a_stride, int lda, double* ev, int64_t ev_stride,
                      double* d, double* e, int64_t sc_stride, double* R, int64_t r_stride, int32_t* infos, int vectors,
                      long long* stamps) {
  const size_t shm = riptrm_eig::eig_lds_bytes(m);
  const char* t = getenv("RIPTRM_EIG_THREADS");
  const char* sp = getenv("RIPTRM_EIG_SPLIT");
  if (!stamps && !(sp && sp[0] == '0') && !(t && atoi(t) == 512)) {
    // four launches: the tridiagonalisation (one workgroup per matrix), the eigenvalues and the
    // vectors of T over ~50 indices per workgroup (four per matrix at m = 199: the whole chip for a
    // batch of 64), the orthogonality pass (one per matrix).  The same arithmetic as one launch.
    const int yv = (m + 49) / 50;
    if (eig_tri_front(m)) {   // T across the chip, then phase 1's split / non-finite test
      riptrm_tri::TriArgs ta{};
      ta.A0 = A;
      ta.a_stride = a_stride;
      ta.lda = lda;
      ta.d0 = d;
      ta.e0 = e;
      ta.de_stride = sc_stride;
      ta.R0 = R;
      ta.r_stride = r_stride;
      ta.infos = infos;
      if (int rc = tri_launch(c, ta, cnt, m)) return rc;
      hipLaunchKernelGGL(riptrm_tri::k_tri_split, dim3(cnt), dim3(256), 0, c->stream, d, e, sc_stride, m, infos, ev, ev_stride);
    } else {
      HIPCHK(c, hipFuncSetAttribute((const void*)riptrm_eig::k_eig_lds<1024, 1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)shm));
      hipLaunchKernelGGL((riptrm_eig::k_eig_lds<1024, 1>), dim3(cnt), dim3(1024), shm, c->stream, A, a_stride, lda, m, ev,
                         ev_stride, d, e, sc_stride, R, r_stride, infos, vectors, nullptr);
    }
    HIPCHK(c, hipFuncSetAttribute((const void*)riptrm_eig::k_eig_lds<512, 2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)shm));
    // the bisection over ~25 eigenvalues per workgroup up to order 128 (four waves of eight-lane
    // groups instead of seven; kq stays 8 for any range <= 64, so the same arithmetic).
    // RIPTRM_EIG_BIS=n (1..64): ~n per workgroup at every order (A/B)
    const char* bs = getenv("RIPTRM_EIG_BIS");
    const int bn = bs ? atoi(bs) : 0;
    const int yb = (bn >= 1 && bn <= 64) ? (m + bn - 1) / bn : (m <= 128 ? (m + 24) / 25 : yv);
    hipLaunchKernelGGL((riptrm_eig::k_eig_lds<512, 2>), dim3(cnt, yb), dim3(512), shm,
                       c->stream, A, a_stride, lda, m, ev, ev_stride, d, e, sc_stride, R, r_stride, infos, vectors, nullptr);
    if (vectors) {
      HIPCHK(c, hipFuncSetAttribute((const void*)riptrm_eig::k_eig_lds<512, 4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)shm));
      hipLaunchKernelGGL((riptrm_eig::k_eig_lds<512, 4>), dim3(cnt, yv), dim3(512), shm, c->stream, A, a_stride, lda, m, ev,
                         ev_stride, d, e, sc_stride, R, r_stride, infos, vectors, nullptr);
      HIPCHK(c, hipFuncSetAttribute((const void*)riptrm_eig::k_eig_lds<1024, 8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)shm));
      hipLaunchKernelGGL((riptrm_eig::k_eig_lds<1024, 8>), dim3(cnt), dim3(1024), shm, c->stream, A, a_stride, lda, m, ev,
                         ev_stride, d, e, sc_stride, R, r_stride, infos, vectors, nullptr);
    }
  } else if (!(t && atoi(t) == 512)) {
    HIPCHK(c, hipFuncSetAttribute((const void*)riptrm_eig::k_eig_lds<1024>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)shm));
    hipLaunchKernelGGL(riptrm_eig::k_eig_lds<1024>, dim3(cnt), dim3(1024), shm, c->stream, A, a_stride, lda, m, ev, ev_stride,
                       d, e, sc_stride, R, r_stride, infos, vectors, stamps);
  } else {
    HIPCHK(c, hipFuncSetAttribute((const void*)riptrm_eig::k_eig_lds<512>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)shm));
    hipLaunchKernelGGL(riptrm_eig::k_eig_lds<512>, dim3(cnt), dim3(512), shm, c->stream, A, a_stride, lda, m, ev, ev_stride,
                       d, e, sc_stride, R, r_stride, infos, vectors, stamps);
  }
  HIPCHK(c, hipGetLastError());
  return RIPTRM_OK;
}

static int eig_batched(riptrm_ctx* c, const Bat& B, int cnt, bool vectors, int m, int64_t aoff, int lda) {
  const char* e = getenv("RIPTRM_BIG_EIG");
  if (eig_compact(m)) {
    // hand-written: one workgroup per matrix, the matrix in LDS
    return launch_eig(c, cnt, m, B.base + aoff, B.sd, lda, B.base + off_vec(B.N, VS_EV), B.sd, B.base + off_vec(B.N, VS_R),
                      B.base + off_vec(B.N, VS_EW), B.sd, B.base + off_refl(B.N), B.sd, B.infos, vectors ? 2 : 0, nullptr);
  }
  if (int rc = big_handle(c)) return rc;
  Solver& s = solver();
  const int ev = vectors ? EVECT_ORIGINAL : EVECT_NONE;
  double* A = B.base + aoff;
  double* W = B.base + off_vec(B.N, VS_EV);
  int st;
  if (e && e[0] == 'j' && s.syevj_sb) {
    int32_t* sweeps = tail_of(c) + 2 * c->big_slots + 8;
    double* resid = (double*)(tail_of(c) + tail_ints(c->big_slots));
    st = s.syevj_sb(c->big_handle, ESORT_ASCENDING, ev, FILL_UPPER, m, A, lda, B.sd, 0.0, resid, 100, sweeps, W, B.sd,
                    B.infos, cnt);
  } else if (e && e[0] == 'd' && e[1] == 'j' && s.syevdj_sb) {
    st = s.syevdj_sb(c->big_handle, ev, FILL_UPPER, m, A, lda, B.sd, W, B.sd, B.infos, cnt);
  } else if (e && e[0] == 's' && s.syevd) {   // one rocsolver_dsyevd call per matrix
    st = 0;
    for (int k = 0; k < cnt && st == 0; ++k)
      st = s.syevd(c->big_handle, ev, FILL_UPPER, m, A + k * B.sd, lda, W + k * B.sd, B.base + off_vec(B.N, VS_EW) + k * B.sd,
                   B.infos + k);
  } else {
    st = s.syevd_sb(c->big_handle, ev, FILL_UPPER, m, A, lda, B.sd, W, B.sd, B.base + off_vec(B.N, VS_EW), B.sd, B.infos,
                    cnt);
  }
  if (st != 0) return fail(c, RIPTRM_E_HIP, "rocsolver batched symmetric eigensolver failed (status " + std::to_string(st) + ")");
  return RIPTRM_OK;
}

// this pass's ids -> the workspace (stream-ordered after the previous pass; synchronises)
static int put_ids(riptrm_ctx* c, const Bat& B, const int32_t* ids, int cnt) {
  HIPCHK(c, hipMemcpyAsync(const_cast<int32_t*>(B.ids), ids, (size_t)cnt * sizeof(int32_t), hipMemcpyHostToDevice,
                           c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return RIPTRM_OK;
}

// the one-workgroup CG when its per-iteration time (A streamed by one CU, ~60 GB/s, or a ~3 us
// latency floor) beats the grid-wide form's (3 launches ~12 us + the pass's matrices at ~5 TB/s)
static bool cg_one_workgroup(int m, int cnt) {
  if (m > CG_WG_MAX) return false;
  const char* e = getenv("RIPTRM_BIG_CG");   // "wg" / "grid": force one form (A/B measurements)
  if (e && e[0] == 'w') return true;
  if (e && e[0] == 'g') return false;
  const double bytes = (double)m * m * 8.0;
  const double t_wg = fmax(3e-6, bytes / 60e9);
  const double t_grid = 12e-6 + cnt * bytes / 5e12;
  return t_wg <= t_grid;
}

// The subproblems min x^T A x / 2 + a^T x s.t. ||x|| <= Delta of the pass's cnt slots: A at slot
// offset aoff with leading dimension lda (m x m), a = v[VS_A], Delta of slot k at D[ids[k] dstride].
// CG (interior candidate), batched dsyevd, secular solve; the solution lands in v[VS_X], the
// scalars in sc.  A is destroyed (eigenvectors).
static int big_cg(riptrm_ctx* c, const Bat& B, int cnt, int64_t aoff, int lda, int m, const double* D, int64_t dstride) {
  hipStream_t st = c->stream;
  const int64_t N = B.N;
  const dim3 one(1, cnt), rows(blocks_of(m, GV / 64), cnt);
  if (m <= CGW_MAX && cg_one_workgroup(m, cnt) && !getenv_is("RIPTRM_CG_WAVE", '0')) {
    const size_t shm = cg_wave_lds(m);
    HIPCHK(c, hipFuncSetAttribute((const void*)k_cg_wave, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
    hipLaunchKernelGGL(k_cg_wave, one, dim3(64), shm, st, B, m, aoff, (int64_t)lda, D, dstride, nullptr, (int64_t)0, 0);
    HIPCHK(c, hipGetLastError());
  } else if (cg_one_workgroup(m, cnt)) {
    const int rl = cg_lds_rows(m);
    const size_t shm = (size_t)rl * m * sizeof(double);
    if (shm > 0)
      HIPCHK(c, hipFuncSetAttribute((const void*)k_cg_wg, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
    hipLaunchKernelGGL(k_cg_wg, one, dim3(WG), shm, st, B, m, aoff, (int64_t)lda, D, dstride, rl);
    HIPCHK(c, hipGetLastError());
  } else {
    hipLaunchKernelGGL(k_cg_init, one, dim3(WG), 0, st, B, m);
    HIPCHK(c, hipGetLastError());
    int32_t* flag = flag_of(c);
    int32_t all = 0;
    for (int it = 0; it < 10 * m + 1; it += CG_POLL) {
      for (int k = 0; k < CG_POLL; ++k) {
        hipLaunchKernelGGL(k_cg_dir, one, dim3(WG), 0, st, B, m);
        hipLaunchKernelGGL(k_gemv, rows, dim3(GV), 0, st, B, aoff, (int64_t)lda, m, m, off_vec(N, VS_P), off_vec(N, VS_Q),
                           off_sc(N) + SC_DONE);
        hipLaunchKernelGGL(k_cg_upd, one, dim3(WG), 0, st, B, m);
      }
      hipLaunchKernelGGL(k_cg_alldone, dim3(1), dim3(64), 0, st, B, cnt, flag);
      HIPCHK(c, hipGetLastError());
      HIPCHK(c, hipMemcpyAsync(&all, flag, sizeof(int32_t), hipMemcpyDeviceToHost, st));
      HIPCHK(c, hipStreamSynchronize(st));
      if (all) break;
    }
    hipLaunchKernelGGL(k_gemv, rows, dim3(GV), 0, st, B, aoff, (int64_t)lda, m, m, off_vec(N, VS_CGX), off_vec(N, VS_Q),
                       (int64_t)-1);
    hipLaunchKernelGGL(k_cg_final, one, dim3(WG), 0, st, B, m, D, dstride);
    HIPCHK(c, hipGetLastError());
  }
  return RIPTRM_OK;
}

// after the eigendecomposition (eigenvectors over the matrix): g = Q^T a, the secular solve, x
static int big_after_eig(riptrm_ctx* c, const Bat& B, int cnt, int64_t aoff, int lda, int m, double tolhc) {
  hipStream_t st = c->stream;
  const int64_t N = B.N;
  const dim3 one(1, cnt), rows(blocks_of(m, GV / 64), cnt);
  // eigenvector k = row k of the row-major view (column k of dsyevd's column-major output); compact:
  // Q^T a = Z^T (H^T a), Q y = H (Z y)
  const bool cpt = eig_compact(m);
  if (cpt)
    if (int rc = refl_apply(c, B, cnt, m, off_vec(N, VS_A), off_vec(N, VS_PE), 0)) return rc;
  hipLaunchKernelGGL(k_gemv, rows, dim3(GV), 0, st, B, aoff, (int64_t)lda, m, m, off_vec(N, cpt ? VS_PE : VS_A),
                     off_vec(N, VS_G), (int64_t)-1);
  hipLaunchKernelGGL(k_secular, one, dim3(WG), 0, st, B, m, tolhc);
  hipLaunchKernelGGL(k_gemv_t, dim3(blocks_of(m, 256), cnt), dim3(256), 0, st, B, aoff, (int64_t)lda, m, m,
                     off_vec(N, VS_PE), off_vec(N, VS_X));
  if (cpt)
    if (int rc = refl_apply(c, B, cnt, m, off_vec(N, VS_X), off_vec(N, VS_X), 1)) return rc;
  hipLaunchKernelGGL(k_pick, dim3(blocks_of(m, 256), cnt), dim3(256), 0, st, B, m);
  HIPCHK(c, hipGetLastError());
  return RIPTRM_OK;
}

// The subproblems of the pass after the hand-written eigensolve (compact eigenvectors over the
// matrix at aoff, lda; eig_compact(m)): g = Q^T a, the boundary candidate (k_secular, choose = 0), the
// CG in eigen-coordinates (k_cg_diag; skip: its certified skip), the interior / boundary choice, and
// x = Q pe.  The matrix itself is not read again.
static int compact_trs(riptrm_ctx* c, const Bat& B, int cnt, int m, int64_t aoff, int lda, const double* D,
                       int64_t dstride, double tolhc, bool skip) {
  hipStream_t st = c->stream;
  const int64_t N = B.N;
  const dim3 one(1, cnt), rows(blocks_of(m, GV / 64), cnt), els(blocks_of(m, 256), cnt);
  if (int rc = refl_apply(c, B, cnt, m, off_vec(N, VS_A), off_vec(N, VS_PE), 0)) return rc;
  hipLaunchKernelGGL(k_gemv, rows, dim3(GV), 0, st, B, aoff, (int64_t)lda, m, m, off_vec(N, VS_PE), off_vec(N, VS_G),
                     (int64_t)-1);
  hipLaunchKernelGGL(k_set_delta, dim3(blocks_of(cnt, 64)), dim3(64), 0, st, B, cnt, D, dstride);
  hipLaunchKernelGGL(k_secular, one, dim3(WG), 0, st, B, m, tolhc, 0);
  hipLaunchKernelGGL(k_cg_diag, one, dim3(64), 0, st, B, m, D, dstride, skip ? 1 : 0);
  hipLaunchKernelGGL(k_choose, dim3(blocks_of(cnt, 64)), dim3(64), 0, st, B, cnt);
  hipLaunchKernelGGL(k_pick_eig, els, dim3(256), 0, st, B, m);
  hipLaunchKernelGGL(k_gemv_t, els, dim3(256), 0, st, B, aoff, (int64_t)lda, m, m, off_vec(N, VS_PE), off_vec(N, VS_X));
  HIPCHK(c, hipGetLastError());
  return refl_apply(c, B, cnt, m, off_vec(N, VS_X), off_vec(N, VS_X), 1);
}

// ---- the tridiagonal path (riptrm_tri.h): orders above the one-workgroup eigensolver ------------------
// RIPTRM_BIG_EIG unset (or 'h'): orders TRI_MIN .. TRI_MAX take it; otherwise rocSOLVER (A/B)
// the tridiagonal path from order TRI_MIN = RIPTRM_TRS_TRI_MIN (RIPTRM_TRI_MIN=k: from k instead, 64 <= k
// <= 200, A/B; 200 keeps the compact eigensolver at every order it serves)
static bool tri_mode(int m) {
  const char* e = getenv("RIPTRM_BIG_EIG");
  const char* t = getenv("RIPTRM_TRI_MIN");
  const int lo = t ? std::min(std::max(atoi(t), 64), riptrm_eig::EIG_LDS_MAX + 1) : riptrm_tri::TRI_MIN;
  return m >= lo && m <= riptrm_tri::TRI_MAX && !(e && e[0] != 'h');
}

template <int EL>
static int tri_launch_el(riptrm_ctx* c, riptrm_tri::TriArgs a, int cnt, int m) {
  constexpr int RW = 32 / EL;
  int G = riptrm_tri::tri_groups(m);
  auto kern = riptrm_tri::k_tridiag_dist<EL, RW>;
  if (EL == 16 && getenv_is("RIPTRM_TRI_RW", '4')) {   // twice the rows per wave, half the workgroups (A/B;
    kern = riptrm_tri::k_tridiag_dist<16, 4>;          // the granule layout's per-parity room covers it)
    G = (m + 31) / 32;
  }
  int nb = 0;
  HIPCHK(c, hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, riptrm_tri::TT, 0));
  const int64_t cap = (int64_t)nb * c->ncu;
  if (nb < 1 || cap < G) return fail(c, RIPTRM_E_HIP, "tridiagonalisation: " + std::to_string(G) + " workgroups per matrix do not fit");
  const int per = (int)std::min<int64_t>(cnt, cap / G);   // matrices per cooperative launch
  const char* spe = getenv("RIPTRM_TRI_SPREAD");   // granule lines every 128 << sp bytes (A/B)
  a.spread = spe ? std::min(std::max(atoi(spe), 0), 8) : 0;
  const size_t gbytes = (size_t)riptrm_tri::tri_grid_bytes(riptrm_tri::tri_granules(m) * per, a.spread);
  if (gbytes >= (size_t)INT32_MAX) return fail(c, RIPTRM_E_HIP, "tridiagonalisation: granule grid above 2 GiB");
  if (c->tri_grid_bytes < gbytes) {
    if (c->tri_grid) HIPCHK(c, hipFree(c->tri_grid));
    c->tri_grid = nullptr;
    c->tri_grid_bytes = 0;
    HIPCHK(c, hipMalloc(&c->tri_grid, gbytes));
    c->tri_grid_bytes = gbytes;
  }
  HIPCHK(c, hipMemsetAsync(a.infos, 0, (size_t)cnt * sizeof(int32_t), c->stream));
  long long* stamps = nullptr;   // RIPTRM_TRI_STAMPS=1: phase cycles of matrix 0's workgroup 0 on stderr
  if (getenv_is("RIPTRM_TRI_STAMPS", '1')) {
    HIPCHK(c, hipMalloc(&stamps, 8 * sizeof(long long)));
    HIPCHK(c, hipMemsetAsync(stamps, 0, 8 * sizeof(long long), c->stream));
  }
  a.stamps = stamps;
  long long* hops = nullptr;   // RIPTRM_TRI_STAMPS=2: every workgroup's gather start / end every 16 steps
  const int ns = (m + 15) / 16;
  if (getenv_is("RIPTRM_TRI_STAMPS", '2')) {
    HIPCHK(c, hipMalloc(&hops, (size_t)G * ns * 2 * sizeof(long long)));
    HIPCHK(c, hipMemsetAsync(hops, 0, (size_t)G * ns * 2 * sizeof(long long), c->stream));
  }
  a.hops = hops;
  {
    const char* sl = getenv("RIPTRM_TRI_SLEEP");   // polling pace (A/B)
    a.sleep = sl ? std::max(1, atoi(sl)) : 1;
  }
  for (int k0 = 0; k0 < cnt; k0 += per) {
    const int nk = std::min(per, cnt - k0);
    HIPCHK(c, hipMemsetAsync(c->tri_grid, 0, (size_t)riptrm_tri::tri_grid_bytes(riptrm_tri::tri_granules(m) * nk, a.spread),
                             c->stream));
    a.k0 = k0;
    a.grid = c->tri_grid;
    a.grid_bytes = (int64_t)c->tri_grid_bytes;
    a.m = m;
    a.G = G;
    void* args[] = {&a};
    HIPCHK(c, hipLaunchCooperativeKernel((const void*)kern, dim3(G, nk), dim3(riptrm_tri::TT), args, 0, c->stream));
    a.stamps = nullptr;
    a.hops = nullptr;
  }
  if (hops) {
    // per sampled step: the publishers' skew (last - first gather start: a workgroup starts its
    // gather right after publishing) and each workgroup's wait past the last publisher
    std::vector<long long> h((size_t)G * ns * 2);
    HIPCHK(c, hipMemcpyAsync(h.data(), hops, h.size() * sizeof(long long), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    (void)hipFree(hops);
    double skew = 0.0, lat = 0.0, own = 0.0, latmax = 0.0;
    int cntv = 0;
    for (int t = 1; t < ns - 1; ++t) {
      long long lo = LLONG_MAX, hi = LLONG_MIN;
      for (int g = 0; g < G; ++g) {
        lo = std::min(lo, h[((size_t)g * ns + t) * 2]);
        hi = std::max(hi, h[((size_t)g * ns + t) * 2]);
      }
      double lt = 0.0, lm = 0.0, ow = 0.0;
      for (int g = 0; g < G; ++g) {
        const long long e = h[((size_t)g * ns + t) * 2 + 1];
        lt += (double)(e - hi);
        lm = std::max(lm, (double)(e - hi));
        ow += (double)(e - h[((size_t)g * ns + t) * 2]);
      }
      skew += (double)(hi - lo);
      lat += lt / G;
      latmax += lm;
      own += ow / G;
      ++cntv;
    }
    if (cntv)
      fprintf(stderr, "[tri hops] m=%d G=%d over %d sampled steps (us): publisher skew %.2f, wait past the last publisher "
              "mean %.2f max %.2f, gather (own start to end) %.2f\n", m, G, cntv, skew / cntv / 100.0, lat / cntv / 100.0,
              latmax / cntv / 100.0, own / cntv / 100.0);
  }
  if (stamps) {
    long long h[8];
    HIPCHK(c, hipMemcpyAsync(h, stamps, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    (void)hipFree(stamps);
    fprintf(stderr, "[tri stamps] m=%d G=%d cnt=%d gather %lld column %lld update %lld cycles (per step %.0f / %.0f / %.0f; "
            "column step: p.v %.0f, w and c %.0f, reflector %.0f)\n", m, G, cnt, h[0], h[1], h[2], h[0] / (double)(m - 1),
            h[1] / (double)(m - 1), h[2] / (double)(m - 1), h[4] / (double)(m - 2), h[5] / (double)(m - 2), h[6] / (double)(m - 2));
  }
  return RIPTRM_OK;
}

// k_tridiag_dist over cnt matrices (a's pointers and strides; infos zeroed first, 3: an exchange
// timed out)
static int tri_launch(riptrm_ctx* c, const riptrm_tri::TriArgs& a, int cnt, int m) {
  switch (riptrm_tri::tri_el(m)) {
    case 4: return tri_launch_el<4>(c, a, cnt, m);
    case 8: return tri_launch_el<8>(c, a, cnt, m);
    default: return tri_launch_el<16>(c, a, cnt, m);
  }
}

// T = H^T A H of the pass's cnt slots (A at slot offset aoff, leading dimension lda): d -> VS_R, e ->
// VS_P, the reflectors at off_refl; infos zeroed first (3: an exchange timed out)
static int tri_tridiag(riptrm_ctx* c, const Bat& B, int cnt, int m, int64_t aoff, int64_t lda) {
  riptrm_tri::TriArgs a{};
  a.A0 = B.base + aoff;
  a.a_stride = B.sd;
  a.lda = lda;
  a.d0 = B.base + off_vec(B.N, VS_R);
  a.e0 = B.base + off_vec(B.N, VS_P);
  a.de_stride = B.sd;
  a.R0 = B.base + off_refl(B.N);
  a.r_stride = B.sd;
  a.infos = B.infos;
  return tri_launch(c, a, cnt, m);
}

// v <- H^T v / H v for the pass's slots (the tridiagonal path's reflectors): one 512-thread workgroup per
// slot, 16 reflections per round (k_refl_blk; the rounds' compact-WY T blocks from k_refl_gram in the
// slot's matrix area, dead once the tridiagonal T is formed: tri_finish makes them); RIPTRM_TRI_REFL=s one reflection per
// round (k_refl_wg), =w one wave with the vector in registers (k_refl_big) (A/B)
static int tri_refl(riptrm_ctx* c, const Bat& B, int cnt, int m, int64_t voff, int64_t ooff, int backward) {
  const dim3 grid(1, cnt);
  if (!getenv_is("RIPTRM_TRI_REFL", 'w') && !getenv_is("RIPTRM_TRI_REFL", 's')) {
    long long* stamps = nullptr;   // RIPTRM_TRI_STAMPS=3: slot 0's phase cycles on stderr
    if (getenv_is("RIPTRM_TRI_STAMPS", '3')) {
      HIPCHK(c, hipMalloc(&stamps, 4 * sizeof(long long)));
      HIPCHK(c, hipMemsetAsync(stamps, 0, 4 * sizeof(long long), c->stream));
    }
    if (getenv_is("RIPTRM_TRI_REFL_E", '1'))
      hipLaunchKernelGGL(riptrm_tri::k_refl_blk<1>, grid, dim3(1024), 0, c->stream, B.base, B.sd, 0, m, off_refl(B.N),
                         (int64_t)0, voff, ooff, backward, stamps);
    else
      hipLaunchKernelGGL(riptrm_tri::k_refl_blk<2>, grid, dim3(512), 0, c->stream, B.base, B.sd, 0, m, off_refl(B.N),
                         (int64_t)0, voff, ooff, backward, stamps);
    HIPCHK(c, hipGetLastError());
    if (stamps) {
      long long h[4];
      HIPCHK(c, hipMemcpyAsync(h, stamps, sizeof(h), hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      (void)hipFree(stamps);
      const int nb = riptrm_tri::refl_blocks(m);
      fprintf(stderr, "[refl stamps] m=%d rounds=%d per round: operands + dots %.0f, solve %.0f, update %.0f cycles\n", m, nb,
              h[0] / (double)nb, h[1] / (double)nb, h[2] / (double)nb);
    }
    return RIPTRM_OK;
  }
  if (getenv_is("RIPTRM_TRI_REFL", 's')) {
    hipLaunchKernelGGL(riptrm_tri::k_refl_wg, grid, dim3(1024), 0, c->stream, B.base, B.sd, 0, m, off_refl(B.N), voff, ooff,
                       backward);
    HIPCHK(c, hipGetLastError());
    return RIPTRM_OK;
  }
  switch (riptrm_tri::tri_el(m)) {
    case 4: hipLaunchKernelGGL(riptrm_tri::k_refl_big<4>, grid, dim3(64), 0, c->stream, B.base, B.sd, 0, m, off_refl(B.N), voff, ooff, backward); break;
    case 8: hipLaunchKernelGGL(riptrm_tri::k_refl_big<8>, grid, dim3(64), 0, c->stream, B.base, B.sd, 0, m, off_refl(B.N), voff, ooff, backward); break;
    default: hipLaunchKernelGGL(riptrm_tri::k_refl_big<16>, grid, dim3(64), 0, c->stream, B.base, B.sd, 0, m, off_refl(B.N), voff, ooff, backward); break;
  }
  HIPCHK(c, hipGetLastError());
  return RIPTRM_OK;
}

template <int EL>
static int tri_solve_el(riptrm_ctx* c, const Bat& B, int cnt, int m, const double* D, int64_t dstride, double tolhc, int mode,
                        bool cg_skip, bool eig_known) {
  const int64_t N = B.N;
  const size_t shm = (size_t)riptrm_tri::TRI_SOLVE_ARRAYS * 64 * EL * sizeof(double);
  auto kern = riptrm_tri::k_tri_solve<EL>;
  HIPCHK(c, hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
  const riptrm_tri::TriSc S{SC_CG_OK, SC_P1OBJ, SC_KIND, SC_LAM1, SC_MINEIG, SC_INTERIOR, SC_DELTA, SC_AN, SC_ATOL, SC_IT,
                            SC_DONE, SC_TRI_FB, SC_RHO_PREV};   // (SC_RHO_PREV: the Newton steps, diagnostics)
  long long* stamps = nullptr;   // RIPTRM_TRI_STAMPS=1: slot 0's phase clocks on stderr
  if (getenv_is("RIPTRM_TRI_STAMPS", '1')) {
    HIPCHK(c, hipMalloc(&stamps, 10 * sizeof(long long)));
    HIPCHK(c, hipMemsetAsync(stamps, 0, 10 * sizeof(long long), c->stream));
  }
  hipLaunchKernelGGL(kern, dim3(1, cnt), dim3(256), shm, c->stream, B.base, B.sd, B.infos, m, off_vec(N, VS_R),
                     off_vec(N, VS_P), off_vec(N, VS_G), off_vec(N, VS_A), off_vec(N, VS_PE), off_vec(N, VS_CGX),
                     off_vec(N, VS_EV), off_sc(N), S, D, dstride, B.ids, tolhc, mode, cg_skip ? 1 : 0, eig_known ? 1 : 0,
                     getenv_is("RIPTRM_TRI_SERIAL", '1') ? 1 : 0, stamps);
  HIPCHK(c, hipGetLastError());
  if (stamps) {
    long long h[10];
    HIPCHK(c, hipMemcpyAsync(h, stamps, sizeof(h), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    (void)hipFree(stamps);
    if (h[0] && mode == 0) {
      const long long par = std::max(std::max(h[2], h[3]), h[8]);   // the concurrent phases' end
      fprintf(stderr, "[tri_solve stamps] m=%d mode=0 eig %lld hard %lld newton %lld (%lld steps) skip-test %lld cg %lld "
              "(%lld it%s) end %lld\n", m, h[1] - h[0], h[2] - h[1], h[3] - h[1], h[6], h[8] ? h[8] - h[1] : 0,
              h[4] ? h[4] - par : 0, h[7], h[9] ? ", skipped" : "", h[5] - h[0]);
    } else if (h[0]) {
      fprintf(stderr, "[tri_solve stamps] m=%d mode=1 eig %lld\n", m, h[1] - h[0]);
    }
  }
  return RIPTRM_OK;
}

// after tri_tridiag (or a cache load of T): mode 1 the smallest eigenvalue only (-> VS_EV[0]); mode 0
// the subproblem min x^T A x / 2 + a^T x, ||x|| <= Delta (a at VS_A): b = H^T a, k_tri_solve, x = H pe
// -> VS_X and the result scalars.  Subproblems it cannot serve set SC_TRI_FB (tri_fallback_ids).
static int tri_finish(riptrm_ctx* c, const Bat& B, int cnt, int m, const double* D, int64_t dstride, double tolhc, int mode,
                      bool cg_skip = false, bool eig_known = false) {
  const int64_t N = B.N;
  if (mode == 0) {
    hipLaunchKernelGGL(riptrm_tri::k_refl_gram, dim3(riptrm_tri::refl_blocks(m), cnt), dim3(256), 0, c->stream, B.base,
                       B.sd, 0, m, off_refl(N), (int64_t)0);
    HIPCHK(c, hipGetLastError());
    if (int rc = tri_refl(c, B, cnt, m, off_vec(N, VS_A), off_vec(N, VS_G), 0)) return rc;
  }
  int rc;
  switch (riptrm_tri::tri_el(m)) {
    case 4: rc = tri_solve_el<4>(c, B, cnt, m, D, dstride, tolhc, mode, cg_skip, eig_known); break;
    case 8: rc = tri_solve_el<8>(c, B, cnt, m, D, dstride, tolhc, mode, cg_skip, eig_known); break;
    default: rc = tri_solve_el<16>(c, B, cnt, m, D, dstride, tolhc, mode, cg_skip, eig_known); break;
  }
  if (rc) return rc;
  if (mode == 0) return tri_refl(c, B, cnt, m, off_vec(N, VS_PE), off_vec(N, VS_X), 1);
  return RIPTRM_OK;
}

// the ids of the pass whose subproblem set SC_TRI_FB (a hard case or a multiple smallest eigenvalue).
// Synchronises.
// (count_skip: the pass ran k_tri_solve's CG skip test; its outcomes into riptrm_trs_skip_stats)
static int tri_fallback_ids(riptrm_ctx* c, const Bat& B, int cnt, const int32_t* ids, std::vector<int32_t>& out,
                            bool count_skip = false) {
  out.clear();
  std::vector<double> fb(cnt), done(count_skip ? cnt : 0);
  HIPCHK(c, hipMemcpy2DAsync(fb.data(), sizeof(double), B.base + off_sc(B.N) + SC_TRI_FB, (size_t)B.sd * sizeof(double),
                             sizeof(double), cnt, hipMemcpyDeviceToHost, c->stream));
  if (count_skip)
    HIPCHK(c, hipMemcpy2DAsync(done.data(), sizeof(double), B.base + off_sc(B.N) + SC_DONE, (size_t)B.sd * sizeof(double),
                               sizeof(double), cnt, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  for (int k = 0; k < cnt; ++k) {
    if (fb[k] != 0.0) {
      out.push_back(ids[k]);
    } else if (count_skip) {   // (a hard case ends before the test)
      c->big_cg_checked += 1;
      c->big_cg_skipped += done[k] == 4.0;
    }
  }
  c->tri_fallbacks += (int64_t)out.size();
  return RIPTRM_OK;
}

static int big_solve(riptrm_ctx* c, const Bat& B, int cnt, int64_t aoff, int lda, int m, const double* D, int64_t dstride,
                     double tolhc) {
  if (int rc = big_cg(c, B, cnt, aoff, lda, m, D, dstride)) return rc;
  if (int rc = eig_batched(c, B, cnt, true, m, aoff, lda)) return rc;
  return big_after_eig(c, B, cnt, aoff, lda, m, tolhc);
}

// matrices of HwCur (trial = 0: at (x, y), the subproblem's linear term from cxCur) or of HwNew
// (trial = 1: at (x_new, y_new)) for the pass's NonnegPCA instances: A at M + n + 1, lda n
static int big_nonnegpca_matrix(riptrm_ctx* c, const Bat& B, int cnt, int trial) {
  hipStream_t st = c->stream;
  const DevParams& P = c->P;
  const int n = P.n;
  const int64_t N = B.N;
  const int xk = trial ? V_IN1 : V_X, yk = trial ? V_YNEW : V_Y;
  const dim3 one(1, cnt), rows(blocks_of(n, GV / 64), cnt);
  hipLaunchKernelGGL(k_dense, dim3(blocks_of((int64_t)n * n, 256), cnt), dim3(256), 0, st, P, B, xk, yk);
  hipLaunchKernelGGL(k_house, one, dim3(WG), 0, st, P, B, xk, yk);
  hipLaunchKernelGGL(k_gemv, rows, dim3(GV), 0, st, B, (int64_t)0, (int64_t)n, n, n, off_vec(N, VS_W), off_vec(N, VS_U),
                     (int64_t)-1);
  hipLaunchKernelGGL(k_gemv_x, rows, dim3(GV), 0, st, P, B, xk);   // M x for x^T S x (k_repmat_vec)
  hipLaunchKernelGGL(k_repmat_vec, one, dim3(WG), 0, st, P, B, xk, trial ? -1 : (int)V_C);
  hipLaunchKernelGGL(k_transform, dim3(blocks_of((int64_t)(n - 1) * (n - 1), 256), cnt), dim3(256), 0, st, n, B);
  HIPCHK(c, hipGetLastError());
  return RIPTRM_OK;
}

// Serve every instance parked at PH_TRS_HOST / PH_MINEIG_HOST, up to big_slots per pass.  Returns
// the number of instances resumed in *served.  Synchronises.
static bool cache_on(const riptrm_ctx* c) {
  return c->big_cache && c->big_cache_order >= c->P.n && c->big_cache_batch >= c->P.batch;
}

// Serve every instance parked at PH_TRS_HOST / PH_MINEIG_HOST, up to big_slots per pass.  With the
// cache bound, the trial point's pass keeps its eigendecomposition per instance, and a subproblem at
// exactly that (x, y) (the step was accepted without dual clipping) builds its matrix and runs CG
// but takes the cached eigenpairs instead of an eigensolve -- the same bits, as the matrices are
// the same bits.  Returns the number of instances resumed in *served.  Synchronises.
int riptrm_big_service(riptrm_ctx* c, int* served) {
  *served = 0;
  const DevParams& P = c->P;
  const int B = P.batch, n = P.n;
  std::vector<double> st((size_t)B * RIPTRM_STAT_NFIELDS);
  HIPCHK(c, hipMemcpyAsync(st.data(), P.stats, st.size() * sizeof(double), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  std::vector<int32_t> ids[2];   // [0] subproblems, [1] trial eigenvalues
  for (int b = 0; b < B; ++b) {
    const int ph = (int)st[(size_t)b * RIPTRM_STAT_NFIELDS + RIPTRM_STAT_PHASE];
    if (ph == PH_TRS_HOST) ids[0].push_back(b);
    if (ph == PH_MINEIG_HOST) ids[1].push_back(b);
  }
  if (ids[0].empty() && ids[1].empty()) return RIPTRM_OK;
  if (!c->big_ws || c->big_order < n || c->big_slots < 1)
    return fail(c, RIPTRM_E_STATE, "Exact_RepMat above dim 96 needs riptrm_trs_bind_workspace (order >= n)");
  const Bat Bt = bat_of(c);
  const bool cached = cache_on(c);
  double* cache = (double*)c->big_cache;
  const int64_t CN = c->big_cache_order;
  const int64_t aoff = n + 1;   // rows / columns 1.. of the n x n buffer
  const int S = c->big_slots;
  // subproblems: split into cache hits and misses
  std::vector<int32_t> miss, hit;
  if (cached && !ids[0].empty()) {
    int32_t* hits = tail_of(c) + 3 * S + 8;
    std::vector<int32_t> h(S);
    for (size_t k0 = 0; k0 < ids[0].size(); k0 += (size_t)S) {
      const int cnt = (int)std::min<size_t>((size_t)S, ids[0].size() - k0);
      if (int rc = put_ids(c, Bt, ids[0].data() + k0, cnt)) return rc;
      hipLaunchKernelGGL(k_cache_check, dim3(1, cnt), dim3(256), 0, c->stream, P, Bt, cache, CN, hits);
      HIPCHK(c, hipGetLastError());
      HIPCHK(c, hipMemcpyAsync(h.data(), hits, (size_t)cnt * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      for (int k = 0; k < cnt; ++k) (h[k] ? hit : miss).push_back(ids[0][k0 + k]);
    }
  } else {
    miss = ids[0];
  }
  // pass kinds: 0 subproblem with its eigensolve, 1 subproblem on cached eigenpairs, 2 trial eigenvalues
  const std::vector<int32_t>* lists[3] = {&miss, &hit, &ids[1]};
  for (int kind = 0; kind < 3; ++kind) {
    const std::vector<int32_t>& L = *lists[kind];
    for (size_t k0 = 0; k0 < L.size(); k0 += (size_t)S) {
      const int cnt = (int)std::min<size_t>((size_t)S, L.size() - k0);
      if (int rc = put_ids(c, Bt, L.data() + k0, cnt)) return rc;
      if (int rc = big_nonnegpca_matrix(c, Bt, cnt, kind == 2)) return rc;
      const bool tri = tri_mode(n - 1);
      if (kind == 2) {
        // eigenvectors too (the next subproblem at this point reuses them); the value is the same
        // computation with or without the cache.  Tridiagonal path: T and its reflectors are kept.
        if (tri) {
          if (int rc = tri_tridiag(c, Bt, cnt, n - 1, aoff, n)) return rc;
          if (int rc = tri_finish(c, Bt, cnt, n - 1, P.st + ST_DELTA, ST_N, P.opt.trs_tolhardcase, 1)) return rc;
        } else if (int rc = eig_batched(c, Bt, cnt, cached, n - 1, aoff, n)) {   // vectors only for the cache
          return rc;
        }
        hipLaunchKernelGGL(k_finish_mineig, dim3(blocks_of(cnt, 64)), dim3(64), 0, c->stream, P, Bt, cnt,
                           eig_compact(n - 1) ? 1 : 0);
        if (cached)
          hipLaunchKernelGGL(k_cache_store, dim3(blocks_of((int64_t)n * n, 256), cnt), dim3(256), 0, c->stream, P, Bt, cache,
                             CN, tri ? 1 : 0);
      } else if (tri) {   // T (or the cached one), then the subproblem in T's coordinates
        if (kind == 1)
          hipLaunchKernelGGL(k_cache_load, dim3(blocks_of((int64_t)n * n, 256), cnt), dim3(256), 0, c->stream, P, Bt, cache,
                             CN, 1);
        else if (int rc = tri_tridiag(c, Bt, cnt, n - 1, aoff, n))
          return rc;
        const bool skip = !getenv_is("RIPTRM_CG_SKIP", '0');
        // (a cache hit's T comes with the extreme eigenvalues its trial pass found: kind 1)
        if (int rc = tri_finish(c, Bt, cnt, n - 1, P.st + ST_DELTA, ST_N, P.opt.trs_tolhardcase, 0, skip, kind == 1)) return rc;
        hipLaunchKernelGGL(k_finish_dir, dim3(1, cnt), dim3(WG), 0, c->stream, P, Bt);
        std::vector<int32_t> fbi;
        if (int rc = tri_fallback_ids(c, Bt, cnt, L.data() + k0, fbi, skip)) return rc;
        for (size_t f0 = 0; f0 < fbi.size(); f0 += (size_t)S) {   // hard cases: the eigendecomposition path
          const int fc = (int)std::min<size_t>((size_t)S, fbi.size() - f0);
          if (int rc = put_ids(c, Bt, fbi.data() + f0, fc)) return rc;
          if (int rc = big_nonnegpca_matrix(c, Bt, fc, 0)) return rc;
          if (int rc = big_cg(c, Bt, fc, aoff, n, n - 1, P.st + ST_DELTA, ST_N)) return rc;
          if (int rc = eig_batched(c, Bt, fc, true, n - 1, aoff, n)) return rc;
          if (int rc = big_after_eig(c, Bt, fc, aoff, n, n - 1, P.opt.trs_tolhardcase)) return rc;
          hipLaunchKernelGGL(k_finish_dir, dim3(1, fc), dim3(WG), 0, c->stream, P, Bt);
        }
      } else if (eig_compact(n - 1)) {   // eigenpairs (or the cached ones), then the CG in eigen-coordinates
        if (kind == 1)
          hipLaunchKernelGGL(k_cache_load, dim3(blocks_of((int64_t)n * n, 256), cnt), dim3(256), 0, c->stream, P, Bt, cache,
                             CN, 0);
        else if (int rc = eig_batched(c, Bt, cnt, true, n - 1, aoff, n))
          return rc;
        if (int rc = compact_trs(c, Bt, cnt, n - 1, aoff, n, P.st + ST_DELTA, ST_N, P.opt.trs_tolhardcase,
                                 !getenv_is("RIPTRM_CG_SKIP", '0')))
          return rc;
        hipLaunchKernelGGL(k_finish_dir, dim3(1, cnt), dim3(WG), 0, c->stream, P, Bt);
      } else {
        if (int rc = big_cg(c, Bt, cnt, aoff, n, n - 1, P.st + ST_DELTA, ST_N)) return rc;
        if (kind == 1)
          hipLaunchKernelGGL(k_cache_load, dim3(blocks_of((int64_t)n * n, 256), cnt), dim3(256), 0, c->stream, P, Bt, cache,
                             CN, 0);
        else if (int rc = eig_batched(c, Bt, cnt, true, n - 1, aoff, n))
          return rc;
        if (int rc = big_after_eig(c, Bt, cnt, aoff, n, n - 1, P.opt.trs_tolhardcase)) return rc;
        hipLaunchKernelGGL(k_finish_dir, dim3(1, cnt), dim3(WG), 0, c->stream, P, Bt);
      }
      HIPCHK(c, hipGetLastError());
      *served += cnt;
    }
  }
  if (cached) c->big_cache_hits += (int64_t)hit.size();
  c->big_subproblems += (int64_t)ids[0].size();
  return RIPTRM_OK;
}

// a new solve: no cache entry is valid (same (x, y) on other data would otherwise hit)
int riptrm_big_reset_cache(riptrm_ctx* c) {
  c->big_cache_hits = c->big_subproblems = 0;
  if (!c->big_cache) return RIPTRM_OK;
  hipLaunchKernelGGL(k_cache_invalidate, dim3(blocks_of(c->big_cache_batch, 256)), dim3(256), 0, c->stream,
                     (double*)c->big_cache, (int64_t)c->big_cache_order, c->big_cache_batch);
  HIPCHK(c, hipGetLastError());
  return RIPTRM_OK;
}

// TRSgep for the subproblems ids[0..count) of a batch laid out as riptrm_trs_gep's arguments (or,
// mineig_only, just the smallest eigenvalue of each A: RIPTRM.py:611), up to big_slots per pass.
// A non-converged eigensolve fails the call naming the subproblem (scipy.linalg.eig raises there),
// or, with per_instance, only marks that subproblem: kind = RIPTRM_TCG_EIGFAIL / mineig = NaN (the
// caller stops that instance, RIPTRM_ERR_EIGEN).  Synchronises.  Serves riptrm_trs_gep above dim 96 and the StableIdentification solve's parked
// instances (riptrm_si.hip).
static_assert(RIPTRM_EIG_COMPACT_MAX == riptrm_eig::EIG_LDS_MAX, "riptrm_ctx.h's copy of EIG_LDS_MAX");
int64_t riptrm_big_kcache_doubles(int dim, int klen) { return kc_doubles(dim, klen); }
bool riptrm_big_kcache_usable(int dim) { return eig_compact(dim) && !tri_mode(dim); }

// the instances ids whose cache entry matches their key (hit) and the others (miss).  Synchronises.
int riptrm_big_kcache_split(riptrm_ctx* c, int dim, const std::vector<int32_t>& ids, const KeyedEigCache& kc,
                            std::vector<int32_t>& hit, std::vector<int32_t>& miss) {
  hit.clear();
  miss.clear();
  if (ids.empty()) return RIPTRM_OK;
  if (!c->big_ws || c->big_order < dim || c->big_slots < 1)
    return fail(c, RIPTRM_E_STATE, "Exact_RepMat above dim 96 needs riptrm_trs_bind_workspace (order >= dim)");
  const Bat Bt = bat_of(c);
  const int S = c->big_slots;
  int32_t* hits = tail_of(c) + 3 * S + 8;
  std::vector<int32_t> h(S);
  for (size_t k0 = 0; k0 < ids.size(); k0 += (size_t)S) {
    const int cnt = (int)std::min<size_t>((size_t)S, ids.size() - k0);
    if (int rc = put_ids(c, Bt, ids.data() + k0, cnt)) return rc;
    hipLaunchKernelGGL(k_kc_check, dim3(1, cnt), dim3(256), 0, c->stream, Bt, kc.keys, kc.kstride, kc.klen, kc.cache,
                       kc.cstride, hits);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(h.data(), hits, (size_t)cnt * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    for (int k = 0; k < cnt; ++k) (h[k] ? hit : miss).push_back(ids[k0 + k]);
  }
  return RIPTRM_OK;
}

int riptrm_big_gep_ids(riptrm_ctx* c, int dim, const int32_t* sel, int count, const double* A, int64_t lda,
                       int64_t a_stride, const double* a, int64_t ldv, const double* Delta, double tolhc, double* x,
                       double* lam1, int32_t* kind, double* mineig, bool mineig_only, bool per_instance,
                       const KeyedEigCache* kc) {
  if (!c->big_ws || c->big_order < dim || c->big_slots < 1)
    return fail(c, RIPTRM_E_STATE, "Exact_RepMat above dim 96 needs riptrm_trs_bind_workspace (order >= dim)");
  const Bat Bt = bat_of(c);
  const int kmode = (kc && kc->cache && eig_compact(dim) && !tri_mode(dim)) ? kc->mode : 0;
  if (kmode == 1 && mineig_only) return fail(c, RIPTRM_E_STATE, "gep_ids: cached eigenpairs serve subproblems only");
  std::vector<int32_t> info(c->big_slots);
  std::vector<double> skip_done;   // SC_DONE of the pass's slots (4 = CG skipped by k_cg_wg's bound)
  for (int b0 = 0; b0 < count; b0 += c->big_slots) {
    const int cnt = std::min(c->big_slots, count - b0);
    skip_done.clear();
    if (int rc = put_ids(c, Bt, sel + b0, cnt)) return rc;
    // (a hit needs only a: the matrix's first dim entries are copied too and then replaced)
    hipLaunchKernelGGL(k_load, dim3(blocks_of(kmode == 1 ? (int64_t)dim : (int64_t)dim * dim, 256), cnt), dim3(256), 0,
                       c->stream, Bt, dim, A, lda, a_stride, a, ldv);
    HIPCHK(c, hipGetLastError());
    std::vector<int32_t> fb_ids;   // subproblems the tridiagonal path hands to the eigendecomposition path
    if (mineig_only && tri_mode(dim)) {
      if (int rc = tri_tridiag(c, Bt, cnt, dim, 0, dim)) return rc;
      if (int rc = tri_finish(c, Bt, cnt, dim, Delta, 1, tolhc, 1)) return rc;
    } else if (mineig_only) {
      if (int rc = eig_batched(c, Bt, cnt, kmode == 2, dim, 0, dim)) return rc;
      if (kmode == 2)
        hipLaunchKernelGGL(k_kc_store, dim3(blocks_of((int64_t)dim * dim, 256), cnt), dim3(256), 0, c->stream, Bt, dim,
                           kc->keys, kc->kstride, kc->klen, kc->cache, kc->cstride);
    } else if (tri_mode(dim)) {   // T = H^T A H across the chip, the subproblem in T's coordinates
      if (int rc = tri_tridiag(c, Bt, cnt, dim, 0, dim)) return rc;
      const bool skip = per_instance && !getenv_is("RIPTRM_CG_SKIP", '0');
      if (int rc = tri_finish(c, Bt, cnt, dim, Delta, 1, tolhc, 0, skip)) return rc;
      if (int rc = tri_fallback_ids(c, Bt, cnt, sel + b0, fb_ids, skip)) return rc;
    } else if (eig_compact(dim)) {
      // eigenpairs first (or the cached ones), then the CG in eigen-coordinates (k_cg_diag), skipped
      // where the certified bound shows its candidate cannot win (per_instance; RIPTRM_CG_SKIP=0: never)
      const bool skip = per_instance && !getenv_is("RIPTRM_CG_SKIP", '0');
      if (kmode == 1)
        hipLaunchKernelGGL(k_kc_load, dim3(blocks_of((int64_t)dim * dim, 256), cnt), dim3(256), 0, c->stream, Bt, dim,
                           kc->klen, kc->cache, kc->cstride);
      else if (int rc = eig_batched(c, Bt, cnt, true, dim, 0, dim))
        return rc;
      if (int rc = compact_trs(c, Bt, cnt, dim, 0, dim, Delta, 1, tolhc, skip)) return rc;
      if (skip) {
        skip_done.resize(cnt);
        HIPCHK(c, hipMemcpy2DAsync(skip_done.data(), sizeof(double), Bt.base + off_sc(Bt.N) + SC_DONE,
                                   (size_t)Bt.sd * sizeof(double), sizeof(double), cnt, hipMemcpyDeviceToHost, c->stream));
      }
    } else if (per_instance && cg_one_workgroup(dim, cnt) && !getenv_is("RIPTRM_CG_SKIP", '0')) {
      // eigenpairs, g = Q^T a and the boundary candidate first; the CG then reads A from the
      // caller's array and is skipped where the eigenpairs prove the interior candidate cannot win
      // (k_cg_wg's bound), so the choice is the one the CG-first order makes (RIPTRM_CG_SKIP=0)
      if (int rc = eig_batched(c, Bt, cnt, true, dim, 0, dim)) return rc;
      hipStream_t st = c->stream;
      const int64_t N = Bt.N;
      const bool cpt = eig_compact(dim);
      if (cpt)
        if (int rc = refl_apply(c, Bt, cnt, dim, off_vec(N, VS_A), off_vec(N, VS_PE), 0)) return rc;
      hipLaunchKernelGGL(k_gemv, dim3(blocks_of(dim, GV / 64), cnt), dim3(GV), 0, st, Bt, (int64_t)0, (int64_t)dim, dim,
                         dim, off_vec(N, cpt ? VS_PE : VS_A), off_vec(N, VS_G), (int64_t)-1);
      hipLaunchKernelGGL(k_set_delta, dim3(blocks_of(cnt, 64)), dim3(64), 0, st, Bt, cnt, Delta, (int64_t)1);
      hipLaunchKernelGGL(k_secular, dim3(1, cnt), dim3(WG), 0, st, Bt, dim, tolhc, 0);
      if (dim <= CGW_MAX && !getenv_is("RIPTRM_CG_WAVE", '0')) {
        const size_t shm = cg_wave_lds(dim);
        HIPCHK(c, hipFuncSetAttribute((const void*)k_cg_wave, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
        hipLaunchKernelGGL(k_cg_wave, dim3(1, cnt), dim3(64), shm, st, Bt, dim, (int64_t)0, lda, Delta, (int64_t)1, A,
                           a_stride, 1);
      } else {
        const int rl = cg_lds_rows(dim);
        const size_t shm = (size_t)rl * dim * sizeof(double);
        if (shm > 0)
          HIPCHK(c, hipFuncSetAttribute((const void*)k_cg_wg, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
        hipLaunchKernelGGL(k_cg_wg, dim3(1, cnt), dim3(WG), shm, st, Bt, dim, (int64_t)0, lda, Delta, (int64_t)1, rl, A,
                           a_stride, 1);
      }
      skip_done.resize(cnt);
      HIPCHK(c, hipMemcpy2DAsync(skip_done.data(), sizeof(double), Bt.base + off_sc(N) + SC_DONE, (size_t)Bt.sd * sizeof(double),
                                 sizeof(double), cnt, hipMemcpyDeviceToHost, st));
      hipLaunchKernelGGL(k_choose, dim3(blocks_of(cnt, 64)), dim3(64), 0, st, Bt, cnt);
      hipLaunchKernelGGL(k_gemv_t, dim3(blocks_of(dim, 256), cnt), dim3(256), 0, st, Bt, (int64_t)0, (int64_t)dim, dim, dim,
                         off_vec(N, VS_PE), off_vec(N, VS_X));
      if (cpt)
        if (int rc = refl_apply(c, Bt, cnt, dim, off_vec(N, VS_X), off_vec(N, VS_X), 1)) return rc;
      hipLaunchKernelGGL(k_pick, dim3(blocks_of(dim, 256), cnt), dim3(256), 0, st, Bt, dim);
      HIPCHK(c, hipGetLastError());
    } else if (int rc = big_solve(c, Bt, cnt, 0, dim, dim, Delta, 1, tolhc)) {
      return rc;
    }
    HIPCHK(c, hipMemcpyAsync(info.data(), Bt.infos, (size_t)cnt * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->big_cg_checked += (int64_t)skip_done.size();
    for (double v : skip_done) c->big_cg_skipped += v == 4.0;
    for (int k = 0; k < cnt; ++k)
      if (info[k] != 0 && !per_instance)
        return fail(c, RIPTRM_E_HIP, "Exact_RepMat: rocsolver_dsyevd did not converge (info " + std::to_string(info[k]) +
                                         ") on subproblem " + std::to_string(sel[b0 + k]));
    if (mineig_only)
      hipLaunchKernelGGL(k_min_out, dim3(blocks_of(cnt, 64)), dim3(64), 0, c->stream, Bt, cnt, mineig,
                         (eig_compact(dim) || tri_mode(dim)) ? 1 : 0);
    else
      hipLaunchKernelGGL(k_gep_out, dim3(blocks_of(dim, 256), cnt), dim3(256), 0, c->stream, Bt, dim, ldv, x, lam1, kind,
                         mineig);
    HIPCHK(c, hipGetLastError());
    if (!mineig_only) {
      static const int32_t eigfail = RIPTRM_TCG_EIGFAIL;
      for (int k = 0; k < cnt; ++k)
        if (info[k] != 0)
          HIPCHK(c, hipMemcpyAsync(kind + sel[b0 + k], &eigfail, sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
    }
    // hard cases of the tridiagonal path: the eigendecomposition path (rocSOLVER dsyevd), one more pass
    if (!fb_ids.empty()) {
      const int fc = (int)fb_ids.size();   // <= cnt <= big_slots
      if (int rc = put_ids(c, Bt, fb_ids.data(), fc)) return rc;
      hipLaunchKernelGGL(k_load, dim3(blocks_of((int64_t)dim * dim, 256), fc), dim3(256), 0, c->stream, Bt, dim, A, lda,
                         a_stride, a, ldv);
      HIPCHK(c, hipGetLastError());
      if (int rc = big_solve(c, Bt, fc, 0, dim, dim, Delta, 1, tolhc)) return rc;
      HIPCHK(c, hipMemcpyAsync(info.data(), Bt.infos, (size_t)fc * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
      HIPCHK(c, hipStreamSynchronize(c->stream));
      for (int k = 0; k < fc; ++k)
        if (info[k] != 0 && !per_instance)
          return fail(c, RIPTRM_E_HIP, "Exact_RepMat: rocsolver_dsyevd did not converge (info " + std::to_string(info[k]) +
                                           ") on subproblem " + std::to_string(fb_ids[k]));
      hipLaunchKernelGGL(k_gep_out, dim3(blocks_of(dim, 256), fc), dim3(256), 0, c->stream, Bt, dim, ldv, x, lam1, kind,
                         mineig);
      HIPCHK(c, hipGetLastError());
      static const int32_t eigfail2 = RIPTRM_TCG_EIGFAIL;
      for (int k = 0; k < fc; ++k)
        if (info[k] != 0)
          HIPCHK(c, hipMemcpyAsync(kind + fb_ids[k], &eigfail2, sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
    }
  }
  return RIPTRM_OK;
}

// riptrm_trs_gep for dim > RIPTRM_TRS_DIM_MAX
int riptrm_big_trs_gep(riptrm_ctx* c, int dim, int batch, const double* A, int64_t lda, int64_t a_stride, const double* a,
                       int64_t ldv, const double* Delta, double tolhc, double* x, double* lam1, int32_t* kind,
                       double* mineig) {
  std::vector<int32_t> ids(batch);
  for (int b = 0; b < batch; ++b) ids[b] = b;
  return riptrm_big_gep_ids(c, dim, ids.data(), batch, A, lda, a_stride, a, ldv, Delta, tolhc, x, lam1, kind, mineig,
                            false, false);
}

extern "C" {

int riptrm_trs_backend_status(char* msg, int32_t len) {
  Solver& s = solver();
  if (msg && len > 0) {
    const std::string t = s.ok ? std::string("rocBLAS + rocSOLVER dsyevd_strided_batched loaded") : s.why;
    std::strncpy(msg, t.c_str(), (size_t)len - 1);
    msg[len - 1] = 0;
  }
  return s.ok ? RIPTRM_OK : RIPTRM_E_HIP;
}

int64_t riptrm_trs_workspace_bytes(int32_t order, int32_t slots) {
  if (order < 1 || slots < 1) return 0;
  return slot_doubles(order) * 8 * (int64_t)slots + tail_bytes(slots) + 256;
}

int64_t riptrm_trs_cache_bytes(int32_t order, int32_t batch) {
  if (order < 1 || batch < 1) return 0;
  return cache_doubles(order) * 8 * (int64_t)batch;
}

int riptrm_trs_bind_cache(riptrm_ctx* ctx, void* cache, int64_t bytes, int32_t order, int32_t batch) {
  if (!ctx) return RIPTRM_E_ARG;
  if (!cache) {   // unbind
    ctx->big_cache = nullptr;
    ctx->big_cache_order = ctx->big_cache_batch = 0;
    return RIPTRM_OK;
  }
  if (order < 1 || batch < 1 || bytes < riptrm_trs_cache_bytes(order, batch) || ((uintptr_t)cache % 256) != 0)
    return fail(ctx, RIPTRM_E_ARG, "trs_bind_cache: need order, batch >= 1, 256-byte alignment and "
                                   "riptrm_trs_cache_bytes(order, batch) bytes");
  ctx->big_cache = (char*)cache;
  ctx->big_cache_order = order;
  ctx->big_cache_batch = batch;
  return riptrm_big_reset_cache(ctx);
}

int riptrm_trs_cache_stats(riptrm_ctx* ctx, int64_t* hits, int64_t* subproblems) {
  if (!ctx) return RIPTRM_E_ARG;
  if (hits) *hits = ctx->big_cache_hits;
  if (subproblems) *subproblems = ctx->big_subproblems;
  return RIPTRM_OK;
}

int riptrm_sym_eig(riptrm_ctx* ctx, int32_t dim, int32_t batch, double* A, int64_t lda, int64_t a_stride, double* w,
                   int64_t w_stride, int32_t* info, int32_t vectors) {
  if (!ctx) return RIPTRM_E_ARG;
  if (dim < 1 || dim > riptrm_eig::EIG_LDS_MAX || batch < 1 || !A || !w || !info || lda < dim ||
      a_stride < (int64_t)dim * lda || w_stride < dim)
    return fail(ctx, RIPTRM_E_ARG, "sym_eig: need 1 <= dim <= " + std::to_string(riptrm_eig::EIG_LDS_MAX) +
                                       ", batch >= 1, lda >= dim, a_stride >= dim * lda, w_stride >= dim");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const int64_t sc = riptrm_eig::vpad_eig(dim);
  const int64_t per = 2 * sc + (int64_t)riptrm_eig::refl_doubles(dim);   // d, e, reflectors + tau
  const size_t need = (size_t)per * batch * sizeof(double);
  if (ctx->eig_scratch_bytes < need) {
    if (ctx->eig_scratch) HIPCHK(ctx, hipFree(ctx->eig_scratch));
    ctx->eig_scratch = nullptr;
    ctx->eig_scratch_bytes = 0;
    HIPCHK(ctx, hipMalloc(&ctx->eig_scratch, need));
    ctx->eig_scratch_bytes = need;
  }
  double* s = (double*)ctx->eig_scratch;
  long long* stamps = nullptr;   // RIPTRM_EIG_STAMPS=1: per-phase clocks of matrix 0 on stderr (diagnostics)
  const bool want_stamps = getenv_is("RIPTRM_EIG_STAMPS", '1');
  if (want_stamps) HIPCHK(ctx, hipMalloc(&stamps, (size_t)batch * 8 * sizeof(long long)));
  if (int rc = launch_eig(ctx, batch, dim, A, a_stride, (int)lda, w, w_stride, s, s + sc, per, s + 2 * sc, per, info,
                          vectors == 2 ? 2 : (vectors ? 1 : 0), stamps))
    return rc;
  if (want_stamps) {
    std::vector<long long> h((size_t)batch * 8);
    HIPCHK(ctx, hipMemcpyAsync(h.data(), stamps, h.size() * sizeof(long long), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    (void)hipFree(stamps);
    const long long* t = h.data();
    fprintf(stderr, "[eig stamps] m=%d load+tridiag %lld (reflector %lld symv %lld) bisect %lld vectors(twisted+backtransform) %lld "
            "orthog %lld total %lld\n",
            dim, t[1] - t[0], t[6], t[7], t[2] - t[1], t[3] - t[2], t[5] - t[4], t[5] - t[0]);
  }
  return RIPTRM_OK;
}

int riptrm_sym_tridiag(riptrm_ctx* ctx, int32_t dim, int32_t batch, const double* A, int64_t lda, int64_t a_stride,
                       double* d, double* e, int64_t de_stride, int32_t* info) {
  if (!ctx) return RIPTRM_E_ARG;
  if (dim < 64 || dim > riptrm_tri::TRI_MAX || batch < 1 || !A || !d || !e || !info || lda < dim ||
      a_stride < (int64_t)dim * lda || de_stride < dim)
    return fail(ctx, RIPTRM_E_ARG, "sym_tridiag: need 64 <= dim <= " + std::to_string(riptrm_tri::TRI_MAX) +
                                       ", batch >= 1, lda >= dim, a_stride >= dim * lda, de_stride >= dim");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const int64_t per = (int64_t)riptrm_eig::refl_doubles(dim);   // the reflectors + tau of one matrix
  const size_t need = (size_t)per * batch * sizeof(double);
  if (ctx->eig_scratch_bytes < need) {
    if (ctx->eig_scratch) HIPCHK(ctx, hipFree(ctx->eig_scratch));
    ctx->eig_scratch = nullptr;
    ctx->eig_scratch_bytes = 0;
    HIPCHK(ctx, hipMalloc(&ctx->eig_scratch, need));
    ctx->eig_scratch_bytes = need;
  }
  riptrm_tri::TriArgs a{};
  a.A0 = A;
  a.a_stride = a_stride;
  a.lda = lda;
  a.d0 = d;
  a.e0 = e;
  a.de_stride = de_stride;
  a.R0 = (double*)ctx->eig_scratch;
  a.r_stride = per;
  a.infos = info;
  return tri_launch(ctx, a, batch, dim);
}

int riptrm_trs_skip_stats(riptrm_ctx* ctx, int64_t* checked, int64_t* skipped) {
  if (!ctx) return RIPTRM_E_ARG;
  if (checked) *checked = ctx->big_cg_checked;
  if (skipped) *skipped = ctx->big_cg_skipped;
  return RIPTRM_OK;
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
