// riptrm_si.hip — RIPTRM (tCG path) for StableIdentification on MI355X (gfx950).
//
// Problem (src/StableIdentification/coordinator.py:13-152): Product(SkewSymmetric(d), SPD(d),
// SPD(d)) with f(J,R,Q) = tr(E E^T)/N, E = XP - (I + h A) X, A = (J-R)Q, and m box constraints on
// entries of A.  Everything is d x d (the fixture has d = 5, m = 16, N = 95), so one workgroup runs
// one instance's WHOLE solve in one launch: thread l < d*d owns element (l / d, l % d) of every
// d x d block; products go through LDS (one staging write + d reads per operand).  No S-pass, no
// host round trip.
//   d <= 8:  one 64-lane wave; inner products / norms are wave butterflies, R^-1 / Q^-1 and the
//            evaluation's Cholesky / Jacobi eigenvalues (dist, manifold violation) run serially in
//            the registers of 2 / 4 lanes.
//   8 < d <= RIPTRM_SI_DMAX:  NT = 64 ceil(d^2 / 64) threads (one element each); inner products are
//            workgroup reductions (riptrm_trs::Blk), lane reads go through LDS, and the dense
//            solvers run on the whole workgroup: Gauss-Jordan inverse with partial pivoting and a
//            right-looking Cholesky, one pivot per step, and the SPD distance's eigenvalues by the
//            parallel Jacobi of riptrm_trs.h.
//
// Math = oracle/si_oracle.py::SIVectorized (the Lagrangian aggregated through dL/dA), i.e.
//   HessL[v]  = e2rh(x, chain(G_L), chain_hess(G_L, dG_L, v), v)        RIPTRM.py:491-523
//   Gx(w)     = -e2rg(x, chain(sum_i w_i dg_i/dA))                        RIPTRM.py:525-551
//   Gxaj(v)_i = -(dg_i/dA) : dA(v)                                        RIPTRM.py:553-571
// with pymanopt's SPD (affine-invariant) and SkewSymmetric formulas restated.
// Control flow = RIPTRM.py:41-216 (tCG), :574-629, :631-705, :707-896, :909-976 — the same as
// the NonnegPCA state machine in riptrm_kernels.hip, written as plain loops.
#include <hip/hip_runtime.h>
#include <math.h>
#include <cstring>
#include <string>
#include <vector>
#include "riptrm_ctx.h"
#include "riptrm_wave.h"
#include "riptrm_trs.h"

namespace riptrm_si {

#pragma clang fp contract(off)

constexpr int W = 64;
constexpr int DMAX = RIPTRM_SI_DMAX;
constexpr int MMAX = RIPTRM_SI_MMAX;
constexpr int CF = RIPTRM_SI_CONS_FIELDS;

enum Mode : int { MODE_SOLVE = 0, MODE_HVP = 1, MODE_TCG = 2, MODE_RESUME = 3 };

struct SIParams {
  int32_t d, N, m, batch, cap, mode, tab_len, pad;
  double h, clock_hz;
  const double* X;
  const double* XP;
  int64_t data_stride;
  const double* cons;
  int64_t cons_stride;
  double* x;       // batch x 3dd   current point / result
  double* y;       // batch x m
  double* eta;     // batch x 3dd
  double* heta;    // batch x 3dd
  double* escr;    // batch x d x N residual scratch
  double* stats;   // batch x RIPTRM_STAT_NFIELDS
  double* log;     // batch x cap x RIPTRM_LOG_NFIELDS
  double* prof;    // optional: batch x RIPTRM_SI_PROF_NFIELDS device-clock ticks per section
  const double* in_x;
  const double* in_y;
  const double* in_mu;
  const double* in_delta;
  const double* in_v;
  double* out_v;
  const double* mu_tab;
  const double* tolL_tab;
  const double* tolC_tab;
  // Exact_RepMat above RIPTRM_TRS_DIM_MAX (si_hbm_trs): the parked subproblems and the resume records
  double* trsA;      // batch x tdim x tdim   matrix of HwCur / HwNew in the tangent frame
  double* trsP;      // batch x (3dd + m + 1) the point (x, y) and mu of the parked subproblem's matrix
  int32_t* trsids;   // 2 batch                the instances of a k_si_repmat launch
  double* trsE;      // batch x tdim x d x N   k_si_repmat's residual scratch when d N does not fit LDS
  double* trsa;      // batch x tdp           coordinates of cxCur
  double* trsx;      // batch x tdp           the subproblem's solution (host service)
  double* trsD;      // batch                 Delta
  double* trslam;    // batch                 lam1 (host service)
  int32_t* trskind;  // batch                 RIPTRM_TRS_* (host service)
  double* trsmin;    // batch                 smallest eigenvalue of HwNew's matrix (host service)
  double* rs;        // batch x rs_doubles    resume records
  double* trsW;      // batch x SI_PREP_F x nt the park point's prepare / frame / X X^T per lane (k_si_prep)
  double* trsC;      // batch x trsC_stride   the service's keyed eigendecomposition cache (tdim <= 199)
  int64_t trsC_stride;
  int32_t tdim, tdp;
  riptrm_options opt;
};

struct Layout {
  int64_t off_x, off_y, off_eta, off_heta, off_escr, off_stats, off_log, total;
  int64_t off_tA, off_tP, off_tids, off_tE, off_ta, off_tx, off_tD, off_tlam, off_tkind, off_tmin, off_rs;   // 0: no HBM subproblem path
  int64_t off_tC, tC_stride;   // the keyed eigendecomposition cache (0: none)
  int64_t off_tW;              // k_si_prep's per-lane records
};

inline int64_t rup(int64_t a, int64_t m) { return (a + m - 1) / m * m; }

// manifold.dim of Product(Skew(d), SPD(d), SPD(d)) and whether its Exact_RepMat subproblem takes the
// HBM path (parked instances served by the host's batched TRS service, riptrm_trs_big.hip)
__host__ __device__ constexpr int si_manifold_dim(int d) { return d * (d - 1) / 2 + d * (d + 1); }
__host__ __device__ constexpr bool si_hbm_trs(int d) { return si_manifold_dim(d) > RIPTRM_TRS_DIM_MAX; }
__host__ __device__ constexpr int si_tdp(int d) { return (si_manifold_dim(d) + 31) / 32 * 32; }
// resume record: 32 scalars (incl. the section ticks), then 21 rows of one double per thread
// (x, xI, xPrev, xHead, x0, eta as 3 rows each; y, yI, y0)
constexpr int RS_NSC = 32, RS_PT = 20, RS_ROWS = 21;
// k_si_repmat keeps each workgroup's residual E (d x N) in LDS up to this size, else in its own
// slice of an HBM scratch (every workgroup of an instance computes the same E: a shared one would
// be a race on identical values)
constexpr int SI_REPMAT_E_LDS = 48 * 1024;
__host__ __device__ constexpr bool si_repmat_e_lds(int d, int N) { return (int64_t)d * N * 8 <= SI_REPMAT_E_LDS; }
__host__ __device__ constexpr int si_nt(int d) { return d <= 8 ? 64 : (d * d + 63) / 64 * 64; }
__host__ __device__ constexpr int64_t si_rs_doubles(int d) { return RS_NSC + (int64_t)RS_ROWS * si_nt(d); }
// k_si_prep's record per lane: AtX (x 3, metric 2, A Gf GL sgR sgQ f, s w y, c 3), Frame 4, M2
constexpr int SI_PREP_F = 22;

inline Layout make_layout(int d, int N, int m, int batch, int cap) {
  Layout L;
  const int64_t v3 = 3LL * d * d;
  int64_t o = 0;
  L.off_x = o;     o = rup(o + 8 * batch * v3, 256);
  L.off_y = o;     o = rup(o + 8LL * batch * m, 256);
  L.off_eta = o;   o = rup(o + 8 * batch * v3, 256);
  L.off_heta = o;  o = rup(o + 8 * batch * v3, 256);
  L.off_escr = o;  o = rup(o + 8LL * batch * d * N, 256);
  L.off_stats = o; o = rup(o + 8LL * batch * RIPTRM_STAT_NFIELDS, 256);
  L.off_log = o;   o = rup(o + 8LL * batch * cap * RIPTRM_LOG_NFIELDS, 256);
  L.off_tA = L.off_tP = L.off_tids = L.off_tE = L.off_ta = L.off_tx = L.off_tD = L.off_tlam = L.off_tkind = L.off_tmin = L.off_rs = 0;
  L.off_tC = L.tC_stride = L.off_tW = 0;
  if (si_hbm_trs(d)) {
    const int64_t td = si_manifold_dim(d), tp = si_tdp(d);
    L.off_tA = o;    o = rup(o + 8 * batch * td * td, 256);
    L.off_tP = o;    o = rup(o + 8LL * batch * (3LL * d * d + m + 1), 256);
    L.off_tids = o;  o = rup(o + 4LL * 2 * batch, 256);
    if (!si_repmat_e_lds(d, N)) {
      L.off_tE = o;  o = rup(o + 8 * batch * td * d * N, 256);
    }
    L.off_ta = o;    o = rup(o + 8 * batch * tp, 256);
    L.off_tx = o;    o = rup(o + 8 * batch * tp, 256);
    L.off_tD = o;    o = rup(o + 8LL * batch, 256);
    L.off_tlam = o;  o = rup(o + 8LL * batch, 256);
    L.off_tkind = o; o = rup(o + 4LL * batch, 256);
    L.off_tmin = o;  o = rup(o + 8LL * batch, 256);
    L.off_rs = o;    o = rup(o + 8 * batch * si_rs_doubles(d), 256);
    L.off_tW = o;    o = rup(o + 8LL * batch * SI_PREP_F * si_nt(d), 256);
    if (td <= RIPTRM_EIG_COMPACT_MAX) {   // keyed by the park point (x, y, mu): 3dd + m + 1 doubles
      L.tC_stride = rup(riptrm_big_kcache_doubles((int)td, 3 * d * d + m + 1), 32);
      L.off_tC = o;  o = rup(o + 8 * batch * L.tC_stride, 256);
    }
  }
  L.total = o;
  return L;
}

// numpy.minimum / numpy.maximum (NaN-propagating), RIPTRM.py:681-683
__device__ __forceinline__ double np_min(double a, double b) { return (isnan(a) || isnan(b)) ? NAN : (b < a ? b : a); }
__device__ __forceinline__ double np_max(double a, double b) { return (isnan(a) || isnan(b)) ? NAN : (b > a ? b : a); }

// value of v on lane src.  A wave op: call it on every lane (never inside a lane-dependent
// branch or ?:), inactive source lanes read as 0.
__device__ __forceinline__ double lane_read(double v, int src) {
  const int addr = src << 2;
  const int lo = __builtin_amdgcn_ds_bpermute(addr, __double2loint(v));
  const int hi = __builtin_amdgcn_ds_bpermute(addr, __double2hiint(v));
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double wsum(double v) { return riptrm_wave::wave_sum(v); }
__device__ __forceinline__ double wmin(double v) { return riptrm_wave::wave_min(v); }
__device__ __forceinline__ double wmax(double v) { return riptrm_wave::wave_max(v); }

// a point / tangent vector of the product: this lane's element of J, R and Q
struct PV {
  double j, r, q;
};
__device__ __forceinline__ PV pv_add(PV a, PV b) { return PV{a.j + b.j, a.r + b.r, a.q + b.q}; }
__device__ __forceinline__ PV pv_sub(PV a, PV b) { return PV{a.j - b.j, a.r - b.r, a.q - b.q}; }
__device__ __forceinline__ PV pv_scale(double s, PV a) { return PV{s * a.j, s * a.r, s * a.q}; }
__device__ __forceinline__ PV pv_neg(PV a) { return PV{-a.j, -a.r, -a.q}; }

struct Info {  // inner-iteration record of solver_status (RIPTRM.py:986-1023)
  double has, num, status, tr, dxtype, normdx, minx, miny, compl_, hasratio, ratio, ru, dc, hasmin, mineig;
};

// ---- serial d x d linear algebra on ONE lane, register arrays, fully unrolled for D ---------
// (numpy.linalg.solve / inv, cholesky and eigvalsh analogues; evaluation-only except inv)
template <int D>
__device__ __forceinline__ void inv_reg(const double (&a0)[D * D], double (&out)[D * D]) {
  double a[D * D];
#pragma unroll
  for (int i = 0; i < D * D; ++i) { a[i] = a0[i]; out[i] = 0.0; }
#pragma unroll
  for (int i = 0; i < D; ++i) out[i * D + i] = 1.0;
#pragma unroll
  for (int k = 0; k < D; ++k) {  // Gauss-Jordan with partial pivoting
    int p = k;
    double best = fabs(a[k * D + k]);
#pragma unroll
    for (int r = k + 1; r < D; ++r) {
      const double v = fabs(a[r * D + k]);
      if (v > best) { best = v; p = r; }
    }
#pragma unroll
    for (int r = k + 1; r < D; ++r)
      if (r == p) {
#pragma unroll
        for (int c = 0; c < D; ++c) {
          double t = a[k * D + c]; a[k * D + c] = a[r * D + c]; a[r * D + c] = t;
          t = out[k * D + c]; out[k * D + c] = out[r * D + c]; out[r * D + c] = t;
        }
      }
    const double piv = a[k * D + k];
#pragma unroll
    for (int c = 0; c < D; ++c) { a[k * D + c] = a[k * D + c] / piv; out[k * D + c] = out[k * D + c] / piv; }
#pragma unroll
    for (int r = 0; r < D; ++r) {
      if (r == k) continue;
      const double f = a[r * D + k];
#pragma unroll
      for (int c = 0; c < D; ++c) {
        a[r * D + c] = a[r * D + c] - f * a[k * D + c];
        out[r * D + c] = out[r * D + c] - f * out[k * D + c];
      }
    }
  }
}

// cyclic Jacobi: eigenvalues of symmetric a end on its diagonal
template <int D>
__device__ __forceinline__ void jacobi_reg(double (&a)[D * D]) {
  for (int sweep = 0; sweep < 60; ++sweep) {
    double off = 0.0, dg = 0.0;
#pragma unroll
    for (int p = 0; p < D; ++p) {
      dg += a[p * D + p] * a[p * D + p];
#pragma unroll
      for (int q = p + 1; q < D; ++q) off += a[p * D + q] * a[p * D + q];
    }
    if (off <= 1e-36 * dg) break;   // converged far below the eigenvalues' rounding
#pragma unroll
    for (int p = 0; p < D; ++p)
#pragma unroll
      for (int q = p + 1; q < D; ++q) {
        const double apq = a[p * D + q];
        if (apq != 0.0) {
          const double app = a[p * D + p], aqq = a[q * D + q];
          const double theta = (aqq - app) / (2.0 * apq);
          const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
          const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
#pragma unroll
          for (int k = 0; k < D; ++k) {
            const double akp = a[k * D + p], akq = a[k * D + q];
            a[k * D + p] = c * akp - s * akq;
            a[k * D + q] = s * akp + c * akq;
          }
#pragma unroll
          for (int k = 0; k < D; ++k) {
            const double apk = a[p * D + k], aqk = a[q * D + k];
            a[p * D + k] = c * apk - s * aqk;
            a[q * D + k] = s * apk + c * aqk;
          }
        }
      }
  }
}

// all eigenvalues of symmetric a > 0 (numpy.linalg.eigvalsh reads the lower triangle)
template <int D>
__device__ __forceinline__ bool pd_reg(double (&a)[D * D]) {
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = i + 1; j < D; ++j) a[i * D + j] = a[j * D + i];
  jacobi_reg<D>(a);
  bool pd = true;
#pragma unroll
  for (int i = 0; i < D; ++i) pd = pd && (a[i * D + i] > 0.0);
  return pd;
}

// lower Cholesky factor L of A (NaN entries if A is not PD) and L^-1 (Exact_RepMat tangent frame)
template <int D>
__device__ __forceinline__ void chol_inv_reg(const double (&A)[D * D], double (&Lm)[D * D], double (&Li)[D * D]) {
#pragma unroll
  for (int i = 0; i < D * D; ++i) { Lm[i] = 0.0; Li[i] = 0.0; }
#pragma unroll
  for (int j = 0; j < D; ++j) {
    double s = A[j * D + j];
#pragma unroll
    for (int k = 0; k < j; ++k) s -= Lm[j * D + k] * Lm[j * D + k];
    const double cjj = sqrt(s);
    Lm[j * D + j] = cjj;
#pragma unroll
    for (int i = j + 1; i < D; ++i) {
      double t = A[i * D + j];
#pragma unroll
      for (int k = 0; k < j; ++k) t -= Lm[i * D + k] * Lm[j * D + k];
      Lm[i * D + j] = t / cjj;
    }
  }
#pragma unroll
  for (int j = 0; j < D; ++j) {
    Li[j * D + j] = 1.0 / Lm[j * D + j];
#pragma unroll
    for (int i = j + 1; i < D; ++i) {
      double t = 0.0;
#pragma unroll
      for (int k = j; k < i; ++k) t -= Lm[i * D + k] * Li[k * D + j];
      Li[i * D + j] = t / Lm[i * D + i];
    }
  }
}

// pymanopt SPD dist: ||logm(C^-1 B C^-T)||_F, C = cholesky(A); NaN if A is not PD
template <int D>
__device__ __forceinline__ double spd_dist_reg(const double (&A)[D * D], const double (&B)[D * D]) {
  double Cm[D * D];
#pragma unroll
  for (int i = 0; i < D * D; ++i) Cm[i] = 0.0;
  bool ok = true;
#pragma unroll
  for (int j = 0; j < D; ++j) {
    double s = A[j * D + j];
#pragma unroll
    for (int k = 0; k < j; ++k) s -= Cm[j * D + k] * Cm[j * D + k];
    ok = ok && (s > 0.0);
    const double cjj = sqrt(s > 0.0 ? s : 1.0);
    Cm[j * D + j] = cjj;
#pragma unroll
    for (int i = j + 1; i < D; ++i) {
      double t = A[i * D + j];
#pragma unroll
      for (int k = 0; k < j; ++k) t -= Cm[i * D + k] * Cm[j * D + k];
      Cm[i * D + j] = t / cjj;
    }
  }
  double Ci[D * D];  // C^-1, lower triangular
#pragma unroll
  for (int i = 0; i < D * D; ++i) Ci[i] = 0.0;
#pragma unroll
  for (int j = 0; j < D; ++j) {
    Ci[j * D + j] = 1.0 / Cm[j * D + j];
#pragma unroll
    for (int i = j + 1; i < D; ++i) {
      double t = 0.0;
#pragma unroll
      for (int k = j; k < i; ++k) t -= Cm[i * D + k] * Ci[k * D + j];
      Ci[i * D + j] = t / Cm[i * D + i];
    }
  }
  double T[D * D];   // B Ci^T
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = 0; j < D; ++j) {
      double t = 0.0;
#pragma unroll
      for (int k = 0; k < D; ++k) t += B[i * D + k] * Ci[j * D + k];
      T[i * D + j] = t;
    }
  double M[D * D];   // Ci (B Ci^T)
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = 0; j < D; ++j) {
      double t = 0.0;
#pragma unroll
      for (int k = 0; k < D; ++k) t += Ci[i * D + k] * T[k * D + j];
      M[i * D + j] = t;
    }
#pragma unroll
  for (int i = 0; i < D; ++i)
#pragma unroll
    for (int j = i + 1; j < D; ++j) {
      const double sm = 0.5 * (M[i * D + j] + M[j * D + i]);
      M[i * D + j] = sm;
      M[j * D + i] = sm;
    }
  jacobi_reg<D>(M);
  double s2 = 0.0;
#pragma unroll
  for (int i = 0; i < D; ++i) {
    const double lg = log(M[i * D + i]);
    s2 += lg * lg;
  }
  return ok ? sqrt(s2) : NAN;
}

// threads of the workgroup for block size D: one wave up to D = 8, one thread per element above
__host__ __device__ constexpr int si_threads(int D) { return si_nt(D); }

// LDS doubles a big-D workgroup needs besides its static arrays: the broadcast buffer, the
// reduction buffers, the dense solvers' row / column buffers and the Jacobi work area
__host__ __device__ constexpr int si_big_lds_doubles(int D) {
  return si_threads(D) + 2 * (si_threads(D) / 64) + 4 * D + riptrm_trs::work_doubles(D);
}

// sum_t a_t b_t in t order (one sequential chain), the loads issued eight at a time: a loop of
// load, wait, multiply-add waits out one memory latency per term (N = 95 terms on the data)
__device__ __forceinline__ double dot_seq(const double* a, const double* b, int N) {
  double acc = 0.0;
  int t = 0;
  for (; t + 8 <= N; t += 8) {
    double x[8], y[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      x[u] = a[t + u];
      y[u] = b[t + u];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc = acc + x[u] * y[u];
  }
  for (; t < N; ++t) acc = acc + a[t] * b[t];
  return acc;
}

template <int D, int NT = si_threads(D)>
struct Eng {
  static constexpr int d = D, dd = D * D;
  static constexpr bool BIG = NT > W;
  const SIParams& P;
  const int b, l, m, N;
  const int li, lj;
  const bool act, cact;
  double* sh;      // LDS staging: 2 x 64 doubles
  double* ser;     // LDS scratch for the per-lane serial solvers: 8 x 64 doubles
  int* cr_s;       // LDS constraint rows / cols / kinds
  int* cc_s;
  double* tl;      // LDS work area of the Exact_RepMat subproblem (riptrm_trs.h), null for tCG;
                   // big D: bc (NT), red (2 NT / 64), colv / rowa / rowo / rowx (D each), the Jacobi work
  // constraint of this lane (l < m)
  int ck, cr, cc;
  double cp0, cp1;
  double M2;       // (X X^T)_{li,lj}
  const double* Xd;
  const double* XPd;
  double* E;
  double pt[RIPTRM_SI_PROF_NFIELDS];   // section tick totals (riptrm_si_profile_*)
  __device__ __forceinline__ double tick() const { return P.prof ? (double)wall_clock64() : 0.0; }

  double* bc;      // big D: LDS broadcast buffer (NT)
  riptrm_trs::Blk<NT> blk;   // big D: workgroup reductions
  double* colv;    // big D: the dense solvers' pivot column / rows (D each)
  double* rowa;
  double* rowo;
  double* rowx;
  double* jw;      // big D: riptrm_trs Work area of the SPD distance's eigenvalues

  __device__ __forceinline__ Eng(const SIParams& P_, int b_, double* sh_, double* ser_, int* crs, int* ccs, double* tl_,
                                 bool with_m2 = true)
      : P(P_), b(b_), l((int)threadIdx.x), m(P_.m), N(P_.N),
        li((int)threadIdx.x / D), lj((int)threadIdx.x % D), act((int)threadIdx.x < D * D),
        cact((int)threadIdx.x < P_.m), sh(sh_), ser(ser_), cr_s(crs), cc_s(ccs), tl(tl_),
        bc(tl_), blk(BIG ? tl_ + NT : nullptr) {
    // one wave: the row / column buffers of par_inv in the serial solvers' spare slot 6 of ser
    colv = BIG ? tl_ + NT + 2 * (NT / 64) : ser_ + 6 * W;
    rowa = colv + D;
    rowo = rowa + D;
    rowx = rowo + D;
    jw = rowx + D;
    Xd = P.X + (int64_t)b * P.data_stride;
    XPd = P.XP + (int64_t)b * P.data_stride;
    E = P.escr + (int64_t)b * d * N;
    const double* cs = P.cons + (int64_t)b * P.cons_stride;
    ck = 0; cr = 0; cc = 0; cp0 = 0.0; cp1 = 0.0;
    if (cact) {
      ck = (int)cs[l * CF + 0];
      cr = (int)cs[l * CF + 1];
      cc = (int)cs[l * CF + 2];
      cp0 = cs[l * CF + 3];
      cp1 = cs[l * CF + 4];
      cr_s[l] = cr;
      cc_s[l] = cc;
    }
    // X X^T (f's Hessian, coordinator.py:92-98)
    double acc = 0.0;
    if (act && with_m2)   // (k_si_repmat on k_si_prep's record takes M2 from there)
      acc = dot_seq(Xd + li * N, Xd + lj * N, N);
    M2 = acc;
#pragma unroll
    for (int k = 0; k < RIPTRM_SI_PROF_NFIELDS; ++k) pt[k] = 0.0;
    __syncthreads();
  }

  // ---- reductions / lane reads: wave ops for one wave, workgroup ops above -------------------
  __device__ __forceinline__ double rsum(double v) {
    if constexpr (BIG) return blk.sum(v);
    else return wsum(v);
  }
  __device__ __forceinline__ double rmin(double v) {
    if constexpr (BIG) return blk.min(v);
    else return wmin(v);
  }
  __device__ __forceinline__ double rmax(double v) {
    if constexpr (BIG) return blk.max(v);
    else return wmax(v);
  }
  // value of v on thread src: call on every thread
  __device__ __forceinline__ double lread(double v, int src) {
    if constexpr (BIG) {
      bc[l] = v;
      __syncthreads();
      const double r = bc[src < NT ? src : 0];
      __syncthreads();
      return r;
    } else {
      return lane_read(v, src);
    }
  }

  // ---- d x d block primitives (one element per lane) ---------------------------------------
  __device__ __forceinline__ double tr(double a) {
    sh[l] = a;
    __syncthreads();
    const double v = act ? sh[lj * d + li] : 0.0;
    __syncthreads();
    return v;
  }
  // op(a) op(b), ta / tb transpose the operand
  __device__ __forceinline__ double mm(double a, double b, bool ta = false, bool tb = false) {
    sh[l] = a;
    sh[NT + l] = b;
    __syncthreads();
    double acc = 0.0;
    if (act) {
#pragma unroll
      for (int k = 0; k < D; ++k) {
        const double av = ta ? sh[k * d + li] : sh[li * d + k];
        const double bv = tb ? sh[NT + lj * d + k] : sh[NT + k * d + lj];
        acc = acc + av * bv;
      }
    }
    __syncthreads();
    return acc;
  }
  __device__ __forceinline__ double sym(double a) { return 0.5 * (a + tr(a)); }
  __device__ __forceinline__ double skew(double a) { return 0.5 * (a - tr(a)); }
  __device__ __forceinline__ double elem(double a, int i, int j) { return lread(a, i * d + j); }

  // stage blocks into LDS slots (slot k = ser + k*W), every lane
  __device__ __forceinline__ void stage(int slot, double a) {
    if (act) ser[slot * W + l] = a;
  }
  __device__ __forceinline__ void load_reg(int slot, double (&r)[D * D]) {
#pragma unroll
    for (int i = 0; i < D * D; ++i) r[i] = ser[slot * W + i];
  }
  // ---- big D: dense solvers on the whole workgroup, one element per thread --------------------
  // A^-1 by Gauss-Jordan with partial pivoting: inv_reg's arithmetic (first row of largest |a_rk|,
  // row swap, pivot row divided by the pivot, the other rows eliminated), one pivot per step
  __device__ __forceinline__ double par_inv(double a) {
    double o = (act && li == lj) ? 1.0 : 0.0;
    for (int k = 0; k < D; ++k) {
      if (act && lj == k) colv[li] = a;   // column k
      __syncthreads();
      int p = k;
      double best = fabs(colv[k]);
      for (int r = k + 1; r < D; ++r) {
        const double v = fabs(colv[r]);
        if (v > best) { best = v; p = r; }
      }
      const double piv = colv[p];
      const double f = (li == p) ? colv[k] : (act ? colv[li] : 0.0);   // a_rk after the swap
      if (act && li == p) { rowa[lj] = a; rowo[lj] = o; }             // the new row k
      if (act && li == k && p != k) { rowx[lj] = a; sh[lj] = o; }     // the old row k -> row p
      __syncthreads();
      if (act) {
        const double sa = rowa[lj] / piv, so = rowo[lj] / piv;
        if (li == k) {
          a = sa;
          o = so;
        } else {
          const double ar = li == p ? rowx[lj] : a, orr = li == p ? sh[lj] : o;
          a = ar - f * sa;
          o = orr - f * so;
        }
      }
      __syncthreads();
    }
    return o;
  }
  // lower Cholesky factor (this thread's element; 0 above the diagonal), right-looking in pivot
  // order: the same operations and order as chol_inv_reg / spd_dist_reg.  ok = every pivot > 0.
  __device__ __forceinline__ double par_chol(double a, bool& ok) {
    double L = 0.0;
    ok = true;
    for (int k = 0; k < D; ++k) {
      if (act && lj == k) colv[li] = a;
      __syncthreads();
      const double sk = colv[k];
      ok = ok && (sk > 0.0);
      const double ckk = sqrt(sk > 0.0 ? sk : 1.0);
      if (act) {
        if (lj == k && li >= k) L = li == k ? ckk : a / ckk;
        else if (li > k && lj > k) a = a - (colv[li] / ckk) * (colv[lj] / ckk);
      }
      __syncthreads();
    }
    return L;
  }
  // L^-1 of this lane's element of lower-triangular L, chol_inv_reg's arithmetic: Li_jj = 1 / L_jj,
  // Li_ij = (0 - sum_{k = j .. i-1} L_ik Li_kj) / L_ii (k ascending), one row of Li per step
  __device__ __forceinline__ double par_trinv(double L) {
    sh[l] = act ? L : 0.0;
    double v = 0.0;
    __syncthreads();
    for (int i = 0; i < D; ++i) {
      if (act && li == i && lj <= i) {
        if (lj == i) {
          v = 1.0 / sh[i * d + i];
        } else {
          double t = 0.0;
          for (int k = lj; k < i; ++k) t -= sh[i * d + k] * sh[NT + k * d + lj];
          v = t / sh[i * d + i];
        }
        sh[NT + i * d + lj] = v;
      }
      __syncthreads();
    }
    return v;
  }
  // pymanopt SPD dist ||logm(C^-1 B C^-T)||_F, C = cholesky(A) (spd_dist_reg on the workgroup;
  // the eigenvalues by riptrm_trs.h's parallel Jacobi); NaN if A is not PD
  __device__ __forceinline__ double par_dist(double A, double Bm) {
    bool ok;
    const double C = par_chol(A, ok);
    const double Ci = par_inv(C);
    const double T = mm(Bm, Ci, false, true);
    const double M = sym(mm(Ci, T));
    riptrm_trs::Work w = riptrm_trs::make_work(jw, D);
    if (act) w.A[li * w.lda + lj] = M;
    __syncthreads();
    riptrm_trs::jacobi<NT>(blk, w, false);
    __syncthreads();
    double s2 = 0.0;
    for (int i = 0; i < D; ++i) {
      const double lg = log(w.ev[i]);
      s2 += lg * lg;
    }
    __syncthreads();
    return ok ? sqrt(s2) : NAN;
  }

  // R^-1 and Q^-1 at once: lane 0 inverts slot 0, lane 1 slot 1 (Gauss-Jordan, partial pivoting).
  // From D = 6 on the serial form's two D x D register arrays live in scratch memory (k_si<8>: 832
  // bytes per lane), so those sizes take par_inv: the same arithmetic, one element per lane
  __device__ __forceinline__ void inv2(double r, double q, double& ri, double& qi) {
    if constexpr (BIG || D >= 6) {
      ri = par_inv(r);
      qi = par_inv(q);
      return;
    }
    stage(0, r);
    stage(1, q);
    __syncthreads();
    if (l < 2) {
      double a[D * D], o[D * D];
      load_reg(l, a);
      inv_reg<D>(a, o);
#pragma unroll
      for (int i = 0; i < D * D; ++i) ser[(2 + l) * W + i] = o[i];
    }
    __syncthreads();
    ri = act ? ser[2 * W + l] : 0.0;
    qi = act ? ser[3 * W + l] : 0.0;
    __syncthreads();
  }
  // evaluation's dense solvers, four lanes in parallel: PD(R), PD(Q), dist(Rp,R), dist(Qp,Q)
  __device__ __forceinline__ void eval_solvers(double rp, double r, double qp, double q, bool& pdr, bool& pdq, double& dR, double& dQ) {
    if constexpr (BIG) {   // PD by Cholesky (the serial path: all Jacobi eigenvalues > 0)
      (void)par_chol(r, pdr);
      (void)par_chol(q, pdq);
      dR = par_dist(rp, r);
      dQ = par_dist(qp, q);
      return;
    }
    stage(0, r);
    stage(1, q);
    stage(2, rp);
    stage(3, qp);
    __syncthreads();
    if (l < 4) {
      double a[D * D];
      double res;
      if (l < 2) {
        load_reg(l, a);
        res = pd_reg<D>(a) ? 1.0 : 0.0;
      } else {
        double bm[D * D];
        load_reg(l, a);        // previous point (Cholesky factor side)
        load_reg(l - 2, bm);   // current point
        res = spd_dist_reg<D>(a, bm);
      }
      ser[4 * W + l] = res;
    }
    __syncthreads();
    pdr = ser[4 * W + 0] != 0.0;
    pdq = ser[4 * W + 1] != 0.0;
    dR = ser[4 * W + 2];
    dQ = ser[4 * W + 3];
    __syncthreads();
  }

  // ---- manifold (pymanopt Product(SkewSymmetric, SPD, SPD)) ---------------------------------
  struct Metric {
    double XiR, XiQ;  // R^-1, Q^-1 at the base point
  };
  __device__ __forceinline__ Metric metric(PV x) {
    Metric g;
    inv2(x.r, x.q, g.XiR, g.XiQ);
    return g;
  }
  __device__ __forceinline__ double spd_inner(double Xi, double u, double v) {
    const double pu = mm(Xi, u);
    const double pv = mm(Xi, v);
    return rsum(pu * tr(pv));
  }
  __device__ __forceinline__ double inner(const Metric& g, PV u, PV v) {
    const double a = rsum(u.j * v.j);
    const double br = spd_inner(g.XiR, u.r, v.r);
    const double bq = spd_inner(g.XiQ, u.q, v.q);
    return ((0.0 + a) + br) + bq;
  }
  __device__ __forceinline__ double norm(const Metric& g, PV u) { return sqrt(inner(g, u, u)); }
  __device__ __forceinline__ PV proj(PV u) { return PV{skew(u.j), sym(u.r), sym(u.q)}; }
  // euclidean_to_riemannian_gradient: (skew(gJ), R sym(gR) R, Q sym(gQ) Q)
  __device__ __forceinline__ PV e2rg(PV x, PV g) {
    return PV{skew(g.j), mm(mm(x.r, sym(g.r)), x.r), mm(mm(x.q, sym(g.q)), x.q)};
  }
  // SPD retraction sym(X + U + U X^-1 U / 2); skew retraction X + U
  __device__ __forceinline__ PV retract(PV x, const Metric& g, PV u) {
    const double ur = mm(u.r, mm(g.XiR, u.r));
    const double uq = mm(u.q, mm(g.XiQ, u.q));
    return PV{x.j + u.j, sym((x.r + u.r) + ur / 2.0), sym((x.q + u.q) + uq / 2.0)};
  }

  // ---- problem ------------------------------------------------------------------------------
  __device__ __forceinline__ double Aof(PV x) { return mm(x.j - x.r, x.q); }
  // chain rule of phi(A(J,R,Q)) from G = dphi/dA
  __device__ __forceinline__ PV chain(PV x, double G) {
    const double gq = mm(G, x.q, false, true);
    return PV{gq, -gq, mm(x.j - x.r, G, true, false)};
  }
  // constraint value g_k(x) on constraint lanes from A (this lane's element)
  __device__ __forceinline__ double cons_val(double A) {
    const double a = lread(A, cr * d + cc);
    if (!cact) return 0.0;
    return ck == 0 ? (-a + cp0) : (ck == 1 ? (a - cp0) : (-((a - cp0) * (a - cp0)) + cp1));
  }
  __device__ __forceinline__ double cons_w(double A) {
    const double a = lread(A, cr * d + cc);
    if (!cact) return 0.0;
    return ck == 0 ? -1.0 : (ck == 1 ? 1.0 : -2.0 * (a - cp0));
  }
  // element lane (i,j) <- sum over constraints k with (r_k, c_k) = (i, j) of v_k, k ascending
  __device__ __forceinline__ double scatter(double v) {
    sh[l] = cact ? v : 0.0;
    __syncthreads();
    double acc = 0.0;
    if (act)
      for (int k = 0; k < m; ++k)
        if (cr_s[k] == li && cc_s[k] == lj) acc = acc + sh[k];
    __syncthreads();
    return act ? acc : 0.0;
  }
  // f(x) and G_f = df/dA = -(2h/N) E X^T (E kept in the instance's scratch)
  __device__ __forceinline__ void cost_grad(double A, double& f, double& Gf) {
    const double At = ((li == lj) ? 1.0 : 0.0) + P.h * A;
    sh[l] = act ? At : 0.0;
    __syncthreads();
    double part = 0.0;
    const int tot = d * N;
    int e = l;
    // two residual entries per step: both entries' data loads issued before either's sums (the same
    // sums in the same order as one at a time)
    for (; e + NT < tot; e += 2 * NT) {
      const int e2 = e + NT;
      const int i = e / N, t = e - i * N, i2 = e2 / N, t2 = e2 - i2 * N;
      double xa[D], xb[D];
#pragma unroll
      for (int k = 0; k < D; ++k) {
        xa[k] = Xd[k * N + t];
        xb[k] = Xd[k * N + t2];
      }
      const double pa = XPd[i * N + t], pb = XPd[i2 * N + t2];
      double s = 0.0, s2 = 0.0;
#pragma unroll
      for (int k = 0; k < D; ++k) {
        s = s + sh[i * d + k] * xa[k];
        s2 = s2 + sh[i2 * d + k] * xb[k];
      }
      const double ev = pa - s, ev2 = pb - s2;
      E[e] = ev;
      E[e2] = ev2;
      part = part + ev * ev;
      part = part + ev2 * ev2;
    }
    for (; e < tot; e += NT) {
      const int i = e / N, t = e - i * N;
      double s = 0.0;
      for (int k = 0; k < d; ++k) s = s + sh[i * d + k] * Xd[k * N + t];
      const double ev = XPd[i * N + t] - s;
      E[e] = ev;
      part = part + ev * ev;
    }
    __syncthreads();
    f = rsum(part) / (double)N;
    double g = 0.0;
    if (act) g = dot_seq(E + li * N, Xd + lj * N, N);
    Gf = act ? -(2.0 * P.h / (double)N) * g : 0.0;
    __syncthreads();
  }

  // everything HwCur / cxCur need at (x, y, mu): RIPTRM.py:720-730
  struct AtX {
    PV x;
    Metric g;
    double A, Gf, GL, sgR, sgQ, f;
    double s, w, y;  // constraint lanes
    PV c;            // cxCur
  };
  __device__ __forceinline__ void prepare(AtX& a, PV x, double y, double mu) {
    a.x = x;
    a.y = y;
    a.g = metric(x);
    a.A = Aof(x);
    cost_grad(a.A, a.f, a.Gf);
    const double g0 = cons_val(a.A);   // wave op: evaluate on every lane, then select
    a.s = cact ? -g0 : 1.0;
    a.w = cons_w(a.A);
    a.GL = a.Gf + scatter(y * a.w);
    const PV cg = chain(x, a.GL);
    a.sgR = sym(cg.r);
    a.sgQ = sym(cg.q);
    // c = rgrad f - Gx(mu / s);  Gx(v) = e2rg(chain(scatter(-(v w))))
    const PV rgf = e2rg(x, chain(x, a.Gf));
    const double q = cact ? (mu / a.s) : 0.0;
    const PV gx = e2rg(x, chain(x, scatter(-(q * a.w))));
    a.c = pv_sub(rgf, gx);
  }
  __device__ __forceinline__ double dAof(const AtX& a, PV v) {
    return mm(v.j - v.r, a.x.q) + mm(a.x.j - a.x.r, v.q);
  }
  // Gxaj(v) on constraint lanes from dA(v)
  __device__ __forceinline__ double gxaj(const AtX& a, double dA) {
    const double da = lread(dA, cr * d + cc);
    return cact ? -(a.w * da) : 0.0;
  }
  // HwCur(v) = HessL[v] + Gx(y Gxaj(v) / s)
  __device__ __forceinline__ PV hw(const AtX& a, PV v) {
    const PV x = a.x;
    const double dA = dAof(a, v);
    double dG = (2.0 * P.h * P.h / (double)N) * mm(dA, M2);
    {  // two-box second derivatives, constraint order
      const double da = lread(dA, cr * d + cc);
      const double t = (cact && ck == 2) ? a.y * (-2.0 * da) : 0.0;
      sh[l] = t;
      __syncthreads();
      double acc = dG;
      if (act)
        for (int k = 0; k < m; ++k)
          if (cr_s[k] == li && cc_s[k] == lj) acc = acc + sh[k];
      __syncthreads();
      dG = act ? acc : 0.0;
    }
    // chain_hess(x, G_L, dG, v)
    const double t = mm(dG, x.q, false, true) + mm(a.GL, v.q, false, true);
    const PV h{t, -t, mm(v.j - v.r, a.GL, true, false) + mm(x.j - x.r, dG, true, false)};
    // e2rh: (skew(hJ), R sym(hR) R + sym(vR sym(gR) R), Q sym(hQ) Q + sym(vQ sym(gQ) Q))
    const double hr = mm(mm(x.r, sym(h.r)), x.r) + sym(mm(mm(v.r, a.sgR), x.r));
    const double hq = mm(mm(x.q, sym(h.q)), x.q) + sym(mm(mm(v.q, a.sgQ), x.q));
    const PV hl{skew(h.j), hr, hq};
    const double gj = gxaj(a, dA);     // wave op outside the lane select
    const double q = cact ? (a.y * gj) / a.s : 0.0;
    const PV gx = e2rg(x, chain(x, scatter(-(q * a.w))));
    return pv_add(hl, gx);
  }
  // gradLagrangefun (RIPTRM.py:475-489) and its norm at (x, y)
  __device__ __forceinline__ double gradlag_norm(PV x, double y, double& f_out, double& A_out) {
    const Metric g = metric(x);
    const double A = Aof(x);
    double f, Gf;
    cost_grad(A, f, Gf);
    const double w = cons_w(A);
    const double G = Gf + scatter(y * w);
    const PV gl = e2rg(x, chain(x, G));
    f_out = f;
    A_out = A;
    return norm(g, gl);
  }

  // ---- tCG, RIPTRM.py:41-216 (eta0 = 0, identity preconditioner) ----------------------------
  __device__ __forceinline__ int tcg(const AtX& a, double Delta, PV& eta, PV& Heta, int& jout, double& hvps) {
    const double theta = P.opt.tcg_theta, kappa = P.opt.tcg_kappa;
    const int mininner = P.opt.tcg_mininner;
    const int maxinner = P.d * (P.d - 1) / 2 + P.d * (P.d + 1);  // manifold.dim
    eta = PV{0.0, 0.0, 0.0};
    Heta = PV{0.0, 0.0, 0.0};
    PV r = a.c;
    double e_Pe = 0.0;
    double r_r = inner(a.g, r, r);
    double norm_r = sqrt(r_r);
    const double norm_r0 = norm_r;
    PV z = r;
    double z_r = inner(a.g, z, r);
    double d_Pd = z_r;
    PV delta = pv_neg(z);
    double e_Pd = 0.0;
    double model = 0.0;
    int stop = RIPTRM_TCG_MAX_INNER_ITER;
    int j = 0;
    for (j = 0; j < maxinner; ++j) {
      const double th0 = tick();
      const PV Hd = hw(a, delta);
      pt[RIPTRM_SI_PROF_HVP] += tick() - th0;
      hvps += 1.0;
      const double d_Hd = inner(a.g, delta, Hd);
      double alpha = 0.0, e_Pe_new;
      if (d_Hd != 0.0) {
        alpha = z_r / d_Hd;
        e_Pe_new = (e_Pe + 2.0 * alpha * e_Pd) + (alpha * alpha) * d_Pd;
      } else {
        e_Pe_new = e_Pe;
      }
      const double D2 = Delta * Delta;
      if (d_Hd <= 0.0 || e_Pe_new >= D2) {
        const double tau = (-e_Pd + sqrt(e_Pd * e_Pd + d_Pd * (D2 - e_Pe))) / d_Pd;
        eta = pv_add(eta, pv_scale(tau, delta));
        Heta = pv_add(Heta, pv_scale(tau, Hd));
        stop = d_Hd <= 0.0 ? RIPTRM_TCG_NEGATIVE_CURVATURE : RIPTRM_TCG_EXCEEDED_TR;
        break;
      }
      e_Pe = e_Pe_new;
      const PV ne = pv_add(eta, pv_scale(alpha, delta));
      const PV nh = pv_add(Heta, pv_scale(alpha, Hd));
      const double nm = inner(a.g, ne, a.c) + 0.5 * inner(a.g, ne, nh);
      if (nm >= model) {
        stop = RIPTRM_TCG_MODEL_INCREASED;
        break;
      }
      eta = ne;
      Heta = nh;
      model = nm;
      r = pv_add(r, pv_scale(alpha, Hd));
      r_r = inner(a.g, r, r);
      norm_r = sqrt(r_r);
      if (j >= mininner && norm_r <= norm_r0 * fmin(pow(norm_r0, theta), kappa)) {
        stop = kappa < pow(norm_r0, theta) ? RIPTRM_TCG_REACHED_TARGET_LINEAR : RIPTRM_TCG_REACHED_TARGET_SUPERLINEAR;
        break;
      }
      z = r;
      const double zold = z_r;
      z_r = r_r;   // inner(z, r) with z = r: pymanopt reuses solve(x, r) for both operands -> == r_r
      const double beta = z_r / zold;
      delta = pv_add(pv_neg(z), pv_scale(beta, delta));
      delta = proj(delta);
      e_Pd = beta * (e_Pd + alpha * d_Pd);
      d_Pd = z_r + (beta * beta) * d_Pd;
    }
    if (j >= maxinner) j = maxinner - 1;  // Python's range loop variable after exhaustion
    jout = j;
    return stop;
  }

  // ---- Exact_RepMat, RIPTRM.py:433-444 (+ the second-order test :599-617) ---------------------
  // Tangent basis of T_x(Skew x SPD x SPD), orthonormal in the product metric (oracle/trs_oracle.py
  // ::si_tangent_basis): skew pairs (E_ij - E_ji)/sqrt2 (i < j), then for R and Q the images
  // L B_k L^T of the Frobenius-orthonormal symmetric basis (E_ii, (E_ij + E_ji)/sqrt2, i <= j) under
  // the Cholesky factor L of the point: <L B L^T, L C L^T>_X = tr(B C).  The reference draws a random
  // basis (utils.py:388-397); the subproblem's solution does not depend on the basis.
  static constexpr int NS = D * (D - 1) / 2, NY = D * (D + 1) / 2, DIMM = NS + 2 * NY;
  static constexpr bool HBMT = si_hbm_trs(D);   // the subproblem's matrix lives in HBM (host service)
  static constexpr int TDP = si_tdp(D);
  static constexpr double RS2 = 0.7071067811865475;   // 1 / np.sqrt(2)
  __device__ __forceinline__ static int skew_idx(int i, int j) { return i * (2 * D - i - 1) / 2 + (j - i - 1); }
  __device__ __forceinline__ static int sym_idx(int i, int j) { return i * D - i * (i - 1) / 2 + (j - i); }
  struct Frame {
    double Lr, Lq, Lri, Lqi;   // this lane's element of chol(R), chol(Q) and their inverses
  };
  __device__ __forceinline__ Frame frame(PV x) {
    if constexpr (BIG) {   // the workgroup's Cholesky / Gauss-Jordan (one element per thread)
      bool ok;
      Frame F;
      F.Lr = par_chol(x.r, ok);
      F.Lq = par_chol(x.q, ok);
      F.Lri = par_inv(F.Lr);
      F.Lqi = par_inv(F.Lq);
      return F;
    } else if constexpr (D >= 6) {
      // one wave from D = 6: chol_inv_reg's arithmetic one element per lane (par_chol is its
      // Cholesky step for step; par_trinv its triangular inverse), not two lanes' scratch-resident
      // arrays.  At a non-PD point every lane's factor is NaN (above the diagonal and past the
      // block too), where chol_inv_reg's are NaN from the failing pivot on and 0 above the diagonal:
      // the same arithmetic on PD points only; either way the non-finite guard stops the instance
      bool okr, okq;
      Frame F;
      F.Lr = par_chol(x.r, okr);
      F.Lq = par_chol(x.q, okq);
      if (!okr) F.Lr = NAN;
      if (!okq) F.Lq = NAN;
      F.Lri = par_trinv(F.Lr);   // every lane (barriers inside); 0 above the diagonal and off the block
      F.Lqi = par_trinv(F.Lq);
      return F;
    }
    stage(0, x.r);
    stage(1, x.q);
    __syncthreads();
    if (l < 2) {
      double a[D * D], Lm[D * D], Li[D * D];
      load_reg(l, a);
      chol_inv_reg<D>(a, Lm, Li);
#pragma unroll
      for (int i = 0; i < D * D; ++i) {
        ser[(2 + l) * W + i] = Lm[i];
        ser[(4 + l) * W + i] = Li[i];
      }
    }
    __syncthreads();
    Frame F;
    F.Lr = act ? ser[2 * W + l] : 0.0;
    F.Lq = act ? ser[3 * W + l] : 0.0;
    F.Lri = act ? ser[4 * W + l] : 0.0;
    F.Lqi = act ? ser[5 * W + l] : 0.0;
    __syncthreads();
    return F;
  }
  // sum_k c_k b_k (c in LDS, DIMM entries)
  __device__ __forceinline__ PV from_coords(const Frame& F, const double* c) {
    double vj = 0.0, cr = 0.0, cq = 0.0;
    if (act) {
      if (li < lj) vj = c[skew_idx(li, lj)] * RS2;
      else if (li > lj) vj = -(c[skew_idx(lj, li)] * RS2);
      const int i0 = li < lj ? li : lj, j0 = li < lj ? lj : li;
      const double f = li == lj ? 1.0 : RS2;
      cr = c[NS + sym_idx(i0, j0)] * f;
      cq = c[NS + NY + sym_idx(i0, j0)] * f;
    }
    const double r = mm(mm(F.Lr, cr), F.Lr, false, true);
    const double q = mm(mm(F.Lq, cq), F.Lq, false, true);
    return PV{vj, r, q};
  }
  // out_k = <b_k, w>_x  (SPD part: <B_k, L^-1 W L^-T>_F)
  __device__ __forceinline__ void to_coords(const Frame& F, PV w, double* out) {
    const double jt = tr(w.j);
    const double wr = mm(mm(F.Lri, w.r), F.Lri, false, true);
    const double wq = mm(mm(F.Lqi, w.q), F.Lqi, false, true);
    const double wrt = tr(wr), wqt = tr(wq);
    if (act && li < lj) out[skew_idx(li, lj)] = (w.j - jt) * RS2;
    if (act && li <= lj) {
      out[NS + sym_idx(li, lj)] = li == lj ? wr : (wr + wrt) * RS2;
      out[NS + NY + sym_idx(li, lj)] = li == lj ? wq : (wq + wqt) * RS2;
    }
    __syncthreads();
  }
  // selfadj_operator2matrix (utils.py:565-573): A[i][j] = <b_i, Hw(b_j)> for i <= j, mirrored;
  // and the coordinates of cxCur (RIPTRM.py:438-440)
  __device__ __forceinline__ riptrm_trs::Work repmat(const AtX& a, const Frame& F, double& hvps) {
    riptrm_trs::Work w = riptrm_trs::make_work(tl, DIMM);
    for (int j = 0; j < DIMM; ++j) {
      for (int k = l; k < DIMM; k += NT) w.p[k] = (k == j) ? 1.0 : 0.0;
      __syncthreads();
      const PV bj = from_coords(F, (const double*)w.p);
      const PV h = hw(a, bj);
      hvps += 1.0;
      to_coords(F, h, (double*)w.q);
      for (int k = l; k <= j; k += NT) {
        w.A[k * w.lda + j] = w.q[k];
        w.A[j * w.lda + k] = w.q[k];
      }
      __syncthreads();
    }
    to_coords(F, a.c, (double*)w.a);
    return w;
  }
  // compute_direction's Exact_RepMat branch: returns the RIPTRM_TRS_* type
  __device__ __forceinline__ int trs_direction(const AtX& a, double Delta, PV& eta, double& hvps) {
    if constexpr (HBMT) {   // solve() parks instead (k_si_repmat)
      eta = PV{0.0, 0.0, 0.0};
      return RIPTRM_TRS_BOUNDARY;
    }
    const Frame F = frame(a.x);
    riptrm_trs::Work w = repmat(a, F, hvps);
    riptrm_trs::Blk<W> B(nullptr);
    const riptrm_trs::Result r = riptrm_trs::trs_solve<W>(B, w, Delta, P.opt.trs_tolhardcase);
    eta = from_coords(F, (const double*)w.x);
    return RIPTRM_TRS_BOUNDARY + r.kind;
  }
  // smallest eigenvalue of HwNew's matrix at (xN, yN, mu) (RIPTRM.py:599-613)
  __device__ __forceinline__ double mineig_at(PV xN, double yN, double mu, double& hvps) {
    if constexpr (HBMT) return 0.0;   // solve() parks instead (k_si_repmat)
    AtX aN;
    prepare(aN, xN, yN, mu);
    const Frame F = frame(xN);
    riptrm_trs::Work w = repmat(aN, F, hvps);
    riptrm_trs::Blk<W> B(nullptr);
    return riptrm_trs::min_eig<W>(B, w);
  }

  // manifold.dim > RIPTRM_TRS_DIM_MAX: selfadj_operator2matrix (utils.py:565-573) into HBM by
  // k_si_repmat, one workgroup per basis vector j: the point of the parked subproblem (park_point),
  // the frame, column j's HVP and its coordinates, written as repmat writes them (entries (k, j) and
  // (j, k) for k <= j: HVP j's coordinate k), so the matrix is the sequential loop's bit for bit.
  // With want_c, also the coordinates of cxCur (RIPTRM.py:438-440).  uv: 2 TDP doubles of LDS.
  // Each workgroup has its own residual scratch E (k_si_repmat sets it: LDS or an HBM slice).
  __device__ __forceinline__ int64_t tp_stride() const { return 3LL * dd + m + 1; }
  __device__ __forceinline__ void park_point(PV px, double py, double mu) {
    double* t = P.trsP + (int64_t)b * tp_stride();
    store_pv(t, px);
    if (cact) t[3 * dd + l] = py;
    if (l == 0) t[3 * dd + m] = mu;
  }
  // k_si_prep: prepare / frame at the park point (and X X^T) once per instance, one record per lane,
  // so the matrix's tdim workgroups load them instead of each recomputing the same values
  __device__ __forceinline__ double* prep_rec() const { return P.trsW + (int64_t)b * SI_PREP_F * NT; }
  __device__ void prep_park() {
    const double* t = P.trsP + (int64_t)b * tp_stride();
    const PV x = load_pv(t);
    const double y = cact ? t[3 * dd + l] : 0.0;
    const double mu = t[3 * dd + m];
    AtX a;
    prepare(a, x, y, mu);
    const Frame F = frame(x);
    double* r = prep_rec() + l;
    const double v[SI_PREP_F] = {a.x.j, a.x.r, a.x.q, a.g.XiR, a.g.XiQ, a.A, a.Gf, a.GL, a.sgR, a.sgQ, a.f,
                                 a.s, a.w, a.y, a.c.j, a.c.r, a.c.q, F.Lr, F.Lq, F.Lri, F.Lqi, M2};
#pragma unroll
    for (int k = 0; k < SI_PREP_F; ++k) r[(int64_t)k * NT] = v[k];
  }
  __device__ void prep_load(AtX& a, Frame& F) {
    const double* r = prep_rec() + l;
    double v[SI_PREP_F];
#pragma unroll
    for (int k = 0; k < SI_PREP_F; ++k) v[k] = r[(int64_t)k * NT];
    a.x = PV{v[0], v[1], v[2]};
    a.g.XiR = v[3], a.g.XiQ = v[4];
    a.A = v[5], a.Gf = v[6], a.GL = v[7], a.sgR = v[8], a.sgQ = v[9], a.f = v[10];
    a.s = v[11], a.w = v[12], a.y = v[13];
    a.c = PV{v[14], v[15], v[16]};
    F.Lr = v[17], F.Lq = v[18], F.Lri = v[19], F.Lqi = v[20];
    M2 = v[21];
  }
  __device__ void repmat_col(int j, bool want_c, double* uv, bool only_c = false, bool pre = false) {
    AtX a;
    Frame F;
    if (pre) {
      prep_load(a, F);
    } else {
      const double* t = P.trsP + (int64_t)b * tp_stride();
      const PV x = load_pv(t);
      const double y = cact ? t[3 * dd + l] : 0.0;
      const double mu = t[3 * dd + m];
      prepare(a, x, y, mu);
      F = frame(x);
    }
    if (only_c) {   // a cached eigendecomposition serves the matrix: the coordinates of cxCur only
      to_coords(F, a.c, P.trsa + (int64_t)b * TDP);
      return;
    }
    double* e = uv;
    double* q = uv + TDP;
    for (int k = l; k < DIMM; k += NT) e[k] = (k == j) ? 1.0 : 0.0;
    __syncthreads();
    const PV bj = from_coords(F, e);
    const PV h = hw(a, bj);
    to_coords(F, h, q);
    double* A = P.trsA + (int64_t)b * DIMM * DIMM;
    for (int k = l; k <= j; k += NT) {
      A[(int64_t)k * DIMM + j] = q[k];
      A[(int64_t)j * DIMM + k] = q[k];
    }
    if (want_c) to_coords(F, a.c, P.trsa + (int64_t)b * TDP);
  }

  // ---- resume records (HBM subproblem path) ------------------------------------------------
  __device__ __forceinline__ double* rs_base() const { return P.rs + (int64_t)b * si_rs_doubles(D); }
  __device__ __forceinline__ void rs_put(double* r, int row, double v) { r[RS_NSC + (int64_t)row * NT + l] = v; }
  __device__ __forceinline__ double rs_get(const double* r, int row) const { return r[RS_NSC + (int64_t)row * NT + l]; }
  __device__ __forceinline__ void rs_put_pv(double* r, int k, PV v) {
    rs_put(r, 3 * k, v.j);
    rs_put(r, 3 * k + 1, v.r);
    rs_put(r, 3 * k + 2, v.q);
  }
  __device__ __forceinline__ PV rs_get_pv(const double* r, int k) const {
    return PV{rs_get(r, 3 * k), rs_get(r, 3 * k + 1), rs_get(r, 3 * k + 2)};
  }

  // ---- evaluation, src/solver/utils.py:342-368 (+ compute_residual :269-340) ----------------
  // ev: cost, distance, residual, gradnorm, complvio, dualvio, manvio, maxvio, meanvio, maxabsy
  __device__ __forceinline__ void evaluation(PV xprev, PV x, double y, double (&ev)[10]) {
    double f, A;
    const double gradnorm = gradlag_norm(x, y, f, A);
    const double g = cons_val(A);
    const double cv = cact ? y * g : 0.0;
    const double sq_compl = rsum(cv * cv);
    const double nv = cact ? fmax(-y, 0.0) : 0.0;
    const double sq_nonneg = rsum(nv * nv);
    const double iv = cact ? fmax(g, 0.0) : 0.0;
    const double sq_ineq = rsum(iv * iv);
    const double maxvio = rmax(cact ? iv : 0.0);
    const double meanvio = rsum(iv) / (double)m;
    const double maxy = rmax(cact ? fabs(y) : -INFINITY);
    double manvio = 0.0;
    if (P.opt.manvio_kind == RIPTRM_MANVIO_SI) {
      const double aj = x.j + tr(x.j), ar = x.r - tr(x.r), aq = x.q - tr(x.q);
      manvio = (sqrt(rsum(aj * aj)) + sqrt(rsum(ar * ar))) + sqrt(rsum(aq * aq));
    }
    bool pr, pq;
    double dR, dQ;
    eval_solvers(xprev.r, x.r, xprev.q, x.q, pr, pq, dR, dQ);
    if (P.opt.manvio_kind == RIPTRM_MANVIO_SI && (!pr || !pq)) manvio = INFINITY;
    const double dj = x.j - xprev.j;
    const double dJ = sqrt(rsum(dj * dj));
    ev[0] = f;
    ev[1] = sqrt((dJ * dJ + dR * dR) + dQ * dQ);
    ev[2] = sqrt(((((gradnorm * gradnorm + sq_compl) + sq_nonneg) + sq_ineq) + 0.0) + manvio * manvio);
    ev[3] = gradnorm;
    ev[4] = sqrt(sq_compl);
    ev[5] = sqrt(sq_nonneg);
    ev[6] = manvio;
    ev[7] = maxvio;
    ev[8] = meanvio;
    ev[9] = maxy;
  }

  __device__ __forceinline__ double now() {
    double t = (l == 0) ? (double)wall_clock64() : -INFINITY;
    return rmax(t);
  }

  __device__ __forceinline__ void log_row(const double (&ev)[10], double outer_it, double mu, const Info* inf, double tcg_iters,
                          double t_now, double t_start, double& count, double& overflow) {
    if (l == 0) {
      const int cnt = (int)count;
      const int64_t capl = P.opt.log_capacity < P.cap ? P.opt.log_capacity : P.cap;
      if (capl > 0) {
        if (cnt >= capl) overflow += 1.0;   // a record leaves the middle of the log (head + latest kept)
        double* L = P.log + ((int64_t)b * P.cap + riptrm::log_slot(cnt, capl)) * RIPTRM_LOG_NFIELDS;
        for (int k = 0; k < RIPTRM_LOG_NFIELDS; ++k) L[k] = 0.0;
        L[RIPTRM_LOG_ITERATION] = outer_it;
        L[RIPTRM_LOG_TIME] = (cnt == 0) ? 0.0 : (t_now - t_start) / P.clock_hz;
        L[RIPTRM_LOG_COST] = ev[0];
        L[RIPTRM_LOG_DISTANCE] = ev[1];
        L[RIPTRM_LOG_RESIDUAL] = ev[2];
        L[RIPTRM_LOG_GRADNORM] = ev[3];
        L[RIPTRM_LOG_COMPLVIOLATION] = ev[4];
        L[RIPTRM_LOG_DUALVIOLATION] = ev[5];
        L[RIPTRM_LOG_MANVIOLATION] = ev[6];
        L[RIPTRM_LOG_MAXVIOLATION] = ev[7];
        L[RIPTRM_LOG_MEANVIOLATION] = ev[8];
        L[RIPTRM_LOG_MU] = mu;
        L[RIPTRM_LOG_MAXABSLAGMULT] = ev[9];
        L[RIPTRM_LOG_TCG_ITERS] = tcg_iters;
        L[RIPTRM_LOG_DUAL_CLIPPING] = -1.0;
        if (inf) {
          L[RIPTRM_LOG_HAS_INFO] = inf->has;
          L[RIPTRM_LOG_NUM_INNER] = inf->num;
          L[RIPTRM_LOG_INNER_STATUS] = inf->status;
          L[RIPTRM_LOG_TR_RADIUS] = inf->tr;
          L[RIPTRM_LOG_DXTYPE] = inf->dxtype;
          L[RIPTRM_LOG_NORMDX] = inf->normdx;
          L[RIPTRM_LOG_MINXFEASI] = inf->minx;
          L[RIPTRM_LOG_MINYFEASI] = inf->miny;
          L[RIPTRM_LOG_COMPL] = inf->compl_;
          L[RIPTRM_LOG_HAS_RATIO] = inf->hasratio;
          L[RIPTRM_LOG_ARED_PRED] = inf->ratio;
          L[RIPTRM_LOG_RADIUS_UPDATE] = inf->ru;
          L[RIPTRM_LOG_DUAL_CLIPPING] = inf->dc;
          L[RIPTRM_LOG_HAS_MINEIG] = inf->hasmin;
          L[RIPTRM_LOG_MINEIGVALHW] = inf->mineig;
        }
      } else {
        overflow += 1.0;
      }
    }
    count += 1.0;
  }

  __device__ __forceinline__ PV load_pv(const double* base) {
    if (!act) return PV{0.0, 0.0, 0.0};
    return PV{base[l], base[dd + l], base[2 * dd + l]};
  }
  __device__ __forceinline__ void store_pv(double* base, PV v) {
    if (act) {
      base[l] = v.j;
      base[dd + l] = v.r;
      base[2 * dd + l] = v.q;
    }
  }
  __device__ __forceinline__ double mu_at(int idx) const {
    const int i = idx < P.tab_len ? idx : P.tab_len - 1;
    return P.mu_tab[i];
  }

  // ---- the whole run: RIPTRM.run / outer_step / inner_run / inner_step ----------------------
  // resume = false: a new solve from P.in_x / P.in_y.  resume = true (HBM subproblem path only): an
  // instance parked at PH_TRS_HOST / PH_MINEIG_HOST continues from its resume record with the host
  // service's answer; every other instance returns at once.
  __device__ __forceinline__ void solve(bool resume) {
    const int64_t v3 = 3LL * dd;
    PV x, xI, xPrev, xHead, x0, eta_r;   // xPrev: inner_run's (RIPTRM.py:787); xHead: run's (:929, :947)
    double y, yI, y0;
    double outer_it = 0.0, mu_idx = 0.0, mu = mu_at(0), Delta = P.opt.initial_tr_radius;
    double inner_total = 0.0, tcg_total = 0.0, hvps = 0.0, log_count = 0.0, log_over = 0.0;
    double stop_code = RIPTRM_STOP_NONE, stop_rt = 0.0, residual = 0.0, last_j = 0.0, last_stop = 0.0;
    double t_start, t_tick0, Delta0 = 0.0, inner_it = 0.0, t_inner = 0.0;
    int rph = 0;       // resumed: 1 with the subproblem's solution, 2 with HwNew's smallest eigenvalue
    int tstop_r = 0;   // the direction type of a phase-2 resume
    int err = RIPTRM_ERR_NONE;   // RIPTRM_ERR_EIGEN: the host's eigensolve failed (RIPTRM.py:961-966 break)
    if (!resume) {
      x = load_pv(P.in_x + b * v3);
      y = cact ? P.in_y[(int64_t)b * m + l] : 0.0;
      xI = xPrev = xHead = x0 = x;
      yI = y0 = y;
      eta_r = PV{0.0, 0.0, 0.0};
      t_start = now();
      t_tick0 = (double)wall_clock64();
    } else {
      if constexpr (!HBMT) {
        return;
      } else {
        const double ph = P.stats[(int64_t)b * RIPTRM_STAT_NFIELDS + RIPTRM_STAT_PHASE];
        if (ph != (double)riptrm::PH_TRS_HOST && ph != (double)riptrm::PH_MINEIG_HOST) return;
        rph = ph == (double)riptrm::PH_TRS_HOST ? 1 : 2;
        const double* r = rs_base();
        outer_it = r[0], mu_idx = r[1], mu = r[2], Delta = r[3], inner_total = r[4], tcg_total = r[5];
        hvps = r[6], log_count = r[7], log_over = r[8], residual = r[9], last_j = r[10], last_stop = r[11];
        t_start = r[12], t_tick0 = r[13], inner_it = r[14], Delta0 = r[15], t_inner = r[16];
        tstop_r = (int)r[17];
        for (int k = 0; k < RIPTRM_SI_PROF_NFIELDS; ++k) pt[k] = r[RS_PT + k];
        x = rs_get_pv(r, 0), xI = rs_get_pv(r, 1), xPrev = rs_get_pv(r, 2), xHead = rs_get_pv(r, 3);
        x0 = rs_get_pv(r, 4), eta_r = rs_get_pv(r, 5);
        y = rs_get(r, 18), yI = rs_get(r, 19), y0 = rs_get(r, 20);
      }
    }
    // park at phase ph: the resume record, then the host serves the subproblem (riptrm_si_solve)
    auto park = [&](int ph, int tstop_now, PV eta_now) {
      double* r = rs_base();
      if (l == 0) {
        r[0] = outer_it, r[1] = mu_idx, r[2] = mu, r[3] = Delta, r[4] = inner_total, r[5] = tcg_total;
        r[6] = hvps, r[7] = log_count, r[8] = log_over, r[9] = residual, r[10] = last_j, r[11] = last_stop;
        r[12] = t_start, r[13] = t_tick0, r[14] = inner_it, r[15] = Delta0, r[16] = t_inner;
        r[17] = (double)tstop_now;
        for (int k = 0; k < RIPTRM_SI_PROF_NFIELDS; ++k) r[RS_PT + k] = pt[k];
        P.trsD[b] = Delta;
        double* o = P.stats + (int64_t)b * RIPTRM_STAT_NFIELDS;
        o[RIPTRM_STAT_PHASE] = (double)ph;
        o[RIPTRM_STAT_OUTER_ITERS] = outer_it;
        o[RIPTRM_STAT_LOG_COUNT] = log_count;
      }
      rs_put_pv(r, 0, x), rs_put_pv(r, 1, xI), rs_put_pv(r, 2, xPrev), rs_put_pv(r, 3, xHead);
      rs_put_pv(r, 4, x0), rs_put_pv(r, 5, eta_now);
      rs_put(r, 18, y), rs_put(r, 19, yI), rs_put(r, 20, y0);
    };
    Info info{};
    bool have_info = resume;   // a resumed instance is inside an inner iteration: info is set before use
    const bool save_inner = P.opt.save_inner_iteration != 0;
    while (true) {
      double ev[10];
      double tn = 0.0;
     if (rph == 0) {
      // outer loop head, RIPTRM.py:931-959
      evaluation(xHead, x, y, ev);
      tn = now();
      if (outer_it == 0.0 || !save_inner)
        log_row(ev, outer_it, mu, (outer_it != 0.0 && have_info) ? &info : nullptr, last_j + 1.0, tn, t_start,
                log_count, log_over);
      residual = ev[2];
      xHead = x;
      const double rt = (tn - t_start) / P.clock_hz;
      int stop = RIPTRM_STOP_NONE;
      if (rt >= P.opt.maxtime) stop = RIPTRM_STOP_MAXTIME;
      else if (outer_it >= (double)P.opt.maxiter) stop = RIPTRM_STOP_MAXITER;
      if (ev[2] <= P.opt.tolresid) stop = RIPTRM_STOP_TOLRESID;
      if (stop != RIPTRM_STOP_NONE) {
        stop_code = stop;
        stop_rt = rt;
        break;
      }
      // restart_every cycling (benchmark windows)
      const int k = P.opt.restart_every;
      if (k > 0 && outer_it > 0.0 && fmod(outer_it, (double)k) == 0.0) {
        x = xI;
        y = yI;
        xPrev = x;
        mu_idx = 0.0;
        mu = mu_at(0);
        Delta = P.opt.initial_tr_radius;
      }
      outer_it += 1.0;
      x0 = x;
      y0 = y;
      Delta0 = Delta;
      xPrev = x;
      inner_it = 0.0;
      t_inner = now();
     }
      const int ti = (int)mu_idx < P.tab_len ? (int)mu_idx : P.tab_len - 1;
      const double tolL = P.tolL_tab[ti], tolC = P.tolC_tab[ti];
      while (true) {  // inner_run, RIPTRM.py:785-847
        if (rph == 0) inner_it += 1.0;
        const double DeltaStep = Delta;   // a parked instance resumes with Delta unchanged
        double tq = tick();
        AtX a;
        prepare(a, x, y, mu);
        pt[RIPTRM_SI_PROF_PREPARE] += tick() - tq;
        tq = tick();
        PV eta, Heta;
        int jj = 0;
        const bool exact = P.opt.trs_solver == RIPTRM_TRS_SOLVER_EXACT_REPMAT;
        int tstop;
        if constexpr (HBMT) {
          if (exact && rph == 0) {   // park; the host builds the matrix (k_si_repmat) and solves TRSgep
            park_point(x, y, mu);
            hvps += (double)DIMM;
            park((int)riptrm::PH_TRS_HOST, 0, PV{0.0, 0.0, 0.0});
            return;
          }
          if (exact && rph == 1 && P.trskind[b] == RIPTRM_TCG_EIGFAIL) {
            err = RIPTRM_ERR_EIGEN;   // scipy.linalg.eig raised inside outer_step
            break;
          }
          if (exact && rph == 1) {
            const Frame F = frame(a.x);
            eta = from_coords(F, P.trsx + (int64_t)b * TDP);
            tstop = P.trskind[b];
          } else if (exact) {
            eta = eta_r;
            tstop = tstop_r;
          } else {
            tstop = tcg(a, Delta, eta, Heta, jj, hvps);
          }
        } else {
          tstop = exact ? trs_direction(a, Delta, eta, hvps) : tcg(a, Delta, eta, Heta, jj, hvps);
        }
        if (exact) jj = -1;   // no tCG iterations
        pt[RIPTRM_SI_PROF_TCG] += tick() - tq;
        tq = tick();
        tcg_total += (double)jj + 1.0;
        last_j = jj;
        last_stop = tstop;
        const double normdx = norm(a.g, eta);
        const double dA = dAof(a, eta);
        const double gj = gxaj(a, dA);
        const double dy = cact ? ((-y + mu * (1.0 / a.s)) - (y * gj) / a.s) : 0.0;
        const PV xN = retract(x, a.g, eta);
        const double yN = cact ? y + dy : 0.0;
        const double AN = Aof(xN);
        const double gN = cons_val(AN);
        const double sN = cact ? -gN : 1.0;
        const double minx = rmin(cact ? sN : INFINITY);
        const double miny = rmin(cact ? yN : INFINITY);
        const bool xfeas = minx > 0.0 && rmin(cact ? (sN > 0.0 ? 1.0 : 0.0) : 1.0) > 0.0;
        const bool yfeas = rmin(cact ? (yN > 0.0 ? 1.0 : 0.0) : 1.0) > 0.0;
        const double cvv = cact ? yN * sN - mu : 0.0;
        const double compl_ = sqrt(rsum(cvv * cvv));
        info = Info{1.0, inner_it, 0.0, DeltaStep, (double)tstop, normdx, minx, miny, compl_, 0.0, 0.0, 0.0, -1.0,
                    0.0, 0.0};
        have_info = true;
        bool mineig_ok = true;
        if (exact && P.opt.second_order_stationarity) {   // RIPTRM.py:599-613
          double me;
          if constexpr (HBMT) {
            if (rph != 2) {   // park; the host builds HwNew's matrix and computes its eigenvalues
              park_point(xN, yN, mu);
              hvps += (double)DIMM;
              park((int)riptrm::PH_MINEIG_HOST, tstop, eta);
              return;
            }
            me = P.trsmin[b];
            if (!isfinite(me)) {   // the eigensolve failed (scipy raises inside outer_step)
              err = RIPTRM_ERR_EIGEN;
              break;
            }
          } else {
            me = mineig_at(xN, yN, mu, hvps);
          }
          const double tol2 = P.opt.tol2_table ? P.opt.tol2_table[ti] : mu;
          mineig_ok = me >= -tol2;
          info.hasmin = 1.0;
          info.mineig = me;
        }
        rph = 0;
        bool converged = false;
        double fN = 0.0, AN2 = 0.0;
        if (xfeas) {
          const double normgl = gradlag_norm(xN, yN, fN, AN2);
          converged = yfeas && normgl <= tolL && compl_ <= tolC && mineig_ok;
        }
        if (converged) {  // RIPTRM.py:762-766
          x = xN;
          y = yN;
          info.status = RIPTRM_IS_CONVERGED;
        } else if (!xfeas) {  // RIPTRM.py:769-775
          info.status = RIPTRM_IS_PRIMAL_INFEASIBLE;
          Delta = P.opt.gamma * normdx;
        } else {  // update_xy_TR_radius, RIPTRM.py:631-705
          const double ls = rsum(cact ? log(a.s) : 0.0);
          const double lsN = rsum(cact ? log(sN) : 0.0);
          const double lb_c = a.f - mu * ls;
          const double lb_n = fN - mu * lsN;
          double ared = lb_c - lb_n;
          const PV Hdx = hw(a, eta);
          hvps += 1.0;
          double pred = (0.0 - 0.5 * inner(a.g, Hdx, eta)) - inner(a.g, a.c, eta);
          const double red_reg = fmax(1.0, fabs(lb_c)) * 2.220446049250313e-16 * P.opt.reduction_regularization;
          ared = ared + red_reg;
          pred = pred + red_reg;
          const double ratio = ared / pred;
          double Dn;
          int ru;
          if (ared < 0.25 * pred) {
            ru = RIPTRM_RU_REDUCED;
            Dn = 0.25 * Delta;
          } else if (ared >= 0.75 * pred && fabs(normdx - Delta) <= 1e-15) {
            ru = RIPTRM_RU_EXPANDED;
            const double d2 = 2.0 * Delta;
            Dn = d2 < P.opt.maximal_tr_radius ? d2 : P.opt.maximal_tr_radius;
          } else {
            ru = RIPTRM_RU_UNCHANGED;
            Dn = Delta;
          }
          info.hasratio = 1.0;
          info.ratio = ratio;
          info.ru = ru;
          if (ared > P.opt.rho * pred) {
            const double cl = P.opt.const_left, crr = P.opt.const_right;
            const double iright = np_max(crr, crr / mu);   // RIPTRM.py:682 (3-arg np.maximum quirk)
            double yc = 0.0;
            if (cact) {
              const double il = cl * np_min(np_min(y, mu / sN), 1.0);
              yc = np_min(np_max(yN, il), iright);
            }
            const double nd = rsum((cact && yc != yN) ? 1.0 : 0.0);
            x = xN;
            y = yc;
            info.status = RIPTRM_IS_SUCCESSFUL;
            info.dc = nd > 0.0 ? 1.0 : 0.0;
          } else {
            info.status = RIPTRM_IS_UNSUCCESSFUL;
          }
          Delta = Dn;
        }
        // inner_run tail, RIPTRM.py:810-847
        pt[RIPTRM_SI_PROF_TRIAL] += tick() - tq;
        tq = tick();
        inner_total += 1.0;
        tn = now();
        if (save_inner) {
          evaluation(xPrev, x, y, ev);
          log_row(ev, outer_it, mu, &info, last_j + 1.0, tn, t_start, log_count, log_over);
        }
        pt[RIPTRM_SI_PROF_EVAL] += tick() - tq;
        xPrev = x;
        bool exitflag = converged;
        double rti, lim;
        if (P.opt.inner_maxtime < 0.0) {
          lim = P.opt.maxtime;
          rti = (tn - t_start) / P.clock_hz;
        } else {
          lim = P.opt.inner_maxtime;
          rti = (tn - t_inner) / P.clock_hz;
        }
        const bool tmo = rti >= lim;
        const bool imax = P.opt.inner_maxiter >= 0 && inner_it >= (double)P.opt.inner_maxiter;
        if (tmo || imax) {
          info.status = imax ? RIPTRM_IS_MAX_ITER_EXCEEDED : RIPTRM_IS_MAX_TIME_EXCEEDED;
          exitflag = true;
          x = x0;
          y = y0;
          xPrev = x0;
          Delta = Delta0;
        }
        if (exitflag) break;
      }
      if (err != RIPTRM_ERR_NONE) {   // the reference's do_exit_on_error break: the outer step's start
        x = x0;
        y = y0;
        stop_rt = (now() - t_start) / P.clock_hz;
        break;
      }
      // outer_step tail, RIPTRM.py:889-896
      mu_idx += 1.0;
      mu = mu_at((int)mu_idx);
      const double mn = P.opt.minimal_initial_tr_radius;
      Delta = Delta > mn ? Delta : mn;
    }
    store_pv(P.x + b * v3, x);
    if (cact) P.y[(int64_t)b * m + l] = y;
    if (l == 0) {
      double* o = P.stats + (int64_t)b * RIPTRM_STAT_NFIELDS;
      for (int k = 0; k < RIPTRM_STAT_NFIELDS; ++k) o[k] = 0.0;
      o[RIPTRM_STAT_OUTER_ITERS] = outer_it;
      o[RIPTRM_STAT_INNER_ITERS] = inner_total;
      o[RIPTRM_STAT_TCG_ITERS] = tcg_total;
      o[RIPTRM_STAT_PASSES] = hvps;
      o[RIPTRM_STAT_STOP_CODE] = stop_code;
      o[RIPTRM_STAT_STOP_RUNTIME] = stop_rt;
      o[RIPTRM_STAT_FINAL_RESIDUAL] = residual;
      o[RIPTRM_STAT_LOG_COUNT] = log_count;
      o[RIPTRM_STAT_LOG_OVERFLOW] = log_over;
      o[RIPTRM_STAT_PHASE] = err != RIPTRM_ERR_NONE ? riptrm::PH_ERROR : riptrm::PH_DONE;
      o[RIPTRM_STAT_ERROR] = err;
      o[RIPTRM_STAT_MU] = mu;
      o[RIPTRM_STAT_TR_RADIUS] = Delta;
      o[RIPTRM_STAT_TCG_LAST_J] = last_j;
      o[RIPTRM_STAT_TCG_LAST_STOP] = last_stop;
      if (P.prof) {
        pt[RIPTRM_SI_PROF_TOTAL] = (double)wall_clock64() - t_tick0;
        for (int k = 0; k < RIPTRM_SI_PROF_NFIELDS; ++k) P.prof[(int64_t)b * RIPTRM_SI_PROF_NFIELDS + k] = pt[k];
      }
    }
  }

  __device__ __forceinline__ void op_hvp() {
    const int64_t v3 = 3LL * dd;
    const PV x = load_pv(P.in_x + b * v3);
    const double y = cact ? P.in_y[(int64_t)b * m + l] : 0.0;
    AtX a;
    prepare(a, x, y, P.in_mu[b]);
    const PV v = load_pv(P.in_v + b * v3);
    const PV h = hw(a, v);
    store_pv(P.out_v + b * v3, h);
  }

  __device__ __forceinline__ void op_tcg() {
    const int64_t v3 = 3LL * dd;
    const PV x = load_pv(P.in_x + b * v3);
    const double y = cact ? P.in_y[(int64_t)b * m + l] : 0.0;
    AtX a;
    prepare(a, x, y, P.in_mu[b]);
    PV eta, Heta;
    int j = 0;
    double hv = 0.0;
    const int stop = tcg(a, P.in_delta[b], eta, Heta, j, hv);
    store_pv(P.eta + b * v3, eta);
    store_pv(P.heta + b * v3, Heta);
    if (l == 0) {
      double* o = P.stats + (int64_t)b * RIPTRM_STAT_NFIELDS;
      o[RIPTRM_STAT_TCG_LAST_J] = j;
      o[RIPTRM_STAT_TCG_LAST_STOP] = stop;
      o[RIPTRM_STAT_PASSES] = hv;
    }
  }
};

template <int D>
__global__ void __launch_bounds__(si_threads(D)) k_si(SIParams P) {
  constexpr int NT = si_threads(D);
  __shared__ double sh[2 * NT];
  __shared__ double ser[NT == W ? 8 * W : 1];   // the one-wave serial solvers' slots
  __shared__ int crs[NT], ccs[NT];
  extern __shared__ double trs_lds[];   // one wave: Exact_RepMat only (size 0 otherwise); big D: si_big_lds_doubles
  const int b = blockIdx.x;
  if (b >= P.batch) return;
  Eng<D> e(P, b, sh, ser, crs, ccs, trs_lds);
  if (P.mode == MODE_SOLVE || P.mode == MODE_RESUME) e.solve(P.mode == MODE_RESUME);
  else if (P.mode == MODE_HVP) e.op_hvp();
  else e.op_tcg();
}

// the parked instances' prepare / frame / X X^T records (ids[blockIdx.y]): Eng::prep_park (its E is
// the first column workgroup's slice, free until k_si_repmat runs)
template <int D>
__global__ void __launch_bounds__(si_threads(D)) k_si_prep(SIParams P, int32_t ids_off) {
  constexpr int NT = si_threads(D);
  __shared__ double sh[2 * NT];
  __shared__ double ser[NT == W ? 8 * W : 1];
  __shared__ int crs[NT], ccs[NT];
  extern __shared__ double trs_lds[];
  const int b = P.trsids[ids_off + blockIdx.y];
  Eng<D> e(P, b, sh, ser, crs, ccs, trs_lds);
  const int64_t en = (int64_t)D * P.N;
  e.E = P.trsE ? P.trsE + (int64_t)b * si_manifold_dim(D) * en : trs_lds + (D > 8 ? si_big_lds_doubles(D) : 0);
  if constexpr (si_hbm_trs(D)) e.prep_park();
}

// the parked instances' subproblem matrices (ids[blockIdx.y], basis vector blockIdx.x): Eng::repmat_col;
// pre: on k_si_prep's records
template <int D>
__global__ void __launch_bounds__(si_threads(D)) k_si_repmat(SIParams P, int32_t ids_off, int want_c, int only_c, int pre) {
  constexpr int NT = si_threads(D);
  __shared__ double sh[2 * NT];
  __shared__ double ser[NT == W ? 8 * W : 1];
  __shared__ int crs[NT], ccs[NT];
  __shared__ double uv[2 * si_tdp(D)];
  extern __shared__ double trs_lds[];   // big D: si_big_lds_doubles; then E when it fits (si_repmat_e_lds)
  const int b = P.trsids[ids_off + blockIdx.y];
  Eng<D> e(P, b, sh, ser, crs, ccs, trs_lds, pre == 0);
  const int64_t en = (int64_t)D * P.N;
  e.E = P.trsE ? P.trsE + ((int64_t)b * si_manifold_dim(D) + blockIdx.x) * en
               : trs_lds + (D > 8 ? si_big_lds_doubles(D) : 0);
  if constexpr (si_hbm_trs(D)) e.repmat_col((int)blockIdx.x, want_c != 0 && blockIdx.x == 0, uv, only_c != 0, pre != 0);
}

struct Bound {
  riptrm_si_problem prob;
  int batch = 0, cap = 0;
  Layout L{};
  char* ws = nullptr;
  double* prof = nullptr;   // device, batch x RIPTRM_SI_PROF_NFIELDS (riptrm_si_profile_enable)
  bool prof_on = false;
};

}  // namespace riptrm_si

using namespace riptrm_si;

void riptrm_si_release(riptrm_si::Bound* s) {
  if (s && s->prof) (void)hipFree(s->prof);
  delete s;
}

static bool si_dims_ok(int32_t d, int32_t N, int32_t m, int32_t batch, int32_t cap) {
  return d >= 1 && d <= DMAX && N >= 1 && m >= 1 && m <= MMAX && m <= si_threads(d) && batch >= 1 && cap >= 0;
}

static SIParams si_params(riptrm_ctx* c, int mode) {
  Bound* s = c->si;
  SIParams P;
  std::memset(&P, 0, sizeof(P));
  P.d = s->prob.d;
  P.N = s->prob.N;
  P.m = s->prob.m;
  P.batch = s->batch;
  P.cap = s->cap;
  P.mode = mode;
  P.h = s->prob.h;
  P.clock_hz = c->clock_hz;
  P.X = s->prob.X;
  P.XP = s->prob.XP;
  P.data_stride = s->prob.data_stride;
  P.cons = s->prob.cons;
  P.cons_stride = s->prob.cons_stride;
  P.x = (double*)(s->ws + s->L.off_x);
  P.y = (double*)(s->ws + s->L.off_y);
  P.eta = (double*)(s->ws + s->L.off_eta);
  P.heta = (double*)(s->ws + s->L.off_heta);
  P.escr = (double*)(s->ws + s->L.off_escr);
  P.stats = (double*)(s->ws + s->L.off_stats);
  P.log = (double*)(s->ws + s->L.off_log);
  P.prof = s->prof_on ? s->prof : nullptr;
  if (si_hbm_trs(P.d)) {
    P.trsA = (double*)(s->ws + s->L.off_tA);
    P.trsP = (double*)(s->ws + s->L.off_tP);
    P.trsids = (int32_t*)(s->ws + s->L.off_tids);
    P.trsE = s->L.off_tE ? (double*)(s->ws + s->L.off_tE) : nullptr;
    P.trsa = (double*)(s->ws + s->L.off_ta);
    P.trsx = (double*)(s->ws + s->L.off_tx);
    P.trsD = (double*)(s->ws + s->L.off_tD);
    P.trslam = (double*)(s->ws + s->L.off_tlam);
    P.trskind = (int32_t*)(s->ws + s->L.off_tkind);
    P.trsmin = (double*)(s->ws + s->L.off_tmin);
    P.rs = (double*)(s->ws + s->L.off_rs);
    P.trsW = (double*)(s->ws + s->L.off_tW);
    P.trsC = s->L.off_tC ? (double*)(s->ws + s->L.off_tC) : nullptr;
    P.trsC_stride = s->L.tC_stride;
    P.tdim = si_manifold_dim(P.d);
    P.tdp = si_tdp(P.d);
  }
  P.opt.struct_size = (int32_t)sizeof(riptrm_options);
  P.opt.tcg_theta = 1.0;   // RIPTRM.py:330-332 defaults for the operator entry points
  P.opt.tcg_kappa = 0.1;
  P.opt.tcg_mininner = 1;
  return P;
}

template <int D>
static int si_launch_d(riptrm_ctx* c, const SIParams& P) {
  const bool exact = (P.mode == MODE_SOLVE || P.mode == MODE_RESUME) && P.opt.trs_solver == RIPTRM_TRS_SOLVER_EXACT_REPMAT;
  const size_t shm = D > 8 ? (size_t)si_big_lds_doubles(D) * sizeof(double)
                     : (exact && !si_hbm_trs(D)) ? (size_t)riptrm_trs::work_doubles(si_manifold_dim(D)) * sizeof(double)
                                                 : 0;
  if (shm > 64 * 1024)
    HIPCHK(c, hipFuncSetAttribute((const void*)k_si<D>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
  hipLaunchKernelGGL(k_si<D>, dim3((unsigned)P.batch), dim3(si_threads(D)), shm, c->stream, P);
  HIPCHK(c, hipGetLastError());
  return RIPTRM_OK;
}

static int si_launch(riptrm_ctx* c, const SIParams& P) {
  switch (P.d) {  // the block size is a template parameter: unrolled products, register solvers
    case 1: return si_launch_d<1>(c, P);
    case 2: return si_launch_d<2>(c, P);
    case 3: return si_launch_d<3>(c, P);
    case 4: return si_launch_d<4>(c, P);
    case 5: return si_launch_d<5>(c, P);
    case 6: return si_launch_d<6>(c, P);
    case 7: return si_launch_d<7>(c, P);
    case 8: return si_launch_d<8>(c, P);
    case 9: return si_launch_d<9>(c, P);
    case 10: return si_launch_d<10>(c, P);
    case 11: return si_launch_d<11>(c, P);
    case 12: return si_launch_d<12>(c, P);
    case 13: return si_launch_d<13>(c, P);
    case 14: return si_launch_d<14>(c, P);
    case 15: return si_launch_d<15>(c, P);
    default: return si_launch_d<16>(c, P);
  }
}

template <int D>
static int si_repmat_d(riptrm_ctx* c, const SIParams& P, int ids_off, int cnt, int want_c, int only_c) {
  const size_t shm = ((D > 8 ? (size_t)si_big_lds_doubles(D) : 0) + (P.trsE ? 0 : (size_t)D * P.N)) * sizeof(double);
  if (shm > 64 * 1024)
    HIPCHK(c, hipFuncSetAttribute((const void*)k_si_repmat<D>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
  // prepare / frame once per instance (k_si_prep), then the tdim column workgroups on its records;
  // RIPTRM_SI_PREP=0: every workgroup recomputes them (A/B; the same values)
  const char* pe = getenv("RIPTRM_SI_PREP");
  const int pre = (pe && pe[0] == '0') ? 0 : 1;
  if (pre) {
    if (shm > 64 * 1024)
      HIPCHK(c, hipFuncSetAttribute((const void*)k_si_prep<D>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
    hipLaunchKernelGGL(k_si_prep<D>, dim3(1u, (unsigned)cnt), dim3(si_threads(D)), shm, c->stream, P, ids_off);
  }
  hipLaunchKernelGGL(k_si_repmat<D>, dim3(only_c ? 1u : (unsigned)si_manifold_dim(D), (unsigned)cnt), dim3(si_threads(D)), shm,
                     c->stream, P, ids_off, want_c, only_c, pre);
  HIPCHK(c, hipGetLastError());
  return RIPTRM_OK;
}

// the subproblem matrices of the parked instances ids (HBM path: d >= 8), one workgroup per entry of
// the tangent basis
// (only_c: just the coordinates of cxCur, for subproblems a cached eigendecomposition serves)
static int si_repmat(riptrm_ctx* c, const SIParams& P, const std::vector<int32_t>& ids, int ids_off, int want_c,
                     int only_c = 0) {
  if (ids.empty()) return RIPTRM_OK;
  HIPCHK(c, hipMemcpyAsync(P.trsids + ids_off, ids.data(), ids.size() * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
  const int cnt = (int)ids.size();
  int rc;
  switch (P.d) {
    case 8: rc = si_repmat_d<8>(c, P, ids_off, cnt, want_c, only_c); break;
    case 9: rc = si_repmat_d<9>(c, P, ids_off, cnt, want_c, only_c); break;
    case 10: rc = si_repmat_d<10>(c, P, ids_off, cnt, want_c, only_c); break;
    case 11: rc = si_repmat_d<11>(c, P, ids_off, cnt, want_c, only_c); break;
    case 12: rc = si_repmat_d<12>(c, P, ids_off, cnt, want_c, only_c); break;
    case 13: rc = si_repmat_d<13>(c, P, ids_off, cnt, want_c, only_c); break;
    case 14: rc = si_repmat_d<14>(c, P, ids_off, cnt, want_c, only_c); break;
    case 15: rc = si_repmat_d<15>(c, P, ids_off, cnt, want_c, only_c); break;
    default: rc = si_repmat_d<16>(c, P, ids_off, cnt, want_c, only_c); break;
  }
  if (rc) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));   // ids (host memory) may go after the copy has run
  return RIPTRM_OK;
}

extern "C" {

int64_t riptrm_si_workspace_bytes(int32_t d, int32_t N, int32_t m, int32_t batch, int32_t cap) {
  if (!si_dims_ok(d, N, m, batch, cap)) return -1;
  return make_layout(d, N, m, batch, cap).total;
}

int64_t riptrm_si_workspace_offset(int32_t d, int32_t N, int32_t m, int32_t batch, int32_t cap, int32_t kind) {
  if (!si_dims_ok(d, N, m, batch, cap)) return -1;
  const riptrm_si::Layout L = make_layout(d, N, m, batch, cap);
  switch (kind) {
    case 0: return L.off_x;
    case 1: return L.off_y;
    case 2: return L.off_eta;
    case 3: return L.off_heta;
    case 4: return L.off_stats;
    case 5: return L.off_log;
    default: return -1;
  }
}

int riptrm_si_bind(riptrm_ctx* ctx, const riptrm_si_problem* prob, int32_t batch, void* ws, int64_t ws_bytes,
                   int32_t cap) {
  if (!ctx) return RIPTRM_E_ARG;
  if (!prob || prob->struct_size != (int32_t)sizeof(riptrm_si_problem))
    return fail(ctx, RIPTRM_E_ARG, "si_bind: riptrm_si_problem.struct_size mismatch");
  if (!si_dims_ok(prob->d, prob->N, prob->m, batch, cap))
    return fail(ctx, RIPTRM_E_ARG, "si_bind: need 1 <= d <= RIPTRM_SI_DMAX, N >= 1, 1 <= m <= 64 (d <= 8) or "
                                   "m <= 64 ceil(d^2 / 64) (d > 8), batch >= 1");
  if (!prob->X || !prob->XP || !prob->cons || !ws || prob->data_stride < 0 || prob->cons_stride < 0)
    return fail(ctx, RIPTRM_E_ARG, "si_bind: bad argument");
  if (prob->data_stride != 0 && prob->data_stride < (int64_t)prob->d * prob->N)
    return fail(ctx, RIPTRM_E_ARG, "si_bind: data_stride smaller than d*N");
  if (prob->cons_stride != 0 && prob->cons_stride < (int64_t)prob->m * RIPTRM_SI_CONS_FIELDS)
    return fail(ctx, RIPTRM_E_ARG, "si_bind: cons_stride smaller than m*RIPTRM_SI_CONS_FIELDS");
  if (((uintptr_t)ws % 256) != 0) return fail(ctx, RIPTRM_E_ARG, "si_bind: workspace must be 256-byte aligned");
  const riptrm_si::Layout L = make_layout(prob->d, prob->N, prob->m, batch, cap);
  if (ws_bytes < L.total) return fail(ctx, RIPTRM_E_ARG, "si_bind: workspace too small");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  HIPCHK(ctx, hipMemsetAsync(ws, 0, (size_t)L.total, ctx->stream));
  if (!ctx->si) ctx->si = new Bound();
  if (ctx->si->prof && ctx->si->batch != batch) {
    (void)hipFree(ctx->si->prof);
    ctx->si->prof = nullptr;
    ctx->si->prof_on = false;
  }
  ctx->si->prob = *prob;
  ctx->si->batch = batch;
  ctx->si->cap = cap;
  ctx->si->L = L;
  ctx->si->ws = (char*)ws;
  return RIPTRM_OK;
}

int riptrm_si_hvp(riptrm_ctx* ctx, const double* x, const double* y, const double* mu, const double* v, double* out) {
  if (!ctx) return RIPTRM_E_ARG;
  if (!ctx->si) return fail(ctx, RIPTRM_E_STATE, "si_hvp: riptrm_si_bind first");
  if (!x || !y || !mu || !v || !out) return fail(ctx, RIPTRM_E_ARG, "si_hvp: bad argument");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  SIParams P = si_params(ctx, MODE_HVP);
  P.in_x = x;
  P.in_y = y;
  P.in_mu = mu;
  P.in_v = v;
  P.out_v = out;
  return si_launch(ctx, P);
}

int riptrm_si_tcg(riptrm_ctx* ctx, const riptrm_options* opt, const double* x, const double* y, const double* mu,
                  const double* delta) {
  if (!ctx) return RIPTRM_E_ARG;
  if (!ctx->si) return fail(ctx, RIPTRM_E_STATE, "si_tcg: riptrm_si_bind first");
  if (!x || !y || !mu || !delta) return fail(ctx, RIPTRM_E_ARG, "si_tcg: bad argument");
  if (opt && opt->struct_size != (int32_t)sizeof(riptrm_options))
    return fail(ctx, RIPTRM_E_ARG, "si_tcg: riptrm_options.struct_size mismatch");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  SIParams P = si_params(ctx, MODE_TCG);
  if (opt) P.opt = *opt;
  P.in_x = x;
  P.in_y = y;
  P.in_mu = mu;
  P.in_delta = delta;
  return si_launch(ctx, P);
}

int riptrm_si_solve(riptrm_ctx* ctx, const riptrm_options* opt, const double* x0, const double* y0,
                    const double* mu_table, const double* tolL_table, const double* tolC_table, int32_t table_len) {
  if (!ctx) return RIPTRM_E_ARG;
  if (!ctx->si) return fail(ctx, RIPTRM_E_STATE, "si_solve: riptrm_si_bind first");
  if (!opt || opt->struct_size != (int32_t)sizeof(riptrm_options))
    return fail(ctx, RIPTRM_E_ARG, "si_solve: riptrm_options.struct_size mismatch");
  if (!x0 || !y0 || !mu_table || !tolL_table || !tolC_table || table_len <= 0)
    return fail(ctx, RIPTRM_E_ARG, "si_solve: bad argument");
  if (opt->log_capacity > ctx->si->cap) return fail(ctx, RIPTRM_E_ARG, "si_solve: log_capacity exceeds bound capacity");
  if (opt->trs_solver != RIPTRM_TRS_SOLVER_TCG && opt->trs_solver != RIPTRM_TRS_SOLVER_EXACT_REPMAT)
    return fail(ctx, RIPTRM_E_ARG, "si_solve: unknown trs_solver");
  const int d = ctx->si->prob.d, tdim = si_manifold_dim(d);
  const bool hbm = opt->trs_solver == RIPTRM_TRS_SOLVER_EXACT_REPMAT && si_hbm_trs(d);
  if (hbm && (!ctx->big_ws || ctx->big_order < tdim || ctx->big_slots < 1))
    return fail(ctx, RIPTRM_E_STATE, "si_solve: Exact_RepMat above RIPTRM_TRS_DIM_MAX (d >= 8) needs "
                                     "riptrm_trs_bind_workspace(order >= manifold.dim) first");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  SIParams P = si_params(ctx, MODE_SOLVE);
  P.opt = *opt;
  P.in_x = x0;
  P.in_y = y0;
  P.mu_tab = mu_table;
  P.tolL_tab = tolL_table;
  P.tolC_tab = tolC_table;
  P.tab_len = table_len;
  if (int rc = si_launch(ctx, P)) return rc;
  if (!hbm) return RIPTRM_OK;
  // HBM subproblem path: the kernel parks an instance at each subproblem (and each trial point's
  // eigenvalue test); serve every parked instance in batched passes, resume, until none is parked.
  // With the keyed cache (tdim <= 199, RIPTRM_SI_CACHE=1; off by default), the trial point's
  // eigensolve keeps its compact eigenpairs keyed by the park point (x_new, y_new, mu), and a
  // subproblem parked at exactly that point -- the step was accepted without dual clipping, mu
  // unchanged -- is served from them: its matrix is not built (only the coordinates of cxCur) and
  // not decomposed; the matrix would be the same bits (the same k_si_repmat arithmetic at the same
  // point), so the solve is the uncached one bit for bit (RIPTRM.py:686-692 reuses HwNewmatrix the
  // same way).  Measured (d = 8 x 64, `OUT=r5w`): 71% of the subproblems hit, yet the line runs at
  // 246 vs 307 outer it/s without it -- the service is bound by each pass's latency, not by its
  // number of matrices: a pass with one miss costs the eigensolve of a full one, and the hits' CG
  // runs as a second pass.  Kept as an opt-in.
  const int B = ctx->si->batch;
  std::vector<double> st((size_t)B * RIPTRM_STAT_NFIELDS);
  P.mode = MODE_RESUME;
  const char* ce = getenv("RIPTRM_SI_CACHE");
  const bool cache = P.trsC && ce && ce[0] == '1' && riptrm_big_kcache_usable(tdim);
  KeyedEigCache kc;
  kc.keys = P.trsP;
  kc.kstride = kc.klen = 3 * d * d + ctx->si->prob.m + 1;
  kc.cache = P.trsC;
  kc.cstride = P.trsC_stride;
  ctx->big_cache_hits = ctx->big_subproblems = 0;
  if (cache)   // no entry of an earlier solve is valid
    HIPCHK(ctx, hipMemset2DAsync(P.trsC, (size_t)P.trsC_stride * sizeof(double), 0, sizeof(double), B, ctx->stream));
  std::vector<int32_t> hit, miss;
  while (true) {
    HIPCHK(ctx, hipMemcpyAsync(st.data(), P.stats, st.size() * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    std::vector<int32_t> trs, mine;
    for (int b = 0; b < B; ++b) {
      const double ph = st[(size_t)b * RIPTRM_STAT_NFIELDS + RIPTRM_STAT_PHASE];
      if (ph == (double)riptrm::PH_TRS_HOST) trs.push_back(b);
      else if (ph == (double)riptrm::PH_MINEIG_HOST) mine.push_back(b);
    }
    if (trs.empty() && mine.empty()) break;
    const int64_t tp = si_tdp(d);
    if (cache) {
      if (int rc = riptrm_big_kcache_split(ctx, tdim, trs, kc, hit, miss)) return rc;
    } else {
      miss = trs;
      hit.clear();
    }
    ctx->big_cache_hits += (int64_t)hit.size();
    ctx->big_subproblems += (int64_t)trs.size();
    if (int rc = si_repmat(ctx, P, miss, 0, 1)) return rc;
    if (int rc = si_repmat(ctx, P, hit, (int)miss.size(), 1, 1)) return rc;
    if (int rc = si_repmat(ctx, P, mine, B, 0)) return rc;
    if (!miss.empty())
      if (int rc = riptrm_big_gep_ids(ctx, tdim, miss.data(), (int)miss.size(), P.trsA, tdim, (int64_t)tdim * tdim, P.trsa,
                                      tp, P.trsD, opt->trs_tolhardcase, P.trsx, P.trslam, P.trskind, nullptr, false,
                                      true))
        return rc;
    if (!hit.empty()) {
      kc.mode = 1;
      if (int rc = riptrm_big_gep_ids(ctx, tdim, hit.data(), (int)hit.size(), P.trsA, tdim, (int64_t)tdim * tdim, P.trsa,
                                      tp, P.trsD, opt->trs_tolhardcase, P.trsx, P.trslam, P.trskind, nullptr, false,
                                      true, &kc))
        return rc;
    }
    if (!mine.empty()) {
      kc.mode = 2;
      if (int rc = riptrm_big_gep_ids(ctx, tdim, mine.data(), (int)mine.size(), P.trsA, tdim, (int64_t)tdim * tdim,
                                      P.trsa, tp, P.trsD, opt->trs_tolhardcase, nullptr, nullptr, nullptr, P.trsmin, true,
                                      true, cache ? &kc : nullptr))
        return rc;
    }
    if (int rc = si_launch(ctx, P)) return rc;
  }
  return RIPTRM_OK;
}

int riptrm_si_profile_enable(riptrm_ctx* ctx, int32_t on) {
  if (!ctx) return RIPTRM_E_ARG;
  if (!ctx->si) return fail(ctx, RIPTRM_E_STATE, "si_profile_enable: riptrm_si_bind first");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  Bound* s = ctx->si;
  if (on && !s->prof) HIPCHK(ctx, hipMalloc(&s->prof, (size_t)s->batch * RIPTRM_SI_PROF_NFIELDS * 8));
  if (on) HIPCHK(ctx, hipMemsetAsync(s->prof, 0, (size_t)s->batch * RIPTRM_SI_PROF_NFIELDS * 8, ctx->stream));
  s->prof_on = on != 0;
  return RIPTRM_OK;
}

int riptrm_si_profile_read(riptrm_ctx* ctx, double* seconds) {
  if (!ctx || !seconds) return RIPTRM_E_ARG;
  if (!ctx->si || !ctx->si->prof) return fail(ctx, RIPTRM_E_STATE, "si_profile_read: riptrm_si_profile_enable first");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  const int B = ctx->si->batch;
  std::string buf((size_t)B * RIPTRM_SI_PROF_NFIELDS * 8, '\0');
  HIPCHK(ctx, hipMemcpy(&buf[0], ctx->si->prof, buf.size(), hipMemcpyDeviceToHost));
  const double* h = (const double*)buf.data();
  for (int k = 0; k < RIPTRM_SI_PROF_NFIELDS; ++k) {
    double t = 0.0;
    for (int b = 0; b < B; ++b) t += h[(size_t)b * RIPTRM_SI_PROF_NFIELDS + k];
    seconds[k] = t / ctx->clock_hz;
  }
  return RIPTRM_OK;
}

}  // extern "C"
