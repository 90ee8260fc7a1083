// riptrm_trs.h — the Exact_RepMat trust-region subproblem solve on one workgroup (gfx950).
//
// Reference: TRSgep (src/solver/RIPTRM.py:218-299), called by compute_direction's Exact_RepMat
// branch (RIPTRM.py:433-444) with B = I on the matrix of HwCur in an orthonormal tangent basis
// (selfadj_operator2matrix, src/solver/utils.py:565-573), and the second-order stationarity test
// (RIPTRM.py:599-617: smallest eigenvalue of the same matrix at the trial point).
//
//   minimize x^T A x / 2 + a^T x   s.t.  ||x|| <= Delta
//
// The reference takes the rightmost eigenpair of the 2n x 2n pencil (MM0, -MM1) (Adachi et al.
// 2017).  Its rightmost eigenvalue is the rightmost root lam1 of ||(A + lam I)^-1 a|| = Delta on
// (-lam_min, inf), so the device solves the same three-candidate problem from the symmetric
// eigendecomposition A = Q diag(lam) Q^T (restated in oracle/trs_oracle.py::trs_eigh):
//   * interior candidate p1: SciPy's CG on A p = -a (RIPTRM.py:245-251, loop for loop as
//     scipy.sparse.linalg.cg 1.15: x0 = 0, rtol 1e-5, maxiter 10 n), kept iff
//     ||A p1 + a|| / ||a|| < 1e-5 and p1^T p1 < Delta^2;
//   * hard case (a orthogonal to the lam_min eigenspace and ||x2|| < Delta): lam1 = -lam_min,
//     x = x2 + alp q_min (RIPTRM.py:266-291);
//   * boundary: safeguarded Newton on 1/||x(lam)|| - 1/Delta from lam = -lam_min + ||a||/Delta,
//     x = -(A + lam1 I)^-1 a rescaled to ||x|| = Delta (RIPTRM.py:262);
//   * interior wins if its model value is <= the boundary one (RIPTRM.py:294-298).
// The eigendecomposition is a parallel two-sided cyclic Jacobi (round-robin pair ordering: all
// dim/2 rotations of a round are disjoint and applied at once by the whole workgroup) on the
// matrix held in LDS — eigenvalues to high relative accuracy, no library call, no host round trip.
//
// Every thread of the NT-thread workgroup must call every function here (they synchronise).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include "riptrm_wave.h"

namespace riptrm_trs {

#pragma clang fp contract(off)

#ifdef RIPTRM_TRS_PROBE
__device__ double g_probe[96];   // tools/trs_probe.hip only: per-sweep off / diag norms
#endif

constexpr int DIM_MAX = 96;

// Everything below lives in LDS and is reached through these address-space-3 pointers, so the
// (noinline) solver bodies compile to ds_read / ds_write — through generic pointers they became
// flat loads/stores at several times the latency (measured: 5.7k cycles per Jacobi column stage
// at dim 16).
typedef __attribute__((address_space(3))) double lds_f64;   // LDS: 2 * 96 * 97 doubles = 146 KiB (matrix + eigenvectors)

enum Kind : int { K_BOUNDARY = 0, K_INTERIOR = 1, K_HARDCASE_1 = 2 };

// odd row stride: column walks of the Jacobi rotations spread over the LDS banks
__host__ __device__ constexpr int lda_of(int dim) { return dim | 1; }

constexpr int ROT_FIELDS = 7;   // per pair of a Jacobi round: c, s, t, a_pp', a_qq', p, q

// LDS doubles of a Work area for dim (matrix, eigenvectors, vectors, rotation table)
__host__ __device__ constexpr int work_doubles(int dim) {
  return 2 * dim * lda_of(dim) + 8 * DIM_MAX + ROT_FIELDS * (DIM_MAX / 2 + 1);
}

struct Work {
  lds_f64* A;    // dim x lda  (destroyed: eigenvalues end on the diagonal)
  lds_f64* V;    // dim x lda  eigenvectors (columns)
  lds_f64* a;    // dim   linear term
  lds_f64* x;    // dim   solution
  lds_f64* p;    // dim   CG direction / scratch
  lds_f64* r;    // dim   CG residual / scratch
  lds_f64* q;    // dim   CG A p / scratch
  lds_f64* cgx;  // dim   CG iterate (the interior candidate p1)
  lds_f64* g;    // dim   Q^T a
  lds_f64* ev;   // dim   eigenvalues (copied off the diagonal)
  lds_f64* rot;  // ROT_FIELDS x (DIM_MAX/2 + 1)  (c, s, t, a_pp, a_qq, p, q) per pair
  int dim, lda;
};

// carve a Work out of an LDS area of work_doubles(dim) doubles
__device__ __forceinline__ Work make_work(double* base_generic, int dim) {
  lds_f64* base = (lds_f64*)base_generic;
  Work w;
  w.dim = dim;
  w.lda = lda_of(dim);
  const int mat = dim * w.lda;
  w.A = base;
  w.V = base + mat;
  lds_f64* v = base + 2 * mat;
  w.a = v;
  w.x = v + DIM_MAX;
  w.p = v + 2 * DIM_MAX;
  w.r = v + 3 * DIM_MAX;
  w.q = v + 4 * DIM_MAX;
  w.cgx = v + 5 * DIM_MAX;
  w.g = v + 6 * DIM_MAX;
  w.ev = v + 7 * DIM_MAX;
  w.rot = v + 8 * DIM_MAX;
  return w;
}

// Workgroup reductions for NT threads: in-wave DPP/permlane reduction (riptrm_wave.h), then the
// NW wave partials through LDS in wave order.  Every thread gets the bitwise-identical value.
template <int NT>
struct Blk {
  static constexpr int NW = NT / 64;
  lds_f64* red;  // LDS, 2 * NW doubles (unused when NW == 1)
  int par;
  __device__ __forceinline__ explicit Blk(double* red_) : red((lds_f64*)red_), par(0) {}
  template <int OP>
  __device__ __forceinline__ double reduce(double v) {
    v = riptrm_wave::wave_reduce<OP>(v);
    if constexpr (NW == 1) {
      return v;
    } else {
      lds_f64* b = red + par * NW;
      par ^= 1;
      if ((threadIdx.x & 63) == 0) b[threadIdx.x >> 6] = v;
      __syncthreads();
      double s = b[0];
#pragma unroll
      for (int i = 1; i < NW; ++i) s = riptrm_wave::comb<OP>(s, b[i]);
      return s;
    }
  }
  __device__ __forceinline__ double sum(double v) { return reduce<0>(v); }
  __device__ __forceinline__ double min(double v) { return reduce<1>(v); }
  __device__ __forceinline__ double max(double v) { return reduce<2>(v); }
};

// round-robin tournament: pair k of round r among me (even) players, p < q
__device__ __forceinline__ void pair_of(int r, int k, int me, int& p, int& q) {
  const int m1 = me - 1;
  int u, v;
  if (k == 0) {
    u = 0;
    v = 1 + r % m1;
  } else {
    u = 1 + (r + k) % m1;
    v = 1 + (r + m1 - k) % m1;
  }
  p = u < v ? u : v;
  q = u < v ? v : u;
}

// Parallel cyclic Jacobi on the symmetric dim x dim matrix w.A (LDS).  On return w.ev holds the
// eigenvalues (diagonal order) and, if want_v, w.V the eigenvectors as columns (A0 = V diag V^T).
// Rotation formulas: Numerical Recipes' (same as the serial jacobi_reg of riptrm_si.hip).
template <int NT>
__device__ __forceinline__ void jacobi(Blk<NT>& B, Work& w, bool want_v) {
  constexpr int NWV = NT / 64;
  constexpr int CH = 4;   // pairs per wave per load/store batch
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int m = w.dim, lda = w.lda;
  lds_f64* A = w.A;
  lds_f64* V = w.V;
  lds_f64* rot = w.rot;
  // rows are walked by waves and columns by lanes: no integer division on the hot loops
  if (want_v)
    for (int i = wv; i < m; i += NWV)
      for (int j = lane; j < m; j += 64) V[i * lda + j] = (i == j) ? 1.0 : 0.0;
  const int me = m + (m & 1);
  const int np = me / 2;
  __syncthreads();
  for (int sweep = 0; sweep < 40 && m > 1; ++sweep) {
    double off = 0.0, dg = 0.0;
    for (int i = wv; i < m; i += NWV)
      for (int j = lane; j < m; j += 64) {
        const double v = A[i * lda + j];
        if (j > i) off += v * v;
        else if (j == i) dg += v * v;
      }
    off = B.sum(off);
    dg = B.sum(dg);
#ifdef RIPTRM_TRS_PROBE
    if (tid == 0 && sweep < 40) { g_probe[2 * sweep] = off; g_probe[2 * sweep + 1] = dg; g_probe[80] = sweep; }
#endif
    if (off <= 1e-36 * dg) break;   // off-diagonal far below the eigenvalues' rounding
    for (int r = 0; r < me - 1; ++r) {
#ifdef RIPTRM_TRS_PROBE
      long long pc0 = clock64();
#endif
      for (int k = tid; k < np; k += NT) {
        int p, q;
        pair_of(r, k, me, p, q);
        double c = 1.0, s = 0.0, t = 0.0, app = 0.0, aqq = 0.0;
        if (q < m) {
          const double apq = A[p * lda + q];
          app = A[p * lda + p];
          aqq = A[q * lda + q];
          if (apq != 0.0) {
            const double theta = (aqq - app) / (2.0 * apq);
            t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
            c = 1.0 / sqrt(t * t + 1.0);
            s = t * c;
            app = app - t * apq;
            aqq = aqq + t * apq;
          }
        }
        lds_f64* R = rot + ROT_FIELDS * k;
        R[0] = c;
        R[1] = s;
        R[2] = t;
        R[3] = app;
        R[4] = aqq;
        R[5] = (double)p;
        R[6] = (double)q;
      }
      __syncthreads();
#ifdef RIPTRM_TRS_PROBE
      long long pc1 = clock64();
#endif
      // columns p, q of A (and V): A <- A J, then rows p, q: A <- J^T A.  A wave takes CH of its
      // pairs at once: every LDS load of the chunk is issued before any store (the pairs of a
      // round touch disjoint columns / rows), so a chunk costs two LDS round trips, not 2 CH.
      for (int k0 = wv; k0 < np; k0 += NWV * CH) {
        double cc[CH], ss[CH];
        int pp[CH], qq[CH];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
          const int k = k0 + u * NWV;
          const lds_f64* R = rot + ROT_FIELDS * (k < np ? k : 0);
          cc[u] = R[0];
          ss[u] = k < np ? R[1] : 0.0;
          pp[u] = (int)R[5];
          qq[u] = (int)R[6];
        }
        for (int i = lane; i < m; i += 64) {
          double ap[CH], aq[CH], vp[CH], vq[CH];
#pragma unroll
          for (int u = 0; u < CH; ++u) {
            if (ss[u] != 0.0) {
              ap[u] = A[i * lda + pp[u]];
              aq[u] = A[i * lda + qq[u]];
              if (want_v) {
                vp[u] = V[i * lda + pp[u]];
                vq[u] = V[i * lda + qq[u]];
              }
            }
          }
#pragma unroll
          for (int u = 0; u < CH; ++u) {
            if (ss[u] != 0.0) {
              A[i * lda + pp[u]] = cc[u] * ap[u] - ss[u] * aq[u];
              A[i * lda + qq[u]] = ss[u] * ap[u] + cc[u] * aq[u];
              if (want_v) {
                V[i * lda + pp[u]] = cc[u] * vp[u] - ss[u] * vq[u];
                V[i * lda + qq[u]] = ss[u] * vp[u] + cc[u] * vq[u];
              }
            }
          }
        }
      }
      __syncthreads();
#ifdef RIPTRM_TRS_PROBE
      long long pc2 = clock64();
#endif
      for (int k0 = wv; k0 < np; k0 += NWV * CH) {
        double cc[CH], ss[CH];
        int pp[CH], qq[CH];
#pragma unroll
        for (int u = 0; u < CH; ++u) {
          const int k = k0 + u * NWV;
          const lds_f64* R = rot + ROT_FIELDS * (k < np ? k : 0);
          cc[u] = R[0];
          ss[u] = k < np ? R[1] : 0.0;
          pp[u] = (int)R[5];
          qq[u] = (int)R[6];
        }
        for (int j = lane; j < m; j += 64) {
          double ap[CH], aq[CH];
#pragma unroll
          for (int u = 0; u < CH; ++u) {
            if (ss[u] != 0.0) {
              ap[u] = A[pp[u] * lda + j];
              aq[u] = A[qq[u] * lda + j];
            }
          }
#pragma unroll
          for (int u = 0; u < CH; ++u) {
            if (ss[u] != 0.0) {
              A[pp[u] * lda + j] = cc[u] * ap[u] - ss[u] * aq[u];
              A[qq[u] * lda + j] = ss[u] * ap[u] + cc[u] * aq[u];
            }
          }
        }
      }
      __syncthreads();
#ifdef RIPTRM_TRS_PROBE
      long long pc3 = clock64();
#endif
      // the rotated 2 x 2 block exactly: a_pq = 0, a_pp / a_qq by the stable update
      for (int k = tid; k < np; k += NT) {
        const lds_f64* R = rot + ROT_FIELDS * k;
        if (R[1] == 0.0) continue;
        const int p = (int)R[5], q = (int)R[6];
        A[p * lda + q] = 0.0;
        A[q * lda + p] = 0.0;
        A[p * lda + p] = R[3];
        A[q * lda + q] = R[4];
      }
      __syncthreads();
#ifdef RIPTRM_TRS_PROBE
      long long pc4 = clock64();
      if (tid == 0) { g_probe[84] += pc1 - pc0; g_probe[85] += pc2 - pc1; g_probe[86] += pc3 - pc2; g_probe[87] += pc4 - pc3; g_probe[88] += 1; }
#endif
    }
  }
  for (int i = tid; i < m; i += NT) w.ev[i] = A[i * lda + i];
  __syncthreads();
}

// smallest eigenvalue of w.A (destroys w.A): RIPTRM.py:611-612
template <int NT>
__device__ __forceinline__ double min_eig(Blk<NT>& B, Work& w) {
  jacobi<NT>(B, w, false);
  double v = INFINITY;
  for (int i = threadIdx.x; i < w.dim; i += NT) v = fmin(v, w.ev[i]);
  return B.min(v);
}

// y = A v over the LDS matrix, one thread per row (row sums in column order)
template <int NT>
__device__ __forceinline__ void matvec(const Work& w, const lds_f64* v, lds_f64* y) {
  const int m = w.dim, lda = w.lda;
  for (int i = threadIdx.x; i < m; i += NT) {
    const lds_f64* row = w.A + i * lda;
    double acc = 0.0;
    for (int k = 0; k < m; ++k) acc += row[k] * v[k];
    y[i] = acc;
  }
}

struct Result {
  double lam1;
  int kind;
};

// TRSgep(A, a, I, Delta, tolhardcase): w.A, w.a filled by the caller (A symmetric).  Writes the
// solution into w.x; w.A is destroyed.
template <int NT>
__device__ __forceinline__ Result trs_solve(Blk<NT>& B, Work& w, double Delta, double tolhardcase) {
  const int tid = threadIdx.x;
  const int m = w.dim;
  const double D2 = Delta * Delta;
  // ---- interior candidate: scipy.sparse.linalg.cg(A, -a) (RIPTRM.py:245) -----------------
  double an = 0.0;
  for (int i = tid; i < m; i += NT) {
    const double b = -w.a[i];
    w.cgx[i] = 0.0;
    w.r[i] = b;
    an += b * b;
  }
  an = sqrt(B.sum(an));   // ||b|| = ||a||
  __syncthreads();
  bool cg_ok = false;
  double p1obj = 0.0;
  if (an == 0.0) {
    // cg returns b itself (= -a = 0); the residual test divides by ||a|| = 0 -> not eligible
    cg_ok = false;
  } else {
    const double atol = 1e-5 * an;
    double rho_prev = 1.0;
    for (int it = 0; it < 10 * m; ++it) {
      double rr = 0.0;
      for (int i = tid; i < m; i += NT) rr += w.r[i] * w.r[i];
      rr = B.sum(rr);
      if (sqrt(rr) < atol) break;
      const double rho = rr;   // dot(r, z) with z = r (no preconditioner)
      const double beta = it > 0 ? rho / rho_prev : 0.0;
      for (int i = tid; i < m; i += NT) w.p[i] = it > 0 ? w.p[i] * beta + w.r[i] : w.r[i];
      __syncthreads();
      matvec<NT>(w, w.p, w.q);
      __syncthreads();
      double pq = 0.0;
      for (int i = tid; i < m; i += NT) pq += w.p[i] * w.q[i];
      pq = B.sum(pq);
      const double alpha = rho / pq;
      for (int i = tid; i < m; i += NT) {
        w.cgx[i] += alpha * w.p[i];
        w.r[i] -= alpha * w.q[i];
      }
      rho_prev = rho;
      __syncthreads();
    }
    // ||A p1 + a|| / ||a|| < 1e-5 and p1^T p1 < Delta^2 (RIPTRM.py:246-251)
    matvec<NT>(w, w.cgx, w.q);
    __syncthreads();
    double v3[3] = {0.0, 0.0, 0.0};
    for (int i = tid; i < m; i += NT) {
      const double res = w.q[i] + w.a[i];
      v3[0] += res * res;
      v3[1] += w.cgx[i] * w.cgx[i];
      v3[2] += w.cgx[i] * w.q[i];
    }
    const double res2 = B.sum(v3[0]);
    const double pp = B.sum(v3[1]);
    const double pAp = B.sum(v3[2]);
    double ap = 0.0;
    for (int i = tid; i < m; i += NT) ap += w.a[i] * w.cgx[i];
    ap = B.sum(ap);
    cg_ok = (sqrt(res2) / an < 1e-5) && (pp < D2);
    p1obj = 0.5 * pAp + ap;
  }
  // ---- eigendecomposition ------------------------------------------------------------------
  jacobi<NT>(B, w, true);
  const int lda = w.lda;
  double lmin = INFINITY, lmax_abs = 0.0;
  for (int i = tid; i < m; i += NT) {
    lmin = fmin(lmin, w.ev[i]);
    lmax_abs = fmax(lmax_abs, fabs(w.ev[i]));
  }
  lmin = B.min(lmin);
  lmax_abs = B.max(lmax_abs);
  // index of lmin (the lowest such index) and g = Q^T a
  double imin = INFINITY;
  for (int i = tid; i < m; i += NT) {
    if (w.ev[i] == lmin) imin = fmin(imin, (double)i);
    double acc = 0.0;
    for (int k = 0; k < m; ++k) acc += w.V[k * lda + i] * w.a[k];
    w.g[i] = acc;
  }
  const double kd = B.min(imin);   // no index when every eigenvalue is NaN: never form one from inf
  const int kmin = (kd >= 0.0 && kd < (double)m) ? (int)kd : 0;
  __syncthreads();
  const double hard_tol = 1e-12 * fmax(1.0, lmax_abs);
  double gh = 0.0, gg = 0.0;
  for (int i = tid; i < m; i += NT) {
    const double gi = w.g[i];
    gg += gi * gi;
    if (fabs(w.ev[i] - lmin) <= hard_tol) gh += gi * gi;
  }
  const double ghard = sqrt(B.sum(gh));
  const double gn = sqrt(B.sum(gg));
  const double lo = -lmin;
  Result res{0.0, K_BOUNDARY};
  bool have = false;
  double xobj = 0.0;
  if (ghard <= tolhardcase * gn) {
    // hard case candidate: x2 = -(A - lmin I)^+ a on the non-hard eigenvectors
    double x2 = 0.0;
    for (int i = tid; i < m; i += NT) {
      const bool hs = fabs(w.ev[i] - lmin) <= hard_tol;
      const double c = hs ? 0.0 : -w.g[i] / (w.ev[i] - lmin);
      w.p[i] = c;   // eigen coordinates
      x2 += c * c;
    }
    x2 = B.sum(x2);
    if (x2 < D2) {
      const double alp = sqrt(D2 - x2);
      __syncthreads();
      if (tid == 0) w.p[kmin] += alp;   // x = Q (x2c + alp e_kmin)
      __syncthreads();
      res.lam1 = lo;
      res.kind = K_HARDCASE_1;
      have = true;
    }
  }
  if (!have) {
    // boundary: Newton on phi(l) = 1/||x(l)|| - 1/Delta, x(l) = -(Lam + l)^-1 g
    double l1 = lo + gn / Delta;
    for (int itn = 0; itn < 100; ++itn) {
      double s2 = 0.0, s3 = 0.0;
      for (int i = tid; i < m; i += NT) {
        const double den = w.ev[i] + l1;
        const double gi = w.g[i];
        s2 += (gi / den) * (gi / den);
        s3 += (gi * gi) / (den * den * den);
      }
      s2 = B.sum(s2);
      s3 = B.sum(s3);
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
    for (int i = tid; i < m; i += NT) {
      const double c = -w.g[i] / (w.ev[i] + l1);
      w.p[i] = c;
      s2 += c * c;
    }
    const double sc = Delta / sqrt(B.sum(s2));   // x / ||x|| * Delta (RIPTRM.py:262)
    __syncthreads();
    for (int i = tid; i < m; i += NT) w.p[i] = w.p[i] * sc;
    res.lam1 = l1;
    res.kind = K_BOUNDARY;
  }
  __syncthreads();
  // model value of the eigen-coordinate candidate: sum lam c^2 / 2 + g.c
  double o2[2] = {0.0, 0.0};
  for (int i = tid; i < m; i += NT) {
    const double c = w.p[i];
    o2[0] += w.ev[i] * c * c;
    o2[1] += w.g[i] * c;
  }
  xobj = 0.5 * B.sum(o2[0]) + B.sum(o2[1]);
  const bool interior = cg_ok && p1obj <= xobj;   // RIPTRM.py:294-298
  for (int i = tid; i < m; i += NT) {
    if (interior) {
      w.x[i] = w.cgx[i];
    } else {
      double acc = 0.0;
      for (int k = 0; k < m; ++k) acc += w.V[i * lda + k] * w.p[k];
      w.x[i] = acc;
    }
  }
  if (interior) {
    res.lam1 = 0.0;
    res.kind = K_INTERIOR;
  }
  __syncthreads();
  return res;
}

}  // namespace riptrm_trs
