// riptrm_eig.h — batched symmetric eigensolver for the HBM Exact_RepMat service, one workgroup per
// matrix, the matrix resident in LDS (orders up to EIG_LDS_MAX; csrc/riptrm_trs_big.hip eig_batched).
//
// Reference: TRSgep (src/solver/RIPTRM.py:218-299) needs the spectrum of the subproblem's matrix
// (the rightmost eigenpair of its 2n x 2n pencil; the build takes A = Q diag(lam) Q^T and solves the
// secular equation in that basis, riptrm_trs_big.hip k_secular), and the second-order test
// (RIPTRM.py:599-617) its smallest eigenvalue.  Rounds 3-4 called rocSOLVER dsyevd_strided_batched
// for orders above 96: ~78% of the n = 200 Exact line's GPU time (sytd2 + divide and conquer on
// 199 x 199 matrices, latency-bound).  This is the hand-written replacement:
//   1. Householder tridiagonalisation (LAPACK dsytd2, lower) with the lower triangle PACKED in LDS
//      (m (m + 1) / 2 doubles: 159 KB at m = 199), the reflectors stored in place of the columns
//      they annihilate; per column one wave forms the reflector, the workgroup runs the symmetric
//      mat-vec (wave per row, both halves of the packed triangle) and the rank-two update;
//   2. eigenvalues of the tridiagonal T by bisection on Sturm counts, one thread per eigenvalue
//      (absolute accuracy eps ||T||, the tridiagonalisation's own error);
//   3. eigenvectors of T by twisted factorisations (the LDL^T and UDU^T of T - lam I meet at the
//      index of the smallest |gamma|), one thread per eigenvector, in its output row;
//   4. back-transformation q = H_0 ... H_{m-2} z with the reflectors from LDS, a wave per group of
//      four vectors (each vector spread over the wave's lanes, wave reductions for the dots);
//   5. block Gram-Schmidt among eigenvectors of close eigenvalues (the twisted vectors are
//      orthogonal only to eps ||T|| / gap), Cholesky-QR inside a block.
// Numerically multiple eigenvalues: T is split where e_j^2 <= eps^2 |d_j d_{j+1}| and each member of
// such a run takes its vector on a different block.
// Output as rocSOLVER's: eigenvalues ascending, eigenvector k in row k of the row-major view of the
// input (column k of the column-major matrix), info = 0 (non-finite input: info = 1).  Fixed
// reduction orders: a matrix's results do not depend on the batch it is in.
#pragma once
#include <hip/hip_runtime.h>
#include <float.h>
#include <math.h>
#include "riptrm_wave.h"

namespace riptrm_eig {

#pragma clang fp contract(off)

constexpr int EW = 512;                    // threads per matrix
constexpr int EIG_LDS_MAX = 199;           // packed lower triangle + two vectors fit 160 KiB
constexpr int EIG_MAX_M = 256;             // four elements per lane in the back-transformation

__host__ __device__ constexpr int poff(int i) { return i * (i + 1) / 2; }
__host__ __device__ constexpr int vpad_eig(int m) { return (m + 7) / 8 * 8; }
constexpr int GB = 32;                     // row block of the Gram-Schmidt phase
// dynamic LDS: the packed triangle + d / e (phases 1-4), or two GB-row blocks + their Gram and its
// Cholesky inverse (phase 5)
__host__ __device__ constexpr size_t eig_lds_bytes(int m) {
  return (poff(m) + 2 * (size_t)vpad_eig(m) > 2 * (size_t)GB * vpad_eig(m) + 2 * GB * (GB + 1)
              ? poff(m) + 2 * (size_t)vpad_eig(m)
              : 2 * (size_t)GB * vpad_eig(m) + 2 * GB * (GB + 1)) *
         sizeof(double);
}

typedef __attribute__((address_space(3))) double lds_t;

// the number of eigenvalues of T (diagonal d, off-diagonal e) below x (Sturm count, LAPACK dlaneg's
// recurrence with pivmin guarding zero pivots)
__device__ __forceinline__ int sturm_count(const lds_t* d, const lds_t* e, int m, double x, double pivmin) {
  double q = d[0] - x;
  if (fabs(q) < pivmin) q = -pivmin;
  int c = q < 0.0;
  for (int j = 1; j < m; ++j) {
    const double ej = e[j - 1];
    q = (d[j] - x) - (ej * ej) / q;
    if (fabs(q) < pivmin) q = -pivmin;
    c += q < 0.0;
  }
  return c;
}

// Matrix k = blockIdx.x: the m x m symmetric matrix at A0 + k a_stride (leading dimension lda; the
// lower triangle is read) -> eigenvalues ascending at ev0 + k ev_stride, eigenvectors (vectors != 0)
// in the rows of the same matrix.  Scratch per matrix (three vectors of >= m doubles, k sc_stride
// apart): d at d0, e at e0, tau at t0.
__global__ void __launch_bounds__(EW) k_eig_lds(double* A0, int64_t a_stride, int lda, int m, double* ev0,
                                                int64_t ev_stride, double* d0, double* e0, double* t0,
                                                int64_t sc_stride, int32_t* infos, int vectors) {
  extern __shared__ double smem[];
  __shared__ double scal[2];
  __shared__ int bad;
  lds_t* P = (lds_t*)smem;                    // packed lower triangle, row i at poff(i)
  lds_t* vb = P + poff(m);                    // the reflector (phase 1), then d (phases 2-3)
  lds_t* pb = vb + vpad_eig(m);               // p (phase 1), then e (phases 2-3), then tau (phase 4)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr int NW = EW / 64;
  const int k = blockIdx.x;
  double* A = A0 + (int64_t)k * a_stride;
  double* ev = ev0 + (int64_t)k * ev_stride;
  double* dg = d0 + (int64_t)k * sc_stride;
  double* eg = e0 + (int64_t)k * sc_stride;
  double* tg = t0 + (int64_t)k * sc_stride;
  if (tid == 0) bad = 0;
  __syncthreads();
  for (int64_t q = tid; q < (int64_t)m * m; q += EW) {
    const int i = (int)(q / m), j = (int)(q - (int64_t)i * m);
    if (j <= i) {
      const double a = A[(int64_t)i * lda + j];
      if (!isfinite(a)) bad = 1;
      P[poff(i) + j] = a;
    }
  }
  __syncthreads();
  if (bad) {
    if (tid == 0) infos[k] = 1;
    for (int i = tid; i < m; i += EW) ev[i] = NAN;
    return;
  }
  if (tid == 0) infos[k] = 0;

  // ---- 1. tridiagonalisation (dsytd2, lower) ----------------------------------------------------
  for (int i = 0; i < m - 1; ++i) {
    const int r = m - i - 1;   // the trailing rows / columns i + 1 .. m - 1
    if (w == 0) {
      double s = 0.0;
      for (int j = i + 2 + lane; j < m; j += 64) {
        const double x = P[poff(j) + i];
        s += x * x;
      }
      s = riptrm_wave::wave_sum(s);
      const double alpha = P[poff(i + 1) + i];
      double tau = 0.0, beta = alpha, scl = 0.0;
      if (s != 0.0) {   // dlarfg: H (alpha, x) = (beta, 0), H = I - tau v v^T, v(0) = 1
        beta = -copysign(sqrt(alpha * alpha + s), alpha);
        tau = (beta - alpha) / beta;
        scl = 1.0 / (alpha - beta);
      }
      for (int l = lane; l < r; l += 64) {
        double v = 1.0;
        if (l > 0) {
          v = P[poff(i + 1 + l) + i] * scl;
          P[poff(i + 1 + l) + i] = v;   // the reflector replaces the column it annihilates
        }
        vb[l] = v;
      }
      if (lane == 0) {
        scal[0] = tau;
        P[poff(i + 1) + i] = beta;
        eg[i] = beta;
        tg[i] = tau;
      }
    }
    __syncthreads();
    const double tau = scal[0];
    if (tau != 0.0) {   // uniform
      // p = tau A22 v: a wave per row, the row's lower part and its column below the diagonal
      for (int l = w; l < r; l += NW) {
        const int gl = i + 1 + l;
        double acc = 0.0;
        for (int j = lane; j < r; j += 64) {
          const int gj = i + 1 + j;
          const double a = j <= l ? P[poff(gl) + gj] : P[poff(gj) + gl];
          acc += a * vb[j];
        }
        acc = riptrm_wave::wave_sum(acc);
        if (lane == 0) pb[l] = tau * acc;
      }
      __syncthreads();
      // alpha2 = -tau (p . v) / 2 (every wave the same tree), w = p + alpha2 v, A22 -= v w^T + w v^T
      double s = 0.0;
      for (int l = lane; l < r; l += 64) s += pb[l] * vb[l];
      s = riptrm_wave::wave_sum(s);
      const double a2 = -0.5 * tau * s;
      for (int l = w; l < r; l += NW) {
        const double vl = vb[l], wl = pb[l] + a2 * vl;
        lds_t* row = P + poff(i + 1 + l) + i + 1;
        for (int j = lane; j <= l; j += 64) {
          const double vj = vb[j];
          const double wj = pb[j] + a2 * vj;
          row[j] = row[j] - (vl * wj + wl * vj);
        }
      }
    }
    __syncthreads();
  }
  // d, e into LDS (vb, pb) and the slot
  for (int i = tid; i < m; i += EW) {
    const double di = P[poff(i) + i];
    vb[i] = di;
    dg[i] = di;
    if (i < m - 1) pb[i] = P[poff(i + 1) + i];
  }
  __syncthreads();
  const double eps = DBL_EPSILON;
  // splitting: e_j -> 0 where |e_j| <= 4 eps ||T|| (the tridiagonalisation's own rounding level, so
  // the eigenvalues move by no more than its error); a multiple eigenvalue of A then lives in
  // separate blocks of T (an unreduced tridiagonal has simple eigenvalues)
  double tn0 = 0.0;
  for (int j = 0; j < m; ++j)
    tn0 = fmax(tn0, fabs(vb[j]) + (j > 0 ? fabs(pb[j - 1]) : 0.0) + (j < m - 1 ? fabs(pb[j]) : 0.0));
  __syncthreads();
  for (int j = tid; j < m - 1; j += EW)
    if (fabs(pb[j]) <= 4.0 * eps * tn0) pb[j] = 0.0;
  __syncthreads();
  const lds_t* d = vb;
  const lds_t* e = pb;

  // ---- 2. eigenvalues: bisection on Sturm counts, one thread per eigenvalue ------------------------
  double tnorm = 0.0, glo = INFINITY, ghi = -INFINITY, emax2 = 0.0;
  for (int j = 0; j < m; ++j) {   // every thread the same (broadcast LDS reads)
    const double r0 = j > 0 ? fabs(e[j - 1]) : 0.0, r1 = j < m - 1 ? fabs(e[j]) : 0.0;
    glo = fmin(glo, d[j] - r0 - r1);
    ghi = fmax(ghi, d[j] + r0 + r1);
    tnorm = fmax(tnorm, fabs(d[j]) + r0 + r1);
    if (j < m - 1) emax2 = fmax(emax2, e[j] * e[j]);
  }
  const double pivmin = DBL_MIN * fmax(1.0, emax2);
  const double fudge = 2.0 * eps * tnorm + 2.0 * pivmin;
  double lam = 0.0;
  if (tid < m) {
    double lo = glo - fudge, hi = ghi + fudge;
    for (int it = 0; it < 128; ++it) {
      const double tol = fmax(2.0 * eps * fmax(fabs(lo), fabs(hi)), eps * tnorm);
      if (hi - lo <= tol) break;
      const double mid = 0.5 * (lo + hi);
      if (mid <= lo || mid >= hi) break;
      if (sturm_count(d, e, m, mid, pivmin) > tid) hi = mid;
      else lo = mid;
    }
    lam = 0.5 * (lo + hi);
    ev[tid] = lam;
  }
  if (!vectors) return;
  __syncthreads();   // every eigenvalue in ev (the block assignment below reads its neighbours)

  // ---- 3. eigenvectors of T: twisted factorisation at lam on its block, in the thread's row ----------
  if (tid < m) {
    double* Z = A + (int64_t)tid * lda;
    const double tiny = pivmin;
    // numerically equal eigenvalues (within delta) take distinct blocks: member k of the run
    // i0 .. takes the block where the running count of block eigenvalues in [lam - delta,
    // lam + delta] passes k (per-block Sturm counts at both ends)
    const double delta = 16.0 * eps * tnorm;
    int i0 = tid;
    while (i0 > 0 && lam - ev[i0 - 1] <= delta) --i0;
    const int kk = tid - i0;
    int blo = 0, bhi = m - 1, acc = 0, bs = 0, ca = 0, cb = 0;
    bool found = false;
    double qa = 0.0, qb = 0.0;
    for (int j = 0; j < m; ++j) {
      const bool start = j == bs;
      const double ej2 = start ? 0.0 : e[j - 1] * e[j - 1];
      qa = (d[j] - (lam - delta)) - (start ? 0.0 : ej2 / qa);
      if (fabs(qa) < pivmin) qa = -pivmin;
      qb = (d[j] - (lam + delta)) - (start ? 0.0 : ej2 / qb);
      if (fabs(qb) < pivmin) qb = -pivmin;
      ca += qa < 0.0;
      cb += qb < 0.0;
      if (j == m - 1 || e[j] == 0.0) {   // block bs .. j ends
        if (!found && acc + (cb - ca) > kk) {
          found = true;
          blo = bs;
          bhi = j;
        }
        acc += cb - ca;
        ca = cb = 0;
        bs = j + 1;
      }
    }
    for (int j = 0; j < blo; ++j) Z[j] = 0.0;
    for (int j = bhi + 1; j < m; ++j) Z[j] = 0.0;
    double dp = d[blo] - lam;
    if (fabs(dp) < tiny) dp = -tiny;
    Z[blo] = dp;   // D+_j (LDL^T of T - lam I on the block)
    for (int j = blo + 1; j <= bhi; ++j) {
      const double ej = e[j - 1];
      dp = (d[j] - lam) - (ej * ej) / dp;
      if (fabs(dp) < tiny) dp = -tiny;
      Z[j] = dp;
    }
    // UDU^T from the block's bottom; gamma_j = D+_j + D-_j - (d_j - lam), the twist at min |gamma|
    double dm = d[bhi] - lam;
    if (fabs(dm) < tiny) dm = -tiny;
    double best = fabs(Z[bhi]);
    int r = bhi;
    for (int j = bhi - 1; j >= blo; --j) {
      const double ej = e[j];
      dm = (d[j] - lam) - (ej * ej) / dm;
      if (fabs(dm) < tiny) dm = -tiny;
      const double g = fabs(Z[j] + dm - (d[j] - lam));
      if (g < best) {
        best = g;
        r = j;
      }
    }
    // D-_j for j > r into the row (D+ is kept below the twist)
    dm = d[bhi] - lam;
    if (fabs(dm) < tiny) dm = -tiny;
    for (int j = bhi; j > r; --j) {
      if (j < bhi) {
        const double ej = e[j];
        dm = (d[j] - lam) - (ej * ej) / dm;
        if (fabs(dm) < tiny) dm = -tiny;
      }
      Z[j] = dm;
    }
    double z = 1.0, nrm = 1.0;
    for (int j = r + 1; j <= bhi; ++j) {   // z_j = -(e_{j-1} / D-_j) z_{j-1}
      z = -(e[j - 1] / Z[j]) * z;
      Z[j] = z;
      nrm += z * z;
    }
    z = 1.0;
    for (int j = r - 1; j >= blo; --j) {  // z_j = -(e_j / D+_j) z_{j+1}
      z = -(e[j] / Z[j]) * z;
      Z[j] = z;
      nrm += z * z;
    }
    Z[r] = 1.0;
    const double inv = 1.0 / sqrt(nrm);
    for (int j = blo; j <= bhi; ++j) Z[j] = Z[j] * inv;
  }
  __syncthreads();
  for (int i = tid; i < m - 1; i += EW) pb[i] = tg[i];   // tau into LDS (e is done with)
  __threadfence_block();
  __syncthreads();

  // ---- 4. back-transformation q = H_0 H_1 ... H_{m-2} z, four vectors per wave at a time ----------
  constexpr int NV = 4;
  for (int v0 = w * NV; v0 < m; v0 += NW * NV) {
    double z[NV][4];
    double* R[NV];
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      const int t = v0 + u < m ? v0 + u : m - 1;
      R[u] = A + (int64_t)t * lda;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = lane + 64 * q;
        z[u][q] = j < m ? R[u][j] : 0.0;
      }
    }
    for (int i = m - 2; i >= 0; --i) {
      const double tau = pb[i];
      if (tau == 0.0) continue;   // uniform
      double v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = lane + 64 * q;
        v[q] = j == i + 1 ? 1.0 : ((j > i + 1 && j < m) ? P[poff(j) + i] : 0.0);
      }
      double s[NV];
#pragma unroll
      for (int u = 0; u < NV; ++u) {
        s[u] = 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q) s[u] += v[q] * z[u][q];
      }
#pragma unroll
      for (int u = 0; u < NV; ++u) s[u] = riptrm_wave::wave_sum(s[u]);
#pragma unroll
      for (int u = 0; u < NV; ++u) {
        const double f = tau * s[u];
#pragma unroll
        for (int q = 0; q < 4; ++q) z[u][q] = z[u][q] - f * v[q];
      }
    }
#pragma unroll
    for (int u = 0; u < NV; ++u) {
      if (v0 + u >= m) continue;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = lane + 64 * q;
        if (j < m) R[u][j] = z[u][q];
      }
    }
  }
  __threadfence_block();
  __syncthreads();

  // ---- 5. orthogonality: block Gram-Schmidt over close eigenvalues ---------------------------------
  // The twisted vectors are orthogonal to ~eps ||T|| / gap: ~1e-9 for the frame matrices of
  // Exact_RepMat (a few diagonal entries y_i / x_i ~ 1e6 over O(1) eigenvalues).  Row blocks of GB
  // vectors, in order: block J loses its components along every earlier block I that holds
  // eigenvalues within CTOL ||T|| of its own (classical GS against the already orthonormal rows,
  // E = Q_I Q_J^T), then is orthonormalised itself (Cholesky-QR of its Gram).  The sweep repeats
  // while some |E| exceeded 1e-8, at most three times; a row that is (numerically) in the span of
  // its block's earlier rows is rebuilt from the orthogonal complement of all the others; if that
  // fails, info = 2.
  {
    const double ctol = 1e-2 * tnorm;
    const int nb = (m + GB - 1) / GB;
    const int mp = vpad_eig(m);
    lds_t* QJ = P;                         // [GB][mp]
    lds_t* QI = P + GB * mp;               // [GB][mp]
    lds_t* E = P + 2 * GB * mp;            // [GB][GB + 1]
    __shared__ int eflag, again, ndrop;
    __shared__ int dropped[16];
    if (tid == 0) eflag = 0;
    for (int pass = 0; pass < 3; ++pass) {
    __syncthreads();
    if (tid == 0) again = 0, ndrop = 0;
    for (int J = 0; J < nb; ++J) {
      const int j0 = J * GB, jn = min(GB, m - j0);
      __syncthreads();
      for (int q = tid; q < GB * mp; q += EW) {
        const int a = q / mp, c = q - a * mp;
        QJ[q] = (a < jn && c < m) ? A[(int64_t)(j0 + a) * lda + c] : 0.0;
      }
      for (int I = 0; I <= J; ++I) {
        const int i0b = I * GB, in = min(GB, m - i0b);
        // eigenvalues sorted: block I is close to block J iff its last one is within ctol of J's first
        if (I < J && ev[j0] - ev[i0b + in - 1] > ctol) continue;   // uniform
        __syncthreads();
        if (I < J)
          for (int q = tid; q < GB * mp; q += EW) {
            const int a = q / mp, c = q - a * mp;
            QI[q] = (a < in && c < m) ? A[(int64_t)(i0b + a) * lda + c] : 0.0;
          }
        __syncthreads();
        const lds_t* QA = I < J ? QI : QJ;
        // E[a][b] = Q_I[a] . Q_J[b] (a 2 x 1 register block per thread: GB x GB / 512)
        for (int q = tid; q < GB * GB; q += EW) {
          const int a = q / GB, b = q - a * GB;
          double sacc = 0.0;
          for (int c = 0; c < m; ++c) sacc += QA[a * mp + c] * QJ[b * mp + c];
          const double eab = (I == J && a == b) ? sacc - 1.0 : sacc;
          E[a * (GB + 1) + b] = eab;
          if (a < in && b < jn) {
            if (fabs(eab) > 1e-8) again = 1;
          }
        }
        __syncthreads();
        if (I == J) {
          // exact orthonormalisation of the block: G = Q_J Q_J^T = L L^T (wave 0, right-looking, lane c
          // owns row c), Q_J <- L^-1 Q_J.  A pivot below 1/4 (a vector nearly in the span of the
          // block's earlier ones: a numerically multiple eigenvalue T did not split) drops the row;
          // it is rebuilt from the orthogonal complement of all other vectors after the sweep.
          lds_t* Li = E + GB * (GB + 1);   // L^-1, [GB][GB + 1]
          if (w == 0 && lane < GB) {
            const int c = lane;
            E[c * (GB + 1) + c] += 1.0;   // G = E + I
            if (c >= jn) E[c * (GB + 1) + c] = 1.0;   // padding rows: identity
            for (int kk = 0; kk < GB; ++kk) {
              const double piv = E[kk * (GB + 1) + kk];
              const bool drop = kk < jn && piv < 0.25;
              if (drop && c == 0) dropped[ndrop < 16 ? ndrop : 15] = j0 + kk, ndrop = ndrop + 1;
              const double sq = drop ? 1.0 : sqrt(piv);
              double lck = 0.0;
              if (c > kk) lck = drop ? 0.0 : E[c * (GB + 1) + kk] / sq;
              asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // lanes exchange through LDS
              if (c == kk) E[c * (GB + 1) + kk] = sq;
              if (c > kk) {
                E[c * (GB + 1) + kk] = lck;
                for (int c2 = kk + 1; c2 <= c; ++c2) {
                  // L[c2][kk] of another lane: read after every lane wrote its column entry
                  const double l2 = c2 == c ? lck : E[c2 * (GB + 1) + kk];
                  E[c * (GB + 1) + c2] -= lck * l2;
                }
              }
              asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // lanes exchange through LDS
            }
            // column c of L^-1 (lower)
            for (int rr = 0; rr < GB; ++rr) Li[rr * (GB + 1) + c] = 0.0;
            Li[c * (GB + 1) + c] = 1.0 / E[c * (GB + 1) + c];
            for (int rr = c + 1; rr < GB; ++rr) {
              double acc = 0.0;
              for (int ss = c; ss < rr; ++ss) acc += E[rr * (GB + 1) + ss] * Li[ss * (GB + 1) + c];
              Li[rr * (GB + 1) + c] = -acc / E[rr * (GB + 1) + rr];
            }
          }
          __syncthreads();
          for (int q = tid; q < GB * mp; q += EW) {
            const int b = q / mp, c = q - b * mp;
            double v = 0.0;
            for (int a = 0; a <= b; ++a) v += Li[b * (GB + 1) + a] * QJ[a * mp + c];
            bool dr = false;
            for (int z2 = 0; z2 < (ndrop < 16 ? ndrop : 16); ++z2) dr |= dropped[z2] == j0 + b;
            QI[b * mp + c] = dr ? 0.0 : v;   // QI is free here (I == J is the last of the loop)
          }
          __syncthreads();
          for (int q = tid; q < GB * mp; q += EW) QJ[q] = QI[q];
        } else {
          // Q_J[b] -= sum_a E[a][b] Q_I[a]
          for (int q = tid; q < GB * mp; q += EW) {
            const int b = q / mp, c = q - b * mp;
            double corr = 0.0;
            for (int a = 0; a < in; ++a) corr += E[a * (GB + 1) + b] * QI[a * mp + c];
            QJ[q] = QJ[q] - corr;
          }
        }
      }
      __syncthreads();
      for (int q = tid; q < jn * m; q += EW) {
        const int a = q / m, c = q - a * m;
        A[(int64_t)(j0 + a) * lda + c] = QJ[a * mp + c];
      }
      __threadfence_block();
    }
    __syncthreads();
    if (ndrop > 16) eflag = 1;
    // dropped rows: a unit vector made orthogonal (twice) to every other row spans what the others
    // leave of the eigenspace -- an eigenvector when they are eigenvectors
    for (int z2 = 0; z2 < (ndrop < 16 ? ndrop : 16); ++z2) {
      const int t = dropped[z2];
      lds_t* u = QI;   // [mp]
      lds_t* cf = QJ;  // coefficients [m]
      for (int tr = 0; tr < 4; ++tr) {
        const int e1 = (t * 131 + 7 + 53 * tr) % m;
        for (int c = tid; c < mp; c += EW) u[c] = c == e1 ? 1.0 : 0.0;
        __syncthreads();
        for (int rep = 0; rep < 2; ++rep) {
          for (int rr = w; rr < m; rr += NW) {   // cf[rr] = q_rr . u (row t itself is zero)
            double acc = 0.0;
            for (int c = lane; c < m; c += 64) acc += A[(int64_t)rr * lda + c] * u[c];
            acc = riptrm_wave::wave_sum(acc);
            if (lane == 0) cf[rr] = rr == t ? 0.0 : acc;
          }
          __syncthreads();
          for (int c = tid; c < m; c += EW) {
            double acc = 0.0;
            for (int rr = 0; rr < m; ++rr) acc += cf[rr] * A[(int64_t)rr * lda + c];
            u[c] = u[c] - acc;
          }
          __syncthreads();
        }
        double nn = 0.0;
        for (int c = lane; c < m; c += 64) nn += u[c] * u[c];
        nn = riptrm_wave::wave_sum(nn);   // every wave the same
        if (nn > 1e-2) {   // uniform
          const double inv = 1.0 / sqrt(nn);
          for (int c = tid; c < m; c += EW) A[(int64_t)t * lda + c] = u[c] * inv;
          __threadfence_block();
          __syncthreads();
          break;
        }
        if (tr == 3 && tid == 0) eflag = 1;
        __syncthreads();
      }
      if (tid == 0) again = 1;   // verify with another sweep
    }
    __syncthreads();
    if (!again) break;   // uniform
    }
    if (tid == 0 && eflag) infos[k] = 2;
  }
}

}  // namespace riptrm_eig
