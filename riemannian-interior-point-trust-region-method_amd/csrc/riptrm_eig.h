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

constexpr int EW = 512;                    // threads per matrix (the default; k_eig_lds<TW> takes 512 or 1024)
constexpr int EIG_LDS_MAX = 199;           // packed lower triangle + two vectors fit 160 KiB
constexpr int EIG_MAX_M = 256;             // four elements per lane in the back-transformation

__host__ __device__ constexpr int poff(int i) { return i * (i + 1) / 2; }
__host__ __device__ constexpr int vpad_eig(int m) { return (m + 7) / 8 * 8; }
constexpr int GB = 32;                     // row block of the Gram-Schmidt phase
constexpr int ZB = 64;                     // eigenvectors per block of the twisted + back-transform phase
constexpr int RB = 16;                     // reflectors staged in LDS at a time
__host__ __device__ constexpr int ms_of(int m) { return vpad_eig(m) + 1; }   // odd LDS row stride
__host__ __device__ constexpr size_t smax(size_t a, size_t b) { return a > b ? a : b; }
// compact eigenvectors (vectors = 2, no back-transformation): blocks of zc_of(m) vectors, row stride
// msc_of(m) (odd), as many as fit beside d and e
__host__ __device__ constexpr int msc_of(int m) { return m | 1; }
__host__ __device__ constexpr int zc_of(int m) {
  return m < (20480 - 2 * vpad_eig(m) - 16) / msc_of(m) ? m : (20480 - 2 * vpad_eig(m) - 16) / msc_of(m);
}
// doubles before d / e / tau: the packed triangle (phase 1), a ZB-vector block + a reflector stage
// (vectors = 1) or a zc-vector block (vectors = 2)
__host__ __device__ constexpr size_t de_off(int m) {
  return smax(smax((size_t)poff(m), (size_t)(ZB + RB) * ms_of(m)), (size_t)zc_of(m) * msc_of(m));
}
// the reflectors in HBM (vectors != 0): reflector i (v_{i+1} = 1, ..., v_{m-1}) contiguous from
// refl_col(m, i), then tau from refl_tau(m); m (m + 1) / 2 doubles in all, rounded to 8
__host__ __device__ constexpr int refl_col(int m, int i) { return i * (m - 1) - i * (i - 1) / 2; }
__host__ __device__ constexpr int refl_tau(int m) { return m * (m - 1) / 2; }
__host__ __device__ constexpr size_t refl_doubles(int m) { return ((size_t)poff(m) + 7) / 8 * 8; }
// tau (phase 4 only): in the triangle's space behind the vector block + stage when that fits (m = 199:
// the triangle is dead by then), else behind d and e
__host__ __device__ constexpr size_t tau_off(int m) {
  return (size_t)(ZB + RB) * ms_of(m) + vpad_eig(m) <= de_off(m) ? (size_t)(ZB + RB) * ms_of(m)
                                                                   : de_off(m) + 2 * (size_t)vpad_eig(m);
}
// dynamic LDS: phases 1-4 (packed triangle or vector block + stage, then d, e, tau), or phase 5
// (two GB-row blocks + their Gram and its Cholesky inverse)
__host__ __device__ constexpr size_t eig_lds_bytes(int m) {
  return smax(smax(de_off(m) + 2 * (size_t)vpad_eig(m), tau_off(m) + vpad_eig(m)),
              2 * (size_t)GB * ms_of(m) + 2 * GB * (GB + 1)) * sizeof(double);
}
static_assert(eig_lds_bytes(EIG_LDS_MAX) <= 160 * 1024, "EIG_LDS_MAX exceeds the LDS");

typedef __attribute__((address_space(3))) double lds_t;

// 1 / q by v_rcp_f64 and two Newton steps (a shorter dependent chain than the IEEE division)
__device__ __forceinline__ double rcp_nr(double q) {
  double r = __builtin_amdgcn_rcp(q);
  double t = fma(-q, r, 1.0);
  r = fma(r, t, r);
  t = fma(-q, r, 1.0);
  return fma(r, t, r);
}

// the number of eigenvalues of T (diagonal d, off-diagonal e) below x (Sturm count, LAPACK dlaneg's
// recurrence with pivmin guarding zero pivots).  (A division-free form -- the sign changes of
// p_j = (d_j - x) p_{j-1} - e_{j-1}^2 p_{j-2}, rescaled every four steps -- measured 6-10% slower: it
// issues more instructions per step, and the counts are issue-bound, not latency-bound.)
__device__ __forceinline__ int sturm_count(const lds_t* d, const lds_t* e, int m, double x, double pivmin) {
  double q = d[0] - x;
  if (fabs(q) < pivmin) q = -pivmin;
  int c = q < 0.0;
  int j = 1;
  for (; j + 3 < m; j += 4) {   // the next four entries' loads issued ahead of the dependent chain
    const double d0 = d[j], d1 = d[j + 1], d2 = d[j + 2], d3 = d[j + 3];
    const double f0 = e[j - 1], f1 = e[j], f2 = e[j + 1], f3 = e[j + 2];
    q = (d0 - x) - (f0 * f0) * rcp_nr(q);
    if (fabs(q) < pivmin) q = -pivmin;
    c += q < 0.0;
    q = (d1 - x) - (f1 * f1) * rcp_nr(q);
    if (fabs(q) < pivmin) q = -pivmin;
    c += q < 0.0;
    q = (d2 - x) - (f2 * f2) * rcp_nr(q);
    if (fabs(q) < pivmin) q = -pivmin;
    c += q < 0.0;
    q = (d3 - x) - (f3 * f3) * rcp_nr(q);
    if (fabs(q) < pivmin) q = -pivmin;
    c += q < 0.0;
  }
  for (; j < m; ++j) {
    const double ej = e[j - 1];
    q = (d[j] - x) - (ej * ej) * rcp_nr(q);
    if (fabs(q) < pivmin) q = -pivmin;
    c += q < 0.0;
  }
  return c;
}

// The eigenvector of T (d, e; split where e_j = 0) for eigenvalue t (lt = ev[t], ev ascending) into
// Z[0 .. m): the twisted factorisation of T - lt I (LAPACK dlar1v's), z_r = 1 at the twist r where
// |gamma_r| is least.  Numerically equal eigenvalues (within delta) take distinct blocks of the split T:
// member kk of the run i0 .. t takes the block where the running count of block eigenvalues in
// [lt - delta, lt + delta] passes kk.  Passes: forward (the Sturm counts at lt -+ delta and D+, which
// restarts at every split: three independent chains), backward over the block (D- and gamma; D- over
// D+), forward again below the twist (D+), then the solve outward from r and the normalisation.
__device__ __forceinline__ void twisted_vector(lds_t* Z, const lds_t* d, const lds_t* e, const double* ev, int m, int t,
                                               double delta, double pivmin) {
  const double lt = ev[t];
  int i0 = t;
  while (i0 > 0 && lt - ev[i0 - 1] <= delta) --i0;
  const int kk = t - i0;
  const double xa = lt - delta, xb = lt + delta;
  int blo = 0, bhi = m - 1, acc = 0, bs = 0, ca = 0, cb = 0;
  bool found = false;
  double qa = 0.0, qb = 0.0, dp = 0.0;
  for (int j = 0; j < m; ++j) {
    const bool start = j == bs;
    const double dj = d[j];
    const double ej2 = start ? 0.0 : e[j - 1] * e[j - 1];
    qa = (dj - xa) - (start ? 0.0 : ej2 * rcp_nr(qa));
    qb = (dj - xb) - (start ? 0.0 : ej2 * rcp_nr(qb));
    dp = (dj - lt) - (start ? 0.0 : ej2 * rcp_nr(dp));
    if (fabs(qa) < pivmin) qa = -pivmin;
    if (fabs(qb) < pivmin) qb = -pivmin;
    if (fabs(dp) < pivmin) dp = -pivmin;
    Z[j] = dp;
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
  // gamma_j = D+_j + D-_j - (d_j - lt); gamma_bhi = D+_bhi
  double dm = d[bhi] - lt;
  if (fabs(dm) < pivmin) dm = -pivmin;
  double best = fabs(Z[bhi]);
  int r = bhi;
  Z[bhi] = dm;
  for (int j = bhi - 1; j >= blo; --j) {
    const double ej = e[j];
    const double djl = d[j] - lt;
    dm = djl - (ej * ej) * rcp_nr(dm);
    if (fabs(dm) < pivmin) dm = -pivmin;
    const double g = fabs(Z[j] + dm - djl);
    Z[j] = dm;
    if (g < best) {
      best = g;
      r = j;
    }
  }
  if (r > blo) {   // D+ below the twist
    dp = d[blo] - lt;
    if (fabs(dp) < pivmin) dp = -pivmin;
    Z[blo] = dp;
    for (int j = blo + 1; j < r; ++j) {
      const double ej = e[j - 1];
      dp = (d[j] - lt) - (ej * ej) * rcp_nr(dp);
      if (fabs(dp) < pivmin) dp = -pivmin;
      Z[j] = dp;
    }
  }
  double z = 1.0, nrm = 1.0;
  for (int j = r + 1; j <= bhi; ++j) {   // z_j = -(e_{j-1} / D-_j) z_{j-1}
    z = -(e[j - 1] / Z[j]) * z;
    Z[j] = z;
    nrm += z * z;
  }
  z = 1.0;
  for (int j = r - 1; j >= blo; --j) {   // z_j = -(e_j / D+_j) z_{j+1}
    z = -(e[j] / Z[j]) * z;
    Z[j] = z;
    nrm += z * z;
  }
  Z[r] = 1.0;
  const double inv = 1.0 / sqrt(nrm);
  for (int j = 0; j < m; ++j) Z[j] = (j < blo || j > bhi) ? 0.0 : Z[j] * inv;
}

// Block Gram-Schmidt algebra on the matrix cores (v_mfma_f64_16x16x4_f64: A operand lane (i = l & 15,
// k = l >> 4), B operand (k = l >> 4, j = l & 15), D rows 4 q + (l >> 4), column l & 15).
typedef double eig_d4 __attribute__((ext_vector_type(4)));
// Out[b][c] = (SUB ? Base[b][c] : 0) -+ sum_a W[b][a] X[a][c] for the GB x m block (b < GB, c < m): W is
// GB x GB at stride GB + 1 (TRANS: W[b][a] read as W[a][b]), X, Out, Base GB x m at stride mp (X's
// columns past m are zero).  (2 x ceil(m / 16)) 16 x 16 tiles dealt to the NWV waves, K = GB in eight steps.
template <bool TRANS, bool SUB, int NWV>
__device__ __forceinline__ void gs_wmul(lds_t* Out, const lds_t* Base, const lds_t* W, const lds_t* X, int mp, int m,
                                        int w, int lane) {
  const int c16 = lane & 15, kk = lane >> 4;
  const int nct = (m + 15) / 16;
  for (int t = w; t < 2 * nct; t += NWV) {
    const int b0 = (t & 1) * 16, c0 = (t >> 1) * 16;
    const int col = c0 + c16 < mp ? c0 + c16 : mp - 1;
    eig_d4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int a0 = 0; a0 < GB; a0 += 8) {
      const double av0 = TRANS ? W[(a0 + kk) * (GB + 1) + b0 + c16] : W[(b0 + c16) * (GB + 1) + a0 + kk];
      const double av1 = TRANS ? W[(a0 + 4 + kk) * (GB + 1) + b0 + c16] : W[(b0 + c16) * (GB + 1) + a0 + 4 + kk];
      const double bv0 = X[(a0 + kk) * mp + col], bv1 = X[(a0 + 4 + kk) * mp + col];
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av0, bv0, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av1, bv1, acc1, 0, 0, 0);
    }
    if (c0 + c16 < m) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int b = b0 + kk + 4 * q;
        const double v = acc0[q] + acc1[q];
        Out[b * mp + c0 + c16] = SUB ? Base[b * mp + c0 + c16] - v : v;
      }
    }
  }
}

// rows r0 .. r0 + rn - 1 of A (m columns, leading dimension lda) -> X [GB][mp], zero past rn / m:
// unconditional loads of clamped addresses, eight in flight per thread, (row, column) stepped
// incrementally (NT threads = qs mp + rs)
template <int NT>
__device__ __forceinline__ void gs_load(lds_t* X, const double* A, int64_t lda, int r0, int rn, int m, int mp, int tid) {
  const int tot = GB * mp, qs = NT / mp, rs = NT - qs * mp;
  int a0 = tid / mp, c0 = tid - (tid / mp) * mp;
  for (int q0 = 0; q0 < tot; q0 += NT * 8) {
    double v[8];
    int aa[8], cc[8];
    int a = a0, c = c0;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      aa[u] = a;
      cc[u] = c;
      v[u] = A[(a < rn && c < m) ? (int64_t)(r0 + a) * lda + c : (int64_t)r0 * lda];
      c += rs;
      a += qs;
      if (c >= mp) {
        c -= mp;
        ++a;
      }
    }
    a0 = a;
    c0 = c;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (aa[u] < GB) X[aa[u] * mp + cc[u]] = (aa[u] < rn && cc[u] < m) ? v[u] : 0.0;
  }
}

// Matrix k = blockIdx.x: the m x m symmetric matrix at A0 + k a_stride (leading dimension lda; the
// lower triangle is read) -> eigenvalues ascending at ev0 + k ev_stride and, with vectors, in the
// rows of the same matrix: vectors = 1 the eigenvectors of A; vectors = 2 those of the tridiagonal
// T = H^T A H (compact form: an eigenvector of A is H z = H_0 ... H_{m-2} z, applied by the caller,
// k_refl_apply).  Scratch per matrix (two vectors of >= m doubles, k sc_stride apart): d at d0, e at
// e0; the reflectors and tau (refl_doubles(m), layout refl_col / refl_tau) at R0 + k r_stride.
// PH selects the phases one launch runs (bit 0 tridiagonalisation, 1 eigenvalues, 2 eigenvectors of T,
// 3 orthogonality; 15: all, one workgroup per matrix).  The split launches (k_eig_split) run them as
// four kernels so the eigenvalue and eigenvector phases spread over gridDim.y workgroups per matrix
// (eigenvalues / vectors m y / Y .. m (y + 1) / Y of workgroup y): d and the split e travel through
// the slot (d0, e0), the eigenvalues through ev, the vectors through A.
template <int TW, int PH = 15>
__global__ void __launch_bounds__(TW) k_eig_lds(double* A0, int64_t a_stride, int lda, int m, double* ev0,
                                                int64_t ev_stride, double* d0, double* e0, int64_t sc_stride,
                                                double* R0, int64_t r_stride, int32_t* infos, int vectors,
                                                long long* stamps = nullptr) {
  constexpr int EW = TW;
  static_assert(TW == 512 || TW == 1024, "k_eig_lds: 512 or 1024 threads");
  extern __shared__ double smem[];
  __shared__ double scal[2];
  __shared__ int bad;
  lds_t* P = (lds_t*)smem;                    // packed lower triangle, row i at poff(i)
  lds_t* vb = P + de_off(m);                  // the reflector (phase 1), then d (phases 2-3)
  lds_t* pb = vb + vpad_eig(m);               // p (phase 1), then e (phases 2-3)
  lds_t* tb = P + tau_off(m);                 // tau (phase 4)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  constexpr int NW = EW / 64;
  const int k = blockIdx.x;
  double* A = A0 + (int64_t)k * a_stride;
  double* ev = ev0 + (int64_t)k * ev_stride;
  double* dg = d0 + (int64_t)k * sc_stride;
  double* eg = e0 + (int64_t)k * sc_stride;
  double* Rg = R0 + (int64_t)k * r_stride;
  const double eps = DBL_EPSILON;
  const int ylo = (int)((int64_t)m * blockIdx.y / gridDim.y), yhi = (int)((int64_t)m * (blockIdx.y + 1) / gridDim.y);
  long long* stp = (PH == 15 && stamps && tid == 0) ? stamps + (int64_t)k * 8 : nullptr;   // phase clocks (diagnostics)
  if constexpr ((PH & 1) == 0) {   // a later phase: d, split e from the slot
    if (infos[k] == 1) return;     // non-finite input: the eigenvalues are NaN already
    for (int i = tid; i < m; i += EW) {
      vb[i] = dg[i];
      if (i < m - 1) pb[i] = eg[i];
    }
    __syncthreads();
  } else {
  if (tid == 0) bad = 0;
  if (stp) stp[0] = clock64();
  __syncthreads();
  // the lower triangle into the packed LDS image, eight loads in flight per thread (a load-then-store
  // loop waits out one memory latency per element); element q = i m + j of thread tid, u-th of a
  // batch, stepped incrementally (EW = qs m + rs)
  {
    const int mm2 = m * m, qs = EW / m, rs = EW - qs * m;
    int i0 = tid / m, j0 = tid - (tid / m) * m;   // element tid
    for (int q0 = 0; q0 < mm2; q0 += EW * 8) {
      double v[8];
      int ii[8], jj[8];
      int i = i0, j = j0;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        ii[u] = i;
        jj[u] = j;
        // an unconditional load of a clamped address (a guarded load is sunk into a branch that waits)
        v[u] = A[(i < m && j <= i) ? (int64_t)i * lda + j : 0];
        j += rs;
        i += qs;
        if (j >= m) {
          j -= m;
          ++i;
        }
      }
      i0 = i;
      j0 = j;
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (ii[u] < m && jj[u] <= ii[u]) {
          if (!isfinite(v[u])) bad = 1;
          P[poff(ii[u]) + jj[u]] = v[u];
        }
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
  long long acc_refl = 0, acc_symv = 0, tq = 0;   // stamps: cycles in the reflector / symv sections
  for (int i = 0; i < m - 1; ++i) {
    const int r = m - i - 1;   // the trailing rows / columns i + 1 .. m - 1
    if (stp) tq = clock64();
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
        if (vectors) Rg[refl_col(m, i) + l] = v;
      }
      if (lane == 0) {
        scal[0] = tau;
        P[poff(i + 1) + i] = beta;
        eg[i] = beta;
        if (vectors) Rg[refl_tau(m) + i] = tau;
      }
    }
    __syncthreads();
    if (stp) {
      const long long t1 = clock64();
      acc_refl += t1 - tq;
      tq = t1;
    }
    const double tau = scal[0];
    if (tau != 0.0) {   // uniform
      // p = tau A22 v: TPR threads per row (EW / 256, or 8 once r <= 128 on 1024 threads), each over
      // a part of the row -- its part of the packed row (contiguous) and, past the diagonal, its part
      // of the column below the diagonal (an incremental offset, no multiplies) -- then the partners'
      // parts (DPP xor 1, xor 2, half mirror)
      {
        const int TPR = (EW == 1024 && r <= 128) ? 8 : EW / 256;   // uniform
        const int l = tid / TPR, h = tid & (TPR - 1);
        const int half = (r + TPR - 1) / TPR;
        double acc0 = 0.0, acc1 = 0.0;
        if (l < r) {
          const int gl = i + 1 + l;
          const int jb = h * half, je = min(r, jb + half);
          const int jm = max(jb, min(je, l + 1));
          const lds_t* rowp = P + poff(gl) + i + 1;
          double acc2 = 0.0, acc3 = 0.0;
          int j = jb;
          for (; j + 3 < jm; j += 4) {
            acc0 += rowp[j] * vb[j];
            acc1 += rowp[j + 1] * vb[j + 1];
            acc2 += rowp[j + 2] * vb[j + 2];
            acc3 += rowp[j + 3] * vb[j + 3];
          }
          for (; j < jm; ++j) acc0 += rowp[j] * vb[j];
          int off = poff(i + 1 + j) + gl;   // element (i + 1 + j, gl) of the packed lower triangle
          for (; j + 3 < je; j += 4) {
            const int o1 = off + i + 1 + j + 1;   // poff(k + 1) = poff(k) + k + 1
            const int o2 = o1 + i + 1 + j + 2;
            const int o3 = o2 + i + 1 + j + 3;
            acc0 += P[off] * vb[j];
            acc1 += P[o1] * vb[j + 1];
            acc2 += P[o2] * vb[j + 2];
            acc3 += P[o3] * vb[j + 3];
            off = o3 + i + 1 + j + 4;
          }
          for (; j < je; ++j) {
            acc0 += P[off] * vb[j];
            off += i + 1 + j + 1;
          }
          acc0 = (acc0 + acc1) + (acc2 + acc3);
          acc1 = 0.0;
        }
        double acc = acc0 + acc1;
        acc = acc + riptrm_wave::dpp<riptrm_wave::DPP_XOR1>(acc);
        if (TPR >= 4) acc = acc + riptrm_wave::dpp<riptrm_wave::DPP_XOR2>(acc);
        if (TPR == 8) acc = acc + riptrm_wave::dpp<riptrm_wave::DPP_HALF_MIRROR>(acc);   // lane ^ 7 of the 8
        if (l < r && h == 0) pb[l] = tau * acc;
      }
      __syncthreads();
      if (stp) acc_symv += clock64() - tq;
      // alpha2 = -tau (p . v) / 2 (every wave the same tree), w = p + alpha2 v, A22 -= v w^T + w v^T:
      // lanes over columns (v_j, w_j in registers), waves over rows
      double s = 0.0;
      for (int l = lane; l < r; l += 64) s += pb[l] * vb[l];
      s = riptrm_wave::wave_sum(s);
      const double a2 = -0.5 * tau * s;
      double vj[4], wj[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = lane + 64 * q;
        vj[q] = j < r ? vb[j] : 0.0;
        wj[q] = j < r ? pb[j] + a2 * vj[q] : 0.0;
      }
      for (int l = w; l < r; l += NW) {
        const double vl = vb[l], wl = pb[l] + a2 * vl;
        lds_t* row = P + poff(i + 1 + l) + i + 1;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int j = lane + 64 * q;
          if (j <= l) row[j] = row[j] - (vl * wj[q] + wl * vj[q]);
        }
      }
    }
    __syncthreads();
  }
  if (stp) {
    stp[1] = clock64();
    stp[6] = acc_refl;
    stp[7] = acc_symv;
  }
  // d, e into LDS (vb, pb) and the slot
  for (int i = tid; i < m; i += EW) {
    const double di = P[poff(i) + i];
    vb[i] = di;
    dg[i] = di;
    if (i < m - 1) pb[i] = P[poff(i + 1) + i];
  }
  __syncthreads();
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
  if constexpr (PH == 1) {   // the split e for the later launches
    for (int j = tid; j < m - 1; j += EW) eg[j] = pb[j];
    return;
  }
  }   // PH & 1
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
  // multisection: kq (1, 2, 4 or 8) consecutive lanes per eigenvalue test kq points of its interval
  // at once and keep the sub-interval the counts select (the same on every lane of the group)
  if constexpr ((PH & 2) != 0) {
    // ~512 lanes per workgroup: kq = 2 for all 199 eigenvalues of one launch (the counts are
    // issue-bound there: more lanes only add work), 8 for the ~50 of a split launch's workgroup (every
    // path the service and riptrm_sym_eig take is split: the same eigenvalues with or without vectors)
    int kq = 512 / (yhi - ylo);
    kq = kq >= 8 ? 8 : (kq >= 4 ? 4 : (kq >= 2 ? 2 : 1));
    const int ei = ylo + tid / kq, sub = tid % kq, base = (int)(threadIdx.x & 63) - sub;
    if (ei < yhi) {
      double lo = glo - fudge, hi = ghi + fudge;
      for (int it = 0; it < 128; ++it) {
        const double tol = fmax(2.0 * eps * fmax(fabs(lo), fabs(hi)), eps * tnorm);
        if (hi - lo <= tol) break;   // uniform over the group
        const double step = (hi - lo) / (kq + 1);
        const double x = lo + step * (sub + 1);
        const int c = (x > lo && x < hi) ? sturm_count(d, e, m, x, pivmin) : (x <= lo ? 0 : m);
        double nlo = lo, nhi = hi;
        for (int s2 = 0; s2 < kq; ++s2) {
          const int cs = __shfl(c, base + s2);
          const double xs = lo + step * (s2 + 1);
          if (cs > ei) nhi = fmin(nhi, xs);
          else nlo = fmax(nlo, xs);
        }
        if (nlo >= nhi || (nlo == lo && nhi == hi)) break;
        lo = nlo;
        hi = nhi;
      }
      if (sub == 0) ev[ei] = 0.5 * (lo + hi);
    }
  }
  __threadfence_block();
  __syncthreads();
  if (stp) stp[2] = clock64();
  if (!vectors || (PH & 12) == 0) return;

  // ---- 3 + 4. per block of eigenvectors, in LDS: the twisted vectors of T, then (vectors = 1)
  // q = H_0 ... H_{m-2} z
  const int ms = ms_of(m);
  const bool cpt = vectors == 2;
  const int zs = cpt ? msc_of(m) : ms;   // row stride of the block
  const int zb = cpt ? zc_of(m) : ZB;    // vectors per block
  lds_t* Zb = P;                         // [zb][zs]
  lds_t* St = P + ZB * ms;               // [RB][ms]: reflectors i_hi - RB + 1 .. i_hi, v_i[j] dense
  if (!cpt)
    for (int i = tid; i < m - 1; i += EW) tb[i] = Rg[refl_tau(m) + i];
  const double delta = 16.0 * eps * tnorm;
  for (int t0 = (PH & 4) ? ylo : m; t0 < yhi; t0 += zb) {
    __syncthreads();   // the previous block's rows are out, tau is in
    if (tid < zb && t0 + tid < yhi) twisted_vector(Zb + tid * zs, d, e, ev, m, t0 + tid, delta, pivmin);
    // back-transformation of the block: reflectors i = m - 2 .. 0, RB at a time staged from Rg; eight
    // lanes per vector (lane c8 takes j = c8, c8 + 8, ...: its own elements only, so the wave needs
    // no LDS ordering between reflectors), the dot product closed by three butterfly steps
    const int u = tid >> 3, c8 = tid & 7;
    for (int ihi = vectors == 1 ? m - 2 : -1; ihi >= 0; ihi -= RB) {
      const int ilo = ihi - RB + 1 > 0 ? ihi - RB + 1 : 0;
      __syncthreads();   // the block's vectors are in; the previous stage is done with
      for (int q = tid; q < (ihi - ilo + 1) * ms; q += EW) {
        const int ii = q / ms, j = q - ii * ms;
        const int i = ilo + ii;
        St[q] = (j > i && j < m) ? Rg[refl_col(m, i) + j - i - 1] : 0.0;
      }
      __syncthreads();
      if (u < ZB && t0 + u < yhi) {   // (1024 threads: the upper half idles)
        lds_t* Zu = Zb + u * zs;
        for (int i = ihi; i >= ilo; --i) {
          const double tau = tb[i];
          if (tau == 0.0) continue;   // uniform
          const lds_t* vi = St + (i - ilo) * ms;
          const int jb = i + 1 + ((c8 - (i + 1)) & 7);   // my first j >= i + 1
          double s0 = 0.0, s1 = 0.0;
          int j = jb;
          for (; j + 8 < m; j += 16) {
            s0 += vi[j] * Zu[j];
            s1 += vi[j + 8] * Zu[j + 8];
          }
          if (j < m) s0 += vi[j] * Zu[j];
          double sv = s0 + s1;
          sv = sv + riptrm_wave::dpp<riptrm_wave::DPP_XOR1>(sv);
          sv = sv + riptrm_wave::dpp<riptrm_wave::DPP_XOR2>(sv);
          sv = sv + riptrm_wave::dpp<riptrm_wave::DPP_HALF_MIRROR>(sv);   // lane ^ 7 within the row of 8
          const double f = tau * sv;
          for (j = jb; j < m; j += 8) Zu[j] = Zu[j] - f * vi[j];
        }
      }
    }
    __syncthreads();
    for (int q = tid; q < zb * m; q += EW) {
      const int uu = q / m, c = q - uu * m;
      if (t0 + uu < yhi) A[(int64_t)(t0 + uu) * lda + c] = Zb[uu * zs + c];
    }
  }
  __threadfence_block();
  __syncthreads();
  if (stp) stp[3] = stp[4] = clock64();
  if constexpr ((PH & 8) == 0) return;

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
    const int mp = vpad_eig(m) + 1;        // odd row stride: a wave's 32 rows at one column hit distinct banks
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
      gs_load<EW>(QJ, A, lda, j0, jn, m, mp, tid);
      for (int I = 0; I <= J; ++I) {
        const int i0b = I * GB, in = min(GB, m - i0b);
        // eigenvalues sorted: block I is close to block J iff its last one is within ctol of J's first
        if (I < J && ev[j0] - ev[i0b + in - 1] > ctol) continue;   // uniform
        __syncthreads();
        if (I < J)
          gs_load<EW>(QI, A, lda, i0b, in, m, mp, tid);
        __syncthreads();
        const lds_t* QA = I < J ? QI : QJ;
        // E[a][b] = Q_I[a] . Q_J[b] on the matrix cores: waves 0-3 one 16 x 16 tile each, the k steps
        // over the columns (zero past m) alternating between two accumulators
        if (w < 4) {
          const int a0 = (w >> 1) * 16, b0 = (w & 1) * 16, c16 = lane & 15, kq = lane >> 4;
          eig_d4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
          const lds_t* xa = QA + (a0 + c16) * mp + kq;
          const lds_t* xb = QJ + (b0 + c16) * mp + kq;
          int k0 = 0;
          for (; k0 + 4 < m; k0 += 8) {
            acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[k0], xb[k0], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[k0 + 4], xb[k0 + 4], acc1, 0, 0, 0);
          }
          if (k0 < m) acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(xa[k0], xb[k0], acc0, 0, 0, 0);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int a = a0 + kq + 4 * q, b = b0 + c16;
            const double sacc = acc0[q] + acc1[q];
            const double eab = (I == J && a == b) ? sacc - 1.0 : sacc;
            E[a * (GB + 1) + b] = eab;
            if (a < in && b < jn && fabs(eab) > 1e-8) again = 1;
          }
        }
        __syncthreads();
        __shared__ int bigE;
        if (I == J) {
          if (tid == 0) bigE = 0;
          __syncthreads();
          for (int q = tid; q < GB * GB; q += EW) {
            const int a = q / GB, b = q - a * GB;
            if (a < jn && b < jn && fabs(E[a * (GB + 1) + b]) > 1e-6) bigE = 1;
          }
          __syncthreads();
        }
        if (I == J && !bigE) {   // uniform: |E| <= 1e-6, first order (the dropped terms are <= 1e-12)
          // Q_J[b] <- Q_J[b] - sum_{a < b} E[a][b] Q_J[a] - E[b][b] / 2 Q_J[b] = Q_J - W Q_J with
          // W[b][a] = E[a][b] (a < b), E[b][b] / 2 (a = b)
          lds_t* Wm = E + GB * (GB + 1);
          for (int q = tid; q < GB * GB; q += EW) {
            const int b = q / GB, a = q - b * GB;
            Wm[b * (GB + 1) + a] = a < b ? E[a * (GB + 1) + b] : (a == b ? 0.5 * E[b * (GB + 1) + b] : 0.0);
          }
          __syncthreads();
          gs_wmul<false, true, EW / 64>(QI, QJ, Wm, QJ, mp, m, w, lane);
          __syncthreads();
          for (int q = tid; q < GB * mp; q += EW)   // columns past m stay zero (the Gram's k steps read them)
            if (q - (q / mp) * mp < m) QJ[q] = QI[q];
        } else if (I == J) {
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
          gs_wmul<false, false, EW / 64>(QI, QI, Li, QJ, mp, m, w, lane);   // QI is free (I == J is the last)
          __syncthreads();
          for (int q = tid; q < GB * mp; q += EW) {
            const int b = q / mp;
            if (q - b * mp >= m) continue;   // columns past m stay zero
            bool dr = false;
            for (int z2 = 0; z2 < (ndrop < 16 ? ndrop : 16); ++z2) dr |= dropped[z2] == j0 + b;
            QJ[q] = dr ? 0.0 : QI[q];
          }
        } else {
          // Q_J[b] -= sum_a E[a][b] Q_I[a] (rows of Q_I past `in` are zero)
          gs_wmul<true, true, EW / 64>(QJ, QJ, E, QI, mp, m, w, lane);
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
        if (nn > 1e-8) {   // uniform (a unit vector's share of a one-dimensional complement is ~1 / m)
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
  if (stp) stp[5] = clock64();
}

}  // namespace riptrm_eig
