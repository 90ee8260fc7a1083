// riptrm_tri.h — Exact_RepMat's subproblem above the one-workgroup eigensolver's orders
// (riptrm_eig::EIG_LDS_MAX < m <= TRI_MAX), without eigenvectors: the matrix is reduced to a
// tridiagonal T = H^T A H by workgroups that hold its rows in REGISTERS across the chip, and TRSgep
// (src/solver/RIPTRM.py:218-299) is solved in T's coordinates.
//
// Reference: TRSgep takes the rightmost eigenpair of a 2m x 2m pencil (scipy.linalg.eig, :251) and
// SciPy's CG for the interior candidate (:243-248); the second-order test takes the smallest
// eigenvalue of the same matrix (:599-617, scipy.linalg.eigh).  Rounds 3-5 ran rocSOLVER dsyevd on
// the m x m matrix above order 199 (25 ms per eigendecomposition at m = 999, 96% of the n = 1000
// Exact line's GPU time: profiles/r6_exact1000_rocsolver_rocprofv3_kernel_stats.csv).  Here:
//   1. k_tridiag_dist: dsytd2 (lower) on G = ceil(m / 8 RW) workgroups per matrix, row l on workgroup
//      l mod G (cyclic, so the shrinking trailing matrix stays balanced), each wave holding RW rows
//      with EL elements per lane in registers.  ONE exchange per column: every workgroup publishes
//      p_l = tau A v for its rows and the owner of row i + 1 publishes that row; each workgroup then
//      forms w = p - tau (p.v) v / 2, the next column c = row_{i+1} - (v w_{i+1} + w v_{i+1}) and its
//      reflector redundantly (the same arithmetic everywhere: bitwise the same values), and runs the
//      rank-two update of its rows fused with the next column's p.  The exchange is the k_persist
//      protocol: 16-byte granules {value, tag} written by one write-through store each, polled with
//      sc1 loads (MI355X_MICROARCH.md, persistent hand-offs), two parities, plus one arrival granule
//      per workgroup and pass so no workgroup overwrites a parity another still reads.
//   2. k_refl_big: b = H^T a (and x = H y at the end) with the reflectors from HBM, one wave.
//   3. k_tri_solve: the extreme eigenvalues of T by Sturm bisection (riptrm_eig.h's counts), the
//      hard-case test on lam_min's eigenvector (a twisted factorisation), the secular Newton of
//      k_secular with (T + lam I)^-1 applied by LDL^T solves instead of an eigenbasis, and SciPy's CG
//      on T y = -b (k_cg_diag's loop: the CG on A x = -a generates x_k = H y_k, the same iterate up to
//      rounding, O(m) per iteration).  A hard case (or a multiple smallest eigenvalue) sets a flag and
//      the host serves that subproblem with the eigendecomposition path instead.
#pragma once
#include <hip/hip_runtime.h>
#include <float.h>
#include <math.h>
#include "riptrm_eig.h"
#include "riptrm_wave.h"

namespace riptrm_tri {

#pragma clang fp contract(off)

using riptrm_eig::lds_t;

constexpr int TT = 512;                          // threads per tridiagonalisation workgroup
constexpr int TRI_MIN = riptrm_eig::EIG_LDS_MAX + 1;
constexpr int TRI_MAX = 1024;                    // (EL = 32 for 2048 spilled the rows to scratch)
constexpr unsigned long long TRI_TIMEOUT = 200000000ull;   // 2 s of the 100 MHz wall clock

// elements per lane (EL) and rows per wave (RW) of order m: 32 doubles of the matrix per lane
__host__ __device__ constexpr int tri_el(int m) { return m <= 256 ? 4 : (m <= 512 ? 8 : 16); }
__host__ __device__ constexpr int tri_rw(int m) { return 32 / tri_el(m); }
__host__ __device__ constexpr int tri_groups(int m) { return (m + 8 * tri_rw(m) - 1) / (8 * tri_rw(m)); }
// granules per matrix: 2 parities x [p: m][row: m][arrivals: G]
__host__ __device__ constexpr int64_t tri_par(int m) { return 2 * (int64_t)m + tri_groups(m); }
__host__ __device__ constexpr int64_t tri_granules(int m) { return 2 * tri_par(m); }

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ unsigned tag_check(unsigned lo, unsigned hi, unsigned pass) {
  return lo ^ hi ^ (pass * 0x9E3779B9u);
}
__device__ __forceinline__ void st_gran(__amdgpu_buffer_rsrc_t rs, int64_t g, double v, unsigned pass) {
  const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  const u32x4 q = {lo, hi, tag_check(lo, hi, pass), pass};
  __builtin_amdgcn_raw_buffer_store_b128(q, rs, (int)(g * 16), 0, 16);   // aux 16: sc1 (write-through)
}

struct TriArgs {
  int k0;                // matrix of blockIdx.y = 0
  const double* A0;      // matrix k at A0 + k a_stride (rows of lda doubles; the whole matrix is read)
  int64_t a_stride, lda;
  double *d0, *e0;       // d (m) and e (m - 1) of matrix k at + k de_stride
  int64_t de_stride;
  double* R0;            // reflectors + tau of matrix k at R0 + k r_stride (riptrm_eig refl_col / refl_tau)
  int64_t r_stride;
  int32_t* infos;        // per matrix (3: an exchange timed out)
  void* grid;            // granules, tri_granules(m) per launch slot (zeroed before the launch)
  int64_t grid_bytes;
  int m, G;
  long long* stamps;     // diagnostics (RIPTRM_TRI_STAMPS=1): workgroup 0 of matrix 0 accumulates clock64
                         // cycles in [0] the gather, [1] wave 0's section + barrier, [2] the update + publish
};

// the reflector of the column c[i+1 .. m) (dlarfg: H (alpha, x) = (beta, 0), v(i+1) = 1) into vo, by
// one wave (lane-strided sums, then the wave tree); returns tau, beta through the references
template <int EL>
__device__ __forceinline__ void make_reflector(const lds_t* c, int i, int m, lds_t* vo, int lane, double& tau,
                                               double& beta, double& scl) {
  double s = 0.0;
#pragma unroll
  for (int q = 0; q < EL; ++q) {
    const int j = lane + 64 * q;
    const double x = c[j];
    s += (j >= i + 2 && j < m) ? x * x : 0.0;
  }
  s = riptrm_wave::wave_sum(s);
  const double alpha = c[i + 1];
  tau = 0.0;
  beta = alpha;
  scl = 0.0;
  if (s != 0.0) {
    beta = -copysign(sqrt(alpha * alpha + s), alpha);
    tau = (beta - alpha) / beta;
    scl = 1.0 / (alpha - beta);
  }
#pragma unroll
  for (int q = 0; q < EL; ++q) {
    const int j = lane + 64 * q;
    vo[j] = (j <= i || j >= m) ? 0.0 : (j == i + 1 ? 1.0 : c[j] * scl);
  }
}

// a workgroup barrier that waits for this wave's LDS accesses only: the granule / reflector stores in
// flight need not complete here (__syncthreads() drains them with vmcnt(0): each write-through store is
// a round trip to memory, ~1.5 us of the step at m = 999 by the phase stamps)
__device__ __forceinline__ void bar_lds() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// dsytd2 (lower) of the m x m matrix of slot k0 + blockIdx.y on gridDim.x = G workgroups: d, e, the
// reflectors and tau into the slot.  Row l lives on workgroup l mod G, wave (l / G) mod 8, register
// row (l / G) / 8, lane j mod 64 holding columns j = lane + 64 q.
template <int EL, int RW>
__global__ void __launch_bounds__(TT) k_tridiag_dist(TriArgs a) {
  __shared__ double Vbuf[2][EL * 64];   // v_i and v_{i+1} (by step parity)
  __shared__ double GP[EL * 64];        // gathered p (written by the gather, read by wave 0 only)
  __shared__ double W[EL * 64];         // w = p + a2 v (wave 0 -> every wave after the barrier)
  __shared__ double C[EL * 64];         // gathered row i + 1, then the column c of step i + 1 (wave 0)
  // (a wave that finishes its rows early starts the next gather while others still read W, Vbuf: the
  // gather writes only GP and C, which nobody reads after the step's barrier)
  __shared__ double scal[2];
  __shared__ int failflag;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = blockIdx.x, ks = blockIdx.y, k = a.k0 + ks;
  if (tid == 0) failflag = 0;
  const int m = a.m, G = a.G;
  const double* A = a.A0 + (int64_t)k * a.a_stride;
  double* dv = a.d0 + (int64_t)k * a.de_stride;
  double* ev = a.e0 + (int64_t)k * a.de_stride;
  double* R = a.R0 + (int64_t)k * a.r_stride;
  const bool writer = g == (m - 1) % G;   // owns row m - 1, active to the last step: writes d, e, H
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.grid, 0, (int)a.grid_bytes, 0x00020000);
  const int64_t gbase = (int64_t)ks * tri_granules(m);
  const int64_t par = tri_par(m);

  // own rows into registers (unconditional loads of clamped addresses)
  double Ar[RW][EL];
  int rowid[RW];
#pragma unroll
  for (int s = 0; s < RW; ++s) {
    const int l = g + G * (w + 8 * s);
    rowid[s] = l;
#pragma unroll
    for (int q = 0; q < EL; ++q) {
      const int j = lane + 64 * q;
      const bool ok = l < m && j < m;   // the lower triangle (as dsytd2 'L' and riptrm_eig.h read it)
      Ar[s][q] = A[ok ? (j <= l ? (int64_t)l * a.lda + j : (int64_t)j * a.lda + l) : 0];
    }
  }
  // column 0 = row 0 of the input, its reflector (wave 0 of every workgroup)
  if (w == 0) {
#pragma unroll
    for (int q = 0; q < EL; ++q) {
      const int j = lane + 64 * q;
      C[j] = A[j < m ? (int64_t)j * a.lda : 0];   // column 0 of the lower triangle
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the wave's lanes exchange through LDS
    double tau, beta, scl;
    make_reflector<EL>((const lds_t*)C, 0, m, (lds_t*)Vbuf[0], lane, tau, beta, scl);
    if (lane == 0) scal[0] = tau;
    if (writer) {
      if (lane == 0) {
        dv[0] = C[0];
        ev[0] = beta;
        R[riptrm_eig::refl_tau(m) + 0] = tau;
      }
#pragma unroll
      for (int q = 0; q < EL; ++q) {
        const int j = lane + 64 * q;
        if (j >= 1 && j < m) R[riptrm_eig::refl_col(m, 0) + j - 1] = Vbuf[0][j];
      }
    }
  }
  __syncthreads();
  double tau_c = scal[0];
  // pass 1: p^(0)_l = tau_0 A_l. v_0 for own rows l >= 1, row 1 by its owner, this workgroup's arrival
  {
    const int64_t pb = gbase + (int64_t)(1 & 1) * par;
    double vq[EL];
#pragma unroll
    for (int q = 0; q < EL; ++q) vq[q] = Vbuf[0][lane + 64 * q];
#pragma unroll
    for (int s = 0; s < RW; ++s) {
      const int l = rowid[s];
      if (l >= 1 && l < m) {
        double acc = 0.0;
#pragma unroll
        for (int q = 0; q < EL; ++q) acc += (lane + 64 * q >= 1) ? Ar[s][q] * vq[q] : 0.0;
        const double p = tau_c * riptrm_wave::wave_sum(acc);
        if (lane == 0) st_gran(rs, pb + l, p, 1u);
        if (l == 1 && m > 1) {
#pragma unroll
          for (int q = 0; q < EL; ++q) {
            const int j = lane + 64 * q;
            if (j >= 1 && j < m) st_gran(rs, pb + m + j, Ar[s][q], 1u);
          }
        }
      }
    }
    if (tid == 0) st_gran(rs, pb + 2 * m + g, 0.0, 1u);
  }

  constexpr int NG = (2 * 64 * EL + 256 + TT - 1) / TT;   // granules polled per thread (upper bound)
  bool failed = false;
  long long* stp = (a.stamps && g == 0 && k == 0 && tid == 0) ? a.stamps : nullptr;
  long long acc0 = 0, acc1 = 0, acc2 = 0, tq = stp ? clock64() : 0, sa = 0, sb = 0, sc = 0, sd = 0;
  for (int i = 0; i <= m - 2; ++i) {
    const unsigned pass = (unsigned)(i + 1);
    const int64_t pb = gbase + (int64_t)(pass & 1) * par;
    const int r = m - i - 1;   // trailing indices i + 1 .. m - 1
    const int ng = 2 * r + G;
    // gather: p_j, row_{i+1}[j] (j > i) and every workgroup's arrival, polled until the tags say this pass
    {
      int pend = 0;
      int64_t gi[NG];
#pragma unroll
      for (int u = 0; u < NG; ++u) {
        const int t = tid + TT * u;
        int64_t gx = 0;
        if (t < r) gx = pb + i + 1 + t;
        else if (t < 2 * r) gx = pb + m + i + 1 + (t - r);
        else if (t < ng) gx = pb + 2 * m + (t - 2 * r);
        gi[u] = gx;
        if (t < ng) pend |= 1 << u;
      }
      const unsigned long long t0 = wall_clock64();
      while (true) {
        u32x4 qv[NG];
#pragma unroll
        for (int u = 0; u < NG; ++u)
          if (pend & (1 << u)) qv[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(gi[u] * 16), 0, 16);
#pragma unroll
        for (int u = 0; u < NG; ++u)
          if (pend & (1 << u)) {
            const u32x4 q = qv[u];
            if (q.w == pass && q.z == tag_check(q.x, q.y, pass)) {
              const int t = tid + TT * u;
              const double v = __hiloint2double((int)q.y, (int)q.x);
              if (t < r) GP[i + 1 + t] = v;
              else if (t < 2 * r) C[i + 1 + (t - r)] = v;
              pend &= ~(1 << u);
            }
          }
        if (!__any(pend != 0)) break;
        if (wall_clock64() - t0 > TRI_TIMEOUT) {
          failed = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    if (failed) failflag = 1;
    bar_lds();
    if (failflag) {   // uniform after the barrier (only ever set, then every wave returns)
      if (tid == 0) a.infos[k] = 3;
      return;
    }
    if (stp) {
      const long long t1 = clock64();
      acc0 += t1 - tq;
      tq = t1;
    }
    // this workgroup has read pass i + 1: the parity of pass i + 2 (= pass i's) may be reused
    const int64_t pn = gbase + (int64_t)((pass + 1) & 1) * par;
    const bool more = i + 1 <= m - 2;
    if (tid == 0 && more) st_gran(rs, pn + 2 * m + g, 0.0, pass + 1);
    lds_t* Vc = (lds_t*)Vbuf[i & 1];
    lds_t* Vn = (lds_t*)Vbuf[(i + 1) & 1];
    if (w == 0) {
      const long long q0s = stp ? clock64() : 0;
      // w = p + a2 v, a2 = -tau (p . v) / 2; the column i + 1 of the updated matrix; its reflector.
      // Every operand is loaded in one batch first (loads inside the selects were issued one
      // latency at a time: 3 us of the 7.6 us step at m = 999), the column stays in registers.
      const int i2 = i + 2 < m ? i + 2 : i + 1;
      const double gp1 = GP[i + 1], vi1 = Vc[i + 1], cr1 = C[i + 1];
      const double gp2 = GP[i2], vc2 = Vc[i2], cr2 = C[i2];
      // (chunks of four columns: every chunk's loads in flight together, few registers live beside the rows)
      double s = 0.0;
#pragma unroll
      for (int q0 = 0; q0 < EL; q0 += 4) {
        double gp[4], vc[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          gp[u] = GP[lane + 64 * (q0 + u)];
          vc[u] = Vc[lane + 64 * (q0 + u)];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int j = lane + 64 * (q0 + u);
          s += (j > i && j < m) ? gp[u] * vc[u] : 0.0;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      s = riptrm_wave::wave_sum(s);
      const double a2 = -0.5 * tau_c * s;
      const long long q1s = stp ? clock64() : 0;
      const double wi1 = gp1 + a2 * vi1;
      double sn = 0.0;   // the reflector's sum over c_j^2, j >= i + 3
#pragma unroll
      for (int q0 = 0; q0 < EL; q0 += 4) {
        double gp[4], vc[4], cr[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          gp[u] = GP[lane + 64 * (q0 + u)];
          vc[u] = Vc[lane + 64 * (q0 + u)];
          cr[u] = C[lane + 64 * (q0 + u)];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int j = lane + 64 * (q0 + u);
          const double wj = (j > i && j < m) ? gp[u] + a2 * vc[u] : 0.0;
          W[j] = wj;
          const double cj = (j > i + 1 && j < m) ? cr[u] - (vc[u] * wi1 + wj * vi1) : 0.0;   // row j's update at column i + 1
          C[j] = cj;
          sn += j >= i + 3 ? cj * cj : 0.0;
        }
        __builtin_amdgcn_sched_barrier(0);   // keep the next chunk's loads behind this one (register pressure)
      }
      const double di1 = cr1 - (vi1 * wi1 + wi1 * vi1);
      const long long q2s = stp ? clock64() : 0;
      if (writer && lane == 0) dv[i + 1] = di1;
      if (more) {
        // dlarfg on c[i+2 .. m): alpha = c[i+2] (its update formula, every lane), the sum over j >= i + 3
        const double alpha = cr2 - (vc2 * wi1 + (gp2 + a2 * vc2) * vi1);
        sn = riptrm_wave::wave_sum(sn);
        double tau = 0.0, beta = alpha, scl = 0.0;
        if (sn != 0.0) {
          beta = -copysign(sqrt(alpha * alpha + sn), alpha);
          tau = (beta - alpha) / beta;
          scl = 1.0 / (alpha - beta);
        }
#pragma unroll
        for (int q = 0; q < EL; ++q) {   // (each lane reads back its own c_j)
          const int j = lane + 64 * q;
          Vn[j] = (j <= i + 1 || j >= m) ? 0.0 : (j == i + 2 ? 1.0 : C[j] * scl);
        }
        if (lane == 0) scal[(i + 1) & 1] = tau;
        if (stp) {
          const long long q3s = clock64();
          sa += q1s - q0s;
          sb += q2s - q1s;
          sc += q3s - q2s;
        }
        if (writer) {
          if (lane == 0) {
            ev[i + 1] = beta;
            R[riptrm_eig::refl_tau(m) + i + 1] = tau;
          }
          const int64_t co = riptrm_eig::refl_col(m, i + 1) - (i + 2);
#pragma unroll
          for (int q = 0; q < EL; ++q) {
            const int j = lane + 64 * q;
            if (j >= i + 2 && j < m) R[co + j] = Vn[j];
          }
        }
      }
    }
    bar_lds();
    if (stp) {
      const long long t1 = clock64();
      acc1 += t1 - tq;
      tq = t1;
    }
    if (!more) break;
    const double tau_n = scal[(i + 1) & 1];
    // rank-two update of own rows l >= i + 2 (row i + 1 is finished: its diagonal is d_{i+1}), fused
    // with p^(i+1)_l = tau_{i+1} A'_l. v_{i+1}; publish pass i + 2
    // (v, w, v_{i+1} read from LDS per row: held in registers beside the rows they spill)
#pragma unroll
    for (int s = 0; s < RW; ++s) {
      const int l = rowid[s];
      if (l >= i + 2 && l < m) {   // uniform over the wave
        const double vl = Vc[l], wl = W[l];
        double acc = 0.0;
#pragma unroll
        for (int q = 0; q < EL; ++q) {
          const int j = lane + 64 * q;
          const double x = Ar[s][q] - (vl * W[j] + wl * Vc[j]);
          Ar[s][q] = x;
          acc += (j >= i + 2) ? x * Vn[j] : 0.0;
        }
        const double p = tau_n * riptrm_wave::wave_sum(acc);
        if (lane == 0) st_gran(rs, pn + l, p, pass + 1);
        if (l == i + 2) {
#pragma unroll
          for (int q = 0; q < EL; ++q) {
            const int j = lane + 64 * q;
            if (j >= i + 2 && j < m) st_gran(rs, pn + m + j, Ar[s][q], pass + 1);
          }
        }
      }
    }
    tau_c = tau_n;
    if (stp) {
      const long long t1 = clock64();
      acc2 += t1 - tq;
      tq = t1;
    }
  }
  if (stp) {
    stp[0] = acc0;
    stp[1] = acc1;
    stp[2] = acc2;
    stp[4] = sa;
    stp[5] = sb;
    stp[6] = sc;
  }
}

// After k_tridiag_dist for the hand-written eigensolver's later phases (riptrm_eig.h k_eig_lds with
// PH & 1 == 0, which read d and the SPLIT e): e_j -> 0 where |e_j| <= 4 eps ||T|| (phase 1's split),
// and a non-finite T marks info = 1 with NaN eigenvalues (phase 1's non-finite input test).  One
// workgroup of 256 threads per matrix.
__global__ void __launch_bounds__(256) k_tri_split(double* d0, double* e0, int64_t de_stride, int m, int32_t* infos,
                                                   double* ev0, int64_t ev_stride) {
  __shared__ double red[4];
  __shared__ int badw;
  const int k = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const double* d = d0 + (int64_t)k * de_stride;
  double* e = e0 + (int64_t)k * de_stride;
  if (tid == 0) badw = 0;
  double tn0 = 0.0;
  int bad = 0;
  for (int j = tid; j < m; j += 256) {
    const double ej = j < m - 1 ? e[j] : 0.0, ep = j > 0 ? e[j - 1] : 0.0;
    bad |= !isfinite(d[j]) | !isfinite(ej);
    tn0 = fmax(tn0, fabs(d[j]) + fabs(ep) + fabs(ej));
  }
  tn0 = riptrm_wave::wave_max(tn0);
  if (lane == 0) red[w] = tn0;
  __syncthreads();
  if (bad) badw = 1;
  tn0 = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
  __syncthreads();
  if (badw || infos[k] != 0) {
    if (tid == 0 && infos[k] == 0) infos[k] = 1;
    for (int j = tid; j < m; j += 256) ev0[(int64_t)k * ev_stride + j] = NAN;
    return;
  }
  for (int j = tid; j < m - 1; j += 256)
    if (fabs(e[j]) <= 4.0 * DBL_EPSILON * tn0) e[j] = 0.0;
}

// v <- H^T v (backward = 0: H_{m-2} ... H_0 v) or H v (backward = 1), H the reflectors of slot k0 +
// blockIdx.y at r_off (riptrm_eig layout), from slot offset voff to ooff; one wave, lane l holding
// elements l + 64 q (the k_refl_apply arithmetic).  The reflectors stream from HBM / L2 through a ring
// of RD register sets: reflector t + RD is requested while t is applied (one reflection is ~0.2 us
// of arithmetic against ~1-2 us of load latency).
template <int EL>
__global__ void __launch_bounds__(64) k_refl_big(double* base, int64_t sd, int k0, int m, int64_t r_off, int64_t voff,
                                                 int64_t ooff, int backward) {
  constexpr int RD = EL <= 8 ? 8 : 4;   // ring depth (EL = 16: 4 x 16 doubles in flight per lane)
  double* sb = base + (int64_t)(k0 + blockIdx.y) * sd;
  const double* R = sb + r_off;
  const int lane = threadIdx.x;
  double v[EL];
#pragma unroll
  for (int q = 0; q < EL; ++q) {
    const int j = lane + 64 * q;
    v[q] = j < m ? sb[voff + j] : 0.0;
  }
  const int nt = riptrm_eig::refl_tau(m), nr = m - 1;
  double ring[RD][EL], rtau[RD];
  auto fetch = [&](int t, double (&u)[EL], double& tau) {
    const int i = backward ? m - 2 - t : t;
    const bool live = t < nr;
    tau = R[live ? nt + i : nt];
    const int c = riptrm_eig::refl_col(m, i) - i - 1;
#pragma unroll
    for (int q = 0; q < EL; ++q) {
      const int j = lane + 64 * q;
      const bool ok = live && j > i && j < m;
      u[q] = R[ok ? c + j : nt];
    }
  };
#pragma unroll
  for (int r = 0; r < RD; ++r) fetch(r, ring[r], rtau[r]);
  for (int t0 = 0; t0 < nr; t0 += RD) {
#pragma unroll
    for (int r = 0; r < RD; ++r) {
      const int t = t0 + r;
      if (t < nr) {   // uniform
        const int i = backward ? m - 2 - t : t;
        double u[EL];
#pragma unroll
        for (int q = 0; q < EL; ++q) {
          const int j = lane + 64 * q;
          u[q] = (j > i && j < m) ? ring[r][q] : 0.0;
        }
        const double tau = rtau[r];
        fetch(t + RD, ring[r], rtau[r]);   // the slot is free: request reflector t + RD
        if (tau != 0.0) {   // uniform
          double s = 0.0;
#pragma unroll
          for (int q = 0; q < EL; ++q) s += u[q] * v[q];
          const double f = tau * riptrm_wave::wave_sum(s);
#pragma unroll
          for (int q = 0; q < EL; ++q) v[q] = v[q] - f * u[q];
        }
      }
    }
  }
#pragma unroll
  for (int q = 0; q < EL; ++q) {
    const int j = lane + 64 * q;
    if (j < m) sb[ooff + j] = v[q];
  }
}

// The number of eigenvalues of T below x by the sign changes of its leading principal minors
// p_j = (d_j - x) p_{j-1} - e_{j-1}^2 p_{j-2} (p_{-1} = 1; e2 = e^2): two dependent operations per step
// where riptrm_eig.h's LDL^T count (dlaneg) waits on a reciprocal (one thread's chain here, not the
// issue-bound many-lane counts there: ~20 vs ~110 cycles per step).  Exact powers of two rescale
// (p_j, p_{j-1}) every four steps; a zero minor takes the sign opposite to the previous one (a tiny
// negative pivot: dlaneg's pivmin convention).
__device__ __forceinline__ int sturm_count_df(const lds_t* d, const lds_t* e2, int m, double x) {
  double pm = 1.0, p = d[0] - x;
  if (p == 0.0) p = -DBL_MIN;
  int c = p < 0.0;
  int j = 1;
  for (; j + 3 < m; j += 4) {
    const double d0 = d[j], d1 = d[j + 1], d2 = d[j + 2], d3 = d[j + 3];
    const double f0 = e2[j - 1], f1 = e2[j], f2 = e2[j + 1], f3 = e2[j + 2];
    double pn = (d0 - x) * p - f0 * pm;
    if (pn == 0.0) pn = -copysign(DBL_MIN, p);
    c += (pn < 0.0) != (p < 0.0);
    pm = p; p = pn;
    pn = (d1 - x) * p - f1 * pm;
    if (pn == 0.0) pn = -copysign(DBL_MIN, p);
    c += (pn < 0.0) != (p < 0.0);
    pm = p; p = pn;
    pn = (d2 - x) * p - f2 * pm;
    if (pn == 0.0) pn = -copysign(DBL_MIN, p);
    c += (pn < 0.0) != (p < 0.0);
    pm = p; p = pn;
    pn = (d3 - x) * p - f3 * pm;
    if (pn == 0.0) pn = -copysign(DBL_MIN, p);
    c += (pn < 0.0) != (p < 0.0);
    pm = p; p = pn;
    int ex;
    (void)frexp(p, &ex);
    p = ldexp(p, -ex);
    pm = ldexp(pm, -ex);
  }
  for (; j < m; ++j) {
    double pn = (d[j] - x) * p - e2[j - 1] * pm;
    if (pn == 0.0) pn = -copysign(DBL_MIN, p);
    c += (pn < 0.0) != (p < 0.0);
    pm = p;
    p = pn;
  }
  return c;
}

// the smallest (hi = false) or largest eigenvalue of T by one wave's multisection (64 points per
// step; riptrm_eig.h phase 2's tolerance max(2 eps |lambda|, eps ||T||))
__device__ __forceinline__ double extreme_eig(const lds_t* d, const lds_t* e2, int m, bool hi_end, double glo, double ghi,
                                              double fudge, double tnorm, int lane) {
  const double eps = DBL_EPSILON;
  const int ei = hi_end ? m - 1 : 0;
  double lo = glo - fudge, hi = ghi + fudge;
  for (int it = 0; it < 128; ++it) {
    const double tol = fmax(2.0 * eps * fmax(fabs(lo), fabs(hi)), eps * tnorm);
    if (hi - lo <= tol) break;   // uniform
    const double step = (hi - lo) / 65.0;
    const double x = lo + step * (lane + 1);
    const int c = (x > lo && x < hi) ? sturm_count_df(d, e2, m, x) : (x <= lo ? 0 : m);
    // the new interval: the largest point with count <= ei, the smallest with count > ei
    const double nlo = riptrm_wave::wave_max(c > ei ? -INFINITY : x);
    const double nhi = riptrm_wave::wave_min(c > ei ? x : INFINITY);
    const double nl = fmax(lo, nlo), nh = fmin(hi, nhi);
    if (nl >= nh || (nl == lo && nh == hi)) break;
    lo = nl;
    hi = nh;
  }
  return 0.5 * (lo + hi);
}

// One Newton step's solves of the secular equation, by one thread: (T + lam I) = L D L^T (no pivoting:
// positive definite for lam > -lam_min), y = (T + lam I)^-1 b and, with second, t = (T + lam I)^-1 y;
// returns s2 = y . y (and s3 = y . t).  The pivots come from the leading minors P_j = (d_j + lam)
// P_{j-1} - e_{j-1}^2 P_{j-2} (D_j = P_j / P_{j-1}, 1 / D_j = P_{j-1} / P_j, L_j = e_j / D_j), so the dependent
// chain is two operations per step and each reciprocal is off it (exact powers of two rescale the pair
// every four steps: the ratios are unchanged).  Then the forward and backward sweeps (one FMA chain
// each), their next four entries' loads issued ahead.  lf, rd: L and 1/D.
__device__ __forceinline__ void ldl_newton(const lds_t* d, const lds_t* e, const lds_t* e2, int m, double lam,
                                           const lds_t* b, lds_t* y, lds_t* t2, lds_t* lf, lds_t* rd, bool second,
                                           double& s2, double& s3) {
  double Pm = 1.0, P = d[0] + lam;
  int j = 0;
  for (; j + 4 < m; j += 4) {
    const double d1 = d[j + 1], d2 = d[j + 2], d3 = d[j + 3], d4 = d[j + 4];
    const double f0 = e2[j], f1 = e2[j + 1], f2 = e2[j + 2], f3 = e2[j + 3];
    const double e0 = e[j], e1 = e[j + 1], ee2 = e[j + 2], e3 = e[j + 3];
    const double P0 = P;
    const double P1 = (d1 + lam) * P0 - f0 * Pm;
    const double P2 = (d2 + lam) * P1 - f1 * P0;
    const double P3 = (d3 + lam) * P2 - f2 * P1;
    const double P4 = (d4 + lam) * P3 - f3 * P2;
    const double r0 = Pm * riptrm_eig::rcp_nr(P0), r1 = P0 * riptrm_eig::rcp_nr(P1);
    const double r2 = P1 * riptrm_eig::rcp_nr(P2), r3 = P2 * riptrm_eig::rcp_nr(P3);
    rd[j] = r0; lf[j] = e0 * r0;
    rd[j + 1] = r1; lf[j + 1] = e1 * r1;
    rd[j + 2] = r2; lf[j + 2] = ee2 * r2;
    rd[j + 3] = r3; lf[j + 3] = e3 * r3;
    int ex;
    (void)frexp(P4, &ex);
    P = ldexp(P4, -ex);
    Pm = ldexp(P3, -ex);
  }
  for (; j + 1 < m; ++j) {
    const double Pn = (d[j + 1] + lam) * P - e2[j] * Pm;
    const double r = Pm * riptrm_eig::rcp_nr(P);
    rd[j] = r;
    lf[j] = e[j] * r;
    Pm = P;
    P = Pn;
  }
  rd[m - 1] = Pm * riptrm_eig::rcp_nr(P);
  // forward: z_0 = b_0, z_{j+1} = b_{j+1} - L_j z_j (into y)
  double z = b[0];
  y[0] = z;
  j = 0;
  for (; j + 4 < m; j += 4) {
    const double l0 = lf[j], l1 = lf[j + 1], l2 = lf[j + 2], l3 = lf[j + 3];
    const double b1 = b[j + 1], b2 = b[j + 2], b3 = b[j + 3], b4 = b[j + 4];
    z = b1 - l0 * z; y[j + 1] = z;
    z = b2 - l1 * z; y[j + 2] = z;
    z = b3 - l2 * z; y[j + 3] = z;
    z = b4 - l3 * z; y[j + 4] = z;
  }
  for (; j + 1 < m; ++j) {
    z = b[j + 1] - lf[j] * z;
    y[j + 1] = z;
  }
  // backward: y_{m-1} = z_{m-1} / D_{m-1}, y_j = z_j / D_j - L_j y_{j+1}; s2
  double x = y[m - 1] * rd[m - 1];
  y[m - 1] = x;
  double a2 = x * x;
  j = m - 2;
  for (; j - 3 >= 0; j -= 4) {
    const double z0 = y[j], z1 = y[j - 1], z2 = y[j - 2], z3 = y[j - 3];
    const double r0 = rd[j], r1 = rd[j - 1], r2 = rd[j - 2], r3 = rd[j - 3];
    const double l0 = lf[j], l1 = lf[j - 1], l2 = lf[j - 2], l3 = lf[j - 3];
    x = z0 * r0 - l0 * x; y[j] = x; a2 += x * x;
    x = z1 * r1 - l1 * x; y[j - 1] = x; a2 += x * x;
    x = z2 * r2 - l2 * x; y[j - 2] = x; a2 += x * x;
    x = z3 * r3 - l3 * x; y[j - 3] = x; a2 += x * x;
  }
  for (; j >= 0; --j) {
    x = y[j] * rd[j] - lf[j] * x;
    y[j] = x;
    a2 += x * x;
  }
  s2 = a2;
  s3 = 0.0;
  if (!second) return;
  // t = (T + lam I)^-1 y with the same factor; s3 = y . t
  z = y[0];
  t2[0] = z;
  j = 0;
  for (; j + 4 < m; j += 4) {
    const double l0 = lf[j], l1 = lf[j + 1], l2 = lf[j + 2], l3 = lf[j + 3];
    const double y1 = y[j + 1], y2 = y[j + 2], y3 = y[j + 3], y4 = y[j + 4];
    z = y1 - l0 * z; t2[j + 1] = z;
    z = y2 - l1 * z; t2[j + 2] = z;
    z = y3 - l2 * z; t2[j + 3] = z;
    z = y4 - l3 * z; t2[j + 4] = z;
  }
  for (; j + 1 < m; ++j) {
    z = y[j + 1] - lf[j] * z;
    t2[j + 1] = z;
  }
  x = t2[m - 1] * rd[m - 1];
  double a3 = y[m - 1] * x;
  j = m - 2;
  for (; j - 3 >= 0; j -= 4) {
    const double z0 = t2[j], z1 = t2[j - 1], z2 = t2[j - 2], z3 = t2[j - 3];
    const double r0 = rd[j], r1 = rd[j - 1], r2 = rd[j - 2], r3 = rd[j - 3];
    const double l0 = lf[j], l1 = lf[j - 1], l2 = lf[j - 2], l3 = lf[j - 3];
    const double y0 = y[j], y1 = y[j - 1], y2 = y[j - 2], y3 = y[j - 3];
    x = z0 * r0 - l0 * x; a3 += y0 * x;
    x = z1 * r1 - l1 * x; a3 += y1 * x;
    x = z2 * r2 - l2 * x; a3 += y2 * x;
    x = z3 * r3 - l3 * x; a3 += y3 * x;
  }
  for (; j >= 0; --j) {
    x = t2[j] * rd[j] - lf[j] * x;
    a3 += y[j] * x;
  }
  s3 = a3;
}

// scalar slots this header uses (riptrm_trs_big.hip Sc)
struct TriSc {
  int cg_ok, p1obj, kind, lam1, mineig, interior, delta, an, atol, it, done, fallback, newton;
};

// After k_tridiag_dist (and the reflector application: b = H^T a at boff): mode 0 the subproblem, mode 1
// the smallest eigenvalue only.  One workgroup of 256 threads per slot: waves 0 / 1 the extreme
// eigenvalues; then, at once, wave 0 the secular Newton (lane 0), wave 1 SciPy's CG on T y = -b and
// wave 2 the hard-case test (lam_min's multiplicity and the component of b on its twisted eigenvector;
// a hard case discards the other two and sets the fallback flag).  Writes the boundary / interior
// candidate in T coordinates at peoff (the host applies H), lam_min at evoff[0].
constexpr int TRI_SOLVE_ARRAYS = 10;   // LDS vectors of 64 EL doubles
template <int EL>
__global__ void __launch_bounds__(256) k_tri_solve(double* base, int64_t sd, int32_t* infos, int m, int64_t d_off,
                                                   int64_t e_off, int64_t boff, int64_t aoff_vec, int64_t peoff,
                                                   int64_t cgxoff, int64_t evoff, int64_t scoff, TriSc S,
                                                   const double* Dg, int64_t dstride, const int32_t* ids, double tolhc,
                                                   int mode, long long* stamps) {
  // stamps (diagnostics, RIPTRM_TRI_STAMPS=1; slot 0): clock64 at [0] start, [1] extreme eigenvalues,
  // [2] hard-case test done (wave 2), [3] the Newton done (wave 0), [4] the CG done (wave 1), [5] end;
  // [6] Newton steps, [7] CG iterations
  long long* stp = (stamps && blockIdx.y == 0) ? stamps : nullptr;
  if (stp && threadIdx.x == 0) stp[0] = clock64();
  extern __shared__ double smem[];
  constexpr int V = 64 * EL;
  lds_t* d = (lds_t*)smem;
  lds_t* e = d + V;
  lds_t* e2 = e + V;   // e^2 (the Sturm counts and the minors)
  lds_t* b = e2 + V;
  lds_t* y = b + V;    // Newton: y, then the boundary candidate
  lds_t* t2 = y + V;
  lds_t* lf = t2 + V;
  lds_t* rd = lf + V;
  lds_t* z = rd + V;   // the twisted eigenvector
  lds_t* cx = z + V;   // the CG's iterate
  __shared__ double red[8];
  __shared__ double xs[10];   // lam_min, lam_max, multiplicity, xobj, lam1, CG ok, p1obj, Newton steps, ghard
  const int k = blockIdx.y;
  double* sb = base + (int64_t)k * sd;
  double* sc = sb + scoff;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const double eps = DBL_EPSILON;
  for (int j = tid; j < V; j += 256) {
    d[j] = j < m ? sb[d_off + j] : 0.0;
    e[j] = j < m - 1 ? sb[e_off + j] : 0.0;
    b[j] = (mode == 0 && j < m) ? sb[boff + j] : 0.0;
  }
  __syncthreads();
  // non-finite T (input or exchange failure): info 1 (3 stays), NaN out
  int bad = 0;
  for (int j = tid; j < m; j += 256) bad |= !isfinite(d[j]) | (j < m - 1 && !isfinite(e[j]));
  bad = __syncthreads_or(bad) || infos[k] != 0;
  if (bad) {
    if (tid == 0) {
      if (infos[k] == 0) infos[k] = 1;
      sb[evoff] = NAN;
      sc[S.fallback] = 0.0;
      sc[S.mineig] = NAN;
      sc[S.kind] = 0.0;
      sc[S.lam1] = NAN;
      sc[S.interior] = 0.0;
    }
    for (int j = tid; j < m; j += 256) sb[peoff + j] = NAN;
    return;
  }
  // split where |e_j| <= 4 eps ||T|| (riptrm_eig.h), Gershgorin interval, pivmin
  double tn0 = 0.0;
  for (int j = tid; j < m; j += 256)
    tn0 = fmax(tn0, fabs(d[j]) + (j > 0 ? fabs(e[j - 1]) : 0.0) + (j < m - 1 ? fabs(e[j]) : 0.0));
  tn0 = riptrm_wave::wave_max(tn0);
  if (lane == 0) red[w] = tn0;
  __syncthreads();
  tn0 = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
  __syncthreads();
  for (int j = tid; j < V; j += 256) {
    double ej = e[j];
    if (j < m - 1 && fabs(ej) <= 4.0 * eps * tn0) ej = 0.0;
    e[j] = ej;
    e2[j] = ej * ej;
  }
  __syncthreads();
  double glo = INFINITY, ghi = -INFINITY, tnorm = 0.0, emax2 = 0.0;
  for (int j = tid; j < m; j += 256) {
    const double r0 = j > 0 ? fabs(e[j - 1]) : 0.0, r1 = j < m - 1 ? fabs(e[j]) : 0.0;
    glo = fmin(glo, d[j] - r0 - r1);
    ghi = fmax(ghi, d[j] + r0 + r1);
    tnorm = fmax(tnorm, fabs(d[j]) + r0 + r1);
    if (j < m - 1) emax2 = fmax(emax2, e[j] * e[j]);
  }
  glo = riptrm_wave::wave_min(glo);
  ghi = riptrm_wave::wave_max(ghi);
  tnorm = riptrm_wave::wave_max(tnorm);
  emax2 = riptrm_wave::wave_max(emax2);
  if (lane == 0) {
    red[w] = glo;
    red[4 + w] = ghi;
    xs[w] = tnorm;
    xs[4 + w] = emax2;
  }
  __syncthreads();
  glo = fmin(fmin(red[0], red[1]), fmin(red[2], red[3]));
  ghi = fmax(fmax(red[4], red[5]), fmax(red[6], red[7]));
  tnorm = fmax(fmax(xs[0], xs[1]), fmax(xs[2], xs[3]));
  emax2 = fmax(fmax(xs[4], xs[5]), fmax(xs[6], xs[7]));
  __syncthreads();
  const double pivmin = DBL_MIN * fmax(1.0, emax2);
  const double fudge = 2.0 * eps * tnorm + 2.0 * pivmin;
  // lam_min (wave 0) and lam_max (wave 1)
  if (w < 2) {
    const double lx = extreme_eig(d, e2, m, w == 1, glo, ghi, fudge, tnorm, lane);
    if (lane == 0) xs[w] = lx;
  }
  __syncthreads();
  const double lmin = xs[0], lmaxv = xs[1];
  if (stp && tid == 0) stp[1] = clock64();
  __syncthreads();
  if (mode == 1) {
    if (tid == 0) {
      sb[evoff] = lmin;
      sc[S.mineig] = lmin;
      infos[k] = 0;
    }
    return;
  }
  const double Delta = Dg[(int64_t)ids[k] * dstride];
  const double D2 = Delta * Delta;
  // ||a|| (the CG's scale, as k_cg_diag) and ||b|| = ||H^T a||
  double an = 0.0, gg = 0.0;
  for (int j = tid; j < m; j += 256) {
    const double aj = sb[aoff_vec + j];
    an += aj * aj;
    gg += b[j] * b[j];
  }
  an = riptrm_wave::wave_sum(an);
  gg = riptrm_wave::wave_sum(gg);
  if (lane == 0) {
    red[w] = an;
    red[4 + w] = gg;
  }
  __syncthreads();
  an = sqrt((red[0] + red[1]) + (red[2] + red[3]));
  const double gn = sqrt((red[4] + red[5]) + (red[6] + red[7]));
  __syncthreads();
  if (w == 0) {
    // the secular Newton of k_secular: ||(T + l1 I)^-1 b|| = Delta from l1 = -lam_min + ||b|| / Delta
    if (lane == 0) {
      const double lo = -lmin;
      double l1 = lo + gn / Delta;
      int itn = 0;
      for (; itn < 100; ++itn) {
        double s2, s3;
        ldl_newton(d, e, e2, m, l1, b, y, t2, lf, rd, true, s2, s3);
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
      double s2, s3;
      ldl_newton(d, e, e2, m, l1, b, y, t2, lf, rd, false, s2, s3);
      const double scl = Delta / sqrt(s2);
      double o0 = 0.0, o1 = 0.0;
      for (int j = 0; j < m; ++j) {
        const double c = -y[j] * scl;
        y[j] = c;
      }
      for (int j = 0; j < m; ++j) {   // xobj = pe^T T pe / 2 + b^T pe
        const double tp = d[j] * y[j] + (j > 0 ? e[j - 1] * y[j - 1] : 0.0) + (j < m - 1 ? e[j] * y[j + 1] : 0.0);
        o0 += y[j] * tp;
        o1 += b[j] * y[j];
      }
      xs[3] = 0.5 * o0 + o1;
      xs[4] = l1;
      xs[7] = (double)itn;
      if (stp) {
        stp[3] = clock64();
        stp[6] = itn;
      }
    }
  } else if (w == 1) {
    // SciPy's CG on T y = -b (k_cg_diag's loop; lane l owns elements l EL .. l EL + EL - 1, its diagonal
    // and off-diagonal entries held in registers)
    double x[EL], r[EL], p[EL], tq[EL], dg[EL], er[EL];
    const int j0 = lane * EL;
#pragma unroll
    for (int u = 0; u < EL; ++u) {
      const int j = j0 + u;
      r[u] = j < m ? -b[j] : 0.0;
      x[u] = p[u] = 0.0;
      dg[u] = j < m ? d[j] : 0.0;
      er[u] = j < m - 1 ? e[j] : 0.0;
    }
    const double el0 = j0 > 0 && j0 < m ? e[j0 - 1] : 0.0;   // the coupling to the previous lane's last element
    const double atol = 1e-5 * an;
    double done = an == 0.0 ? 2.0 : 0.0, it = 0.0, rho_prev = 1.0;
    auto tmul = [&](const double (&pv)[EL], double (&out)[EL]) {
      const double left = __shfl(pv[EL - 1], lane > 0 ? lane - 1 : 0);    // element j0 - 1
      const double right = __shfl(pv[0], lane < 63 ? lane + 1 : 63);     // element j0 + EL
#pragma unroll
      for (int u = 0; u < EL; ++u) {
        const double pl = u > 0 ? pv[u - 1] : (lane > 0 ? left : 0.0);
        const double pr = u < EL - 1 ? pv[u + 1] : (lane < 63 ? right : 0.0);
        const double el = u > 0 ? er[u - 1] : el0;
        out[u] = (el * pl + dg[u] * pv[u]) + er[u] * pr;
      }
    };
    while (done == 0.0) {   // uniform
      if (it >= 10.0 * m) {
        done = 3.0;
        break;
      }
      double rr = 0.0;
#pragma unroll
      for (int u = 0; u < EL; ++u) rr += r[u] * r[u];
      rr = riptrm_wave::wave_sum(rr);
      if (sqrt(rr) < atol) {
        done = 1.0;
        break;
      }
      const double rho = rr;
      const double beta = it > 0.0 ? rho / rho_prev : 0.0;
#pragma unroll
      for (int u = 0; u < EL; ++u) p[u] = it > 0.0 ? p[u] * beta + r[u] : r[u];
      tmul(p, tq);
      double pq = 0.0;
#pragma unroll
      for (int u = 0; u < EL; ++u) pq += p[u] * tq[u];
      pq = riptrm_wave::wave_sum(pq);
      const double alpha = rho / pq;
#pragma unroll
      for (int u = 0; u < EL; ++u) {
        x[u] += alpha * p[u];
        r[u] -= alpha * tq[u];
      }
      rho_prev = rho;
      it += 1.0;
    }
    tmul(x, tq);
    double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0;
#pragma unroll
    for (int u = 0; u < EL; ++u) {
      const int j = j0 + u;
      if (j < m) {
        const double res = tq[u] + b[j];
        v0 += res * res;
        v1 += x[u] * x[u];
        v2 += x[u] * tq[u];
        v3 += b[j] * x[u];
        sb[cgxoff + j] = x[u];
        cx[j] = x[u];
      }
    }
    v0 = riptrm_wave::wave_sum(v0);
    v1 = riptrm_wave::wave_sum(v1);
    v2 = riptrm_wave::wave_sum(v2);
    v3 = riptrm_wave::wave_sum(v3);
    if (lane == 0) {
      const double ok = (an != 0.0 && sqrt(v0) / an < 1e-5 && v1 < D2) ? 1.0 : 0.0;   // RIPTRM.py:246-251
      sc[S.an] = an;
      sc[S.atol] = atol;
      sc[S.it] = it;
      sc[S.done] = done;
      sc[S.cg_ok] = ok;
      sc[S.p1obj] = 0.5 * v2 + v3;
      sc[S.delta] = Delta;
      xs[5] = ok;
      xs[6] = 0.5 * v2 + v3;
      if (stp) {
        stp[4] = clock64();
        stp[7] = (long long)it;
      }
    }
  } else if (w == 2) {
    // hard-case test (k_secular): the component of b on the eigenspace of lam_min (eigenvalues within
    // 1e-12 max(1, max |lambda|)); a multiple lam_min or a hard case goes to the eigendecomposition path
    const double hard_tol = 1e-12 * fmax(1.0, fmax(fabs(lmin), fabs(lmaxv)));
    if (lane == 0) {
      xs[2] = (double)sturm_count_df(d, e2, m, lmin + hard_tol);
      double evl[1] = {lmin};
      riptrm_eig::twisted_vector(z, d, e, evl, m, 0, 16.0 * eps * tnorm, pivmin);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // lane 0's vector -> the wave
    double zb = 0.0;
    for (int j = lane; j < m; j += 64) zb += z[j] * b[j];
    zb = riptrm_wave::wave_sum(zb);
    if (lane == 0) {
      xs[8] = fabs(zb);
      if (stp) stp[2] = clock64();
    }
  }
  __syncthreads();
  const bool fb = xs[2] > 1.5 || xs[8] <= tolhc * gn;
  if (fb) {   // uniform
    if (tid == 0) {
      sc[S.fallback] = 1.0;
      sb[evoff] = lmin;
      infos[k] = 0;
    }
    return;
  }
  // the interior / boundary choice (RIPTRM.py:294-298) and the candidate in T coordinates
  const bool interior = xs[5] != 0.0 && xs[6] <= xs[3];
  if (stp && tid == 0) stp[5] = clock64();
  for (int j = tid; j < m; j += 256) sb[peoff + j] = interior ? cx[j] : y[j];
  if (tid == 0) {
    sc[S.interior] = interior ? 1.0 : 0.0;
    sc[S.kind] = interior ? 1.0 : 0.0;   // riptrm_trs::Kind: boundary 0, interior 1
    sc[S.lam1] = interior ? 0.0 : xs[4];
    sc[S.mineig] = lmin;
    sc[S.fallback] = 0.0;
    sc[S.newton] = xs[7];
    sb[evoff] = lmin;
    infos[k] = 0;
  }
}

// v <- H^T v (backward = 0: H_{m-2} ... H_0 v) or H v (backward = 1) for orders up to 1024 on one
// 1024-thread workgroup (element j on thread j): per reflection each wave's share of the dot product,
// one workgroup barrier, the 16 wave partials added in a fixed order (two parities of the partial
// buffer, so a wave may run one reflection ahead); reflector t + 8 is requested while t is applied.
// ~0.1 us per reflection where one wave with the vector in registers waited on the reflectors' loads.
__global__ void __launch_bounds__(1024) k_refl_wg(double* base, int64_t sd, int k0, int m, int64_t r_off, int64_t voff,
                                                  int64_t ooff, int backward) {
  constexpr int RD = 8;
  __shared__ double red[2][16];
  double* sb = base + (int64_t)(k0 + blockIdx.y) * sd;
  const double* R = sb + r_off;
  const int j = threadIdx.x, lane = j & 63, w = j >> 6;
  double v = j < m ? sb[voff + j] : 0.0;
  const int nt = riptrm_eig::refl_tau(m), nr = m - 1;
  double ring[RD], rtau[RD];
  auto fetch = [&](int t, double& u, double& tau) {
    const int i = backward ? m - 2 - t : t;
    const bool live = t < nr;
    tau = R[live ? nt + i : nt];
    const bool ok = live && j > i && j < m;
    u = R[ok ? riptrm_eig::refl_col(m, i) - i - 1 + j : nt];
  };
#pragma unroll
  for (int r = 0; r < RD; ++r) fetch(r, ring[r], rtau[r]);
  for (int t0 = 0; t0 < nr; t0 += RD) {
#pragma unroll
    for (int r = 0; r < RD; ++r) {
      const int t = t0 + r;
      if (t < nr) {   // uniform
        const int i = backward ? m - 2 - t : t;
        const double u = (j > i && j < m) ? ring[r] : 0.0;
        const double tau = rtau[r];
        fetch(t + RD, ring[r], rtau[r]);
        if (tau != 0.0) {   // uniform
          const double s = riptrm_wave::wave_sum(u * v);
          if (lane == 0) red[t & 1][w] = s;
          __syncthreads();
          double S = 0.0;
#pragma unroll
          for (int q = 0; q < 16; ++q) S += red[t & 1][q];
          v = v - (tau * S) * u;
        }
      }
    }
  }
  if (j < m) sb[ooff + j] = v;
}

}  // namespace riptrm_tri
