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
//      with EL elements per lane in registers.  ONE exchange per column: every workgroup publishes,
//      per row l, the pair {p_l = tau A_l . v, A_{l, i+1}} (row i + 1 of the updated matrix is its
//      column i + 1: the bitwise-symmetric update keeps it so); each workgroup then forms
//      w = p - tau (p.v) v / 2, the next column c = col_{i+1} - (v w_{i+1} + w v_{i+1}) and its
//      reflector redundantly (the same arithmetic everywhere: bitwise the same values), and runs the
//      rank-two update of its rows fused with the next column's p.  The exchange: 16-byte granules
//      {p_l, A_{l, i+1}} written by one write-through store each, their mantissas' last bits set to the
//      pass's tag bit (a rounding-level change every workgroup sees alike), polled with sc1 loads
//      (MI355X_MICROARCH.md, persistent hand-offs), two parities, plus one arrival granule {value,
//      check, pass} per workgroup and pass so no workgroup overwrites a parity another still reads.
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
#include "../../include/riptrm.h"

namespace riptrm_tri {

#pragma clang fp contract(off)

using riptrm_eig::lds_t;

constexpr int TT = 512;                          // threads per tridiagonalisation workgroup
constexpr int TRI_MIN = RIPTRM_TRS_TRI_MIN;      // (m = 199 x 64: 10.0k vs 7.7k outer it/s by the
                                                 // eigensolver path, OUT=r6e200)
constexpr int TRI_MAX = RIPTRM_TRS_TRI_MAX;      // (EL = 32 for 2048 spilled the rows to scratch)
static_assert(TRI_MIN > 64 && TRI_MIN <= riptrm_eig::EIG_LDS_MAX + 1 && TRI_MAX == 1024, "riptrm_tri: orders");
constexpr unsigned long long TRI_TIMEOUT = 200000000ull;   // 2 s of the 100 MHz wall clock

// elements per lane (EL) and rows per wave (RW) of order m: 32 doubles of the matrix per lane
__host__ __device__ constexpr int tri_el(int m) { return m <= 256 ? 4 : (m <= 512 ? 8 : 16); }
__host__ __device__ constexpr int tri_rw(int m) { return 32 / tri_el(m); }
__host__ __device__ constexpr int tri_groups(int m) { return (m + 8 * tri_rw(m) - 1) / (8 * tri_rw(m)); }
// granules per matrix: 2 parities x [{p, column}: m][arrivals: G]
__host__ __device__ constexpr int64_t tri_par(int m) { return (int64_t)m + tri_groups(m); }
__host__ __device__ constexpr int64_t tri_granules(int m) { return 2 * tri_par(m); }
// byte offset of granule g: eight granules (one 128-byte line) every 128 << sp bytes (sp = 0: packed;
// larger sp spreads the lines every workgroup polls over more memory channels)
__host__ __device__ constexpr int64_t gran_off(int64_t g, int sp) { return ((g >> 3) << (7 + sp)) + ((g & 7) << 4); }
__host__ __device__ constexpr int64_t tri_grid_bytes(int64_t granules, int sp) { return ((granules + 7) >> 3) << (7 + sp); }

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ unsigned tag_check(unsigned lo, unsigned hi, unsigned pass) {
  return lo ^ hi ^ (pass * 0x9E3779B9u);
}
__device__ __forceinline__ void st_gran(__amdgpu_buffer_rsrc_t rs, int64_t g, int sp, double v, unsigned pass) {
  const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  const u32x4 q = {lo, hi, tag_check(lo, hi, pass), pass};
  __builtin_amdgcn_raw_buffer_store_b128(q, rs, (int)gran_off(g, sp), 0, 16);   // aux 16: sc1 (write-through)
}

// the pair granule {a, b} of pass `pass`: both mantissas' last bits = the pass's tag bit, which
// alternates between the passes sharing a parity (and is 1 on each parity's first pass: the grid
// starts zeroed); a reader takes it when both bits match (a granule torn between passes mixes them)
__device__ __forceinline__ unsigned pair_bit(unsigned pass) { return ((pass + 1) >> 1) & 1u; }
__device__ __forceinline__ void st_pair(__amdgpu_buffer_rsrc_t rs, int64_t g, int sp, double a, double b, unsigned pass) {
  const unsigned t = pair_bit(pass);
  const u32x4 q = {((unsigned)__double2loint(a) & ~1u) | t, (unsigned)__double2hiint(a),
                   ((unsigned)__double2loint(b) & ~1u) | t, (unsigned)__double2hiint(b)};
  __builtin_amdgcn_raw_buffer_store_b128(q, rs, (int)gran_off(g, sp), 0, 16);   // aux 16: sc1 (write-through)
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
  int sleep;             // s_sleep 1 rounds between polls (RIPTRM_TRI_SLEEP; default 1)
  int spread;            // gran_off's sp (RIPTRM_TRI_SPREAD)
  long long* hops;       // diagnostics (RIPTRM_TRI_STAMPS=2): matrix 0, every workgroup, steps i = 16 s: the
                         // wall clock (100 MHz, chip-wide) at [g][s][0] its gather's start, [1] its end
  long long* stamps;     // diagnostics (RIPTRM_TRI_STAMPS=1): workgroup 0 of matrix 0 accumulates clock64
                         // cycles in [0] the gather, [1] the column step, [2] the update + publish
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
  __shared__ double GP[EL * 64];        // gathered p (written by the gather, read by the column step)
  __shared__ double W[EL * 64];         // w = p + a2 v (column step -> every wave's update)
  __shared__ double C[EL * 64];         // gathered column (= row) i + 1 (column 0 of the input in the prologue)
  __shared__ double red[2][8];          // the column step's per-wave partial sums
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
  const int gsp = a.spread;
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
  // pass 1: {p^(0)_l = tau_0 A_l. v_0, A_{l,1}} for own rows l >= 1 (lane 1 holds column 1), this
  // workgroup's arrival
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
        if (lane == 1) st_pair(rs, pb + l, gsp, p, Ar[s][0], 1u);
      }
    }
    if (tid == 0) st_gran(rs, pb + m + g, gsp, 0.0, 1u);
  }

  constexpr int NG = (64 * EL + 64 + TT - 1) / TT;   // granules polled per thread (upper bound)
  bool failed = false;
  long long* stp = (a.stamps && g == 0 && k == 0 && tid == 0) ? a.stamps : nullptr;
  long long acc0 = 0, acc1 = 0, acc2 = 0, tq = stp ? clock64() : 0, sa = 0, sb = 0, sc = 0, sd = 0;
  for (int i = 0; i <= m - 2; ++i) {
    const unsigned pass = (unsigned)(i + 1);
    const int64_t pb = gbase + (int64_t)(pass & 1) * par;
    const int r = m - i - 1;   // trailing indices i + 1 .. m - 1
    const int ng = r + G;
    lds_t* Vc = (lds_t*)Vbuf[i & 1];
    lds_t* Vn = (lds_t*)Vbuf[(i + 1) & 1];
    long long* hp = (a.hops && k == 0 && tid == 0 && (i & 15) == 0) ? a.hops + ((int64_t)g * ((m + 15) / 16) + (i >> 4)) * 2 : nullptr;
    if (hp) hp[0] = (long long)wall_clock64();
    // gather: p_j, row_{i+1}[j] (j > i) and every workgroup's arrival, polled until the tags say this
    // pass; each p_j as it lands goes into this wave's share of p . v (the column step's first sum, its
    // wave tree and partial ahead of the gather's barrier: one barrier less per step)
    {
      double sp = 0.0;
      int pend = 0;
      int64_t gi[NG];
#pragma unroll
      for (int u = 0; u < NG; ++u) {
        const int t = tid + TT * u;
        int64_t gx = 0;
        if (t < r) gx = pb + i + 1 + t;
        else if (t < ng) gx = pb + m + (t - r);
        gi[u] = gx;
        if (t < ng) pend |= 1 << u;
      }
      const unsigned long long t0 = wall_clock64();
      while (true) {
        u32x4 qv[NG];
#pragma unroll
        for (int u = 0; u < NG; ++u)
          if (pend & (1 << u)) qv[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)gran_off(gi[u], gsp), 0, 16);
#pragma unroll
        for (int u = 0; u < NG; ++u)
          if (pend & (1 << u)) {
            const u32x4 q = qv[u];
            const int t = tid + TT * u;
            const unsigned tb = pair_bit(pass);
            if (t < r ? ((q.x & 1u) == tb && (q.z & 1u) == tb) : (q.w == pass && q.z == tag_check(q.x, q.y, pass))) {
              if (t < r) {   // {p_j, A_{j, i+1}}, j = i + 1 + t
                const double pv = __hiloint2double((int)q.y, (int)q.x);
                GP[i + 1 + t] = pv;
                C[i + 1 + t] = __hiloint2double((int)q.w, (int)q.z);
                sp += pv * Vc[i + 1 + t];
              }
              pend &= ~(1 << u);
            }
          }
        if (!__any(pend != 0)) break;
        if (wall_clock64() - t0 > TRI_TIMEOUT) {
          failed = true;
          break;
        }
        for (int z = 0; z < a.sleep; ++z) __builtin_amdgcn_s_sleep(1);
      }
      sp = riptrm_wave::wave_sum(sp);
      if (lane == 0) red[0][w] = sp;
    }
    if (failed) failflag = 1;
    bar_lds();
    if (failflag) {   // uniform after the barrier (only ever set, then every wave returns)
      if (tid == 0) a.infos[k] = 3;
      return;
    }
    if (hp) hp[1] = (long long)wall_clock64();
    if (stp) {
      const long long t1 = clock64();
      acc0 += t1 - tq;
      tq = t1;
    }
    // this workgroup has read pass i + 1: the parity of pass i + 2 (= pass i's) may be reused
    const int64_t pn = gbase + (int64_t)((pass + 1) & 1) * par;
    const bool more = i + 1 <= m - 2;
    if (tid == 0 && more) st_gran(rs, pn + m + g, gsp, 0.0, pass + 1);
    // The column step, spread over the eight waves (wave w owns the columns j = lane + 64 q, q = w + 8 t):
    // w = p + a2 v with a2 = -tau (p . v) / 2, the column i + 1 of the updated matrix, its reflector.
    // Two block sums (p . v, its wave partials made in the gather, and the reflector's sum of squares:
    // wave trees then eight partials in a fixed order, so every thread of every workgroup holds the
    // same tau); the column stays in registers.  (One wave doing all of it was a 2.4 us latency chain
    // of the 7 us step at m = 999.)
    constexpr int QT = (EL + 7) / 8;
    const long long q0s = stp ? clock64() : 0;
    const int i2 = i + 2 < m ? i + 2 : i + 1;
    const double gp1 = GP[i + 1], vi1 = Vc[i + 1], cr1 = C[i + 1];
    const double gp2 = GP[i2], vc2 = Vc[i2], cr2 = C[i2];
    double gq[QT], vq[QT], cq[QT];
#pragma unroll
    for (int t = 0; t < QT; ++t) {
      const int q = w + 8 * t, j = lane + 64 * q;
      const bool on = q < EL;   // uniform over the wave
      gq[t] = on ? GP[j] : 0.0;
      vq[t] = on ? Vc[j] : 0.0;
      cq[t] = on ? C[j] : 0.0;
    }
    const long long q1s = stp ? clock64() : 0;
    double s = 0.0;   // p . v from the gather's partials
#pragma unroll
    for (int u = 0; u < 8; ++u) s += red[0][u];
    const double a2 = -0.5 * tau_c * s;
    const double wi1 = gp1 + a2 * vi1;
    double sn = 0.0, cn[QT];   // the reflector's sum over c_j^2, j >= i + 3
#pragma unroll
    for (int t = 0; t < QT; ++t) {
      const int q = w + 8 * t, j = lane + 64 * q;
      const bool on = q < EL;
      const double wj = (on && j > i && j < m) ? gq[t] + a2 * vq[t] : 0.0;
      cn[t] = (on && j > i + 1 && j < m) ? cq[t] - (vq[t] * wi1 + wj * vi1) : 0.0;   // row j's update at column i + 1
      if (on) W[j] = wj;
      sn += j >= i + 3 ? cn[t] * cn[t] : 0.0;
    }
    sn = riptrm_wave::wave_sum(sn);
    if (lane == 0) red[1][w] = sn;
    bar_lds();
    const long long q2s = stp ? clock64() : 0;
    sn = 0.0;
#pragma unroll
    for (int u = 0; u < 8; ++u) sn += red[1][u];
    if (writer && tid == 0) dv[i + 1] = cr1 - (vi1 * wi1 + wi1 * vi1);
    double tau_n = 0.0;
    if (more) {
      // dlarfg on c[i+2 .. m): alpha = c[i+2] by its update formula (every thread)
      const double alpha = cr2 - (vc2 * wi1 + (gp2 + a2 * vc2) * vi1);
      double beta = alpha, scl = 0.0;
      if (sn != 0.0) {
        beta = -copysign(sqrt(alpha * alpha + sn), alpha);
        tau_n = (beta - alpha) / beta;
        scl = 1.0 / (alpha - beta);
      }
      const int64_t co = riptrm_eig::refl_col(m, i + 1) - (i + 2);
#pragma unroll
      for (int t = 0; t < QT; ++t) {
        const int q = w + 8 * t, j = lane + 64 * q;
        if (q < EL) {
          const double vn = (j <= i + 1 || j >= m) ? 0.0 : (j == i + 2 ? 1.0 : cn[t] * scl);
          Vn[j] = vn;
          if (writer && j >= i + 2 && j < m) R[co + j] = vn;
        }
      }
      if (writer && tid == 0) {
        ev[i + 1] = beta;
        R[riptrm_eig::refl_tau(m) + i + 1] = tau_n;
      }
      if (stp) {
        const long long q3s = clock64();
        sa += q1s - q0s;
        sb += q2s - q1s;
        sc += q3s - q2s;
      }
    }
    // (v_{i+1} complete in LDS before the update's dot products.  Taking it as c scl from a copy of c
    // instead, without this barrier, was slower: OUT=r6tri13, 14.4k vs 13.2k cycles per step -- the
    // waves then publish and start polling at spread times)
    bar_lds();
    if (stp) {
      const long long t1 = clock64();
      acc1 += t1 - tq;
      tq = t1;
    }
    if (!more) break;
    // rank-two update of own rows l >= i + 2 (row i + 1 is finished: its diagonal is d_{i+1}), fused
    // with p^(i+1)_l = tau_{i+1} A'_l. v_{i+1}; publish pass i + 2.  (v, w, v_{i+1} read from LDS per
    // row: held in registers beside the rows they spill.  Columns outer with each w_j, v_j read once for
    // all RW rows measured no faster: 5.70 vs 5.71 ms per reduction at m = 999, slower at 199 x 64 --
    // the rows then publish together at the end, OUT=r6upd)
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
        // {p_l, A_{l, i+2}}: column i + 2 sits in lane (i + 2) mod 64, register (i + 2) / 64
        const int qc = (i + 2) >> 6;
        double ac = Ar[s][0];
#pragma unroll
        for (int q = 1; q < EL; ++q) ac = q == qc ? Ar[s][q] : ac;
        if (lane == ((i + 2) & 63)) st_pair(rs, pn + l, gsp, p, ac, pass + 1);
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

// (T + lam I) y = r on ONE wave by partitioned elimination: lane k owns rows kL .. kL + L - 1 (L = EL;
// rows past m padded as decoupled unit rows), its first L - 1 rows interior, the last a separator.
// Each lane factors its interior block (LDL^T, pivots in registers) and solves it for the right-hand
// side (z) and for the couplings to the separator before (u) and its own (w); the separators' 64 x 64
// tridiagonal Schur complement is solved by lane 0 (Thomas); interiors x = z - u x_prev - w x_sep.
// A symmetric reordering of the LDL^T the serial ldl_newton runs (stable for T + lam I positive
// definite, what the secular Newton keeps); for an indefinite T (the CG skip test at lam = 0) a tiny
// pivot shows up as a large residual, which that test checks.  u, w live in LDS (UT, WT: element i of
// lane k at i 64 + k, bank-conflict free), the Schur complement's rows and factors in RS[7][64].
template <int L>
struct PartSolve {
  double rpv[L - 1], lo[L - 1];   // interior pivots' reciprocals and L multipliers
  double a_s, o_l2, o_l1;         // separator diagonal (+ lam), e at rows L - 2 and L - 1
  lds_t *UT, *WT, *RS;
  int lane, base, m;
  // RS rows: 0 Lc, 1 D, 2 Uc, 3 rhs, 4 denom, 5 c', 6 x
  __device__ __forceinline__ void factor(const lds_t* d, const lds_t* e, int m_, double lam, lds_t* ut, lds_t* wt, lds_t* rs,
                                         int lane_) {
    UT = ut;
    WT = wt;
    RS = rs;
    lane = lane_;
    m = m_;
    base = lane * L;
    double a[L], o[L];
#pragma unroll
    for (int i = 0; i < L; ++i) {
      const int j = base + i;
      a[i] = j < m ? d[j] + lam : 1.0;
      o[i] = j < m - 1 ? e[j] : 0.0;
    }
    const double eprev = (base > 0 && base - 1 < m - 1) ? e[base - 1] : 0.0;
    a_s = a[L - 1];
    o_l2 = o[L - 2];
    o_l1 = o[L - 1];
    double pv = a[0];
#pragma unroll
    for (int i = 1; i < L - 1; ++i) {
      rpv[i - 1] = riptrm_eig::rcp_nr(pv);
      lo[i - 1] = o[i - 1] * rpv[i - 1];
      pv = a[i] - lo[i - 1] * o[i - 1];
    }
    rpv[L - 2] = riptrm_eig::rcp_nr(pv);
    const double* rp = rpv;
    // u: right-hand side eprev at interior row 0
    double g = eprev, gu[L - 1];
    gu[0] = g;
#pragma unroll
    for (int i = 1; i < L - 1; ++i) gu[i] = -lo[i - 1] * gu[i - 1];
    double u = gu[L - 2] * rp[L - 2];
    UT[(L - 2) * 64 + lane] = u;
    const double u_last = u;
#pragma unroll
    for (int i = L - 3; i >= 0; --i) {
      u = gu[i] * rp[i] - lo[i] * u;
      UT[i * 64 + lane] = u;
    }
    const double u_first = u;
    // w: right-hand side o[L - 2] at interior row L - 2
    double w = o_l2 * rp[L - 2];
    WT[(L - 2) * 64 + lane] = w;
    const double w_last = w;
#pragma unroll
    for (int i = L - 3; i >= 0; --i) {
      w = -lo[i] * w;
      WT[i * 64 + lane] = w;
    }
    const double w_first = w;
    // the separators' Schur complement: row k couples x_{s_{k-1}} (Lc), x_{s_k} (D), x_{s_{k+1}} (Uc)
    const double u_nx = __shfl(u_first, lane < 63 ? lane + 1 : 63), w_nx = __shfl(w_first, lane < 63 ? lane + 1 : 63);
    RS[0 * 64 + lane] = -o_l2 * u_last;
    RS[1 * 64 + lane] = (a_s - o_l2 * w_last) - (lane < 63 ? o_l1 * u_nx : 0.0);
    RS[2 * 64 + lane] = lane < 63 ? -o_l1 * w_nx : 0.0;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) {   // Thomas factors: 1 / denom_k, c'_k
      double cp = 0.0;
#pragma unroll 8
      for (int k = 0; k < 64; ++k) {
        const double rden = riptrm_eig::rcp_nr(RS[1 * 64 + k] - (k > 0 ? RS[0 * 64 + k] * cp : 0.0));
        cp = RS[2 * 64 + k] * rden;
        RS[4 * 64 + k] = rden;
        RS[5 * 64 + k] = cp;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  // y = (T + lam I)^-1 r into y (natural order); returns the wave's sum of y_j * q_j over j < m
  // (q = y when q is null: ||y||^2)
  __device__ __forceinline__ double solve(const lds_t* r, lds_t* y, const lds_t* q) {
    double rr[L];
#pragma unroll
    for (int i = 0; i < L; ++i) rr[i] = base + i < m ? r[base + i] : 0.0;
    double gz[L - 1];
    gz[0] = rr[0];
#pragma unroll
    for (int i = 1; i < L - 1; ++i) gz[i] = rr[i] - lo[i - 1] * gz[i - 1];
    double z[L - 1];
    z[L - 2] = gz[L - 2] * rpv[L - 2];
#pragma unroll
    for (int i = L - 3; i >= 0; --i) z[i] = gz[i] * rpv[i] - lo[i] * z[i + 1];
    const double z_nx = __shfl(z[0], lane < 63 ? lane + 1 : 63);
    RS[3 * 64 + lane] = (rr[L - 1] - o_l2 * z[L - 2]) - (lane < 63 ? o_l1 * z_nx : 0.0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) {
      double yp = 0.0;
#pragma unroll 8
      for (int k = 0; k < 64; ++k) {
        yp = (RS[3 * 64 + k] - (k > 0 ? RS[0 * 64 + k] * yp : 0.0)) * RS[4 * 64 + k];
        RS[6 * 64 + k] = yp;
      }
      double x = RS[6 * 64 + 63];
#pragma unroll 8
      for (int k = 62; k >= 0; --k) {
        x = RS[6 * 64 + k] - RS[5 * 64 + k] * x;
        RS[6 * 64 + k] = x;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const double xs = RS[6 * 64 + lane], xp = lane > 0 ? RS[6 * 64 + lane - 1] : 0.0;
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < L - 1; ++i) {
      const double x = (z[i] - UT[i * 64 + lane] * xp) - WT[i * 64 + lane] * xs;
      const int j = base + i;
      if (j < m) {
        const double qv = q ? q[j] : x;
        y[j] = x;
        acc += x * qv;
      }
    }
    if (base + L - 1 < m) {
      const double qv = q ? q[base + L - 1] : xs;
      y[base + L - 1] = xs;
      acc += xs * qv;
    }
    return riptrm_wave::wave_sum(acc);
  }
};

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

// The eigenvector of T (d, e, e2 = e^2; split where e_j = 0) for its smallest eigenvalue lt, unnormalised,
// into Z[0 .. m) by one thread: riptrm_eig::twisted_vector for t = 0 (dlar1v's twisted factorisation of
// T - lt I, z_r = 1 at the twist r where |gamma_r| is least, in the first block of the split T holding
// an eigenvalue within delta of lt), restructured for one thread's latency: every pass loads four
// steps' operands ahead, the pivots' reciprocals come off the chains (the pass that needs D+ ratios
// reads them from DP, the last pass is one multiply per step), no divisions.  DP: scratch (D+).
// split: T has some e_j = 0 (j < m - 1).  Without one the block is the whole T and the forward pass is
// the D+ chain alone (the block search's two Sturm counts, and its per-step branches, only matter
// between splits): one dependent chain per step instead of three.
__device__ __forceinline__ void twisted_min(lds_t* Z, lds_t* DP, const lds_t* d, const lds_t* e, const lds_t* e2, int m,
                                            double lt, double delta, double pivmin, bool split) {
  using riptrm_eig::rcp_nr;
  const double xa = lt - delta, xb = lt + delta;
  int blo = 0, bhi = m - 1, bs = 0, ca = 0, cb = 0;
  bool found = false;
  double qa = 0.0, qb = 0.0, dp = 0.0;
  if (!split) {
    dp = d[0] - lt;
    if (fabs(dp) < pivmin) dp = -pivmin;
    DP[0] = dp;
    int j = 1;
    for (; j + 4 <= m; j += 4) {
      const double d0 = d[j], d1 = d[j + 1], d2 = d[j + 2], d3 = d[j + 3];
      const double f0 = e2[j - 1], f1 = e2[j], f2 = e2[j + 1], f3 = e2[j + 2];
      dp = (d0 - lt) - f0 * rcp_nr(dp);
      if (fabs(dp) < pivmin) dp = -pivmin;
      DP[j] = dp;
      dp = (d1 - lt) - f1 * rcp_nr(dp);
      if (fabs(dp) < pivmin) dp = -pivmin;
      DP[j + 1] = dp;
      dp = (d2 - lt) - f2 * rcp_nr(dp);
      if (fabs(dp) < pivmin) dp = -pivmin;
      DP[j + 2] = dp;
      dp = (d3 - lt) - f3 * rcp_nr(dp);
      if (fabs(dp) < pivmin) dp = -pivmin;
      DP[j + 3] = dp;
    }
    for (; j < m; ++j) {
      dp = (d[j] - lt) - e2[j - 1] * rcp_nr(dp);
      if (fabs(dp) < pivmin) dp = -pivmin;
      DP[j] = dp;
    }
  }
  // forward: the Sturm counts at lt -+ delta (the block) and D+ (restarting at every split)
  auto fstep = [&](int j, double dj, double ejm, double ej) {
    const bool start = j == bs;
    const double ej2 = start ? 0.0 : ejm * ejm;
    qa = (dj - xa) - (start ? 0.0 : ej2 * rcp_nr(qa));
    qb = (dj - xb) - (start ? 0.0 : ej2 * rcp_nr(qb));
    dp = (dj - lt) - (start ? 0.0 : ej2 * rcp_nr(dp));
    if (fabs(qa) < pivmin) qa = -pivmin;
    if (fabs(qb) < pivmin) qb = -pivmin;
    if (fabs(dp) < pivmin) dp = -pivmin;
    DP[j] = dp;
    ca += qa < 0.0;
    cb += qb < 0.0;
    if (j == m - 1 || ej == 0.0) {   // block bs .. j ends: the first one with an eigenvalue near lt
      if (!found && cb - ca > 0) {
        found = true;
        blo = bs;
        bhi = j;
      }
      ca = cb = 0;
      bs = j + 1;
    }
  };
  if (split) {
    int j = 0;
    for (; j + 4 <= m; j += 4) {
      const double d0 = d[j], d1 = d[j + 1], d2 = d[j + 2], d3 = d[j + 3];
      const double em = j > 0 ? e[j - 1] : 0.0, e0 = e[j], e1 = e[j + 1], e2v = e[j + 2], e3 = j + 3 < m - 1 ? e[j + 3] : 0.0;
      fstep(j, d0, em, e0);
      fstep(j + 1, d1, e0, e1);
      fstep(j + 2, d2, e1, e2v);
      fstep(j + 3, d3, e2v, e3);
    }
    for (; j < m; ++j) fstep(j, d[j], j > 0 ? e[j - 1] : 0.0, j < m - 1 ? e[j] : 0.0);
  }
  // backward over the block: D- and gamma_j = D+_j + D-_j - (d_j - lt) (gamma_bhi = D+_bhi); Z[j] =
  // e_{j-1} / D-_j for the solve above the twist
  double dm = d[bhi] - lt;
  if (fabs(dm) < pivmin) dm = -pivmin;
  double best = fabs(DP[bhi]);
  int r = bhi;
  if (bhi > blo) Z[bhi] = e[bhi - 1] * rcp_nr(dm);
  auto bstep = [&](int i, double di, double ei, double dpi, double eim) {
    const double dil = di - lt;
    dm = dil - (ei * ei) * rcp_nr(dm);
    if (fabs(dm) < pivmin) dm = -pivmin;
    const double g = fabs(dpi + dm - dil);
    const bool better = g < best;
    best = better ? g : best;
    r = better ? i : r;
    Z[i] = eim * rcp_nr(dm);
  };
  int i = bhi - 1;
  for (; i - 3 >= blo; i -= 4) {
    const double d0 = d[i], d1 = d[i - 1], d2 = d[i - 2], d3 = d[i - 3];
    const double e0 = e[i], e1 = e[i - 1], e2v = e[i - 2], e3 = e[i - 3];
    const double p0 = DP[i], p1 = DP[i - 1], p2 = DP[i - 2], p3 = DP[i - 3];
    const double e4 = i - 4 >= 0 ? e[i - 4] : 0.0;
    bstep(i, d0, e0, p0, e1);
    bstep(i - 1, d1, e1, p1, e2v);
    bstep(i - 2, d2, e2v, p2, e3);
    bstep(i - 3, d3, e3, p3, e4);
  }
  for (; i >= blo; --i) bstep(i, d[i], e[i], DP[i], i > 0 ? e[i - 1] : 0.0);
  // the solve outward from the twist: z_j = -(e_{j-1} / D-_j) z_{j-1} above, -(e_j / D+_j) z_{j+1} below
  double z = 1.0;
  for (int k = r + 1; k <= bhi; ++k) {
    z = -Z[k] * z;
    Z[k] = z;
  }
  z = 1.0;
  for (int k = r - 1; k >= blo; --k) {
    z = -(e[k] * rcp_nr(DP[k])) * z;
    Z[k] = z;
  }
  Z[r] = 1.0;
  for (int k = 0; k < blo; ++k) Z[k] = 0.0;
  for (int k = bhi + 1; k < m; ++k) Z[k] = 0.0;
}

// scalar slots this header uses (riptrm_trs_big.hip Sc)
struct TriSc {
  int cg_ok, p1obj, kind, lam1, mineig, interior, delta, an, atol, it, done, fallback, newton;
};

// After k_tridiag_dist (and the reflector application: b = H^T a at boff): mode 0 the subproblem, mode 1
// the smallest eigenvalue only.  One workgroup of 256 threads per slot: waves 0 / 1 the extreme
// eigenvalues; then, at once, wave 0 the secular Newton (lane 0) and the boundary candidate's model
// value, waves 1 and 3 the CG's certified skip test (cg_skip; k_cg_wg's bounds) and wave 2 the
// hard-case test (lam_min's multiplicity and the component of b on its twisted eigenvector; a hard
// case sets the fallback flag and ends there); then wave 1 SciPy's CG on T y = -b unless the skip
// test shows that its candidate cannot win.  Writes the boundary / interior candidate in T
// coordinates at peoff (the host applies H), lam_min at evoff[0].
constexpr int TRI_SOLVE_ARRAYS = 13;   // LDS vectors of 64 EL doubles
template <int EL>
__global__ void __launch_bounds__(256) k_tri_solve(double* base, int64_t sd, int32_t* infos, int m, int64_t d_off,
                                                   int64_t e_off, int64_t boff, int64_t aoff_vec, int64_t peoff,
                                                   int64_t cgxoff, int64_t evoff, int64_t scoff, TriSc S,
                                                   const double* Dg, int64_t dstride, const int32_t* ids, double tolhc,
                                                   int mode, int cg_skip, int eig_known, int serial, long long* stamps) {
  // stamps (diagnostics, RIPTRM_TRI_STAMPS=1; slot 0): clock64 at [0] start, [1] extreme eigenvalues,
  // [2] hard-case test done (wave 2), [3] the Newton done (wave 0), [4] the CG done or skipped (wave 1),
  // [5] end, [6] Newton steps, [7] CG iterations, [8] the skip test done (wave 1), [9] 1: CG skipped
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
  lds_t* pz = cx + V;  // the skip test: T^-1 b and its LDL^T factor
  lds_t* lz = pz + V;
  lds_t* rz = lz + V;
  __shared__ double red[8];
  // lam_min, lam_max, multiplicity, xobj, lam1, CG ok, p1obj, Newton steps, ghard, -Delta / ||y||,
  // ||T^-1 b||, b . T^-1 b, its residual
  __shared__ double xs[13];
  __shared__ int ic[128];   // the skip test's Sturm counts
  __shared__ double rs0[7 * 64], rs1[7 * 64];   // PartSolve's Schur complements (Newton, skip test)
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
  int sp0 = 0;
  for (int j = tid; j < V; j += 256) {
    double ej = e[j];
    if (j < m - 1 && fabs(ej) <= 4.0 * eps * tn0) ej = 0.0;
    e[j] = ej;
    e2[j] = ej * ej;
    sp0 |= j < m - 1 && ej == 0.0;
  }
  const bool split = __syncthreads_or(sp0);
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
  // lam_min (wave 0) and lam_max (wave 1), or (eig_known, mode 0) the ones a mode-1 pass over the same
  // T left at evoff[0], evoff[1] (the eigendecomposition cache hands them on with T: same bits)
  if (w < 2) {
    const double lx = (eig_known && mode == 0) ? sb[evoff + w] : extreme_eig(d, e2, m, w == 1, glo, ghi, fudge, tnorm, lane);
    if (lane == 0) xs[w] = lx;
  }
  __syncthreads();
  const double lmin = xs[0], lmaxv = xs[1];
  if (stp && tid == 0) stp[1] = clock64();
  __syncthreads();
  if (mode == 1) {
    if (tid == 0) {
      sb[evoff] = lmin;
      sb[evoff + 1] = lmaxv;
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
  const double lmx = fmax(fabs(lmin), fabs(lmaxv));
  if (w == 0) {
    // the secular Newton of k_secular: ||(T + l1 I)^-1 b|| = Delta from l1 = -lam_min + ||b|| / Delta;
    // the solves by the whole wave (PartSolve), or by lane 0 alone (ldl_newton; serial = 1, A/B)
    if (!serial) {
      const double lo = -lmin;
      double l1 = lo + gn / Delta, bl = lo, br = INFINITY;
      int itn = 0;
      PartSolve<EL> ps;
      for (; itn < 100; ++itn) {   // (uniform: every lane holds the same sums)
        ps.factor(d, e, m, l1, lf, rd, (lds_t*)rs0, lane);
        const double s2 = ps.solve(b, y, nullptr);
        const double s3 = ps.solve(y, t2, y);
        const double xn = sqrt(s2);
        const double f = 1.0 / xn - 1.0 / Delta;
        const double fp = s3 / (xn * xn * xn);
        if (fabs(f) * Delta <= 4.0 * eps) break;
        if (f > 0.0) br = fmin(br, l1);
        else bl = fmax(bl, l1);
        double nl = l1 - f / fp;
        if (nl <= bl) nl = 0.5 * (bl + l1);
        const double tol = 1e-15 * fmax(1.0, fabs(l1));
        if (fabs(nl - l1) <= tol || br - bl <= tol) {
          l1 = nl;
          break;
        }
        l1 = nl;
      }
      ps.factor(d, e, m, l1, lf, rd, (lds_t*)rs0, lane);
      const double s2 = ps.solve(b, y, nullptr);
      if (lane == 0) {
        xs[4] = l1;
        xs[7] = (double)itn;
        xs[9] = -Delta / sqrt(s2);
        if (stp) stp[6] = itn;
      }
    } else if (lane == 0) {
      // The iterates bracket the root: f > 0 right of it, f < 0 left (bl starts at the pole -lam_min).
      // A step to or below bl bisects towards it (k_secular bisects towards the pole: the same
      // sequence while no iterate has landed left of the root); a step past br is taken (bisecting
      // there costs ~45 steps where f bends the wrong way: OUT=r6tri9), and a bracket shrunk to the
      // stopping tolerance, or |f| at rounding level, ends the loop (near a hard case the LDL^T's f is
      // rounding noise at the step tolerance: 100 steps without these)
      const double lo = -lmin;
      double l1 = lo + gn / Delta, bl = lo, br = INFINITY;
      int itn = 0;
      for (; itn < 100; ++itn) {
        double s2, s3;
        ldl_newton(d, e, e2, m, l1, b, y, t2, lf, rd, true, s2, s3);
        const double xn = sqrt(s2);
        const double f = 1.0 / xn - 1.0 / Delta;
        const double fp = s3 / (xn * xn * xn);
        if (fabs(f) * Delta <= 4.0 * eps) break;   // ||y|| = Delta to rounding: no step can do better
        if (f > 0.0) br = fmin(br, l1);
        else bl = fmax(bl, l1);
        double nl = l1 - f / fp;
        if (nl <= bl) nl = 0.5 * (bl + l1);
        const double tol = 1e-15 * fmax(1.0, fabs(l1));
        if (fabs(nl - l1) <= tol || br - bl <= tol) {
          l1 = nl;
          break;
        }
        l1 = nl;
      }
      double s2, s3;
      ldl_newton(d, e, e2, m, l1, b, y, t2, lf, rd, false, s2, s3);
      xs[4] = l1;
      xs[7] = (double)itn;
      xs[9] = -Delta / sqrt(s2);
      if (stp) stp[6] = itn;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // lane 0's solve -> the wave
    // the boundary candidate pe = -Delta y / ||y|| and xobj = pe^T T pe / 2 + b^T pe (lane-strided)
    const double scl = xs[9];
    double o0 = 0.0, o1 = 0.0;
    for (int j = lane; j < m; j += 64) {
      const double yj = y[j] * scl;
      const double tp = d[j] * yj + (j > 0 ? e[j - 1] * (y[j - 1] * scl) : 0.0) + (j < m - 1 ? e[j] * (y[j + 1] * scl) : 0.0);
      o0 += yj * tp;
      o1 += b[j] * yj;
    }
    for (int j = lane; j < m; j += 64) y[j] *= scl;   // (after every lane's reads: one wave, in order)
    o0 = riptrm_wave::wave_sum(o0);
    o1 = riptrm_wave::wave_sum(o1);
    if (lane == 0) {
      xs[3] = 0.5 * o0 + o1;
      if (stp) stp[3] = clock64();
    }
  } else if (w == 1 || w == 3) {
    // The CG's certified skip (k_cg_wg's bounds, from T alone): lam_s <= min |lambda_i| by Sturm counts
    // at 64 points either side of 0 (x = -+ lmx 2^(-7 l / 16), down to 2e-9 lmx; wave 1 the negative
    // side and 0 itself, wave 3 the positive side), and p* = -T^-1 b by the LDL^T at 0 with its
    // residual, whose error ||T^-1 res|| <= ||res|| / lam_s enters both bounds.
    const double x = w == 1 ? (lane == 63 ? 0.0 : -lmx * exp2(-7.0 * (62 - lane) / 16.0)) : lmx * exp2(-7.0 * lane / 16.0);
    const int cnt = (cg_skip && lmx > 0.0) ? sturm_count_df(d, e2, m, x) : 0;
    ic[w == 1 ? lane : 64 + lane] = cnt;
    if (w == 1 && cg_skip) {
      if (!serial) {
        PartSolve<EL> ps;
        ps.factor(d, e, m, 0.0, lz, rz, (lds_t*)rs1, lane);
        (void)ps.solve(b, pz, nullptr);
      } else if (lane == 0) {
        double s2, s3;
        ldl_newton(d, e, e2, m, 0.0, b, pz, nullptr, lz, rz, false, s2, s3);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (w == 1 && cg_skip) {   // the residual T ps - b and b . ps (ps = T^-1 b, p* = -ps)
      double rr = 0.0, bp = 0.0, pp = 0.0;
      for (int j = lane; j < m; j += 64) {
        const double tp = d[j] * pz[j] + (j > 0 ? e[j - 1] * pz[j - 1] : 0.0) + (j < m - 1 ? e[j] * pz[j + 1] : 0.0);
        rr += (tp - b[j]) * (tp - b[j]);
        bp += b[j] * pz[j];
        pp += pz[j] * pz[j];
      }
      rr = riptrm_wave::wave_sum(rr);
      bp = riptrm_wave::wave_sum(bp);
      pp = riptrm_wave::wave_sum(pp);
      if (lane == 0) {
        xs[10] = sqrt(pp);
        xs[11] = bp;
        xs[12] = sqrt(rr);
        if (stp) stp[8] = clock64();
      }
    }
  } else if (w == 2) {
    // hard-case test (k_secular): the component of b on the eigenspace of lam_min (eigenvalues within
    // 1e-12 max(1, max |lambda|)); a multiple lam_min or a hard case goes to the eigendecomposition path
    const double hard_tol = 1e-12 * fmax(1.0, lmx);
    if (lane == 0) {
      xs[2] = (double)sturm_count_df(d, e2, m, lmin + hard_tol);
      twisted_min(z, cx, d, e, e2, m, lmin, 16.0 * eps * tnorm, pivmin, split);   // (cx: the CG's, free until the barrier)
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // lane 0's vector -> the wave
    double zb = 0.0, zz = 0.0;
    for (int j = lane; j < m; j += 64) {
      zb += z[j] * b[j];
      zz += z[j] * z[j];
    }
    zb = riptrm_wave::wave_sum(zb);
    zz = riptrm_wave::wave_sum(zz);
    if (lane == 0) {
      xs[8] = fabs(zb) / sqrt(zz);
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
  // the skip: no iterate with ||T p1 + b|| <= e := 1e-5 ||a|| can pass RIPTRM.py:294-298 when
  //   ||p1|| >= ||p*|| - e / lam_s >= Delta   or   p1obj >= -b^T T^-1 b / 2 - e^2 / (2 lam_s) > xobj
  // (k_cg_wg), with ||p*|| >= ||ps|| - ||res|| / lam_s and b^T T^-1 b <= b . ps + ||b|| ||res|| / lam_s
  bool skip = false;
  if (cg_skip) {
    const int c0 = ic[63];   // eigenvalues below 0
    // the strongest bounds: the largest |x| with every negative eigenvalue below x (count c0), the
    // largest x > 0 with none in [0, x) (count c0); none certified: 0 (no skip)
    double ng = 0.0, ps = 0.0;
    for (int l = 0; l < 63; ++l)
      if (ic[l] == c0) ng = fmax(ng, lmx * exp2(-7.0 * (62 - l) / 16.0));
    for (int l = 0; l < 64; ++l)
      if (ic[64 + l] == c0) ps = fmax(ps, lmx * exp2(-7.0 * l / 16.0));
    if (c0 == 0) ng = INFINITY;
    if (c0 == m) ps = INFINITY;
    const double lam_s = fmin(ng, ps) * (1.0 - 1e-6) - 4.0 * m * eps * tnorm;
    const double pn = xs[10], bp = xs[11], resn = xs[12], xobj = xs[3];
    if (lam_s > 1e-8 * lmx && isfinite(pn) && isfinite(bp) && isfinite(resn) && isfinite(xobj)) {
      const double e1 = 1e-5 * an;
      const bool far = (pn - resn / lam_s) * (1.0 - 1e-6) - e1 / lam_s >= Delta;
      const double s2u = bp + gn * resn / lam_s;
      const double p1lo = -0.5 * s2u - 0.5 * e1 * e1 / lam_s;
      const bool worse = p1lo - xobj > 1e-6 * (fabs(s2u) + fabs(xobj)) + 1e-10 * (e1 * 1e5) * Delta;
      skip = far || worse;
    }
  }
  if (skip) {   // uniform
    if (tid == 0) {
      sc[S.an] = an;
      sc[S.atol] = 1e-5 * an;
      sc[S.it] = 0.0;
      sc[S.done] = 4.0;
      sc[S.cg_ok] = 0.0;
      sc[S.p1obj] = 0.0;
      sc[S.delta] = Delta;
      xs[5] = 0.0;
      xs[6] = 0.0;
      if (stp) {
        stp[4] = clock64();
        stp[9] = 1;
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
  }
  __syncthreads();
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

// ---- blocked reflector application ----------------------------------------------------------------
// RB consecutive reflections H_a = I - tau_a u_a u_a^T (a = 0 .. RB - 1) compose to H_0 ... H_{RB-1} =
// I - U T U^T with T upper triangular (the compact WY form, LAPACK dlarft's forward columnwise recurrence:
// T_aa = tau_a, T_{0:a, a} = -tau_a T_{0:a, 0:a} G_{0:a, a}, G_ab = u_a . u_b).  Applied first-to-last
// (v <- H_{RB-1} ... H_0 v) the block maps v to v - U T^T s, last-to-first to v - U T s, s = U^T v: the
// reflections' exact composition, the sums in another order.  T depends on the reflectors only:
// k_refl_gram forms the blocks' T once per tridiagonalisation, for both applications.
constexpr int RB = 16;
__host__ __device__ constexpr int refl_blocks(int m) { return (m - 1 + RB - 1) / RB; }
__host__ __device__ constexpr int64_t refl_gram_doubles(int m) { return (int64_t)refl_blocks(m) * RB * RB; }

// u_i[j] of reflector i (riptrm_eig refl_col layout: j = i + 1 .. m - 1, u_i[i + 1] = 1), 0 elsewhere
__device__ __forceinline__ double refl_u(const double* R, int m, int i, int j) {
  const bool ok = i < m - 1 && j > i && j < m;
  return ok ? R[riptrm_eig::refl_col(m, i) - i - 1 + j] : 0.0;
}

// T of block blockIdx.x (reflectors b RB .. b RB + RB - 1; absent ones tau 0) of slot k0 + blockIdx.y into
// the slot at goff + b RB^2 (row-major RB x RB, zero below the diagonal): G's upper triangle by thread
// (a, c) < 120 over chunks of 128 rows staged in LDS (coalesced: consecutive threads, consecutive rows of
// one reflector), two accumulation chains; then thread a < RB forms row a of T (its own earlier entries
// and G only: no barrier per column).  (Round 6 first form: 120 accumulators per thread and 120 wave
// sums, 31.5 us per 13 x 64 blocks at order 199, 17.9 us at 999.)
__global__ void __launch_bounds__(256) k_refl_gram(double* base, int64_t sd, int k0, int m, int64_t r_off, int64_t goff) {
  constexpr int NP = RB * (RB - 1) / 2, CH = 128;
  __shared__ double us[CH][RB + 1];
  __shared__ double gs[RB][RB];
  double* sb = base + (int64_t)(k0 + blockIdx.y) * sd;
  const double* R = sb + r_off;
  const int b = blockIdx.x, i0 = b * RB, tid = threadIdx.x;
  int pa = 0, pc = 1;
  if (tid < NP) {
    int x = tid;
    while (x >= RB - 1 - pa) {
      x -= RB - 1 - pa;
      ++pa;
    }
    pc = pa + 1 + x;
  }
  double acc0 = 0.0, acc1 = 0.0;
  for (int j0 = i0 + 1; j0 < m; j0 += CH) {
    __syncthreads();   // (the previous chunk is consumed)
    // all eight loads of a thread issued before any is used: clamped addresses, masked after (a load
    // under the bound's condition is waited for one at a time)
    double x[CH * RB / 256];
#pragma unroll
    for (int r = 0; r < CH * RB / 256; ++r) {
      const int q = tid + 256 * r, a = q / CH, i = i0 + a, j = j0 + q % CH;
      const bool ok = i < m - 1 && j > i && j < m;
      x[r] = R[ok ? riptrm_eig::refl_col(m, i) - i - 1 + j : 0];
    }
#pragma unroll
    for (int r = 0; r < CH * RB / 256; ++r) {
      const int q = tid + 256 * r, a = q / CH, i = i0 + a, j = j0 + q % CH;
      us[q % CH][a] = (i < m - 1 && j > i && j < m) ? x[r] : 0.0;
    }
    __syncthreads();
    if (tid < NP) {
#pragma unroll 8
      for (int jj = 0; jj < CH; jj += 2) {
        acc0 += us[jj][pa] * us[jj][pc];
        acc1 += us[jj + 1][pa] * us[jj + 1][pc];
      }
    }
  }
  if (tid < NP) gs[pa][pc] = acc0 + acc1;
  __syncthreads();
  if (tid < RB) {
    const int nt = riptrm_eig::refl_tau(m);
    double tr[RB];   // row tid of T
#pragma unroll
    for (int c = 0; c < RB; ++c) {
      const double tc = i0 + c < m - 1 ? R[nt + i0 + c] : 0.0;
      double x = c == tid ? tc : 0.0;
      if (tid < c) {
        double z = 0.0;
#pragma unroll
        for (int l = 0; l < c; ++l)
          if (l >= tid) z += tr[l] * gs[l][c];
        x = -tc * z;
      }
      tr[c] = x;
    }
    double* T = sb + goff + (int64_t)b * RB * RB + tid * RB;
#pragma unroll
    for (int c = 0; c < RB; ++c) T[c] = tr[c];
  }
}

// v <- H^T v (backward = 0: H_{m-2} ... H_0 v) or H v (backward = 1) for orders up to 1024 on one
// 512-thread workgroup (elements j = t and t + 512 on thread t), RB reflections per round: the RB dot
// products s = U^T v (one reduce-scatter per wave, eight partials per value summed in a fixed order),
// then every wave forms c = T^T s (T s backward) itself -- lane a < 16 one row, the s_b and then the c_a
// broadcast by readlane -- and subtracts its sums of c_a u_a[j]: one barrier per round (the partials and
// T double-buffered by round parity, so a wave one round ahead cannot overwrite what a slower one still
// reads).  The next round's reflector entries and T block are loaded during the current one into the
// other of two register sets (the round loop unrolled twice, no copies), unconditionally (a load under a
// condition made the compiler wait for every outstanding load, the prefetch included).
// Instruction issue, not memory, bounds the round (OUT=r6refl: 612 VALU + 325 SALU per wave per round,
// 8.1k of 10k cycles before the first barrier, with wave 0's sequential 16-step solve 1.7k more): the
// address of u_i[j] is the wave-uniform start of reflector i (a buffer load's soffset) plus a per-thread
// byte offset fixed for the whole launch (j clamped into 1 .. m - 1, so every load stays inside the
// reflector triangle), no vector instruction per load; the masks (j > i, j < m) are applied only by
// the one or two waves whose element range straddles the round's reflectors or the order, and a wave
// whose elements all lie at or above the block (or past m) skips its dot products and update.
// Measured (OUT=r6chk3/r6chk4/r6help, m = 999): 255 -> 208 us per application; the first phase still
// 5.8k cycles per round and insensitive to bytes and to where they come from -- reading only live lines
// (no change) and 1, 2 or 4 L2-prefetch workgroups on workgroup 0's XCD (no change) -- so the floor is
// the CU's own vector-memory return path (32 x 512 B per wave per round) and the reduction's issue.
// E elements per thread (1024 / E threads): E = 2 the default, E = 1 four waves per SIMD (A/B,
// RIPTRM_TRI_REFL_E=1)
template <int E>
__global__ void __launch_bounds__(1024 / E) k_refl_blk(double* base, int64_t sd, int k0, int m, int64_t r_off, int64_t goff,
                                                  int64_t voff, int64_t ooff, int backward, long long* stamps) {
  // stamps (RIPTRM_TRI_STAMPS=3, slot 0, thread 0): clock64 cycles summed over the rounds in [0] the
  // operands' arrival + the dot products to the barrier, [1] c, [2] the update
  constexpr int NT = 1024 / E, NW = NT / 64;
  __shared__ double part[2][NW][RB];
  __shared__ double gl[2][RB * RB];   // the round's T (forward: gl[b RB + a] = T_ba; backward T_ab)
  double* sb = base + (int64_t)(k0 + blockIdx.y) * sd;
  const double* R = sb + r_off;
  const double* Gall = sb + goff;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const int nb = refl_blocks(m);
  double v[E];
  unsigned jb[E];   // bytes from u_i[0]'s position to element j (clamped into 1 .. m - 1)
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int j = t + NT * e;
    v[e] = j < m ? sb[voff + j] : 0.0;
    jb[e] = (unsigned)(j < 1 ? 1 : (j > m - 1 ? m - 1 : j)) * 8u;
  }
  // buffer loads: R - 1 as the base, the reflector's start (uniform) as soffset, jb as voffset
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(R - 1), (short)0, 0x7fffffff, 0x00020000);
  const int tg = t < RB * RB ? t : 0, tl = backward ? (tg & (RB - 1)) * RB + (tg >> 4) : tg;
  auto load = [&](int bi, double (&un)[E][RB], double& gn) {
    int b = backward ? nb - 1 - bi : bi;
    b = b < 0 ? 0 : (b >= nb ? nb - 1 : b);
    // elements at or above the block's first reflector all read its first entry's position (one line
    // per wave, not the previous reflectors' tails: half the bytes of a full-width read)
    const unsigned lo = (unsigned)(b * RB + 1) * 8u;
    unsigned jv[E];
#pragma unroll
    for (int e = 0; e < E; ++e) jv[e] = jb[e] > lo ? jb[e] : lo;
#pragma unroll
    for (int a = 0; a < RB; ++a) {
      // (reflectors past m - 2 reread m - 2's entries; their T rows and columns are 0)
      const int i = min(b * RB + a, m - 2), d = i * (m - 2) - (i * (i - 1) >> 1);   // refl_col(m, i) - i
#pragma unroll
      for (int e = 0; e < E; ++e)
        un[e][a] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rsrc, (int)jv[e], d * 8, 0));
    }
    gn = Gall[(int64_t)b * RB * RB + tg];
  };
  long long* stp = (stamps && blockIdx.y == 0 && threadIdx.x == 0) ? stamps : nullptr;
  long long s0 = 0, s1 = 0, s2 = 0, tq = stp ? clock64() : 0;
  auto round = [&](int bi, double (&u)[E][RB], double g, double (&un)[E][RB], double& gn) {
    const int b = backward ? nb - 1 - bi : bi, i0 = b * RB, p = bi & 1;
    bool use[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int jmin = 64 * wu + NT * e, jmax = jmin + 63;   // (uniform)
      use[e] = jmax > i0 && jmin < m;
      if (use[e] && (jmin <= i0 + RB - 1 || jmax >= m)) {
        const int j = t + NT * e;
#pragma unroll
        for (int a = 0; a < RB; ++a) u[e][a] = (j > i0 + a && j < m) ? u[e][a] : 0.0;
      }
    }
    if (t < RB * RB) gl[p][tl] = g;
    load(bi + 1, un, gn);
    {
      static_assert(RB == 16, "k_refl_blk: one reduce-scatter of sixteen sums");
      double pr[RB];
      if constexpr (E == 1) {
#pragma unroll
        for (int a = 0; a < RB; ++a) pr[a] = use[0] ? u[0][a] * v[0] : 0.0;
      } else if (use[0] && use[1]) {
#pragma unroll
        for (int a = 0; a < RB; ++a) pr[a] = u[0][a] * v[0] + u[1][a] * v[1];
      } else if (use[0]) {
#pragma unroll
        for (int a = 0; a < RB; ++a) pr[a] = u[0][a] * v[0];
      } else if (use[1]) {
#pragma unroll
        for (int a = 0; a < RB; ++a) pr[a] = u[1][a] * v[1];
      } else {
#pragma unroll
        for (int a = 0; a < RB; ++a) pr[a] = 0.0;
      }
      const double x = riptrm_wave::wave_sum16(pr);
      if ((lane & 3) == 0) part[p][w][riptrm_wave::wave_sum16_index(lane)] = x;
    }
    bar_lds();   // (not __syncthreads(): its vmcnt(0) would wait for the next round's prefetch)
    if (stp) {
      const long long t1 = clock64();
      s0 += t1 - tq;
      tq = t1;
    }
    double cv[RB];
    {
      const int a = lane & (RB - 1);
      double sa = 0.0;
#pragma unroll
      for (int q = 0; q < NW; ++q) sa += part[p][q][a];
      double ca = 0.0;
#pragma unroll
      for (int c = 0; c < RB; ++c) ca += gl[p][c * RB + a] * riptrm_wave::read_lane(sa, c);
#pragma unroll
      for (int c = 0; c < RB; ++c) cv[c] = riptrm_wave::read_lane(ca, c);
    }
    if (stp) {
      const long long t1 = clock64();
      s1 += t1 - tq;
      tq = t1;
    }
#pragma unroll
    for (int e = 0; e < E; ++e) {
      if (use[e]) {
        double dv = 0.0;
#pragma unroll
        for (int a = 0; a < RB; ++a) dv += cv[a] * u[e][a];
        v[e] -= dv;
      }
    }
    if (stp) {
      const long long t1 = clock64();
      s2 += t1 - tq;
      tq = t1;
    }
  };
  double ua[E][RB], ub[E][RB], ga, gb;
  load(0, ua, ga);
  for (int bi = 0; bi < nb; bi += 2) {
    round(bi, ua, ga, ub, gb);
    if (bi + 1 < nb) round(bi + 1, ub, gb, ua, ga);
  }
#pragma unroll
  for (int e = 0; e < E; ++e)
    if (t + NT * e < m) sb[ooff + t + NT * e] = v[e];
  if (stp) {
    stp[0] = s0;
    stp[1] = s1;
    stp[2] = s2;
  }
}

}  // namespace riptrm_tri
