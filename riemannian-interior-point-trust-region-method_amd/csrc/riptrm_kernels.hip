// riptrm_kernels.hip — MI355X (gfx950) kernels for the RIPTRM tCG hot path + the C-ABI.
//
// Work per lock-step iteration of a batch of independent NonnegPCA instances:
//   k_gemv   : one pass over every active instance's S = Z + Z^T (fp64, HBM-bound):
//              out0 = S*in0 (and out1 = S*in1 for the trial point's 2-RHS pass).
//   k_state  : one 1024-thread workgroup per active instance advances the RIPTRM state machine
//              (barrier Hessian epilogue, tCG iteration, trial point, ratio test, dual clipping,
//              inner/outer loop control, KKT evaluation + log row) until it needs the next S-pass.
// Reference restated: src/solver/RIPTRM.py:41-216 (tCG), :491-571 + :729-730 (barrier Hessian
// and gradient), :574-629 (inner stopping test), :631-705 (acceptance / TR radius), :707-896
// (inner/outer loops), :909-976 (run), src/solver/utils.py:269-368 (KKT residual, evaluation).
#include <hip/hip_runtime.h>
#include <math.h>
#include <string>
#include <vector>
#include <cstring>
#include <cstdio>
#include <type_traits>
#include "riptrm_device.h"
#include "riptrm_ctx.h"
#include "riptrm_wave.h"
#include "riptrm_trs.h"

namespace riptrm {

// Elementwise arithmetic must round exactly like NumPy (no contraction into FMA).
#pragma clang fp contract(off)

typedef double dbl2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ double* vp(const DevParams& P, int k, int b) {
  return P.vec + ((int64_t)k * P.batch + b) * P.ld;
}

// An active-list entry carries the instance and its right-hand-side count (1 or 2), so a consumer
// learns both from ONE load, issued together with the list-count load (slot < grid bound <= batch
// keeps the read in bounds): one dependent memory round trip less at the head of every S-pass and
// state-kernel workgroup.
__device__ __forceinline__ int32_t le_make(int b, int nrhs) { return b * 2 + (nrhs - 1); }
__device__ __forceinline__ int le_b(int32_t e) { return e >> 1; }
__device__ __forceinline__ int le_nrhs(int32_t e) { return (e & 1) + 1; }

// ------------------------------------------------------------------------------------------
// Workgroup reductions (ST_THREADS threads).  Every thread ends with the bitwise-identical
// result, so all scalar control flow downstream is uniform across the workgroup.
// op per slot: 0 = sum, 1 = min (NaN-ignoring), 2 = max (NaN-ignoring).
// ------------------------------------------------------------------------------------------
constexpr int RED_MAX = 10;
struct Red {
  double* buf;  // LDS [2][ST_WAVES][RED_MAX]
  int parity;
};

// lane l <- lane (l ^ off) for one double: two ds_bpermute_b32, no bounds select (64 lanes)
__device__ __forceinline__ double xor_lane(double v, int off) {
  const int addr = ((int)__lane_id() ^ off) << 2;
  const int lo = __builtin_amdgcn_ds_bpermute(addr, __double2loint(v));
  const int hi = __builtin_amdgcn_ds_bpermute(addr, __double2hiint(v));
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double comb(int op, double a, double b) {
  return op == 0 ? a + b : (op == 1 ? fmin(a, b) : fmax(a, b));
}

template <int K>
__device__ __forceinline__ void bred(Red& R, double (&v)[K], const int (&op)[K]) {
  static_assert(K <= RED_MAX, "too many reduction slots");
#pragma unroll
  for (int k = 0; k < K; ++k) {  // in-wave: DPP / permlane reduction (riptrm_wave.h), no LDS
    v[k] = op[k] == 0 ? riptrm_wave::wave_sum(v[k])
                      : (op[k] == 1 ? riptrm_wave::wave_min(v[k]) : riptrm_wave::wave_max(v[k]));
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double* b = R.buf + R.parity * (ST_WAVES * RED_MAX);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < K; ++k) b[w * RED_MAX + k] = v[k];
  }
  __syncthreads();
  static_assert(ST_WAVES == 8, "bred: pairwise tree over 8 wave partials");
#pragma unroll
  for (int k = 0; k < K; ++k) {   // fixed pairwise tree: 3 dependent combines instead of 7
    const double s01 = comb(op[k], b[k], b[RED_MAX + k]);
    const double s23 = comb(op[k], b[2 * RED_MAX + k], b[3 * RED_MAX + k]);
    const double s45 = comb(op[k], b[4 * RED_MAX + k], b[5 * RED_MAX + k]);
    const double s67 = comb(op[k], b[6 * RED_MAX + k], b[7 * RED_MAX + k]);
    v[k] = comb(op[k], comb(op[k], s01, s23), comb(op[k], s45, s67));
  }
  R.parity ^= 1;
}

template <int K>
__device__ __forceinline__ void bsum(Red& R, double (&v)[K]) {
  int op[K];
#pragma unroll
  for (int k = 0; k < K; ++k) op[k] = 0;
  bred<K>(R, v, op);
}

// numpy.minimum / numpy.maximum (NaN-propagating) used by the dual clipping (RIPTRM.py:681-683)
__device__ __forceinline__ double np_min(double a, double b) {
  return (isnan(a) || isnan(b)) ? NAN : (b < a ? b : a);
}
__device__ __forceinline__ double np_max(double a, double b) {
  return (isnan(a) || isnan(b)) ? NAN : (b > a ? b : a);
}

// ------------------------------------------------------------------------------------------
// k_gemv: batched fp64 mat-vec over the active instances.  Workgroup = GV_RB rows of one
// instance; each wave owns GV_RW rows and streams them in 1 KiB (64 lanes x 16 B) column
// chunks, v read as 16 B per lane (L1/L2-resident, 32 KiB per instance at n = 4000), FMAs into
// per-lane partials, then a 64-lane butterfly per row.  S is read exactly once per pass.
// ------------------------------------------------------------------------------------------
template <int NR>
__device__ __forceinline__ void gemv_rows(const DevParams& P, int b, int rb) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int row0 = rb * GV_RB + w * GV_RW;
  const int64_t ld = P.ld;
  const double* __restrict__ Sb = P.S + (int64_t)b * P.inst_stride + (int64_t)row0 * ld;
  const double* __restrict__ v0 = vp(P, V_IN0, b);
  const double* __restrict__ v1 = vp(P, V_IN1, b);
  double a0[GV_RW], a1[GV_RW];
#pragma unroll
  for (int k = 0; k < GV_RW; ++k) { a0[k] = 0.0; a1[k] = 0.0; }

  int64_t col = 2 * lane;
  // main loop: two 1 KiB chunks per row in flight per iteration
  for (; col + 128 < ld; col += 256) {
    dbl2 s[2][GV_RW];
#pragma unroll
    for (int k = 0; k < GV_RW; ++k) {
      s[0][k] = __builtin_nontemporal_load((const dbl2*)(Sb + k * ld + col));
      s[1][k] = __builtin_nontemporal_load((const dbl2*)(Sb + k * ld + col + 128));
    }
    const dbl2 x00 = *(const dbl2*)(v0 + col);
    const dbl2 x01 = *(const dbl2*)(v0 + col + 128);
    dbl2 x10 = dbl2{0.0, 0.0}, x11 = dbl2{0.0, 0.0};
    if (NR == 2) {
      x10 = *(const dbl2*)(v1 + col);
      x11 = *(const dbl2*)(v1 + col + 128);
    }
#pragma unroll
    for (int k = 0; k < GV_RW; ++k) {
      a0[k] = __builtin_fma(s[0][k].x, x00.x, a0[k]);
      a0[k] = __builtin_fma(s[0][k].y, x00.y, a0[k]);
      a0[k] = __builtin_fma(s[1][k].x, x01.x, a0[k]);
      a0[k] = __builtin_fma(s[1][k].y, x01.y, a0[k]);
      if (NR == 2) {
        a1[k] = __builtin_fma(s[0][k].x, x10.x, a1[k]);
        a1[k] = __builtin_fma(s[0][k].y, x10.y, a1[k]);
        a1[k] = __builtin_fma(s[1][k].x, x11.x, a1[k]);
        a1[k] = __builtin_fma(s[1][k].y, x11.y, a1[k]);
      }
    }
  }
  if (col < ld) {  // last (possibly partial) chunk
    dbl2 s[GV_RW];
#pragma unroll
    for (int k = 0; k < GV_RW; ++k) s[k] = __builtin_nontemporal_load((const dbl2*)(Sb + k * ld + col));
    const dbl2 x0 = *(const dbl2*)(v0 + col);
    dbl2 x1 = dbl2{0.0, 0.0};
    if (NR == 2) x1 = *(const dbl2*)(v1 + col);
#pragma unroll
    for (int k = 0; k < GV_RW; ++k) {
      a0[k] = __builtin_fma(s[k].x, x0.x, a0[k]);
      a0[k] = __builtin_fma(s[k].y, x0.y, a0[k]);
      if (NR == 2) {
        a1[k] = __builtin_fma(s[k].x, x1.x, a1[k]);
        a1[k] = __builtin_fma(s[k].y, x1.y, a1[k]);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < GV_RW; ++k) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      a0[k] += xor_lane(a0[k], off);
      if (NR == 2) a1[k] += xor_lane(a1[k], off);
    }
  }
  if (lane == 0) {
    double* o0 = vp(P, V_OUT0, b);
    double* o1 = vp(P, V_OUT1, b);
#pragma unroll
    for (int k = 0; k < GV_RW; ++k) {
      const int row = row0 + k;
      if (row < P.n) {
        o0[row] = a0[k];
        if (NR == 2) o1[row] = a1[k];
      }
    }
  }
}

// list_in: which ping-pong list holds the active instances; zero_cnt: counter to clear for the
// state kernel that follows.
__global__ void __launch_bounds__(GV_THREADS) k_gemv(DevParams P, int list_in, int zero_cnt) {
  if (zero_cnt >= 0 && blockIdx.x == 0 && threadIdx.x == 0) P.cnt[zero_cnt] = 0;
  const int slot = blockIdx.x / P.nrb;
  const int nact = P.cnt[list_in];
  const int32_t e = P.lists[list_in * P.batch + slot];
  if (slot >= nact) return;
  const int b = le_b(e);
  const int rb = blockIdx.x - slot * P.nrb;
  if (le_nrhs(e) == 2) gemv_rows<2>(P, b, rb);
  else gemv_rows<1>(P, b, rb);
}

// ------------------------------------------------------------------------------------------
// Symmetric-tile S-pass.  S = Z + Z^T is stored as its upper triangle of 128 x 128 tiles; tile
// (I, J), I <= J, gives y_I += S_IJ v_J ("row part") and, off the diagonal, y_J += S_IJ^T v_I
// ("column part"), so every S byte is read once per pass for two output blocks: ~half the
// HBM traffic of the full matrix.  One 8-wave workgroup per tile; lane l owns columns 2l, 2l+1
// (16 B non-temporal loads, 1 KiB per wave instruction), each wave 16 rows in two 8-row
// batches (tools/spass_bench.hip: 8 waves 6.22 TB/s vs 4 waves 5.90, 16 waves 6.06, a pure
// non-temporal streaming read of the same bytes 6.47; plain loads 10% slower).  Row sums
// use an 8-row reduce-scatter across the wave (~3.5 lane exchanges per row); column sums
// accumulate per lane and are combined across the 4 waves through LDS.  Results go to a
// partial-sum grid P[b][I][J][0..127] (every slot written exactly once per pass) that the
// state kernel sums in fixed J order: deterministic, no atomics.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void tile_ij(int t, int nt, int& I, int& J) {
  int i = 0, rem = t, len = nt;
  while (rem >= len) { rem -= len; ++i; --len; }
  I = i;
  J = i + rem;
}

// gfx950 half exchanges on one double: swap32 trades lanes 32-63 of a with lanes 0-31 of b,
// swap16 trades the odd 16-lane rows of a with the even rows of b (v_permlane{32,16}_swap_b32).
__device__ __forceinline__ void swap32(double& a, double& b) {
  const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)__double2loint(a), (unsigned)__double2loint(b), false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(a), (unsigned)__double2hiint(b), false, false);
  a = __hiloint2double((int)hi[0], (int)lo[0]);
  b = __hiloint2double((int)hi[1], (int)lo[1]);
}
__device__ __forceinline__ void swap16(double& a, double& b) {
  const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)__double2loint(a), (unsigned)__double2loint(b), false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(a), (unsigned)__double2hiint(b), false, false);
  a = __hiloint2double((int)hi[0], (int)lo[0]);
  b = __hiloint2double((int)hi[1], (int)lo[1]);
}

// Reduce-scatter of 8 per-lane row partials over the 64 lanes: afterwards lane l holds the
// full sum of row rs_row(l) = 4 b5 + 2 b4 + b3 (b_k = bit k of l); the 8 lanes sharing bits
// 3-5 agree.  8->4 rows by swap32 and 4->2 by swap16 (no lane selects), 2->1 by a lane
// exchange with a per-lane choice of the kept half, then a butterfly over bits 0-2.
__device__ __forceinline__ double reduce_scatter8(double (&a)[8]) {
  const int lane = (int)__lane_id();
#pragma unroll
  for (int k = 0; k < 4; ++k) {  // lanes 0-31 keep rows k, lanes 32-63 rows k+4
    swap32(a[k], a[k + 4]);
    a[k] = a[k] + a[k + 4];
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {  // even 16-lane rows keep k, odd rows k+2
    swap16(a[k], a[k + 2]);
    a[k] = a[k] + a[k + 2];
  }
  const double r0 = a[0], r1 = a[1];
  const bool b3 = (lane & 8) != 0;
  const double snd = b3 ? r0 : r1, kp = b3 ? r1 : r0;
  double v = kp + xor_lane(snd, 8);
  v += xor_lane(v, 4);
  v += xor_lane(v, 2);
  v += xor_lane(v, 1);
  return v;
}

template <int NR>
__device__ __forceinline__ void spass_tile(const DevParams& P, int b, int t) {
  int I, J;
  tile_ij(t, P.nt, I, J);
  const int lane = (int)__lane_id();
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nt = P.nt, wl = P.wl;
  const int rowsT = (I == nt - 1) ? wl : TS;   // stored rows / columns of this tile
  const int colsT = (J == nt - 1) ? wl : TS;
  const bool cl = 2 * lane < colsT;            // this lane's two columns are stored
  const double* __restrict__ T = P.S + (int64_t)b * P.inst_stride + sym_off(I, J, nt, wl);
  const double* __restrict__ v0 = vp(P, V_IN0, b);
  const double* __restrict__ v1 = vp(P, V_IN1, b);
  const dbl2 vj0 = *(const dbl2*)(v0 + J * TS + 2 * lane);
  dbl2 vj1 = dbl2{0.0, 0.0};
  if (NR == 2) vj1 = *(const dbl2*)(v1 + J * TS + 2 * lane);
  const int64_t nn = (int64_t)P.nt * P.nt * TS;
  double* __restrict__ pb0 = P.pbuf + (int64_t)b * nn;
  double* __restrict__ pb1 = P.pbuf + ((int64_t)P.pbatch + b) * nn;
  double c0x = 0.0, c0y = 0.0, c1x = 0.0, c1y = 0.0;
  const int rrow = 4 * ((lane >> 5) & 1) + 2 * ((lane >> 4) & 1) + ((lane >> 3) & 1);
  constexpr int ROWS = TS / SP_WAVES;  // rows per wave
#pragma unroll 1
  for (int rb = 0; rb < ROWS / 8; ++rb) {
    const int r0 = w * ROWS + rb * 8;
    if (r0 >= rowsT) break;   // corner tile: rows beyond wl are not stored (wave-uniform)
    dbl2 sv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
      sv[k] = cl ? __builtin_nontemporal_load((const dbl2*)(T + (r0 + k) * colsT + 2 * lane)) : dbl2{0.0, 0.0};
    double a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const double vi0 = v0[I * TS + r0 + k];
      a[k] = __builtin_fma(sv[k].y, vj0.y, sv[k].x * vj0.x);
      c0x = __builtin_fma(sv[k].x, vi0, c0x);
      c0y = __builtin_fma(sv[k].y, vi0, c0y);
    }
    const double s0 = reduce_scatter8(a);
    if ((lane & 7) == 0) pb0[((int64_t)I * P.nt + J) * TS + r0 + rrow] = s0;
    if (NR == 2) {  // second right-hand side reuses the loaded tile rows
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const double vi1 = v1[I * TS + r0 + k];
        a[k] = __builtin_fma(sv[k].y, vj1.y, sv[k].x * vj1.x);
        c1x = __builtin_fma(sv[k].x, vi1, c1x);
        c1y = __builtin_fma(sv[k].y, vi1, c1y);
      }
      const double s1 = reduce_scatter8(a);
      if ((lane & 7) == 0) pb1[((int64_t)I * P.nt + J) * TS + r0 + rrow] = s1;
    }
  }
  if (I != J) {
    __shared__ double cs[2][SP_WAVES][TS];
    cs[0][w][2 * lane] = c0x;
    cs[0][w][2 * lane + 1] = c0y;
    if (NR == 2) {
      cs[1][w][2 * lane] = c1x;
      cs[1][w][2 * lane + 1] = c1y;
    }
    __syncthreads();
    if (threadIdx.x < TS) {
      const int c = threadIdx.x;
      double s0 = cs[0][0][c];
#pragma unroll
      for (int q = 1; q < SP_WAVES; ++q) s0 += cs[0][q][c];
      pb0[((int64_t)J * P.nt + I) * TS + c] = s0;
      if (NR == 2) {
        double s1 = cs[1][0][c];
#pragma unroll
        for (int q = 1; q < SP_WAVES; ++q) s1 += cs[1][q][c];
        pb1[((int64_t)J * P.nt + I) * TS + c] = s1;
      }
    }
  }
}

__global__ void __launch_bounds__(SP_THREADS, 4) k_spass_sym(DevParams P, int list_in, int zero_cnt) {
  if (zero_cnt >= 0 && blockIdx.x == 0 && threadIdx.x == 0) P.cnt[zero_cnt] = 0;
  const int slot = blockIdx.x / P.ntiles;
  const int nact = P.cnt[list_in];
  const int32_t e = P.lists[list_in * P.batch + slot];
  if (slot >= nact) return;
  const int b = le_b(e);
  const int t = blockIdx.x - slot * P.ntiles;
  if (le_nrhs(e) == 2) spass_tile<2>(P, b, t);
  else spass_tile<1>(P, b, t);
}

// ------------------------------------------------------------------------------------------
// Persistent super-tile S-pass (P.smode = 1; launches with >= 1 unit per CU).  Same arithmetic
// per stored tile as spass_tile, but one 8-wave workgroup per CU walks units u = g, g + G, ... of
// SB x SB stored tiles: row sums accumulate over a unit's tile columns, column sums over its
// tile rows (8 waves, then LDS across waves in wave order), and each unit's two SW-element
// partial vectors are kept in LDS and written in bursts of up to SUP_OCAP doubles.  Why: the
// partial-sum writes of the per-tile kernel, 1.5% of the bytes, cost 13% of its streaming rate
// when they trickle out between the reads (tools/spass_glds_bench.hip: 6.15 TB/s with the writes,
// 7.15 without, 6.79-6.82 for this kernel on the same box).  Partial grid [b][P][Q][SW]: slot
// (P, Q) holds unit (P, Q)'s row part (P <= Q; the whole symmetric block on the diagonal) and
// slot (Q, P) its column part; every slot is written by exactly one unit: deterministic.
// ------------------------------------------------------------------------------------------
constexpr int SUP_OCAP = 15360;                 // doubles of buffered unit results (120 KiB)
constexpr int SUP_MAXU = SUP_OCAP / (2 * SW);   // units per burst at one right-hand side

typedef double (*sup_red_t)[SP_WAVES][SW];

template <int NR>
// One right-hand side: the wave's 16 row entries of v for tile row I are loaded once per tile row
// and reused across the unit's tile columns (same-box A/B: 80.6 vs 80.0 outer it/s, 194 VGPRs, no
// scratch either way; with two right-hand sides the second set would not fit in registers).
// red: column-sum scratch; one right-hand side uses red[rsel] (alternating between units, so a
// unit's cross-wave column reduction needs no trailing barrier: the next unit zeroes the other
// buffer), two use red[0] and red[1] between a leading and a trailing barrier
__device__ __forceinline__ void sup_unit(const DevParams& P, int b, int Pq, int Qq, sup_red_t red, double* out, int rsel) {
  const int lane = (int)__lane_id();
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nt = P.nt, wl = P.wl;
  constexpr int ROWS = TS / SP_WAVES;
  const double* __restrict__ Sb = P.S + (int64_t)b * P.inst_stride;
  const double* __restrict__ v0 = vp(P, V_IN0, b);
  const double* __restrict__ v1 = vp(P, V_IN1, b);
  const int rrow = 4 * ((lane >> 5) & 1) + 2 * ((lane >> 4) & 1) + ((lane >> 3) & 1);
  double racc[NR][SB][2];
#pragma unroll
  for (int k = 0; k < NR; ++k)
#pragma unroll
    for (int i = 0; i < SB; ++i) racc[k][i][0] = racc[k][i][1] = 0.0;
  if (NR == 2) __syncthreads();   // the previous unit's reduction may still read either buffer
  const int r0sel = NR == 2 ? 0 : rsel;
#pragma unroll
  for (int k = 0; k < NR; ++k)
    for (int jl = 0; jl < SB; ++jl) {
      red[r0sel + k][w][jl * TS + 2 * lane] = 0.0;
      red[r0sel + k][w][jl * TS + 2 * lane + 1] = 0.0;
    }
#pragma unroll
  for (int il = 0; il < SB; ++il) {
    const int I = SB * Pq + il;
    if (I >= nt) break;
    const int rowsT = (I == nt - 1) ? wl : TS;
    constexpr bool hoist = NR == 1;
    double vih[ROWS];
    if (hoist) {
#pragma unroll
      for (int k = 0; k < ROWS; ++k) vih[k] = v0[I * TS + w * ROWS + k];
    }
#pragma unroll 1
    for (int jl = 0; jl < SB; ++jl) {
      const int J = SB * Qq + jl;
      if (J >= nt || J < I) continue;
      const int colsT = (J == nt - 1) ? wl : TS;
      const bool cl = 2 * lane < colsT;
      const double* __restrict__ T = Sb + sym_off(I, J, nt, wl);
      // vector entries first, then the wave's 16 S rows (both 8-row batches) with no branches
      // (clamped addresses + selects), so the compiler can wait for batch 0 while batch 1 is
      // still in flight (one workgroup per CU has no sibling workgroups to cover its latency)
      const dbl2 vj0 = *(const dbl2*)(v0 + J * TS + 2 * lane);
      dbl2 vj1 = dbl2{0.0, 0.0};
      if (NR == 2) vj1 = *(const dbl2*)(v1 + J * TS + 2 * lane);
      double vi0[ROWS], vi1[ROWS];
#pragma unroll
      for (int k = 0; k < ROWS; ++k) {
        vi0[k] = hoist ? vih[k] : v0[I * TS + w * ROWS + k];
        vi1[k] = NR == 2 ? v1[I * TS + w * ROWS + k] : 0.0;
      }
      __builtin_amdgcn_sched_barrier(0);   // keep the vector loads ahead of the S rows
      double c0x = 0.0, c0y = 0.0, c1x = 0.0, c1y = 0.0;
      dbl2 sv2[ROWS / 8][8];
#pragma unroll
      for (int rb = 0; rb < ROWS / 8; ++rb)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int row = w * ROWS + rb * 8 + k;
          const bool ok = cl && row < rowsT;   // corner / narrow tiles: not stored
          const dbl2 x = __builtin_nontemporal_load((const dbl2*)(T + (row < rowsT ? row : 0) * colsT + (cl ? 2 * lane : 0)));
          sv2[rb][k] = ok ? x : dbl2{0.0, 0.0};
        }
#pragma unroll
      for (int rb = 0; rb < ROWS / 8; ++rb) {
        const int r0 = w * ROWS + rb * 8;
        if (r0 >= rowsT) break;   // wave-uniform
        const dbl2 (&sv)[8] = sv2[rb];
        double a[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const double vi = vi0[rb * 8 + k];
          a[k] = __builtin_fma(sv[k].y, vj0.y, sv[k].x * vj0.x);
          c0x = __builtin_fma(sv[k].x, vi, c0x);
          c0y = __builtin_fma(sv[k].y, vi, c0y);
        }
        racc[0][il][rb] += reduce_scatter8(a);
        if (NR == 2) {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const double vi = vi1[rb * 8 + k];
            a[k] = __builtin_fma(sv[k].y, vj1.y, sv[k].x * vj1.x);
            c1x = __builtin_fma(sv[k].x, vi, c1x);
            c1y = __builtin_fma(sv[k].y, vi, c1y);
          }
          racc[NR - 1][il][rb] += reduce_scatter8(a);
        }
      }
      if (I != J) {   // column part (the diagonal tile is stored whole: row part only)
        red[r0sel][w][jl * TS + 2 * lane] += c0x;
        red[r0sel][w][jl * TS + 2 * lane + 1] += c0y;
        if (NR == 2) {
          red[NR - 1][w][jl * TS + 2 * lane] += c1x;
          red[NR - 1][w][jl * TS + 2 * lane + 1] += c1y;
        }
      }
    }
  }
  // unit result out[k][0] = rows of super-block Pq, out[k][1] = columns of super-block Qq
  if ((lane & 7) == 0) {
#pragma unroll
    for (int k = 0; k < NR; ++k)
#pragma unroll
      for (int il = 0; il < SB; ++il) {
        out[(2 * k) * SW + il * TS + w * ROWS + rrow] = racc[k][il][0];
        out[(2 * k) * SW + il * TS + w * ROWS + 8 + rrow] = racc[k][il][1];
      }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < NR * SW; t += SP_THREADS) {
    const int k = t / SW, c = t - k * SW;
    double cs = red[r0sel + k][0][c];
#pragma unroll
    for (int q = 1; q < SP_WAVES; ++q) cs += red[r0sel + k][q][c];
    if (Pq == Qq) out[(2 * k) * SW + c] += cs;   // diagonal unit: both parts land in block Pq
    else out[(2 * k + 1) * SW + c] = cs;
  }
  if (NR == 2) __syncthreads();
}

__device__ __forceinline__ void sup_flush(const DevParams& P, const double* outb, const int (*meta)[2], int nslot,
                                          int list_in) {
  __syncthreads();
  const int64_t nn = (int64_t)P.nst * P.nst * SW;
  int off = 0;
  for (int s = 0; s < nslot; ++s) {
    const int u = meta[s][0], nr = meta[s][1];
    const int slot = u / P.nsup;
    const int b = le_b(P.lists[list_in * P.batch + slot]);
    int Pq, Qq;
    tile_ij(u - slot * P.nsup, P.nst, Pq, Qq);
    const int t = threadIdx.x, side = t / SW, c = t - side * SW;   // 512 threads: row side, column side
    for (int k = 0; k < nr; ++k) {
      double* pb = P.pbuf + ((int64_t)k * P.pbatch + b) * nn;
      if (side == 0) pb[((int64_t)Pq * P.nst + Qq) * SW + c] = outb[off + (2 * k) * SW + c];
      else if (Pq != Qq) pb[((int64_t)Qq * P.nst + Pq) * SW + c] = outb[off + (2 * k + 1) * SW + c];
    }
    off += nr * 2 * SW;
  }
  __syncthreads();
}

// Unit order: static (u = g, g + G, ...) or, with P.sup_dyn, tickets from a per-list counter
// (cnt[8 + list_in]): a workgroup takes its next unit when it finishes one, so CUs that also run
// the other group's state kernel, and units of 3 vs 4 tiles or two right-hand sides, no longer
// decide the launch's end.  The next ticket is fetched at the start of the current unit (its
// latency overlaps the unit's first loads); the last workgroup to finish resets the counter for
// the next launch.  Every unit writes its fixed slots, so results do not depend on the order.
__global__ void __launch_bounds__(SP_THREADS, 1) k_spass_sup(DevParams P, int list_in, int zero_cnt) {
  static_assert(SP_THREADS == 2 * SW, "sup_flush: one thread per element of the two sides");
  __shared__ double red[2][SP_WAVES][SW];
  __shared__ double outb[SUP_OCAP];
  __shared__ int meta[SUP_MAXU][2];
  __shared__ int tick_next;
  if (zero_cnt >= 0 && blockIdx.x == 0 && threadIdx.x == 0) P.cnt[zero_cnt] = 0;
  const int nact = P.cnt[list_in];
  const int total = nact * P.nsup;
  int used = 0, nslot = 0, rsel = 0;
  const bool dyn = P.sup_dyn != 0;
  unsigned int* tick = (unsigned int*)P.cnt + 8 + list_in;
  unsigned int* done = (unsigned int*)P.cnt + 12 + list_in;
  int u = blockIdx.x;
  if (dyn) {
    if (threadIdx.x == 0) tick_next = (int)atomicAdd(tick, 1u);
    __syncthreads();
    u = tick_next;
  }
  while (u < total) {
    unsigned int pre = 0;
    if (dyn && threadIdx.x == 0) pre = atomicAdd(tick, 1u);   // next unit, in flight during this one
    const int slot = u / P.nsup;
    const int32_t e = P.lists[list_in * P.batch + slot];
    const int b = le_b(e), nr = le_nrhs(e);
    int Pq, Qq;
    tile_ij(u - slot * P.nsup, P.nst, Pq, Qq);
    if (used + nr * 2 * SW > SUP_OCAP) {
      sup_flush(P, outb, meta, nslot, list_in);
      used = 0;
      nslot = 0;
    }
    if (nr == 2) {
      sup_unit<2>(P, b, Pq, Qq, red, outb + used, 0);
    } else {
      sup_unit<1>(P, b, Pq, Qq, red, outb + used, rsel);
      rsel ^= 1;
    }
    if (threadIdx.x == 0) {
      meta[nslot][0] = u;
      meta[nslot][1] = nr;
    }
    used += nr * 2 * SW;
    ++nslot;
    if (dyn) {
      __syncthreads();                 // every thread has read tick_next (and meta is ordered)
      if (threadIdx.x == 0) tick_next = (int)pre;
      __syncthreads();
      u = tick_next;
    } else {
      u += gridDim.x;
    }
  }
  if (nslot > 0) sup_flush(P, outb, meta, nslot, list_in);
  if (dyn && threadIdx.x == 0) {
    // every workgroup has drawn its last ticket before it counts itself done: the last one resets
    if (atomicAdd(done, 1u) == gridDim.x - 1) {
      atomicExch(tick, 0u);
      atomicExch(done, 0u);
    }
  }
}

// ------------------------------------------------------------------------------------------
// Shared-S (multi-start) S-pass on the fp64 matrix cores: every active instance multiplies the
// SAME S, so one pass is the dense product Y^T = V^T S over the active right-hand sides
// (column c = active slot for in0, bound + slot for in1 when the instance asked for two).
// v_mfma_f64_16x16x4_f64: A = 16 right-hand sides x 4 k, B = 4 k x 16 rows of S (S is
// symmetric, so row i of S is column i of S^T), D = 16 x 16 fp64 accumulators.
//
// A workgroup (MM_WAVES = 16 waves, four per SIMD) owns CT = 16 WM right-hand sides x RT rows of S over one
// of MM_KZ K slices.  Each 32-deep K step stages V[CT][32] and S[RT][32] into LDS with
// global_load_lds_dwordx4 (256-B rows; 16-B chunk c of row r kept at chunk c ^ (r & 15), written
// through the SOURCE address since the LDS side of the copy is lane-linear, so the fragment reads
// below are bank-conflict free), in a ring of NST = 3 stages where it fits LDS (else 2): step
// t + NST - 1's copy is in flight while the waves run step t's MFMAs out of LDS, one barrier per
// step.  The waves form a rows x columns grid over the tile (8 x 2 for 128-row tiles; 4 x 4 for
// 64-row tiles, the shape at n = 4000 where 4 K slices x 63 row blocks fill the chip) and read, for MFMA pair jj,
// lane (r, q)'s 16 B at k = 8q + 2jj: MFMA m = 2 jj + {0,1} sums k in {m, 8+m, 16+m, 24+m} — the
// same order for every kernel shape, so an instance's product does not depend on CT / RT or on
// the other right-hand sides.  The next pair's fragments are read while the current pair's
// MFMAs issue, and the SIMD's other waves cover one wave's LDS reads and barrier wait.  Partial
// slabs of the MM_KZ slices are added in slice order by the state kernel (deterministic, no
// atomics).  Linear block id -> slice = id % MM_KZ, so a slice (and the V columns it reads)
// stays on one XCD.  4 slices rather than 8: the state kernel adds half the slabs (k_state 37.9 ->
// 29.8 us per launch in the n = 4000 multi-start solve) at an equal S-pass time (82 us).
// tools/mfma_bench.hip at n = 4000, 128 right-hand sides: 72.5 us = 56.5 TFLOP/s with 128-row
// tiles and 8 slices (4 waves: 81.5 us; the register-fed tile this replaced: 115 us; issue-rate
// probe 70.8).
// ------------------------------------------------------------------------------------------
typedef double dbl4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) unsigned char lds_u8;
#ifndef RIPTRM_MM_WAVES
#define RIPTRM_MM_WAVES 16   // A/B builds: -DRIPTRM_MM_WAVES=8 (the round-2 workgroup)
#endif
// tools/mfma_bench.hip at n = 4000, 128 right-hand sides (profiles/r3_mfma_tile_sweep.jsonl):
// 64-row tiles 4 waves 81.5 us, 8 waves (4 x 2 grid) 75.4 us, 16 waves (4 x 4) 70.8 us
constexpr int MM_WAVES = RIPTRM_MM_WAVES;
typedef __attribute__((address_space(3))) dbl2 lds_dbl2;
#ifndef RIPTRM_MM_NST
#define RIPTRM_MM_NST 3   // A/B builds: -DRIPTRM_MM_NST=2 (the round-2 double buffer)
#endif

// Wait until at most N of this wave's LDS copies are in flight, then a bare workgroup barrier.
// __syncthreads() would add a release fence, which waits for every copy (vmcnt(0)) and so would
// serialise the copy of the step after next with this one.  The "memory" clobber keeps the
// compiler from moving LDS reads across.
template <int N>
__device__ __forceinline__ void mm_wait_barrier() {
#define MM_WB_CASE(K) else if constexpr (N == K) asm volatile("s_waitcnt vmcnt(" #K ")\n\ts_barrier" ::: "memory");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  MM_WB_CASE(1) MM_WB_CASE(2) MM_WB_CASE(3) MM_WB_CASE(4) MM_WB_CASE(5) MM_WB_CASE(6) MM_WB_CASE(7)
  MM_WB_CASE(8) MM_WB_CASE(9) MM_WB_CASE(10) MM_WB_CASE(11) MM_WB_CASE(12)
#undef MM_WB_CASE
  else static_assert(N < 0, "mm_wait_barrier: add the count");
}

template <int WM, int RT>
struct MmShape {
  static constexpr int NW = MM_WAVES;                  // waves per workgroup (NW / 4 per SIMD)
  static constexpr int CT = 16 * WM;                   // right-hand sides per workgroup
  // wave grid: rows x columns; waves past NWR x NWC (narrow in1 tiles) only copy
  static constexpr int NWR = NW < RT / 16 ? NW : RT / 16;
  static constexpr int NWC = NW / NWR < WM ? NW / NWR : WM, NACT = NWR * NWC;
  static constexpr int WMW = WM / NWC;                 // 16-column accumulator rows per wave
  static constexpr int RW = RT / NWR, WN = RW / 16;    // rows per wave, 16-row accumulator columns
  static constexpr int VT = CT * 256;                  // V tile bytes per stage
  static constexpr int STAGE = VT + RT * 256;          // + S tile
  // glds wave-instructions (4 rows of 256 B each) per stage: waves < VW copy VP of V's, < SW SP of S's
  static constexpr int VW = NW < CT / 4 ? NW : CT / 4, VP = CT / 4 / VW;
  static constexpr int SW = NW < RT / 4 ? NW : RT / 4, SP = RT / 4 / SW;
  // LDS stages: three where they fit next to the in1 map (64-row tiles: 3 x 48 KiB), else two
  static constexpr int NST = RIPTRM_MM_NST >= 3 && 3 * STAGE + 32 * 4 <= 160 * 1024 ? 3 : 2;
  static_assert(WMW >= 1 && WN >= 1 && WM % NWC == 0 && VP * VW * 4 == CT && SP * SW * 4 == RT, "tile shape");
};

// One tile: right-hand-side columns v = 0..CT-1 of the tile are instance slots slot_of(v) (valid
// while v < nv), reading V kind vk and writing slab (z, which).  slot_of(v) = s0 + v for in0
// tiles, the v-th entry of an LDS map for compacted in1 tiles.
template <int WM, int RT, typename SlotOf>
__device__ __forceinline__ void mm_tile(const DevParams& P, lds_u8* smem, const int32_t* lst, int vk, int which, int nv,
                                        SlotOf slot_of, int z, int i0, int rows) {
  using Sh = MmShape<WM, RT>;
  constexpr int CT = Sh::CT, WN = Sh::WN, WMW = Sh::WMW, RW = Sh::RW, NWR = Sh::NWR;
  constexpr int VT = Sh::VT, STAGE = Sh::STAGE, VP = Sh::VP, SP = Sh::SP, NST = Sh::NST;
  constexpr int VW = Sh::VW, SW = Sh::SW, NACT = Sh::NACT;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  const int wr = w % NWR, wc = w / NWR;  // this wave's rows RW wr .. and columns 16 WMW wc ..
  const int r = lane & 15, q = lane >> 4;
  const int64_t ld = P.ld;
  const double* vsrc[VP];
  const double* ssrc[SP];
#pragma unroll
  for (int p = 0; p < VP; ++p) {
    const int row = 4 * (VP * w + p) + q;
    vsrc[p] = vp(P, vk, le_b(lst[slot_of(min(row, nv - 1))])) + 2 * (r ^ (row & 15));   // row < CT when w < VW
  }
#pragma unroll
  for (int p = 0; p < SP; ++p) {
    const int row = 4 * (SP * w + p) + q;
    const int i = min(i0 + row, rows - 1);
    ssrc[p] = P.S + (int64_t)i * ld + 2 * (r ^ (row & 15));
  }
  const int nch = (int)(ld / 32), per = (nch + MM_KZ - 1) / MM_KZ;
  const int lo = z * per, hi = min(nch, lo + per);
  auto issue = [&](int ch, int buf) {
    const int64_t k0 = (int64_t)ch * 32;
    lds_u8* vb = smem + buf * STAGE;
#pragma unroll
    for (int p = 0; p < VP; ++p)
      if (VW == Sh::NW || w < VW)   // wave-uniform
        __builtin_amdgcn_global_load_lds((const void*)(vsrc[p] + k0), vb + 4 * (VP * w + p) * 256, 16, 0, 0);
#pragma unroll
    for (int p = 0; p < SP; ++p)
      if (SW == Sh::NW || w < SW)
        __builtin_amdgcn_global_load_lds((const void*)(ssrc[p] + k0), vb + VT + 4 * (SP * w + p) * 256, 16, 0, 0);
  };
  dbl4 acc[WMW][WN];
#pragma unroll
  for (int a = 0; a < WMW; ++a)
#pragma unroll
    for (int c = 0; c < WN; ++c) acc[a][c] = dbl4{0.0, 0.0, 0.0, 0.0};
  // wave-uniform: rows of the tile past n, and column groups past the tile's last column, idle
  const bool live = w < NACT && i0 + RW * wr < P.n && 16 * WMW * wc < nv;
  // NST-stage ring: step ch + NST - 1's copy is issued right after the barrier of step ch (the
  // buffer step ch - 1 read), so a copy has NST - 1 steps of MFMA work to land
  if (lo < hi) issue(lo, 0);
  if (NST == 3 && lo + 1 < hi) issue(lo + 1, 1);
  int s = 0;
  for (int ch = lo; ch < hi; ++ch) {
    // this wave's copies of step ch landed (the NST - 2 later steps' may still fly); after the
    // barrier everyone's have, and step ch - 1's LDS reads are done
    if (NST == 3 && ch + 1 < hi) {
      // copies this wave issues per stage (wave-uniform branches, one barrier each)
      if (w < VW && w < SW) mm_wait_barrier<VP + SP>();
      else if (w < VW) mm_wait_barrier<VP>();
      else if (w < SW) mm_wait_barrier<SP>();
      else mm_wait_barrier<0>();
    } else {
      mm_wait_barrier<0>();
    }
    if (ch + NST - 1 < hi) issue(ch + NST - 1, s == 0 ? NST - 1 : s - 1);
    const int sc = s;
    s = s + 1 == NST ? 0 : s + 1;
    if (!live) continue;
    const lds_u8* vb = smem + sc * STAGE + 16 * WMW * wc * 256;
    const lds_u8* sb = smem + sc * STAGE + VT + RW * wr * 256;
    dbl2 fa[2][WMW], fb[2][WN];
    auto frag = [&](int jj, int u) {
      const int off = ((4 * q + jj) ^ r) * 16;
#pragma unroll
      for (int a = 0; a < WMW; ++a) fa[u][a] = *(const lds_dbl2*)(vb + (16 * a + r) * 256 + off);
#pragma unroll
      for (int c = 0; c < WN; ++c) fb[u][c] = *(const lds_dbl2*)(sb + (16 * c + r) * 256 + off);
    };
    frag(0, 0);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int u = jj & 1;
      if (jj < 3) frag(jj + 1, u ^ 1);
#pragma unroll
      for (int mm = 0; mm < 2; ++mm)
#pragma unroll
        for (int a = 0; a < WMW; ++a)
#pragma unroll
          for (int c = 0; c < WN; ++c)
            acc[a][c] = __builtin_amdgcn_mfma_f64_16x16x4f64(mm ? fa[u][a].y : fa[u][a].x, mm ? fb[u][c].y : fb[u][c].x,
                                                             acc[a][c], 0, 0, 0);
    }
  }
  (void)CT;
  if (!live) return;
  // D (f64): column = lane & 15 -> row i of S, row = (lane >> 4) + 4 g -> right-hand side
  double* slab = P.pbuf + ((int64_t)z * 2 + which) * P.batch * ld;
#pragma unroll
  for (int a = 0; a < WMW; ++a)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int v = 16 * (WMW * wc + a) + q + 4 * g;
      if (v >= nv) continue;
      double* o = slab + (int64_t)le_b(lst[slot_of(v)]) * ld;
#pragma unroll
      for (int c = 0; c < WN; ++c) {
        const int i = i0 + RW * wr + 16 * c + r;
        if (i < P.n) o[i] = acc[a][c][g];
      }
    }
}

// dynamic LDS: the stages of the in0 tile shape + the in1 column map (in1 tiles' stages are smaller)
template <int WM0, int RT>
constexpr int mm_shm() { return MmShape<WM0, RT>::NST * MmShape<WM0, RT>::STAGE + 32 * 4; }

// Grid (1-D): MM_KZ slices x row blocks x t0 in0 tiles of 16 WM0 columns.  The second right-hand
// side exists only for the instances that asked for two (le_nrhs): their in1 columns are
// compacted in list order into 32-wide tiles, run by the same workgroups after their in0 tile, so
// a pass where a few instances need two products costs a narrow tile, not a second full-width one.
template <int WM0, int RT>
__global__ void __launch_bounds__(64 * MM_WAVES) k_spass_mm(DevParams P, int list_in, int zero_cnt, int bound) {
  extern __shared__ __attribute__((aligned(16))) unsigned char mm_smem_raw[];
  lds_u8* smem = (lds_u8*)mm_smem_raw;
  if (zero_cnt >= 0 && blockIdx.x == 0 && threadIdx.x == 0) P.cnt[zero_cnt] = 0;
  const int nact = P.cnt[list_in];
  const int rows = (P.n + 31) / 32 * 32;  // rows_of(n)
  const int nrb = (rows + RT - 1) / RT, t0 = (bound + 16 * WM0 - 1) / (16 * WM0);
  const int L = blockIdx.x, z = L % MM_KZ, rest = L / MM_KZ;
  const int i0 = (rest % nrb) * RT, y = rest / nrb;
  const int32_t* lst = P.lists + (int64_t)list_in * P.batch;
  const int s0 = y * 16 * WM0;
  if (s0 < nact)
    mm_tile<WM0, RT>(P, smem, lst, V_IN0, 0, min(16 * WM0, nact - s0), [&](int v) { return s0 + v; }, z, i0, rows);
  // in1 tiles j = y, y + t0, ... of this row block and slice, after the in0 one: their 32 columns
  // are the instances asking for a second product, in list order.  Run by the in0 workgroups
  // rather than as workgroups of their own: in most passes no instance asks, and a grid of idle
  // in1 workgroups, each holding the in0 tile's LDS, dispatched behind the in0 tiles costs
  // ~8 us per launch at n = 4000 (profiles/r3_shared_16w_ab.jsonl vs r3_shared_in1_inline_ab.jsonl).
  const int t1 = (bound + 31) / 32;
  if (y >= t1) return;
  int32_t* map = (int32_t*)(mm_smem_raw + MmShape<WM0, RT>::NST * MmShape<WM0, RT>::STAGE);
  const int lane = threadIdx.x & 63;
  int n2 = 0;   // instances asking for two products (the same in every wave)
  for (int c = 0; c < nact; c += 64) {
    const bool two = c + lane < nact && le_nrhs(lst[c + lane]) == 2;
    n2 += __popcll(__ballot(two));
  }
  for (int j = y; j < t1 && 32 * j < n2; j += t0) {
    const int u0 = 32 * j;
    __syncthreads();   // the previous tile's LDS reads (and map reads) are done
    int k0 = 0;
    for (int c = 0; c < nact; c += 64) {
      const int sl = c + lane;
      const bool two = sl < nact && le_nrhs(lst[sl]) == 2;
      const uint64_t m = __ballot(two);
      const int k = k0 + __popcll(m & ((1ull << lane) - 1));
      if (two && threadIdx.x < 64 && k >= u0 && k < u0 + 32) map[k - u0] = sl;
      k0 += __popcll(m);
    }
    __syncthreads();
    mm_tile<2, RT>(P, smem, lst, V_IN1, 1, min(32, n2 - u0), [&](int v) { return (int)map[v]; }, z, i0, rows);
  }
}

// ------------------------------------------------------------------------------------------
// Packing: S = Z + Z^T from a row-major Z (leading dimension ldz) into either layout, zero
// padded.  32x32 sub-tiles staged through LDS so both Z and Z^T are read coalesced; each
// element is the single rounding of Z_ij + Z_ji (so S_ij == S_ji bit for bit).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void pack_sub32(const double* __restrict__ Zb, int64_t ldz, int n, int i0, int j0,
                                           double* __restrict__ dst, int64_t dst_ld) {
  __shared__ double a[32][33], bt[32][33];
  const int c = threadIdx.x & 31, r8 = threadIdx.x >> 5;  // 256 threads: 32 x 8
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int r = r8 + 8 * k;
    const int i = i0 + r, j = j0 + c;
    a[r][c] = (i < n && j < n) ? Zb[(int64_t)i * ldz + j] : 0.0;
    const int i2 = j0 + r, j2 = i0 + c;               // Z block (J, I)
    bt[r][c] = (i2 < n && j2 < n) ? Zb[(int64_t)i2 * ldz + j2] : 0.0;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int r = r8 + 8 * k;
    const int i = i0 + r, j = j0 + c;
    dst[(int64_t)r * dst_ld + c] = (i < n && j < n) ? a[r][c] + bt[c][r] : 0.0;
  }
  __syncthreads();
}

// grid.x = sub-tiles of the padded square, grid.y = instance
__global__ void __launch_bounds__(256) k_pack(const double* Z, int64_t ldz, int64_t zs, int n, double* S,
                                              int64_t ss, int layout, int64_t ld, int64_t rows) {
  const double* Zb = Z + (int64_t)blockIdx.y * zs;
  double* Sb = S + (int64_t)blockIdx.y * ss;
  const int nsub = (int)(ld / 32);
  const int si = blockIdx.x / nsub, sj = blockIdx.x % nsub;
  const int i0 = si * 32, j0 = sj * 32;
  if (layout != RIPTRM_LAYOUT_SYMTILE) {  // full / shared: row-major
    if (i0 >= rows) return;
    pack_sub32(Zb, ldz, n, i0, j0, Sb + (int64_t)i0 * ld + j0, ld);
  } else {
    const int I = i0 / TS, J = j0 / TS;
    if (I > J) return;
    const int nt = (int)(ld / TS);
    const int wl = (int)(((int64_t)n - (int64_t)(nt - 1) * TS + 31) / 32 * 32);
    const int rowsT = (I == nt - 1) ? wl : TS, colsT = (J == nt - 1) ? wl : TS;
    if (i0 - I * TS >= rowsT || j0 - J * TS >= colsT) return;   // outside the stored part
    pack_sub32(Zb, ldz, n, i0, j0, Sb + sym_off(I, J, nt, wl) + (int64_t)(i0 - I * TS) * colsT + (j0 - J * TS),
               colsT);
  }
}

// ------------------------------------------------------------------------------------------
// The per-instance state machine.
// ------------------------------------------------------------------------------------------
// ACT_CONTINUE: the next phase needs no S-pass; k_state<true> dispatches it in a loop (a direct
// call would recurse through the inner loop whenever trial points are infeasible)
enum Act : int { ACT_YIELD = 0, ACT_DONE = 1, ACT_PAUSE = 2, ACT_CONTINUE = 3 };

// ---- register-path operand loads (free functions: k_state prefetches them before the machine's
// scalars arrive) --------------------------------------------------------------------------------
template <int K>
__device__ __forceinline__ void rl_load(const double* a, int n, double (&r)[K]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int i = tid + k * ST_THREADS;
    r[k] = i < n ? a[i] : 0.0;
  }
}
template <int K>
__device__ __forceinline__ void rl_store(double* a, int n, const double (&r)[K]) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int i = tid + k * ST_THREADS;
    if (i < n) a[i] = r[k];
  }
}
// Partial-grid words handed between workgroups INSIDE a launch (k_persist): written by `sc1`
// (write-through) stores and read by `sc1` loads, which bypass the reading CU's L1, after the
// arrival counter says every producer has drained its stores (MI355X_MICROARCH.md, visibility:
// the counter form with sc1 payload stores and loads).  Agent-scope relaxed atomics on global
// pointers lower to exactly those instructions.
typedef __attribute__((address_space(1))) unsigned long long gu64_t;
typedef __attribute__((address_space(1))) unsigned int gu32_t;
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store((gu64_t*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __longlong_as_double((long long)__hip_atomic_load((gu64_t*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
template <bool SC1>
__device__ __forceinline__ double ldp(const double* p) {
  if constexpr (SC1) return ld_sc1(p);
  else return *p;
}

// S delta of the last S-pass into registers (the layouts' partial sums, in gather_out's order).
// K <= 2 (n <= 1024, nt <= 8): every partial of the element issued at once — one memory round
// trip instead of one per tile column (the partials come from S-pass workgroups on every XCD,
// so they are L2 misses).  pbuf / bp: the partial grid and the instance's slot in it (the
// persistent replicas read their instance's grid; SC1 = the in-launch hand-off loads).
template <int K, bool SC1 = false>
__device__ __forceinline__ void rl_gather(const DevParams& P, const double* pbuf, int bp, double (&u)[K]) {
  const int tid = threadIdx.x, n = P.n;
  if (P.layout == RIPTRM_LAYOUT_SYMTILE) {
    // tile grid [nt][nt][TS] or super-tile grid [nst][nst][SW] (P.smode), summed in block order
    const int nt = P.smode ? P.nst : P.nt;
    const int sh = P.smode ? 8 : 7, wd = 1 << sh;
    static_assert(SW == 256 && TS == 128, "partial-grid shifts");
    const int64_t nn = (int64_t)nt * nt * wd;
    const double* pb = pbuf + (int64_t)bp * nn;
    const double* q[K];
#pragma unroll
    for (int e = 0; e < K; ++e) {
      int i = tid + e * ST_THREADS;
      i = i < n ? i : n - 1;
      const int I = i >> sh, c = i - (I << sh);
      q[e] = pb + (int64_t)I * nt * wd + c;
    }
    if constexpr (K <= 2) {
      constexpr int NTS = 8;
      double t[K][NTS];
#pragma unroll
      for (int e = 0; e < K; ++e)
#pragma unroll
        for (int J = 0; J < NTS; ++J) t[e][J] = (J < nt) ? ldp<SC1>(q[e] + (int64_t)J * wd) : 0.0;
#pragma unroll
      for (int e = 0; e < K; ++e) {
        u[e] = t[e][0];
#pragma unroll
        for (int J = 1; J < NTS; ++J)
          if (J < nt) u[e] += t[e][J];
      }
    } else {
#pragma unroll
      for (int e = 0; e < K; ++e) u[e] = ldp<SC1>(q[e]);
      constexpr int GJ = 2;
      for (int J = 1; J < nt; J += GJ) {
        double t[K][GJ];
#pragma unroll
        for (int e = 0; e < K; ++e)
#pragma unroll
          for (int v = 0; v < GJ; ++v) t[e][v] = (J + v < nt) ? ldp<SC1>(q[e] + (int64_t)(J + v) * wd) : 0.0;
#pragma unroll
        for (int e = 0; e < K; ++e)
#pragma unroll
          for (int v = 0; v < GJ; ++v)
            if (J + v < nt) u[e] += t[e][v];
      }
    }
#pragma unroll
    for (int e = 0; e < K; ++e)
      if (tid + e * ST_THREADS >= n) u[e] = 0.0;
  } else if (P.layout == RIPTRM_LAYOUT_SHARED) {
    const int64_t ld = P.ld, slab = (int64_t)P.batch * ld;
    const double* pb = pbuf + (int64_t)bp * ld;
#pragma unroll
    for (int e = 0; e < K; ++e) {
      const int i = tid + e * ST_THREADS;
      double acc = 0.0;
      if (i < n) {
        acc = pb[i];
#pragma unroll
        for (int z = 1; z < MM_KZ; ++z) acc += pb[(int64_t)z * 2 * slab + i];
      }
      u[e] = acc;
    }
  } else {
    rl_load<K>(vp(P, V_OUT0, bp), P.n, u);
  }
}


// The persistent replicas' slots (k_persist): vectors (NVEC x batch x ld), scalars, stats and
// request words of batch x (reps - 1) replicas, laid out like the instances' own.
struct RepBlock {
  double* vec;
  double* st;
  double* stats;
  int32_t* req;
  int32_t batch;
};

// ---- one tCG iteration (RIPTRM.py:100-214) on register-resident vectors ------------------------
// u = S delta on entry (the S-pass); d, x, y, c, e, he, rv = delta, x, y, cxCur, eta, Heta, r for
// this thread's elements i = tid + k ST_THREADS.  Updates the vectors and the scalars and returns
// TCG_CONTINUE (d is the next direction, j advanced) or the stop code (eta / Heta final, j as the
// reference leaves it).  The hooks load late operands / store results for the workspace-backed
// caller (k_state); the persistent fast path passes no-ops and keeps everything in registers.  One
// body for both, so the two paths are bitwise identical.
struct TcgScalars {
  double coef, z_r, e_Pd, d_Pd, e_Pe, Delta, model, nr0, j;
  double nr0t;   // pow(nr0, tCG_theta): constant over a tCG run (RIPTRM.py:180-182), computed once
};
constexpr int TCG_CONTINUE = -1;

// The part of the barrier-Hessian action that does not need u = S delta: xv = <x, delta>,
// q = y (delta - x xv) / x and xq = <x, q> (the lean path computes it while the S-pass's partial
// sums are in flight).  Each reduction is its own slot of the same tree as before, so the values
// are those of the fused form.
template <int K>
struct HwPre {
  double xv, xq;
  double q[K];
};
template <int K>
__device__ __forceinline__ void tcg_math_pre(HwPre<K>& p, int n, Red& R, const double (&d)[K], const double (&x)[K],
                                             const double (&y)[K]) {
  const int tid = threadIdx.x;
  double r1[1] = {0.0};
#pragma unroll
  for (int k = 0; k < K; ++k) r1[0] += x[k] * d[k];
  bsum<1>(R, r1);
  p.xv = r1[0];
  double r2[1] = {0.0};
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const bool ok = tid + k * ST_THREADS < n;
    p.q[k] = ok ? (y[k] * (d[k] - x[k] * p.xv)) / x[k] : 0.0;
    r2[0] += ok ? x[k] * p.q[k] : 0.0;
  }
  bsum<1>(R, r2);
  p.xq = r2[0];
}

template <int K, class Hooks>
__device__ __forceinline__ int tcg_math(TcgScalars& t, const riptrm_options& opt, int n, Red& R, double (&u)[K],
                                        double (&d)[K], const double (&x)[K], const double (&y)[K],
                                        const double (&c)[K], double (&e)[K], double (&he)[K], double (&rv)[K],
                                        Hooks& h, const HwPre<K>& pre) {
  // hw_apply(U, D, U): xu = <x, S delta>; the u-free part came in `pre`
  double r1[1] = {0.0};
#pragma unroll
  for (int k = 0; k < K; ++k) r1[0] += x[k] * u[k];
  bsum<1>(R, r1);
  h.stamp(0);
  h.stamp(1);
  const double xu = r1[0];
  const double xq = pre.xq;
  const double coef = t.coef;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const double hf = -u[k] + xu * x[k];
    u[k] = (hf + coef * d[k]) + (pre.q[k] - xq * x[k]);
  }
  h.late_ceh();
  double d1[1] = {0.0};
#pragma unroll
  for (int k = 0; k < K; ++k) d1[0] += d[k] * u[k];
  bsum<1>(R, d1);
  h.stamp(2);
  const double d_Hd = d1[0];
  if (!isfinite(d_Hd)) return RIPTRM_TCG_NONFINITE;   // non-finite guard (include/riptrm.h)
  const double z_r = t.z_r, e_Pd = t.e_Pd, d_Pd = t.d_Pd, e_Pe = t.e_Pe;
  const double Delta = t.Delta;
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
#pragma unroll
    for (int k = 0; k < K; ++k) {
      e[k] = e[k] + tau * d[k];
      he[k] = he[k] + tau * u[k];
    }
    h.store_eh();
    return d_Hd <= 0.0 ? RIPTRM_TCG_NEGATIVE_CURVATURE : RIPTRM_TCG_EXCEEDED_TR;
  }
  t.e_Pe = e_Pe_new;
  // one reduction for the model value at eta + alpha delta and <r', r'> of the updated residual
  // r' = r + alpha H delta (computed speculatively, committed only if the model decreased); each
  // value keeps its own slot of the same tree, so both are bitwise what two reductions give
  h.late_r();
  double m3[3] = {0.0, 0.0, 0.0};
  double rn[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const double ne = e[k] + alpha * d[k];
    const double nh = he[k] + alpha * u[k];
    m3[0] += ne * c[k];
    m3[1] += ne * nh;
    rn[k] = rv[k] + alpha * u[k];
    m3[2] += rn[k] * rn[k];
  }
  bsum<3>(R, m3);
  h.stamp(3);
  const double new_model = m3[0] + 0.5 * m3[1];
  if (new_model >= t.model) return RIPTRM_TCG_MODEL_INCREASED;
  t.model = new_model;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    e[k] = e[k] + alpha * d[k];
    he[k] = he[k] + alpha * u[k];
    rv[k] = rn[k];
  }
  h.store_ehr();
  h.stamp(4);
  const double r_r = m3[2];
  const double norm_r = sqrt(r_r);
  const double nr0 = t.nr0;
  const double ka = opt.tcg_kappa;
  const double nr0t = t.nr0t;
  const double j = t.j;
  if (j >= (double)opt.tcg_mininner && norm_r <= nr0 * fmin(nr0t, ka))
    return ka < nr0t ? RIPTRM_TCG_REACHED_TARGET_LINEAR : RIPTRM_TCG_REACHED_TARGET_SUPERLINEAR;
  h.stamp(5);
  const double znew = r_r;
  const double beta = znew / z_r;
  double p1[1] = {0.0};
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const double dn = -rv[k] + beta * d[k];
    d[k] = dn;
    p1[0] += x[k] * dn;
  }
  bsum<1>(R, p1);
  h.stamp(6);
  const double xd = p1[0];
#pragma unroll
  for (int k = 0; k < K; ++k) d[k] = d[k] - xd * x[k];  // to_tangent_space
  h.store_d();
  t.z_r = znew;
  t.e_Pd = beta * (e_Pd + alpha * d_Pd);
  t.d_Pd = znew + (beta * beta) * d_Pd;
  t.j = j + 1.0;
  if (j + 1.0 >= (double)(n - 1)) {  // range(maxinner) exhausted; Python j stays maxinner-1
    t.j = j;
    return RIPTRM_TCG_MAX_INNER_ITER;
  }
  return TCG_CONTINUE;
}

// EXACT = false: the tCG machine (every shipped config); EXACT = true adds the Exact_RepMat
// branches (a separate k_state instantiation, so the tCG kernel carries none of its code or
// register / scratch pressure).  PERSIST = true: a replica inside k_persist (partial grid read
// with sc1 loads from the instance's slot `bp` of the grid `pb`, no active-list appends, the
// clock published at the last in-launch barrier so every replica takes the same decisions).
template <bool EXACT, bool PERSIST = false>
struct MachineT {
  const DevParams P;
  const int b;
  const int tid;
  const int n;
  const int out_list;
  Red R;
  double s[ST_HOT];   // hot scalars: identical in every thread, drive uniform control flow
  double* cold;       // cold scalars (ST_HOT..ST_N): read and written by thread 0 only
  double* tl;         // LDS of the Exact_RepMat subproblem (dynamic; Exact_RepMat solves only)
  const double* pb;   // S-pass partial grid of this step and this instance's slot in it
  int bp;
  // this instance's (or persistent replica's) slots: V(k) = vbase + k vkstride, scalars, stats,
  // request word, log (replicas keep no log)
  double* vbase;
  int64_t vkstride;
  double* ostats;
  int32_t* oreq;
  double* olog;
  int ocap;
  double uclk = 0.0;  // PERSIST: the workgroup-uniform clock of the last in-launch barrier
  int last_nr = 1;    // right-hand sides of the last request()
  bool tcg_cont = false;   // tcg_reg_core ended by requesting the next pass of the SAME tCG run

  // hot: where the hot scalars come from (nullptr = the workspace; k_persist keeps them in LDS
  // between its steps, so they are not live in registers across the tile pass).  use_rep: b is a
  // slot of the persistent replica block rb instead of an instance of P.
  __device__ __forceinline__ MachineT(const DevParams& P_, int b_, int out_list_, double* redbuf, double* tl_ = nullptr,
                                      const double* hot = nullptr, bool use_rep = false, RepBlock rb = RepBlock{})
      : P(P_), b(b_), tid(threadIdx.x), n(P_.n), out_list(out_list_), tl(tl_), pb(P_.pbuf), bp(b_) {
    R.buf = redbuf;
    R.parity = 0;
    vbase = (use_rep ? rb.vec : P.vec) + (int64_t)b * P.ld;
    vkstride = (int64_t)(use_rep ? rb.batch : P.batch) * P.ld;
    double* stb = (use_rep ? rb.st : P.st) + (int64_t)b * ST_N;
    ostats = (use_rep ? rb.stats : P.stats) + (int64_t)b * RIPTRM_STAT_NFIELDS;
    oreq = (use_rep ? rb.req : P.req) + b;
    olog = use_rep ? nullptr : P.log + (int64_t)b * P.cap * RIPTRM_LOG_NFIELDS;
    ocap = use_rep ? 0 : P.cap;
    const double* g = hot ? hot : stb;
#pragma unroll
    for (int k = 0; k < ST_HOT; ++k) s[k] = g[k];
    cold = stb;
  }

  // thread-0-owned counters / info fields
  __device__ __forceinline__ void cadd(int k, double v) { if (tid == 0) cold[k] += v; }
  __device__ __forceinline__ void cset(int k, double v) { if (tid == 0) cold[k] = v; }

  // workgroup-uniform device clock (thread 0 reads it, max-reduction broadcasts it)
  __device__ __forceinline__ double unow() {
    if constexpr (PERSIST) return uclk;
    double t[1] = {tid == 0 ? (double)wall_clock64() : -INFINITY};
    const int op[1] = {2};
    bred<1>(R, t, op);
    return t[0];
  }

  __device__ __forceinline__ double* V(int k) const { return vbase + k * vkstride; }
  __device__ __forceinline__ double elapsed_u(double t0) { return (unow() - t0) / P.clock_hz; }
  __device__ __forceinline__ double mu_at(int idx) const {
    const int i = idx < P.tab_len ? idx : P.tab_len - 1;
    return P.mu_tab[i];
  }

  __device__ __forceinline__ void copy(int dst, int src) {
    double* d = V(dst);
    const double* a = V(src);
    #pragma unroll 4
    for (int i = tid; i < n; i += ST_THREADS) d[i] = a[i];
  }

  // OUT_k = sum_J P_k[b][I][J] for the symmetric-tile layout, J in fixed order.  Each thread
  // sums GE elements at once with GJ partials per element in flight (GE*GJ loads per round),
  // so the ~nt rounds of memory latency of a naive loop become ~nt/GJ.
  // shared layout: out_k[i] = sum over the MM_KZ K-slices, in slice order
  __device__ __forceinline__ void gather_slices(int nr) {
    const int64_t ld = P.ld, slab = (int64_t)P.batch * ld;
    for (int k = 0; k < nr; ++k) {
      const double* pb = P.pbuf + ((int64_t)k * P.batch + b) * ld;
      double* O = V(k == 0 ? V_OUT0 : V_OUT1);
      for (int i = tid; i < n; i += ST_THREADS) {
        double acc = pb[i];
#pragma unroll
        for (int z = 1; z < MM_KZ; ++z) acc += pb[(int64_t)z * 2 * slab + i];
        O[i] = acc;
      }
    }
  }

  __device__ __forceinline__ void gather_out(int nr) {
    constexpr int GE = 8, GJ = 4;
    const int nt = P.smode ? P.nst : P.nt;   // tile or super-tile partial grid
    const int sh = P.smode ? 8 : 7, wd = 1 << sh;
    const int64_t nn = (int64_t)nt * nt * wd;
    for (int k = 0; k < nr; ++k) {
      const double* pbk = pb + ((int64_t)k * P.pbatch + bp) * nn;
      double* O = V(k == 0 ? V_OUT0 : V_OUT1);
      for (int base = tid; base < n; base += ST_THREADS * GE) {
        const double* q[GE];
        double acc[GE];
#pragma unroll
        for (int e = 0; e < GE; ++e) {
          int i = base + e * ST_THREADS;
          i = i < n ? i : n - 1;  // clamp: duplicate work, stored only if in range
          const int I = i >> sh, c = i - (I << sh);
          q[e] = pbk + (int64_t)I * nt * wd + c;
          acc[e] = ldp<PERSIST>(q[e]);
        }
        for (int J = 1; J < nt; J += GJ) {
          double t[GE][GJ];
#pragma unroll
          for (int e = 0; e < GE; ++e)
#pragma unroll
            for (int u = 0; u < GJ; ++u) t[e][u] = (J + u < nt) ? ldp<PERSIST>(q[e] + (int64_t)(J + u) * wd) : 0.0;
#pragma unroll
          for (int e = 0; e < GE; ++e)
#pragma unroll
            for (int u = 0; u < GJ; ++u)
              if (J + u < nt) acc[e] += t[e][u];
        }
#pragma unroll
        for (int e = 0; e < GE; ++e) {
          const int i = base + e * ST_THREADS;
          if (i < n) O[i] = acc[e];
        }
      }
    }
  }

  __device__ __forceinline__ int request(int nrhs) {
    last_nr = nrhs;
    if (tid == 0) {
      *oreq = nrhs;
      if constexpr (!PERSIST) {
        const int slot = atomicAdd(&P.cnt[out_list], 1);
        P.lists[out_list * P.batch + slot] = le_make(b, nrhs);
      }
    }
    cadd(ST_PASSES, 1.0);
    cadd(ST_RHS, (double)nrhs);
    return ACT_YIELD;
  }

  __device__ __forceinline__ void finish_write() {
    if (tid == 0) {
      double* g = cold;
#pragma unroll
      for (int k = 0; k < ST_HOT; ++k) g[k] = s[k];
      double* o = ostats;
      o[RIPTRM_STAT_OUTER_ITERS] = s[ST_OUTER_IT];
      o[RIPTRM_STAT_INNER_ITERS] = g[ST_INNER_TOTAL];
      o[RIPTRM_STAT_TCG_ITERS] = g[ST_TCG_TOTAL];
      o[RIPTRM_STAT_PASSES] = g[ST_PASSES];
      o[RIPTRM_STAT_RHS] = g[ST_RHS];
      o[RIPTRM_STAT_STOP_CODE] = g[ST_STOP_CODE];
      o[RIPTRM_STAT_STOP_RUNTIME] = g[ST_STOP_RUNTIME];
      o[RIPTRM_STAT_FINAL_RESIDUAL] = g[ST_RESIDUAL];
      o[RIPTRM_STAT_LOG_COUNT] = g[ST_LOG_COUNT];
      o[RIPTRM_STAT_LOG_OVERFLOW] = g[ST_LOG_OVERFLOW];
      o[RIPTRM_STAT_PHASE] = s[ST_PHASE];
      o[RIPTRM_STAT_MU] = s[ST_MU];
      o[RIPTRM_STAT_TR_RADIUS] = s[ST_DELTA];
      o[RIPTRM_STAT_TCG_LAST_J] = s[ST_J];
      o[RIPTRM_STAT_TCG_LAST_STOP] = s[ST_TCG_STOP];
      o[RIPTRM_STAT_ERROR] = g[ST_ERROR];
      o[RIPTRM_STAT_LOG_BASE] = g[ST_LOG_BASE];
    }
  }

  // ---- barrier Hessian HwCur(v) (RIPTRM.py:729; closed form SURVEY.md Appendix A) ----------
  // u = S v.  Writes Hw(v) into dst (dst may alias u).  Needs ST_COEF at the current x.
  // Hw(v) = P_x(-u) + coef v + G_x(q),  q = y (v - x (x.v)) / x,  G_x(w) = w - (x.w) x
  __device__ __forceinline__ void hw_apply(const double* u, const double* v, double* dst) {
    const double* X = V(V_X);
    const double* Y = V(V_Y);
    double r1[2] = {0.0, 0.0};
    #pragma unroll 4
    for (int i = tid; i < n; i += ST_THREADS) {
      r1[0] += X[i] * u[i];
      r1[1] += X[i] * v[i];
    }
    bsum<2>(R, r1);
    const double xu = r1[0], xv = r1[1];
    double r2[1] = {0.0};
    #pragma unroll 4
    for (int i = tid; i < n; i += ST_THREADS) {
      const double q = (Y[i] * (v[i] - X[i] * xv)) / X[i];
      r2[0] += X[i] * q;
    }
    bsum<1>(R, r2);
    const double xq = r2[0];
    const double coef = s[ST_COEF];
    #pragma unroll 4
    for (int i = tid; i < n; i += ST_THREADS) {
      const double q = (Y[i] * (v[i] - X[i] * xv)) / X[i];
      const double hf = -u[i] + xu * X[i];
      dst[i] = (hf + coef * v[i]) + (q - xq * X[i]);
    }
  }

  // ---- KKT evaluation, src/solver/utils.py:342-368 (+ compute_residual :269-340) ----------
  // ev: cost, distance, residual, gradnorm, complvio, dualvio, manvio, maxvio, meanvio, maxabsy
  __device__ __forceinline__ void evaluation(int xprev_kind, double (&ev)[10]) {
    const double* X = V(V_X);
    const double* Y = V(V_Y);
    const double* SX = V(V_SX);
    const double* XP = V(xprev_kind);
    double a[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    const int op[9] = {0, 0, 0, 0, 0, 0, 0, 2, 2};
    a[7] = 0.0;
    a[8] = -INFINITY;
    #pragma unroll 4
    for (int i = tid; i < n; i += ST_THREADS) {
      const double x = X[i], y = Y[i];
      a[0] += x * SX[i];                  // x.Sx
      a[1] += XP[i] * x;                  // xPrev.x
      a[2] += y * x;                      // y.x
      a[3] += x * x;                      // x.x
      const double cv = y * (-x);
      a[4] += cv * cv;                    // sum (y_i g_i)^2
      const double nv = fmax(-y, 0.0);
      a[5] += nv * nv;                    // sum max(-y_i,0)^2
      const double iv = fmax(-x, 0.0);
      a[6] += iv * iv;                    // sum max(g_i,0)^2
      a[7] = fmax(a[7], iv);              // max violation
      a[8] = fmax(a[8], fabs(y));         // max |y_i|
    }
    bred<9>(R, a, op);
    const double xSx = a[0], yx = a[2];
    const double xg = -xSx;
    double gg[2] = {0.0, 0.0};
    #pragma unroll 4
    for (int i = tid; i < n; i += ST_THREADS) {
      const double x = X[i];
      const double g = -SX[i];
      const double gl = (g - xg * x) - (Y[i] - yx * x);
      gg[0] += gl * gl;
      gg[1] += fmax(-x, 0.0);
    }
    bsum<2>(R, gg);
    const double gradnorm = sqrt(gg[0]);
    double manvio = 0.0;
    if (P.opt.manvio_kind == RIPTRM_MANVIO_SPHERE) manvio = sqrt(a[3]) - 1.0;
    const double sq = gradnorm * gradnorm + a[4] + a[5] + a[6] + 0.0 + manvio * manvio;
    double inner = a[1];
    inner = inner > 1.0 ? 1.0 : inner;
    inner = inner < -1.0 ? -1.0 : inner;
    ev[0] = -0.5 * xSx;
    ev[1] = acos(inner);
    ev[2] = sqrt(sq);
    ev[3] = gradnorm;
    ev[4] = sqrt(a[4]);
    ev[5] = sqrt(a[5]);
    ev[6] = manvio;
    ev[7] = a[7] > 0.0 ? a[7] : 0.0;
    ev[8] = gg[1] / (double)n;
    ev[9] = a[8];
  }

  // one log row; info == false -> solver_status(..., inner_info=None)
  __device__ __forceinline__ void log_row(const double (&ev)[10], bool info, double t_now) {
    if (tid == 0) {
      const double* c = cold;
      const int cnt = (int)c[ST_LOG_COUNT];
      const int64_t k = (int64_t)(c[ST_LOG_COUNT] - c[ST_LOG_BASE]);
      const int64_t capl = P.opt.log_capacity < ocap ? P.opt.log_capacity : ocap;
      if (capl > 0) {
        if (k >= capl) cold[ST_LOG_OVERFLOW] += 1.0;   // a record leaves the middle of the log
        double* L = olog + log_slot(k, capl) * RIPTRM_LOG_NFIELDS;
        L[RIPTRM_LOG_ITERATION] = s[ST_OUTER_IT];
        L[RIPTRM_LOG_TIME] = (cnt == 0) ? 0.0 : (t_now - s[ST_T_START]) / P.clock_hz;
        L[RIPTRM_LOG_COST] = ev[0];
        L[RIPTRM_LOG_DISTANCE] = ev[1];
        L[RIPTRM_LOG_RESIDUAL] = ev[2];
        L[RIPTRM_LOG_GRADNORM] = ev[3];
        L[RIPTRM_LOG_COMPLVIOLATION] = ev[4];
        L[RIPTRM_LOG_DUALVIOLATION] = ev[5];
        L[RIPTRM_LOG_MANVIOLATION] = ev[6];
        L[RIPTRM_LOG_MAXVIOLATION] = ev[7];
        L[RIPTRM_LOG_MEANVIOLATION] = ev[8];
        L[RIPTRM_LOG_MU] = s[ST_MU];
        L[RIPTRM_LOG_HAS_INFO] = info ? c[ST_I_HAS] : 0.0;
        L[RIPTRM_LOG_NUM_INNER] = c[ST_I_NUM];
        L[RIPTRM_LOG_INNER_STATUS] = c[ST_I_STATUS];
        L[RIPTRM_LOG_TR_RADIUS] = c[ST_I_TR];
        L[RIPTRM_LOG_DXTYPE] = c[ST_I_DXTYPE];
        L[RIPTRM_LOG_NORMDX] = c[ST_I_NORMDX];
        L[RIPTRM_LOG_MINXFEASI] = c[ST_I_MINX];
        L[RIPTRM_LOG_MINYFEASI] = c[ST_I_MINY];
        L[RIPTRM_LOG_COMPL] = c[ST_I_COMPL];
        L[RIPTRM_LOG_HAS_RATIO] = c[ST_I_HASRATIO];
        L[RIPTRM_LOG_ARED_PRED] = c[ST_I_RATIO];
        L[RIPTRM_LOG_RADIUS_UPDATE] = c[ST_I_RU];
        L[RIPTRM_LOG_DUAL_CLIPPING] = c[ST_I_DC];
        L[RIPTRM_LOG_HAS_MINEIG] = c[ST_I_HASMIN];
        L[RIPTRM_LOG_MINEIGVALHW] = c[ST_I_MINEIG];
        L[RIPTRM_LOG_MAXABSLAGMULT] = ev[9];
        L[RIPTRM_LOG_TCG_ITERS] = s[ST_J] + 1.0;
      } else {
        cold[ST_LOG_OVERFLOW] += 1.0;
      }
      cold[ST_LOG_COUNT] += 1.0;
    }
  }

  // Exact_RepMat beyond the LDS solver's size: the host serves the subproblem and the trial-point
  // eigenvalue from HBM (riptrm_trs_big.hip)
  __device__ __forceinline__ bool trs_big() const { return n - 1 > riptrm_trs::DIM_MAX || P.trs_hbm; }

  // Error stop (include/riptrm.h RIPTRM_ERR_NONFINITE / RIPTRM_ERR_EIGEN; RIPTRM.py:961-966):
  // stop the instance; inside an outer step (restore) hand back the iterate that step started
  // from, as the reference's break after an exception in outer_step does.  At the outer loop
  // head (restore = false) the completed iterate stays.  A tCG-only run keeps x, y as they are.
  __device__ __forceinline__ int nonfinite_stop(bool restore = true, int code = RIPTRM_ERR_NONFINITE) {
    if (restore && s[ST_OUTER_IT] > 0.0 && (int)s[ST_MODE] == MODE_SOLVE) {
      copy(V_X, V_X0);
      copy(V_Y, V_Y0);
      copy(V_SX, V_SX0);
    }
    cset(ST_ERROR, (double)code);
    cset(ST_STOP_RUNTIME, (unow() - s[ST_T_START]) / P.clock_hz);
    s[ST_PHASE] = PH_ERROR;
    return ACT_DONE;
  }

  // ---- outer loop head: RIPTRM.py:931-959 + base_solver.check_stoppingcriterion ------------
  __device__ __forceinline__ int outer_top() {
    double ev[10];
    evaluation(V_X0, ev);
    const bool save_inner = P.opt.save_inner_iteration != 0;
    const double tn = unow();
    if (s[ST_OUTER_IT] == 0.0 || !save_inner) log_row(ev, s[ST_OUTER_IT] != 0.0, tn);
    cset(ST_RESIDUAL, ev[2]);
    if (!isfinite(ev[2])) return nonfinite_stop(false);   // deliberate deviation, include/riptrm.h
    const double rt = (tn - s[ST_T_START]) / P.clock_hz;
    int stop = RIPTRM_STOP_NONE;
    if (rt >= P.opt.maxtime) stop = RIPTRM_STOP_MAXTIME;
    else if (s[ST_OUTER_IT] >= (double)P.opt.maxiter) stop = RIPTRM_STOP_MAXITER;
    if (ev[2] <= P.opt.tolresid) stop = RIPTRM_STOP_TOLRESID;
    if (stop != RIPTRM_STOP_NONE) {
      cset(ST_STOP_CODE, stop);
      cset(ST_STOP_RUNTIME, rt);
      s[ST_PHASE] = PH_DONE;
      return ACT_DONE;
    }
    if (s[ST_OUTER_IT] >= (double)P.outer_target) {
      s[ST_PHASE] = PH_PAUSED;
      return ACT_PAUSE;
    }
    return start_outer_step();
  }

  // restart_every cycling (benchmark windows only): back to (x0, y0, mu_0, Delta_0)
  __device__ __forceinline__ void maybe_restart() {
    const int k = P.opt.restart_every;
    if (k > 0 && s[ST_OUTER_IT] > 0.0 && fmod(s[ST_OUTER_IT], (double)k) == 0.0) {
      copy(V_X, V_XI);
      copy(V_Y, V_YI);
      copy(V_SX, V_SXI);
      s[ST_MU_IDX] = 0.0;
      s[ST_MU] = mu_at(0);
      s[ST_DELTA] = P.opt.initial_tr_radius;
    }
  }

  // RIPTRM.py:866-887 + inner_run :785-799
  __device__ __forceinline__ int start_outer_step() {
    maybe_restart();
    s[ST_OUTER_IT] += 1.0;
    const int mi = (int)s[ST_MU_IDX];
    const int ti = mi < P.tab_len ? mi : P.tab_len - 1;
    s[ST_TOLL] = P.tolL_tab[ti];
    s[ST_TOLC] = P.tolC_tab[ti];
    copy(V_X0, V_X);
    copy(V_Y0, V_Y);
    copy(V_SX0, V_SX);
    copy(V_XPREV, V_X);
    s[ST_DELTA0] = s[ST_DELTA];
    s[ST_INNER_IT] = 0.0;
    s[ST_T_INNER] = unow();
    return inner_step_begin();
  }

  // RIPTRM.py:707-733: quantities at x, then tCG start (RIPTRM.py:46-96 with eta = 0)
  __device__ __forceinline__ int inner_step_begin() {
    s[ST_INNER_IT] += 1.0;
    s[ST_DELTA_STEP] = s[ST_DELTA];
    return tcg_begin();
  }

  __device__ __forceinline__ int tcg_begin() {
    const double* X = V(V_X);
    const double* Y = V(V_Y);
    const double* SX = V(V_SX);
    double* C = V(V_C);
    double* Rv = V(V_R);
    double* D = V(V_IN0);
    double* E = V(V_ETA);
    double* HE = V(V_HETA);
    const double mu = s[ST_MU];
    double h[4] = {0.0, 0.0, 0.0, 0.0};
    #pragma unroll 4
    for (int i = tid; i < n; i += ST_THREADS) {
      const double x = X[i];
      h[0] += x * x;
      h[1] += x * SX[i];
      h[2] += Y[i] * x;
      h[3] += x * (mu / x);
    }
    bsum<4>(R, h);
    const double xx = h[0], xSx = h[1], yx = h[2], xm = h[3];
    s[ST_XX] = xx;
    s[ST_XSX] = xSx;
    s[ST_YX] = yx;
    s[ST_COEF] = (xSx + yx) * xx;
    s[ST_FCUR] = -0.5 * xSx;
    const double xg = -xSx;
    double rr[1] = {0.0};
    #pragma unroll 4
    for (int i = tid; i < n; i += ST_THREADS) {
      const double x = X[i];
      const double g = -SX[i];
      const double m = mu / x;
      const double c = (g - xg * x) - (m - xm * x);   // cxCur, RIPTRM.py:730
      C[i] = c;
      Rv[i] = c;
      D[i] = -c;
      E[i] = 0.0;
      HE[i] = 0.0;
      rr[0] += c * c;
    }
    bsum<1>(R, rr);
    s[ST_NORMR0] = sqrt(rr[0]);
    if (!isfinite(s[ST_NORMR0]) || !isfinite(s[ST_DELTA])) return nonfinite_stop();
    s[ST_ZR] = rr[0];
    s[ST_DPD] = rr[0];
    s[ST_EPE] = 0.0;
    s[ST_EPD] = 0.0;
    s[ST_MODEL] = 0.0;
    s[ST_J] = 0.0;
    s[ST_HASMIN] = 0.0;
    s[ST_MINEIG] = 0.0;
    s[ST_MINEIG_OK] = 1.0;
    if constexpr (EXACT) {
      if (P.opt.trs_solver == RIPTRM_TRS_SOLVER_EXACT_REPMAT && (int)s[ST_MODE] == MODE_SOLVE) {
        if (trs_big()) {   // the host serves the subproblem (riptrm_trs_big.hip), then PH_TRS_END
          s[ST_PHASE] = PH_TRS_HOST;
          return ACT_PAUSE;
        }
        s[ST_PHASE] = PH_TRS;
        return ACT_CONTINUE;
      }
    }
    if (n - 1 <= 0) {  // maxinner = manifold.dim = 0: no tCG iteration is possible
      cset(ST_ERROR, (double)RIPTRM_ERR_NO_TCG_ITER);
      s[ST_PHASE] = PH_ERROR;
      return ACT_DONE;
    }
    s[ST_PHASE] = PH_TCG;
    return request(1);
  }

  // one tCG iteration after Hdelta's S-pass: RIPTRM.py:100-214
  __device__ __forceinline__ int tcg_step() {
    double* U = V(V_OUT0);          // S delta, overwritten with Hdelta
    const double* D = V(V_IN0);     // delta
    hw_apply(U, D, U);
    const double* X = V(V_X);
    const double* C = V(V_C);
    double* E = V(V_ETA);
    double* HE = V(V_HETA);
    double* Rv = V(V_R);
    double* Dw = V(V_IN0);
    double d1[1] = {0.0};
    #pragma unroll 4
    for (int i = tid; i < n; i += ST_THREADS) d1[0] += D[i] * U[i];
    bsum<1>(R, d1);
    const double d_Hd = d1[0];
    if (!isfinite(d_Hd)) {   // non-finite guard (include/riptrm.h)
      s[ST_TCG_STOP] = RIPTRM_TCG_NONFINITE;
      return tcg_end();
    }
    const double z_r = s[ST_ZR], e_Pd = s[ST_EPD], d_Pd = s[ST_DPD], e_Pe = s[ST_EPE];
    const double Delta = s[ST_DELTA];
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
      #pragma unroll 4
      for (int i = tid; i < n; i += ST_THREADS) {
        E[i] = E[i] + tau * D[i];
        HE[i] = HE[i] + tau * U[i];
      }
      s[ST_TCG_STOP] = d_Hd <= 0.0 ? RIPTRM_TCG_NEGATIVE_CURVATURE : RIPTRM_TCG_EXCEEDED_TR;
      return tcg_end();
    }
    s[ST_EPE] = e_Pe_new;
    double m2[2] = {0.0, 0.0};
    #pragma unroll 4
    for (int i = tid; i < n; i += ST_THREADS) {
      const double ne = E[i] + alpha * D[i];
      const double nh = HE[i] + alpha * U[i];
      m2[0] += ne * C[i];
      m2[1] += ne * nh;
    }
    bsum<2>(R, m2);
    const double new_model = m2[0] + 0.5 * m2[1];
    if (new_model >= s[ST_MODEL]) {
      s[ST_TCG_STOP] = RIPTRM_TCG_MODEL_INCREASED;
      return tcg_end();
    }
    s[ST_MODEL] = new_model;
    double r2[1] = {0.0};
    #pragma unroll 4
    for (int i = tid; i < n; i += ST_THREADS) {
      E[i] = E[i] + alpha * D[i];
      HE[i] = HE[i] + alpha * U[i];
      const double r = Rv[i] + alpha * U[i];
      Rv[i] = r;
      r2[0] += r * r;
    }
    bsum<1>(R, r2);
    const double r_r = r2[0];
    const double norm_r = sqrt(r_r);
    const double nr0 = s[ST_NORMR0];
    const double th = P.opt.tcg_theta, ka = P.opt.tcg_kappa;
    const double nr0t = pow(nr0, th);
    const double j = s[ST_J];
    if (j >= (double)P.opt.tcg_mininner && norm_r <= nr0 * fmin(nr0t, ka)) {
      s[ST_TCG_STOP] = ka < nr0t ? RIPTRM_TCG_REACHED_TARGET_LINEAR : RIPTRM_TCG_REACHED_TARGET_SUPERLINEAR;
      return tcg_end();
    }
    const double zold = z_r;
    const double znew = r_r;
    const double beta = znew / zold;
    double p1[1] = {0.0};
    #pragma unroll 4
    for (int i = tid; i < n; i += ST_THREADS) {
      const double dn = -Rv[i] + beta * D[i];
      Dw[i] = dn;
      p1[0] += X[i] * dn;
    }
    bsum<1>(R, p1);
    const double xd = p1[0];
    #pragma unroll 4
    for (int i = tid; i < n; i += ST_THREADS) Dw[i] = Dw[i] - xd * X[i];  // to_tangent_space
    s[ST_ZR] = znew;
    s[ST_EPD] = beta * (e_Pd + alpha * d_Pd);
    s[ST_DPD] = znew + (beta * beta) * d_Pd;
    s[ST_J] = j + 1.0;
    if (j + 1.0 >= (double)(n - 1)) {  // range(maxinner) exhausted; Python j stays maxinner-1
      s[ST_J] = j;
      s[ST_TCG_STOP] = RIPTRM_TCG_MAX_INNER_ITER;
      return tcg_end();
    }
    return request(1);
  }

  // ---- register-resident tCG iteration (n <= RT_EPT * ST_THREADS) ------------------------------
  // Same arithmetic, element order and reductions as gather_out + tcg_step (bitwise identical),
  // but every vector is read from memory once and kept in registers across the iteration's six
  // reductions (element i = tid + k * ST_THREADS, k < RT_EPT): one load phase, one store phase.
  static constexpr int RT_EPT = 8;

  template <int K>
  __device__ __forceinline__ void load_reg(int kind, double (&r)[K]) const { rl_load<K>(V(kind), n, r); }
  template <int K>
  __device__ __forceinline__ void store_reg(int kind, const double (&r)[K]) const { rl_store<K>(V(kind), n, r); }
  template <int K>
  __device__ __forceinline__ void gather_reg(double (&u)[K]) { rl_gather<K, PERSIST>(P, pb, bp, u); }

  template <int K>
  struct TcgVecs {
    double d[K], x[K], y[K], c[K], e[K], he[K], rv[K];
  };

  template <int K>
  __device__ __forceinline__ int tcg_step_reg() {
    // every operand loaded up front: one memory round trip per iteration instead of three (the
    // ~150 VGPRs of K = 8 fit the 256 a wave has at two waves per SIMD; one workgroup per
    // instance never fills the chip, so occupancy is not the limit)
    TcgVecs<K> v;
    double u[K];
    gather_reg<K>(u);
    load_reg<K>(V_IN0, v.d);
    load_reg<K>(V_X, v.x);
    load_reg<K>(V_Y, v.y);
    load_reg<K>(V_C, v.c);
    load_reg<K>(V_ETA, v.e);
    load_reg<K>(V_HETA, v.he);
    load_reg<K>(V_R, v.rv);
    return tcg_reg_core<K, true>(v, u);
  }

  // k_persist: every operand already in registers (v carried over from the previous iteration)
  template <int K>
  __device__ __forceinline__ void tcg_fast_load(TcgVecs<K>& v) const {
    load_reg<K>(V_IN0, v.d);
    load_reg<K>(V_X, v.x);
    load_reg<K>(V_Y, v.y);
    load_reg<K>(V_C, v.c);
    load_reg<K>(V_ETA, v.e);
    load_reg<K>(V_HETA, v.he);
    load_reg<K>(V_R, v.rv);
  }
  template <int K>
  __device__ __forceinline__ void tcg_fast_flush(const TcgVecs<K>& v) const {
    store_reg(V_IN0, v.d);
    store_reg(V_ETA, v.e);
    store_reg(V_HETA, v.he);
    store_reg(V_R, v.rv);
  }

  // One tCG iteration on register-resident vectors, u = S delta (tcg_math below).  MEM = true
  // (k_state): the vectors round-trip through the workspace every iteration (stores as each is
  // final, c / e / he / rv loaded late for K > 2).  MEM = false (k_persist's fast path): v holds
  // every operand and stays in registers across iterations; nothing is stored until the tCG stops
  // (then every modified vector is flushed before tcg_end reads it).
  template <int K, bool MEM>
  struct TcgHooks {
    MachineT& M;
    TcgVecs<K>& v;
    __device__ __forceinline__ void late_ceh() {
      // (operands are loaded up front by tcg_step_reg)
    }
    __device__ __forceinline__ void late_r() {
      // (operands are loaded up front by tcg_step_reg)
    }
    __device__ __forceinline__ void store_eh() {
      if constexpr (MEM) {
        M.store_reg(V_ETA, v.e);
        M.store_reg(V_HETA, v.he);
      }
    }
    __device__ __forceinline__ void store_ehr() {
      if constexpr (MEM) {
        M.store_reg(V_ETA, v.e);
        M.store_reg(V_HETA, v.he);
        M.store_reg(V_R, v.rv);
      }
    }
    __device__ __forceinline__ void store_d() {
      if constexpr (MEM) M.store_reg(V_IN0, v.d);
    }
    __device__ __forceinline__ void stamp(int) {}
  };

  __device__ __forceinline__ TcgScalars tcg_scalars() const {
    TcgScalars t;
    t.coef = s[ST_COEF];
    t.z_r = s[ST_ZR];
    t.e_Pd = s[ST_EPD];
    t.d_Pd = s[ST_DPD];
    t.e_Pe = s[ST_EPE];
    t.Delta = s[ST_DELTA];
    t.model = s[ST_MODEL];
    t.nr0 = s[ST_NORMR0];
    t.j = s[ST_J];
    t.nr0t = pow(t.nr0, P.opt.tcg_theta);
    return t;
  }
  __device__ __forceinline__ void tcg_scalars_back(const TcgScalars& t) {
    s[ST_ZR] = t.z_r;
    s[ST_EPD] = t.e_Pd;
    s[ST_DPD] = t.d_Pd;
    s[ST_EPE] = t.e_Pe;
    s[ST_MODEL] = t.model;
    s[ST_J] = t.j;
  }

  template <int K, bool MEM>
  __device__ __forceinline__ int tcg_reg_core(TcgVecs<K>& v, double (&u)[K]) {
    tcg_cont = false;   // a stop may start a new tCG (infeasible trial -> tcg_begin) whose
                        // request must not be mistaken for this run's next pass
    TcgScalars t = tcg_scalars();
    TcgHooks<K, MEM> h{*this, v};
    HwPre<K> pre;
    tcg_math_pre<K>(pre, n, R, v.d, v.x, v.y);
    const int stop = tcg_math<K>(t, P.opt, n, R, u, v.d, v.x, v.y, v.c, v.e, v.he, v.rv, h, pre);
    tcg_scalars_back(t);
    if (stop != TCG_CONTINUE) {
      if constexpr (!MEM) tcg_fast_flush(v);
      s[ST_TCG_STOP] = stop;
      return tcg_end();
    }
    tcg_cont = true;
    return request(1);
  }

  // ---- Exact_RepMat (RIPTRM.py:433-444, :599-617), n - 1 <= RIPTRM_TRS_DIM_MAX ---------------
  // Tangent basis of x^perp: b_k = H e_k (k = 1..n-1) with the Householder reflector
  // H = I - tau w w^T, w = x + sign(x_0) ||x|| e_0 (H x = -sign(x_0) ||x|| e_0, so the b_k are
  // orthonormal and orthogonal to x).  For tangent b_i, b_j the closed form of HwCur
  //  gives <b_i, Hw b_j> = b_i^T (-S + diag(y/x)) b_j + coef delta_ij, so the
  // represented matrix (selfadj_operator2matrix, utils.py:565-573) is the trailing block of
  // H M H = M - tau (w u^T + u w^T) + tau^2 (w^T u) w w^T, u = M w, M = -S + diag(y/x): O(n^2)
  // instead of n HVPs.  The reference's basis is random (utils.py:388-397); the subproblem's
  // solution and the eigenvalues do not depend on it.
  __device__ __forceinline__ double s_at(int i, int j) const {
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
  // LDS: [Work of dim n-1][w: n][u: n][Blk scratch]
  __device__ __forceinline__ riptrm_trs::lds_f64* trs_wvec() const {
    return (riptrm_trs::lds_f64*)tl + riptrm_trs::work_doubles(n - 1);
  }
  __device__ __forceinline__ riptrm_trs::lds_f64* trs_uvec() const { return trs_wvec() + riptrm_trs::DIM_MAX + 1; }
  __device__ __forceinline__ double* trs_red() const { return (double*)(trs_uvec() + riptrm_trs::DIM_MAX + 1); }

  // A <- (H M H)[1:, 1:] + coef I at (X, Y); returns tau (w in trs_wvec)
  __device__ __noinline__ double repmat(riptrm_trs::Blk<ST_THREADS>& B, riptrm_trs::Work& w, const double* X,
                                           const double* Y, double xx, double coef) {
    riptrm_trs::lds_f64* Wv = trs_wvec();
    riptrm_trs::lds_f64* Uv = trs_uvec();
    const double sg = X[0] >= 0.0 ? 1.0 : -1.0;
    double ww = 0.0;
    for (int i = tid; i < n; i += ST_THREADS) {
      const double wi = i == 0 ? X[0] + sg * sqrt(xx) : X[i];
      Wv[i] = wi;
      ww += wi * wi;
    }
    ww = B.sum(ww);
    const double tau = 2.0 / ww;
    __syncthreads();
    double wu = 0.0;
    for (int i = tid; i < n; i += ST_THREADS) {
      double acc = 0.0;
      for (int j = 0; j < n; ++j) acc += s_at(i, j) * Wv[j];
      const double ui = -acc + (Y[i] / X[i]) * Wv[i];
      Uv[i] = ui;
      wu += Wv[i] * ui;
    }
    const double gam = B.sum(wu);
    __syncthreads();
    const int m = n - 1;
    const double t2g = (tau * tau) * gam;
    for (int e = tid; e < m * m; e += ST_THREADS) {
      const int i = e / m + 1, j = e - (i - 1) * m + 1;
      double mij = -s_at(i, j);
      if (i == j) mij += Y[i] / X[i];
      double v = (mij - tau * (Wv[i] * Uv[j] + Uv[i] * Wv[j])) + t2g * (Wv[i] * Wv[j]);
      if (i == j) v += coef;
      w.A[(i - 1) * w.lda + (j - 1)] = v;
    }
    __syncthreads();
    return tau;
  }

  // compute_direction's Exact_RepMat branch: eta <- argmin of the model over the ball, then the
  // rest of the inner step as after tCG
  __device__ __noinline__ int trs_direction() {
    riptrm_trs::Blk<ST_THREADS> B(trs_red());
    riptrm_trs::Work w = riptrm_trs::make_work(tl, n - 1);
    const double* X = V(V_X);
    const double* Y = V(V_Y);
    const double* Cv = V(V_C);
    const double tau = repmat(B, w, X, Y, s[ST_XX], s[ST_COEF]);
    const riptrm_trs::lds_f64* Wv = trs_wvec();
    double wc = 0.0;   // cxCurvector_k = <c, b_k> = (H c)_k (RIPTRM.py:438-440)
    for (int i = tid; i < n; i += ST_THREADS) wc += Wv[i] * Cv[i];
    wc = B.sum(wc);
    for (int k = tid + 1; k < n; k += ST_THREADS) w.a[k - 1] = Cv[k] - tau * Wv[k] * wc;
    __syncthreads();
    const riptrm_trs::Result r = riptrm_trs::trs_solve<ST_THREADS>(B, w, s[ST_DELTA], P.opt.trs_tolhardcase);
    double wz = 0.0;   // dx = sum_k coeff_k b_k = H [0; coeff] (RIPTRM.py:442-444)
    for (int k = tid + 1; k < n; k += ST_THREADS) wz += Wv[k] * w.x[k - 1];
    wz = B.sum(wz);
    double* E = V(V_ETA);
    for (int i = tid; i < n; i += ST_THREADS) E[i] = (i == 0 ? 0.0 : w.x[i - 1]) - tau * Wv[i] * wz;
    __syncthreads();
    s[ST_TCG_STOP] = RIPTRM_TRS_BOUNDARY + r.kind;
    s[ST_J] = -1.0;   // no tCG iterations
    s[ST_PHASE] = PH_TRS_END;
    return ACT_CONTINUE;
  }

  // smallest eigenvalue of HwNew's matrix at (x_new, y_new) = (IN1, YNEW) (RIPTRM.py:599-612);
  // S x_new directly from S (n <= 97)
  __device__ __noinline__ double trial_mineig() {
    riptrm_trs::Blk<ST_THREADS> B(trs_red());
    riptrm_trs::Work w = riptrm_trs::make_work(tl, n - 1);
    const double* XN = V(V_IN1);
    const double* YN = V(V_YNEW);
    double h3[3] = {0.0, 0.0, 0.0};
    for (int i = tid; i < n; i += ST_THREADS) {
      double acc = 0.0;
      for (int j = 0; j < n; ++j) acc += s_at(i, j) * XN[j];
      h3[0] += XN[i] * XN[i];
      h3[1] += XN[i] * acc;
      h3[2] += YN[i] * XN[i];
    }
    const double xx = B.sum(h3[0]), xSx = B.sum(h3[1]), yx = B.sum(h3[2]);
    repmat(B, w, XN, YN, xx, (xSx + yx) * xx);
    return riptrm_trs::min_eig<ST_THREADS>(B, w);
  }

  // after tCG: RIPTRM.py:733-746 (direction, ||dx||, dy, retraction) + feasibility part of :591
  __device__ __forceinline__ int tcg_end() {
    if (s[ST_TCG_STOP] == RIPTRM_TCG_NONFINITE) return nonfinite_stop();
    if (s[ST_TCG_STOP] == RIPTRM_TCG_EIGFAIL) return nonfinite_stop(true, RIPTRM_ERR_EIGEN);
    cadd(ST_TCG_TOTAL, s[ST_J] + 1.0);
    const double* X = V(V_X);
    const double* Y = V(V_Y);
    const double* E = V(V_ETA);
    double e1[2] = {0.0, 0.0};
    #pragma unroll 4
    for (int i = tid; i < n; i += ST_THREADS) {
      e1[0] += E[i] * E[i];
      e1[1] += X[i] * E[i];
    }
    bsum<2>(R, e1);
    const double normdx = sqrt(e1[0]);
    const double xdx = e1[1];
    s[ST_NORMDX] = normdx;
    s[ST_XDX] = xdx;
    if ((int)s[ST_MODE] == MODE_TCG_ONLY) {
      s[ST_PHASE] = PH_DONE;
      return ACT_DONE;
    }
    const double mu = s[ST_MU];
    double* YN = V(V_YNEW);
    double* XN = V(V_IN1);
    double w2[1] = {0.0};
    #pragma unroll 4
    for (int i = tid; i < n; i += ST_THREADS) {
      const double x = X[i], y = Y[i], dx = E[i];
      const double dy = (-y + mu * (1.0 / x)) - (y * (dx - x * xdx)) / x;   // RIPTRM.py:743
      YN[i] = y + dy;
      const double w = x + dx;
      w2[0] += w * w;
    }
    bsum<1>(R, w2);
    const double nw = sqrt(w2[0]);
    double* D = V(V_IN0);
    double c3[5] = {INFINITY, INFINITY, 0.0, 0.0, 0.0};
    const int op3[5] = {1, 1, 0, 0, 0};
    #pragma unroll 4
    for (int i = tid; i < n; i += ST_THREADS) {
      const double dx = E[i];
      const double xn = (X[i] + dx) / nw;   // retraction (x+dx)/||x+dx||
      XN[i] = xn;
      D[i] = dx;
      const double yn = YN[i];
      c3[0] = fmin(c3[0], xn);
      c3[1] = fmin(c3[1], yn);
      c3[2] += (xn > 0.0) ? 0.0 : 1.0;
      c3[3] += (yn > 0.0) ? 0.0 : 1.0;
      const double cv = yn * xn - mu;
      c3[4] += cv * cv;
    }
    bred<5>(R, c3, op3);
    s[ST_MINX] = c3[0];
    s[ST_MINY] = c3[1];
    s[ST_XFEAS] = (c3[2] == 0.0) ? 1.0 : 0.0;
    s[ST_COMPL] = sqrt(c3[4]);
    s[ST_YFEAS] = (c3[3] == 0.0) ? 1.0 : 0.0;
    if (EXACT && P.opt.trs_solver == RIPTRM_TRS_SOLVER_EXACT_REPMAT && P.opt.second_order_stationarity) {
      // compute_inner_stoppingcriteria's eigen-check at (x_new, y_new), RIPTRM.py:599-613
      if (trs_big()) {   // the host takes the smallest eigenvalue, then PH_MINEIG_END
        s[ST_PHASE] = PH_MINEIG_HOST;
        return ACT_PAUSE;
      }
      double me = 0.0;
      if constexpr (EXACT) me = trial_mineig();
      s[ST_MINEIG] = me;
      mineig_test();
    }
    return tcg_end_tail();
  }

  // s[ST_MINEIG] against -forcing_function_second_order(mu) (RIPTRM.py:613)
  __device__ __forceinline__ void mineig_test() {
    const int mi = (int)s[ST_MU_IDX];
    const double tol2 = P.opt.tol2_table ? P.opt.tol2_table[mi < P.tab_len ? mi : P.tab_len - 1] : s[ST_MU];
    s[ST_HASMIN] = 1.0;
    s[ST_MINEIG_OK] = (s[ST_MINEIG] >= -tol2) ? 1.0 : 0.0;
  }

  // the rest of the step after the trial point's criteria: RIPTRM.py:746-775
  __device__ __forceinline__ int tcg_end_tail() {
    if (s[ST_XFEAS] != 0.0) {
      s[ST_PHASE] = PH_TRIAL;
      return request(2);
    }
    // primal infeasible: RIPTRM.py:769-775
    set_info(RIPTRM_IS_PRIMAL_INFEASIBLE, false, 0.0, RIPTRM_RU_NONE, -1.0);
    s[ST_DELTA] = P.opt.gamma * s[ST_NORMDX];
    return inner_loop_tail(false);
  }

  __device__ __forceinline__ void set_info(int status, bool has_ratio, double ratio, int ru, double dc) {
    if (tid == 0) {
      double* c = cold;
      c[ST_I_HAS] = 1.0;
      c[ST_I_NUM] = s[ST_INNER_IT];
      c[ST_I_STATUS] = status;
      c[ST_I_TR] = s[ST_DELTA_STEP];
      c[ST_I_DXTYPE] = s[ST_TCG_STOP];
      c[ST_I_NORMDX] = s[ST_NORMDX];
      c[ST_I_MINX] = s[ST_MINX];
      c[ST_I_MINY] = s[ST_MINY];
      c[ST_I_COMPL] = s[ST_COMPL];
      c[ST_I_HASRATIO] = has_ratio ? 1.0 : 0.0;
      c[ST_I_RATIO] = ratio;
      c[ST_I_RU] = ru;
      c[ST_I_DC] = dc;
      c[ST_I_HASMIN] = s[ST_HASMIN];
      c[ST_I_MINEIG] = s[ST_MINEIG];
    }
  }

  // after the 2-RHS pass (S dx, S x_new): RIPTRM.py:748-783 with :574-629 and :631-705
  __device__ __forceinline__ int trial_eval() {
    const double* X = V(V_X);
    const double* XN = V(V_IN1);
    const double* YN = V(V_YNEW);
    const double* SXN = V(V_OUT1);
    const double mu = s[ST_MU];
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    #pragma unroll 4
    for (int i = tid; i < n; i += ST_THREADS) {
      const double xn = XN[i];
      a[0] += xn * SXN[i];
      a[1] += YN[i] * xn;
      a[2] += log(X[i]);
      a[3] += log(xn);
    }
    bsum<4>(R, a);
    const double xnS = a[0], ynxn = a[1];
    const double xg = -xnS;
    double g2[1] = {0.0};
    #pragma unroll 4
    for (int i = tid; i < n; i += ST_THREADS) {
      const double xn = XN[i];
      const double gl = (-SXN[i] - xg * xn) - (YN[i] - ynxn * xn);   // gradLagrangefun
      g2[0] += gl * gl;
    }
    bsum<1>(R, g2);
    const double normgl = sqrt(g2[0]);
    const bool yfeas = s[ST_YFEAS] != 0.0;
    const bool conv = yfeas && normgl <= s[ST_TOLL] && s[ST_COMPL] <= s[ST_TOLC] && s[ST_MINEIG_OK] != 0.0;
    if (conv) {  // RIPTRM.py:762-766
      copy(V_X, V_IN1);
      copy(V_Y, V_YNEW);
      copy(V_SX, V_OUT1);
      set_info(RIPTRM_IS_CONVERGED, false, 0.0, RIPTRM_RU_NONE, -1.0);
      return inner_loop_tail(true);
    }
    // update_xy_TR_radius, RIPTRM.py:631-705
    const double lb_c = s[ST_FCUR] - mu * a[2];
    const double lb_n = (-0.5 * xnS) - mu * a[3];
    double ared = lb_c - lb_n;
    double* HW = V(V_OUT0);
    const double* DX = V(V_IN0);
    hw_apply(HW, DX, HW);
    const double* C = V(V_C);
    double pp[2] = {0.0, 0.0};
    #pragma unroll 4
    for (int i = tid; i < n; i += ST_THREADS) {
      pp[0] += HW[i] * DX[i];
      pp[1] += C[i] * DX[i];
    }
    bsum<2>(R, pp);
    double pred = (0.0 - 0.5 * pp[0]) - pp[1];
    const double red_reg = fmax(1.0, fabs(lb_c)) * 2.220446049250313e-16 * P.opt.reduction_regularization;
    ared = ared + red_reg;
    pred = pred + red_reg;
    const double ratio = ared / pred;
    const double Delta = s[ST_DELTA];
    double Dn;
    int ru;
    if (ared < 0.25 * pred) {
      ru = RIPTRM_RU_REDUCED;
      Dn = 0.25 * Delta;
    } else if (ared >= 0.75 * pred && fabs(s[ST_NORMDX] - Delta) <= 1e-15) {
      ru = RIPTRM_RU_EXPANDED;
      const double d2 = 2.0 * Delta;
      Dn = d2 < P.opt.maximal_tr_radius ? d2 : P.opt.maximal_tr_radius;
    } else {
      ru = RIPTRM_RU_UNCHANGED;
      Dn = Delta;
    }
    if (ared > P.opt.rho * pred) {
      const double cl = P.opt.const_left, cr = P.opt.const_right;
      const double iright = np_max(cr, cr / mu);   // RIPTRM.py:682 (3-arg np.maximum quirk)
      double* Xw = V(V_X);
      double* Yw = V(V_Y);
      double* SXw = V(V_SX);
      double nd[1] = {0.0};
      #pragma unroll 4
      for (int i = tid; i < n; i += ST_THREADS) {
        const double xn = XN[i], yn = YN[i];
        const double il = cl * np_min(np_min(Yw[i], mu / xn), 1.0);
        const double yc = np_min(np_max(yn, il), iright);
        nd[0] += (yc != yn) ? 1.0 : 0.0;
        Xw[i] = xn;
        Yw[i] = yc;
        SXw[i] = SXN[i];
      }
      bsum<1>(R, nd);
      set_info(RIPTRM_IS_SUCCESSFUL, true, ratio, ru, nd[0] > 0.0 ? 1.0 : 0.0);
    } else {
      set_info(RIPTRM_IS_UNSUCCESSFUL, true, ratio, ru, -1.0);
    }
    s[ST_DELTA] = Dn;
    return inner_loop_tail(false);
  }

  // inner_run after a step: log, time/iteration limits, exit -> outer update (RIPTRM.py:810-896)
  __device__ __forceinline__ int inner_loop_tail(bool converged) {
    cadd(ST_INNER_TOTAL, 1.0);
    const double tn = unow();
    if (P.opt.save_inner_iteration) {
      double ev[10];
      evaluation(V_XPREV, ev);
      log_row(ev, true, tn);
    }
    copy(V_XPREV, V_X);
    bool exitflag = converged;
    double rt, lim;
    if (P.opt.inner_maxtime < 0.0) {
      lim = P.opt.maxtime;
      rt = (tn - s[ST_T_START]) / P.clock_hz;
    } else {
      lim = P.opt.inner_maxtime;
      rt = (tn - s[ST_T_INNER]) / P.clock_hz;
    }
    bool reset = false;
    if (rt >= lim) reset = true;
    if (P.opt.inner_maxiter >= 0 && s[ST_INNER_IT] >= (double)P.opt.inner_maxiter) reset = true;
    if (reset) {
      cset(ST_I_STATUS, s[ST_INNER_IT] * 0.0 + (rt >= lim && !(P.opt.inner_maxiter >= 0 && s[ST_INNER_IT] >= (double)P.opt.inner_maxiter) ? RIPTRM_IS_MAX_TIME_EXCEEDED : RIPTRM_IS_MAX_ITER_EXCEEDED));
      exitflag = true;
      copy(V_X, V_X0);
      copy(V_Y, V_Y0);
      copy(V_SX, V_SX0);
      copy(V_XPREV, V_X0);
      s[ST_DELTA] = s[ST_DELTA0];
    }
    if (!exitflag) return inner_step_begin();
    // outer_step tail: RIPTRM.py:889-896
    s[ST_MU_IDX] += 1.0;
    s[ST_MU] = mu_at((int)s[ST_MU_IDX]);
    const double mn = P.opt.minimal_initial_tr_radius;
    s[ST_DELTA] = s[ST_DELTA] > mn ? s[ST_DELTA] : mn;
    return outer_top();
  }

  __device__ __forceinline__ int dispatch() {
    switch ((int)s[ST_PHASE]) {
      case PH_START:
        copy(V_IN0, V_X);
        s[ST_PHASE] = PH_AFTER_SX0;
        return request(1);
      case PH_AFTER_SX0:
        copy(V_SX, V_OUT0);
        s[ST_T_START] = unow();
        copy(V_X0, V_X);
        copy(V_XI, V_X);
        copy(V_YI, V_Y);
        copy(V_SXI, V_SX);
        return outer_top();
      case PH_TCG:
        return tcg_step();
      case PH_TRIAL:
        return trial_eval();
      case PH_PAUSED:
        return start_outer_step();
      case PH_TCGO_START:
        copy(V_IN0, V_X);
        s[ST_PHASE] = PH_TCGO_SX;
        return request(1);
      case PH_TCGO_SX:
        copy(V_SX, V_OUT0);
        return tcg_begin();
      case PH_TRS:
        if constexpr (EXACT) return trs_direction();
        return ACT_DONE;
      case PH_TRS_END:
        return tcg_end();
      case PH_MINEIG_END:   // the host wrote s[ST_MINEIG] (riptrm_trs_big.hip); NaN: dsyevd failed
        if (!isfinite(s[ST_MINEIG])) return nonfinite_stop(true, RIPTRM_ERR_EIGEN);
        mineig_test();
        return tcg_end_tail();
      default:
        return ACT_DONE;
    }
  }
};
using Machine = MachineT<false>;

// full = 1: workgroup k serves instance full_base + k (k < full_count); else workgroup k
// serves lists[list_in][k].  List ids are group * 2 + parity (two independent instance groups).
template <bool EXACT>
__global__ void __launch_bounds__(ST_THREADS) k_state(DevParams P, int full, int list_in, int list_out,
                                                      int full_base, int full_count) {
  __shared__ double redbuf[2 * ST_WAVES * RED_MAX];
  extern __shared__ double trs_lds[];   // Exact_RepMat only (dynamic size 0 otherwise)
  int b;
  // full = 1: (re)start launch; full = 2: direct lock-step launch, workgroup k = instance
  // full_base + k, active iff it waits for the S-pass that just ran (its phase says so: every
  // instance in that state was queued by request()); full = 0: workgroup k = lists[list_in][k]
  if (full == 1) {
    if ((int)blockIdx.x >= full_count) return;
    b = full_base + blockIdx.x;
    if (b >= P.batch) return;
    // a full launch (solve start / resume) only (re)starts instances that wait for no S-pass
    const double* g = P.st + (int64_t)b * ST_N;
    const int ph = (int)g[ST_PHASE];
    const bool startable = ph == PH_START || ph == PH_TCGO_START || ph == PH_TRS_END || ph == PH_MINEIG_END ||
                           (ph == PH_PAUSED && (double)P.outer_target > g[ST_OUTER_IT]);
    if (!startable) return;
  } else if (full == 2) {
    if ((int)blockIdx.x >= full_count) return;
    b = full_base + blockIdx.x;
    if (b >= P.batch) return;
  } else {
    const int nact = P.cnt[list_in];
    const int32_t e = P.lists[list_in * P.batch + blockIdx.x];
    if ((int)blockIdx.x >= nact) return;
    b = le_b(e);
  }
  MachineT<EXACT> M(P, b, list_out, redbuf, trs_lds);
  const int ph = (int)M.s[ST_PHASE];
  if (ph == PH_DONE || ph == PH_IDLE || ph == PH_ERROR) return;
  if (full == 2 && !(ph == PH_TCG || ph == PH_TRIAL || ph == PH_AFTER_SX0 || ph == PH_TCGO_SX)) return;
  if (full != 1 && ph == PH_TCG && P.n <= Machine::RT_EPT * ST_THREADS) {
    // gathers S delta itself, vectors register-resident (2 elements per thread up to n = 1024)
    if (P.n <= 2 * ST_THREADS) M.template tcg_step_reg<2>();
    else M.template tcg_step_reg<Machine::RT_EPT>();
  } else {
    if (full != 1 && P.layout == RIPTRM_LAYOUT_SYMTILE) M.gather_out(P.req[b]);
    if (full != 1 && P.layout == RIPTRM_LAYOUT_SHARED) M.gather_slices(P.req[b]);
    if constexpr (EXACT) {
      while (M.dispatch() == ACT_CONTINUE) {
      }
    } else {
      M.dispatch();
    }
  }
  M.finish_write();
}

// ------------------------------------------------------------------------------------------
// k_persist: the lock-step loop of a small symmetric-tile batch (tCG) in ONE launch.
// Why: at n = 1000 with one instance (BASELINE configs[1]) a lock-step iteration is a 5 us
// S-pass plus a 12.5 us state kernel, latency and launch bound (profiles/r1_cfg1_*).  Here every
// stored tile of every instance gets one 512-thread workgroup that keeps the tile in LDS for the
// whole launch (S is read from HBM once per launch, not once per pass), and every workgroup of an
// instance runs a private REPLICA of the instance's state machine on identical data: the
// replicas take bitwise identical decisions (same code, same operands, same reduction orders; the
// clock comes from the barrier, below), so no state is ever exchanged.  Per pass each workgroup
// multiplies its tile by its own replica's S-pass vectors (spass_tile's arithmetic, operands from
// LDS) into the instance's partial grid, with write-through (sc1) stores; one arrival counter per
// instance (agent-scope atomic add after every wave drained its stores, sc1 polling) is the only
// synchronisation, and every replica then gathers the grid (sc1 loads) exactly as k_state does.
// Results are bitwise those of the lock-step path (k_spass_sym + k_state), which stays the
// general path.  The partial grid and the published clock alternate between two buffers by pass
// parity, so a fast replica never overwrites what a slow one still reads.  Every spin is bounded.
// Replica 0 of instance b is the instance itself (P); replica t > 0 is slot b (reps - 1) + t - 1
// of the replica block Q.
// ------------------------------------------------------------------------------------------
struct PersistSync {
  unsigned int* ctr;    // [batch] arrivals, zeroed before every launch
  double* clk;          // [2][batch] clock published by replica 0 at each barrier (parity)
  unsigned int* flag;   // [0]: some barrier wait timed out
  double* pbuf2;        // the partial grid's second parity
  double* tgrid;        // the tagged grid of lean passes (zeroed before every launch)
  int tgrid_bytes;
  unsigned long long* trace;   // diagnostics (riptrm_persist_trace): per step of workgroups 0 and
  int trace_cap;               // reps - 1, the device clock at the step's start / tile pass done /
                               // barrier passed / state step done; nullptr = off
};
constexpr unsigned long long PERSIST_TIMEOUT_TICKS = 200000000ull;   // 2 s of the 100 MHz clock

// ---- tagged partial sums (lean tCG passes of k_persist) ---------------------------------------
// A lean pass exchanges its partial sums as 16-byte granules {value, tag} written by ONE 16-B
// write-through store each: the data are their own flag, so the pass needs neither an arrival
// counter nor a separate gather round trip (every consumer polls exactly the granules it sums).
// tag = (pass << 32) | (lo ^ hi ^ pass * 0x9E3779B9): the pass index (unique within a launch; the
// grid is zeroed before every launch) and a check of the value bits, so a granule read half old /
// half new is never accepted.  The grid alternates between two parities by pass, as the plain one.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ unsigned tag_check(unsigned lo, unsigned hi, unsigned pass) {
  return lo ^ hi ^ (pass * 0x9E3779B9u);
}
struct TagOut {
  __amdgpu_buffer_rsrc_t rsrc;   // the tagged grid (both parities)
  int base;                      // granule index of this pass's parity and instance, rhs 0
  unsigned pass;                 // tag of this pass (>= 1)
};
__device__ __forceinline__ void st_tag(const TagOut& to, int g, double v) {
  const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
  const u32x4 q = {lo, hi, tag_check(lo, hi, to.pass), to.pass};
  __builtin_amdgcn_raw_buffer_store_b128(q, to.rsrc, (to.base + g) * 16, 0, 16);   // aux 16 = sc1
}

// spass_tile with the tile in LDS (row stride colsT) and the input vectors' two blocks it needs
// staged in LDS (vl[rhs][0] = block I, vl[rhs][1] = block J); the partial sums go to the
// instance's slot bp of the grid pbase with sc1 stores
// (to != nullptr: tagged granules instead, one right-hand side)
template <int NR>
__device__ __forceinline__ void spass_tile_lds(const DevParams& P, const double* Tl, const double (*vl)[2][TS],
                                               double* pbase, int bp, int t, double (*csl)[SP_WAVES][TS],
                                               unsigned long long* tr = nullptr, const TagOut* to = nullptr) {
  int I, J;
  tile_ij(t, P.nt, I, J);
  const int lane = (int)__lane_id();
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nt = P.nt, wl = P.wl;
  const int rowsT = (I == nt - 1) ? wl : TS;
  const int colsT = (J == nt - 1) ? wl : TS;
  const bool cl = 2 * lane < colsT;
  const dbl2 vj0 = *(const dbl2*)(&vl[0][1][2 * lane]);
  dbl2 vj1 = dbl2{0.0, 0.0};
  if (NR == 2) vj1 = *(const dbl2*)(&vl[1][1][2 * lane]);
  const int64_t nn = (int64_t)P.nt * P.nt * TS;
  double* pb0 = pbase + (int64_t)bp * nn;
  double* pb1 = pbase + ((int64_t)P.pbatch + bp) * nn;
  double c0x = 0.0, c0y = 0.0, c1x = 0.0, c1y = 0.0;
  const int rrow = 4 * ((lane >> 5) & 1) + 2 * ((lane >> 4) & 1) + ((lane >> 3) & 1);
  constexpr int ROWS = TS / SP_WAVES;
  static_assert(ST_THREADS == SP_THREADS, "k_persist: one state workgroup = one tile workgroup");
  // the row sums of both 8-row batches are stored after the loop: on gfx950 loads and stores share
  // one counter, so any load wait after a write-through store would wait for its round trip
  double rs[2][2] = {{0.0, 0.0}, {0.0, 0.0}};
  bool rv[2] = {false, false};
#pragma unroll
  for (int rb = 0; rb < ROWS / 8; ++rb) {
    const int r0 = w * ROWS + rb * 8;
    if (r0 >= rowsT) break;
    dbl2 sv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) sv[k] = cl ? *(const dbl2*)(Tl + (r0 + k) * colsT + 2 * lane) : dbl2{0.0, 0.0};
    double a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const double vi0 = vl[0][0][r0 + k];
      a[k] = __builtin_fma(sv[k].y, vj0.y, sv[k].x * vj0.x);
      c0x = __builtin_fma(sv[k].x, vi0, c0x);
      c0y = __builtin_fma(sv[k].y, vi0, c0y);
    }
    rs[rb][0] = reduce_scatter8(a);
    rv[rb] = true;
    if (NR == 2) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const double vi1 = vl[1][0][r0 + k];
        a[k] = __builtin_fma(sv[k].y, vj1.y, sv[k].x * vj1.x);
        c1x = __builtin_fma(sv[k].x, vi1, c1x);
        c1y = __builtin_fma(sv[k].y, vi1, c1y);
      }
      rs[rb][1] = reduce_scatter8(a);
    }
  }
  if ((lane & 7) == 0) {
#pragma unroll
    for (int rb = 0; rb < ROWS / 8; ++rb) {
      if (!rv[rb]) continue;
      const int r0 = w * ROWS + rb * 8;
      if (to) st_tag(*to, (I * P.nt + J) * TS + r0 + rrow, rs[rb][0]);
      else st_sc1(pb0 + ((int64_t)I * P.nt + J) * TS + r0 + rrow, rs[rb][0]);
      if (NR == 2) st_sc1(pb1 + ((int64_t)I * P.nt + J) * TS + r0 + rrow, rs[rb][1]);
    }
  }
  if (tr) tr[16] = wall_clock64();   // wave 0's rows done
  if (I != J) {   // csl: LDS [2][SP_WAVES][TS], the column sums across waves
    csl[0][w][2 * lane] = c0x;
    csl[0][w][2 * lane + 1] = c0y;
    if (NR == 2) {
      csl[1][w][2 * lane] = c1x;
      csl[1][w][2 * lane + 1] = c1y;
    }
    __syncthreads();
    if (tr) tr[17] = wall_clock64();   // every wave's rows done
    if (threadIdx.x < TS) {
      const int c = threadIdx.x;
      double s0 = csl[0][0][c];
#pragma unroll
      for (int q = 1; q < SP_WAVES; ++q) s0 += csl[0][q][c];
      if (to) st_tag(*to, (J * P.nt + I) * TS + c, s0);
      else st_sc1(pb0 + ((int64_t)J * P.nt + I) * TS + c, s0);
      if (NR == 2) {
        double s1 = csl[1][0][c];
#pragma unroll
        for (int q = 1; q < SP_WAVES; ++q) s1 += csl[1][q][c];
        st_sc1(pb1 + ((int64_t)J * P.nt + I) * TS + c, s1);
      }
    }
    __syncthreads();   // csl is rewritten by the next pass
  }
}

// Arrival of workgroup (b, replica) at in-launch barrier `epoch` (1, 2, ...) of instance b: every
// wave drains its sc1 stores, one lane publishes (replica 0: the clock) and adds to the counter,
// then polls it (relaxed sc1 loads, bounded) until all `reps` workgroups of the instance arrived.
// Returns false on a timeout (then the caller stops; the flag tells the host).
__device__ __forceinline__ bool persist_barrier(const PersistSync& sy, int batch, int b, int reps, bool rep0,
                                                unsigned epoch, double& clk, double* bclk, int* bfail) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    double* cslot = sy.clk + (int64_t)(epoch & 1u) * batch + b;
    gu32_t* ctr = (gu32_t*)(sy.ctr + b);
    if (rep0) {
      st_sc1(cslot, (double)wall_clock64());
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned target = epoch * (unsigned)reps;
    const unsigned long long t0 = wall_clock64();
    int fail = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (wall_clock64() - t0 > PERSIST_TIMEOUT_TICKS) {
        fail = 1;
        break;
      }
    }
    if (fail) __hip_atomic_store((gu32_t*)sy.flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *bclk = fail ? 0.0 : ld_sc1(cslot);
    *bfail = fail;
  }
  __syncthreads();
  clk = *bclk;
  return *bfail == 0;
}

using riptrm_trs::lds_f64;

// What a lean tCG run reads (by value: one copy at the call, then registers).
struct LeanArgs {
  double* vk;          // the replica's vector kind 0 (kind k at vk + k vks)
  int64_t vks;
  double* gcold;       // the replica's scalar slots (ST_PASSES)
  double* pb[2];       // the instance's partial grid, both parities
  double* tg;          // the tagged grid [2 parities][batch][nt][nt][TS] of 16-B granules
  int tg_bytes;
  PersistSync sy;
  int n, b, t, R, I, J, steps, batch;
  int rep0, tsel;
  double kappa, theta;
  int mininner, pbatch, nt, wl;
};
// In / out of a lean run: the next pass index, barrier epoch, published clock, barrier ok, stop code.
struct LeanIO {
  int k;
  unsigned epoch;
  double clk;
  int ok;
  int stop;
};

// A lean tCG run of a k_persist replica: passes of S delta (the instance's tiles multiply the
// direction staged in LDS, the barrier, the partial sums gathered with sc1 loads) and tcg_math on
// register-resident vectors and scalars, until the run stops or the step budget ends; then the
// vectors go back to the workspace, the scalars to the LDS copy `hot`, the passes to ST_PASSES.
// Not inlined: its operands stay in registers (inside the kernel body, next to the inlined state
// machine, the register allocator kept them in scratch and every reload waited on memory).  LDS
// operands come in as address-space-3 pointers, so every access stays a ds_* instruction.
template <int K>
__device__ __noinline__ void lean_tcg_run(LeanArgs a, LeanIO* io, const lds_f64* tile, lds_f64* vl_, lds_f64* csl_,
                                          lds_f64* red_, lds_f64* hot, lds_f64* bclk, int* bfail) {
  const int n = a.n, tid = threadIdx.x;
  double (*vl)[2][TS] = (double (*)[2][TS])(double*)vl_;
  double (*csl)[SP_WAVES][TS] = (double (*)[SP_WAVES][TS])(double*)csl_;
  DevParams Pt;   // the fields spass_tile_lds reads
  Pt.nt = a.nt;
  Pt.wl = a.wl;
  Pt.pbatch = a.pbatch;
  Pt.n = n;
  Pt.smode = 0;
  Pt.layout = RIPTRM_LAYOUT_SYMTILE;
  Pt.nst = 0;
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(a.tg, 0, a.tg_bytes, 0x00020000);
  typename MachineT<false, true>::template TcgVecs<K> tv;
  rl_load<K>(a.vk + V_IN0 * a.vks, n, tv.d);
  rl_load<K>(a.vk + V_X * a.vks, n, tv.x);
  rl_load<K>(a.vk + V_Y * a.vks, n, tv.y);
  rl_load<K>(a.vk + V_C * a.vks, n, tv.c);
  rl_load<K>(a.vk + V_ETA * a.vks, n, tv.e);
  rl_load<K>(a.vk + V_HETA * a.vks, n, tv.he);
  rl_load<K>(a.vk + V_R * a.vks, n, tv.rv);
  TcgScalars ts;
  ts.coef = hot[ST_COEF];
  ts.z_r = hot[ST_ZR];
  ts.e_Pd = hot[ST_EPD];
  ts.d_Pd = hot[ST_DPD];
  ts.e_Pe = hot[ST_EPE];
  ts.Delta = hot[ST_DELTA];
  ts.model = hot[ST_MODEL];
  ts.nr0 = hot[ST_NORMR0];
  ts.j = hot[ST_J];
  ts.nr0t = pow(ts.nr0, a.theta);
  riptrm_options opt;
  opt.tcg_kappa = a.kappa;
  opt.tcg_mininner = a.mininner;
  int k = io->k;
  unsigned epoch = io->epoch;
  double clk = io->clk;
  int ok = 1;
  double passes = 0.0;
  int stop = TCG_CONTINUE;
  while (true) {
#pragma unroll
    for (int q = 0; q < K; ++q) {   // the direction's blocks I and J
      const int i = tid + q * ST_THREADS;
      const double dv = i < n ? tv.d[q] : 0.0;
      if (i / TS == a.I) vl[0][0][i - a.I * TS] = dv;
      if (i / TS == a.J) vl[0][1][i - a.J * TS] = dv;
    }
    __syncthreads();
    unsigned long long* tr = (a.sy.trace && a.tsel >= 0 && k < a.sy.trace_cap && tid == 0)
                                 ? a.sy.trace + ((int64_t)a.tsel * a.sy.trace_cap + k) * 24 : nullptr;
    if (tr) tr[0] = wall_clock64();
    const int nn = a.nt * a.nt * TS;
    TagOut to;
    to.rsrc = rsrc;
    to.base = ((k & 1) * a.batch + a.b) * nn;
    to.pass = (unsigned)k + 1u;
    spass_tile_lds<1>(Pt, (const double*)tile, vl, nullptr, a.b, a.t, csl, tr, &to);
    if (tr) tr[1] = wall_clock64();
    Red Rd;
    Rd.buf = (double*)red_;
    Rd.parity = 0;
    HwPre<K> pre;   // while the granules travel
    tcg_math_pre<K>(pre, n, Rd, tv.d, tv.x, tv.y);
    // gather = poll: each thread's granules of its K elements (the same summation order as
    // rl_gather), re-read until every tag says this pass; bounded
    double u[K];
    {
      constexpr int NTS = K <= 2 ? 8 : 16;
      double tv_[K][NTS];
      int gi[K];
#pragma unroll
      for (int e = 0; e < K; ++e) {
        int i = tid + e * ST_THREADS;
        i = i < n ? i : n - 1;
        const int Ib = i >> 7, c = i & (TS - 1);
        gi[e] = to.base + Ib * a.nt * TS + c;
      }
      unsigned long long pend = 0;
#pragma unroll
      for (int e = 0; e < K; ++e)
#pragma unroll
        for (int J = 0; J < NTS; ++J)
          if (J < a.nt) pend |= 1ull << (e * NTS + J);
      const unsigned long long t0 = wall_clock64();
      while (true) {
        u32x4 q[K][NTS];
#pragma unroll
        for (int e = 0; e < K; ++e)
#pragma unroll
          for (int J = 0; J < NTS; ++J)
            if (pend & (1ull << (e * NTS + J)))
              q[e][J] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (gi[e] + J * TS) * 16, 0, 16);
#pragma unroll
        for (int e = 0; e < K; ++e)
#pragma unroll
          for (int J = 0; J < NTS; ++J)
            if (pend & (1ull << (e * NTS + J))) {
              const u32x4 g = q[e][J];
              if (g.w == to.pass && g.z == tag_check(g.x, g.y, to.pass)) {
                tv_[e][J] = __hiloint2double((int)g.y, (int)g.x);
                pend &= ~(1ull << (e * NTS + J));
              }
            }
        if (!__any(pend != 0)) break;
        if (wall_clock64() - t0 > PERSIST_TIMEOUT_TICKS) {
          if (pend) __hip_atomic_store((gu32_t*)a.sy.flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      ok = __syncthreads_and(ok);
      if (!ok) break;
#pragma unroll
      for (int e = 0; e < K; ++e) {
        u[e] = tv_[e][0];
#pragma unroll
        for (int J = 1; J < NTS; ++J)
          if (J < a.nt) u[e] += tv_[e][J];
        if (tid + e * ST_THREADS >= n) u[e] = 0.0;
      }
    }
    if (tr) tr[4] = tr[2] = wall_clock64();
    ++k;
    struct NoHooks {   // nothing to load or store; optional trace stamps (diagnostics)
      unsigned long long* tr;
      __device__ __forceinline__ void late_ceh() {}
      __device__ __forceinline__ void late_r() {}
      __device__ __forceinline__ void store_eh() {}
      __device__ __forceinline__ void store_ehr() {}
      __device__ __forceinline__ void store_d() {}
      __device__ __forceinline__ void stamp(int i) {
        if (tr) tr[8 + i] = wall_clock64();
      }
    } nohooks{tr};
    stop = tcg_math<K>(ts, opt, n, Rd, u, tv.d, tv.x, tv.y, tv.c, tv.e, tv.he, tv.rv, nohooks, pre);
    if (tr) {
      tr[5] = wall_clock64();
      tr[3] = wall_clock64();
    }
    if (stop != TCG_CONTINUE) break;
    passes += 1.0;   // request(1) of the same run
    if (k >= a.steps) break;
  }
  // flush: vectors to the workspace, scalars to LDS, the requested passes to ST_PASSES
  rl_store<K>(a.vk + V_IN0 * a.vks, n, tv.d);
  rl_store<K>(a.vk + V_ETA * a.vks, n, tv.e);
  rl_store<K>(a.vk + V_HETA * a.vks, n, tv.he);
  rl_store<K>(a.vk + V_R * a.vks, n, tv.rv);
  __syncthreads();
  if (tid == 0) {
    hot[ST_ZR] = ts.z_r;
    hot[ST_EPD] = ts.e_Pd;
    hot[ST_DPD] = ts.d_Pd;
    hot[ST_EPE] = ts.e_Pe;
    hot[ST_MODEL] = ts.model;
    hot[ST_J] = ts.j;
    if (stop != TCG_CONTINUE) hot[ST_TCG_STOP] = stop;
    a.gcold[ST_PASSES] += passes;
    a.gcold[ST_RHS] += passes;   // lean passes carry one right-hand side
    io->k = k;
    io->epoch = epoch;
    io->clk = clk;
    io->ok = ok;
    io->stop = stop;
  }
  __syncthreads();
}

// K: elements per thread of the register-resident tCG iterations (n <= K ST_THREADS; 2 or 4)
// P: the instances' parameters; rq: the replicas' slots (replica t > 0 of instance b is slot
// b (reps - 1) + t - 1)
template <int K>
__global__ void __launch_bounds__(ST_THREADS) k_persist(DevParams P, RepBlock rq, PersistSync sy, int steps) {
  extern __shared__ double tile_lds[];   // TS x TS doubles (the stored tile)
  __shared__ double redbuf[2 * ST_WAVES * RED_MAX];
  __shared__ double csl[2][SP_WAVES][TS];
  __shared__ double vl[2][2][TS];        // the pass inputs' blocks I and J (per right-hand side)
  __shared__ double hot[ST_HOT];         // the replica's hot scalars between steps
  __shared__ double bclk;
  __shared__ int bfail, bnr, bact;
  __shared__ LeanIO lio;
  const int R = P.ntiles;
  const int b = blockIdx.x / R, t = blockIdx.x - b * R;
  if (b >= P.batch || steps <= 0) return;
  const bool rep0 = t == 0;
  const int bm = rep0 ? b : b * (R - 1) + (t - 1);   // the replica's slot in its parameter block
  double* const gst = (rep0 ? P.st : rq.st) + (int64_t)bm * ST_N;
  // every replica of an instance sees the same phase, so these exits are uniform per instance
  const int ph0 = (int)gst[ST_PHASE];
  const bool waiting = ph0 == PH_TCG || ph0 == PH_TRIAL || ph0 == PH_AFTER_SX0 || ph0 == PH_TCGO_SX;
  const bool startable = ph0 == PH_START || ph0 == PH_TCGO_START ||
                         (ph0 == PH_PAUSED && (double)P.outer_target > gst[ST_OUTER_IT]);
  if (!waiting && !startable) return;
  if (threadIdx.x < ST_HOT) hot[threadIdx.x] = gst[threadIdx.x];
  if (threadIdx.x == 0) {
    bnr = (rep0 ? P.req : rq.req)[bm];   // the pass the previous launch left pending (if waiting)
    bact = ACT_YIELD;
  }
  int I, J;
  tile_ij(t, P.nt, I, J);
  {  // the tile, once per launch
    const int rowsT = (I == P.nt - 1) ? P.wl : TS;
    const int colsT = (J == P.nt - 1) ? P.wl : TS;
    const double* T = P.S + (int64_t)b * P.inst_stride + sym_off(I, J, P.nt, P.wl);
    for (int i = 2 * (int)threadIdx.x; i < rowsT * colsT; i += 2 * ST_THREADS)
      *(dbl2*)(tile_lds + i) = __builtin_nontemporal_load((const dbl2*)(T + i));
  }
  double* const vbm = (rep0 ? P.vec : rq.vec) + (int64_t)bm * P.ld;
  const int64_t vks = (int64_t)(rep0 ? P.batch : rq.batch) * P.ld;
  double* const pb0 = P.pbuf;
  double* const pb1 = sy.pbuf2;
  const int tsel = blockIdx.x == 0 ? 0 : ((int)blockIdx.x == R - 1 ? 1 : -1);
  unsigned epoch = 1;
  double clk = 0.0;
  bool ok = persist_barrier(sy, P.batch, b, R, rep0, epoch++, clk, &bclk, &bfail);   // uniform start clock
  // Step k >= 0 = S-pass k, then the state machine until its next request; tCG iterations run as
  // lean runs (lean_tcg_run, not inlined: vectors and scalars in registers across iterations,
  // tcg_math = the function k_state's tcg_step_reg runs, bitwise identical); every other step
  // builds the machine from the LDS copy of its hot scalars, runs it inline, and writes them back.
  int k = startable ? -1 : 0;
  while (ok && bact == ACT_YIELD && k < steps) {
    int stop = TCG_CONTINUE;
    if (k >= 0 && (int)hot[ST_PHASE] == PH_TCG && P.n <= K * ST_THREADS) {
      LeanArgs la;
      la.vk = vbm;
      la.vks = vks;
      la.gcold = gst;
      la.pb[0] = pb0;
      la.pb[1] = pb1;
      la.tg = sy.tgrid;
      la.tg_bytes = sy.tgrid_bytes;
      la.sy = sy;
      la.n = P.n;
      la.b = b;
      la.t = t;
      la.R = R;
      la.I = I;
      la.J = J;
      la.steps = steps;
      la.batch = P.batch;
      la.rep0 = rep0 ? 1 : 0;
      la.tsel = tsel;
      la.kappa = P.opt.tcg_kappa;
      la.theta = P.opt.tcg_theta;
      la.mininner = P.opt.tcg_mininner;
      la.pbatch = P.pbatch;
      la.nt = P.nt;
      la.wl = P.wl;
      if (threadIdx.x == 0) {
        lio.k = k;
        lio.epoch = epoch;
        lio.clk = clk;
      }
      __syncthreads();
      lean_tcg_run<K>(la, &lio, (const lds_f64*)tile_lds, (lds_f64*)&vl[0][0][0], (lds_f64*)&csl[0][0][0],
                      (lds_f64*)redbuf, (lds_f64*)hot, (lds_f64*)&bclk, &bfail);
      k = lio.k;
      epoch = lio.epoch;
      clk = lio.clk;
      ok = lio.ok != 0;
      stop = lio.stop;
      if (!ok || stop == TCG_CONTINUE) continue;   // barrier failure, or the budget ended mid-run
    } else if (k >= 0) {
      // one pass of the machine's request: blocks I and J of its inputs, one load round trip
      const int q = threadIdx.x >> 7, e = threadIdx.x & (TS - 1);   // q: rhs * 2 + block
      if (q < 2 * bnr) vl[q >> 1][q & 1][e] = vbm[(q >> 1 ? V_IN1 : V_IN0) * vks + ((q & 1) ? J : I) * TS + e];
      __syncthreads();
      unsigned long long* tr = (sy.trace && tsel >= 0 && k < sy.trace_cap && threadIdx.x == 0)
                                   ? sy.trace + ((int64_t)tsel * sy.trace_cap + k) * 24 : nullptr;
      if (tr) tr[0] = wall_clock64();
      if (bnr == 2) spass_tile_lds<2>(P, tile_lds, vl, (k & 1) ? pb1 : pb0, b, t, csl);
      else spass_tile_lds<1>(P, tile_lds, vl, (k & 1) ? pb1 : pb0, b, t, csl);
      if (tr) tr[1] = wall_clock64();
      ok = persist_barrier(sy, P.batch, b, R, rep0, epoch++, clk, &bclk, &bfail);
      if (!ok) break;
      if (tr) tr[2] = wall_clock64();
    }
    // the machine: (re)start (k = -1), after a pass, or after a lean run stopped (then tcg_end)
    MachineT<false, true> M(P, bm, 0, redbuf, nullptr, hot, !rep0, rq);
    M.bp = b;
    M.uclk = clk;
    const int kp = k >= 0 ? k : 0;
    M.pb = ((stop != TCG_CONTINUE ? kp - 1 : kp) & 1) ? pb1 : pb0;
    int act;
    if (stop != TCG_CONTINUE) {   // a lean run stopped: the rest of compute_direction + the trial point
      act = M.tcg_end();
    } else {   // one dispatch call site (as in k_state): the machine is inlined once
      if (k >= 0) M.gather_out(bnr);
      act = M.dispatch();
      ++k;
    }
    __syncthreads();   // every thread has read hot / bnr
    if (threadIdx.x == 0) {   // static indices: s[] stays in registers
#pragma unroll
      for (int q = 0; q < ST_HOT; ++q) hot[q] = M.s[q];
      bnr = M.last_nr;
      bact = act;
    }
    if (act != ACT_YIELD) M.finish_write();
    __syncthreads();
  }
  if (ok && bact != ACT_YIELD) return;   // finished or paused: finish_write done in the step
  // still waiting for an S-pass (step budget used up) or a peer never arrived: write the scalars back
  MachineT<false, true> M(P, bm, 0, redbuf, nullptr, hot, !rep0, rq);
  if (!ok) {   // the instance stops with an error (the host reports it)
    M.s[ST_PHASE] = PH_ERROR;
    M.cset(ST_ERROR, (double)RIPTRM_ERR_BARRIER_TIMEOUT);
  }
  M.finish_write();
}

// instances of the batch still running after a persistent launch (waiting for an S-pass, or
// startable): the count the lock-step path keeps in its active list
__global__ void __launch_bounds__(256) k_persist_count(DevParams P, int list) {
  __shared__ int c;
  if (threadIdx.x == 0) c = 0;
  __syncthreads();
  for (int b = threadIdx.x; b < P.batch; b += blockDim.x) {
    const double* g = P.st + (int64_t)b * ST_N;
    const int ph = (int)g[ST_PHASE];
    const bool run = ph == PH_TCG || ph == PH_TRIAL || ph == PH_AFTER_SX0 || ph == PH_TCGO_SX || ph == PH_START ||
                     ph == PH_TCGO_START || (ph == PH_PAUSED && (double)P.outer_target > g[ST_OUTER_IT]);
    if (run) atomicAdd(&c, 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) P.cnt[list] = c;
}

// riptrm_log_rebase: every record logged so far counts as drained
__global__ void __launch_bounds__(256) k_log_rebase(DevParams P) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= P.batch) return;
  double* c = P.st + (int64_t)b * ST_N;
  c[ST_LOG_BASE] = c[ST_LOG_COUNT];
  P.stats[(int64_t)b * RIPTRM_STAT_NFIELDS + RIPTRM_STAT_LOG_BASE] = c[ST_LOG_COUNT];
}

// initialise a solve: x0/y0 -> X/Y, scalars
// rep_div > 1: P is the persistent replicas' block (batch x (reps - 1) slots), slot b replicates
// instance b / rep_div of the caller's arrays
__global__ void __launch_bounds__(256) k_init(DevParams P, const double* x0, const double* y0, int64_t ldv,
                                              const double* mu, const double* delta, int mode, int rep_div) {
  const int b = blockIdx.x;
  const int src = b / rep_div;
  double* X = vp(P, V_X, b);
  double* Y = vp(P, V_Y, b);
  for (int i = threadIdx.x; i < P.n; i += blockDim.x) {
    X[i] = x0[(int64_t)src * ldv + i];
    Y[i] = y0[(int64_t)src * ldv + i];
  }
  if (threadIdx.x == 0) {
    double* s = P.st + (int64_t)b * ST_N;
    for (int k = 0; k < ST_N; ++k) s[k] = 0.0;
    s[ST_MODE] = mode;
    if (mode == MODE_SOLVE) {
      s[ST_PHASE] = PH_START;
      s[ST_MU] = P.mu_tab[0];
      s[ST_DELTA] = P.opt.initial_tr_radius;
    } else {
      s[ST_PHASE] = PH_TCGO_START;
      s[ST_MU] = mu[src];
      s[ST_DELTA] = delta[src];
    }
    s[ST_I_DC] = -1.0;
    s[ST_T_START] = (double)wall_clock64();
  }
}

// HVP entry: copy x, y, v into the workspace and queue all instances for a 2-RHS pass
__global__ void __launch_bounds__(256) k_hvp_prep(DevParams P, const double* x, const double* y, const double* v, int64_t ldv) {
  const int b = blockIdx.x;
  double* X = vp(P, V_X, b);
  double* Y = vp(P, V_Y, b);
  double* I0 = vp(P, V_IN0, b);
  double* I1 = vp(P, V_IN1, b);
  for (int i = threadIdx.x; i < P.n; i += blockDim.x) {
    X[i] = x[(int64_t)b * ldv + i];
    Y[i] = y[(int64_t)b * ldv + i];
    I0[i] = v[(int64_t)b * ldv + i];
    I1[i] = X[i];
  }
  if (threadIdx.x == 0) {
    P.req[b] = 2;
    P.lists[b] = le_make(b, 2);
    if (b == 0) P.cnt[0] = P.batch;
  }
}

__global__ void __launch_bounds__(ST_THREADS) k_hvp_epi(DevParams P, double mu, double* out, int64_t ldv) {
  __shared__ double redbuf[2 * ST_WAVES * RED_MAX];
  const int b = blockIdx.x;
  Machine M(P, b, 0, redbuf);
  if (P.layout == RIPTRM_LAYOUT_SYMTILE) M.gather_out(2);
  if (P.layout == RIPTRM_LAYOUT_SHARED) M.gather_slices(2);
  const double* X = M.V(V_X);
  const double* Y = M.V(V_Y);
  const double* SX = M.V(V_OUT1);
  double h[3] = {0.0, 0.0, 0.0};
  for (int i = threadIdx.x; i < P.n; i += ST_THREADS) {
    h[0] += X[i] * X[i];
    h[1] += X[i] * SX[i];
    h[2] += Y[i] * X[i];
  }
  bsum<3>(M.R, h);
  M.s[ST_COEF] = (h[1] + h[2]) * h[0];
  (void)mu;
  double* U = M.V(V_OUT0);
  M.hw_apply(U, M.V(V_IN0), U);
  for (int i = threadIdx.x; i < P.n; i += ST_THREADS) out[(int64_t)b * ldv + i] = U[i];
}

// RIPM's condensed Newton operator (src/solver/RIPM.py:485-487) after an HVP-style 2-RHS pass
// (k_hvp_prep with y := z):  Aw(v) = P_x(-Sv) + (x^T S x + z^T x)(x^T x) v + P_x(w (v - x x^T v)),
// w = z / s — HwCur's structure with RIPM's multipliers z and separate slacks s.
__global__ void __launch_bounds__(ST_THREADS) k_aw_epi(DevParams P, const double* sl, double* out, int64_t ldv) {
  __shared__ double redbuf[2 * ST_WAVES * RED_MAX];
  const int b = blockIdx.x;
  Machine M(P, b, 0, redbuf);
  if (P.layout == RIPTRM_LAYOUT_SYMTILE) M.gather_out(2);
  if (P.layout == RIPTRM_LAYOUT_SHARED) M.gather_slices(2);
  const int n = P.n;
  const double* X = M.V(V_X);
  const double* Zm = M.V(V_Y);
  const double* SX = M.V(V_OUT1);
  const double* U = M.V(V_OUT0);
  const double* Vv = M.V(V_IN0);
  const double* Sl = sl + (int64_t)b * ldv;
  double h[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
  for (int i = threadIdx.x; i < n; i += ST_THREADS) {
    h[0] += X[i] * X[i];
    h[1] += X[i] * SX[i];
    h[2] += Zm[i] * X[i];
    h[3] += X[i] * U[i];
    h[4] += X[i] * Vv[i];
  }
  bsum<5>(M.R, h);
  const double coef = (h[1] + h[2]) * h[0];
  const double xu = h[3], xv = h[4];
  double r2[1] = {0.0};
  for (int i = threadIdx.x; i < n; i += ST_THREADS) {
    const double q = (Vv[i] - X[i] * xv) * (Zm[i] / Sl[i]);
    r2[0] += X[i] * q;
  }
  bsum<1>(M.R, r2);
  const double xq = r2[0];
  for (int i = threadIdx.x; i < n; i += ST_THREADS) {
    const double q = (Vv[i] - X[i] * xv) * (Zm[i] / Sl[i]);
    out[(int64_t)b * ldv + i] = ((-U[i] + xu * X[i]) + coef * Vv[i]) + (q - xq * X[i]);
  }
}

}  // namespace riptrm

// ==========================================================================================
// C-ABI
// ==========================================================================================
using namespace riptrm;

static hipEvent_t prof_event(riptrm_ctx* c, int* idx) {
  if (c->ev_used == (int)c->ev_pool.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    c->ev_pool.push_back(e);
  }
  *idx = c->ev_used;
  return c->ev_pool[c->ev_used++];
}

// after a stream sync: fold the recorded pairs into the running totals
static void prof_collect(riptrm_ctx* c) {
  for (auto& pr : c->ev_gemv) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, c->ev_pool[pr.first], c->ev_pool[pr.second]) == hipSuccess) c->gemv_ms += ms;
    c->gemv_n++;
  }
  for (auto& pr : c->ev_state) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, c->ev_pool[pr.first], c->ev_pool[pr.second]) == hipSuccess) c->state_ms += ms;
    c->state_n++;
  }
  c->ev_gemv.clear();
  c->ev_state.clear();
  c->ev_used = 0;
}

extern "C" {

int riptrm_abi_version(void) { return RIPTRM_ABI_VERSION; }

int riptrm_ctx_create(riptrm_ctx** out, int device, void* stream) {
  if (!out) return RIPTRM_E_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return RIPTRM_E_NODEV;
  if (device < 0 || device >= ndev) return RIPTRM_E_ARG;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return RIPTRM_E_NODEV;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return RIPTRM_E_NODEV;
  riptrm_ctx* c = new riptrm_ctx();
  c->device = device;
  c->stream = (hipStream_t)stream;
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) == hipSuccess && khz > 0)
    c->clock_hz = (double)khz * 1000.0;
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0) c->ncu = ncu;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_pass[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_pass[1], hipEventDisableTiming) != hipSuccess) {
    riptrm_ctx_destroy(c);
    return RIPTRM_E_HIP;
  }
  *out = c;
  return RIPTRM_OK;
}

int riptrm_ctx_destroy(riptrm_ctx* ctx) {
  if (ctx) {
    if (ctx->gexec) (void)hipGraphExecDestroy(ctx->gexec);
    if (ctx->si) riptrm_si_release(ctx->si);
    riptrm_big_release(ctx);
    for (auto e : ctx->ev_pool) (void)hipEventDestroy(e);
    for (auto e : {ctx->ev_fork, ctx->ev_join, ctx->ev_pass[0], ctx->ev_pass[1]})
      if (e) (void)hipEventDestroy(e);
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
  }
  delete ctx;
  return RIPTRM_OK;
}

const char* riptrm_last_error(const riptrm_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int riptrm_ctx_set_stream(riptrm_ctx* ctx, void* stream) {
  if (!ctx) return RIPTRM_E_ARG;
  ctx->stream = (hipStream_t)stream;
  return RIPTRM_OK;
}

double riptrm_device_clock_hz(riptrm_ctx* ctx) { return ctx ? ctx->clock_hz : 0.0; }

static bool layout_ok(int32_t layout) {
  return layout == RIPTRM_LAYOUT_FULL || layout == RIPTRM_LAYOUT_SYMTILE || layout == RIPTRM_LAYOUT_SHARED;
}

int64_t riptrm_nonnegpca_ld(int32_t n) { return n > 0 ? ld_of(n) : -1; }
int64_t riptrm_nonnegpca_rows(int32_t n) { return n > 0 ? rows_of(n) : -1; }
int64_t riptrm_nonnegpca_s_elems(int32_t n, int32_t layout) {
  return (n > 0 && layout_ok(layout)) ? s_elems_of(n, layout) : -1;
}
int64_t riptrm_workspace_bytes(int32_t n, int32_t batch, int32_t cap, int32_t layout) {
  if (n <= 0 || batch <= 0 || cap < 0 || !layout_ok(layout)) return -1;
  return make_layout(n, batch, cap, layout).total;
}
int64_t riptrm_workspace_offset(int32_t n, int32_t batch, int32_t cap, int32_t layout, int32_t kind) {
  if (n <= 0 || batch <= 0 || cap < 0 || !layout_ok(layout)) return -1;
  const Layout L = make_layout(n, batch, cap, layout);
  switch (kind) {
    case 0: case 1: case 2: case 3:
      return L.off_vec + (int64_t)kind * batch * L.ld * 8;
    case 4: return L.off_stats;
    case 5: return L.off_log;
    default: return -1;
  }
}

int riptrm_nonnegpca_pack(riptrm_ctx* ctx, const double* Z, int64_t ldz, int64_t z_stride, int32_t n, int32_t count,
                          double* S, int32_t layout, int64_t s_stride) {
  if (!ctx) return RIPTRM_E_ARG;
  if (!Z || !S || n <= 0 || count <= 0 || ldz < n || !layout_ok(layout))
    return fail(ctx, RIPTRM_E_ARG, "pack: bad argument");
  if (count > 1 && (z_stride < (int64_t)n * ldz || s_stride < s_elems_of(n, layout)))
    return fail(ctx, RIPTRM_E_ARG, "pack: instance strides too small");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const int64_t ld = ld_of(n);
  const int64_t nsub = ld / 32;
  dim3 grid((unsigned)(nsub * nsub), (unsigned)count);
  hipLaunchKernelGGL(k_pack, grid, dim3(256), 0, ctx->stream, Z, ldz, z_stride, n, S, s_stride, layout, ld,
                     rows_of(n));
  HIPCHK(ctx, hipGetLastError());
  return RIPTRM_OK;
}

// list 0 = instances [base, base + count), one right-hand side each (S-pass calibration)
__global__ void k_list_range(DevParams P, int base, int count) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < count) P.lists[k] = le_make(base + k, 1);
  if (k == 0) P.cnt[0] = count;
}

// Optional (riptrm_set_spass_kind(3) only): which S-pass kernel streams faster on this device for
// this batch.  The two kinds' HBM rates differ by box (the per-tile kernel ran at 5.9-6.7 TB/s in
// the bench on different boxes of the pool, the super-tile kernel at 6.2-6.5 on all of them), so
// kind 3 times both once at bind on a full instance group (3 timed launches each after a warm-up)
// and keeps the faster.  The two kernels add the same products in different fixed orders, so a
// timing-based choice could make two runs of the same solve differ in the last bits; the default
// (kind 1) therefore uses the fixed rule of spass_mode and never times anything.
static int launch_gemv(riptrm_ctx* c, hipStream_t st, int list_in, int zero_cnt, int bound, int smode);
static DevParams params_for(const riptrm_ctx* c, int smode);

// the persistent replicas' parameter block: the instances' parameters with the replica region's
// vectors, scalars, stats and requests (batch x (reps - 1) slots), no log, the instances' grid
static DevParams persist_params(const riptrm_ctx* c) {
  DevParams Q = c->P;
  const Layout& L = c->L;
  Q.batch = c->P.batch * (L.reps > 1 ? L.reps - 1 : 0);
  Q.vec = (double*)(c->ws + L.off_rvec);
  Q.st = (double*)(c->ws + L.off_rstate);
  Q.stats = (double*)(c->ws + L.off_rstats);
  Q.req = (int32_t*)(c->ws + L.off_rreq);
  Q.log = nullptr;
  Q.cap = 0;
  Q.pbatch = c->P.batch;
  Q.smode = 0;
  return Q;
}

static PersistSync persist_sync(const riptrm_ctx* c) {
  const Layout& L = c->L;
  PersistSync sy;
  char* base = c->ws + L.off_sync;
  sy.ctr = (unsigned int*)base;
  sy.clk = (double*)(base + round_up((int64_t)c->P.batch * 4, 16));
  sy.flag = (unsigned int*)(base + round_up((int64_t)c->P.batch * 4, 16) + (int64_t)2 * c->P.batch * 8);
  sy.pbuf2 = (double*)(c->ws + L.off_pbuf2);
  sy.tgrid = (double*)(c->ws + L.off_tgrid);
  sy.tgrid_bytes = (int)L.tgrid_bytes;
  sy.trace = c->persist_trace;
  sy.trace_cap = c->persist_trace_cap;
  return sy;
}

// solve / tCG start: replicas get the instances' starting state too
static int persist_init(riptrm_ctx* c, const double* x, const double* y, int64_t ldv, const double* mu,
                        const double* delta, int mode) {
  c->persist_on = c->persist_ok && c->P.opt.trs_solver == RIPTRM_TRS_SOLVER_TCG;
  c->persist_launched = false;
  if (!c->persist_on || c->L.reps <= 1) return RIPTRM_OK;
  const DevParams Q = persist_params(c);
  hipLaunchKernelGGL(k_init, dim3((unsigned)Q.batch), dim3(256), 0, c->stream, Q, x, y, ldv, mu, delta, mode,
                     c->L.reps - 1);
  HIPCHK(c, hipGetLastError());
  return RIPTRM_OK;
}

static void reset_groups(riptrm_ctx* c) {
  c->parity[0] = c->parity[1] = 0;
  c->active_bound[0] = c->active_bound[1] = 0;
}

// `steps` lock-step iterations of the whole batch in one k_persist launch
static int kick(riptrm_ctx* c);
static int run_steps(riptrm_ctx* c, int steps, int* n_active);

// launch k_persist<K>: cooperative (the runtime refuses a grid that cannot be co-resident instead
// of letting its workgroups spin against each other) unless persist_req == 2
extern "C++" template <int K>
static hipError_t persist_launch(riptrm_ctx* c, unsigned grid, DevParams p, RepBlock rq, PersistSync sy, int steps) {
  const size_t shm = (size_t)TS * TS * sizeof(double);
  if (c->persist_req == 2) {
    hipLaunchKernelGGL(k_persist<K>, dim3(grid), dim3(ST_THREADS), shm, c->stream, p, rq, sy, steps);
    return hipGetLastError();
  }
  if (c->persist_req == 3 && !c->persist_launched) return hipErrorCooperativeLaunchTooLarge;   // test hook
  void* args[] = {&p, &rq, &sy, &steps};
  return hipLaunchCooperativeKernel((const void*)k_persist<K>, dim3(grid), dim3(ST_THREADS), args, (unsigned)shm,
                                    c->stream);
}

static int persist_run(riptrm_ctx* c, int steps, int* n_active) {
  const PersistSync sy = persist_sync(c);
  // the sync block and the tagged grid (adjacent): counters, clocks and tags start at zero
  HIPCHK(c, hipMemsetAsync(c->ws + c->L.off_sync, 0, (size_t)(c->L.off_tgrid - c->L.off_sync + c->L.tgrid_bytes),
                           c->stream));
  if (steps > 0) {
    int i0 = -1, i1 = -1;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (c->prof && (e0 = prof_event(c, &i0)) && (e1 = prof_event(c, &i1))) HIPCHK(c, hipEventRecord(e0, c->stream));
    const unsigned grid = (unsigned)(c->P.batch * c->L.reps);
    const DevParams Q = persist_params(c);
    const RepBlock rq{Q.vec, Q.st, Q.stats, Q.req, Q.batch};
    static_assert(PERSIST_MAX_N <= 4 * ST_THREADS, "k_persist<4> covers every persistent shape");
    const hipError_t le = c->P.n <= 2 * ST_THREADS ? persist_launch<2>(c, grid, params_for(c, 0), rq, sy, steps)
                                                    : persist_launch<4>(c, grid, params_for(c, 0), rq, sy, steps);
    if (le != hipSuccess) {
      (void)hipGetLastError();
      if (c->persist_launched)
        return fail(c, RIPTRM_E_HIP, std::string("persistent lock-step launch refused mid-solve: ") + hipGetErrorString(le));
      // nothing of this solve has run persistently yet: the instances are still at their start
      // (replicas only initialised), so the lock-step pipeline takes over from here
      c->persist_on = false;
      c->persist_fallbacks++;
      c->ev_used -= (e0 ? 1 : 0) + (e1 ? 1 : 0);   // the unused events go back to the pool
      reset_groups(c);
      HIPCHK(c, hipMemsetAsync(c->P.cnt, 0, 4 * sizeof(int32_t), c->stream));
      if (int rc = kick(c)) return rc;
      return run_steps(c, steps, n_active);
    }
    c->persist_launched = true;
    if (c->prof && e1) {
      HIPCHK(c, hipEventRecord(e1, c->stream));
      c->ev_state.push_back({i0, i1});
    }
  }
  hipLaunchKernelGGL(k_persist_count, dim3(1), dim3(256), 0, c->stream, c->P, c->parity[0]);
  HIPCHK(c, hipGetLastError());
  int32_t h = 0;
  uint32_t flag = 0;
  HIPCHK(c, hipMemcpyAsync(&h, c->P.cnt + c->parity[0], sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(&flag, sy.flag, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->prof) prof_collect(c);
  c->active_bound[0] = h;
  if (n_active) *n_active = h;
  if (flag) return fail(c, RIPTRM_E_HIP, "persistent lock-step: a workgroup waited > 2 s at an in-launch barrier "
                                        "(instance stopped with STAT_ERROR = 2)");
  return RIPTRM_OK;
}

static int calibrate_spass(riptrm_ctx* c) {
  c->sup_auto = 1;
  c->spass_cal_ms[0] = c->spass_cal_ms[1] = 0.0f;
  const int count = c->gsize[0];
  if (c->P.layout != RIPTRM_LAYOUT_SYMTILE || c->sup_req != 3 || (int64_t)count * c->P.nsup < (int64_t)4 * c->ncu)
    return RIPTRM_OK;   // calibrated on groups of >= 4 units per CU (the bench's and the headline's case)
  hipLaunchKernelGGL(k_list_range, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, c->stream, c->P, c->gbase[0], count);
  HIPCHK(c, hipGetLastError());
  hipEvent_t ev[4];
  for (auto& e : ev) HIPCHK(c, hipEventCreate(&e));
  float ms[2] = {0.0f, 0.0f};
  int rc = RIPTRM_OK;
  const bool prof = c->prof;
  c->prof = false;   // not part of any measured window
  for (int kind = 0; kind < 2 && rc == RIPTRM_OK; ++kind) {
    rc = launch_gemv(c, c->stream, 0, -1, count, kind);   // warm-up
    if (rc == RIPTRM_OK) rc = hipEventRecord(ev[2 * kind], c->stream) == hipSuccess ? RIPTRM_OK : RIPTRM_E_HIP;
    for (int r = 0; r < 3 && rc == RIPTRM_OK; ++r) rc = launch_gemv(c, c->stream, 0, -1, count, kind);
    if (rc == RIPTRM_OK) rc = hipEventRecord(ev[2 * kind + 1], c->stream) == hipSuccess ? RIPTRM_OK : RIPTRM_E_HIP;
  }
  if (rc == RIPTRM_OK && hipEventSynchronize(ev[3]) == hipSuccess && hipEventElapsedTime(&ms[0], ev[0], ev[1]) == hipSuccess &&
      hipEventElapsedTime(&ms[1], ev[2], ev[3]) == hipSuccess)
    c->sup_auto = ms[1] <= ms[0] ? 1 : 0;
  c->spass_cal_ms[0] = ms[0] / 3.0f;
  c->spass_cal_ms[1] = ms[1] / 3.0f;
  c->prof = prof;
  for (auto& e : ev) (void)hipEventDestroy(e);
  if (rc) return rc;
  HIPCHK(c, hipMemsetAsync(c->P.cnt, 0, 4 * sizeof(int32_t), c->stream));
  return RIPTRM_OK;
}

int riptrm_nonnegpca_bind(riptrm_ctx* ctx, const double* S, int32_t n, int32_t batch, int32_t layout,
                          int64_t inst_stride, void* workspace, int64_t workspace_bytes, int32_t cap) {
  if (!ctx) return RIPTRM_E_ARG;
  if (!S || !workspace || n < 2 || batch <= 0 || cap < 0 || !layout_ok(layout))
    return fail(ctx, RIPTRM_E_ARG, "bind: bad argument (need n >= 2, batch >= 1, a known layout)");
  if (layout == RIPTRM_LAYOUT_SHARED) {
    if (inst_stride != 0) return fail(ctx, RIPTRM_E_ARG, "bind: the shared layout needs inst_stride = 0");
  } else if (inst_stride < s_elems_of(n, layout) || (inst_stride % 2) != 0) {
    return fail(ctx, RIPTRM_E_ARG, "bind: instance stride smaller than riptrm_nonnegpca_s_elems (or odd)");
  }
  if (((uintptr_t)S % 16) != 0 || ((uintptr_t)workspace % 256) != 0)
    return fail(ctx, RIPTRM_E_ARG, "bind: S must be 16-byte and workspace 256-byte aligned");
  const Layout L = make_layout(n, batch, cap, layout);
  if (workspace_bytes < L.total) return fail(ctx, RIPTRM_E_ARG, "bind: workspace too small");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  HIPCHK(ctx, hipMemsetAsync(workspace, 0, (size_t)L.total, ctx->stream));
  ctx->L = L;
  ctx->S = S;
  ctx->inst_stride = inst_stride;
  ctx->ws = (char*)workspace;
  DevParams& P = ctx->P;
  std::memset(&P, 0, sizeof(P));
  P.S = S;
  P.inst_stride = inst_stride;
  P.ld = L.ld;
  P.n = n;
  P.batch = batch;
  P.cap = cap;
  P.nrb = (int)(rows_of(n) / GV_RB);
  P.layout = layout;
  P.nt = L.nt;
  P.ntiles = (int)ntiles_of(n);
  P.wl = edge_w_of(n);
  P.nst = nst_of(n);
  P.nsup = (int32_t)nsup_of(n);
  P.smode = 0;
  P.pbuf = (double*)(ctx->ws + L.off_pbuf);
  P.vec = (double*)(ctx->ws + L.off_vec);
  P.st = (double*)(ctx->ws + L.off_state);
  P.stats = (double*)(ctx->ws + L.off_stats);
  P.log = (double*)(ctx->ws + L.off_log);
  P.lists = (int32_t*)(ctx->ws + L.off_lists);
  P.req = (int32_t*)(ctx->ws + L.off_req);
  P.cnt = (int32_t*)(ctx->ws + L.off_cnt);
  P.pbatch = batch;
  {   // S-pass unit order (k_spass_sup): RIPTRM_SUP_DYNAMIC=0 / 1 overrides the default
    const char* ev = getenv("RIPTRM_SUP_DYNAMIC");
    P.sup_dyn = ev ? (atoi(ev) != 0) : 0;
  }
  P.clock_hz = ctx->clock_hz;
  P.outer_target = INT32_MAX;
  // persistent mode: the workspace has the replica region and every workgroup fits on its own CU
  ctx->persist_ok = ctx->persist_req != 0 && L.reps > 0 && (int64_t)batch * L.reps <= ctx->ncu;
  ctx->persist_on = false;
  ctx->persist_fallbacks = 0;
  if (ctx->persist_ok) {
    HIPCHK(ctx, hipFuncSetAttribute((const void*)k_persist<2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)(TS * TS * sizeof(double))));
    HIPCHK(ctx, hipFuncSetAttribute((const void*)k_persist<4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)(TS * TS * sizeof(double))));
    // every workgroup must be resident at once: ask the occupancy calculator with the launch's
    // dynamic LDS (one 128 KiB tile per workgroup -> at most one per CU), and the device for
    // cooperative launch support
    int nb = 0, coop = 0;
    const void* kp = n <= 2 * ST_THREADS ? (const void*)k_persist<2> : (const void*)k_persist<4>;
    HIPCHK(ctx, hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kp, ST_THREADS, (size_t)TS * TS * sizeof(double)));
    HIPCHK(ctx, hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, ctx->device));
    ctx->persist_ok = nb >= 1 && (int64_t)batch * L.reps <= (int64_t)nb * ctx->ncu && (coop || ctx->persist_req == 2);
  }
  if (layout == RIPTRM_LAYOUT_SHARED) {  // the MFMA S-pass stages two K steps of V and S tiles in LDS
    HIPCHK(ctx, hipFuncSetAttribute((const void*)k_spass_mm<8, 128>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    mm_shm<8, 128>()));
    HIPCHK(ctx, hipFuncSetAttribute((const void*)k_spass_mm<8, 64>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    mm_shm<8, 64>()));
    HIPCHK(ctx, hipFuncSetAttribute((const void*)k_spass_mm<2, 128>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    mm_shm<2, 128>()));
    HIPCHK(ctx, hipFuncSetAttribute((const void*)k_spass_mm<2, 64>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    mm_shm<2, 64>()));
  }
  // two groups only when one group's S-pass is long enough (>= ~0.6 GB, ~100 us) to hide the
  // other group's state kernel; small batches are launch/latency bound and lose from the split
  ctx->ngroups = (layout != RIPTRM_LAYOUT_SHARED && batch >= 8 &&
                  (double)batch * s_elems_of(n, layout) * 8.0 >= 1.2e9) ? 2 : 1;
  if (ctx->groups_req > 0) ctx->ngroups = (ctx->groups_req >= 2 && batch >= 2) ? 2 : 1;
  ctx->gbase[0] = 0;
  ctx->gsize[0] = ctx->ngroups == 2 ? (batch + 1) / 2 : batch;
  ctx->gbase[1] = ctx->gsize[0];
  ctx->gsize[1] = batch - ctx->gsize[0];
  ctx->bound = true;
  ctx->solving = false;
  ctx->pver++;
  return calibrate_spass(ctx);
}

// S-pass kind of the symmetric-tile layout.  Kind 1 (default): the persistent super-tile kernel
// for problems of at least SUP_MIN_UNITS 2 x 2-tile units per instance (n >= 2561), the per-tile
// kernel below that.  The rule depends on n alone, never on how many instances are active: the
// two kernels add the same products in different fixed orders, so a rule that followed the
// active count would make an instance's last bits depend on the other instances of its batch
// (and on when they finish).  With it, an instance gives bitwise the same results alone or inside
// any batch, run after run.  Kind 3 keeps the older rule (super-tile once every CU gets a unit,
// if the bind-time timing preferred it; fastest, not batch-independent).  The state kernel that
// gathers the pass gets the same mode.
constexpr int SUP_MIN_UNITS = 64;
static int spass_mode(const riptrm_ctx* c, int bound) {
  if (c->P.layout != RIPTRM_LAYOUT_SYMTILE || c->sup_req == 0) return 0;
  if (c->sup_req == 2) return 1;
  if (c->sup_req == 1) return c->P.nsup >= SUP_MIN_UNITS ? 1 : 0;
  const bool wide = (int64_t)bound * c->P.nsup >= (int64_t)c->ncu;
  return (wide && c->sup_auto) ? 1 : 0;
}

static DevParams params_for(const riptrm_ctx* c, int smode) {
  DevParams P = c->P;
  P.smode = smode;
  return P;
}

static int launch_gemv(riptrm_ctx* c, hipStream_t st, int list_in, int zero_cnt, int bound, int smode) {
  if (bound <= 0) return RIPTRM_OK;
  const bool sym = c->P.layout == RIPTRM_LAYOUT_SYMTILE;
  const int64_t blocks = (int64_t)bound * (sym ? c->P.ntiles : c->P.nrb);
  int i0 = -1, i1 = -1;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (c->prof && (e0 = prof_event(c, &i0)) && (e1 = prof_event(c, &i1))) HIPCHK(c, hipEventRecord(e0, st));
  if (c->P.layout == RIPTRM_LAYOUT_SHARED) {
    // 128 right-hand sides per workgroup for wide batches, 32 for narrow ones; 128-row tiles when
    // they alone give every CU a workgroup, else 64 (the k order, hence every product, is the same)
    const int rows = rows_of(c->P.n);
    const bool rt128 = (int64_t)((rows + 127) / 128) * MM_KZ >= c->ncu;
    const int nrb = rt128 ? (rows + 127) / 128 : (rows + 63) / 64;
    const int t0 = bound > 32 ? (bound + 127) / 128 : (bound + 31) / 32;
    const dim3 grid((unsigned)(nrb * t0 * MM_KZ));   // in1 tiles run inside these workgroups
    if (bound > 32) {
      if (rt128)
        hipLaunchKernelGGL((k_spass_mm<8, 128>), grid, dim3(64 * MM_WAVES), (mm_shm<8, 128>()), st, c->P, list_in, zero_cnt, bound);
      else
        hipLaunchKernelGGL((k_spass_mm<8, 64>), grid, dim3(64 * MM_WAVES), (mm_shm<8, 64>()), st, c->P, list_in, zero_cnt, bound);
    } else {
      if (rt128)
        hipLaunchKernelGGL((k_spass_mm<2, 128>), grid, dim3(64 * MM_WAVES), (mm_shm<2, 128>()), st, c->P, list_in, zero_cnt, bound);
      else
        hipLaunchKernelGGL((k_spass_mm<2, 64>), grid, dim3(64 * MM_WAVES), (mm_shm<2, 64>()), st, c->P, list_in, zero_cnt, bound);
    }
  } else if (sym && smode) {
    const int64_t units = (int64_t)bound * c->P.nsup;
    const unsigned grid = (unsigned)(units < c->ncu ? units : c->ncu);
    hipLaunchKernelGGL(k_spass_sup, dim3(grid), dim3(SP_THREADS), 0, st, params_for(c, 1), list_in, zero_cnt);
  } else if (sym)
    hipLaunchKernelGGL(k_spass_sym, dim3((unsigned)blocks), dim3(SP_THREADS), 0, st, c->P, list_in, zero_cnt);
  else
    hipLaunchKernelGGL(k_gemv, dim3((unsigned)blocks), dim3(GV_THREADS), 0, st, c->P, list_in, zero_cnt);
  HIPCHK(c, hipGetLastError());
  if (c->prof && e1) {
    HIPCHK(c, hipEventRecord(e1, st));
    c->ev_gemv.push_back({i0, i1});
  }
  return RIPTRM_OK;
}

// dynamic LDS of k_state: the Exact_RepMat work area (Machine::trs_wvec / trs_uvec / trs_red)
static size_t state_lds_bytes(const DevParams& P) {
  if (P.opt.trs_solver != RIPTRM_TRS_SOLVER_EXACT_REPMAT || P.n - 1 > riptrm_trs::DIM_MAX) return 0;
  return ((size_t)riptrm_trs::work_doubles(P.n - 1) + 2 * (riptrm_trs::DIM_MAX + 1) + 2 * ST_WAVES) * sizeof(double);
}

static int launch_state(riptrm_ctx* c, hipStream_t st, int full, int list_in, int list_out, int bound,
                        int full_base, int smode) {
  const int blocks = bound;
  if (blocks <= 0) return RIPTRM_OK;
  int i0 = -1, i1 = -1;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (c->prof && (e0 = prof_event(c, &i0)) && (e1 = prof_event(c, &i1))) HIPCHK(c, hipEventRecord(e0, st));
  if (c->P.opt.trs_solver == RIPTRM_TRS_SOLVER_EXACT_REPMAT)
    hipLaunchKernelGGL(k_state<true>, dim3((unsigned)blocks), dim3(ST_THREADS), state_lds_bytes(c->P), st,
                       params_for(c, smode), full,
                       list_in, list_out, full_base, bound);
  else
    hipLaunchKernelGGL(k_state<false>, dim3((unsigned)blocks), dim3(ST_THREADS), 0, st, params_for(c, smode), full,
                       list_in, list_out,
                       full_base, bound);
  HIPCHK(c, hipGetLastError());
  if (c->prof && e1) {
    HIPCHK(c, hipEventRecord(e1, st));
    c->ev_state.push_back({i0, i1});
  }
  return RIPTRM_OK;
}

// group 1's stream starts after everything already enqueued on the caller's stream
static int fork_streams(riptrm_ctx* c) {
  c->gstream[0] = c->stream;
  c->gstream[1] = c->own_stream;
  if (c->ngroups < 2) return RIPTRM_OK;
  HIPCHK(c, hipEventRecord(c->ev_fork, c->stream));
  HIPCHK(c, hipStreamWaitEvent(c->own_stream, c->ev_fork, 0));
  return RIPTRM_OK;
}

// the caller's stream continues after group 1's work
static int join_streams(riptrm_ctx* c) {
  if (c->ngroups < 2) return RIPTRM_OK;
  HIPCHK(c, hipEventRecord(c->ev_join, c->own_stream));
  HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_join, 0));
  return RIPTRM_OK;
}

int riptrm_nonnegpca_hvp(riptrm_ctx* ctx, const double* x, const double* y, double mu, const double* v, double* out, int64_t ldv) {
  if (!ctx) return RIPTRM_E_ARG;
  if (!ctx->bound) return fail(ctx, RIPTRM_E_STATE, "hvp: bind first");
  if (!x || !y || !v || !out || ldv < ctx->P.n) return fail(ctx, RIPTRM_E_ARG, "hvp: bad argument");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const int B = ctx->P.batch;
  hipLaunchKernelGGL(k_hvp_prep, dim3(B), dim3(256), 0, ctx->stream, ctx->P, x, y, v, ldv);
  HIPCHK(ctx, hipGetLastError());
  const int sm = spass_mode(ctx, B);
  int rc = launch_gemv(ctx, ctx->stream, 0, -1, B, sm);
  if (rc) return rc;
  hipLaunchKernelGGL(k_hvp_epi, dim3(B), dim3(ST_THREADS), 0, ctx->stream, params_for(ctx, sm), mu, out, ldv);
  HIPCHK(ctx, hipGetLastError());
  ctx->solving = false;
  return RIPTRM_OK;
}

int riptrm_nonnegpca_operator_aw(riptrm_ctx* ctx, const double* x, const double* z, const double* s, const double* v,
                                 double* out, int64_t ldv) {
  if (!ctx) return RIPTRM_E_ARG;
  if (!ctx->bound) return fail(ctx, RIPTRM_E_STATE, "operator_aw: bind first");
  if (!x || !z || !s || !v || !out || ldv < ctx->P.n) return fail(ctx, RIPTRM_E_ARG, "operator_aw: bad argument");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  const int B = ctx->P.batch;
  hipLaunchKernelGGL(k_hvp_prep, dim3(B), dim3(256), 0, ctx->stream, ctx->P, x, z, v, ldv);
  HIPCHK(ctx, hipGetLastError());
  const int sm = spass_mode(ctx, B);
  int rc = launch_gemv(ctx, ctx->stream, 0, -1, B, sm);
  if (rc) return rc;
  hipLaunchKernelGGL(k_aw_epi, dim3(B), dim3(ST_THREADS), 0, ctx->stream, params_for(ctx, sm), s, out, ldv);
  HIPCHK(ctx, hipGetLastError());
  ctx->solving = false;
  return RIPTRM_OK;
}

// `steps` lock-step iterations of every group.  Per step and group: S-pass then state kernel on
// the group's stream.  The S-passes of the two groups are chained by events so they never run
// concurrently (each gets the whole HBM; per-launch timing stays clean), while a group's state
// kernel runs beside the other group's S-pass.
constexpr int GRAPH_STEPS = 8;   // even: the ping-pong lists are back at the same parity

// (re)capture GRAPH_STEPS lock-step iterations of group 0 on the private stream
static int capture_graph(riptrm_ctx* c, int bound) {
  if (c->gexec) {
    (void)hipGraphExecDestroy(c->gexec);
    c->gexec = nullptr;
  }
  hipStream_t st = c->own_stream;
  HIPCHK(c, hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  int par = c->parity[0];
  int rc = RIPTRM_OK;
  for (int s = 0; s < GRAPH_STEPS && rc == RIPTRM_OK; ++s) {
    const int lin = par, lout = par ^ 1;
    const int sm = spass_mode(c, bound);
    rc = launch_gemv(c, st, lin, lout, bound, sm);
    if (rc == RIPTRM_OK) rc = launch_state(c, st, 2, lin, lout, c->gsize[0], c->gbase[0], sm);
    par ^= 1;
  }
  hipGraph_t g = nullptr;
  const hipError_t e = hipStreamEndCapture(st, &g);
  if (rc) {
    if (g) (void)hipGraphDestroy(g);
    return rc;
  }
  if (e != hipSuccess) return fail(c, RIPTRM_E_HIP, std::string("hipStreamEndCapture: ") + hipGetErrorString(e));
  const hipError_t e2 = hipGraphInstantiate(&c->gexec, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  if (e2 != hipSuccess) return fail(c, RIPTRM_E_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(e2));
  c->g_bound = bound;
  c->g_parity = c->parity[0];
  c->g_pver = c->pver;
  return RIPTRM_OK;
}

static int run_steps(riptrm_ctx* c, int steps, int* n_active) {
  if (c->persist_on) return persist_run(c, steps, n_active);
  // short kernels (small n x batch): replay a captured graph of GRAPH_STEPS iterations instead of
  // launching 2 kernels per step from the host
  const bool small = (double)c->P.batch * (double)s_elems_of(c->P.n, c->P.layout) * 8.0 < 2.0e8 ||
                     c->P.layout == RIPTRM_LAYOUT_SHARED;
  // Exact_RepMat's k_state needs up to 156 KiB of dynamic LDS: raised by hipFuncSetAttribute for
  // direct launches, but a replayed graph's kernel node ran without it (LDS accesses past 64 KiB
  // faulted, n = 97) -> direct launches whenever the state kernel needs more than the default
  const bool graph_ok = state_lds_bytes(c->P) <= 64 * 1024;
  if (c->graphs && !c->prof && c->ngroups == 1 && c->active_bound[0] > 0 && small && steps > 0 && graph_ok) {
    int bound = 1;
    while (bound < c->active_bound[0]) bound *= 2;
    if (bound > c->P.batch) bound = c->P.batch;
    if (!c->gexec || c->g_bound != bound || c->g_parity != c->parity[0] || c->g_pver != c->pver) {
      const int rc = capture_graph(c, bound);
      if (rc) return rc;
    }
    for (int s = 0; s < steps; s += GRAPH_STEPS) HIPCHK(c, hipGraphLaunch(c->gexec, c->stream));
    int32_t h = 0;
    HIPCHK(c, hipMemcpyAsync(&h, c->P.cnt + c->parity[0], sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    c->active_bound[0] = h;
    if (n_active) *n_active = h;
    return RIPTRM_OK;
  }
  int rc = fork_streams(c);
  if (rc) return rc;
  const int G = c->ngroups;
  for (int s = 0; s < steps; ++s) {
    for (int g = 0; g < G; ++g) {
      if (c->active_bound[g] <= 0) continue;  // nothing queued: keep the list (and its count 0)
      hipStream_t st = c->gstream[g];
      const int lin = g * 2 + c->parity[g], lout = g * 2 + (c->parity[g] ^ 1);
      if (G == 2) HIPCHK(c, hipStreamWaitEvent(st, c->ev_pass[g ^ 1], 0));
      const int sm = spass_mode(c, c->active_bound[g]);
      rc = launch_gemv(c, st, lin, lout, c->active_bound[g], sm);
      if (rc) return rc;
      if (G == 2) HIPCHK(c, hipEventRecord(c->ev_pass[g], st));
      rc = launch_state(c, st, 2, lin, lout, c->gsize[g], c->gbase[g], sm);
      if (rc) return rc;
      c->parity[g] ^= 1;
    }
  }
  int32_t h[2] = {0, 0};
  for (int g = 0; g < G; ++g)
    HIPCHK(c, hipMemcpyAsync(&h[g], c->P.cnt + g * 2 + c->parity[g], sizeof(int32_t), hipMemcpyDeviceToHost,
                             c->gstream[g]));
  rc = join_streams(c);
  if (rc) return rc;
  for (int g = 0; g < G; ++g) HIPCHK(c, hipStreamSynchronize(c->gstream[g]));
  if (c->prof) prof_collect(c);
  for (int g = 0; g < G; ++g) c->active_bound[g] = h[g];
  if (n_active) *n_active = h[0] + (G == 2 ? h[1] : 0);
  return RIPTRM_OK;
}

// (re)start instances that wait for no S-pass (START / raised-target PAUSED): a full state
// launch per group that APPENDS their requests to the group's list `parity`, the one its next
// S-pass reads, so the requests of instances already in flight stay queued.
static int kick(riptrm_ctx* c) {
  if (c->persist_on) {   // k_persist starts startable instances itself (with the uniform clock)
    c->active_bound[0] = c->P.batch;
    return RIPTRM_OK;
  }
  int rc = fork_streams(c);
  if (rc) return rc;
  for (int g = 0; g < c->ngroups; ++g) {
    const int l = g * 2 + c->parity[g];
    rc = launch_state(c, c->gstream[g], 1, l, l, c->gsize[g], c->gbase[g], 0);
    if (rc) return rc;
    c->active_bound[g] = c->gsize[g];
  }
  return join_streams(c);
}


int riptrm_tcg(riptrm_ctx* ctx, const double* x, const double* y, int64_t ldv, const double* mu, const double* delta,
               int32_t* iters, int32_t* stop, int32_t max_steps) {
  if (!ctx) return RIPTRM_E_ARG;
  if (!ctx->bound) return fail(ctx, RIPTRM_E_STATE, "tcg: bind first");
  if (!x || !y || !mu || !delta || ldv < ctx->P.n) return fail(ctx, RIPTRM_E_ARG, "tcg: bad argument");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  DevParams& P = ctx->P;
  if (P.opt.struct_size == 0) {  // tCG defaults (RIPTRM.py:330-332) when no solve options were set
    P.opt.tcg_theta = 1.0;
    P.opt.tcg_kappa = 0.1;
    P.opt.tcg_mininner = 1;
    ctx->pver++;
  }
  hipLaunchKernelGGL(k_init, dim3(P.batch), dim3(256), 0, ctx->stream, P, x, y, ldv, mu, delta, (int)MODE_TCG_ONLY, 1);
  HIPCHK(ctx, hipGetLastError());
  if (int rc0 = persist_init(ctx, x, y, ldv, mu, delta, (int)MODE_TCG_ONLY)) return rc0;
  reset_groups(ctx);
  HIPCHK(ctx, hipMemsetAsync(P.cnt, 0, 4 * sizeof(int32_t), ctx->stream));
  int rc = kick(ctx);
  if (rc) return rc;
  int act = P.batch;
  int total = 0;
  int chunk = 4;
  while (act > 0) {
    if (max_steps > 0 && total >= max_steps) return fail(ctx, RIPTRM_E_STATE, "tcg: step limit reached");
    rc = run_steps(ctx, chunk, &act);
    if (rc) return rc;
    total += chunk;
    if (chunk < 256) chunk *= 2;
  }
  if (iters || stop) {
    const int B = P.batch;
    double* h = new double[(size_t)B * RIPTRM_STAT_NFIELDS];
    hipError_t e = hipMemcpy(h, P.stats, (size_t)B * RIPTRM_STAT_NFIELDS * 8, hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
      delete[] h;
      return fail(ctx, RIPTRM_E_HIP, "tcg: stats copy failed");
    }
    for (int b = 0; b < B; ++b) {
      if (iters) iters[b] = (int32_t)h[b * RIPTRM_STAT_NFIELDS + RIPTRM_STAT_TCG_LAST_J];
      if (stop) stop[b] = (int32_t)h[b * RIPTRM_STAT_NFIELDS + RIPTRM_STAT_TCG_LAST_STOP];
    }
    delete[] h;
  }
  ctx->solving = false;
  return RIPTRM_OK;
}

// the subproblems of Exact_RepMat go to the HBM service (riptrm_trs_big.hip): above the LDS solver's
// size, or everywhere with RIPTRM_TRS_HBM=1 (read at riptrm_solve_begin)
static bool big_trs_path(const riptrm_ctx* c) { return c->P.n - 1 > RIPTRM_TRS_DIM_MAX || c->P.trs_hbm; }

int riptrm_solve_begin(riptrm_ctx* ctx, const riptrm_options* opt, const double* x0, const double* y0, int64_t ldv,
                       const double* mu_table, const double* tolL_table, const double* tolC_table, int32_t table_len) {
  if (!ctx) return RIPTRM_E_ARG;
  if (!ctx->bound) return fail(ctx, RIPTRM_E_STATE, "solve_begin: bind first");
  if (!opt || opt->struct_size != (int32_t)sizeof(riptrm_options))
    return fail(ctx, RIPTRM_E_ARG, "solve_begin: riptrm_options.struct_size mismatch");
  if (opt->trs_solver != RIPTRM_TRS_SOLVER_TCG && opt->trs_solver != RIPTRM_TRS_SOLVER_EXACT_REPMAT)
    return fail(ctx, RIPTRM_E_ARG, "solve_begin: unknown trs_solver");
  if (opt->trs_solver == RIPTRM_TRS_SOLVER_EXACT_REPMAT && ctx->P.n < 2)
    return fail(ctx, RIPTRM_E_ARG, "solve_begin: Exact_RepMat needs n >= 2");
  {   // A/B: the HBM subproblem path below its size limit too (comparisons with the LDS solver)
    const char* e = getenv("RIPTRM_TRS_HBM");
    ctx->P.trs_hbm = (e && e[0] == '1') ? 1 : 0;
  }
  if (opt->trs_solver == RIPTRM_TRS_SOLVER_EXACT_REPMAT && big_trs_path(ctx) &&
      (!ctx->big_ws || ctx->big_order < ctx->P.n || ctx->big_slots < 1))
    return fail(ctx, RIPTRM_E_STATE, "solve_begin: Exact_RepMat above RIPTRM_TRS_DIM_MAX + 1 needs "
                                     "riptrm_trs_bind_workspace(order >= n) first");
  if (!x0 || !y0 || ldv < ctx->P.n || !mu_table || !tolL_table || !tolC_table || table_len <= 0)
    return fail(ctx, RIPTRM_E_ARG, "solve_begin: bad argument");
  if (opt->log_capacity > ctx->L.cap) return fail(ctx, RIPTRM_E_ARG, "solve_begin: log_capacity exceeds bound capacity");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  DevParams& P = ctx->P;
  P.opt = *opt;
  if (const size_t shm = state_lds_bytes(P))
    HIPCHK(ctx, hipFuncSetAttribute((const void*)k_state<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
  P.mu_tab = mu_table;
  P.tolL_tab = tolL_table;
  P.tolC_tab = tolC_table;
  P.tab_len = table_len;
  P.outer_target = INT32_MAX;
  ctx->pver++;
  hipLaunchKernelGGL(k_init, dim3(P.batch), dim3(256), 0, ctx->stream, P, x0, y0, ldv, (const double*)nullptr,
                     (const double*)nullptr, (int)MODE_SOLVE, 1);
  HIPCHK(ctx, hipGetLastError());
  if (int rc0 = persist_init(ctx, x0, y0, ldv, nullptr, nullptr, (int)MODE_SOLVE)) return rc0;
  reset_groups(ctx);
  HIPCHK(ctx, hipMemsetAsync(P.cnt, 0, 4 * sizeof(int32_t), ctx->stream));
  if (int rc0 = riptrm_big_reset_cache(ctx)) return rc0;
  ctx->solving = true;
  return kick(ctx);
}

int riptrm_set_stream_groups(riptrm_ctx* ctx, int32_t groups) {
  if (!ctx || groups < 0 || groups > 2) return RIPTRM_E_ARG;
  if (ctx->solving) return fail(ctx, RIPTRM_E_STATE, "set_stream_groups: call before riptrm_nonnegpca_bind");
  ctx->groups_req = groups;
  return RIPTRM_OK;
}

int riptrm_get_spass_calibration(riptrm_ctx* ctx, double* ms_tile, double* ms_super, int32_t* chosen) {
  if (!ctx || !ms_tile || !ms_super || !chosen) return RIPTRM_E_ARG;
  *ms_tile = ctx->spass_cal_ms[0];
  *ms_super = ctx->spass_cal_ms[1];
  *chosen = spass_mode(ctx, ctx->P.batch);
  return RIPTRM_OK;
}

int riptrm_set_spass_kind(riptrm_ctx* ctx, int32_t kind) {
  if (!ctx || kind < 0 || kind > 3) return RIPTRM_E_ARG;
  ctx->sup_req = kind;
  ctx->pver++;   // a captured graph holds the old kernel
  return RIPTRM_OK;
}

int riptrm_set_persistent(riptrm_ctx* ctx, int32_t mode) {
  if (!ctx || mode < 0 || mode > 3) return RIPTRM_E_ARG;
  if (ctx->solving) return fail(ctx, RIPTRM_E_STATE, "set_persistent: call before riptrm_nonnegpca_bind");
  ctx->persist_req = mode;
  return RIPTRM_OK;
}

int riptrm_persist_trace(riptrm_ctx* ctx, uint64_t* buf, int32_t cap) {
  if (!ctx || cap < 0 || (cap > 0 && !buf)) return RIPTRM_E_ARG;
  ctx->persist_trace = cap > 0 ? (unsigned long long*)buf : nullptr;
  ctx->persist_trace_cap = cap;
  return RIPTRM_OK;
}

int riptrm_get_persistent(riptrm_ctx* ctx, int32_t* possible, int32_t* active) {
  if (!ctx || !possible || !active) return RIPTRM_E_ARG;
  *possible = ctx->persist_ok ? 1 : 0;
  *active = ctx->persist_on ? 1 : 0;
  return RIPTRM_OK;
}

int riptrm_persist_fallbacks(riptrm_ctx* ctx, int32_t* count) {
  if (!ctx || !count) return RIPTRM_E_ARG;
  *count = ctx->persist_fallbacks;
  return RIPTRM_OK;
}

int riptrm_set_graphs(riptrm_ctx* ctx, int32_t on) {
  if (!ctx || on < 0 || on > 1) return RIPTRM_E_ARG;
  ctx->graphs = on;
  return RIPTRM_OK;
}

int riptrm_profile_enable(riptrm_ctx* ctx, int32_t on) {
  if (!ctx) return RIPTRM_E_ARG;
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->own_stream));
  prof_collect(ctx);
  ctx->prof = on != 0;
  ctx->gemv_ms = ctx->state_ms = 0.0;
  ctx->gemv_n = ctx->state_n = 0;
  return RIPTRM_OK;
}

int riptrm_profile_read(riptrm_ctx* ctx, double* gemv_ms, int64_t* gemv_launches, double* state_ms,
                        int64_t* state_launches) {
  if (!ctx) return RIPTRM_E_ARG;
  HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
  HIPCHK(ctx, hipStreamSynchronize(ctx->own_stream));
  prof_collect(ctx);
  if (gemv_ms) *gemv_ms = ctx->gemv_ms;
  if (gemv_launches) *gemv_launches = ctx->gemv_n;
  if (state_ms) *state_ms = ctx->state_ms;
  if (state_launches) *state_launches = ctx->state_n;
  return RIPTRM_OK;
}

int riptrm_log_rebase(riptrm_ctx* ctx) {
  if (!ctx) return RIPTRM_E_ARG;
  if (!ctx->bound) return fail(ctx, RIPTRM_E_STATE, "log_rebase: bind first");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  hipLaunchKernelGGL(k_log_rebase, dim3((unsigned)((ctx->P.batch + 255) / 256)), dim3(256), 0, ctx->stream, ctx->P);
  HIPCHK(ctx, hipGetLastError());
  return RIPTRM_OK;
}

int riptrm_solve_advance(riptrm_ctx* ctx, int32_t steps, int32_t outer_target, int32_t* n_active) {
  if (!ctx) return RIPTRM_E_ARG;
  if (!ctx->solving) return fail(ctx, RIPTRM_E_STATE, "solve_advance: call riptrm_solve_begin first");
  if (steps < 0) return fail(ctx, RIPTRM_E_ARG, "solve_advance: steps < 0");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  if (outer_target != ctx->P.outer_target) {
    const bool raised = outer_target > ctx->P.outer_target;
    ctx->P.outer_target = outer_target;
    ctx->pver++;
    if (raised) {  // resume paused instances
      int rc = kick(ctx);
      if (rc) return rc;
    }
  }
  int act = 0;
  if (int rc = run_steps(ctx, steps, &act)) return rc;
  if (ctx->P.opt.trs_solver == RIPTRM_TRS_SOLVER_EXACT_REPMAT && big_trs_path(ctx)) {
    // instances parked for a host-served subproblem / trial eigenvalue (riptrm_trs_big.hip): serve
    // them and let them run on from PH_TRS_END / PH_MINEIG_END with the next chunk
    int served = 0;
    if (int rc = riptrm_big_service(ctx, &served)) return rc;
    if (served > 0) {
      if (int rc = kick(ctx)) return rc;
      act += served;
    }
  }
  if (n_active) *n_active = act;
  return RIPTRM_OK;
}

}  // extern "C"
