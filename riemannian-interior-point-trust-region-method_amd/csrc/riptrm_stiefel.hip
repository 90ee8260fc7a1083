// riptrm_stiefel.hip — batched Stiefel(n, p) manifold operations on MI355X (gfx950).
//
// north_star asks for "the Sphere/Stiefel projection+retraction from
// pymanopt re-implemented as HIP kernels"; the reference itself has no Stiefel problem, so the
// formulas are pymanopt 2.x's (oracle/stiefel_oracle.py, parity unpinned):
//   projection  P_X(U) = U - X sym(X^T U)              (= euclidean_to_riemannian_gradient)
//   retraction  qf(X + U), the QR factor with diag(R) > 0
//   e2rh        P_X(H - U sym(X^T G))
//   inner       tr(U^T V)
// One 512-thread workgroup (8 waves) per instance.  Both products of a projection run on the fp64
// matrix cores: the symmetric Gram sym(X^T U) streamed row-chunk-wise into registers by all eight
// waves at once (gram_sym), the n x p update X sym(.) with the p x p factor in LDS; per projection
// 3 n p doubles of HBM traffic (read X, U, write the result; the update's re-reads hit L2).
// At p = 50 the two products are ~4 n p^2 flops against 24 n p bytes (p / 6 flop/B, the fp64
// ridge is 78.6 TFLOP/s / 8 TB/s ~ 10): v_mfma_f64_16x16x4_f64 keeps its SIMD busy 64 cycles
// (SQ_VALU_MFMA_BUSY_CYCLES / SQ_INSTS_VALU_MFMA_F64 measured), so one point per CU is
// latency-bound on its chain of loads, MFMAs and barriers.  The retraction is CholeskyQR2 (Q = A R^-1
// with R = chol(A^T A), twice): diag(R) > 0 by construction, so it is pymanopt's qf up to
// rounding for full-rank A.  k_st_retr2 keeps the point in LDS; its first factor is blocked
// (r3_factor_blocked: 16-column diagonal blocks on one wave, the rest on MFMA), its second is taken
// in closed form when Q1 is orthonormal to 1e-10 (r2_inverse_first_order).
#include <hip/hip_runtime.h>
#include <math.h>
#include "riptrm_ctx.h"

namespace riptrm_stiefel {

#pragma clang fp contract(off)

constexpr int NW = 8;          // waves per workgroup (one workgroup per point)
constexpr int T = NW * 64;     // threads per workgroup
constexpr int PMAX = RIPTRM_STIEFEL_PMAX;
constexpr int PS = PMAX + 1;   // LDS row stride of p x p matrices: odd, so a column walk (one row per
                               // lane, the Cholesky) is 2-way banked at worst
constexpr int UB = 13;         // 4-row groups per gram load batch (loads of a batch in flight together;
                               // 2 batches per wave at n = 200)

// LDS (dynamic): M (p x p, stride PS: sym(A^T B), then the Cholesky factor in its lower triangle)
// and red (the k-half partials of the Gram: 4 block rows x 4 block columns x 256 doubles).
// address-space-3 pointers: ds_read / ds_write, not flat accesses through generic pointers
typedef __attribute__((address_space(3))) double lds_f64;
struct Smem {
  lds_f64* M;
  lds_f64* red;
};
constexpr int LDS_DOUBLES = PMAX * PS + 16 * 256;

__device__ __forceinline__ Smem smem_of(double* base_generic) {
  lds_f64* base = (lds_f64*)base_generic;
  return Smem{base, base + PMAX * PS};
}

typedef double dbl4 __attribute__((ext_vector_type(4)));
typedef double dbl2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) dbl2 lds_dbl2;

// Diagnostic builds only (tools/stiefel_stamps.hip defines ST_STAMPS): s_memtime at phase ends,
// thread 0 of each workgroup, into a buffer nothing else reads.
#ifdef ST_STAMPS
__device__ long long* g_st_stamps;
#define ST_STAMP(k)                                                                      \
  do {                                                                                   \
    if (threadIdx.x == 0) g_st_stamps[blockIdx.x * 16 + (k)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define ST_STAMP(k) \
  do {              \
  } while (0)
#endif

// Guarded operand loads: load a clamped (always valid) address and scale by a 0/1 mask, so the
// load cannot be sunk into a branch (a select on a runtime bound makes hipcc branch around every
// load and wait vmcnt(0) after each — one memory latency per element).  Data are finite.
__device__ __forceinline__ double mask01(bool ok) { return ok ? 1.0 : 0.0; }

// sm.M <- sym(A^T B) = (M + M^T) / 2 with M = A^T B, n x p row-major A, B (exactly symmetric:
// M_ij + M_ji is the same sum both ways).  v_mfma_f64_16x16x4_f64 blocks M_IJ (16 x 16, I, J <
// ceil(p/16)): wave w = 4 kg + I owns block row I over the 4-row groups g = kg, kg + 2, ... (the
// k dimension is the n rows), A operand = A[4g + kk][16 I + c] (the block of A^T), B operand =
// B[4g + kk][16 J + c]; loads for UB groups issue together.  The two k halves meet once in LDS
// (kg = 1 writes, kg = 0 adds): a fixed order, bitwise deterministic.  AEQB: A == B (A^T A), the
// B operand of column block I is the A operand.
template <bool AEQB, int P16, bool SUM = false>
__device__ __forceinline__ void gram(Smem& sm, const double* __restrict__ A, const double* __restrict__ B, int n,
                                     int p) {
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  const int c = l & 15, kk = l >> 4;
  const int kg = w >> 2, I = w & 3;
  const int G = (n + 3) / 4;
  dbl4 acc[4];
#pragma unroll
  for (int J = 0; J < 4; ++J) acc[J] = dbl4{0.0, 0.0, 0.0, 0.0};
  if (I < P16) {
    const int colA = 16 * I + c;
    for (int g0 = kg; g0 < G; g0 += 2 * UB) {
      double av[UB], bv[UB][4];
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const int row = 4 * (g0 + 2 * u) + kk;
        const bool rok = row < n;
        const int64_t rb = (int64_t)(rok ? row : n - 1) * p;
        const int64_t ea = rb + (colA < p ? colA : p - 1);
        av[u] = (SUM ? A[ea] + B[ea] : A[ea]) * mask01(rok && colA < p);
#pragma unroll
        for (int J = 0; J < 4; ++J) {   // J, P16: constants
          const int col = 16 * J + c;
          const int64_t eb = rb + (col < p ? col : p - 1);
          const double vb = AEQB ? (SUM ? A[eb] + B[eb] : A[eb]) : B[eb];
          bv[u][J] = J < P16 ? vb * mask01(rok && col < p) : 0.0;
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // every load of the batch issues before the first MFMA
#pragma unroll
      for (int u = 0; u < UB; ++u) {   // groups past the last are zero operands: no branch between loads
#pragma unroll
        for (int J = 0; J < 4; ++J)
          if (J < P16) acc[J] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u], bv[u][J], acc[J], 0, 0, 0);
      }
    }
  }
  if (kg == 1 && I < P16) {
#pragma unroll
    for (int J = 0; J < 4; ++J)
#pragma unroll
      for (int q = 0; q < 4; ++q) sm.red[(I * 4 + J) * 256 + q * 64 + l] = acc[J][q];
  }
  __syncthreads();
  if (kg == 0 && I < P16) {
#pragma unroll
    for (int J = 0; J < 4; ++J) {
      if (J < P16) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const double v = acc[J][q] + sm.red[(I * 4 + J) * 256 + q * 64 + l];
          // D (f64): row = kk + 4q of the block, column = c
          const int i = 16 * I + kk + 4 * q, j = 16 * J + c;
          if (i < p && j < p) sm.M[i * PS + j] = v;
        }
      }
    }
  }
  __syncthreads();
  for (int e = t; e < p * p; e += T) {   // symmetric part: one thread per pair i < j
    const int i = e / p, j = e - (e / p) * p;
    if (i < j) {
      const double v = 0.5 * (sm.M[i * PS + j] + sm.M[j * PS + i]);
      sm.M[i * PS + j] = v;
      sm.M[j * PS + i] = v;
    }
  }
  __syncthreads();
}

// out = C + sgn * A K (K = sm.M, p x p) on the matrix cores.  Units (16-row block R, pair of
// 16-column blocks) are dealt round-robin to the 8 waves; a unit's operands — A[16R + c][4s + kk]
// for every k step, its C values and the K column slices from LDS — are all loaded ahead of a
// scheduling barrier, then its MFMAs run (k steps past p are skipped by a wave-uniform test on
// the MFMA alone, never around a load).  out must not alias A (another wave may still read those
// rows); it may alias C.
template <int P16>
__device__ __forceinline__ void update(Smem& sm, const double* __restrict__ A, const double* C, double sgn,
                                       double* out, int n, int p) {
  constexpr int S4 = 4 * P16;    // k steps of 4 covering 16 P16 columns
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = l & 15, kk = l >> 4;
  const int R16 = (n + 15) / 16, P4 = (p + 3) / 4;
  constexpr int H = (P16 + 1) / 2;   // column-block pairs
  for (int u = w; u < R16 * H; u += NW) {
    const int R = u / H, J0 = 2 * (u - R * H);
    const int arow = 16 * R + c;
    const int64_t ab = (int64_t)(arow < n ? arow : n - 1) * p;
    double ar[S4], bk[2][S4], cv[2][4];
#pragma unroll
    for (int s = 0; s < S4; ++s) {
      const int k = 4 * s + kk;
      ar[s] = A[ab + (k < p ? k : p - 1)] * mask01(arow < n && k < p);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int j = 16 * (J0 + h) + c;
      const bool jok = J0 + h < P16 && j < p;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int i = 16 * R + kk + 4 * g;
        cv[h][g] = C[(int64_t)(i < n ? i : n - 1) * p + (jok ? j : p - 1)] * mask01(jok && i < n);
      }
      const lds_f64* pb = sm.M + kk * PS + (jok ? j : 0);
#pragma unroll
      for (int s = 0; s < S4; ++s) bk[h][s] = pb[(4 * s + kk < p ? 4 * s : 0) * PS] * mask01(jok && 4 * s + kk < p);
    }
    __builtin_amdgcn_sched_barrier(0);
    dbl4 acc[2] = {dbl4{0.0, 0.0, 0.0, 0.0}, dbl4{0.0, 0.0, 0.0, 0.0}};
#pragma unroll
    for (int s = 0; s < S4; ++s)
      if (s < P4) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
          if (J0 + h < P16) acc[h] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[s], bk[h][s], acc[h], 0, 0, 0);
      }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (J0 + h < P16) {
        const int j = 16 * (J0 + h) + c;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int i = 16 * R + kk + 4 * g;
          if (i < n && j < p) out[(int64_t)i * p + j] = cv[h][g] + sgn * acc[h][g];
        }
      }
    }
  }
  __syncthreads();
}

template <int P16>
__global__ void __launch_bounds__(T) k_st_proj(int n, int p, int64_t stride, const double* X, const double* U, double* out) {
  extern __shared__ double lds[];
  Smem sm = smem_of(lds);
  const int64_t o = (int64_t)blockIdx.x * stride;
  ST_STAMP(0);
  gram<false, P16>(sm, X + o, U + o, n, p);
  ST_STAMP(1);
  update<P16>(sm, X + o, U + o, -1.0, out + o, n, p);
  ST_STAMP(2);
}

// ---- projection, round 3: the point resident in LDS, every operand read from HBM once -----------
// k_st_proj above streams X and U from global memory twice (Gram, then update) in register batches,
// so each phase waits on memory latency several times.  Here the whole point is copied into LDS up
// front (X then U, row-major with their own stride p: 2 n p doubles, 160 KB at (200, 50)) by one
// burst of 16-B loads from every thread, and both products run out of LDS:
//   Gram  M = X^T U: the 16 x 16 blocks M_IJ, two per wave, each wave either a transposed pair
//         (M_IJ, M_JI) or two diagonal blocks, all n rows (k) in order: one accumulator chain per
//         block, no cross-wave sum; the blocks land in LDS where U's rows were, after every wave has
//         taken its own output blocks' U values (the update's C operand) into registers;
//   update out = U - X sym(M): unit (16-row block R, 16-column block J); wave w keeps J = w % 4, so
//         its B operand sym(M)[k][J] = (M[k][j] + M[j][k]) / 2 (exactly symmetric) is read once.
// HBM traffic: 24 n p bytes per point, the minimum.  Needs n p even and 2 n p (+ the 64 x 64 M when
// U's area is smaller) doubles of LDS; other shapes run k_st_proj.
constexpr int P3_LDS_DOUBLES = 160 * 1024 / 8;

__host__ __device__ inline int p3_lds_doubles(int n, int p, int P16) {
  const int S = 16 * P16;
  return 2 * n * p + (n * p >= S * S ? 0 : S * S);
}

template <int P16>
__device__ __forceinline__ void p3_unit(int w, int& I0, int& J0, int& I1, int& J1) {
  constexpr int NP = P16 * (P16 - 1) / 2;   // off-diagonal pairs (I < J)
  I0 = J0 = I1 = J1 = -1;
  if (w < NP) {   // pair index w -> (I, J), row by row
    int i = 0, r = w;
#pragma unroll
    for (int q = 0; q < P16; ++q)
      if (r >= P16 - 1 - i && i < P16 - 1) {
        r -= P16 - 1 - i;
        ++i;
      }
    I0 = i; J0 = i + 1 + r;
    I1 = J0; J1 = I0;
  } else {
    const int d = 2 * (w - NP);
    if (d < P16) { I0 = d; J0 = d; }
    if (d + 1 < P16) { I1 = d + 1; J1 = d + 1; }
  }
}

// the Gram of k_st_proj3 over the 4-row groups [g0, g1), GB groups per batch of LDS reads; RMASK: a
// batch runs past row rend = min(n, 4 g1), those rows are masked
constexpr int P3_GB = 5;
template <bool RMASK>
__device__ __forceinline__ void p3_gram(const lds_f64* Xs, const lds_f64* Us, int n, int p, int kk, int a0, int b0,
                                        int a1, int b1, int gs, int ge, dbl4& acc0, dbl4& acc1) {
  constexpr int GB = P3_GB;
  const int rend = 4 * ge < n ? 4 * ge : n;
  for (int g0 = gs; g0 < ge; g0 += GB) {
    double xa0[GB], ub0[GB], xa1[GB], ub1[GB];
#pragma unroll
    for (int u = 0; u < GB; ++u) {
      const int r = 4 * (g0 + u) + kk;
      const lds_f64* xr = Xs + (!RMASK || r < rend ? r : rend - 1) * p;
      const lds_f64* ur = Us + (!RMASK || r < rend ? r : rend - 1) * p;
      const double rm = RMASK ? mask01(r < rend) : 1.0;
      xa0[u] = RMASK ? xr[a0] * rm : xr[a0];
      ub0[u] = ur[b0];
      xa1[u] = RMASK ? xr[a1] * rm : xr[a1];
      ub1[u] = ur[b1];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < GB; ++u) {
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(xa0[u], ub0[u], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(xa1[u], ub1[u], acc1, 0, 0, 0);
    }
  }
}

// the update of k_st_proj3: out = U - X sym(M) for this wave's units (16-row block R, column block J),
// two at a time (two independent accumulator chains per wave, four per SIMD), each unit's P4T k steps
// in order (P4T = ceil(p / 4) as a template parameter: with a runtime bound every MFMA pair sat
// behind its own branch; measured 21.9k ticks for the update at (200, 50))
// units (independent accumulator chains) per wave per step of the update; measured at (200, 50):
// 2 / 3 / 4 -> 22.9k / 22.9k / 23.5k ticks (4 spills): the update is not bound by its chains
// hk(q) after every step q (all waves; k_st_proj4 frees X's rows there)
template <int P16, int P4T, int UMAX, class HK>
__device__ __forceinline__ void p3_update(const lds_f64* Xs, const double (&bk)[4 * P16], const double (&cv)[UMAX][4],
                                          double* out, int n, int p, int w, int c, int kk, int J, int nunits, HK hk) {
  constexpr int UB = 2;
#pragma unroll
  for (int q = 0; q < UMAX; q += UB) {
    if (q > 0) hk(q - UB);
    if (w + NW * q >= nunits) continue;   // wave-uniform (no break: the loop stays unrolled)
    int R[UB];
    bool on[UB];
#pragma unroll
    for (int b = 0; b < UB; ++b) {
      const int u = w + NW * (q + b);
      on[b] = q + b < UMAX && u < nunits;
      R[b] = (on[b] ? u : w + NW * q) / P16;
    }
    double a[UB][P4T];
#pragma unroll
    for (int b = 0; b < UB; ++b) {
      const int ar = 16 * R[b] + c;
      const lds_f64* xr = Xs + (ar < n ? ar : n - 1) * p;
#pragma unroll
      for (int s = 0; s < P4T; ++s) {   // unmasked: sym(M) is zero at k >= p, rows past n are not stored
        const int k = 4 * s + kk;
        a[b][s] = xr[k < p ? k : p - 1];
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    dbl4 acc[UB];
#pragma unroll
    for (int b = 0; b < UB; ++b) acc[b] = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < P4T; ++s)
#pragma unroll
      for (int b = 0; b < UB; ++b) acc[b] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[b][s], bk[s], acc[b], 0, 0, 0);
    const int j = 16 * J + c;
#pragma unroll
    for (int b = 0; b < UB; ++b)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int i = 16 * R[b] + kk + 4 * g;
        if (on[b] && i < n && j < p) out[(int64_t)i * p + j] = cv[q + b < UMAX ? q + b : UMAX - 1][g] - acc[b][g];
      }
  }
  hk((UMAX - 1) / UB * UB);
}

// one projection out of LDS (X at Xs, U at Us, M over U's rows): the Gram, M, and the update; `pf()`
// runs once every wave holds its operands of the update in registers and U's LDS area (M included)
// is free -- k_st_proj4 starts the next point's U copy there
template <int P16, class PF, class HK>
__device__ __forceinline__ void p3_body(int n, int p, const lds_f64* Xs, lds_f64* Us, double* outp, PF pf, HK hk) {
  constexpr int S = 16 * P16;
  lds_f64* Ms = (n * p >= S * S) ? Us : Us + n * p;   // M over U's rows once they are consumed
  const int t = threadIdx.x, l = t & 63, w = t >> 6, c = l & 15, kk = l >> 4;
  (void)t;
  (void)l;
  // Gram: this wave's two blocks over all n rows
  int I0, J0, I1, J1;
  p3_unit<P16>(w, I0, J0, I1, J1);
  dbl4 acc0 = dbl4{0.0, 0.0, 0.0, 0.0}, acc1 = dbl4{0.0, 0.0, 0.0, 0.0};
  if (I0 >= 0) {
    // columns past p are clamped, not masked: they only feed M's rows / columns past p, which are
    // stored as zero below (a 0/1 factor on each operand would make every read's multiply wait on
    // that read inside the batch)
    const int ca0 = 16 * I0 + c, cb0 = 16 * J0 + c;
    const int ca1 = 16 * (I1 >= 0 ? I1 : I0) + c, cb1 = 16 * (J1 >= 0 ? J1 : J0) + c;
    const int a0 = ca0 < p ? ca0 : p - 1, b0 = cb0 < p ? cb0 : p - 1;
    const int a1 = ca1 < p ? ca1 : p - 1, b1 = cb1 < p ? cb1 : p - 1;
    const int G = (n + 3) / 4;
    if (n % (4 * P3_GB) == 0) p3_gram<false>(Xs, Us, n, p, kk, a0, b0, a1, b1, 0, G, acc0, acc1);
    else p3_gram<true>(Xs, Us, n, p, kk, a0, b0, a1, b1, 0, G, acc0, acc1);
  }
  ST_STAMP(2);
  // the update's C operand (U at this wave's output blocks) while U is still in LDS
  constexpr int UMAX = 7;   // units per wave: ceil(R16 P16 / 8) <= 7 for n <= 208 at P16 = 4
  const int R16 = (n + 15) / 16;
  const int J = w % P16;
  const int nunits = R16 * P16;
  double cv[UMAX][4];
#pragma unroll
  for (int q = 0; q < UMAX; ++q) {
    const int u = w + NW * q;
    const int R = u / P16;
    const int j = 16 * J + c;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int i = 16 * R + kk + 4 * g;
      const bool ok = u < nunits && i < n && j < p;
      cv[q][g] = Us[(ok ? i : 0) * p + (ok ? j : 0)];   // unmasked: outputs past n or p are not stored
    }
  }
  __syncthreads();   // every read of U in LDS is done: M may overwrite it
  if (I0 >= 0) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {   // M is zero outside [0, p)^2 (the update's k steps past p rely on it)
      const int i0 = 16 * I0 + kk + 4 * g, j0 = 16 * J0 + c, i1 = 16 * I1 + kk + 4 * g, j1 = 16 * J1 + c;
      Ms[i0 * S + (j0 ^ (i0 & 15))] = acc0[g] * mask01(i0 < p && j0 < p);   // column XOR row: see bk below
      if (I1 >= 0) Ms[i1 * S + (j1 ^ (i1 & 15))] = acc1[g] * mask01(i1 < p && j1 < p);
    }
  }
  __syncthreads();
  ST_STAMP(3);
  // update: B = sym(M)[4s + kk][16 J + c] for this wave's column block J, read once
  constexpr int S4 = 4 * P16;
  const int P4 = (p + 3) / 4;
  double bk[S4];
#pragma unroll
  for (int s = 0; s < S4; ++s) {
    const int k = 4 * s + kk, j = 16 * J + c;
    // zero past p (M is zero there).  M's columns are XOR-swizzled by the row, so the transposed read
    // (16 lanes on 16 rows of one column) is bank-conflict free (unswizzled: 16-way)
    bk[s] = 0.5 * (Ms[k * S + (j ^ (k & 15))] + Ms[j * S + (k ^ (j & 15))]);
  }
  pf();
  switch (P4) {   // the update specialised on the k steps, so no MFMA sits behind a per-step branch
    case 13: p3_update<P16, 13, UMAX>(Xs, bk, cv, outp, n, p, w, c, kk, J, nunits, hk); break;
    case 14: p3_update<P16, 14, UMAX>(Xs, bk, cv, outp, n, p, w, c, kk, J, nunits, hk); break;
    case 15: p3_update<P16, 15, UMAX>(Xs, bk, cv, outp, n, p, w, c, kk, J, nunits, hk); break;
    default: p3_update<P16, 16, UMAX>(Xs, bk, cv, outp, n, p, w, c, kk, J, nunits, hk); break;
  }
  ST_STAMP(4);
}

template <int P16>
__global__ void __launch_bounds__(T) k_st_proj3(int n, int p, int64_t stride, const double* X, const double* U,
                                                double* out) {
  constexpr int UL = 10;   // 16-B copies per thread per matrix in flight
  extern __shared__ double lds[];
  lds_f64* Xs = (lds_f64*)lds;
  lds_f64* Us = Xs + n * p;
  const int t = threadIdx.x;
  const int64_t o = (int64_t)blockIdx.x * stride;
  ST_STAMP(0);
  {   // X, U -> LDS: np / 2 16-byte chunks each, every load of a batch in flight together (loading the
      // second row half while the Gram runs over the first measured slower: 33.8 vs 31.3 us)
    const int nc = n * p / 2;
    const dbl2* Xg = (const dbl2*)(X + o);
    const dbl2* Ug = (const dbl2*)(U + o);
    for (int e0 = 0; e0 < nc; e0 += T * UL) {
      dbl2 vx[UL], vu[UL];
#pragma unroll
      for (int u = 0; u < UL; ++u) {
        const int e = e0 + u * T + t;
        const int ec = e < nc ? e : nc - 1;
        vx[u] = Xg[ec];
        vu[u] = Ug[ec];
      }
#pragma unroll
      for (int u = 0; u < UL; ++u) {
        const int e = e0 + u * T + t;
        if (e < nc) {
          *(__attribute__((address_space(3))) dbl2*)(Xs + 2 * e) = vx[u];
          *(__attribute__((address_space(3))) dbl2*)(Us + 2 * e) = vu[u];
        }
      }
    }
  }
  __syncthreads();
  ST_STAMP(1);
  p3_body<P16>(n, p, Xs, Us, out + o, [] {}, [](int) {});
}

// n p / 2 16-byte chunks from global memory into LDS (lane-linear image) by LDS-DMA: wave w's
// instruction k copies chunks 64 (w + NW k) .. + 63; no VGPR destination, nothing waits on them until
// the caller's vmcnt(0) (a __syncthreads()).  Chunks past nc are not issued (exec mask).
__device__ __forceinline__ void p4_dma(const double* g, lds_f64* l, int c0, int c1) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int e0 = c0 + 64 * w; e0 < c1; e0 += 64 * NW) {
    const int e = e0 + lane;
    if (e < c1)
      __builtin_amdgcn_global_load_lds((const void*)(g + 2 * (int64_t)e), (__attribute__((address_space(3))) void*)(l + 2 * e0),
                                       16, 0, 0);
  }
}

// a workgroup barrier that leaves LDS-DMA copies in flight: this wave's LDS reads are complete
// (lgkmcnt(0)), no vmcnt wait (a __syncthreads() would drain the copies); the memory clobber keeps
// the compiler from moving LDS accesses across it
__device__ __forceinline__ void p4_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// k_st_proj3 as a persistent loop over the points b = blockIdx.x, + gridDim.x, ... (one workgroup per
// CU, the point resident in LDS): the next point's U is copied into U's LDS area by LDS-DMA while the
// update runs (M and the update's operands are in registers by then), and its X once the update has
// read X; the copies run beside the update's matrix-core work instead of in front of the Gram.
template <int P16>
__global__ void __launch_bounds__(T) k_st_proj4(int n, int p, int64_t stride, int batch, const double* X,
                                                const double* U, double* out) {
  extern __shared__ double lds[];
  lds_f64* Xs = (lds_f64*)lds;
  lds_f64* Us = Xs + n * p;
  const int nc = n * p / 2;
  int b = blockIdx.x;
  if (b >= batch) return;
  p4_dma(X + (int64_t)b * stride, Xs, 0, nc);
  p4_dma(U + (int64_t)b * stride, Us, 0, nc);
  __syncthreads();   // vmcnt(0): this point's copies landed
  for (; b < batch; b += gridDim.x) {
    const int nb = b + (int)gridDim.x;
    // opaque per iteration: keeps the body's per-lane LDS addresses from being hoisted out of the loop
    // (live across it they pushed the inlined body past 256 VGPRs)
    int n_ = n, p_ = p;
    asm volatile("" : "+s"(n_), "+s"(p_));
    const double* Xn = X + (int64_t)nb * stride;
    int rdone = 0;   // rows of X whose next-point copy is issued
    ST_STAMP(0);
    ST_STAMP(1);
    p3_body<P16>(n_, p_, Xs, Us, out + (int64_t)b * stride, [&] {
      if (nb < batch) {
        __syncthreads();   // every wave's M reads are done: U's area is free
        p4_dma(U + (int64_t)nb * stride, Us, 0, nc);
      }
    }, [&](int q) {
      // after update step q every unit u < NW (q + 2) is done: X's rows below 16 (NW (q + 2) / P16)
      // are read for good, and the next point's rows go there while the update goes on
      if (nb < batch) {
        int r1 = 16 * ((NW * (q + 2)) / P16);
        r1 = r1 < n_ ? r1 & ~1 : n_;   // whole 16-B chunks (n p even; an even row count keeps r p even)
        if (r1 > rdone) {
          p4_barrier();
          p4_dma(Xn, Xs, rdone * p_ / 2, r1 * p_ / 2);
          rdone = r1;
        }
      }
    });
    if (nb < batch) __syncthreads();   // vmcnt(0): the next point's copies landed
    ST_STAMP(5);
  }
}

template <int P16>
__global__ void __launch_bounds__(T) k_st_e2rh(int n, int p, int64_t stride, const double* X, const double* G,
                                               const double* H, const double* U, double* out) {
  extern __shared__ double lds[];
  Smem sm = smem_of(lds);
  const int64_t o = (int64_t)blockIdx.x * stride;
  gram<false, P16>(sm, X + o, G + o, n, p);              // sym(X^T G)
  update<P16>(sm, U + o, H + o, -1.0, out + o, n, p);    // W = H - U sym(X^T G) into out
  gram<false, P16>(sm, X + o, out + o, n, p);            // sym(X^T W)
  update<P16>(sm, X + o, out + o, -1.0, out + o, n, p);  // P_X(W)
}

// ---- retraction (CholeskyQR2): the round-1 kernel, kept as measured best ----------------------
// Its own LDS layout: M and L (p x p, stride 16 ceil(p/16)) and the 8-wave Gram tree's partials.
// Redesigns tried this round and measured slower at (200, 50) x 256 (tools/stiefel_stamps.hip
// phase stamps, profiles/r2_stiefel_phase_stamps.jsonl): single-wave Cholesky
// variants, a column-oriented row solve with data-dependent LDS reads, a first Gram reading X + U
// directly, and a 16-column-blocked factor + solve (MFMA off-diagonal blocks, 16-step row
// chains; agrees with this kernel to 2.8e-16) — 222-349 µs in total against this kernel's 191 µs.
constexpr int NBLK = 10;       // upper-triangular 16 x 16 blocks of a p x p matrix at p <= 64
constexpr int GMAX = 8;        // 4-row groups per wave per streamed chunk (8 waves x 32 rows = 256 rows)
struct SmemR {
  lds_f64* M;
  lds_f64* L;
  lds_f64* red;
};
constexpr int LDS_DOUBLES_R = 2 * PMAX * PMAX + (NW / 2) * NBLK * 256;
__device__ __forceinline__ SmemR smem_of_r(double* base_generic) {
  lds_f64* base = (lds_f64*)base_generic;
  return SmemR{base, base + PMAX * PMAX, base + 2 * PMAX * PMAX};
}
__device__ __forceinline__ int pstride(int p) { return ((p + 15) / 16) * 16; }

// sm.M <- sym(A^T B) = (A^T B + B^T A) / 2 for n x p row-major A, B, exactly symmetric, on the fp64
// matrix cores.  Every wave streams its own rows straight into registers — each lane loads the
// 4 x 16 operand fragments of v_mfma_f64_16x16x4_f64 for GMAX 4-row groups and all p columns at
// once (one memory latency per 256-row chunk, all loads of the workgroup in flight together) —
// and accumulates the upper-triangular blocks S_IJ = A_I^T B_J + B_I^T A_J (I <= J).  The eight
// wave partials meet in a fixed LDS tree (bitwise deterministic); wave 0 writes S / 2.
__device__ __forceinline__ void gram_sym_r(SmemR& sm, const double* __restrict__ A, const double* __restrict__ B,
                                         int n, int p) {
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  const int c = l & 15, kk = l >> 4;
  const int P16 = (p + 15) / 16, PS = P16 * 16;
  dbl4 acc[NBLK];
#pragma unroll
  for (int b = 0; b < NBLK; ++b) acc[b] = dbl4{0.0, 0.0, 0.0, 0.0};
  for (int r0 = 0; r0 < n; r0 += NW * GMAX * 4) {
    double ar[GMAX][4], br[GMAX][4];
#pragma unroll
    for (int g = 0; g < GMAX; ++g) {
      const int row = r0 + (w * GMAX + g) * 4 + kk;
#pragma unroll
      for (int I = 0; I < 4; ++I) {
        const int col = 16 * I + c;
        const bool ok = row < n && col < p;
        const int64_t e = ok ? (int64_t)row * p + col : 0;
        const double va = A[e], vb = B[e];
        ar[g][I] = ok ? va : 0.0;
        br[g][I] = ok ? vb : 0.0;
      }
    }
#pragma unroll
    for (int g = 0; g < GMAX; ++g) {
      if (r0 + (w * GMAX + g) * 4 >= n) break;   // wave-uniform: rows past n are all zero
      int b = 0;
#pragma unroll
      for (int I = 0; I < 4; ++I)
#pragma unroll
        for (int J = I; J < 4; ++J) {
          if (J < P16) {
            acc[b] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[g][I], br[g][J], acc[b], 0, 0, 0);
            acc[b] = __builtin_amdgcn_mfma_f64_16x16x4f64(br[g][I], ar[g][J], acc[b], 0, 0, 0);
          }
          ++b;
        }
    }
  }
  // tree over the waves: upper half writes, lower half adds (4 -> 2 -> 1)
#pragma unroll
  for (int h = NW / 2; h >= 1; h >>= 1) {
    if (w >= h && w < 2 * h) {
      lds_f64* r = sm.red + (int64_t)(w - h) * NBLK * 256;
#pragma unroll
      for (int b = 0; b < NBLK; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) r[b * 256 + q * 64 + l] = acc[b][q];
    }
    __syncthreads();
    if (w < h) {
      const lds_f64* r = sm.red + (int64_t)w * NBLK * 256;
#pragma unroll
      for (int b = 0; b < NBLK; ++b)
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[b][q] = acc[b][q] + r[b * 256 + q * 64 + l];
    }
    __syncthreads();
  }
  for (int e = t; e < PS * PS; e += T) sm.M[e] = 0.0;
  __syncthreads();
  if (w == 0) {
    int b = 0;
#pragma unroll
    for (int I = 0; I < 4; ++I)
#pragma unroll
      for (int J = I; J < 4; ++J) {
        if (J < P16) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int i = I * 16 + kk + 4 * q, j = J * 16 + c;
            if (i < p && j < p && (I < J || i <= j)) {   // one writer per symmetric pair
              const double v = 0.5 * acc[b][q];
              sm.M[i * PS + j] = v;
              sm.M[j * PS + i] = v;
            }
          }
        }
        ++b;
      }
  }
  __syncthreads();
}

// sm.M (SPD p x p, stride PS) -> sm.L = lower Cholesky factor (A^T A = L L^T, diag > 0)
__device__ __forceinline__ void chol_lower_r(SmemR& sm, int p) {
  const int t = threadIdx.x, PS = pstride(p);
  lds_f64* G = sm.M;
  lds_f64* L = sm.L;
  for (int e = t; e < PS * PS; e += T) L[e] = 0.0;
  __syncthreads();
  for (int k = 0; k < p; ++k) {
    const double lkk = sqrt(G[k * PS + k]);   // final since step k - 1; every thread takes it
    if (t == 0) L[k * PS + k] = lkk;
    for (int i = k + 1 + t; i < p; i += T) L[i * PS + k] = G[i * PS + k] / lkk;
    __syncthreads();
    const int m = p - k - 1;
    for (int e = t; e < m * m; e += T) {
      const int i = k + 1 + e / m, j = k + 1 + (e - (e / m) * m);
      if (j <= i) G[i * PS + j] = G[i * PS + j] - L[i * PS + k] * L[j * PS + k];
    }
    __syncthreads();
  }
}

// A <- A R^-1 (R = L^T) row by row: row a_i solves q R = a_i by forward substitution, all n rows in
// parallel with the row in registers and L read as LDS broadcasts — no serial p^2 inverse.
__device__ __forceinline__ void rows_solve_r(const SmemR& sm, double* A, int n, int p) {
  const int PS = pstride(p);
  for (int i = threadIdx.x; i < n; i += T) {
    double q[PMAX];
#pragma unroll
    for (int j = 0; j < PMAX; ++j) q[j] = (j < p) ? A[(int64_t)i * p + j] : 0.0;
#pragma unroll
    for (int j = 0; j < PMAX; ++j) {
      if (j < p) {
        double s = q[j];
#pragma unroll
        for (int k = 0; k < j; ++k) s = s - q[k] * sm.L[j * PS + k];
        q[j] = s / sm.L[j * PS + j];
      }
    }
#pragma unroll
    for (int j = 0; j < PMAX; ++j)
      if (j < p) A[(int64_t)i * p + j] = q[j];
  }
  __syncthreads();
}

__global__ void __launch_bounds__(T) k_st_retr_r(int n, int p, int64_t stride, const double* X, const double* U, double* out) {
  extern __shared__ double lds[];
  SmemR sm = smem_of_r(lds);
  const int64_t o = (int64_t)blockIdx.x * stride;
  double* A = out + o;
  for (int e = threadIdx.x; e < n * p; e += T) A[e] = X[o + e] + U[o + e];
  __syncthreads();
  for (int pass = 0; pass < 2; ++pass) {   // CholeskyQR2
    gram_sym_r(sm, A, A, n, p);                // (A^T A + A^T A) / 2 = A^T A exactly
    chol_lower_r(sm, p);
    rows_solve_r(sm, A, n, p);                 // A R^-1
  }
}

// ---- retraction, round 2: the point resident in LDS ---------------------------------------------
// The round-1 kernel above re-reads A from global memory in every phase and spends most of its time
// in LDS-latency chains (a row solve that waits on one L read per FMA; a factor with an integer
// division per element and two barriers per step).  This one keeps A = X + U (then Q1) in LDS for
// the whole CholeskyQR2 and turns every O(n p^2) step into fp64 MFMA work:
//   1. A -> LDS, row-major with stride S = 16 ceil(p/16), zero padded to NR = 16 ceil(n/16) rows,
//      element (r, c) at r S + (c ^ (r & 15)) (XOR swizzle inside 16-column groups: the Gram reads a
//      row's 16 consecutive columns per lane group, the product reads 16 rows of one column; a
//      32-lane ds_read_b64 group still spans only 32 of the 64 banks, 2-way — swapping odd rows'
//      16-column blocks in pairs removes that but measured no faster: Gram 16.5k vs 16.9k ticks,
//      load 17.4k vs 14.7k; profiles/r3_stiefel_retr_block_pair_swizzle_stamps.jsonl);
//   2. G = A^T A: the upper 16 x 16 blocks (I <= J), each split over two k halves, the
//      (block, half) tasks dealt to the 8 waves; halves meet once in a fixed order;
//   3. E = L^-1 (G = L L^T) by symmetric Gauss-Jordan elimination on registers: thread (j = lane,
//      rows 8 w .. 8 w + 7) holds G[i][j] and E[i][j]; per step k the lane-k threads publish G's
//      column k and wave k / 8 publishes E's row k (double-buffered in LDS, ONE barrier per step),
//      then every thread applies E_i -= (G_ik / G_kk) E_k, G_ij -= (G_ik / G_kk) G_jk (i > k); row k
//      is scaled by G_kk^-1/2 after the loop — no division by a runtime size, no second barrier;
//   4. Q = A R^-1 = A E^T on MFMA (E^T upper triangular: only the K <= J blocks), the wave's 16-row
//      blocks in registers; Q1 overwrites A in LDS, the second pass writes Q to global memory.
// diag(R) = diag(L^T) > 0 by construction: pymanopt's qf up to rounding, as the round-1 kernel.
template <int P16>
__host__ __device__ constexpr int r2_lds_doubles_nr(int NR) {
  return NR * 16 * P16 + (16 * P16) * (16 * P16) + (P16 * (P16 + 1) / 2) * 256;
}

template <int P16>
__device__ __forceinline__ void r2_block_ij(int b, int& I, int& J) {
  int i = 0;
#pragma unroll
  for (int q = 0; q < P16; ++q)
    if (b >= P16 - i) {
      b -= P16 - i;
      ++i;
    }
  I = i;
  J = i + b;
}

// The Gram writes only G's upper triangle: the blocked factor (r3_factor_blocked) and the
// first-order inverse read nothing else.

// MASK = false when every batch is full (both halves a multiple of the batch size, e.g. n = 200): the
// 0/1 factor on each A operand is then dropped — with it in, each read's multiply waits on that read
// inside the batch (s_waitcnt lgkmcnt after every 4 reads), which serialises the batch's LDS latency.
// hsel: run only the tasks of k half hsel (0 or 1; -1: both)
template <int P16, bool MASK, int UB2>
__device__ __forceinline__ void r2_gram_tasks(lds_f64* As, lds_f64* Gm, lds_f64* red, int NR, int hsel) {
  constexpr int S = 16 * P16, NB = P16 * (P16 + 1) / 2;
  const int t = threadIdx.x, l = t & 63, w = t >> 6, c = l & 15, kk = l >> 4;
  const int NG = NR / 4, H0 = NG / 2;   // k groups of 4 rows; half 0 = [0, H0), half 1 = [H0, NG)
  for (int task = w; task < 2 * NB; task += NW) {   // wave-uniform
    const int b = task % NB, h = task / NB;
    if (hsel >= 0 && h != hsel) continue;
    int I, J;
    r2_block_ij<P16>(b, I, J);
    const int g0 = h ? H0 : 0, g1 = h ? NG : H0;
    dbl4 acc2[2] = {dbl4{0.0, 0.0, 0.0, 0.0}, dbl4{0.0, 0.0, 0.0, 0.0}};   // two chains: MFMAs of a batch overlap
    for (int g = g0; g < g1; g += UB2) {
      double av[UB2], bv[UB2];
#pragma unroll
      for (int u = 0; u < UB2; ++u) {
        const bool ok = !MASK || g + u < g1;
        const int r = 4 * (ok ? g + u : g1 - 1) + kk;
        const lds_f64* row = As + r * S;
        av[u] = MASK ? row[(16 * I + c) ^ (r & 15)] * mask01(ok) : row[(16 * I + c) ^ (r & 15)];
        bv[u] = row[(16 * J + c) ^ (r & 15)];
      }
      __builtin_amdgcn_sched_barrier(0);   // the batch's reads issue together
#pragma unroll
      for (int u = 0; u < UB2; ++u)
        acc2[u & 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u], bv[u], acc2[u & 1], 0, 0, 0);
    }
    const dbl4 acc = acc2[0] + acc2[1];
    lds_f64* dst = (h ? red : Gm) + b * 256;   // half 0 partials in Gm's space, half 1 in red
#pragma unroll
    for (int q = 0; q < 4; ++q) dst[q * 64 + l] = acc[q];
  }
}

template <int P16>
__device__ __forceinline__ void r2_gram_half(lds_f64* As, lds_f64* Gm, lds_f64* red, int NR, int hsel) {
  const int NG = NR / 4, H0 = NG / 2;
  if (H0 % 13 == 0 && (NG - H0) % 13 == 0) r2_gram_tasks<P16, false, 13>(As, Gm, red, NR, hsel);   // n = 200: 2 x 13 per half
  else r2_gram_tasks<P16, true, 14>(As, Gm, red, NR, hsel);
}

// the halves' partials (half 0 in Gm's area, half 1 in red) -> the symmetric G in Gm
template <int P16>
__device__ __forceinline__ void r2_gram_finish(lds_f64* Gm, lds_f64* red) {
  constexpr int S = 16 * P16, NB = P16 * (P16 + 1) / 2;
  const int t = threadIdx.x;
  __syncthreads();
  constexpr int PER = (NB * 256 + T - 1) / T;
  double v[PER];
#pragma unroll
  for (int m = 0; m < PER; ++m) {
    const int e = t + m * T;
    v[m] = e < NB * 256 ? Gm[e] + red[e] : 0.0;   // fixed order: half 0 + half 1
  }
  __syncthreads();
#pragma unroll
  for (int m = 0; m < PER; ++m) {
    const int e = t + m * T;
    if (e < NB * 256) {
      const int b = e >> 8, q = (e >> 6) & 3, ll = e & 63;
      int I, J;
      r2_block_ij<P16>(b, I, J);
      const int i = 16 * I + (ll >> 4) + 4 * q, j = 16 * J + (ll & 15);   // f64 D: row (l >> 4) + 4 q, col l & 15
      if (I < J || i <= j) {   // one writer per symmetric pair: G exactly symmetric
        Gm[i * S + j] = v[m];
      }
    }
  }
  __syncthreads();
}

template <int P16>
__device__ __forceinline__ void r2_gram(lds_f64* As, lds_f64* Gm, lds_f64* red, int NR) {
  r2_gram_half<P16>(As, Gm, red, NR, -1);
  r2_gram_finish<P16>(Gm, red);
}

// The Gram with a narrow last column block (P16 = 4, tw = p - 48 <= 4 valid columns in it, e.g.
// p = 50): the 16 x 16 MFMA blocks that touch that block (4 of the 10) do the work of 2 columns in
// 16, so they are dropped — the matrix cores take the 6 blocks of the first 48 columns and the VALU
// takes the tw last columns: wave w sums rows [26 w, 26 w + 26) of A[r][i] A[r][48 + t] in lane i,
// the 8 wave partials meet in wave order.  G's last column block is written whole (zeros past p),
// upper triangle only (the blocked factor reads nothing else).  Unmasked batches only.
template <int TW>
__device__ __forceinline__ void r4t_gram(lds_f64* As, lds_f64* Gm, lds_f64* red, int NR, int n, int p) {
  constexpr int S = 64, PM = 3, NBm = 6, c0 = 48, UB2 = 13;
  const int t = threadIdx.x, l = t & 63, w = t >> 6, c = l & 15, kk = l >> 4;
  const int NG = NR / 4, H0 = NG / 2;
  // (1) MFMA: the 6 upper blocks of the first 48 columns, both k halves
  for (int task = w; task < 2 * NBm; task += NW) {   // wave-uniform
    const int b = task % NBm, h = task / NBm;
    int I, J;
    r2_block_ij<PM>(b, I, J);
    const int g0 = h ? H0 : 0, g1 = h ? NG : H0;
    dbl4 acc2[2] = {dbl4{0.0, 0.0, 0.0, 0.0}, dbl4{0.0, 0.0, 0.0, 0.0}};
    for (int g = g0; g < g1; g += UB2) {
      double av[UB2], bv[UB2];
#pragma unroll
      for (int u = 0; u < UB2; ++u) {
        const int r = 4 * (g + u) + kk;
        const lds_f64* row = As + r * S;
        av[u] = row[(16 * I + c) ^ (r & 15)];
        bv[u] = row[(16 * J + c) ^ (r & 15)];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < UB2; ++u)
        acc2[u & 1] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u], bv[u], acc2[u & 1], 0, 0, 0);
    }
    const dbl4 acc = acc2[0] + acc2[1];
    lds_f64* dst = (h ? red : Gm) + b * 256;   // half 0 partials in Gm's space, half 1 in red
#pragma unroll
    for (int q = 0; q < 4; ++q) dst[q * 64 + l] = acc[q];
  }
  // (2) VALU: this wave's rows of the tw last columns, column i = lane
  lds_f64* tb = Gm + 2048;   // [NW][4][64] wave partials (past the half-0 MFMA partials)
  {
    const int RB = (NR + NW - 1) / NW, r0 = w * RB, r1 = r0 + RB < n ? r0 + RB : n;
    const int ic = l < p ? l : p - 1;
    double sum[TW];
#pragma unroll
    for (int q = 0; q < TW; ++q) sum[q] = 0.0;
    for (int r = r0; r < r1; ++r) {
      const lds_f64* row = As + r * S;
      const double ai = row[(ic & ~15) | ((ic & 15) ^ (r & 15))];
#pragma unroll
      for (int q = 0; q < TW; ++q) sum[q] = __builtin_fma(ai, row[c0 + (q ^ (r & 15))], sum[q]);
    }
#pragma unroll
    for (int q = 0; q < TW; ++q) tb[(w * 4 + q) * 64 + l] = sum[q];
  }
  __syncthreads();
  // (3) partial sums into registers (MFMA halves in a fixed order; the tail in wave order)
  constexpr int PER = (NBm * 256 + T - 1) / T;
  double v[PER];
#pragma unroll
  for (int m = 0; m < PER; ++m) {
    const int e = t + m * T;
    v[m] = e < NBm * 256 ? Gm[e] + red[e] : 0.0;
  }
  double tv = 0.0;
  if (t < TW * 64) {
    const int q = t >> 6, i = t & 63;
    tv = tb[q * 64 + i];
#pragma unroll
    for (int ww = 1; ww < NW; ++ww) tv = tv + tb[(ww * 4 + q) * 64 + i];
  }
  __syncthreads();
#pragma unroll
  for (int m = 0; m < PER; ++m) {
    const int e = t + m * T;
    if (e < NBm * 256) {
      const int b = e >> 8, q = (e >> 6) & 3, ll = e & 63;
      int I, J;
      r2_block_ij<PM>(b, I, J);
      const int i = 16 * I + (ll >> 4) + 4 * q, j = 16 * J + (ll & 15);
      if (I < J || i <= j) Gm[i * S + j] = v[m];
    }
  }
  // the last column block: the tail sums at rows i < p, zero elsewhere (upper part)
  for (int e = t; e < S * 16; e += T) {
    const int i = e >> 4, jj = e & 15, j = c0 + jj;
    if (i <= j && !(jj < TW && i < p)) Gm[i * S + j] = 0.0;
  }
  if (t < TW * 64) {
    const int q = t >> 6, i = t & 63;
    if (i < p && i <= c0 + q) Gm[i * S + c0 + q] = tv;
  }
  __syncthreads();
}

// r4t_gram where it applies (P16 = 4, 1 <= p - 48 <= 4, whole batches, the blocked factor), else r2_gram
template <int P16>
__device__ __forceinline__ void r2_gram_any(lds_f64* As, lds_f64* Gm, lds_f64* red, int NR, int n, int p) {
  if (P16 == 4) {
    const int NG = NR / 4, H0 = NG / 2;
    if (H0 % 13 == 0 && (NG - H0) % 13 == 0) {
      switch (p - 48) {
        case 1: r4t_gram<1>(As, Gm, red, NR, n, p); return;
        case 2: r4t_gram<2>(As, Gm, red, NR, n, p); return;
        case 3: r4t_gram<3>(As, Gm, red, NR, n, p); return;
        case 4: r4t_gram<4>(As, Gm, red, NR, n, p); return;
        default: break;
      }
    }
  }
  r2_gram<P16>(As, Gm, red, NR);
}

// ---- blocked factor (round 3): 16-column diagonal blocks on one wave, the rest on MFMA -----------
// A Gauss-Jordan factor spread over the 8 waves (round 2) paid one workgroup barrier and one
// cross-wave LDS round trip per pivot pair (~1.4k ticks per column at p = 50).  Here the chain of p pivots runs inside ONE wave on 16 x 16
// diagonal blocks with lane shuffles only, and everything else is block algebra on the matrix cores
// with three barriers per 16-column block:
//   for K = 0 .. ceil(p/16) - 1 (E starts as the identity):
//     (a) F = L_KK^-1 from the current G_KK: Gauss-Jordan on [G_KK | I] in registers of one wave
//         (lane = (row group q, column j), 4 rows each; pivot row and column by ds_bpermute, pivot by
//         readlane), row i scaled by D_i^-1/2 — no LDS, no barrier inside;
//     (b) C_IK = L_IK = G_IK F^T (I > K) and E_KJ <- F E_KJ (J < K; E_KK = F);
//     (c) G_IJ -= C_IK C_JK^T (K < J <= I, the trailing Schur complement) and E_IJ -= C_IK E_KJ
//         (I > K, J <= K); the wave that updates G_{K+1,K+1} goes straight on to (a) of K + 1.
//   E = L^-1, and W = R^-1 = E^T.
// Storage: G's trailing blocks are kept in Gm's UPPER triangle (G_IK read as G_KI^T, so every
// operand read walks 16 consecutive doubles), C_IK in Gm's lower block (I, K) and E's lower blocks
// (block-major, 256 doubles each) in the exchange area; both with the column XOR-swizzled by the
// row (element (a, b) at column b ^ a), so the MFMA operand reads of a column are bank-conflict
// free.  Columns past p are the identity (W = diag(W_p, I)).
__device__ __forceinline__ double r3_shfl(double v, int src) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_ds_bpermute(src << 2, (int)b);
  const int hi = __builtin_amdgcn_ds_bpermute(src << 2, (int)(b >> 32));
  return __longlong_as_double((long long)(unsigned)lo | ((long long)hi << 32));
}
__device__ __forceinline__ double r3_readlane(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double((long long)(unsigned)lo | ((long long)hi << 32));
}
__device__ __forceinline__ double r3_recip(double d) {
  // v_rcp_f64 + two Newton steps (measured 37.9k vs 39.3k ticks per factor against IEEE division
  // at (200, 50))
  double r = __builtin_amdgcn_rcp(d);
  r = __builtin_fma(r, __builtin_fma(-d, r, 1.0), r);
  return __builtin_fma(r, __builtin_fma(-d, r, 1.0), r);
}
__device__ __forceinline__ int r3_eb(int I, int J) { return (I * (I + 1) / 2 + J) * 256; }   // E block (I, J), J <= I

// (a): one wave; Fb = the E block (K, K) (swizzled)
template <int P16>
__device__ __forceinline__ void r3_diag_factor(const lds_f64* Gm, lds_f64* Fb, int K, int p) {
  constexpr int S = 16 * P16;
  const int l = threadIdx.x & 63, q = l >> 4, j = l & 15;
  const int kmax = p - 16 * K < 16 ? p - 16 * K : 16;   // pivots past p: identity rows
  const int jj = 16 * K + j;
  double g[4], e[4], piv[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int a = 4 * q + s, i = 16 * K + a;
    // the upper triangle of the block (the Gram writes only the upper half of G; the trailing
    // updates keep the diagonal blocks' upper half exact), mirrored below the diagonal
    const double vu = Gm[i * S + jj], vl = Gm[jj * S + i];   // always in range (i, jj < S)
    const double v = a <= j ? vu : vl;
    g[s] = (i < p && jj < p) ? v : (a == j ? 1.0 : 0.0);
    e[s] = a == j ? 1.0 : 0.0;
    piv[s] = 1.0;
  }
  // one pivot per step.  Measured alternatives at (200, 50): two pivots per step (a 2 x 2 pivot block,
  // independent reciprocals) 9.2k vs 8.8k ticks per 16-column block; the pivot row through LDS (one
  // lane group writes, all read back, wave-scope fences) 8.9k: each step is a dependent chain
  // (exchange -> reciprocal -> update of the next pivot row) of ~500 ticks however the row travels
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if (k >= kmax) continue;   // uniform (a break here keeps the loop from unrolling: runtime slot indices)
    const int kq = k >> 2, ks = k & 3;
    const double gk = r3_shfl(g[ks], 16 * kq + j);   // G[k][j]
    const double ek = r3_shfl(e[ks], 16 * kq + j);   // E[k][j]
    double ck[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) ck[s] = r3_shfl(g[s], 16 * q + k);   // G[4q + s][k]
    const double d = r3_readlane(g[ks], 16 * kq + k);                // G[k][k]
    const double inv = r3_recip(d);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int a = 4 * q + s;
      const double m = ck[s] * inv * mask01(a > k);   // 0 leaves rows <= k bitwise unchanged
      g[s] = g[s] - m * gk;
      e[s] = e[s] - m * ek;
      if (a == k) piv[s] = d;
    }
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int a = 4 * q + s;
    Fb[a * 16 + (j ^ a)] = e[s] * (1.0 / sqrt(piv[s]));
  }
}

// (b) C_IK = G_IK F^T into Gm's lower block (I, K)
template <int P16>
__device__ __forceinline__ void r3_task_C(lds_f64* Gm, const lds_f64* Fb, int I, int K) {
  constexpr int S = 16 * P16;
  const int l = threadIdx.x & 63, c = l & 15, kk = l >> 4;
  double a[4], b[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int x = 4 * s + kk;
    a[s] = Gm[(16 * K + x) * S + 16 * I + c];   // G_IK[c][x] = G_KI[x][c]
    b[s] = Fb[c * 16 + (x ^ c)];               // F^T[x][c] = F[c][x]
  }
  dbl4 acc = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[s], acc, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = kk + 4 * r;
    Gm[(16 * I + row) * S + 16 * K + (c ^ row)] = acc[r];
  }
}

// (b) E_KJ <- F E_KJ (in place)
__device__ __forceinline__ void r3_task_EF(lds_f64* Ea, int K, int J) {
  const int l = threadIdx.x & 63, c = l & 15, kk = l >> 4;
  const lds_f64* Fb = Ea + r3_eb(K, K);
  lds_f64* R = Ea + r3_eb(K, J);
  double a[4], b[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int x = 4 * s + kk;
    a[s] = Fb[c * 16 + (x ^ c)];
    b[s] = R[x * 16 + (c ^ x)];
  }
  dbl4 acc = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[s], acc, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = kk + 4 * r;
    R[row * 16 + (c ^ row)] = acc[r];
  }
}

// (c) G_JI -= C_JK C_IK^T (K < J <= I; upper storage, the diagonal block whole)
template <int P16>
__device__ __forceinline__ void r3_task_G(lds_f64* Gm, int J, int I, int K) {
  constexpr int S = 16 * P16;
  const int l = threadIdx.x & 63, c = l & 15, kk = l >> 4;
  double a[4], b[4];
  dbl4 acc;
#pragma unroll
  for (int r = 0; r < 4; ++r) acc[r] = Gm[(16 * J + kk + 4 * r) * S + 16 * I + c];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int x = 4 * s + kk;
    a[s] = -Gm[(16 * J + c) * S + 16 * K + (x ^ c)];   // -C_JK[c][x]
    b[s] = Gm[(16 * I + c) * S + 16 * K + (x ^ c)];    //  C_IK[c][x]
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[s], acc, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 4; ++r) Gm[(16 * J + kk + 4 * r) * S + 16 * I + c] = acc[r];
}

// (c) E_IJ -= C_IK E_KJ (I > K, J <= K)
template <int P16>
__device__ __forceinline__ void r3_task_R(const lds_f64* Gm, lds_f64* Ea, int I, int J, int K) {
  constexpr int S = 16 * P16;
  const int l = threadIdx.x & 63, c = l & 15, kk = l >> 4;
  lds_f64* R = Ea + r3_eb(I, J);
  const lds_f64* Ek = Ea + r3_eb(K, J);
  double a[4], b[4];
  dbl4 acc;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = kk + 4 * r;
    acc[r] = R[row * 16 + (c ^ row)];
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int x = 4 * s + kk;
    a[s] = -Gm[(16 * I + c) * S + 16 * K + (x ^ c)];   // -C_IK[c][x]
    b[s] = Ek[x * 16 + (c ^ x)];                       //  E_KJ[x][c]
  }
#pragma unroll
  for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[s], acc, 0, 0, 0);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = kk + 4 * r;
    R[row * 16 + (c ^ row)] = acc[r];
  }
}

// Gm (G, stride S, both triangles) -> Gm (W = E^T in the upper blocks, stride S); Ea: P16 (P16 + 1) / 2
// blocks of 256 doubles (the Gram's partial-sum area)
// STAMPS: the first call's sub-phases go to stamp slots 8..15 (tools/stiefel_stamps.hip only)
template <int P16, bool STAMPS = false>
__device__ __forceinline__ void r3_factor_blocked(lds_f64* Gm, lds_f64* Ea, int p) {
  constexpr int S = 16 * P16, NB = P16 * (P16 + 1) / 2;
  const int t = threadIdx.x, w = t >> 6;
  if (STAMPS) ST_STAMP(8);
  for (int e = t; e < NB * 256; e += T) {   // E's off-diagonal blocks start at zero (the diagonal ones are written by (a))
    const int blk = e >> 8;
    bool diag = false;
#pragma unroll
    for (int I = 0; I < P16; ++I) diag = diag || blk == I * (I + 3) / 2;
    if (!diag) Ea[e] = 0.0;
  }
  if (w == 0) r3_diag_factor<P16>(Gm, Ea + r3_eb(0, 0), 0, p);
  if (STAMPS) ST_STAMP(9);
  __syncthreads();
  for (int K = 0; K < P16; ++K) {
    const int nC = P16 - 1 - K;
    for (int task = w; task < nC + K; task += NW) {   // (b)
      if (task < nC) r3_task_C<P16>(Gm, Ea + r3_eb(K, K), K + 1 + task, K);
      else r3_task_EF(Ea, K, task - nC);
    }
    __syncthreads();
    if (STAMPS && K < 2) ST_STAMP(10 + 3 * K);
    if (K == P16 - 1) break;
    if (w == 0) {   // (c) G_{K+1,K+1}, then (a) of K + 1
      r3_task_G<P16>(Gm, K + 1, K + 1, K);
      r3_diag_factor<P16>(Gm, Ea + r3_eb(K + 1, K + 1), K + 1, p);
      if (STAMPS && K < 2) ST_STAMP(11 + 3 * K);
    } else {
      const int m = P16 - 1 - K;             // trailing block rows
      const int nG = m * (m + 1) / 2 - 1;    // pairs (J, I), K < J <= I, without (K + 1, K + 1)
      const int nR = m * (K + 1);
      for (int task = w - 1; task < nG + nR; task += NW - 1) {
        if (task < nG) {
          int u = task + 1, J = K + 1;
          while (u >= P16 - J) {   // row J of the pair triangle holds P16 - J pairs
            u -= P16 - J;
            ++J;
          }
          r3_task_G<P16>(Gm, J, J + u, K);
        } else {
          const int u = task - nG;
          r3_task_R<P16>(Gm, Ea, K + 1 + u / (K + 1), u % (K + 1), K);
        }
      }
    }
    __syncthreads();
    if (STAMPS && K == 0) ST_STAMP(12);
  }
  for (int e = t; e < NB * 256; e += T) {   // W[16 J + b][16 I + a] = E_IJ[a][b]; consecutive lanes: consecutive a
    const int blk = e >> 8, b = (e >> 4) & 15, a = e & 15;
    int I = 0;
#pragma unroll
    for (int q = 1; q < P16; ++q) I += blk >= q * (q + 1) / 2;
    const int J = blk - I * (I + 1) / 2;
    Gm[(16 * J + b) * S + 16 * I + a] = Ea[blk * 256 + a * 16 + (b ^ a)];
  }
  __syncthreads();
  if (STAMPS) ST_STAMP(15);
}

// The second CholeskyQR pass factors G2 = Q1^T Q1 = I + D with D at the rounding level of the first
// pass (~kappa(A)^2 eps).  Then L2 = I + N with N = tril(D, -1) + diag(D) / 2 up to O(D^2), and
// W2 = R2^-1 = (L2^-1)^T = I - N^T up to O(D^2): elementwise, no dependent chain.  Used when
// max |D_ij| <= FO_MAX, where the dropped O(D^2) terms (<= 1e-20) sit far below the rounding of
// the full factor; otherwise (a badly conditioned A) the exact factor runs.  Gm: G2 in, W2 out
// (stride S, W2[i][j] at i S + j, upper triangular, identity past p).  Returns the uniform verdict.
constexpr double FO_MAX = 1e-10;

template <int P16>
__device__ __forceinline__ bool r2_inverse_first_order(lds_f64* Gm, lds_f64* red, int p) {
  constexpr int S = 16 * P16;
  const int t = threadIdx.x;
  double dev = 0.0;
  for (int e = t; e < S * S; e += T) {   // the upper triangle (the Gram writes only that half)
    const int i = e / S, j = e - (e / S) * S;
    if (i <= j && j < p) dev = fmax(dev, fabs(Gm[e] - (i == j ? 1.0 : 0.0)));
  }
  for (int off = 32; off > 0; off >>= 1) dev = fmax(dev, __shfl_xor(dev, off));
  if ((t & 63) == 0) red[t >> 6] = dev;
  __syncthreads();
  double mx = red[0];
#pragma unroll
  for (int w = 1; w < NW; ++w) mx = fmax(mx, red[w]);
  if (!(mx <= FO_MAX)) return false;   // NaN-safe: the exact factor decides then
  for (int e = t; e < S * S; e += T) {
    const int i = e / S, j = e - (e / S) * S;
    double v;
    if (i >= p || j >= p) v = (i == j) ? 1.0 : 0.0;
    else if (i == j) v = 1.0 - 0.5 * (Gm[e] - 1.0);
    else v = (i < j) ? -Gm[e] : 0.0;
    Gm[e] = v;   // every thread reads only the element it writes
  }
  __syncthreads();
  return true;
}

// Q = A W (W upper triangular): wave w owns the 16-row blocks R = w, w + 8, ...; FINAL writes Q to
// global memory, otherwise Q overwrites A in LDS (a wave writes only the rows it read)
// KSL: k steps of the last 16-column block that hold columns of A (ceil((p - 16 (P16 - 1)) / 4)): a
// template parameter, so no MFMA sits behind a per-step branch
// (Dealing the last NRB % 8 row blocks as (row block, column block) units in a snake over the waves,
// so the SIMDs get 123 instead of 148 MFMAs at (200, 50), measured 12.5k vs 12.2k ticks per apply:
// not kept; profiles/r3_stiefel_apply_snake_balance_stamps.jsonl)
template <int P16, bool FINAL, int KSL>
__device__ __forceinline__ void r2_apply_k(lds_f64* As, const lds_f64* Wt, int NR, int n, int p, double* out) {
  constexpr int S = 16 * P16;
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6, c = l & 15, kk = l >> 4;
  double wf[P16][P16][4];
#pragma unroll
  for (int K = 0; K < P16; ++K)
#pragma unroll
    for (int J = K; J < P16; ++J)
#pragma unroll
      for (int s = 0; s < 4; ++s) wf[K][J][s] = Wt[(16 * K + 4 * s + kk) * S + 16 * J + c];
  for (int R = w; R < NR / 16; R += NW) {
    double af[P16][4];
    const int row = 16 * R + c;
#pragma unroll
    for (int K = 0; K < P16; ++K)
#pragma unroll
      for (int s = 0; s < 4; ++s) af[K][s] = As[row * S + ((16 * K + 4 * s + kk) ^ c)];
    dbl4 acc[P16];
#pragma unroll
    for (int J = 0; J < P16; ++J) acc[J] = dbl4{0.0, 0.0, 0.0, 0.0};
    // (K, s) outer, J inner: consecutive MFMAs feed different accumulators; A's columns past p are
    // zero, so k steps past p are skipped
#pragma unroll
    for (int K = 0; K < P16; ++K)
#pragma unroll
      for (int s = 0; s < (K == P16 - 1 ? KSL : 4); ++s) {
#pragma unroll
        for (int J = K; J < P16; ++J) acc[J] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[K][s], wf[K][J][s], acc[J], 0, 0, 0);
      }
#pragma unroll
    for (int J = 0; J < P16; ++J)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = 16 * R + kk + 4 * q, col = 16 * J + c;
        if (FINAL) {
          if (r < n && col < p) out[(int64_t)r * p + col] = acc[J][q];
        } else {
          As[r * S + (col ^ (r & 15))] = acc[J][q];
        }
      }
  }
  __syncthreads();
}

template <int P16, bool FINAL>
__device__ __forceinline__ void r2_apply(lds_f64* As, const lds_f64* Wt, int NR, int n, int p, double* out) {
  switch ((p - 16 * (P16 - 1) + 3) / 4) {
    case 1: r2_apply_k<P16, FINAL, 1>(As, Wt, NR, n, p, out); break;
    case 2: r2_apply_k<P16, FINAL, 2>(As, Wt, NR, n, p, out); break;
    case 3: r2_apply_k<P16, FINAL, 3>(As, Wt, NR, n, p, out); break;
    default: r2_apply_k<P16, FINAL, 4>(As, Wt, NR, n, p, out); break;
  }
}

// the second pass's exact factor (rare: only when Q1 is not orthonormal to 1e-10) as a call, so its
// code does not sit inline in the kernel (the kernel is ~54 KB with it inlined)
template <int P16>
__device__ __noinline__ void r3_factor_blocked_call(lds_f64* Gm, lds_f64* Ea, int p) {
  r3_factor_blocked<P16>(Gm, Ea, p);
}

template <int P16>
__global__ void __launch_bounds__(T) k_st_retr2(int n, int p, int64_t stride, const double* __restrict__ X,
                                                const double* __restrict__ U, double* out) {   // out may alias X or U (all reads precede the first write)
  constexpr int S = 16 * P16, UL = 8;
  extern __shared__ double lds[];
  const int NR = (n + 15) & ~15;
  lds_f64* As = (lds_f64*)lds;
  lds_f64* Gm = As + NR * S;
  lds_f64* red = Gm + S * S;
  const int t = threadIdx.x;
  const int64_t o = (int64_t)blockIdx.x * stride;
  ST_STAMP(0);
  // (loading the second row half while the first half's Gram tasks run measured slower: 35.1k vs
  // 32.6k ticks for load + Gram)
  const int tot = NR * S;
  for (int e0 = 0; e0 < tot; e0 += T * UL) {
    double v[UL];
#pragma unroll
    for (int u = 0; u < UL; ++u) {
      const int e = e0 + u * T + t;
      const int r = e / S, col = e - (e / S) * S;
      const bool ok = r < n && col < p;
      const int64_t gi = o + (ok ? (int64_t)r * p + col : 0);
      v[u] = (X[gi] + U[gi]) * mask01(ok);
    }
#pragma unroll
    for (int u = 0; u < UL; ++u) {
      const int e = e0 + u * T + t;
      const int r = e / S, col = e - (e / S) * S;
      if (e < tot) As[r * S + (col ^ (r & 15))] = v[u];
    }
  }
  __syncthreads();
  ST_STAMP(1);
  r2_gram_any<P16>(As, Gm, red, NR, n, p);
  ST_STAMP(2);
#ifdef ST_STAMPS
  r3_factor_blocked<P16, true>(Gm, red, p);
#else
  r3_factor_blocked<P16>(Gm, red, p);
#endif
  ST_STAMP(3);
  r2_apply<P16, false>(As, Gm, NR, n, p, out + o);
  ST_STAMP(4);
  r2_gram_any<P16>(As, Gm, red, NR, n, p);
  ST_STAMP(5);
  if (!r2_inverse_first_order<P16>(Gm, red, p)) r3_factor_blocked_call<P16>(Gm, red, p);
  ST_STAMP(6);
  r2_apply<P16, true>(As, Gm, NR, n, p, out + o);
  ST_STAMP(7);
}

__global__ void __launch_bounds__(T) k_st_inner(int n, int p, int64_t stride, const double* U, const double* V, double* out) {
  __shared__ double red[T / 64];
  const int64_t o = (int64_t)blockIdx.x * stride;
  double s = 0.0;
  for (int e = threadIdx.x; e < n * p; e += T) s = s + U[o + e] * V[o + e];
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double r = red[0];
    for (int i = 1; i < T / 64; ++i) r = r + red[i];
    out[blockIdx.x] = r;
  }
}

}  // namespace riptrm_stiefel

using namespace riptrm_stiefel;

constexpr int R2_LDS_MAX = 160 * 1024;   // LDS per workgroup on gfx950

static int st_check(riptrm_ctx* c, int32_t n, int32_t p, int32_t batch, int64_t stride) {
  if (n < 1 || p < 1 || p > PMAX || p > n || batch < 1 || stride < (int64_t)n * p)
    return fail(c, RIPTRM_E_ARG, "stiefel: need 1 <= p <= min(n, 64), batch >= 1, stride >= n*p");
  HIPCHK(c, hipSetDevice(c->device));
  static bool attr[64] = {};   // per device: dynamic LDS above the 64 KiB default
  if (c->device < 0 || c->device >= 64 || !attr[c->device]) {
    const int shm = (int)(LDS_DOUBLES * sizeof(double));
    const void* fns[] = {(const void*)k_st_proj<1>, (const void*)k_st_proj<2>, (const void*)k_st_proj<3>,
                         (const void*)k_st_proj<4>, (const void*)k_st_e2rh<1>, (const void*)k_st_e2rh<2>,
                         (const void*)k_st_e2rh<3>, (const void*)k_st_e2rh<4>};
    for (const void* f : fns) HIPCHK(c, hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, shm));
    HIPCHK(c, hipFuncSetAttribute((const void*)k_st_retr_r, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)(LDS_DOUBLES_R * sizeof(double))));
    const void* fr[] = {(const void*)k_st_retr2<1>, (const void*)k_st_retr2<2>, (const void*)k_st_retr2<3>,
                        (const void*)k_st_retr2<4>, (const void*)k_st_proj3<4>, (const void*)k_st_proj4<4>};
    for (const void* f : fr) HIPCHK(c, hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, R2_LDS_MAX));
    if (c->device >= 0 && c->device < 64) attr[c->device] = true;
  }
  return RIPTRM_OK;
}

constexpr size_t SHM = LDS_DOUBLES * sizeof(double);

// LDS bytes of k_st_retr2 at (n, p), 0 if the point does not fit (the round-1 kernel runs then)
static size_t retr2_lds_bytes(int n, int p) {
  const int NR = ((n + 15) / 16) * 16;
  int d = 0;
  switch ((p + 15) / 16) {
    case 1: d = r2_lds_doubles_nr<1>(NR); break;
    case 2: d = r2_lds_doubles_nr<2>(NR); break;
    case 3: d = r2_lds_doubles_nr<3>(NR); break;
    default: d = r2_lds_doubles_nr<4>(NR); break;
  }
  const size_t b = (size_t)d * sizeof(double);
  return b <= (size_t)R2_LDS_MAX ? b : 0;
}

// RIPTRM_STIEFEL_RETR=r1 forces the round-1 retraction kernel (A/B measurements)
static bool retr_force_r1() {
  const char* e = getenv("RIPTRM_STIEFEL_RETR");
  return e && e[0] == 'r' && e[1] == '1';
}
constexpr size_t SHM_R = LDS_DOUBLES_R * sizeof(double);

// k_st_proj3 (point resident in LDS) for 49 <= p <= 64 when the point fits 160 KB, n p is even (16-B
// copies) and the stride keeps points 16-B aligned; RIPTRM_STIEFEL_PROJ=r2 forces k_st_proj (A/B)
static bool proj3_ok(int n, int p, int64_t stride) {
  const char* e = getenv("RIPTRM_STIEFEL_PROJ");
  if (e && e[0] == 'r' && e[1] == '2') return false;
  return (p + 15) / 16 == 4 && (n * p) % 2 == 0 && stride % 2 == 0 && (n + 15) / 16 <= 14 &&
         p3_lds_doubles(n, p, 4) <= P3_LDS_DOUBLES;
}

// kernels are specialised on ceil(p / 16) (the 16-column blocks), so no operand load sits behind
// a runtime branch
#define ST_LAUNCH(K, p, ...)                                                                              \
  switch (((p) + 15) / 16) {                                                                             \
    case 1: hipLaunchKernelGGL(K<1>, __VA_ARGS__); break;                                              \
    case 2: hipLaunchKernelGGL(K<2>, __VA_ARGS__); break;                                              \
    case 3: hipLaunchKernelGGL(K<3>, __VA_ARGS__); break;                                              \
    default: hipLaunchKernelGGL(K<4>, __VA_ARGS__); break;                                             \
  }

extern "C" {

int riptrm_stiefel_inner(riptrm_ctx* ctx, int32_t n, int32_t p, int32_t batch, int64_t stride, const double* X,
                         const double* U, const double* V, double* out) {
  if (!ctx) return RIPTRM_E_ARG;
  if (!U || !V || !out) return fail(ctx, RIPTRM_E_ARG, "stiefel_inner: null pointer");
  (void)X;
  int rc = st_check(ctx, n, p, batch, stride);
  if (rc) return rc;
  hipLaunchKernelGGL(k_st_inner, dim3(batch), dim3(T), 0, ctx->stream, n, p, stride, U, V, out);
  HIPCHK(ctx, hipGetLastError());
  return RIPTRM_OK;
}

int riptrm_stiefel_proj(riptrm_ctx* ctx, int32_t n, int32_t p, int32_t batch, int64_t stride, const double* X,
                        const double* U, double* out) {
  if (!ctx) return RIPTRM_E_ARG;
  if (!X || !U || !out || out == X) return fail(ctx, RIPTRM_E_ARG, "stiefel_proj: bad pointer (out must not alias X)");
  int rc = st_check(ctx, n, p, batch, stride);
  if (rc) return rc;
  if (proj3_ok(n, p, stride)) {
    const size_t shm = (size_t)p3_lds_doubles(n, p, 4) * sizeof(double);
    const int ncu = ctx->ncu > 0 ? ctx->ncu : 256;
    // (a Gram that left the 2-column tail of p = 50 to the VALU and split the 9 remaining MFMA blocks
    // over two k halves measured slower: 29.98 vs 27.62 us at 256 points, 246 vs 191 us at 2048)
    const char* e = getenv("RIPTRM_STIEFEL_PROJ");   // "p3": one point per workgroup always (A/B)
    if (batch > ncu && !(e && e[0] == 'p' && e[1] == '3'))   // several points per CU: the prefetching loop
      hipLaunchKernelGGL(k_st_proj4<4>, dim3(ncu), dim3(T), shm, ctx->stream, n, p, stride, batch, X, U, out);
    else
      hipLaunchKernelGGL(k_st_proj3<4>, dim3(batch), dim3(T), shm, ctx->stream, n, p, stride, X, U, out);
    HIPCHK(ctx, hipGetLastError());
    return RIPTRM_OK;
  }
  ST_LAUNCH(k_st_proj, p, dim3(batch), dim3(T), SHM, ctx->stream, n, p, stride, X, U, out);
  HIPCHK(ctx, hipGetLastError());
  return RIPTRM_OK;
}

int riptrm_stiefel_retr(riptrm_ctx* ctx, int32_t n, int32_t p, int32_t batch, int64_t stride, const double* X,
                        const double* U, double* out) {
  if (!ctx) return RIPTRM_E_ARG;
  if (!X || !U || !out) return fail(ctx, RIPTRM_E_ARG, "stiefel_retr: null pointer");
  int rc = st_check(ctx, n, p, batch, stride);
  if (rc) return rc;
  const size_t shm2 = retr_force_r1() ? 0 : retr2_lds_bytes(n, p);
  if (shm2) {
    ST_LAUNCH(k_st_retr2, p, dim3(batch), dim3(T), shm2, ctx->stream, n, p, stride, X, U, out);
  } else {
    hipLaunchKernelGGL(k_st_retr_r, dim3(batch), dim3(T), SHM_R, ctx->stream, n, p, stride, X, U, out);
  }
  HIPCHK(ctx, hipGetLastError());
  return RIPTRM_OK;
}

int riptrm_stiefel_ehess2rhess(riptrm_ctx* ctx, int32_t n, int32_t p, int32_t batch, int64_t stride, const double* X,
                               const double* G, const double* H, const double* U, double* out) {
  if (!ctx) return RIPTRM_E_ARG;
  if (!X || !G || !H || !U || !out || out == X || out == U)
    return fail(ctx, RIPTRM_E_ARG, "stiefel_ehess2rhess: bad pointer (out must not alias X or U)");
  int rc = st_check(ctx, n, p, batch, stride);
  if (rc) return rc;
  ST_LAUNCH(k_st_e2rh, p, dim3(batch), dim3(T), SHM, ctx->stream, n, p, stride, X, G, H, U, out);
  HIPCHK(ctx, hipGetLastError());
  return RIPTRM_OK;
}

}  // extern "C"
