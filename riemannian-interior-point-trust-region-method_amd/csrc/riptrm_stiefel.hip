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
// rounding for full-rank A.
#include <hip/hip_runtime.h>
#include <math.h>
#include "riptrm_ctx.h"

namespace riptrm_stiefel {

#pragma clang fp contract(off)

constexpr int NW = 8;          // waves per workgroup (one workgroup per point)
constexpr int T = NW * 64;     // threads per workgroup
constexpr int PMAX = RIPTRM_STIEFEL_PMAX;
constexpr int GMAX = 8;        // 4-row groups per wave per streamed chunk (8 waves x 32 rows = 256 rows)
constexpr int NBLK = 10;       // upper-triangular 16 x 16 blocks of a p x p matrix at p <= 64

// LDS (dynamic): M and L are p x p (padded stride PS <= 64), red holds the wave partials of the
// Gram reduction tree (NW / 2 waves x NBLK blocks x 256 doubles).
// address-space-3 pointers: ds_read / ds_write, not flat accesses through generic pointers
typedef __attribute__((address_space(3))) double lds_f64;
struct Smem {
  lds_f64* M;     // p x p (Gram / sym / R^-1)
  lds_f64* L;     // Cholesky factor
  lds_f64* red;
};
constexpr int LDS_DOUBLES = 2 * PMAX * PMAX + (NW / 2) * NBLK * 256;

__device__ __forceinline__ Smem smem_of(double* base_generic) {
  lds_f64* base = (lds_f64*)base_generic;
  return Smem{base, base + PMAX * PMAX, base + 2 * PMAX * PMAX};
}

typedef double dbl4 __attribute__((ext_vector_type(4)));

// Small p x p matrices live in LDS with the padded row stride PS = 16 ceil(p / 16) and zeros
// outside p x p, so the MFMA loops read operands without bounds tests (no divergent branches).
__device__ __forceinline__ int pstride(int p) { return ((p + 15) / 16) * 16; }

// sm.M <- sym(A^T B) = (A^T B + B^T A) / 2 for n x p row-major A, B, exactly symmetric, on the fp64
// matrix cores.  Every wave streams its own rows straight into registers — each lane loads the
// 4 x 16 operand fragments of v_mfma_f64_16x16x4_f64 for GMAX 4-row groups and all p columns at
// once (one memory latency per 256-row chunk, all loads of the workgroup in flight together) —
// and accumulates the upper-triangular blocks S_IJ = A_I^T B_J + B_I^T A_J (I <= J).  The eight
// wave partials meet in a fixed LDS tree (bitwise deterministic); wave 0 writes S / 2.
__device__ __forceinline__ void gram_sym(Smem& sm, const double* __restrict__ A, const double* __restrict__ B,
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

// out = C + sgn * A K (K = sm.M, p x p, padded) on the matrix cores.  A wave owns 16-row blocks
// of the output and computes ALL their column blocks before writing, reading its A rows only:
// out may alias A or C.  C = nullptr gives out = A K.
__device__ __forceinline__ void update(Smem& sm, const double* A, const double* C, double sgn, double* out,
                                       int n, int p) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int P16 = (p + 15) / 16, R16 = (n + 15) / 16, PS = P16 * 16;
  const int c = l & 15, kk = l >> 4;
  const int P4 = (p + 3) / 4;
  for (int I = w; I < R16; I += NW) {
    dbl4 acc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = dbl4{0.0, 0.0, 0.0, 0.0};
    const int arow = I * 16 + c;
    double ar[PMAX / 4];   // this lane's A operands for every k step, loaded at once
#pragma unroll
    for (int k4 = 0; k4 < PMAX / 4; ++k4) {
      const int k = k4 * 4 + kk;
      const bool ok = k4 < P4 && arow < n && k < p;
      const double v = A[ok ? (int64_t)arow * p + k : 0];
      ar[k4] = ok ? v : 0.0;
    }
#pragma unroll
    for (int J = 0; J < 4; ++J) {
      if (J < P16) {
        const lds_f64* pb = sm.M + kk * PS + J * 16 + c;
#pragma unroll
        for (int k4 = 0; k4 < PMAX / 4; ++k4)
          if (k4 < P4) acc[J] = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[k4], pb[k4 * 4 * PS], acc[J], 0, 0, 0);
      }
    }
    // every lane of the wave has read its A rows before any lane writes them
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int J = 0; J < 4; ++J) {
      if (J < P16) {
        const int j = J * 16 + c;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int i = I * 16 + kk + 4 * g;
          if (i < n && j < p) {
            const int64_t e = (int64_t)i * p + j;
            out[e] = C ? C[e] + sgn * acc[J][g] : acc[J][g];
          }
        }
      }
    }
  }
  __syncthreads();
}

__global__ void __launch_bounds__(T) k_st_proj(int n, int p, int64_t stride, const double* X, const double* U, double* out) {
  extern __shared__ double lds[];
  Smem sm = smem_of(lds);
  const int64_t o = (int64_t)blockIdx.x * stride;
  gram_sym(sm, X + o, U + o, n, p);
  update(sm, X + o, U + o, -1.0, out + o, n, p);
}

__global__ void __launch_bounds__(T) k_st_e2rh(int n, int p, int64_t stride, const double* X, const double* G,
                                               const double* H, const double* U, double* out) {
  extern __shared__ double lds[];
  Smem sm = smem_of(lds);
  const int64_t o = (int64_t)blockIdx.x * stride;
  gram_sym(sm, X + o, G + o, n, p);                // sym(X^T G)
  update(sm, U + o, H + o, -1.0, out + o, n, p);   // W = H - U sym(X^T G) into out
  gram_sym(sm, X + o, out + o, n, p);              // sym(X^T W)
  update(sm, X + o, out + o, -1.0, out + o, n, p);  // P_X(W)
}

// sm.M (SPD p x p, stride PS) -> sm.L = lower Cholesky factor (A^T A = L L^T, diag > 0)
__device__ __forceinline__ void chol_lower(Smem& sm, int p) {
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
__device__ __forceinline__ void rows_solve(const Smem& sm, double* A, int n, int p) {
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

__global__ void __launch_bounds__(T) k_st_retr(int n, int p, int64_t stride, const double* X, const double* U, double* out) {
  extern __shared__ double lds[];
  Smem sm = smem_of(lds);
  const int64_t o = (int64_t)blockIdx.x * stride;
  double* A = out + o;
  for (int e = threadIdx.x; e < n * p; e += T) A[e] = X[o + e] + U[o + e];
  __syncthreads();
  for (int pass = 0; pass < 2; ++pass) {   // CholeskyQR2
    gram_sym(sm, A, A, n, p);                // (A^T A + A^T A) / 2 = A^T A exactly
    chol_lower(sm, p);
    rows_solve(sm, A, n, p);                 // A R^-1
  }
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

static int st_check(riptrm_ctx* c, int32_t n, int32_t p, int32_t batch, int64_t stride) {
  if (n < 1 || p < 1 || p > PMAX || p > n || batch < 1 || stride < (int64_t)n * p)
    return fail(c, RIPTRM_E_ARG, "stiefel: need 1 <= p <= min(n, 64), batch >= 1, stride >= n*p");
  HIPCHK(c, hipSetDevice(c->device));
  static bool attr[64] = {};   // per device: dynamic LDS above the 64 KiB default
  if (c->device < 0 || c->device >= 64 || !attr[c->device]) {
    const int shm = (int)(LDS_DOUBLES * sizeof(double));
    HIPCHK(c, hipFuncSetAttribute((const void*)k_st_proj, hipFuncAttributeMaxDynamicSharedMemorySize, shm));
    HIPCHK(c, hipFuncSetAttribute((const void*)k_st_e2rh, hipFuncAttributeMaxDynamicSharedMemorySize, shm));
    HIPCHK(c, hipFuncSetAttribute((const void*)k_st_retr, hipFuncAttributeMaxDynamicSharedMemorySize, shm));
    if (c->device >= 0 && c->device < 64) attr[c->device] = true;
  }
  return RIPTRM_OK;
}

constexpr size_t SHM = LDS_DOUBLES * sizeof(double);

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
  hipLaunchKernelGGL(k_st_proj, dim3(batch), dim3(T), SHM, ctx->stream, n, p, stride, X, U, out);
  HIPCHK(ctx, hipGetLastError());
  return RIPTRM_OK;
}

int riptrm_stiefel_retr(riptrm_ctx* ctx, int32_t n, int32_t p, int32_t batch, int64_t stride, const double* X,
                        const double* U, double* out) {
  if (!ctx) return RIPTRM_E_ARG;
  if (!X || !U || !out) return fail(ctx, RIPTRM_E_ARG, "stiefel_retr: null pointer");
  int rc = st_check(ctx, n, p, batch, stride);
  if (rc) return rc;
  hipLaunchKernelGGL(k_st_retr, dim3(batch), dim3(T), SHM, ctx->stream, n, p, stride, X, U, out);
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
  hipLaunchKernelGGL(k_st_e2rh, dim3(batch), dim3(T), SHM, ctx->stream, n, p, stride, X, G, H, U, out);
  HIPCHK(ctx, hipGetLastError());
  return RIPTRM_OK;
}

}  // extern "C"
