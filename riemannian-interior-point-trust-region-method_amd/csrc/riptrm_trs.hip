// riptrm_trs.hip — batched TRSgep (src/solver/RIPTRM.py:218-299) behind the C-ABI: one
// 256-thread workgroup per subproblem runs riptrm_trs::trs_solve (riptrm_trs.h) on its matrix
// staged in LDS.  The same device solver is what the NonnegPCA state machine and the
// StableIdentification kernel call in-kernel for TRS_solver = 'Exact_RepMat'.
#include <hip/hip_runtime.h>
#include "riptrm_ctx.h"
#include "riptrm_trs.h"

namespace riptrm_trs {

constexpr int TRS_THREADS = 256;

__global__ void __launch_bounds__(TRS_THREADS) k_trs_gep(int dim, const double* __restrict__ A, int64_t lda,
                                                         int64_t a_stride, const double* __restrict__ a, int64_t ldv,
                                                         const double* __restrict__ Delta, double tolhc, double* x,
                                                         double* lam1, int32_t* kind, double* mineig) {
  extern __shared__ double lds[];
  __shared__ double red[2 * (TRS_THREADS / 64)];
  const int b = blockIdx.x;
  Work w = make_work(lds, dim);
  Blk<TRS_THREADS> B(red);
  const double* Ab = A + (int64_t)b * a_stride;
  for (int e = threadIdx.x; e < dim * dim; e += TRS_THREADS) {
    const int i = e / dim, j = e - i * dim;
    w.A[i * w.lda + j] = Ab[(int64_t)i * lda + j];
  }
  for (int i = threadIdx.x; i < dim; i += TRS_THREADS) w.a[i] = a[(int64_t)b * ldv + i];
  __syncthreads();
  const Result r = trs_solve<TRS_THREADS>(B, w, Delta[b], tolhc);
  for (int i = threadIdx.x; i < dim; i += TRS_THREADS) x[(int64_t)b * ldv + i] = w.x[i];
  double mn = INFINITY;
  for (int i = threadIdx.x; i < dim; i += TRS_THREADS) mn = fmin(mn, w.ev[i]);
  mn = B.min(mn);
  if (threadIdx.x == 0) {
    lam1[b] = r.lam1;
    kind[b] = RIPTRM_TRS_BOUNDARY + r.kind;
    if (mineig) mineig[b] = mn;
  }
}

}  // namespace riptrm_trs

extern "C" int riptrm_trs_gep(riptrm_ctx* ctx, int32_t dim, int32_t batch, const double* A, int64_t lda,
                              int64_t a_stride, const double* a, int64_t ldv, const double* Delta, double tolhardcase,
                              double* x, double* lam1, int32_t* kind, double* mineig) {
  using namespace riptrm_trs;
  if (!ctx) return RIPTRM_E_ARG;
  if (dim < 1) return fail(ctx, RIPTRM_E_ARG, "trs_gep: dim must be >= 1");
  if (batch < 0 || lda < dim || ldv < dim || (batch > 1 && a_stride < (int64_t)dim * lda))
    return fail(ctx, RIPTRM_E_ARG, "trs_gep: bad batch / lda / a_stride / ldv");
  if (batch == 0) return RIPTRM_OK;
  if (!A || !a || !Delta || !x || !lam1 || !kind) return fail(ctx, RIPTRM_E_ARG, "trs_gep: null pointer");
  HIPCHK(ctx, hipSetDevice(ctx->device));
  if (dim > DIM_MAX)   // HBM-resident matrix, rocSOLVER eigendecomposition (riptrm_trs_big.hip)
    return riptrm_big_trs_gep(ctx, dim, batch, A, lda, a_stride, a, ldv, Delta, tolhardcase, x, lam1, kind, mineig);
  const size_t shm = (size_t)work_doubles(dim) * sizeof(double);
  HIPCHK(ctx, hipFuncSetAttribute((const void*)k_trs_gep, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm));
  hipLaunchKernelGGL(k_trs_gep, dim3(batch), dim3(TRS_THREADS), shm, ctx->stream, (int)dim, A, lda, a_stride, a, ldv,
                     Delta, tolhardcase, x, lam1, kind, mineig);
  HIPCHK(ctx, hipGetLastError());
  return RIPTRM_OK;
}
