// trs_probe.hip — latency probe of the device TRS pieces (riptrm_trs.h) on one workgroup:
// device wall-clock (100 MHz) around jacobi (with / without eigenvectors) and trs_solve.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I<csrc> tools/trs_probe.hip -o trs_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define RIPTRM_TRS_PROBE 1
#include "riptrm_trs.h"

using namespace riptrm_trs;
constexpr int NT = 256;

__global__ void probe(int dim, const double* A, const double* a, double Delta, double* out) {
  extern __shared__ double lds[];
  __shared__ double red[2 * (NT / 64)];
  Work w = make_work(lds, dim);
  Blk<NT> B(red);
  auto load = [&]() {
    for (int e = threadIdx.x; e < dim * dim; e += NT) w.A[(e / dim) * w.lda + e % dim] = A[e];
    for (int i = threadIdx.x; i < dim; i += NT) w.a[i] = a[i];
    __syncthreads();
  };
  load();
  double t0 = (double)wall_clock64();
  jacobi<NT>(B, w, true);
  double t1 = (double)wall_clock64();
  load();
  double t2 = (double)wall_clock64();
  jacobi<NT>(B, w, false);
  double t3 = (double)wall_clock64();
  load();
  double t4 = (double)wall_clock64();
  Result r = trs_solve<NT>(B, w, Delta, 1e-8);
  double t5 = (double)wall_clock64();
  if (threadIdx.x == 0) {
    out[0] = (t1 - t0) * 10.0;   // ns
    out[1] = (t3 - t2) * 10.0;
    out[2] = (t5 - t4) * 10.0;
    out[3] = r.kind;
  }
}

int main(int argc, char** argv) {
  for (int dim : {16, 40, 49, 96}) {
    std::vector<double> A(dim * dim), a(dim);
    srand(dim);
    for (int i = 0; i < dim; ++i)
      for (int j = 0; j <= i; ++j) A[i * dim + j] = A[j * dim + i] = (rand() / (double)RAND_MAX) - 0.5;
    for (int i = 0; i < dim; ++i) a[i] = (rand() / (double)RAND_MAX) - 0.5;
    double *dA, *da, *dout;
    hipMalloc(&dA, 8 * dim * dim);
    hipMalloc(&da, 8 * dim);
    hipMalloc(&dout, 8 * 4);
    hipMemcpy(dA, A.data(), 8 * dim * dim, hipMemcpyHostToDevice);
    hipMemcpy(da, a.data(), 8 * dim, hipMemcpyHostToDevice);
    const size_t shm = (size_t)work_doubles(dim) * 8;
    hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    double out[4];
    for (int rep = 0; rep < 2; ++rep) {
      hipLaunchKernelGGL(probe, dim3(1), dim3(NT), shm, 0, dim, dA, da, 0.5, dout);
      hipMemcpy(out, dout, 32, hipMemcpyDeviceToHost);
    }
    double pr[96];
    hipMemcpyFromSymbol(pr, HIP_SYMBOL(g_probe), sizeof(pr));
    printf("sweeps(last trs_solve jacobi) %.0f:", pr[80]);
    for (int k = 0; k <= (int)pr[80] && k < 40; ++k) printf(" %.1e", pr[2 * k] / pr[2 * k + 1]);
    printf("\n  cycles per round: rot %.0f cols %.0f rows %.0f fix %.0f (rounds %.0f)\n", pr[84] / pr[88], pr[85] / pr[88],
           pr[86] / pr[88], pr[87] / pr[88], pr[88]);
    double z[16] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(g_probe), z, sizeof(z), 84 * sizeof(double));
    printf("{\"dim\": %d, \"jacobi_vec_us\": %.1f, \"jacobi_val_us\": %.1f, \"trs_solve_us\": %.1f, \"kind\": %.0f}\n", dim,
           out[0] / 1e3, out[1] / 1e3, out[2] / 1e3, out[3]);
    hipFree(dA); hipFree(da); hipFree(dout);
  }
  return 0;
}
