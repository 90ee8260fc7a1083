// stiefel_stamps.hip — phase timing of the Stiefel kernels (diagnostic build, s_memtime stamps).
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I<pkg>/csrc -I include tools/stiefel_stamps.hip
// Runs k_st_proj / k_st_retr_r / k_st_retr2 at (n, p, batch) on random data and prints, per phase, the median
// over workgroups of the stamp deltas (s_memtime ticks) and the kernel's event time.
#define ST_STAMPS 1
#include "riptrm_stiefel.hip"
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 200, p = argc > 2 ? atoi(argv[2]) : 50, B = argc > 3 ? atoi(argv[3]) : 256;
  const size_t N = (size_t)B * n * p;
  std::vector<double> h(N);
  srand(7);
  for (auto& v : h) v = (double)rand() / RAND_MAX - 0.5;
  double *X, *U, *O;
  long long* st;
  CK(hipMalloc(&X, N * 8));
  CK(hipMalloc(&U, N * 8));
  CK(hipMalloc(&O, N * 8));
  CK(hipMalloc(&st, (size_t)B * 16 * 8));
  CK(hipMemcpy(X, h.data(), N * 8, hipMemcpyHostToDevice));
  for (auto& v : h) v *= 0.01;
  CK(hipMemcpy(U, h.data(), N * 8, hipMemcpyHostToDevice));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(g_st_stamps), &st, sizeof(st)));
  const int shm = LDS_DOUBLES * 8;
  CK(hipFuncSetAttribute((const void*)k_st_proj<4>, hipFuncAttributeMaxDynamicSharedMemorySize, shm));
  CK(hipFuncSetAttribute((const void*)k_st_retr_r, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_DOUBLES_R * 8));
  const int shm2 = r2_lds_doubles_nr<4>((n + 15) / 16 * 16) * 8;
  CK(hipFuncSetAttribute((const void*)k_st_retr2<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CK(hipFuncSetAttribute((const void*)k_st_proj3<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CK(hipFuncSetAttribute((const void*)k_st_proj4<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  int ncu = 256;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const int shm3 = p3_lds_doubles(n, p, 4) * 8;

  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int which = 0; which < 5; ++which) {
    for (int r = 0; r < 20; ++r) {
      CK(hipEventRecord(a, 0));
      if (which == 0) hipLaunchKernelGGL(k_st_proj<4>, dim3(B), dim3(T), shm, 0, n, p, (int64_t)n * p, X, U, O);
      else if (which == 1) hipLaunchKernelGGL(k_st_retr_r, dim3(B), dim3(T), LDS_DOUBLES_R * 8, 0, n, p, (int64_t)n * p, X, U, O);
      else if (which == 2) hipLaunchKernelGGL(k_st_retr2<4>, dim3(B), dim3(T), shm2, 0, n, p, (int64_t)n * p, X, U, O);
      else if (which == 3) hipLaunchKernelGGL(k_st_proj3<4>, dim3(B), dim3(T), shm3, 0, n, p, (int64_t)n * p, X, U, O);
      else hipLaunchKernelGGL(k_st_proj4<4>, dim3(B < ncu ? B : ncu), dim3(T), shm3, 0, n, p, (int64_t)n * p, B, X, U, O);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
    }
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<long long> s((size_t)B * 16);
    CK(hipMemcpy(s.data(), st, s.size() * 8, hipMemcpyDeviceToHost));
    if (which == 1) {   // the round-1 retraction kernel carries no stamps: event time only
      printf("{\"kernel\": \"k_st_retr_r\", \"n\": %d, \"p\": %d, \"B\": %d, \"event_us\": %.2f}\n", n, p, B, ms * 1e3);
      continue;
    }
    const int np = which == 2 ? 7 : which == 3 ? 4 : which == 4 ? 5 : 2;
    const int Bw = which == 4 && B > ncu ? ncu : B;   // k_st_proj4: one workgroup per CU, its last point's stamps
    printf("{\"kernel\": \"%s\", \"n\": %d, \"p\": %d, \"B\": %d, \"event_us\": %.2f, \"phase_ticks_median\": [",
           which == 0 ? "k_st_proj" : which == 3 ? "k_st_proj3 (load, gram, M to LDS, update)"
           : which == 4 ? "k_st_proj4 per point (-, gram, M to LDS, update + X copy, U/X copy drain)"
                        : "k_st_retr2 (load, gram1, factor1, apply1, gram2, factor2, apply2)", n, p, B, ms * 1e3);
    for (int k = 0; k < np; ++k) {
      std::vector<long long> d(Bw);
      for (int g = 0; g < Bw; ++g) d[g] = s[g * 16 + k + 1] - s[g * 16 + k];
      std::sort(d.begin(), d.end());
      printf("%s%lld", k ? ", " : "", d[Bw / 2]);
    }
    std::vector<long long> t(Bw);
    for (int g = 0; g < Bw; ++g) t[g] = s[g * 16 + np] - s[g * 16];
    std::sort(t.begin(), t.end());
    printf("], \"total_ticks_median\": %lld, \"total_ticks_max\": %lld", t[Bw / 2], t[Bw - 1]);
    if (which == 2) {   // blocked factor sub-phases (first factor): diag0, b0, G11+diag1 (wave 0), wait, b1, G22+diag2, rest
      printf(", \"factor1_sub_ticks_median\": [");
      for (int k = 8; k < 15; ++k) {
        std::vector<long long> d(B);
        for (int g = 0; g < B; ++g) d[g] = s[g * 16 + k + 1] - s[g * 16 + k];
        std::sort(d.begin(), d.end());
        printf("%s%lld", k > 8 ? ", " : "", d[B / 2]);
      }
      printf("]");
    }
    printf("}\n");
  }
  return 0;
}
