// mfma_bench.hip — tuning harness for the shared-S multi-start S-pass (fp64 MFMA) on MI355X.
// Builds standalone: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mfma_bench.hip -o mfma_bench
// Y[c][i] = sum_k V[c][k] * S[i][k] for C right-hand sides sharing one n x n S (row-major, ld).
// Checks the v_mfma_f64_16x16x4_f64 operand/result layout against a host fp64 product and
// times the tile variants (TFLOP/s of 2 n^2 C).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
#include <string>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

typedef double dbl2 __attribute__((ext_vector_type(2)));
typedef double dbl4 __attribute__((ext_vector_type(4)));

// K chunk of 32 per wave step: lane l covers k0 + 8*(l>>4) .. +8 for row/col (l & 15); MFMA m
// (0..7) consumes element m, i.e. the k order inside a chunk is permuted identically for A and B.
template <int WM, int WN, int KS>
__global__ void __launch_bounds__(64 * KS) k_mm(const double* __restrict__ S, const double* __restrict__ V,
                                                double* __restrict__ Y, int n, int rows, int64_t ld, int C) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i0 = blockIdx.x * 16 * WN, c0 = blockIdx.y * 16 * WM;
  const int r = lane & 15, q = lane >> 4;
  const double* ap[WM];
  const double* bp[WN];
#pragma unroll
  for (int a = 0; a < WM; ++a) {
    int c = c0 + 16 * a + r;
    c = c < C ? c : C - 1;
    ap[a] = V + (int64_t)c * ld + 8 * q;
  }
#pragma unroll
  for (int b = 0; b < WN; ++b) {
    int i = i0 + 16 * b + r;
    i = i < rows ? i : rows - 1;
    bp[b] = S + (int64_t)i * ld + 8 * q;
  }
  dbl4 acc[WM][WN];
#pragma unroll
  for (int a = 0; a < WM; ++a)
#pragma unroll
    for (int b = 0; b < WN; ++b) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
  const int nch = (int)(ld / 32);
  for (int ch = w; ch < nch; ch += KS) {
    const int64_t k0 = (int64_t)ch * 32;
    dbl2 fa[WM][4], fb[WN][4];
#pragma unroll
    for (int a = 0; a < WM; ++a)
#pragma unroll
      for (int h = 0; h < 4; ++h) fa[a][h] = *(const dbl2*)(ap[a] + k0 + 2 * h);
#pragma unroll
    for (int b = 0; b < WN; ++b)
#pragma unroll
      for (int h = 0; h < 4; ++h) fb[b][h] = __builtin_nontemporal_load((const dbl2*)(bp[b] + k0 + 2 * h));
#pragma unroll
    for (int m = 0; m < 8; ++m)
#pragma unroll
      for (int a = 0; a < WM; ++a)
#pragma unroll
        for (int b = 0; b < WN; ++b) {
          const double av = (m & 1) ? fa[a][m >> 1].y : fa[a][m >> 1].x;
          const double bv = (m & 1) ? fb[b][m >> 1].y : fb[b][m >> 1].x;
          acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[a][b], 0, 0, 0);
        }
  }
  if (KS > 1) {
    __shared__ dbl4 red[KS > 1 ? KS - 1 : 1][WM][WN][64];
    if (w > 0)
#pragma unroll
      for (int a = 0; a < WM; ++a)
#pragma unroll
        for (int b = 0; b < WN; ++b) red[w - 1][a][b][lane] = acc[a][b];
    __syncthreads();
    if (w != 0) return;
    for (int s = 0; s < KS - 1; ++s)
#pragma unroll
      for (int a = 0; a < WM; ++a)
#pragma unroll
        for (int b = 0; b < WN; ++b) acc[a][b] += red[s][a][b][lane];
  }
  // D layout (f64): col = lane & 15 (-> i), row = (lane >> 4) + 4 * reg (-> c)
#pragma unroll
  for (int a = 0; a < WM; ++a)
#pragma unroll
    for (int b = 0; b < WN; ++b) {
      const int i = i0 + 16 * b + r;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = c0 + 16 * a + q + 4 * g;
        if (i < n && c < C) Y[(int64_t)c * ld + i] = acc[a][b][g];
      }
    }
}

struct Variant {
  std::string name;
  void (*launch)(const double*, const double*, double*, int, int, int64_t, int, hipStream_t);
};

template <int WM, int WN, int KS>
void launch_mm(const double* S, const double* V, double* Y, int n, int rows, int64_t ld, int C, hipStream_t st) {
  dim3 grid((rows + 16 * WN - 1) / (16 * WN), (C + 16 * WM - 1) / (16 * WM));
  hipLaunchKernelGGL((k_mm<WM, WN, KS>), grid, dim3(64 * KS), 0, st, S, V, Y, n, rows, ld, C);
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4000;
  const int C = argc > 2 ? atoi(argv[2]) : 128;
  const int64_t ld = (n + 127) / 128 * 128;
  const int rows = (n + 31) / 32 * 32;
  std::vector<double> hS((size_t)rows * ld, 0.0), hV((size_t)C * ld, 0.0);
  srand(12345);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j <= i; ++j) {
      const double v = (double)rand() / RAND_MAX - 0.5;
      hS[(size_t)i * ld + j] = v;
      hS[(size_t)j * ld + i] = v;
    }
  for (int c = 0; c < C; ++c)
    for (int k = 0; k < n; ++k) hV[(size_t)c * ld + k] = (double)rand() / RAND_MAX - 0.5;
  std::vector<double> ref((size_t)C * n);
  for (int c = 0; c < C; ++c)
    for (int i = 0; i < n; ++i) {
      long double s = 0;
      for (int k = 0; k < n; ++k) s += (long double)hS[(size_t)i * ld + k] * hV[(size_t)c * ld + k];
      ref[(size_t)c * n + i] = (double)s;
    }
  double *S, *V, *Y;
  CHK(hipMalloc(&S, hS.size() * 8));
  CHK(hipMalloc(&V, hV.size() * 8));
  CHK(hipMalloc(&Y, (size_t)C * ld * 8));
  CHK(hipMemcpy(S, hS.data(), hS.size() * 8, hipMemcpyHostToDevice));
  CHK(hipMemcpy(V, hV.data(), hV.size() * 8, hipMemcpyHostToDevice));
  std::vector<Variant> vs = {
      {"wm2 wn2 ks4", launch_mm<2, 2, 4>}, {"wm2 wn2 ks2", launch_mm<2, 2, 2>}, {"wm2 wn2 ks8", launch_mm<2, 2, 8>},
      {"wm2 wn4 ks4", launch_mm<2, 4, 4>}, {"wm4 wn2 ks4", launch_mm<4, 2, 4>}, {"wm4 wn4 ks4", launch_mm<4, 4, 4>},
      {"wm1 wn4 ks4", launch_mm<1, 4, 4>}, {"wm2 wn1 ks4", launch_mm<2, 1, 4>}, {"wm4 wn4 ks2", launch_mm<4, 4, 2>},
      {"wm8 wn2 ks4", launch_mm<8, 2, 4>}, {"wm2 wn8 ks4", launch_mm<2, 8, 4>},
  };
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  std::vector<double> hY((size_t)C * ld);
  for (auto& v : vs) {
    CHK(hipMemset(Y, 0, (size_t)C * ld * 8));
    v.launch(S, V, Y, n, rows, ld, C, 0);
    CHK(hipDeviceSynchronize());
    CHK(hipMemcpy(hY.data(), Y, hY.size() * 8, hipMemcpyDeviceToHost));
    double maxrel = 0;
    for (int c = 0; c < C; ++c)
      for (int i = 0; i < n; ++i) {
        const double d = fabs(hY[(size_t)c * ld + i] - ref[(size_t)c * n + i]);
        maxrel = fmax(maxrel, d / (fabs(ref[(size_t)c * n + i]) + 1e-3));
      }
    const int reps = 50;
    CHK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; ++r) v.launch(S, V, Y, n, rows, ld, C, 0);
    CHK(hipEventRecord(e1, 0));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const double t = ms / reps;
    printf("{\"variant\": \"%s\", \"n\": %d, \"C\": %d, \"us\": %.2f, \"TFLOPs\": %.2f, \"maxrelerr\": %.2e}\n",
           v.name.c_str(), n, C, t * 1e3, 2.0 * n * n * C / (t * 1e-3) / 1e12, maxrel);
  }
  return 0;
}
