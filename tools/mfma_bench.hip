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
  Y += (int64_t)blockIdx.z * C * ld;
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
  const int nch_all = (int)(ld / 32), per = (nch_all + gridDim.z - 1) / gridDim.z;
  const int ch_lo = blockIdx.z * per, nch = min(nch_all, ch_lo + per);
  for (int ch = ch_lo + w; ch < nch; ch += KS) {
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
  if (KS > 1) {  // waves 1..KS-1 accumulate in turn into one LDS slab, wave 0 adds it last
    __shared__ dbl4 red[WM][WN][64];
    for (int s = 1; s < KS; ++s) {
      if (w == s)
#pragma unroll
        for (int a = 0; a < WM; ++a)
#pragma unroll
          for (int b = 0; b < WN; ++b) red[a][b][lane] = s == 1 ? acc[a][b] : red[a][b][lane] + acc[a][b];
      __syncthreads();
    }
    if (w != 0) return;
#pragma unroll
    for (int a = 0; a < WM; ++a)
#pragma unroll
      for (int b = 0; b < WN; ++b) acc[a][b] += red[a][b][lane];
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

// sum of KZ partial slabs in fixed order into slab 0
__global__ void k_red(double* Y, int64_t slab, int kz) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= slab) return;
  double s = Y[e];
  for (int z = 1; z < kz; ++z) s += Y[(int64_t)z * slab + e];
  Y[e] = s;
}

// f64 MFMA issue-rate probe: independent accumulator chains, no memory
template <int NACC>
__global__ void k_peak(double* out, int iters) {
  dbl4 acc[NACC];
  for (int a = 0; a < NACC; ++a) acc[a] = dbl4{0.0, 0.0, 0.0, 0.0};
  double x = threadIdx.x * 1e-3, y = 1.0 + threadIdx.x * 1e-4;
  for (int it = 0; it < iters; ++it)
#pragma unroll
    for (int a = 0; a < NACC; ++a) acc[a] = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc[a], 0, 0, 0);
  double s = 0;
  for (int a = 0; a < NACC; ++a) s += acc[a][0] + acc[a][1] + acc[a][2] + acc[a][3];
  if (s == 12345.678) out[0] = s;
}

struct Variant {
  std::string name;
  void (*launch)(const double*, const double*, double*, int, int, int64_t, int, hipStream_t);
};

template <int WM, int WN, int KS, int KZ = 1>
void launch_mm(const double* S, const double* V, double* Y, int n, int rows, int64_t ld, int C, hipStream_t st) {
  dim3 grid((rows + 16 * WN - 1) / (16 * WN), (C + 16 * WM - 1) / (16 * WM), KZ);
  hipLaunchKernelGGL((k_mm<WM, WN, KS>), grid, dim3(64 * KS), 0, st, S, V, Y, n, rows, ld, C);
  if (KZ > 1) {
    const int64_t slab = (int64_t)C * ld;
    hipLaunchKernelGGL(k_red, dim3((unsigned)((slab + 255) / 256)), dim3(256), 0, st, Y, slab, KZ);
  }
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
  CHK(hipMalloc(&Y, (size_t)4 * C * ld * 8));
  {
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    for (int waves : {1024, 2048, 4096}) {
      const int iters = 4000;
      hipLaunchKernelGGL(k_peak<4>, dim3(waves / 4), dim3(256), 0, 0, Y, 10);
      CHK(hipEventRecord(a, 0));
      hipLaunchKernelGGL(k_peak<4>, dim3(waves / 4), dim3(256), 0, 0, Y, iters);
      CHK(hipEventRecord(b, 0));
      CHK(hipEventSynchronize(b));
      float ms = 0;
      CHK(hipEventElapsedTime(&ms, a, b));
      const double fl = (double)waves * iters * 4 * 2048.0;
      printf("{\"variant\": \"mfma_f64_16x16x4 peak probe\", \"waves\": %d, \"TFLOPs\": %.2f}\n", waves, fl / (ms * 1e-3) / 1e12);
    }
  }
  CHK(hipMemcpy(S, hS.data(), hS.size() * 8, hipMemcpyHostToDevice));
  CHK(hipMemcpy(V, hV.data(), hV.size() * 8, hipMemcpyHostToDevice));
  std::vector<Variant> vs = {
      {"wm8 wn2 ks4", launch_mm<8, 2, 4>},      {"wm8 wn2 ks8", launch_mm<8, 2, 8>},
      {"wm8 wn2 ks16", launch_mm<8, 2, 16>},    {"wm4 wn4 ks8", launch_mm<4, 4, 8>},
      {"wm4 wn4 ks16", launch_mm<4, 4, 16>},    {"wm4 wn2 ks8", launch_mm<4, 2, 8>},
      {"wm4 wn2 ks16", launch_mm<4, 2, 16>},    {"wm2 wn2 ks16", launch_mm<2, 2, 16>},
      {"wm8 wn2 ks4 kz4", launch_mm<8, 2, 4, 4>}, {"wm8 wn2 ks8 kz2", launch_mm<8, 2, 8, 2>},
      {"wm4 wn4 ks4 kz4", launch_mm<4, 4, 4, 4>}, {"wm4 wn2 ks4 kz4", launch_mm<4, 2, 4, 4>},
      {"wm2 wn1 ks4 kz4", launch_mm<2, 1, 4, 4>}, {"wm2 wn1 ks8", launch_mm<2, 1, 8>},
      {"wm2 wn2 ks8 kz2", launch_mm<2, 2, 8, 2>}, {"wm1 wn2 ks8", launch_mm<1, 2, 8>},
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
