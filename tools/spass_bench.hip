// spass_bench.hip — tuning harness for the symmetric-tile S-pass (k_spass_sym) on MI355X.
// Builds standalone: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/spass_bench.hip -o spass_bench
// Times variants of the tile kernel on B instances of a random packed S (all instances active),
// reports device time per pass and TB/s of stored S bytes, and checks every variant's result
// against variant 0 (relative error).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
#include <string>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

typedef double dbl2 __attribute__((ext_vector_type(2)));
constexpr int TS = 128;

__device__ __forceinline__ double xor_lane(double v, int off) {
  const int addr = ((int)__lane_id() ^ off) << 2;
  const int lo = __builtin_amdgcn_ds_bpermute(addr, __double2loint(v));
  const int hi = __builtin_amdgcn_ds_bpermute(addr, __double2hiint(v));
  return __hiloint2double(hi, lo);
}
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
__device__ __forceinline__ double rs8(double (&a)[8]) {
  const int lane = (int)__lane_id();
#pragma unroll
  for (int k = 0; k < 4; ++k) { swap32(a[k], a[k + 4]); a[k] = a[k] + a[k + 4]; }
#pragma unroll
  for (int k = 0; k < 2; ++k) { swap16(a[k], a[k + 2]); a[k] = a[k] + a[k + 2]; }
  const double r0 = a[0], r1 = a[1];
  const bool b3 = (lane & 8) != 0;
  const double snd = b3 ? r0 : r1, kp = b3 ? r1 : r0;
  double v = kp + xor_lane(snd, 8);
  v += xor_lane(v, 4); v += xor_lane(v, 2); v += xor_lane(v, 1);
  return v;
}
__device__ __forceinline__ void tile_ij(int t, int nt, int& I, int& J) {
  int i = 0, rem = t, len = nt;
  while (rem >= len) { rem -= len; ++i; --len; }
  I = i; J = i + rem;
}

template <bool NT>
__device__ __forceinline__ dbl2 ld2(const double* p) {
  if (NT) return __builtin_nontemporal_load((const dbl2*)p);
  return *(const dbl2*)p;
}

struct Args {
  const double* S; int64_t inst_stride; int nt, ntiles, batch, ld;
  const double* v; double* pb;
};

// WAVES waves per tile; each wave ROWS = 128/WAVES rows in batches of 8; PF = prefetch next batch;
// TPW = tiles per workgroup (consecutive tiles of the same instance)
template <int WAVES, bool PF, bool NT, int TPW>
__global__ void __launch_bounds__(WAVES * 64) k_var(Args A) {
  constexpr int ROWS = TS / WAVES;
  constexpr int NB = ROWS / 8;
  const int lane = (int)__lane_id();
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int per_inst = (A.ntiles + TPW - 1) / TPW;
  const int b = blockIdx.x / per_inst;
  const int t0 = (blockIdx.x - b * per_inst) * TPW;
  const double* v0 = A.v + (int64_t)b * A.ld;
  const int64_t nn = (int64_t)A.nt * A.nt * TS;
  double* pb0 = A.pb + (int64_t)b * nn;
  const int rrow = 4 * ((lane >> 5) & 1) + 2 * ((lane >> 4) & 1) + ((lane >> 3) & 1);
  __shared__ double cs[WAVES][TS];
  for (int tt = 0; tt < TPW; ++tt) {
    const int t = t0 + tt;
    if (t >= A.ntiles) break;
    int I, J; tile_ij(t, A.nt, I, J);
    const double* T = A.S + (int64_t)b * A.inst_stride + (int64_t)t * TS * TS;
    const dbl2 vj0 = *(const dbl2*)(v0 + J * TS + 2 * lane);
    double cx = 0.0, cy = 0.0;
    dbl2 nxt[8];
    if (PF) {
#pragma unroll
      for (int k = 0; k < 8; ++k) nxt[k] = ld2<NT>(T + (w * ROWS + k) * TS + 2 * lane);
    }
#pragma unroll 1
    for (int rb = 0; rb < NB; ++rb) {
      const int r0 = w * ROWS + rb * 8;
      dbl2 sv[8];
      if (PF) {
#pragma unroll
        for (int k = 0; k < 8; ++k) sv[k] = nxt[k];
        if (rb + 1 < NB) {
#pragma unroll
          for (int k = 0; k < 8; ++k) nxt[k] = ld2<NT>(T + (r0 + 8 + k) * TS + 2 * lane);
        }
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) sv[k] = ld2<NT>(T + (r0 + k) * TS + 2 * lane);
      }
      double a[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const double vi0 = v0[I * TS + r0 + k];
        a[k] = __builtin_fma(sv[k].y, vj0.y, sv[k].x * vj0.x);
        cx = __builtin_fma(sv[k].x, vi0, cx);
        cy = __builtin_fma(sv[k].y, vi0, cy);
      }
      const double s0 = rs8(a);
      if ((lane & 7) == 0) pb0[((int64_t)I * A.nt + J) * TS + r0 + rrow] = s0;
    }
    if (I != J) {
      cs[w][2 * lane] = cx;
      cs[w][2 * lane + 1] = cy;
      __syncthreads();
      if (threadIdx.x < TS) {
        double s = cs[0][threadIdx.x];
#pragma unroll
        for (int q = 1; q < WAVES; ++q) s += cs[q][threadIdx.x];
        pb0[((int64_t)J * A.nt + I) * TS + threadIdx.x] = s;
      }
      __syncthreads();
    }
  }
}

__global__ void k_fill(double* p, int64_t n, uint64_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull; z ^= z >> 31;
    p[i] = (double)(z >> 11) * (1.0 / 9007199254740992.0) - 0.5;
  }
}

// pure streaming read of the same bytes: the achievable HBM read rate for this footprint
template <bool NT>
__global__ void __launch_bounds__(256) k_stream(const double* S, int64_t n2, double* out) {
  double acc = 0.0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 2;
  for (int64_t i = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) * 2; i < n2; i += stride * 4) {
    dbl2 a = ld2<NT>(S + i), b = (i + stride < n2) ? ld2<NT>(S + i + stride) : dbl2{0, 0};
    dbl2 c = (i + 2 * stride < n2) ? ld2<NT>(S + i + 2 * stride) : dbl2{0, 0};
    dbl2 d = (i + 3 * stride < n2) ? ld2<NT>(S + i + 3 * stride) : dbl2{0, 0};
    acc += a.x + a.y + b.x + b.y + c.x + c.y + d.x + d.y;
  }
  if (acc == 123.456) out[0] = acc;
}

typedef void (*KFn)(Args);
struct Var { const char* name; KFn fn; int threads; int tpw; };

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4000;
  const int B = argc > 2 ? atoi(argv[2]) : 128;
  const int reps = argc > 3 ? atoi(argv[3]) : 20;
  const int ld = (n + TS - 1) / TS * TS, nt = ld / TS, ntiles = nt * (nt + 1) / 2;
  const int64_t inst = (int64_t)ntiles * TS * TS;
  double *S, *v, *pb;
  CHK(hipMalloc(&S, (size_t)B * inst * 8));
  CHK(hipMalloc(&v, (size_t)B * ld * 8));
  CHK(hipMalloc(&pb, (size_t)B * nt * nt * TS * 8));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, S, (int64_t)B * inst, 1ull);
  hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, 0, v, (int64_t)B * ld, 7ull);
  CHK(hipDeviceSynchronize());
  Args A{S, inst, nt, ntiles, B, ld, v, pb};
  Var vars[] = {
      {"w4 nt noPF tpw1 (current)", k_var<4, false, true, 1>, 256, 1},
      {"w4 nt PF tpw1", k_var<4, true, true, 1>, 256, 1},
      {"w4 plain noPF tpw1", k_var<4, false, false, 1>, 256, 1},
      {"w4 plain PF tpw1", k_var<4, true, false, 1>, 256, 1},
      {"w8 nt noPF tpw1", k_var<8, false, true, 1>, 512, 1},
      {"w8 nt PF tpw1", k_var<8, true, true, 1>, 512, 1},
      {"w4 nt PF tpw2", k_var<4, true, true, 2>, 256, 2},
      {"w4 nt PF tpw4", k_var<4, true, true, 4>, 256, 4},
      {"w2 nt PF tpw1", k_var<2, true, true, 1>, 128, 1},
      {"w16 nt noPF tpw1", k_var<16, false, true, 1>, 1024, 1},
  };
  const double bytes = (double)B * inst * 8;
  std::vector<double> ref((size_t)B * nt * nt * TS), got(ref.size());
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  for (size_t vi = 0; vi < sizeof(vars) / sizeof(vars[0]); ++vi) {
    const Var& V = vars[vi];
    const int per = (ntiles + V.tpw - 1) / V.tpw;
    dim3 grid(B * per);
    CHK(hipMemset(pb, 0, ref.size() * 8));
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(V.fn, grid, dim3(V.threads), 0, 0, A);
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(V.fn, grid, dim3(V.threads), 0, 0, A);
    CHK(hipEventRecord(e1, 0));
    CHK(hipEventSynchronize(e1));
    float ms = 0; CHK(hipEventElapsedTime(&ms, e0, e1));
    const double per_ms = ms / reps;
    CHK(hipMemcpy(got.data(), pb, got.size() * 8, hipMemcpyDeviceToHost));
    double err = 0.0, nrm = 0.0;
    if (vi == 0) ref = got;
    for (size_t i = 0; i < got.size(); ++i) { err = fmax(err, fabs(got[i] - ref[i])); nrm = fmax(nrm, fabs(ref[i])); }
    printf("{\"variant\": \"%s\", \"n\": %d, \"B\": %d, \"ms\": %.4f, \"TBps\": %.3f, \"maxrelerr\": %.2e}\n",
           V.name, n, B, per_ms, bytes / (per_ms * 1e-3) / 1e12, nrm > 0 ? err / nrm : 0.0);
    fflush(stdout);
  }
  for (int ntv = 0; ntv < 2; ++ntv) {
    for (int grid : {1024, 2048, 4096, 8192}) {
      auto fn = ntv ? k_stream<true> : k_stream<false>;
      for (int r = 0; r < 2; ++r) hipLaunchKernelGGL(fn, dim3(grid), dim3(256), 0, 0, S, (int64_t)B * inst, pb);
      CHK(hipDeviceSynchronize());
      CHK(hipEventRecord(e0, 0));
      for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(fn, dim3(grid), dim3(256), 0, 0, S, (int64_t)B * inst, pb);
      CHK(hipEventRecord(e1, 0));
      CHK(hipEventSynchronize(e1));
      float ms = 0; CHK(hipEventElapsedTime(&ms, e0, e1));
      printf("{\"variant\": \"stream read %s grid %d\", \"ms\": %.4f, \"TBps\": %.3f}\n", ntv ? "nt" : "plain", grid,
             ms / reps, bytes / (ms / reps * 1e-3) / 1e12);
    }
  }
  return 0;
}
