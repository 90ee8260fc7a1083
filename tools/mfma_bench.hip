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

// Software-pipelined variant: K chunks of 16 (lane l loads 4 consecutive k = 32 B of row l & 15
// at offset 4 (l >> 4); MFMA m of the chunk consumes element m), the next chunk's operands
// loaded into a second register set while the current one feeds the MFMAs (one wave per SIMD
// cannot hide a load phase behind another wave).  Loop manually unrolled by two so the buffers
// swap without register moves.
template <int WM, int WN>
struct MmFrag {
  dbl2 a[WM][2], b[WN][2];
};

template <int WM, int WN>
__device__ __forceinline__ void mm_load(MmFrag<WM, WN>& f, const double* const* ap, const double* const* bp, int64_t k0) {
#pragma unroll
  for (int a = 0; a < WM; ++a)
#pragma unroll
    for (int h = 0; h < 2; ++h) f.a[a][h] = *(const dbl2*)(ap[a] + k0 + 2 * h);
#pragma unroll
  for (int b = 0; b < WN; ++b)
#pragma unroll
    for (int h = 0; h < 2; ++h) f.b[b][h] = __builtin_nontemporal_load((const dbl2*)(bp[b] + k0 + 2 * h));
}

template <int WM, int WN>
__device__ __forceinline__ void mm_fma(dbl4 (&acc)[WM][WN], const MmFrag<WM, WN>& f) {
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int a = 0; a < WM; ++a)
#pragma unroll
      for (int b = 0; b < WN; ++b) {
        const double av = (m & 1) ? f.a[a][m >> 1].y : f.a[a][m >> 1].x;
        const double bv = (m & 1) ? f.b[b][m >> 1].y : f.b[b][m >> 1].x;
        acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[a][b], 0, 0, 0);
      }
}

template <int WM, int WN, int KS>
__global__ void __launch_bounds__(64 * KS) k_mm2(const double* __restrict__ S, const double* __restrict__ V,
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
    ap[a] = V + (int64_t)c * ld + 4 * q;
  }
#pragma unroll
  for (int b = 0; b < WN; ++b) {
    int i = i0 + 16 * b + r;
    i = i < rows ? i : rows - 1;
    bp[b] = S + (int64_t)i * ld + 4 * q;
  }
  dbl4 acc[WM][WN];
#pragma unroll
  for (int a = 0; a < WM; ++a)
#pragma unroll
    for (int b = 0; b < WN; ++b) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
  const int nch_all = (int)(ld / 16), per = (nch_all + gridDim.z - 1) / gridDim.z;
  const int ch_lo = blockIdx.z * per, ch_hi = min(nch_all, ch_lo + per);
  int ch = ch_lo + w;
  MmFrag<WM, WN> f0, f1;
  if (ch < ch_hi) mm_load(f0, ap, bp, (int64_t)ch * 16);
  while (ch < ch_hi) {
    const int c1 = ch + KS;
    if (c1 < ch_hi) mm_load(f1, ap, bp, (int64_t)c1 * 16);
    mm_fma(acc, f0);
    if (c1 >= ch_hi) break;
    const int c2 = c1 + KS;
    if (c2 < ch_hi) mm_load(f0, ap, bp, (int64_t)c2 * 16);
    mm_fma(acc, f1);
    ch = c2;
  }
  if (KS > 1) {
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

// LDS-staged variant: a workgroup owns 128 right-hand sides x 128 rows of S over one K slice;
// each 32-deep K step stages V[128][32] and S[128][32] (256-B rows, 16-B chunk c of row r kept at
// chunk c ^ (r & 15)) with global_load_lds_dwordx4, double-buffered: the next step's copy is in
// flight while the 4 waves (32 rows each, 8 x 2 accumulators) run this step's 128 MFMAs from
// LDS.  One barrier per step.  Linear block id -> (slice = id % kz, so a K slice stays on one
// XCD and its V slice in that XCD's L2; row block; column block).
constexpr int M3_VT = 128 * 256;  // bytes of the V tile per stage
typedef __attribute__((address_space(3))) unsigned char lds_u8;
typedef __attribute__((address_space(3))) dbl2 lds_dbl2;

template <int RT>
struct M3 {
  static constexpr int STAGE = M3_VT + RT * 256;  // V tile + S tile
};

// NW waves per workgroup, each owning RT / NW rows of the tile (WN = RT / (16 NW) accumulator
// columns): NW = 8 puts two waves on every SIMD, so one wave's LDS reads / barrier wait hide
// under the other's MFMAs.
template <int RT, bool PF, int NW = 4>
__global__ void __launch_bounds__(64 * NW) k_mm3(const double* __restrict__ S, const double* __restrict__ V,
                                                 double* __restrict__ Y, int n, int rows, int64_t ld, int C, int kz) {
  constexpr int RW = RT / NW, WN = RW / 16, STAGE = M3<RT>::STAGE;
  constexpr int VPW = 32 / NW, SPW = RT / 4 / NW;  // glds per wave per stage
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  lds_u8* smem = (lds_u8*)smem_raw;
  const int L = blockIdx.x, z = L % kz, rest = L / kz;
  const int nrb = (rows + RT - 1) / RT;
  const int i0 = (rest % nrb) * RT, c0 = (rest / nrb) * 128;
  Y += (int64_t)z * C * ld;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, q = lane >> 4;
  const double* vsrc[VPW];
  const double* ssrc[SPW];
#pragma unroll
  for (int p = 0; p < VPW; ++p) {
    const int row = 4 * (VPW * w + p) + q;
    const int c = min(c0 + row, C - 1);
    vsrc[p] = V + (int64_t)c * ld + 2 * (r ^ (row & 15));
  }
#pragma unroll
  for (int p = 0; p < SPW; ++p) {
    const int row = 4 * (SPW * w + p) + q;
    const int i = min(i0 + row, rows - 1);
    ssrc[p] = S + (int64_t)i * ld + 2 * (r ^ (row & 15));
  }
  const int nch = (int)(ld / 32), per = (nch + kz - 1) / kz;
  const int lo = z * per, hi = min(nch, lo + per);
  auto issue = [&](int ch, int buf) {
    const int64_t k0 = (int64_t)ch * 32;
    lds_u8* vb = smem + buf * STAGE;
#pragma unroll
    for (int p = 0; p < VPW; ++p)
      __builtin_amdgcn_global_load_lds((const void*)(vsrc[p] + k0), (lds_u8*)(vb + 4 * (VPW * w + p) * 256), 16, 0, 0);
#pragma unroll
    for (int p = 0; p < SPW; ++p)
      __builtin_amdgcn_global_load_lds((const void*)(ssrc[p] + k0), (lds_u8*)(vb + M3_VT + 4 * (SPW * w + p) * 256), 16, 0, 0);
  };
  dbl4 acc[8][WN];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < WN; ++b) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
  const bool live = i0 + RW * w < n;
  if (lo < hi) issue(lo, 0);
  for (int ch = lo; ch < hi; ++ch) {
    const int s = (ch - lo) & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (ch + 1 < hi) issue(ch + 1, s ^ 1);
    if (!live) continue;
    const lds_u8* vb = smem + s * STAGE;
    const lds_u8* sb = vb + M3_VT;
    dbl2 fa[2][8], fb[2][WN];
    auto frag = [&](int jj, int u) {
      const int off = ((4 * q + jj) ^ r) * 16;
#pragma unroll
      for (int a = 0; a < 8; ++a) fa[u][a] = *(const lds_dbl2*)(vb + (16 * a + r) * 256 + off);
#pragma unroll
      for (int b = 0; b < WN; ++b) fb[u][b] = *(const lds_dbl2*)(sb + (RW * w + 16 * b + r) * 256 + off);
    };
    frag(0, 0);
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int u = PF ? (jj & 1) : 0;
      if (PF && jj < 3) frag(jj + 1, u ^ 1);
#pragma unroll
      for (int mm = 0; mm < 2; ++mm)
#pragma unroll
        for (int a = 0; a < 8; ++a)
#pragma unroll
          for (int b = 0; b < WN; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(mm ? fa[u][a].y : fa[u][a].x, mm ? fb[u][b].y : fb[u][b].x,
                                                             acc[a][b], 0, 0, 0);
      if (!PF && jj < 3) frag(jj + 1, 0);
    }
  }
  if (!live) return;
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < WN; ++b) {
      const int i = i0 + RW * w + 16 * b + r;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = c0 + 16 * a + q + 4 * g;
        if (i < n && c < C) Y[(int64_t)c * ld + i] = acc[a][b][g];
      }
    }
}

// The solver's tile (csrc/riptrm_kernels.hip mm_tile) with the wave grid as parameters: NWR x NWC
// waves over RT rows x 128 columns (WMW = 8 / NWC 16-column and WN = RT / NWR / 16 16-row
// accumulators per wave), NST-stage LDS ring, bare barrier after an explicit vmcnt wait.
// SCHED interleaves each fragment read group with the previous group's MFMAs
// (__builtin_amdgcn_sched_group_barrier: 1 DS read, then MFMAs).
template <int RT, int NWR, int NWC, int NST, bool SCHED>
__global__ void __launch_bounds__(64 * NWR * NWC) k_mm4(const double* __restrict__ S, const double* __restrict__ V,
                                                        double* __restrict__ Y, int n, int rows, int64_t ld, int C, int kz) {
  constexpr int NW = NWR * NWC, WMW = 8 / NWC, RW = RT / NWR, WN = RW / 16, STAGE = M3<RT>::STAGE;
  constexpr int VP = 32 / NW, SP = RT / 4 / NW;
  static_assert(VP >= 1 && SP >= 1 && WMW >= 1 && WN >= 1, "shape");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  lds_u8* smem = (lds_u8*)smem_raw;
  const int L = blockIdx.x, z = L % kz, rest = L / kz;
  const int nrb = (rows + RT - 1) / RT;
  const int i0 = (rest % nrb) * RT, c0 = (rest / nrb) * 128;
  Y += (int64_t)z * C * ld;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w % NWR, wc = w / NWR;
  const int r = lane & 15, q = lane >> 4;
  const double* vsrc[VP];
  const double* ssrc[SP];
#pragma unroll
  for (int p = 0; p < VP; ++p) {
    const int row = 4 * (VP * w + p) + q;
    vsrc[p] = V + (int64_t)min(c0 + row, C - 1) * ld + 2 * (r ^ (row & 15));
  }
#pragma unroll
  for (int p = 0; p < SP; ++p) {
    const int row = 4 * (SP * w + p) + q;
    ssrc[p] = S + (int64_t)min(i0 + row, rows - 1) * ld + 2 * (r ^ (row & 15));
  }
  const int nch = (int)(ld / 32), per = (nch + kz - 1) / kz;
  const int lo = z * per, hi = min(nch, lo + per);
  auto issue = [&](int ch, int buf) {
    const int64_t k0 = (int64_t)ch * 32;
    lds_u8* vb = smem + buf * STAGE;
#pragma unroll
    for (int p = 0; p < VP; ++p)
      __builtin_amdgcn_global_load_lds((const void*)(vsrc[p] + k0), (lds_u8*)(vb + 4 * (VP * w + p) * 256), 16, 0, 0);
#pragma unroll
    for (int p = 0; p < SP; ++p)
      __builtin_amdgcn_global_load_lds((const void*)(ssrc[p] + k0), (lds_u8*)(vb + M3_VT + 4 * (SP * w + p) * 256), 16, 0, 0);
  };
  dbl4 acc[WMW][WN];
#pragma unroll
  for (int a = 0; a < WMW; ++a)
#pragma unroll
    for (int b = 0; b < WN; ++b) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
  const bool live = i0 + RW * wr < n;
  if (lo < hi) issue(lo, 0);
  if (NST == 3 && lo + 1 < hi) issue(lo + 1, 1);
  int s = 0;
  for (int ch = lo; ch < hi; ++ch) {
    if (NST == 3 && ch + 1 < hi) {
#define WB(K) if constexpr (VP + SP == K) asm volatile("s_waitcnt vmcnt(" #K ")\n\ts_barrier" ::: "memory");
      WB(1) WB(2) WB(3) WB(4) WB(5) WB(6) WB(7) WB(8) WB(9) WB(10) WB(12)
#undef WB
    } else {
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
    if (ch + NST - 1 < hi) issue(ch + NST - 1, s == 0 ? NST - 1 : s - 1);
    const int sc = s;
    s = s + 1 == NST ? 0 : s + 1;
    if (!live) continue;
    const lds_u8* vb = smem + sc * STAGE + 16 * WMW * wc * 256;
    const lds_u8* sb = smem + sc * STAGE + M3_VT + RW * wr * 256;
    dbl2 fa[2][WMW], fb[2][WN];
    auto frag = [&](int jj, int u) {
      const int off = ((4 * q + jj) ^ r) * 16;
#pragma unroll
      for (int a = 0; a < WMW; ++a) fa[u][a] = *(const lds_dbl2*)(vb + (16 * a + r) * 256 + off);
#pragma unroll
      for (int b = 0; b < WN; ++b) fb[u][b] = *(const lds_dbl2*)(sb + (16 * b + r) * 256 + off);
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
          for (int b = 0; b < WN; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(mm ? fa[u][a].y : fa[u][a].x, mm ? fb[u][b].y : fb[u][b].x,
                                                             acc[a][b], 0, 0, 0);
      if constexpr (SCHED) {
        if (jj < 3) {
          // next group's reads spread over this group's MFMAs
#pragma unroll
          for (int t = 0; t < WMW + WN; ++t) {
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
          }
          __builtin_amdgcn_sched_group_barrier(0x008, 2 * WMW * WN - (WMW + WN) > 0 ? 2 * WMW * WN - (WMW + WN) : 0, 0);
        }
      }
    }
  }
  if (!live) return;
#pragma unroll
  for (int a = 0; a < WMW; ++a)
#pragma unroll
    for (int b = 0; b < WN; ++b) {
      const int i = i0 + RW * wr + 16 * b + r;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = c0 + 16 * (WMW * wc + a) + q + 4 * g;
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

static bool g_red = true;  // timing loops skip the slab sum (the solver's state kernel does it)

struct Variant {
  std::string name;
  void (*launch)(const double*, const double*, double*, int, int, int64_t, int, hipStream_t);
};

template <int WM, int WN, int KS, int KZ = 1>
void launch_mm(const double* S, const double* V, double* Y, int n, int rows, int64_t ld, int C, hipStream_t st) {
  dim3 grid((rows + 16 * WN - 1) / (16 * WN), (C + 16 * WM - 1) / (16 * WM), KZ);
  hipLaunchKernelGGL((k_mm<WM, WN, KS>), grid, dim3(64 * KS), 0, st, S, V, Y, n, rows, ld, C);
  if (KZ > 1 && g_red) {
    const int64_t slab = (int64_t)C * ld;
    hipLaunchKernelGGL(k_red, dim3((unsigned)((slab + 255) / 256)), dim3(256), 0, st, Y, slab, KZ);
  }
}

template <int WM, int WN, int KS, int KZ = 1>
void launch_mm2(const double* S, const double* V, double* Y, int n, int rows, int64_t ld, int C, hipStream_t st) {
  dim3 grid((rows + 16 * WN - 1) / (16 * WN), (C + 16 * WM - 1) / (16 * WM), KZ);
  hipLaunchKernelGGL((k_mm2<WM, WN, KS>), grid, dim3(64 * KS), 0, st, S, V, Y, n, rows, ld, C);
  if (KZ > 1 && g_red) {
    const int64_t slab = (int64_t)C * ld;
    hipLaunchKernelGGL(k_red, dim3((unsigned)((slab + 255) / 256)), dim3(256), 0, st, Y, slab, KZ);
  }
}

template <int RT, bool PF, int KZ, int NW = 4>
void launch_mm3(const double* S, const double* V, double* Y, int n, int rows, int64_t ld, int C, hipStream_t st) {
  const int nrb = (rows + RT - 1) / RT, ncb = (C + 127) / 128;
  hipLaunchKernelGGL((k_mm3<RT, PF, NW>), dim3(nrb * ncb * KZ), dim3(64 * NW), M3<RT>::STAGE * 2, st, S, V, Y, n, rows, ld,
                     C, KZ);
  if (KZ > 1 && g_red) {
    const int64_t slab = (int64_t)C * ld;
    hipLaunchKernelGGL(k_red, dim3((unsigned)((slab + 255) / 256)), dim3(256), 0, st, Y, slab, KZ);
  }
}

template <int RT, int NWR, int NWC, int NST, int KZ, bool SCHED = false>
void launch_mm4(const double* S, const double* V, double* Y, int n, int rows, int64_t ld, int C, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    CHK(hipFuncSetAttribute((const void*)k_mm4<RT, NWR, NWC, NST, SCHED>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            M3<RT>::STAGE * NST));
    attr = true;
  }
  const int nrb = (rows + RT - 1) / RT, ncb = (C + 127) / 128;
  hipLaunchKernelGGL((k_mm4<RT, NWR, NWC, NST, SCHED>), dim3(nrb * ncb * KZ), dim3(64 * NWR * NWC), M3<RT>::STAGE * NST, st,
                     S, V, Y, n, rows, ld, C, KZ);
  if (KZ > 1 && g_red) {
    const int64_t slab = (int64_t)C * ld;
    hipLaunchKernelGGL(k_red, dim3((unsigned)((slab + 255) / 256)), dim3(256), 0, st, Y, slab, KZ);
  }
}

int main(int argc, char** argv) {
  CHK(hipFuncSetAttribute((const void*)k_mm3<128, false>, hipFuncAttributeMaxDynamicSharedMemorySize, M3<128>::STAGE * 2));
  CHK(hipFuncSetAttribute((const void*)k_mm3<128, true>, hipFuncAttributeMaxDynamicSharedMemorySize, M3<128>::STAGE * 2));
  CHK(hipFuncSetAttribute((const void*)k_mm3<64, false>, hipFuncAttributeMaxDynamicSharedMemorySize, M3<64>::STAGE * 2));
  CHK(hipFuncSetAttribute((const void*)k_mm3<64, true>, hipFuncAttributeMaxDynamicSharedMemorySize, M3<64>::STAGE * 2));
  CHK(hipFuncSetAttribute((const void*)k_mm3<128, true, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, M3<128>::STAGE * 2));
  CHK(hipFuncSetAttribute((const void*)k_mm3<64, true, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, M3<64>::STAGE * 2));
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
  CHK(hipMalloc(&Y, (size_t)16 * C * ld * 8));
  const char* only = argc > 3 ? argv[3] : nullptr;  // run only variants whose name contains this
  if (!only) {
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    auto probe = [&](auto kern, int nacc, int waves) {
      const int iters = 4000;
      hipLaunchKernelGGL(kern, dim3(waves / 4), dim3(256), 0, 0, Y, 10);
      CHK(hipEventRecord(a, 0));
      hipLaunchKernelGGL(kern, dim3(waves / 4), dim3(256), 0, 0, Y, iters);
      CHK(hipEventRecord(b, 0));
      CHK(hipEventSynchronize(b));
      float ms = 0;
      CHK(hipEventElapsedTime(&ms, a, b));
      const double fl = (double)waves * iters * nacc * 2048.0;
      printf("{\"variant\": \"mfma_f64_16x16x4 peak probe\", \"chains\": %d, \"waves\": %d, \"TFLOPs\": %.2f}\n", nacc, waves,
             fl / (ms * 1e-3) / 1e12);
    };
    for (int waves : {1024, 2048, 4096}) probe(k_peak<4>, 4, waves);
    for (int waves : {1024, 2048}) probe(k_peak<8>, 8, waves);
    probe(k_peak<16>, 16, 1024);
    probe(k_peak<2>, 2, 2048);
    probe(k_peak<1>, 1, 4096);
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
      {"pipe wm8 wn2 ks4 kz4", launch_mm2<8, 2, 4, 4>}, {"pipe wm8 wn2 ks4 kz2", launch_mm2<8, 2, 4, 2>},
      {"pipe wm8 wn2 ks4 kz1", launch_mm2<8, 2, 4, 1>}, {"pipe wm4 wn4 ks4 kz4", launch_mm2<4, 4, 4, 4>},
      {"pipe wm8 wn4 ks4 kz4", launch_mm2<8, 4, 4, 4>}, {"pipe wm4 wn2 ks4 kz4", launch_mm2<4, 2, 4, 4>},
      {"pipe wm4 wn2 ks8 kz4", launch_mm2<4, 2, 8, 4>}, {"pipe wm8 wn1 ks4 kz4", launch_mm2<8, 1, 4, 4>},
      {"pipe wm2 wn1 ks4 kz4", launch_mm2<2, 1, 4, 4>},
      {"glds r128 kz8", launch_mm3<128, false, 8>}, {"glds r128 pf kz8", launch_mm3<128, true, 8>},
      {"glds r64 kz4", launch_mm3<64, false, 4>},   {"glds r64 pf kz4", launch_mm3<64, true, 4>},
      {"glds r64 pf kz8", launch_mm3<64, true, 8>}, {"glds r128 pf kz16", launch_mm3<128, true, 16>},
      {"glds r128 pf kz8 nw8", launch_mm3<128, true, 8, 8>}, {"glds r64 pf kz8 nw8", launch_mm3<64, true, 8, 8>},
      // t4: the solver's tile shape family (rows x cols wave grid, stages, K slices)
      {"t4 r64 4x2 st2 kz4", launch_mm4<64, 4, 2, 2, 4>},  {"t4 r64 4x2 st3 kz4", launch_mm4<64, 4, 2, 3, 4>},
      {"t4 r64 4x2 st2 kz4 sched", launch_mm4<64, 4, 2, 2, 4, true>},
      {"t4 r64 2x4 st2 kz4", launch_mm4<64, 2, 4, 2, 4>},  {"t4 r64 4x4 st2 kz4", launch_mm4<64, 4, 4, 2, 4>},
      {"t4 r64 2x8 st2 kz4", launch_mm4<64, 2, 8, 2, 4>},  {"t4 r64 4x1 st2 kz4", launch_mm4<64, 4, 1, 2, 4>},
      {"t4 r64 2x2 st2 kz4", launch_mm4<64, 2, 2, 2, 4>},  {"t4 r64 2x4 st3 kz4", launch_mm4<64, 2, 4, 3, 4>},
      {"t4 r128 8x1 st2 kz8", launch_mm4<128, 8, 1, 2, 8>}, {"t4 r128 4x2 st2 kz8", launch_mm4<128, 4, 2, 2, 8>},
      {"t4 r128 8x2 st2 kz8", launch_mm4<128, 8, 2, 2, 8>}, {"t4 r128 4x4 st2 kz8", launch_mm4<128, 4, 4, 2, 8>},
      {"t4 r128 4x2 st2 kz4", launch_mm4<128, 4, 2, 2, 4>}, {"t4 r32 2x4 st3 kz4", launch_mm4<32, 2, 4, 3, 4>},
      {"t4 r32 2x4 st3 kz2", launch_mm4<32, 2, 4, 3, 2>},
  };
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  std::vector<double> hY((size_t)C * ld);
  for (auto& v : vs) {
    if (only && v.name.find(only) == std::string::npos) continue;
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
    g_red = false;
    CHK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; ++r) v.launch(S, V, Y, n, rows, ld, C, 0);
    CHK(hipEventRecord(e1, 0));
    CHK(hipEventSynchronize(e1));
    g_red = true;
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const double t = ms / reps;
    printf("{\"variant\": \"%s\", \"n\": %d, \"C\": %d, \"us\": %.2f, \"TFLOPs\": %.2f, \"maxrelerr\": %.2e}\n",
           v.name.c_str(), n, C, t * 1e3, 2.0 * n * n * C / (t * 1e-3) / 1e12, maxrel);
  }
  return 0;
}
