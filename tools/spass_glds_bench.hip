// spass_glds_bench.hip — LDS-DMA (global_load_lds) variant of the symmetric-tile S-pass.
// Builds standalone: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/spass_glds_bench.hip -o spass_glds_bench
//
// One wave streams whole 128x128 tiles (no cross-wave combination, so no barriers): rows go
// global -> LDS by global_load_lds_dwordx4 (1 KiB per wave instruction) into a private ring of
// D stages of 8 rows, the wave waits with a counted vmcnt for the oldest stage only, reads it
// with ds_read_b128 and does the same row / column arithmetic as k_spass_sym.  Persistent grid:
// wave g takes tiles g, g + G, ... of the flattened (instance, tile) list.
// Checked against the register-path tile kernel (same partial grid, same summation order per
// row; the column sums differ in order, so compared with a relative tolerance).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

typedef double dbl2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) double lds_f64;
typedef __attribute__((address_space(3))) dbl2 lds_dbl2;
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

// ---- reference: the register-path kernel as shipped (8 waves per tile, 16 rows per wave) ----
template <int SM>
__global__ void __launch_bounds__(512) k_ref(const double* __restrict__ S, int64_t inst, int nt, int ntiles, int ld,
                                             const double* __restrict__ v, double* __restrict__ pb) {
  constexpr int W = 8, ROWS = TS / W;
  const int lane = (int)__lane_id();
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = blockIdx.x / ntiles, t = blockIdx.x - b * ntiles;
  int I, J; tile_ij(t, nt, I, J);
  const double* T = S + (int64_t)b * inst + (int64_t)t * TS * TS;
  const double* v0 = v + (int64_t)b * ld;
  const int64_t nn = (int64_t)nt * nt * TS;
  double* pb0 = pb + (int64_t)b * nn;
  const int rrow = 4 * ((lane >> 5) & 1) + 2 * ((lane >> 4) & 1) + ((lane >> 3) & 1);
  const dbl2 vj0 = *(const dbl2*)(v0 + J * TS + 2 * lane);
  double cx = 0.0, cy = 0.0;
  __shared__ double cs[W][TS];
#pragma unroll 1
  for (int rb = 0; rb < ROWS / 8; ++rb) {
    const int r0 = w * ROWS + rb * 8;
    dbl2 sv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) sv[k] = __builtin_nontemporal_load((const dbl2*)(T + (r0 + k) * TS + 2 * lane));
    double a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const double vi0 = v0[I * TS + r0 + k];
      a[k] = __builtin_fma(sv[k].y, vj0.y, sv[k].x * vj0.x);
      cx = __builtin_fma(sv[k].x, vi0, cx);
      cy = __builtin_fma(sv[k].y, vi0, cy);
    }
    const double s0 = rs8(a);
    if (SM == 1 || SM == 2) { cx += s0 * 1e-300; continue; }
    if ((lane & 7) == 0) {
      if (SM == 4) __builtin_nontemporal_store(s0, pb0 + ((int64_t)I * nt + J) * TS + r0 + rrow);
      else pb0[((int64_t)I * nt + J) * TS + r0 + rrow] = s0;
    }
  }
  if (SM == 1 || SM == 3) { if (cx + cy == 123.456) pb0[0] = cx; return; }
  if (I != J) {
    cs[w][2 * lane] = cx;
    cs[w][2 * lane + 1] = cy;
    __syncthreads();
    if (threadIdx.x < TS) {
      double s = cs[0][threadIdx.x];
#pragma unroll
      for (int q = 1; q < W; ++q) s += cs[q][threadIdx.x];
      if (SM == 4) __builtin_nontemporal_store(s, pb0 + ((int64_t)J * nt + I) * TS + threadIdx.x);
      else pb0[((int64_t)J * nt + I) * TS + threadIdx.x] = s;
    }
  }
}

// s_waitcnt with only vmcnt constrained (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] | lgkmcnt[11:8] | vmcnt_hi[15:14])
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

template <int AUX>
__device__ __forceinline__ void glds16(const double* g, lds_f64* l) {
  __builtin_amdgcn_global_load_lds((const void*)g, (__attribute__((address_space(3))) void*)l, 16, 0, AUX);
}

// one wave = one workgroup; D stages of 8 rows (8 KiB) + 2 x (vJ, vI) slots (4 KiB)
template <int D, int AUX, int SM>
__global__ void __launch_bounds__(64) k_glds(const double* __restrict__ S, int64_t inst, int nt, int ntiles, int batch,
                                             int ld, const double* __restrict__ v, double* __restrict__ pb) {
  __shared__ __attribute__((aligned(16))) double lds_raw[D * 8 * TS + 5 * TS];
  lds_f64* const ring = (lds_f64*)lds_raw;
  lds_f64* const vsl = ring + D * 8 * TS;   // [2][vJ | vI][128]
  lds_f64* const osl = vsl + 4 * TS;        // row sums of the current tile (SM 2)
  const int lane = (int)__lane_id();
  const int G = gridDim.x, g = blockIdx.x;
  const int total = batch * ntiles;
  const int my_tiles = g < total ? (total - 1 - g) / G + 1 : 0;
  const int nbat = my_tiles * (TS / 8);
  const int64_t nn = (int64_t)nt * nt * TS;
  const int rrow = 4 * ((lane >> 5) & 1) + 2 * ((lane >> 4) & 1) + ((lane >> 3) & 1);

  // producer: issue batch q (tile q / 16 of this wave, rows 8 (q % 16) ..)
  auto issue = [&](int q) {
    const int k = q >> 4, rb = q & 15;
    const int tt = g + k * G;
    const int b = tt / ntiles, t = tt - b * ntiles;
    const double* T = S + (int64_t)b * inst + (int64_t)t * TS * TS + rb * 8 * TS + 2 * lane;
    lds_f64* st = ring + (q % D) * 8 * TS;
#pragma unroll
    for (int r = 0; r < 8; ++r) glds16<AUX>(T + r * TS, st + r * TS);
    if (rb == 0) {
      int I, J; tile_ij(t, nt, I, J);
      const double* vb = v + (int64_t)b * ld;
      lds_f64* sl = vsl + (k & 1) * 2 * TS;
      glds16<0>(vb + J * TS + 2 * lane, sl);
      glds16<0>(vb + I * TS + 2 * lane, sl + TS);
    }
  };
  const int pro = nbat < D ? nbat : D;
  for (int q = 0; q < pro; ++q) issue(q);
  double cx = 0.0, cy = 0.0, sink = 0.0;
  dbl2 vj = dbl2{0.0, 0.0};
  int I = 0, J = 0, b = 0;
  for (int q = 0; q < nbat; ++q) {
    const int k = q >> 4, rb = q & 15;
    // batch q landed: at most (D - 1) later batches (8 glds + 1 store each, + tile-start vector
    // glds / column-sum store: the count is a lower bound, so the wait is conservative)
    if (q + D - 1 < nbat) wait_vm<(D - 1) * 8>();
    else wait_vm<0>();
    if (rb == 0) {
      if (SM == 5 && k > 0) wait_vm<0>();
      if ((SM == 2 || SM == 4) && k > 0) {   // previous tile's results, issued right after a wait
        const dbl2 rsum = *(const lds_dbl2*)(osl + 2 * lane);
        double* pbp = SM == 4 ? pb + (int64_t)g * 2 * TS - ((int64_t)I * nt + J) * TS : pb + (int64_t)b * nn;
        *(dbl2*)(pbp + ((int64_t)I * nt + J) * TS + 2 * lane) = rsum;
        if (I != J) *(dbl2*)(pbp + (SM == 4 ? ((int64_t)I * nt + J) * TS + TS : ((int64_t)J * nt + I) * TS) + 2 * lane) = dbl2{cx, cy};
      }
      const int tt = g + k * G;
      b = tt / ntiles;
      tile_ij(tt - b * ntiles, nt, I, J);
      cx = cy = 0.0;
      vj = *(const lds_dbl2*)(vsl + (k & 1) * 2 * TS + 2 * lane);
    }
    const lds_f64* st = ring + (q % D) * 8 * TS;
    const lds_f64* vi = vsl + (k & 1) * 2 * TS + TS + rb * 8;
    dbl2 sv[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) sv[r] = *(const lds_dbl2*)(st + r * TS + 2 * lane);
    double a[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const double vi0 = vi[r];
      a[r] = __builtin_fma(sv[r].y, vj.y, sv[r].x * vj.x);
      cx = __builtin_fma(sv[r].x, vi0, cx);
      cy = __builtin_fma(sv[r].y, vi0, cy);
    }
    const double s0 = rs8(a);
    double* pb0 = pb + (int64_t)b * nn;
    if (SM == 0) {
      if ((lane & 7) == 0) pb0[((int64_t)I * nt + J) * TS + rb * 8 + rrow] = s0;
      if (rb == 15 && I != J) *(dbl2*)(pb0 + ((int64_t)J * nt + I) * TS + 2 * lane) = dbl2{cx, cy};
    } else if (SM == 2 || SM == 4) {
      if ((lane & 7) == 0) osl[rb * 8 + rrow] = s0;
    } else {
      sink += s0 + cx + cy;
    }
    __builtin_amdgcn_s_waitcnt((15) | (7 << 4) | (0 << 8) | (3 << 14));   // lgkmcnt(0): stage reads done
    if (q + D < nbat) issue(q + D);
  }
  if (SM == 2 && nbat > 0) {
    const dbl2 rsum = *(const lds_dbl2*)(osl + 2 * lane);
    double* pbp = pb + (int64_t)b * nn;
    *(dbl2*)(pbp + ((int64_t)I * nt + J) * TS + 2 * lane) = rsum;
    if (I != J) *(dbl2*)(pbp + ((int64_t)J * nt + I) * TS + 2 * lane) = dbl2{cx, cy};
  }
  if ((SM == 1 || SM == 5) && sink == 123.456) pb[0] = sink;
}


// streamer + writer: wave 0 streams and computes (its vmcnt sees only its glds), wave 1 issues
// the partial-sum stores of finished tiles, handed over through LDS with one s_barrier per tile
template <int D, bool NTS>
__global__ void __launch_bounds__(128) k_glds_w(const double* __restrict__ S, int64_t inst, int nt, int ntiles, int batch,
                                                int ld, const double* __restrict__ v, double* __restrict__ pb) {
  __shared__ __attribute__((aligned(16))) double lds_raw[D * 8 * TS + 8 * TS];
  lds_f64* const ring = (lds_f64*)lds_raw;
  lds_f64* const vsl = ring + D * 8 * TS;   // [2][vJ | vI][128]
  lds_f64* const osl = vsl + 4 * TS;        // [2][row sums | column sums][128]
  const int lane = (int)__lane_id();
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int G = gridDim.x, g = blockIdx.x;
  const int total = batch * ntiles;
  const int my_tiles = g < total ? (total - 1 - g) / G + 1 : 0;
  const int64_t nn = (int64_t)nt * nt * TS;
  if (wv == 1) {   // writer
    for (int k = 0; k < my_tiles; ++k) {
      __builtin_amdgcn_s_barrier();
      const int tt = g + k * G;
      const int b = tt / ntiles;
      int I, J; tile_ij(tt - b * ntiles, nt, I, J);
      const lds_f64* o = osl + (k & 1) * 2 * TS;
      const dbl2 rsum = *(const lds_dbl2*)(o + 2 * lane);
      const dbl2 csum = *(const lds_dbl2*)(o + TS + 2 * lane);
      double* pbp = pb + (int64_t)b * nn;
      if (NTS) {
        __builtin_nontemporal_store(rsum, (dbl2*)(pbp + ((int64_t)I * nt + J) * TS + 2 * lane));
        if (I != J) __builtin_nontemporal_store(csum, (dbl2*)(pbp + ((int64_t)J * nt + I) * TS + 2 * lane));
      } else {
        *(dbl2*)(pbp + ((int64_t)I * nt + J) * TS + 2 * lane) = rsum;
        if (I != J) *(dbl2*)(pbp + ((int64_t)J * nt + I) * TS + 2 * lane) = csum;
      }
    }
    return;
  }
  const int nbat = my_tiles * (TS / 8);
  const int rrow = 4 * ((lane >> 5) & 1) + 2 * ((lane >> 4) & 1) + ((lane >> 3) & 1);
  auto issue = [&](int q) {
    const int k = q >> 4, rb = q & 15;
    const int tt = g + k * G;
    const int b = tt / ntiles, t = tt - b * ntiles;
    const double* T = S + (int64_t)b * inst + (int64_t)t * TS * TS + rb * 8 * TS + 2 * lane;
    lds_f64* st = ring + (q % D) * 8 * TS;
#pragma unroll
    for (int r = 0; r < 8; ++r) glds16<2>(T + r * TS, st + r * TS);
    if (rb == 0) {
      int I, J; tile_ij(t, nt, I, J);
      const double* vb = v + (int64_t)b * ld;
      lds_f64* sl = vsl + (k & 1) * 2 * TS;
      glds16<0>(vb + J * TS + 2 * lane, sl);
      glds16<0>(vb + I * TS + 2 * lane, sl + TS);
    }
  };
  const int pro = nbat < D ? nbat : D;
  for (int q = 0; q < pro; ++q) issue(q);
  double cx = 0.0, cy = 0.0;
  dbl2 vj = dbl2{0.0, 0.0};
  for (int q = 0; q < nbat; ++q) {
    const int k = q >> 4, rb = q & 15;
    if (q + D - 1 < nbat) wait_vm<(D - 1) * 8>();
    else wait_vm<0>();
    if (rb == 0) {
      cx = cy = 0.0;
      vj = *(const lds_dbl2*)(vsl + (k & 1) * 2 * TS + 2 * lane);
    }
    const lds_f64* st = ring + (q % D) * 8 * TS;
    const lds_f64* vi = vsl + (k & 1) * 2 * TS + TS + rb * 8;
    dbl2 sv[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) sv[r] = *(const lds_dbl2*)(st + r * TS + 2 * lane);
    double a[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const double vi0 = vi[r];
      a[r] = __builtin_fma(sv[r].y, vj.y, sv[r].x * vj.x);
      cx = __builtin_fma(sv[r].x, vi0, cx);
      cy = __builtin_fma(sv[r].y, vi0, cy);
    }
    const double s0 = rs8(a);
    lds_f64* o = osl + (k & 1) * 2 * TS;
    if ((lane & 7) == 0) o[rb * 8 + rrow] = s0;
    if (rb == 15) *(lds_dbl2*)(o + TS + 2 * lane) = dbl2{cx, cy};
    __builtin_amdgcn_s_waitcnt((15) | (7 << 4) | (0 << 8) | (3 << 14));   // lgkmcnt(0)
    if (q + D < nbat) issue(q + D);
    if (rb == 15) __builtin_amdgcn_s_barrier();   // hand the tile to the writer
  }
}

// super-tiles: one 8-wave workgroup per SB x SB block of stored tiles; row sums accumulate over
// the block's tile columns and column sums over its tile rows, so a workgroup writes one
// 8*SB*128-byte partial per side instead of one per tile (partial grid [b][P][Q][SB*128]).
template <int SB>
__global__ void __launch_bounds__(512) k_sup(const double* __restrict__ S, int64_t inst, int nt, int nst, int nsup,
                                             int ld, const double* __restrict__ v, double* __restrict__ pp) {
  constexpr int W = 8, ROWS = TS / W, SW = SB * TS;
  __shared__ double red[W][SW];
  __shared__ double obuf[2][SW];
  const int lane = (int)__lane_id();
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = blockIdx.x / nsup, u = blockIdx.x - b * nsup;
  int P, Q; tile_ij(u, nst, P, Q);
  const double* Sb = S + (int64_t)b * inst;
  const double* v0 = v + (int64_t)b * ld;
  const int rrow = 4 * ((lane >> 5) & 1) + 2 * ((lane >> 4) & 1) + ((lane >> 3) & 1);
  double racc[SB][ROWS / 8];
  double cax[SB], cay[SB];
#pragma unroll
  for (int i = 0; i < SB; ++i) {
    cax[i] = cay[i] = 0.0;
#pragma unroll
    for (int r = 0; r < ROWS / 8; ++r) racc[i][r] = 0.0;
  }
#pragma unroll
  for (int il = 0; il < SB; ++il) {
    const int I = SB * P + il;
    if (I >= nt) break;
#pragma unroll
    for (int jl = 0; jl < SB; ++jl) {
      const int J = SB * Q + jl;
      if (J >= nt || J < I) continue;
      const int64_t toff = ((int64_t)I * nt - (int64_t)I * (I - 1) / 2 + (J - I)) * TS * TS;
      const double* T = Sb + toff;
      const dbl2 vj = *(const dbl2*)(v0 + J * TS + 2 * lane);
      const bool off = I != J;
#pragma unroll
      for (int rb = 0; rb < ROWS / 8; ++rb) {
        const int r0 = w * ROWS + rb * 8;
        dbl2 sv[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) sv[k] = __builtin_nontemporal_load((const dbl2*)(T + (r0 + k) * TS + 2 * lane));
        double a[8];
        double tx = 0.0, ty = 0.0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const double vi0 = v0[I * TS + r0 + k];
          a[k] = __builtin_fma(sv[k].y, vj.y, sv[k].x * vj.x);
          tx = __builtin_fma(sv[k].x, vi0, tx);
          ty = __builtin_fma(sv[k].y, vi0, ty);
        }
        if (off) { cax[jl] += tx; cay[jl] += ty; }
        racc[il][rb] += rs8(a);
      }
    }
  }
#pragma unroll
  for (int il = 0; il < SB; ++il)
#pragma unroll
    for (int rb = 0; rb < ROWS / 8; ++rb)
      if ((lane & 7) == 0) obuf[0][il * TS + w * ROWS + rb * 8 + rrow] = racc[il][rb];
#pragma unroll
  for (int jl = 0; jl < SB; ++jl) {
    red[w][jl * TS + 2 * lane] = cax[jl];
    red[w][jl * TS + 2 * lane + 1] = cay[jl];
  }
  __syncthreads();
  for (int t = threadIdx.x; t < SW; t += 512) {
    double c = red[0][t];
#pragma unroll
    for (int q = 1; q < W; ++q) c += red[q][t];
    if (P == Q) obuf[0][t] += c;
    else obuf[1][t] = c;
  }
  __syncthreads();
  double* pb0 = pp + (int64_t)b * nst * nst * SW;
  for (int t = threadIdx.x; t < SW; t += 512) {
    pb0[((int64_t)P * nst + Q) * SW + t] = obuf[0][t];
    if (P != Q) pb0[((int64_t)Q * nst + P) * SW + t] = obuf[1][t];
  }
}

template <int SB, bool NTS = false>
__global__ void __launch_bounds__(512) k_sup2(const double* __restrict__ S, int64_t inst, int nt, int nst, int nsup,
                                             int ld, const double* __restrict__ v, double* __restrict__ pp) {
  constexpr int W = 8, ROWS = TS / W, SW = SB * TS;
  __shared__ double red[W][SW];
  __shared__ double obuf[2][SW];
  const int lane = (int)__lane_id();
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = blockIdx.x / nsup, u = blockIdx.x - b * nsup;
  int P, Q; tile_ij(u, nst, P, Q);
  const double* Sb = S + (int64_t)b * inst;
  const double* v0 = v + (int64_t)b * ld;
  const int rrow = 4 * ((lane >> 5) & 1) + 2 * ((lane >> 4) & 1) + ((lane >> 3) & 1);
  double racc[SB][ROWS / 8];
#pragma unroll
  for (int i = 0; i < SB; ++i) {
#pragma unroll
    for (int r = 0; r < ROWS / 8; ++r) racc[i][r] = 0.0;
  }
  for (int jl = 0; jl < SB; ++jl) { red[w][jl * TS + 2 * lane] = 0.0; red[w][jl * TS + 2 * lane + 1] = 0.0; }
#pragma unroll
  for (int il = 0; il < SB; ++il) {
    const int I = SB * P + il;
    if (I >= nt) break;
#pragma unroll 1
    for (int jl = 0; jl < SB; ++jl) {
      const int J = SB * Q + jl;
      if (J >= nt || J < I) continue;
      const int64_t toff = ((int64_t)I * nt - (int64_t)I * (I - 1) / 2 + (J - I)) * TS * TS;
      const double* T = Sb + toff;
      const dbl2 vj = *(const dbl2*)(v0 + J * TS + 2 * lane);
      const bool off = I != J;
      double txs = 0.0, tys = 0.0;
#pragma unroll 1
      for (int rb = 0; rb < ROWS / 8; ++rb) {
        const int r0 = w * ROWS + rb * 8;
        dbl2 sv[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) sv[k] = __builtin_nontemporal_load((const dbl2*)(T + (r0 + k) * TS + 2 * lane));
        double a[8];
        double tx = 0.0, ty = 0.0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const double vi0 = v0[I * TS + r0 + k];
          a[k] = __builtin_fma(sv[k].y, vj.y, sv[k].x * vj.x);
          tx = __builtin_fma(sv[k].x, vi0, tx);
          ty = __builtin_fma(sv[k].y, vi0, ty);
        }
        txs += tx; tys += ty;
        const double rs = rs8(a);
        if (rb == 0) racc[il][0] += rs;
        else racc[il][1] += rs;
      }
      if (off) { red[w][jl * TS + 2 * lane] += txs; red[w][jl * TS + 2 * lane + 1] += tys; }
    }
  }
#pragma unroll
  for (int il = 0; il < SB; ++il)
#pragma unroll
    for (int rb = 0; rb < ROWS / 8; ++rb)
      if ((lane & 7) == 0) obuf[0][il * TS + w * ROWS + rb * 8 + rrow] = racc[il][rb];
  __syncthreads();
  for (int t = threadIdx.x; t < SW; t += 512) {
    double c = red[0][t];
#pragma unroll
    for (int q = 1; q < W; ++q) c += red[q][t];
    if (P == Q) obuf[0][t] += c;
    else obuf[1][t] = c;
  }
  __syncthreads();
  double* pb0 = pp + (int64_t)b * nst * nst * SW;
  for (int t = threadIdx.x; t < SW; t += 512) {
    if (NTS) {
      __builtin_nontemporal_store(obuf[0][t], pb0 + ((int64_t)P * nst + Q) * SW + t);
      if (P != Q) __builtin_nontemporal_store(obuf[1][t], pb0 + ((int64_t)Q * nst + P) * SW + t);
    } else {
      pb0[((int64_t)P * nst + Q) * SW + t] = obuf[0][t];
      if (P != Q) pb0[((int64_t)Q * nst + P) * SW + t] = obuf[1][t];
    }
  }
}

// persistent super-tiles: one 8-wave workgroup per CU walks units u = g, g + G, ... (SB x SB
// blocks of tiles) and keeps each unit's two partial vectors in LDS, writing FL units' results
// in one burst: HBM sees reads only between the bursts.
template <int SB, int FL, bool NTS>
__global__ void __launch_bounds__(512) k_psup(const double* __restrict__ S, int64_t inst, int nt, int nst, int nsup,
                                              int batch, int ld, const double* __restrict__ v, double* __restrict__ pp) {
  constexpr int W = 8, ROWS = TS / W, SW = SB * TS;
  __shared__ double red[W][SW];
  __shared__ double outb[FL][2][SW];
  const int lane = (int)__lane_id();
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int G = gridDim.x, g = blockIdx.x;
  const int total = batch * nsup;
  const int my = g < total ? (total - 1 - g) / G + 1 : 0;
  const int rrow = 4 * ((lane >> 5) & 1) + 2 * ((lane >> 4) & 1) + ((lane >> 3) & 1);
  auto flush = [&](int k0, int cnt) {
    __syncthreads();
    for (int s = 0; s < cnt; ++s) {
      const int uu = g + (k0 + s) * G;
      const int b = uu / nsup;
      int P, Q; tile_ij(uu - b * nsup, nst, P, Q);
      double* pb0 = pp + (int64_t)b * nst * nst * SW;
      for (int t = threadIdx.x; t < SW; t += 512) {
        if (NTS) {
          __builtin_nontemporal_store(outb[s][0][t], pb0 + ((int64_t)P * nst + Q) * SW + t);
          if (P != Q) __builtin_nontemporal_store(outb[s][1][t], pb0 + ((int64_t)Q * nst + P) * SW + t);
        } else {
          pb0[((int64_t)P * nst + Q) * SW + t] = outb[s][0][t];
          if (P != Q) pb0[((int64_t)Q * nst + P) * SW + t] = outb[s][1][t];
        }
      }
    }
    __syncthreads();
  };
  int k0 = 0;
  for (int k = 0; k < my; ++k) {
    const int u = g + k * G;
    const int b = u / nsup;
    int P, Q; tile_ij(u - b * nsup, nst, P, Q);
    const int slot = k - k0;
    const double* Sb = S + (int64_t)b * inst;
    const double* v0 = v + (int64_t)b * ld;
    double racc[SB][ROWS / 8];
#pragma unroll
    for (int i = 0; i < SB; ++i)
#pragma unroll
      for (int r = 0; r < ROWS / 8; ++r) racc[i][r] = 0.0;
    for (int jl = 0; jl < SB; ++jl) { red[w][jl * TS + 2 * lane] = 0.0; red[w][jl * TS + 2 * lane + 1] = 0.0; }
#pragma unroll
    for (int il = 0; il < SB; ++il) {
      const int I = SB * P + il;
      if (I >= nt) break;
#pragma unroll 1
      for (int jl = 0; jl < SB; ++jl) {
        const int J = SB * Q + jl;
        if (J >= nt || J < I) continue;
        const int64_t toff = ((int64_t)I * nt - (int64_t)I * (I - 1) / 2 + (J - I)) * TS * TS;
        const double* T = Sb + toff;
        const dbl2 vj = *(const dbl2*)(v0 + J * TS + 2 * lane);
        double txs = 0.0, tys = 0.0;
#pragma unroll 1
        for (int rb = 0; rb < ROWS / 8; ++rb) {
          const int r0 = w * ROWS + rb * 8;
          dbl2 sv[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) sv[q] = __builtin_nontemporal_load((const dbl2*)(T + (r0 + q) * TS + 2 * lane));
          double a[8];
          double tx = 0.0, ty = 0.0;
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const double vi0 = v0[I * TS + r0 + q];
            a[q] = __builtin_fma(sv[q].y, vj.y, sv[q].x * vj.x);
            tx = __builtin_fma(sv[q].x, vi0, tx);
            ty = __builtin_fma(sv[q].y, vi0, ty);
          }
          txs += tx; tys += ty;
          const double rs = rs8(a);
          if (rb == 0) racc[il][0] += rs;
          else racc[il][1] += rs;
        }
        if (I != J) { red[w][jl * TS + 2 * lane] += txs; red[w][jl * TS + 2 * lane + 1] += tys; }
      }
    }
#pragma unroll
    for (int il = 0; il < SB; ++il)
#pragma unroll
      for (int rb = 0; rb < ROWS / 8; ++rb)
        if ((lane & 7) == 0) outb[slot][0][il * TS + w * ROWS + rb * 8 + rrow] = racc[il][rb];
    __syncthreads();
    for (int t = threadIdx.x; t < SW; t += 512) {
      double c = red[0][t];
#pragma unroll
      for (int q = 1; q < W; ++q) c += red[q][t];
      if (P == Q) outb[slot][0][t] += c;
      else outb[slot][1][t] = c;
    }
    __syncthreads();
    if (slot + 1 == FL) { flush(k0, FL); k0 = k + 1; }
  }
  if (my > k0) flush(k0, my - k0);
}

template <int SB>
__global__ void k_gath(const double* pp, int nst, int ld, double* y) {
  constexpr int SW = SB * TS;
  const int b = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ld) return;
  const int P = i / SW, c = i - P * SW;
  const double* q = pp + (int64_t)b * nst * nst * SW + (int64_t)P * nst * SW + c;
  double acc = 0.0;
  for (int j = 0; j < nst; ++j) acc += q[(int64_t)j * SW];
  y[(int64_t)b * ld + i] = acc;
}

__global__ void k_fill(double* p, int64_t n, uint64_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull; z = (z ^ (z >> 27)) * 0x94D049BB133111EBull; z ^= z >> 31;
    p[i] = (double)(z >> 11) * (1.0 / 9007199254740992.0) - 0.5;
  }
}

// pure LDS-DMA stream of the same bytes (one wave per WG, D stages of 8 KiB, no arithmetic)
template <int D, int AUX>
__global__ void __launch_bounds__(64) k_glds_stream(const double* __restrict__ S, int64_t nchunks, double* out) {
  __shared__ __attribute__((aligned(16))) double lds_raw[D * 8 * TS];
  lds_f64* const ring = (lds_f64*)lds_raw;
  const int lane = (int)__lane_id();
  const int64_t G = gridDim.x, g = blockIdx.x;
  const int64_t my = g < nchunks ? (nchunks - 1 - g) / G + 1 : 0;
  auto issue = [&](int64_t q) {
    const double* src = S + (g + q * G) * 8 * TS + 2 * lane;
    lds_f64* st = ring + (q % D) * 8 * TS;
#pragma unroll
    for (int r = 0; r < 8; ++r) glds16<AUX>(src + r * TS, st + r * TS);
  };
  for (int64_t q = 0; q < (my < D ? my : D); ++q) issue(q);
  double acc = 0.0;
  for (int64_t q = 0; q < my; ++q) {
    if (q + D - 1 < my) wait_vm<(D - 1) * 8>();
    else wait_vm<0>();
    const dbl2 x = *(const lds_dbl2*)(ring + (q % D) * 8 * TS + 2 * lane);
    acc += x.x + x.y;
    __builtin_amdgcn_s_waitcnt((15) | (7 << 4) | (0 << 8) | (3 << 14));
    if (q + D < my) issue(q + D);
  }
  if (acc == 123.456) out[0] = acc;
}

template <typename F>
double time_ms(F launch, int reps, hipEvent_t e0, hipEvent_t e1) {
  for (int r = 0; r < 2; ++r) launch();
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0, 0));
  for (int r = 0; r < reps; ++r) launch();
  CHK(hipEventRecord(e1, 0));
  CHK(hipEventSynchronize(e1));
  float ms = 0; CHK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 4000;
  const int B = argc > 2 ? atoi(argv[2]) : 64;
  const int reps = argc > 3 ? atoi(argv[3]) : 20;
  const int ld = (n + TS - 1) / TS * TS, nt = ld / TS, ntiles = nt * (nt + 1) / 2;
  const int64_t inst = (int64_t)ntiles * TS * TS;
  double *S, *v, *pb, *pb2;
  const size_t pbn = (size_t)B * nt * nt * TS;
  CHK(hipMalloc(&S, (size_t)B * inst * 8));
  CHK(hipMalloc(&v, (size_t)B * ld * 8));
  CHK(hipMalloc(&pb, pbn * 8));
  CHK(hipMalloc(&pb2, pbn * 8));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, S, (int64_t)B * inst, 1ull);
  hipLaunchKernelGGL(k_fill, dim3(256), dim3(256), 0, 0, v, (int64_t)B * ld, 7ull);
  CHK(hipMemset(pb, 0, pbn * 8));
  CHK(hipDeviceSynchronize());
  const double bytes = (double)B * inst * 8;
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  const double ms_rns = time_ms([&] { hipLaunchKernelGGL(k_ref<1>, dim3(B * ntiles), dim3(512), 0, 0, S, inst, nt, ntiles, ld, v, pb); }, reps, e0, e1);
  printf("{\"variant\": \"ref NOSTORE\", \"ms\": %.4f, \"TBps\": %.3f}\n", ms_rns, bytes / (ms_rns * 1e-3) / 1e12);
  const double ms_c = time_ms([&] { hipLaunchKernelGGL(k_ref<2>, dim3(B * ntiles), dim3(512), 0, 0, S, inst, nt, ntiles, ld, v, pb); }, reps, e0, e1);
  printf("{\"variant\": \"ref column stores only\", \"ms\": %.4f, \"TBps\": %.3f}\n", ms_c, bytes / (ms_c * 1e-3) / 1e12);
  const double ms_r = time_ms([&] { hipLaunchKernelGGL(k_ref<3>, dim3(B * ntiles), dim3(512), 0, 0, S, inst, nt, ntiles, ld, v, pb); }, reps, e0, e1);
  printf("{\"variant\": \"ref row stores only\", \"ms\": %.4f, \"TBps\": %.3f}\n", ms_r, bytes / (ms_r * 1e-3) / 1e12);
  const double ms_n = time_ms([&] { hipLaunchKernelGGL(k_ref<4>, dim3(B * ntiles), dim3(512), 0, 0, S, inst, nt, ntiles, ld, v, pb); }, reps, e0, e1);
  printf("{\"variant\": \"ref nt stores\", \"ms\": %.4f, \"TBps\": %.3f}\n", ms_n, bytes / (ms_n * 1e-3) / 1e12);
  const double ms_ref = time_ms([&] { hipLaunchKernelGGL(k_ref<0>, dim3(B * ntiles), dim3(512), 0, 0, S, inst, nt, ntiles, ld, v, pb); }, reps, e0, e1);
  printf("{\"variant\": \"ref (k_spass_sym shape)\", \"n\": %d, \"B\": %d, \"ms\": %.4f, \"TBps\": %.3f}\n", n, B, ms_ref, bytes / (ms_ref * 1e-3) / 1e12);
  std::vector<double> ref(pbn), got(pbn);
  CHK(hipMemcpy(ref.data(), pb, pbn * 8, hipMemcpyDeviceToHost));
  fflush(stdout);
  struct V { const char* name; void (*fn)(const double*, int64_t, int, int, int, int, const double*, double*); int wpc; };
  V vars[] = {
      {"glds D4 nt wpc4", k_glds<4, 2, 0>, 4},
      {"glds D4 nt wpc4 NOSTORE", k_glds<4, 2, 1>, 4},
      {"glds D4 nt wpc4 TILESTORE", k_glds<4, 2, 2>, 4},

  };
  {
    double* y0; double* y1;
    CHK(hipMalloc(&y0, (size_t)B * ld * 8));
    CHK(hipMalloc(&y1, (size_t)B * ld * 8));
    std::vector<double> ya((size_t)B * ld), yb((size_t)B * ld);
    hipLaunchKernelGGL(k_gath<1>, dim3(ld / 128, B), dim3(128), 0, 0, pb, nt, ld, y0);
    CHK(hipMemcpy(ya.data(), y0, ya.size() * 8, hipMemcpyDeviceToHost));
    struct SV2 { const char* name; void (*fn)(const double*, int64_t, int, int, int, int, const double*, double*); void (*g)(const double*, int, int, double*); int sb; };
    SV2 sv2[] = {{"super 1x1", k_sup<1>, k_gath<1>, 1}, {"super 2x2", k_sup<2>, k_gath<2>, 2}, {"super 4x4", k_sup<4>, k_gath<4>, 4},
                   {"super2 2x2", k_sup2<2>, k_gath<2>, 2}, {"super2 4x4", k_sup2<4>, k_gath<4>, 4}, {"super2 4x4 ntstore", k_sup2<4, true>, k_gath<4>, 4}, {"super2 2x2 ntstore", k_sup2<2, true>, k_gath<2>, 2}};
    struct SV3 { const char* name; void (*fn)(const double*, int64_t, int, int, int, int, int, const double*, double*); void (*g)(const double*, int, int, double*); int sb; int grid; };
    SV3 sv3[] = {{"persist 2x2 FL32 g256", k_psup<2, 32, false>, k_gath<2>, 2, 256},
                 {"persist 2x2 FL32 g256 nts", k_psup<2, 32, true>, k_gath<2>, 2, 256},
                 {"persist 2x2 FL8 g512", k_psup<2, 8, false>, k_gath<2>, 2, 512},
                 {"persist 2x2 FL16 g256", k_psup<2, 16, false>, k_gath<2>, 2, 256},
                 {"persist 4x4 FL8 g256", k_psup<4, 8, false>, k_gath<4>, 4, 256}};
    for (const SV3& X : sv3) {
      const int nst = (nt + X.sb - 1) / X.sb, nsup = nst * (nst + 1) / 2;
      CHK(hipMemset(pb2, 0, pbn * 8));
      const double ms = time_ms([&] { hipLaunchKernelGGL(X.fn, dim3(X.grid), dim3(512), 0, 0, S, inst, nt, nst, nsup, B, ld, v, pb2); }, reps, e0, e1);
      CHK(hipGetLastError());
      hipLaunchKernelGGL(X.g, dim3(ld / 128, B), dim3(128), 0, 0, pb2, nst, ld, y1);
      CHK(hipMemcpy(yb.data(), y1, yb.size() * 8, hipMemcpyDeviceToHost));
      double err = 0.0, nrm = 0.0;
      for (size_t i = 0; i < ya.size(); ++i) { err = fmax(err, fabs(yb[i] - ya[i])); nrm = fmax(nrm, fabs(ya[i])); }
      printf("{\"variant\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f, \"y_maxrelerr\": %.2e}\n", X.name, ms, bytes / (ms * 1e-3) / 1e12, err / nrm);
      fflush(stdout);
    }
    for (const SV2& X : sv2) {
      const int nst = (nt + X.sb - 1) / X.sb, nsup = nst * (nst + 1) / 2;
      CHK(hipMemset(pb2, 0, pbn * 8));
      const double ms = time_ms([&] { hipLaunchKernelGGL(X.fn, dim3(B * nsup), dim3(512), 0, 0, S, inst, nt, nst, nsup, ld, v, pb2); }, reps, e0, e1);
      hipLaunchKernelGGL(X.g, dim3(ld / 128, B), dim3(128), 0, 0, pb2, nst, ld, y1);
      CHK(hipMemcpy(yb.data(), y1, yb.size() * 8, hipMemcpyDeviceToHost));
      double err = 0.0, nrm = 0.0;
      for (size_t i = 0; i < ya.size(); ++i) { err = fmax(err, fabs(yb[i] - ya[i])); nrm = fmax(nrm, fabs(ya[i])); }
      printf("{\"variant\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f, \"y_maxrelerr\": %.2e}\n", X.name, ms, bytes / (ms * 1e-3) / 1e12, err / nrm);
      fflush(stdout);
    }
  }
  {
    int occ = 0;
    CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_glds_w<4, false>, 128, 0));
    int occ3 = 0;
    CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ3, k_glds_w<3, false>, 128, 0));
    int occ2 = 0;
    CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ2, k_glds_w<2, false>, 128, 0));
    printf("{\"occupancy\": [%d, %d, %d]}\n", occ2, occ3, occ);
    struct W { const char* name; void (*fn)(const double*, int64_t, int, int, int, int, const double*, double*); int wpc; };
    W ws[] = {{"glds+writer D4", k_glds_w<4, false>, occ}, {"glds+writer D4 ntstore", k_glds_w<4, true>, occ},
              {"glds+writer D2 ntstore", k_glds_w<2, true>, occ2}};
    for (const W& X : ws) {
      CHK(hipMemset(pb2, 0, pbn * 8));
      const int grid = 256 * X.wpc;
      const double ms = time_ms([&] { hipLaunchKernelGGL(X.fn, dim3(grid), dim3(128), 0, 0, S, inst, nt, ntiles, B, ld, v, pb2); }, reps, e0, e1);
      CHK(hipMemcpy(got.data(), pb2, pbn * 8, hipMemcpyDeviceToHost));
      double err = 0.0, nrm = 0.0;
      for (size_t i = 0; i < pbn; ++i) { err = fmax(err, fabs(got[i] - ref[i])); nrm = fmax(nrm, fabs(ref[i])); }
      printf("{\"variant\": \"%s wpc%d\", \"ms\": %.4f, \"TBps\": %.3f, \"maxrelerr\": %.2e}\n", X.name, X.wpc, ms, bytes / (ms * 1e-3) / 1e12, err / nrm);
      fflush(stdout);
    }
  }
  for (const V& X : vars) {
    CHK(hipMemset(pb2, 0, pbn * 8));
    const int grid = 256 * X.wpc;
    const double ms = time_ms([&] { hipLaunchKernelGGL(X.fn, dim3(grid), dim3(64), 0, 0, S, inst, nt, ntiles, B, ld, v, pb2); }, reps, e0, e1);
    CHK(hipMemcpy(got.data(), pb2, pbn * 8, hipMemcpyDeviceToHost));
    double err = 0.0, nrm = 0.0;
    for (size_t i = 0; i < pbn; ++i) { err = fmax(err, fabs(got[i] - ref[i])); nrm = fmax(nrm, fabs(ref[i])); }
    printf("{\"variant\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f, \"maxrelerr\": %.2e}\n", X.name, ms, bytes / (ms * 1e-3) / 1e12, err / nrm);
    fflush(stdout);
  }
  const int64_t nchunks = (int64_t)B * inst / (8 * TS);
  struct SV { const char* name; void (*fn)(const double*, int64_t, double*); int wpc; };
  SV svars[] = {{"glds stream D2 nt wpc8", k_glds_stream<2, 2>, 8}, {"glds stream D3 nt wpc6", k_glds_stream<3, 2>, 6},
                {"glds stream D4 nt wpc4", k_glds_stream<4, 2>, 4}, {"glds stream D3 plain wpc6", k_glds_stream<3, 0>, 6}};
  for (const SV& X : svars) {
    const double ms = time_ms([&] { hipLaunchKernelGGL(X.fn, dim3(256 * X.wpc), dim3(64), 0, 0, S, nchunks, pb2); }, reps, e0, e1);
    printf("{\"variant\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f}\n", X.name, ms, bytes / (ms * 1e-3) / 1e12);
    fflush(stdout);
  }
  return 0;
}
