// riptrm_wave.h — 64-lane wave reductions for fp64 without LDS (gfx950).
//
// A sum over the wave in six VALU steps: two quad_perm DPP exchanges (lane ^ 1, lane ^ 2), the
// half-row and row mirrors (lane i <-> 7 - i, i <-> 15 - i), then v_permlane16_swap (row pairs)
// and v_permlane32_swap (wave halves).  Every step pairs lanes by an involution and adds the
// two partial sums, so all 64 lanes end with the bitwise-identical result (a + b == b + a) and
// control flow that depends on it stays uniform.  Replaces a ds_bpermute butterfly (12 LDS-path
// exchanges per double) on the latency-critical state machines.
#pragma once
#include <hip/hip_runtime.h>

namespace riptrm_wave {

template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

constexpr int DPP_XOR1 = 0xB1;         // quad_perm [1,0,3,2]
constexpr int DPP_XOR2 = 0x4E;         // quad_perm [2,3,0,1]
constexpr int DPP_HALF_MIRROR = 0x141;
constexpr int DPP_MIRROR = 0x140;

// (v of the even row of my row pair, v of the odd row) / (v of my wave half 0, v of half 1)
__device__ __forceinline__ void pair16(double v, double& ev, double& od) {
  const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)__double2loint(v), (unsigned)__double2loint(v), false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)__double2hiint(v), (unsigned)__double2hiint(v), false, false);
  ev = __hiloint2double((int)hi[0], (int)lo[0]);
  od = __hiloint2double((int)hi[1], (int)lo[1]);
}
__device__ __forceinline__ void pair32(double v, double& h0, double& h1) {
  const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)__double2loint(v), (unsigned)__double2loint(v), false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)__double2hiint(v), (unsigned)__double2hiint(v), false, false);
  h0 = __hiloint2double((int)hi[0], (int)lo[0]);
  h1 = __hiloint2double((int)hi[1], (int)lo[1]);
}

// op: 0 = sum, 1 = min (NaN-ignoring fmin), 2 = max (NaN-ignoring fmax)
template <int OP>
__device__ __forceinline__ double comb(double a, double b) {
  return OP == 0 ? a + b : (OP == 1 ? fmin(a, b) : fmax(a, b));
}

template <int OP>
__device__ __forceinline__ double wave_reduce(double v) {
  v = comb<OP>(v, dpp<DPP_XOR1>(v));
  v = comb<OP>(v, dpp<DPP_XOR2>(v));
  v = comb<OP>(v, dpp<DPP_HALF_MIRROR>(v));
  v = comb<OP>(v, dpp<DPP_MIRROR>(v));
  double a, b;
  pair16(v, a, b);
  v = comb<OP>(a, b);
  pair32(v, a, b);
  return comb<OP>(a, b);
}

__device__ __forceinline__ double wave_sum(double v) { return wave_reduce<0>(v); }
__device__ __forceinline__ double wave_min(double v) { return wave_reduce<1>(v); }
__device__ __forceinline__ double wave_max(double v) { return wave_reduce<2>(v); }

// The wave sums of 16 values at once (reduce-scatter): every level pairs lanes by an involution that
// flips one lane bit (permlane32 / permlane16 swaps, row mirror, half-row mirror), each lane keeps the
// half of its values selected by that bit and adds the partner's copy of that half (the partner sends
// the half it does not keep); then the last two bits (quad DPP) complete the single remaining value.
// Lane L returns the wave's sum of v[idx], idx = 8 b5 + 4 b4 + 2 b3 + b2 (b = the bits of L); the four
// lanes sharing bits 5..2 hold bitwise the same sum.  30 half-exchanges instead of 16 x 6 for sixteen
// wave_sum calls.
__device__ __forceinline__ double wave_sum16(const double (&v)[16]) {
  const unsigned lane = __lane_id();
  const bool b5 = lane & 32, b4 = lane & 16, b3 = lane & 8, b2 = lane & 4;
  double x8[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    double h0, h1;
    pair32(b5 ? v[k] : v[k + 8], h0, h1);   // the half the partner keeps
    x8[k] = (b5 ? v[k + 8] : v[k]) + (b5 ? h0 : h1);
  }
  double x4[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    double ev, od;
    pair16(b4 ? x8[k] : x8[k + 4], ev, od);
    x4[k] = (b4 ? x8[k + 4] : x8[k]) + (b4 ? ev : od);
  }
  double x2[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) x2[k] = (b3 ? x4[k + 2] : x4[k]) + dpp<DPP_MIRROR>(b3 ? x4[k] : x4[k + 2]);
  double x = (b2 ? x2[1] : x2[0]) + dpp<DPP_HALF_MIRROR>(b2 ? x2[0] : x2[1]);
  x = x + dpp<DPP_XOR2>(x);
  return x + dpp<DPP_XOR1>(x);
}
__host__ __device__ constexpr int wave_sum16_index(int lane) {
  return ((lane >> 5) & 1) * 8 + ((lane >> 4) & 1) * 4 + ((lane >> 3) & 1) * 2 + ((lane >> 2) & 1);
}

// v from lane l (uniform l): two readlanes, no LDS
__device__ __forceinline__ double read_lane(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

}  // namespace riptrm_wave
