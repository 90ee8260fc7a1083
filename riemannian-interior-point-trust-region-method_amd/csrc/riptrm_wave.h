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

}  // namespace riptrm_wave
