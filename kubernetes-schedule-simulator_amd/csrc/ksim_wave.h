// ksim_wave.h — wave64 reductions and scans on DPP (gfx9-family row controls: quad_perm,
// row_shr, row_(half_)mirror, row_bcast15/31) instead of ds_bpermute shuffles: each step is
// one VALU op with a DPP source instead of an LDS-crossbar round trip.  Results are
// checked against naive lane loops by ksim_selftest_wave() (tests/test_gpu_parity.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ksimw {

// dpp controls (CDNA / GFX9 encoding)
constexpr int QP_1032 = 0xB1;       // quad_perm [1,0,3,2]
constexpr int QP_2301 = 0x4E;       // quad_perm [2,3,0,1]
constexpr int ROW_SHR1 = 0x111;
constexpr int ROW_SHR2 = 0x112;
constexpr int ROW_SHR3 = 0x113;
constexpr int ROW_SHR4 = 0x114;
constexpr int ROW_SHR8 = 0x118;
constexpr int ROW_MIRROR = 0x140;
constexpr int ROW_HALF_MIRROR = 0x141;
constexpr int ROW_BCAST15 = 0x142;
constexpr int ROW_BCAST31 = 0x143;

template <int CTRL, int ROW_MASK = 0xF, int BANK_MASK = 0xF, bool BOUND_ZERO = false>
__device__ __forceinline__ int dpp(int old, int v) {
  return __builtin_amdgcn_update_dpp(old, v, CTRL, ROW_MASK, BANK_MASK, BOUND_ZERO);
}

// max over the wave, result in every lane (signed)
__device__ __forceinline__ int32_t max_i32(int32_t v) {
  constexpr int ID = INT32_MIN;
  v = max(v, dpp<QP_1032>(ID, v));
  v = max(v, dpp<QP_2301>(ID, v));
  v = max(v, dpp<ROW_HALF_MIRROR>(ID, v));
  v = max(v, dpp<ROW_MIRROR>(ID, v));
  v = max(v, dpp<ROW_BCAST15, 0xA>(ID, v));
  v = max(v, dpp<ROW_BCAST31, 0xC>(ID, v));
  return __builtin_amdgcn_readlane(v, 63);
}

// sum over the wave, result in every lane
__device__ __forceinline__ int32_t sum_i32(int32_t v) {
  v += dpp<QP_1032>(0, v);
  v += dpp<QP_2301>(0, v);
  v += dpp<ROW_HALF_MIRROR>(0, v);
  v += dpp<ROW_MIRROR>(0, v);
  v += dpp<ROW_BCAST15, 0xA>(0, v);
  v += dpp<ROW_BCAST31, 0xC>(0, v);
  return __builtin_amdgcn_readlane(v, 63);
}

// inclusive prefix sum over lanes 0..l (rows of 16 via row_shr, then row broadcasts)
__device__ __forceinline__ int32_t prefix_incl_i32(int32_t v) {
  int32_t x = v + dpp<ROW_SHR1, 0xF, 0xF, true>(0, v);
  x += dpp<ROW_SHR2, 0xF, 0xF, true>(0, v);
  x += dpp<ROW_SHR3, 0xF, 0xF, true>(0, v);
  x += dpp<ROW_SHR4, 0xF, 0xE, true>(0, x);
  x += dpp<ROW_SHR8, 0xF, 0xC, true>(0, x);
  x += dpp<ROW_BCAST15, 0xA, 0xF, false>(0, x);
  x += dpp<ROW_BCAST31, 0xC, 0xF, false>(0, x);
  return x;
}

// 64-bit forms: the two halves move through the same DPP control, the compare / add is 64-bit.
template <int CTRL, int ROW_MASK = 0xF, int BANK_MASK = 0xF, bool BOUND_ZERO = false>
__device__ __forceinline__ int64_t dpp64(int64_t old, int64_t v) {
  const int lo = dpp<CTRL, ROW_MASK, BANK_MASK, BOUND_ZERO>((int)(uint32_t)old, (int)(uint32_t)v);
  const int hi = dpp<CTRL, ROW_MASK, BANK_MASK, BOUND_ZERO>((int)(old >> 32), (int)(v >> 32));
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

__device__ __forceinline__ int64_t readlane64(int64_t v, int l) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), l);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ int64_t max_i64(int64_t v) {
  constexpr int64_t ID = INT64_MIN;
  int64_t t;
  t = dpp64<QP_1032>(ID, v); v = t > v ? t : v;
  t = dpp64<QP_2301>(ID, v); v = t > v ? t : v;
  t = dpp64<ROW_HALF_MIRROR>(ID, v); v = t > v ? t : v;
  t = dpp64<ROW_MIRROR>(ID, v); v = t > v ? t : v;
  t = dpp64<ROW_BCAST15, 0xA>(ID, v); v = t > v ? t : v;
  t = dpp64<ROW_BCAST31, 0xC>(ID, v); v = t > v ? t : v;
  return readlane64(v, 63);
}

__device__ __forceinline__ int64_t min_i64(int64_t v) {
  constexpr int64_t ID = INT64_MAX;
  int64_t t;
  t = dpp64<QP_1032>(ID, v); v = t < v ? t : v;
  t = dpp64<QP_2301>(ID, v); v = t < v ? t : v;
  t = dpp64<ROW_HALF_MIRROR>(ID, v); v = t < v ? t : v;
  t = dpp64<ROW_MIRROR>(ID, v); v = t < v ? t : v;
  t = dpp64<ROW_BCAST15, 0xA>(ID, v); v = t < v ? t : v;
  t = dpp64<ROW_BCAST31, 0xC>(ID, v); v = t < v ? t : v;
  return readlane64(v, 63);
}

__device__ __forceinline__ int64_t sum_i64(int64_t v) {
  v += dpp64<QP_1032>(0, v);
  v += dpp64<QP_2301>(0, v);
  v += dpp64<ROW_HALF_MIRROR>(0, v);
  v += dpp64<ROW_MIRROR>(0, v);
  v += dpp64<ROW_BCAST15, 0xA>(0, v);
  v += dpp64<ROW_BCAST31, 0xC>(0, v);
  return readlane64(v, 63);
}

// Over the first 16 lanes only (one DPP row: four steps, no row broadcasts), result from lane 0.
__device__ __forceinline__ int64_t max16_i64(int64_t v) {
  constexpr int64_t ID = INT64_MIN;
  int64_t t;
  t = dpp64<QP_1032>(ID, v); v = t > v ? t : v;
  t = dpp64<QP_2301>(ID, v); v = t > v ? t : v;
  t = dpp64<ROW_HALF_MIRROR>(ID, v); v = t > v ? t : v;
  t = dpp64<ROW_MIRROR>(ID, v); v = t > v ? t : v;
  return readlane64(v, 0);
}

__device__ __forceinline__ int32_t sum16_i32(int32_t v) {
  v += dpp<QP_1032>(0, v);
  v += dpp<QP_2301>(0, v);
  v += dpp<ROW_HALF_MIRROR>(0, v);
  v += dpp<ROW_MIRROR>(0, v);
  return __builtin_amdgcn_readlane(v, 0);
}

}  // namespace ksimw
