// Shared helpers for the gfx950 (CDNA4) kernels of neuroimagedisttraining_amd.
// Wave = 64 lanes; blocks are multiples of 64 threads.  All kernels are written for gfx950 only.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <string>

#define NIDT_CHECK(expr)                                                                 \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess)                                                                \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e) +      \
                               " at " __FILE__ ":" + std::to_string(__LINE__));          \
  } while (0)

#define NIDT_REQUIRE(cond, msg)                                                          \
  do {                                                                                   \
    if (!(cond)) throw std::invalid_argument(std::string("nidt: ") + (msg));             \
  } while (0)

namespace nidt {

constexpr int kWave = 64;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Block-wide sum; result valid in every thread. `red` must hold blockDim.x/64 floats.
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

__device__ __forceinline__ float bf16_to_f32(uint16_t b) { return __uint_as_float(((uint32_t)b) << 16); }

// f32 -> bf16 bits, round-to-nearest-even (NaN stays NaN): the gfx950 hardware conversion
// (v_cvt_pk_bf16_f32), one VALU op per PAIR instead of a ~6-op software rounding per value.
__device__ __forceinline__ uint16_t f32_to_bf16(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }

__device__ __forceinline__ uint32_t pack_bf16x2(float lo, float hi) {
  typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
  const bf2 v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(uint32_t, v);
}

// 27-bit in-bounds mask of the 3x3x3 taps (t = 9 jd + 3 jh + jw) of an output position whose window starts at
// (d0, h0, w0): three 3-bit per-dimension masks combined with shifts (~20 VALU instead of 27 x 6 compares).
__device__ __forceinline__ uint32_t tap_mask3(int d0, int h0, int w0, int D, int H, int W) {
  uint32_t md = 0, mh = 0, mw = 0;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    md |= (uint32_t)((unsigned)(d0 + j) < (unsigned)D) << j;
    mh |= (uint32_t)((unsigned)(h0 + j) < (unsigned)H) << j;
    mw |= (uint32_t)((unsigned)(w0 + j) < (unsigned)W) << j;
  }
  const uint32_t hw = ((mh & 1u) ? mw : 0u) | ((mh & 2u) ? mw << 3 : 0u) | ((mh & 4u) ? mw << 6 : 0u);
  return ((md & 1u) ? hw : 0u) | ((md & 2u) ? hw << 9 : 0u) | ((md & 4u) ? hw << 18 : 0u);
}

inline hipStream_t as_stream(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

template <typename T>
inline T* ptr(uintptr_t p) { return reinterpret_cast<T*>(p); }

inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// Bijective XCD-aware remap of a 1-D block id (cdna_hip_programming.md §5, "XCD swizzle must be bijective"):
// consecutive logical tiles land on the same XCD so neighbouring tiles share that XCD's L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

}  // namespace nidt
