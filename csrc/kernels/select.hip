// SNIP saliency accumulation, global top-k threshold by radix select, and mask utilities.
//
// Reference: fedml_api/standalone/sailentgrads/snip.py:21-116 — saliency |dL/dmask| = |w * dL/dw| per
// maskable (conv/linear) weight, averaged over IterSNIP batches and clients, then a global top-k at
// keep_ratio over the concatenated normalised scores and mask = (score >= k-th largest) (ties kept, quirk Q7).
// Selection here is an exact radix select over the fp32 bit patterns (scores are >= 0, so unsigned order ==
// float order): four 8-bit digit passes, each one histogram kernel + one single-block scan kernel, entirely
// on device (no host round trip, identical result on every rank given identical scores).
#include "common.h"

namespace nidt {

// score[g][i] += |theta[g][i] * grad[g][i]| * alpha for i in [0, P)
__global__ void k_saliency_acc(const float* __restrict__ theta, const float* __restrict__ grad, int64_t ld, int64_t P,
                               int G, float alpha, float* __restrict__ score, int64_t lds) {
  const int64_t tot = (int64_t)G * P;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    const int g = (int)(e / P);
    const int64_t i = e - (int64_t)g * P;
    score[(int64_t)g * lds + i] += fabsf(theta[(int64_t)g * ld + i] * grad[(int64_t)g * ld + i]) * alpha;
  }
}

void saliency_acc(uintptr_t theta, uintptr_t grad, int64_t ld, int64_t P, int G, float alpha, uintptr_t score,
                  int64_t lds, uintptr_t stream) {
  const int64_t tot = (int64_t)G * P;
  hipLaunchKernelGGL(k_saliency_acc, dim3((unsigned)std::min<int64_t>(8192, (tot + 255) / 256)), dim3(256), 0,
                     as_stream(stream), ptr<const float>(theta), ptr<const float>(grad), ld, P, G, alpha,
                     ptr<float>(score), lds);
  NIDT_CHECK(hipGetLastError());
}

// state: [0] prefix bits, [1] prefix mask, [2] remaining k, [3] threshold bits (result)
__global__ __launch_bounds__(256) void k_radix_hist(const float* __restrict__ v, int64_t n,
                                                    const uint32_t* __restrict__ state, int shift,
                                                    uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t pre = state[0], pm = state[1];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t b = __float_as_uint(v[i]);
    if ((b & pm) == pre) atomicAdd(&h[(b >> shift) & 0xff], 1u);
  }
  __syncthreads();
  if (h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}

__global__ void k_radix_scan(uint32_t* __restrict__ state, int shift, uint32_t* __restrict__ hist) {
  if (threadIdx.x != 0) return;
  uint32_t k = state[2];
  uint32_t acc = 0;
  int d = 255;
  for (; d > 0; --d) {
    if (acc + hist[d] >= k) break;
    acc += hist[d];
  }
  state[0] |= (uint32_t)d << shift;
  state[1] |= 0xffu << shift;
  state[2] = k - acc;
  state[3] = state[0];
  for (int i = 0; i < 256; ++i) hist[i] = 0;
}

// k-th largest (1-based) of v[0..n) -> state[3] (bit pattern); workspace: state[4] + hist[256] (uint32)
void radix_select_kth(uintptr_t v, int64_t n, int64_t k, uintptr_t state, uintptr_t hist, uintptr_t stream) {
  NIDT_REQUIRE(k >= 1 && k <= n, "radix_select_kth: 1 <= k <= n");
  hipStream_t s = as_stream(stream);
  uint32_t init[4] = {0u, 0u, (uint32_t)k, 0u};
  NIDT_CHECK(hipMemcpyAsync(ptr<void>(state), init, sizeof(init), hipMemcpyHostToDevice, s));
  NIDT_CHECK(hipMemsetAsync(ptr<void>(hist), 0, 256 * sizeof(uint32_t), s));
  const unsigned nb = (unsigned)std::min<int64_t>(2048, (n + 255) / 256);
  for (int shift = 24; shift >= 0; shift -= 8) {
    hipLaunchKernelGGL(k_radix_hist, dim3(nb), dim3(256), 0, s, ptr<const float>(v), n, ptr<const uint32_t>(state),
                       shift, ptr<uint32_t>(hist));
    hipLaunchKernelGGL(k_radix_scan, dim3(1), dim3(64), 0, s, ptr<uint32_t>(state), shift, ptr<uint32_t>(hist));
  }
  NIDT_CHECK(hipGetLastError());
  NIDT_CHECK(hipStreamSynchronize(s));  // the init array lives on the host stack
}

// mask[i] = v[i] >= threshold(state[3]) ? 1 : 0
__global__ void k_threshold_mask(const float* __restrict__ v, int64_t n, const uint32_t* __restrict__ state,
                                 float* __restrict__ mask) {
  const float thr = __uint_as_float(state[3]);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    mask[i] = v[i] >= thr ? 1.f : 0.f;
}

void threshold_mask(uintptr_t v, int64_t n, uintptr_t state, uintptr_t mask, uintptr_t stream) {
  hipLaunchKernelGGL(k_threshold_mask, dim3((unsigned)std::min<int64_t>(8192, (n + 255) / 256)), dim3(256), 0,
                     as_stream(stream), ptr<const float>(v), n, ptr<const uint32_t>(state), ptr<float>(mask));
  NIDT_CHECK(hipGetLastError());
}

// count of non-zeros and Hamming distance between two float masks (mask != 0), uint64 counters
__global__ void k_mask_stats(const float* __restrict__ a, const float* __restrict__ b, int64_t n,
                             unsigned long long* __restrict__ out) {
  unsigned long long nz = 0, hd = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const bool x = a[i] != 0.f;
    nz += x;
    if (b) hd += (x != (b[i] != 0.f));
  }
  for (int o = 32; o > 0; o >>= 1) {
    nz += __shfl_xor(nz, o, 64);
    hd += __shfl_xor(hd, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(out, nz);
    atomicAdd(out + 1, hd);
  }
}

void mask_stats(uintptr_t a, uintptr_t b, int64_t n, uintptr_t out, uintptr_t stream) {
  NIDT_CHECK(hipMemsetAsync(ptr<void>(out), 0, 2 * sizeof(unsigned long long), as_stream(stream)));
  hipLaunchKernelGGL(k_mask_stats, dim3((unsigned)std::min<int64_t>(2048, (n + 255) / 256)), dim3(256), 0,
                     as_stream(stream), ptr<const float>(a), ptr<const float>(b), n,
                     ptr<unsigned long long>(out));
  NIDT_CHECK(hipGetLastError());
}

}  // namespace nidt
