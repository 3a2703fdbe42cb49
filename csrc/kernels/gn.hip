// GroupNorm(32) forward / backward for client-grouped channels-last activations [N = G*B][S][C] (bf16), the
// normalisation of the reference's CIFAR ResNet-18-GN (fedml_api/model/cv/resnet.py:91-124: BatchNorm swapped for
// GroupNorm(32, C), per-client affine).
//
// One block (512 threads) per sample.  The whole sample (S*C <= 65536 elements: 32x32x64 at layer 1) stays in
// registers as packed bf16 (<= 16 x 16-B chunks per thread), so the activation is read from HBM once: statistics
// (two-pass: mean, then sum of squared deviations), normalisation, affine, optional residual add and ReLU are
// applied from registers.  Each thread owns one 8-channel chunk column (512 % (C/8) == 0), so per-channel partial
// sums reduce through LDS in a fixed order (deterministic, no atomics, no library workspaces: hipGraph-safe).
// The backward recomputes x-hat from the saved (mean, rstd), forms the per-channel sums A_c = sum dy and
// B_c = sum dy * xhat (= the per-sample dbeta / dgamma partials), from them the group means of dy*gamma and
// dy*gamma*xhat, and writes dt in bf16; k_gn_param_grads sums the per-sample partials of each client into its
// gradient row.
#include "common.h"
#include "dma.h"

namespace nidt {

constexpr int kGnThreads = 512;
constexpr int kGnGroups = 32;
constexpr float kGnEps = 1e-5f;

__device__ __forceinline__ void unpack8(const uint4 v, float* f) {
  const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[2 * j] = __uint_as_float(u[j] << 16);
    f[2 * j + 1] = __uint_as_float(u[j] & 0xffff0000u);
  }
}

// Per-channel sums of this thread's 8-channel partials -> per-group totals in grp[32] (valid after the call).
// part: this thread's 8 values; sm: LDS [512][9] scratch; chs: LDS [512]; grp: LDS [32].
__device__ __forceinline__ void gn_reduce_groups(const float* part, float* sm, float* chs, float* grp, int C,
                                                 int nch) {
  const int tid = threadIdx.x;
#pragma unroll
  for (int e = 0; e < 8; ++e) sm[tid * 9 + e] = part[e];
  __syncthreads();
  const int rows = kGnThreads / nch;
  for (int c = tid; c < C; c += kGnThreads) {
    const int j = c >> 3, e = c & 7;
    float s = 0.f;
    for (int r = 0; r < rows; ++r) s += sm[(r * nch + j) * 9 + e];
    chs[c] = s;
  }
  __syncthreads();
  if (tid < kGnGroups) {
    const int cg = C / kGnGroups;
    float s = 0.f;
    for (int i = 0; i < cg; ++i) s += chs[tid * cg + i];
    grp[tid] = s;
  }
  __syncthreads();
}

// Per-channel totals over the block of this thread's 8 channel partials p (channels 8j .. 8j+7 of chunk column
// j = tid % nch): the lanes of a wave sharing j by xor shuffles over the lane bits >= log2(nch), then the 8 waves in
// a fixed order through LDS (deterministic).  red: LDS [8][512]; out: LDS [C] (valid after the call; p is clobbered).
__device__ __forceinline__ void gn_chan_sums(float* p, float* red, float* out, int C, int nch) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int o = nch; o < 64; o <<= 1)
#pragma unroll
    for (int e = 0; e < 8; ++e) p[e] += __shfl_xor(p[e], o, 64);
  if (lane < nch) {
    float4* r = reinterpret_cast<float4*>(red + w * 512 + 8 * lane);
    r[0] = make_float4(p[0], p[1], p[2], p[3]);
    r[1] = make_float4(p[4], p[5], p[6], p[7]);
  }
  __syncthreads();
  for (int c = tid; c < C; c += kGnThreads) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < kGnThreads / 64; ++q) s += red[q * 512 + c];
    out[c] = s;
  }
  __syncthreads();
}

__device__ __forceinline__ uint4 as_u4(i32x4_t v) {
  return make_uint4((uint32_t)v.x, (uint32_t)v.y, (uint32_t)v.z, (uint32_t)v.w);
}

// Opaque redefinition of the held chunks between passes: the compiler may not keep a pass's unpacked fp32 copies
// alive for the next pass (2x the registers of the packed bf16 chunks).
template <int NV>
__device__ __forceinline__ void gn_fence(i32x4_t (&v)[NV]) {
#pragma unroll
  for (int k = 0; k < NV; ++k) asm volatile("" : "+v"(v[k]));
}

// [GN-REG] Register-resident forward: the sample's 16-B chunks are read once through a raw buffer resource (a 32-bit
// VGPR offset per chunk row; rows past the sample read zeros and their stores are dropped by the range check, so no
// 64-bit address per chunk stays live) and kept packed; <= 128 VGPRs at NV = 16 -> two 512-thread blocks per CU (the
// global-pointer version needed 184 VGPRs: one block per CU, its load / reduce / store phases never overlapped).
template <int NV, bool RES, bool RELU>
__global__ __launch_bounds__(kGnThreads, 4) void k_gn_fwd(const uint16_t* __restrict__ t,
                                                          const uint16_t* __restrict__ res,
                                                          const float* __restrict__ theta, int64_t ldt, int64_t off_w,
                                                          int64_t off_b, uint16_t* __restrict__ y,
                                                          float* __restrict__ stats, int B, int S, int C) {
  __shared__ __attribute__((aligned(16))) float red[kGnThreads / 64 * 512];
  __shared__ float chs[512];
  __shared__ float gmean[kGnGroups], grstd[kGnGroups];
  const int n = blockIdx.x, g = n / B, tid = threadIdx.x;
  const int nch = C >> 3, nchunk = S * nch;
  const int64_t base = (int64_t)n * S * C;
  const uint32_t bytes = (uint32_t)S * C * 2;
  const int j = tid % nch;  // this thread's channel chunk (512 % nch == 0)
  const int cg = C / kGnGroups;
  const int vo = tid * 16;
  const i32x4_t rt = make_rsrc(t + base, bytes);
  i32x4_t v[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = nidt_raw_buffer_load_v4i32(rt, vo + k * kGnThreads * 16, 0, 0);
  float part[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) part[e] = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {  // rows past the sample read zeros: no guard in the sum
    float f[8];
    unpack8(as_u4(v[k]), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) part[e] += f[e];
  }
  gn_chan_sums(part, red, chs, C, nch);
  if (tid < kGnGroups) {
    float s = 0.f;
    for (int i = 0; i < cg; ++i) s += chs[tid * cg + i];
    gmean[tid] = s / (float)(S * cg);
  }
  __syncthreads();
  gn_fence(v);
  float mu[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mu[e] = gmean[(8 * j + e) / cg];
    part[e] = 0.f;
  }
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    if (tid + k * kGnThreads < nchunk) {
      float f[8];
      unpack8(as_u4(v[k]), f);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = f[e] - mu[e];
        part[e] = fmaf(d, d, part[e]);
      }
    }
  }
  gn_chan_sums(part, red, chs, C, nch);
  if (tid < kGnGroups) {
    float s = 0.f;
    for (int i = 0; i < cg; ++i) s += chs[tid * cg + i];
    const float rs = rsqrtf(s / (float)(S * cg) + kGnEps);
    grstd[tid] = rs;
    stats[((int64_t)n * kGnGroups + tid) * 2] = gmean[tid];
    stats[((int64_t)n * kGnGroups + tid) * 2 + 1] = rs;
  }
  __syncthreads();
  float sc[8], sh[8];
  const float* gw = theta + (int64_t)g * ldt + off_w;
  const float* gb = theta + (int64_t)g * ldt + off_b;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = 8 * j + e;
    sc[e] = gw[c] * grstd[c / cg];
    sh[e] = gb[c] - mu[e] * sc[e];
  }
  gn_fence(v);
  const i32x4_t ry = make_rsrc(y + base, bytes);
  i32x4_t rr;
  if (RES) rr = make_rsrc(res + base, bytes);
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    float f[8], r[8];
    unpack8(as_u4(v[k]), f);
    if (RES) unpack8(as_u4(nidt_raw_buffer_load_v4i32(rr, vo + k * kGnThreads * 16, 0, 0)), r);
    i32x4_t o;
    int* op = reinterpret_cast<int*>(&o);
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      float a0 = fmaf(f[e], sc[e], sh[e]), a1 = fmaf(f[e + 1], sc[e + 1], sh[e + 1]);
      if (RES) {
        a0 += r[e];
        a1 += r[e + 1];
      }
      if (RELU) {
        a0 = fmaxf(a0, 0.f);
        a1 = fmaxf(a1, 0.f);
      }
      op[e >> 1] = (int)pack_bf16x2(a0, a1);
    }
    nidt_raw_buffer_store_v4i32(o, ry, vo + k * kGnThreads * 16, 0, 0);  // rows past the sample: dropped
  }
}

// dy: fp32 (DYB = false) or bf16; mask (optional, bf16 post-ReLU activation): dy *= (mask > 0).
// [GN-REG] HOLD (bf16 dy): t and the masked dy are read once and held packed; otherwise t is held and dy (and the
// mask) are read again by the apply pass (fewer registers: more resident blocks for the 16-row samples).
// [GN-RMASK] RM: the ReLU mask of a GroupNorm WITHOUT residual (y = relu(gamma xhat + beta)) recomputed from the held t
// and the saved statistics with the forward's own arithmetic (sc = gamma rstd, sh = beta - mu sc, y > 0 <=>
// fma(t, sc, sh) > 0): no mask tensor read, the same dt bit for bit (off_b = the beta offset).
template <int NV, bool DYB, bool MASK, bool HOLD, bool RM = false>
__global__ __launch_bounds__(kGnThreads, (HOLD || NV >= 16) ? 2 : 4) void k_gn_bwd(const void* __restrict__ dyv, const uint16_t* __restrict__ mask,
                                                       const uint16_t* __restrict__ t, const float* __restrict__ stats,
                                                       const float* __restrict__ theta, int64_t ldt, int64_t off_w,
                                                       uint16_t* __restrict__ dt, float* __restrict__ part_out, int B,
                                                       int S, int C, int64_t off_b = 0) {
  static_assert(!HOLD || DYB, "k_gn_bwd: held dy is bf16");
  static_assert(!(RM && MASK), "k_gn_bwd: one mask source");
  __shared__ __attribute__((aligned(16))) float red[kGnThreads / 64 * 512];
  __shared__ float chA[512], chB[512];
  __shared__ float gm1[kGnGroups], gm2[kGnGroups];
  const int n = blockIdx.x, g = n / B, tid = threadIdx.x;
  const int nch = C >> 3, nchunk = S * nch;
  const int64_t base = (int64_t)n * S * C;
  const uint32_t bytes = (uint32_t)S * C * 2;
  const int j = tid % nch;
  const int cg = C / kGnGroups;
  const int vo = tid * 16;
  float mu[8], rs[8], gw[8], msc[8], msh[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = 8 * j + e;
    mu[e] = stats[((int64_t)n * kGnGroups + c / cg) * 2];
    rs[e] = stats[((int64_t)n * kGnGroups + c / cg) * 2 + 1];
    gw[e] = theta[(int64_t)g * ldt + off_w + c];
    if (RM) {  // k_gn_fwd's coefficients, same expressions
      msc[e] = gw[e] * rs[e];
      msh[e] = theta[(int64_t)g * ldt + off_b + c] - mu[e] * msc[e];
    }
  }
  auto rmask = [&](const float* f, float* d) {  // [GN-RMASK] dy *= (relu input > 0)
    if (RM) {
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] = fmaf(f[e], msc[e], msh[e]) > 0.f ? d[e] : 0.f;
    }
  };
  const i32x4_t rt = make_rsrc(t + base, bytes);
  i32x4_t rm, rd;
  if (MASK) rm = make_rsrc(mask + base, bytes);
  if (DYB) rd = make_rsrc(reinterpret_cast<const uint16_t*>(dyv) + base, bytes);
  auto mask_bits = [&](i32x4_t dvk, i32x4_t mk) {  // keep the dy halves whose mask value is > 0
    float m[8];
    unpack8(as_u4(mk), m);
    int* dp = reinterpret_cast<int*>(&dvk);
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const uint32_t u = (uint32_t)dp[h];
      dp[h] = (int)((m[2 * h] > 0.f ? (u & 0xffffu) : 0u) | (m[2 * h + 1] > 0.f ? (u & 0xffff0000u) : 0u));
    }
    return dvk;
  };
  auto load_d = [&](int k, float* d) {  // dy row k (masked), not held
    const int q = tid + k * kGnThreads;
    if constexpr (DYB) {
      i32x4_t x = nidt_raw_buffer_load_v4i32(rd, vo + k * kGnThreads * 16, 0, 0);
      if (MASK) x = mask_bits(x, nidt_raw_buffer_load_v4i32(rm, vo + k * kGnThreads * 16, 0, 0));
      unpack8(as_u4(x), d);
    } else if (q < nchunk) {
      const float4* p = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(dyv) + base + (int64_t)q * 8);
      const float4 a = p[0], b = p[1];
      d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w; d[4] = b.x; d[5] = b.y; d[6] = b.z; d[7] = b.w;
      if (MASK) {
        float m[8];
        unpack8(*reinterpret_cast<const uint4*>(mask + base + (int64_t)q * 8), m);
#pragma unroll
        for (int e = 0; e < 8; ++e) d[e] = m[e] > 0.f ? d[e] : 0.f;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] = 0.f;
    }
  };
  i32x4_t v[NV];
  i32x4_t dv[HOLD ? NV : 1];
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = nidt_raw_buffer_load_v4i32(rt, vo + k * kGnThreads * 16, 0, 0);
  if constexpr (HOLD) {
    constexpr int KB = NV < 4 ? NV : 4;  // dy + mask in batches of 4 rows (bounded in-flight registers)
#pragma unroll
    for (int k0 = 0; k0 < NV; k0 += KB) {
      i32x4_t mk[KB];
#pragma unroll
      for (int k = k0; k < k0 + KB; ++k) {
        dv[k] = nidt_raw_buffer_load_v4i32(rd, vo + k * kGnThreads * 16, 0, 0);
        if (MASK) mk[k - k0] = nidt_raw_buffer_load_v4i32(rm, vo + k * kGnThreads * 16, 0, 0);
      }
      if (MASK) {
#pragma unroll
        for (int k = k0; k < k0 + KB; ++k) dv[k] = mask_bits(dv[k], mk[k - k0]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  float pa[8], pb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) pa[e] = pb[e] = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    float f[8], d[8];
    unpack8(as_u4(v[k]), f);
    if constexpr (HOLD) unpack8(as_u4(dv[k]), d);
    else load_d(k, d);
    rmask(f, d);
    if (tid + k * kGnThreads < nchunk) {  // rows past the sample: dy reads zero, but (f - mu) does not
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        pa[e] += d[e];
        pb[e] = fmaf(d[e], (f[e] - mu[e]) * rs[e], pb[e]);
      }
    }
  }
  // per-channel A_c (= dbeta partial) and B_c (= dgamma partial); group sums of gamma-weighted values
  gn_chan_sums(pa, red, chA, C, nch);
  gn_chan_sums(pb, red, chB, C, nch);
  for (int c = tid; c < C; c += kGnThreads) {
    part_out[((int64_t)n * C + c) * 2] = chA[c];
    part_out[((int64_t)n * C + c) * 2 + 1] = chB[c];
  }
  if (tid < kGnGroups) {
    float s1 = 0.f, s2 = 0.f;
    const float* gwr = theta + (int64_t)g * ldt + off_w;
    for (int i = 0; i < cg; ++i) {
      const int c = tid * cg + i;
      s1 = fmaf(gwr[c], chA[c], s1);
      s2 = fmaf(gwr[c], chB[c], s2);
    }
    gm1[tid] = s1 / (float)(S * cg);
    gm2[tid] = s2 / (float)(S * cg);
  }
  __syncthreads();
  float m1[8], m2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    m1[e] = gm1[(8 * j + e) / cg];
    m2[e] = gm2[(8 * j + e) / cg];
  }
  gn_fence(v);
  if constexpr (HOLD) gn_fence(dv);
  const i32x4_t rdt = make_rsrc(dt + base, bytes);
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    float f[8], d[8];
    unpack8(as_u4(v[k]), f);
    if constexpr (HOLD) unpack8(as_u4(dv[k]), d);
    else load_d(k, d);
    rmask(f, d);
    i32x4_t o;
    int* op = reinterpret_cast<int*>(&o);
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      const float x0 = (f[e] - mu[e]) * rs[e], x1 = (f[e + 1] - mu[e + 1]) * rs[e + 1];
      const float r0 = rs[e] * (d[e] * gw[e] - m1[e] - x0 * m2[e]);
      const float r1 = rs[e + 1] * (d[e + 1] * gw[e + 1] - m1[e + 1] - x1 * m2[e + 1]);
      op[e >> 1] = (int)pack_bf16x2(r0, r1);
    }
    nidt_raw_buffer_store_v4i32(o, rdt, vo + k * kGnThreads * 16, 0, 0);  // rows past the sample: dropped
  }
}

// Streaming variants for samples larger than the register-resident limit (S*C > 65536, e.g. the 64x64x64 maps of
// the Tiny-ImageNet ResNet-18): the same arithmetic and reduction order per element, with the sample re-read from
// memory in each pass (mean, squared deviations, apply) instead of held in registers.
template <bool RES, bool RELU>
__global__ __launch_bounds__(kGnThreads) void k_gn_fwd_stream(const uint16_t* __restrict__ t,
                                                              const uint16_t* __restrict__ res,
                                                              const float* __restrict__ theta, int64_t ldt,
                                                              int64_t off_w, int64_t off_b, uint16_t* __restrict__ y,
                                                              float* __restrict__ stats, int B, int S, int C) {
  __shared__ float sm[kGnThreads * 9];
  __shared__ float chs[512];
  __shared__ float grp[kGnGroups], gmean[kGnGroups], grstd[kGnGroups];
  const int n = blockIdx.x, g = n / B, tid = threadIdx.x;
  const int nch = C >> 3, nchunk = S * nch;
  const int64_t base = (int64_t)n * S * C;
  const int j = tid % nch;
  const int cg = C / kGnGroups;
  float part[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) part[e] = 0.f;
  for (int q = tid; q < nchunk; q += kGnThreads) {
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(t + base + (int64_t)q * 8), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) part[e] += f[e];
  }
  gn_reduce_groups(part, sm, chs, grp, C, nch);
  if (tid < kGnGroups) gmean[tid] = grp[tid] / (float)(S * cg);
  __syncthreads();
  float mu[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mu[e] = gmean[(8 * j + e) / cg];
    part[e] = 0.f;
  }
  for (int q = tid; q < nchunk; q += kGnThreads) {
    float f[8];
    unpack8(*reinterpret_cast<const uint4*>(t + base + (int64_t)q * 8), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = f[e] - mu[e];
      part[e] = fmaf(d, d, part[e]);
    }
  }
  gn_reduce_groups(part, sm, chs, grp, C, nch);
  if (tid < kGnGroups) {
    const float rs = rsqrtf(grp[tid] / (float)(S * cg) + kGnEps);
    grstd[tid] = rs;
    stats[((int64_t)n * kGnGroups + tid) * 2] = gmean[tid];
    stats[((int64_t)n * kGnGroups + tid) * 2 + 1] = rs;
  }
  __syncthreads();
  float sc[8], sh[8];
  const float* gw = theta + (int64_t)g * ldt + off_w;
  const float* gb = theta + (int64_t)g * ldt + off_b;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = 8 * j + e;
    sc[e] = gw[c] * grstd[c / cg];
    sh[e] = gb[c] - mu[e] * sc[e];
  }
  for (int q = tid; q < nchunk; q += kGnThreads) {
    float f[8], r[8];
    unpack8(*reinterpret_cast<const uint4*>(t + base + (int64_t)q * 8), f);
    if (RES) unpack8(*reinterpret_cast<const uint4*>(res + base + (int64_t)q * 8), r);
    uint32_t o[4];
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      float a0 = fmaf(f[e], sc[e], sh[e]), a1 = fmaf(f[e + 1], sc[e + 1], sh[e + 1]);
      if (RES) {
        a0 += r[e];
        a1 += r[e + 1];
      }
      if (RELU) {
        a0 = fmaxf(a0, 0.f);
        a1 = fmaxf(a1, 0.f);
      }
      o[e >> 1] = pack_bf16x2(a0, a1);
    }
    *reinterpret_cast<uint4*>(y + base + (int64_t)q * 8) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

template <bool DYB, bool MASK>
__global__ __launch_bounds__(kGnThreads) void k_gn_bwd_stream(const void* __restrict__ dyv,
                                                              const uint16_t* __restrict__ mask,
                                                              const uint16_t* __restrict__ t,
                                                              const float* __restrict__ stats,
                                                              const float* __restrict__ theta, int64_t ldt,
                                                              int64_t off_w, uint16_t* __restrict__ dt,
                                                              float* __restrict__ part_out, int B, int S, int C) {
  __shared__ float sm[kGnThreads * 9];
  __shared__ float chs[512];
  __shared__ float grp[kGnGroups], gm1[kGnGroups], gm2[kGnGroups];
  __shared__ float chA[512];
  const int n = blockIdx.x, g = n / B, tid = threadIdx.x;
  const int nch = C >> 3, nchunk = S * nch;
  const int64_t base = (int64_t)n * S * C;
  const int j = tid % nch;
  const int cg = C / kGnGroups;
  float mu[8], rs[8], gw[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = 8 * j + e;
    mu[e] = stats[((int64_t)n * kGnGroups + c / cg) * 2];
    rs[e] = stats[((int64_t)n * kGnGroups + c / cg) * 2 + 1];
    gw[e] = theta[(int64_t)g * ldt + off_w + c];
  }
  auto load_dy = [&](int q, float* d) {
    if (DYB) {
      unpack8(*reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(dyv) + base + (int64_t)q * 8), d);
    } else {
      const float4* p = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(dyv) + base + (int64_t)q * 8);
      const float4 a = p[0], b = p[1];
      d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w; d[4] = b.x; d[5] = b.y; d[6] = b.z; d[7] = b.w;
    }
    if (MASK) {
      float m[8];
      unpack8(*reinterpret_cast<const uint4*>(mask + base + (int64_t)q * 8), m);
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] = m[e] > 0.f ? d[e] : 0.f;
    }
  };
  float pa[8], pb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) pa[e] = pb[e] = 0.f;
  for (int q = tid; q < nchunk; q += kGnThreads) {
    float f[8], d[8];
    unpack8(*reinterpret_cast<const uint4*>(t + base + (int64_t)q * 8), f);
    load_dy(q, d);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      pa[e] += d[e];
      pb[e] = fmaf(d[e], (f[e] - mu[e]) * rs[e], pb[e]);
    }
  }
  gn_reduce_groups(pa, sm, chs, grp, C, nch);
  for (int c = tid; c < C; c += kGnThreads) chA[c] = chs[c];
  __syncthreads();
  gn_reduce_groups(pb, sm, chs, grp, C, nch);
  for (int c = tid; c < C; c += kGnThreads) {
    part_out[((int64_t)n * C + c) * 2] = chA[c];
    part_out[((int64_t)n * C + c) * 2 + 1] = chs[c];
  }
  if (tid < kGnGroups) {
    float s1 = 0.f, s2 = 0.f;
    const float* gwr = theta + (int64_t)g * ldt + off_w;
    for (int i = 0; i < cg; ++i) {
      const int c = tid * cg + i;
      s1 = fmaf(gwr[c], chA[c], s1);
      s2 = fmaf(gwr[c], chs[c], s2);
    }
    gm1[tid] = s1 / (float)(S * cg);
    gm2[tid] = s2 / (float)(S * cg);
  }
  __syncthreads();
  float m1[8], m2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    m1[e] = gm1[(8 * j + e) / cg];
    m2[e] = gm2[(8 * j + e) / cg];
  }
  for (int q = tid; q < nchunk; q += kGnThreads) {
    float f[8], d[8];
    unpack8(*reinterpret_cast<const uint4*>(t + base + (int64_t)q * 8), f);
    load_dy(q, d);
    uint32_t o[4];
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      const float x0 = (f[e] - mu[e]) * rs[e], x1 = (f[e + 1] - mu[e + 1]) * rs[e + 1];
      const float r0 = rs[e] * (d[e] * gw[e] - m1[e] - x0 * m2[e]);
      const float r1 = rs[e + 1] * (d[e + 1] * gw[e + 1] - m1[e + 1] - x1 * m2[e + 1]);
      o[e >> 1] = pack_bf16x2(r0, r1);
    }
    *reinterpret_cast<uint4*>(dt + base + (int64_t)q * 8) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// grads[g][off_w + c] = sum_b part[g*B + b][c][1] (dgamma), grads[g][off_b + c] = sum_b part[..][c][0] (dbeta)
__global__ void k_gn_param_grads(const float* __restrict__ part, int B, int C, float* __restrict__ grads, int64_t ldg,
                                 int64_t off_w, int64_t off_b) {
  const int g = blockIdx.x;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float a = 0.f, b = 0.f;
    for (int i = 0; i < B; ++i) {
      const float* p = part + (((int64_t)g * B + i) * C + c) * 2;
      a += p[0];
      b += p[1];
    }
    grads[(int64_t)g * ldg + off_w + c] = b;
    grads[(int64_t)g * ldg + off_b + c] = a;
  }
}

// Residual-stream gradient of a basic block: out = dx1 + (dx2 if given, else da * (mask > 0)); dx1/dx2 bf16 (the two
// convolutions' data gradients), da (the block output gradient) and out bf16 or fp32, mask bf16 (the block's
// post-ReLU output).  One pass instead of the four elementwise torch ops (two up-casts, a compare-multiply, an add).
// The engines keep the residual gradient stream in bf16 (OB, DB): it is re-read by the normalisation backward of
// every block, and fp32 doubled those passes' bytes (config 5: the fp32-dy BN backward was 16 % of a round).
__device__ __forceinline__ void store8(void* out, int64_t q, const float (&v)[8], bool bf) {
  if (bf) {
    *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(out) + q * 8) =
        make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
  } else {
    float4* o = reinterpret_cast<float4*>(reinterpret_cast<float*>(out) + q * 8);
    o[0] = make_float4(v[0], v[1], v[2], v[3]);
    o[1] = make_float4(v[4], v[5], v[6], v[7]);
  }
}

// [OMASK] omask (optional): the output is also multiplied by [omask > 0] — the ReLU mask of the previous block's
// output, so the stream handed on is the gradient at that block's BatchNorm output (pre-ReLU) and its BN backward
// and identity shortcut read no mask (config 5: two fewer passes over the widest tensor per block).  mask == null
// with dx2 == null: da is already masked.
template <bool OB, bool DB>
__global__ void k_res_grad(void* __restrict__ out, const uint16_t* __restrict__ dx1, const uint16_t* __restrict__ dx2,
                           const void* __restrict__ da, const uint16_t* __restrict__ mask,
                           const uint16_t* __restrict__ omask, int64_t n8) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n8; q += (int64_t)gridDim.x * blockDim.x) {
    float a[8], b[8];
    unpack8(*reinterpret_cast<const uint4*>(dx1 + q * 8), a);
    if (dx2) {
      unpack8(*reinterpret_cast<const uint4*>(dx2 + q * 8), b);
    } else {
      float m[8], d[8];
      if (mask) {
        unpack8(*reinterpret_cast<const uint4*>(mask + q * 8), m);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) m[e] = 1.f;
      }
      if (DB) {
        unpack8(*reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(da) + q * 8), d);
      } else {
        const float* df = reinterpret_cast<const float*>(da);
        const float4 d0 = *reinterpret_cast<const float4*>(df + q * 8), d1 = *reinterpret_cast<const float4*>(df + q * 8 + 4);
        d[0] = d0.x; d[1] = d0.y; d[2] = d0.z; d[3] = d0.w; d[4] = d1.x; d[5] = d1.y; d[6] = d1.z; d[7] = d1.w;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) b[e] = m[e] > 0.f ? d[e] : 0.f;
    }
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = a[e] + b[e];
    if (omask) {
      float om[8];
      unpack8(*reinterpret_cast<const uint4*>(omask + q * 8), om);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = om[e] > 0.f ? v[e] : 0.f;
    }
    store8(out, q, v, OB);
  }
}

// flags: bit 0 = out bf16, bit 1 = da bf16.  res_grad_om: with the [OMASK] output mask (and mask optional)
void res_grad_om(uintptr_t out, uintptr_t dx1, uintptr_t dx2, uintptr_t da, uintptr_t mask, uintptr_t omask, int64_t n,
                 int flags, uintptr_t stream) {
  NIDT_REQUIRE(n % 8 == 0 && (dx2 || da), "res_grad: n % 8 == 0 and (dx2 or da)");
  const int64_t n8 = n / 8;
  const dim3 grid((unsigned)std::min<int64_t>(8192, (n8 + 255) / 256));
  hipStream_t s = as_stream(stream);
#define RG(OB, DB)                                                                                             \
  hipLaunchKernelGGL((k_res_grad<OB, DB>), grid, dim3(256), 0, s, ptr<void>(out), ptr<const uint16_t>(dx1),     \
                     ptr<const uint16_t>(dx2), ptr<const void>(da), ptr<const uint16_t>(mask),                  \
                     ptr<const uint16_t>(omask), n8)
  switch (flags & 3) {
    case 0: RG(false, false); break;
    case 1: RG(true, false); break;
    case 2: RG(false, true); break;
    default: RG(true, true); break;
  }
#undef RG
  NIDT_CHECK(hipGetLastError());
}

void res_grad(uintptr_t out, uintptr_t dx1, uintptr_t dx2, uintptr_t da, uintptr_t mask, int64_t n, int flags,
              uintptr_t stream) {
  NIDT_REQUIRE(dx2 || (da && mask), "res_grad: dx2 or da+mask");
  res_grad_om(out, dx1, dx2, da, mask, 0, n, flags, stream);
}

// Residual-stream gradient of a downsampling block: out = dx1 + (dx2 at the even pixels), with the 1x1(x1) stride-2
// shortcut's data gradient given at half resolution (dx2s [N][Do][Ho][Wo][C], Ho = ceil(H/2); D = 1 for 2-D maps):
// the shortcut conv read only the even positions, so no full-size zero-filled scatter of its gradient is needed.
template <bool OB>
__global__ void k_res_grad_s2(void* __restrict__ out, const uint16_t* __restrict__ dx1,
                              const uint16_t* __restrict__ dx2s, const uint16_t* __restrict__ omask, int64_t n8, int D,
                              int H, int W, int C) {
  const int C8 = C / 8, Do = D > 1 ? (D + 1) / 2 : 1, Ho = (H + 1) / 2, Wo = (W + 1) / 2;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n8; q += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(q % C8);
    const int64_t pix = q / C8;
    const int x = (int)(pix % W);
    int64_t r = pix / W;
    const int y = (int)(r % H);
    r /= H;
    const int z = (int)(r % D);
    const int64_t n = r / D;
    const int zz = D > 1 ? z : 0;
    float a[8], b[8];
    unpack8(*reinterpret_cast<const uint4*>(dx1 + q * 8), a);
    if (((x | y | zz) & 1) == 0) {
      const int64_t o = (((n * Do + (zz >> 1)) * Ho + (y >> 1)) * Wo + (x >> 1)) * C8 + c8;
      unpack8(*reinterpret_cast<const uint4*>(dx2s + o * 8), b);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) b[e] = 0.f;
    }
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = a[e] + b[e];
    if (omask) {  // [OMASK]
      float om[8];
      unpack8(*reinterpret_cast<const uint4*>(omask + q * 8), om);
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = om[e] > 0.f ? v[e] : 0.f;
    }
    store8(out, q, v, OB);
  }
}

void res_grad_s2_om(uintptr_t out, uintptr_t dx1, uintptr_t dx2s, uintptr_t omask, int N, int D, int H, int W, int C,
                    int out_bf16, uintptr_t stream) {
  NIDT_REQUIRE(C % 8 == 0 && D >= 1, "res_grad_s2: C % 8 == 0");
  const int64_t n8 = (int64_t)N * D * H * W * C / 8;
  const dim3 grid((unsigned)std::min<int64_t>(8192, (n8 + 255) / 256));
  if (out_bf16)
    hipLaunchKernelGGL(k_res_grad_s2<true>, grid, dim3(256), 0, as_stream(stream), ptr<void>(out),
                       ptr<const uint16_t>(dx1), ptr<const uint16_t>(dx2s), ptr<const uint16_t>(omask), n8, D, H, W, C);
  else
    hipLaunchKernelGGL(k_res_grad_s2<false>, grid, dim3(256), 0, as_stream(stream), ptr<void>(out),
                       ptr<const uint16_t>(dx1), ptr<const uint16_t>(dx2s), ptr<const uint16_t>(omask), n8, D, H, W, C);
  NIDT_CHECK(hipGetLastError());
}

void res_grad_s2(uintptr_t out, uintptr_t dx1, uintptr_t dx2s, int N, int D, int H, int W, int C, int out_bf16,
                 uintptr_t stream) {
  res_grad_s2_om(out, dx1, dx2s, 0, N, D, H, W, C, out_bf16, stream);
}

static int gn_nv(int S, int C) {
  const int chunks = S * C / 8;
  const int nv = ceil_div(chunks, kGnThreads);
  return nv <= 1 ? 1 : nv <= 2 ? 2 : nv <= 4 ? 4 : nv <= 8 ? 8 : 16;
}

static void gn_check(int N, int B, int S, int C, const char* who) {
  NIDT_REQUIRE(N > 0 && B > 0 && N % B == 0, std::string(who) + ": N % B");
  NIDT_REQUIRE(C % kGnGroups == 0 && C % 64 == 0 && C <= 512 && (kGnThreads % (C / 8)) == 0,
               std::string(who) + ": C must be a multiple of 64, <= 512");
}

static bool gn_streaming(int S, int C) { return (int64_t)S * C > 16 * 8 * kGnThreads; }

void gn_fwd(uintptr_t t, uintptr_t res, uintptr_t theta, int64_t ldt, int64_t off_w, int64_t off_b, uintptr_t y,
            uintptr_t stats, int N, int B, int S, int C, int relu, uintptr_t stream) {
  gn_check(N, B, S, C, "gn_fwd");
  hipStream_t s = as_stream(stream);
  if (gn_streaming(S, C)) {
#define GNFS(R, L)                                                                                             \
  hipLaunchKernelGGL((k_gn_fwd_stream<R, L>), dim3(N), dim3(kGnThreads), 0, s, ptr<const uint16_t>(t),          \
                     ptr<const uint16_t>(res), ptr<const float>(theta), ldt, off_w, off_b, ptr<uint16_t>(y),     \
                     ptr<float>(stats), B, S, C)
    if (res) { if (relu) GNFS(true, true); else GNFS(true, false); }
    else { if (relu) GNFS(false, true); else GNFS(false, false); }
#undef GNFS
    NIDT_CHECK(hipGetLastError());
    return;
  }
  const int nv = gn_nv(S, C);
#define GNF(NVV, R, L)                                                                                         \
  hipLaunchKernelGGL((k_gn_fwd<NVV, R, L>), dim3(N), dim3(kGnThreads), 0, s, ptr<const uint16_t>(t),            \
                     ptr<const uint16_t>(res), ptr<const float>(theta), ldt, off_w, off_b, ptr<uint16_t>(y),     \
                     ptr<float>(stats), B, S, C)
#define GNF_RL(NVV)                                                                                            \
  if (res) { if (relu) GNF(NVV, true, true); else GNF(NVV, true, false); }                                     \
  else { if (relu) GNF(NVV, false, true); else GNF(NVV, false, false); }
  switch (nv) {
    case 1: GNF_RL(1) break;
    case 2: GNF_RL(2) break;
    case 4: GNF_RL(4) break;
    case 8: GNF_RL(8) break;
    default: GNF_RL(16) break;
  }
#undef GNF_RL
#undef GNF
  NIDT_CHECK(hipGetLastError());
}

void gn_bwd(uintptr_t dy, int dy_bf16, uintptr_t mask, uintptr_t t, uintptr_t stats, uintptr_t theta, int64_t ldt,
            int64_t off_w, uintptr_t dt, uintptr_t part, int N, int B, int S, int C, uintptr_t stream) {
  gn_check(N, B, S, C, "gn_bwd");
  hipStream_t s = as_stream(stream);
  if (gn_streaming(S, C)) {
#define GNBS(DB, M)                                                                                            \
  hipLaunchKernelGGL((k_gn_bwd_stream<DB, M>), dim3(N), dim3(kGnThreads), 0, s, ptr<const void>(dy),            \
                     ptr<const uint16_t>(mask), ptr<const uint16_t>(t), ptr<const float>(stats),               \
                     ptr<const float>(theta), ldt, off_w, ptr<uint16_t>(dt), ptr<float>(part), B, S, C)
    if (dy_bf16) { if (mask) GNBS(true, true); else GNBS(true, false); }
    else { if (mask) GNBS(false, true); else GNBS(false, false); }
#undef GNBS
    NIDT_CHECK(hipGetLastError());
    return;
  }
  const int nv = gn_nv(S, C);
  // [GN-REG] hold the bf16 dy in registers up to NIDT_GN_HOLD rows per thread (round 5: 4 — at 8 rows holding cost
  // the second resident block; round 6, with the ReLU masks no longer read here ([GN-RMASK], [OMASK]): 16, CIFAR SubAvg
  // +0.8 %, DisPFL +0.2 % vs 4, profiles/r6_gn_masks.txt)
  static const int hold_max = [] {
    const char* e = getenv("NIDT_GN_HOLD");
    return e ? atoi(e) : 16;
  }();
  const bool hold = dy_bf16 && nv <= hold_max;
#define GNB(NVV, DB, M)                                                                                        \
  if (DB && hold) hipLaunchKernelGGL((k_gn_bwd<NVV, DB, M, DB>), dim3(N), dim3(kGnThreads), 0, s,               \
                     ptr<const void>(dy), ptr<const uint16_t>(mask), ptr<const uint16_t>(t), ptr<const float>(stats), \
                     ptr<const float>(theta), ldt, off_w, ptr<uint16_t>(dt), ptr<float>(part), B, S, C);        \
  else hipLaunchKernelGGL((k_gn_bwd<NVV, DB, M, false>), dim3(N), dim3(kGnThreads), 0, s, ptr<const void>(dy),  \
                     ptr<const uint16_t>(mask), ptr<const uint16_t>(t), ptr<const float>(stats),               \
                     ptr<const float>(theta), ldt, off_w, ptr<uint16_t>(dt), ptr<float>(part), B, S, C)
#define GNB_DM(NVV)                                                                                            \
  if (dy_bf16) { if (mask) GNB(NVV, true, true); else GNB(NVV, true, false); }                                 \
  else { if (mask) GNB(NVV, false, true); else GNB(NVV, false, false); }
  switch (nv) {
    case 1: GNB_DM(1) break;
    case 2: GNB_DM(2) break;
    case 4: GNB_DM(4) break;
    case 8: GNB_DM(8) break;
    default: GNB_DM(16) break;
  }
#undef GNB_DM
#undef GNB
  NIDT_CHECK(hipGetLastError());
}

// [GN-EPI] GroupNorm forward from the producing conv's epilogue statistics: part [N * nb][C][2] = (mean, M2) of each
// channel over each of the sample's nb blocks of bp positions (conv2d_fwd_slab_stats).  The sample's 32 group
// statistics are combined from them (Chan: mean = the mean of the block means, M2 = sum M2 + bp sum (block mean -
// mean)^2, population variance as k_gn_fwd), then normalisation + affine (+ residual) (+ ReLU) is a pure streaming
// pass over many blocks per sample: no reduction phases between the sample's load and store, the grid fills the chip
// (k_gn_fwd: one block per sample, its phases serialised).  Block (sample n, chunk range); block 0 of a sample writes
// the saved (mean, rstd).  sc / sh exactly as k_gn_fwd (the backward's [GN-RMASK] recomputes them).
constexpr int kGnApplyThreads = 256, kGnApplyChunks = 4;  // 16-B chunks per thread
template <bool RES, bool RELU>
__global__ __launch_bounds__(kGnApplyThreads) void k_gn_apply(const uint16_t* __restrict__ t,
                                                              const uint16_t* __restrict__ res,
                                                              const float* __restrict__ part, int nb, float bp,
                                                              const float* __restrict__ theta, int64_t ldt,
                                                              int64_t off_w, int64_t off_b, uint16_t* __restrict__ y,
                                                              float* __restrict__ stats, int B, int S, int C, int nblk) {
  __shared__ float gmean[kGnGroups], grstd[kGnGroups];
  const int n = blockIdx.x / nblk, q = blockIdx.x - n * nblk, g = n / B, tid = threadIdx.x;
  const int cg = C / kGnGroups;
  if (tid < kGnGroups) {  // group statistics of sample n (fixed order: deterministic)
    const float* pp = part + (int64_t)n * nb * C * 2;
    const int k = nb * cg;
    float m = 0.f;
    for (int b = 0; b < nb; ++b)
      for (int i = 0; i < cg; ++i) m += pp[((int64_t)b * C + tid * cg + i) * 2];
    m /= (float)k;
    float m2 = 0.f;
    for (int b = 0; b < nb; ++b)
      for (int i = 0; i < cg; ++i) {
        const float* e = pp + ((int64_t)b * C + tid * cg + i) * 2;
        const float d = e[0] - m;
        m2 += e[1] + bp * d * d;
      }
    const float rs = rsqrtf(m2 / (bp * (float)k) + kGnEps);
    gmean[tid] = m;
    grstd[tid] = rs;
    if (q == 0) {
      stats[((int64_t)n * kGnGroups + tid) * 2] = m;
      stats[((int64_t)n * kGnGroups + tid) * 2 + 1] = rs;
    }
  }
  __syncthreads();
  const int nch = C >> 3;
  const int64_t base = (int64_t)n * S * C;
  const int nchunk = S * nch;
  const float* gw = theta + (int64_t)g * ldt + off_w;
  const float* gb = theta + (int64_t)g * ldt + off_b;
#pragma unroll
  for (int k = 0; k < kGnApplyChunks; ++k) {
    const int ch = (q * kGnApplyChunks + k) * kGnApplyThreads + tid;  // 16-B chunk of the sample
    if (ch >= nchunk) break;
    const int j = ch % nch;  // 8-channel column
    float f[8], r[8];
    unpack8(*reinterpret_cast<const uint4*>(t + base + (int64_t)ch * 8), f);
    if (RES) unpack8(*reinterpret_cast<const uint4*>(res + base + (int64_t)ch * 8), r);
    uint32_t o[4];
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      float v[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = 8 * j + e + h;
        const float mu = gmean[c / cg];
        const float sc = gw[c] * grstd[c / cg];
        const float sh = gb[c] - mu * sc;
        float a = fmaf(f[e + h], sc, sh);
        if (RES) a += r[e + h];
        if (RELU) a = fmaxf(a, 0.f);
        v[h] = a;
      }
      o[e >> 1] = pack_bf16x2(v[0], v[1]);
    }
    *reinterpret_cast<uint4*>(y + base + (int64_t)ch * 8) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

void gn_apply(uintptr_t t, uintptr_t res, uintptr_t part, int nb, int bp, uintptr_t theta, int64_t ldt, int64_t off_w,
              int64_t off_b, uintptr_t y, uintptr_t stats, int N, int B, int S, int C, int relu, uintptr_t stream) {
  gn_check(N, B, S, C, "gn_apply");
  NIDT_REQUIRE(nb >= 1 && bp >= 1 && (int64_t)nb * bp == S && part != 0, "gn_apply: partials must tile the sample");
  const int nchunk = S * (C >> 3);
  const int nblk = ceil_div(nchunk, kGnApplyThreads * kGnApplyChunks);
  hipStream_t s = as_stream(stream);
#define GNA(R, L)                                                                                              \
  hipLaunchKernelGGL((k_gn_apply<R, L>), dim3((unsigned)((int64_t)N * nblk)), dim3(kGnApplyThreads), 0, s,       \
                     ptr<const uint16_t>(t), ptr<const uint16_t>(res), ptr<const float>(part), nb, (float)bp,    \
                     ptr<const float>(theta), ldt, off_w, off_b, ptr<uint16_t>(y), ptr<float>(stats), B, S, C, nblk)
  if (res) { if (relu) GNA(true, true); else GNA(true, false); }
  else { if (relu) GNA(false, true); else GNA(false, false); }
#undef GNA
  NIDT_CHECK(hipGetLastError());
}

// [GN-RMASK] gn_bwd of a GroupNorm + ReLU without residual, the ReLU mask recomputed from t (no mask tensor); the
// register-resident shapes only (gn_rm_ok), the streaming ones keep the mask tensor
int gn_rm_ok(int S, int C) { return gn_streaming(S, C) ? 0 : 1; }

void gn_bwd_rm(uintptr_t dy, int dy_bf16, uintptr_t t, uintptr_t stats, uintptr_t theta, int64_t ldt, int64_t off_w,
               int64_t off_b, uintptr_t dt, uintptr_t part, int N, int B, int S, int C, uintptr_t stream) {
  gn_check(N, B, S, C, "gn_bwd_rm");
  NIDT_REQUIRE(!gn_streaming(S, C), "gn_bwd_rm: register-resident shapes only (gn_rm_ok)");
  hipStream_t s = as_stream(stream);
  const int nv = gn_nv(S, C);
  static const int hold_max = [] {
    const char* e = getenv("NIDT_GN_HOLD");
    return e ? atoi(e) : 16;
  }();
  const bool hold = dy_bf16 && nv <= hold_max;
#define GNR(NVV, DB, H)                                                                                        \
  hipLaunchKernelGGL((k_gn_bwd<NVV, DB, false, H, true>), dim3(N), dim3(kGnThreads), 0, s, ptr<const void>(dy), \
                     nullptr, ptr<const uint16_t>(t), ptr<const float>(stats), ptr<const float>(theta), ldt, off_w,  \
                     ptr<uint16_t>(dt), ptr<float>(part), B, S, C, off_b)
#define GNR_D(NVV)                                                                                             \
  if (dy_bf16) { if (hold) GNR(NVV, true, true); else GNR(NVV, true, false); }                                 \
  else GNR(NVV, false, false);
  switch (nv) {
    case 1: GNR_D(1) break;
    case 2: GNR_D(2) break;
    case 4: GNR_D(4) break;
    case 8: GNR_D(8) break;
    default: GNR_D(16) break;
  }
#undef GNR_D
#undef GNR
  NIDT_CHECK(hipGetLastError());
}

void gn_param_grads(uintptr_t part, int G, int B, int C, uintptr_t grads, int64_t ldg, int64_t off_w, int64_t off_b,
                    uintptr_t stream) {
  NIDT_REQUIRE(C <= 512, "gn_param_grads: C <= 512");
  hipLaunchKernelGGL(k_gn_param_grads, dim3(G), dim3(256), 0, as_stream(stream), ptr<const float>(part), B, C,
                     ptr<float>(grads), ldg, off_w, off_b);
  NIDT_CHECK(hipGetLastError());
}

}  // namespace nidt
