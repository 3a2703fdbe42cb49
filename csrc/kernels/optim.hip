// Fused per-client optimizer step over the client-stacked flat parameter matrix [C, stride].
//
// Reproduces, per client row c (reference sailentgrads/my_model_trainer.py:221-231):
//   total = ||g_c||_2                                   (torch.nn.utils.clip_grad_norm_, fp32)
//   coef  = min(1, max_norm / (total + 1e-6));  g *= coef
//   d     = g + wd * w                                  (SGD weight_decay)
//   buf   = first ? d : mom * buf + d;  d = buf         (SGD momentum, dampening 0; skipped if mom==0)
//   w    -= lr * d
//   w    *= mask                                        (SalientGrads: mask applied to WEIGHTS, Q2)
// plus optional emission of a bf16 copy of the updated weights for the MFMA conv kernels.
//
// Two launches, no float atomics (bitwise reproducible): (1) per-(client, block) partial sums of
// g^2 written to a [C, nblk] slab; (2) every block of client c re-reduces that client's nblk
// partials (<= 1024 floats, L2-resident) and updates its chunk with 16-B vector accesses.
#include "common.h"

namespace nidt {

constexpr int kOptThreads = 256;

__global__ __launch_bounds__(kOptThreads) void k_row_sqnorm_partial(const float* __restrict__ g, int64_t P,
                                                                    int64_t stride, int64_t chunk,
                                                                    float* __restrict__ part, int nblk) {
  __shared__ float red[kOptThreads / 64];
  const int c = blockIdx.y;
  const int64_t s = (int64_t)blockIdx.x * chunk;
  const int64_t e = s + chunk < P ? s + chunk : P;
  const float* row = g + (int64_t)c * stride;
  float acc = 0.f;
  // vectorised body: chunk is a multiple of 4 and row base is 16-B aligned (stride % 4 == 0)
  const int64_t e4 = s + ((e - s) & ~int64_t(3));
  for (int64_t i = s + 4 * threadIdx.x; i < e4; i += 4 * kOptThreads) {
    float4 v = *reinterpret_cast<const float4*>(row + i);
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  for (int64_t i = e4 + threadIdx.x; i < e; i += kOptThreads) acc += row[i] * row[i];
  float t = block_sum(acc, red);
  if (threadIdx.x == 0) part[(int64_t)c * nblk + blockIdx.x] = t;
}

template <bool HAS_MASK, bool HAS_MOM, bool EMIT_BF16>
__global__ __launch_bounds__(kOptThreads) void k_clip_sgd_mask(
    float* __restrict__ w, float* __restrict__ g, float* __restrict__ buf, const float* __restrict__ mask,
    const float* __restrict__ part, int nblk, int64_t P, int64_t stride, int64_t chunk, float lr, float wd,
    float mom, int first, float max_norm, float* __restrict__ coef_out, uint16_t* __restrict__ wbf,
    const float* __restrict__ lr_dev, int keep_grad) {
  __shared__ float red[kOptThreads / 64];
  const int c = blockIdx.y;
  if (lr_dev) lr = *lr_dev;  // hipGraph replays: the round's learning rate lives on the device
  float t = 0.f;
  for (int i = threadIdx.x; i < nblk; i += kOptThreads) t += part[(int64_t)c * nblk + i];
  t = block_sum(t, red);
  float coef = max_norm / (sqrtf(t) + 1e-6f);
  coef = coef < 1.f ? coef : 1.f;
  if (blockIdx.x == 0 && threadIdx.x == 0 && coef_out) coef_out[c] = coef;
  const int64_t s = (int64_t)blockIdx.x * chunk;
  const int64_t e = s + chunk < P ? s + chunk : P;
  float* wr = w + (int64_t)c * stride;
  float* gr = g + (int64_t)c * stride;
  float* br = HAS_MOM ? buf + (int64_t)c * stride : nullptr;
  uint16_t* wb = EMIT_BF16 ? wbf + (int64_t)c * stride : nullptr;
  const int64_t e4 = s + ((e - s) & ~int64_t(3));
  for (int64_t i = s + 4 * threadIdx.x; i < e4; i += 4 * kOptThreads) {
    float4 gv = *reinterpret_cast<float4*>(gr + i);
    float4 wv = *reinterpret_cast<float4*>(wr + i);
    float gg[4] = {gv.x, gv.y, gv.z, gv.w};
    float ww[4] = {wv.x, wv.y, wv.z, wv.w};
    float bb[4];
    if (HAS_MOM) {
      float4 bv = *reinterpret_cast<float4*>(br + i);
      bb[0] = bv.x; bb[1] = bv.y; bb[2] = bv.z; bb[3] = bv.w;
    }
    float mm[4] = {1.f, 1.f, 1.f, 1.f};
    if (HAS_MASK) {
      float4 mv = *reinterpret_cast<const float4*>(mask + i);
      mm[0] = mv.x; mm[1] = mv.y; mm[2] = mv.z; mm[3] = mv.w;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float gj = gg[j] * coef;
      gg[j] = gj;
      float d = fmaf(wd, ww[j], gj);
      if (HAS_MOM) {
        bb[j] = first ? d : fmaf(mom, bb[j], d);
        d = bb[j];
      }
      ww[j] = fmaf(-lr, d, ww[j]);
      if (HAS_MASK) ww[j] *= mm[j];
    }
    if (keep_grad) *reinterpret_cast<float4*>(gr + i) = make_float4(gg[0], gg[1], gg[2], gg[3]);
    *reinterpret_cast<float4*>(wr + i) = make_float4(ww[0], ww[1], ww[2], ww[3]);
    if (HAS_MOM) *reinterpret_cast<float4*>(br + i) = make_float4(bb[0], bb[1], bb[2], bb[3]);
    if (EMIT_BF16) {
      ushort4 o;
      o.x = f32_to_bf16(ww[0]); o.y = f32_to_bf16(ww[1]); o.z = f32_to_bf16(ww[2]); o.w = f32_to_bf16(ww[3]);
      *reinterpret_cast<ushort4*>(wb + i) = o;
    }
  }
  for (int64_t i = e4 + threadIdx.x; i < e; i += kOptThreads) {
    float gj = gr[i] * coef;
    if (keep_grad) gr[i] = gj;
    float d = fmaf(wd, wr[i], gj);
    if (HAS_MOM) {
      float b = first ? d : fmaf(mom, br[i], d);
      br[i] = b;
      d = b;
    }
    float nw = fmaf(-lr, d, wr[i]);
    if (HAS_MASK) nw *= mask[i];
    wr[i] = nw;
    if (EMIT_BF16) wb[i] = f32_to_bf16(nw);
  }
}

static int64_t opt_chunk(int64_t P, int* nblk) {
  // ~ 256 threads x 4 floats x 8 iterations per block; cap blocks per row at 1024
  int64_t chunk = 8192;
  int64_t nb = (P + chunk - 1) / chunk;
  if (nb > 1024) {
    chunk = ((P + 1023) / 1024 + 3) & ~int64_t(3);
    nb = (P + chunk - 1) / chunk;
  }
  *nblk = (int)nb;
  return chunk;
}

int64_t clip_sgd_mask_workspace(int64_t C, int64_t P) {
  int nb;
  opt_chunk(P, &nb);
  return C * nb;
}

void clip_sgd_mask(uintptr_t w, uintptr_t g, uintptr_t buf, uintptr_t mask, uintptr_t part, uintptr_t coef_out,
                   uintptr_t wbf, int64_t C, int64_t P, int64_t stride, float lr, float wd, float mom, int first,
                   float max_norm, uintptr_t lr_dev, int keep_grad, uintptr_t stream) {
  NIDT_REQUIRE(stride % 4 == 0 && stride >= P, "stride must be >= P and a multiple of 4");
  NIDT_REQUIRE((w & 15) == 0 && (g & 15) == 0 && (buf & 15) == 0 && (mask & 15) == 0 && (wbf & 7) == 0,
               "buffers must be 16-byte aligned");
  int nblk;
  int64_t chunk = opt_chunk(P, &nblk);
  hipStream_t st = as_stream(stream);
  dim3 grid(nblk, (unsigned)C);
  hipLaunchKernelGGL(k_row_sqnorm_partial, grid, dim3(kOptThreads), 0, st, ptr<const float>(g), P, stride, chunk,
                     ptr<float>(part), nblk);
  const bool hm = mask != 0, hmo = (buf != 0 && mom != 0.f), hb = wbf != 0;
#define NIDT_LAUNCH(M, MO, B)                                                                                   \
  hipLaunchKernelGGL((k_clip_sgd_mask<M, MO, B>), grid, dim3(kOptThreads), 0, st, ptr<float>(w), ptr<float>(g),      \
                     ptr<float>(buf), ptr<const float>(mask), ptr<const float>(part), nblk, P, stride, chunk, lr, wd,   \
                     mom, first, max_norm, ptr<float>(coef_out), ptr<uint16_t>(wbf), ptr<const float>(lr_dev),  \
                     keep_grad)
  if (hm && hmo && hb) NIDT_LAUNCH(true, true, true);
  else if (hm && hmo && !hb) NIDT_LAUNCH(true, true, false);
  else if (hm && !hmo && hb) NIDT_LAUNCH(true, false, true);
  else if (hm && !hmo && !hb) NIDT_LAUNCH(true, false, false);
  else if (!hm && hmo && hb) NIDT_LAUNCH(false, true, true);
  else if (!hm && hmo && !hb) NIDT_LAUNCH(false, true, false);
  else if (!hm && !hmo && hb) NIDT_LAUNCH(false, false, true);
  else NIDT_LAUNCH(false, false, false);
#undef NIDT_LAUNCH
  NIDT_CHECK(hipGetLastError());
}

// ---- weighted reduction over the client axis: out[p] = sum_c wts[c] * rows[c, p] (+ beta*out) ----
__global__ __launch_bounds__(256) void k_weighted_rows_sum(const float* __restrict__ rows, const float* __restrict__ wts,
                                                           int C, int64_t P, int64_t stride, float beta,
                                                           float* __restrict__ out) {
  const int64_t i = 4 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= P) return;
  if (i + 3 < P) {
    float4 acc = beta != 0.f ? *reinterpret_cast<const float4*>(out + i) : make_float4(0, 0, 0, 0);
    acc.x *= beta; acc.y *= beta; acc.z *= beta; acc.w *= beta;
    for (int c = 0; c < C; ++c) {
      const float wc = wts[c];
      float4 v = *reinterpret_cast<const float4*>(rows + (int64_t)c * stride + i);
      acc.x = fmaf(wc, v.x, acc.x); acc.y = fmaf(wc, v.y, acc.y);
      acc.z = fmaf(wc, v.z, acc.z); acc.w = fmaf(wc, v.w, acc.w);
    }
    *reinterpret_cast<float4*>(out + i) = acc;
  } else {
    for (int64_t j = i; j < P; ++j) {
      float acc = beta != 0.f ? beta * out[j] : 0.f;
      for (int c = 0; c < C; ++c) acc = fmaf(wts[c], rows[(int64_t)c * stride + j], acc);
      out[j] = acc;
    }
  }
}

void weighted_rows_sum(uintptr_t rows, uintptr_t wts, int64_t C, int64_t P, int64_t stride, float beta, uintptr_t out,
                       uintptr_t stream) {
  NIDT_REQUIRE(stride % 4 == 0 && (rows & 15) == 0 && (out & 15) == 0, "alignment");
  const int64_t n4 = (P + 3) / 4;
  hipLaunchKernelGGL(k_weighted_rows_sum, dim3(ceil_div(n4, 256)), dim3(256), 0, as_stream(stream),
                     ptr<const float>(rows), ptr<const float>(wts), (int)C, P, stride, beta, ptr<float>(out));
  NIDT_CHECK(hipGetLastError());
}

// ---- broadcast one row into C rows (round start: every client starts from w_global) ----
__global__ void k_broadcast_row(const float* __restrict__ src, int64_t P, int64_t stride, int C, float* __restrict__ dst) {
  const int64_t i = 4 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= P) return;
  if (i + 3 < P) {
    float4 v = *reinterpret_cast<const float4*>(src + i);
    for (int c = 0; c < C; ++c) *reinterpret_cast<float4*>(dst + (int64_t)c * stride + i) = v;
  } else {
    for (int64_t j = i; j < P; ++j)
      for (int c = 0; c < C; ++c) dst[(int64_t)c * stride + j] = src[j];
  }
}

void broadcast_row(uintptr_t src, int64_t P, int64_t stride, int64_t C, uintptr_t dst, uintptr_t stream) {
  NIDT_REQUIRE(stride % 4 == 0 && (src & 15) == 0 && (dst & 15) == 0, "alignment");
  const int64_t n4 = (P + 3) / 4;
  hipLaunchKernelGGL(k_broadcast_row, dim3(ceil_div(n4, 256)), dim3(256), 0, as_stream(stream), ptr<const float>(src), P,
                     stride, (int)C, ptr<float>(dst));
  NIDT_CHECK(hipGetLastError());
}

}  // namespace nidt
