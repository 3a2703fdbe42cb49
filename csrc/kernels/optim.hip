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
#include "pack.h"

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

// ------------------------------------------------------------------------------------------------
// Generalised fused local step for every algorithm of the harness, per client row c:
//   g' = g * m_c            (mask_mode GRAD: SubAvg masks gradients before clipping, subavg/my_model_trainer.py:66-68)
//   g' += mu * (w - ref_c)  (FedProx proximal gradient, inside the clipped norm like a loss term)
//   coef = min(1, max_norm / (||g'|| + 1e-6));  d = coef g' + wd w;  buf = mom buf + d (buf zeroed at round start)
//   w -= lr d
//   w -= lr * lamda * (w - pref_c)   (Ditto personal pull after the step, ditto/my_model_trainer.py:63-64)
//   w *= m_c                (mask_mode WEIGHT: SalientGrads / DisPFL re-zero masked weights, Q2)
// Masks are bit rows (uint32 words, bit i of word i>>5); mstride = 0 shares one mask row between all clients
// (SalientGrads' global SNIP mask).  ref/pref row strides may be 0 (w_global shared by every client).
struct LocalOpt {
  float* w; float* g; float* buf; int64_t ld;
  const uint32_t* mbits; int64_t mstride;
  const float* ref; int64_t ref_ld; float mu;
  const float* pref; int64_t pref_ld; float lamda;
  float lr, wd, mom, max_norm;
  const float* lr_dev;
  int keep_grad;
};

enum { kMaskNone = 0, kMaskWeight = 1, kMaskGrad = 2 };

template <int MASK>
__device__ __forceinline__ uint32_t mask4(const LocalOpt& a, int c, int64_t i) {
  if (MASK == kMaskNone) return 0xfu;
  return (a.mbits[(int64_t)c * a.mstride + (i >> 5)] >> (i & 31)) & 0xfu;
}

template <int MASK>
__global__ __launch_bounds__(kOptThreads) void k_local_sqnorm(LocalOpt a, int64_t P, int64_t chunk,
                                                              float* __restrict__ part, int nblk) {
  __shared__ float red[kOptThreads / 64];
  const int c = blockIdx.y;
  const int64_t s = (int64_t)blockIdx.x * chunk;
  const int64_t e = s + chunk < P ? s + chunk : P;
  const float* gr = a.g + (int64_t)c * a.ld;
  const float* wr = a.w + (int64_t)c * a.ld;
  const float* rr = a.mu != 0.f ? a.ref + (int64_t)c * a.ref_ld : nullptr;
  float acc = 0.f;
  const int64_t e4 = s + ((e - s) & ~int64_t(3));
  for (int64_t i = s + 4 * threadIdx.x; i < e4; i += 4 * kOptThreads) {
    const float4 gv = *reinterpret_cast<const float4*>(gr + i);
    float gg[4] = {gv.x, gv.y, gv.z, gv.w};
    if (MASK == kMaskGrad) {
      const uint32_t m = mask4<MASK>(a, c, i);
#pragma unroll
      for (int j = 0; j < 4; ++j) gg[j] = ((m >> j) & 1u) ? gg[j] : 0.f;
    }
    if (rr) {
      const float4 wv = *reinterpret_cast<const float4*>(wr + i), rv = *reinterpret_cast<const float4*>(rr + i);
      gg[0] = fmaf(a.mu, wv.x - rv.x, gg[0]); gg[1] = fmaf(a.mu, wv.y - rv.y, gg[1]);
      gg[2] = fmaf(a.mu, wv.z - rv.z, gg[2]); gg[3] = fmaf(a.mu, wv.w - rv.w, gg[3]);
    }
    acc += gg[0] * gg[0] + gg[1] * gg[1] + gg[2] * gg[2] + gg[3] * gg[3];
  }
  for (int64_t i = e4 + threadIdx.x; i < e; i += kOptThreads) {
    float gj = gr[i];
    if (MASK == kMaskGrad && !((a.mbits[(int64_t)c * a.mstride + (i >> 5)] >> (i & 31)) & 1u)) gj = 0.f;
    if (rr) gj = fmaf(a.mu, wr[i] - rr[i], gj);
    acc += gj * gj;
  }
  const float t = block_sum(acc, red);
  if (threadIdx.x == 0) part[(int64_t)c * nblk + blockIdx.x] = t;
}

// clip coefficient of client row c from its sqnorm partials (every thread of the block takes part)
__device__ __forceinline__ float opt_coef(const LocalOpt& a, const float* __restrict__ part, int nblk, int c,
                                          float* red) {
  float t = 0.f;
  for (int i = threadIdx.x; i < nblk; i += kOptThreads) t += part[(int64_t)c * nblk + i];
  t = block_sum(t, red);
  const float coef = a.max_norm / (sqrtf(t) + 1e-6f);
  return coef < 1.f ? coef : 1.f;
}

// the step on elements [s, e) of client row c (16-B accesses on the 4-aligned body, scalars at the ends); stage
// (optional, LDS): the updated weights at stage[i - s]
template <int MASK, bool HAS_MOM>
__device__ __forceinline__ void opt_range(const LocalOpt& a, int c, float coef, float lr, int64_t s, int64_t e,
                                          float* stage) {
  float* wr = a.w + (int64_t)c * a.ld;
  float* gr = a.g + (int64_t)c * a.ld;
  float* br = HAS_MOM ? a.buf + (int64_t)c * a.ld : nullptr;
  const float* rr = a.mu != 0.f ? a.ref + (int64_t)c * a.ref_ld : nullptr;
  const float* pr = a.lamda != 0.f ? a.pref + (int64_t)c * a.pref_ld : nullptr;
  const float pull = lr * a.lamda;
  auto one = [&](float& ww, float& gg, float& bb, float rv, float pv, bool m) {
    float gj = (MASK == kMaskGrad && !m) ? 0.f : gg;
    if (rr) gj = fmaf(a.mu, ww - rv, gj);
    gj *= coef;
    gg = gj;
    float d = fmaf(a.wd, ww, gj);
    if (HAS_MOM) {
      bb = fmaf(a.mom, bb, d);
      d = bb;
    }
    ww = fmaf(-lr, d, ww);
    if (pr) ww = fmaf(-pull, ww - pv, ww);
    if (MASK == kMaskWeight && !m) ww = 0.f;
  };
  auto scalar = [&](int64_t i) {
    float ww = wr[i], gg = gr[i], bb = HAS_MOM ? br[i] : 0.f;
    const bool m = MASK == kMaskNone ? true : ((a.mbits[(int64_t)c * a.mstride + (i >> 5)] >> (i & 31)) & 1u);
    one(ww, gg, bb, rr ? rr[i] : 0.f, pr ? pr[i] : 0.f, m);
    if (a.keep_grad) gr[i] = gg;
    wr[i] = ww;
    if (HAS_MOM) br[i] = bb;
    if (stage) stage[i - s] = ww;
  };
  int64_t s4 = (s + 3) & ~int64_t(3);
  if (s4 > e) s4 = e;
  const int64_t e4 = s4 + ((e - s4) & ~int64_t(3));
  for (int64_t i = s + threadIdx.x; i < s4; i += kOptThreads) scalar(i);
  for (int64_t i = s4 + 4 * threadIdx.x; i < e4; i += 4 * kOptThreads) {
    const float4 gv = *reinterpret_cast<const float4*>(gr + i);
    const float4 wv = *reinterpret_cast<const float4*>(wr + i);
    float gg[4] = {gv.x, gv.y, gv.z, gv.w}, ww[4] = {wv.x, wv.y, wv.z, wv.w};
    float bb[4] = {0.f, 0.f, 0.f, 0.f}, rv[4] = {0.f, 0.f, 0.f, 0.f}, pv[4] = {0.f, 0.f, 0.f, 0.f};
    if (HAS_MOM) {
      const float4 v = *reinterpret_cast<const float4*>(br + i);
      bb[0] = v.x; bb[1] = v.y; bb[2] = v.z; bb[3] = v.w;
    }
    if (rr) {
      const float4 v = *reinterpret_cast<const float4*>(rr + i);
      rv[0] = v.x; rv[1] = v.y; rv[2] = v.z; rv[3] = v.w;
    }
    if (pr) {
      const float4 v = *reinterpret_cast<const float4*>(pr + i);
      pv[0] = v.x; pv[1] = v.y; pv[2] = v.z; pv[3] = v.w;
    }
    const uint32_t m = mask4<MASK>(a, c, i);
#pragma unroll
    for (int j = 0; j < 4; ++j) one(ww[j], gg[j], bb[j], rv[j], pv[j], (m >> j) & 1u);
    if (a.keep_grad) *reinterpret_cast<float4*>(gr + i) = make_float4(gg[0], gg[1], gg[2], gg[3]);
    *reinterpret_cast<float4*>(wr + i) = make_float4(ww[0], ww[1], ww[2], ww[3]);
    if (HAS_MOM) *reinterpret_cast<float4*>(br + i) = make_float4(bb[0], bb[1], bb[2], bb[3]);
    if (stage) {
#pragma unroll
      for (int j = 0; j < 4; ++j) stage[i - s + j] = ww[j];
    }
  }
  for (int64_t i = e4 + threadIdx.x; i < e; i += kOptThreads) scalar(i);
}

template <int MASK, bool HAS_MOM>
__global__ __launch_bounds__(kOptThreads) void k_local_step(LocalOpt a, const float* __restrict__ part, int nblk,
                                                            int64_t P, int64_t chunk) {
  __shared__ float red[kOptThreads / 64];
  const int c = blockIdx.y;
  const float lr = a.lr_dev ? *a.lr_dev : a.lr;
  const float coef = opt_coef(a, part, nblk, c, red);
  const int64_t s = (int64_t)blockIdx.x * chunk;
  const int64_t e = s + chunk < P ? s + chunk : P;
  opt_range<MASK, HAS_MOM>(a, c, coef, lr, s, e, nullptr);
}

// [PACK-FUSE] The step with the next forward's bf16 weight images written from the updated values (no k_pack_plain
// re-read of the fp32 rows).  Blocks [0, nconv): one plain-grid chunk of a conv layer each (desc: blk_plain prefixes
// over every conv layer, 1x1 included), updated into LDS and written as image rows (pack.h pack_image_chunk);
// blocks [nconv, nconv + nrest): the ranges of the other parameters (rest: {start, length} pairs).
template <int MASK, bool HAS_MOM>
__global__ __launch_bounds__(kOptThreads) void k_local_step_pack(LocalOpt a, const float* __restrict__ part, int nblk,
                                                                 const PackDesc* __restrict__ desc, int nd, int nconv,
                                                                 const int64_t* __restrict__ rest,
                                                                 uint16_t* __restrict__ out) {
  extern __shared__ float row[];
  __shared__ float red[kOptThreads / 64];
  const int c = blockIdx.y;
  const float lr = a.lr_dev ? *a.lr_dev : a.lr;
  const float coef = opt_coef(a, part, nblk, c, red);
  if ((int)blockIdx.x >= nconv) {
    const int64_t* r = rest + 2 * ((int64_t)blockIdx.x - nconv);
    opt_range<MASK, HAS_MOM>(a, c, coef, lr, r[0], r[0] + r[1], nullptr);
    return;
  }
  const int li = find_layer(desc, nd, blockIdx.x, 0);
  const PackDesc& d = desc[li];
  const int Cin = d.cin_p, kt = d.kt, cs = d.cin_src;
  const int CC = pack_cc(Cin, kt), nch = (Cin + CC - 1) / CC;
  const int b = blockIdx.x - d.blk_plain, co = b / nch, ci0 = (b - co * nch) * CC;
  const int cw = min(CC, Cin - ci0);
  const int cc = max(0, min(CC, cs - ci0));
  const int64_t s = d.src_off + ((int64_t)co * cs + ci0) * kt;
  opt_range<MASK, HAS_MOM>(a, c, coef, lr, s, s + (int64_t)cc * kt, row);
  __syncthreads();
  pack_image_chunk(d, row, out, c, co, ci0, cw, cc);
}

// [PACK-WT] The step writing BOTH bf16 images of the next training step: the forward image wp[g][Cout][kt][Cin_p] and
// the data-gradient image wt[g][Cin_p][slot(t)][Cout] (pack.hip's layouts), so no k_pack_trans pass re-reads wp and
// writes wt in the next step.  Conv blocks are tiles of kWtCo output x kWtCi input channels x all taps: the tile's
// updated weights go to LDS as bf16 in PyTorch order ([co][ci][t]: 72 KB at kt = 9, two blocks per CU), the forward
// image is written in 128-B runs (64 input channels of one (co, t)) and the transposed image in 128-B runs (64 output
// channels of one (ci, slot)) — bit-identical to k_pack_plain + k_pack_trans.  Opt-in (NIDT_PACK_WT=1): measured
// slower than k_pack_trans overlapped on the side stream, with 16- and 64-channel tiles (profiles/r6_pack_wt.txt).  Blocks
// [nconv, nconv + nrest): the other parameter ranges, as k_local_step_pack.  desc.blk_plain = this tiled grid's
// prefixes (host: wt_tiles).
constexpr int kWtCo = 64, kWtCi = 64;
int wt_tiles(int cout, int cin_p) { return ((cout + kWtCo - 1) / kWtCo) * ((cin_p + kWtCi - 1) / kWtCi); }
int wt_tile_lds(int kt) { return kWtCo * kWtCi * kt * 2; }

template <int MASK, bool HAS_MOM>
__global__ __launch_bounds__(kOptThreads) void k_local_step_pack_wt(LocalOpt a, const float* __restrict__ part,
                                                                    int nblk, const PackDesc* __restrict__ desc, int nd,
                                                                    int nconv, const int64_t* __restrict__ rest,
                                                                    uint16_t* __restrict__ out) {
  extern __shared__ uint16_t rowh[];
  __shared__ float red[kOptThreads / 64];
  const int c = blockIdx.y;
  const float lr = a.lr_dev ? *a.lr_dev : a.lr;
  const float coef = opt_coef(a, part, nblk, c, red);
  if ((int)blockIdx.x >= nconv) {
    const int64_t* r = rest + 2 * ((int64_t)blockIdx.x - nconv);
    opt_range<MASK, HAS_MOM>(a, c, coef, lr, r[0], r[0] + r[1], nullptr);
    return;
  }
  const int li = find_layer(desc, nd, blockIdx.x, 0);
  const PackDesc& d = desc[li];
  const int Cin = d.cin_p, kt = d.kt, cs = d.cin_src, Cout = d.cout;
  const int nci = (Cin + kWtCi - 1) / kWtCi;
  const int b = blockIdx.x - d.blk_plain, co0 = (b / nci) * kWtCo, ci0 = (b - (b / nci) * nci) * kWtCi;
  const int nco = min(kWtCo, Cout - co0), cw = min(kWtCi, Cin - ci0), cc = max(0, min(kWtCi, cs - ci0));
  const int RS = kWtCi * kt;  // LDS elements per output channel of the tile
  const int L = cc * kt;      // live elements per output channel (contiguous in the PyTorch row)
  const int64_t base = d.src_off + (int64_t)co0 * cs * kt + (int64_t)ci0 * kt, rstr = (int64_t)cs * kt;
  float* wr = a.w + (int64_t)c * a.ld;
  float* gr = a.g + (int64_t)c * a.ld;
  float* br = HAS_MOM ? a.buf + (int64_t)c * a.ld : nullptr;
  const float* rr = a.mu != 0.f ? a.ref + (int64_t)c * a.ref_ld : nullptr;
  const float* pr = a.lamda != 0.f ? a.pref + (int64_t)c * a.pref_ld : nullptr;
  const float pull = lr * a.lamda;
  auto step1 = [&](float& ww, float& gg, float& bb, int64_t gi, bool m) {  // the element step of opt_range
    float gj = (MASK == kMaskGrad && !m) ? 0.f : gg;
    if (rr) gj = fmaf(a.mu, ww - rr[gi], gj);
    gj *= coef;
    gg = gj;
    float dd = fmaf(a.wd, ww, gj);
    if (HAS_MOM) {
      bb = fmaf(a.mom, bb, dd);
      dd = bb;
    }
    ww = fmaf(-lr, dd, ww);
    if (pr) ww = fmaf(-pull, ww - pr[gi], ww);
    if (MASK == kMaskWeight && !m) ww = 0.f;
  };
  if (L % 4 == 0 && (base & 3) == 0 && (rstr & 3) == 0) {  // the tile's rows as one flat loop of 16-B accesses
    const int L4 = L >> 2;
    for (int e = threadIdx.x; e < nco * L4; e += kOptThreads) {
      const int r = e / L4, i = (e - r * L4) * 4;
      const int64_t gi = base + r * rstr + i;
      const float4 gv = *reinterpret_cast<const float4*>(gr + gi), wv = *reinterpret_cast<const float4*>(wr + gi);
      float gg[4] = {gv.x, gv.y, gv.z, gv.w}, ww[4] = {wv.x, wv.y, wv.z, wv.w}, bb[4] = {0.f, 0.f, 0.f, 0.f};
      if (HAS_MOM) {
        const float4 v = *reinterpret_cast<const float4*>(br + gi);
        bb[0] = v.x; bb[1] = v.y; bb[2] = v.z; bb[3] = v.w;
      }
      const uint32_t m = mask4<MASK>(a, c, gi);
#pragma unroll
      for (int j = 0; j < 4; ++j) step1(ww[j], gg[j], bb[j], gi + j, (m >> j) & 1u);
      if (a.keep_grad) *reinterpret_cast<float4*>(gr + gi) = make_float4(gg[0], gg[1], gg[2], gg[3]);
      *reinterpret_cast<float4*>(wr + gi) = make_float4(ww[0], ww[1], ww[2], ww[3]);
      if (HAS_MOM) *reinterpret_cast<float4*>(br + gi) = make_float4(bb[0], bb[1], bb[2], bb[3]);
      *reinterpret_cast<uint2*>(rowh + r * RS + i) = make_uint2(pack_bf16x2(ww[0], ww[1]), pack_bf16x2(ww[2], ww[3]));
    }
  } else {  // unaligned rows (the 3-channel stem): element by element
    for (int e = threadIdx.x; e < nco * L; e += kOptThreads) {
      const int r = e / L, i = e - r * L;
      const int64_t gi = base + r * rstr + i;
      float ww = wr[gi], gg = gr[gi], bb = HAS_MOM ? br[gi] : 0.f;
      const bool m = MASK == kMaskNone ? true : ((a.mbits[(int64_t)c * a.mstride + (gi >> 5)] >> (gi & 31)) & 1u);
      step1(ww, gg, bb, gi, m);
      if (a.keep_grad) gr[gi] = gg;
      wr[gi] = ww;
      if (HAS_MOM) br[gi] = bb;
      rowh[r * RS + i] = f32_to_bf16(ww);
    }
  }
  __syncthreads();
  auto w_at = [&](int r, int ci, int t) -> uint32_t { return ci < cc ? (uint32_t)rowh[r * RS + ci * kt + t] : 0u; };
  uint16_t* wp = out + d.wp_off + (int64_t)c * Cout * kt * Cin;
  const int nq = cw >> 3;
  for (int e = threadIdx.x; e < nco * kt * nq; e += kOptThreads) {
    const int q = e % nq, rt = e / nq, t = rt % kt, r = rt / kt;
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = w_at(r, 8 * q + 2 * k, t) | (w_at(r, 8 * q + 2 * k + 1, t) << 16);
    *reinterpret_cast<uint4*>(wp + ((int64_t)(co0 + r) * kt + t) * Cin + ci0 + 8 * q) = make_uint4(w[0], w[1], w[2], w[3]);
  }
  if (d.wt_off < 0) return;
  uint16_t* wt = out + d.wt_off + (int64_t)c * Cin * kt * Cout;
  const int nq2 = nco >> 3;
  for (int e = threadIdx.x; e < cw * kt * nq2; e += kOptThreads) {
    const int q = e % nq2, rt = e / nq2, t = rt % kt, ci = rt / kt;
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = w_at(8 * q + 2 * k, ci, t) | (w_at(8 * q + 2 * k + 1, ci, t) << 16);
    *reinterpret_cast<uint4*>(wt + ((int64_t)(ci0 + ci) * kt + d.slot[t]) * Cout + co0 + 8 * q) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

void local_opt(uintptr_t w, uintptr_t g, uintptr_t buf, int64_t ld, uintptr_t mbits, int64_t mstride, int mask_mode,
               uintptr_t ref, int64_t ref_ld, float mu, uintptr_t pref, int64_t pref_ld, float lamda, uintptr_t part,
               int64_t C, int64_t P, float lr, float wd, float mom, float max_norm, uintptr_t lr_dev, int keep_grad,
               uintptr_t stream) {
  NIDT_REQUIRE(ld % 4 == 0 && ld >= P, "local_opt: row stride must be >= P and a multiple of 4");
  NIDT_REQUIRE((w & 15) == 0 && (g & 15) == 0 && (buf & 15) == 0, "local_opt: 16-byte alignment");
  NIDT_REQUIRE(mask_mode == kMaskNone || (mbits != 0 && mstride % 4 == 0 && (mbits & 15) == 0), "local_opt: mask");
  NIDT_REQUIRE(mu == 0.f || (ref != 0 && ref_ld % 4 == 0 && (ref & 15) == 0), "local_opt: prox reference");
  NIDT_REQUIRE(lamda == 0.f || (pref != 0 && pref_ld % 4 == 0 && (pref & 15) == 0), "local_opt: pull reference");
  if (C == 0) return;
  LocalOpt a{ptr<float>(w), ptr<float>(g), ptr<float>(buf), ld, ptr<const uint32_t>(mbits), mstride,
             ptr<const float>(ref), ref_ld, mu, ptr<const float>(pref), pref_ld, lamda, lr, wd, mom, max_norm,
             ptr<const float>(lr_dev), keep_grad};
  int nblk;
  const int64_t chunk = opt_chunk(P, &nblk);
  hipStream_t st = as_stream(stream);
  dim3 grid(nblk, (unsigned)C);
  if (mask_mode == kMaskGrad)
    hipLaunchKernelGGL(k_local_sqnorm<kMaskGrad>, grid, dim3(kOptThreads), 0, st, a, P, chunk, ptr<float>(part), nblk);
  else
    hipLaunchKernelGGL(k_local_sqnorm<kMaskNone>, grid, dim3(kOptThreads), 0, st, a, P, chunk, ptr<float>(part), nblk);
  const bool hm = buf != 0 && mom != 0.f;
#define NIDT_LS(M, MO)                                                                                            \
  hipLaunchKernelGGL((k_local_step<M, MO>), grid, dim3(kOptThreads), 0, st, a, ptr<const float>(part), nblk, P, chunk)
  switch (mask_mode * 2 + (hm ? 1 : 0)) {
    case 0: NIDT_LS(kMaskNone, false); break;
    case 1: NIDT_LS(kMaskNone, true); break;
    case 2: NIDT_LS(kMaskWeight, false); break;
    case 3: NIDT_LS(kMaskWeight, true); break;
    case 4: NIDT_LS(kMaskGrad, false); break;
    case 5: NIDT_LS(kMaskGrad, true); break;
    default: NIDT_REQUIRE(false, "local_opt: mask_mode");
  }
#undef NIDT_LS
  NIDT_CHECK(hipGetLastError());
}

// local_opt + the forward images of the conv layers (k_local_step_pack): desc / nd / nconv = the fused plain grid,
// rest / nrest = the other parameter ranges, lds = bytes of the largest chunk, out = the packed image buffer
static void local_opt_pack_impl(uintptr_t w, uintptr_t g, uintptr_t buf, int64_t ld, uintptr_t mbits,
                                int64_t mstride, int mask_mode, uintptr_t ref, int64_t ref_ld, float mu,
                                uintptr_t pref, int64_t pref_ld, float lamda, uintptr_t part, int64_t C, int64_t P,
                                float lr, float wd, float mom, float max_norm, uintptr_t lr_dev, int keep_grad,
                                uintptr_t desc, int nd, int nconv, uintptr_t rest, int nrest, int lds, uintptr_t out,
                                uintptr_t stream, bool wt) {
  NIDT_REQUIRE(ld % 4 == 0 && ld >= P, "local_opt_pack: row stride must be >= P and a multiple of 4");
  NIDT_REQUIRE((w & 15) == 0 && (g & 15) == 0 && (buf & 15) == 0, "local_opt_pack: 16-byte alignment");
  NIDT_REQUIRE(mask_mode == kMaskNone || (mbits != 0 && mstride % 4 == 0 && (mbits & 15) == 0), "local_opt_pack: mask");
  NIDT_REQUIRE(mu == 0.f || (ref != 0 && ref_ld % 4 == 0 && (ref & 15) == 0), "local_opt_pack: prox reference");
  NIDT_REQUIRE(lamda == 0.f || (pref != 0 && pref_ld % 4 == 0 && (pref & 15) == 0), "local_opt_pack: pull reference");
  NIDT_REQUIRE(desc != 0 && nd > 0 && nconv > 0 && nrest >= 0 && (nrest == 0 || rest != 0) && out != 0 && lds > 0 &&
               lds <= (wt ? 80 : 64) * 1024, "local_opt_pack: bad pack plan");
  if (C == 0) return;
  LocalOpt a{ptr<float>(w), ptr<float>(g), ptr<float>(buf), ld, ptr<const uint32_t>(mbits), mstride,
             ptr<const float>(ref), ref_ld, mu, ptr<const float>(pref), pref_ld, lamda, lr, wd, mom, max_norm,
             ptr<const float>(lr_dev), keep_grad};
  int nblk;
  const int64_t chunk = opt_chunk(P, &nblk);
  hipStream_t st = as_stream(stream);
  const dim3 grid(nblk, (unsigned)C);
  if (mask_mode == kMaskGrad)
    hipLaunchKernelGGL(k_local_sqnorm<kMaskGrad>, grid, dim3(kOptThreads), 0, st, a, P, chunk, ptr<float>(part), nblk);
  else
    hipLaunchKernelGGL(k_local_sqnorm<kMaskNone>, grid, dim3(kOptThreads), 0, st, a, P, chunk, ptr<float>(part), nblk);
  const bool hm = buf != 0 && mom != 0.f;
  const dim3 pgrid((unsigned)(nconv + nrest), (unsigned)C);
#define NIDT_LSP(M, MO)                                                                                        \
  if (wt) {                                                                                                    \
    NIDT_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_local_step_pack_wt<M, MO>),                   \
                                   hipFuncAttributeMaxDynamicSharedMemorySize, lds));                            \
    hipLaunchKernelGGL((k_local_step_pack_wt<M, MO>), pgrid, dim3(kOptThreads), lds, st, a, ptr<const float>(part), \
                       nblk, ptr<const PackDesc>(desc), nd, nconv, ptr<const int64_t>(rest), ptr<uint16_t>(out));  \
  } else                                                                                                       \
    hipLaunchKernelGGL((k_local_step_pack<M, MO>), pgrid, dim3(kOptThreads), lds, st, a, ptr<const float>(part), \
                       nblk, ptr<const PackDesc>(desc), nd, nconv, ptr<const int64_t>(rest), ptr<uint16_t>(out))
  switch (mask_mode * 2 + (hm ? 1 : 0)) {
    case 0: NIDT_LSP(kMaskNone, false); break;
    case 1: NIDT_LSP(kMaskNone, true); break;
    case 2: NIDT_LSP(kMaskWeight, false); break;
    case 3: NIDT_LSP(kMaskWeight, true); break;
    case 4: NIDT_LSP(kMaskGrad, false); break;
    case 5: NIDT_LSP(kMaskGrad, true); break;
    default: NIDT_REQUIRE(false, "local_opt_pack: mask_mode");
  }
#undef NIDT_LSP
  NIDT_CHECK(hipGetLastError());
}

void local_opt_pack(uintptr_t w, uintptr_t g, uintptr_t buf, int64_t ld, uintptr_t mbits, int64_t mstride,
                    int mask_mode, uintptr_t ref, int64_t ref_ld, float mu, uintptr_t pref, int64_t pref_ld,
                    float lamda, uintptr_t part, int64_t C, int64_t P, float lr, float wd, float mom, float max_norm,
                    uintptr_t lr_dev, int keep_grad, uintptr_t desc, int nd, int nconv, uintptr_t rest, int nrest,
                    int lds, uintptr_t out, uintptr_t stream) {
  local_opt_pack_impl(w, g, buf, ld, mbits, mstride, mask_mode, ref, ref_ld, mu, pref, pref_ld, lamda, part, C, P, lr,
                      wd, mom, max_norm, lr_dev, keep_grad, desc, nd, nconv, rest, nrest, lds, out, stream, false);
}

// [PACK-WT] local_opt_pack over the tiled grid (desc.blk_plain = wt_tiles prefixes; lds = wt_tile_lds(max kt)), also
// writing the data-gradient images of the layers with wt_off >= 0 (every layer: Cout % 16 == 0, Cin_p % 8 == 0)
void local_opt_pack_wt(uintptr_t w, uintptr_t g, uintptr_t buf, int64_t ld, uintptr_t mbits, int64_t mstride,
                       int mask_mode, uintptr_t ref, int64_t ref_ld, float mu, uintptr_t pref, int64_t pref_ld,
                       float lamda, uintptr_t part, int64_t C, int64_t P, float lr, float wd, float mom, float max_norm,
                       uintptr_t lr_dev, int keep_grad, uintptr_t desc, int nd, int nconv, uintptr_t rest, int nrest,
                       int lds, uintptr_t out, uintptr_t stream) {
  local_opt_pack_impl(w, g, buf, ld, mbits, mstride, mask_mode, ref, ref_ld, mu, pref, pref_ld, lamda, part, C, P, lr,
                      wd, mom, max_norm, lr_dev, keep_grad, desc, nd, nconv, rest, nrest, lds, out, stream, true);
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

// ---- non-zero count per row (the reference's count_communication_params, once per round per client) ----
// grid (nblk, R): block b of row r counts [b * chunk, (b + 1) * chunk) with 16-B loads and writes one int32
// partial (no atomics); the caller sums the [R, nblk] partials.  torch.count_nonzero(dim=1) ran at ~0.15 TB/s.
__global__ __launch_bounds__(256) void k_rows_nnz(const float* __restrict__ rows, int64_t P, int64_t stride,
                                                  int64_t chunk, int* __restrict__ part, int nblk) {
  __shared__ int red[4];
  const int r = blockIdx.y;
  const float* row = rows + (int64_t)r * stride;
  const int64_t s = (int64_t)blockIdx.x * chunk;
  const int64_t e = s + chunk < P ? s + chunk : P;
  int cnt = 0;
  const int64_t e4 = s + ((e - s) & ~int64_t(3));
  for (int64_t i = s + 4 * threadIdx.x; i < e4; i += 4 * 256) {
    const float4 v = *reinterpret_cast<const float4*>(row + i);
    cnt += (v.x != 0.f) + (v.y != 0.f) + (v.z != 0.f) + (v.w != 0.f);
  }
  for (int64_t i = e4 + threadIdx.x; i < e; i += 256) cnt += row[i] != 0.f;
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_down(cnt, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) part[(int64_t)r * nblk + blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

int64_t rows_nnz_blocks(int64_t P) {
  int nb;
  opt_chunk(P, &nb);
  return nb;
}

void rows_nnz(uintptr_t rows, int64_t R, int64_t P, int64_t stride, uintptr_t part, uintptr_t stream) {
  NIDT_REQUIRE(stride % 4 == 0 && (rows & 15) == 0, "rows_nnz: 16-byte aligned rows");
  if (R == 0 || P == 0) return;
  int nblk;
  const int64_t chunk = opt_chunk(P, &nblk);
  hipLaunchKernelGGL(k_rows_nnz, dim3(nblk, (unsigned)R), dim3(256), 0, as_stream(stream), ptr<const float>(rows), P,
                     stride, chunk, ptr<int>(part), nblk);
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

// ---- masked rows: dst[c][i] = (src ? src[i] : dst[c][i]) * bit(c, i) ----
// (SubAvg's per-client evaluation models w_global * mask_c, the real_prune of the trained rows, DisPFL's masked start
// rows).  The torch form (unpack the bit rows to an int64 [C, 32 W] tensor, then to floats, then multiply) moved ~30 GB
// for 100 CIFAR ResNet-18 rows (13.5 ms per SubAvg evaluation); this reads the bits once and writes the rows once.
// Thread = one 32-bit mask word (32 elements, 8 x 16-B accesses on the 4-aligned body); bits rows at stride mstride
// words (0: one mask shared by every row).
__global__ __launch_bounds__(256) void k_masked_rows(const float* __restrict__ src, const uint32_t* __restrict__ bits,
                                                     int64_t mstride, int64_t P, int64_t ld, float* __restrict__ dst) {
  const int c = blockIdx.y;
  const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, i0 = 32 * w;
  if (i0 >= P) return;
  const uint32_t b = bits[(int64_t)c * mstride + w];
  float* d = dst + (int64_t)c * ld;
  if (i0 + 32 <= P) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t i = i0 + 4 * j;
      float4 v = src ? *reinterpret_cast<const float4*>(src + i) : *reinterpret_cast<const float4*>(d + i);
      v.x = (b >> (4 * j)) & 1u ? v.x : 0.f;
      v.y = (b >> (4 * j + 1)) & 1u ? v.y : 0.f;
      v.z = (b >> (4 * j + 2)) & 1u ? v.z : 0.f;
      v.w = (b >> (4 * j + 3)) & 1u ? v.w : 0.f;
      *reinterpret_cast<float4*>(d + i) = v;
    }
    return;
  }
  for (int64_t i = i0; i < P; ++i) {
    const float v = src ? src[i] : d[i];
    d[i] = (b >> (i - i0)) & 1u ? v : 0.f;
  }
}

// ---- bit rows -> [R, P] 0/1 rows (uint8 for bool, or fp32): 4 elements per thread (one nibble of a mask word),
// consecutive threads on consecutive elements: 4-B / 16-B coalesced stores ----
template <bool F32>
__global__ __launch_bounds__(256) void k_unpack_bits(const uint32_t* __restrict__ bits, int64_t mstride, int64_t P,
                                                     void* __restrict__ out) {
  const int r = blockIdx.y;
  const int64_t i = 4 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= P) return;
  const uint32_t nib = (bits[(int64_t)r * mstride + (i >> 5)] >> (i & 31)) & 0xfu;
  if (F32) {
    float* o = reinterpret_cast<float*>(out) + (int64_t)r * P + i;
    const float v[4] = {(float)(nib & 1u), (float)((nib >> 1) & 1u), (float)((nib >> 2) & 1u), (float)(nib >> 3)};
    if (i + 3 < P && (P & 3) == 0) {
      *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
    } else {
      for (int j = 0; j < 4 && i + j < P; ++j) o[j] = v[j];
    }
  } else {
    uint8_t* o = reinterpret_cast<uint8_t*>(out) + (int64_t)r * P + i;
    if (i + 3 < P && (P & 3) == 0) {
      *reinterpret_cast<uint32_t*>(o) = (nib & 1u) | (((nib >> 1) & 1u) << 8) | (((nib >> 2) & 1u) << 16) | ((nib >> 3) << 24);
    } else {
      for (int j = 0; j < 4 && i + j < P; ++j) o[j] = (uint8_t)((nib >> j) & 1u);
    }
  }
}

void unpack_bits_dev(uintptr_t bits, int64_t mstride, int64_t R, int64_t P, int f32, uintptr_t out, uintptr_t stream) {
  NIDT_REQUIRE(bits != 0 && out != 0 && R > 0 && P > 0 && (out & 15) == 0, "unpack_bits_dev: arguments");
  const dim3 grid((unsigned)ceil_div((P + 3) / 4, 256), (unsigned)R);
  if (f32)
    hipLaunchKernelGGL(k_unpack_bits<true>, grid, dim3(256), 0, as_stream(stream), ptr<const uint32_t>(bits), mstride, P,
                       ptr<void>(out));
  else
    hipLaunchKernelGGL(k_unpack_bits<false>, grid, dim3(256), 0, as_stream(stream), ptr<const uint32_t>(bits), mstride,
                       P, ptr<void>(out));
  NIDT_CHECK(hipGetLastError());
}

void masked_rows(uintptr_t src, uintptr_t bits, int64_t mstride, int64_t C, int64_t P, int64_t ld, uintptr_t dst,
                 uintptr_t stream) {
  NIDT_REQUIRE(ld % 4 == 0 && (dst & 15) == 0 && (src & 15) == 0 && bits != 0 && C > 0 && P > 0 && ld >= P,
               "masked_rows: 16-B aligned rows (ld % 4 == 0), bits");
  const int64_t nw = (P + 31) / 32;
  hipLaunchKernelGGL(k_masked_rows, dim3((unsigned)ceil_div(nw, 256), (unsigned)C), dim3(256), 0, as_stream(stream),
                     ptr<const float>(src), ptr<const uint32_t>(bits), mstride, P, ld, ptr<float>(dst));
  NIDT_CHECK(hipGetLastError());
}

void broadcast_row(uintptr_t src, int64_t P, int64_t stride, int64_t C, uintptr_t dst, uintptr_t stream) {
  NIDT_REQUIRE(stride % 4 == 0 && (src & 15) == 0 && (dst & 15) == 0, "alignment");
  const int64_t n4 = (P + 3) / 4;
  hipLaunchKernelGGL(k_broadcast_row, dim3(ceil_div(n4, 256)), dim3(256), 0, as_stream(stream), ptr<const float>(src), P,
                     stride, (int)C, ptr<float>(dst));
  NIDT_CHECK(hipGetLastError());
}

}  // namespace nidt
