// Client-grouped 3x3x3 stride-1 Conv3d on gfx950 MFMA (bf16 in, fp32 accumulate), channels-last.
//
// Serves AlexNet3D conv2..conv5 (reference fedml_api/model/cv/salient_models.py:152-165) for G
// virtual clients at once: activations are [G*B, D, H, W, C] (client-major), weights [G, Cout, 27, Cin]
// (one weight set per client).  Three kernels:
//
//  * k_conv_fwd  — implicit GEMM  C[co][pos] = sum_k W[co][k] * patch[pos][k]  (k = tap*Cin + ci).
//                  A = weights (rows co), B = im2col patches (cols = output positions), both staged through
//                  LDS as [row][32 k] with an XOR swizzle that makes the ds_read_b128 fragment reads
//                  bank-conflict free; register-staged double buffer (one barrier per 32-deep k-step).
//                  Optional fused input transform relu(x*s+t) (= the previous layer's BatchNorm+ReLU,
//                  so BN3/BN4 outputs are never materialised), bias add, bf16 store, and per-block BN
//                  statistics (block mean + M2 per channel, merged later with Chan's formula).
//                  Also used for dgrad: dX = conv(dY, flip(W)^T) with pad' = 2 - pad.
//  * k_conv_wgrad — dW[co][k] = sum_pos dY[pos][co] * patch[pos][k]: both operands are stored
//                  [pos][channel] in LDS and read with the gfx950 transposing ds_read_b64_tr_b16, so the
//                  reduction (position) axis lands in the MFMA k slots without any shuffles.  Split over
//                  positions into fp32 slabs; k_wgrad_reduce sums slabs and writes the PyTorch
//                  [Cout][Cin][3][3][3] layout straight into the flat per-client gradient rows.
//  * k_pack_conv_w — fp32 flat master weights -> bf16 [G][Cout][27][Cin] (+ flipped/transposed copy
//                  for dgrad), scaled by an optional factor.
#include <cmath>
#include <array>
#include <cstdlib>
#include <map>
#include <type_traits>

#include <vector>

#include "common.h"
#include "dma.h"

namespace nidt {

// ------------------------------------------------------------------------------------------------
struct ConvFwdArgs {
  const uint16_t* x;    // [G*B, D, H, W, Cin] bf16
  const uint16_t* w;    // [G, Cout, 27, Cin] bf16
  const float* bias;    // [G, Cout] or null
  const float* xs;      // [G, Cin] input scale (transform) or null
  const float* xt;      // [G, Cin] input shift
  uint16_t* y;          // [G*B, Do, Ho, Wo, Cout] bf16
  float* stats;         // [G, nPB, Cout, 2] or null
  int B, D, H, W, Cin, Do, Ho, Wo, Cout, pad;
  int Mg;               // output positions per client
  int nPB;              // position blocks per client (grid.x)
  int ksplit = 1;       // split-K factor (LDS-DMA path): > 1 writes fp32 partials, k_fwd_splitk_fin finishes
  int G = 0;            // clients (split-K partial indexing)
  int64_t bias_ld = 0;  // bias row stride per client (0 = Cout; the flat parameter row stride to read theta directly)
  float* part = nullptr;  // [ksplit, G, Mg, Cout] fp32 partial sums
  // geometry (LDS-DMA path): kt taps per output (27 = 3x3x3, 9 = 1x3x3 (2-D convs as D = 1 volumes), 1 = 1x1x1),
  // stride st in every dimension, depth padding padd (the h/w padding is pad)
  int kt = 27, st = 1, padd = 0;
  // sub-pixel (phase) data gradient of a stride-2 conv (LDS-DMA path, conv_dgrad_s2_g): nph > 0 phases, each a
  // stride-1 conv over the dy grid with pnt[ph] taps — window taps ptap[pt0[ph] + j] (geometry and padding mask),
  // weights at tap slots pt0[ph] + j of w [Cout][kt][Cin] — whose output (od, oh, ow) lands at (2od + bit2(poff),
  // 2oh + bit1(poff), 2ow + bit0(poff)) of the [Dx][Hx][Wx] output (positions outside are skipped)
  int nph = 0, Dx = 0, Hx = 0, Wx = 0;
  unsigned char pnt[8] = {0}, pt0[8] = {0}, poff[8] = {0}, ptap[28] = {0};
  int kd1 = 0;          // k_conv_fwd_slab: depth tap kd = 1 only (2-D maps batched along depth, conv2d_fwd_slab_bd)
  int dbg = 0;          // timing diagnostics only (NIDT_SLAB_DBG): 1 = k_conv_fwd_slab keeps its first union
};

constexpr int kFwdBP = 128;  // positions per block
constexpr int kMaxCin = 512; // LDS-DMA paths (Cin % 64 == 0); the register-staged / transform paths keep 192
constexpr int kBK = 32;      // k per step

__device__ __forceinline__ int swz_fwd(int r) { return ((r >> 3) & 1) * 3; }

__device__ __forceinline__ uint4 xform8(uint4 v, const float* s, const float* t, bool valid) {
  if (!valid) return make_uint4(0, 0, 0, 0);
  uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float lo = __uint_as_float(u[j] << 16), hi = __uint_as_float(u[j] & 0xffff0000u);
    lo = fmaxf(fmaf(lo, s[2 * j], t[2 * j]), 0.f);
    hi = fmaxf(fmaf(hi, s[2 * j + 1], t[2 * j + 1]), 0.f);
    u[j] = pack_bf16x2(lo, hi);
  }
  return make_uint4(u[0], u[1], u[2], u[3]);
}

// [DPP-SUM] sum over the 16 lanes of a DPP row, every lane getting the same total: quad swaps (lane ^ 1, lane ^ 2),
// then the half-row and row mirrors — four v_add_f32 with a DPP source operand instead of four __shfl_xor
// (ds_bpermute_b32: an LDS-pipeline round trip each; profiles/r6_dpp_stats.txt).
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float row_sum16(float s) {
  s += dpp_f32<0xB1>(s);   // quad_perm [1, 0, 3, 2]
  s += dpp_f32<0x4E>(s);   // quad_perm [2, 3, 0, 1]
  s += dpp_f32<0x141>(s);  // row_half_mirror: lane i <- 7 - i within each 8
  s += dpp_f32<0x140>(s);  // row_mirror: lane i <- 15 - i
  return s;
}

// Shared epilogue of the forward kernels: bias, bf16 store, per-block BN statistics (block mean + M2 per
// channel).  C layout (16x16x32): C[row = 4*fq + r][col = fr]; rows = co, cols = positions.
template <int BCO, int BP, int WM, int WN, bool BIAS, bool STATS, int TCO, int TP>
__device__ __forceinline__ void conv_fwd_epilogue(const ConvFwdArgs& a, f32x4 (&acc)[TCO][TP], float* red, int g,
                                                  int pb, int co0, int wco, int wp, int fr, int fq, int tid,
                                                  int ph = 0, int mb = -1, int me = -1) {
  // block positions [mb, me) of the client (default: [pb BP, min(pb BP + BP, Mg)), the fixed-size blocks)
  constexpr int WCO = BCO / WM, WP = BP / WN;
  if (mb < 0) {
    mb = pb * BP;
    me = a.Mg;
  }
  float bias_r[TCO][4];
#pragma unroll
  for (int i = 0; i < TCO; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      bias_r[i][r] = BIAS ? a.bias[(int64_t)g * (a.bias_ld ? a.bias_ld : a.Cout) + co0 + wco * WCO + i * 16 + 4 * fq + r]
                          : 0.f;
  const int posw = mb + wp * WP + fr;
#pragma unroll
  for (int j = 0; j < TP; ++j) {
    const int m = posw + j * 16;
    if (m < me) {
      int64_t yo = (int64_t)g * a.Mg + m;
      if (a.nph) {  // phase output: scatter to the strided positions of the full-resolution gradient
        const int S = a.Do * a.Ho * a.Wo, nl = m / S, sr = m - nl * S;
        const int od = sr / (a.Ho * a.Wo), r2 = sr - od * a.Ho * a.Wo, oh = r2 / a.Wo, ow = r2 - oh * a.Wo;
        const int po = a.poff[ph];
        const int zd = a.Dx > 1 ? 2 * od + ((po >> 2) & 1) : od, zh = 2 * oh + ((po >> 1) & 1), zw = 2 * ow + (po & 1);
        if (zd >= a.Dx || zh >= a.Hx || zw >= a.Wx) continue;
        yo = (((int64_t)g * a.B + nl) * a.Dx + zd) * a.Hx * a.Wx + (int64_t)zh * a.Wx + zw;
      }
      uint16_t* yp = a.y + yo * a.Cout + co0 + wco * WCO + 4 * fq;
#pragma unroll
      for (int i = 0; i < TCO; ++i) {
        float v0 = acc[i][j][0] + bias_r[i][0], v1 = acc[i][j][1] + bias_r[i][1];
        float v2 = acc[i][j][2] + bias_r[i][2], v3 = acc[i][j][3] + bias_r[i][3];
        uint2 o = make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2, v3));
        *reinterpret_cast<uint2*>(yp + i * 16) = o;
      }
    }
  }
  if (STATS) {
    // [WSTATS] each wave's (mean, M2) per channel over its own WP positions (one pass, DPP only: the wave mean
    // needs no block-wide round), then ONE LDS round: the WN wave partials merged per channel (Chan: mean = count-
    // weighted mean of the wave means, M2 = sum M2 + sum cnt (wave mean - mean)^2).  Two barriers instead of four.
    // red: [WN (wp)][BCO][2] floats of LDS scratch
    const int cntw = max(0, min(WP, me - (mb + wp * WP)));  // valid positions of this wave (uniform)
    float m_[TCO][4], q_[TCO][4];
#pragma unroll
    for (int i = 0; i < TCO; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // [ONEPASS] sum and sum of squares in one sweep, shifted by one sample of the channel (the row's lane 0,
        // first position: row_newbcast:0 hands it to the 16 reduced lanes; valid whenever cntw > 0), so q - s^2/n
        // cancels only at the channel's spread, not its mean (exact shifted-data variance; the bias only moves the
        // mean).  The two DPP chains are independent and interleave.
        const float k0 = __int_as_float(
            __builtin_amdgcn_update_dpp(0, __float_as_int(acc[i][0][r]), 0x150, 0xf, 0xf, false));
        float s = 0.f, q = 0.f;
#pragma unroll
        for (int j = 0; j < TP; ++j)
          if (posw + j * 16 < me) {
            const float v = acc[i][j][r] - k0;
            s += v;
            q = fmaf(v, v, q);
          }
        s = row_sum16(s);
        q = row_sum16(q);
        const float dw = cntw > 0 ? s / (float)cntw : 0.f;
        m_[i][r] = (cntw > 0 ? k0 + dw : 0.f) + bias_r[i][r];
        q_[i][r] = fmaxf(q - s * dw, 0.f);
      }
    __syncthreads();  // red aliases the operand staging
    if (fr == 0) {
#pragma unroll
      for (int i = 0; i < TCO; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float* e = red + 2 * (wp * BCO + wco * WCO + i * 16 + 4 * fq + r);
          e[0] = m_[i][r];
          e[1] = q_[i][r];
        }
    }
    __syncthreads();
    for (int c = tid; c < BCO; c += (int)blockDim.x) {
      float n = 0.f, sm = 0.f;
#pragma unroll
      for (int w = 0; w < WN; ++w) {
        const float cw = (float)max(0, min(WP, me - (mb + w * WP)));
        n += cw;
        sm = fmaf(cw, red[2 * (w * BCO + c)], sm);
      }
      const float mean = n > 0.f ? sm / n : 0.f;
      float m2 = 0.f;
#pragma unroll
      for (int w = 0; w < WN; ++w) {
        const float cw = (float)max(0, min(WP, me - (mb + w * WP)));
        const float d = red[2 * (w * BCO + c)] - mean;
        m2 += red[2 * (w * BCO + c) + 1] + cw * d * d;
      }
      float* st = a.stats + (((int64_t)g * a.nPB + pb) * a.Cout + co0 + c) * 2;
      st[0] = mean;
      st[1] = m2;
    }
  }
}

template <int BCO, bool XF, bool BIAS, bool STATS>
__global__ __launch_bounds__(256, 2) void k_conv_fwd(ConvFwdArgs a) {
  constexpr int BP = kFwdBP;
  constexpr int WCO = BCO / 2, WP = BP / 2;
  constexpr int TCO = WCO / 16, TP = WP / 16;
  constexpr int A_CHUNKS = BCO * 4 / 256;  // 16-B chunks of the A tile per thread (2 or 1)
  __shared__ __attribute__((aligned(16))) uint16_t sA[2][BCO * kBK];
  __shared__ __attribute__((aligned(16))) uint16_t sB[2][BP * kBK];
  __shared__ float sXS[XF ? 192 : 1], sXT[XF ? 192 : 1];

  const int g = blockIdx.z, pb = blockIdx.x, co0 = blockIdx.y * BCO;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wco = wid >> 1, wp = wid & 1;
  const int Cin = a.Cin, nck = Cin / kBK, nks = 27 * nck;
  if (XF) {
    for (int i = tid; i < Cin; i += 256) {
      sXS[i] = a.xs[(int64_t)g * Cin + i];
      sXT[i] = a.xt[(int64_t)g * Cin + i];
    }
  }
  // ---- B-tile rows owned by this thread (fixed over the k loop) ----
  const int q = tid & 3;
  int bn[2], bd[2], bh[2], bw[2];
  bool bv[2];
  const int S = a.Do * a.Ho * a.Wo;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = pb * BP + (tid >> 2) + 64 * i;
    bv[i] = m < a.Mg;
    const int mm = bv[i] ? m : 0;
    const int nl = mm / S, s = mm - nl * S;
    bn[i] = g * a.B + nl;
    bd[i] = s / (a.Ho * a.Wo);
    const int r = s - bd[i] * a.Ho * a.Wo;
    bh[i] = r / a.Wo;
    bw[i] = r - bh[i] * a.Wo;
  }
  uint4 rA0, rA1, rB0, rB1;
  const float* sxs = sXS;
  const float* sxt = sXT;
#define CONV_LOAD_B(I, DST, KD, KH, KW, C)                                                                      \
  {                                                                                                             \
    const int id = bd[I] + (KD) - a.pad, ih = bh[I] + (KH) - a.pad, iw = bw[I] + (KW) - a.pad;                  \
    const bool ok = bv[I] && id >= 0 && id < a.D && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;                 \
    uint4 v = make_uint4(0, 0, 0, 0);                                                                           \
    if (ok) v = *reinterpret_cast<const uint4*>(a.x + ((((int64_t)bn[I] * a.D + id) * a.H + ih) * a.W + iw) * Cin + (C)); \
    if (XF) v = xform8(v, sxs + (C), sxt + (C), ok);                                                            \
    DST = v;                                                                                                    \
  }
#define CONV_LOAD(KS)                                                                                           \
  {                                                                                                             \
    const int t_ = (KS) / nck, cc_ = (KS) - t_ * nck;                                                           \
    const int kd_ = t_ / 9, kh_ = (t_ / 3) % 3, kw_ = t_ % 3;                                                   \
    const int c_ = cc_ * kBK + q * 8;                                                                           \
    CONV_LOAD_B(0, rB0, kd_, kh_, kw_, c_)                                                                      \
    CONV_LOAD_B(1, rB1, kd_, kh_, kw_, c_)                                                                      \
    rA0 = *reinterpret_cast<const uint4*>(a.w + (((int64_t)g * a.Cout + co0 + (tid >> 2)) * 27 + t_) * Cin + c_); \
    if (A_CHUNKS > 1)                                                                                           \
      rA1 = *reinterpret_cast<const uint4*>(a.w + (((int64_t)g * a.Cout + co0 + (tid >> 2) + 64) * 27 + t_) * Cin + c_); \
  }
#define CONV_STORE(BUF)                                                                                         \
  {                                                                                                             \
    const int r0_ = tid >> 2, r1_ = r0_ + 64;                                                                   \
    *reinterpret_cast<uint4*>(&sB[BUF][r0_ * kBK + ((q ^ swz_fwd(r0_)) << 3)]) = rB0;                           \
    *reinterpret_cast<uint4*>(&sB[BUF][r1_ * kBK + ((q ^ swz_fwd(r1_)) << 3)]) = rB1;                           \
    *reinterpret_cast<uint4*>(&sA[BUF][r0_ * kBK + ((q ^ swz_fwd(r0_)) << 3)]) = rA0;                           \
    if (A_CHUNKS > 1) *reinterpret_cast<uint4*>(&sA[BUF][r1_ * kBK + ((q ^ swz_fwd(r1_)) << 3)]) = rA1;         \
  }

  f32x4 acc[TCO][TP];
#pragma unroll
  for (int i = 0; i < TCO; ++i)
#pragma unroll
    for (int j = 0; j < TP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (XF) __syncthreads();
  CONV_LOAD(0)
  CONV_STORE(0)
  __syncthreads();
  const int fr = lane & 15, fq = lane >> 4;
  const int fchunk = (fq ^ swz_fwd(fr)) << 3;
  for (int ks = 0; ks < nks; ++ks) {
    const int cur = ks & 1;
    const bool more = ks + 1 < nks;
    if (more) CONV_LOAD(ks + 1)
    bf16x8 fa[TCO], fb[TP];
#pragma unroll
    for (int i = 0; i < TCO; ++i)
      fa[i] = *reinterpret_cast<const bf16x8*>(&sA[cur][(wco * WCO + i * 16 + fr) * kBK + fchunk]);
#pragma unroll
    for (int j = 0; j < TP; ++j)
      fb[j] = *reinterpret_cast<const bf16x8*>(&sB[cur][(wp * WP + j * 16 + fr) * kBK + fchunk]);
#pragma unroll
    for (int i = 0; i < TCO; ++i)
#pragma unroll
      for (int j = 0; j < TP; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    if (more) CONV_STORE(cur ^ 1)
    __syncthreads();
  }
#undef CONV_LOAD_B
#undef CONV_LOAD
#undef CONV_STORE

  conv_fwd_epilogue<BCO, BP, 2, 2, BIAS, STATS, TCO, TP>(a, acc, reinterpret_cast<float*>(&sB[0][0]), g, pb, co0,
                                                         wco, wp, fr, fq, tid);
}

// ------------------------------------------------------------------------------------------------
// k_conv_fwd_dma — the Cin % 64 == 0 forward/dgrad path: BK = 64 (one tap x 64 channels per k-step, a
// 128-B row per position / output channel), both tiles filled by buffer_load ... lds (LDS-DMA, no staging
// VGPRs, no ds_write).  The LDS image is lane-linear per wave instruction, so the bank swizzle
// chunk' = chunk ^ ((row >> 1) & 7) is applied to the per-lane SOURCE offset and undone on the
// ds_read_b128 fragment reads (conflict-free for the 16x16x32 fragment pattern: each 16-lane group of a
// b128 read touches 16 distinct 16-B bank slots).  Out-of-range taps (padding) and positions past the
// end read past the buffer range and get zeros.  Per-row tap validity is a 27-bit mask computed once per
// block, so the k-loop's address work is one 32-bit add + select per 16-B chunk.  1-D grid with the XCD
// remap: the co-tiles of one position tile and neighbouring position tiles share an XCD's L2 (the 27
// taps re-read the same input rows).
__device__ __forceinline__ int swz_dma(int r) { return (r >> 1) & 7; }

// [SCHED] one 64-deep k-step (two 32-deep MFMA halves) of a wave's TCO x TP fragment tile with every fragment in its
// own registers: the second half's LDS reads issue between the first half's MFMAs, so the wave waits on LDS about
// once per k-step.  The compiler's own schedule of the same loop re-reads each weight fragment into one register set
// (an LDS round trip per TP MFMAs), which two waves per SIMD cannot cover.  fa_at(kk, i) / fb_at(kk, j) read the
// fragments with RPF LDS read instructions each (2 for the transposed-read pairs of the weight-gradient kernels).  The
// closing sched_barrier keeps the MFMAs ahead of the caller's wait + barrier: hoisted above it, they would leave the
// next k-step's tile loads only a few MFMAs to land in.
template <int TCO, int TP, int RPF = 1, class FA, class FB>
__device__ __forceinline__ void kstep_sched(f32x4 (&acc)[TCO][TP], FA fa_at, FB fb_at) {
  bf16x8 fa[2][TCO], fb[2][TP];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
    for (int i = 0; i < TCO; ++i) fa[kk][i] = fa_at(kk, i);
#pragma unroll
    for (int j = 0; j < TP; ++j) fb[kk][j] = fb_at(kk, j);
  }
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int i = 0; i < TCO; ++i)
#pragma unroll
      for (int j = 0; j < TP; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[kk][i], fb[kk][j], acc[i][j], 0, 0, 0);
  __builtin_amdgcn_sched_group_barrier(0x100, RPF * (TCO + TP), 0);  // DS_READ: first half's fragments
#pragma unroll
  for (int x = 0; x < TCO + TP; ++x) {
    __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);      // MFMA
    __builtin_amdgcn_sched_group_barrier(0x100, RPF, 0);  // DS_READ of the second half
  }
  __builtin_amdgcn_sched_group_barrier(0x8, 2 * TCO * TP - (TCO + TP), 0);
  __builtin_amdgcn_sched_barrier(0);
}

// [SCHED-half] the register-lean form for blocks at four waves per SIMD (<= 128 VGPRs): one 32-deep half's
// fragments at a time, all of its reads ahead of its MFMAs
template <int TCO, int TP, class FA, class FB>
__device__ __forceinline__ void kstep_sched_half(f32x4 (&acc)[TCO][TP], FA fa_at, FB fb_at) {
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    bf16x8 fa[TCO], fb[TP];
#pragma unroll
    for (int i = 0; i < TCO; ++i) fa[i] = fa_at(kk, i);
#pragma unroll
    for (int j = 0; j < TP; ++j) fb[j] = fb_at(kk, j);
#pragma unroll
    for (int i = 0; i < TCO; ++i)
#pragma unroll
      for (int j = 0; j < TP; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, TCO + TP, 0);
    __builtin_amdgcn_sched_group_barrier(0x8, TCO * TP, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
}

// [SCHED] on the forward blocks (dma_sched: NIDT_DMA_SCHED)
template <int BCO, int WM, int WN, int NST, bool BIAS, bool STATS, int SCHED = 0>
__global__ __launch_bounds__(64 * WM * WN, ((NST == 2 ? 8 : 4) / (WM * WN)) > 0 ? (NST == 2 ? 8 : 4) / (WM * WN) : 1) void k_conv_fwd_dma(ConvFwdArgs a, int nCO) {
  // waves: WM (co) x WN (positions); each wave owns (BCO/WM) co x 64 positions
  constexpr int NW = WM * WN, BP = 64 * WN, BK = 64;
  constexpr int WCO = BCO / WM, WP = 64;
  constexpr int TCO = WCO / 16, TP = WP / 16;
  constexpr int A_ELEMS = BCO * BK, B_ELEMS = BP * BK, BUF = A_ELEMS + B_ELEMS;
  constexpr int A_INSTR = BCO / (8 * NW);  // 1-KB glds wave-instructions per wave for the A tile
  constexpr int B_INSTR = BP / (8 * NW);   // ... and for the B tile (8 rows each)
  constexpr int NI = A_INSTR + B_INSTR;    // glds per wave per stage (the vmcnt unit)
  // NST LDS stages: NST-1 tiles in flight while one is consumed.  With NST = 3 the loads of two k-steps
  // stay in flight across the barrier (counted vmcnt + raw s_barrier; a __syncthreads() would drain them).
  __shared__ __attribute__((aligned(16))) uint16_t smem[NST * BUF];

  const int nwg = gridDim.x;
  const int id = xcd_remap(blockIdx.x, nwg);
  const int cot = id % nCO, rest = id / nCO;
  const int pb = rest % a.nPB, rest2 = rest / a.nPB;
  const int nph = a.nph > 0 ? a.nph : 1;
  const int sp = rest2 % a.ksplit, gp = rest2 / a.ksplit;
  const int ph = gp % nph, g = gp / nph;
  const int ntap = a.nph ? (int)a.pnt[ph] : a.kt, tbase = a.nph ? (int)a.pt0[ph] : 0;
  const int co0 = cot * BCO;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: LDS destinations stay in SGPRs
  const int wco = wid / WN, wp = wid % WN;
  const int Cin = a.Cin, nck = Cin / BK, nks = ntap * nck;
  int ks0 = nks * sp / a.ksplit, ks1 = nks * (sp + 1) / a.ksplit;  // this split's k-steps
  const int lrow = lane >> 3, slot = lane & 7;
  const int S = a.Do * a.Ho * a.Wo;
  if (a.kt == 27 && !a.nph && a.padd > 0) {
    // depth taps kd that read only padding for EVERY position of this block are skipped (their B rows are all
    // zeros): the conv2 data gradient (pad 2 over 17 dy planes) spends 27 % of its MACs on padding, and blocks
    // inside the border output planes need only 1 or 2 of the 3 kd.  Positions of one sample only; a block that
    // spans two samples keeps every kd.  The result is bitwise unchanged (only zero products are dropped).
    const int m_lo = pb * BP, m_hi = min(m_lo + BP, a.Mg) - 1;
    int od_lo = 0, od_hi = a.Do - 1;
    if (m_lo / S == m_hi / S) {
      od_lo = (m_lo % S) / (a.Ho * a.Wo);
      od_hi = (m_hi % S) / (a.Ho * a.Wo);
    }
    const int kd_lo = max(0, a.padd - od_hi * a.st), kd_hi = min(2, a.D - 1 + a.padd - od_lo * a.st);
    ks0 = max(ks0, 9 * kd_lo * nck);
    ks1 = min(ks1, 9 * (kd_hi + 1) * nck);
  }

  // ---- per-thread B rows: one per LDS-DMA instruction, fixed over the k loop (byte offsets in the client's input;
  // rows past the end and padding taps read out of range -> zeros) ----
  int roff[B_INSTR];
  uint32_t tmask[B_INSTR];
#pragma unroll
  for (int i = 0; i < B_INSTR; ++i) {
    const int row = 8 * (B_INSTR * wid + i) + lrow;
    const int m = pb * BP + row;
    tmask[i] = 0u;
    roff[i] = 0;
    if (m < a.Mg) {
      const int nl = m / S, s = m - nl * S;
      const int od = s / (a.Ho * a.Wo), r2 = s - od * a.Ho * a.Wo;
      const int oh = r2 / a.Wo, ow = r2 - oh * a.Wo;
      const int d0 = od * a.st - a.padd, h0 = oh * a.st - a.pad, w0 = ow * a.st - a.pad;
      // may be negative for padded windows; only taps inside the volume (tmask) are ever read
      roff[i] = ((((nl * a.D + d0) * a.H + h0) * a.W + w0) * Cin + ((slot ^ swz_dma(row)) << 3)) * 2;
      tmask[i] = tap_mask3(d0, h0, w0, a.D, a.H, a.W);
    }
  }
  int aoff[A_INSTR];
#pragma unroll
  for (int i = 0; i < A_INSTR; ++i) {
    const int row = 8 * (wid * A_INSTR + i) + lrow;
    aoff[i] = ((co0 + row) * a.kt * Cin + ((slot ^ swz_dma(row)) << 3)) * 2;
  }
  const int64_t xcl = (int64_t)a.B * a.D * a.H * a.W * Cin;
  const i32x4_t rxs = make_rsrc(a.x + (int64_t)g * xcl, (uint32_t)(xcl * 2));
  const i32x4_t rws = make_rsrc(a.w + (int64_t)g * a.Cout * a.kt * Cin, (uint32_t)(a.Cout * a.kt * Cin * 2));

#define DMA_ISSUE(KS, BUFI)                                                                                   \
  {                                                                                                           \
    const int l_ = (KS) / nck, cc_ = (KS) - l_ * nck;                                                         \
    const int t_ = a.nph ? (int)a.ptap[tbase + l_] : l_;  /* window tap: geometry + padding mask */           \
    const int toff_ = (((((t_ / 9)) * a.H + (t_ / 3) % 3) * a.W + t_ % 3) * Cin + cc_ * BK) * 2;              \
    const int woff_ = ((tbase + l_) * Cin + cc_ * BK) * 2;  /* weight tap slot */                             \
    uint16_t* sA_ = smem + (BUFI) * BUF;                                                                      \
    uint16_t* sB_ = sA_ + A_ELEMS;                                                                            \
    _Pragma("unroll") for (int i_ = 0; i_ < A_INSTR; ++i_)                                                    \
      blds16(rws, aoff[i_] + woff_, sA_ + (wid * A_INSTR + i_) * 512);                                        \
    _Pragma("unroll") for (int i_ = 0; i_ < B_INSTR; ++i_)                                                    \
      blds16(rxs, ((tmask[i_] >> t_) & 1u) ? roff[i_] + toff_ : kBufOOB, sB_ + (B_INSTR * wid + i_) * 512);   \
  }

  f32x4 acc[TCO][TP];
#pragma unroll
  for (int i = 0; i < TCO; ++i)
#pragma unroll
    for (int j = 0; j < TP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  if (ks0 < ks1) {  // block-uniform; empty only for a split-K slice outside the block's live kd range
  // prologue: stages 0 .. NST-2 in flight, wait for stage 0 only
  DMA_ISSUE(ks0, 0)
#pragma unroll
  for (int s_ = 1; s_ < NST - 1; ++s_)
    if (ks0 + s_ < ks1) DMA_ISSUE(ks0 + s_, s_)
  {
    const int younger = min(NST - 2, ks1 - ks0 - 1);
    if (younger >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NI) : "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  int cur = 0;
  for (int ks = ks0; ks < ks1; ++ks) {
    if (ks + NST - 1 < ks1) {
      int nb = cur + NST - 1;
      nb = nb >= NST ? nb - NST : nb;
      DMA_ISSUE(ks + NST - 1, nb)
    }
    const uint16_t* sA = smem + cur * BUF;
    const uint16_t* sB = sA + A_ELEMS;
    auto fa_at = [&](int kk, int i) {
      const int r = wco * WCO + i * 16 + fr;
      return *reinterpret_cast<const bf16x8*>(&sA[r * BK + (((4 * kk + fq) ^ swz_dma(r)) << 3)]);
    };
    auto fb_at = [&](int kk, int j) {
      const int r = wp * WP + j * 16 + fr;
      return *reinterpret_cast<const bf16x8*>(&sB[r * BK + (((4 * kk + fq) ^ swz_dma(r)) << 3)]);
    };
    if constexpr (SCHED == 1) {
      kstep_sched<TCO, TP>(acc, fa_at, fb_at);
    } else if constexpr (SCHED == 2) {
      kstep_sched_half<TCO, TP>(acc, fa_at, fb_at);
    } else {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[TCO], fb[TP];
#pragma unroll
      for (int i = 0; i < TCO; ++i) {
        const int r = wco * WCO + i * 16 + fr;
        fa[i] = *reinterpret_cast<const bf16x8*>(&sA[r * BK + (((4 * kk + fq) ^ swz_dma(r)) << 3)]);
      }
#pragma unroll
      for (int j = 0; j < TP; ++j) {
        const int r = wp * WP + j * 16 + fr;
        fb[j] = *reinterpret_cast<const bf16x8*>(&sB[r * BK + (((4 * kk + fq) ^ swz_dma(r)) << 3)]);
      }
#pragma unroll
      for (int i = 0; i < TCO; ++i)
#pragma unroll
        for (int j = 0; j < TP; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    }
    // retire stage ks+1 (this wave's own glds), keep the younger stages in flight, then one barrier so
    // every wave's part of stage ks+1 has landed and every wave is done reading stage ks.
    {
      const int younger = min(NST - 2, ks1 - ks - 2);  // stages issued after ks+1 that may stay in flight
      if (younger >= 2) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(2 * NI) : "memory");
      else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(NI) : "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    cur = cur + 1 == NST ? 0 : cur + 1;
  }
  }
#undef DMA_ISSUE
  if (a.ksplit > 1) {  // raw fp32 partials; bias, bf16 output and statistics come from k_fwd_splitk_fin
    const int posw = pb * BP + wp * WP + fr;
#pragma unroll
    for (int j = 0; j < TP; ++j) {
      const int m = posw + j * 16;
      if (m < a.Mg) {
        float* pp = a.part + (((int64_t)sp * a.G + g) * a.Mg + m) * a.Cout + co0 +
                    wco * WCO + 4 * fq;
#pragma unroll
        for (int i = 0; i < TCO; ++i)
          *reinterpret_cast<float4*>(pp + i * 16) = make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
      }
    }
    return;
  }
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);
  conv_fwd_epilogue<BCO, BP, WM, WN, BIAS, STATS, TCO, TP>(a, acc, red, g, pb, co0, wco, wp, fr, fq, tid, ph);
}

// ------------------------------------------------------------------------------------------------
// k_conv_fwd_tri — 3x3x3 stride-1 forward/dgrad with the B operand staged once per (kd, kh, 64-channel chunk)
// triplet for the three kw taps.  k_conv_fwd_dma fetches a [BP positions][64 channels] B tile per tap; with the
// B fetch removed from its k-loop (diagnostic build) the conv2 dgrad ran 3.79 -> 2.62 ms and conv2 fwd 3.33 ->
// 2.77 ms at 64 clients, so the per-tap B traffic, not the MFMA work, sets their pace.  The rows the three kw taps
// of a band of BP consecutive output positions read form a union of runs of consecutive padded-input rows (288
// for conv2 fwd/dgrad, 360 for the padded 5x7x5 convs, vs 3 x 256); the block stages that union once per triplet
// (single buffer: it is reloaded after the triplet's last tap, while the other block on the CU computes) and
// double-buffers only the per-tap weight tile.  Union table (k_union_table with P = BP): per band the union rows'
// sources and each position's union row; tap kw of position p reads union row idx(p) + kw.  Block numbering,
// statistics blocks and epilogue are those of k_conv_fwd_dma (BP = 256), so the BN buffers are unchanged.
// Chunk swizzle of the union rows: 2 * ((r >> 1) & 3).  The union rows a fragment reads are 16 consecutive rows
// from an arbitrary start (plus 2-row jumps at output-row wraps); swz_dma ((r >> 1) & 7) is conflict-free only for
// starts aligned to 16 (the ds_read_b128 lane groups pair fq 0 / fq 1 lanes whose rows then differ by 2 in one
// aligned quad); an even swizzle can never map a fq-0 chunk and its fq-1 neighbour (c ^ 1) to one slot, and
// (r >> 1) & 3 still separates the 4 same-parity rows of one fq in a group: conflict-free for any start without
// wraps (exhaustive check over starts and wrap positions: 29 % fewer conflicts than swz_dma with wraps).
__device__ __forceinline__ int swz_un(int r) { return ((r >> 1) & 3) << 1; }

template <int BCO, int WM, int WN, int U, bool PADDED, bool BIAS, bool STATS>
__global__ __launch_bounds__(64 * WM * WN, 2) void k_conv_fwd_tri(ConvFwdArgs a, int nCO, const int* __restrict__ utab) {
  constexpr int NW = WM * WN, BP = 64 * WN, BK = 64;
  constexpr int WCO = BCO / WM, WP = 64, TCO = WCO / 16, TP = WP / 16;
  constexpr int A_ELEMS = BCO * BK, ST = 2 * U + BP;
  constexpr int A_INSTR = BCO / (8 * NW);
  constexpr int UP = U / 8, UPW = (UP + NW - 1) / NW;  // union pieces (8 rows) per wave
  static_assert(A_INSTR >= 1 && U % 8 == 0, "tile split");
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * A_ELEMS + U * BK];
  uint16_t* const sAb = smem;
  uint16_t* const sU = smem + 2 * A_ELEMS;

  const int nwg = gridDim.x;
  const int id = xcd_remap(blockIdx.x, nwg);
  const int cot = id % nCO, rest = id / nCO;
  const int pb = rest % a.nPB, g = rest / a.nPB;
  const int co0 = cot * BCO;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wco = wid / WN, wp = wid % WN;
  const int Cin = a.Cin, nck = Cin / BK, ntr = 9 * nck, nks = 3 * ntr;
  const int lrow = lane >> 3, slot = lane & 7;
  const int fr = lane & 15, fq = lane >> 4;
  const int* ent = utab + (int64_t)pb * ST;
  int uoff[UPW], ucode[UPW];
#pragma unroll
  for (int i = 0; i < UPW; ++i) {
    const int u = 8 * (wid * UPW + i) + lrow;
    uoff[i] = 0;
    ucode[i] = 1023;
    if (wid * UPW + i < UP) {
      uoff[i] = ent[2 * u] * (Cin * 2) + ((slot ^ swz_un(u)) << 4);
      ucode[i] = ent[2 * u + 1];
    }
  }
  int hrow[TP];
#pragma unroll
  for (int j = 0; j < TP; ++j) hrow[j] = ent[2 * U + wp * WP + j * 16 + fr];
  int aoff[A_INSTR];
#pragma unroll
  for (int i = 0; i < A_INSTR; ++i) {
    const int row = 8 * (wid * A_INSTR + i) + lrow;
    aoff[i] = ((co0 + row) * 27 * Cin + ((slot ^ swz_dma(row)) << 3)) * 2;
  }
  const int64_t xcl = (int64_t)a.B * a.D * a.H * a.W * Cin;
  const i32x4_t rxs = make_rsrc(a.x + (int64_t)g * xcl, (uint32_t)(xcl * 2));
  const i32x4_t rws = make_rsrc(a.w + (int64_t)g * a.Cout * 27 * Cin, (uint32_t)(a.Cout * 27 * Cin * 2));

  auto issue_a = [&](int ks, int buf) {  // weight tile of tap kw of triplet q = ks / 3
    const int q = ks / 3, kw = ks - 3 * q, trip = q / nck, cc = q - trip * nck;
    const int woff = ((trip * 3 + kw) * Cin + cc * BK) * 2;  // tap = kd*9 + kh*3 + kw = trip*3 + kw
    uint16_t* sA = sAb + buf * A_ELEMS;
#pragma unroll
    for (int i = 0; i < A_INSTR; ++i) blds16(rws, aoff[i] + woff, sA + (wid * A_INSTR + i) * 512);
  };
  auto issue_u = [&](int q) {  // union rows of triplet q (its (kd, kh) shift and 64-channel chunk)
    const int trip = q / nck, cc = q - trip * nck, kd = trip / 3, kh = trip - 3 * kd;
    const int add = ((kd * a.H + kh) * a.W) * (Cin * 2) + cc * (BK * 2);
    const int dlo = a.pad - kd, hlo = a.pad - kh;
#pragma unroll
    for (int i = 0; i < UPW; ++i) {
      if (wid * UPW + i >= UP) continue;
      const int c = ucode[i];
      const bool ok = PADDED ? ((unsigned)((c & 1023) - dlo) < (unsigned)a.D &&
                                (unsigned)(((c >> 10) & 1023) - hlo) < (unsigned)a.H &&
                                (unsigned)((c >> 20) - a.pad) < (unsigned)a.W)
                             : (c & 1023) != 1023;
      blds16(rxs, ok ? uoff[i] + add : kBufOOB, sU + (wid * UPW + i) * 512);
    }
  };

  f32x4 acc[TCO][TP];
#pragma unroll
  for (int i = 0; i < TCO; ++i)
#pragma unroll
    for (int j = 0; j < TP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue_u(0);
  issue_a(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int ks = 0; ks < nks; ++ks) {
    const int q = ks / 3, kw = ks - 3 * q;
    if (ks + 1 < nks) issue_a(ks + 1, (ks + 1) & 1);
    const uint16_t* sA = sAb + (ks & 1) * A_ELEMS;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[TCO], fb[TP];
#pragma unroll
      for (int i = 0; i < TCO; ++i) {
        const int r = wco * WCO + i * 16 + fr;
        fa[i] = *reinterpret_cast<const bf16x8*>(&sA[r * BK + (((4 * kk + fq) ^ swz_dma(r)) << 3)]);
      }
#pragma unroll
      for (int j = 0; j < TP; ++j) {
        const int r = hrow[j] + kw;
        fb[j] = *reinterpret_cast<const bf16x8*>(&sU[r * BK + (((4 * kk + fq) ^ swz_un(r)) << 3)]);
      }
#pragma unroll
      for (int i = 0; i < TCO; ++i)
#pragma unroll
        for (int j = 0; j < TP; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kw == 2 && q + 1 < ntr) {  // every wave is done with this triplet's union: reload it for the next one
      issue_u(q + 1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }
  __syncthreads();
  conv_fwd_epilogue<BCO, BP, WM, WN, BIAS, STATS, TCO, TP>(a, acc, reinterpret_cast<float*>(smem), g, pb, co0, wco, wp, fr,
                                                         fq, tid);
}

// k_conv_fwd_slab — 3x3x3 stride-1 forward/dgrad with the B operand staged once per (kd, 64-channel chunk) slab for
// all nine (kh, kw) taps.  k_conv_fwd_tri reloads a union per (kd, kh) triplet (3 x ~288 rows per kd for conv2); the
// runs of a slab union are whole windows b(p) .. b(p) + 2 Wp + 2 of the padded input (k_union_table with
// ext = 2 Wp + 2), so tap (kh, kw) of position p reads union row idx(p) + kh Wp + kw and one union of <= 384 rows
// (~352 on average for conv2) serves 9 k-steps: 2.3x fewer B bytes than the triplet unions, 6x fewer than
// per-tap tiles, and one exposed union reload per 9 k-steps instead of per 3.  The weight tile is double-buffered
// per tap as in k_conv_fwd_tri; 256-position blocks and the k_conv_fwd_dma epilogue / statistics layout.  Depth taps
// that read only padding for every position of a block (border output planes of the padded data gradient) are
// skipped.  LDS: 48 KB union + 2 weight tiles (16 / 32 KB): two blocks per CU also at 128 output channels.
// [LSWZ] the 16-B chunk swizzle of a union row is keyed by the row's output-space index L = (d Ho + h) Wo + w (its
// padded coordinates of the kd = 0 union) instead of its union position u: the 16 positions of a B fragment read the
// 16 CONSECUTIVE L values p + kh Wo + kw for every tap, across output-row and plane boundaries, where their union
// positions jump by Wp - Wo + 1 (3 for a 3x3 window).  With the pair swizzle ((x >> 1) & 3) << 1 the rows of one
// ds_read_b128 lane group then land on 16 distinct 4-bank slots; keyed by u, every fragment that crosses an output
// row put two rows on one slot (modelled: 1.84 / 1.79 LDS cycles per B read for the AlexNet conv2 forward / data
// gradient -> 1.00; measured 23-28 % LDS bank-conflict cycles, profiles/r3_s2_pmc_alexnet_g64.txt).  Measured
// (profiles/r4_ab_lds_swizzle.txt): bank conflicts 23.4 / 28.3 % -> 0.1 %, but conv2 forward / data gradient time
// unchanged (2.55 / 3.30 vs 2.55 / 3.25 ms) — the B reads are not what these blocks wait on.  Opt-in
// (NIDT_SLAB_LSWZ=1); the union-position swizzle stays the default.
__device__ __forceinline__ int swz_l(int l) { return ((l >> 1) & 3) << 1; }

// [NA] weight-tile stages: 2 = double buffer (the tile of k-step ks + 1 lands under k-step ks), 3 = two tiles in
// flight (the 64-channel blocks: 3 x 8 KB + the union still leave two blocks per CU).  Measured not faster (conv2
// data gradient 3.32-3.35 vs 3.25 ms, profiles/r4_ab_slab_stages.txt): NA = 3 is opt-in (NIDT_SLAB_NA=3).
template <int BCO, int WM, int WN, int U, bool PADDED, bool BIAS, bool STATS, bool LSW = true, int NA = 2,
          int SCHED = 0>
__global__ __launch_bounds__(64 * WM * WN, 2) void k_conv_fwd_slab(ConvFwdArgs a, int nCO, const int* __restrict__ utab) {
  constexpr int NW = WM * WN, BP = 64 * WN, BK = 64;
  constexpr int WCO = BCO / WM, WP = 64, TCO = WCO / 16, TP = WP / 16;
  constexpr int A_ELEMS = BCO * BK, ST = 2 * U + BP;
  constexpr int A_INSTR = BCO / (8 * NW);
  constexpr int UP = U / 8, UPW = (UP + NW - 1) / NW;  // union pieces (8 rows) per wave
  static_assert(A_INSTR >= 1 && U % 8 == 0, "tile split");
  static_assert(NA == 2 || NA == 3, "weight stages");
  __shared__ __attribute__((aligned(16))) uint16_t smem[NA * A_ELEMS + U * BK];
  uint16_t* const sAb = smem;
  uint16_t* const sU = smem + NA * A_ELEMS;

  const int nwg = gridDim.x;
  const int id = xcd_remap(blockIdx.x, nwg);
  const int cot = id % nCO, rest = id / nCO;
  const int pb = rest % a.nPB, g = rest / a.nPB;
  const int co0 = cot * BCO;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wco = wid / WN, wp = wid % WN;
  const int Cin = a.Cin, nck = Cin / BK, Wp = a.W + 2 * a.pad;
  // depth taps of this block (see k_conv_fwd_dma): slabs q = kd * nck + cc for kd in [kd_lo, kd_hi]
  int kd_lo = 0, kd_hi = 2;
  if (PADDED) {
    const int S = a.Do * a.Ho * a.Wo, m_lo = pb * BP, m_hi = min(m_lo + BP, a.Mg) - 1;
    if (m_lo / S == m_hi / S) {
      const int od_lo = (m_lo % S) / (a.Ho * a.Wo), od_hi = (m_hi % S) / (a.Ho * a.Wo);
      kd_lo = max(0, a.pad - od_hi);
      kd_hi = min(2, a.D - 1 + a.pad - od_lo);
    }
  }
  if (a.kd1) kd_lo = kd_hi = 1;
  const int q0 = kd_lo * nck, nq = (kd_hi + 1) * nck - q0, nks = 9 * nq;
  const int lrow = lane >> 3, slot = lane & 7;
  const int fr = lane & 15, fq = lane >> 4;
  const int* ent = utab + (int64_t)pb * ST;
  int uoff[UPW], ucode[UPW];
#pragma unroll
  for (int i = 0; i < UPW; ++i) {
    const int u = 8 * (wid * UPW + i) + lrow;
    uoff[i] = 0;
    ucode[i] = 1023;
    if (wid * UPW + i < UP) {
      const int c = ent[2 * u + 1];
      const int sw = LSW ? swz_l(((c & 1023) * a.Ho + ((c >> 10) & 1023)) * a.Wo + (c >> 20)) : swz_un(u);
      uoff[i] = ent[2 * u] * (Cin * 2) + ((slot ^ sw) << 4);
      ucode[i] = c;
    }
  }
  int hrow[TP], hl[TP];  // union row and output-space index L of tap (0, 0) of each fragment position
  const int So = a.Do * a.Ho * a.Wo;
#pragma unroll
  for (int j = 0; j < TP; ++j) {
    const int pl = wp * WP + j * 16 + fr;
    hrow[j] = ent[2 * U + pl];
    hl[j] = (pb * BP + pl) % So;
  }
  int aoff[A_INSTR];
#pragma unroll
  for (int i = 0; i < A_INSTR; ++i) {
    const int row = 8 * (wid * A_INSTR + i) + lrow;
    aoff[i] = ((co0 + row) * a.kt * Cin + ((slot ^ swz_dma(row)) << 3)) * 2;
  }
  // a.kt = 27 (3-D) or 9: a 2-D 3x3 conv as a D = 1, pad 1 volume whose blocks all lie inside one sample, so the
  // depth-tap skip above leaves kd = 1 only and that slab's weights are the 9-tap image itself
  const int kdw = a.kt == 27 ? 9 : 0;
  const int64_t xcl = (int64_t)a.B * a.D * a.H * a.W * Cin;
  const i32x4_t rxs = make_rsrc(a.x + (int64_t)g * xcl, (uint32_t)(xcl * 2));
  const i32x4_t rws = make_rsrc(a.w + (int64_t)g * a.Cout * a.kt * Cin, (uint32_t)(a.Cout * a.kt * Cin * 2));

  auto issue_a = [&](int ks, int buf) {  // weight tile of tap (kd, t = kh * 3 + kw) of slab q0 + ks / 9
    const int q = q0 + ks / 9, t = ks % 9, kd = q / nck, cc = q - kd * nck;
    const int woff = ((kd * kdw + t) * Cin + cc * BK) * 2;
    uint16_t* sA = sAb + buf * A_ELEMS;
#pragma unroll
    for (int i = 0; i < A_INSTR; ++i) blds16(rws, aoff[i] + woff, sA + (wid * A_INSTR + i) * 512);
  };
  auto issue_u = [&](int q) {  // union rows of slab q (its kd shift and 64-channel chunk)
    const int kd = q / nck, cc = q - kd * nck;
    const int add = kd * a.H * a.W * (Cin * 2) + cc * (BK * 2);
    const int dlo = a.pad - kd;
#pragma unroll
    for (int i = 0; i < UPW; ++i) {
      if (wid * UPW + i >= UP) continue;
      const int c = ucode[i];
      const bool ok = PADDED ? ((unsigned)((c & 1023) - dlo) < (unsigned)a.D &&
                                (unsigned)(((c >> 10) & 1023) - a.pad) < (unsigned)a.H &&
                                (unsigned)((c >> 20) - a.pad) < (unsigned)a.W)
                             : (c & 1023) != 1023;
      blds16(rxs, ok ? uoff[i] + add : kBufOOB, sU + (wid * UPW + i) * 512);
    }
  };

  f32x4 acc[TCO][TP];
#pragma unroll
  for (int i = 0; i < TCO; ++i)
#pragma unroll
    for (int j = 0; j < TP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue_u(q0);
  issue_a(0, 0);
  if (NA == 3 && nks > 1) issue_a(1, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  int bcur = 0;  // buffer of k-step ks (ks % NA)
  for (int ks = 0; ks < nks; ++ks) {
    const int ql = ks / 9, t = ks - 9 * ql, kh = t / 3, kw = t - 3 * kh;
    const int bnext = bcur + 1 == NA ? 0 : bcur + 1;
    if (NA == 2) {
      if (ks + 1 < nks) issue_a(ks + 1, bnext);
    } else if (ks + 2 < nks) {
      issue_a(ks + 2, bnext + 1 == NA ? 0 : bnext + 1);
    }
    const uint16_t* sA = sAb + bcur * A_ELEMS;
    bcur = bnext;
    const int toff = kh * Wp + kw, loff = kh * a.Wo + kw;
    auto fa_at = [&](int kk, int i) {
      const int r = wco * WCO + i * 16 + fr;
      return *reinterpret_cast<const bf16x8*>(&sA[r * BK + (((4 * kk + fq) ^ swz_dma(r)) << 3)]);
    };
    auto fb_at = [&](int kk, int j) {
      const int r = hrow[j] + toff;
      const int sw = LSW ? swz_l(hl[j] + loff) : swz_un(r);
      return *reinterpret_cast<const bf16x8*>(&sU[r * BK + (((4 * kk + fq) ^ sw) << 3)]);
    };
    if constexpr (SCHED == 1) {  // [SCHED] (kstep_sched)
      kstep_sched<TCO, TP>(acc, fa_at, fb_at);
    } else if constexpr (SCHED == 2) {  // [SCHED-half]
      kstep_sched_half<TCO, TP>(acc, fa_at, fb_at);
    } else {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[TCO], fb[TP];
#pragma unroll
      for (int i = 0; i < TCO; ++i) {
        const int r = wco * WCO + i * 16 + fr;
        fa[i] = *reinterpret_cast<const bf16x8*>(&sA[r * BK + (((4 * kk + fq) ^ swz_dma(r)) << 3)]);
      }
#pragma unroll
      for (int j = 0; j < TP; ++j) {
        const int r = hrow[j] + toff;
        const int sw = LSW ? swz_l(hl[j] + loff) : swz_un(r);
        fb[j] = *reinterpret_cast<const bf16x8*>(&sU[r * BK + (((4 * kk + fq) ^ sw) << 3)]);
      }
#pragma unroll
      for (int i = 0; i < TCO; ++i)
#pragma unroll
        for (int j = 0; j < TP; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    }
    // the tile of k-step ks + 1 must have landed; with three stages the one of ks + 2 may stay in flight
    if (NA == 3 && ks + 2 < nks) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(A_INSTR) : "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t == 8 && ql + 1 < nq && a.dbg != 1) {  // every wave is done with this slab's union: reload it for the next one
      issue_u(q0 + ql + 1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }
  __syncthreads();
  conv_fwd_epilogue<BCO, BP, WM, WN, BIAS, STATS, TCO, TP>(a, acc, reinterpret_cast<float*>(smem), g, pb, co0, wco, wp, fr,
                                                         fq, tid);
}

// k_conv_fwd_vol — 3x3x3 stride-1 forward/dgrad of small volumes (the AlexNet3D 5x7x5 conv3-5 layers) with the B
// operand of a whole padded SAMPLE staged once per 64-channel chunk for all 27 taps.  Blocks are (sample, output-
// channel chunk) with BP = 64 WN >= Do Ho Wo positions; the padded sample (Dp Hp Wp <= U rows, padding rows read out of
// the buffer range as zeros) is the union of every tap's rows, so tap (kd, kh, kw) of output p reads union row
// idx(p) + kd Hp Wp + kh Wp + kw — no table.  Against the per-tap kernel (one B tile per tap) this moves 27x fewer B
// bytes per k-step; weights double-buffered per tap as in k_conv_fwd_slab.  Per-sample BN statistics blocks
// (nPB = B, block size Do Ho Wo).
template <int BCO, int WM, int WN, int U, bool BIAS, bool STATS>
__global__ __launch_bounds__(64 * WM * WN, 2) void k_conv_fwd_vol(ConvFwdArgs a, int nCO) {
  constexpr int NW = WM * WN, BP = 64 * WN, BK = 64;
  constexpr int WCO = BCO / WM, WP = 64, TCO = WCO / 16, TP = WP / 16;
  constexpr int A_ELEMS = BCO * BK;
  constexpr int AI = BCO / 8, AIW = (AI + NW - 1) / NW;   // weight-tile pieces (8 rows) and per wave
  constexpr int UP = U / 8, UPW = (UP + NW - 1) / NW;     // union pieces and per wave
  static_assert(U % 8 == 0 && TCO >= 1, "tile split");
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * A_ELEMS + U * BK];
  uint16_t* const sAb = smem;
  uint16_t* const sU = smem + 2 * A_ELEMS;

  const int nwg = gridDim.x;
  const int id = xcd_remap(blockIdx.x, nwg);
  const int cot = id % nCO, rest = id / nCO;
  const int n = rest % a.B, g = rest / a.B;
  const int co0 = cot * BCO;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wco = wid / WN, wp = wid % WN;
  const int Cin = a.Cin, nck = Cin / BK, pad = a.pad;
  const int Hp = a.H + 2 * pad, Wp = a.W + 2 * pad, HWp = Hp * Wp, R = (a.D + 2 * pad) * HWp;
  const int S = a.Do * a.Ho * a.Wo, HoWo = a.Ho * a.Wo;
  const int lrow = lane >> 3, slot = lane & 7;
  const int fr = lane & 15, fq = lane >> 4;
  const int64_t vol = (int64_t)a.D * a.H * a.W;
  // union pieces of this lane: padded row r -> source voxel of sample n (or out of range: zeros)
  int uoff[UPW];
#pragma unroll
  for (int i = 0; i < UPW; ++i) {
    const int u = 8 * (wid + NW * i) + lrow;
    uoff[i] = kBufOOB;
    if (wid + NW * i < UP && u < R) {
      const int d = u / HWp - pad, h = (u / Wp) % Hp - pad, w = u % Wp - pad;
      if ((unsigned)d < (unsigned)a.D && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W)
        uoff[i] = (int)(((n * vol + ((int64_t)d * a.H + h) * a.W + w) * Cin) * 2) + ((slot ^ swz_un(u)) << 4);
    }
  }
  int hrow[TP];
#pragma unroll
  for (int j = 0; j < TP; ++j) {
    int p = wp * WP + j * 16 + fr;
    p = p < S ? p : 0;
    const int od = p / HoWo, r2 = p - od * HoWo, oh = r2 / a.Wo, ow = r2 - oh * a.Wo;
    hrow[j] = od * HWp + oh * Wp + ow;
  }
  int aoff[AIW];
#pragma unroll
  for (int i = 0; i < AIW; ++i) {
    const int row = 8 * (wid + NW * i) + lrow;
    aoff[i] = ((co0 + row) * 27 * Cin + ((slot ^ swz_dma(row)) << 3)) * 2;
  }
  const int64_t xcl = (int64_t)a.B * vol * Cin;
  const i32x4_t rxs = make_rsrc(a.x + (int64_t)g * xcl, (uint32_t)(xcl * 2));
  const i32x4_t rws = make_rsrc(a.w + (int64_t)g * a.Cout * 27 * Cin, (uint32_t)(a.Cout * 27 * Cin * 2));

  auto issue_a = [&](int ks, int buf) {  // weight tile of tap t = ks % 27 of channel chunk ks / 27
    const int cc = ks / 27, t = ks - 27 * cc;
    const int woff = (t * Cin + cc * BK) * 2;
    uint16_t* sA = sAb + buf * A_ELEMS;
#pragma unroll
    for (int i = 0; i < AIW; ++i)
      if (wid + NW * i < AI) blds16(rws, aoff[i] + woff, sA + (wid + NW * i) * 512);
  };
  auto issue_u = [&](int cc) {
#pragma unroll
    for (int i = 0; i < UPW; ++i) {
      if (wid + NW * i >= UP) continue;
      const int o = uoff[i];
      blds16(rxs, o == kBufOOB ? kBufOOB : o + cc * (BK * 2), sU + (wid + NW * i) * 512);
    }
  };

  f32x4 acc[TCO][TP];
#pragma unroll
  for (int i = 0; i < TCO; ++i)
#pragma unroll
    for (int j = 0; j < TP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nks = 27 * nck;
  issue_u(0);
  issue_a(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  for (int ks = 0; ks < nks; ++ks) {
    const int cc = ks / 27, t = ks - 27 * cc, kd = t / 9, kh = (t / 3) % 3, kw = t % 3;
    if (ks + 1 < nks) issue_a(ks + 1, (ks + 1) & 1);
    const uint16_t* sA = sAb + (ks & 1) * A_ELEMS;
    const int toff = kd * HWp + kh * Wp + kw;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[TCO], fb[TP];
#pragma unroll
      for (int i = 0; i < TCO; ++i) {
        const int r = wco * WCO + i * 16 + fr;
        fa[i] = *reinterpret_cast<const bf16x8*>(&sA[r * BK + (((4 * kk + fq) ^ swz_dma(r)) << 3)]);
      }
#pragma unroll
      for (int j = 0; j < TP; ++j) {
        const int r = hrow[j] + toff;
        fb[j] = *reinterpret_cast<const bf16x8*>(&sU[r * BK + (((4 * kk + fq) ^ swz_un(r)) << 3)]);
      }
#pragma unroll
      for (int i = 0; i < TCO; ++i)
#pragma unroll
        for (int j = 0; j < TP; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (t == 26 && cc + 1 < nck) {  // every wave is done with this chunk's union: reload it for the next one
      issue_u(cc + 1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
  }
  __syncthreads();
  conv_fwd_epilogue<BCO, BP, WM, WN, BIAS, STATS, TCO, TP>(a, acc, reinterpret_cast<float*>(smem), g, n, co0, wco, wp, fr,
                                                         fq, tid, 0, n * S, n * S + S);
}

// Finish of a split-K forward without bias / statistics: y = bf16(sum over the ksplit slabs), 4 values per thread
__global__ __launch_bounds__(256) void k_fwd_splitk_sum(const float* __restrict__ part, int ksplit, int64_t n4,
                                                        uint16_t* __restrict__ y) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4; q += (int64_t)gridDim.x * blockDim.x) {
    float4 acc = reinterpret_cast<const float4*>(part)[q];
    for (int sp = 1; sp < ksplit; ++sp) {
      const float4 v = reinterpret_cast<const float4*>(part)[sp * n4 + q];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    reinterpret_cast<uint2*>(y)[q] = make_uint2(pack_bf16x2(acc.x, acc.y), pack_bf16x2(acc.z, acc.w));
  }
}

// Finish a split-K forward: y = bf16(sum of the partials + bias) and the same per-block BN statistics as the
// fused epilogue (block mean and M2 per channel over the block's BP positions, fp32 values before rounding).
// Block (pb, g), 1024 threads: lane -> channel c = lane + 64 u, wave -> positions m0 + wave + 16 v; the 16 wave
// partial sums are combined in a fixed order (deterministic).
constexpr int kFinPG = 16;      // position groups (waves)
constexpr int kFinMaxCU = 4;    // Cout <= 256
constexpr int kFinMaxPV = 16;   // positions per group (BP = 256)
template <bool BIAS, bool STATS>
__global__ __launch_bounds__(1024) void k_fwd_splitk_fin(const float* __restrict__ part, int ksplit,
                                                         const float* __restrict__ bias, uint16_t* __restrict__ y,
                                                         float* __restrict__ stats, int G, int Mg, int Cout, int BP,
                                                         int nPB, int64_t bias_ld) {
  __shared__ float red[kFinPG][256];
  __shared__ float smean[256];
  const int pb = blockIdx.x, g = blockIdx.y;
  const int lane = threadIdx.x & 63, pg = threadIdx.x >> 6;
  const int m0 = pb * BP, cnt = min(BP, Mg - m0);
  const int ncu = Cout / 64;
  const int64_t pst = (int64_t)G * Mg * Cout;
  float v[kFinMaxCU][kFinMaxPV];
  float s[kFinMaxCU];
#pragma unroll
  for (int u = 0; u < kFinMaxCU; ++u) {
    s[u] = 0.f;
    if (u >= ncu) continue;
    const int c = lane + 64 * u;
    const float bv = BIAS ? bias[(int64_t)g * bias_ld + c] : 0.f;
#pragma unroll
    for (int q = 0; q < kFinMaxPV; ++q) {
      const int m = pg + kFinPG * q;
      v[u][q] = 0.f;
      if (m < cnt) {
        const int64_t o = ((int64_t)g * Mg + m0 + m) * Cout + c;
        float acc = 0.f;
        for (int sp = 0; sp < ksplit; ++sp) acc += part[sp * pst + o];
        const float t = acc + bv;
        v[u][q] = t;
        y[o] = f32_to_bf16(t);
        s[u] += t;
      }
    }
  }
  if (!STATS) return;
#pragma unroll
  for (int u = 0; u < kFinMaxCU; ++u)
    if (u < ncu) red[pg][lane + 64 * u] = s[u];
  __syncthreads();
  for (int c = threadIdx.x; c < Cout; c += 1024) {
    float t = 0.f;
    for (int q = 0; q < kFinPG; ++q) t += red[q][c];
    smean[c] = t / (float)cnt;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kFinMaxCU; ++u) {
    if (u >= ncu) continue;
    const float mu = smean[lane + 64 * u];
    float q2 = 0.f;
#pragma unroll
    for (int q = 0; q < kFinMaxPV; ++q)
      if (pg + kFinPG * q < cnt) {
        const float d = v[u][q] - mu;
        q2 = fmaf(d, d, q2);
      }
    s[u] = q2;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < kFinMaxCU; ++u)
    if (u < ncu) red[pg][lane + 64 * u] = s[u];
  __syncthreads();
  for (int c = threadIdx.x; c < Cout; c += 1024) {
    float t = 0.f;
    for (int q = 0; q < kFinPG; ++q) t += red[q][c];
    float* st = stats + (((int64_t)g * nPB + pb) * Cout + c) * 2;
    st[0] = smean[c];
    st[1] = t;
  }
}

int conv3d_fwd_bp(int Cin, int Cout, int xf, int G, int Mg);

// launch one k_conv_fwd_dma variant; the 3-stage pipeline only where 3 LDS stages fit in 160 KB
// [SCHED] on the per-tap forward blocks: 1 = the 64-channel blocks, 2 (default) = the 128-channel blocks too (each of
// the three A/Bs the same sign: 8-client step -0.6 %, 8-client round 15.25 -> 15.29 rounds/s, config 5 12.16 ->
// 12.12 s/round; profiles/r4_ab_dma_sched.txt, r4_ab_sched_more.txt, r4_ab_dma_sched128.txt); 0 = off (A/B)
static int dma_sched() {
  static const int env = [] {
    const char* e = getenv("NIDT_DMA_SCHED");
    return e ? atoi(e) : 2;
  }();
  return env;
}

template <int BC, int WM, int WN, bool BI, bool ST>
static void launch_fwd_dma(int nst, dim3 g, hipStream_t s, const ConvFwdArgs& a, int nCO) {
  constexpr int kStageBytes = (BC + 64 * WN) * 64 * 2;
  if constexpr (BC == 64 && WM == 1) {
    if (dma_sched()) {
      if constexpr (3 * kStageBytes <= 160 * 1024) {
        if (nst == 3) {
          hipLaunchKernelGGL((k_conv_fwd_dma<BC, WM, WN, 3, BI, ST, 1>), g, dim3(64 * WM * WN), 0, s, a, nCO);
          return;
        }
      }
      hipLaunchKernelGGL((k_conv_fwd_dma<BC, WM, WN, 2, BI, ST, 1>), g, dim3(64 * WM * WN), 0, s, a, nCO);
      return;
    }
  }
  if constexpr (BC == 128 && WM == 2) {
    if (dma_sched() == 2) {
      if constexpr (3 * kStageBytes <= 160 * 1024) {
        if (nst == 3) {
          hipLaunchKernelGGL((k_conv_fwd_dma<BC, WM, WN, 3, BI, ST, 1>), g, dim3(64 * WM * WN), 0, s, a, nCO);
          return;
        }
      }
      hipLaunchKernelGGL((k_conv_fwd_dma<BC, WM, WN, 2, BI, ST, 1>), g, dim3(64 * WM * WN), 0, s, a, nCO);
      return;
    }
  }
  if constexpr (3 * kStageBytes <= 160 * 1024) {
    if (nst == 3) {
      hipLaunchKernelGGL((k_conv_fwd_dma<BC, WM, WN, 3, BI, ST>), g, dim3(64 * WM * WN), 0, s, a, nCO);
      return;
    }
  }
  hipLaunchKernelGGL((k_conv_fwd_dma<BC, WM, WN, 2, BI, ST>), g, dim3(64 * WM * WN), 0, s, a, nCO);
}

// output channels per forward block: 128 (8 waves, one resident block per CU) where Cout allows, else 64 (4 waves,
// two blocks per CU).  NIDT_FWD_BCO=64 forces 64-channel blocks everywhere (A/B).
static int fwd_bco(int Cout) {
  static const int env = [] {
    const char* e = getenv("NIDT_FWD_BCO");
    return e ? atoi(e) : 0;
  }();
  if (env == 64) return 64;
  return (Cout % 128 == 0) ? 128 : 64;
}

// output extent of one dimension: taps k (3 or 1), stride st, padding p
static inline int conv_out_dim(int n, int k, int st, int p) { return (n + 2 * p - k) / st + 1; }

struct PhasePlan;
static void conv3d_fwd_impl(uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t xs, uintptr_t xt, uintptr_t y,
                            uintptr_t stats, int G, int B, int D, int H, int W, int Cin, int Cout, int pad,
                            uintptr_t stream, int ksplit, uintptr_t part, int64_t bias_ld = 0, int kt = 27,
                            int stride = 1, int padd = -1, const PhasePlan* pp = nullptr, int Dx = 0, int Hx = 0,
                            int Wx = 0);

// Sub-pixel decomposition of the data gradient of a k=3, pad=1, stride-2 conv: per dimension, output phase 0 (even
// positions 2i) takes kernel tap k=1 from dy row i (window index 1 of a pad-1 3-window), phase 1 (2i+1) takes k=0
// from dy row i+1 (window 2) and k=2 from row i (window 1).  A 3x3(x3) conv therefore splits into 4 (8) stride-1
// convs over the dy grid with 1,2,2,4 (,2,4,4,8) taps — 9 (27) taps in all instead of 9 (27) taps on a 4x (8x)
// larger zero-upsampled grid.  Slots number the taps phase-major (phase = d,h,w bits), window order inside.
struct PhasePlan {
  int nph = 0;
  int pnt[8] = {0}, pt0[8] = {0}, poff[8] = {0}, ptap[27] = {0};
  int slot_of_tap[27] = {0};  // fwd kernel tap (kd*9 + kh*3 + kw) -> slot
};

static PhasePlan conv_s2_phase_plan(int kt) {
  PhasePlan pl;
  const int nd = kt == 27 ? 2 : 1;  // depth phases (2-D convs run as D = 1 volumes: one depth tap, window 0)
  static const int nk[2] = {1, 2}, kk[2][2] = {{1, -1}, {0, 2}}, ww[2][2] = {{1, -1}, {2, 1}};
  int slot = 0;
  for (int ad = 0; ad < nd; ++ad)
    for (int ah = 0; ah < 2; ++ah)
      for (int aw = 0; aw < 2; ++aw) {
        const int p = pl.nph++;
        pl.pt0[p] = slot;
        pl.poff[p] = (ad << 2) | (ah << 1) | aw;
        const int ndt = kt == 27 ? nk[ad] : 1;
        for (int i = 0; i < ndt; ++i)
          for (int j = 0; j < nk[ah]; ++j)
            for (int l = 0; l < nk[aw]; ++l) {
              const int kd = kt == 27 ? kk[ad][i] : 0, wd = kt == 27 ? ww[ad][i] : 0;
              const int t_fwd = kd * 9 + kk[ah][j] * 3 + kk[aw][l];
              const int t_win = wd * 9 + ww[ah][j] * 3 + ww[aw][l];
              pl.ptap[slot] = t_win;
              pl.slot_of_tap[t_fwd] = slot;
              ++slot;
            }
        pl.pnt[p] = slot - pl.pt0[p];
      }
  return pl;
}

static void conv3d_fwd_impl(uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t xs, uintptr_t xt, uintptr_t y,
                            uintptr_t stats, int G, int B, int D, int H, int W, int Cin, int Cout, int pad,
                            uintptr_t stream, int ksplit, uintptr_t part, int64_t bias_ld, int kt,
                            int stride, int padd, const PhasePlan* pp, int Dx, int Hx, int Wx) {
  NIDT_REQUIRE(Cin % 32 == 0, "conv3d_fwd: Cin must be a multiple of 32");
  NIDT_REQUIRE((xs == 0 && Cin % 64 == 0) ? (int64_t)Cin * kt <= 27 * kMaxCin : Cin <= 192,
               "conv3d_fwd: taps x Cin <= 27 x 512 (LDS-DMA path: Cin % 64 == 0, no input transform), else Cin <= 192");
  NIDT_REQUIRE(Cout % 64 == 0, "conv3d_fwd: Cout must be a multiple of 64");
  NIDT_REQUIRE(pad >= 0 && pad <= 2, "conv3d_fwd: pad in [0,2]");
  NIDT_REQUIRE(kt == 27 || kt == 9 || kt == 1, "conv3d_fwd: taps 27 (3x3x3), 9 (1x3x3) or 1 (1x1x1)");
  NIDT_REQUIRE(stride == 1 || stride == 2, "conv3d_fwd: stride 1 or 2");
  if (padd < 0) padd = pad;
  NIDT_REQUIRE(padd >= 0 && padd <= 2 && (kt == 27 || padd == 0) && (kt != 1 || pad == 0),
               "conv3d_fwd: padding must fit the kernel extent");
  NIDT_REQUIRE((kt == 27 && stride == 1 && padd == pad) || (xs == 0 && Cin % 64 == 0),
               "conv3d_fwd: 9/1-tap or strided convs need the LDS-DMA path (Cin % 64 == 0, no input transform)");
  NIDT_REQUIRE((int64_t)B * D * H * W * Cin * 2 < (1ll << 31),
               "conv3d_fwd: per-client input must stay below 2 GiB (32-bit buffer offsets)");
  ConvFwdArgs a;
  a.x = ptr<const uint16_t>(x); a.w = ptr<const uint16_t>(w); a.bias = ptr<const float>(bias);
  a.xs = ptr<const float>(xs); a.xt = ptr<const float>(xt); a.y = ptr<uint16_t>(y); a.stats = ptr<float>(stats);
  a.B = B; a.D = D; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.pad = pad;
  a.kt = kt; a.st = stride; a.padd = padd;
  const int kd = kt == 27 ? 3 : 1, khw = kt == 1 ? 1 : 3;
  a.Do = conv_out_dim(D, kd, stride, padd); a.Ho = conv_out_dim(H, khw, stride, pad); a.Wo = conv_out_dim(W, khw, stride, pad);
  NIDT_REQUIRE(a.Do > 0 && a.Ho > 0 && a.Wo > 0, "conv3d_fwd: empty output");
  a.Mg = B * a.Do * a.Ho * a.Wo;
  a.nPB = ceil_div(a.Mg, kFwdBP);
  a.G = G;
  a.bias_ld = bias_ld;
  if (pp) {
    NIDT_REQUIRE(stride == 1 && bias == 0 && stats == 0 && xs == 0 && ksplit <= 1 && Cin % 64 == 0,
                 "conv_dgrad_s2: phase convs are plain stride-1 LDS-DMA convs without split-K");
    a.nph = pp->nph; a.Dx = Dx; a.Hx = Hx; a.Wx = Wx;
    for (int p = 0; p < pp->nph; ++p) {
      a.pnt[p] = (unsigned char)pp->pnt[p]; a.pt0[p] = (unsigned char)pp->pt0[p]; a.poff[p] = (unsigned char)pp->poff[p];
    }
    for (int t = 0; t < kt; ++t) a.ptap[t] = (unsigned char)pp->ptap[t];
  }
  const bool xf = xs != 0, hb = bias != 0, st = stats != 0;
  NIDT_REQUIRE(!st || hb, "conv3d_fwd: statistics require a bias");
  const int bco = fwd_bco(Cout);
  hipStream_t s = as_stream(stream);
  if (!xf && Cin % 64 == 0) {
    // 256 positions per block: BCO=128 -> 8 waves (2 co x 4 pos, 512 threads), BCO=64 -> 4 waves (1 x 4);
    // every wave owns a 64x64 output tile (the A tile is re-read from L2 once per 256 positions).  When that
    // grid would not fill the chip (few clients per GPU, e.g. 8 clients x the 5x7x5 conv3-5 layers at 8 GPUs)
    // the block shrinks to one 64-position column of waves (4x the blocks).
    const int bp = conv3d_fwd_bp(Cin, Cout, 0, G * (a.nph > 0 ? a.nph : 1), a.Mg);
    a.nPB = ceil_div(a.Mg, bp);
    const int nCO = Cout / bco;
    if (ksplit > 1) {
      NIDT_REQUIRE(part != 0 && ((!hb && !st) || (bp <= 256 && Cout <= 256)),
                   "conv3d_fwd_splitk: needs a partial buffer (with bias/statistics: <= 256-position blocks, Cout <= 256)");
      a.ksplit = ksplit;
      a.part = ptr<float>(part);
    }
    const int64_t nwg = (int64_t)a.nPB * nCO * G * a.ksplit * (a.nph > 0 ? a.nph : 1);
    NIDT_REQUIRE(nwg < (1ll << 31), "conv3d_fwd: grid too large");
    dim3 g1((unsigned)nwg);
    // small grids (64-position blocks: conv3-5 at 8 clients per GPU) run at ~1 wave per SIMD: a third LDS stage
    // keeps two k-steps of LDS-DMA in flight to cover the load latency the missing waves cannot hide.
    static const int nst_env = [] {
      const char* e = getenv("NIDT_FWD_NST");
      return e ? atoi(e) : 0;
    }();
    const int nst = nst_env ? nst_env : (bp == 64 ? 3 : 2);  // measured: 3 stages only pay with 64-position blocks
#define NIDT_DMA(BC, WM, WN, BI, ST) launch_fwd_dma<BC, WM, WN, BI, ST>(nst, g1, s, a, nCO)
#define NIDT_DMA_WN(WN)                                                                                     \
    if (bco == 128) {                                                                                       \
      if (st) NIDT_DMA(128, 2, WN, true, true); else if (hb) NIDT_DMA(128, 2, WN, true, false);             \
      else NIDT_DMA(128, 2, WN, false, false);                                                              \
    } else {                                                                                                \
      if (st) NIDT_DMA(64, 1, WN, true, true); else if (hb) NIDT_DMA(64, 1, WN, true, false);               \
      else NIDT_DMA(64, 1, WN, false, false);                                                               \
    }
    if (bp == 256) { NIDT_DMA_WN(4) } else if (bp == 512) { NIDT_DMA_WN(8) } else if (bp == 128) { NIDT_DMA_WN(2) } else { NIDT_DMA_WN(1) }
#undef NIDT_DMA_WN
#undef NIDT_DMA
    NIDT_CHECK(hipGetLastError());
    if (a.ksplit > 1 && !hb && !st) {  // plain sum of the partial slabs -> bf16
      const int64_t n4 = (int64_t)G * a.Mg * Cout / 4;
      hipLaunchKernelGGL(k_fwd_splitk_sum, dim3((unsigned)std::min<int64_t>(8192, (n4 + 255) / 256)), dim3(256), 0, s,
                         a.part, a.ksplit, n4, a.y);
      NIDT_CHECK(hipGetLastError());
    } else if (a.ksplit > 1) {
      const dim3 fg(a.nPB, G);
      if (st) hipLaunchKernelGGL((k_fwd_splitk_fin<true, true>), fg, dim3(1024), 0, s, a.part, a.ksplit, a.bias, a.y, a.stats, G, a.Mg, Cout, bp, a.nPB, a.bias_ld ? a.bias_ld : (int64_t)Cout);
      else if (hb) hipLaunchKernelGGL((k_fwd_splitk_fin<true, false>), fg, dim3(1024), 0, s, a.part, a.ksplit, a.bias, a.y, a.stats, G, a.Mg, Cout, bp, a.nPB, a.bias_ld ? a.bias_ld : (int64_t)Cout);
      else hipLaunchKernelGGL((k_fwd_splitk_fin<false, false>), fg, dim3(1024), 0, s, a.part, a.ksplit, a.bias, a.y, a.stats, G, a.Mg, Cout, bp, a.nPB, a.bias_ld ? a.bias_ld : (int64_t)Cout);
      NIDT_CHECK(hipGetLastError());
    }
    return;
  }
  NIDT_REQUIRE(ksplit <= 1, "conv3d_fwd: split-K needs the LDS-DMA path (Cin % 64 == 0, no input transform)");
  dim3 grid(a.nPB, Cout / bco, G);
#define NIDT_FWD(BC, X, BI, ST) hipLaunchKernelGGL((k_conv_fwd<BC, X, BI, ST>), grid, dim3(256), 0, s, a)
  if (bco == 128) {
    if (xf) { if (st) NIDT_FWD(128, true, true, true); else if (hb) NIDT_FWD(128, true, true, false); else NIDT_FWD(128, true, false, false); }
    else { if (st) NIDT_FWD(128, false, true, true); else if (hb) NIDT_FWD(128, false, true, false); else NIDT_FWD(128, false, false, false); }
  } else {
    if (xf) { if (st) NIDT_FWD(64, true, true, true); else if (hb) NIDT_FWD(64, true, true, false); else NIDT_FWD(64, true, false, false); }
    else { if (st) NIDT_FWD(64, false, true, true); else if (hb) NIDT_FWD(64, false, true, false); else NIDT_FWD(64, false, false, false); }
  }
#undef NIDT_FWD
  NIDT_CHECK(hipGetLastError());
}

// Data gradient of a k=3, pad=1, stride-2 client-grouped conv by sub-pixel phases (conv_s2_phase_plan): dy
// [G*B][D][H][W][Cin] (the forward's output grid and channels), w [G][Cout][kt][Cin] with the taps in slot order
// (pack_convs), dx [G*B][Dx][Hx][Wx][Cout] written completely (every position belongs to exactly one phase) — no
// zero-upsampled copy of dy and no memset.  kt = 9 (2-D, D = 1) or 27.
void conv_dgrad_s2_g(uintptr_t dy, uintptr_t w, uintptr_t dx, int G, int B, int D, int H, int W, int Cin, int Cout,
                     int kt, int Dx, int Hx, int Wx, uintptr_t stream) {
  NIDT_REQUIRE(kt == 9 || kt == 27, "conv_dgrad_s2_g: 3x3 (kt 9) or 3x3x3 (kt 27) kernels");
  NIDT_REQUIRE(Hx <= 2 * H && Hx >= 2 * H - 1 && Wx <= 2 * W && Wx >= 2 * W - 1 &&
               (kt == 9 ? (D == 1 && Dx == 1) : (Dx <= 2 * D && Dx >= 2 * D - 1)),
               "conv_dgrad_s2_g: dx extent must be the stride-2 input of the dy grid");
  static const PhasePlan pl9 = conv_s2_phase_plan(9), pl27 = conv_s2_phase_plan(27);
  conv3d_fwd_impl(dy, w, 0, 0, 0, dx, 0, G, B, D, H, W, Cin, Cout, 1, stream, 1, 0, 0, kt, 1, kt == 27 ? 1 : 0,
                  kt == 27 ? &pl27 : &pl9, Dx, Hx, Wx);
}

// tap slot permutation of the dgrad weight image (pack_convs): stride 1 -> flipped taps, stride 2 (k = 3) -> the
// sub-pixel phase order, 1x1 -> identity
std::vector<int> conv_tap_slots(int kt, int stride) {
  std::vector<int> out(kt);
  if (kt == 1) { out[0] = 0; return out; }
  if (stride == 1) {
    for (int t = 0; t < kt; ++t) out[t] = kt - 1 - t;
    return out;
  }
  const PhasePlan pl = conv_s2_phase_plan(kt);
  for (int t = 0; t < kt; ++t) out[t] = pl.slot_of_tap[t];
  return out;
}

void conv3d_fwd(uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t xs, uintptr_t xt, uintptr_t y, uintptr_t stats,
                int G, int B, int D, int H, int W, int Cin, int Cout, int pad, uintptr_t stream) {
  conv3d_fwd_impl(x, w, bias, xs, xt, y, stats, G, B, D, H, W, Cin, Cout, pad, stream, 1, 0);
}

// Split-K forward for grids that would not fill the chip (few clients per GPU x the 5x7x5 conv3-5 layers):
// ksplit blocks share one output tile, each over 1/ksplit of the 27*Cin reduction, writing fp32 partials
// [ksplit, G, Mg, Cout] (part); k_fwd_splitk_fin adds them (fixed order), the bias, and emits y and the BN stats.
// Forward whose per-client bias rows live at stride bias_ld (e.g. read straight from the flat parameter rows
// theta[g][off_bias ..] instead of a per-step copy into a contiguous [G, Cout] buffer).
void conv3d_fwd_bld(uintptr_t x, uintptr_t w, uintptr_t bias, int64_t bias_ld, uintptr_t y, uintptr_t stats, int G, int B,
                    int D, int H, int W, int Cin, int Cout, int pad, uintptr_t stream) {
  conv3d_fwd_impl(x, w, bias, 0, 0, y, stats, G, B, D, H, W, Cin, Cout, pad, stream, 1, 0, bias_ld);
}

// Split-K factor of the general forward: grids that cannot fill the chip (few output tiles: deep layers at small
// spatial size, few clients per GPU) but have long reductions get their k-steps split over ksplit blocks (>= 12
// k-steps each), finished by k_fwd_splitk_sum.  NIDT_FWDG_KSPLIT=1 disables it (A/B), =k forces k.
int conv_fwd_g_ksplit(int G, int B, int D, int H, int W, int Cin, int Cout, int kt, int st, int pad, int padd) {
  static const int env = [] {
    const char* e = getenv("NIDT_FWDG_KSPLIT");
    return e ? atoi(e) : 0;
  }();
  const int kd = kt == 27 ? 3 : 1, khw = kt == 1 ? 1 : 3;
  const int Mg = B * conv_out_dim(D, kd, st, padd) * conv_out_dim(H, khw, st, pad) * conv_out_dim(W, khw, st, pad);
  const int nks = kt * Cin / 64;
  if (env > 0) return std::max(1, std::min(env, nks));
  const int bco = fwd_bco(Cout);
  const int bp = conv3d_fwd_bp(Cin, Cout, 0, G, Mg);
  const int64_t nwg = (int64_t)ceil_div(Mg, bp) * (Cout / bco) * G;
  const int64_t slots = 256 * (bco == 128 ? 1 : 2);
  if (nwg >= slots || nks < 24) return 1;
  const int ks = (int)std::min<int64_t>(std::min<int64_t>(ceil_div(2 * slots, nwg), nks / 12), 8);
  return std::max(1, ks);
}

// General client-grouped conv forward with split-K partials (part: ksplit * G * Mg * Cout fp32, ksplit > 1)
void conv_fwd_gk(uintptr_t x, uintptr_t w, uintptr_t y, uintptr_t part, int ksplit, int G, int B, int D, int H, int W,
                 int Cin, int Cout, int kt, int st, int pad, int padd, uintptr_t stream) {
  NIDT_REQUIRE(Cin % 64 == 0, "conv_fwd_gk: Cin must be a multiple of 64 (pad the channels)");
  conv3d_fwd_impl(x, w, 0, 0, 0, y, 0, G, B, D, H, W, Cin, Cout, pad, stream, ksplit, part, 0, kt, st, padd);
}

// General client-grouped conv forward (no bias / statistics): kt taps (27, 9 = 2-D 3x3 on D = 1 volumes, 1 = 1x1),
// stride st (1 or 2), h/w padding pad, depth padding padd.  w: [G][Cout][kt][Cin] bf16 (pack_conv_wk).
void conv_fwd_g(uintptr_t x, uintptr_t w, uintptr_t y, int G, int B, int D, int H, int W, int Cin, int Cout, int kt,
                int st, int pad, int padd, uintptr_t stream) {
  NIDT_REQUIRE(Cin % 64 == 0, "conv_fwd_g: Cin must be a multiple of 64 (pad the channels)");
  conv3d_fwd_impl(x, w, 0, 0, 0, y, 0, G, B, D, H, W, Cin, Cout, pad, stream, 1, 0, 0, kt, st, padd);
}

void conv3d_fwd_splitk(uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, uintptr_t stats, uintptr_t part,
                       int ksplit, int G, int B, int D, int H, int W, int Cin, int Cout, int pad, uintptr_t stream) {
  conv3d_fwd_impl(x, w, bias, 0, 0, y, stats, G, B, D, H, W, Cin, Cout, pad, stream, ksplit, part);
}

// Split-K factor for conv3d_fwd_splitk (forward with bias + BN block statistics, and the dgrad convs): only grids
// with fewer blocks than CUs and a long reduction, i.e. the 5x7x5 conv3-5 layers at one or two clients per launch
// (the partial-batch launches of ragged federations): there a block runs 36-81 sequential k-steps on a third of
// the chip.  ks = min(ceil(512 / blocks), k-steps / 12, 8), finished by k_fwd_splitk_fin / k_fwd_splitk_sum.
// Measured at 8 clients per GPU (264-block grids) a split made the step slower (3.97 -> 4.16 ms,
// profiles/r1_ab_fwd_splitk.txt), hence the < 256-block rule.  NIDT_FWD_KSPLIT=1 disables it, =k > 1 forces k.
int conv3d_fwd_ksplit(int Cin, int Cout, int G, int Mg) {
  if (Cin % 64 != 0 || Cout > 256 || Cout % 64 != 0) return 1;
  static const int env = [] {
    const char* e = getenv("NIDT_FWD_KSPLIT");
    return e ? atoi(e) : 0;
  }();
  const int nks = 27 * Cin / 64;
  if (env == 1) return 1;
  if (env > 1) return std::max(1, std::min(env, nks / 8));
  const int bp = conv3d_fwd_bp(Cin, Cout, 0, G, Mg);
  const int64_t nwg = (int64_t)ceil_div(Mg, bp) * (Cout / fwd_bco(Cout)) * G;
  if (nwg >= 256 || nks < 24) return 1;
  return (int)std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(ceil_div(512, nwg), nks / 12), 8));
}

// positions per block (= per BN-statistics block) of conv3d_fwd for this layer shape and client count
int conv3d_fwd_bp(int Cin, int Cout, int xf, int G, int Mg) {
  if (xf || Cin % 64 != 0) return kFwdBP;
  const int bco = fwd_bco(Cout);
  const int64_t nwg256 = (int64_t)ceil_div(Mg, 256) * (Cout / bco) * G;
  static const int thresh = [] {
    const char* e = getenv("NIDT_FWD_BP_THRESH");
    return e ? atoi(e) : 256;
  }();
  if (nwg256 < thresh) return 64;  // fewer blocks than CUs: 64-position blocks (measured: only then a win)
  // one 4-wave 64-channel block per CU (e.g. conv3-5 at 8 clients per GPU: 264 blocks): 128-position blocks of
  // 2 waves put two blocks on every CU instead
  static const int bp128 = [] {
    const char* e = getenv("NIDT_FWD_BP128");
    return e ? atoi(e) : 1;
  }();
  if (bp128 && bco == 64 && nwg256 < 512) return 128;
  // large grids: 512-position blocks (16 waves for 128 channels, 160 KB of LDS) raise the MFMA work per byte of
  // LDS-DMA by 20 % and give each SIMD 4 waves.  NIDT_FWD_BP512=1 enables it (A/B).
  static const int bp512 = [] {
    const char* e = getenv("NIDT_FWD_BP512");
    return e ? atoi(e) : 0;
  }();
  if (bp512 && nwg256 >= 4096) return 512;
  return 256;
}

static int union_umax(int B, int D, int H, int W, int pad, int P, int ext = 2);
__global__ void k_union_table(int* tab, int U, int P, int Mg, int D, int H, int W, int pad, int ext);

static inline int ft_ucap(int umax) { return umax <= 320 ? 320 : (umax <= 384 ? 384 : 0); }

// k_conv_fwd_tri is used for this forward/dgrad (3x3x3 stride 1, 256-position blocks, union <= 384 rows, no split-K,
// and measured faster for the shape): NIDT_FWD_TRI=0 turns it off (A/B against k_conv_fwd_dma)
// the shape is supported by k_conv_fwd_tri (any client count; 256-position blocks)
int conv3d_fwd_tri_ok(int B, int D, int H, int W, int Cin, int Cout, int pad) {
  if (Cin % 64 != 0 || Cout % 64 != 0 || pad < 0 || pad > 2 || (int64_t)Cin * 27 > 27 * kMaxCin) return 0;
  const int Mg = B * (D + 2 * pad - 2) * (H + 2 * pad - 2) * (W + 2 * pad - 2);
  if (D + 2 * pad < 3 || H + 2 * pad < 3 || W + 2 * pad < 3 || Mg <= 0) return 0;
  return ft_ucap(union_umax(B, D, H, W, pad, 256)) > 0 ? 1 : 0;
}

int conv3d_fwd_tri_pick(int G, int B, int D, int H, int W, int Cin, int Cout, int pad) {
  static const int env = [] {
    const char* e = getenv("NIDT_FWD_TRI");
    return e ? atoi(e) : 1;
  }();
  if (!env || !conv3d_fwd_tri_ok(B, D, H, W, Cin, Cout, pad)) return 0;
  const int Mg = B * (D + 2 * pad - 2) * (H + 2 * pad - 2) * (W + 2 * pad - 2);
  if (conv3d_fwd_bp(Cin, Cout, 0, G, Mg) != 256 || conv3d_fwd_ksplit(Cin, Cout, G, Mg) > 1) return 0;
  const int U = ft_ucap(union_umax(B, D, H, W, pad, 256));
  // measured (profiles/r2_ab_fwd_tri.txt): conv2 fwd (unpadded) 3.25 -> 2.71 ms at 64 clients, 0.43 -> 0.34 at 8;
  // conv2 dgrad (pad 2, 320-row unions) 3.80 -> 3.67 on one box but 3.65 -> 3.68 on another (and 8-wave 64-channel
  // blocks 3.85), 0.48 -> 0.49 at 8 clients; the padded 5x7x5 convs (384-row unions) 5-25 % slower.  So: unpadded
  // convs only (the single union buffer's per-triplet reload is not hidden for the 4-wave 64-channel blocks).
  (void)U;
  return pad == 0 ? 1 : 0;
}

int conv3d_fwd_tri_table_size(int B, int D, int H, int W, int pad) {
  const int Mg = B * (D + 2 * pad - 2) * (H + 2 * pad - 2) * (W + 2 * pad - 2);
  const int U = ft_ucap(union_umax(B, D, H, W, pad, 256));
  NIDT_REQUIRE(U > 0, "conv3d_fwd_tri_table_size: shape not eligible");
  return ceil_div(Mg, 256) * (2 * U + 256);
}

void conv3d_fwd_tri_table(uintptr_t tab, int B, int D, int H, int W, int pad, uintptr_t stream) {
  const int Mg = B * (D + 2 * pad - 2) * (H + 2 * pad - 2) * (W + 2 * pad - 2);
  const int U = ft_ucap(union_umax(B, D, H, W, pad, 256));
  NIDT_REQUIRE(U > 0, "conv3d_fwd_tri_table: shape not eligible");
  NIDT_REQUIRE(D + 2 * pad < 1024 && H + 2 * pad < 1024 && W + 2 * pad < 1024, "conv3d_fwd_tri_table: extents < 1024");
  hipLaunchKernelGGL(k_union_table, dim3(ceil_div(Mg, 256)), dim3(256), 0, as_stream(stream), ptr<int>(tab), U, 256, Mg,
                     D, H, W, pad, 2);
  NIDT_CHECK(hipGetLastError());
}

// forward (bias + BN block statistics optional; bias rows at stride bias_ld, 0 = Cout) through k_conv_fwd_tri
void conv3d_fwd_tri(uintptr_t x, uintptr_t w, uintptr_t bias, int64_t bias_ld, uintptr_t y, uintptr_t stats, int G,
                    int B, int D, int H, int W, int Cin, int Cout, int pad, uintptr_t utab, uintptr_t stream) {
  NIDT_REQUIRE(conv3d_fwd_tri_ok(B, D, H, W, Cin, Cout, pad) && utab != 0, "conv3d_fwd_tri: shape not supported");
  NIDT_REQUIRE((int64_t)B * D * H * W * Cin * 2 < (1ll << 31), "conv3d_fwd_tri: per-client input below 2 GiB");
  const bool hb = bias != 0, st = stats != 0;
  NIDT_REQUIRE(!st || hb, "conv3d_fwd_tri: statistics require a bias");
  ConvFwdArgs a;
  a.x = ptr<const uint16_t>(x); a.w = ptr<const uint16_t>(w); a.bias = ptr<const float>(bias);
  a.xs = nullptr; a.xt = nullptr; a.y = ptr<uint16_t>(y); a.stats = ptr<float>(stats);
  a.B = B; a.D = D; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.pad = pad; a.padd = pad; a.kt = 27; a.st = 1;
  a.Do = D + 2 * pad - 2; a.Ho = H + 2 * pad - 2; a.Wo = W + 2 * pad - 2;
  a.Mg = B * a.Do * a.Ho * a.Wo;
  a.nPB = ceil_div(a.Mg, 256);
  a.G = G;
  a.bias_ld = bias_ld;
  const int U = ft_ucap(union_umax(B, D, H, W, pad, 256));
  const int bco = fwd_bco(Cout), nCO = Cout / bco;
  const dim3 grid((unsigned)((int64_t)a.nPB * nCO * G));
  hipStream_t s = as_stream(stream);
  const int* tab = ptr<const int>(utab);
#define NIDT_FT(BC, WM, UU, PD, BI, STT) \
  hipLaunchKernelGGL((k_conv_fwd_tri<BC, WM, 4, UU, PD, BI, STT>), grid, dim3(256 * WM), 0, s, a, nCO, tab)
#define NIDT_FT_B(BC, WM, UU, PD) \
  if (st) NIDT_FT(BC, WM, UU, PD, true, true); else if (hb) NIDT_FT(BC, WM, UU, PD, true, false); else NIDT_FT(BC, WM, UU, PD, false, false);
#define NIDT_FT_U(BC, WM)                                                                                        \
  if (pad) { if (U == 320) { NIDT_FT_B(BC, WM, 320, true) } else { NIDT_FT_B(BC, WM, 384, true) } }             \
  else { if (U == 320) { NIDT_FT_B(BC, WM, 320, false) } else { NIDT_FT_B(BC, WM, 384, false) } }
  if (bco == 128) { NIDT_FT_U(128, 2) } else { NIDT_FT_U(64, 1) }
#undef NIDT_FT_U
#undef NIDT_FT_B
#undef NIDT_FT
  NIDT_CHECK(hipGetLastError());
}

// ---- k_conv_fwd_slab host side (union rows <= 384 per 256-position band; ext = 2 Wp + 2) ----
// (512-position blocks, one 8-wave block per CU with 704-row unions, measured slower for the conv2 data gradient:
// 3.79 vs 3.28 ms, profiles/r3_ab_fwd_slab.txt — not kept)
static inline int slab_ext(int W, int pad) { return 2 * (W + 2 * pad) + 2; }
// union rows per band: 384, or 416 for 64-channel blocks (48 + 4 KB more LDS still leaves two blocks per CU: the
// 31x37x31 layer-1 convs of the 3D ResNet need up to 408)
static inline int slab_u(int B, int D, int H, int W, int pad) {
  const int um = union_umax(B, D, H, W, pad, 256, slab_ext(W, pad));
  return um <= 384 ? 384 : (um <= 416 ? 416 : 0);
}

// largest kd-slab union (rows) of a 256-position band: exposed for host-side tests of the slab rule
int conv3d_slab_umax(int B, int D, int H, int W, int pad) { return union_umax(B, D, H, W, pad, 256, slab_ext(W, pad)); }

int conv3d_fwd_slab_ok(int B, int D, int H, int W, int Cin, int Cout, int pad) {
  if (Cin % 64 != 0 || Cout % 64 != 0 || pad < 0 || pad > 2 || (int64_t)Cin * 27 > 27 * kMaxCin) return 0;
  const int Mg = B * (D + 2 * pad - 2) * (H + 2 * pad - 2) * (W + 2 * pad - 2);
  if (D + 2 * pad < 3 || H + 2 * pad < 3 || W + 2 * pad < 3 || Mg <= 0) return 0;
  if (D + 2 * pad >= 1024 || H + 2 * pad >= 1024 || W + 2 * pad >= 1024) return 0;
  const int U = slab_u(B, D, H, W, pad);
  return (U == 384 || (U == 416 && fwd_bco(Cout) == 64)) ? 1 : 0;
}

// Chosen for every eligible shape (measured, profiles/r3_ab_fwd_slab.txt, 64 clients: conv2 dgrad 3.60 -> 3.26 ms
// against the per-tap kernel, conv2 fwd 2.65 -> 2.52 ms against k_conv_fwd_tri).  NIDT_FWD_SLAB=0 turns it off,
// =1 keeps it to padded convs (A/B).
int conv3d_fwd_slab_pick(int G, int B, int D, int H, int W, int Cin, int Cout, int pad) {
  static const int env = [] {
    const char* e = getenv("NIDT_FWD_SLAB");
    return e ? atoi(e) : 2;
  }();
  if (!env || !conv3d_fwd_slab_ok(B, D, H, W, Cin, Cout, pad)) return 0;
  const int Mg = B * (D + 2 * pad - 2) * (H + 2 * pad - 2) * (W + 2 * pad - 2);
  if (conv3d_fwd_bp(Cin, Cout, 0, G, Mg) != 256 || conv3d_fwd_ksplit(Cin, Cout, G, Mg) > 1) return 0;
  return (pad > 0 || env == 2) ? 1 : 0;
}

int conv3d_fwd_slab_table_size(int B, int D, int H, int W, int pad) {
  const int Mg = B * (D + 2 * pad - 2) * (H + 2 * pad - 2) * (W + 2 * pad - 2);
  const int U = slab_u(B, D, H, W, pad);
  NIDT_REQUIRE(U > 0, "conv3d_fwd_slab_table_size: shape not eligible");
  return ceil_div(Mg, 256) * (2 * U + 256);
}

void conv3d_fwd_slab_table(uintptr_t tab, int B, int D, int H, int W, int pad, uintptr_t stream) {
  const int Mg = B * (D + 2 * pad - 2) * (H + 2 * pad - 2) * (W + 2 * pad - 2);
  const int U = slab_u(B, D, H, W, pad);
  NIDT_REQUIRE(U > 0, "conv3d_fwd_slab_table: shape not eligible");
  hipLaunchKernelGGL(k_union_table, dim3(ceil_div(Mg, 256)), dim3(256), 0, as_stream(stream), ptr<int>(tab), U, 256, Mg,
                     D, H, W, pad, slab_ext(W, pad));
  NIDT_CHECK(hipGetLastError());
}

static int slab_bd_u(int B, int H, int W, int bp = 256);

static void fwd_slab_impl(uintptr_t x, uintptr_t w, uintptr_t bias, int64_t bias_ld, uintptr_t y, uintptr_t stats,
                          int G, int B, int D, int H, int W, int Cin, int Cout, int pad, int kt, uintptr_t utab,
                          uintptr_t stream, int kd1 = 0, int bp = 256) {
  NIDT_REQUIRE((kd1 ? slab_bd_u(D, H, W, bp) > 0 : conv3d_fwd_slab_ok(B, D, H, W, Cin, Cout, pad)) && utab != 0,
               "conv3d_fwd_slab: shape not supported");
  NIDT_REQUIRE(bp == 256 || (bp == 128 && kd1 && !bias && !stats && Cout % 128 == 0),
               "conv3d_fwd_slab: 128-position blocks only for the depth-batched 2-D form, 128-channel blocks");
  NIDT_REQUIRE((int64_t)B * D * H * W * Cin * 2 < (1ll << 31), "conv3d_fwd_slab: per-client input below 2 GiB");
  const bool hb = bias != 0, st = stats != 0;
  NIDT_REQUIRE(!st || hb, "conv3d_fwd_slab: statistics require a bias");
  ConvFwdArgs a;
  a.x = ptr<const uint16_t>(x); a.w = ptr<const uint16_t>(w); a.bias = ptr<const float>(bias);
  a.xs = nullptr; a.xt = nullptr; a.y = ptr<uint16_t>(y); a.stats = ptr<float>(stats);
  a.B = B; a.D = D; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.pad = pad; a.padd = pad; a.kt = kt; a.st = 1;
  a.Do = D + 2 * pad - 2; a.Ho = H + 2 * pad - 2; a.Wo = W + 2 * pad - 2;
  a.Mg = B * a.Do * a.Ho * a.Wo;
  a.nPB = ceil_div(a.Mg, bp);
  a.G = G;
  a.bias_ld = bias_ld;
  static const int slab_dbg = [] {  // timing diagnostics only (wrong results): NIDT_SLAB_DBG=1 skips union reloads
    const char* e = getenv("NIDT_SLAB_DBG");
    return e ? atoi(e) : 0;
  }();
  a.dbg = slab_dbg;
  a.kd1 = kd1;
  if (bp == 128) {  // [SLAB-BD] 128-position bands (4x4 maps: 8 padded samples = 288 union rows)
    const int nCO = Cout / 128;
    const dim3 grid((unsigned)((int64_t)a.nPB * nCO * G));
    hipLaunchKernelGGL((k_conv_fwd_slab<128, 2, 2, 384, true, false, false, false>), grid, dim3(256), 0,
                       as_stream(stream), a, nCO, ptr<const int>(utab));
    NIDT_CHECK(hipGetLastError());
    return;
  }
  const int bco = (kd1 && slab_u(B, D, H, W, pad) == 416) ? 64 : fwd_bco(Cout), nCO = Cout / bco;
  const dim3 grid((unsigned)((int64_t)a.nPB * nCO * G));
  hipStream_t s = as_stream(stream);
  const int* tab = ptr<const int>(utab);
  static const int lswz = [] {  // NIDT_SLAB_LSWZ=1: output-space swizzle (A/B: no gain measured, see [LSWZ])
    const char* e = getenv("NIDT_SLAB_LSWZ");
    return e ? atoi(e) : 0;
  }();
  static const int na3 = [] {  // NIDT_SLAB_NA=3: three weight-tile stages for the 64-channel blocks (A/B)
    const char* e = getenv("NIDT_SLAB_NA");
    return e ? (atoi(e) == 3) : 0;
  }();
  // [SCHED] fragment schedule for the 64-channel blocks (AlexNet conv2 data gradient 3.25 -> 3.00 ms at 64 clients,
  // profiles/r4_ab_slab_sched.txt; the 128-channel blocks would need > 128 VGPRs and lose their second block per CU:
  // conv2 forward 2.55 -> 3.23 ms).  NIDT_SLAB_SCHED=0: the compiler's schedule (A/B); =2 adds [SCHED-half] on the
  // 128-channel blocks (A/B)
  static const int sched = [] {
    const char* e = getenv("NIDT_SLAB_SCHED");
    return e ? atoi(e) : 1;
  }();
#define NIDT_FS_U(BC, WM, UU, PD, BI, STT)                                                                        \
  if (lswz) hipLaunchKernelGGL((k_conv_fwd_slab<BC, WM, 4, UU, PD, BI, STT, true>), grid, dim3(256 * WM), 0, s, a,   \
                               nCO, tab);                                                                          \
  else if (na3 && BC == 64)                                                                                        \
    hipLaunchKernelGGL((k_conv_fwd_slab<BC, WM, 4, UU, PD, BI, STT, false, (BC == 64 ? 3 : 2)>), grid,            \
                       dim3(256 * WM), 0, s, a, nCO, tab);                                                         \
  else if (sched && BC == 64)                                                                                      \
    hipLaunchKernelGGL((k_conv_fwd_slab<BC, WM, 4, UU, PD, BI, STT, false, 2, (BC == 64 ? 1 : 0)>), grid,         \
                       dim3(256 * WM), 0, s, a, nCO, tab);                                                         \
  else if (sched == 2 && BC == 128 && !PD)                                                                         \
    hipLaunchKernelGGL((k_conv_fwd_slab<BC, WM, 4, UU, PD, BI, STT, false, 2, (BC == 128 && !PD ? 2 : 0)>), grid, \
                       dim3(256 * WM), 0, s, a, nCO, tab);                                                         \
  else hipLaunchKernelGGL((k_conv_fwd_slab<BC, WM, 4, UU, PD, BI, STT, false>), grid, dim3(256 * WM), 0, s, a, nCO, tab)
#define NIDT_FS_B(BC, WM, UU, PD)                                                                                  \
  if (st) NIDT_FS_U(BC, WM, UU, PD, true, true); else if (hb) NIDT_FS_U(BC, WM, UU, PD, true, false);            \
  else NIDT_FS_U(BC, WM, UU, PD, false, false);
  // (8-wave 64-channel blocks, two 32-channel halves: conv2 data gradient 3.49 vs 3.25 ms — more VALU per MFMA from
  // the duplicated B addressing; profiles/r4_ab_slab_sched.txt, not kept)
  if (bco == 128) {
    if (pad) { NIDT_FS_B(128, 2, 384, true) } else { NIDT_FS_B(128, 2, 384, false) }
  } else if (slab_u(B, D, H, W, pad) == 416) {
    if (pad) { NIDT_FS_B(64, 1, 416, true) } else { NIDT_FS_B(64, 1, 416, false) }
  } else {
    if (pad) { NIDT_FS_B(64, 1, 384, true) } else { NIDT_FS_B(64, 1, 384, false) }
  }
#undef NIDT_FS_B
#undef NIDT_FS_U
  NIDT_CHECK(hipGetLastError());
}

void conv3d_fwd_slab(uintptr_t x, uintptr_t w, uintptr_t bias, int64_t bias_ld, uintptr_t y, uintptr_t stats, int G,
                     int B, int D, int H, int W, int Cin, int Cout, int pad, uintptr_t utab, uintptr_t stream) {
  fwd_slab_impl(x, w, bias, bias_ld, y, stats, G, B, D, H, W, Cin, Cout, pad, 27, utab, stream);
}

// 2-D 3x3 stride-1 pad-1 convs (the CIFAR / Tiny ResNet-18 layers 1-2 and their data gradients) on the slab kernel:
// one union per 64-channel chunk serves all nine taps.  Weights [G][Cout][9][Cin]; the union table is
// conv3d_fwd_slab_table(B, 1, H, W, 1).  Eligible when every 256-position block lies inside one sample (H W % 256
// == 0, so the depth-tap skip keeps kd = 1 only) and the band unions fit.
int conv2d_fwd_slab_ok(int B, int H, int W, int Cin, int Cout) {
  return (H * W) % 256 == 0 && conv3d_fwd_slab_ok(B, 1, H, W, Cin, Cout, 1) ? 1 : 0;
}

// Chosen (measured per layer, profiles/r3_ab_conv2d_slab.txt, B = 16): 64-channel blocks always (0.77-1.01 of the
// per-tap kernel's time), 128-channel blocks once the grid has >= 160 of them (0.64-0.96; with 16-128 blocks the
// slab's one-block-per-CU grid loses to the per-tap kernel's 64-position / split-K blocks: 1.09-1.56).
// NIDT_2D_SLAB=0 turns it off, =2 forces it for every eligible shape (A/B).
int conv2d_fwd_slab_pick(int G, int B, int H, int W, int Cin, int Cout) {
  static const int env = [] {
    const char* e = getenv("NIDT_2D_SLAB");
    return e ? atoi(e) : 1;
  }();
  if (!env || !conv2d_fwd_slab_ok(B, H, W, Cin, Cout)) return 0;
  const int bco = fwd_bco(Cout);
  const int64_t blocks = (int64_t)ceil_div(B * H * W, 256) * (Cout / bco) * G;
  return (env == 2 || bco == 64 || blocks >= 160) ? 1 : 0;
}

void conv2d_fwd_slab(uintptr_t x, uintptr_t w, uintptr_t y, int G, int B, int H, int W, int Cin, int Cout,
                     uintptr_t utab, uintptr_t stream) {
  NIDT_REQUIRE(conv2d_fwd_slab_ok(B, H, W, Cin, Cout), "conv2d_fwd_slab: shape not supported");
  fwd_slab_impl(x, w, 0, 0, y, 0, G, B, 1, H, W, Cin, Cout, 1, 9, utab, stream);
}

// [GN-EPI] the same conv with the per-block channel statistics (mean, M2 over the block's 256 positions, from the fp32
// accumulators) written to stats [G][nPB][Cout][2] by the shared epilogue: every block lies inside one sample (H W %
// 256 == 0), so a sample's blocks pb = n (H W / 256) .. are its GroupNorm partials (gn.hip gn_apply).  The epilogue's
// statistics need its bias path: zb is a [G][Cout] zero bias (the ResNet convs have none)
void conv2d_fwd_slab_stats(uintptr_t x, uintptr_t w, uintptr_t zb, uintptr_t y, uintptr_t stats, int G, int B, int H,
                           int W, int Cin, int Cout, uintptr_t utab, uintptr_t stream) {
  NIDT_REQUIRE(conv2d_fwd_slab_ok(B, H, W, Cin, Cout) && zb != 0 && stats != 0, "conv2d_fwd_slab_stats: shape");
  fwd_slab_impl(x, w, zb, 0, y, stats, G, B, 1, H, W, Cin, Cout, 1, 9, utab, stream);
}

// [SLAB-BD] 2-D 3x3 stride-1 pad-1 convs on maps whose 256-position blocks span several samples (8x8: four samples
// per block; the CIFAR / Tiny ResNet-18 layer 3 and the 16x16 / 8x8 maps of the Tiny layers): the client's B samples
// are the depth planes of ONE volume [1][B][H][W] and the conv is the 3-D slab conv restricted to depth tap kd = 1
// (k_conv_fwd_slab with a.kd1): plane d reads only plane d, i.e. each sample's own 2-D conv, and one union of
// consecutive whole padded planes (4 x 100 rows for 8x8 maps) serves the block's nine taps.  Eligible when the union
// fits (416 rows: 64-channel blocks).
// bp = 256: the slab kernel's union sizes (384 / 416 rows); bp = 128 (4x4 maps, 128-channel blocks): <= 384 rows
static int slab_bd_u(int B, int H, int W, int bp) {
  if (B + 2 >= 1024 || H + 2 >= 1024 || W + 2 >= 1024) return 0;
  if (bp == 128) return union_umax(1, B, H, W, 1, 128, slab_ext(W, 1)) <= 384 ? 384 : 0;
  return slab_u(1, B, H, W, 1);
}

// block positions of the depth-batched form for a shape (256, 128, or 0 = not eligible)
static int slab_bd_bp(int B, int H, int W, int Cin, int Cout) {
  if (Cin % 64 != 0 || Cout % 64 != 0 || Cin > kMaxCin || (H * W) % 256 == 0) return 0;
  if (slab_bd_u(B, H, W, 256) > 0) return 256;
  return (Cout % 128 == 0 && slab_bd_u(B, H, W, 128) > 0) ? 128 : 0;
}

int conv2d_fwd_slab_bd_ok(int B, int H, int W, int Cin, int Cout) { return slab_bd_bp(B, H, W, Cin, Cout) > 0 ? 1 : 0; }

// Chosen for every eligible 256-position shape: CIFAR layer-3 convs 0.158 -> 0.129 ms at 100 clients x 16, 0.625 ->
// 0.502 ms at 100 x 62 (764 -> 934 TF/s), 0.032 -> 0.031 at 10 x 16; the 128-position form (4x4 maps) from 512 blocks
// (tools/bench_conv2d.py, profiles/r5_slab_bd.txt).
// NIDT_2D_SLAB_BD=0 keeps the per-tap kernel (A/B)
int conv2d_fwd_slab_bd_pick(int G, int B, int H, int W, int Cin, int Cout) {
  static const int env = [] {
    const char* e = getenv("NIDT_2D_SLAB_BD");
    return e ? atoi(e) : 1;
  }();
  const int bp = env ? slab_bd_bp(B, H, W, Cin, Cout) : 0;
  if (bp == 128) {  // one 8-wave block per band and 128 channels: small grids lose to the per-tap kernel's split-K
    // (4x4 maps at 10 clients x 16: 0.041 -> 0.062 ms; at 100 x 16: 0.193 -> 0.177; 100 x 62: 0.615 -> 0.548)
    const int64_t blocks = (int64_t)ceil_div(B * H * W, 128) * (Cout / 128) * G;
    return blocks >= 512 ? 1 : 0;
  }
  return bp > 0 ? 1 : 0;
}

// union tables per (B, H, W, block positions): the caller passes the Cin / Cout of the layer so the same blocking is
// chosen here and in conv2d_fwd_slab_bd
int conv2d_fwd_slab_bd_table_size(int B, int H, int W, int Cin, int Cout) {
  const int bp = slab_bd_bp(B, H, W, Cin, Cout);
  NIDT_REQUIRE(bp > 0, "conv2d_fwd_slab_bd_table_size: shape not eligible");
  if (bp == 256) return conv3d_fwd_slab_table_size(1, B, H, W, 1);
  return ceil_div(B * H * W, 128) * (2 * 384 + 128);
}

void conv2d_fwd_slab_bd_table(uintptr_t tab, int B, int H, int W, int Cin, int Cout, uintptr_t stream) {
  const int bp = slab_bd_bp(B, H, W, Cin, Cout);
  NIDT_REQUIRE(bp > 0, "conv2d_fwd_slab_bd_table: shape not eligible");
  if (bp == 256) {
    conv3d_fwd_slab_table(tab, 1, B, H, W, 1, stream);
    return;
  }
  const int Mg = B * H * W;
  hipLaunchKernelGGL(k_union_table, dim3(ceil_div(Mg, 128)), dim3(256), 0, as_stream(stream), ptr<int>(tab), 384, 128,
                     Mg, B, H, W, 1, slab_ext(W, 1));
  NIDT_CHECK(hipGetLastError());
}

void conv2d_fwd_slab_bd(uintptr_t x, uintptr_t w, uintptr_t y, int G, int B, int H, int W, int Cin, int Cout,
                        uintptr_t utab, uintptr_t stream) {
  const int bp = slab_bd_bp(B, H, W, Cin, Cout);
  NIDT_REQUIRE(bp > 0, "conv2d_fwd_slab_bd: shape not supported");
  fwd_slab_impl(x, w, 0, 0, y, 0, G, 1, B, H, W, Cin, Cout, 1, 9, utab, stream, 1, bp);
}

// ---- k_conv_fwd_vol host side (whole padded sample <= 448 rows, <= 256 output positions per sample) ----
constexpr int kVolU = 448;
int conv3d_fwd_vol_ok(int B, int D, int H, int W, int Cin, int Cout, int pad) {
  if (Cin % 64 != 0 || Cout % 64 != 0 || pad < 0 || pad > 2 || Cin > kMaxCin || B < 1) return 0;
  const int Do = D + 2 * pad - 2, Ho = H + 2 * pad - 2, Wo = W + 2 * pad - 2;
  if (Do < 1 || Ho < 1 || Wo < 1 || Do * Ho * Wo > 256) return 0;
  return (D + 2 * pad) * (H + 2 * pad) * (W + 2 * pad) <= kVolU ? 1 : 0;
}

// Opt-in (NIDT_FWD_VOL=1): measured slower than the per-tap kernel for the 5x7x5 conv3-5 at 64 clients (fwd + dgrad
// 2.19 vs 1.71 ms per step: 3-wave blocks, one exposed weight-tile wait per tap) and within 1 % at 8 clients
// (profiles/r3_ab_fwd_vol.txt).  When enabled: grids of >= NIDT_FWD_VOL_MINB (256) blocks without split-K.
int conv3d_fwd_vol_pick(int G, int B, int D, int H, int W, int Cin, int Cout, int pad) {
  static const int env = [] {
    const char* e = getenv("NIDT_FWD_VOL");
    return e ? atoi(e) : 0;
  }();
  static const int minb = [] {
    const char* e = getenv("NIDT_FWD_VOL_MINB");
    return e ? atoi(e) : 256;
  }();
  if (!env || !conv3d_fwd_vol_ok(B, D, H, W, Cin, Cout, pad)) return 0;
  const int Mg = B * (D + 2 * pad - 2) * (H + 2 * pad - 2) * (W + 2 * pad - 2);
  if (conv3d_fwd_ksplit(Cin, Cout, G, Mg) > 1) return 0;
  return (int64_t)G * B * (Cout / 64) >= minb ? 1 : 0;
}

void conv3d_fwd_vol(uintptr_t x, uintptr_t w, uintptr_t bias, int64_t bias_ld, uintptr_t y, uintptr_t stats, int G,
                    int B, int D, int H, int W, int Cin, int Cout, int pad, uintptr_t stream) {
  NIDT_REQUIRE(conv3d_fwd_vol_ok(B, D, H, W, Cin, Cout, pad), "conv3d_fwd_vol: shape not supported");
  NIDT_REQUIRE((int64_t)B * D * H * W * Cin * 2 < (1ll << 31), "conv3d_fwd_vol: per-client input below 2 GiB");
  const bool hb = bias != 0, st = stats != 0;
  NIDT_REQUIRE(!st || hb, "conv3d_fwd_vol: statistics require a bias");
  ConvFwdArgs a;
  a.x = ptr<const uint16_t>(x); a.w = ptr<const uint16_t>(w); a.bias = ptr<const float>(bias);
  a.xs = nullptr; a.xt = nullptr; a.y = ptr<uint16_t>(y); a.stats = ptr<float>(stats);
  a.B = B; a.D = D; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.pad = pad; a.padd = pad; a.kt = 27; a.st = 1;
  a.Do = D + 2 * pad - 2; a.Ho = H + 2 * pad - 2; a.Wo = W + 2 * pad - 2;
  a.Mg = B * a.Do * a.Ho * a.Wo;
  a.nPB = B;  // statistics blocks = samples
  a.G = G;
  a.bias_ld = bias_ld;
  const int S = a.Do * a.Ho * a.Wo, wn = ceil_div(S, 64), nCO = Cout / 64;
  static const int wm = [] {
    const char* e = getenv("NIDT_FWD_VOL_WM");
    return e ? atoi(e) : 1;
  }();
  const dim3 grid((unsigned)((int64_t)G * B * nCO));
  hipStream_t s = as_stream(stream);
#define NIDT_FV(WM, WN, BI, STT) \
  hipLaunchKernelGGL((k_conv_fwd_vol<64, WM, WN, kVolU, BI, STT>), grid, dim3(64 * WM * WN), 0, s, a, nCO)
#define NIDT_FV_B(WM, WN) \
  if (st) NIDT_FV(WM, WN, true, true); else if (hb) NIDT_FV(WM, WN, true, false); else NIDT_FV(WM, WN, false, false);
#define NIDT_FV_N(WM) \
  if (wn == 1) { NIDT_FV_B(WM, 1) } else if (wn == 2) { NIDT_FV_B(WM, 2) } else if (wn == 3) { NIDT_FV_B(WM, 3) } else { NIDT_FV_B(WM, 4) }
  if (wm == 2) { NIDT_FV_N(2) } else { NIDT_FV_N(1) }
#undef NIDT_FV_N
#undef NIDT_FV_B
#undef NIDT_FV
  NIDT_CHECK(hipGetLastError());
}

int conv3d_fwd_nblocks(int B, int D, int H, int W, int pad, int bp) {
  const int Mg = B * (D + 2 * pad - 2) * (H + 2 * pad - 2) * (W + 2 * pad - 2);
  return ceil_div(Mg, bp);
}

// ------------------------------------------------------------------------------------------------
// wgrad
struct ConvWgArgs {
  const uint16_t* x;    // [G*B, D, H, W, Cin]
  const float* xs;      // transform or null
  const float* xt;
  const uint16_t* dy;   // [G*B, Do, Ho, Wo, Cout]
  float* part;          // [nsplit, G, Cout, K]
  int B, D, H, W, Cin, Do, Ho, Wo, Cout, pad, Mg, K, nsplit, chunk, G;
};

constexpr int kWgCO = 64;    // co per block
constexpr int kWgKC = 256;   // k columns per block (4 waves x 64)

// swizzles of the [32 pos][64 co] (128-B rows) and [32 pos][256 k] (512-B rows) tiles, in 32-B segments
__device__ __forceinline__ int swz_dy(int r) { return ((r >> 1) & 1) | (((r >> 3) & 1) << 1); }
__device__ __forceinline__ int swz_x(int r) { return (r & 3) | (((r >> 3) & 1) << 2); }

__device__ __forceinline__ bf16x8 tr_pair(const uint16_t* p0, const uint16_t* p1) {
  typedef short v4s __attribute__((ext_vector_type(4)));
  v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p0));
  v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p1));
  typedef short v8s __attribute__((ext_vector_type(8)));
  v8s r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

template <bool XF>
__global__ __launch_bounds__(256, 2) void k_conv_wgrad(ConvWgArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t sD[2][32 * kWgCO];
  __shared__ __attribute__((aligned(16))) uint16_t sX[2][32 * kWgKC];
  __shared__ float sXS[XF ? 192 : 1], sXT[XF ? 192 : 1];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int kc0 = blockIdx.x * kWgKC;
  const int co0 = blockIdx.y * kWgCO;
  const int g = blockIdx.z / a.nsplit, sp = blockIdx.z - g * a.nsplit;
  const int p_begin = sp * a.chunk, p_end = min(a.Mg, p_begin + a.chunk);
  const int Cin = a.Cin;
  if (XF) {
    for (int i = tid; i < Cin; i += 256) {
      sXS[i] = a.xs[(int64_t)g * Cin + i];
      sXT[i] = a.xt[(int64_t)g * Cin + i];
    }
    __syncthreads();
  }
  const int S = a.Do * a.Ho * a.Wo;
  const int lrow = tid >> 3, lch = tid & 7;  // loader: row (position) and 16-B chunk
  // the x-tile chunks of this thread: columns kc0 + 8*(lch + 8u), u = 0..3 -> (tap, ci)
  int xt_[4], xc_[4];
  bool xk_[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int kk = kc0 + 8 * (lch + 8 * u);
    xk_[u] = kk < a.K;
    xt_[u] = xk_[u] ? kk / Cin : 0;
    xc_[u] = xk_[u] ? kk - xt_[u] * Cin : 0;
  }
  uint4 rD, rX[4];
  auto load = [&](int p0) {
    const int m = p0 + lrow;
    const bool mv = m < p_end;
    const int mm = mv ? m : p_begin;
    const int nl = mm / S, s = mm - nl * S;
    const int n = g * a.B + nl;
    const int od = s / (a.Ho * a.Wo), r = s - od * a.Ho * a.Wo, oh = r / a.Wo, ow = r - oh * a.Wo;
    rD = mv ? *reinterpret_cast<const uint4*>(a.dy + ((int64_t)g * a.Mg + mm) * a.Cout + co0 + 8 * lch)
            : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int t = xt_[u];
      const int id = od + t / 9 - a.pad, ih = oh + (t / 3) % 3 - a.pad, iw = ow + t % 3 - a.pad;
      const bool ok = mv && xk_[u] && id >= 0 && id < a.D && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (ok) v = *reinterpret_cast<const uint4*>(a.x + ((((int64_t)n * a.D + id) * a.H + ih) * a.W + iw) * Cin + xc_[u]);
      if (XF) v = xform8(v, sXS + xc_[u], sXT + xc_[u], ok);
      rX[u] = v;
    }
  };
  auto store = [&](int buf) {
    {
      const int seg = lch >> 1, half = lch & 1;
      const int pc = (((seg ^ swz_dy(lrow)) << 1) | half);
      *reinterpret_cast<uint4*>(&sD[buf][lrow * kWgCO + pc * 8]) = rD;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int ch = lch + 8 * u, seg = ch >> 1, half = ch & 1;
      const int pc = (((seg ^ swz_x(lrow)) << 1) | half);
      *reinterpret_cast<uint4*>(&sX[buf][lrow * kWgKC + pc * 8]) = rX[u];
    }
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed-read addressing: 16-lane group gq = lane>>4 covers positions 8*gq .. 8*gq+7 (two reads of 4 rows);
  // within the group lane 4*qq+pp supplies row (qq) and columns 4*pp..4*pp+3 of a 16-column segment.
  const int gq = lane >> 4, li = lane & 15, qq = li >> 2, pp = li & 3;
  const int r0 = 8 * gq + qq, r1 = r0 + 4;
  const int nsteps = (p_end - p_begin + 31) / 32;
  if (nsteps > 0) {
    load(p_begin);
    store(0);
    __syncthreads();
  }
  for (int st = 0; st < nsteps; ++st) {
    const int cur = st & 1;
    if (st + 1 < nsteps) load(p_begin + 32 * (st + 1));
    bf16x8 fa[4], fb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // A = dy^T: co segment i (16 co) -> 32-B segment i of the dy row
      const uint16_t* p0 = &sD[cur][r0 * kWgCO + ((i ^ swz_dy(r0)) << 4) + 4 * pp];
      const uint16_t* p1 = &sD[cur][r1 * kWgCO + ((i ^ swz_dy(r1)) << 4) + 4 * pp];
      fa[i] = tr_pair(p0, p1);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // B = patches: wave's 64 columns = segments 4*wid + j
      const int sg = 4 * wid + j;
      const uint16_t* p0 = &sX[cur][r0 * kWgKC + ((sg ^ swz_x(r0)) << 4) + 4 * pp];
      const uint16_t* p1 = &sX[cur][r1 * kWgKC + ((sg ^ swz_x(r1)) << 4) + 4 * pp];
      fb[j] = tr_pair(p0, p1);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    if (st + 1 < nsteps) store(cur ^ 1);
    __syncthreads();
  }
  // store partial slab: C[co = 16 i + 4 fq + r][k = 16 j + fr]
  const int fr = lane & 15, fq = lane >> 4;
  float* out = a.part + (((int64_t)sp * a.G + g) * a.Cout + co0) * a.K;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = kc0 + 64 * wid + 16 * j + fr;
    if (k < a.K) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) out[(int64_t)(16 * i + 4 * fq + r) * a.K + k] = acc[i][j][r];
    }
  }
}

// sum the split slabs; write PyTorch layout grad[g][off + (co*Cin + ci)*27 + t] for k = t*Cin + ci (scaled).
// Block = (co, g): the K-row is summed into LDS (16-B loads), then written out in [ci][t] order (coalesced).
// The LDS row is padded to a (Cin + 1) stride per tap: the transposed read row[t][ci] with t fastest across
// lanes would otherwise hit one bank ~27 times (Cin is a multiple of 32).  Dynamic LDS sized to the layer
// (27 (Cin + 1) floats) instead of the 512-channel maximum: more resident blocks to cover the HBM latency.
__global__ __launch_bounds__(256) void k_wgrad_reduce(const float* __restrict__ part, int nsplit, int G, int Cout,
                                                      int Cin, int kt, float* grad, int64_t ldg, int64_t off,
                                                      float scale) {
  extern __shared__ float row[];  // [kt][Cin + 1]
  const int co = blockIdx.x, g = blockIdx.y;
  const int K = kt * Cin, RS = Cin + 1;
  const int64_t tot = (int64_t)G * Cout * K;
  const float* src = part + ((int64_t)g * Cout + co) * K;  // 16-B aligned: K = 27 * 64 * n
  for (int k = 4 * threadIdx.x; k < K; k += 4 * 256) {
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int sp = 0; sp < nsplit; ++sp) {
      const float4 v = *reinterpret_cast<const float4*>(src + (int64_t)sp * tot + k);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    const int t = k / Cin, ci = k - t * Cin;  // k .. k+3 share the tap (Cin % 4 == 0)
    float* r = row + t * RS + ci;
    r[0] = s.x * scale; r[1] = s.y * scale; r[2] = s.z * scale; r[3] = s.w * scale;
  }
  __syncthreads();
  float* dst = grad + (int64_t)g * ldg + off + (int64_t)co * K;
  for (int e = threadIdx.x; e < K; e += 256) {
    const int ci = e / kt, t = e - ci * kt;
    dst[e] = row[t * RS + ci];
  }
}

void k_wgrad_reduce_launch(const float* part, int nsplit, int G, int Cout, int Cin, int kt, float* grad, int64_t ldg,
                           int64_t off, float scale, hipStream_t s) {
  hipLaunchKernelGGL(k_wgrad_reduce, dim3(Cout, G), dim3(256), kt * (Cin + 1) * sizeof(float), s, part, nsplit, G, Cout,
                     Cin, kt, grad, ldg, off, scale);
  NIDT_CHECK(hipGetLastError());
}

// 1x1x1 stride-1 weight gradients on the streaming kernel of wgrad1x1.hip (default); NIDT_WG1X1=0 keeps them on
// k_conv_wgrad_dma (A/B)
int wgrad1x1_ok(int N, int K);
int wgrad1x1_chunks(int G, int64_t Mg, int N, int K);
void wgrad1x1_g(uintptr_t x, uintptr_t dy, uintptr_t part, uintptr_t grad, int64_t ldg, int64_t off, int G, int64_t Mg,
                int N, int K, int nMB, float scale, uintptr_t stream);
static bool wg1x1_on(int Cin, int Cout, int kt, int st) {
  static const bool on = [] {
    const char* e = getenv("NIDT_WG1X1");
    return !(e && e[0] == '0');
  }();
  return on && kt == 1 && st == 1 && wgrad1x1_ok(Cout, Cin);
}

// Split-K factor for the wgrad: blocks are equally long (chunk positions each), so the run time is
// waves x block time with waves = ceil(blocks / slots), slots = 256 CUs x 2 resident blocks (80 KB LDS each),
// plus the fp32 slab traffic (ns x G x Cout x K, written once and read once by k_wgrad_reduce).  The model
// (one 64-position step ~1.28 us per block slot, ~12 steps of prologue/epilogue, ~5 TB/s slab traffic) picks the
// ns with the smallest estimate; ties go to the smaller ns.  NIDT_WG_NSPLIT_LEGACY=1 restores the old rule
// (ceil(2048 / tiles), capped) for A/B measurements.
static int wgrad_nsplit_mk(int G, int Mg, int K, int Cout);

int conv3d_wgrad_nsplit(int G, int B, int D, int H, int W, int Cin, int Cout, int pad) {
  return wgrad_nsplit_mk(G, B * (D + 2 * pad - 2) * (H + 2 * pad - 2) * (W + 2 * pad - 2), 27 * Cin, Cout);
}

int conv_wgrad_nsplit_g(int G, int B, int D, int H, int W, int Cin, int Cout, int kt, int st, int pad, int padd) {
  const int kd = kt == 27 ? 3 : 1, khw = kt == 1 ? 1 : 3;
  const int Mg = B * conv_out_dim(D, kd, st, padd) * conv_out_dim(H, khw, st, pad) * conv_out_dim(W, khw, st, pad);
  if (wg1x1_on(Cin, Cout, kt, st) && pad == 0) return wgrad1x1_chunks(G, Mg, Cout, Cin);
  return wgrad_nsplit_mk(G, Mg, kt * Cin, Cout);
}

static int wgrad_nsplit_base(int base, int G, int Mg, int K, int Cout, double step_us, double overhead_steps,
                             double slots);

static int wgrad_nsplit_mk(int G, int Mg, int K, int Cout) {
  return wgrad_nsplit_base(G * (Cout / kWgCO) * ceil_div(K, kWgKC), G, Mg, K, Cout, 1.28, 12.0, 512.0);
}

// base = output tiles (blocks per split) of the wgrad kernel in use; step_us / overhead_steps = its cost per
// 64-position step per block slot and its fixed cost in steps
static int wgrad_nsplit_base(int base, int G, int Mg, int K, int Cout, double step_us, double overhead_steps,
                             double slots) {
  static const bool legacy = [] {
    const char* e = getenv("NIDT_WG_NSPLIT_LEGACY");
    return e && e[0] == '1';
  }();
  static const int force = [] {  // A/B experiments only: one split factor for every layer
    const char* e = getenv("NIDT_WG_NSPLIT_FORCE");
    return e ? atoi(e) : 0;
  }();
  if (force > 0) return std::max(1, std::min(force, std::max(1, Mg / 64)));
  if (legacy) {
    const int ns = ceil_div(2048, base);
    const int maxns = max(1, Mg / (K >= 3000 ? 1024 : 512));
    return max(1, min(ns, maxns));
  }
  constexpr double kBytesPerUs = 5.0e6;
  const double kSlots = slots;  // resident blocks chip-wide
  const double kStepUs = step_us, kOverheadSteps = overhead_steps;
  const double slab_bytes = 8.0 * G * Cout * K;  // fp32 write + read per split
  const int maxns = max(1, min(64, Mg / 512));  // keep >= 8 steps per block
  int best = 1;
  double best_t = 1e30;
  for (int ns = 1; ns <= maxns; ++ns) {
    const double waves = ceil((double)base * ns / kSlots);
    const double steps = ceil(ceil((double)Mg / ns) / 64.0);
    const double t = waves * (steps + kOverheadSteps) * kStepUs + ns * slab_bytes / kBytesPerUs;
    if (t < best_t * 0.995) {
      best_t = t;
      best = ns;
    }
  }
  return best;
}

// ------------------------------------------------------------------------------------------------
// k_conv_wgrad_dma — dW[co][k] = sum_pos dY[pos][co] * X[pos + tap(k)][ci(k)], 64 positions per k-step,
// both tiles filled by global_load_lds.  A block owns 64 co x 256 k-cols = 4 "groups" of 64 k-cols (each
// group is one tap x 64 input channels, a 128-B row per position, so every glds wave-instruction reads
// 8 whole 128-B rows: coalesced).  Wave w stages X group w (8 instructions, rows 8i + lane/8) and two of
// the eight 8-row slices of dY.  The MFMA operands want the position axis in the k slots: they are read
// with ds_read_b64_tr_b16 (4 positions x 4 channels per lane).  Rows are 128 B, so the 16-B chunk index is
// XORed with f(r) = bit1(r)<<1 | bit3(r)<<2 (applied to the glds SOURCE address, undone on the read): every
// 32-lane group of a tr read then hits 32 distinct 8-B bank slots.  Position table (k_conv_pos_table): per
// client-local output position, the input-voxel offset of tap 0 and the 27-bit in-bounds tap mask; one
// global load per lane per step, distributed to the 8 rows a lane stages with __shfl.
struct ConvWgDmaArgs {
  const uint16_t* x;    // [G*B, D, H, W, Cin]
  const uint16_t* dy;   // [G*B, Do, Ho, Wo, Cout] == [G, Mg, Cout]
  const int2* ptab;     // [Mg] {input voxel offset of tap (0,0,0) relative to the client's first voxel, tap mask}
  float* part;          // [nsplit, G, Cout, K]
  int D, H, W, Cin, Cout, Mg, K, nsplit, chunk, G, nKT, nCT;
  int64_t xclient;      // elements per client in x (B*D*H*W*Cin)
  // nsplit == 1: the epilogue writes the PyTorch-layout gradient rows itself (grad[g][off + (co*Cin + ci)*kt + t],
  // times scale) and k_wgrad_reduce is skipped; null -> fp32 slabs into part
  float* grad;
  int64_t ldg, off;
  float scale;
  int kt;
};

__global__ void k_conv_pos_table(int2* tab, int Mg, int D, int H, int W, int Do, int Ho, int Wo, int st, int padd,
                                 int pad) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= Mg) return;
  const int S = Do * Ho * Wo;
  const int nl = m / S, s = m - nl * S;
  const int od = s / (Ho * Wo), r = s - od * Ho * Wo, oh = r / Wo, ow = r - oh * Wo;
  const int d0 = od * st - padd, h0 = oh * st - pad, w0 = ow * st - pad;
  uint32_t mask = 0;
  mask = tap_mask3(d0, h0, w0, D, H, W);
  tab[m] = make_int2(((nl * D + d0) * H + h0) * W + w0, (int)mask);
}

constexpr int kWdPos = 64;                       // positions per k-step
constexpr int kWdRow = 64;                       // bf16 per 128-B row
constexpr int kWdGroup = kWdPos * kWdRow;        // one 64-col group: 8 KB
constexpr int kWdBuf = 5 * kWdGroup;             // 4 X groups + dY
__device__ __forceinline__ int swz_wd(int r) { return (r & 2) | ((r >> 1) & 4); }

// NCH = 64-channel output halves per block: 1 -> 4 waves (64 co x 256 k-cols), 2 -> 8 waves (128 co x 256 k-cols:
// the X tile of a k-step feeds twice the MFMAs, 48 KB of LDS-DMA per 256 MFMAs instead of 40 KB per 128).
// Wave (wc, wk) = (wid / 4, wid % 4) computes co half wc x X group wk; it stages 8/NCH of group wk's 8 X
// instructions and dY half wc's slices 2wk, 2wk+1.
// [ADMA] as k_conv_wgrad_tri: the stage DMA from inline asm, the position-table loads issued before it
template <int NCH, bool SCHED = false, bool ADMA = false>
__global__ __launch_bounds__(256 * NCH, 2 / NCH) void k_conv_wgrad_dma(ConvWgDmaArgs a) {
  constexpr int BUFE = (4 + NCH) * kWdGroup;  // elements per stage: 4 X groups + NCH dY halves
  constexpr int XI = 8 / NCH;                  // X instructions per wave per stage
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * BUFE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: LDS destinations stay in SGPRs
  const int wc = wid >> 2, wk = wid & 3;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int kt = id % a.nKT, r1 = id / a.nKT;
  const int ct = r1 % a.nCT, r2 = r1 / a.nCT;
  const int sp = r2 % a.nsplit, g = r2 / a.nsplit;
  const int kc0 = kt * kWgKC, co0 = ct * (kWgCO * NCH);
  const int p_begin = sp * a.chunk, p_end = min(a.Mg, p_begin + a.chunk);
  const int Cin = a.Cin;
  const i32x4_t rx = make_rsrc(a.x + (int64_t)g * a.xclient, (uint32_t)(a.xclient * 2));
  const i32x4_t rd = make_rsrc(a.dy + (int64_t)g * a.Mg * a.Cout, (uint32_t)((int64_t)a.Mg * a.Cout * 2));
  const i32x4_t rt = make_rsrc(a.ptab, (uint32_t)a.Mg * 8u);  // rows past Mg read {0, mask 0}: no taps valid
  // this wave's X group: k-cols kc0 + 64 wk .. +63 = one tap, 64 channels
  const int kg = kc0 + 64 * wk;
  const bool gval = kg < a.K;
  const int gtap = gval ? kg / Cin : 31;  // 31: never set in a tap mask -> out-of-range read -> zeros
  const int gcol = gval ? (((gtap / 9) * a.H + (gtap / 3) % 3) * a.W + gtap % 3) * Cin + (kg - gtap * Cin) : 0;
  const int lr = lane >> 3, ls = lane & 7;
  const int xi0 = wc * XI;  // this wave's first X instruction (row block) of group wk
  // per-lane constant parts of the byte offsets: X row r = 8i + lr, chunk (ls ^ swz(r)); dY likewise
  int xcol[XI], dcol[2];
#pragma unroll
  for (int i = 0; i < XI; ++i) xcol[i] = (gcol + ((ls ^ swz_wd(8 * (xi0 + i) + lr)) << 3)) * 2;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = 8 * (2 * wk + i) + lr;
    dcol[i] = (r * a.Cout + co0 + 64 * wc + ((ls ^ swz_wd(r)) << 3)) * 2;
  }
  i32x2_t tn[XI];  // ptab entries {voxel offset, tap mask} of this lane's X rows, one step ahead
#define WD_FETCH(P0)                                                                                          \
  {                                                                                                           \
    _Pragma("unroll") for (int i_ = 0; i_ < XI; ++i_)                                                         \
      tn[i_] = nidt_raw_buffer_load_v2i32(rt, ((P0) + 8 * (xi0 + i_) + lr) * 8, 0, 0);                        \
  }
  auto wd_dma = [](i32x4_t r, int off, uint16_t* dst) {
    if constexpr (ADMA) blds16_asm(r, off, dst);
    else blds16(r, off, dst);
  };
#define WD_ISSUE_T(P0, BUFI, TN)                                                                              \
  {                                                                                                           \
    uint16_t* sX_ = smem + (BUFI) * BUFE + wk * kWdGroup;                                                     \
    uint16_t* sD_ = smem + (BUFI) * BUFE + (4 + wc) * kWdGroup;                                               \
    _Pragma("unroll") for (int i_ = 0; i_ < XI; ++i_) {                                                       \
      const bool ok_ = (TN[i_].y >> gtap) & 1;                                                                \
      wd_dma(rx, ok_ ? TN[i_].x * (2 * Cin) + xcol[i_] : kBufOOB, sX_ + (xi0 + i_) * 512);                    \
    }                                                                                                         \
    _Pragma("unroll") for (int i_ = 0; i_ < 2; ++i_)                                                          \
      wd_dma(rd, (P0) * (2 * a.Cout) + dcol[i_], sD_ + (2 * wk + i_) * 512);                                  \
  }
#define WD_ISSUE(P0, BUFI) WD_ISSUE_T(P0, BUFI, tn)

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed reads: 16-lane group gq covers positions 8gq..8gq+7 (two 4-row reads); lane 4qq+pp reads row qq,
  // columns 4pp..4pp+3 of a 16-column segment s = chunks 2s + (pp >> 1), half (pp & 1).
  const int gq = lane >> 4, li = lane & 15, qq = li >> 2, pp = li & 3;
  const int rr0 = 8 * gq + qq, rr1 = rr0 + 4;
  const int nsteps = (p_end - p_begin + kWdPos - 1) / kWdPos;
  if (nsteps > 0) {
    WD_FETCH(p_begin)
    WD_ISSUE(p_begin, 0)
    if (nsteps > 1) WD_FETCH(p_begin + kWdPos)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int st = 0; st < nsteps; ++st) {
    const int cur = st & 1;
    if constexpr (ADMA) {
      i32x2_t tdma[XI];  // the table entries of step st + 1, fetched a step ago
#pragma unroll
      for (int i = 0; i < XI; ++i) tdma[i] = tn[i];
      if (st + 1 < nsteps) {
        if (st + 2 < nsteps) WD_FETCH(p_begin + kWdPos * (st + 2))
        WD_ISSUE_T(p_begin + kWdPos * (st + 1), cur ^ 1, tdma)
      }
    } else if (st + 1 < nsteps) {
      WD_ISSUE(p_begin + kWdPos * (st + 1), cur ^ 1)
      if (st + 2 < nsteps) WD_FETCH(p_begin + kWdPos * (st + 2))
    }
    const uint16_t* sX = smem + cur * BUFE + wk * kWdGroup;
    const uint16_t* sD = smem + cur * BUFE + (4 + wc) * kWdGroup;
    if constexpr (SCHED) {  // [SCHED] (kstep_sched)
      auto frag = [&](const uint16_t* base, int kk, int i) {
        const int ra = 32 * kk + rr0, rb = 32 * kk + rr1, c = 2 * i + (pp >> 1);
        return tr_pair(base + ra * kWdRow + ((c ^ swz_wd(ra)) << 3) + (pp & 1) * 4,
                       base + rb * kWdRow + ((c ^ swz_wd(rb)) << 3) + (pp & 1) * 4);
      };
      kstep_sched<4, 4, 2>(acc, [&](int kk, int i) { return frag(sD, kk, i); },
                           [&](int kk, int j) { return frag(sX, kk, j); });
    } else {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {  // two 32-position MFMA k-steps
      const int ra = 32 * kk + rr0, rb = 32 * kk + rr1;
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = 2 * i + (pp >> 1);
        fa[i] = tr_pair(sD + ra * kWdRow + ((c ^ swz_wd(ra)) << 3) + (pp & 1) * 4,
                        sD + rb * kWdRow + ((c ^ swz_wd(rb)) << 3) + (pp & 1) * 4);
        fb[i] = tr_pair(sX + ra * kWdRow + ((c ^ swz_wd(ra)) << 3) + (pp & 1) * 4,
                        sX + rb * kWdRow + ((c ^ swz_wd(rb)) << 3) + (pp & 1) * 4);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    }
    if constexpr (ADMA) {
      __builtin_amdgcn_s_waitcnt(7 << 4);  // vmcnt(0) lgkmcnt(0), visible to the waitcnt pass (k_conv_wgrad_tri)
    } else {
      // retire this step's LDS-DMA (next stage) but leave the XI position-table loads for step st+2 in flight: they
      // are the youngest vector-memory ops and are only consumed by the next step's DMA issue
      if (st + 2 < nsteps) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(XI) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  }
#undef WD_ISSUE
#undef WD_ISSUE_T
#undef WD_FETCH
  const int fr = lane & 15, fq = lane >> 4;
  if (a.grad) {  // single split: final layout straight from the accumulators (this wave's group is one tap)
    float* out = a.grad + (int64_t)g * a.ldg + a.off + (int64_t)(co0 + 64 * wc) * a.K;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = kc0 + 64 * wk + 16 * j + fr;
      if (k < a.K) {
        const int dk = (k - gtap * Cin) * a.kt + gtap;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) out[(int64_t)(16 * i + 4 * fq + r) * a.K + dk] = acc[i][j][r] * a.scale;
      }
    }
    return;
  }
  float* out = a.part + (((int64_t)sp * a.G + g) * a.Cout + co0 + 64 * wc) * a.K;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = kc0 + 64 * wk + 16 * j + fr;
    if (k < a.K) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) out[(int64_t)(16 * i + 4 * fq + r) * a.K + k] = acc[i][j][r];
    }
  }
}

// ------------------------------------------------------------------------------------------------
// k_conv_wgrad_tri — wgrad of a 3x3x3 stride-1 conv (AlexNet3D conv2-5) with the X operand staged once per
// k-step for THREE taps.
//
// k_conv_wgrad_dma stages, per 64-position k-step, one [64 positions][64 channels] X tile per tap of its 4-tap
// k-column block plus the dY tile: 40 KB of LDS-DMA per 128 MFMAs, ~78 B/clk/CU at the matrix rate against the
// ~33 B/clk/CU one CU pulls from L2 by LDS-DMA (MI355X_MICROARCH.md, gather into LDS), so it runs at 29 % MFMA
// busy with its waves parked on the DMA 55 % of the time (profiles/r2_pmc_alexnet_g64.txt).  The taps kw = 0,1,2
// of one (kd, kh) read padded-input rows b(p) + kw: for 64 consecutive output positions the union of those rows
// is a few runs of consecutive padded rows (74 for conv2, 92 for the padded 5x7x5 conv3-5; one run per band of
// output rows, split where the band crosses a depth slice or a sample).  A block owns 64 NCH output channels x
// one (kd, kh, 64-channel chunk) triplet = 192 k-columns; per k-step it stages the union (<= U rows) and the dY
// tile: conv2 (NCH 2) 26 KB per 192 MFMAs, 2.3x fewer bytes per MFMA.  Wave (wc, kw) computes co block wc x tap
// kw; its X fragment rows are union row idx(p) + kw.  Step table (k_union_table, per 64-position step of a
// client): per union row {voxel offset of its (kd, kh) = (0, 0) source, padded (d, h, w) code} and idx(p); a
// row whose source for this block's (kd, kh) lies in the padding reads out of range -> 0.
template <int U>
struct WtTab {
  static constexpr int kST = 2 * U + 64;  // ints per step entry: int2 rows[U], int idx[64]
};
struct ConvWgTriArgs {
  const uint16_t* x;    // [G*B, D, H, W, Cin]
  const uint16_t* dy;   // [G, Mg, Cout]
  const int* stab;      // [nsteps][2U + 64]
  float* part;          // [nsplit, G, Cout, K]
  int D, H, W, Cin, Cout, Mg, K, nsplit, chunk, G, nKT, nCT, nstab, pad;
  int64_t xclient;
};

static inline int wt_umax_cap(int umax) { return umax <= 80 ? 80 : (umax <= 96 ? 96 : 0); }

// Union table of a 3x3x3 stride-1 conv (pad in every dimension), one entry per band of P consecutive output positions
// of a client: int2 rows[U] = {voxel offset of the union row's (kd, kh) = (0, 0) source, padded (d, h, w) code},
// int idx[P] = union row of each position's tap (0, 0, 0).  The union is the set of padded-input rows b(p) + e
// (e = 0..ext) over the band, in increasing order; rows past the union get a depth code that no range admits.
// ext = 2: the three kw taps of one (kd, kh) (k_conv_fwd_tri, k_conv_wgrad_tri); ext = 2 Wp + 2: all nine (kh, kw)
// taps of one kd, whose rows are idx(p) + kh Wp + kw because every run is whole (k_conv_fwd_slab).
// One block of P threads per band (P <= 512); one thread merges the runs (allocation time only).
__global__ __launch_bounds__(512) void k_union_table(int* tab, int U, int P, int Mg, int D, int H, int W, int pad,
                                                      int ext) {
  __shared__ int b[512];
  const int Dp = D + 2 * pad, Hp = H + 2 * pad, Wp = W + 2 * pad, Do = Dp - 2, Ho = Hp - 2, Wo = Wp - 2;
  const int S = Do * Ho * Wo, VOL = Dp * Hp * Wp + 8;  // sample n's padded rows live at n * VOL + padded index
  const int s = blockIdx.x, p = threadIdx.x, m = P * s + p;
  int key = -1;
  if (p < P && m < Mg) {
    const int nl = m / S, r = m - nl * S, od = r / (Ho * Wo), r2 = r - od * Ho * Wo, oh = r2 / Wo, ow = r2 - oh * Wo;
    key = nl * VOL + (od * Hp + oh) * Wp + ow;
  }
  if (p < P) b[p] = key;
  __syncthreads();
  if (p != 0) return;
  int* rows = tab + (int64_t)s * (2 * U + P);
  int* idx = rows + 2 * U;
  int cnt = 0, last = -10;
  for (int q = 0; q < P; ++q) {  // keys increase with q: rows of the current run are contiguous up to `last`
    const int bq = b[q];
    if (bq < 0) { idx[q] = 0; continue; }
    int first;
    if (cnt > 0 && bq <= last) { idx[q] = cnt - 1 - (last - bq); first = last + 1; }
    else { idx[q] = cnt; first = bq; }
    for (int r = first; r <= bq + ext; ++r) {
      if (cnt < U) {
        const int n = r / VOL, l = r - n * VOL, dp = l / (Hp * Wp), l2 = l - dp * Hp * Wp, hp = l2 / Wp, wp = l2 - hp * Wp;
        rows[2 * cnt] = ((n * D + dp - pad) * H + hp - pad) * W + wp - pad;
        rows[2 * cnt + 1] = dp | (hp << 10) | (wp << 20);
      }
      ++cnt;
    }
    last = max(last, bq + ext);
  }
  for (int u = cnt; u < U; ++u) {
    rows[2 * u] = 0;
    rows[2 * u + 1] = 1023;  // depth code out of every range: never read
  }
}

// largest union of one P-position band (same rule as k_union_table), cached per shape
static int union_umax(int B, int D, int H, int W, int pad, int P, int ext) {
  static std::map<std::array<int, 7>, int> cache;
  const std::array<int, 7> key{B, D, H, W, pad, P, ext};
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  const int Dp = D + 2 * pad, Hp = H + 2 * pad, Wp = W + 2 * pad, Do = Dp - 2, Ho = Hp - 2, Wo = Wp - 2;
  const int S = Do * Ho * Wo, Mg = B * S, VOL = Dp * Hp * Wp + 8;
  int mx = 0;
  for (int s0 = 0; s0 < Mg; s0 += P) {
    int cnt = 0, last = -10;
    for (int m = s0; m < std::min(s0 + P, Mg); ++m) {
      const int nl = m / S, r = m - nl * S, od = r / (Ho * Wo), r2 = r - od * Ho * Wo, oh = r2 / Wo, ow = r2 - oh * Wo;
      const int bq = nl * VOL + (od * Hp + oh) * Wp + ow;
      const int first = (cnt > 0 && bq <= last) ? last + 1 : bq;
      cnt += std::max(0, bq + ext + 1 - first);
      last = std::max(last, bq + ext);
    }
    mx = std::max(mx, cnt);
  }
  cache[key] = mx;
  return mx;
}

static int wgrad_tri_umax(int B, int D, int H, int W, int pad) { return union_umax(B, D, H, W, pad, 64); }

// largest union (rows) of a P-position band: exposed for host-side tests of the union rule
int conv3d_union_umax(int B, int D, int H, int W, int pad, int P) { return union_umax(B, D, H, W, pad, P); }

// [LSW] as k_conv_fwd_slab: the X union rows' chunk swizzle is keyed by their output-space index L = (d Ho + h) Wo + w
// (the positions of one ds_read_b64_tr_b16 read L = p + kw for 8 positions p, consecutive within the step except at
// the 32-position kk halves, where the union rows jump at output-row ends; modelled for conv2: 1.52 LDS cycles per X
// read -> 1.00).  The dY rows are the step's positions themselves and keep swz_wd of their row.  Measured: conflicts
// 20.8 / 33.2 % -> 0.1 / 1.7 % (conv2 / conv3-5) but conv2 2.92-2.98 -> 3.22-3.29 ms (the per-step swizzle of the
// DMA addresses sits on the issue path); opt-in NIDT_WGTRI_LSWZ=1 (profiles/r4_ab_lds_swizzle.txt).
// [ADMA] the stage DMA issued from inline asm (blds16_asm) instead of the intrinsic: the compiler's waitcnt pass
// treats an intrinsic LDS-DMA as a write to LDS that the fragment reads of the current stage may alias, and put a
// vmcnt wait for the next stage's DMA (issued at the top of the step) in front of them — the double buffer never
// overlapped a transfer with the MFMAs of its own wave.  The kernel's counted waits at the end of each step already
// order every DMA before its stage is read; M0 is used by nothing else here.
template <int NCH, int U, bool PADDED, bool LSW = true, bool SCHED = false, bool ADMA = false>
__global__ __launch_bounds__(192 * NCH, 2) void k_conv_wgrad_tri(ConvWgTriArgs a) {
  constexpr int NW = 3 * NCH, XG = U * kWdRow, BUFE = XG + NCH * kWdGroup, ST = WtTab<U>::kST;
  constexpr int XP = U / 8, XPW = (XP + NW - 1) / NW;       // union pieces (8 rows each) per wave
  constexpr int DP = 8 * NCH, DPW = (DP + NW - 1) / NW;     // dY pieces (8 positions x 64 co) per wave
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * BUFE];
  auto stage = [&](int k) -> uint16_t* { return smem + k * BUFE; };
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wid / 3, kw = wid - 3 * wc;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int kt = id % a.nKT, r1 = id / a.nKT;
  const int ct = r1 % a.nCT, r2 = r1 / a.nCT;
  const int sp = r2 % a.nsplit, g = r2 / a.nsplit;
  const int Cin = a.Cin, nck = Cin / 64;
  const int trip = kt / nck, cc = kt - trip * nck;  // trip = kd * 3 + kh
  const int kd = trip / 3, kh = trip - 3 * kd;
  const int co0 = ct * 64 * NCH;
  const int p_begin = sp * a.chunk, p_end = min(a.Mg, p_begin + a.chunk);
  const i32x4_t rx = make_rsrc(a.x + (int64_t)g * a.xclient, (uint32_t)(a.xclient * 2));
  const i32x4_t rd = make_rsrc(a.dy + (int64_t)g * a.Mg * a.Cout, (uint32_t)((int64_t)a.Mg * a.Cout * 2));
  const i32x4_t rt = make_rsrc(a.stab, (uint32_t)a.nstab * ST * 4u);
  const int lr = lane >> 3, ls = lane & 7;
  const int xadd = (kd * a.H + kh) * a.W;                   // voxel offset of tap (kd, kh, 0)
  const int dlo = a.pad - kd, hlo = a.pad - kh;             // code ranges of sources inside the volume
  int xcol[XPW], dcol[DPW], dls[DPW];
#pragma unroll
  for (int i = 0; i < XPW; ++i) {
    const int u = 8 * (wid * XPW + i) + lr;
    xcol[i] = (cc * 64 + (LSW ? 0 : ((ls ^ swz_wd(u)) << 3))) * 2;
  }
  const int Ho = a.H + 2 * a.pad - 2, Wo = a.W + 2 * a.pad - 2, So = (a.D + 2 * a.pad - 2) * Ho * Wo;
#pragma unroll
  for (int i = 0; i < DPW; ++i) {
    const int dp = min(wid * DPW + i, DP - 1), h = dp >> 3, sl = dp & 7, r = 8 * sl + lr;
    dcol[i] = (r * a.Cout + co0 + 64 * h + ((ls ^ swz_wd(r)) << 3)) * 2;
    dls[i] = h * kWdGroup + sl * 512;
  }
  const int gq = lane >> 4, li = lane & 15, qq = li >> 2, pp = li & 3;
  const int rr0 = 8 * gq + qq, rr1 = rr0 + 4;
  i32x2_t trow[XPW];
  int tix[4], tixn[4];
  auto wt_dma = [](i32x4_t r, int off, uint16_t* dst) {
    if constexpr (ADMA) blds16_asm(r, off, dst);
    else blds16(r, off, dst);
  };
#define WT_FETCH_ROWS(S)                                                                                      \
  {                                                                                                           \
    _Pragma("unroll") for (int i_ = 0; i_ < XPW; ++i_)                                                        \
      trow[i_] = nidt_raw_buffer_load_v2i32(rt, ((S) * ST + 2 * (8 * (wid * XPW + i_) + lr)) * 4, 0, 0);      \
  }
#define WT_FETCH_IDX(S, DST)                                                                                  \
  {                                                                                                           \
    _Pragma("unroll") for (int k_ = 0; k_ < 4; ++k_)                                                          \
      DST[k_] = nidt_raw_buffer_load_i32(rt, ((S) * ST + 2 * U + 32 * (k_ >> 1) + ((k_ & 1) ? rr1 : rr0)) * 4, \
                                         0, 0);                                                               \
  }
#define WT_ISSUE_R(S, BUFI, TR)                                                                               \
  {                                                                                                           \
    uint16_t* sX_ = stage(BUFI);                                                                              \
    uint16_t* sD_ = sX_ + XG;                                                                                 \
    _Pragma("unroll") for (int i_ = 0; i_ < XPW; ++i_)                                                        \
      if (wid * XPW + i_ < XP) {                                                                              \
        const int c_ = TR[i_].y;                                                                              \
        const bool ok_ = PADDED ? ((unsigned)((c_ & 1023) - dlo) < (unsigned)a.D &&                            \
                                   (unsigned)(((c_ >> 10) & 1023) - hlo) < (unsigned)a.H &&                   \
                                   (unsigned)((c_ >> 20) - a.pad) < (unsigned)a.W)                            \
                                : (c_ & 1023) != 1023;                                                        \
        const int sw_ = LSW ? ((ls ^ swz_wd(((c_ & 1023) * Ho + ((c_ >> 10) & 1023)) * Wo + (c_ >> 20))) << 4) : 0; \
        wt_dma(rx, ok_ ? (TR[i_].x + xadd) * (2 * Cin) + xcol[i_] + sw_ : kBufOOB, sX_ + (wid * XPW + i_) * 512); \
      }                                                                                                       \
    _Pragma("unroll") for (int i_ = 0; i_ < DPW; ++i_)                                                        \
      if (wid * DPW + i_ < DP) wt_dma(rd, (S) * 64 * (2 * a.Cout) + dcol[i_], sD_ + dls[i_]);               \
  }
#define WT_ISSUE(S, BUFI) WT_ISSUE_R(S, BUFI, trow)

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int s0 = p_begin / 64, nsteps = (p_end - p_begin + 63) / 64;
  // output-space index (within the sample) of the four fragment positions of this lane, advanced by 64 per step
  int lpos[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) lpos[k] = (s0 * 64 + 32 * (k >> 1) + ((k & 1) ? rr1 : rr0)) % So;
  // the k-step: 32 MFMAs per wave from stage buffer `buf` with union-row indices tx of this step's positions
  auto compute = [&](const uint16_t* sX, const int (&tx)[4]) {
    const uint16_t* sD = sX + XG + wc * kWdGroup;
    if constexpr (SCHED) {  // [SCHED] (kstep_sched)
      kstep_sched<4, 4, 2>(
          acc,
          [&](int kk, int i) {
            const int ra = 32 * kk + rr0, rb = 32 * kk + rr1, c = 2 * i + (pp >> 1);
            return tr_pair(sD + ra * kWdRow + ((c ^ swz_wd(ra)) << 3) + (pp & 1) * 4,
                           sD + rb * kWdRow + ((c ^ swz_wd(rb)) << 3) + (pp & 1) * 4);
          },
          [&](int kk, int j) {
            const int xa = tx[2 * kk] + kw, xb = tx[2 * kk + 1] + kw, c = 2 * j + (pp >> 1);
            const int sxa = swz_wd(LSW ? lpos[2 * kk] + kw : xa), sxb = swz_wd(LSW ? lpos[2 * kk + 1] + kw : xb);
            return tr_pair(sX + xa * kWdRow + ((c ^ sxa) << 3) + (pp & 1) * 4,
                           sX + xb * kWdRow + ((c ^ sxb) << 3) + (pp & 1) * 4);
          });
    } else {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int ra = 32 * kk + rr0, rb = 32 * kk + rr1;
        const int xa = tx[2 * kk] + kw, xb = tx[2 * kk + 1] + kw;
        const int sxa = swz_wd(LSW ? lpos[2 * kk] + kw : xa), sxb = swz_wd(LSW ? lpos[2 * kk + 1] + kw : xb);
        bf16x8 fa[4], fb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = 2 * i + (pp >> 1);
          fa[i] = tr_pair(sD + ra * kWdRow + ((c ^ swz_wd(ra)) << 3) + (pp & 1) * 4,
                          sD + rb * kWdRow + ((c ^ swz_wd(rb)) << 3) + (pp & 1) * 4);
          fb[i] = tr_pair(sX + xa * kWdRow + ((c ^ sxa) << 3) + (pp & 1) * 4,
                          sX + xb * kWdRow + ((c ^ sxb) << 3) + (pp & 1) * 4);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      lpos[k] += 64;
      lpos[k] -= lpos[k] >= So ? So : 0;  // So >= 64 for every eligible shape (host check)
    }
  };
  if (nsteps > 0) {
    WT_FETCH_ROWS(s0)
    WT_FETCH_IDX(s0, tixn)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    WT_ISSUE(s0, 0)
    if (nsteps > 1) WT_FETCH_ROWS(s0 + 1)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int st = 0; st < nsteps; ++st) {
    const int cur = st & 1;
#pragma unroll
    for (int k = 0; k < 4; ++k) tix[k] = tixn[k];
    if constexpr (ADMA) {
      // [ADMA] the step-table loads (rows of st + 2, indices of st + 1) go out first, then the asm DMA of st + 1 from
      // the rows fetched a step ago (rdma): the compiler, which counts only the loads it sees, never has to wait for
      // anything younger than the DMA to feed it, and nothing of this step reads those new registers, so the only
      // wait for the DMA is ours at the end of the step — the transfer overlaps this step's MFMAs
      i32x2_t rdma[XPW];
#pragma unroll
      for (int i = 0; i < XPW; ++i) rdma[i] = trow[i];
      if (st + 1 < nsteps) {
        if (st + 2 < nsteps) WT_FETCH_ROWS(s0 + st + 2)
        WT_FETCH_IDX(s0 + st + 1, tixn)
        WT_ISSUE_R(s0 + st + 1, cur ^ 1, rdma)
      }
      compute(stage(cur), tix);
      // s_waitcnt vmcnt(0) lgkmcnt(0) as the builtin, which the waitcnt pass sees (with an asm wait it would still
      // count this step's table loads as pending and wait for them in front of the next step's DMA)
      __builtin_amdgcn_s_waitcnt(7 << 4);
    } else {
      if (st + 1 < nsteps) {
        WT_ISSUE(s0 + st + 1, cur ^ 1)
        if (st + 2 < nsteps) WT_FETCH_ROWS(s0 + st + 2)
        WT_FETCH_IDX(s0 + st + 1, tixn)
      }
      compute(stage(cur), tix);
      // retire the next stage's LDS-DMA; the step-table loads issued after it (rows for st+2, idx for st+1) may stay
      if (st + 2 < nsteps) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(XPW + 4) : "memory");
      else if (st + 1 < nsteps) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  }
#undef WT_ISSUE
#undef WT_ISSUE_R
#undef WT_FETCH_IDX
#undef WT_FETCH_ROWS
  const int fr = lane & 15, fq = lane >> 4;
  float* out = a.part + (((int64_t)sp * a.G + g) * a.Cout + co0 + 64 * wc) * a.K;
  const int kcol = ((kd * 9 + kh * 3 + kw) * Cin) + cc * 64;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = kcol + 16 * j + fr;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(int64_t)(16 * i + 4 * fq + r) * a.K + k] = acc[i][j][r];
  }
}

// k_conv_wgrad_slab — the weight gradient with one X union per (kd, 64-channel chunk) slab for all nine (kh, kw)
// taps: per 64-position step the block stages the whole-window union of the step's positions (k_union_table with
// ext = 2 Wp + 2, <= 152 rows for conv2 vs 3 x <= 80 for the three (kd, kh) triplets of k_conv_wgrad_tri) and the
// step's dY tile, and 12 waves compute 64 co x 9 taps x 64 ci from them: 288 MFMAs per 27 KB of LDS-DMA instead of
// 96 per 18 KB (k_conv_wgrad_tri, which the PMC shows waiting on those transfers).  Wave (kh, j) = (wid / 4,
// wid % 4) owns ci tile j of taps (kh, 0..2) for all four co tiles: X row of tap (kh, kw) = idx(p) + kh Wp + kw.
// Output: fp32 slabs per split (k_wgrad_reduce finishes), as k_conv_wgrad_tri.
// [ADMA] as k_conv_wgrad_tri: the stage DMA from inline asm, the step-table loads issued before it, the builtin wait
template <int U, bool PADDED, bool ADMA = false>
__global__ __launch_bounds__(768, 1) void k_conv_wgrad_slab(ConvWgTriArgs a) {
  constexpr int NW = 12, XG = U * kWdRow, BUFE = XG + kWdGroup, ST = WtTab<U>::kST;
  constexpr int XP = U / 8, XPW = (XP + NW - 1) / NW;   // union pieces (8 rows each) per wave
  __shared__ __attribute__((aligned(16))) uint16_t smem[2 * BUFE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kh = wid >> 2, jt = wid & 3;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int kt = id % a.nKT, r1 = id / a.nKT;
  const int ct = r1 % a.nCT, r2 = r1 / a.nCT;
  const int sp = r2 % a.nsplit, g = r2 / a.nsplit;
  const int Cin = a.Cin, nck = Cin / 64;
  const int kd = kt / nck, cc = kt - kd * nck;
  const int co0 = ct * 64, Wp = a.W + 2 * a.pad;
  const int p_begin = sp * a.chunk, p_end = min(a.Mg, p_begin + a.chunk);
  const i32x4_t rx = make_rsrc(a.x + (int64_t)g * a.xclient, (uint32_t)(a.xclient * 2));
  const i32x4_t rd = make_rsrc(a.dy + (int64_t)g * a.Mg * a.Cout, (uint32_t)((int64_t)a.Mg * a.Cout * 2));
  const i32x4_t rt = make_rsrc(a.stab, (uint32_t)a.nstab * ST * 4u);
  const int lr = lane >> 3, ls = lane & 7;
  const int xadd = kd * a.H * a.W;                          // voxel offset of tap (kd, 0, 0)
  const int dlo = a.pad - kd;                               // depth code range of sources inside the volume
  int xcol[XPW];
#pragma unroll
  for (int i = 0; i < XPW; ++i) {
    const int u = 8 * (wid * XPW + i) + lr;
    xcol[i] = (cc * 64 + ((ls ^ swz_wd(u)) << 3)) * 2;
  }
  const bool dload = wid < 8;                               // waves 0-7 stage dY slice wid (8 positions x 64 co)
  const int dr = 8 * (wid & 7) + lr;
  const int dcol = (dr * a.Cout + co0 + ((ls ^ swz_wd(dr)) << 3)) * 2;
  const int gq = lane >> 4, li = lane & 15, qq = li >> 2, pp = li & 3;
  const int rr0 = 8 * gq + qq, rr1 = rr0 + 4;
  i32x2_t trow[XPW];
  int tix[4], tixn[4];
#define WS_FETCH_ROWS(S)                                                                                      \
  {                                                                                                           \
    _Pragma("unroll") for (int i_ = 0; i_ < XPW; ++i_)                                                        \
      trow[i_] = nidt_raw_buffer_load_v2i32(rt, ((S) * ST + 2 * (8 * (wid * XPW + i_) + lr)) * 4, 0, 0);      \
  }
#define WS_FETCH_IDX(S, DST)                                                                                  \
  {                                                                                                           \
    _Pragma("unroll") for (int k_ = 0; k_ < 4; ++k_)                                                          \
      DST[k_] = nidt_raw_buffer_load_i32(rt, ((S) * ST + 2 * U + 32 * (k_ >> 1) + ((k_ & 1) ? rr1 : rr0)) * 4, \
                                         0, 0);                                                               \
  }
  auto ws_dma = [](i32x4_t r, int off, uint16_t* dst) {
    if constexpr (ADMA) blds16_asm(r, off, dst);
    else blds16(r, off, dst);
  };
#define WS_ISSUE_R(S, BUFI, TR)                                                                               \
  {                                                                                                           \
    uint16_t* sX_ = smem + (BUFI) * BUFE;                                                                     \
    _Pragma("unroll") for (int i_ = 0; i_ < XPW; ++i_)                                                        \
      if (wid * XPW + i_ < XP) {                                                                              \
        const int c_ = TR[i_].y;                                                                              \
        const bool ok_ = PADDED ? ((unsigned)((c_ & 1023) - dlo) < (unsigned)a.D &&                            \
                                   (unsigned)(((c_ >> 10) & 1023) - a.pad) < (unsigned)a.H &&                 \
                                   (unsigned)((c_ >> 20) - a.pad) < (unsigned)a.W)                            \
                                : (c_ & 1023) != 1023;                                                        \
        ws_dma(rx, ok_ ? (TR[i_].x + xadd) * (2 * Cin) + xcol[i_] : kBufOOB, sX_ + (wid * XPW + i_) * 512);    \
      }                                                                                                       \
    if (dload) ws_dma(rd, (S) * 64 * (2 * a.Cout) + dcol, sX_ + XG + (wid & 7) * 512);                       \
  }
#define WS_ISSUE(S, BUFI) WS_ISSUE_R(S, BUFI, trow)

  f32x4 acc[3][4];
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int s0 = p_begin / 64, nsteps = (p_end - p_begin + 63) / 64;
  if (nsteps > 0) {
    WS_FETCH_ROWS(s0)
    WS_FETCH_IDX(s0, tixn)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    WS_ISSUE(s0, 0)
    if (nsteps > 1) WS_FETCH_ROWS(s0 + 1)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  const int toff = kh * Wp;
  for (int st = 0; st < nsteps; ++st) {
    const int cur = st & 1;
#pragma unroll
    for (int k = 0; k < 4; ++k) tix[k] = tixn[k];
    if constexpr (ADMA) {
      i32x2_t rdma[XPW];
#pragma unroll
      for (int i = 0; i < XPW; ++i) rdma[i] = trow[i];
      if (st + 1 < nsteps) {
        if (st + 2 < nsteps) WS_FETCH_ROWS(s0 + st + 2)
        WS_FETCH_IDX(s0 + st + 1, tixn)
        WS_ISSUE_R(s0 + st + 1, cur ^ 1, rdma)
      }
    } else if (st + 1 < nsteps) {
      WS_ISSUE(s0 + st + 1, cur ^ 1)
      if (st + 2 < nsteps) WS_FETCH_ROWS(s0 + st + 2)
      WS_FETCH_IDX(s0 + st + 1, tixn)
    }
    const uint16_t* sX = smem + cur * BUFE;
    const uint16_t* sD = sX + XG;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int ra = 32 * kk + rr0, rb = 32 * kk + rr1;
      bf16x8 fa[4], fb[3];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = 2 * i + (pp >> 1);
        fa[i] = tr_pair(sD + ra * kWdRow + ((c ^ swz_wd(ra)) << 3) + (pp & 1) * 4,
                        sD + rb * kWdRow + ((c ^ swz_wd(rb)) << 3) + (pp & 1) * 4);
      }
      const int c = 2 * jt + (pp >> 1);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int xa = tix[2 * kk] + toff + kw, xb = tix[2 * kk + 1] + toff + kw;
        fb[kw] = tr_pair(sX + xa * kWdRow + ((c ^ swz_wd(xa)) << 3) + (pp & 1) * 4,
                         sX + xb * kWdRow + ((c ^ swz_wd(xb)) << 3) + (pp & 1) * 4);
      }
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[kw][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[kw], acc[kw][i], 0, 0, 0);
    }
    if constexpr (ADMA) {
      __builtin_amdgcn_s_waitcnt(7 << 4);  // vmcnt(0) lgkmcnt(0), visible to the waitcnt pass (k_conv_wgrad_tri)
    } else {
      // retire the next stage's LDS-DMA; the step-table loads issued after it (rows for st+2, idx for st+1) may stay
      if (st + 2 < nsteps) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(XPW + 4) : "memory");
      else if (st + 1 < nsteps) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  }
#undef WS_ISSUE
#undef WS_ISSUE_R
#undef WS_FETCH_IDX
#undef WS_FETCH_ROWS
  const int fr = lane & 15, fq = lane >> 4;
  float* out = a.part + (((int64_t)sp * a.G + g) * a.Cout + co0) * a.K;
#pragma unroll
  for (int kw = 0; kw < 3; ++kw) {
    const int k = ((kd * 9 + kh * 3 + kw) * Cin) + cc * 64 + 16 * jt + fr;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[(int64_t)(16 * i + 4 * fq + r) * a.K + k] = acc[kw][i][r];
  }
}

static inline int conv_out_n(int n, int pad) { return n + 2 * pad - 2; }

// output channels per k_conv_wgrad_tri block: 64 (3 waves).  NIDT_WG_TRI_NCH=2 gives 128-channel blocks (6 waves)
// where Cout allows (A/B: slower on every AlexNet layer, conv2 3.28 vs 3.06 ms at 64 clients,
// profiles/r2_ab_wgrad_tri.txt)
static int wt_nch(int Cout) {
  static const int env = [] {
    const char* e = getenv("NIDT_WG_TRI_NCH");
    return e ? atoi(e) : 1;
  }();
  return (Cout % 128 == 0 && env == 2) ? 2 : 1;
}

// split factor of k_conv_wgrad_tri: the wgrad cost model over its own tiles (9 x Cin/64 triplets x co blocks x G)
int conv3d_wgrad_tri_nsplit(int G, int B, int D, int H, int W, int Cin, int Cout, int pad) {
  static const int ns_env = [] {  // NIDT_WG_TRI_NS=<n>: force the split of the unpadded (conv2) launch (A/B)
    const char* e = getenv("NIDT_WG_TRI_NS");
    return e ? atoi(e) : 0;
  }();
  if (ns_env > 0 && pad == 0) return ns_env;
  const int Mg = B * conv_out_n(D, pad) * conv_out_n(H, pad) * conv_out_n(W, pad);
  const int nch = wt_nch(Cout);
  // step cost ~1 us per block slot, no fixed term (128-channel blocks at 64 clients, conv2: ns 4 / 6 / 8 / 12 ->
  // 3.27 / 3.28 / 3.09 / 3.12 ms, profiles/r2_ab_wgrad_tri.txt)
  const int U = wt_umax_cap(wgrad_tri_umax(B, D, H, W, pad));
  const int lds = 2 * (U * 128 + nch * 8192);  // bytes per block; 4 waves per SIMD by registers
  const int per_cu = std::max(1, std::min(163840 / std::max(lds, 1), 16 / (3 * nch)));
  const int base = G * (Cout / (64 * nch)) * 9 * (Cin / 64);
  const double slots = 256.0 * per_cu;
  const int ns = wgrad_nsplit_base(base, G, Mg, 27 * Cin, Cout, 1.0, 0.0, slots);
  // a single-wave pick (small lockstep groups) ends with its slowest block: every block runs the whole launch, so
  // uneven progress of co-resident blocks sets the time.  Going about three waves deep measured faster in the full
  // step although the isolated launch is slower (AlexNet conv2 at 8 clients: step 3.62 -> 3.48 ms with 24 splits,
  // 3.50 with 16, 3.58 with 8; isolated wgrad 0.363 -> 0.415 ms; profiles/r4_kbench_g8.txt)
  if (pad == 0 && base * ns <= slots) {
    const int deep = ceil_div((int)(3 * slots), base);
    return std::max(ns, std::min(deep, std::max(1, std::min(64, Mg / 512))));
  }
  return ns;
}

// step table for k_conv_wgrad_tri: ceil(Mg / 64) entries of 2U + 64 ints
int conv3d_wgrad_tri_table_size(int B, int D, int H, int W, int pad) {
  const int Mg = B * conv_out_n(D, pad) * conv_out_n(H, pad) * conv_out_n(W, pad);
  const int U = wt_umax_cap(wgrad_tri_umax(B, D, H, W, pad));
  NIDT_REQUIRE(U > 0, "conv3d_wgrad_tri_table_size: shape not eligible");
  return ceil_div(Mg, 64) * (2 * U + 64);
}

void conv3d_wgrad_tri_table(uintptr_t tab, int B, int D, int H, int W, int pad, uintptr_t stream) {
  const int Mg = B * conv_out_n(D, pad) * conv_out_n(H, pad) * conv_out_n(W, pad);
  const int U = wt_umax_cap(wgrad_tri_umax(B, D, H, W, pad));
  NIDT_REQUIRE(U > 0, "conv3d_wgrad_tri_table: shape not eligible");
  NIDT_REQUIRE(D + 2 * pad < 1024 && H + 2 * pad < 1024 && W + 2 * pad < 1024, "conv3d_wgrad_tri_table: extents < 1024");
  hipLaunchKernelGGL(k_union_table, dim3(ceil_div(Mg, 64)), dim3(64), 0, as_stream(stream), ptr<int>(tab), U, 64, Mg,
                     D, H, W, pad, 2);
  NIDT_CHECK(hipGetLastError());
}

// k_conv_wgrad_tri applies (3x3x3 stride 1, pad <= 2, 64-channel multiples, every step's union <= 96 rows) and is
// not switched off (NIDT_WG_TRI=0 -> k_conv_wgrad_dma everywhere, A/B; NIDT_WG_TRI=2 -> only unpadded convs)
int conv3d_wgrad_tri_ok(int B, int D, int H, int W, int Cin, int Cout, int pad) {
  static const int env = [] {
    const char* e = getenv("NIDT_WG_TRI");
    return e ? atoi(e) : 1;
  }();
  if (!env || (env == 2 && pad != 0) || pad < 0 || pad > 2 || Cin % 64 != 0 || Cout % 64 != 0) return 0;
  if (conv_out_n(D, pad) < 1 || conv_out_n(H, pad) < 1 || conv_out_n(W, pad) < 1) return 0;
  return wt_umax_cap(wgrad_tri_umax(B, D, H, W, pad)) > 0 ? 1 : 0;
}

// k_conv_wgrad_tri is the faster choice for this layer and client count: always for unpadded convs (conv2); padded
// convs with >= 8 K output positions per launch (the 5x7x5 conv3-5 at 64 clients: 0.47/0.64/0.45 -> 0.37/0.52/0.36
// ms).  Since its stage DMA overlaps the MFMAs ([ADMA]) it also wins at 8 clients (22 K positions): conv3 / conv5
// 0.076 -> 0.059 / 0.060 ms, conv4 0.081 -> 0.085 (kbench 8: step 3.07-3.15 -> 3.01 ms, profiles/r6_g8_sweep.txt);
// the threshold was 64 K before [ADMA]
int conv3d_wgrad_tri_pick(int G, int B, int D, int H, int W, int Cin, int Cout, int pad) {
  if (!conv3d_wgrad_tri_ok(B, D, H, W, Cin, Cout, pad)) return 0;
  static const int64_t minpos = [] {  // NIDT_WG_TRI_MINPOS: the padded-conv threshold (A/B)
    const char* e = getenv("NIDT_WG_TRI_MINPOS");
    return e ? (int64_t)atoll(e) : (int64_t)8192;
  }();
  const int64_t pos = (int64_t)G * B * conv_out_n(D, pad) * conv_out_n(H, pad) * conv_out_n(W, pad);
  return (pad == 0 || pos >= minpos) ? 1 : 0;
}

void conv3d_wgrad_tri(uintptr_t x, uintptr_t dy, uintptr_t part, uintptr_t grad, int64_t ldg, int64_t off, int G, int B,
                      int D, int H, int W, int Cin, int Cout, int pad, int nsplit, float scale, uintptr_t stab,
                      uintptr_t stream) {
  NIDT_REQUIRE(conv3d_wgrad_tri_ok(B, D, H, W, Cin, Cout, pad), "conv3d_wgrad_tri: shape not eligible");
  NIDT_REQUIRE(stab != 0 && nsplit >= 1, "conv3d_wgrad_tri: needs the step table");
  const int U = wt_umax_cap(wgrad_tri_umax(B, D, H, W, pad));
  ConvWgTriArgs d;
  d.x = ptr<const uint16_t>(x); d.dy = ptr<const uint16_t>(dy); d.stab = ptr<const int>(stab); d.part = ptr<float>(part);
  d.D = D; d.H = H; d.W = W; d.Cin = Cin; d.Cout = Cout; d.pad = pad;
  d.Mg = B * conv_out_n(D, pad) * conv_out_n(H, pad) * conv_out_n(W, pad);
  d.K = 27 * Cin; d.nsplit = nsplit; d.G = G;
  d.chunk = ((ceil_div(d.Mg, nsplit) + 63) / 64) * 64;
  const int nch = wt_nch(Cout);
  d.nKT = 9 * (Cin / 64); d.nCT = Cout / (64 * nch);
  d.nstab = ceil_div(d.Mg, 64);
  d.xclient = (int64_t)B * D * H * W * Cin;
  NIDT_REQUIRE(d.xclient * 2 < (1ll << 31) && (int64_t)d.Mg * Cout * 2 < (1ll << 31),
               "conv3d_wgrad_tri: per-client tensors must stay below 2 GiB (32-bit buffer offsets)");
  const int64_t nwg = (int64_t)d.nKT * d.nCT * nsplit * G;
  NIDT_REQUIRE(nwg < (1ll << 31), "conv3d_wgrad_tri: grid too large");
  hipStream_t s = as_stream(stream);
  const dim3 grid((unsigned)nwg);
  static const int lsw_env = [] {  // NIDT_WGTRI_LSWZ=1: output-space swizzle of the X rows (A/B: slower, see [LSW])
    const char* e = getenv("NIDT_WGTRI_LSWZ");
    return e ? atoi(e) : 0;
  }();
  const bool lsw = lsw_env && d.Mg / B >= 64;  // the kernel advances its output-space indices by 64 per step
  // [SCHED] k-step schedule (kstep_sched): AlexNet conv2-5 weight gradients at 64 clients 4.28 -> 4.24 ms
  // (profiles/r4_ab_sched_more.txt); NIDT_WGT_SCHED=0: the compiler's schedule (A/B)
  static const int tsched = [] {
    const char* e = getenv("NIDT_WGT_SCHED");
    return e ? atoi(e) : 1;
  }();
  // [ADMA] asm-issued stage DMA (NIDT_WGT_ADMA=0: the intrinsic, A/B)
  static const int tadma = [] {
    const char* e = getenv("NIDT_WGT_ADMA");
    return e ? atoi(e) : 1;
  }();
#define NIDT_TRI(NC, UU)                                                                                       \
  if (tsched && !lsw && tadma) {                                                                               \
    if (pad) hipLaunchKernelGGL((k_conv_wgrad_tri<NC, UU, true, false, true, true>), grid, dim3(192 * NC), 0, s, d); \
    else hipLaunchKernelGGL((k_conv_wgrad_tri<NC, UU, false, false, true, true>), grid, dim3(192 * NC), 0, s, d); \
  } else if (tsched && !lsw) {                                                                                        \
    if (pad) hipLaunchKernelGGL((k_conv_wgrad_tri<NC, UU, true, false, true>), grid, dim3(192 * NC), 0, s, d); \
    else hipLaunchKernelGGL((k_conv_wgrad_tri<NC, UU, false, false, true>), grid, dim3(192 * NC), 0, s, d);    \
  } else if (lsw) {                                                                                            \
    if (pad) hipLaunchKernelGGL((k_conv_wgrad_tri<NC, UU, true, true>), grid, dim3(192 * NC), 0, s, d);        \
    else hipLaunchKernelGGL((k_conv_wgrad_tri<NC, UU, false, true>), grid, dim3(192 * NC), 0, s, d);           \
  } else {                                                                                                     \
    if (pad) hipLaunchKernelGGL((k_conv_wgrad_tri<NC, UU, true, false>), grid, dim3(192 * NC), 0, s, d);       \
    else hipLaunchKernelGGL((k_conv_wgrad_tri<NC, UU, false, false>), grid, dim3(192 * NC), 0, s, d);          \
  }
  if (nch == 2) {
    if (U == 80) { NIDT_TRI(2, 80) } else { NIDT_TRI(2, 96) }
  } else {
    if (U == 80) { NIDT_TRI(1, 80) } else { NIDT_TRI(1, 96) }
  }
#undef NIDT_TRI
  NIDT_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_wgrad_reduce, dim3(Cout, G), dim3(256), 27 * (Cin + 1) * sizeof(float), s, ptr<const float>(part),
                     nsplit, G, Cout, Cin, 27, ptr<float>(grad), ldg, off, scale);
  NIDT_CHECK(hipGetLastError());
}

// ---- k_conv_wgrad_slab host side: 64-position steps, whole-window unions (ext = 2 Wp + 2) of <= 152 rows ----
static inline int ws_u(int B, int D, int H, int W, int pad) {
  return union_umax(B, D, H, W, pad, 64, 2 * (W + 2 * pad) + 2) <= 152 ? 152 : 0;
}

int conv3d_wgrad_slab_ok(int B, int D, int H, int W, int Cin, int Cout, int pad) {
  if (pad < 0 || pad > 2 || Cin % 64 != 0 || Cout % 64 != 0) return 0;
  if (conv_out_n(D, pad) < 1 || conv_out_n(H, pad) < 1 || conv_out_n(W, pad) < 1) return 0;
  if (D + 2 * pad >= 1024 || H + 2 * pad >= 1024 || W + 2 * pad >= 1024) return 0;
  return ws_u(B, D, H, W, pad) > 0 ? 1 : 0;
}

// Off by default (NIDT_WG_SLAB=1 opts in where k_conv_wgrad_tri would run): measured slower at 64 clients, conv2 wgrad
// 3.83 vs 3.03 ms, conv3-5 0.44-0.63 vs 0.36-0.53 ms (profiles/r3_ab_wgrad_slab.txt) — one 12-wave block per CU
// (114 VGPRs) re-reads the dY tile from LDS in every wave and waits at each step's barrier with no second block
// to cover it; the triplet kernel's two 3-wave blocks per CU overlap those waits.
int conv3d_wgrad_slab_pick(int G, int B, int D, int H, int W, int Cin, int Cout, int pad) {
  static const int env = [] {
    const char* e = getenv("NIDT_WG_SLAB");
    return e ? atoi(e) : 0;
  }();
  if (!env || !conv3d_wgrad_slab_ok(B, D, H, W, Cin, Cout, pad)) return 0;
  return conv3d_wgrad_tri_pick(G, B, D, H, W, Cin, Cout, pad) || env == 2 ? 1 : 0;
}

int conv3d_wgrad_slab_nsplit(int G, int B, int D, int H, int W, int Cin, int Cout, int pad) {
  const int Mg = B * conv_out_n(D, pad) * conv_out_n(H, pad) * conv_out_n(W, pad);
  // one 12-wave block per CU; ~3x the MFMAs of a k_conv_wgrad_tri step
  return wgrad_nsplit_base(G * (Cout / 64) * 3 * (Cin / 64), G, Mg, 27 * Cin, Cout, 1.5, 0.0, 256.0);
}

int conv3d_wgrad_slab_table_size(int B, int D, int H, int W, int pad) {
  const int Mg = B * conv_out_n(D, pad) * conv_out_n(H, pad) * conv_out_n(W, pad);
  const int U = ws_u(B, D, H, W, pad);
  NIDT_REQUIRE(U > 0, "conv3d_wgrad_slab_table_size: shape not eligible");
  return ceil_div(Mg, 64) * (2 * U + 64);
}

void conv3d_wgrad_slab_table(uintptr_t tab, int B, int D, int H, int W, int pad, uintptr_t stream) {
  const int Mg = B * conv_out_n(D, pad) * conv_out_n(H, pad) * conv_out_n(W, pad);
  const int U = ws_u(B, D, H, W, pad);
  NIDT_REQUIRE(U > 0, "conv3d_wgrad_slab_table: shape not eligible");
  hipLaunchKernelGGL(k_union_table, dim3(ceil_div(Mg, 64)), dim3(64), 0, as_stream(stream), ptr<int>(tab), U, 64, Mg,
                     D, H, W, pad, 2 * (W + 2 * pad) + 2);
  NIDT_CHECK(hipGetLastError());
}

void conv3d_wgrad_slab(uintptr_t x, uintptr_t dy, uintptr_t part, uintptr_t grad, int64_t ldg, int64_t off, int G,
                       int B, int D, int H, int W, int Cin, int Cout, int pad, int nsplit, float scale, uintptr_t stab,
                       uintptr_t stream) {
  NIDT_REQUIRE(conv3d_wgrad_slab_ok(B, D, H, W, Cin, Cout, pad), "conv3d_wgrad_slab: shape not eligible");
  NIDT_REQUIRE(stab != 0 && nsplit >= 1, "conv3d_wgrad_slab: needs the step table");
  ConvWgTriArgs d;
  d.x = ptr<const uint16_t>(x); d.dy = ptr<const uint16_t>(dy); d.stab = ptr<const int>(stab); d.part = ptr<float>(part);
  d.D = D; d.H = H; d.W = W; d.Cin = Cin; d.Cout = Cout; d.pad = pad;
  d.Mg = B * conv_out_n(D, pad) * conv_out_n(H, pad) * conv_out_n(W, pad);
  d.K = 27 * Cin; d.nsplit = nsplit; d.G = G;
  d.chunk = ((ceil_div(d.Mg, nsplit) + 63) / 64) * 64;
  d.nKT = 3 * (Cin / 64); d.nCT = Cout / 64;
  d.nstab = ceil_div(d.Mg, 64);
  d.xclient = (int64_t)B * D * H * W * Cin;
  NIDT_REQUIRE(d.xclient * 2 < (1ll << 31) && (int64_t)d.Mg * Cout * 2 < (1ll << 31),
               "conv3d_wgrad_slab: per-client tensors must stay below 2 GiB (32-bit buffer offsets)");
  const int64_t nwg = (int64_t)d.nKT * d.nCT * nsplit * G;
  NIDT_REQUIRE(nwg < (1ll << 31), "conv3d_wgrad_slab: grid too large");
  hipStream_t s = as_stream(stream);
  // [ADMA] asm-issued stage DMA (k_conv_wgrad_tri); NIDT_WGS_ADMA=0: the intrinsic (A/B)
  static const int sadma = [] {
    const char* e = getenv("NIDT_WGS_ADMA");
    return e ? atoi(e) : 1;
  }();
  if (sadma) {
    if (pad) hipLaunchKernelGGL((k_conv_wgrad_slab<152, true, true>), dim3((unsigned)nwg), dim3(768), 0, s, d);
    else hipLaunchKernelGGL((k_conv_wgrad_slab<152, false, true>), dim3((unsigned)nwg), dim3(768), 0, s, d);
  } else if (pad) {
    hipLaunchKernelGGL((k_conv_wgrad_slab<152, true>), dim3((unsigned)nwg), dim3(768), 0, s, d);
  } else {
    hipLaunchKernelGGL((k_conv_wgrad_slab<152, false>), dim3((unsigned)nwg), dim3(768), 0, s, d);
  }
  NIDT_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_wgrad_reduce, dim3(Cout, G), dim3(256), 27 * (Cin + 1) * sizeof(float), s, ptr<const float>(part),
                     nsplit, G, Cout, Cin, 27, ptr<float>(grad), ldg, off, scale);
  NIDT_CHECK(hipGetLastError());
}

// positions table of a general conv (kt taps, stride st, h/w padding pad, depth padding padd): Mg = B*Do*Ho*Wo rows
void conv_pos_table_g(uintptr_t tab, int B, int D, int H, int W, int kt, int st, int pad, int padd, uintptr_t stream) {
  const int kd = kt == 27 ? 3 : 1, khw = kt == 1 ? 1 : 3;
  const int Do = conv_out_dim(D, kd, st, padd), Ho = conv_out_dim(H, khw, st, pad), Wo = conv_out_dim(W, khw, st, pad);
  NIDT_REQUIRE(Do > 0 && Ho > 0 && Wo > 0, "conv_pos_table: empty output");
  const int Mg = B * Do * Ho * Wo;
  NIDT_REQUIRE((int64_t)B * D * H * W < (1ll << 31), "conv3d_pos_table: volume too large for 32-bit offsets");
  hipLaunchKernelGGL(k_conv_pos_table, dim3(ceil_div(Mg, 256)), dim3(256), 0, as_stream(stream), ptr<int2>(tab), Mg,
                     D, H, W, Do, Ho, Wo, st, padd, pad);
  NIDT_CHECK(hipGetLastError());
}

void conv3d_pos_table(uintptr_t tab, int B, int D, int H, int W, int pad, uintptr_t stream) {
  conv_pos_table_g(tab, B, D, H, W, 27, 1, pad, pad, stream);
}

static void conv_wgrad_impl(uintptr_t x, uintptr_t xs, uintptr_t xt, uintptr_t dy, uintptr_t part, uintptr_t grad,
                            int64_t ldg, int64_t off, int G, int B, int D, int H, int W, int Cin, int Cout, int pad,
                            int nsplit, float scale, uintptr_t ptab, uintptr_t stream, int kt, int st, int padd) {
  NIDT_REQUIRE(Cin % 64 == 0, "conv3d_wgrad: Cin must be a multiple of 64");
  NIDT_REQUIRE(kt == 27 || kt == 9 || kt == 1, "conv_wgrad: taps 27, 9 or 1");
  NIDT_REQUIRE((kt == 27 && st == 1 && padd == pad) || (ptab && !xs),
               "conv_wgrad: 9/1-tap or strided convs need the LDS-DMA path (position table, no input transform)");
  NIDT_REQUIRE(nsplit >= 1, "conv_wgrad: nsplit >= 1");
  NIDT_REQUIRE((ptab && !xs) ? (int64_t)Cin * kt <= 27 * kMaxCin : Cin <= 192,
               "conv3d_wgrad: taps x Cin <= 27 x 512 (LDS-DMA path with a position table), else Cin <= 192");
  NIDT_REQUIRE(Cout % kWgCO == 0, "conv3d_wgrad: Cout must be a multiple of 64");
  if (wg1x1_on(Cin, Cout, kt, st) && pad == 0 && padd == 0 && !xs) {  // rows of X and dY are the same positions
    wgrad1x1_g(x, dy, part, grad, ldg, off, G, (int64_t)B * D * H * W, Cout, Cin, nsplit, scale, stream);
    return;
  }
  ConvWgArgs a;
  a.x = ptr<const uint16_t>(x); a.xs = ptr<const float>(xs); a.xt = ptr<const float>(xt);
  a.dy = ptr<const uint16_t>(dy); a.part = ptr<float>(part);
  a.B = B; a.D = D; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.pad = pad; a.G = G;
  {
    const int kd = kt == 27 ? 3 : 1, khw = kt == 1 ? 1 : 3;
    a.Do = conv_out_dim(D, kd, st, padd); a.Ho = conv_out_dim(H, khw, st, pad); a.Wo = conv_out_dim(W, khw, st, pad);
  }
  NIDT_REQUIRE(a.Do > 0 && a.Ho > 0 && a.Wo > 0, "conv_wgrad: empty output");
  a.Mg = B * a.Do * a.Ho * a.Wo;
  a.K = kt * Cin;
  a.nsplit = nsplit;
  a.chunk = ((ceil_div(a.Mg, nsplit) + 31) / 32) * 32;
  hipStream_t s = as_stream(stream);
  bool direct = false;
  if (ptab && !xs) {
    ConvWgDmaArgs d;
    d.x = a.x; d.dy = a.dy; d.ptab = ptr<const int2>(ptab); d.part = a.part;
    d.D = D; d.H = H; d.W = W; d.Cin = Cin; d.Cout = Cout; d.Mg = a.Mg; d.K = a.K; d.nsplit = nsplit; d.G = G;
    d.chunk = ((ceil_div(a.Mg, nsplit) + kWdPos - 1) / kWdPos) * kWdPos;
    // NIDT_WG_NCH=2: 128-channel blocks where Cout allows (8 waves, the X tile feeds both halves).  Measured slower
    // than two resident 64-channel blocks per CU (conv2 wgrad 3.91 -> 4.14 ms at 64 clients, 0.505 -> 0.542 ms
    // at 8; profiles/r2_ab_wgrad_nch.txt): the kernel is latency/barrier bound, not L2->LDS bandwidth bound.
    static const int nch_env = [] {
      const char* e = getenv("NIDT_WG_NCH");
      return e ? atoi(e) : 0;
    }();
    const int nch = (Cout % 128 == 0 && nch_env == 2) ? 2 : 1;
    d.nKT = ceil_div(a.K, kWgKC); d.nCT = Cout / (kWgCO * nch);
    d.xclient = (int64_t)B * D * H * W * Cin;
    // [WG-DIRECT] one split: the kernel writes the gradient rows (no fp32 slab round trip, no reduce launch).  The
    // rows are [Cout][Cin][kt] and a block owns 1-4 taps of a channel slice, so for kt > 1 its stores are 4-B
    // scatters at a kt-float stride: CIFAR DisPFL (100 clients) -70 ms/round net, SubAvg (10 clients) +10 ms
    // (profiles/r5_pack_fuse_wg_direct.txt).  NIDT_WG_DIRECT=1 (default): 1x1 layers only (contiguous rows), 2: every layer,
    // 0: off (A/B; the results are bitwise equal either way)
    static const int direct_env = [] {
      const char* e = getenv("NIDT_WG_DIRECT");
      return e ? atoi(e) : 1;
    }();
    direct = nsplit == 1 && (direct_env == 2 || (direct_env == 1 && kt == 1));
    d.grad = direct ? ptr<float>(grad) : nullptr;
    d.ldg = ldg; d.off = off; d.scale = scale; d.kt = kt;
    NIDT_REQUIRE(d.xclient * 2 < (1ll << 31) && (int64_t)a.Mg * Cout * 2 < (1ll << 31),
                 "conv3d_wgrad: per-client tensors must stay below 2 GiB (32-bit buffer offsets)");
    const int64_t nwg = (int64_t)d.nKT * d.nCT * nsplit * G;
    NIDT_REQUIRE(nwg < (1ll << 31), "conv3d_wgrad: grid too large");
    // [SCHED] k-step schedule (kstep_sched): AlexNet conv3-5 weight gradients at 8 clients -2.7 %, config 5 12.16 ->
    // 12.10 s/round (profiles/r4_ab_sched_more.txt); NIDT_WGD_SCHED=0: the compiler's schedule (A/B)
    static const int wsched = [] {
      const char* e = getenv("NIDT_WGD_SCHED");
      return e ? atoi(e) : 1;
    }();
    // [ADMA] asm-issued stage DMA (k_conv_wgrad_tri); NIDT_WGD_ADMA=0: the intrinsic (A/B)
    static const int wadma = [] {
      const char* e = getenv("NIDT_WGD_ADMA");
      return e ? atoi(e) : 1;
    }();
    if (wsched && wadma) {
      if (nch == 2) hipLaunchKernelGGL((k_conv_wgrad_dma<2, true, true>), dim3((unsigned)nwg), dim3(512), 0, s, d);
      else hipLaunchKernelGGL((k_conv_wgrad_dma<1, true, true>), dim3((unsigned)nwg), dim3(256), 0, s, d);
    } else if (wsched) {
      if (nch == 2) hipLaunchKernelGGL((k_conv_wgrad_dma<2, true>), dim3((unsigned)nwg), dim3(512), 0, s, d);
      else hipLaunchKernelGGL((k_conv_wgrad_dma<1, true>), dim3((unsigned)nwg), dim3(256), 0, s, d);
    } else if (nch == 2) {
      hipLaunchKernelGGL(k_conv_wgrad_dma<2>, dim3((unsigned)nwg), dim3(512), 0, s, d);
    } else {
      hipLaunchKernelGGL(k_conv_wgrad_dma<1>, dim3((unsigned)nwg), dim3(256), 0, s, d);
    }
  } else {
    dim3 grid(ceil_div(a.K, kWgKC), Cout / kWgCO, G * nsplit);
    if (xs) hipLaunchKernelGGL((k_conv_wgrad<true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((k_conv_wgrad<false>), grid, dim3(256), 0, s, a);
  }
  NIDT_CHECK(hipGetLastError());
  if (direct) return;
  hipLaunchKernelGGL(k_wgrad_reduce, dim3(Cout, G), dim3(256), kt * (Cin + 1) * sizeof(float), s,
                     ptr<const float>(part), nsplit, G, Cout, Cin, kt,
                     ptr<float>(grad), ldg, off, scale);
  NIDT_CHECK(hipGetLastError());
}

void conv3d_wgrad(uintptr_t x, uintptr_t xs, uintptr_t xt, uintptr_t dy, uintptr_t part, uintptr_t grad, int64_t ldg,
                  int64_t off, int G, int B, int D, int H, int W, int Cin, int Cout, int pad, int nsplit, float scale,
                  uintptr_t ptab, uintptr_t stream) {
  conv_wgrad_impl(x, xs, xt, dy, part, grad, ldg, off, G, B, D, H, W, Cin, Cout, pad, nsplit, scale, ptab, stream, 27, 1,
                  pad);
}

// General wgrad (position table from conv_pos_table_g with the same geometry): grad rows get PyTorch-layout
// [Cout][Cin][kt] fp32 at offset off (times scale).
void conv_wgrad_g(uintptr_t x, uintptr_t dy, uintptr_t part, uintptr_t grad, int64_t ldg, int64_t off, int G, int B,
                  int D, int H, int W, int Cin, int Cout, int kt, int st, int pad, int padd, int nsplit, float scale,
                  uintptr_t ptab, uintptr_t stream) {
  NIDT_REQUIRE(ptab != 0, "conv_wgrad_g: needs a position table");
  conv_wgrad_impl(x, 0, 0, dy, part, grad, ldg, off, G, B, D, H, W, Cin, Cout, pad, nsplit, scale, ptab, stream, kt, st,
                  padd);
}

// ------------------------------------------------------------------------------------------------
// Pack fp32 PyTorch-layout weights [Cout][Cin][27] (row g of theta at offset off) into
// wp [G][Cout][27][Cin] bf16 (block per (co, g): coalesced read of the [Cin][27] row, LDS transpose) and, for dgrad,
// wt [G][Cin][27][Cout] with the taps flipped (64x64 LDS-tiled transpose of wp per tap).
__global__ __launch_bounds__(256) void k_pack_wp(const float* __restrict__ theta, int64_t ldt, int64_t off, int Cout,
                                                 int Cin, int kt, int cin_src, float scale, uint16_t* __restrict__ wp) {
  extern __shared__ float row[];  // [Cin][kt], dynamic: sized to the layer (not the 512-channel maximum)
  const int co = blockIdx.x, g = blockIdx.y;
  const int K = kt * Cin, Ks = kt * cin_src;  // source rows may carry fewer input channels (zero-padded here)
  const float* src = theta + (int64_t)g * ldt + off + (int64_t)co * Ks;
  if (Ks == K && (reinterpret_cast<uintptr_t>(src) & 15) == 0 && K % 4 == 0) {  // 16-B source loads
    for (int e = 4 * threadIdx.x; e < K; e += 4 * 256)
      *reinterpret_cast<float4*>(row + e) = *reinterpret_cast<const float4*>(src + e);
  } else {
    for (int e = threadIdx.x; e < K; e += 256) row[e] = e < Ks ? src[e] : 0.f;
  }
  __syncthreads();
  uint16_t* dst = wp + ((int64_t)g * Cout + co) * K;
  if (Cin % 8 == 0) {  // 16-B stores: 8 channels of one tap per lane (K % 8 == 0: aligned)
    for (int e = 8 * threadIdx.x; e < K; e += 8 * 256) {
      const int t = e / Cin, ci = e - t * Cin;
      const float* r = row + ci * kt + t;
      *reinterpret_cast<uint4*>(dst + e) =
          make_uint4(pack_bf16x2(r[0] * scale, r[kt] * scale), pack_bf16x2(r[2 * kt] * scale, r[3 * kt] * scale),
                     pack_bf16x2(r[4 * kt] * scale, r[5 * kt] * scale), pack_bf16x2(r[6 * kt] * scale, r[7 * kt] * scale));
    }
    return;
  }
  for (int e = 2 * threadIdx.x; e < K; e += 2 * 256) {  // e, e+1 share the tap (Cin even); K even: 4-B aligned pairs
    const int t = e / Cin, ci = e - t * Cin;
    *reinterpret_cast<uint32_t*>(dst + e) = pack_bf16x2(row[ci * kt + t] * scale, row[(ci + 1) * kt + t] * scale);
  }
}

__global__ __launch_bounds__(256) void k_pack_wt(const uint16_t* __restrict__ wp, int Cout, int Cin, int kt,
                                                 uint16_t* __restrict__ wt) {
  // 16-B global pieces (8 channels per lane), transpose through a padded LDS tile (as pack.hip k_pack_trans)
  __shared__ uint16_t tile[64][72];  // [co][ci]
  const int ci0 = blockIdx.x * 64, co0 = blockIdx.y * 64;
  const int g = blockIdx.z / kt, t = blockIdx.z - g * kt;
  const int q = threadIdx.x & 7, r0 = threadIdx.x >> 3;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = r0 + 32 * h, co = co0 + r, ci = ci0 + 8 * q;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (co < Cout && ci < Cin) v = *reinterpret_cast<const uint4*>(wp + (((int64_t)g * Cout + co) * kt + t) * Cin + ci);
    *reinterpret_cast<uint4*>(&tile[r][8 * q]) = v;
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = r0 + 32 * h, ci = ci0 + r, co = co0 + 8 * q;
    if (ci >= Cin || co >= Cout) continue;
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      w[k] = (uint32_t)tile[8 * q + 2 * k][r] | ((uint32_t)tile[8 * q + 2 * k + 1][r] << 16);
    *reinterpret_cast<uint4*>(wt + (((int64_t)g * Cin + ci) * kt + (kt - 1 - t)) * Cout + co) =
        make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// General pack: theta rows hold [Cout][cin_src][kt] fp32 (PyTorch layout); wp [G][Cout][kt][Cin] bf16 with input
// channels cin_src..Cin-1 zero (channel-padded first layers), wt (dgrad, optional) [G][Cin][kt][Cout] tap-flipped.
void pack_conv_wk(uintptr_t theta, int64_t ldt, int64_t off, int G, int Cout, int Cin, int kt, int cin_src,
                  float scale, uintptr_t wp, uintptr_t wt, uintptr_t stream) {
  NIDT_REQUIRE((int64_t)Cin * kt <= 27 * kMaxCin && Cin % 2 == 0, "pack_conv_w: Cin even, taps x Cin <= 27 x 512");
  NIDT_REQUIRE(kt == 27 || kt == 9 || kt == 1, "pack_conv_w: taps 27, 9 or 1");
  NIDT_REQUIRE(cin_src >= 1 && cin_src <= Cin, "pack_conv_w: 1 <= cin_src <= Cin");
  NIDT_REQUIRE(!wt || (Cin % 8 == 0 && Cout % 8 == 0), "pack_conv_w: the transposed image needs Cin, Cout % 8 == 0");
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(k_pack_wp, dim3(Cout, G), dim3(256), kt * Cin * sizeof(float), s, ptr<const float>(theta), ldt,
                     off, Cout, Cin, kt, cin_src, scale, ptr<uint16_t>(wp));
  NIDT_CHECK(hipGetLastError());
  if (wt) {
    hipLaunchKernelGGL(k_pack_wt, dim3(ceil_div(Cin, 64), ceil_div(Cout, 64), G * kt), dim3(256), 0, s,
                       ptr<const uint16_t>(wp), Cout, Cin, kt, ptr<uint16_t>(wt));
    NIDT_CHECK(hipGetLastError());
  }
}

void pack_conv_w(uintptr_t theta, int64_t ldt, int64_t off, int G, int Cout, int Cin, float scale, uintptr_t wp,
                 uintptr_t wt, uintptr_t stream) {
  pack_conv_wk(theta, ldt, off, G, Cout, Cin, 27, Cin, scale, wp, wt, stream);
}

// h = relu(y * s + t) in bf16 (materialises BN+ReLU once so the consuming conv and its wgrad read it plain)
__global__ void k_bn_relu_apply(const uint16_t* __restrict__ y, const float* __restrict__ sc,
                                const float* __restrict__ sh, uint16_t* __restrict__ h, int64_t npos, int C, int S) {
  const int C8 = C / 8;
  const int64_t tot = npos * C8;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    const int cg = (int)(e % C8);
    const int64_t pos = e / C8;
    const int g = (int)(pos / S);
    const uint4 v = *reinterpret_cast<const uint4*>(y + pos * C + cg * 8);
    *reinterpret_cast<uint4*>(h + pos * C + cg * 8) = xform8(v, sc + (int64_t)g * C + cg * 8, sh + (int64_t)g * C + cg * 8, true);
  }
}

// y: [G*B*S_per_sample positions][C]; S = positions per client (B * D*H*W)
void bn_relu_apply(uintptr_t y, uintptr_t sc, uintptr_t sh, uintptr_t h, int64_t npos, int C, int S, uintptr_t stream) {
  NIDT_REQUIRE(C % 8 == 0, "bn_relu_apply: C % 8");
  const int64_t tot = npos * (C / 8);
  hipLaunchKernelGGL(k_bn_relu_apply, dim3((unsigned)std::min<int64_t>(16384, (tot + 255) / 256)), dim3(256), 0,
                     as_stream(stream), ptr<const uint16_t>(y), ptr<const float>(sc), ptr<const float>(sh),
                     ptr<uint16_t>(h), npos, C, S);
  NIDT_CHECK(hipGetLastError());
}

}  // namespace nidt
