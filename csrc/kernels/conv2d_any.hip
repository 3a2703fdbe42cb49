// Client-grouped 2-D convolution of any kernel size / channel count (the reference's small image models: lenet5,
// cnn_cifar10/100, the EMNIST CNNs, VGG-11/16 — fedml_experiments/standalone/subavg/main_subavg.py:143-158,
// fedml_api/model/cv/{lenet5,cnn_cifar10,cnn,vgg}.py), replacing the per-layer vmapped library convolutions of the
// batched 2-D engine.  The ResNet-18 engine's kernels (conv3d.hip) need 64-channel multiples and 1x1 / 3x3 taps;
// these models have 5x5 taps and 1 / 3 / 6 / 20 / 50-channel layers.
//
//  * forward (and the stride-1 data gradient, as a forward over dY with the flipped, transposed weights and padding
//    k - 1 - p): an implicit GEMM on channels-last rows, Y[g][m][co] = sum_{t, ci} X[g][pix(m, t)][ci] W[g][co][t][ci],
//    16x16x32 bf16 MFMA, block = 4 waves = 64 positions x 64 output channels, wave = 32 x 32.  K = kt x Cinp
//    (Cinp = Cin rounded up to 8) walks 32 at a time; a lane's 8 consecutive k are 8 channels of one tap: one 16-B load
//    when the channel stride allows it, element loads otherwise (first layers); out-of-image taps read zeros;
//  * weight gradient: per (client, tap, 64 x 64 channel tile, 256-position chunk) block, dY and the tap-shifted X rows
//    staged through LDS as fp32, 4 x 4 register micro-tiles of fp32 FMAs, one deterministic fp32 partial per chunk
//    (the host sums the chunks in a fixed order).
#include "common.h"

namespace nidt {

struct C2Args {
  const uint16_t* x;   // [G*B][H][W][cs]   bf16
  const uint16_t* w;   // [G][coutp][kt][cinp] bf16 (zero padded)
  const float* bias;   // [G][cout] or null
  uint16_t* y;         // [G*B][Ho][Wo][cout] bf16
  int G, B, H, W, cin, cs, cinp, cout, coutp, k, pad, Ho, Wo;
};

template <bool VEC>
__device__ __forceinline__ bf16x8 c2_xfrag(const C2Args& a, const uint16_t* xb, int oh, int ow, bool mval, int k0) {
  const int t = k0 / a.cinp, ci0 = k0 - t * a.cinp;
  const int kh = t / a.k, kw = t - kh * a.k;
  const int ih = oh + kh - a.pad, iw = ow + kw - a.pad;
  bf16x8 v = {};
  if (!mval || t >= a.k * a.k || (unsigned)ih >= (unsigned)a.H || (unsigned)iw >= (unsigned)a.W) return v;
  const uint16_t* p = xb + ((int64_t)ih * a.W + iw) * a.cs + ci0;
  if (VEC) return *reinterpret_cast<const bf16x8*>(p);
  uint16_t e[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) e[j] = ci0 + j < a.cin ? p[j] : (uint16_t)0;
  return __builtin_bit_cast(bf16x8, make_uint4(e[0] | (uint32_t)e[1] << 16, e[2] | (uint32_t)e[3] << 16,
                                               e[4] | (uint32_t)e[5] << 16, e[6] | (uint32_t)e[7] << 16));
}

// VEC: cs % 8 == 0 and cin % 8 == 0 (every 8-channel piece is a whole, aligned 16-B load)
template <bool VEC>
__global__ __launch_bounds__(256) void k_conv2d_any_fwd(C2Args a) {
  const int g = blockIdx.z, co0 = blockIdx.y * 64;
  const int M = a.B * a.Ho * a.Wo;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int wp = wid & 1, wc = wid >> 1;           // wave: positions half wp, channels half wc
  const int mb = blockIdx.x * 64 + wp * 32;
  // this lane's two B columns (positions mb + fr, mb + 16 + fr)
  const uint16_t* xb[2];
  int oh[2], ow[2];
  bool mv[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int m = mb + 16 * j + fr;
    mv[j] = m < M;
    const int mm = mv[j] ? m : 0;
    const int n = mm / (a.Ho * a.Wo), r = mm - n * a.Ho * a.Wo;
    oh[j] = r / a.Wo;
    ow[j] = r - oh[j] * a.Wo;
    xb[j] = a.x + ((int64_t)(g * a.B + n) * a.H * a.W) * a.cs;
  }
  const int KT = a.k * a.k * a.cinp, nks = (KT + 31) / 32;
  const uint16_t* wg = a.w + (int64_t)g * a.coutp * (a.k * a.k) * a.cinp;
  f32x4 acc[2][2] = {};
  for (int s = 0; s < nks; ++s) {
    const int k0 = 32 * s + 8 * fq;
    bf16x8 fa[2], fb[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int co = co0 + wc * 32 + 16 * i + fr;
      fa[i] = k0 < KT ? *reinterpret_cast<const bf16x8*>(wg + (int64_t)co * KT + k0) : bf16x8{};
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) fb[j] = c2_xfrag<VEC>(a, xb[j], oh[j], ow[j], mv[j] && k0 < KT, k0);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
  }
  // lane: output channels co0 + wc 32 + 16 i + 4 fq + r (r = 0..3) of position mb + 16 j + fr
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int m = mb + 16 * j + fr;
    if (m >= M) continue;
    uint16_t* yp = a.y + ((int64_t)g * M + m) * a.cout;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = co0 + wc * 32 + 16 * i + 4 * fq;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + (a.bias && c + r < a.cout ? a.bias[g * a.cout + c + r] : 0.f);
      if (c + 3 < a.cout && (a.cout & 3) == 0) {
        *reinterpret_cast<uint2*>(yp + c) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (c + r < a.cout) yp[c + r] = f32_to_bf16(v[r]);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// weight gradient partials: part[chunk][g][co][t][ci] = sum over the chunk's positions m of
// dY[g][m][co] * X[g][pix(m, t)][ci]  (stride 1)
constexpr int kC2WgM = 256;   // positions per block
constexpr int kC2WgS = 32;    // positions per LDS stage

struct C2WgArgs {
  const uint16_t* x;    // [G*B][H][W][cs]
  const uint16_t* dy;   // [G*B][Ho][Wo][cout]
  float* part;          // [nchunk][G][cout][kt][cin]
  int G, B, H, W, cin, cs, cout, k, pad, Ho, Wo, nchunk;
};

__global__ __launch_bounds__(256) void k_conv2d_any_wgrad(C2WgArgs a) {
  __shared__ float sd[kC2WgS][64 + 1];
  __shared__ float sx[kC2WgS][64 + 1];
  const int chunk = blockIdx.x, t = blockIdx.y;
  const int nco = (a.cout + 63) / 64, nci = (a.cin + 63) / 64;
  int z = blockIdx.z;
  const int cit = z % nci;
  z /= nci;
  const int cot = z % nco, g = z / nco;
  const int co0 = cot * 64, ci0 = cit * 64;
  const int kh = t / a.k, kw = t - kh * a.k;
  const int M = a.B * a.Ho * a.Wo;
  const int m0 = chunk * kC2WgM, m1 = min(M, m0 + kC2WgM);
  const int tid = threadIdx.x, ty = tid >> 4, tx = tid & 15;  // micro-tile: co 4 ty .. +3, ci 4 tx .. +3
  float acc[4][4] = {};
  for (int ms = m0; ms < m1; ms += kC2WgS) {
    // stage 32 positions x 64 channels of dY and of the tap-shifted X (8 elements per thread each)
    for (int e = tid; e < kC2WgS * 64; e += 256) {
      const int r = e >> 6, c = e & 63, m = ms + r;
      float dv = 0.f, xv = 0.f;
      if (m < m1) {
        const int n = m / (a.Ho * a.Wo), q = m - n * a.Ho * a.Wo;
        const int oh = q / a.Wo, ow = q - oh * a.Wo;
        if (co0 + c < a.cout) dv = bf16_to_f32(a.dy[((int64_t)g * M + m) * a.cout + co0 + c]);
        const int ih = oh + kh - a.pad, iw = ow + kw - a.pad;
        if (ci0 + c < a.cin && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W)
          xv = bf16_to_f32(a.x[(((int64_t)(g * a.B + n) * a.H + ih) * a.W + iw) * a.cs + ci0 + c]);
      }
      sd[r][c] = dv;
      sx[r][c] = xv;
    }
    __syncthreads();
#pragma unroll 4
    for (int r = 0; r < kC2WgS; ++r) {
      float d[4], x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        d[u] = sd[r][4 * ty + u];
        x[u] = sx[r][4 * tx + u];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[u][v] = fmaf(d[u], x[v], acc[u][v]);
    }
    __syncthreads();
  }
  const int kt = a.k * a.k;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int co = co0 + 4 * ty + u;
    if (co >= a.cout) continue;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int ci = ci0 + 4 * tx + v;
      if (ci < a.cin) a.part[((((int64_t)chunk * a.G + g) * a.cout + co) * kt + t) * a.cin + ci] = acc[u][v];
    }
  }
}

void conv2d_any_fwd(uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, int G, int B, int H, int W, int cin, int cs,
                    int cout, int k, int pad, uintptr_t stream) {
  C2Args a;
  a.x = ptr<const uint16_t>(x);
  a.w = ptr<const uint16_t>(w);
  a.bias = ptr<const float>(bias);
  a.y = ptr<uint16_t>(y);
  a.G = G; a.B = B; a.H = H; a.W = W; a.cin = cin; a.cs = cs; a.cinp = (cin + 7) / 8 * 8;
  a.cout = cout; a.coutp = (cout + 63) / 64 * 64; a.k = k; a.pad = pad;
  a.Ho = H + 2 * pad - k + 1;
  a.Wo = W + 2 * pad - k + 1;
  NIDT_REQUIRE(G > 0 && B > 0 && a.Ho > 0 && a.Wo > 0 && cs >= cin && k >= 1, "conv2d_any_fwd: shape");
  NIDT_REQUIRE((int64_t)G * a.coutp * k * k * a.cinp < (int64_t(1) << 31), "conv2d_any_fwd: weight image size");
  const int M = B * a.Ho * a.Wo;
  const dim3 grid((M + 63) / 64, a.coutp / 64, G);
  if (cs % 8 == 0 && cin % 8 == 0)
    hipLaunchKernelGGL(k_conv2d_any_fwd<true>, grid, dim3(256), 0, as_stream(stream), a);
  else
    hipLaunchKernelGGL(k_conv2d_any_fwd<false>, grid, dim3(256), 0, as_stream(stream), a);
  NIDT_CHECK(hipGetLastError());
}

int conv2d_any_wgrad_chunks(int B, int Ho, int Wo) { return (B * Ho * Wo + kC2WgM - 1) / kC2WgM; }

void conv2d_any_wgrad(uintptr_t x, uintptr_t dy, uintptr_t part, int G, int B, int H, int W, int cin, int cs, int cout,
                      int k, int pad, uintptr_t stream) {
  C2WgArgs a;
  a.x = ptr<const uint16_t>(x);
  a.dy = ptr<const uint16_t>(dy);
  a.part = ptr<float>(part);
  a.G = G; a.B = B; a.H = H; a.W = W; a.cin = cin; a.cs = cs; a.cout = cout; a.k = k; a.pad = pad;
  a.Ho = H + 2 * pad - k + 1;
  a.Wo = W + 2 * pad - k + 1;
  NIDT_REQUIRE(G > 0 && B > 0 && a.Ho > 0 && a.Wo > 0 && cs >= cin, "conv2d_any_wgrad: shape");
  a.nchunk = conv2d_any_wgrad_chunks(B, a.Ho, a.Wo);
  const int nco = (cout + 63) / 64, nci = (cin + 63) / 64;
  const dim3 grid(a.nchunk, k * k, G * nco * nci);
  hipLaunchKernelGGL(k_conv2d_any_wgrad, grid, dim3(256), 0, as_stream(stream), a);
  NIDT_CHECK(hipGetLastError());
}

}  // namespace nidt
