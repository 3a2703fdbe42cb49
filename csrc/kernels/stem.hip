// Stem of the 3D ResNet (BASELINE config 5; models/resnet3d.py ResNet3D: Conv3d(1, 64, 7, stride 2, pad 3, no bias)
// -> BatchNorm3d -> ReLU -> MaxPool3d(3, stride 2, pad 1)) on full-resolution 1x121x145x121 volumes, client-grouped
// (per-client weights, BN affine and batch statistics), forward and backward — the largest-activation layer of the
// network (61x73x61x64 per sample), which the conv-kernel family of conv3d.hip does not serve (7^3 taps, 1 channel).
//
// Polyphase form.  Input voxel 2o + k - 3 of output o and tap k in [0, 7) is written 2(o + j - 2) + r with
// k = 2j + r - 1, j in [0, 4), r in {0, 1} (7 of the 8 (j, r) pairs are taps).  The uint8 volume becomes a
// polyphase image Xp[z'][y'][x'][r] = X[2z' - 4 + rd][2y' - 4 + rh][2x' - 4 + rw] (zero outside) of 64 x 76 x 64
// voxels x 8 phases, and the stride-2 7^3 conv a stride-1 4^3 conv over 8 phase channels: K = 64 tap groups x 8
// phases = 512 MFMA k-slots (343 live).  uint8 values are exact in bf16, the 1/255 input scale is applied to the
// fp32 accumulators.
//
//  k_stem_polyphase   raw uint8 [N][121][145][121] -> Xp (forward, [z'][y'][x'][8]) and the phase-major copy
//                     Xq [8][z'][y'][x'] the weight gradient stages from.
//  k_stem_fwd         block = (sample, output plane od): walks the 73 output rows; the input rows of the 4 x 4
//                     (jd, jh) taps live in an LDS ring (one new y' row per output row), A = packed bf16 weights in
//                     registers (4 waves x 32 channels x 32 positions), 16 k-steps of 16x16x32 bf16 MFMA per row;
//                     epilogue: bf16 output + per-block BN statistics (shifted sums -> block mean and M2, the
//                     format bn.hip's k_bn_finalize merges).
//  k_stem_pool        z = relu(y * scale + shift), 3^3 / stride 2 / pad 1 max with the first-max-in-(d,h,w)-order
//                     argmax of PyTorch's max_pool3d -> pooled bf16 + uint8 window index.
//  k_stem_unpool      dz at conv resolution = sum of the (bf16) pooled gradients of the (<= 8) windows whose argmax is this
//                     voxel, times the ReLU mask; per-block sums of dz and dz * xhat for the BN backward.
//  k_stem_bn_bwd_fin  dgamma / dbeta into the gradient rows and the coefficients of dy = a dz + b y + d.
//  k_stem_wgrad       dW[c][slot] = sum_pos dy[pos][c] Xq[pos + tap][phase]: block = (sample, chunk of od planes,
//                     jd); A = dy^T read with ds_read_b64_tr_b16 from a [pos][c] LDS tile, B = four x-shifted
//                     copies (jw = 0..3) of the phase-major input rows so every fragment is an aligned 16-B read;
//                     fp32 partial slabs, k_stem_wgrad_fin sums them per client into the PyTorch-layout row.
#include "common.h"

namespace nidt {

// extents: input D x H x W (ABCD: 121 x 145 x 121), conv output O* = (n - 1) / 2 + 1 (61 x 73 x 61, at most 64 wide:
// one block row), polyphase grid P* = O* + 3, pooled Q* = (O* - 1) / 2 + 1 (31 x 37 x 31)
struct StemDims {
  int D, H, W, OD, OH, OW, PZ, PY, PX, QD, QH, QW;
};
static StemDims stem_dims(int D, int H, int W) {
  StemDims d;
  d.D = D; d.H = H; d.W = W;
  d.OD = (D - 1) / 2 + 1; d.OH = (H - 1) / 2 + 1; d.OW = (W - 1) / 2 + 1;
  d.PZ = d.OD + 3; d.PY = d.OH + 3; d.PX = d.OW + 3;
  d.QD = (d.OD - 1) / 2 + 1; d.QH = (d.OH - 1) / 2 + 1; d.QW = (d.OW - 1) / 2 + 1;
  return d;
}
constexpr int kSC = 64;                          // stem channels
constexpr int kSK = 512;                         // k-slots (64 tap groups x 8 phases)
constexpr int kSRing = 5;                        // y' ring rows of the forward halo
constexpr int kSHX = 68;                         // halo x extent (64 positions + 3 taps, padded)
constexpr int kWgOD = 8;                         // od planes per wgrad block

// slot s -> (tap group t = 16 jd + 4 jh + jw, phase r) ; fwd kernel tap per dim k = 2j + r - 1 (valid 0..6)
__host__ __device__ __forceinline__ int stem_tap(int s) {
  const int t = s >> 3, r = s & 7;
  const int kd = 2 * (t >> 4) + (r >> 2) - 1, kh = 2 * ((t >> 2) & 3) + ((r >> 1) & 1) - 1, kw = 2 * (t & 3) + (r & 1) - 1;
  if (kd < 0 || kh < 0 || kw < 0 || kd > 6 || kh > 6 || kw > 6) return -1;
  return (kd * 7 + kh) * 7 + kw;
}

// ------------------------------------------------------------------------------------------------ polyphase
__global__ void k_stem_polyphase(StemDims d, const uint8_t* __restrict__ src, const int* __restrict__ idx, int N,
                                 uint8_t* __restrict__ xp, uint8_t* __restrict__ xq) {
  const int64_t vox = (int64_t)d.PZ * d.PY * d.PX;
  const int64_t tot = (int64_t)N * vox;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t v = e;
    const int x = (int)(v % d.PX); v /= d.PX;
    const int y = (int)(v % d.PY); v /= d.PY;
    const int z = (int)(v % d.PZ);
    const int n = (int)(v / d.PZ);
    const uint8_t* s = src + (int64_t)idx[n] * d.D * d.H * d.W;
    uint32_t lo = 0, hi = 0;
    uint8_t b[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int zz = 2 * z - 4 + (r >> 2), h = 2 * y - 4 + ((r >> 1) & 1), w = 2 * x - 4 + (r & 1);
      b[r] = (zz >= 0 && zz < d.D && h >= 0 && h < d.H && w >= 0 && w < d.W) ? s[((int64_t)zz * d.H + h) * d.W + w] : 0;
      if (r < 4) lo |= (uint32_t)b[r] << (8 * r); else hi |= (uint32_t)b[r] << (8 * (r - 4));
    }
    *reinterpret_cast<uint2*>(xp + e * 8) = make_uint2(lo, hi);
    if (xq) {  // training only (the weight gradient's layout)
      const int64_t sv = (((int64_t)z * d.PY + y) * d.PX + x);
#pragma unroll
      for (int r = 0; r < 8; ++r) xq[((int64_t)n * 8 + r) * vox + sv] = b[r];
    }
  }
}

// weights: theta [64][343] fp32 (PyTorch conv1.weight) -> wk [G][64][512] bf16 in slot order (0 in empty slots)
__global__ void k_stem_pack(const float* __restrict__ theta, int64_t ldt, int64_t off, int G, uint16_t* __restrict__ wk) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= G * kSC * kSK) return;
  const int g = i / (kSC * kSK), rem = i - g * kSC * kSK, c = rem / kSK, s = rem - c * kSK;
  const int k = stem_tap(s);
  wk[i] = k >= 0 ? f32_to_bf16(theta[(int64_t)g * ldt + off + c * 343 + k]) : (uint16_t)0;
}

__device__ __forceinline__ uint4 u8x8_to_bf16(uint2 v) {
  uint4 o;
  o.x = pack_bf16x2((float)(v.x & 0xff), (float)((v.x >> 8) & 0xff));
  o.y = pack_bf16x2((float)((v.x >> 16) & 0xff), (float)(v.x >> 24));
  o.z = pack_bf16x2((float)(v.y & 0xff), (float)((v.y >> 8) & 0xff));
  o.w = pack_bf16x2((float)((v.y >> 16) & 0xff), (float)(v.y >> 24));
  return o;
}

// ------------------------------------------------------------------------------------------------ forward conv
// halo ring: [4 jd][kSRing y' slots][kSHX x'][8 phases] bf16
constexpr int kSHalo = 4 * kSRing * kSHX * 8;

__global__ __launch_bounds__(256, 2) void k_stem_fwd(StemDims d, const uint8_t* __restrict__ xp, const uint16_t* __restrict__ wk,
                                                     int B, uint16_t* __restrict__ y, float* __restrict__ stats) {
  __shared__ __attribute__((aligned(16))) uint16_t halo[kSHalo];
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int od = bid % d.OD, n = bid / d.OD, g = n / B;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int ch = wid & 1, ph = wid >> 1;
  const uint8_t* xs = xp + (int64_t)n * d.PZ * d.PY * d.PX * 8;
  // stage one y' row of the 4 jd planes into ring slot (yrow % kSRing): 4 x kSHX voxels of 8 phases
  auto stage = [&](int yrow) {
    for (int e = tid; e < 4 * kSHX; e += 256) {
      const int jd = e / kSHX, xx = e - jd * kSHX;
      uint2 v = make_uint2(0, 0);
      if (xx < d.PX && yrow < d.PY) v = *reinterpret_cast<const uint2*>(xs + (((int64_t)(od + jd) * d.PY + yrow) * d.PX + xx) * 8);
      *reinterpret_cast<uint4*>(&halo[((jd * kSRing + yrow % kSRing) * kSHX + xx) * 8]) = u8x8_to_bf16(v);
    }
  };
  bf16x8 fa[2][16];
  const uint16_t* wg = wk + (int64_t)g * kSC * kSK;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int s = 0; s < 16; ++s)
      fa[i][s] = *reinterpret_cast<const bf16x8*>(wg + (32 * ch + 16 * i + fr) * kSK + 32 * s + 8 * fq);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int s = 0; s < 16; ++s) asm volatile("" : "+v"(fa[i][s]));
  // per-(channel, position-lane) shifted sums for the block statistics; shift = the first row's value
  float sh[2][4], s1[2][4], s2[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) { sh[i][r] = 0.f; s1[i][r] = 0.f; s2[i][r] = 0.f; }
  for (int yy = 0; yy < 3; ++yy) stage(yy);
  const float inv255 = 1.0f / 255.0f;
  for (int oh = 0; oh < d.OH; ++oh) {
    stage(oh + 3);  // the row the last jh tap of this output row reads (slot not in use by row oh - 1 any more)
    __syncthreads();
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    int rbase[4];
#pragma unroll
    for (int jh = 0; jh < 4; ++jh) rbase[jh] = ((oh + jh) % kSRing) * kSHX * 8;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int t = 4 * s + fq;
      const int jd = t >> 4, jh = (t >> 2) & 3, jw = t & 3;
      const int base = jd * kSRing * kSHX * 8 + rbase[jh] + (32 * ph + fr + jw) * 8;
      const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(&halo[base]);
      const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(&halo[base + 16 * 8]);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        acc[i][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][s], b0, acc[i][0], 0, 0, 0);
        acc[i][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][s], b1, acc[i][1], 0, 0, 0);
      }
    }
    // epilogue: C[row = 4 fq + r][col = fr] -> channel 32 ch + 16 i + 4 fq + r, position 32 ph + 16 j + fr
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int ow = 32 * ph + 16 * j + fr;
      const bool valid = ow < d.OW;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = acc[i][j][r] * inv255;
          // the stored (bf16) value is what BN normalises in the reference (conv output in the activation dtype)
          v[r] = bf16_to_f32(f32_to_bf16(v[r]));
          if (oh == 0 && j == 0) sh[i][r] = v[r];
          if (valid) {
            const float dv = v[r] - sh[i][r];
            s1[i][r] += dv;
            s2[i][r] = fmaf(dv, dv, s2[i][r]);
          }
        }
        if (valid) {
          uint16_t* yp = y + ((((int64_t)n * d.OD + od) * d.OH + oh) * d.OW + ow) * kSC + 32 * ch + 16 * i + 4 * fq;
          *reinterpret_cast<uint2*>(yp) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
        }
      }
    }
    // no trailing barrier: the next row stages slot (oh + 4) % 5, which this row does not read, and a wave can
    // only run one row ahead of the slowest (the barrier above)
  }
  // block statistics: sum over the 16 position lanes, then the two position halves (waves ph = 0, 1).  The shift
  // differs per lane, so convert each lane's shifted sums to (count, mean, M2) and merge with Chan's formula.
  const float cnt_lane = (float)d.OH * (float)((32 * ph + fr < d.OW ? 1 : 0) + (32 * ph + 16 + fr < d.OW ? 1 : 0));
  __shared__ float part[4][kSC][3];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float n_ = cnt_lane, mu = n_ > 0 ? sh[i][r] + s1[i][r] / n_ : 0.f;
      float m2 = n_ > 0 ? fmaxf(s2[i][r] - s1[i][r] * s1[i][r] / n_, 0.f) : 0.f;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const float n2 = __shfl_xor(n_, o, 64), mu2 = __shfl_xor(mu, o, 64), q2 = __shfl_xor(m2, o, 64);
        const float nn = n_ + n2;
        if (nn > 0) {
          const float dm = mu2 - mu;
          m2 = m2 + q2 + dm * dm * n_ * n2 / nn;
          mu = mu + dm * n2 / nn;
          n_ = nn;
        }
      }
      if (fr == 0) {
        const int c = 32 * ch + 16 * i + 4 * fq + r;
        part[wid][c][0] = n_;
        part[wid][c][1] = mu;
        part[wid][c][2] = m2;
      }
    }
  __syncthreads();
  if (tid < kSC) {
    const int c = tid, chh = c >> 5;  // waves (ch = chh, ph = 0 / 1) = wid chh and chh + 2
    const float n1 = part[chh][c][0], m1 = part[chh][c][1], q1 = part[chh][c][2];
    const float n2 = part[chh + 2][c][0], m2_ = part[chh + 2][c][1], q2 = part[chh + 2][c][2];
    const float nn = n1 + n2, dm = m2_ - m1;
    const float mean = m1 + dm * n2 / nn, M2 = q1 + q2 + dm * dm * n1 * n2 / nn;
    const int b = (n % B) * d.OD + od;  // block index within the client (B samples x 61 planes, BP = 73 x 61)
    float* st = stats + (((int64_t)g * B * d.OD + b) * kSC + c) * 2;
    st[0] = mean;
    st[1] = M2;
  }
}

// ------------------------------------------------------------------------------------------------ BN + ReLU + pool
// thread per (n, pz, py, px, 8-channel chunk)
__global__ void k_stem_pool(StemDims d, const uint16_t* __restrict__ y, const float* __restrict__ scale,
                            const float* __restrict__ shift, int N, int B, uint16_t* __restrict__ out,
                            uint8_t* __restrict__ amax) {
  const int64_t tot = (int64_t)N * d.QD * d.QH * d.QW * (kSC / 8);
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t v = e;
    const int cg = (int)(v % (kSC / 8)); v /= (kSC / 8);
    const int px = (int)(v % d.QW); v /= d.QW;
    const int py = (int)(v % d.QH); v /= d.QH;
    const int pz = (int)(v % d.QD);
    const int n = (int)(v / d.QD), g = n / B;
    float sc[8], sf[8], best[8];
    int arg[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      sc[q] = scale[g * kSC + cg * 8 + q];
      sf[q] = shift[g * kSC + cg * 8 + q];
      best[q] = -INFINITY;
      arg[q] = 0;
    }
    // the window's 9 voxels of one depth plane are loaded before their max (clamped addresses + a validity mask): the
    // round-4 loop's per-voxel bounds `continue` made the 27 loads dependent round trips; all 27 at once held 108
    // VGPRs and ran slower (5.5 vs 2.2 ms per config-5 step)
    const uint16_t* yn = y + (int64_t)n * d.OD * d.OH * d.OW * kSC + cg * 8;
    for (int kd = 0; kd < 3; ++kd) {
      const int zd = 2 * pz - 1 + kd;
      if (zd < 0 || zd >= d.OD) continue;
      uint4 raw[9];
      uint32_t valid = 0;
#pragma unroll
      for (int a9 = 0; a9 < 9; ++a9) {
        const int zh = 2 * py - 1 + a9 / 3, zw = 2 * px - 1 + a9 % 3;
        const bool ok = zh >= 0 && zh < d.OH && zw >= 0 && zw < d.OW;
        valid |= (uint32_t)ok << a9;
        const int ch = min(max(zh, 0), d.OH - 1), cw = min(max(zw, 0), d.OW - 1);
        raw[a9] = *reinterpret_cast<const uint4*>(yn + (((int64_t)zd * d.OH + ch) * d.OW + cw) * kSC);
      }
#pragma unroll
      for (int a9 = 0; a9 < 9; ++a9) {
        if (!((valid >> a9) & 1u)) continue;
        const int a = kd * 9 + a9;
        const uint32_t u[4] = {raw[a9].x, raw[a9].y, raw[a9].z, raw[a9].w};
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const float yv = __uint_as_float((q & 1) ? (u[q >> 1] & 0xffff0000u) : (u[q >> 1] << 16));
          const float z = fmaxf(fmaf(yv, sc[q], sf[q]), 0.f);
          if (z > best[q]) { best[q] = z; arg[q] = a; }
        }
      }
    }
    const int64_t o = e * 8;
    *reinterpret_cast<uint4*>(out + o) = make_uint4(pack_bf16x2(best[0], best[1]), pack_bf16x2(best[2], best[3]),
                                                    pack_bf16x2(best[4], best[5]), pack_bf16x2(best[6], best[7]));
    *reinterpret_cast<uint2*>(amax + o) = make_uint2((uint32_t)arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24),
                                                     (uint32_t)arg[4] | (arg[5] << 8) | (arg[6] << 16) | (arg[7] << 24));
  }
}

// ------------------------------------------------------------------------------------------------ pool / BN backward
// block = (n, od); thread: fixed 8-channel chunk cg = tid & 7, positions (oh, ow) strided by 32.  dz (bf16) and
// per-block sums of dz and dz * xhat (xhat = (y - mean) * invstd) per channel -> part [G][B*61][64][2].
__global__ __launch_bounds__(256) void k_stem_unpool(StemDims d, const uint16_t* __restrict__ dpool, const uint8_t* __restrict__ amax,
                                                     const uint16_t* __restrict__ y, const float* __restrict__ scale,
                                                     const float* __restrict__ shift, const float* __restrict__ mean,
                                                     const float* __restrict__ invstd, int B,
                                                     uint16_t* __restrict__ dz, float* __restrict__ part) {
  __shared__ float red[32][kSC][2];
  const int od = blockIdx.x % d.OD, n = blockIdx.x / d.OD, g = n / B;
  const int tid = threadIdx.x, cg = tid & 7, pl = tid >> 3;
  float sc[8], sf[8], mu[8], is[8], a1[8], a2[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int c = g * kSC + cg * 8 + q;
    sc[q] = scale[c]; sf[q] = shift[c]; mu[q] = mean[c]; is[q] = invstd[c];
    a1[q] = 0.f; a2[q] = 0.f;
  }
  const int qd0 = od >> 1, qd1 = (od + 1) >> 1;
  for (int p = pl; p < d.OH * d.OW; p += 32) {
    const int oh = p / d.OW, ow = p - oh * d.OW;
    float dv[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) dv[q] = 0.f;
    // the (<= 8) pooling windows containing this voxel: windows qd in {od >> 1, (od + 1) >> 1} (one when od is even),
    // likewise qh, qw; their argmax bytes and gradients are loaded before any is used (clamped addresses, validity
    // bits) instead of one dependent round trip per window, and summed in the round-4 loop's (qd, qh, qw) order
    const int qh0 = oh >> 1, qh1 = (oh + 1) >> 1, qw0 = ow >> 1, qw1 = (ow + 1) >> 1;
    const int64_t yo = ((((int64_t)n * d.OD + od) * d.OH + oh) * d.OW + ow) * kSC + cg * 8;
    const uint4 raw = *reinterpret_cast<const uint4*>(y + yo);
    uint2 am[8];
    uint4 gr[8];
    uint32_t wvalid = 0;
#pragma unroll
    for (int w8 = 0; w8 < 8; ++w8) {
      const int qd = (w8 & 4) ? qd1 : qd0, qh = (w8 & 2) ? qh1 : qh0, qw = (w8 & 1) ? qw1 : qw0;
      const bool ok = ((w8 & 4) == 0 || qd1 != qd0) && ((w8 & 2) == 0 || qh1 != qh0) && ((w8 & 1) == 0 || qw1 != qw0) &&
                      qd < d.QD && qh < d.QH && qw < d.QW;
      wvalid |= (uint32_t)ok << w8;
      const int64_t qo = ((((int64_t)n * d.QD + min(qd, d.QD - 1)) * d.QH + min(qh, d.QH - 1)) * d.QW +
                          min(qw, d.QW - 1)) * kSC + cg * 8;
      am[w8] = *reinterpret_cast<const uint2*>(amax + qo);
      gr[w8] = *reinterpret_cast<const uint4*>(dpool + qo);  // bf16 (the engine's residual stream)
    }
#pragma unroll
    for (int w8 = 0; w8 < 8; ++w8) {
      if (!((wvalid >> w8) & 1u)) continue;
      const int qd = (w8 & 4) ? qd1 : qd0, qh = (w8 & 2) ? qh1 : qh0, qw = (w8 & 1) ? qw1 : qw0;
      const int a = (od - (2 * qd - 1)) * 9 + (oh - (2 * qh - 1)) * 3 + (ow - (2 * qw - 1));
      const uint32_t gu[4] = {gr[w8].x, gr[w8].y, gr[w8].z, gr[w8].w};
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float gv = __uint_as_float((q & 1) ? (gu[q >> 1] & 0xffff0000u) : (gu[q >> 1] << 16));
        const int aq = (int)(((q < 4 ? am[w8].x : am[w8].y) >> (8 * (q & 3))) & 0xffu);
        if (aq == a) dv[q] += gv;
      }
    }
    const uint32_t u[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float yv = __uint_as_float((q & 1) ? (u[q >> 1] & 0xffff0000u) : (u[q >> 1] << 16));
      if (fmaf(yv, sc[q], sf[q]) <= 0.f) dv[q] = 0.f;  // ReLU mask
      a1[q] += dv[q];
      a2[q] = fmaf(dv[q], (yv - mu[q]) * is[q], a2[q]);
    }
    *reinterpret_cast<uint4*>(dz + yo) = make_uint4(pack_bf16x2(dv[0], dv[1]), pack_bf16x2(dv[2], dv[3]),
                                                    pack_bf16x2(dv[4], dv[5]), pack_bf16x2(dv[6], dv[7]));
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    red[pl][cg * 8 + q][0] = a1[q];
    red[pl][cg * 8 + q][1] = a2[q];
  }
  __syncthreads();
  if (tid < kSC * 2) {
    const int c = tid >> 1, k = tid & 1;
    float s = 0.f;
    for (int r = 0; r < 32; ++r) s += red[r][c][k];
    part[(((int64_t)g * B * d.OD + (n % B) * d.OD + od) * kSC + c) * 2 + k] = s;
  }
}

// per (g, c): dbeta = sum dz, dgamma = sum dz xhat; coefficients of dy = a dz + b y + d (BN train backward)
__global__ void k_stem_bn_bwd_fin(StemDims d, const float* __restrict__ part, int B, int G, const float* __restrict__ mean,
                                  const float* __restrict__ invstd, const float* __restrict__ theta, int64_t ldt,
                                  int64_t off_g, float* __restrict__ grad, int64_t ldg, int64_t goff_g, int64_t goff_b,
                                  float* __restrict__ coef) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= G * kSC) return;
  const int g = i / kSC, c = i - g * kSC;
  double s1 = 0, s2 = 0;
  const int nb = B * d.OD;
  for (int b = 0; b < nb; ++b) {
    const float* p = part + (((int64_t)g * nb + b) * kSC + c) * 2;
    s1 += p[0];
    s2 += p[1];
  }
  const double M = (double)B * d.OD * d.OH * d.OW;
  const double gm = theta[(int64_t)g * ldt + off_g + c], is = invstd[i], mu = mean[i];
  grad[(int64_t)g * ldg + goff_g + c] = (float)s2;
  grad[(int64_t)g * ldg + goff_b + c] = (float)s1;
  // dy = gm is (dz - s1/M - xhat s2/M), xhat = (y - mu) is
  const double ca = gm * is, cb = -gm * is * is * s2 / M, cd = -gm * is * s1 / M + gm * is * is * mu * s2 / M;
  coef[i * 3 + 0] = (float)ca;
  coef[i * 3 + 1] = (float)cb;
  coef[i * 3 + 2] = (float)cd;
}

// ------------------------------------------------------------------------------------------------ weight gradient
// block = (n, od chunk, jd); 4 waves: channel half (w & 1) x slot half (w >> 1) of the block's 128 slots
// (jh 4 x jw 4 x phase 8; slot-in-block = (jh * 4 + jw) * 8 + r).  Per output row: dy tile [64 pos][64 c] bf16 in LDS
// (A = dy^T by transposed reads), B = x-shifted phase-major input rows in a ring of kSRing y' rows:
// bq[slot y'][r][jw][64 pos] bf16.
constexpr int kWgB = kSRing * 8 * 4 * 64;  // B ring elements
__global__ __launch_bounds__(256, 2) void k_stem_wgrad(StemDims d, const uint8_t* __restrict__ xq, const uint16_t* __restrict__ dz,
                                                       const uint16_t* __restrict__ y, const float* __restrict__ coef,
                                                       int B, float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) uint16_t bq[kWgB];
  __shared__ __attribute__((aligned(16))) uint16_t dyt[64 * 64];
  __shared__ uint8_t rawrow[8][72];
  const int nchunk = (d.OD + kWgOD - 1) / kWgOD;
  const int bid = blockIdx.x;
  const int jd = bid & 3, oc = (bid >> 2) % nchunk, n = (bid >> 2) / nchunk, g = n / B;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int chh = wid & 1, shh = wid >> 1;
  const int64_t vox = (int64_t)d.PZ * d.PY * d.PX;
  // dy coefficients of this thread's channel chunk (dy tile build: thread -> (position, chunk) items)
  const int cg = tid & 7;
  float ca[8], cb[8], cd[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int c = g * kSC + cg * 8 + q;
    ca[q] = coef[c * 3]; cb[q] = coef[c * 3 + 1]; cd[q] = coef[c * 3 + 2];
  }
  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // stage y' row yrow of plane z' into ring slot yrow % kSRing: raw phase-major bytes -> 4 x-shifted bf16 copies
  auto stage = [&](int zp, int yrow) {
    __syncthreads();  // rawrow reuse
    for (int e = tid; e < 8 * 72; e += 256) {
      const int r = e / 72, xx = e - r * 72;
      uint8_t v = 0;
      if (xx < d.PX && yrow < d.PY) v = xq[((int64_t)n * 8 + r) * vox + ((int64_t)zp * d.PY + yrow) * d.PX + xx];
      rawrow[r][xx] = v;
    }
    __syncthreads();
    {  // thread -> (r, jw, 8-position group): 8 x 4 x 8 = 256 items
      const int r = tid >> 5, jw = (tid >> 3) & 3, p0 = (tid & 7) * 8;
      float f[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = (float)rawrow[r][p0 + jw + k];
      *reinterpret_cast<uint4*>(&bq[(((yrow % kSRing) * 8 + r) * 4 + jw) * 64 + p0]) =
          make_uint4(pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3]), pack_bf16x2(f[4], f[5]), pack_bf16x2(f[6], f[7]));
    }
  };
  const int od0 = oc * kWgOD, od1 = min(d.OD, od0 + kWgOD);
  for (int od = od0; od < od1; ++od) {
    const int zp = od + jd;
    for (int yy = 0; yy < 3; ++yy) stage(zp, yy);
    for (int oh = 0; oh < d.OH; ++oh) {
      stage(zp, oh + 3);
      // dy tile: [pos][c], positions >= 61 zero
      for (int e = tid; e < 64 * 8; e += 256) {
        const int p = e >> 3;  // e & 7 == cg (256 % 8 == 0)
        uint4 o = make_uint4(0, 0, 0, 0);
        if (p < d.OW) {
          const int64_t yo = ((((int64_t)n * d.OD + od) * d.OH + oh) * d.OW + p) * kSC + cg * 8;
          const uint4 zr = *reinterpret_cast<const uint4*>(dz + yo), yr = *reinterpret_cast<const uint4*>(y + yo);
          const uint32_t zu[4] = {zr.x, zr.y, zr.z, zr.w}, yu[4] = {yr.x, yr.y, yr.z, yr.w};
          float v[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const float zv = __uint_as_float((q & 1) ? (zu[q >> 1] & 0xffff0000u) : (zu[q >> 1] << 16));
            const float yv = __uint_as_float((q & 1) ? (yu[q >> 1] & 0xffff0000u) : (yu[q >> 1] << 16));
            v[q] = fmaf(ca[q], zv, fmaf(cb[q], yv, cd[q]));
          }
          o = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
        }
        *reinterpret_cast<uint4*>(&dyt[p * 64 + cg * 8]) = o;
      }
      __syncthreads();
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        // A fragments (rows = channels c0 + fr, k = positions 32 ks + 8 fq + e): two transposed 4-row reads
        bf16x8 fa[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int c0 = 32 * chh + 16 * i;
          const int q = fr >> 2, pp = fr & 3;
          s16x4 lo, hi;
          const uint16_t* a0 = &dyt[(32 * ks + 8 * fq + q) * 64 + c0 + 4 * pp];
          const uint16_t* a1 = &dyt[(32 * ks + 8 * fq + 4 + q) * 64 + c0 + 4 * pp];
          lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a0);
          hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a1);
          typedef short s16x8 __attribute__((ext_vector_type(8)));
          const s16x8 f = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          fa[i] = __builtin_bit_cast(bf16x8, f);
        }
        // B fragments: column = slot (jh, jw, r) of this wave's half, k = positions
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int sl = 64 * shh + 16 * j + fr;  // slot in block
          const int jh = sl >> 5, jw = (sl >> 3) & 3, r = sl & 7;
          const bf16x8 fb = *reinterpret_cast<const bf16x8*>(
              &bq[((((oh + jh) % kSRing) * 8 + r) * 4 + jw) * 64 + 32 * ks + 8 * fq]);
#pragma unroll
          for (int i = 0; i < 2; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb, acc[i][j], 0, 0, 0);
        }
      }
    }
  }
  // slab [block][64 c][128 slots]: C[row = 4 fq + r][col = fr] -> channel 32 chh + 16 i + 4 fq + r, slot 64 shh + 16 j + fr
  float* sp = slab + (int64_t)bid * kSC * 128;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) sp[(32 * chh + 16 * i + 4 * fq + r) * 128 + 64 * shh + 16 * j + fr] = acc[i][j][r];
}

// [WG4] k_stem_wgrad with the four depth tap groups jd in ONE block.  k_stem_wgrad is a block per (sample, od chunk,
// jd): every one of the four builds the same dy tile from dz and y, so the two 64-channel bf16 tensors (4.45 GB each
// at config 5) were read four times — 35.6 GB, the kernel ran at ~4.3 TB/s and 8.3 ms per step
// (profiles/r5_config5_steady.txt).  Here 8 waves = jd (w >> 1) x slot half (w & 1), 64 channels x 64 slots each, share
// one dy tile per output row; the input rows of the four planes z' = od + jd live in per-jd rings of 4 y' rows
// (row oh reads y' = oh .. oh + 3 and writes oh + 3 into the slot row oh - 1 read last).  Software-pipelined: the dz / y
// chunk and the raw input bytes of row oh + 1 are loaded into registers while the MFMAs of row oh run; one barrier
// after the LDS writes, one after the MFMAs.  Same slab layout as k_stem_wgrad (k_stem_wgrad_fin unchanged).
constexpr int kW4Ring = 4;
__global__ __launch_bounds__(512, 2) void k_stem_wgrad4(StemDims d, const uint8_t* __restrict__ xq,
                                                        const uint16_t* __restrict__ dz, const uint16_t* __restrict__ y,
                                                        const float* __restrict__ coef, int B, float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) uint16_t bq[4 * kW4Ring * 8 * 4 * 64];  // [jd][ring][r][jw][64 pos]
  __shared__ __attribute__((aligned(16))) uint16_t dyt[64 * 64];                  // [pos][c]
  const int nchunk = (d.OD + kWgOD - 1) / kWgOD;
  const int bid = blockIdx.x;
  const int oc = bid % nchunk, n = bid / nchunk, g = n / B;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int jdw = wid >> 1, shh = wid & 1;
  const int64_t vox = (int64_t)d.PZ * d.PY * d.PX;
  // dy item: position pt, channel chunk cg
  const int cg = tid & 7, pt = tid >> 3;
  float ca[8], cb[8], cd[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int c = g * kSC + cg * 8 + q;
    ca[q] = coef[c * 3]; cb[q] = coef[c * 3 + 1]; cd[q] = coef[c * 3 + 2];
  }
  // staging items it = tid + 512 h: (jd, r, jw, 8-position group)
  int s_jd[2], s_r[2], s_jw[2], s_p0[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int it = tid + 512 * h;
    s_jd[h] = it >> 8; s_r[h] = (it >> 5) & 7; s_jw[h] = (it >> 3) & 3; s_p0[h] = (it & 7) * 8;
  }
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint2 rlo[2], rhi[2];  // raw input bytes p0 .. p0 + 15 of the staged row, per item
  uint4 zr, yr;          // dz / y chunk of the dy item
  auto ld_raw = [&](int od, int yrow) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      rlo[h] = rhi[h] = make_uint2(0, 0);
      if (yrow < d.PY) {
        const uint8_t* row = xq + ((int64_t)n * 8 + s_r[h]) * vox + ((int64_t)(od + s_jd[h]) * d.PY + yrow) * d.PX;
        rlo[h] = *reinterpret_cast<const uint2*>(row + s_p0[h]);
        if (s_p0[h] + 8 < d.PX) rhi[h] = *reinterpret_cast<const uint2*>(row + s_p0[h] + 8);
      }
    }
  };
  auto st_raw = [&](int yrow) {  // the 4 x-shifted bf16 copies of the loaded row into ring slot yrow % kW4Ring
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint64_t lo = ((uint64_t)rlo[h].y << 32) | rlo[h].x, hi = ((uint64_t)rhi[h].y << 32) | rhi[h].x;
      const int sh = 8 * s_jw[h];
      const uint64_t v = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
      *reinterpret_cast<uint4*>(&bq[((((s_jd[h] * kW4Ring + yrow % kW4Ring) * 8 + s_r[h]) * 4 + s_jw[h]) * 64) +
                                    s_p0[h]]) = u8x8_to_bf16(make_uint2((uint32_t)v, (uint32_t)(v >> 32)));
    }
  };
  auto ld_dy = [&](int od, int oh) {
    zr = yr = make_uint4(0, 0, 0, 0);
    if (pt < d.OW) {
      const int64_t yo = ((((int64_t)n * d.OD + od) * d.OH + oh) * d.OW + pt) * kSC + cg * 8;
      zr = *reinterpret_cast<const uint4*>(dz + yo);
      yr = *reinterpret_cast<const uint4*>(y + yo);
    }
  };
  auto st_dy = [&]() {
    uint4 o = make_uint4(0, 0, 0, 0);
    if (pt < d.OW) {
      const uint32_t zu[4] = {zr.x, zr.y, zr.z, zr.w}, yu[4] = {yr.x, yr.y, yr.z, yr.w};
      float v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float zv = __uint_as_float((q & 1) ? (zu[q >> 1] & 0xffff0000u) : (zu[q >> 1] << 16));
        const float yv = __uint_as_float((q & 1) ? (yu[q >> 1] & 0xffff0000u) : (yu[q >> 1] << 16));
        v[q] = fmaf(ca[q], zv, fmaf(cb[q], yv, cd[q]));
      }
      o = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
    }
    *reinterpret_cast<uint4*>(&dyt[pt * 64 + cg * 8]) = o;
  };

  const int od0 = oc * kWgOD, od1 = min(d.OD, od0 + kWgOD);
  const uint16_t* bqw = bq + jdw * kW4Ring * 8 * 4 * 64;
  for (int od = od0; od < od1; ++od) {
    for (int yy = 0; yy < 3; ++yy) {  // ring rows 0..2 (the previous plane's last MFMAs are behind a barrier)
      ld_raw(od, yy);
      st_raw(yy);
    }
    ld_dy(od, 0);
    ld_raw(od, 3);
    for (int oh = 0; oh < d.OH; ++oh) {
      st_dy();
      st_raw(oh + 3);
      __syncthreads();
      if (oh + 1 < d.OH) {  // next row's operands in flight under this row's MFMAs
        ld_dy(od, oh + 1);
        ld_raw(od, oh + 4);
      }
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 fa[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int q = fr >> 2, pp = fr & 3;
          const uint16_t* a0 = &dyt[(32 * ks + 8 * fq + q) * 64 + 16 * i + 4 * pp];
          const uint16_t* a1 = &dyt[(32 * ks + 8 * fq + 4 + q) * 64 + 16 * i + 4 * pp];
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a0);
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)a1);
          typedef short s16x8 __attribute__((ext_vector_type(8)));
          const s16x8 f = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          fa[i] = __builtin_bit_cast(bf16x8, f);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int sl = 64 * shh + 16 * j + fr;
          const int jh = sl >> 5, jw = (sl >> 3) & 3, r = sl & 7;
          const bf16x8 fb = *reinterpret_cast<const bf16x8*>(
              &bqw[((((oh + jh) % kW4Ring) * 8 + r) * 4 + jw) * 64 + 32 * ks + 8 * fq]);
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb, acc[i][j], 0, 0, 0);
        }
      }
      __syncthreads();
    }
  }
  float* sp = slab + ((int64_t)bid * 4 + jdw) * kSC * 128;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) sp[(16 * i + 4 * fq + r) * 128 + 64 * shh + 16 * j + fr] = acc[i][j][r];
}

// per (g, c, tap k): sum of the client's slabs at the tap's slot, / 255 (the input scale), PyTorch layout [64][343]
__global__ void k_stem_wgrad_fin(StemDims d, const float* __restrict__ slab, int B, int G, float* __restrict__ grad, int64_t ldg,
                                 int64_t goff) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= G * kSC * kSK) return;
  const int g = i / (kSC * kSK), rem = i - g * kSC * kSK, c = rem / kSK, s = rem - c * kSK;
  const int k = stem_tap(s);
  if (k < 0) return;
  const int t = s >> 3, r = s & 7, jd = t >> 4, sl = ((t & 15) * 8) + r;  // slot in the jd block: (jh*4+jw)*8 + r
  const int nchunk = (d.OD + kWgOD - 1) / kWgOD;
  double acc = 0;
  for (int n = g * B; n < (g + 1) * B; ++n)
    for (int oc = 0; oc < nchunk; ++oc)
      acc += slab[((int64_t)((n * nchunk + oc) * 4 + jd) * kSC + c) * 128 + sl];
  grad[(int64_t)g * ldg + goff + c * 343 + k] = (float)(acc / 255.0);
}

// ------------------------------------------------------------------------------------------------ host API
void stem_polyphase(uintptr_t src, uintptr_t idx, int N, int D, int H, int W, uintptr_t xp, uintptr_t xq,
                    uintptr_t stream) {
  const StemDims d = stem_dims(D, H, W);
  const int64_t tot = (int64_t)N * d.PZ * d.PY * d.PX;
  hipLaunchKernelGGL(k_stem_polyphase, dim3((unsigned)std::min<int64_t>(65536, (tot + 255) / 256)), dim3(256), 0,
                     as_stream(stream), d, ptr<const uint8_t>(src), ptr<const int>(idx), N, ptr<uint8_t>(xp),
                     ptr<uint8_t>(xq));
  NIDT_CHECK(hipGetLastError());
}

void stem_fwd(uintptr_t xp, uintptr_t theta, int64_t ldt, int64_t off_w, int N, int B, int D, int H, int W, uintptr_t wk,
              uintptr_t y, uintptr_t stats, uintptr_t stream) {
  const StemDims d = stem_dims(D, H, W);
  NIDT_REQUIRE(d.OW <= 64 && d.OW >= 2 && d.OH >= 2 && d.OD >= 2, "stem_fwd: output rows must fit one 64-wide block");
  NIDT_REQUIRE(N % B == 0, "stem_fwd: N % B");
  hipStream_t s = as_stream(stream);
  const int G = N / B;
  hipLaunchKernelGGL(k_stem_pack, dim3(ceil_div(G * kSC * kSK, 256)), dim3(256), 0, s, ptr<const float>(theta), ldt,
                     off_w, G, ptr<uint16_t>(wk));
  NIDT_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_stem_fwd, dim3(N * d.OD), dim3(256), 0, s, d, ptr<const uint8_t>(xp), ptr<const uint16_t>(wk), B,
                     ptr<uint16_t>(y), ptr<float>(stats));
  NIDT_CHECK(hipGetLastError());
}

void stem_pool(uintptr_t y, uintptr_t scale, uintptr_t shift, int N, int B, int D, int H, int W, uintptr_t out,
               uintptr_t amax, uintptr_t stream) {
  const StemDims d = stem_dims(D, H, W);
  const int64_t tot = (int64_t)N * d.QD * d.QH * d.QW * (kSC / 8);
  hipLaunchKernelGGL(k_stem_pool, dim3((unsigned)std::min<int64_t>(65536, (tot + 255) / 256)), dim3(256), 0,
                     as_stream(stream), d, ptr<const uint16_t>(y), ptr<const float>(scale), ptr<const float>(shift), N, B,
                     ptr<uint16_t>(out), ptr<uint8_t>(amax));
  NIDT_CHECK(hipGetLastError());
}

void stem_bwd(uintptr_t dpool, uintptr_t amax, uintptr_t y, uintptr_t xq, uintptr_t scale, uintptr_t shift,
              uintptr_t mean, uintptr_t invstd, int N, int B, int D, int H, int W, uintptr_t theta, int64_t ldt, int64_t off_g,
              uintptr_t grad, int64_t ldg, int64_t goff_w, int64_t goff_g, int64_t goff_b, uintptr_t dz,
              uintptr_t part, uintptr_t coef, uintptr_t slab, uintptr_t stream) {
  NIDT_REQUIRE(N % B == 0, "stem_bwd: N % B");
  const StemDims d = stem_dims(D, H, W);
  NIDT_REQUIRE(d.OW <= 64, "stem_bwd: output rows must fit one 64-wide block");
  hipStream_t s = as_stream(stream);
  const int G = N / B;
  hipLaunchKernelGGL(k_stem_unpool, dim3(N * d.OD), dim3(256), 0, s, d, ptr<const uint16_t>(dpool),
                     ptr<const uint8_t>(amax), ptr<const uint16_t>(y), ptr<const float>(scale),
                     ptr<const float>(shift), ptr<const float>(mean), ptr<const float>(invstd), B, ptr<uint16_t>(dz),
                     ptr<float>(part));
  NIDT_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_stem_bn_bwd_fin, dim3(ceil_div(G * kSC, 64)), dim3(64), 0, s, d, ptr<const float>(part), B, G,
                     ptr<const float>(mean), ptr<const float>(invstd), ptr<const float>(theta), ldt, off_g,
                     ptr<float>(grad), ldg, goff_g, goff_b, ptr<float>(coef));
  NIDT_CHECK(hipGetLastError());
  const int nchunk = (d.OD + kWgOD - 1) / kWgOD;
  // [WG4] one block per (sample, od chunk) for all four jd (NIDT_STEM_WG4=0: k_stem_wgrad, A/B); its raw-row loads
  // are 8-byte words, so the polyphase rows must be a multiple of 8 bytes (64 at the ABCD shape)
  static const bool wg4 = [] {
    const char* e = getenv("NIDT_STEM_WG4");
    return !(e && e[0] == '0');
  }();
  if (wg4 && d.PX % 8 == 0)
    hipLaunchKernelGGL(k_stem_wgrad4, dim3(N * nchunk), dim3(512), 0, s, d, ptr<const uint8_t>(xq),
                       ptr<const uint16_t>(dz), ptr<const uint16_t>(y), ptr<const float>(coef), B, ptr<float>(slab));
  else
    hipLaunchKernelGGL(k_stem_wgrad, dim3(N * nchunk * 4), dim3(256), 0, s, d, ptr<const uint8_t>(xq),
                       ptr<const uint16_t>(dz), ptr<const uint16_t>(y), ptr<const float>(coef), B, ptr<float>(slab));
  NIDT_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_stem_wgrad_fin, dim3(ceil_div(G * kSC * kSK, 256)), dim3(256), 0, s, d, ptr<const float>(slab), B,
                     G, ptr<float>(grad), ldg, goff_w);
  NIDT_CHECK(hipGetLastError());
}

// scratch sizes (elements) for the Python side
std::vector<int64_t> stem_sizes(int N, int D, int H, int W) {
  const StemDims d = stem_dims(D, H, W);
  const int nchunk = (d.OD + kWgOD - 1) / kWgOD;
  return {(int64_t)N * d.PZ * d.PY * d.PX * 8,             // xp / xq bytes
          (int64_t)N * d.OD * d.OH * d.OW * kSC,           // y / dz bf16
          (int64_t)N * d.QD * d.QH * d.QW * kSC,           // pooled / amax
          (int64_t)N * d.OD * kSC * 2,                     // stats / part fp32
          (int64_t)N * nchunk * 4 * kSC * 128,             // wgrad slab fp32
          (int64_t)kSC * kSK};                             // packed weights per client (bf16)
}

}  // namespace nidt
