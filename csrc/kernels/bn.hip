// BatchNorm3d (+ReLU, +MaxPool3d(3,3)) forward/backward for client-grouped channels-last activations.
//
// Reference semantics: torch.nn.BatchNorm3d in training mode (biased variance for normalisation,
// unbiased for running_var, momentum 0.1, eps 1e-5, num_batches_tracked += 1), followed by ReLU and
// (for conv1/conv2/conv5) MaxPool3d(kernel 3, stride 3, floor mode) — salient_models.py:146-168.
// Every (client g, channel c) pair has its own statistics (per-client BatchNorm).
//
//  k_bn_finalize   merge per-block (mean, M2) partials from the conv epilogue (Chan's parallel formula),
//                  update running stats in the flat per-client buffer rows, emit scale/shift (z = y*s+t).
//  k_bn_eval       scale/shift from running stats (model.eval()).
//  k_bn_relu_pool  z = y*s + t, max over the 27-voxel window (first max in d,h,w scan order, like
//                  PyTorch), relu -> pooled bf16 output + uint8 argmax (backward needs no dense mask).
//  k_bn_bwd_reduce sum(dz), sum(dz * xhat) per (g,c) as slabs; dz is reconstructed on the fly from the
//                  pooled gradient + argmax (POOL) or from the next layer's dgrad and the ReLU mask.
//  k_bn_bwd_fin    dgamma/dbeta into the flat gradient rows, conv-bias grad (exactly 0 before BN),
//                  and the affine coefficients of dy = A*dz + Bc + Cc*y.
//  k_bn_bwd_dx     dense bf16 dy (grad wrt the conv output), consumed by dgrad and wgrad.
#include "common.h"

namespace nidt {

struct BNPtrs {
  const float* theta; int64_t ldt; int64_t off_g, off_b;      // gamma/beta rows
  float* bufs; int64_t ldb; int64_t off_rm, off_rv, off_nbt;  // running stats rows
};

__global__ void k_bn_finalize(const float* __restrict__ stats, int nPB, int BP, int Mg, int G, int C, BNPtrs p,
                              float momentum, float eps, float* scale, float* shift, float* mean_o, float* invstd_o,
                              int update_running) {
  const int lane = threadIdx.x & 63;
  const int pair = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (pair >= G * C) return;
  const int g = pair / C, c = pair - g * C;
  double n = 0, mean = 0, m2 = 0;
  for (int b = lane; b < nPB; b += 64) {
    const float* s = stats + (((int64_t)g * nPB + b) * C + c) * 2;
    const double nb = (double)min(BP, Mg - b * BP);
    const double mb = s[0], qb = s[1];
    const double nn = n + nb, d = mb - mean;
    mean += d * nb / nn;
    m2 += qb + d * d * n * nb / nn;
    n = nn;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double n2 = __shfl_xor(n, o, 64), mean2 = __shfl_xor(mean, o, 64), m22 = __shfl_xor(m2, o, 64);
    const double nn = n + n2;
    if (nn > 0) {
      const double d = mean2 - mean;
      m2 = m2 + m22 + d * d * n * n2 / nn;
      mean = mean + d * n2 / nn;
      n = nn;
    }
  }
  if (lane == 0) {
    const double var = m2 / n;
    const float inv = (float)(1.0 / sqrt(var + (double)eps));
    const float gm = p.theta[(int64_t)g * p.ldt + p.off_g + c], bt = p.theta[(int64_t)g * p.ldt + p.off_b + c];
    const float sc = gm * inv;
    scale[pair] = sc;
    shift[pair] = bt - (float)mean * sc;
    mean_o[pair] = (float)mean;
    invstd_o[pair] = inv;
    if (update_running) {
      float* rm = p.bufs + (int64_t)g * p.ldb + p.off_rm + c;
      float* rv = p.bufs + (int64_t)g * p.ldb + p.off_rv + c;
      *rm = (1.f - momentum) * *rm + momentum * (float)mean;
      *rv = (1.f - momentum) * *rv + momentum * (float)(var * n / (n - 1.0));
      if (c == 0) p.bufs[(int64_t)g * p.ldb + p.off_nbt] += 1.f;
    }
  }
}

void bn_finalize(uintptr_t stats, int nPB, int BP, int Mg, int G, int C, uintptr_t theta, int64_t ldt, int64_t off_g,
                 int64_t off_b, uintptr_t bufs, int64_t ldb, int64_t off_rm, int64_t off_rv, int64_t off_nbt,
                 float momentum, float eps, uintptr_t scale, uintptr_t shift, uintptr_t mean, uintptr_t invstd,
                 int update_running, uintptr_t stream) {
  BNPtrs p{ptr<const float>(theta), ldt, off_g, off_b, ptr<float>(bufs), ldb, off_rm, off_rv, off_nbt};
  const int pairs = G * C;
  hipLaunchKernelGGL(k_bn_finalize, dim3(ceil_div(pairs, 4)), dim3(256), 0, as_stream(stream), ptr<const float>(stats),
                     nPB, BP, Mg, G, C, p, momentum, eps, ptr<float>(scale), ptr<float>(shift), ptr<float>(mean),
                     ptr<float>(invstd), update_running);
  NIDT_CHECK(hipGetLastError());
}

// eval-mode coefficients; mean_o / invstd_o (optional) receive the running mean and 1/sqrt(running_var + eps) for an
// eval-mode backward (DisPFL screen_gradients runs the model in eval(): DisPFL/my_model_trainer.py:166-189)
__global__ void k_bn_eval(int G, int C, BNPtrs p, float eps, float* scale, float* shift, float* mean_o,
                          float* invstd_o) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= G * C) return;
  const int g = i / C, c = i - g * C;
  const float rm = p.bufs[(int64_t)g * p.ldb + p.off_rm + c], rv = p.bufs[(int64_t)g * p.ldb + p.off_rv + c];
  const float gm = p.theta[(int64_t)g * p.ldt + p.off_g + c], bt = p.theta[(int64_t)g * p.ldt + p.off_b + c];
  const float inv = 1.f / sqrtf(rv + eps);
  const float sc = gm / sqrtf(rv + eps);
  scale[i] = sc;
  shift[i] = bt - rm * sc;
  if (mean_o) mean_o[i] = rm;
  if (invstd_o) invstd_o[i] = inv;
}

void bn_eval(int G, int C, uintptr_t theta, int64_t ldt, int64_t off_g, int64_t off_b, uintptr_t bufs, int64_t ldb,
             int64_t off_rm, int64_t off_rv, float eps, uintptr_t scale, uintptr_t shift, uintptr_t mean,
             uintptr_t invstd, uintptr_t stream) {
  BNPtrs p{ptr<const float>(theta), ldt, off_g, off_b, ptr<float>(bufs), ldb, off_rm, off_rv, 0};
  hipLaunchKernelGGL(k_bn_eval, dim3(ceil_div(G * C, 256)), dim3(256), 0, as_stream(stream), G, C, p, eps,
                     ptr<float>(scale), ptr<float>(shift), ptr<float>(mean), ptr<float>(invstd));
  NIDT_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// pooled forward: thread = (pooled voxel, 8-channel group)
__global__ __launch_bounds__(256) void k_bn_relu_pool(const uint16_t* __restrict__ y, const float* __restrict__ scale,
                                                      const float* __restrict__ shift, uint16_t* __restrict__ out,
                                                      uint8_t* __restrict__ amax, int NB, int B, int D, int H, int W,
                                                      int C) {
  const int Dp = D / 3, Hp = H / 3, Wp = W / 3, C8 = C / 8;
  const int64_t tot = (int64_t)NB * Dp * Hp * Wp * C8;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    const int cg = (int)(e % C8);
    int64_t v = e / C8;
    const int pw = (int)(v % Wp); v /= Wp;
    const int ph = (int)(v % Hp); v /= Hp;
    const int pd = (int)(v % Dp);
    const int n = (int)(v / Dp);
    const int g = n / B;
    float s[8], t[8], best[8];
    int bi[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s[j] = scale[g * C + cg * 8 + j];
      t[j] = shift[g * C + cg * 8 + j];
      best[j] = -INFINITY;
      bi[j] = 0;
    }
    for (int dd = 0; dd < 3; ++dd)
      for (int dh = 0; dh < 3; ++dh)
#pragma unroll
        for (int dw = 0; dw < 3; ++dw) {
          const int64_t idx = ((((int64_t)n * D + 3 * pd + dd) * H + 3 * ph + dh) * W + 3 * pw + dw) * C + cg * 8;
          const uint4 u = *reinterpret_cast<const uint4*>(y + idx);
          const uint32_t w4[4] = {u.x, u.y, u.z, u.w};
          const int li = dd * 9 + dh * 3 + dw;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const uint32_t bits = (j & 1) ? (w4[j >> 1] & 0xffff0000u) : (w4[j >> 1] << 16);
            const float z = fmaf(__uint_as_float(bits), s[j], t[j]);
            if (z > best[j]) { best[j] = z; bi[j] = li; }
          }
        }
    const int64_t o = e * 8;
    uint32_t pk[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) pk[j] = pack_bf16x2(fmaxf(best[2 * j], 0.f), fmaxf(best[2 * j + 1], 0.f));
    *reinterpret_cast<uint4*>(out + o) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
    uint2 ab;
    ab.x = (uint32_t)bi[0] | ((uint32_t)bi[1] << 8) | ((uint32_t)bi[2] << 16) | ((uint32_t)bi[3] << 24);
    ab.y = (uint32_t)bi[4] | ((uint32_t)bi[5] << 8) | ((uint32_t)bi[6] << 16) | ((uint32_t)bi[7] << 24);
    *reinterpret_cast<uint2*>(amax + o) = ab;
  }
}

void bn_relu_pool(uintptr_t y, uintptr_t scale, uintptr_t shift, uintptr_t out, uintptr_t amax, int NB, int B, int D,
                  int H, int W, int C, uintptr_t stream) {
  NIDT_REQUIRE(C % 8 == 0, "bn_relu_pool: C % 8");
  const int64_t tot = (int64_t)NB * (D / 3) * (H / 3) * (W / 3) * (C / 8);
  hipLaunchKernelGGL(k_bn_relu_pool, dim3((unsigned)std::min<int64_t>(16384, (tot + 255) / 256)), dim3(256), 0,
                     as_stream(stream), ptr<const uint16_t>(y), ptr<const float>(scale), ptr<const float>(shift),
                     ptr<uint16_t>(out), ptr<uint8_t>(amax), NB, B, D, H, W, C);
  NIDT_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// backward
struct BwdSrc {
  const uint16_t* y;      // conv output (pre-BN) [NB, D, H, W, C]
  const uint16_t* dsrc;   // POOL: dL/d(pooled relu out) [NB, Dp, Hp, Wp, C]; DENSE: dL/d(relu out) [NB, D, H, W, C]
  const uint16_t* pout;   // POOL: pooled relu output
  const uint8_t* amax;    // POOL: argmax
  const float* scale;     // [G, C] forward BN scale (DENSE relu mask)
  const float* shift;
  const float* mean;      // [G, C]
  const float* invstd;
  int NB, B, D, H, W, C;
};

__device__ __forceinline__ void unpack8(uint4 u, float* f) {
  const uint32_t w4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[2 * j] = __uint_as_float(w4[j] << 16);
    f[2 * j + 1] = __uint_as_float(w4[j] & 0xffff0000u);
  }
}

// One block = (chunk of positions of client g); threads = rows x channel groups.
template <bool POOL>
__global__ __launch_bounds__(256) void k_bn_bwd_reduce(BwdSrc s, int nchunk, float* __restrict__ part) {
  __shared__ float red[2][256 * 8];
  const int g = blockIdx.y, ch = blockIdx.x;
  const int C8 = s.C / 8;
  const int rows = 256 / C8;
  const int tid = threadIdx.x;
  const int row = tid / C8, cg = tid - row * C8;
  const int Dp = s.D / 3, Hp = s.H / 3, Wp = s.W / 3;
  const int64_t per = POOL ? (int64_t)s.B * Dp * Hp * Wp : (int64_t)s.B * s.D * s.H * s.W;
  const int64_t cs = (per + nchunk - 1) / nchunk;
  const int64_t b0 = ch * cs, b1 = min(per, b0 + cs);
  float sdz[8], sdx[8], mn[8], iv[8], sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sdz[j] = 0.f; sdx[j] = 0.f;
    if (row < rows) {
      mn[j] = s.mean[g * s.C + cg * 8 + j];
      iv[j] = s.invstd[g * s.C + cg * 8 + j];
      sc[j] = s.scale[g * s.C + cg * 8 + j];
      sh[j] = s.shift[g * s.C + cg * 8 + j];
    }
  }
  if (row < rows) {
    for (int64_t q = b0 + row; q < b1; q += rows) {
      const int64_t gq = (int64_t)g * per + q;  // global index of the (pooled) position
      float d[8], yv[8];
      if (POOL) {
        const int64_t o = gq * s.C + cg * 8;
        float dp[8], pv[8];
        unpack8(*reinterpret_cast<const uint4*>(s.dsrc + o), dp);
        unpack8(*reinterpret_cast<const uint4*>(s.pout + o), pv);
        const uint2 ab = *reinterpret_cast<const uint2*>(s.amax + o);
        int64_t v = gq;
        const int pw = (int)(v % Wp); v /= Wp;
        const int ph = (int)(v % Hp); v /= Hp;
        const int pd = (int)(v % Dp);
        const int n = (int)(v / Dp);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int a = (int)(((j < 4 ? ab.x : ab.y) >> (8 * (j & 3))) & 0xff);
          const int dd = a / 9, dh = (a / 3) % 3, dw = a % 3;
          const int64_t yi = ((((int64_t)n * s.D + 3 * pd + dd) * s.H + 3 * ph + dh) * s.W + 3 * pw + dw) * s.C + cg * 8 + j;
          yv[j] = bf16_to_f32(s.y[yi]);
          d[j] = pv[j] > 0.f ? dp[j] : 0.f;
        }
      } else {
        const int64_t o = gq * s.C + cg * 8;
        float dv[8];
        unpack8(*reinterpret_cast<const uint4*>(s.dsrc + o), dv);
        unpack8(*reinterpret_cast<const uint4*>(s.y + o), yv);
#pragma unroll
        for (int j = 0; j < 8; ++j) d[j] = fmaf(yv[j], sc[j], sh[j]) > 0.f ? dv[j] : 0.f;
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sdz[j] += d[j];
        sdx[j] = fmaf(d[j], (yv[j] - mn[j]) * iv[j], sdx[j]);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][tid * 8 + j] = sdz[j];
    red[1][tid * 8 + j] = sdx[j];
  }
  __syncthreads();
  for (int c = tid; c < s.C; c += 256) {
    const int cgi = c / 8, j = c % 8;
    float a0 = 0.f, a1 = 0.f;
    for (int r = 0; r < rows; ++r) {
      a0 += red[0][(r * C8 + cgi) * 8 + j];
      a1 += red[1][(r * C8 + cgi) * 8 + j];
    }
    part[(((int64_t)g * nchunk + ch) * s.C + c) * 2] = a0;
    part[(((int64_t)g * nchunk + ch) * s.C + c) * 2 + 1] = a1;
  }
}

// per (g,c): reduce chunks, write dgamma/dbeta (+ zero conv-bias grad), affine dx coefficients
// One wave per (g, c): lanes take the chunk partials (fixed-order shuffle tree: deterministic), lane 0 finishes.
// (A thread per (g, c) walking the 64 chunks serially was latency-bound: 18 us per call at 8 clients.)
__global__ __launch_bounds__(256) void k_bn_bwd_fin(const float* __restrict__ part, int nchunk, int G, int C,
                                                    double Ncount, const float* __restrict__ mean,
                                                    const float* __restrict__ invstd, const float* theta, int64_t ldt,
                                                    int64_t off_g, float* grad, int64_t ldg, int64_t goff_g,
                                                    int64_t goff_b, int64_t goff_convb, float* __restrict__ coef,
                                                    int eval_mode) {
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (i >= G * C) return;
  const int g = i / C, c = i - g * C;
  double sdz = 0, sdx = 0;
  for (int k = lane; k < nchunk; k += 64) {
    sdz += part[(((int64_t)g * nchunk + k) * C + c) * 2];
    sdx += part[(((int64_t)g * nchunk + k) * C + c) * 2 + 1];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    sdz += __shfl_xor(sdz, o, 64);
    sdx += __shfl_xor(sdx, o, 64);
  }
  if (lane != 0) return;
  const float gm = theta[(int64_t)g * ldt + off_g + c];
  const double iv = invstd[i], mu = mean[i];
  grad[(int64_t)g * ldg + goff_g + c] = (float)sdx;
  grad[(int64_t)g * ldg + goff_b + c] = (float)sdz;
  if (eval_mode) {  // running statistics are constants: dy = gamma * invstd * dz, conv bias grad = sum dy
    if (goff_convb >= 0) grad[(int64_t)g * ldg + goff_convb + c] = (float)(gm * iv * sdz);
    coef[i * 3 + 0] = (float)(gm * iv);
    coef[i * 3 + 1] = 0.f;
    coef[i * 3 + 2] = 0.f;
    return;
  }
  if (goff_convb >= 0) grad[(int64_t)g * ldg + goff_convb + c] = 0.f;
  // dy = gm*iv*(dz - sdz/N - xhat*sdx/N), xhat = (y - mu)*iv
  const double A = gm * iv;
  const double Cc = -gm * iv * iv * sdx / Ncount;
  const double Bc = -gm * iv * sdz / Ncount + gm * iv * iv * mu * sdx / Ncount;
  coef[i * 3 + 0] = (float)A;
  coef[i * 3 + 1] = (float)Bc;
  coef[i * 3 + 2] = (float)Cc;
}

template <bool POOL>
// Block (chunk, sample n): lane -> channel group cg (8 channels, fixed per thread, so the dy = A dz + Bc + Cc y
// coefficients and the ReLU affine are loaded once), threads stride over the chunk's positions with 32-bit
// index math.  (The flat 64-bit grid-stride version spent its issue slots on 64-bit div/mod and 24 coefficient
// loads per 16 B of output: ~3.2 TB/s on the 1.6 GB conv2 tensors.)
__global__ __launch_bounds__(256) void k_bn_bwd_dx(BwdSrc s, const float* __restrict__ coef, uint16_t* __restrict__ dy) {
  const int C8 = s.C / 8, npl = 256 / C8;
  const int cg = threadIdx.x % C8, pl = threadIdx.x / C8;
  if (pl >= npl) return;
  const int n = blockIdx.y, g = n / s.B;
  const int HW = s.H * s.W, S = s.D * HW;
  const int chunk = (S + gridDim.x - 1) / gridDim.x;
  const int p0 = blockIdx.x * chunk, p1 = min(S, p0 + chunk);
  const int Dp = s.D / 3, Hp = s.H / 3, Wp = s.W / 3;
  float cA[8], cB[8], cC[8], sc[8], sh[8];
  {
    const float4* cf = reinterpret_cast<const float4*>(coef + (int64_t)(g * s.C + cg * 8) * 3);  // 96-B aligned
    float t[24];
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const float4 v = cf[q];
      t[4 * q] = v.x; t[4 * q + 1] = v.y; t[4 * q + 2] = v.z; t[4 * q + 3] = v.w;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) { cA[j] = t[3 * j]; cB[j] = t[3 * j + 1]; cC[j] = t[3 * j + 2]; }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sc[j] = POOL ? 0.f : s.scale[g * s.C + cg * 8 + j];
      sh[j] = POOL ? 0.f : s.shift[g * s.C + cg * 8 + j];
    }
  }
  const uint16_t* yb = s.y + (int64_t)n * S * s.C + cg * 8;
  uint16_t* db = dy + (int64_t)n * S * s.C + cg * 8;
  for (int p = p0 + pl; p < p1; p += npl) {
    const int d = p / HW, r = p - d * HW, h = r / s.W, w = r - h * s.W;
    const int64_t pos = (int64_t)n * S + p;
    float yv[8], dz[8];
    unpack8(*reinterpret_cast<const uint4*>(yb + (int64_t)p * s.C), yv);
    if (POOL) {
#pragma unroll
      for (int j = 0; j < 8; ++j) dz[j] = 0.f;
      const int pd = d / 3, ph = h / 3, pw = w / 3;
      if (pd < Dp && ph < Hp && pw < Wp) {
        const int64_t pq = ((((int64_t)n * Dp + pd) * Hp + ph) * Wp + pw) * s.C + cg * 8;
        const int li = (d - 3 * pd) * 9 + (h - 3 * ph) * 3 + (w - 3 * pw);
        const uint2 ab = *reinterpret_cast<const uint2*>(s.amax + pq);
        float dp[8], pv[8];
        unpack8(*reinterpret_cast<const uint4*>(s.dsrc + pq), dp);
        unpack8(*reinterpret_cast<const uint4*>(s.pout + pq), pv);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int a = (int)(((j < 4 ? ab.x : ab.y) >> (8 * (j & 3))) & 0xff);
          dz[j] = (a == li && pv[j] > 0.f) ? dp[j] : 0.f;
        }
      }
    } else {
      float dv[8];
      unpack8(*reinterpret_cast<const uint4*>(s.dsrc + pos * s.C + cg * 8), dv);
#pragma unroll
      for (int j = 0; j < 8; ++j) dz[j] = fmaf(yv[j], sc[j], sh[j]) > 0.f ? dv[j] : 0.f;
    }
    uint32_t pk[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float o0 = fmaf(cA[2 * j], dz[2 * j], fmaf(cC[2 * j], yv[2 * j], cB[2 * j]));
      const float o1 = fmaf(cA[2 * j + 1], dz[2 * j + 1], fmaf(cC[2 * j + 1], yv[2 * j + 1], cB[2 * j + 1]));
      pk[j] = pack_bf16x2(o0, o1);
    }
    *reinterpret_cast<uint4*>(db + (int64_t)p * s.C) = make_uint4(pk[0], pk[1], pk[2], pk[3]);
  }
}

void bn_bwd(int pool, uintptr_t y, uintptr_t dsrc, uintptr_t pout, uintptr_t amax, uintptr_t scale, uintptr_t shift,
            uintptr_t mean, uintptr_t invstd, int NB, int B, int D, int H, int W, int C, uintptr_t part, int nchunk,
            uintptr_t theta, int64_t ldt, int64_t off_g, uintptr_t grad, int64_t ldg, int64_t goff_g, int64_t goff_b,
            int64_t goff_convb, uintptr_t coef, uintptr_t dy, int eval_mode, uintptr_t stream) {
  NIDT_REQUIRE(C % 8 == 0 && C <= 256, "bn_bwd: C");
  BwdSrc s{ptr<const uint16_t>(y), ptr<const uint16_t>(dsrc), ptr<const uint16_t>(pout), ptr<const uint8_t>(amax),
           ptr<const float>(scale), ptr<const float>(shift), ptr<const float>(mean), ptr<const float>(invstd),
           NB, B, D, H, W, C};
  const int G = NB / B;
  hipStream_t st = as_stream(stream);
  dim3 grid(nchunk, G);
  if (pool) hipLaunchKernelGGL((k_bn_bwd_reduce<true>), grid, dim3(256), 0, st, s, nchunk, ptr<float>(part));
  else hipLaunchKernelGGL((k_bn_bwd_reduce<false>), grid, dim3(256), 0, st, s, nchunk, ptr<float>(part));
  NIDT_CHECK(hipGetLastError());
  const double Ncount = (double)B * D * H * W;
  hipLaunchKernelGGL(k_bn_bwd_fin, dim3(ceil_div(G * C, 4)), dim3(256), 0, st, ptr<const float>(part), nchunk, G, C,
                     Ncount, ptr<const float>(mean), ptr<const float>(invstd), ptr<const float>(theta), ldt, off_g,
                     ptr<float>(grad), ldg, goff_g, goff_b, goff_convb, ptr<float>(coef), eval_mode);
  NIDT_CHECK(hipGetLastError());
  NIDT_REQUIRE((int64_t)D * H * W * C < (1ll << 31), "bn_bwd: per-sample tensor too large for 32-bit offsets");
  const int S = D * H * W, npl = 256 / (C / 8);
  // ~8k blocks in total, each chunk at least one position per thread row
  const int nch = std::max(1, std::min(std::max(1, 8192 / NB), (S + npl - 1) / npl));
  dim3 g2(nch, NB);
  if (pool) hipLaunchKernelGGL((k_bn_bwd_dx<true>), g2, dim3(256), 0, st, s, ptr<const float>(coef), ptr<uint16_t>(dy));
  else hipLaunchKernelGGL((k_bn_bwd_dx<false>), g2, dim3(256), 0, st, s, ptr<const float>(coef), ptr<uint16_t>(dy));
  NIDT_CHECK(hipGetLastError());
}

}  // namespace nidt
