// BatchNorm3d (training and eval mode) for client-grouped channels-last activations [G][M = B*D*H*W][C] (bf16), the
// normalisation of the 3D ResNets (fedml_api/model/cv/salient_models.py:8-139 BasicBlock/Bottleneck; the config-5
// ResNet-50): per-client statistics over the client's batch, per-client affine and running statistics (rows of
// theta / bufs).
//
// Statistics are two-stage and deterministic: k_bnr_partial reduces a chunk of positions of one client for every
// channel (thread = 8-channel chunk x position row; LDS merge of the rows in a fixed order) into fp32 partial sums,
// k_bnr_finalize combines the chunks in fp64 per (client, channel) and updates the running mean / unbiased variance
// (momentum 0.1) and num_batches_tracked exactly like nn.BatchNorm3d.  The apply kernel fuses the residual add and
// ReLU; the backward reuses the partial kernel for sum(dy) and sum(dy * xhat) (ReLU mask folded in) and writes
// dgamma / dbeta straight into the client's gradient row.  No atomics, no library workspaces: hipGraph-safe.
#include "common.h"

namespace nidt {

constexpr int kBnrThreads = 256;
constexpr int kBnrChunk = 2048;  // positions per partial block

__device__ __forceinline__ void bnr_unpack8(const uint4 v, float* f) {
  const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    f[2 * j] = __uint_as_float(u[j] << 16);
    f[2 * j + 1] = __uint_as_float(u[j] & 0xffff0000u);
  }
}

// [TMASK] the BN affine of the forward apply, written so that every kernel computes it bit-identically (explicit
// fmaf, no contraction choices): sc = gamma rstd, sf = beta - mu sc, x = t sc + sf.  The backward of a BN + ReLU
// without residual (the Bottleneck's bn1 / bn2) then recomputes the ReLU mask of the stored output from t instead of
// reading that bf16 tensor: mask = bf16(relu(x)) > 0, exactly the stored value's test.
__device__ __forceinline__ void bnr_affine(float gamma, float beta, float mu, float rs, float& sc, float& sf) {
  sc = gamma * rs;
  sf = fmaf(-mu, sc, beta);
}
__device__ __forceinline__ bool bnr_relu_live(float t, float sc, float sf) {
  return __uint_as_float((uint32_t)f32_to_bf16(fmaxf(fmaf(t, sc, sf), 0.f)) << 16) > 0.f;
}

// MODE 0: part = (sum t, sum t^2); MODE 1: part = (sum dy', sum dy' * xhat) with dy' = dy * (mask > 0) (mask optional),
// xhat = (t - mean) * rstd from stats [G][C][2].  dy: fp32 (DYB false) or bf16.
// TM: the mask from t ([TMASK]; theta rows give gamma / beta)
template <int MODE, bool DYB, bool TM = false>
__global__ __launch_bounds__(kBnrThreads) void k_bnr_partial(const uint16_t* __restrict__ t, const void* __restrict__ dyv,
                                                             const uint16_t* __restrict__ mask,
                                                             const float* __restrict__ stats, int M, int C,
                                                             float* __restrict__ part, const float* __restrict__ theta = nullptr,
                                                             int64_t ldt = 0, int64_t off_w = 0, int64_t off_b = 0) {
  __shared__ float sm[kBnrThreads * 17];
  const int chunk = blockIdx.x, g = blockIdx.y, nchunk = gridDim.x, tid = threadIdx.x;
  const int nch = C >> 3, rows = kBnrThreads / nch;
  const int j = tid % nch, r = tid / nch;
  const int p0 = chunk * kBnrChunk, p1 = min(M, p0 + kBnrChunk);
  const int64_t base = (int64_t)g * M * C;
  float a[8], b[8], mu[8], rs[8], tsc[8], tsf[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    a[e] = b[e] = 0.f;
    if (MODE == 1) {
      mu[e] = stats[((int64_t)g * C + 8 * j + e) * 2];
      rs[e] = stats[((int64_t)g * C + 8 * j + e) * 2 + 1];
      if (TM) bnr_affine(theta[(int64_t)g * ldt + off_w + 8 * j + e], theta[(int64_t)g * ldt + off_b + 8 * j + e], mu[e],
                         rs[e], tsc[e], tsf[e]);
    }
  }
  // per position: the t chunk, and for MODE 1 the dy / mask chunks; four positions' loads are issued before
  // their arithmetic (a thread walks ~kBnrChunk / rows positions, one dependent HBM round trip each otherwise)
  struct Ld {
    uint4 t, m, d0, d1;
  };
  auto load = [&](int p) {
    Ld v;
    const int64_t o = base + (int64_t)p * C + 8 * j;
    v.t = *reinterpret_cast<const uint4*>(t + o);
    if (MODE == 1) {
      if (DYB) {
        v.d0 = *reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(dyv) + o);
      } else {
        const uint4* q = reinterpret_cast<const uint4*>(reinterpret_cast<const float*>(dyv) + o);
        v.d0 = q[0];
        v.d1 = q[1];
      }
      if (!TM && mask) v.m = *reinterpret_cast<const uint4*>(mask + o);
    }
    return v;
  };
  auto step = [&](const Ld& v) {
    float f[8];
    bnr_unpack8(v.t, f);
    if (MODE == 0) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        a[e] += f[e];
        b[e] = fmaf(f[e], f[e], b[e]);
      }
    } else {
      float d[8];
      if (DYB) {
        bnr_unpack8(v.d0, d);
      } else {
        const uint32_t u[8] = {v.d0.x, v.d0.y, v.d0.z, v.d0.w, v.d1.x, v.d1.y, v.d1.z, v.d1.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) d[e] = __uint_as_float(u[e]);
      }
      if (TM) {
#pragma unroll
        for (int e = 0; e < 8; ++e) d[e] = bnr_relu_live(f[e], tsc[e], tsf[e]) ? d[e] : 0.f;
      } else if (mask) {
        float mk[8];
        bnr_unpack8(v.m, mk);
#pragma unroll
        for (int e = 0; e < 8; ++e) d[e] = mk[e] > 0.f ? d[e] : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        a[e] += d[e];
        b[e] = fmaf(d[e], (f[e] - mu[e]) * rs[e], b[e]);
      }
    }
  };
  if (r < rows) {
    int p = p0 + r;
    for (; p + 3 * rows < p1; p += 4 * rows) {
      const Ld v0 = load(p), v1 = load(p + rows), v2 = load(p + 2 * rows), v3 = load(p + 3 * rows);
      step(v0);
      step(v1);
      step(v2);
      step(v3);
    }
    for (; p < p1; p += rows) step(load(p));
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sm[tid * 17 + e] = a[e];
    sm[tid * 17 + 8 + e] = b[e];
  }
  __syncthreads();
  for (int c = tid; c < C; c += kBnrThreads) {
    const int jj = c >> 3, e = c & 7;
    float sa = 0.f, sb = 0.f;
    for (int rr = 0; rr < rows; ++rr) {
      sa += sm[(rr * nch + jj) * 17 + e];
      sb += sm[(rr * nch + jj) * 17 + 8 + e];
    }
    float* o = part + (((int64_t)chunk * gridDim.y + g) * C + c) * 2;
    o[0] = sa;
    o[1] = sb;
  }
  (void)nchunk;
}

// [RESBN] the residual-stream gradient of a Bottleneck (res_grad with the [OMASK] output mask) fused with the
// backward statistics of the BatchNorms that consume it next: the previous block's bn3 and, when that block has a
// projection, its downsample BN.  out = (dx1 + (dx2 | da [mask > 0])) [omask > 0] is the gradient at their outputs
// (bf16), and this pass also reduces part3 = (sum out, sum out xhat3) and partd = (sum out, sum out xhatd) per chunk
// of kBnrChunk positions, the layout k_bnr_partial writes — so their backward runs k_bnr_bwd_fin + k_bnr_bwd_apply
// only, without its own pass over (t, dy).  Sums of the stored (bf16-rounded) out, as the unfused path sums it.
template <bool HAS_D>
__global__ __launch_bounds__(kBnrThreads) void k_bnr_res_partial(
    uint16_t* __restrict__ out, const uint16_t* __restrict__ dx1, const uint16_t* __restrict__ dx2,
    const uint16_t* __restrict__ da, const uint16_t* __restrict__ mask, const uint16_t* __restrict__ omask,
    const uint16_t* __restrict__ t3, const float* __restrict__ s3, float* __restrict__ part3,
    const uint16_t* __restrict__ td, const float* __restrict__ sd, float* __restrict__ partd, int M, int C) {
  __shared__ float sm[kBnrThreads * 25];
  const int chunk = blockIdx.x, g = blockIdx.y, tid = threadIdx.x;
  const int nch = C >> 3, rows = kBnrThreads / nch;
  const int j = tid % nch, r = tid / nch;
  const int p0 = chunk * kBnrChunk, p1 = min(M, p0 + kBnrChunk);
  const int64_t base = (int64_t)g * M * C;
  float a[8], b3[8], bd[8], mu3[8], rs3[8], mud[8], rsd[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    a[e] = b3[e] = bd[e] = 0.f;
    mu3[e] = s3[((int64_t)g * C + 8 * j + e) * 2];
    rs3[e] = s3[((int64_t)g * C + 8 * j + e) * 2 + 1];
    if (HAS_D) {
      mud[e] = sd[((int64_t)g * C + 8 * j + e) * 2];
      rsd[e] = sd[((int64_t)g * C + 8 * j + e) * 2 + 1];
    }
  }
  // loads of four positions are issued before their arithmetic (k_bnr_partial)
  struct Ld {
    uint4 x1, x2, mk, om, t3, td;
  };
  auto load = [&](int p) {
    Ld v;
    const int64_t o = base + (int64_t)p * C + 8 * j;
    v.x1 = *reinterpret_cast<const uint4*>(dx1 + o);
    v.x2 = *reinterpret_cast<const uint4*>((dx2 ? dx2 : da) + o);
    if (!dx2 && mask) v.mk = *reinterpret_cast<const uint4*>(mask + o);
    v.om = *reinterpret_cast<const uint4*>(omask + o);
    v.t3 = *reinterpret_cast<const uint4*>(t3 + o);
    if (HAS_D) v.td = *reinterpret_cast<const uint4*>(td + o);
    return v;
  };
  auto step = [&](int p, const Ld& v) {
    const int64_t o = base + (int64_t)p * C + 8 * j;
    float x1[8], x2[8], om[8], f3[8], fd[8];
    bnr_unpack8(v.x1, x1);
    bnr_unpack8(v.x2, x2);
    if (!dx2 && mask) {
      float mk[8];
      bnr_unpack8(v.mk, mk);
#pragma unroll
      for (int e = 0; e < 8; ++e) x2[e] = mk[e] > 0.f ? x2[e] : 0.f;
    }
    bnr_unpack8(v.om, om);
    bnr_unpack8(v.t3, f3);
    if (HAS_D) bnr_unpack8(v.td, fd);
    uint32_t w[4];
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      const float v0 = om[e] > 0.f ? x1[e] + x2[e] : 0.f, v1 = om[e + 1] > 0.f ? x1[e + 1] + x2[e + 1] : 0.f;
      w[e >> 1] = pack_bf16x2(v0, v1);
    }
    *reinterpret_cast<uint4*>(out + o) = make_uint4(w[0], w[1], w[2], w[3]);
    float d[8];
    bnr_unpack8(make_uint4(w[0], w[1], w[2], w[3]), d);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      a[e] += d[e];
      b3[e] = fmaf(d[e], (f3[e] - mu3[e]) * rs3[e], b3[e]);
      if (HAS_D) bd[e] = fmaf(d[e], (fd[e] - mud[e]) * rsd[e], bd[e]);
    }
  };
  if (r < rows) {
    int p = p0 + r;
    for (; p + 3 * rows < p1; p += 4 * rows) {
      const Ld v0 = load(p), v1 = load(p + rows), v2 = load(p + 2 * rows), v3 = load(p + 3 * rows);
      step(p, v0);
      step(p + rows, v1);
      step(p + 2 * rows, v2);
      step(p + 3 * rows, v3);
    }
    for (; p < p1; p += rows) step(p, load(p));
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sm[tid * 25 + e] = a[e];
    sm[tid * 25 + 8 + e] = b3[e];
    sm[tid * 25 + 16 + e] = bd[e];
  }
  __syncthreads();
  for (int c = tid; c < C; c += kBnrThreads) {
    const int jj = c >> 3, e = c & 7;
    float sa = 0.f, sb = 0.f, sdd = 0.f;
    for (int rr = 0; rr < rows; ++rr) {
      sa += sm[(rr * nch + jj) * 25 + e];
      sb += sm[(rr * nch + jj) * 25 + 8 + e];
      sdd += sm[(rr * nch + jj) * 25 + 16 + e];
    }
    float* o3 = part3 + (((int64_t)chunk * gridDim.y + g) * C + c) * 2;
    o3[0] = sa;
    o3[1] = sb;
    if (HAS_D) {
      float* od = partd + (((int64_t)chunk * gridDim.y + g) * C + c) * 2;
      od[0] = sa;
      od[1] = sdd;
    }
  }
}

// per (client, channel): stats = (mean, rstd); running stats rows updated (train mode)
__global__ void k_bnr_finalize(const float* __restrict__ part, int nchunk, int G, int C, int M, float eps, float mom,
                               float* __restrict__ stats, float* bufs, int64_t ldb, int64_t off_rm, int64_t off_rv,
                               int64_t off_nbt) {
  const int g = blockIdx.x;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    double s = 0.0, q = 0.0;
    for (int k = 0; k < nchunk; ++k) {
      const float* p = part + (((int64_t)k * G + g) * C + c) * 2;
      s += p[0];
      q += p[1];
    }
    const double mean = s / M;
    const double var = fmax(q / M - mean * mean, 0.0);
    stats[((int64_t)g * C + c) * 2] = (float)mean;
    stats[((int64_t)g * C + c) * 2 + 1] = (float)(1.0 / sqrt(var + eps));
    if (bufs) {
      float* rm = bufs + (int64_t)g * ldb + off_rm;
      float* rv = bufs + (int64_t)g * ldb + off_rv;
      const double unb = M > 1 ? var * M / (M - 1) : var;
      rm[c] = (float)((1.0 - mom) * rm[c] + mom * mean);
      rv[c] = (float)((1.0 - mom) * rv[c] + mom * unb);
      if (c == 0 && off_nbt >= 0) bufs[(int64_t)g * ldb + off_nbt] += 1.f;
    }
  }
}

// eval mode: stats from the running statistics rows
__global__ void k_bnr_eval_stats(int G, int C, float eps, const float* __restrict__ bufs, int64_t ldb, int64_t off_rm,
                                 int64_t off_rv, float* __restrict__ stats) {
  const int g = blockIdx.x;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    stats[((int64_t)g * C + c) * 2] = bufs[(int64_t)g * ldb + off_rm + c];
    stats[((int64_t)g * C + c) * 2 + 1] = rsqrtf(bufs[(int64_t)g * ldb + off_rv + c] + eps);
  }
}

template <bool RES, bool RELU>
__global__ __launch_bounds__(256) void k_bnr_apply(const uint16_t* __restrict__ t, const uint16_t* __restrict__ res,
                                                   const float* __restrict__ stats, const float* __restrict__ theta,
                                                   int64_t ldt, int64_t off_w, int64_t off_b, uint16_t* __restrict__ y,
                                                   int64_t M, int C) {
  const int nch = C >> 3;
  const int64_t per = M * nch, tot = per * gridDim.y;
  (void)tot;
  const int g = blockIdx.y;
  // the grid stride (a multiple of 256 threads) is a multiple of nch = C/8 <= 256: a thread's channel chunk j never
  // changes, so its 8 channels' scale/shift are loaded once (they were 4 global loads per channel per chunk)
  const int64_t q0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int j = (int)(q0 % nch);
  float sc[8], sf[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = 8 * j + e;
    const float mu = stats[((int64_t)g * C + c) * 2], rs = stats[((int64_t)g * C + c) * 2 + 1];
    bnr_affine(theta[(int64_t)g * ldt + off_w + c], theta[(int64_t)g * ldt + off_b + c], mu, rs, sc[e], sf[e]);
  }
  for (int64_t q = q0; q < per; q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t o = ((int64_t)g * M * nch + q) * 8;
    float f[8], rr[8];
    bnr_unpack8(*reinterpret_cast<const uint4*>(t + o), f);
    if (RES) bnr_unpack8(*reinterpret_cast<const uint4*>(res + o), rr);
    uint32_t out[4];
#pragma unroll
    for (int e = 0; e < 8; e += 2) {
      float v[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        float x = fmaf(f[e + h], sc[e + h], sf[e + h]);
        if (RES) x += rr[e + h];
        if (RELU) x = fmaxf(x, 0.f);
        v[h] = x;
      }
      out[e >> 1] = pack_bf16x2(v[0], v[1]);
    }
    *reinterpret_cast<uint4*>(y + o) = make_uint4(out[0], out[1], out[2], out[3]);
  }
}

// dgamma / dbeta rows from the backward partials; coef [G][C][2] = (sum dy'/M, sum dy'*xhat/M)
__global__ void k_bnr_bwd_fin(const float* __restrict__ part, int nchunk, int G, int C, int M, float* __restrict__ grads,
                              int64_t ldg, int64_t off_w, int64_t off_b, float* __restrict__ coef) {
  const int g = blockIdx.x;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    double a = 0.0, b = 0.0;
    for (int k = 0; k < nchunk; ++k) {
      const float* p = part + (((int64_t)k * G + g) * C + c) * 2;
      a += p[0];
      b += p[1];
    }
    grads[(int64_t)g * ldg + off_w + c] = (float)b;
    grads[(int64_t)g * ldg + off_b + c] = (float)a;
    coef[((int64_t)g * C + c) * 2] = (float)(a / M);
    coef[((int64_t)g * C + c) * 2 + 1] = (float)(b / M);
  }
}

// dt = rstd * gamma * (dy' - mean(dy') - xhat * mean(dy' xhat))   (eval mode: coef = 0 -> rstd * gamma * dy')
template <bool DYB, bool TM = false>
__global__ __launch_bounds__(256) void k_bnr_bwd_apply(const uint16_t* __restrict__ t, const void* __restrict__ dyv,
                                                       const uint16_t* __restrict__ mask,
                                                       const float* __restrict__ stats, const float* __restrict__ coef,
                                                       const float* __restrict__ theta, int64_t ldt, int64_t off_w,
                                                       uint16_t* __restrict__ dt, int64_t M, int C, int64_t off_b = 0) {
  const int nch = C >> 3;
  const int64_t per = M * nch;
  const int g = blockIdx.y;
  // loop-invariant channel chunk (see k_bnr_apply): dt = A dy' + K1 + K2 t with A = rstd gamma,
  // K2 = -A rstd m2, K1 = -A m1 - K2 mu
  const int64_t q0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int j = (int)(q0 % nch);
  float A[8], K1[8], K2[8], tsc[8], tsf[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = 8 * j + e;
    const float mu = stats[((int64_t)g * C + c) * 2], rs = stats[((int64_t)g * C + c) * 2 + 1];
    if (TM) bnr_affine(theta[(int64_t)g * ldt + off_w + c], theta[(int64_t)g * ldt + off_b + c], mu, rs, tsc[e], tsf[e]);
    const float m1 = coef ? coef[((int64_t)g * C + c) * 2] : 0.f;
    const float m2 = coef ? coef[((int64_t)g * C + c) * 2 + 1] : 0.f;
    A[e] = rs * theta[(int64_t)g * ldt + off_w + c];
    K2[e] = -A[e] * rs * m2;
    K1[e] = -A[e] * m1 - K2[e] * mu;
  }
  for (int64_t q = q0; q < per; q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t o = ((int64_t)g * M * nch + q) * 8;
    float f[8], d[8];
    bnr_unpack8(*reinterpret_cast<const uint4*>(t + o), f);
    if (DYB) {
      bnr_unpack8(*reinterpret_cast<const uint4*>(reinterpret_cast<const uint16_t*>(dyv) + o), d);
    } else {
      const float4* p = reinterpret_cast<const float4*>(reinterpret_cast<const float*>(dyv) + o);
      const float4 x0 = p[0], x1 = p[1];
      d[0] = x0.x; d[1] = x0.y; d[2] = x0.z; d[3] = x0.w; d[4] = x1.x; d[5] = x1.y; d[6] = x1.z; d[7] = x1.w;
    }
    if (TM) {
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] = bnr_relu_live(f[e], tsc[e], tsf[e]) ? d[e] : 0.f;
    } else if (mask) {
      float mk[8];
      bnr_unpack8(*reinterpret_cast<const uint4*>(mask + o), mk);
#pragma unroll
      for (int e = 0; e < 8; ++e) d[e] = mk[e] > 0.f ? d[e] : 0.f;
    }
    uint32_t out[4];
#pragma unroll
    for (int e = 0; e < 8; e += 2)
      out[e >> 1] = pack_bf16x2(fmaf(A[e], d[e], fmaf(K2[e], f[e], K1[e])),
                                fmaf(A[e + 1], d[e + 1], fmaf(K2[e + 1], f[e + 1], K1[e + 1])));
    *reinterpret_cast<uint4*>(dt + o) = make_uint4(out[0], out[1], out[2], out[3]);
  }
}

static void bnr_check(int G, int64_t M, int C, const char* who) {
  NIDT_REQUIRE(G > 0 && M > 0 && C % 8 == 0 && C <= 2048 && kBnrThreads % (C / 8) == 0,
               std::string(who) + ": C a power-of-two multiple of 8, <= 2048");
  NIDT_REQUIRE(M < (1ll << 31), std::string(who) + ": positions per client < 2^31");
}

static int bnr_nchunk(int64_t M) { return (int)((M + kBnrChunk - 1) / kBnrChunk); }

int bnr_workspace(int G, int64_t M, int C) { return bnr_nchunk(M) * G * C * 2; }

// training-mode statistics (+ running stats) -> stats [G][C][2]; ws: bnr_workspace floats
void bnr_stats(uintptr_t t, int G, int64_t M, int C, float eps, float mom, uintptr_t ws, uintptr_t stats,
               uintptr_t bufs, int64_t ldb, int64_t off_rm, int64_t off_rv, int64_t off_nbt, uintptr_t stream) {
  bnr_check(G, M, C, "bnr_stats");
  NIDT_REQUIRE(C / 8 <= kBnrThreads, "bnr_stats: C <= 2048");
  hipStream_t s = as_stream(stream);
  const int nc = bnr_nchunk(M);
  hipLaunchKernelGGL((k_bnr_partial<0, false>), dim3(nc, G), dim3(kBnrThreads), 0, s, ptr<const uint16_t>(t), nullptr,
                     nullptr, nullptr, (int)M, C, ptr<float>(ws));
  NIDT_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_bnr_finalize, dim3(G), dim3(256), 0, s, ptr<const float>(ws), nc, G, C, (int)M, eps, mom,
                     ptr<float>(stats), ptr<float>(bufs), ldb, off_rm, off_rv, off_nbt);
  NIDT_CHECK(hipGetLastError());
}

// training-mode statistics from precomputed chunk partials part [nchunk][G][C][2] (e.g. gemm1x1.hip's [STATS]
// epilogue) -> stats [G][C][2] (+ running stats); the k_bnr_partial pass over t is skipped
void bnr_finalize_part(uintptr_t part, int nchunk, int G, int64_t M, int C, float eps, float mom, uintptr_t stats,
                       uintptr_t bufs, int64_t ldb, int64_t off_rm, int64_t off_rv, int64_t off_nbt, uintptr_t stream) {
  bnr_check(G, M, C, "bnr_finalize_part");
  NIDT_REQUIRE(nchunk > 0, "bnr_finalize_part: nchunk");
  hipLaunchKernelGGL(k_bnr_finalize, dim3(G), dim3(256), 0, as_stream(stream), ptr<const float>(part), nchunk, G, C,
                     (int)M, eps, mom, ptr<float>(stats), ptr<float>(bufs), ldb, off_rm, off_rv, off_nbt);
  NIDT_CHECK(hipGetLastError());
}

void bnr_eval_stats(int G, int C, float eps, uintptr_t bufs, int64_t ldb, int64_t off_rm, int64_t off_rv,
                    uintptr_t stats, uintptr_t stream) {
  hipLaunchKernelGGL(k_bnr_eval_stats, dim3(G), dim3(256), 0, as_stream(stream), G, C, eps, ptr<const float>(bufs), ldb,
                     off_rm, off_rv, ptr<float>(stats));
  NIDT_CHECK(hipGetLastError());
}

static dim3 bnr_grid(int G, int64_t M, int C) {
  const int64_t per = M * (C / 8);
  return dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(4096 / std::max(1, G) + 1, (per + 255) / 256)), G);
}

void bnr_apply(uintptr_t t, uintptr_t res, uintptr_t stats, uintptr_t theta, int64_t ldt, int64_t off_w, int64_t off_b,
               uintptr_t y, int G, int64_t M, int C, int relu, uintptr_t stream) {
  bnr_check(G, M, C, "bnr_apply");
  hipStream_t s = as_stream(stream);
  const dim3 grid = bnr_grid(G, M, C);
#define BNRA(R, L)                                                                                             \
  hipLaunchKernelGGL((k_bnr_apply<R, L>), grid, dim3(256), 0, s, ptr<const uint16_t>(t), ptr<const uint16_t>(res), \
                     ptr<const float>(stats), ptr<const float>(theta), ldt, off_w, off_b, ptr<uint16_t>(y), M, C)
  if (res) { if (relu) BNRA(true, true); else BNRA(true, false); }
  else { if (relu) BNRA(false, true); else BNRA(false, false); }
#undef BNRA
  NIDT_CHECK(hipGetLastError());
}

// backward: dgamma/dbeta rows (train mode) and dt.  eval_mode: BN used running stats (no statistics gradient).
// bnr_bwd_tm with tmask: the ReLU mask recomputed from t ([TMASK]; the forward was bnr_apply with relu, no residual,
// and the same stats / theta rows); mask must be null then.
void bnr_bwd_tm(uintptr_t t, uintptr_t dy, int dy_bf16, uintptr_t mask, uintptr_t stats, uintptr_t theta, int64_t ldt,
                int64_t off_w, int64_t off_b, uintptr_t grads, int64_t ldg, uintptr_t ws, uintptr_t coef, uintptr_t dt,
                int G, int64_t M, int C, int eval_mode, int tmask, uintptr_t stream) {
  bnr_check(G, M, C, "bnr_bwd");
  NIDT_REQUIRE(C / 8 <= kBnrThreads, "bnr_bwd: C <= 2048");
  NIDT_REQUIRE(!tmask || (!mask && dy_bf16), "bnr_bwd: tmask replaces the mask tensor (bf16 dy)");
  hipStream_t s = as_stream(stream);
  const int nc = bnr_nchunk(M);
  if (tmask) {
    hipLaunchKernelGGL((k_bnr_partial<1, true, true>), dim3(nc, G), dim3(kBnrThreads), 0, s, ptr<const uint16_t>(t),
                       ptr<const void>(dy), nullptr, ptr<const float>(stats), (int)M, C, ptr<float>(ws),
                       ptr<const float>(theta), ldt, off_w, off_b);
    NIDT_CHECK(hipGetLastError());
    hipLaunchKernelGGL(k_bnr_bwd_fin, dim3(G), dim3(256), 0, s, ptr<const float>(ws), nc, G, C, (int)M,
                       ptr<float>(grads), ldg, off_w, off_b, ptr<float>(coef));
    NIDT_CHECK(hipGetLastError());
    hipLaunchKernelGGL((k_bnr_bwd_apply<true, true>), bnr_grid(G, M, C), dim3(256), 0, s, ptr<const uint16_t>(t),
                       ptr<const void>(dy), nullptr, ptr<const float>(stats),
                       eval_mode ? nullptr : ptr<const float>(coef), ptr<const float>(theta), ldt, off_w,
                       ptr<uint16_t>(dt), M, C, off_b);
    NIDT_CHECK(hipGetLastError());
    return;
  }
  if (dy_bf16)
    hipLaunchKernelGGL((k_bnr_partial<1, true>), dim3(nc, G), dim3(kBnrThreads), 0, s, ptr<const uint16_t>(t),
                       ptr<const void>(dy), ptr<const uint16_t>(mask), ptr<const float>(stats), (int)M, C, ptr<float>(ws));
  else
    hipLaunchKernelGGL((k_bnr_partial<1, false>), dim3(nc, G), dim3(kBnrThreads), 0, s, ptr<const uint16_t>(t),
                       ptr<const void>(dy), ptr<const uint16_t>(mask), ptr<const float>(stats), (int)M, C, ptr<float>(ws));
  NIDT_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_bnr_bwd_fin, dim3(G), dim3(256), 0, s, ptr<const float>(ws), nc, G, C, (int)M, ptr<float>(grads),
                     ldg, off_w, off_b, ptr<float>(coef));
  NIDT_CHECK(hipGetLastError());
  const dim3 grid = bnr_grid(G, M, C);
  const float* cf = eval_mode ? nullptr : ptr<const float>(coef);
  if (dy_bf16)
    hipLaunchKernelGGL(k_bnr_bwd_apply<true>, grid, dim3(256), 0, s, ptr<const uint16_t>(t), ptr<const void>(dy),
                       ptr<const uint16_t>(mask), ptr<const float>(stats), cf, ptr<const float>(theta), ldt, off_w,
                       ptr<uint16_t>(dt), M, C);
  else
    hipLaunchKernelGGL(k_bnr_bwd_apply<false>, grid, dim3(256), 0, s, ptr<const uint16_t>(t), ptr<const void>(dy),
                       ptr<const uint16_t>(mask), ptr<const float>(stats), cf, ptr<const float>(theta), ldt, off_w,
                       ptr<uint16_t>(dt), M, C);
  NIDT_CHECK(hipGetLastError());
}

void bnr_bwd(uintptr_t t, uintptr_t dy, int dy_bf16, uintptr_t mask, uintptr_t stats, uintptr_t theta, int64_t ldt,
             int64_t off_w, int64_t off_b, uintptr_t grads, int64_t ldg, uintptr_t ws, uintptr_t coef, uintptr_t dt,
             int G, int64_t M, int C, int eval_mode, uintptr_t stream) {
  bnr_bwd_tm(t, dy, dy_bf16, mask, stats, theta, ldt, off_w, off_b, grads, ldg, ws, coef, dt, G, M, C, eval_mode, 0,
             stream);
}

// [RESBN] host side: out and the chunk partials of bn3 (ws3) and, with td, of the downsample BN (wsd); flags bit 1:
// da bf16 (required: the engines keep the stream in bf16)
void bnr_res_partial(uintptr_t out, uintptr_t dx1, uintptr_t dx2, uintptr_t da, uintptr_t mask, uintptr_t omask,
                     uintptr_t t3, uintptr_t s3, uintptr_t ws3, uintptr_t td, uintptr_t sd, uintptr_t wsd, int G,
                     int64_t M, int C, uintptr_t stream) {
  bnr_check(G, M, C, "bnr_res_partial");
  NIDT_REQUIRE(C / 8 <= kBnrThreads && omask && t3 && s3 && ws3 && (dx2 || da) && (!td || (sd && wsd)),
               "bnr_res_partial: operands");
  hipStream_t s = as_stream(stream);
  const dim3 grid(bnr_nchunk(M), G);
  if (td)
    hipLaunchKernelGGL(k_bnr_res_partial<true>, grid, dim3(kBnrThreads), 0, s, ptr<uint16_t>(out),
                       ptr<const uint16_t>(dx1), ptr<const uint16_t>(dx2), ptr<const uint16_t>(da),
                       ptr<const uint16_t>(mask), ptr<const uint16_t>(omask), ptr<const uint16_t>(t3),
                       ptr<const float>(s3), ptr<float>(ws3), ptr<const uint16_t>(td), ptr<const float>(sd),
                       ptr<float>(wsd), (int)M, C);
  else
    hipLaunchKernelGGL(k_bnr_res_partial<false>, grid, dim3(kBnrThreads), 0, s, ptr<uint16_t>(out),
                       ptr<const uint16_t>(dx1), ptr<const uint16_t>(dx2), ptr<const uint16_t>(da),
                       ptr<const uint16_t>(mask), ptr<const uint16_t>(omask), ptr<const uint16_t>(t3),
                       ptr<const float>(s3), ptr<float>(ws3), nullptr, nullptr, nullptr, (int)M, C);
  NIDT_CHECK(hipGetLastError());
}

// backward from precomputed chunk partials ws [nchunk][G][C][2] of (sum dy', sum dy' xhat) (k_bnr_res_partial):
// dgamma / dbeta rows and dt, no statistics pass; dy bf16, no mask (the partials' producer applied it)
void bnr_bwd_part(uintptr_t t, uintptr_t dy, uintptr_t stats, uintptr_t theta, int64_t ldt, int64_t off_w,
                  int64_t off_b, uintptr_t grads, int64_t ldg, uintptr_t ws, uintptr_t coef, uintptr_t dt, int G,
                  int64_t M, int C, uintptr_t stream) {
  bnr_check(G, M, C, "bnr_bwd_part");
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(k_bnr_bwd_fin, dim3(G), dim3(256), 0, s, ptr<const float>(ws), bnr_nchunk(M), G, C, (int)M,
                     ptr<float>(grads), ldg, off_w, off_b, ptr<float>(coef));
  NIDT_CHECK(hipGetLastError());
  hipLaunchKernelGGL((k_bnr_bwd_apply<true, false>), bnr_grid(G, M, C), dim3(256), 0, s, ptr<const uint16_t>(t),
                     ptr<const void>(dy), nullptr, ptr<const float>(stats), ptr<const float>(coef),
                     ptr<const float>(theta), ldt, off_w, ptr<uint16_t>(dt), M, C, (int64_t)0);
  NIDT_CHECK(hipGetLastError());
}

}  // namespace nidt
