// AlexNet3D classifier head + BCEWithLogits loss, forward and backward in one kernel per client.
//
// Reference: salient_models.py:171-176 (Dropout, Linear(256,64), ReLU, Dropout, Linear(64,C)) and the
// trainer's criterion nn.BCEWithLogitsLoss (sailentgrads/my_model_trainer.py:207,221).  The flattened feature
// order follows PyTorch's NCDHW flatten of the [128,1,2,1] pooled map: f = c*2 + h.
// Dropout masks come from a counter-based hash of (seed, client, sample, feature, layer), so the backward
// regenerates them instead of storing them.
#include "common.h"

namespace nidt {

__device__ __forceinline__ uint32_t hash4(uint64_t seed, uint32_t a, uint32_t b, uint32_t c) {
  uint64_t z = seed ^ (0x9e3779b97f4a7c15ull * (((uint64_t)a << 40) ^ ((uint64_t)b << 20) ^ (uint64_t)c));
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}

struct HeadArgs {
  const uint16_t* p5;   // [NB, 2, 128] bf16 pooled conv5 output (channels-last, h major)
  const float* theta;   // [G, ldt]
  int64_t ldt, off_w1, off_b1, off_w2, off_b2;
  const float* y;       // [NB] labels (train)
  float* logits;        // [NB]
  float* loss;          // [G] mean BCE (train)
  float* grad;          // [G, ldg]
  int64_t ldg;
  uint16_t* dp5;        // [NB, 2, 128] bf16 (train)
  int B, nout, train;
  float keep;           // dropout keep probability (1 = no dropout)
  uint64_t seed;
  const int* cids;      // [G] global client ids (dropout streams are per client, independent of sharding)
  const int64_t* seed_dev;  // optional: device step counter added to seed (hipGraph replays change it on device)
};

constexpr int kHF = 256, kHH = 64, kHMaxB = 32;
constexpr int kHT = 1024;  // 16 waves per client: the head is latency-bound (one block per client)

__global__ __launch_bounds__(kHT) void k_head(HeadArgs a) {
  __shared__ float F[kHMaxB][kHF + 1];
  __shared__ float Z1[kHMaxB][kHH + 1];
  __shared__ float Hd[kHMaxB][kHH + 1];
  __shared__ float Z2[kHMaxB];
  __shared__ float DZ2[kHMaxB];
  __shared__ float W1s[kHH][kHF + 1];  // w1 staged once (the dot products below read it ~nb times)
  const int g = blockIdx.x, tid = threadIdx.x;
  const uint32_t cid = a.cids ? (uint32_t)a.cids[g] : (uint32_t)g;
  const uint64_t seed = a.seed + (a.seed_dev ? (uint64_t)*a.seed_dev : 0ull);
  const float* th = a.theta + (int64_t)g * a.ldt;
  const float* w1 = th + a.off_w1;
  const float* b1 = th + a.off_b1;
  const float* w2 = th + a.off_w2;
  const float b2 = th[a.off_b2];
  const float inv_keep = a.keep > 0.f ? 1.f / a.keep : 0.f;
  const uint32_t thr = a.keep >= 1.f ? 0xffffffffu : (uint32_t)(a.keep * 4294967296.0);
  const bool drop = a.train && a.keep < 1.f;
  for (int e = tid; e < kHH * kHF; e += kHT) W1s[e / kHF][e % kHF] = w1[e];  // rows are not 16-B aligned
  // train mode processes the whole batch in one chunk (B <= 32 asserted on the host)
  for (int b0 = 0; b0 < a.B; b0 += kHMaxB) {
    const int nb = min(kHMaxB, a.B - b0);
    __syncthreads();
    for (int e = tid; e < nb * kHF; e += kHT) {
      const int b = e / kHF, f = e - b * kHF;
      const int c = f >> 1, h = f & 1;
      const int n = g * a.B + b0 + b;
      float v = bf16_to_f32(a.p5[((int64_t)n * 2 + h) * 128 + c]);
      if (drop) v = (hash4(seed, cid, b0 + b, f) < thr) ? v * inv_keep : 0.f;
      F[b][f] = v;
    }
    __syncthreads();
    for (int e = tid; e < nb * kHH; e += kHT) {
      const int b = e / kHH, o = e - b * kHH;
      float z = b1[o];
#pragma unroll 8
      for (int f = 0; f < kHF; ++f) z = fmaf(W1s[o][f], F[b][f], z);
      Z1[b][o] = z;
      float h = fmaxf(z, 0.f);
      if (drop) h = (hash4(seed ^ 0x5bd1e995ull, cid, b0 + b, o) < thr) ? h * inv_keep : 0.f;
      Hd[b][o] = h;
    }
    __syncthreads();
    if (tid < nb) {
      float z = b2;
      for (int o = 0; o < kHH; ++o) z = fmaf(w2[o], Hd[tid][o], z);
      Z2[tid] = z;
      a.logits[(int64_t)g * a.B + b0 + tid] = z;
    }
    __syncthreads();
  }
  if (!a.train) return;
  const int nb = a.B;
  // loss and dlogits (mean over the client's batch)
  if (tid < 64) {
    float l = 0.f;
    if (tid < nb) {
      const float z = Z2[tid], yy = a.y[(int64_t)g * a.B + tid];
      l = fmaxf(z, 0.f) - z * yy + log1pf(expf(-fabsf(z)));
      DZ2[tid] = (1.f / (1.f + expf(-z)) - yy) / (float)nb;
    }
    l = wave_sum(l);
    if (tid == 0) a.loss[g] = l / (float)nb;
  }
  __syncthreads();
  float* gr = a.grad + (int64_t)g * a.ldg;
  if (tid == 0) {
    float s = 0.f;
    for (int b = 0; b < nb; ++b) s += DZ2[b];
    gr[a.off_b2] = s;
  }
  if (tid < kHH) {
    float s = 0.f;
    for (int b = 0; b < nb; ++b) s = fmaf(DZ2[b], Hd[b][tid], s);
    gr[a.off_w2 + tid] = s;
  }
  // dz1 (overwrite Z1)
  __syncthreads();
  for (int e = tid; e < nb * kHH; e += kHT) {
    const int b = e / kHH, o = e - b * kHH;
    float d = DZ2[b] * w2[o];
    if (drop) d = (hash4(seed ^ 0x5bd1e995ull, cid, b, o) < thr) ? d * inv_keep : 0.f;
    Z1[b][o] = Z1[b][o] > 0.f ? d : 0.f;
  }
  __syncthreads();
  if (tid < kHH) {
    float s = 0.f;
    for (int b = 0; b < nb; ++b) s += Z1[b][tid];
    gr[a.off_b1 + tid] = s;
  }
  for (int e = tid; e < kHH * kHF; e += kHT) {
    const int o = e / kHF, f = e - o * kHF;
    float s = 0.f;
    for (int b = 0; b < nb; ++b) s = fmaf(Z1[b][o], F[b][f], s);
    gr[a.off_w1 + e] = s;
  }
  for (int e = tid; e < nb * kHF; e += kHT) {
    const int b = e / kHF, f = e - b * kHF;
    float s = 0.f;
#pragma unroll 8
    for (int o = 0; o < kHH; ++o) s = fmaf(Z1[b][o], W1s[o][f], s);
    if (drop) s = (hash4(seed, cid, b, f) < thr) ? s * inv_keep : 0.f;
    const int c = f >> 1, h = f & 1;
    a.dp5[(((int64_t)g * a.B + b) * 2 + h) * 128 + c] = f32_to_bf16(s);
  }
}

void head(uintptr_t p5, uintptr_t theta, int64_t ldt, int64_t off_w1, int64_t off_b1, int64_t off_w2, int64_t off_b2,
          uintptr_t y, uintptr_t logits, uintptr_t loss, uintptr_t grad, int64_t ldg, uintptr_t dp5, int G, int B,
          int train, float keep, uint64_t seed, uintptr_t cids, uintptr_t seed_dev, uintptr_t stream) {
  NIDT_REQUIRE(!train || B <= kHMaxB, "head: training batch per client must be <= 32");
  HeadArgs a{ptr<const uint16_t>(p5), ptr<const float>(theta), ldt, off_w1, off_b1, off_w2, off_b2,
             ptr<const float>(y), ptr<float>(logits), ptr<float>(loss), ptr<float>(grad), ldg, ptr<uint16_t>(dp5),
             B, 1, train, keep, seed, ptr<const int>(cids), ptr<const int64_t>(seed_dev)};
  hipLaunchKernelGGL(k_head, dim3(G), dim3(kHT), 0, as_stream(stream), a);
  NIDT_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// ResNet-18 classifier head + CrossEntropy, forward and backward (train step of the client-batched ResNet engine):
// pooled = mean over the final H x W map, logits = pooled W^T + b, loss = -log softmax(logits)[y] (mean over the
// client's batch), dlogits = (softmax - onehot) / B, dW / db rows, and the broadcast input gradient
// da[n, hw, c] = (dlogits W)[c] / (H W) in bf16.  Reference: resnet.py ResNet.forward (avg_pool2d(4) / adaptive
// pool, linear) with nn.CrossEntropyLoss in the trainers.  Two launches replace ~20 framework kernels per step.
//
// k_cls_head_fwd: one block per sample.  a: [N, HW, C] bf16; writes pooled [N, C], dlog [N, K] (already / B),
// lossn [N] (per-sample CE) and da.
constexpr int kCHT = 256;
constexpr int kCHMaxC = 512, kCHMaxK = 256;
__global__ __launch_bounds__(kCHT) void k_cls_head_fwd(const uint16_t* __restrict__ a, const float* __restrict__ theta,
                                                       int64_t ldt, int64_t off_w, int64_t off_b,
                                                       const int64_t* __restrict__ y, int B, int HW, int C, int K,
                                                       float* __restrict__ pooled, float* __restrict__ dlog,
                                                       float* __restrict__ lossn, uint16_t* __restrict__ da) {
  __shared__ float sP[kCHMaxC];
  __shared__ float sZ[kCHMaxK];
  __shared__ float red[kCHT / 64];
  const int n = blockIdx.x, g = n / B, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const float* W = theta + (int64_t)g * ldt + off_w;  // [K, C]
  const float* bias = theta + (int64_t)g * ldt + off_b;
  const uint16_t* an = a + (int64_t)n * HW * C;
  const float inv_hw = 1.f / (float)HW;
  for (int c = 2 * tid; c < C; c += 2 * kCHT) {  // pooled: channel pairs, one 4-B load per (hw, pair)
    float s0 = 0.f, s1 = 0.f;
    for (int hw = 0; hw < HW; ++hw) {
      const uint32_t v = *reinterpret_cast<const uint32_t*>(an + (int64_t)hw * C + c);
      s0 += bf16_to_f32((uint16_t)(v & 0xffffu));
      s1 += bf16_to_f32((uint16_t)(v >> 16));
    }
    s0 *= inv_hw;
    s1 *= inv_hw;
    sP[c] = s0;
    sP[c + 1] = s1;
    pooled[(int64_t)n * C + c] = s0;
    pooled[(int64_t)n * C + c + 1] = s1;
  }
  __syncthreads();
  for (int k = wid; k < K; k += kCHT / 64) {  // logits: one wave per class row
    float z = 0.f;
    for (int c = lane; c < C; c += 64) z = fmaf(W[(int64_t)k * C + c], sP[c], z);
    z = wave_sum(z);
    if (lane == 0) sZ[k] = z + bias[k];
  }
  __syncthreads();
  // softmax statistics (one wave; K <= 256)
  if (wid == 0) {
    float m = -INFINITY;
    for (int k = lane; k < K; k += 64) m = fmaxf(m, sZ[k]);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    float se = 0.f;
    for (int k = lane; k < K; k += 64) se += expf(sZ[k] - m);
    se = wave_sum(se);
    if (lane == 0) {
      red[0] = m;
      red[1] = se;
    }
  }
  __syncthreads();
  const float m = red[0], se = red[1], lse = m + logf(se);
  const int yy = (int)y[n];
  if (tid == 0) lossn[n] = lse - sZ[yy];
  __syncthreads();  // every thread has read sZ[yy] before it is overwritten below
  const float invB = 1.f / (float)B;
  for (int k = tid; k < K; k += kCHT) {
    const float d = (expf(sZ[k] - m) / se - (k == yy ? 1.f : 0.f)) * invB;
    sZ[k] = d;
    dlog[(int64_t)n * K + k] = d;
  }
  __syncthreads();
  for (int c = 2 * tid; c < C; c += 2 * kCHT) {  // dpool = dlog W, broadcast / HW over the map
    float d0 = 0.f, d1 = 0.f;
    for (int k = 0; k < K; ++k) {
      const float2 w = *reinterpret_cast<const float2*>(W + (int64_t)k * C + c);
      d0 = fmaf(sZ[k], w.x, d0);
      d1 = fmaf(sZ[k], w.y, d1);
    }
    const uint32_t pk = pack_bf16x2(d0 * inv_hw, d1 * inv_hw);
    for (int hw = 0; hw < HW; ++hw) *reinterpret_cast<uint32_t*>(da + ((int64_t)n * HW + hw) * C + c) = pk;
  }
}

// k_cls_head_grad: dW[g][k][c] = sum_b dlog[g B + b][k] pooled[g B + b][c] into the grads rows (one thread per
// (k, c), fixed order over b: deterministic); the extra block column (blockIdx.y == ncol) writes db and the client's
// mean loss.
__global__ __launch_bounds__(kCHT) void k_cls_head_grad(const float* __restrict__ pooled, const float* __restrict__ dlog,
                                                        const float* __restrict__ lossn, int B, int C, int K,
                                                        float* __restrict__ grad, int64_t ldg, int64_t off_w,
                                                        int64_t off_b, float* __restrict__ losses) {
  const int g = blockIdx.x, col = blockIdx.y, tid = threadIdx.x;
  const int ncol = (K * C + kCHT - 1) / kCHT;
  float* gr = grad + (int64_t)g * ldg;
  const float* P = pooled + (int64_t)g * B * C;
  const float* D = dlog + (int64_t)g * B * K;
  if (col < ncol) {
    const int e = col * kCHT + tid;
    if (e >= K * C) return;
    const int k = e / C, c = e - k * C;
    float s = 0.f;
    for (int b = 0; b < B; ++b) s = fmaf(D[(int64_t)b * K + k], P[(int64_t)b * C + c], s);
    gr[off_w + e] = s;
    return;
  }
  for (int k = tid; k < K; k += kCHT) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += D[(int64_t)b * K + k];
    gr[off_b + k] = s;
  }
  if (tid < 64) {
    float l = 0.f;
    for (int b = tid; b < B; b += 64) l += lossn[(int64_t)g * B + b];
    l = wave_sum(l);
    if (tid == 0) losses[g] = l / (float)B;
  }
}

void cls_head_train(uintptr_t a, uintptr_t theta, int64_t ldt, int64_t off_w, int64_t off_b, uintptr_t y, int G, int B,
                    int HW, int C, int K, uintptr_t pooled, uintptr_t dlog, uintptr_t lossn, uintptr_t losses,
                    uintptr_t grad, int64_t ldg, uintptr_t da, uintptr_t stream) {
  NIDT_REQUIRE(C % 2 == 0 && C <= kCHMaxC && K >= 1 && K <= kCHMaxK && B >= 1 && HW >= 1,
               "cls_head_train: C even <= 512, 1 <= K <= 256");
  NIDT_REQUIRE(off_w % 2 == 0 && ldt % 2 == 0, "cls_head_train: 8-B aligned weight rows");
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(k_cls_head_fwd, dim3(G * B), dim3(kCHT), 0, s, ptr<const uint16_t>(a), ptr<const float>(theta), ldt,
                     off_w, off_b, ptr<const int64_t>(y), B, HW, C, K, ptr<float>(pooled), ptr<float>(dlog),
                     ptr<float>(lossn), ptr<uint16_t>(da));
  const int ncol = (K * C + kCHT - 1) / kCHT;
  hipLaunchKernelGGL(k_cls_head_grad, dim3(G, ncol + 1), dim3(kCHT), 0, s, ptr<const float>(pooled),
                     ptr<const float>(dlog), ptr<const float>(lossn), B, C, K, ptr<float>(grad), ldg, off_w, off_b,
                     ptr<float>(losses));
  NIDT_CHECK(hipGetLastError());
}

}  // namespace nidt
