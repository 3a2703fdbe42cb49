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

}  // namespace nidt
