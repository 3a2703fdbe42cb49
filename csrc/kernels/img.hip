// Image input stage of the client-batched 2-D ResNet engine: gather + train-time augmentation + normalisation +
// channel padding in one pass (reference transforms: fedml_api/data_preprocessing/cifar10/data_loader.py:46-52,
// cifar100/data_loader.py:33-39, tiny_imagenet/data_loader.py:51-57 — ToPILImage, RandomCrop(S, padding=4),
// RandomHorizontalFlip, ToTensor, Normalize(mean, std)).
//
// out[n][y][x][c] (bf16, c < 3: (pix / 255 - mean_c) / std_c, 3 <= c < CP: 0) for the uint8 HWC image
// src[idx[n]].  With augmentation, sample n (client cids[n / B], batch position n % B) draws from a counter-based
// hash of (step seed, client id, position): crop offsets oy, ox uniform in [0, 2 pad] and a flip bit, so
//   out(y, x) = padded(y + oy, (flip ? W-1-x : x) + ox),  padded(a, b) = src(a - pad, b - pad) or 0 outside,
// i.e. torchvision's RandomCrop (zero-padded PIL image) followed by RandomHorizontalFlip.  The step seed is read
// from device memory (seed_base + *seed_dev), so a captured hipGraph replays with fresh draws every step, and the
// draw depends only on (run seed, round, epoch, step, client, position): the same on any grouping or sharding.
#include "common.h"

namespace nidt {

// splitmix64 finaliser of (seed, a, b); the torch twin is engine/resnet2d_hip.py:aug_draws
__device__ __forceinline__ uint64_t mix64(uint64_t seed, uint64_t a, uint64_t b) {
  uint64_t z = seed ^ (0x9e3779b97f4a7c15ull * ((a << 32) ^ b));
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

struct ImgArgs {
  const uint8_t* src;   // [Ns][H][W][3]
  const int* idx;       // [N]
  uint16_t* out;        // [N][H][W][CP] bf16
  const int64_t* seed_dev;
  const int* cids;      // [N / B] global client ids
  int64_t seed_base;
  int N, H, W, CP, B, pad, aug;
  float sc[3], sh[3];   // x * sc + sh = (x / 255 - mean) / std
};

// one thread per output pixel; 8-channel (16-B) stores
__global__ __launch_bounds__(256) void k_img_input(ImgArgs a) {
  const int64_t tot = (int64_t)a.N * a.H * a.W;
  const int span = 2 * a.pad + 1;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(e % a.W);
    const int64_t r = e / a.W;
    const int y = (int)(r % a.H);
    const int n = (int)(r / a.H);
    int sy = y, sx = x;
    if (a.aug) {
      const uint64_t h = mix64((uint64_t)(a.seed_base + *a.seed_dev), (uint64_t)(uint32_t)a.cids[n / a.B],
                               (uint64_t)(n % a.B));
      const uint32_t lo = (uint32_t)h, hi = (uint32_t)(h >> 32);
      const int oy = (int)(lo % (uint32_t)span), ox = (int)((lo / (uint32_t)span) % (uint32_t)span);
      const int fx = (hi & 1u) ? (a.W - 1 - x) : x;
      sy = y + oy - a.pad;
      sx = fx + ox - a.pad;
    }
    float v[3] = {0.f, 0.f, 0.f};  // zero padding (pixel value 0, normalised below like any pixel)
    if (sy >= 0 && sy < a.H && sx >= 0 && sx < a.W) {
      const uint8_t* p = a.src + (((int64_t)a.idx[n] * a.H + sy) * a.W + sx) * 3;
      v[0] = (float)p[0];
      v[1] = (float)p[1];
      v[2] = (float)p[2];
    }
    uint4 c0;
    c0.x = pack_bf16x2(fmaf(v[0], a.sc[0], a.sh[0]), fmaf(v[1], a.sc[1], a.sh[1]));
    c0.y = pack_bf16x2(fmaf(v[2], a.sc[2], a.sh[2]), 0.f);
    c0.z = 0u;
    c0.w = 0u;
    uint4* o = reinterpret_cast<uint4*>(a.out + e * a.CP);
    o[0] = c0;
    for (int c = 1; c < a.CP / 8; ++c) o[c] = make_uint4(0u, 0u, 0u, 0u);
  }
}

// [STEM-FOLD] The stem's 3x3 pad-1 window folded into the channels: out[n][y][x][3 t + c] (t = 3 kh + kw) is the
// normalised augmented pixel (y + kh - 1, x + kw - 1) of channel c, 0 outside the image (the conv's zero padding),
// channels 27 .. CP-1 zero.  The 3 -> 64 stem then runs as a 1x1 conv with K = 27 (padded to 64) instead of nine
// 64-channel taps of which 61 channels are zero: 9x fewer MACs in the forward and the weight gradient, the same
// input bytes (the padded image was 64 channels wide too).  Same values, in bf16, as the unfolded input.
__device__ __forceinline__ float img_pixel(const ImgArgs& a, int n, int y, int x, int c, int oy, int ox, bool flip) {
  // augmented (crop + flip) normalised pixel (y, x) of sample n, channel c; y, x inside the image
  int sy = y, sx = x;
  if (a.aug) {
    sy = y + oy - a.pad;
    sx = (flip ? (a.W - 1 - x) : x) + ox - a.pad;
  }
  float v = 0.f;  // RandomCrop's zero padding: pixel value 0, normalised like any pixel
  if (sy >= 0 && sy < a.H && sx >= 0 && sx < a.W) v = (float)a.src[(((int64_t)a.idx[n] * a.H + sy) * a.W + sx) * 3 + c];
  return fmaf(v, a.sc[c], a.sh[c]);
}

__global__ __launch_bounds__(256) void k_img_fold(ImgArgs a) {
  const int64_t tot = (int64_t)a.N * a.H * a.W;
  const int span = 2 * a.pad + 1;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(e % a.W);
    const int64_t r = e / a.W;
    const int y = (int)(r % a.H);
    const int n = (int)(r / a.H);
    int oy = 0, ox = 0;
    bool flip = false;
    if (a.aug) {
      const uint64_t h = mix64((uint64_t)(a.seed_base + *a.seed_dev), (uint64_t)(uint32_t)a.cids[n / a.B],
                               (uint64_t)(n % a.B));
      const uint32_t lo = (uint32_t)h, hi = (uint32_t)(h >> 32);
      oy = (int)(lo % (uint32_t)span);
      ox = (int)((lo / (uint32_t)span) % (uint32_t)span);
      flip = (hi & 1u) != 0u;
    }
    float v[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) v[k] = 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
      if (yy >= 0 && yy < a.H && xx >= 0 && xx < a.W) {
#pragma unroll
        for (int c = 0; c < 3; ++c) v[3 * t + c] = img_pixel(a, n, yy, xx, c, oy, ox, flip);
      }
    }
    uint4* o = reinterpret_cast<uint4*>(a.out + e * a.CP);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      o[q] = make_uint4(pack_bf16x2(v[8 * q], v[8 * q + 1]), pack_bf16x2(v[8 * q + 2], v[8 * q + 3]),
                        pack_bf16x2(v[8 * q + 4], v[8 * q + 5]), pack_bf16x2(v[8 * q + 6], v[8 * q + 7]));
    for (int q = 4; q < a.CP / 8; ++q) o[q] = make_uint4(0u, 0u, 0u, 0u);
  }
}

static ImgArgs img_args(uintptr_t src, uintptr_t idx, uintptr_t out, int N, int H, int W, int CP, float m0, float m1,
                        float m2, float s0, float s1, float s2, int aug, int pad, uintptr_t seed_dev,
                        int64_t seed_base, uintptr_t cids, int B) {
  ImgArgs a;
  a.src = ptr<const uint8_t>(src); a.idx = ptr<const int>(idx); a.out = ptr<uint16_t>(out);
  a.seed_dev = ptr<const int64_t>(seed_dev); a.cids = ptr<const int>(cids); a.seed_base = seed_base;
  a.N = N; a.H = H; a.W = W; a.CP = CP; a.B = B > 0 ? B : 1; a.pad = pad; a.aug = aug;
  const float mean[3] = {m0, m1, m2}, sd[3] = {s0, s1, s2};
  for (int c = 0; c < 3; ++c) {
    a.sc[c] = 1.f / (255.f * sd[c]);
    a.sh[c] = -mean[c] / sd[c];
  }
  return a;
}

void img_input_fold(uintptr_t src, uintptr_t idx, uintptr_t out, int N, int H, int W, int CP, float m0, float m1,
                    float m2, float s0, float s1, float s2, int aug, int pad, uintptr_t seed_dev, int64_t seed_base,
                    uintptr_t cids, int B, uintptr_t stream) {
  NIDT_REQUIRE(CP % 8 == 0 && CP >= 32, "img_input_fold: CP must be a multiple of 8 and >= 32 (27 folded channels)");
  NIDT_REQUIRE(!aug || (seed_dev && cids && B > 0 && N % B == 0 && pad >= 0), "img_input_fold: augmentation needs "
               "the step seed, the client ids and N % B == 0");
  const ImgArgs a = img_args(src, idx, out, N, H, W, CP, m0, m1, m2, s0, s1, s2, aug, pad, seed_dev, seed_base, cids, B);
  const int64_t tot = (int64_t)N * H * W;
  hipLaunchKernelGGL(k_img_fold, dim3((unsigned)std::min<int64_t>(16384, (tot + 255) / 256)), dim3(256), 0,
                     as_stream(stream), a);
  NIDT_CHECK(hipGetLastError());
}

void img_input(uintptr_t src, uintptr_t idx, uintptr_t out, int N, int H, int W, int CP, float m0, float m1, float m2,
               float s0, float s1, float s2, int aug, int pad, uintptr_t seed_dev, int64_t seed_base, uintptr_t cids,
               int B, uintptr_t stream) {
  NIDT_REQUIRE(CP % 8 == 0 && CP >= 8, "img_input: padded channels CP must be a multiple of 8");
  NIDT_REQUIRE(!aug || (seed_dev && cids && B > 0 && N % B == 0 && pad >= 0), "img_input: augmentation needs "
               "the step seed, the client ids and N % B == 0");
  ImgArgs a;
  a.src = ptr<const uint8_t>(src); a.idx = ptr<const int>(idx); a.out = ptr<uint16_t>(out);
  a.seed_dev = ptr<const int64_t>(seed_dev); a.cids = ptr<const int>(cids); a.seed_base = seed_base;
  a.N = N; a.H = H; a.W = W; a.CP = CP; a.B = B > 0 ? B : 1; a.pad = pad; a.aug = aug;
  const float mean[3] = {m0, m1, m2}, sd[3] = {s0, s1, s2};
  for (int c = 0; c < 3; ++c) {
    a.sc[c] = 1.f / (255.f * sd[c]);
    a.sh[c] = -mean[c] / sd[c];
  }
  const int64_t tot = (int64_t)N * H * W;
  hipLaunchKernelGGL(k_img_input, dim3((unsigned)std::min<int64_t>(16384, (tot + 255) / 256)), dim3(256), 0,
                     as_stream(stream), a);
  NIDT_CHECK(hipGetLastError());
}

}  // namespace nidt
