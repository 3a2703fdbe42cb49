// AlexNet3D conv1 (Conv3d(1, 64, k=5, s=2) + BatchNorm3d + ReLU + MaxPool3d(3,3)), salient_models.py:146-150,
// the layer that carries 53 % of the model's FLOPs at 1x121x145x121.
//
// Design (MI355X-first, not a translation of cuDNN's path):
//  * Input volumes live in HBM as uint8 in a *polyphase* layout [N][61][73][61][8]: voxel (d,h,w) is stored at
//    (d>>1, h>>1, w>>1) phase ((d&1)<<2 | (h&1)<<1 | (w&1)).  The stride-2 5^3 conv becomes a stride-1 3^3 conv
//    over 8 "phase channels": every MFMA B fragment (8 consecutive k = the 8 phases of one tap) is one 16-B
//    contiguous read.  K = 27 taps x 8 phases = 216 (125 live), padded to 224 = 7 k-steps of 32.
//    uint8 values are exact in bf16, so B = u8 and A = bf16(w/255): conv == sum w * (u8/255).
//  * BatchNorm batch statistics need no pass over the 253 M-element conv output: with per-sample patch moments
//    m1 = sum_pos p, m2 = sum_pos p p^T (computed once when the data is loaded; exact int-valued fp64),
//    mean_c = w_c.mu + b_c and var_c = w_c^T Cov w_c.  The forward kernel therefore fuses conv + BN + ReLU +
//    max-pool and writes only the pooled bf16 output and a uint8 argmax (the conv1 activation never exists).
//  * Backward needs no dense activation either: with dz only non-zero at the argmax voxels,
//      S_c = sum dz p (sparse gather, k_conv1_wgrad), D_c = sum dz,
//      dgamma = invstd w.(S - D mu),  dbeta = D,
//      dw = gamma invstd (S - D mu - dgamma invstd Cov w),  db = 0
//    which is exactly the gradient autograd computes through conv -> BN(train) -> ReLU -> pool.
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "conv1_wgrad_layout.h"
#include "conv1_mx_layout.h"

namespace nidt {

constexpr int kPZ = 61, kPY = 73, kPX = 61;          // polyphase grid of a 121x145x121 volume
constexpr int kOD = 59, kOH = 71, kOW = 59;          // conv1 output
constexpr int kPD = 19, kPH = 23, kPW = 19;          // pooled output
constexpr int kC1 = 64;
constexpr int kK1 = 224;                              // padded k (27 taps x 8 phases = 216)
constexpr int kNM = 125 + 125 * 125;                  // per-sample moment vector length

// phase r = (rd<<2)|(rh<<1)|rw ; tap t = jd*9+jh*3+jw ; original k = kd*25+kh*5+kw with kd = 2 jd + rd
__host__ __device__ constexpr bool tp_valid(int t, int r) {
  const int jd = t / 9, jh = (t / 3) % 3, jw = t % 3;
  return (2 * jd + (r >> 2) < 5) && (2 * jh + ((r >> 1) & 1) < 5) && (2 * jw + (r & 1) < 5);
}
__host__ __device__ constexpr int tp_to_k(int t, int r) {
  const int jd = t / 9, jh = (t / 3) % 3, jw = t % 3;
  return (2 * jd + (r >> 2)) * 25 + (2 * jh + ((r >> 1) & 1)) * 5 + (2 * jw + (r & 1));
}

// ------------------------------------------------------------------------------------------------
// polyphase conversion of uint8 volumes [N][121][145][121] -> [N][61][73][61][8]
__global__ void k_polyphase(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int64_t N) {
  const int64_t tot = N * kPZ * kPY * kPX;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    int64_t v = e;
    const int x = (int)(v % kPX); v /= kPX;
    const int y = (int)(v % kPY); v /= kPY;
    const int z = (int)(v % kPZ);
    const int64_t n = v / kPZ;
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int d = 2 * z + (r >> 2), h = 2 * y + ((r >> 1) & 1), w = 2 * x + (r & 1);
      uint32_t b = 0;
      if (d < 121 && h < 145 && w < 121) b = src[((n * 121 + d) * 145 + h) * 121 + w];
      if (r < 4) lo |= b << (8 * r); else hi |= b << (8 * (r - 4));
    }
    *reinterpret_cast<uint2*>(dst + e * 8) = make_uint2(lo, hi);
  }
}

void polyphase(uintptr_t src, uintptr_t dst, int64_t N, uintptr_t stream) {
  const int64_t tot = N * kPZ * kPY * kPX;
  hipLaunchKernelGGL(k_polyphase, dim3((unsigned)std::min<int64_t>(65536, (tot + 255) / 256)), dim3(256), 0,
                     as_stream(stream), ptr<const uint8_t>(src), ptr<uint8_t>(dst), N);
  NIDT_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// per-sample patch moments, exact (integer products summed in fp32 chunks of <= 256 positions, then fp64)
// grid (N, 59 od); block 256: thread owns an 8x8 block of the (padded 128x128) second-moment matrix.
__global__ __launch_bounds__(256) void k_conv1_moments_sample(const uint8_t* __restrict__ x8, double* __restrict__ mom) {
  __shared__ float P[64][129];
  const int n = blockIdx.x, od = blockIdx.y, tid = threadIdx.x;
  const int kb1 = tid >> 4, kb2 = tid & 15;
  const bool active = kb1 <= kb2;  // symmetric: compute upper block triangle only
  float acc[8][8];
  double accd[8][8];
  float s1 = 0.f;
  double s1d = 0.0;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) { acc[i][j] = 0.f; accd[i][j] = 0.0; }
  const uint8_t* xs = x8 + (int64_t)n * kPZ * kPY * kPX * 8;
  const int npos = kOH * kOW;
  int since = 0;
  for (int p0 = 0; p0 < npos; p0 += 64) {
    __syncthreads();
    for (int e = tid; e < 64 * 128; e += 256) {
      const int pl = e >> 7, k = e & 127;
      const int pos = p0 + pl;
      float v = 0.f;
      if (pos < npos && k < 125) {
        const int oh = pos / kOW, ow = pos - oh * kOW;
        const int kd = k / 25, kh = (k / 5) % 5, kw = k % 5;
        const int z = od + (kd >> 1), y = oh + (kh >> 1), xx = ow + (kw >> 1);
        const int r = ((kd & 1) << 2) | ((kh & 1) << 1) | (kw & 1);
        v = (float)xs[(((int64_t)z * kPY + y) * kPX + xx) * 8 + r];
      }
      P[pl][k] = v;
    }
    __syncthreads();
    if (active) {
      for (int pl = 0; pl < 64; ++pl) {
        float a[8], b[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) { a[i] = P[pl][8 * kb1 + i]; b[i] = P[pl][8 * kb2 + i]; }
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[i][j] = fmaf(a[i], b[j], acc[i][j]);
      }
    }
    if (tid < 128) for (int pl = 0; pl < 64; ++pl) s1 += P[pl][tid];
    since += 64;
    if (since >= 256 || p0 + 64 >= npos) {  // flush (each fp32 partial <= 256*255*255 < 2^24: exact)
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) { accd[i][j] += (double)acc[i][j]; acc[i][j] = 0.f; }
      s1d += (double)s1;
      s1 = 0.f;
      since = 0;
    }
  }
  double* m = mom + (int64_t)n * kNM;
  if (tid < 125) atomicAdd(m + tid, s1d);
  if (active) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k1 = 8 * kb1 + i, k2 = 8 * kb2 + j;
        if (k1 < 125 && k2 < 125) {
          atomicAdd(m + 125 + k1 * 125 + k2, accd[i][j]);
          if (kb1 != kb2) atomicAdd(m + 125 + k2 * 125 + k1, accd[i][j]);
        }
      }
  }
}

void conv1_sample_moments(uintptr_t x8, int64_t N, uintptr_t mom, uintptr_t stream) {
  NIDT_CHECK(hipMemsetAsync(ptr<void>(mom), 0, (size_t)N * kNM * sizeof(double), as_stream(stream)));
  hipLaunchKernelGGL(k_conv1_moments_sample, dim3((unsigned)N, kOD), dim3(256), 0, as_stream(stream),
                     ptr<const uint8_t>(x8), ptr<double>(mom));
  NIDT_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// 128-slot K packing of the forward (4 MFMA k-steps instead of 7).  The 27 polyphase tap groups t = 9 jd + 3 jh +
// jw carry 8 valid phases when every j < 2 (8 groups "F"), 4 when one j = 2 (D: jd, H: jh, W: jw; 4 groups each),
// 2 when two are (DH, DW, HW; 2 each) and 1 for jd = jh = jw = 2 — 125 taps.  Each lane group fq of a k-step holds
// 8 consecutive k: k-steps 0-1 = the 8 F groups (one 16-B halo read each); k-step 2 = D[fq] (phases 0-3: the first
// 8 bytes) + H[fq] (phases 0,1,4,5: dwords 0 and 2); k-step 3 = W[fq] (phases 0,2,4,6: the low halves of the 4
// dwords, two v_perm) + two 2-phase groups (or DHW) picked by one v_cndmask + v_perm each.  Only 3 of 128 slots are
// empty (vs 99 of 224 in the 27 x 8 layout).
// [RO]: RO = 1 orders the groups of k-steps 0-2 so that the two lane quarters of each ds_read_b128 lane group (fq 0
// with 1, fq 2 with 3) read tap groups of the same jw (their halo offsets then differ by whole 1-KB (dd, dh) rows:
// the same banks for the same column, no conflict); RO = 0 is the original order and the
// default (RO = 1 measured slower, NIDT_C1_TAPORD=1 for A/B)
__device__ constexpr int kC1F2[2][8] = {{0, 1, 3, 4, 9, 10, 12, 13}, {0, 3, 1, 4, 9, 12, 10, 13}};
__device__ constexpr int kC1D2[2][4] = {{18, 19, 21, 22}, {18, 21, 19, 22}};
__device__ constexpr int kC1H2[2][4] = {{6, 7, 15, 16}, {6, 15, 7, 16}};
__device__ constexpr int kC1W[4] = {2, 5, 11, 14};
__device__ constexpr int kC1X1[4] = {24, 20, 8, 26};   // DH0, DW0, HW0, DHW
__device__ constexpr int kC1X2[4] = {25, 23, 17, 26};  // DH1, DW1, HW1, (empty)
__device__ constexpr int kC1XR[4][2] = {{0, 1}, {0, 2}, {0, 4}, {0, -1}};
// RO = 2 (opt-in, NIDT_C1_TAPORD=2): every B operand is one conflict-free ds_read_b128.  A ds_read_b128 is served in 16-lane
// groups {fq0 fr0-3,12-15 + fq1 fr4-11} (and the fq2/fq3 mirror): when the two lane quarters of a group read tap
// groups of the same jw, their 16 lanes touch 16 distinct 16-B slots of the 256-B bank row.  k-steps 0-2 take the
// RO = 1 order (paired jw); k-step 3 holds W[fq] (phases 0,2,4,6) + X1[fq] (phases 0,2: DW0, DW1, DHW, empty) +
// X2[fq] (phases 0,1 for DH0/DH1, 0,4 for HW0/HW1).  Only X2 of the fq0/fq1 quarters (DH0: jw 0 vs DH1: jw 1) is
// 2-way.  The narrow reads of RO = 0/1 (ds_read_b64 / b32 at a 16-B lane stride: 2- and 4-way) were the kernel's
// 45.7 % LDS bank conflicts (profiles/r5_c1fwd_w64_pmc.txt).
__device__ constexpr int kC1X1b[4] = {20, 23, 26, -1};  // DW0, DW1, DHW, empty
__device__ constexpr int kC1X2b[4] = {24, 25, 8, 17};   // DH0, DH1, HW0, HW1

// (tap group, phase) of slot kk of the 128-slot layout, or t = -1 for an empty slot
template <int RO>
__device__ __forceinline__ void c1_slot128(int kk, int& t, int& r) {
  constexpr int R1 = RO ? 1 : 0;
  const int st = kk >> 5, fq = (kk >> 3) & 3, e = kk & 7;
  t = -1;
  r = 0;
  if (st < 2) { t = kC1F2[R1][4 * st + fq]; r = e; return; }
  if (st == 2) {
    if (e < 4) { t = kC1D2[R1][fq]; r = e; }
    else { t = kC1H2[R1][fq]; r = (e - 4 < 2) ? e - 4 : e - 4 + 2; }
    return;
  }
  if (e < 4) { t = kC1W[fq]; r = 2 * e; return; }
  if (RO == 2) {
    if (e < 6) { t = kC1X1b[fq]; r = e == 4 ? 0 : 2; }  // DHW's phase 2 is invalid: tp_valid zeroes its weight
    else { t = kC1X2b[fq]; r = e == 6 ? 0 : (fq < 2 ? 1 : 4); }
    return;
  }
  const int x = (e - 4) >> 1, h = e & 1;
  if (x == 1 && fq == 3) return;
  const int rr = kC1XR[fq][h];
  if (rr < 0) return;
  t = x == 0 ? kC1X1[fq] : kC1X2[fq];
  r = rr;
}

// weight packing: theta row g at off: [64][125] fp32 -> w8 [G][64][KS] f16 bits of f16(w) (the forward's MFMA
// A operand, against raw uint8 voxels; KS = 128 slots, or 224 = 27 x 8 for the legacy layout), w125 [G][64][125]
// f32 = f16(w) * scale (scale = 1/255): the exact effective weights of conv(x / 255) that the moment math (BN
// statistics) and the closed-form backward use.
template <int RO>
__global__ void k_pack_conv1_w(const float* __restrict__ theta, int64_t ldt, int64_t off, int64_t off_sign, int G,
                               float scale, int KS, uint16_t* __restrict__ w8, float* __restrict__ w125) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= G * kC1 * KS) return;
  const int g = i / (kC1 * KS), rem = i - g * kC1 * KS, c = rem / KS, kk = rem - c * KS;
  int t, r;
  if (KS == 128) {
    c1_slot128<RO>(kk, t, r);
  } else {
    t = kk >> 3;
    r = kk & 7;
  }
  uint16_t v = 0;
  if (t >= 0 && t < 27 && tp_valid(t, r)) {
    const int k = tp_to_k(t, r);
    const _Float16 h = (_Float16)theta[(int64_t)g * ldt + off + c * 125 + k];
    v = __builtin_bit_cast(uint16_t, h);
    w125[((int64_t)g * kC1 + c) * 125 + k] = (float)h * scale;
    // the fused forward expects sign(gamma_c) folded into its MFMA weights (exact sign flip)
    if (off_sign >= 0 && theta[(int64_t)g * ldt + off_sign + c] < 0.f) v ^= 0x8000u;
  }
  w8[i] = v;
}

// K slots of the forward's packed weights: 128 (default) or the legacy 27 x 8 = 224 (NIDT_C1_K224=1, A/B)
// tap-group order of the 128-slot forward layout (pack and forward must agree): the original order by default;
// NIDT_C1_TAPORD=1 selects the bank-paired order (slower at 64 clients: conv1 forward 4.38 vs 4.25 ms,
// profiles/r4_kbench_g64.txt)
// NIDT_C1_TAPORD=2 (A/B, the w64 forward only): the all-b128 layout [RO = 2]: LDS bank conflicts 45.7 % -> 0.0 %
// with the forward's time unchanged (3.28 ms per 64-client step either way, profiles/r6_conv1_b128.txt) — the
// conflicts are not what the kernel waits on.  Its fp32 sums differ from RO = 0 by rounding (another k order), which
// flips near-tie max-pool / ReLU decisions downstream; RO = 0 stays the default.  The pipe kernel knows RO 0 / 1.
int conv1_kslots();
int conv1_fwd_variant();
int conv1_tapord() {
  static const int env = [] {
    const char* e = getenv("NIDT_C1_TAPORD");
    return e ? atoi(e) : 0;
  }();
  if (conv1_fwd_variant() == 1 && conv1_kslots() == 128) return env >= 0 && env <= 2 ? env : 0;
  return env == 1 ? 1 : 0;
}

int conv1_kslots() {
  static const int ks = [] {
    const char* e = getenv("NIDT_C1_K224");
    return (e && atoi(e) == 1) ? kK1 : 128;
  }();
  return ks;
}

void pack_conv1_w(uintptr_t theta, int64_t ldt, int64_t off, int64_t off_sign, int G, float scale, uintptr_t w8,
                  uintptr_t w125, uintptr_t stream) {
  const int KS = conv1_kslots();
  // w125 entries of empty taps are never read; every valid (t, r) appears in exactly one slot of either layout
  const int ro = conv1_tapord();
  if (ro == 2)
    hipLaunchKernelGGL(k_pack_conv1_w<2>, dim3(ceil_div(G * kC1 * KS, 256)), dim3(256), 0, as_stream(stream),
                       ptr<const float>(theta), ldt, off, off_sign, G, scale, KS, ptr<uint16_t>(w8), ptr<float>(w125));
  else if (ro == 1)
    hipLaunchKernelGGL(k_pack_conv1_w<1>, dim3(ceil_div(G * kC1 * KS, 256)), dim3(256), 0, as_stream(stream),
                       ptr<const float>(theta), ldt, off, off_sign, G, scale, KS, ptr<uint16_t>(w8), ptr<float>(w125));
  else
    hipLaunchKernelGGL(k_pack_conv1_w<0>, dim3(ceil_div(G * kC1 * KS, 256)), dim3(256), 0, as_stream(stream),
                       ptr<const float>(theta), ldt, off, off_sign, G, scale, KS, ptr<uint16_t>(w8), ptr<float>(w125));
  NIDT_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// batch moments: Mb[g][e] = sum_b mom[idx[g*B+b]][e]
__global__ void k_conv1_batch_moments(const double* __restrict__ mom, const int* __restrict__ idx, int B, int G,
                                      double* __restrict__ Mb) {
  const int g = blockIdx.y;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= kNM) return;
  double s = 0;
  for (int b = 0; b < B; ++b) s += mom[(int64_t)idx[g * B + b] * kNM + e];
  Mb[(int64_t)g * kNM + e] = s;
}

// BN1 statistics per (g, c) from the batch moments.  block = 128 threads (k1), grid (64, G).
// Outputs: scale/shift for conv-without-bias; mean (incl. bias) & invstd; covw[g][c][k] = (Cov w)_k; running stats.
// Block = (group of kBnCPB channels, client): the 125x125 patch covariance row k1 is formed once per thread and
// applied to the block's channel filters (one block per channel re-reads the client's 125 KB moment matrix 64
// times; 8 channels per block when there are >= 32 clients, else 1 to keep the grid wide).  Per channel the
// arithmetic and reduction order are the same either way.
template <int kBnCPB>
__global__ __launch_bounds__(128) void k_conv1_bnstats(const double* __restrict__ Mb, const float* __restrict__ w125,
                                                       const float* __restrict__ theta, int64_t ldt, int64_t off_bias,
                                                       int64_t off_g, int64_t off_b, float* bufs, int64_t ldb,
                                                       int64_t off_rm, int64_t off_rv, int64_t off_nbt, double Npos,
                                                       float momentum, float eps, int update_running, float* scale,
                                                       float* shift, float* mean_o, float* invstd_o, float* mu_o,
                                                       float* covw_o) {
  __shared__ double sw[kBnCPB][128], smu[128], red[kBnCPB][2][2];
  const int c0 = blockIdx.x * kBnCPB, g = blockIdx.y, k1 = threadIdx.x;
  const double* M = Mb + (int64_t)g * kNM;
  smu[k1] = k1 < 125 ? M[k1] / Npos : 0.0;
#pragma unroll
  for (int cc = 0; cc < kBnCPB; ++cc) sw[cc][k1] = k1 < 125 ? (double)w125[((int64_t)g * kC1 + c0 + cc) * 125 + k1] : 0.0;
  __syncthreads();
  double t[kBnCPB];
#pragma unroll
  for (int cc = 0; cc < kBnCPB; ++cc) t[cc] = 0;
  if (k1 < 125) {
    for (int k2 = 0; k2 < 125; ++k2) {
      const double cov = M[125 + k1 * 125 + k2] / Npos - smu[k1] * smu[k2];
#pragma unroll
      for (int cc = 0; cc < kBnCPB; ++cc) t[cc] += cov * sw[cc][k2];
    }
#pragma unroll
    for (int cc = 0; cc < kBnCPB; ++cc) covw_o[((int64_t)g * kC1 + c0 + cc) * 125 + k1] = (float)t[cc];
    if (c0 == 0) mu_o[(int64_t)g * 125 + k1] = (float)smu[k1];
  }
#pragma unroll
  for (int cc = 0; cc < kBnCPB; ++cc) {
    double v = sw[cc][k1] * t[cc], m = sw[cc][k1] * smu[k1];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { v += __shfl_xor(v, o, 64); m += __shfl_xor(m, o, 64); }
    if ((k1 & 63) == 0) { red[cc][0][k1 >> 6] = v; red[cc][1][k1 >> 6] = m; }
  }
  __syncthreads();
  if (k1 < kBnCPB) {
    const int c = c0 + k1;
    const double var = red[k1][0][0] + red[k1][0][1];
    const double mnb = red[k1][1][0] + red[k1][1][1];  // mean of the conv output without bias
    const float bias = theta[(int64_t)g * ldt + off_bias + c];
    const float gm = theta[(int64_t)g * ldt + off_g + c], bt = theta[(int64_t)g * ldt + off_b + c];
    const double vv = var > 0 ? var : 0.0;
    const float inv = (float)(1.0 / sqrt(vv + (double)eps));
    const int i = g * kC1 + c;
    scale[i] = gm * inv;
    shift[i] = bt - (float)mnb * gm * inv;
    mean_o[i] = (float)(mnb + bias);
    invstd_o[i] = inv;
    if (update_running) {
      float* rm = bufs + (int64_t)g * ldb + off_rm + c;
      float* rv = bufs + (int64_t)g * ldb + off_rv + c;
      *rm = (1.f - momentum) * *rm + momentum * (float)(mnb + bias);
      *rv = (1.f - momentum) * *rv + momentum * (float)(vv * Npos / (Npos - 1.0));
      if (c == 0) bufs[(int64_t)g * ldb + off_nbt] += 1.f;
    }
  }
}

void conv1_bnstats(uintptr_t mom, uintptr_t idx, int B, int G, uintptr_t Mb, uintptr_t w125, uintptr_t theta,
                   int64_t ldt, int64_t off_bias, int64_t off_g, int64_t off_b, uintptr_t bufs, int64_t ldb,
                   int64_t off_rm, int64_t off_rv, int64_t off_nbt, float momentum, float eps, int update_running,
                   uintptr_t scale, uintptr_t shift, uintptr_t mean, uintptr_t invstd, uintptr_t mu, uintptr_t covw,
                   uintptr_t stream) {
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(k_conv1_batch_moments, dim3(ceil_div(kNM, 256), G), dim3(256), 0, s, ptr<const double>(mom),
                     ptr<const int>(idx), B, G, ptr<double>(Mb));
  NIDT_CHECK(hipGetLastError());
  const double Npos = (double)B * kOD * kOH * kOW;
#define NIDT_BNSTATS(CPB)                                                                                      \
  hipLaunchKernelGGL(k_conv1_bnstats<CPB>, dim3(kC1 / CPB, G), dim3(128), 0, s, ptr<const double>(Mb),           \
                     ptr<const float>(w125), ptr<const float>(theta), ldt, off_bias, off_g, off_b, ptr<float>(bufs), \
                     ldb, off_rm, off_rv, off_nbt, Npos, momentum, eps, update_running, ptr<float>(scale),          \
                     ptr<float>(shift), ptr<float>(mean), ptr<float>(invstd), ptr<float>(mu), ptr<float>(covw))
  if (G >= 32) NIDT_BNSTATS(8);
  else NIDT_BNSTATS(1);
#undef NIDT_BNSTATS
  NIDT_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// Fused forward: conv1 (MFMA) -> z = conv*scale + shift -> max over 3x3x3 -> relu, k_conv1_fwd_pool_pipe.
// One block (4 waves) walks all 23 pooled rows (ph) of a (sample, pd) slab; wave w owns 32 output channels
// (ch = w & 1) x 2 column groups of 15 conv columns (op = w >> 1); the next row's 5x5x64 polyphase halo is
// prefetched into registers while the MFMAs of the current row run, then written into the other LDS buffer.
// 1-D grid, XCD-remapped so the 19 pd-slabs of a sample (overlapping by 2 z-planes) share an L2.
//
// The kernel is VALU-issue bound, not MFMA bound (rocprofv3 PMC, profiles/r1_pmc_v4.txt: 1330 VALU vs 252
// MFMA per wave-row), so every per-voxel and per-output VALU op counts:
//  * operands are f16, not bf16.  A uint8 voxel becomes the f16 magic number 1024 + x with ONE v_perm per two
//    voxels (exponent byte 0x64 spliced next to each data byte) instead of 8 cvt + 4 perm per 8 voxels; the
//    weights are f16(w) (11-bit mantissa, more precise than bf16).  The +1024 offset is cancelled exactly by
//    starting every accumulator at -1024 * sum_k A[c][k] (A = the packed, sign-folded row of channel c), so
//    acc = sum_k A x = 255 * conv(x/255) with no cancellation in the final value;
//  * the 3^3 window's argmax index (dd*9 + dh*3 + dw, dw = this lane's column in the window) rides in the 5
//    low mantissa bits of each candidate: one v_and_or_b32 + one v_max (v_max3 across two dh rows);
//  * the cross-lane (dw) part of the pool is two DPP row shifts + one v_max3 on the tagged values; the bf16
//    output is one v_cvt_pk_bf16_f32 per two channels.
__device__ __forceinline__ uint4 u8x8_to_f16magic(uint2 v) {
  const uint32_t e = 0x64646464u;  // f16 0x64xx = 1024 + xx
  uint4 o;
  o.x = __builtin_amdgcn_perm(e, v.x, 0x04010400u);
  o.y = __builtin_amdgcn_perm(e, v.x, 0x04030402u);
  o.z = __builtin_amdgcn_perm(e, v.y, 0x04010400u);
  o.w = __builtin_amdgcn_perm(e, v.y, 0x04030402u);
  return o;
}

__device__ __forceinline__ float tag_idx(float acc, uint32_t tag) {
  return __uint_as_float((__float_as_uint(acc) & ~31u) | tag);
}

// plain v_max_f32 / v_max3_f32: fmaxf would first "canonicalise" each bit-built operand with an extra
// v_max(x, x) (IEEE NaN quieting) — one wasted VALU op per candidate in this VALU-bound loop
__device__ __forceinline__ float vmax2(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ float vmax3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}


typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

// B fragment of k-step s (of KS per (dd, dh) row) for one output column: the lane's 8 consecutive k of the packed
// layout read from the f16 halo at row offset ro.  KS = 7: tap group 4 s + fq, one 16-B read.  KS = 4: the
// 128-slot layout of c1_slot128 (ga/gh/gx1/gx2: the lane's group offsets; xsrc2: lane picks dword 2 instead of 1
// of its 2-phase groups; xsel1/xsel2: v_perm selectors of those groups).
template <int KS>
__device__ __forceinline__ f16x8 c1_bfrag(const uint16_t* hb, int s, int ro, const int* ga, int gh, int gx1, int gx2,
                                          bool xsrc2, uint32_t xsel1, uint32_t xsel2) {
  if (KS == 7 || s < 2) return *reinterpret_cast<const f16x8*>(&hb[ro + ga[s]]);
  if (s == 2) {
    const uint2 d = *reinterpret_cast<const uint2*>(&hb[ro + ga[2]]);  // D: phases 0-3
    const uint32_t h0 = *reinterpret_cast<const uint32_t*>(&hb[ro + gh]);      // H: phases 0,1
    const uint32_t h2 = *reinterpret_cast<const uint32_t*>(&hb[ro + gh + 4]);  // H: phases 4,5
    const uint4 v = make_uint4(d.x, d.y, h0, h2);
    return __builtin_bit_cast(f16x8, v);
  }
  const uint4 w = *reinterpret_cast<const uint4*>(&hb[ro + ga[3]]);
  const uint4 a = *reinterpret_cast<const uint4*>(&hb[ro + gx1]);
  const uint4 b = *reinterpret_cast<const uint4*>(&hb[ro + gx2]);
  uint4 v;
  v.x = __builtin_amdgcn_perm(w.y, w.x, 0x05040100u);  // phases 0, 2 (low halves)
  v.y = __builtin_amdgcn_perm(w.w, w.z, 0x05040100u);  // phases 4, 6
  v.z = __builtin_amdgcn_perm(xsrc2 ? a.z : a.y, a.x, xsel1);
  v.w = __builtin_amdgcn_perm(xsrc2 ? b.z : b.y, b.x, xsel2);
  return __builtin_bit_cast(f16x8, v);
}

// PF: B-fragment prefetch distance in k-steps; KS: k-steps per (dd, dh) row (7 or 4); OCC: blocks per CU the
// register budget is cut for (2: 256 VGPRs; 3: 168, with spills — A/B NIDT_C1_OCC)
template <int PF, int KS, int OCC = 2, int DDU = 1, int RO = 1>
__global__ __launch_bounds__(256, OCC) void k_conv1_fwd_pool_pipe(const uint8_t* __restrict__ x8,
                                                                const int* __restrict__ idx,
                                                                const uint16_t* __restrict__ w8,
                                                                const float* __restrict__ scale,
                                                                const float* __restrict__ shift, int B,
                                                                uint16_t* __restrict__ out, uint8_t* __restrict__ amax,
                                                                int nq) {
  constexpr int HX = 64;
  constexpr int HALO = 5 * 5 * HX * 8;  // f16 elements per buffer
  constexpr int NLD = (5 * 5 * HX + 255) / 256;  // 7 halo voxels per thread
  __shared__ __attribute__((aligned(16))) uint16_t halo[2 * HALO];
  // block = (sample n, pd slab, row range q of nq): few clients per GPU split the 23 pooled rows of a slab over
  // nq blocks (more, shorter blocks: a wider grid and a shorter tail of the last wave)
  const int bid0 = xcd_remap(blockIdx.x, gridDim.x);
  const int q = bid0 % nq, bid = bid0 / nq;
  const int pd = bid % kPD, n = bid / kPD;
  const int ph_lo = (kPH * q) / nq, ph_hi = (kPH * (q + 1)) / nq;
  const int g = n / B;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const uint8_t* xs = x8 + (int64_t)idx[n] * kPZ * kPY * kPX * 8;
  uint2 pre[NLD];
#define C1_LOAD(PH)                                                                                           \
  _Pragma("unroll") for (int u_ = 0; u_ < NLD; ++u_) {                                                        \
    const int e_ = tid + 256 * u_;                                                                            \
    const int xh_ = e_ & (HX - 1), yz_ = e_ >> 6, yh_ = yz_ % 5, zh_ = yz_ / 5;                                \
    pre[u_] = make_uint2(0, 0);                                                                               \
    if (e_ < 5 * 5 * HX && xh_ < kPX)                                                                         \
      pre[u_] = *reinterpret_cast<const uint2*>(xs + (((int64_t)(3 * pd + zh_) * kPY + 3 * (PH) + yh_) * kPX + xh_) * 8); \
  }
#define C1_STORE(BUF)                                                                                         \
  _Pragma("unroll") for (int u_ = 0; u_ < NLD; ++u_) {                                                        \
    const int e_ = tid + 256 * u_;                                                                            \
    if (e_ < 5 * 5 * HX) *reinterpret_cast<uint4*>(&halo[(BUF) * HALO + e_ * 8]) = u8x8_to_f16magic(pre[u_]); \
  }
  C1_LOAD(ph_lo)
  const int fr = lane & 15, fq = lane >> 4;
  const int ch = wid & 1, op = wid >> 1;
  constexpr int KW = KS * 32;  // packed slots per channel row
  f16x8 fa[2][KS];
  const uint16_t* wg = w8 + (int64_t)g * kC1 * KW;
  float rs[2] = {0.f, 0.f};  // partial row sums of A (row 32ch + 16i + fr, this lane's k chunks)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      fa[i][s] = *reinterpret_cast<const f16x8*>(wg + (32 * ch + 16 * i + fr) * KW + 32 * s + 8 * fq);
#pragma unroll
      for (int e = 0; e < 8; ++e) rs[i] += (float)fa[i][s][e];
    }
  // full row sums (the 4 fq lanes of a row hold disjoint k chunks), then fetch the sums of the C rows this
  // lane accumulates (rows 4fq + r of each 16-row tile) -> accumulator start values -1024 * sum A
  f32x4 cinit[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    rs[i] += __shfl_xor(rs[i], 16, 64);
    rs[i] += __shfl_xor(rs[i], 32, 64);
#pragma unroll
    for (int r = 0; r < 4; ++r) cinit[i][r] = -1024.f * __shfl(rs[i], 4 * fq + r, 64);
  }
  // w8 carries sign(gamma) = sign(sc) per output channel (k_pack_conv1_w, exact), so the argmax of
  // z = sc*acc + sh is the argmax of the accumulator and the pooled value is |sc| * max + sh.  acc is
  // 255 x the conv of x/255 (f16(w) weights against raw uint8), hence |sc| / 255.
  float sc[2][4], sh[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      sc[i][r] = fabsf(scale[g * kC1 + 32 * ch + 16 * i + 4 * fq + r]) * (1.0f / 255.0f);
      sh[i][r] = shift[g * kC1 + 32 * ch + 16 * i + 4 * fq + r];
    }
  // Retire the one-time loads here: an empty asm that "redefines" each register makes the waitcnt pass see
  // them complete before the row loop, so it does not insert vmcnt waits on the halo prefetch inside the
  // MFMA loop (which would serialise the prefetch with the matrix work).
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int s = 0; s < KS; ++s) asm volatile("" : "+v"(fa[i][s]));
#pragma unroll
    for (int r = 0; r < 4; ++r) asm volatile("" : "+v"(sc[i][r]), "+v"(sh[i][r]), "+v"(cinit[i][r]));
  }
  // halo offsets of this lane's tap groups (relative to the (dd, dh) row and the output column)
  auto goff = [](int t) { return (((t / 9) * 5 + (t / 3) % 3) * HX + (t % 3)) * 8; };
  int toff[KS];
  int gh = 0, gx1 = 0, gx2 = 0;
  bool xsrc2 = false;
  uint32_t xsel1 = 0, xsel2 = 0;
  if (KS == 7) {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      int t = 4 * s + fq;
      t = t < 27 ? t : 26;
      toff[s] = goff(t);
    }
  } else {
    toff[0] = goff(kC1F2[RO][fq]);
    toff[1] = goff(kC1F2[RO][4 + fq]);
    toff[2] = goff(kC1D2[RO][fq]);
    toff[3 % KS] = goff(kC1W[fq]);
    gh = goff(kC1H2[RO][fq]);
    gx1 = goff(kC1X1[fq]);
    gx2 = goff(kC1X2[fq]);
    xsrc2 = fq == 2;
    xsel1 = fq == 0 ? 0x03020100u : fq == 3 ? 0x0c0c0100u : 0x05040100u;
    xsel2 = fq == 0 ? 0x03020100u : fq == 3 ? 0x0c0c0c0cu : 0x05040100u;
  }
  const int colbase0 = (15 * (2 * op) + fr) * 8, colbase1 = colbase0 + 15 * 8;
  const int wloc = fr / 3, dw = fr - 3 * wloc;
  C1_STORE(0)
  __syncthreads();
  for (int ph = ph_lo; ph < ph_hi; ++ph) {
    const int cur = (ph - ph_lo) & 1;
    if (ph + 1 < ph_hi) C1_LOAD(ph + 1)
    const uint16_t* hb = halo + cur * HALO;
    float best[2][2][4], pend[2][2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) best[i][j][r] = -INFINITY;
#pragma unroll DDU
    for (int dd = 0; dd < 3; ++dd) {
      // 3 KS k-steps (3 dh rows x KS); the B fragments are read PF steps ahead of their MFMAs (a ring of PF + 1
      // register pairs), so an LDS read's latency is covered by PF steps of matrix work, not one
      constexpr int NQ = 3 * KS;
      f16x8 rb0[PF + 1], rb1[PF + 1];
#pragma unroll
      for (int p = 0; p < PF; ++p) {
        const int ro = ((dd * 5 + p / KS) * HX) * 8;
        rb0[p] = c1_bfrag<KS>(hb + colbase0, p % KS, ro, toff, gh, gx1, gx2, xsrc2, xsel1, xsel2);
        rb1[p] = c1_bfrag<KS>(hb + colbase1, p % KS, ro, toff, gh, gx1, gx2, xsrc2, xsel1, xsel2);
      }
      f32x4 acc[2][2];
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int dh = q / KS, s = q % KS;
        if (s == 0) {
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = cinit[i];
        }
        if (q + PF < NQ) {
          const int qn = q + PF, ro = ((dd * 5 + qn / KS) * HX) * 8;
          rb0[qn % (PF + 1)] = c1_bfrag<KS>(hb + colbase0, qn % KS, ro, toff, gh, gx1, gx2, xsrc2, xsel1, xsel2);
          rb1[qn % (PF + 1)] = c1_bfrag<KS>(hb + colbase1, qn % KS, ro, toff, gh, gx1, gx2, xsrc2, xsel1, xsel2);
        }
        const f16x8 fb0 = rb0[q % (PF + 1)], fb1 = rb1[q % (PF + 1)];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          acc[i][0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[i][s], fb0, acc[i][0], 0, 0, 0);
          acc[i][1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[i][s], fb1, acc[i][1], 0, 0, 0);
        }
        if (PF > 1) asm volatile("" ::: "memory");  // keep step q+PF's LDS reads in step q (no re-hoisting)
        if (s != KS - 1) continue;
        const uint32_t tag = (uint32_t)(dd * 9 + dh * 3 + dw);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float e = tag_idx(acc[i][j][r], tag);
              if (dh == 0) pend[i][j][r] = e;
              else if (dh == 1) best[i][j][r] = vmax3(best[i][j][r], pend[i][j][r], e);
              else best[i][j][r] = vmax2(best[i][j][r], e);
            }
      }
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int pw = 5 * (2 * op + j) + wloc;
      const bool writer = (dw == 0) && (fr < 15) && (pw < kPW);
      uint32_t pk[2][2], ab[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        ab[i] = 0;
        float o4[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          // max over the window's 3 columns = this lane (dw = 0) and the next two lanes of the 16-lane row
          const uint32_t b0 = __float_as_uint(best[i][j][r]);
          const uint32_t b1 = __builtin_amdgcn_update_dpp(0u, b0, 0x101, 0xf, 0xf, false);  // row_shl:1
          const uint32_t b2 = __builtin_amdgcn_update_dpp(0u, b0, 0x102, 0xf, 0xf, false);  // row_shl:2
          const uint32_t bb = __float_as_uint(vmax3(__uint_as_float(b0), __uint_as_float(b1), __uint_as_float(b2)));
          o4[r] = fmaxf(fmaf(__uint_as_float(bb & ~31u), sc[i][r], sh[i][r]), 0.f);
          ab[i] |= (bb & 31u) << (8 * r);
        }
        pk[i][0] = pack_bf16x2(o4[0], o4[1]);
        pk[i][1] = pack_bf16x2(o4[2], o4[3]);
      }
      if (writer) {
        const int64_t o = ((((int64_t)n * kPD + pd) * kPH + ph) * kPW + pw) * kC1 + 32 * ch + 4 * fq;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          *reinterpret_cast<uint2*>(out + o + 16 * i) = make_uint2(pk[i][0], pk[i][1]);
          *reinterpret_cast<uint32_t*>(amax + o + 16 * i) = ab[i];
        }
      }
    }
    if (ph + 1 < ph_hi) C1_STORE(cur ^ 1)
    __syncthreads();
  }
#undef C1_LOAD
#undef C1_STORE
}

// max over the 3 columns of a pooling window = this lane and the next two of its 16-lane row: two VOP2 DPP maxes
// (the lanes whose window leaves the row are not writers and keep garbage); one s_nop 1 covers the VALU -> DPP
// read hazard of all four inputs
__device__ __forceinline__ void pool3_dpp4(const float (&b)[4], float (&m)[4]) {
  asm volatile(
      "s_nop 1\n\t"
      "v_max_f32_dpp %0, %4, %4 row_shl:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_max_f32_dpp %1, %5, %5 row_shl:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_max_f32_dpp %2, %6, %6 row_shl:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_max_f32_dpp %3, %7, %7 row_shl:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_max_f32_dpp %0, %4, %0 row_shl:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_max_f32_dpp %1, %5, %1 row_shl:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_max_f32_dpp %2, %6, %2 row_shl:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_max_f32_dpp %3, %7, %3 row_shl:2 row_mask:0xf bank_mask:0xf"
      : "=&v"(m[0]), "=&v"(m[1]), "=&v"(m[2]), "=&v"(m[3])
      : "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]));
}

// Wave-tile variant of the fused forward (k_conv1_fwd_w64): each wave owns ALL 64 output channels of one group of
// 15 conv columns (op = wave), instead of 32 channels x 2 column groups.  The B fragment of a (dd, dh, k-step) is
// then read and assembled once for 4 MFMAs instead of twice for 2 each, which halves the LDS traffic (the pipe
// kernel's LDS array time was ~80 % of its MFMA time before its 34 % bank conflicts) and the B-assembly VALU
// (v_perm / v_cndmask / v_mov of k-steps 2-3).  The A operand (64 x 128 f16) stays in 64 VGPRs.  Halo loads are
// unconditional (columns >= 61 clamp to 60: they only feed conv columns >= 59, which no pooled cell reads) with a
// scalar row base and a per-thread 32-bit offset; the max-pool starts from the first candidate pair instead of -inf.
template <int PF, int RO>
__global__ __launch_bounds__(256, 2) void k_conv1_fwd_w64(const uint8_t* __restrict__ x8, const int* __restrict__ idx,
                                                          const uint16_t* __restrict__ w8,
                                                          const float* __restrict__ scale,
                                                          const float* __restrict__ shift, int B,
                                                          uint16_t* __restrict__ out, uint8_t* __restrict__ amax,
                                                          int nq) {
  constexpr int HX = 64, KS = 4, KW = KS * 32;
  constexpr int HALO = 5 * 5 * HX * 8;           // f16 elements per buffer
  constexpr int NV = 5 * 5 * HX;                 // 1600 halo voxels
  constexpr int NLD = (NV + 255) / 256;          // 7 per thread (the 7th: wave 0 only)
  __shared__ __attribute__((aligned(16))) uint16_t halo[2 * HALO];
  __shared__ __attribute__((aligned(16))) float scsh[2][kC1];  // |scale| / 255 and shift (read by the epilogue)
  const int bid0 = xcd_remap(blockIdx.x, gridDim.x);
  const int q = bid0 % nq, bid = bid0 / nq;
  const int pd = bid % kPD, n = bid / kPD;
  const int ph_lo = (kPH * q) / nq, ph_hi = (kPH * (q + 1)) / nq;
  const int g = n / B;
  const int tid = threadIdx.x, lane = tid & 63, op = tid >> 6;
  if (tid < kC1) {
    scsh[0][tid] = fabsf(scale[g * kC1 + tid]) * (1.0f / 255.0f);
    scsh[1][tid] = shift[g * kC1 + tid];
  }
  const uint8_t* xs = x8 + ((int64_t)idx[n] * kPZ * kPY * kPX + (int64_t)(3 * pd) * kPY * kPX) * 8;
  int lofs[NLD];
#pragma unroll
  for (int u = 0; u < NLD; ++u) {
    const int e = min(tid + 256 * u, NV - 1);
    const int xh = min(e & (HX - 1), kPX - 1), yz = e >> 6, yh = yz % 5, zh = yz / 5;
    lofs[u] = ((zh * kPY + yh) * kPX + xh) * 8;
  }
  uint2 pre[NLD];
  auto load_row = [&](int ph) {
    const uint8_t* rp = xs + (int64_t)(3 * ph) * kPX * 8;
#pragma unroll
    for (int u = 0; u < NLD; ++u) pre[u] = *reinterpret_cast<const uint2*>(rp + lofs[u]);
  };
  auto store_row = [&](int buf) {
#pragma unroll
    for (int u = 0; u < NLD; ++u) {
      const int e = tid + 256 * u;
      if (u < NLD - 1 || e < NV) *reinterpret_cast<uint4*>(&halo[buf * HALO + e * 8]) = u8x8_to_f16magic(pre[u]);
    }
  };
  load_row(ph_lo);
  const int fr = lane & 15, fq = lane >> 4;
  f16x8 fa[4][KS];
  const uint16_t* wg = w8 + (int64_t)g * kC1 * KW;
  float rs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      fa[i][s] = *reinterpret_cast<const f16x8*>(wg + (16 * i + fr) * KW + 32 * s + 8 * fq);
#pragma unroll
      for (int e = 0; e < 8; ++e) rs[i] += (float)fa[i][s][e];
    }
  f32x4 cinit[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    rs[i] += __shfl_xor(rs[i], 16, 64);
    rs[i] += __shfl_xor(rs[i], 32, 64);
#pragma unroll
    for (int r = 0; r < 4; ++r) cinit[i][r] = -1024.f * __shfl(rs[i], 4 * fq + r, 64);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int s = 0; s < KS; ++s) asm volatile("" : "+v"(fa[i][s]));
#pragma unroll
    for (int r = 0; r < 4; ++r) asm volatile("" : "+v"(cinit[i][r]));
  }
  auto goff = [](int t) { return (((t / 9) * 5 + (t / 3) % 3) * HX + (t % 3)) * 8; };
  constexpr int R1 = RO ? 1 : 0;
  int toff[KS];
  toff[0] = goff(kC1F2[R1][fq]);
  toff[1] = goff(kC1F2[R1][4 + fq]);
  toff[2] = goff(kC1D2[R1][fq]);
  toff[3] = goff(kC1W[fq]);
  const int gh = goff(kC1H2[R1][fq]);
  // RO = 2: the empty X1 quarter (fq 3) reads the DHW group of its jw-paired quarter (zero weights)
  const int gx1 = RO == 2 ? goff(kC1X1b[fq < 3 ? fq : 2]) : goff(kC1X1[fq]);
  const int gx2 = RO == 2 ? goff(kC1X2b[fq]) : goff(kC1X2[fq]);
  const bool xsrc2 = fq == 2;
  const uint32_t xsel1 = fq == 0 ? 0x03020100u : fq == 3 ? 0x0c0c0100u : 0x05040100u;
  const uint32_t xsel2 = RO == 2 ? (fq < 2 ? 0x03020100u : 0x05040100u)
                                 : fq == 0 ? 0x03020100u : fq == 3 ? 0x0c0c0c0cu : 0x05040100u;
  // k-step 3's two 2-phase groups: the second dword of each is picked by address (dword 2 for the HW groups of
  // fq = 2, dword 1 otherwise) instead of a v_cndmask after a 16-B read
  const int gx1s = gx1 + (xsrc2 ? 4 : 2), gx2s = gx2 + (xsrc2 ? 4 : 2);
  // a whole 16-B read whose value is only partly used: the opaque asm keeps all four dwords live, so the load is
  // not narrowed back to a conflicting ds_read_b64 / ds_read2_b32
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  auto rd128 = [](const uint16_t* p) -> uint4 {
    u32x4 v = *reinterpret_cast<const u32x4*>(p);
    asm("" : "+v"(v));
    return make_uint4(v[0], v[1], v[2], v[3]);
  };
  auto bfrag = [&](const uint16_t* hb, int s, int ro) -> f16x8 {
    if (RO == 2) {
      if (s < 2) return *reinterpret_cast<const f16x8*>(&hb[ro + toff[s]]);
      if (s == 2) {
        const uint4 d = rd128(&hb[ro + toff[2]]), h = rd128(&hb[ro + gh]);
        return __builtin_bit_cast(f16x8, make_uint4(d.x, d.y, h.x, h.z));  // D: phases 0-3, H: phases 0,1,4,5
      }
      const uint4 w = rd128(&hb[ro + toff[3]]), a = rd128(&hb[ro + gx1]), b = rd128(&hb[ro + gx2]);
      uint4 v;
      v.x = __builtin_amdgcn_perm(w.y, w.x, 0x05040100u);  // W: phases 0, 2
      v.y = __builtin_amdgcn_perm(w.w, w.z, 0x05040100u);  // W: phases 4, 6
      v.z = __builtin_amdgcn_perm(a.y, a.x, 0x05040100u);  // X1: phases 0, 2
      v.w = __builtin_amdgcn_perm(b.z, b.x, xsel2);        // X2: phases 0, 1 (DH) or 0, 4 (HW)
      return __builtin_bit_cast(f16x8, v);
    }
    if (s < 3) return c1_bfrag<KS>(hb, s, ro, toff, gh, gx1, gx2, xsrc2, xsel1, xsel2);
    const uint4 w = *reinterpret_cast<const uint4*>(&hb[ro + toff[3]]);
    const uint32_t a0 = *reinterpret_cast<const uint32_t*>(&hb[ro + gx1]);
    const uint32_t a1 = *reinterpret_cast<const uint32_t*>(&hb[ro + gx1s]);
    const uint32_t b0 = *reinterpret_cast<const uint32_t*>(&hb[ro + gx2]);
    const uint32_t b1 = *reinterpret_cast<const uint32_t*>(&hb[ro + gx2s]);
    uint4 v;
    v.x = __builtin_amdgcn_perm(w.y, w.x, 0x05040100u);  // phases 0, 2 (low halves)
    v.y = __builtin_amdgcn_perm(w.w, w.z, 0x05040100u);  // phases 4, 6
    v.z = __builtin_amdgcn_perm(a1, a0, xsel1);
    v.w = __builtin_amdgcn_perm(b1, b0, xsel2);
    return __builtin_bit_cast(f16x8, v);
  };
  const int colbase = (15 * op + fr) * 8;
  const int wloc = fr / 3, dw = fr - 3 * wloc;
  const int pw = 5 * op + wloc;
  const bool writer = (dw == 0) && (fr < 15) && (pw < kPW);
  store_row(0);
  __syncthreads();
  for (int ph = ph_lo; ph < ph_hi; ++ph) {
    const int cur = (ph - ph_lo) & 1;
    if (ph + 1 < ph_hi) load_row(ph + 1);
    const uint16_t* hb = halo + cur * HALO + colbase;
    float best[4][4], pend[4][4], pend2[4][4];
#pragma unroll
    for (int dd = 0; dd < 3; ++dd) {
      constexpr int NQ = 3 * KS;
      f16x8 rb[PF + 1];
#pragma unroll
      for (int p = 0; p < PF; ++p)
        rb[p] = bfrag(hb, p % KS, ((dd * 5 + p / KS) * HX) * 8);
      f32x4 acc[4];
#pragma unroll
      for (int qq = 0; qq < NQ; ++qq) {
        const int dh = qq / KS, s = qq % KS;
        if (qq + PF < NQ) {
          const int qn = qq + PF;
          rb[qn % (PF + 1)] = bfrag(hb, qn % KS, ((dd * 5 + qn / KS) * HX) * 8);
        }
        const f16x8 fb = rb[qq % (PF + 1)];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[i][s], fb, s == 0 ? cinit[i] : acc[i], 0, 0, 0);
        if (PF > 1) asm volatile("" ::: "memory");
        if (s != KS - 1) continue;
        // the 9 (dd, dh) candidates of a lane fold into the running max with 4 v_max3: k = 0, 1 wait, k = 2 starts
        // the max, then every even k folds itself and the odd one before it
        const uint32_t tag = (uint32_t)(dd * 9 + dh * 3 + dw);
        const int k = dd * 3 + dh;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float e = tag_idx(acc[i][r], tag);
            if (k == 0) pend2[i][r] = e;
            else if (k & 1) pend[i][r] = e;
            else if (k == 2) best[i][r] = vmax3(pend2[i][r], pend[i][r], e);
            else best[i][r] = vmax3(best[i][r], pend[i][r], e);
          }
      }
    }
    const int64_t o = ((((int64_t)n * kPD + pd) * kPH + ph) * kPW + pw) * kC1 + 4 * fq;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float m[4];
      pool3_dpp4(best[i], m);
      const f32x4 scv = *reinterpret_cast<const f32x4*>(&scsh[0][16 * i + 4 * fq]);
      const f32x4 shv = *reinterpret_cast<const f32x4*>(&scsh[1][16 * i + 4 * fq]);
      uint32_t u[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) u[r] = __float_as_uint(m[r]);
      // argmax tags: the low byte of each candidate, gathered by two v_perm, then masked to 5 bits
      const uint32_t t01 = __builtin_amdgcn_perm(u[1], u[0], 0x0c0c0400u);
      const uint32_t t23 = __builtin_amdgcn_perm(u[3], u[2], 0x04000c0cu);
      const uint32_t ab = (t01 | t23) & 0x1f1f1f1fu;
      f32x2 v01 = {__uint_as_float(u[0] & ~31u), __uint_as_float(u[1] & ~31u)};
      f32x2 v23 = {__uint_as_float(u[2] & ~31u), __uint_as_float(u[3] & ~31u)};
      const f32x2 s01 = {scv[0], scv[1]}, s23 = {scv[2], scv[3]}, h01 = {shv[0], shv[1]}, h23 = {shv[2], shv[3]};
      v01 = v01 * s01 + h01;
      v23 = v23 * s23 + h23;
      // relu on the packed bf16 pair: a signed 16-bit max with 0 zeroes exactly the negative values (and -0)
      typedef short s16x2 __attribute__((ext_vector_type(2)));
      const s16x2 z = {0, 0};
      const s16x2 p01 = __builtin_elementwise_max(__builtin_bit_cast(s16x2, pack_bf16x2(v01[0], v01[1])), z);
      const s16x2 p23 = __builtin_elementwise_max(__builtin_bit_cast(s16x2, pack_bf16x2(v23[0], v23[1])), z);
      if (writer) {
        *reinterpret_cast<uint2*>(out + o + 16 * i) =
            make_uint2(__builtin_bit_cast(uint32_t, p01), __builtin_bit_cast(uint32_t, p23));
        *reinterpret_cast<uint32_t*>(amax + o + 16 * i) = ab;
      }
    }
    if (ph + 1 < ph_hi) store_row(cur ^ 1);
    __syncthreads();
  }
}

// forward variant: NIDT_C1_FWD=1 (default) the wave-tile kernel (k_conv1_fwd_w64: 4.20 -> 3.33 ms per 64-client
// step, 0.59 -> 0.47 ms at 8 clients, profiles/r5_c1fwd_w64.txt), 0 the channel-split pipe kernel;
// conv1_fwd_mode(m) overrides it at run time (tests: m = 0 / 1, -1 back to the environment / default)
static int g_c1fwd_mode = -1;
void conv1_fwd_mode(int mode) { g_c1fwd_mode = mode; }
int conv1_fwd_variant() {
  static const int v = [] {
    const char* e = getenv("NIDT_C1_FWD");
    return e ? atoi(e) : 1;
  }();
  return g_c1fwd_mode >= 0 ? g_c1fwd_mode : v;
}

void conv1_fwd_pool(uintptr_t x8, uintptr_t idx, uintptr_t w8, uintptr_t scale, uintptr_t shift, int NB, int B,
                    uintptr_t out, uintptr_t amax, uintptr_t stream) {
  NIDT_REQUIRE(NB % B == 0, "conv1_fwd_pool: NB % B");
  if (conv1_fwd_variant() == 1 && conv1_kslots() == 128) {
    static const int nq1 = [] {
      const char* e = getenv("NIDT_C1_NQ");
      return e ? std::max(1, std::min(kPH, atoi(e))) : 1;
    }();
    // B-fragment prefetch distance of the RO = 2 kernel in k-steps (NIDT_C1_WPF, A/B), default 4 (3.28 ms per
    // 64-client step vs 3.35 at 2; the RO = 0 kernel, 45.7 % bank conflicts, also 3.28: profiles/r6_conv1_b128.txt)
    static const int wpf = [] {
      const char* e = getenv("NIDT_C1_WPF");
      return e ? atoi(e) : 4;
    }();
    if (conv1_tapord() == 2 && wpf == 3)
      hipLaunchKernelGGL((k_conv1_fwd_w64<3, 2>), dim3(kPD * NB * nq1), dim3(256), 0, as_stream(stream),
                         ptr<const uint8_t>(x8), ptr<const int>(idx), ptr<const uint16_t>(w8), ptr<const float>(scale),
                         ptr<const float>(shift), B, ptr<uint16_t>(out), ptr<uint8_t>(amax), nq1);
    else if (conv1_tapord() == 2 && wpf == 4)
      hipLaunchKernelGGL((k_conv1_fwd_w64<4, 2>), dim3(kPD * NB * nq1), dim3(256), 0, as_stream(stream),
                         ptr<const uint8_t>(x8), ptr<const int>(idx), ptr<const uint16_t>(w8), ptr<const float>(scale),
                         ptr<const float>(shift), B, ptr<uint16_t>(out), ptr<uint8_t>(amax), nq1);
    else if (conv1_tapord() == 2)
      hipLaunchKernelGGL((k_conv1_fwd_w64<2, 2>), dim3(kPD * NB * nq1), dim3(256), 0, as_stream(stream),
                         ptr<const uint8_t>(x8), ptr<const int>(idx), ptr<const uint16_t>(w8), ptr<const float>(scale),
                         ptr<const float>(shift), B, ptr<uint16_t>(out), ptr<uint8_t>(amax), nq1);
    else if (conv1_tapord() == 1)
      hipLaunchKernelGGL((k_conv1_fwd_w64<2, 1>), dim3(kPD * NB * nq1), dim3(256), 0, as_stream(stream),
                         ptr<const uint8_t>(x8), ptr<const int>(idx), ptr<const uint16_t>(w8), ptr<const float>(scale),
                         ptr<const float>(shift), B, ptr<uint16_t>(out), ptr<uint8_t>(amax), nq1);
    else
      hipLaunchKernelGGL((k_conv1_fwd_w64<2, 0>), dim3(kPD * NB * nq1), dim3(256), 0, as_stream(stream),
                         ptr<const uint8_t>(x8), ptr<const int>(idx), ptr<const uint16_t>(w8), ptr<const float>(scale),
                         ptr<const float>(shift), B, ptr<uint16_t>(out), ptr<uint8_t>(amax), nq1);
    NIDT_CHECK(hipGetLastError());
    return;
  }
  // B-fragment prefetch distance (k-steps); NIDT_C1_PF=1/2/3 selects it (A/B), default 2
  static const int pf = [] {
    const char* e = getenv("NIDT_C1_PF");
    return e ? atoi(e) : 2;
  }();
  static const int occ = [] {
    const char* e = getenv("NIDT_C1_OCC");
    return e ? atoi(e) : 2;
  }();
  // pooled-row split per slab: NIDT_C1_NQ (A/B), default 1
  static const int nq_env = [] {
    const char* e = getenv("NIDT_C1_NQ");
    return e ? std::max(1, std::min(kPH, atoi(e))) : 1;
  }();
  const int nq = nq_env;
#define NIDT_C1(PF, KSS)                                                                                       \
  if (occ == 3 && (PF) == 2 && (KSS) == 4)                                                                     \
    hipLaunchKernelGGL((k_conv1_fwd_pool_pipe<2, 4, 3>), dim3(kPD * NB * nq), dim3(256), 0, as_stream(stream),     \
                       ptr<const uint8_t>(x8), ptr<const int>(idx), ptr<const uint16_t>(w8), ptr<const float>(scale), \
                       ptr<const float>(shift), B, ptr<uint16_t>(out), ptr<uint8_t>(amax), nq);                      \
  else                                                                                                         \
  hipLaunchKernelGGL((k_conv1_fwd_pool_pipe<PF, KSS>), dim3(kPD * NB * nq), dim3(256), 0, as_stream(stream),      \
                     ptr<const uint8_t>(x8), ptr<const int>(idx), ptr<const uint16_t>(w8), ptr<const float>(scale),  \
                     ptr<const float>(shift), B, ptr<uint16_t>(out), ptr<uint8_t>(amax), nq)
  // the three dd rows of the 3^3 window unrolled: each row's pooling epilogue overlaps the next row's MFMAs and the
  // body needs 208 instead of 248 VGPRs (4.30 -> 4.17 ms per 64-client step, profiles/r3_ab_conv1_fwd_ddu.txt);
  // NIDT_C1_DDU=1 keeps the rolled loop (A/B)
  static const int ddu = [] {
    const char* e = getenv("NIDT_C1_DDU");
    return e ? atoi(e) : 3;
  }();
  if (conv1_kslots() == 128 && ddu == 3 && pf == 2 && occ != 3 && conv1_tapord() == 0) {
    hipLaunchKernelGGL((k_conv1_fwd_pool_pipe<2, 4, 2, 3, 0>), dim3(kPD * NB * nq), dim3(256), 0, as_stream(stream),
                       ptr<const uint8_t>(x8), ptr<const int>(idx), ptr<const uint16_t>(w8), ptr<const float>(scale),
                       ptr<const float>(shift), B, ptr<uint16_t>(out), ptr<uint8_t>(amax), nq);
  } else if (conv1_kslots() == 128 && ddu == 3 && pf == 2 && occ != 3) {
    hipLaunchKernelGGL((k_conv1_fwd_pool_pipe<2, 4, 2, 3>), dim3(kPD * NB * nq), dim3(256), 0, as_stream(stream),
                       ptr<const uint8_t>(x8), ptr<const int>(idx), ptr<const uint16_t>(w8), ptr<const float>(scale),
                       ptr<const float>(shift), B, ptr<uint16_t>(out), ptr<uint8_t>(amax), nq);
  } else if (conv1_kslots() == 128) {
    if (pf == 1) NIDT_C1(1, 4); else if (pf == 3) NIDT_C1(3, 4); else NIDT_C1(2, 4);
  } else {
    if (pf == 1) NIDT_C1(1, 7); else if (pf == 3) NIDT_C1(3, 7); else NIDT_C1(2, 7);
  }
#undef NIDT_C1
  NIDT_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// Sparse wgrad: S[c][k] = sum over pooled voxels of dz * patch(argmax voxel), D[c] = sum dz.
// Block = (n, pd); thread = (wave w, channel c = lane).  Per stage of kWgRows pooled rows (ph) the block stages
// (a) the polyphase input halo as raw uint8 (8 B per voxel) and (b) one 32-bit record per (cell, channel):
// dz = (pooled > 0 ? dL/dpooled : 0) as bf16 bits in the low half, the halo offset of the argmax patch in the
// high half.  Staging the per-cell metadata with the whole block's loads in flight at once (instead of each
// lane walking its cells with a one-cell global prefetch) takes the L2/HBM latency out of the cell loop, which
// PMC showed parked 42 % of wave time in s_waitcnt.  Halo strides are padded so that the 27 possible argmax
// offsets (aw + 67 ah + 553 ad voxels apart: 3 and 9 mod 32) fall on 27 distinct ds_read_b64 bank pairs: the
// 64 channel-lanes of a wave, which read at their own argmax, never bank-conflict.
// Output slab: part[n*19 + pd][64][126] (125 S entries + D).
constexpr int kWgRows = 2;                       // pooled rows (ph) per stage
constexpr int kWgHY = 3 * kWgRows + 2;           // halo y extent (8)
constexpr int kWgRS = 67;                        // row stride in voxels   (67 = 3 mod 32)
constexpr int kWgZS = 553;                       // plane stride in voxels (553 = 9 mod 32, >= 8*67)
constexpr int kWgHalo = 5 * kWgZS;               // voxels per halo buffer
constexpr int kWgMeta = kWgRows * kPW * kC1;     // metadata records per stage
__device__ __forceinline__ int bid_slab(int n_pd, int q, int nq) { return n_pd * nq + q; }  // slab of (n, pd, q)

// Reduce slabs per client and apply the closed form.  grid (64 c, G), block 1024: the B*19*nq slabs are split
// over the 16 waves (lane = k, k + 64; 4 independent loads in flight per lane; 16 waves per block because at few
// clients per GPU there are only 64*G blocks to cover the L2/HBM latency), merged through LDS in a fixed order
// (deterministic), then threads 0..127 (k) apply the closed form.
constexpr int kFinW = 16;
__global__ __launch_bounds__(64 * kFinW) void k_conv1_wgrad_fin(const float* __restrict__ part, int nslab,
                                                         const float* __restrict__ w125, const float* __restrict__ mu,
                                                         const float* __restrict__ covw,
                                                         const float* __restrict__ invstd, const float* theta,
                                                         int64_t ldt, int64_t off_g, float* grad, int64_t ldg,
                                                         int64_t goff_w, int64_t goff_bias, int64_t goff_g,
                                                         int64_t goff_b, float wscale, const float* __restrict__ emean) {
  __shared__ double red[2];
  __shared__ double sD, sdg;
  __shared__ double wpart[kFinW][128];
  const int c = blockIdx.x, g = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  {
    const float* base = part + ((int64_t)g * nslab * kC1 + c) * 126;
    const int64_t sst = (int64_t)kC1 * 126;  // slab stride
    double a0 = 0, a1 = 0;
    const bool hi = lane + 64 < 126;
    int sl = wid;
    for (; sl + 3 * kFinW < nslab; sl += 4 * kFinW) {
      float v0[4], v1[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float* o = base + (int64_t)(sl + kFinW * u) * sst;
        v0[u] = o[lane];
        v1[u] = hi ? o[lane + 64] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) { a0 += v0[u]; a1 += v1[u]; }
    }
    for (; sl < nslab; sl += kFinW) {
      const float* o = base + (int64_t)sl * sst;
      a0 += o[lane];
      if (hi) a1 += o[lane + 64];
    }
    wpart[wid][lane] = a0;
    wpart[wid][lane + 64] = a1;
  }
  __syncthreads();
  if (tid < 128) {  // fixed-order tree over the 16 wave partials
    double t[kFinW];
#pragma unroll
    for (int w = 0; w < kFinW; ++w) t[w] = wpart[w][tid];
#pragma unroll
    for (int h = kFinW / 2; h > 0; h >>= 1)
#pragma unroll
      for (int w = 0; w < h; ++w) t[w] += t[w + h];
    wpart[0][tid] = t[0];
  }
  __syncthreads();
  if (tid >= 128) return;
  const int k = tid;
  double S = k < 125 ? wpart[0][k] : 0.0;
  if (k == 0) sD = wpart[0][125];
  __syncthreads();
  double D = sD;
  const int i = g * kC1 + c;
  const double iv = invstd[i];
  const double gm = theta[(int64_t)g * ldt + off_g + c];
  const double muk = k < 125 ? mu[(int64_t)g * 125 + k] : 0.0;
  const double wk = k < 125 ? w125[(int64_t)i * 125 + k] : 0.0;
  // eval mode (emean != null, running statistics): y = w.p + b, z = gamma*(y - rm)*iv + beta, so
  // dW = gamma*iv*S, dbias = gamma*iv*D, dgamma = iv*(w.S - D*(rm - b)) with emean = rm - b
  const bool ev = emean != nullptr;
  const double r = k < 125 ? (ev ? S : S - D * muk) : 0.0;
  double v = wk * r;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((k & 63) == 0) red[k >> 6] = v;
  __syncthreads();
  if (k == 0) sdg = ev ? iv * (red[0] + red[1] - D * (double)emean[i]) : iv * (red[0] + red[1]);
  __syncthreads();
  const double dg = sdg;
  if (k < 125) {
    const double dw = ev ? gm * iv * r : gm * iv * (r - dg * iv * covw[(int64_t)i * 125 + k]);
    grad[(int64_t)g * ldg + goff_w + (int64_t)c * 125 + k] = (float)(dw * wscale);
  }
  if (k == 0) {
    grad[(int64_t)g * ldg + goff_g + c] = (float)dg;
    grad[(int64_t)g * ldg + goff_b + c] = (float)D;
    grad[(int64_t)g * ldg + goff_bias + c] = ev ? (float)(gm * iv * D) : 0.f;
  }
}

// k_conv1_wgrad_split — the sparse wgrad with the 125 taps split over the 4 waves instead of the cells:
// every wave walks all cells of the slab for its channel (lane) but accumulates only its ~31 taps, so the
// accumulators shrink from 125 to <= 32 VGPRs (4+ waves/SIMD instead of 2, which hides the LDS and L2
// latency of the per-lane argmax gathers) and no cross-wave reduction is needed: each wave writes its own
// disjoint taps of the slab row.  Polyphase offsets t = 9jd+3jh+jw carry 8/4/2/1 valid taps (j=2 drops
// the odd phase in that dimension); the sets below balance taps (32/32/30/31).
__device__ constexpr int kWgSet0[] = {0, 1, 3, 4};
__device__ constexpr int kWgSet1[] = {9, 10, 12, 13};
__device__ constexpr int kWgSet2[] = {2, 5, 11, 14, 6, 7, 15, 8};
__device__ constexpr int kWgSet3[] = {16, 18, 19, 21, 22, 17, 20, 23, 24, 25, 26};
template <int W> struct WgSet;
template <> struct WgSet<0> { static constexpr int n = 4; __device__ static constexpr int t(int i) { return kWgSet0[i]; } };
template <> struct WgSet<1> { static constexpr int n = 4; __device__ static constexpr int t(int i) { return kWgSet1[i]; } };
template <> struct WgSet<2> { static constexpr int n = 8; __device__ static constexpr int t(int i) { return kWgSet2[i]; } };
template <> struct WgSet<3> { static constexpr int n = 11; __device__ static constexpr int t(int i) { return kWgSet3[i]; } };

__host__ __device__ constexpr int tp_count(int t) {
  return (t / 9 < 2 ? 2 : 1) * ((t / 3) % 3 < 2 ? 2 : 1) * (t % 3 < 2 ? 2 : 1);
}

// byte b of w as fp32: one v_cvt_f32_ubyteN.  Written out because the compiler merges the two dwords of a
// ds_read_b64 into one 64-bit value for some tap sets and then converts (w64 >> 8n) & 0xff through the u64->f32
// sequence (lshl_b64, min, or, cvt_f32_u32, ldexp: ~5 VALU per byte, ~20 extra per cell on waves 1-2, which
// pace the block's per-stage barrier).
__device__ __forceinline__ float u8f(uint32_t w, int b) {
  float f;
  switch (b) {
    case 0: asm("v_cvt_f32_ubyte0 %0, %1" : "=v"(f) : "v"(w)); break;
    case 1: asm("v_cvt_f32_ubyte1 %0, %1" : "=v"(f) : "v"(w)); break;
    case 2: asm("v_cvt_f32_ubyte2 %0, %1" : "=v"(f) : "v"(w)); break;
    default: asm("v_cvt_f32_ubyte3 %0, %1" : "=v"(f) : "v"(w)); break;
  }
  return f;
}

// one cell of the sparse wgrad: its (dz, argmax offset) record and the 8-phase halo voxels of the wave's taps
template <class SET>
__device__ __forceinline__ void conv1_wg_load(const uint32_t* meta, const uint2* halo, int it, int c, float& dz,
                                              uint2 (&u)[SET::n]) {
  const uint32_t m = meta[it * kC1 + c];
  dz = bf16_to_f32((uint16_t)(m & 0xffffu));
  const uint2* base = halo + (m >> 16);
  // volatile 8-B LDS reads (lds_u64, below): one ds_read_b64 per tap group, in this order.  Plain loads of
  // neighbouring voxels are merged by the compiler into ds_read2_b64, which costs 8 LDS cycles for 16 B (two
  // ds_read_b64: 4) and banks by (a/4) mod 32, so the padded strides no longer keep the 27 argmax offsets apart
#pragma unroll
  for (int i = 0; i < SET::n; ++i) {
    const int t = SET::t(i);
    const uint64_t v = ((const volatile __attribute__((address_space(3))) uint64_t*)base)[(t / 9) * kWgZS +
                                                                                        ((t / 3) % 3) * kWgRS + t % 3];
    u[i] = make_uint2((uint32_t)v, (uint32_t)(v >> 32));
  }
}

// S += dz * x over the wave's valid taps; consecutive taps are paired into packed-FP32 FMAs (v_pk_fma_f32)
template <class SET>
__device__ __forceinline__ void conv1_wg_fma(float dz, const uint2 (&u)[SET::n], f32x2* S2) {
  const f32x2 dz2 = {dz, dz};
  int slot = 0;
  float pend = 0.f;
#pragma unroll
  for (int i = 0; i < SET::n; ++i) {
    const int t = SET::t(i);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      if (tp_valid(t, r)) {
        const float xv = u8f(r < 4 ? u[i].x : u[i].y, r & 3);
        if ((slot & 1) == 0) {
          pend = xv;
        } else {
          const f32x2 x2 = {pend, xv};
          S2[slot >> 1] = __builtin_elementwise_fma(dz2, x2, S2[slot >> 1]);
        }
        ++slot;
      }
    }
  }
  if (slot & 1) S2[slot >> 1].x = fmaf(dz, pend, S2[slot >> 1].x);
}

template <int W, int UNR>
__device__ __forceinline__ void conv1_wg_wave(const uint8_t* __restrict__ xs, const uint16_t* __restrict__ dp,
                                              const uint16_t* __restrict__ pout, const uint8_t* __restrict__ amax,
                                              float* __restrict__ part, uint2* halo, uint32_t* meta, int n, int pd,
                                              int tid, int c, int ph_begin, int ph_end, int slab) {
  using SET = WgSet<W>;
  constexpr int NS = 32;  // >= taps of any set
  f32x2 S2[NS / 2];
#pragma unroll
  for (int k = 0; k < NS / 2; ++k) S2[k] = f32x2{0.f, 0.f};
  float Dsum = 0.f;
  const int64_t rowbase = ((int64_t)n * kPD + pd) * kPH;
  for (int ph0 = ph_begin; ph0 < ph_end; ph0 += kWgRows) {
    const int nph = min(kWgRows, ph_end - ph0);
    const int ny = 3 * nph + 2;
    __syncthreads();
    for (int e = tid; e < 5 * ny * 64; e += 256) {
      const int xh = e & 63, r = e >> 6, yh = r % ny, zh = r / ny;
      const int z = 3 * pd + zh, y = 3 * ph0 + yh;
      uint2 v = make_uint2(0, 0);
      if (xh < kPX) v = *reinterpret_cast<const uint2*>(xs + (((int64_t)z * kPY + y) * kPX + xh) * 8);
      halo[zh * kWgZS + yh * kWgRS + xh] = v;
    }
    const int ncell = nph * kPW;
    const int64_t obase = ((rowbase + ph0) * kPW) * kC1;
    for (int e = tid; e < ncell * kC1; e += 256) {  // (cell, channel) records, channel-fastest: coalesced
      const int cell = e >> 6;
      const uint16_t pv = pout[obase + e], g = dp[obase + e];
      const int a = amax[obase + e];
      const int phl = cell / kPW, pw = cell - phl * kPW;
      const int off = (a / 9) * kWgZS + (3 * phl + (a / 3) % 3) * kWgRS + 3 * pw + a % 3;
      const uint32_t dzb = bf16_to_f32(pv) > 0.f ? (uint32_t)g : 0u;
      meta[e] = dzb | ((uint32_t)off << 16);
    }
    __syncthreads();
    // UNR cells per iteration: every cell's metadata and halo reads are issued before any of their FMAs, so the
    // LDS latency of cell it+1 hides behind cell it's arithmetic inside one wave
    int it = 0;
    for (; it + UNR <= ncell; it += UNR) {
      float dz[UNR];
      uint2 u[UNR][SET::n];
#pragma unroll
      for (int q = 0; q < UNR; ++q) conv1_wg_load<SET>(meta, halo, it + q, c, dz[q], u[q]);
#pragma unroll
      for (int q = 0; q < UNR; ++q) {
        if (W == 0) Dsum += dz[q];
        conv1_wg_fma<SET>(dz[q], u[q], S2);
      }
    }
    for (; it < ncell; ++it) {
      float dz;
      uint2 u[SET::n];
      conv1_wg_load<SET>(meta, halo, it, c, dz, u);
      if (W == 0) Dsum += dz;
      conv1_wg_fma<SET>(dz, u, S2);
    }
  }
  float* op = part + ((int64_t)slab * kC1 + c) * 126;
  int slot = 0;
#pragma unroll
  for (int i = 0; i < SET::n; ++i) {
    const int t = SET::t(i);
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      if (tp_valid(t, r)) {
        op[tp_to_k(t, r)] = (slot & 1) ? S2[slot >> 1].y : S2[slot >> 1].x;
        ++slot;
      }
    }
  }
  if (W == 0) op[125] = Dsum;
}

// grid = NB * 19 * nq: block (n, pd, q) walks pooled rows [q * rq, (q + 1) * rq) of its slab (nq = 2 when one
// slab per (sample, pd) would give the chip fewer than ~4 blocks per CU: few clients per GPU)
template <int UNR>
__global__ __launch_bounds__(256) void k_conv1_wgrad_split(const uint8_t* __restrict__ x8, const int* __restrict__ idx,
                                                           const uint16_t* __restrict__ dp,
                                                           const uint16_t* __restrict__ pout,
                                                           const uint8_t* __restrict__ amax, float* __restrict__ part,
                                                           int nq) {
  __shared__ __attribute__((aligned(16))) uint2 halo[kWgHalo];
  __shared__ uint32_t meta[kWgMeta];
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int q = bid % nq, rest = bid / nq;
  const int pd = rest % kPD, n = rest / kPD;
  const int rq = ((kPH + nq - 1) / nq + kWgRows - 1) / kWgRows * kWgRows;
  const int ph_begin = q * rq, ph_end = min(kPH, ph_begin + rq);
  const int tid = threadIdx.x, c = tid & 63, wid = tid >> 6;
  const uint8_t* xs = x8 + (int64_t)idx[n] * kPZ * kPY * kPX * 8;
  switch (wid) {
    case 0: conv1_wg_wave<0, UNR>(xs, dp, pout, amax, part, halo, meta, n, pd, tid, c, ph_begin, ph_end, bid_slab(rest, q, nq)); break;
    case 1: conv1_wg_wave<1, UNR>(xs, dp, pout, amax, part, halo, meta, n, pd, tid, c, ph_begin, ph_end, bid_slab(rest, q, nq)); break;
    case 2: conv1_wg_wave<2, UNR>(xs, dp, pout, amax, part, halo, meta, n, pd, tid, c, ph_begin, ph_end, bid_slab(rest, q, nq)); break;
    default: conv1_wg_wave<3, UNR>(xs, dp, pout, amax, part, halo, meta, n, pd, tid, c, ph_begin, ph_end, bid_slab(rest, q, nq)); break;
  }
}

// k_conv1_wgrad_dot — the same sparse wgrad with CELL-PAIRED bf16 dot products: uint8 inputs are exact in bf16, so
// the halo is staged once per stage as bf16 (two planes of 4 phases, each an 8-B voxel read with the padded strides
// above: the 27 argmax offsets stay on 27 distinct bank pairs), and each lane takes two cells at a time:
// v_perm_b32 interleaves the two cells' values of a tap into one bf16 pair and v_dot2c_f32_bf16 adds both products
// to the tap's fp32 accumulator — 1 VALU per MAC (one perm + one dot2 per two MACs) instead of 1.5
// (v_cvt_f32_ubyte per value + half a v_pk_fma_f32).  The dz pair (bf16, as stored) is one perm per cell pair.
__device__ __forceinline__ uint32_t bf2_pack(float lo, float hi) {  // exact for integers < 257
  return __builtin_amdgcn_perm(__float_as_uint(hi), __float_as_uint(lo), 0x07060302u);
}
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float dot2bf(uint32_t a, uint32_t b, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2v, a), __builtin_bit_cast(bf16x2v, b), c, false);
}

// the 8-B halo reads of one cell for a wave's tap set: phases 0-3 (hlo) of every group that has a live tap there,
// then phases 4-7 (hhi)
template <class SET>
__device__ constexpr int wd_nreads() {
  int n = 0;
  for (int h = 0; h < 2; ++h)
    for (int i = 0; i < SET::n; ++i) {
      bool need = false;
      for (int r = 0; r < 4; ++r) need = need || tp_valid(SET::t(i), 4 * h + r);
      n += need ? 1 : 0;
    }
  return n;
}

// volatile 8-B reads: one ds_read_b64 each (2 LDS cycles, 64-bank rule), issued in this order.  Plain loads of
// neighbouring voxels get merged into ds_read2_b64 (8 cycles for the same 16 B, 32-bank rule: the padded strides
// no longer separate the argmax offsets) or split into ds_read2_b32.
typedef const volatile __attribute__((address_space(3))) uint64_t lds_u64;
template <class SET, int NR>
__device__ __forceinline__ void conv1_wd_load(const uint2* hlo, const uint2* hhi, uint32_t m, uint64_t (&v)[NR]) {
  int k = 0;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < SET::n; ++i) {
      const int t = SET::t(i);
      bool need = false;
#pragma unroll
      for (int r = 0; r < 4; ++r) need = need || tp_valid(t, 4 * h + r);
      if (!need) continue;
      const int off = (t / 9) * kWgZS + ((t / 3) % 3) * kWgRS + t % 3;
      v[k++] = ((lds_u64*)((h ? hhi : hlo) + (m >> 16)))[off];
    }
}

template <class SET, int NR>
__device__ __forceinline__ void conv1_wd_fma(uint32_t dzp, const uint64_t (&a)[NR], const uint64_t (&b)[NR], float* S) {
  int k = 0, slot = 0;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < SET::n; ++i) {
      const int t = SET::t(i);
      bool need = false;
#pragma unroll
      for (int r = 0; r < 4; ++r) need = need || tp_valid(t, 4 * h + r);
      if (!need) continue;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const uint32_t aj = (uint32_t)(a[k] >> (32 * j)), bj = (uint32_t)(b[k] >> (32 * j));
        if (tp_valid(t, 4 * h + 2 * j)) {
          S[slot] = dot2bf(dzp, __builtin_amdgcn_perm(bj, aj, 0x05040100u), S[slot]);
          ++slot;
        }
        if (tp_valid(t, 4 * h + 2 * j + 1)) {
          S[slot] = dot2bf(dzp, __builtin_amdgcn_perm(bj, aj, 0x07060302u), S[slot]);
          ++slot;
        }
      }
      ++k;
    }
}

// slot order of the accumulators: phases 0-3 of every group of the set, then phases 4-7 (conv1_wd_half order)
template <class SET>
__device__ __forceinline__ void conv1_wd_store(const float* S, float* op) {
  int slot = 0;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < SET::n; ++i) {
      const int t = SET::t(i);
      bool need = false;
#pragma unroll
      for (int r = 0; r < 4; ++r) need = need || tp_valid(t, 4 * h + r);
      if (!need) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (tp_valid(t, 4 * h + r)) op[tp_to_k(t, 4 * h + r)] = S[slot++];
    }
}

template <int W>
__device__ __forceinline__ void conv1_wd_wave(const uint8_t* __restrict__ xs, const uint16_t* __restrict__ dp,
                                              const uint16_t* __restrict__ pout, const uint8_t* __restrict__ amax,
                                              float* __restrict__ part, uint2* hlo, uint2* hhi, uint32_t* meta, int n,
                                              int pd, int tid, int c, int ph_begin, int ph_end, int slab) {
  using SET = WgSet<W>;
  constexpr int NS = 32;
  float S[NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) S[k] = 0.f;
  float Dsum = 0.f;
  const int64_t rowbase = ((int64_t)n * kPD + pd) * kPH;
  // the next stage's global reads (halo voxels, pooled value / gradient / argmax per (cell, channel)) are issued into
  // registers before this stage's dot products and written to LDS after them: with 54 KB of LDS per block only 2
  // blocks share a CU, too few to cover the staging latency by switching blocks
  constexpr int kHV = (5 * kWgHY * 64 + 255) / 256, kMV = (kWgMeta + 255) / 256;
  uint2 hv[kHV];
  uint16_t pvr[kMV], gvr[kMV];
  uint8_t avr[kMV];
  auto prefetch = [&](int ph0) {
    const int nph = min(kWgRows, ph_end - ph0), ny = 3 * nph + 2, ncell = nph * kPW;
    const int64_t obase = ((rowbase + ph0) * kPW) * kC1;
#pragma unroll
    for (int k = 0; k < kHV; ++k) {
      const int e = tid + 256 * k;
      const int xh = e & 63, r = e >> 6, yh = r % ny, zh = r / ny;
      hv[k] = make_uint2(0, 0);
      if (e < 5 * ny * 64 && xh < kPX)
        hv[k] = *reinterpret_cast<const uint2*>(xs + (((int64_t)(3 * pd + zh) * kPY + 3 * ph0 + yh) * kPX + xh) * 8);
    }
#pragma unroll
    for (int k = 0; k < kMV; ++k) {
      const int e = tid + 256 * k;
      if (e < ncell * kC1) {
        pvr[k] = pout[obase + e];
        gvr[k] = dp[obase + e];
        avr[k] = amax[obase + e];
      }
    }
  };
  auto commit = [&](int ph0) {
    const int nph = min(kWgRows, ph_end - ph0), ny = 3 * nph + 2, ncell = nph * kPW;
#pragma unroll
    for (int k = 0; k < kHV; ++k) {
      const int e = tid + 256 * k;
      if (e < 5 * ny * 64) {
        const int xh = e & 63, r = e >> 6, yh = r % ny, zh = r / ny;
        const int hi = zh * kWgZS + yh * kWgRS + xh;
        const uint2 v = hv[k];
        hlo[hi] = make_uint2(bf2_pack(u8f(v.x, 0), u8f(v.x, 1)), bf2_pack(u8f(v.x, 2), u8f(v.x, 3)));
        hhi[hi] = make_uint2(bf2_pack(u8f(v.y, 0), u8f(v.y, 1)), bf2_pack(u8f(v.y, 2), u8f(v.y, 3)));
      }
    }
#pragma unroll
    for (int k = 0; k < kMV; ++k) {
      const int e = tid + 256 * k;
      if (e < ncell * kC1) {
        const int cell = e >> 6, a = avr[k];
        const int phl = cell / kPW, pw = cell - phl * kPW;
        const int off = (a / 9) * kWgZS + (3 * phl + (a / 3) % 3) * kWgRS + 3 * pw + a % 3;
        const uint32_t dzb = bf16_to_f32(pvr[k]) > 0.f ? (uint32_t)gvr[k] : 0u;
        meta[e] = dzb | ((uint32_t)off << 16);
      }
    }
  };
  prefetch(ph_begin);
  for (int ph0 = ph_begin; ph0 < ph_end; ph0 += kWgRows) {
    const int nph = min(kWgRows, ph_end - ph0);
    const int ncell = nph * kPW;
    __syncthreads();  // previous stage's reads done
    commit(ph0);
    __syncthreads();
    if (ph0 + kWgRows < ph_end) prefetch(ph0 + kWgRows);
    // two cells per step; the next pair's halo reads are issued before this pair's dot products (registers X/Y
    // alternate, so no copies)
    constexpr int NR = wd_nreads<SET>();
    auto pair_meta = [&](int it, uint32_t& m0, uint32_t& m1) {
      m0 = meta[it * kC1 + c];
      m1 = it + 1 < ncell ? meta[(it + 1) * kC1 + c] : (m0 & 0xffff0000u);  // odd tail: dz = 0
    };
    auto pair_fma = [&](uint32_t m0, uint32_t m1, const uint64_t (&a)[NR], const uint64_t (&b)[NR]) {
      if (W == 0) Dsum += bf16_to_f32((uint16_t)(m0 & 0xffffu)) + bf16_to_f32((uint16_t)(m1 & 0xffffu));
      conv1_wd_fma<SET, NR>(__builtin_amdgcn_perm(m1, m0, 0x05040100u), a, b, S);  // dz pair (dz0, dz1)
    };
    uint64_t xa[NR], xb[NR], ya[NR], yb[NR];
    uint32_t xm0, xm1, ym0, ym1;
    pair_meta(0, xm0, xm1);
    conv1_wd_load<SET, NR>(hlo, hhi, xm0, xa);
    conv1_wd_load<SET, NR>(hlo, hhi, xm1, xb);
    for (int it = 0; it < ncell; it += 4) {
      const bool more1 = it + 2 < ncell, more2 = it + 4 < ncell;
      if (more1) {
        pair_meta(it + 2, ym0, ym1);
        conv1_wd_load<SET, NR>(hlo, hhi, ym0, ya);
        conv1_wd_load<SET, NR>(hlo, hhi, ym1, yb);
      }
      pair_fma(xm0, xm1, xa, xb);
      if (!more1) break;
      if (more2) {
        pair_meta(it + 4, xm0, xm1);
        conv1_wd_load<SET, NR>(hlo, hhi, xm0, xa);
        conv1_wd_load<SET, NR>(hlo, hhi, xm1, xb);
      }
      pair_fma(ym0, ym1, ya, yb);
    }
  }
  float* op = part + ((int64_t)slab * kC1 + c) * 126;
  conv1_wd_store<SET>(S, op);
  if (W == 0) op[125] = Dsum;
}

__global__ __launch_bounds__(256, 2) void k_conv1_wgrad_dot(const uint8_t* __restrict__ x8, const int* __restrict__ idx,
                                                         const uint16_t* __restrict__ dp,
                                                         const uint16_t* __restrict__ pout,
                                                         const uint8_t* __restrict__ amax, float* __restrict__ part,
                                                         int nq) {
  __shared__ __attribute__((aligned(256))) uint2 hlo[kWgHalo];
  __shared__ __attribute__((aligned(256))) uint2 hhi[kWgHalo];
  __shared__ uint32_t meta[kWgMeta];
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int q = bid % nq, rest = bid / nq;
  const int pd = rest % kPD, n = rest / kPD;
  const int rq = ((kPH + nq - 1) / nq + kWgRows - 1) / kWgRows * kWgRows;
  const int ph_begin = q * rq, ph_end = min(kPH, ph_begin + rq);
  const int tid = threadIdx.x, c = tid & 63, wid = tid >> 6;
  const uint8_t* xs = x8 + (int64_t)idx[n] * kPZ * kPY * kPX * 8;
  switch (wid) {
    case 0: conv1_wd_wave<0>(xs, dp, pout, amax, part, hlo, hhi, meta, n, pd, tid, c, ph_begin, ph_end, bid_slab(rest, q, nq)); break;
    case 1: conv1_wd_wave<1>(xs, dp, pout, amax, part, hlo, hhi, meta, n, pd, tid, c, ph_begin, ph_end, bid_slab(rest, q, nq)); break;
    case 2: conv1_wd_wave<2>(xs, dp, pout, amax, part, hlo, hhi, meta, n, pd, tid, c, ph_begin, ph_end, bid_slab(rest, q, nq)); break;
    default: conv1_wd_wave<3>(xs, dp, pout, amax, part, hlo, hhi, meta, n, pd, tid, c, ph_begin, ph_end, bid_slab(rest, q, nq)); break;
  }
}

// ------------------------------------------------------------------------------------------------
// k_conv1_wgrad_smf — the same S[c][k] / D[c] slabs on 2:4-sparse MATRIX cores (v_smfmac_f32_32x32x32_bf16).
//
// S[c][k] = sum_pos dY[c][pos] X[2 pos + k] over the conv-output positions of the pooled region, with dY = dz at each
// (cell, channel)'s argmax voxel and 0 elsewhere — an implicit-GEMM weight gradient with M = 64 channels (2 tiles of
// 32), N = 125 taps (4 tiles of 32, 3 dummy columns), K = the conv positions x of one conv row (57 live, 2 k-steps of
// 32).  Along x a group of 4 consecutive positions touches at most 2 pooling cells (cells are 3 wide) and a cell has
// exactly ONE argmax per channel, so each group of 4 K of a channel's dY row holds <= 2 non-zeros: dY is exactly 2:4
// structured-sparse, and smfmac computes the dense-equivalent product at twice the dense MFMA rate (the 32x32x32
// smfmac issues at the cycles of the dense 32x32x16: profiles/r4_smfmac_probe.txt).  This replaces the per-(cell,
// channel) gather on the VALU (k_conv1_wgrad_split: 0 MFMA, ~35 TF/s).
//
// Operand layouts (gfx950, measured with tools/probes/smfmac_probe.hip): B lane (n = l % 32, q = l / 32) holds the 16
// consecutive K = 16 q .. 16 q + 15 of column n; A lane (m = l % 32, p = l / 32) holds 8 compressed values, element j
// covering the 4-group at K = 16 (j >> 2) + 8 p + 4 ((j >> 1) & 1), its position in that group in bits 2j..2j+1 of
// the index VGPR (abid 0).  With K = x, tap k = (kd, kh, kw)'s B fragment is 16 consecutive x of the input's phase
// plane r(k) shifted by jw = kw >> 1.  Misaligned ds_read_b128 are exact on gfx950 but ~11x slower (probe), so the
// stage holds three shifted copies J = jw of the bf16 phase planes (J = 2 only for rw = 0: 20 planes), laid out by
// tools/probes/c1wg_layout_gen.py so that no ds_read_b128 lane group has two taps on one bank.
//
// A is built in registers: per stage each lane reads, for its 8 slots of each M-tile, the (dz, argmax) record of the
// slot's cell from LDS and folds "argmax inside this 4-group" into a row key; per conv row a slot is dz if its key is
// that row, else 0 (the position index word is row-independent).  Block = (sample, pd[, row range]), stage = pooled
// row ph: wave w runs k-step w & 1 over 5 or 4 of the 9 conv rows (alternating per stage), 8 smfmac per row.  Slabs
// are reduced across the 4 waves in a fixed order (deterministic), in the VALU kernel's part[slab][64][126] format.
// Block = 8 waves, warp-specialised and double-buffered (one block per CU): waves 4-7 are producers — they issue the
// global loads of stage s + 2, convert and store stage s + 1 (the 20 bf16 phase-plane copies and the record table)
// into the other LDS buffer; waves 0-3 are consumers — each runs k-step w & 1 of stage s over 5 or 4 of its 9 conv
// rows (8 smfmac per row, the next row's B fragments loaded under the current row's MFMAs).  One barrier per stage.
constexpr int kSmBufBytes = (kC1sBElems * 2 + 15) / 16 * 16;        // one stage's B planes
constexpr int kSmMetaBytes = kPW * kC1 * 4;                          // one stage's record table
constexpr int kSmBytes = 2 * kSmBufBytes + 2 * kSmMetaBytes;
static_assert(kSmBytes >= 4 * 32 * 128 * 4 + 4 * 64 * 4, "reduction scratch must fit in the stage buffers");
static_assert(kSmBytes <= 160 * 1024, "LDS budget");

typedef __bf16 bf16x16 __attribute__((ext_vector_type(16)));
typedef short s16x2 __attribute__((ext_vector_type(2)));

// producer side: one stage's global data held in registers between its load and its LDS store
struct C1sStage {
  uint2 vx[10];        // 10 polyphase voxels (x0 .. x0 + 9) of this thread's staged input row
  uint32_t rpg[5];     // pooled value | dL/dpooled << 16 of this thread's 5 records
  uint32_t ra[5];      // argmax of the records
};

__device__ __forceinline__ void c1s_load(C1sStage& st, const uint8_t* xs, const uint16_t* dp, const uint16_t* pout,
                                         const uint8_t* amax, int64_t rowbase, int pd, int ph, int ptid) {
  const int brow = ptid >> 3, bx0 = 8 * (ptid & 7);
  const int bzi = brow / 5, byi = brow - 5 * (brow / 5);
#pragma unroll
  for (int v = 0; v < 10; ++v) {
    const int x = bx0 + v;
    st.vx[v] = make_uint2(0, 0);
    if (ptid < 200 && x < kPX)
      st.vx[v] = *reinterpret_cast<const uint2*>(xs + (((int64_t)(3 * pd + bzi) * kPY + 3 * ph + byi) * kPX + x) * 8);
  }
  const int rc = ptid & 63, rcg = ptid >> 6;
  const int64_t obase = (rowbase + ph) * kPW * kC1;
#pragma unroll
  for (int u = 0; u < 5; ++u) {
    const int pw = rcg + 4 * u;
    st.rpg[u] = 0;
    st.ra[u] = 0;
    if (pw < kPW) {
      st.rpg[u] = (uint32_t)pout[obase + pw * kC1 + rc] | ((uint32_t)dp[obase + pw * kC1 + rc] << 16);
      st.ra[u] = amax[obase + pw * kC1 + rc];
    }
  }
}

__device__ __forceinline__ void c1s_store(const C1sStage& st, uint16_t* bsm, uint32_t* meta, int ptid, float& Dloc) {
  if (ptid < 200) {
    const int brow = ptid >> 3, bx0 = 8 * (ptid & 7);
    const int bzi = brow / 5, byi = brow - 5 * (brow / 5);
    const int roff = bzi * kC1sZS + byi * kC1sRS + bx0;
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      float f[10];
#pragma unroll
      for (int v = 0; v < 10; ++v) f[v] = u8f(r < 4 ? st.vx[v].x : st.vx[v].y, r & 3);
      const uint32_t e0 = bf2_pack(f[0], f[1]), e1 = bf2_pack(f[2], f[3]), e2 = bf2_pack(f[4], f[5]);
      const uint32_t e3 = bf2_pack(f[6], f[7]), e4 = bf2_pack(f[8], f[9]);
      *reinterpret_cast<uint4*>(&bsm[kC1sPlaneBase[kC1sPlaneOf[0][r]] + roff]) = make_uint4(e0, e1, e2, e3);
      *reinterpret_cast<uint4*>(&bsm[kC1sPlaneBase[kC1sPlaneOf[1][r]] + roff]) =
          make_uint4(bf2_pack(f[1], f[2]), bf2_pack(f[3], f[4]), bf2_pack(f[5], f[6]), bf2_pack(f[7], f[8]));
      if ((r & 1) == 0)
        *reinterpret_cast<uint4*>(&bsm[kC1sPlaneBase[kC1sPlaneOf[2][r]] + roff]) = make_uint4(e1, e2, e3, e4);
    }
  }
  const int rc = ptid & 63, rcg = ptid >> 6;
#pragma unroll
  for (int u = 0; u < 5; ++u) {
    const int pw = rcg + 4 * u;
    const uint32_t dzb = bf16_to_f32((uint16_t)(st.rpg[u] & 0xffffu)) > 0.f ? (st.rpg[u] >> 16) : 0u;
    Dloc += bf16_to_f32((uint16_t)dzb);
    if (pw < kPW) {
      const int a = st.ra[u];
      const int ad = a / 9, ah = (a / 3) % 3, aw = a % 3;
      meta[pw * kC1 + rc] = dzb | ((uint32_t)(3 * pw + aw) << 16) | ((uint32_t)(ad * 3 + ah) << 24);
    }
  }
}

__global__ __launch_bounds__(512, 1) void k_conv1_wgrad_smf(const uint8_t* __restrict__ x8, const int* __restrict__ idx,
                                                           const uint16_t* __restrict__ dp,
                                                           const uint16_t* __restrict__ pout,
                                                           const uint8_t* __restrict__ amax, float* __restrict__ part,
                                                           int nq) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[kSmBytes];
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int q = bid % nq, rest = bid / nq;
  const int pd = rest % kPD, n = rest / kPD;
  const int rq = ((kPH + nq - 1) / nq + kWgRows - 1) / kWgRows * kWgRows;
  const int ph_begin = q * rq, ph_end = min(kPH, ph_begin + rq);
  const int nst = ph_end - ph_begin;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const bool producer = wid >= 4;
  const uint8_t* xs = x8 + (int64_t)idx[n] * kPZ * kPY * kPX * 8;
  const int64_t rowbase = ((int64_t)n * kPD + pd) * kPH;
  auto bbuf = [&](int s) { return reinterpret_cast<uint16_t*>(smem + (s & 1) * kSmBufBytes); };
  auto mbuf = [&](int s) { return reinterpret_cast<uint32_t*>(smem + 2 * kSmBufBytes + (s & 1) * kSmMetaBytes); };

  float Dloc = 0.f;
  f32x16 acc[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int T = 0; T < 4; ++T)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[t][T][i] = 0.f;

  if (producer) {  // ------------------------------------------------------------------------------ producers
    const int ptid = tid - 256;
    C1sStage cur, nxt;
    c1s_load(cur, xs, dp, pout, amax, rowbase, pd, ph_begin, ptid);
    if (nst > 1) c1s_load(nxt, xs, dp, pout, amax, rowbase, pd, ph_begin + 1, ptid);
    c1s_store(cur, bbuf(0), mbuf(0), ptid, Dloc);
    __syncthreads();                                  // stage 0 ready
    for (int s = 0; s < nst; ++s) {
      if (s + 1 < nst) {
        cur = nxt;
        if (s + 2 < nst) c1s_load(nxt, xs, dp, pout, amax, rowbase, pd, ph_begin + s + 2, ptid);
        c1s_store(cur, bbuf(s + 1), mbuf(s + 1), ptid, Dloc);
      }
      __syncthreads();                                // stage s consumed, stage s + 1 ready
    }
  } else {  // ------------------------------------------------------------------------------------- consumers
    const int ks = wid & 1;  // this wave's k-step (x 0-31 or 32-63)
    int bbase[4];
#pragma unroll
    for (int T = 0; T < 4; ++T) {
      int k = kC1sSlotTap[32 * T + (lane & 31)];
      k = k >= 1000 ? k - 1000 : k;
      const int kd = k / 25, kh = (k / 5) % 5, kw = k % 5;
      const int r = ((kd & 1) << 2) | ((kh & 1) << 1) | (kw & 1);
      bbase[T] = kC1sPlaneBase[kC1sPlaneOf[kw >> 1][r]] + (kd >> 1) * kC1sZS + (kh >> 1) * kC1sRS + 16 * (lane >> 5) +
                 32 * ks;
    }
    // this lane's 4-groups g at x = xg (slot 0 = the group's first cell, slot 1 = the next one)
    const int xg0 = 32 * ks + 8 * (lane >> 5);
    __syncthreads();                                  // stage 0 ready
    for (int s = 0; s < nst; ++s) {
      const uint16_t* bsm = bbuf(s);
      const uint32_t* meta = mbuf(s);
      // per-stage A operands: per 4-group g the slots' dz values packed as one bf16 pair (W) and their conv rows as
      // one-hot bits (low half slot 0, high half slot 1; none when the argmax falls outside the group); the index
      // word holds each argmax's position in its group
      uint32_t wv[2][4], oh[2][4], ix[2] = {0u, 0u};
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int xg = xg0 + 16 * (g >> 1) + 4 * (g & 1);
        const int C0 = xg / 3;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          uint32_t w = 0, o = 0;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int C = C0 + h;
            const uint32_t mw = C < kPW ? meta[C * kC1 + 32 * t + (lane & 31)] : 0u;
            const uint32_t d = ((mw >> 16) & 0xffu) - (uint32_t)xg;
            const bool in = d <= 3u && C < kPW;
            w |= (in ? (mw & 0xffffu) : 0u) << (16 * h);
            o |= (in ? (1u << (mw >> 24)) : 0u) << (16 * h);
            ix[t] |= (in ? d : 0u) << (2 * (2 * g + h));
          }
          wv[t][g] = w;
          oh[t][g] = o;
        }
      }
      const int half = (wid >> 1) ^ (s & 1);
      const int rr0 = half ? 5 : 0, rr1 = half ? 9 : 5;
      // B fragments of row rr: software-pipelined one row ahead
      bf16x16 bv[4], bn[4];
      auto loadB = [&](int rr, bf16x16 (&dst)[4]) {
        const int roff = (rr / 3) * kC1sZS + (rr % 3) * kC1sRS;
#pragma unroll
        for (int T = 0; T < 4; ++T) {
          const uint16_t* bp = &bsm[bbase[T] + roff];
          const bf16x8 lo = *reinterpret_cast<const bf16x8*>(bp);
          const bf16x8 hi = *reinterpret_cast<const bf16x8*>(bp + 8);
          dst[T] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
        }
      };
      loadB(rr0, bv);
      for (int rr = rr0; rr < rr1; ++rr) {
        if (rr + 1 < rr1) loadB(rr + 1, bn);
        // A of row rr: shifting a one-hot pair left by 15 - rr puts bit rr of each half into that half's sign bit;
        // a packed 16-bit arithmetic shift by 15 makes it a 0xffff / 0 mask per slot (3 VALU per 4-group)
        bf16x8 av[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          uint32_t w[4];
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const s16x2 sh = __builtin_bit_cast(s16x2, oh[t][g] << (15 - rr));
            const s16x2 m = sh >> (s16x2){15, 15};
            w[g] = wv[t][g] & __builtin_bit_cast(uint32_t, m);
          }
          av[t] = __builtin_bit_cast(bf16x8, make_uint4(w[0], w[1], w[2], w[3]));
        }
#pragma unroll
        for (int T = 0; T < 4; ++T) {
          acc[0][T] = __builtin_amdgcn_smfmac_f32_32x32x32_bf16(av[0], bv[T], acc[0][T], (int)ix[0], 0, 0);
          acc[1][T] = __builtin_amdgcn_smfmac_f32_32x32x32_bf16(av[1], bv[T], acc[1][T], (int)ix[1], 0, 0);
        }
#pragma unroll
        for (int T = 0; T < 4; ++T) bv[T] = bn[T];
      }
      __syncthreads();                                // stage s consumed, stage s + 1 ready
    }
  }
  // fixed-order reduction over the 4 consumer waves, one M-tile (32 channels) at a time, and D over the producers'
  // 4 cell groups
  float* red = reinterpret_cast<float*>(smem);           // [4 w][32 m][128 slot]
  float* dred = red + 4 * 32 * 128;                      // [4 cg][64 c]
  float* op = part + (int64_t)bid_slab(rest, q, nq) * kC1 * 126;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    __syncthreads();
    if (!producer) {
#pragma unroll
      for (int T = 0; T < 4; ++T)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int m = 8 * (i >> 2) + 4 * (lane >> 5) + (i & 3);
          red[(wid * 32 + m) * 128 + 32 * T + (lane & 31)] = acc[t][T][i];
        }
    } else if (t == 0) {
      const int ptid = tid - 256;
      dred[(ptid >> 6) * 64 + (ptid & 63)] = Dloc;
    }
    __syncthreads();
    for (int e = tid; e < 32 * 126; e += 512) {
      const int m = e / 126, k = e - 126 * (e / 126);
      float v;
      if (k < 125) {
        const int sl = kC1sTapSlot[k];
        v = red[(0 * 32 + m) * 128 + sl] + red[(1 * 32 + m) * 128 + sl];
        v += red[(2 * 32 + m) * 128 + sl] + red[(3 * 32 + m) * 128 + sl];
      } else {
        const int c = 32 * t + m;
        v = dred[0 * 64 + c] + dred[1 * 64 + c] + dred[2 * 64 + c] + dred[3 * 64 + c];
      }
      op[(32 * t + m) * 126 + k] = v;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// k_conv1_wgrad_mx — the conv1 weight-gradient slabs on 2:4-sparse matrix cores with the argmax ROW in the sparsity
// index (v_smfmac_f32_32x32x32_bf16).
//
// K of S[c][k] = sum_pos dY[c][pos] X[2 pos + k] is ordered (dh, x, dd): a 4-group of K is the three conv positions
// dd = 0, 1, 2 of one pooling-window column (dh, x) plus a pad slot.  A window column holds at most one argmax per
// channel (a cell has one argmax, at (dd, dh, dw)), so every 4-group of a channel's dY row has <= 1 non-zero — legal
// 2:4 — and its position in the group IS the argmax's dd.  Hence:
//  * A (dY, 32 channels x 32 K per M-tile) is the same for the three dh of a pooled row: element 2i = dz of the
//    cell covering the lane's x (dY = dz only where the argmax column is x: aw == x mod 3), element 2i + 1 = 0.  Only
//    the 2-bit indices change with dh: dd where the argmax is in row dh, else 3 (the pad slot, whose B value is 0).
//    The three index words come from ONE 32-bit OR per (channel, x) and stage — fields at bits 4i (dh 0), 16 + 4i
//    (dh 1, read with abid 1) and 4i + 2 (dh 2: the dead element's field, read after a 2-bit shift) — instead of a
//    per-row value mask (k_conv1_wgrad_smf: 23 VALU per smfmac);
//  * B (input, 32 K x 32 taps per N-tile) comes from "dd-slot images": per jd = kd >> 1 an image of 4-slot groups
//    [z' = 3 pd + jd + dd for dd = 0..2, 0] per (y', phase r, x'), so a tap's 16 K (4 groups at x' = x + jw) are 32
//    contiguous bytes, 8-B aligned for every jw: no shifted copies, four ds_read_b64 per fragment, and all 125 taps
//    share one A (4 N-tiles).
// The images keep y' rows in an 8-slot ring (3 new rows per pooled row, 5 at a new pd slab); per-plane offsets and the
// tap -> column order (conv1_mx_layout.h, tools/probes/c1mx_layout_gen.py) put the 32 taps of every N-tile on 32
// distinct LDS bank pairs.  Cost: 4/3 of the minimal K (the pad slot) = 192 smfmac per pooled row and sample.
//
// Block = 8 waves, one per CU by LDS = (sample, range of pd slabs); wave w owns x = 8w .. 8w + 7 (one 32-K k-step per
// dh) for all 64 channels (2 M-tiles) x 128 tap columns (4 N-tiles): 24 smfmac per pooled row, 128 accumulators.  The
// next pooled row's staging (3 y' rows: uint8 -> bf16 into the three images; the row's (dz, argmax) records) is
// loaded into registers before this row's MFMAs and stored after them: one barrier per pooled row.  Output
// part[block][64][126] (125 S + D), summed per client by k_conv1_wgrad_fin.
constexpr int kMxRing = 8;                         // y' ring slots (+ 2 mirrors of slots 0, 1: see below)
constexpr int kMxSS8 = kMxSS * 8;                  // bytes per slot
constexpr int kMxImgBytes = (kMxRing + 2) * kMxSS8;
constexpr int kMxRecCells = kPW + 1;               // + a zero cell for the x beyond the pooled region
constexpr int kMxRecBytes = kMxRecCells * kC1 * 8;
constexpr int kMxLdsBytes = 135168;                // also the [8 waves][32][128] fp32 reduction scratch
static_assert(kMxImgBytes + 2 * kMxRecBytes + 32 * 4 <= kMxLdsBytes, "LDS budget");
static_assert(8 * 32 * 128 * 4 <= kMxLdsBytes && kMxLdsBytes <= 163840, "reduction scratch");
static_assert(2 * kMxSS8 + 24 < 65536, "dh offsets must fit the ds_read immediate");
constexpr int kMxRecItems = kPW * 16;              // (cell, channel quad) record items of a pooled row

struct MxRec { uint2 pv, gv; uint32_t av; };      // 4 channels of one cell: pooled, dL/dpooled (bf16), argmax

// y' row task (row, phase half H) of one wave: lane = x' (< 61); the 5 (H = 0) or 4 (H = 1) z' = 3 pd + z bytes
template <int H>
__device__ __forceinline__ void mx_load_row(uint32_t (&v)[5], const uint8_t* xs, int pd, int y, int xp) {
  // lanes x' >= 61 read x' = 60 (their stores are skipped): unpredicated loads
  const uint8_t* src = xs + (((int64_t)(3 * pd) * kPY + y) * kPX + min(xp, kPX - 1)) * 8 + 4 * H;
  constexpr int64_t zs = (int64_t)kPY * kPX * 8;
#pragma unroll
  for (int z = 0; z < 5; ++z) v[z] = (H == 0 || z < 4) ? *reinterpret_cast<const uint32_t*>(src + z * zs) : 0u;
}

// into the images at ring slot s (wave-uniform; and its mirror s + 8 for s < 2): group [z' jd, jd + 1, jd + 2, 0] of
// plane 8 jd + r, straight-line stores with immediate plane offsets
template <int H>
__device__ __forceinline__ void mx_store_row(const uint32_t (&v)[5], uint8_t* img, int s, int xp) {
  constexpr int NJ = H == 0 ? 3 : 2;
  uint2 g[NJ][4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    float f[5];
#pragma unroll
    for (int z = 0; z < NJ + 2; ++z) f[z] = u8f(v[z], r);
#pragma unroll
    for (int jd = 0; jd < NJ; ++jd) g[jd][r] = make_uint2(bf2_pack(f[jd], f[jd + 1]), __float_as_uint(f[jd + 2]) >> 16);
  }
  if (xp >= kPX) return;  // x' >= 61 stays the zero of the initialisation
  uint8_t* base = img + s * kMxSS8 + xp * 8;
#pragma unroll
  for (int jd = 0; jd < NJ; ++jd)
#pragma unroll
    for (int r = 0; r < 4; ++r) *reinterpret_cast<uint2*>(base + kMxPO[8 * jd + 4 * H + r] * 8) = g[jd][r];
  if (s < 2) {
    base += 8 * kMxSS8;
#pragma unroll
    for (int jd = 0; jd < NJ; ++jd)
#pragma unroll
      for (int r = 0; r < 4; ++r) *reinterpret_cast<uint2*>(base + kMxPO[8 * jd + 4 * H + r] * 8) = g[jd][r];
  }
}

__device__ __forceinline__ void mx_load_rec(MxRec& st, const uint16_t* dp, const uint16_t* pout, const uint8_t* amax,
                                            int n, int pd, int ph, int item) {
  const int pw = item >> 4, cq = item & 15;
  const int64_t o = ((((int64_t)n * kPD + pd) * kPH + ph) * kPW + pw) * kC1 + 4 * cq;
  st.pv = *reinterpret_cast<const uint2*>(pout + o);
  st.gv = *reinterpret_cast<const uint2*>(dp + o);
  st.av = *reinterpret_cast<const uint32_t*>(amax + o);
}

// record = (dz as bf16 in the low half, lut[argmax]): dz = dL/dpooled where the pooled value is > 0 (ReLU), else 0
__device__ __forceinline__ void mx_store_rec(const MxRec& st, uint8_t* rec, const uint32_t* lut, int item) {
  const int pw = item >> 4, cq = item & 15;
  uint32_t o[8];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t pw2 = j < 2 ? st.pv.x : st.pv.y, gw2 = j < 2 ? st.gv.x : st.gv.y;
    const uint32_t p16 = (pw2 >> (16 * (j & 1))) & 0xffffu, g16 = (gw2 >> (16 * (j & 1))) & 0xffffu;
    o[2 * j] = (int16_t)p16 > 0 ? g16 : 0u;
    o[2 * j + 1] = lut[(st.av >> (8 * j)) & 0xffu];
  }
  uint4* d = reinterpret_cast<uint4*>(rec + (pw * kC1 + 4 * cq) * 8);
  d[0] = make_uint4(o[0], o[1], o[2], o[3]);
  d[1] = make_uint4(o[4], o[5], o[6], o[7]);
}

// stage S of a block (flat over its pd slabs x 23 pooled rows): slab, pooled row, ring offset (+5 per slab: the
// first 5 rows of a new slab go to slots the last stage of the old one leaves free / frees at its end)
struct MxStage {
  int pd, ph, ro;
};
__device__ __forceinline__ MxStage mx_stage(int pd0, int S) {
  const int sl = S / kPH;
  return MxStage{pd0 + sl, S - sl * kPH, (5 * sl) & 7};
}

template <int DBG>
__global__ __launch_bounds__(512, 1) void k_conv1_wgrad_mx(const uint8_t* __restrict__ x8, const int* __restrict__ idx,
                                                          const uint16_t* __restrict__ dp,
                                                          const uint16_t* __restrict__ pout,
                                                          const uint8_t* __restrict__ amax, float* __restrict__ part,
                                                          int npb, int nblk) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[kMxLdsBytes];
  uint8_t* img = smem;
  uint8_t* recb = smem + kMxImgBytes;
  uint32_t* lut = reinterpret_cast<uint32_t*>(smem + kMxImgBytes + 2 * kMxRecBytes);
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int n = bid / nblk, jb = bid - n * nblk;
  const int pd0 = jb * npb, pd1 = min(kPD, pd0 + npb);
  const int nstage = (pd1 - pd0) * kPH;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int m = lane & 31, q = lane >> 5;
  const uint8_t* xs = x8 + (int64_t)idx[n] * kPZ * kPY * kPX * 8;

  // ---- initialisation: zero images (x' >= 61, pads), the constant ones plane [1, 1, 1, 0] of every slot, the zero
  // cell of both record buffers, and the argmax lut: a -> the dd ^ 3 index field at the bit of its row dh (0: bit 0,
  // 1: bit 16, 2: bit 2; "no argmax here" = 0 -> index 3 after the final NOT) and its column aw in bits 30-31
  for (int e = tid; e < kMxImgBytes / 16; e += 512) reinterpret_cast<uint4*>(img)[e] = make_uint4(0, 0, 0, 0);
  __syncthreads();
  for (int e = tid; e < (kMxRing + 2) * 66; e += 512) {
    const int s = e / 66, xp = e - 66 * s;
    *reinterpret_cast<uint2*>(img + s * kMxSS8 + (kMxPO[20] + xp) * 8) = make_uint2(0x3f803f80u, 0x3f80u);
  }
  if (tid < 27) {
    const int ad = tid / 9, ah = (tid / 3) % 3, aw = tid % 3;
    lut[tid] = ((uint32_t)(ad ^ 3) << (ah == 0 ? 0 : ah == 1 ? 16 : 2)) | ((uint32_t)aw << 30);
  }
  if (tid >= 64 && tid < 64 + 2 * kC1) {
    const int b = (tid - 64) / kC1, c = (tid - 64) % kC1;
    *reinterpret_cast<uint2*>(recb + b * kMxRecBytes + (kPW * kC1 + c) * 8) = make_uint2(0, 0);
  }

  // ---- per-lane constants of the MFMA part (wave w = k-step: x = 8 w .. 8 w + 7)
  int roff[4], awi[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int gi = (i & 1) + 2 * q + 4 * (i >> 1);  // A element 2i covers 4-group gi = 2q, 2q + 1, 4 + 2q, 5 + 2q
    const int x = 8 * w + gi;
    const int cell = x < 3 * kPW ? x / 3 : kPW;
    roff[i] = (cell * kC1 + m) * 8;
    awi[i] = x % 3;
  }
  int col8[4], jhT[4];
#pragma unroll
  for (int T = 0; T < 4; ++T) {
    int k = kMxTap[32 * T + m];
    if (k == 999) {  // the ones column: D = sum of dz (any slot, any x)
      col8[T] = (kMxPO[20] + 8 * w + 4 * q) * 8;
      jhT[T] = 0;
      continue;
    }
    k = k >= 1000 ? k - 1000 : k;
    const int kd = k / 25, kh = (k / 5) % 5, kw = k % 5;
    const int p = 8 * (kd >> 1) + 4 * (kd & 1) + 2 * (kh & 1) + (kw & 1);
    col8[T] = (kMxPO[p] + 8 * w + 4 * q + (kw >> 1)) * 8;
    jhT[T] = kh >> 1;
  }

  // ---- staging roles.  The two waves of a SIMD (w, w + 4) run in opposite phases: waves 0-3 stage the NEXT pooled
  // row after their MFMAs (loads issued at the start of the row), waves 4-7 before them (loaded one row earlier), so
  // one wave's conversion VALU runs beside the other's matrix work.  Waves 0-2 / 4-6: y' row tasks (row, half) 0-2 /
  // 3-5 of the 3 new rows; waves 3 / 7: record items {l, 128 + l, 256 + l} / {64 + l, 192 + l}.  At a new slab its
  // rows 0, 1 (tasks 6-9) are written by waves 0-3 after the last barrier of the old slab.  Each role runs its own
  // copy of the loop with unconditional (index-clamped) loads: loads under role branches made the compiler copy the
  // loaded registers at the joins behind a vmcnt(0) wait, exposing the HBM latency before every row's MFMAs.
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const int wl = wu & 3;

  // prologue: stage 0 (its 5 rows and records) by every wave
  __syncthreads();  // lut, zeros
  {
    const MxStage st = mx_stage(pd0, 0);
    for (int t = wu; t < 10; t += 8) {
      uint32_t v[5];
      if ((t & 1) == 0) {
        mx_load_row<0>(v, xs, st.pd, t >> 1, lane);
        mx_store_row<0>(v, img, ((t >> 1) + st.ro) & 7, lane);
      } else {
        mx_load_row<1>(v, xs, st.pd, t >> 1, lane);
        mx_store_row<1>(v, img, ((t >> 1) + st.ro) & 7, lane);
      }
    }
    for (int it = tid; it < kMxRecItems; it += 512) {
      MxRec r;
      mx_load_rec(r, dp, pout, amax, n, st.pd, st.ph, it);
      mx_store_rec(r, recb, lut, it);
    }
  }

  f32x16 acc[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int T = 0; T < 4; ++T)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[t][T][e] = 0.f;

  auto run = [&](auto early_c, auto meta_c) {
    constexpr bool EARLY = decltype(early_c)::value, META = decltype(meta_c)::value;
    constexpr int NREC = META ? (EARLY ? 2 : 3) : 0;
    const int rec0 = EARLY ? 64 : 0;
    const int bt = META ? 0 : (EARLY ? 3 : 0) + wl;  // y' row task: row bt >> 1 of the new rows, phase half bt & 1
    const int bh = bt & 1;
    // two register sets, alternating per pooled row, so a row's staging data is loaded two rows before it is stored
    // (one row of MFMA work did not cover the HBM latency: the same kernel ran 3.60 vs 2.43 ms with the loads
    // redirected to L2-resident rows).  The row loop is unrolled by 2 so the sets never need register copies.
    struct Set {
      uint32_t bv[5], xv[5];
      MxRec rv[NREC > 0 ? NREC : 1];
    };
    Set sa, sb;
    auto load_stage = [&](Set& X, int S) {  // S clamped to a valid stage: the loads never sit under a branch
      S = min(S, nstage - 1);
      const MxStage st = mx_stage(pd0, DBG ? 0 : S);  // DBG: diagnostic, every row re-reads stage 0 (L2 hits)
      if constexpr (META) {
#pragma unroll
        for (int k = 0; k < NREC; ++k)
          mx_load_rec(X.rv[k], dp, pout, amax, n, st.pd, st.ph, min(rec0 + 128 * k + lane, kMxRecItems - 1));
      } else {
        const uint8_t* src = xs + (((int64_t)(3 * st.pd) * kPY + 3 * st.ph + 2 + (bt >> 1)) * kPX +
                                   min(lane, kPX - 1)) * 8 + 4 * bh;
#pragma unroll
        for (int z = 0; z < 5; ++z) X.bv[z] = *reinterpret_cast<const uint32_t*>(src + z * (int64_t)kPY * kPX * 8);
      }
      if constexpr (!EARLY) {  // rows 0, 1 of S's slab (used only when S starts a new slab)
        const uint8_t* src = xs + (((int64_t)(3 * st.pd) * kPY + (wl >> 1)) * kPX + min(lane, kPX - 1)) * 8 + 4 * (wl & 1);
#pragma unroll
        for (int z = 0; z < 5; ++z) X.xv[z] = *reinterpret_cast<const uint32_t*>(src + z * (int64_t)kPY * kPX * 8);
      }
    };
    auto store_stage = [&](const Set& X, int S) {
      const MxStage st = mx_stage(pd0, S);
      if constexpr (META) {
#pragma unroll
        for (int k = 0; k < NREC; ++k)
          if (rec0 + 128 * k + lane < kMxRecItems)
            mx_store_rec(X.rv[k], recb + (S & 1) * kMxRecBytes, lut, rec0 + 128 * k + lane);
      } else {
        const int sl = (3 * st.ph + 2 + (bt >> 1) + st.ro) & 7;
        if (bh == 0) mx_store_row<0>(X.bv, img, sl, lane);
        else mx_store_row<1>(X.bv, img, sl, lane);
      }
    };
    // row s: early waves store row s + 1 from set X (loaded at row s - 2) and reload X with row s + 3; late waves load
    // row s + 2 into X and store row s + 1 from Y (loaded at row s - 1) after their MFMAs
    auto body = [&](int s, Set& X, Set& Y) {
      const MxStage cur = mx_stage(pd0, s);
      if constexpr (EARLY) {
        if (s + 1 < nstage) store_stage(X, s + 1);
        load_stage(X, s + 3);
      } else {
        load_stage(X, s + 2);
      }
      // ---- A of this pooled row (both M-tiles): values and the three index words
      const uint8_t* rb = recb + (s & 1) * kMxRecBytes;
      uint32_t av[2][4], om[2] = {0u, 0u};
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint64_t r = *((lds_u64*)(rb + roff[i] + 256 * t));
          const uint32_t rx = (uint32_t)r, ry = (uint32_t)(r >> 32);
          av[t][i] = rx;
          om[t] |= ((ry >> 30) == (uint32_t)awi[i]) ? (ry << (4 * i)) : 0u;
        }
      bf16x8 A[2];
      int W0[2], W2[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        A[t] = __builtin_bit_cast(bf16x8, make_uint4(av[t][0], av[t][1], av[t][2], av[t][3]));
        W0[t] = (int)~om[t];
        W2[t] = (int)(~om[t] >> 2);
      }
      // B base of each N-tile at dh = 0: ring slot of y' = 3 ph + jh; dh = 1, 2 are +1, +2 slots (immediate
      // offsets; the mirrors 8, 9 of slots 0, 1 make that valid across the ring's end)
      int bb[4];
#pragma unroll
      for (int T = 0; T < 4; ++T) bb[T] = ((3 * cur.ph + cur.ro + jhT[T]) & 7) * kMxSS8 + col8[T];
#pragma unroll
      for (int dh = 0; dh < 3; ++dh) {
        bf16x16 B[4];
#pragma unroll
        for (int T = 0; T < 4; ++T) {
          lds_u64* bp = (lds_u64*)(img + bb[T] + dh * kMxSS8);
          typedef uint64_t u64x4 __attribute__((ext_vector_type(4)));
          const u64x4 bq = {bp[0], bp[1], bp[2], bp[3]};
          B[T] = __builtin_bit_cast(bf16x16, bq);
        }
#pragma unroll
        for (int T = 0; T < 4; ++T)
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            if (dh == 0) acc[t][T] = __builtin_amdgcn_smfmac_f32_32x32x32_bf16(A[t], B[T], acc[t][T], W0[t], 0, 0);
            else if (dh == 1) acc[t][T] = __builtin_amdgcn_smfmac_f32_32x32x32_bf16(A[t], B[T], acc[t][T], W0[t], 0, 1);
            else acc[t][T] = __builtin_amdgcn_smfmac_f32_32x32x32_bf16(A[t], B[T], acc[t][T], W2[t], 0, 0);
          }
      }
      if constexpr (!EARLY)
        if (s + 1 < nstage) store_stage(Y, s + 1);
      __syncthreads();
      if (s + 1 < nstage) {
        const MxStage nx = mx_stage(pd0, s + 1);
        if (nx.ph == 0) {  // rows 0, 1 of the new slab take the slots rows 69, 70 of the old one just released
          if constexpr (!EARLY) {
            const int sl = ((wl >> 1) + nx.ro) & 7;
            if ((wl & 1) == 0) mx_store_row<0>(Y.xv, img, sl, lane);
            else mx_store_row<1>(Y.xv, img, sl, lane);
          }
          __syncthreads();
        }
      }
    };
    if constexpr (EARLY) {
      load_stage(sa, 1);
      load_stage(sb, 2);
    } else {
      load_stage(sb, 1);
    }
    __syncthreads();
    int s = 0;
    for (; s + 1 < nstage; s += 2) {
      body(s, sa, sb);
      body(s + 1, sb, sa);
    }
    if (s < nstage) body(s, sa, sb);
  };
  using T1 = std::integral_constant<bool, true>;
  using F1 = std::integral_constant<bool, false>;
  if (wu >= 4) {
    if (wl == 3) run(T1{}, T1{});
    else run(T1{}, F1{});
  } else {
    if (wl == 3) run(F1{}, T1{});
    else run(F1{}, F1{});
  }

  // ---- fixed-order reduction over the 8 waves (one M-tile at a time through the whole LDS); column 999 = D
  float* red = reinterpret_cast<float*>(smem);
  float* op = part + (int64_t)bid * kC1 * 126;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    __syncthreads();
#pragma unroll
    for (int T = 0; T < 4; ++T)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int mm = 8 * (e >> 2) + 4 * q + (e & 3);
        red[(w * 32 + mm) * 128 + 32 * T + m] = acc[t][T][e];
      }
    __syncthreads();
    for (int e = tid; e < 32 * 128; e += 512) {
      const int mm = e >> 7, col = e & 127;
      int k = kMxTap[col];
      if (k >= 1000) continue;
      float v = 0.f;
#pragma unroll
      for (int ww = 0; ww < 8; ++ww) v += red[(ww * 32 + mm) * 128 + col];
      op[(32 * t + mm) * 126 + (k == 999 ? 125 : k)] = v;
    }
  }
}

// pd slabs per block: the whole sample when there are >= 4 samples per CU (one reduction per sample), else fewer so
// the grid still covers the chip ~4 times
int conv1_wgrad_mx_npb(int NB) { return std::max(1, std::min(kPD, NB * kPD / (4 * 256))); }

// conv1 weight-gradient kernel: 0 = VALU gather (k_conv1_wgrad_split), 1 = 2:4 smfmac (k_conv1_wgrad_smf),
// 2 = 2:4 smfmac with the argmax row in the index (k_conv1_wgrad_mx); -1 = the environment default
static int g_c1wg_mode = -1;
void conv1_wgrad_mode(int mode) { g_c1wg_mode = mode; }

int conv1_wgrad_nq(int NB) { return (int64_t)NB * kPD < 4 * 256 * 4 ? 2 : 1; }

void conv1_wgrad(uintptr_t x8, uintptr_t idx, uintptr_t dp, uintptr_t pout, uintptr_t amax, int NB, int B,
                 uintptr_t part, uintptr_t w125, uintptr_t mu, uintptr_t covw, uintptr_t invstd, uintptr_t theta,
                 int64_t ldt, int64_t off_g, uintptr_t grad, int64_t ldg, int64_t goff_w, int64_t goff_bias,
                 int64_t goff_g, int64_t goff_b, float wscale, uintptr_t emean, uintptr_t stream) {
  hipStream_t s = as_stream(stream);
  const int nq = conv1_wgrad_nq(NB);
  // NIDT_C1WG_UNROLL=2|4: unrolled cell loop (A/B: loads of the next cell overlap the current cell's FMAs)
  static const int unr = [] {
    const char* e = getenv("NIDT_C1WG_UNROLL");
    return e ? atoi(e) : 1;
  }();
  // NIDT_C1WG_DOT=1: the cell-paired bf16 dot-product kernel (A/B record: 4.52 ms vs 3.98 ms for this one at
  // 64 clients, profiles/r3_ab_conv1_wgrad_dot.txt — v_dot2c_f32_bf16 does not issue at the v_fma rate)
  static const bool dot = [] {
    const char* e = getenv("NIDT_C1WG_DOT");
    return e && atoi(e) == 1;
  }();
#define NIDT_C1WG(U)                                                                                                \
  hipLaunchKernelGGL(k_conv1_wgrad_split<U>, dim3(kPD * NB * nq), dim3(256), 0, s, ptr<const uint8_t>(x8),          \
                     ptr<const int>(idx), ptr<const uint16_t>(dp), ptr<const uint16_t>(pout), ptr<const uint8_t>(amax), \
                     ptr<float>(part), nq)
  static const int smf_env = [] {
    const char* e = getenv("NIDT_C1WG_SMF");
    return e ? atoi(e) : 0;
  }();
  // NIDT_C1WG_MX=0 falls back from the argmax-row smfmac kernel (default) to the VALU gather
  static const int mx_env = [] {
    const char* e = getenv("NIDT_C1WG_MX");
    return e ? atoi(e) : 1;
  }();
  const int mode = g_c1wg_mode >= 0 ? g_c1wg_mode : (smf_env == 1 ? 1 : mx_env == 1 ? 2 : 0);
  const bool smf = mode == 1;
  int nslab = B * kPD * nq;  // part slabs per client
  if (mode == 2) {
    const int npb = conv1_wgrad_mx_npb(NB), nblk = (kPD + npb - 1) / npb;
    NIDT_REQUIRE(nblk <= kPD * nq, "conv1_wgrad: part buffer");
    static const int dbg = [] {
      const char* e = getenv("NIDT_C1WG_DBG");
      return e ? atoi(e) : 0;
    }();
    if (dbg)
      hipLaunchKernelGGL(k_conv1_wgrad_mx<1>, dim3(NB * nblk), dim3(512), 0, s, ptr<const uint8_t>(x8),
                         ptr<const int>(idx), ptr<const uint16_t>(dp), ptr<const uint16_t>(pout),
                         ptr<const uint8_t>(amax), ptr<float>(part), npb, nblk);
    else
      hipLaunchKernelGGL(k_conv1_wgrad_mx<0>, dim3(NB * nblk), dim3(512), 0, s, ptr<const uint8_t>(x8),
                         ptr<const int>(idx), ptr<const uint16_t>(dp), ptr<const uint16_t>(pout),
                         ptr<const uint8_t>(amax), ptr<float>(part), npb, nblk);
    nslab = B * nblk;
  } else if (smf)
    hipLaunchKernelGGL(k_conv1_wgrad_smf, dim3(kPD * NB * nq), dim3(512), 0, s, ptr<const uint8_t>(x8),
                       ptr<const int>(idx), ptr<const uint16_t>(dp), ptr<const uint16_t>(pout),
                       ptr<const uint8_t>(amax), ptr<float>(part), nq);
  else if (dot)
    hipLaunchKernelGGL(k_conv1_wgrad_dot, dim3(kPD * NB * nq), dim3(256), 0, s, ptr<const uint8_t>(x8),
                       ptr<const int>(idx), ptr<const uint16_t>(dp), ptr<const uint16_t>(pout),
                       ptr<const uint8_t>(amax), ptr<float>(part), nq);
  else if (unr == 4) NIDT_C1WG(4); else if (unr == 2) NIDT_C1WG(2); else NIDT_C1WG(1);
#undef NIDT_C1WG
  NIDT_CHECK(hipGetLastError());
  const int G = NB / B;
  // client g's slabs are contiguous: B samples x (19 pd x nq row ranges | nblk pd ranges)
  hipLaunchKernelGGL(k_conv1_wgrad_fin, dim3(kC1, G), dim3(64 * kFinW), 0, s, ptr<const float>(part), nslab,
                     ptr<const float>(w125), ptr<const float>(mu), ptr<const float>(covw), ptr<const float>(invstd),
                     ptr<const float>(theta), ldt, off_g, ptr<float>(grad), ldg, goff_w, goff_bias, goff_g, goff_b,
                     wscale, ptr<const float>(emean));
  NIDT_CHECK(hipGetLastError());
}

}  // namespace nidt
