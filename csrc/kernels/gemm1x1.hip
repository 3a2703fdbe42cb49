// 1x1x1 stride-1 convolutions of the client-batched 3D ResNet (config 5: the Bottleneck's conv1 / conv3 and the
// stride-1 projection, forward and data gradient) as per-client GEMMs on channels-last rows:
//     Y[g][m][n] = sum_k X[g][m][k] W[g][n][k]      X [G][Mg][K], W [G][N][K] (the packed image), Y [G][Mg][N], bf16
// (reference block: fedml_api/model/cv/salient_models.py:8-139).  The general LDS-DMA conv kernel ran these at
// 14 % MFMA busy and ~1.1 TB/s: one tap and one or a few 64-deep k-steps per block, so its per-row tap/geometry
// setup, its one-stage-per-block load latency and its epilogue were the whole block (profiles/r4_pmc_config5.txt).
// At K = 64 / 256 with N = 256 / 64 (layer 1, 4.5 M rows per step) the GEMM is HBM-bound (51 FLOP/B), so the design
// streams:
//  * a block owns (client g, n-tile) and walks m-tiles mb, mb + nMB, ... (persistent): the [BN][K] weight tile is
//    staged into LDS ONCE; X m-tiles [BM][K] flow through a 3-stage LDS-DMA ring (buffer_load ... lds, raw buffer
//    resources: rows past Mg read zeros), so two tiles' loads are in flight while one is multiplied;
//  * no per-row geometry: row m of client g is at byte (g Mg + m) K 2 (64-bit client base, 32-bit in-client
//    offsets; the host checks Mg K 2 < 2^31);
//  * 8 waves = 2 (m halves) x 4 (n quarters); the MFMA A operand is the weight tile (rows = output channels), B the X
//    rows, so a lane's accumulator holds 4 consecutive channels of one row: 8-B bf16 stores, 128 contiguous bytes per
//    row per wave;
//  * LDS rows are 128 B (one 64-deep k chunk) with the 16-B chunk swizzle (r >> 1) & 7 of conv3d.hip's DMA tiles;
//  * the waits are counted (vmcnt over this wave's own DMA + stores) and one s_barrier per tile.
#include "common.h"
#include "dma.h"

namespace nidt {

constexpr int kG1NST = 3;  // X stages

__device__ __forceinline__ int swz_g1(int r) { return (r >> 1) & 7; }

// s_waitcnt vmcnt(N) lgkmcnt(0) as the builtin (gfx9 encoding: vmcnt[3:0] | expcnt[6:4] = 7 | lgkmcnt[11:8] = 0 |
// vmcnt[5:4] << 14), which the compiler's waitcnt pass sees: with an inline-asm wait it still believes the DMA
// is in flight and adds a vmcnt(0) in front of the first LDS read of every tile
template <int N>
__device__ __forceinline__ void g1_wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | ((N >> 4) << 14));
}

// The tile loop's VMEM traffic — the LDS-DMA of X / W and the Y stores — is issued from inline asm, invisible to the
// compiler's waitcnt pass, and ordered only by the kernel's own counted waits (g1_wait_vm): with the intrinsic DMA
// and plain stores the pass put a vmcnt(1) at the head of every tile (wait for every VMEM op but the DMA just issued,
// i.e. the next tile's DMA and the previous tile's stores), which left one tile in flight and cut the K = 64, N = 256
// shape to ~3 TB/s.  No other code in the kernel uses M0 (the DMA's LDS base).
template <class T>
__device__ __forceinline__ void g1_dma16(i32x4_t rsrc, int voffset, T* lds_wave_base) {
  const uint32_t m0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) T*)lds_wave_base;
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m0), "v"(voffset), "s"(rsrc)
               : "memory");
}

// [STATS] the following BatchNorm's training statistics from the epilogue: per-lane sums of the stored (bf16)
// outputs and their squares over every row the block writes, reduced over the 16 row lanes (DPP/shuffle) and the two
// m-half waves (LDS) into part[mb][g][N][2] = the chunk partials of bnr.hip's k_bnr_finalize (nchunk = nMB), which
// replaces that layer's k_bnr_partial pass over the whole output (a 2.33 GB read per layer-1 conv3 at config 5)
template <int BN, int NKC, int BM, bool STATS>
__global__ __launch_bounds__(512, 1) void k_gemm1x1(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                     uint16_t* __restrict__ y, int G, int Mg, int N, int nNT,
                                                     int nMB, float* __restrict__ part) {
  constexpr int K = 64 * NKC;
  constexpr int W_ELEMS = NKC * BN * 64, X_ELEMS = NKC * BM * 64;
  constexpr int NIW = NKC * BN / 64;           // weight DMA instructions per wave
  constexpr int NIX = NKC * BM / 64;           // X DMA instructions per wave per stage
  constexpr int WN = BN / 4, WM = BM / 2;      // wave tile: WM rows x WN channels
  constexpr int NSUB = WN / 16, MSUB = WM / 16;
  constexpr int NSTORE = NSUB * MSUB;          // 8-B stores per wave per tile
  static_assert(NIX >= 1 && NIW >= 1 && NSUB >= 1 && MSUB >= 1, "tile shape");
  __shared__ __attribute__((aligned(16))) uint16_t sW[W_ELEMS];
  // three separate stage arrays, each used at a compile-time position of the 3x-unrolled tile loop: the DMA into
  // one and the fragment reads of another are then provably disjoint, so the compiler's waitcnt pass does not put a
  // vmcnt(0) (a wait for the DMA just issued) in front of the reads
  __shared__ __attribute__((aligned(16))) uint16_t sX0[X_ELEMS];
  __shared__ __attribute__((aligned(16))) uint16_t sX1[X_ELEMS];
  __shared__ __attribute__((aligned(16))) uint16_t sX2[X_ELEMS];

  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int nt = id % nNT, rest = id / nNT;
  const int mb = rest % nMB, g = rest / nMB;
  const int n0 = nt * BN;
  const int nmt = (Mg + BM - 1) / BM;
  const int T = mb < nmt ? (nmt - 1 - mb) / nMB + 1 : 0;  // m-tiles of this block
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wid & 3, wm = wid >> 2;
  const int lrow = lane >> 3, slot = lane & 7;

  if (T == 0) {  // block-uniform
    if (STATS)
      for (int c = tid; c < 2 * BN; c += 512) part[(((int64_t)mb * G + g) * N + n0) * 2 + c] = 0.f;
    return;
  }
  float s1[NSUB][4], s2[NSUB][4];
#pragma unroll
  for (int i = 0; i < NSUB; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) s1[i][r] = s2[i][r] = 0.f;
  const i32x4_t rx = make_rsrc(x + (int64_t)g * Mg * K, (uint32_t)Mg * K * 2);
  const i32x4_t rw = make_rsrc(w + (int64_t)g * N * K, (uint32_t)N * K * 2);
  // weight tile: instruction j = (k chunk, 8-row group) of [NKC][BN][64]
#pragma unroll
  for (int i = 0; i < NIW; ++i) {
    const int j = wid * NIW + i, kc = j / (BN / 8), rg = j % (BN / 8);
    const int r = rg * 8 + lrow;
    g1_dma16(rw, ((n0 + r) * K + kc * 64 + ((slot ^ swz_g1(r)) << 3)) * 2, sW + kc * BN * 64 + rg * 512);
  }
  // X stage of m-tile t into stage array sb
  auto issue_x = [&](int t, uint16_t* sb) {
    const int m0 = (mb + t * nMB) * BM;
#pragma unroll
    for (int i = 0; i < NIX; ++i) {
      const int j = wid * NIX + i, kc = j / (BM / 8), rg = j % (BM / 8);
      const int r = rg * 8 + lrow;
      const int m = m0 + r;
      g1_dma16(rx, m < Mg ? (m * K + kc * 64 + ((slot ^ swz_g1(r)) << 3)) * 2 : kBufOOB, sb + kc * BM * 64 + rg * 512);
    }
  };
  // every tile issues the DMA of tile t + 2, past the block's last tile as all-out-of-range loads (zeros, no HBM
  // traffic), so the vmcnt arithmetic is the same constant in every tile
  issue_x(0, sX0);
  issue_x(1, sX1);
  g1_wait_vm<NIX>();
  __builtin_amdgcn_s_barrier();

  const int fr = lane & 15, fq = lane >> 4;
  // one tile: DMA of tile t + 2 into sn, MFMAs from sx, stores, wait for tile t + 1, barrier
  auto tile = [&](int t, const uint16_t* sx, uint16_t* sn) {
    issue_x(t + 2, sn);
    f32x4 acc[NSUB][MSUB];
#pragma unroll
    for (int i = 0; i < NSUB; ++i)
#pragma unroll
      for (int j = 0; j < MSUB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kc = 0; kc < NKC; ++kc)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 fa[NSUB], fb[MSUB];
#pragma unroll
        for (int i = 0; i < NSUB; ++i) {
          const int r = wn * WN + 16 * i + fr;
          fa[i] = *reinterpret_cast<const bf16x8*>(&sW[kc * BN * 64 + r * 64 + (((4 * kk + fq) ^ swz_g1(r)) << 3)]);
        }
#pragma unroll
        for (int j = 0; j < MSUB; ++j) {
          const int r = wm * WM + 16 * j + fr;
          fb[j] = *reinterpret_cast<const bf16x8*>(&sx[kc * BM * 64 + r * 64 + (((4 * kk + fq) ^ swz_g1(r)) << 3)]);
        }
#pragma unroll
        for (int i = 0; i < NSUB; ++i)
#pragma unroll
          for (int j = 0; j < MSUB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    // epilogue: lane = (row fr of each 16-row m-subtile, channels 4 fq .. 4 fq + 3 of each n-subtile)
    const int mrow = (mb + t * nMB) * BM + wm * WM + fr;
#pragma unroll
    for (int j = 0; j < MSUB; ++j) {
      const int m = mrow + 16 * j;
      if (m < Mg) {
        uint16_t* yp = y + ((int64_t)g * Mg + m) * N + n0 + wn * WN + 4 * fq;
#pragma unroll
        for (int i = 0; i < NSUB; ++i)
        {
          const uint2 v = make_uint2(pack_bf16x2(acc[i][j][0], acc[i][j][1]), pack_bf16x2(acc[i][j][2], acc[i][j][3]));
          asm volatile("global_store_dwordx2 %0, %1, off" ::"v"(yp + 16 * i), "v"(v) : "memory");
          if (STATS) {
            const float q[4] = {__uint_as_float(v.x << 16), __uint_as_float(v.x & 0xffff0000u),
                                __uint_as_float(v.y << 16), __uint_as_float(v.y & 0xffff0000u)};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              s1[i][r] += q[r];
              s2[i][r] = fmaf(q[r], q[r], s2[i][r]);
            }
          }
        }
      }
    }
    // stage t + 1 landed (younger: the stage t + 2 DMA and this tile's stores; only the client's partial last m-tile,
    // which is its block's last tile and has no successor to wait for, can issue fewer stores), every wave done with t
    g1_wait_vm<NIX + NSTORE>();
    __builtin_amdgcn_s_barrier();
  };
  int t = 0;
  for (; t + 3 <= T; t += 3) {
    tile(t, sX0, sX2);
    tile(t + 1, sX1, sX0);
    tile(t + 2, sX2, sX1);
  }
  if (t < T) tile(t, sX0, sX2);
  if (t + 1 < T) tile(t + 1, sX1, sX0);
  if (STATS) {
#pragma unroll
    for (int i = 0; i < NSUB; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          s1[i][r] += __shfl_xor(s1[i][r], o, 64);
          s2[i][r] += __shfl_xor(s2[i][r], o, 64);
        }
    // [2 m halves][BN][2] in sX0.  The last tile issued (out-of-range) DMAs for tiles T and T + 1, one of which can
    // target sX0 (T % 3 == 2) and land late: drain every wave's DMAs and meet at a barrier before the first write
    g1_wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    float* red = reinterpret_cast<float*>(sX0);
    if (fr == 0) {
#pragma unroll
      for (int i = 0; i < NSUB; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = wn * WN + 16 * i + 4 * fq + r;
          red[(wm * BN + c) * 2] = s1[i][r];
          red[(wm * BN + c) * 2 + 1] = s2[i][r];
        }
    }
    __syncthreads();
    for (int c = tid; c < 2 * BN; c += 512)
      part[(((int64_t)mb * G + g) * N + n0) * 2 + c] = red[c] + red[2 * BN + c];
  }
}

// (BN, NKC, BM) of a (K, N) shape, or 0 when the weight tile does not fit (K >= 1024: the general conv kernel)
static int g1_cfg(int K, int N, int& BN, int& NKC, int& BM) {
  if (K % 64 || N % 64) return 0;
  NKC = K / 64;
  BM = 64;
  const int bn_cap = NKC == 1 ? 256 : NKC == 2 ? 256 : NKC == 4 ? 128 : NKC == 8 ? 64 : 0;
  if (!bn_cap) return 0;
  if (NKC == 8) BM = 32;
  BN = (N % 256 == 0 && bn_cap >= 256) ? 256 : (N % 128 == 0 && bn_cap >= 128) ? 128 : 64;
  return 1;
}

int gemm1x1_ok(int K, int N) {
  int BN, NKC, BM;
  return g1_cfg(K, N, BN, NKC, BM);
}

// m-tile groups per (client, n-tile): about two blocks per CU in all (one resident per CU at the large LDS
// configs) — enough tiles per block to keep the DMA ring full, enough blocks to fill the 256 CUs.  Also the chunk
// count of the [STATS] partials.
int gemm1x1_chunks(int G, int64_t Mg, int K, int N) {
  int BN, NKC, BM;
  NIDT_REQUIRE(g1_cfg(K, N, BN, NKC, BM), "gemm1x1_chunks: unsupported (K, N)");
  const int nNT = N / BN;
  const int nmt = (int)((Mg + BM - 1) / BM);
  const int target = 512;
  return std::max(1, std::min(nmt, (target + G * nNT - 1) / (G * nNT)));
}

// part: 0, or [gemm1x1_chunks][G][N][2] fp32 BatchNorm partial sums of the output (see [STATS])
void gemm1x1_g(uintptr_t x, uintptr_t w, uintptr_t y, int G, int64_t Mg, int K, int N, uintptr_t part,
               uintptr_t stream) {
  int BN, NKC, BM;
  NIDT_REQUIRE(g1_cfg(K, N, BN, NKC, BM), "gemm1x1_g: unsupported (K, N)");
  NIDT_REQUIRE(Mg > 0 && Mg * K * 2 < (int64_t(1) << 31) && Mg * N * 2 < (int64_t(1) << 31),
               "gemm1x1_g: a client's rows must stay below 2 GB (32-bit in-client offsets)");
  const int nNT = N / BN;
  const int nMB = gemm1x1_chunks(G, Mg, K, N);
  const dim3 grid(G * nNT * nMB), block(512);
  hipStream_t s = as_stream(stream);
#define G1(BN_, NKC_, BM_)                                                                                     \
  if (BN == BN_ && NKC == NKC_ && BM == BM_) {                                                                 \
    if (part)                                                                                                  \
      hipLaunchKernelGGL((k_gemm1x1<BN_, NKC_, BM_, true>), grid, block, 0, s, ptr<const uint16_t>(x),         \
                         ptr<const uint16_t>(w), ptr<uint16_t>(y), G, (int)Mg, N, nNT, nMB, ptr<float>(part)); \
    else                                                                                                       \
      hipLaunchKernelGGL((k_gemm1x1<BN_, NKC_, BM_, false>), grid, block, 0, s, ptr<const uint16_t>(x),        \
                         ptr<const uint16_t>(w), ptr<uint16_t>(y), G, (int)Mg, N, nNT, nMB, nullptr);          \
    NIDT_CHECK(hipGetLastError());                                                                             \
    return;                                                                                                    \
  }
  G1(256, 1, 64) G1(128, 1, 64) G1(64, 1, 64)
  G1(256, 2, 64) G1(128, 2, 64) G1(64, 2, 64)
  G1(128, 4, 64) G1(64, 4, 64)
  G1(64, 8, 32)
#undef G1
  NIDT_REQUIRE(false, "gemm1x1_g: no kernel for this tile");
}

}  // namespace nidt
