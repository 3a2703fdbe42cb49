// Weight gradients of the 1x1x1 stride-1 convolutions of the client-batched 3D ResNet (config 5: the Bottleneck's
// conv1 / conv3 and the stride-1 projection; reference block fedml_api/model/cv/salient_models.py:8-139):
//     dW[g][n][k] = sum_m dY[g][m][n] X[g][m][k]      dY [G][Mg][N], X [G][Mg][K] channels-last bf16 rows
// a GEMM whose contraction runs over the Mg ~ 142 k positions of a client, with a [N][K] <= 256 x 256 output.
// At 1 FLOP/B per operand byte it is HBM-bound, so the design is gemm1x1.hip's streaming one turned around:
//  * a block owns (client g, n-tile, k-tile, m-chunk mb) and walks m-tiles mb, mb + nMB, ... (persistent): the
//    output tile stays in the accumulators; the dY and X rows of an m-tile flow through a 3-stage LDS-DMA ring
//    (buffer_load ... lds from inline asm, counted waits), two tiles' loads in flight while one is multiplied;
//  * the MFMA operands want the position axis in the k slots: both are read with ds_read_b64_tr_b16 from
//    [BM positions][64 channels] groups of 128-B rows (the 16-B chunk swizzle of k_conv_wgrad_dma);
//  * every m-tile is read once per (n-tile, k-tile) block: the tile is as large as the accumulators allow
//    (up to 256 x 128), so dY / X are re-read at most (K / KT) / (N / NT) times;
//  * the nMB chunk partials go through k_wgrad_reduce (PyTorch [Cout][Cin] rows, scale), or straight into the
//    gradient rows with one chunk.
// The general LDS-DMA wgrad (k_conv_wgrad_dma, 256 k-columns per block) ran these at 3.1-5.4 TB/s and, at Cin = 64,
// with three of its four waves on all-zero k-columns (profiles/r5_config5_bn_wgrad_bandwidth.txt).
#include "common.h"
#include "dma.h"

namespace nidt {

constexpr int kW1NST = 3;  // m-tile stages

__device__ __forceinline__ int swz_w1(int r) { return (r & 2) | ((r >> 1) & 4); }

template <int N>
__device__ __forceinline__ void w1_wait_vm() {  // s_waitcnt vmcnt(N) lgkmcnt(0), visible to the waitcnt pass
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | ((N >> 4) << 14));
}

__device__ __forceinline__ bf16x8 w1_tr_pair(const uint16_t* p0, const uint16_t* p1) {
  typedef short v4s __attribute__((ext_vector_type(4)));
  v4s lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p0));
  v4s hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(p1));
  typedef short v8s __attribute__((ext_vector_type(8)));
  v8s r = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, r);
}

struct Wg1Args {
  const uint16_t* x;   // [G][Mg][K]
  const uint16_t* dy;  // [G][Mg][N]
  float* part;         // [nMB][G][N][K] (nMB > 1)
  float* grad;         // nMB == 1: grad[g ldg + off + n K + k] = scale dW
  int64_t ldg, off;
  float scale;
  int G, Mg, N, K, nNT, nKT, nMB;
};

// WR x WC waves, wave tile (16 TCO) x (16 TP): block tile NT = 16 WR TCO output channels x KT = 16 WC TP input
// channels; BM positions per m-tile (a multiple of 32: one MFMA k-step per 32)
template <int WR, int WC, int TCO, int TP, int BM>
__global__ __launch_bounds__(64 * WR * WC, 1) void k_wgrad1x1(Wg1Args a) {
  constexpr int NWV = WR * WC, NT = 16 * WR * TCO, KT = 16 * WC * TP;
  constexpr int NGD = NT / 64, NGX = KT / 64, GRP = BM * 64;  // 64-channel groups per stage, elements per group
  constexpr int STE = (NGD + NGX) * GRP;                      // elements per stage
  constexpr int NIT = (NGD + NGX) * (BM / 8);                 // DMA instructions per stage
  constexpr int NIW = NIT / NWV;                              // ... per wave
  static_assert(NT % 64 == 0 && KT % 64 == 0 && BM % 32 == 0 && NIT % NWV == 0, "tile shape");
  __shared__ __attribute__((aligned(16))) uint16_t sS0[STE];
  __shared__ __attribute__((aligned(16))) uint16_t sS1[STE];
  __shared__ __attribute__((aligned(16))) uint16_t sS2[STE];

  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int kt = id % a.nKT, r1 = id / a.nKT;
  const int nt = r1 % a.nNT, r2 = r1 / a.nNT;
  const int mb = r2 % a.nMB, g = r2 / a.nMB;
  const int n0 = nt * NT, k0 = kt * KT;
  const int nmt = (a.Mg + BM - 1) / BM;
  const int T = mb < nmt ? (nmt - 1 - mb) / a.nMB + 1 : 0;  // m-tiles of this block
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / WC, wc = wid % WC;
  const int lrow = lane >> 3, slot = lane & 7;

  const i32x4_t rx = make_rsrc(a.x + (int64_t)g * a.Mg * a.K, (uint32_t)a.Mg * a.K * 2);
  const i32x4_t rd = make_rsrc(a.dy + (int64_t)g * a.Mg * a.N, (uint32_t)a.Mg * a.N * 2);
  // this wave's DMA instructions j = wid NIW + i: group j / (BM / 8) (dY groups first), 8-row block j % (BM / 8)
  int dcol[NIW], drow[NIW], dlds[NIW];
  bool isd[NIW];
#pragma unroll
  for (int i = 0; i < NIW; ++i) {
    const int j = wid * NIW + i, gi = j / (BM / 8), rb = j % (BM / 8);
    const int r = rb * 8 + lrow;
    isd[i] = gi < NGD;
    const int cb = isd[i] ? n0 + 64 * gi : k0 + 64 * (gi - NGD);
    dcol[i] = (cb + ((slot ^ swz_w1(r)) << 3)) * 2;
    drow[i] = r;
    dlds[i] = gi * GRP + rb * 512;
  }
  auto issue = [&](int t, uint16_t* sb) {  // m-tile t of this block (past the last: out-of-range, zeros)
    const int m0 = t < T ? (mb + t * a.nMB) * BM : a.Mg;
#pragma unroll
    for (int i = 0; i < NIW; ++i) {
      const int m = m0 + drow[i];
      const uint32_t m0v = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint16_t*)(sb + dlds[i]);
      const int voff = m < a.Mg ? m * (isd[i] ? a.N : a.K) * 2 + dcol[i] : kBufOOB;
      if (isd[i])
        asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m0v), "v"(voff), "s"(rd)
                     : "memory");
      else
        asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m0v), "v"(voff), "s"(rx)
                     : "memory");
    }
  };

  f32x4 acc[TCO][TP];
#pragma unroll
  for (int i = 0; i < TCO; ++i)
#pragma unroll
    for (int j = 0; j < TP; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed fragment reads (k_conv_wgrad_dma): 16-lane group gq covers positions 8 gq .. 8 gq + 7 of a 32-position
  // k-step (two 4-row reads); lane 4 qq + pp reads row qq, columns 4 pp .. 4 pp + 3 of its 16-channel fragment
  const int gq = lane >> 4, li = lane & 15, qq = li >> 2, pp = li & 3;
  const int rr0 = 8 * gq + qq;
  auto frag = [&](const uint16_t* grp, int cb, int kk) {  // cb: fragment's first channel within the 64-group
    const int ra = 32 * kk + rr0, rb = ra + 4, c = (cb >> 3) + (pp >> 1);
    return w1_tr_pair(grp + ra * 64 + ((c ^ swz_w1(ra)) << 3) + (pp & 1) * 4,
                      grp + rb * 64 + ((c ^ swz_w1(rb)) << 3) + (pp & 1) * 4);
  };
  auto tile = [&](int t, const uint16_t* sx, uint16_t* sn) {
    issue(t + 2, sn);
#pragma unroll
    for (int kk = 0; kk < BM / 32; ++kk) {
      bf16x8 fa[TCO], fb[TP];
#pragma unroll
      for (int i = 0; i < TCO; ++i) {
        const int c = wr * 16 * TCO + 16 * i;
        fa[i] = frag(sx + (c >> 6) * GRP, c & 63, kk);
      }
#pragma unroll
      for (int j = 0; j < TP; ++j) {
        const int c = wc * 16 * TP + 16 * j;
        fb[j] = frag(sx + (NGD + (c >> 6)) * GRP, c & 63, kk);
      }
#pragma unroll
      for (int i = 0; i < TCO; ++i)
#pragma unroll
        for (int j = 0; j < TP; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    // stage t + 1 landed (the younger NIW loads are stage t + 2's), every wave done reading stage t
    w1_wait_vm<NIW>();
    __builtin_amdgcn_s_barrier();
  };
  if (T > 0) {  // block-uniform
    issue(0, sS0);
    issue(1, sS1);
    w1_wait_vm<NIW>();
    __builtin_amdgcn_s_barrier();
    int t = 0;
    for (; t + 3 <= T; t += 3) {
      tile(t, sS0, sS2);
      tile(t + 1, sS1, sS0);
      tile(t + 2, sS2, sS1);
    }
    if (t < T) tile(t, sS0, sS2);
    if (t + 1 < T) tile(t + 1, sS1, sS0);
    w1_wait_vm<0>();  // the trailing out-of-range DMAs, before the block's LDS is released
  }
  // lane (fr, fq): rows (channels n) 16 i + 4 fq + r, column (channel k) 16 j + fr of each fragment
  const int fr = lane & 15, fq = lane >> 4;
  const bool direct = a.nMB == 1;
  float* out = direct ? a.grad + (int64_t)g * a.ldg + a.off
                      : a.part + ((int64_t)mb * a.G + g) * (int64_t)a.N * a.K;
  const float sc = direct ? a.scale : 1.f;
#pragma unroll
  for (int i = 0; i < TCO; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + wr * 16 * TCO + 16 * i + 4 * fq + r;
#pragma unroll
      for (int j = 0; j < TP; ++j) out[(int64_t)n * a.K + k0 + wc * 16 * TP + 16 * j + fr] = acc[i][j][r] * sc;
    }
}

// tile configurations: (WR, WC, TCO, TP, BM) -> NT x KT, waves, LDS
struct W1Cfg {
  int id, NT, KT;
};
static const W1Cfg kW1Cfgs[] = {
    {0, 64, 64},    // <2, 2, 2, 2, 128>: 4 waves, 3 x 32 KB
    {1, 256, 64},   // <4, 2, 4, 2, 64>: 8 waves, 3 x 40 KB
    {2, 64, 256},   // <1, 8, 4, 2, 64>: 8 waves, 3 x 40 KB
    {3, 128, 128},  // <2, 4, 4, 2, 64>: 8 waves, 3 x 32 KB
    {4, 128, 256},  // <2, 4, 4, 4, 32>: 8 waves, 3 x 24 KB
    {5, 256, 128},  // <4, 2, 4, 4, 32>: 8 waves, 3 x 24 KB
};

// the tile that reads the fewest operand bytes (Mg (N nKT + K nNT)); ties -> the larger tile
static int w1_pick(int N, int K) {
  int best = -1;
  int64_t best_b = 0;
  for (const W1Cfg& c : kW1Cfgs) {
    if (N % c.NT || K % c.KT) continue;
    const int64_t b = (int64_t)N * (K / c.KT) + (int64_t)K * (N / c.NT);
    if (best < 0 || b < best_b || (b == best_b && c.NT * c.KT > kW1Cfgs[best].NT * kW1Cfgs[best].KT)) {
      best = c.id;
      best_b = b;
    }
  }
  return best;
}

int wgrad1x1_ok(int N, int K) { return (N % 64 == 0 && K % 64 == 0 && N <= 2048 && K <= 2048) ? 1 : 0; }

// m-chunks per (client, tile): about 512 blocks in all (one or two resident per CU), at least 8 m-tiles per block
int wgrad1x1_chunks(int G, int64_t Mg, int N, int K) {
  NIDT_REQUIRE(wgrad1x1_ok(N, K), "wgrad1x1_chunks: channels must be multiples of 64 (<= 2048)");
  const W1Cfg& c = kW1Cfgs[w1_pick(N, K)];
  const int bm = c.id == 0 ? 128 : (c.id >= 4 ? 32 : 64);
  const int tiles = G * (N / c.NT) * (K / c.KT);
  const int64_t nmt = (Mg + bm - 1) / bm;
  const int want = (512 + tiles - 1) / tiles;
  return (int)std::max<int64_t>(1, std::min<int64_t>(want, nmt / 8));
}

// part: [nMB][G][N][K] fp32 (nMB = wgrad1x1_chunks > 1), reduced by k_wgrad_reduce into grad rows
// grad[g ldg + off + n K + k] = scale dW; with one chunk the kernel writes the rows itself
void k_wgrad_reduce_launch(const float* part, int nsplit, int G, int Cout, int Cin, int kt, float* grad, int64_t ldg,
                           int64_t off, float scale, hipStream_t s);

void wgrad1x1_g(uintptr_t x, uintptr_t dy, uintptr_t part, uintptr_t grad, int64_t ldg, int64_t off, int G, int64_t Mg,
                int N, int K, int nMB, float scale, uintptr_t stream) {
  NIDT_REQUIRE(wgrad1x1_ok(N, K), "wgrad1x1_g: channels must be multiples of 64 (<= 2048)");
  NIDT_REQUIRE(Mg > 0 && Mg * std::max(N, K) * 2 < (int64_t(1) << 31),
               "wgrad1x1_g: a client's rows must stay below 2 GB (32-bit in-client offsets)");
  NIDT_REQUIRE(nMB >= 1 && (nMB == 1 || part), "wgrad1x1_g: nMB > 1 needs the partial buffer");
  const W1Cfg& c = kW1Cfgs[w1_pick(N, K)];
  Wg1Args a;
  a.x = ptr<const uint16_t>(x); a.dy = ptr<const uint16_t>(dy); a.part = ptr<float>(part); a.grad = ptr<float>(grad);
  a.ldg = ldg; a.off = off; a.scale = scale;
  a.G = G; a.Mg = (int)Mg; a.N = N; a.K = K; a.nNT = N / c.NT; a.nKT = K / c.KT; a.nMB = nMB;
  const int64_t nwg = (int64_t)G * a.nNT * a.nKT * nMB;
  NIDT_REQUIRE(nwg < (1ll << 31), "wgrad1x1_g: grid too large");
  hipStream_t s = as_stream(stream);
  const dim3 grid((unsigned)nwg);
  switch (c.id) {
    case 0: hipLaunchKernelGGL((k_wgrad1x1<2, 2, 2, 2, 128>), grid, dim3(256), 0, s, a); break;
    case 1: hipLaunchKernelGGL((k_wgrad1x1<4, 2, 4, 2, 64>), grid, dim3(512), 0, s, a); break;
    case 2: hipLaunchKernelGGL((k_wgrad1x1<1, 8, 4, 2, 64>), grid, dim3(512), 0, s, a); break;
    case 3: hipLaunchKernelGGL((k_wgrad1x1<2, 4, 4, 2, 64>), grid, dim3(512), 0, s, a); break;
    case 4: hipLaunchKernelGGL((k_wgrad1x1<2, 4, 4, 4, 32>), grid, dim3(512), 0, s, a); break;
    default: hipLaunchKernelGGL((k_wgrad1x1<4, 2, 4, 4, 32>), grid, dim3(512), 0, s, a); break;
  }
  NIDT_CHECK(hipGetLastError());
  if (nMB > 1) k_wgrad_reduce_launch(ptr<const float>(part), nMB, G, N, K, 1, ptr<float>(grad), ldg, off, scale, s);
}

}  // namespace nidt
