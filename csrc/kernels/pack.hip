// Batched per-step weight packing of a client-grouped network: every conv layer of G clients' fp32 parameter rows
// (PyTorch layout [Cout][cin][taps]) becomes the bf16 MFMA A-operand images of the conv kernels in TWO launches per
// step (all layers at once), instead of two launches per layer:
//   plain  wp[g][Cout][kt][Cin_p]   (forward; input channels cin..Cin_p-1 zero),
//   dgrad  wt[g][Cin_p][kt][Cout]   with the taps in slot order: slot_of_tap = kt-1-t for a stride-1 conv (the
//          flipped kernel), the sub-pixel phase order of conv_s2_phase_plan (conv3d.hip) for a stride-2 3x3(x3)
//          conv, identity for 1x1.
// The layer of a block comes from a small descriptor table (prefix block counts), so one grid covers layers of
// different shapes; the transposes go through a padded 64x64 LDS tile (coalesced reads and writes).
#include "common.h"

namespace nidt {

struct PackDesc {
  int64_t src_off;   // element offset of the layer in a theta row
  int64_t wp_off;    // element offset of wp (all G clients) in the packed buffer
  int64_t wt_off;    // ... of wt, or -1 (no dgrad image)
  int cout, cin_p, cin_src, kt;
  int blk_plain;     // first block of this layer in the plain grid (Cout blocks per layer; 0 blocks for 1x1 layers
                     // packed by k_pack_plain1)
  int blk_t;         // first block in the transpose grid (ceil(Cin_p/64) * ceil(Cout/64) * kt blocks per layer)
  int blk_plain1;    // first block in the 1x1 grid (ceil(Cout / pack1_rows(Cin_p)) blocks; 0 for the other layers)
  int slot[27];
};
static_assert(sizeof(PackDesc) % 8 == 0, "PackDesc alignment");

// layer of block b in one of the three grids: the last layer whose prefix block count is <= b (prefixes are
// non-decreasing; layers without blocks in a grid repeat the running count and are never the last such layer)
__device__ __forceinline__ int find_layer(const PackDesc* d, int n, int b, int grid) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    const int p = grid == 0 ? d[mid].blk_plain : (grid == 1 ? d[mid].blk_t : d[mid].blk_plain1);
    if (p <= b) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// rows per block of the 1x1 grid: about 8 K elements per block (host twin: resnet2d_hip.WeightPacker)
__host__ __device__ constexpr int pack1_rows(int cin_p) { return cin_p >= 8192 ? 1 : 8192 / cin_p; }

// plain: block (layer row co, channel chunk of pack_cc channels, client g).  The chunk's fp32 source [cc][kt]
// (contiguous in the PyTorch row) is staged in LDS and written as kt runs of image channels (16-B stores).  The round-4 kernel staged
// a whole row per block (kt x Cin x 4 B: 55 KB for a 512-channel 3x3x3 layer), which held it to two blocks per CU and
// ~1.2 TB/s (7.2 ms per config-5 pack); 64-channel chunks need 7 KB (kt = 27) and give Cout x Cin/64 blocks per layer.
// chunk width: as many 64-channel groups as keep the staged chunk within 8 K floats (32 KB), at least one — whole
// rows for the 3x3 layers of the 2-D ResNet (a 64-channel chunk there is 2.3 KB, and the 4096 blocks per 512x512
// layer per client made the pack 5x slower than the per-row kernel), 256 channels for a 512-channel 3x3x3 layer
__host__ __device__ inline int pack_cc(int cin_p, int kt) {
  const int cc = ((8192 / kt) / 64) * 64;
  return cc < 64 ? 64 : (cc > cin_p ? cin_p : cc);
}
__global__ __launch_bounds__(256) void k_pack_plain(const PackDesc* __restrict__ desc, int nd,
                                                    const float* __restrict__ theta, int64_t ldt, int G,
                                                    uint16_t* __restrict__ out) {
  extern __shared__ float row[];  // [CC][kt]
  const int li = find_layer(desc, nd, blockIdx.x, 0);
  const PackDesc& d = desc[li];
  const int Cin = d.cin_p, kt = d.kt, cs = d.cin_src, K = kt * Cin;
  const int CC = pack_cc(Cin, kt), nch = (Cin + CC - 1) / CC;
  const int b = blockIdx.x - d.blk_plain, co = b / nch, ci0 = (b - co * nch) * CC, g = blockIdx.y;
  const int cw = min(CC, Cin - ci0);          // image channels of this chunk
  const int cc = max(0, min(CC, cs - ci0));   // source channels of this chunk
  const int n = cc * kt;
  const float* src = theta + (int64_t)g * ldt + d.src_off + ((int64_t)co * cs + ci0) * kt;
  if ((reinterpret_cast<uintptr_t>(src) & 15) == 0 && n % 4 == 0) {  // 16-B source loads
    for (int e = 4 * threadIdx.x; e < n; e += 4 * 256)
      *reinterpret_cast<float4*>(row + e) = *reinterpret_cast<const float4*>(src + e);
  } else {
    for (int e = threadIdx.x; e < n; e += 256) row[e] = src[e];
  }
  __syncthreads();
  uint16_t* dst = out + d.wp_off + ((int64_t)g * d.cout + co) * K + ci0;
  if (Cin % 8 == 0 && (d.wp_off & 7) == 0) {  // 16-B stores: 8 channels of one tap per lane
    const int nq = cw / 8;
    for (int e = threadIdx.x; e < kt * nq; e += 256) {
      const int t = e / nq, c = (e - t * nq) * 8;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = c + j < cc ? row[(c + j) * kt + t] : 0.f;
      *reinterpret_cast<uint4*>(dst + (int64_t)t * Cin + c) = make_uint4(
          pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
    }
    return;
  }
  for (int e = threadIdx.x; e < kt * cw; e += 256) {
    const int t = e / cw, c = e - t * cw;
    dst[(int64_t)t * Cin + c] = f32_to_bf16(c < cc ? row[c * kt + t] : 0.f);
  }
}

// plain image of the 1x1 layers (kt = 1: the PyTorch row [cin] is already the image row [1][Cin_p] up to the zero
// channels): no transpose and no LDS; block (layer, R = pack1_rows consecutive rows, client g) converts R x Cin_p
// elements, 8 per lane (two 16-B loads, one 16-B store).  The per-row kernel above staged each of these short rows
// in an LDS buffer sized for the largest 3x3x3 row, which held the whole pack to two blocks per CU.
__global__ __launch_bounds__(256) void k_pack_plain1(const PackDesc* __restrict__ desc, int nd,
                                                     const float* __restrict__ theta, int64_t ldt, int G,
                                                     uint16_t* __restrict__ out) {
  const int li = find_layer(desc, nd, blockIdx.x, 2);
  const PackDesc& d = desc[li];
  const int Cin = d.cin_p, cs = d.cin_src, R = pack1_rows(Cin);
  const int r0 = (blockIdx.x - d.blk_plain1) * R, nr = min(R, d.cout - r0), g = blockIdx.y;
  const float* src = theta + (int64_t)g * ldt + d.src_off + (int64_t)r0 * cs;
  uint16_t* dst = out + d.wp_off + ((int64_t)g * d.cout + r0) * Cin;
  const int n8 = nr * (Cin >> 3);
  const bool vec = cs == Cin && (reinterpret_cast<uintptr_t>(src) & 15) == 0;
  for (int e = threadIdx.x; e < n8; e += 256) {
    const int row = e / (Cin >> 3), c = (e - row * (Cin >> 3)) * 8;
    float v[8];
    if (vec) {
      const float4 lo = *reinterpret_cast<const float4*>(src + (int64_t)row * cs + c);
      const float4 hi = *reinterpret_cast<const float4*>(src + (int64_t)row * cs + c + 4);
      v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w; v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = c + j < cs ? src[(int64_t)row * cs + c + j] : 0.f;
    }
    *reinterpret_cast<uint4*>(dst + (int64_t)row * Cin + c) =
        make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
  }
}

// transposed: block (64 ci x 64 co tile, tap t, client g) reads the plain image written by k_pack_plain.  Global
// traffic in 16-B pieces (8 channels per lane: a 64-wide tile row is 8 lanes), the transpose through a padded LDS tile
// (2-B column reads there, where bandwidth is plentiful); 2-B global accesses ran at ~2 TB/s.
__global__ __launch_bounds__(256) void k_pack_trans(const PackDesc* __restrict__ desc, int nd, int G,
                                                    uint16_t* __restrict__ out) {
  __shared__ uint16_t tile[64][72];  // [co][ci], rows padded to 144 B (16-B aligned, staggered banks)
  const int li = find_layer(desc, nd, blockIdx.x, 1);
  const PackDesc& d = desc[li];
  const int Cin = d.cin_p, Cout = d.cout, kt = d.kt;
  const int nci = (Cin + 63) / 64;
  int b = blockIdx.x - d.blk_t;
  const int t = b % kt;
  b /= kt;
  const int ci0 = (b % nci) * 64, co0 = (b / nci) * 64;
  const int g = blockIdx.y;
  const uint16_t* wp = out + d.wp_off + (int64_t)g * Cout * kt * Cin;
  uint16_t* wt = out + d.wt_off + (int64_t)g * Cin * kt * Cout;
  const int q = threadIdx.x & 7, r0 = threadIdx.x >> 3;  // 8-channel piece q of tile row r0 (+ 32)
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = r0 + 32 * h, co = co0 + r, ci = ci0 + 8 * q;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (co < Cout && ci < Cin) v = *reinterpret_cast<const uint4*>(wp + ((int64_t)co * kt + t) * Cin + ci);
    *reinterpret_cast<uint4*>(&tile[r][8 * q]) = v;
  }
  __syncthreads();
  const int s = d.slot[t];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = r0 + 32 * h, ci = ci0 + r, co = co0 + 8 * q;  // output row ci, co piece q
    if (ci >= Cin || co >= Cout) continue;
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      w[k] = (uint32_t)tile[8 * q + 2 * k][r] | ((uint32_t)tile[8 * q + 2 * k + 1][r] << 16);
    *reinterpret_cast<uint4*>(wt + ((int64_t)ci * kt + s) * Cout + co) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}
// desc: device table of nd PackDesc; nplain / nplain1 / ntrans: total blocks of the three grids (the plain grid has
// Cout x ceil(Cin_p / 64) blocks per layer); lds: bytes of one plain-grid chunk (64 x max kt x 4 over its layers)
void pack_convs(uintptr_t desc, int nd, int nplain, int nplain1, int ntrans, int lds, uintptr_t theta, int64_t ldt,
                int G, uintptr_t out, uintptr_t stream) {
  NIDT_REQUIRE(nd > 0 && G > 0 && lds > 0 && lds <= 160 * 1024 && nplain >= 0 && nplain1 >= 0,
               "pack_convs: bad table");
  hipStream_t s = as_stream(stream);
  if (nplain > 0) {
    hipLaunchKernelGGL(k_pack_plain, dim3(nplain, G), dim3(256), lds, s, ptr<const PackDesc>(desc), nd,
                       ptr<const float>(theta), ldt, G, ptr<uint16_t>(out));
    NIDT_CHECK(hipGetLastError());
  }
  if (nplain1 > 0) {
    hipLaunchKernelGGL(k_pack_plain1, dim3(nplain1, G), dim3(256), 0, s, ptr<const PackDesc>(desc), nd,
                       ptr<const float>(theta), ldt, G, ptr<uint16_t>(out));
    NIDT_CHECK(hipGetLastError());
  }
  if (ntrans > 0) {
    hipLaunchKernelGGL(k_pack_trans, dim3(ntrans, G), dim3(256), 0, s, ptr<const PackDesc>(desc), nd, G,
                       ptr<uint16_t>(out));
    NIDT_CHECK(hipGetLastError());
  }
}

int pack_desc_bytes() { return (int)sizeof(PackDesc); }
int pack1_rows_host(int cin_p) { return pack1_rows(cin_p); }
int pack_plain_chunks(int cin_p, int kt) { const int cc = pack_cc(cin_p, kt); return (cin_p + cc - 1) / cc; }
int pack_plain_lds(int cin_p, int kt) { return pack_cc(cin_p, kt) * kt * 4; }

}  // namespace nidt
