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
  int blk_plain;     // first block of this layer in the plain grid (Cout x ceil(Cin_p / 64) blocks per layer)
  int blk_t;         // first block in the transpose grid (ceil(Cin_p/64) * ceil(Cout/64) * kt blocks per layer)
  int slot[27];
};
static_assert(sizeof(PackDesc) % 8 == 0, "PackDesc alignment");

// layer of block b: binary search over the prefix block counts (log2 of ~60 layers, uniform per block)
__device__ __forceinline__ int find_layer(const PackDesc* d, int n, int b, bool plain) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if ((plain ? d[mid].blk_plain : d[mid].blk_t) <= b) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// plain: block (layer row co, 64-channel chunk cc, client g): the chunk's fp32 source rows [64][kt] (contiguous in
// the PyTorch layout) are staged in LDS and written as kt runs of 64 bf16 channels.  Chunked so that a block stages
// at most 64 kt floats (6.9 KB for 3x3x3) instead of a whole [cin][kt] row: the launch's dynamic LDS is sized by its
// largest block, and whole 512-channel rows (55 KB) held the 3D ResNet's pack to two blocks per CU (~1.2 TB/s).
__global__ __launch_bounds__(256) void k_pack_plain(const PackDesc* __restrict__ desc, int nd,
                                                    const float* __restrict__ theta, int64_t ldt, int G,
                                                    uint16_t* __restrict__ out) {
  extern __shared__ float row[];
  const int li = find_layer(desc, nd, blockIdx.x, true);
  const PackDesc& d = desc[li];
  const int Cin = d.cin_p, kt = d.kt, K = kt * Cin, Ks = kt * d.cin_src;
  const int nci = (Cin + 63) >> 6;
  const int b = blockIdx.x - d.blk_plain, co = b / nci, c0 = (b - co * nci) * 64, g = blockIdx.y;
  const int nc = min(64, Cin - c0);                       // output channels of this chunk
  const int ns = max(0, min(64, d.cin_src - c0));         // source channels present in it (the rest are zero)
  const float* src = theta + (int64_t)g * ldt + d.src_off + (int64_t)co * Ks + (int64_t)c0 * kt;
  const int n = ns * kt;
  if ((reinterpret_cast<uintptr_t>(src) & 15) == 0 && n % 4 == 0) {  // 16-B source loads
    for (int e = 4 * threadIdx.x; e < n; e += 4 * 256)
      *reinterpret_cast<float4*>(row + e) = *reinterpret_cast<const float4*>(src + e);
  } else {
    for (int e = threadIdx.x; e < n; e += 256) row[e] = src[e];
  }
  __syncthreads();
  uint16_t* dst = out + d.wp_off + ((int64_t)g * d.cout + co) * K + c0;
  if (Cin % 8 == 0 && nc % 8 == 0 && (d.wp_off & 7) == 0) {  // 16-B stores: 8 channels of one tap per lane
    const int n8 = nc >> 3;
    for (int it = threadIdx.x; it < kt * n8; it += 256) {
      const int t = it / n8, j0 = (it - t * n8) * 8;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = j0 + j < ns ? row[(j0 + j) * kt + t] : 0.f;
      *reinterpret_cast<uint4*>(dst + t * Cin + j0) = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]),
                                                                 pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
    }
    return;
  }
  const int n2 = (nc + 1) >> 1;  // channel pairs (Cin even: a pair never straddles a tap)
  for (int it = threadIdx.x; it < kt * n2; it += 256) {
    const int t = it / n2, j = (it - t * n2) * 2;
    const float a = j < ns ? row[j * kt + t] : 0.f;
    const float c = j + 1 < ns ? row[(j + 1) * kt + t] : 0.f;
    *reinterpret_cast<uint32_t*>(dst + t * Cin + j) = pack_bf16x2(a, c);
  }
}

// transposed: block (64 ci x 64 co tile, tap t, client g) reads the plain image written by k_pack_plain.  Global
// traffic in 16-B pieces (8 channels per lane: a 64-wide tile row is 8 lanes), the transpose through a padded LDS tile
// (2-B column reads there, where bandwidth is plentiful); 2-B global accesses ran at ~2 TB/s.
__global__ __launch_bounds__(256) void k_pack_trans(const PackDesc* __restrict__ desc, int nd, int G,
                                                    uint16_t* __restrict__ out) {
  __shared__ uint16_t tile[64][72];  // [co][ci], rows padded to 144 B (16-B aligned, staggered banks)
  const int li = find_layer(desc, nd, blockIdx.x, false);
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
// desc: device table of nd PackDesc; nplain / ntrans: total blocks of the two grids; lds: bytes for the largest
// plain block (max kt * min(64, cin_src) * 4)
void pack_convs(uintptr_t desc, int nd, int nplain, int ntrans, int lds, uintptr_t theta, int64_t ldt, int G,
                uintptr_t out, uintptr_t stream) {
  NIDT_REQUIRE(nd > 0 && G > 0 && lds > 0 && lds <= 160 * 1024, "pack_convs: bad table");
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(k_pack_plain, dim3(nplain, G), dim3(256), lds, s, ptr<const PackDesc>(desc), nd,
                     ptr<const float>(theta), ldt, G, ptr<uint16_t>(out));
  NIDT_CHECK(hipGetLastError());
  if (ntrans > 0) {
    hipLaunchKernelGGL(k_pack_trans, dim3(ntrans, G), dim3(256), 0, s, ptr<const PackDesc>(desc), nd, G,
                       ptr<uint16_t>(out));
    NIDT_CHECK(hipGetLastError());
  }
}

int pack_desc_bytes() { return (int)sizeof(PackDesc); }

}  // namespace nidt
