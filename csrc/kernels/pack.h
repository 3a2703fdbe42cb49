// Shared descriptors of the batched weight packing (pack.hip) and the optimizer step that writes the forward images
// itself (optim.hip k_local_step_pack).
#pragma once
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
// the forward-image rows of one plain-grid chunk: row = the chunk's fp32 source [cc][kt] (LDS, PyTorch order),
// written as kt runs of cw image channels (channels cc..cw-1 zero) at wp[g][co][t][ci0..]
__device__ __forceinline__ void pack_image_chunk(const PackDesc& d, const float* row, uint16_t* out, int g, int co,
                                                 int ci0, int cw, int cc) {
  const int Cin = d.cin_p, kt = d.kt, K = kt * Cin;
  uint16_t* dst = out + d.wp_off + ((int64_t)g * d.cout + co) * K + ci0;
  if (Cin % 8 == 0 && (d.wp_off & 7) == 0) {  // 16-B stores: 8 channels of one tap per lane
    const int nq = cw / 8;
    for (int e = threadIdx.x; e < kt * nq; e += blockDim.x) {
      const int t = e / nq, c = (e - t * nq) * 8;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = c + j < cc ? row[(c + j) * kt + t] : 0.f;
      *reinterpret_cast<uint4*>(dst + (int64_t)t * Cin + c) = make_uint4(
          pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]), pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
    }
    return;
  }
  for (int e = threadIdx.x; e < kt * cw; e += blockDim.x) {
    const int t = e / cw, c = e - t * cw;
    dst[(int64_t)t * Cin + c] = f32_to_bf16(c < cc ? row[c * kt + t] : 0.f);
  }
}

}  // namespace nidt
