// Batched per-step weight packing of a client-grouped network: every conv layer of G clients' fp32 parameter rows
// (PyTorch layout [Cout][cin][taps]) becomes the bf16 MFMA A-operand images of the conv kernels in TWO launches per
// step (all layers at once), instead of two launches per layer:
//   plain  wp[g][Cout][kt][Cin_p]   (forward; input channels cin..Cin_p-1 zero),
//   dgrad  wt[g][Cin_p][kt][Cout]   with the taps in slot order: slot_of_tap = kt-1-t for a stride-1 conv (the
//          flipped kernel), the sub-pixel phase order of conv_s2_phase_plan (conv3d.hip) for a stride-2 3x3(x3)
//          conv, identity for 1x1.
// The layer of a block comes from a small descriptor table (prefix block counts), so one grid covers layers of
// different shapes; the transposes go through a padded 64x64 LDS tile (coalesced reads and writes).
#include "pack.h"

namespace nidt {

__global__ __launch_bounds__(256) void k_pack_plain(const PackDesc* __restrict__ desc, int nd,
                                                    const float* __restrict__ theta, int64_t ldt, int G,
                                                    uint16_t* __restrict__ out) {
  extern __shared__ float row[];  // [CC][kt]
  const int li = find_layer(desc, nd, blockIdx.x, 0);
  const PackDesc& d = desc[li];
  const int Cin = d.cin_p, kt = d.kt, cs = d.cin_src;
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
  pack_image_chunk(d, row, out, g, co, ci0, cw, cc);
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
