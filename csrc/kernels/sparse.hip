// Per-client sparse-mask kernels: bit-packed mask rows, per-(client, layer) counts / Hamming distances,
// exact segmented top-k selection (DisPFL fire / regrow), per-layer percentile pruning (SubAvg), mask-count
// averaging (SubAvg aggregation), row mixing (D-PSGD / FedFomo / DisPFL gossip) and row-pair distances.
//
// Masks: one uint32 bit row per client, bit i of row r <-> flat parameter i (word i >> 5, bit i & 31); the row
// stride is a multiple of 4 words.  "Segments" are the per-parameter ranges of the flat layout (the reference keys
// masks by parameter name: DisPFL/my_model_trainer.py:31-41, subavg/my_model_trainer.py:28-40).  Work is split into
// tiles (row, segment, [begin, end)) built once on the host, so one launch covers every (client, layer) pair.
//
// Selection (reference DisPFL/client.py:71-99: torch.sort of the masked |w| / |g| per layer):
//   keys are 32-bit unsigned, larger = selected first, 0 = not a candidate:
//     FIRE        candidates: active (bit 1);   key = ~bits(|w|)        (smallest |w| first)   -> clear
//     REGROW_ABS  candidates: inactive (bit 0); key = bits(|g|) + 1     (largest |g| first)    -> set
//     REGROW_RAND candidates: inactive;         key = hash(seed, client, i) | 1  (uniform random subset) -> set
//     ALIVE_MIN   candidates: active and w != 0; key = ~bits(|w|)       (query only: k-th smallest alive |w|)
//   k-th largest key per segment by a 4-pass 8-bit radix select (integer histograms: deterministic), then all
//   keys > T plus the FIRST r keys == T in index order (what a stable sort does with ties) are applied.
#include "common.h"

namespace nidt {

enum SelMode { kFire = 0, kRegrowAbs = 1, kRegrowRand = 2, kAliveMin = 3 };

struct Tile {
  int row, seg, begin, end;  // element range [begin, end) of segment seg in client row row
};

__device__ __forceinline__ uint32_t mix_hash(uint64_t seed, uint32_t a, uint32_t b) {
  uint64_t z = seed ^ (0x9e3779b97f4a7c15ull * (((uint64_t)a << 32) ^ (uint64_t)b));
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}

template <int MODE>
__device__ __forceinline__ uint32_t sel_key(float v, bool bit, uint64_t seed, uint32_t cid, uint32_t i) {
  const uint32_t a = __float_as_uint(v) & 0x7fffffffu;
  if (MODE == kFire) return bit ? ~a : 0u;
  if (MODE == kRegrowAbs) return bit ? 0u : a + 1u;
  if (MODE == kRegrowRand) return bit ? 0u : (mix_hash(seed, cid, i) | 1u);
  return (bit && a != 0u) ? ~a : 0u;  // kAliveMin
}

// words of tile t covered by this thread: w = wbeg + threadIdx.x + k * blockDim.x
__device__ __forceinline__ void tile_words(const Tile& t, int& wbeg, int& wend) {
  wbeg = t.begin >> 5;
  wend = (t.end + 31) >> 5;
}

__device__ __forceinline__ uint32_t word_range_mask(int w, int begin, int end) {
  const int lo = max(begin - (w << 5), 0), hi = min(end - (w << 5), 32);
  if (hi <= lo) return 0u;
  const uint32_t up = hi == 32 ? 0xffffffffu : ((1u << hi) - 1u);
  return up & ~((1u << lo) - 1u);
}

// ------------------------------------------------------------------------------------------------ counts
// mode 0: popcount(A); 1: popcount(A ^ B); 2: popcount(A & (v != 0))
__global__ __launch_bounds__(256) void k_seg_count(const Tile* __restrict__ tiles, const uint32_t* __restrict__ A,
                                                   const uint32_t* __restrict__ Bm, int64_t mstride,
                                                   const float* __restrict__ v, int64_t ldv, int mode, int S,
                                                   int* __restrict__ out) {
  const Tile t = tiles[blockIdx.x];
  int wb, we;
  tile_words(t, wb, we);
  const uint32_t* a = A + (int64_t)t.row * mstride;
  int cnt = 0;
  for (int w = wb + threadIdx.x; w < we; w += blockDim.x) {
    uint32_t x = a[w];
    if (mode == 1) x ^= Bm[(int64_t)t.row * mstride + w];
    if (mode == 2) {
      const float* vr = v + (int64_t)t.row * ldv + ((int64_t)w << 5);
      uint32_t nz = 0;
      for (int j = 0; j < 32; ++j) {
        const int64_t e = ((int64_t)w << 5) + j;
        if (e >= t.begin && e < t.end && vr[j] != 0.f) nz |= 1u << j;
      }
      x &= nz;
    }
    cnt += __popc(x & word_range_mask(w, t.begin, t.end));
  }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  if ((threadIdx.x & 63) == 0 && cnt) atomicAdd(out + t.row * S + t.seg, cnt);
}

// ------------------------------------------------------------------------------------------------ radix select
template <int MODE>
__global__ __launch_bounds__(256) void k_seg_hist(const Tile* __restrict__ tiles, const float* __restrict__ v,
                                                  int64_t ldv, const uint32_t* __restrict__ bits, int64_t mstride,
                                                  const int* __restrict__ cids, uint64_t seed, int S,
                                                  const uint32_t* __restrict__ state, int shift,
                                                  uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[256];
  const Tile t = tiles[blockIdx.x];
  const int sid = t.row * S + t.seg;
  const uint32_t pre = state[sid * 4], pm = state[sid * 4 + 1], krem = state[sid * 4 + 2];
  if (krem == 0) return;  // nothing to select in this segment (uniform per block)
  h[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t cid = cids ? (uint32_t)cids[t.row] : (uint32_t)t.row;
  const float* vr = v + (int64_t)t.row * ldv;
  const uint32_t* br = bits + (int64_t)t.row * mstride;
  for (int e = t.begin + threadIdx.x; e < t.end; e += blockDim.x) {
    const bool b = (br[e >> 5] >> (e & 31)) & 1u;
    const uint32_t key = sel_key<MODE>(MODE == kRegrowRand ? 0.f : vr[e], b, seed, cid, (uint32_t)e);
    if (key != 0u && (key & pm) == pre) atomicAdd(&h[(key >> shift) & 0xffu], 1u);
  }
  __syncthreads();
  if (h[threadIdx.x]) atomicAdd(&hist[(int64_t)sid * 256 + threadIdx.x], h[threadIdx.x]);
}

// one wave per segment: pick the digit holding the krem-th largest key, zero the histogram for the next pass
__global__ void k_seg_scan(uint32_t* __restrict__ state, int shift, uint32_t* __restrict__ hist, int nseg) {
  const int sid = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (sid >= nseg) return;
  uint32_t* hs = hist + (int64_t)sid * 256;
  const uint32_t krem = state[sid * 4 + 2];
  if (krem != 0u && lane == 0) {
    uint32_t acc = 0;
    int d = 255;
    for (; d > 0; --d) {
      if (acc + hs[d] >= krem) break;
      acc += hs[d];
    }
    state[sid * 4] |= (uint32_t)d << shift;
    state[sid * 4 + 1] |= 0xffu << shift;
    state[sid * 4 + 2] = krem - acc;
    state[sid * 4 + 3] = state[sid * 4];
  }
  for (int i = lane; i < 256; i += 64) hs[i] = 0;
}

// number of candidates with key == T per tile
template <int MODE>
__global__ __launch_bounds__(256) void k_seg_ties(const Tile* __restrict__ tiles, const float* __restrict__ v,
                                                  int64_t ldv, const uint32_t* __restrict__ bits, int64_t mstride,
                                                  const int* __restrict__ cids, uint64_t seed, int S,
                                                  const uint32_t* __restrict__ state, int* __restrict__ ties) {
  __shared__ int red[4];
  const Tile t = tiles[blockIdx.x];
  const int sid = t.row * S + t.seg;
  const uint32_t T = state[sid * 4 + 3], krem = state[sid * 4 + 2];
  int c = 0;
  if (krem != 0u) {
    const uint32_t cid = cids ? (uint32_t)cids[t.row] : (uint32_t)t.row;
    const float* vr = v + (int64_t)t.row * ldv;
    const uint32_t* br = bits + (int64_t)t.row * mstride;
    for (int e = t.begin + threadIdx.x; e < t.end; e += blockDim.x) {
      const bool b = (br[e >> 5] >> (e & 31)) & 1u;
      c += sel_key<MODE>(MODE == kRegrowRand ? 0.f : vr[e], b, seed, cid, (uint32_t)e) == T;
    }
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) ties[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// Apply the selection: thread = one 32-bit mask word of the tile; ties are taken in index order (block scan of the
// per-word tie counts, running base across the tile, base of the tile = ties of the segment's earlier tiles).
// [COAL] the keys are computed lane-contiguous: wave w of the block owns words w0 + 64 w .. + 63 (2048 elements);
// in pass j its lanes read elements 64 j + lane of that range (256 contiguous bytes per load instead of a 128-B
// stride per lane) and two ballots give words 2 j and 2 j + 1, which lanes 2 j / 2 j + 1 keep — each thread ends
// with the (gt, eq) bits of its own word, as before.  The mask words are fetched once per lane and shuffled.
// (config 5's sparse update selection: 5.3 ms per call at 1.1 TB/s, profiles/r6_config5_steady.txt)
template <int MODE>
__global__ __launch_bounds__(256) void k_seg_apply(const Tile* __restrict__ tiles, const int* __restrict__ tile_first,
                                                   const float* __restrict__ v, int64_t ldv,
                                                   uint32_t* __restrict__ bits, int64_t mstride,
                                                   const int* __restrict__ cids, uint64_t seed, int S,
                                                   const uint32_t* __restrict__ state, const int* __restrict__ ties) {
  __shared__ int scan[256];
  __shared__ int base_s;
  const Tile t = tiles[blockIdx.x];
  const int sid = t.row * S + t.seg;
  const uint32_t T = state[sid * 4 + 3];
  const int krem = (int)state[sid * 4 + 2];
  if (krem == 0) return;
  (void)tile_first;
  const int prior = ties[blockIdx.x];  // ties of the segment's earlier tiles (k_seg_ties_scan)
  int quota = krem - prior;  // ties this tile may still take
  const uint32_t cid = cids ? (uint32_t)cids[t.row] : (uint32_t)t.row;
  const float* vr = v + (int64_t)t.row * ldv;
  uint32_t* br = bits + (int64_t)t.row * mstride;
  int wb, we;
  tile_words(t, wb, we);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (threadIdx.x == 0) base_s = 0;
  for (int w0 = wb; w0 < we; w0 += blockDim.x) {
    const int w = w0 + threadIdx.x;
    const uint32_t word = w < we ? br[w] : 0u;  // this thread's mask word (read before any write of this pass)
    const int wbase = w0 + 64 * wv;             // first word of this wave
    uint32_t gt = 0, eq = 0;
    if (wbase < we) {  // wave-uniform
      for (int j = 0; j < 32; ++j) {
        const int e = (wbase << 5) + 64 * j + lane;
        const uint32_t wj = __shfl(word, 2 * j + (lane >> 5), 64);
        bool g = false, q = false;
        if (e >= t.begin && e < t.end) {
          const uint32_t key = sel_key<MODE>(MODE == kRegrowRand ? 0.f : vr[e], (wj >> (lane & 31)) & 1u, seed, cid,
                                             (uint32_t)e);
          g = key > T;
          q = key == T && key != 0u;
        }
        const uint64_t bg = __ballot(g), bq = __ballot(q);
        if (lane == 2 * j) {
          gt = (uint32_t)bg;
          eq = (uint32_t)bq;
        } else if (lane == 2 * j + 1) {
          gt = (uint32_t)(bg >> 32);
          eq = (uint32_t)(bq >> 32);
        }
      }
    }
    const int my = __popc(eq);
    __syncthreads();
    scan[threadIdx.x] = my;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {  // inclusive Hillis-Steele scan (256 entries)
      const int add = threadIdx.x >= o ? scan[threadIdx.x - o] : 0;
      __syncthreads();
      scan[threadIdx.x] += add;
      __syncthreads();
    }
    const int before = base_s + scan[threadIdx.x] - my;
    int take = quota - before;
    take = take < 0 ? 0 : (take > my ? my : take);
    uint32_t sel = gt;
    for (uint32_t m = eq; take > 0; --take) {  // lowest-index ties first
      const uint32_t low = m & (~m + 1u);
      sel |= low;
      m ^= low;
    }
    if (w < we && sel) {
      if (MODE == kFire) atomicAnd(br + w, ~sel);
      else atomicOr(br + w, sel);
    }
    __syncthreads();
    if (threadIdx.x == 255) base_s += scan[255];
    __syncthreads();
  }
}

// [TSCAN] per-tile tie counts -> the exclusive prefix over the segment's earlier tiles, in place: one wave per
// segment start walks its tiles 64 at a time (wave prefix sum + running base).  k_seg_apply summed
// ties[tile_first .. b) itself — O(tiles^2) loads per segment, 5.3 ms per call for config 5's whole-row update
// segments (thousands of tiles each)
__global__ void k_seg_ties_scan(const int* __restrict__ tile_first, int* __restrict__ ties, int ntiles) {
  const int b = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (b >= ntiles || tile_first[b] != b) return;  // wave-uniform
  int base = 0;
  for (int j0 = b; j0 < ntiles; j0 += 64) {
    const int j = j0 + lane;
    const bool in = j < ntiles && tile_first[j] == b;
    const int c = in ? ties[j] : 0;
    int inc = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int u = __shfl_up(inc, o, 64);
      if (lane >= o) inc += u;
    }
    if (in) ties[j] = base + inc - c;
    base += __shfl(inc, 63, 64);
    if (!__all(in)) break;  // the segment ended inside this group of 64
  }
}

// ------------------------------------------------------------------------------------------------ host: select
void seg_count(uintptr_t tiles, int ntiles, uintptr_t A, uintptr_t Bm, int64_t mstride, uintptr_t v, int64_t ldv,
               int mode, int S, uintptr_t out, uintptr_t stream) {
  if (ntiles == 0) return;
  hipLaunchKernelGGL(k_seg_count, dim3(ntiles), dim3(256), 0, as_stream(stream), ptr<const Tile>(tiles),
                     ptr<const uint32_t>(A), ptr<const uint32_t>(Bm), mstride, ptr<const float>(v), ldv, mode, S,
                     ptr<int>(out));
  NIDT_CHECK(hipGetLastError());
}

// state [nseg, 4] uint32 must hold {0, 0, k, 0} per segment (k <= candidates); hist [nseg, 256] zeroed.
// query_only: stop after the radix passes (state[.,3] = T, state[.,2] = ties to take).
void seg_select(uintptr_t tiles, uintptr_t tile_first, int ntiles, uintptr_t v, int64_t ldv, uintptr_t bits,
                int64_t mstride, uintptr_t cids, uint64_t seed, int R, int S, int mode, uintptr_t state,
                uintptr_t hist, uintptr_t ties, int query_only, uintptr_t stream) {
  if (ntiles == 0) return;
  hipStream_t st = as_stream(stream);
  const int nseg = R * S;
  const Tile* tl = ptr<const Tile>(tiles);
#define NIDT_SEL(M)                                                                                              \
  for (int shift = 24; shift >= 0; shift -= 8) {                                                                 \
    hipLaunchKernelGGL(k_seg_hist<M>, dim3(ntiles), dim3(256), 0, st, tl, ptr<const float>(v), ldv,              \
                       ptr<const uint32_t>(bits), mstride, ptr<const int>(cids), seed, S,                        \
                       ptr<const uint32_t>(state), shift, ptr<uint32_t>(hist));                                  \
    hipLaunchKernelGGL(k_seg_scan, dim3(ceil_div(nseg, 4)), dim3(256), 0, st, ptr<uint32_t>(state), shift,       \
                       ptr<uint32_t>(hist), nseg);                                                               \
  }                                                                                                              \
  if (!query_only) {                                                                                             \
    hipLaunchKernelGGL(k_seg_ties<M>, dim3(ntiles), dim3(256), 0, st, tl, ptr<const float>(v), ldv,              \
                       ptr<const uint32_t>(bits), mstride, ptr<const int>(cids), seed, S,                        \
                       ptr<const uint32_t>(state), ptr<int>(ties));                                              \
    hipLaunchKernelGGL(k_seg_ties_scan, dim3(ceil_div(ntiles, 4)), dim3(256), 0, st, ptr<const int>(tile_first),     \
                       ptr<int>(ties), ntiles);                                                                  \
    hipLaunchKernelGGL(k_seg_apply<M>, dim3(ntiles), dim3(256), 0, st, tl, ptr<const int>(tile_first),           \
                       ptr<const float>(v), ldv, ptr<uint32_t>(bits), mstride, ptr<const int>(cids), seed, S,    \
                       ptr<const uint32_t>(state), ptr<const int>(ties));                                        \
  }
  switch (mode) {
    case kFire: NIDT_SEL(kFire); break;
    case kRegrowAbs: NIDT_SEL(kRegrowAbs); break;
    case kRegrowRand: NIDT_SEL(kRegrowRand); break;
    case kAliveMin: NIDT_SEL(kAliveMin); break;
    default: NIDT_REQUIRE(false, "seg_select: mode");
  }
#undef NIDT_SEL
  NIDT_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------ percentile prune
// SubAvg fake_prune (subavg/prune_func.py:9-30): thr = numpy.percentile(|alive|, 100 q) with linear interpolation
// between the lo-th and hi-th smallest alive |w| (alive = w * m != 0); new mask = m where |w| >= thr, else 0.
// thr[sid] (fp64) is computed on the host side of the op from the two radix queries; here only the mask update.
// out must hold a copy of the input bits.  prune[seg] = 0 leaves that segment's bits untouched.
__global__ __launch_bounds__(256) void k_seg_prune(const Tile* __restrict__ tiles, const float* __restrict__ v,
                                                   int64_t ldv, uint32_t* __restrict__ out, int64_t mstride,
                                                   const float* __restrict__ thr, const int* __restrict__ prune,
                                                   int S) {
  const Tile t = tiles[blockIdx.x];
  if (!prune[t.seg]) return;
  const float th = thr[t.row * S + t.seg];
  const float* vr = v + (int64_t)t.row * ldv;
  uint32_t* orow = out + (int64_t)t.row * mstride;
  int wb, we;
  tile_words(t, wb, we);
  for (int w = wb + threadIdx.x; w < we; w += blockDim.x) {
    const uint32_t rm = word_range_mask(w, t.begin, t.end);
    uint32_t clr = 0;
    for (int j = 0; j < 32; ++j)
      if ((rm >> j) & 1u) clr |= (fabsf(vr[(w << 5) + j]) < th ? 1u : 0u) << j;
    if (clr) atomicAnd(orow + w, ~clr);
  }
}

void seg_prune(uintptr_t tiles, int ntiles, uintptr_t v, int64_t ldv, uintptr_t out, int64_t mstride, uintptr_t thr,
               uintptr_t prune, int S, uintptr_t stream) {
  if (ntiles == 0) return;
  hipLaunchKernelGGL(k_seg_prune, dim3(ntiles), dim3(256), 0, as_stream(stream), ptr<const Tile>(tiles),
                     ptr<const float>(v), ldv, ptr<uint32_t>(out), mstride, ptr<const float>(thr),
                     ptr<const int>(prune), S);
  NIDT_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------ masked average
// SubAvg aggregation partials (subavg_api.py:123-139): sum[p] += sum_r rows[r][p]; cnt[p] += sum_r bit(r, p)
// (bits == 0: every row counts, i.e. a plain average, used for the BN buffers the reference never masks).
__global__ __launch_bounds__(256) void k_masked_rows_sum(const float* __restrict__ rows, int64_t ld,
                                                         const uint32_t* __restrict__ bits, int64_t mstride, int R,
                                                         int64_t n, float* __restrict__ sum, float* __restrict__ cnt) {
  const int64_t i = 4 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= n) return;
  float s[4] = {0.f, 0.f, 0.f, 0.f}, c[4] = {0.f, 0.f, 0.f, 0.f};
  const bool full = i + 3 < n;
  for (int r = 0; r < R; ++r) {
    const float* rr = rows + (int64_t)r * ld;
    uint32_t b4 = 0xfu;
    if (bits) b4 = (bits[(int64_t)r * mstride + (i >> 5)] >> (i & 31)) & 0xfu;
    if (full) {
      const float4 x = *reinterpret_cast<const float4*>(rr + i);
      s[0] += x.x; s[1] += x.y; s[2] += x.z; s[3] += x.w;
    } else {
      for (int j = 0; j < 4 && i + j < n; ++j) s[j] += rr[i + j];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j] += (float)((b4 >> j) & 1u);
  }
  for (int j = 0; j < 4 && i + j < n; ++j) {
    sum[i + j] += s[j];
    cnt[i + j] += c[j];
  }
}

void masked_rows_sum(uintptr_t rows, int64_t ld, uintptr_t bits, int64_t mstride, int R, int64_t n, uintptr_t sum,
                     uintptr_t cnt, uintptr_t stream) {
  NIDT_REQUIRE(ld % 4 == 0 && (rows & 15) == 0, "masked_rows_sum: alignment");
  NIDT_REQUIRE(!bits || mstride % 4 == 0, "masked_rows_sum: mask stride");
  if (R == 0 || n == 0) return;
  hipLaunchKernelGGL(k_masked_rows_sum, dim3(ceil_div((n + 3) / 4, 256)), dim3(256), 0, as_stream(stream),
                     ptr<const float>(rows), ld, ptr<const uint32_t>(bits), mstride, R, n, ptr<float>(sum),
                     ptr<float>(cnt));
  NIDT_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------ masked neighbour mean
// DisPFL's masked neighbour average (the paper's aggregation; commented out in the reference, dispfl_api.py:138-142),
// every client of the launch at once: out_r[p] = own_r(p) * (sum_k src_k[p] bit_k(p)) / (sum_k bit_k(p)) over its
// neighbours k in [rp[r], rp[r+1]) (0 where no neighbour keeps p).  src / bits / dst / own: device pointer tables
// (fp32 rows 16-B aligned, uint32 bit rows); outputs must not alias sources.  grid (ceil(n/4/256), rows).
__global__ __launch_bounds__(256) void k_masked_mean_rows(const uint64_t* __restrict__ src,
                                                          const uint64_t* __restrict__ sbits,
                                                          const int* __restrict__ rp, const uint64_t* __restrict__ dst,
                                                          const uint64_t* __restrict__ own, int64_t n) {
  const int r = blockIdx.y;
  const int64_t i = 4 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= n) return;
  const int k0 = rp[r], k1 = rp[r + 1];
  float num[4] = {0.f, 0.f, 0.f, 0.f}, cnt[4] = {0.f, 0.f, 0.f, 0.f};
  const bool full = i + 3 < n;
  for (int k = k0; k < k1; ++k) {
    const float* x = reinterpret_cast<const float*>(src[k]);
    const uint32_t b4 = (reinterpret_cast<const uint32_t*>(sbits[k])[i >> 5] >> (i & 31)) & 0xfu;
    float v[4];
    if (full) {
      const float4 q = *reinterpret_cast<const float4*>(x + i);
      v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    } else {
      for (int j = 0; j < 4; ++j) v[j] = i + j < n ? x[i + j] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool on = (b4 >> j) & 1u;
      num[j] += on ? v[j] : 0.f;
      cnt[j] += on ? 1.f : 0.f;
    }
  }
  const uint32_t o4 = (reinterpret_cast<const uint32_t*>(own[r])[i >> 5] >> (i & 31)) & 0xfu;
  float* out = reinterpret_cast<float*>(dst[r]);
  float res[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) res[j] = (cnt[j] > 0.f && ((o4 >> j) & 1u)) ? num[j] / cnt[j] : 0.f;
  if (full) {
    *reinterpret_cast<float4*>(out + i) = make_float4(res[0], res[1], res[2], res[3]);
  } else {
    for (int j = 0; j < 4 && i + j < n; ++j) out[i + j] = res[j];
  }
}

void masked_mean_rows(uintptr_t src, uintptr_t sbits, uintptr_t rp, uintptr_t dst, uintptr_t own, int R, int64_t n,
                      uintptr_t stream) {
  if (R == 0 || n == 0) return;
  hipLaunchKernelGGL(k_masked_mean_rows, dim3(ceil_div((n + 3) / 4, 256), R), dim3(256), 0, as_stream(stream),
                     ptr<const uint64_t>(src), ptr<const uint64_t>(sbits), ptr<const int>(rp), ptr<const uint64_t>(dst),
                     ptr<const uint64_t>(own), n);
  NIDT_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------ row mixing
// out_r = sum_{k in [ptr[r], ptr[r+1])} wts[k] * src_k   for each output row r (addresses are device pointers of
// fp32 rows, 16-B aligned; outputs must not alias any source).  Gossip / neighbour averaging of D-PSGD
// (dpsgd_api.py:169-178), FedFomo's weighted neighbour update (fedfomo_api.py:200-217), DisPFL's mean.
__global__ __launch_bounds__(256) void k_mix_rows(const uint64_t* __restrict__ src, const float* __restrict__ wts,
                                                  const int* __restrict__ rp, const uint64_t* __restrict__ dst,
                                                  int64_t n) {
  const int r = blockIdx.y;
  const int64_t i = 4 * ((int64_t)blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= n) return;
  const int k0 = rp[r], k1 = rp[r + 1];
  float* out = reinterpret_cast<float*>(dst[r]);
  if (i + 3 < n) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int k = k0; k < k1; ++k) {
      const float w = wts[k];
      const float4 x = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(src[k]) + i);
      acc.x = fmaf(w, x.x, acc.x); acc.y = fmaf(w, x.y, acc.y);
      acc.z = fmaf(w, x.z, acc.z); acc.w = fmaf(w, x.w, acc.w);
    }
    *reinterpret_cast<float4*>(out + i) = acc;
  } else {
    for (int64_t j = i; j < n; ++j) {
      float acc = 0.f;
      for (int k = k0; k < k1; ++k) acc = fmaf(wts[k], reinterpret_cast<const float*>(src[k])[j], acc);
      out[j] = acc;
    }
  }
}

void mix_rows(uintptr_t src, uintptr_t wts, uintptr_t rowptr, uintptr_t dst, int R, int64_t n, uintptr_t stream) {
  if (R == 0 || n == 0) return;
  dim3 grid(ceil_div((n + 3) / 4, 256), R);
  hipLaunchKernelGGL(k_mix_rows, grid, dim3(256), 0, as_stream(stream), ptr<const uint64_t>(src),
                     ptr<const float>(wts), ptr<const int>(rowptr), ptr<const uint64_t>(dst), n);
  NIDT_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------ pair distances
// part[k, b] = sum over block b's chunk of (a_k - b_k)^2 (fp32 partials; the caller reduces in fp64)
__global__ __launch_bounds__(256) void k_pair_sqdist(const uint64_t* __restrict__ pa, const uint64_t* __restrict__ pb,
                                                     int64_t n, int64_t chunk, float* __restrict__ part, int nblk) {
  __shared__ float red[4];
  const int k = blockIdx.y;
  const float* a = reinterpret_cast<const float*>(pa[k]);
  const float* b = reinterpret_cast<const float*>(pb[k]);
  const int64_t s = (int64_t)blockIdx.x * chunk, e = min(n, s + chunk);
  float acc = 0.f;
  const int64_t e4 = s + ((e - s) & ~int64_t(3));
  for (int64_t i = s + 4 * threadIdx.x; i < e4; i += 1024) {
    const float4 x = *reinterpret_cast<const float4*>(a + i), y = *reinterpret_cast<const float4*>(b + i);
    const float d0 = x.x - y.x, d1 = x.y - y.y, d2 = x.z - y.z, d3 = x.w - y.w;
    acc += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
  }
  for (int64_t i = e4 + threadIdx.x; i < e; i += 256) {
    const float d = a[i] - b[i];
    acc += d * d;
  }
  const float t = block_sum(acc, red);
  if (threadIdx.x == 0) part[(int64_t)k * nblk + blockIdx.x] = t;
}

int pair_sqdist_nblk(int64_t n) { return (int)std::min<int64_t>(256, std::max<int64_t>(1, (n + 16383) / 16384)); }

void pair_sqdist(uintptr_t pa, uintptr_t pb, int K, int64_t n, uintptr_t part, uintptr_t stream) {
  if (K == 0) return;
  const int nblk = pair_sqdist_nblk(n);
  const int64_t chunk = (((n + nblk - 1) / nblk) + 3) & ~int64_t(3);
  hipLaunchKernelGGL(k_pair_sqdist, dim3(nblk, K), dim3(256), 0, as_stream(stream), ptr<const uint64_t>(pa),
                     ptr<const uint64_t>(pb), n, chunk, ptr<float>(part), nblk);
  NIDT_CHECK(hipGetLastError());
}

}  // namespace nidt
