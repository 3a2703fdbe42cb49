// Probe of gfx950's 2:4-sparse MFMA (v_smfmac_*) operand layouts, their issue rate, and misaligned ds_read_b128.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probes/smfmac_probe.hip -o tools/probes/smfmac_probe
// Run:   tools/probes/smfmac_probe <outdir>   (writes raw probe dumps; tools/probes/smfmac_probe.py decodes them)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// probe p: pattern = p / 1024 (index nibble 0x4: slots at dense positions (0,1); 0xE: (2,3)); the single B one-hot sits
// at lane L = (p % 1024) / 16, element e = p % 16.  A's compressed element j of lane l = 1 + 8 * (l / G) + j (G = lanes
// per K chunk: 16 for 16x16x64, 32 for 32x32x32).
__global__ void k_layout16(float* out) {
  const int p = blockIdx.x, l = threadIdx.x;
  const int pat = p / 1024, L = (p % 1024) / 16, e = p % 16;
  bf16x8 a;
  for (int j = 0; j < 8; ++j) a[j] = (__bf16)(float)(1 + 8 * (l / 16) + j);
  bf16x16 b;
  for (int j = 0; j < 16; ++j) b[j] = (__bf16)((l == L && j == e) ? 1.f : 0.f);
  const int idx = pat ? (int)0xEEEEEEEEu : 0x44444444;
  f32x4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_smfmac_f32_16x16x64_bf16(a, b, c, idx, 0, 0);
  for (int i = 0; i < 4; ++i) out[((size_t)p * 64 + l) * 4 + i] = c[i];
}

__global__ void k_layout32(float* out) {
  const int p = blockIdx.x, l = threadIdx.x;
  const int pat = p / 1024, L = (p % 1024) / 16, e = p % 16;
  bf16x8 a;
  for (int j = 0; j < 8; ++j) a[j] = (__bf16)(float)(1 + 8 * (l / 32) + j);
  bf16x16 b;
  for (int j = 0; j < 16; ++j) b[j] = (__bf16)((l == L && j == e) ? 1.f : 0.f);
  const int idx = pat ? (int)0xEEEEEEEEu : 0x44444444;
  f32x16 c = {};
  c = __builtin_amdgcn_smfmac_f32_32x32x32_bf16(a, b, c, idx, 0, 0);
  for (int i = 0; i < 16; ++i) out[((size_t)p * 64 + l) * 16 + i] = c[i];
}

// index semantics: lane-uniform random compressed A values / indices (incl. duplicate and descending index pairs) and
// random B; the host compares D with its own model of the dense product
__global__ void k_random16(const float* av, const int* ai, const float* bv, float* out, int abid) {
  const int p = blockIdx.x, l = threadIdx.x;
  bf16x8 a;
  bf16x16 b;
  for (int j = 0; j < 8; ++j) a[j] = (__bf16)av[(p * 64 + l) * 8 + j];
  for (int j = 0; j < 16; ++j) b[j] = (__bf16)bv[(p * 64 + l) * 16 + j];
  f32x4 c = {0, 0, 0, 0};
  if (abid) c = __builtin_amdgcn_smfmac_f32_16x16x64_bf16(a, b, c, ai[p * 64 + l], 0, 1);
  else c = __builtin_amdgcn_smfmac_f32_16x16x64_bf16(a, b, c, ai[p * 64 + l], 0, 0);
  for (int i = 0; i < 4; ++i) out[((size_t)p * 64 + l) * 4 + i] = c[i];
}

__global__ void k_random32(const float* av, const int* ai, const float* bv, float* out) {
  const int p = blockIdx.x, l = threadIdx.x;
  bf16x8 a;
  bf16x16 b;
  for (int j = 0; j < 8; ++j) a[j] = (__bf16)av[(p * 64 + l) * 8 + j];
  for (int j = 0; j < 16; ++j) b[j] = (__bf16)bv[(p * 64 + l) * 16 + j];
  f32x16 c = {};
  c = __builtin_amdgcn_smfmac_f32_32x32x32_bf16(a, b, c, ai[p * 64 + l], 0, 0);
  for (int i = 0; i < 16; ++i) out[((size_t)p * 64 + l) * 16 + i] = c[i];
}

// issue rate: 4 independent accumulators, n iterations; cycles per instruction per wave (s_memtime)
template <int KIND>
__global__ void k_rate(float* sink, long long* cyc, int n) {
  const int l = threadIdx.x;
  bf16x8 a;
  bf16x16 b;
  for (int j = 0; j < 8; ++j) a[j] = (__bf16)(float)((l + j) & 3);
  for (int j = 0; j < 16; ++j) b[j] = (__bf16)(float)((l * 3 + j) & 3);
  const bf16x8 b8 = {b[0], b[1], b[2], b[3], b[4], b[5], b[6], b[7]};
  f32x4 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  f32x16 d0 = {}, d1 = {}, d2 = {}, d3 = {};
  const int idx = 0x44444444;
  const long long t0 = clock64();
  for (int i = 0; i < n; ++i) {
    if (KIND == 0) {
      c0 = __builtin_amdgcn_smfmac_f32_16x16x64_bf16(a, b, c0, idx, 0, 0);
      c1 = __builtin_amdgcn_smfmac_f32_16x16x64_bf16(a, b, c1, idx, 0, 0);
      c2 = __builtin_amdgcn_smfmac_f32_16x16x64_bf16(a, b, c2, idx, 0, 0);
      c3 = __builtin_amdgcn_smfmac_f32_16x16x64_bf16(a, b, c3, idx, 0, 0);
    } else if (KIND == 1) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b8, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b8, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b8, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b8, c3, 0, 0, 0);
    } else if (KIND == 2) {
      d0 = __builtin_amdgcn_smfmac_f32_32x32x32_bf16(a, b, d0, idx, 0, 0);
      d1 = __builtin_amdgcn_smfmac_f32_32x32x32_bf16(a, b, d1, idx, 0, 0);
      d2 = __builtin_amdgcn_smfmac_f32_32x32x32_bf16(a, b, d2, idx, 0, 0);
      d3 = __builtin_amdgcn_smfmac_f32_32x32x32_bf16(a, b, d3, idx, 0, 0);
    } else {
      d0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b8, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b8, d1, 0, 0, 0);
      d2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b8, d2, 0, 0, 0);
      d3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b8, d3, 0, 0, 0);
    }
  }
  const long long t1 = clock64();
  float s = 0;
  for (int i = 0; i < 4; ++i) s += c0[i] + c1[i] + c2[i] + c3[i];
  for (int i = 0; i < 16; ++i) s += d0[i] + d1[i] + d2[i] + d3[i];
  sink[blockIdx.x * 64 + l] = s;
  if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

// misaligned ds_read_b128: LDS bytes = byte index; lane reads 16 B at 32 * lane + off; plus a timed loop
__global__ void k_lds(uint32_t* out, long long* cyc, int off, int n) {
  __shared__ __attribute__((aligned(16))) uint8_t s[4096];
  for (int i = threadIdx.x; i < 4096; i += 64) s[i] = (uint8_t)(i * 7 + (i >> 8));
  __syncthreads();
  const int l = threadIdx.x;
  const uint32_t addr = (uint32_t)(uintptr_t)(s) + 32 * l + off;
  uint4 v;
  asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
  out[(blockIdx.x * 64 + l) * 4 + 0] = v.x;
  out[(blockIdx.x * 64 + l) * 4 + 1] = v.y;
  out[(blockIdx.x * 64 + l) * 4 + 2] = v.z;
  out[(blockIdx.x * 64 + l) * 4 + 3] = v.w;
  uint32_t acc = 0;
  const long long t0 = clock64();
  for (int i = 0; i < n; ++i) {
    uint4 w0, w1, w2, w3;
    const uint32_t a2 = addr ^ ((i & 1) << 11);
    asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:512\n\tds_read_b128 %2, %4 offset:1024\n\t"
                 "ds_read_b128 %3, %4 offset:1536\n\ts_waitcnt lgkmcnt(0)"
                 : "=v"(w0), "=v"(w1), "=v"(w2), "=v"(w3) : "v"(a2) : "memory");
    acc += w0.x ^ w1.y ^ w2.z ^ w3.w;
  }
  const long long t1 = clock64();
  out[(gridDim.x * 64 + blockIdx.x * 64 + l) * 4] = acc;
  if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

// ds_read_b128 THROUGHPUT: 4 waves, each lane reads 16 B at 16 * lane + off (+ 1 KiB steps), 8 reads in flight per
// wait; cycles per wave-instruction
__global__ void k_lds_rate(uint32_t* out, long long* cyc, int off, int n) {
  __shared__ __attribute__((aligned(16))) uint8_t s[16384 + 64];
  for (int i = threadIdx.x; i < 16384 + 64; i += blockDim.x) s[i] = (uint8_t)i;
  __syncthreads();
  const int l = threadIdx.x & 63;
  const uint32_t addr = (uint32_t)(uintptr_t)(s) + 16 * l + off + 1024 * (threadIdx.x >> 6);
  uint32_t acc = 0;
  const long long t0 = clock64();
  for (int i = 0; i < n; ++i) {
    uint4 w0, w1, w2, w3, w4, w5, w6, w7;
    asm volatile("ds_read_b128 %0, %8\n\tds_read_b128 %1, %8 offset:4096\n\tds_read_b128 %2, %8 offset:8192\n\t"
                 "ds_read_b128 %3, %8 offset:12288\n\tds_read_b128 %4, %8 offset:2048\n\tds_read_b128 %5, %8 offset:6144\n\t"
                 "ds_read_b128 %6, %8 offset:10240\n\tds_read_b128 %7, %8 offset:14336\n\ts_waitcnt lgkmcnt(0)"
                 : "=v"(w0), "=v"(w1), "=v"(w2), "=v"(w3), "=v"(w4), "=v"(w5), "=v"(w6), "=v"(w7) : "v"(addr) : "memory");
    acc += w0.x ^ w1.y ^ w2.z ^ w3.w ^ w4.x ^ w5.y ^ w6.z ^ w7.w;
  }
  const long long t1 = clock64();
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

static void dump(const char* dir, const char* name, const void* p, size_t bytes) {
  char path[512];
  snprintf(path, sizeof(path), "%s/%s", dir, name);
  FILE* f = fopen(path, "wb");
  fwrite(p, 1, bytes, f);
  fclose(f);
}

int main(int argc, char** argv) {
  const char* dir = argc > 1 ? argv[1] : ".";
  {
    float* d;
    const size_t n16 = 2048 * 64 * 4, n32 = 2048 * 64 * 16;
    CK(hipMalloc(&d, n32 * 4));
    hipLaunchKernelGGL(k_layout16, dim3(2048), dim3(64), 0, 0, d);
    CK(hipDeviceSynchronize());
    std::vector<float> h(n32);
    CK(hipMemcpy(h.data(), d, n16 * 4, hipMemcpyDeviceToHost));
    dump(dir, "layout16.f32", h.data(), n16 * 4);
    hipLaunchKernelGGL(k_layout32, dim3(2048), dim3(64), 0, 0, d);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h.data(), d, n32 * 4, hipMemcpyDeviceToHost));
    dump(dir, "layout32.f32", h.data(), n32 * 4);
    CK(hipFree(d));
    printf("layout probes done\n");
  }
  {
    const int P = 64;
    std::vector<float> av(P * 64 * 8), bv(P * 64 * 16);
    std::vector<int> ai(P * 64);
    srand(7);
    for (auto& x : av) x = (float)(rand() % 17 - 8);
    for (auto& x : bv) x = (float)(rand() % 17 - 8);
    for (auto& x : ai) x = (int)(((uint32_t)rand() << 16) ^ (uint32_t)rand());
    float *dav, *dbv, *dout;
    int* dai;
    CK(hipMalloc(&dav, av.size() * 4));
    CK(hipMalloc(&dbv, bv.size() * 4));
    CK(hipMalloc(&dai, ai.size() * 4));
    CK(hipMalloc(&dout, P * 64 * 4 * 4));
    CK(hipMemcpy(dav, av.data(), av.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dbv, bv.data(), bv.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dai, ai.data(), ai.size() * 4, hipMemcpyHostToDevice));
    dump(dir, "rand_a.f32", av.data(), av.size() * 4);
    dump(dir, "rand_b.f32", bv.data(), bv.size() * 4);
    dump(dir, "rand_i.i32", ai.data(), ai.size() * 4);
    std::vector<float> h(P * 64 * 4);
    for (int abid = 0; abid < 2; ++abid) {
      hipLaunchKernelGGL(k_random16, dim3(P), dim3(64), 0, 0, dav, dai, dbv, dout, abid);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(h.data(), dout, h.size() * 4, hipMemcpyDeviceToHost));
      dump(dir, abid ? "rand_out_abid1.f32" : "rand_out_abid0.f32", h.data(), h.size() * 4);
    }
    float* dout32;
    CK(hipMalloc(&dout32, P * 64 * 16 * 4));
    hipLaunchKernelGGL(k_random32, dim3(P), dim3(64), 0, 0, dav, dai, dbv, dout32);
    CK(hipDeviceSynchronize());
    std::vector<float> h32(P * 64 * 16);
    CK(hipMemcpy(h32.data(), dout32, h32.size() * 4, hipMemcpyDeviceToHost));
    dump(dir, "rand32_out.f32", h32.data(), h32.size() * 4);
    printf("random probes done\n");
  }
  {
    float* sink;
    long long* cyc;
    const int NB = 1024, n = 2000;
    CK(hipMalloc(&sink, NB * 64 * 4));
    CK(hipMalloc(&cyc, NB * 8));
    std::vector<long long> hc(NB);
    const char* names[4] = {"smfmac_f32_16x16x64_bf16", "mfma_f32_16x16x32_bf16", "smfmac_f32_32x32x32_bf16",
                            "mfma_f32_32x32x16_bf16"};
    for (int kind = 0; kind < 4; ++kind) {
      for (int rep = 0; rep < 2; ++rep) {
        if (kind == 0) hipLaunchKernelGGL(k_rate<0>, dim3(NB), dim3(64), 0, 0, sink, cyc, n);
        if (kind == 1) hipLaunchKernelGGL(k_rate<1>, dim3(NB), dim3(64), 0, 0, sink, cyc, n);
        if (kind == 2) hipLaunchKernelGGL(k_rate<2>, dim3(NB), dim3(64), 0, 0, sink, cyc, n);
        if (kind == 3) hipLaunchKernelGGL(k_rate<3>, dim3(NB), dim3(64), 0, 0, sink, cyc, n);
        CK(hipDeviceSynchronize());
      }
      CK(hipMemcpy(hc.data(), cyc, NB * 8, hipMemcpyDeviceToHost));
      double s = 0;
      for (auto c : hc) s += (double)c;
      printf("rate %-28s %.2f cycles (s_memtime) per instruction per wave\n", names[kind], s / NB / (4.0 * n));
    }
  }
  {
    uint32_t* d;
    long long* cyc;
    CK(hipMalloc(&d, 2 * 64 * 4 * 4 * 8));
    CK(hipMalloc(&cyc, 8 * 8));
    std::vector<uint32_t> h(64 * 4);
    std::vector<long long> hc(1);
    for (int off = 0; off < 16; off += 2) {
      hipLaunchKernelGGL(k_lds, dim3(1), dim3(64), 0, 0, d, cyc, off, 4000);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hc.data(), cyc, 8, hipMemcpyDeviceToHost));
      int bad = 0;
      for (int l = 0; l < 64; ++l)
        for (int b = 0; b < 16; ++b) {
          const int i = 32 * l + off + b;
          const uint8_t want = (uint8_t)(i * 7 + (i >> 8));
          const uint8_t got = (uint8_t)(h[l * 4 + b / 4] >> (8 * (b % 4)));
          bad += want != got;
        }
      printf("ds_read_b128 offset %2d: %s (%d wrong bytes), %.2f cycles per 4 reads + wait\n", off,
             bad ? "WRONG" : "exact", bad, (double)hc[0] / 4000.0);
    }
  }
  {
    uint32_t* d;
    long long* cyc;
    CK(hipMalloc(&d, 256 * 256 * 4));
    CK(hipMalloc(&cyc, 256 * 8));
    std::vector<long long> hc(256);
    for (int off = 0; off < 8; off += 2) {
      hipLaunchKernelGGL(k_lds_rate, dim3(256), dim3(256), 0, 0, d, cyc, off, 2000);
      CK(hipDeviceSynchronize());
      hipLaunchKernelGGL(k_lds_rate, dim3(256), dim3(256), 0, 0, d, cyc, off, 2000);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(hc.data(), cyc, 256 * 8, hipMemcpyDeviceToHost));
      double sm = 0;
      for (auto c : hc) sm += (double)c;
      printf("ds_read_b128 throughput, offset %d: %.2f s_memtime cycles per wave-instruction (4 waves/CU, 8 in flight)\n",
             off, sm / 256 / (2000.0 * 8));
    }
  }
  return 0;
}
