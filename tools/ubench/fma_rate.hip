// Issue-rate microbenchmark (MI355X): v_fma_f32 vs v_pk_fma_f32 vs v_fma_mix_f32 (f32 += f32 * f16) vs
// v_cvt_f32_ubyte0 + v_fma_f32, one dependency chain per 8 accumulators, 4 waves per SIMD.  Prints ns per
// wave-instruction per SIMD.  Build: hipcc --offload-arch=gfx950 -O3 fma_rate.hip -o fma_rate
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, int iters, float s) {
  float a[8];
  uint32_t x = threadIdx.x * 0x01010101u;
  for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 0.001f + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (MODE == 0) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(s), "v"(a[(i + 1) & 7]));
      if (MODE == 1) {
        typedef float f2 __attribute__((ext_vector_type(2)));
        f2 v = {a[i], a[(i + 4) & 7]};
        f2 w = {s, s};
        asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(v) : "v"(w), "v"(w));
        a[i] = v.x;
      }
      if (MODE == 2) asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[0,1,0]" : "+v"(a[i]) : "v"(s), "v"(x));
      if (MODE == 3) {
        float f;
        asm volatile("v_cvt_f32_ubyte0 %0, %1" : "=v"(f) : "v"(x));
        asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a[i]) : "v"(s), "v"(f));
      }
    }
  }
  float t = 0.f;
  for (int i = 0; i < 8; ++i) t += a[i];
  out[blockIdx.x * 256 + threadIdx.x] = t;
}

int main() {
  float* out;
  hipMalloc(&out, 256 * 4096 * sizeof(float));
  const int iters = 4096, blocks = 256 * 4;  // 4 blocks of 4 waves per CU -> 4 waves per SIMD
  const char* names[4] = {"v_fma_f32", "v_pk_fma_f32 (2 MAC)", "v_fma_mix_f32 (f16 operand)", "cvt_f32_ubyte0 + v_fma_f32"};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int mode = 0; mode < 4; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f);
      if (mode == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f);
      if (mode == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f);
      if (mode == 3) hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      // per SIMD: 4 waves x iters x 8 instructions (mode 3: 16)
      const double inst = 4.0 * iters * 8.0 * (mode == 3 ? 2 : 1);
      if (rep) printf("%-30s %8.3f ms  %6.3f ns per wave-instruction per SIMD\n", names[mode], ms, ms * 1e6 / inst);
    }
  }
  hipFree(out);
  return 0;
}
