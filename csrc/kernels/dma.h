// Raw buffer-resource loads shared by the LDS-DMA kernels (conv3d.hip, gemm1x1.hip).
#pragma once
#include "common.h"

namespace nidt {

// Raw buffer resources (stride 0, range = bytes): an offset at or past the range reads zeros, which replaces the
// zero page, the 64-bit address arithmetic and the per-row bounds selects of the global_load_lds version (the
// issue loop was VALU-bound: 4.8 VALU per MFMA, profiles/r1_pmc_v4.txt).
typedef int i32x4_t __attribute__((ext_vector_type(4)));
typedef int i32x2_t __attribute__((ext_vector_type(2)));
__device__ i32x2_t nidt_raw_buffer_load_v2i32(i32x4_t rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.load.v2i32");
__device__ int nidt_raw_buffer_load_i32(i32x4_t rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.load.i32");
__device__ void nidt_raw_buffer_load_lds(i32x4_t rsrc, __attribute__((address_space(3))) uint32_t* lds, int size,
                                         int voffset, int soffset, int offset, int aux)
    __asm("llvm.amdgcn.raw.buffer.load.lds");
__device__ i32x4_t nidt_raw_buffer_load_v4i32(i32x4_t rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.load.v4i32");
__device__ void nidt_raw_buffer_store_v4i32(i32x4_t data, i32x4_t rsrc, int voffset, int soffset, int aux)
    __asm("llvm.amdgcn.raw.buffer.store.v4i32");
constexpr int kBufOOB = (int)0x80000000u;

__device__ __forceinline__ i32x4_t make_rsrc(const void* base, uint32_t bytes) {
  const uint64_t p = reinterpret_cast<uint64_t>(base);
  i32x4_t r;
  r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)p);
  r.y = __builtin_amdgcn_readfirstlane((int)(uint32_t)(p >> 32));  // stride 0 (48-bit address)
  r.z = __builtin_amdgcn_readfirstlane((int)bytes);
  r.w = 0x00020000;
  return r;
}

__device__ __forceinline__ void blds16(i32x4_t rsrc, int voffset, uint16_t* lds_wave_base) {
  nidt_raw_buffer_load_lds(rsrc, (__attribute__((address_space(3))) uint32_t*)(lds_wave_base), 16, voffset, 0, 0, 0);
}

// The same 16-B LDS-DMA issued from inline asm: invisible to the compiler's waitcnt pass, which otherwise treats the
// DMA as a write to LDS that every later ds_read may alias and puts a vmcnt wait for it in front of them (the stage
// in flight is then waited for before the current one is computed).  Kernels using it order their DMA with their
// own counted s_waitcnt vmcnt and barriers, and use M0 for nothing else.
__device__ __forceinline__ void blds16_asm(i32x4_t rsrc, int voffset, uint16_t* lds_wave_base) {
  const uint32_t m0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint16_t*)lds_wave_base;
  asm volatile("s_mov_b32 m0, %0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds" ::"s"(m0), "v"(voffset), "s"(rsrc)
               : "memory");
}

}  // namespace nidt
