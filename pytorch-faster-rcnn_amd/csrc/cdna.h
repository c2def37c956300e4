// CDNA4 building blocks shared by the kernels: wave-uniform buffer descriptors,
// DPP wave reductions, LDS-DMA (buffer_load ... lds) and counted vmcnt waits.
#pragma once
#include "common.h"

namespace frh {

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p, int64_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a), hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane((int)bytes);
  void* q = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(q, 0, n, 0x00020000);
}

// Wave-wide min / max with DPP row ops (no LDS round trip); result in every lane.
template <bool kMin>
__device__ __forceinline__ int wave_minmax_i32(int v) {
  const int id = kMin ? 0x7fffffff : (int)0x80000000;
  auto op = [](int a, int b) { return kMin ? min(a, b) : max(a, b); };
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0xb1, 0xf, 0xf, false));   // quad_perm [1,0,3,2]
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x4e, 0xf, 0xf, false));   // quad_perm [2,3,0,1]
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x141, 0xf, 0xf, false));  // row_half_mirror
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x140, 0xf, 0xf, false));  // row_mirror
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x142, 0xa, 0xf, false));  // row_bcast15
  v = op(v, __builtin_amdgcn_update_dpp(id, v, 0x143, 0xc, 0xf, false));  // row_bcast31
  return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ int wave_min_i32(int v) { return wave_minmax_i32<true>(v); }
__device__ __forceinline__ int wave_max_i32(int v) { return wave_minmax_i32<false>(v); }

// buffer_load_dword{,x4} ... lds: kBytes per lane into LDS at lds + 4*kBytes/4 * lane.
// The 16-byte form is a gfx950 instruction the host pass of hipcc cannot check,
// hence the device-pass guard (the host never runs device code).
template <int kBytes>
__device__ __forceinline__ void lds_dma(__amdgpu_buffer_rsrc_t r, float* lds, int voff, int soff) {
#if defined(__HIP_DEVICE_COMPILE__)
  static_assert(kBytes == 4 || kBytes == 16, "LDS-DMA width");
  if constexpr (kBytes == 16)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
  else
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 4, voff, soff, 0, 0);
#endif
}

// gfx950 cache-policy bits of buffer loads / stores (the builtins' aux operand)
constexpr int kCpolSC0 = 1, kCpolNT = 2, kCpolSC1 = 16;

// the same with the destination given as a wave-uniform LDS byte address; kAux is
// the gfx950 cache policy (0 default, 1 sc0, 2 nt, 16 sc1)
template <int kBytes, int kAux = 0>
__device__ __forceinline__ void lds_dma_at(__amdgpu_buffer_rsrc_t r, uint32_t lds_addr, int voff, int soff) {
#if defined(__HIP_DEVICE_COMPILE__)
  static_assert(kBytes == 4 || kBytes == 16, "LDS-DMA width");
  auto* p = (__attribute__((address_space(3))) void*)(uintptr_t)lds_addr;
  if constexpr (kBytes == 16)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, p, 16, voff, soff, 0, kAux);
  else
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, p, 4, voff, soff, 0, kAux);
#endif
}

// s_waitcnt vmcnt(N) with every other counter left alone (gfx9 encoding).  The
// compiler does not wait for LDS-DMA data before ds_reads: these are explicit.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}


}  // namespace frh
