// Url-id bitmaps of the large index lists (DList::bm), device side.
//
// 16-B units of BM_UNIT_IDS = 96 url ids each (yrwi_internal.h).  Unit v:
//   uint32 x, y, z  the bits of ids 96v .. 96v+31, +32..+63, +64..+95
//   uint32 w        the list position of the unit's first id (its rank)
// One 16-B load gives an id's membership and, for a member, its list position
// (rank + the bits below it).  Rounds 1-4 used 16 B per 64 ids (a 64-bit word
// and a 64-bit rank): half of every line was rank, so a probe of a sparse key
// stream fetched one 128-B line per 512 ids; this layout fetches one per 768.
// (A 128-B line of 896 ids behind a 16-B rank header took one more load per
// key: C3 k_probe 783 -> 721 us, but C2's L2-resident probes 116 -> 129 us.)
#pragma once
#include "yrwi_internal.h"

namespace yrwi {

struct BmAt {
  uint32_t unit;  // unit index
  uint32_t bit;   // bit 0..95 within the unit
};

__device__ __forceinline__ BmAt bm_at(uint32_t u) {
  BmAt a;
  a.unit = u / (uint32_t)BM_UNIT_IDS;
  a.bit = u - a.unit * (uint32_t)BM_UNIT_IDS;
  return a;
}

// membership of the id at a in its unit U, and its list position
__device__ __forceinline__ bool bm_test(const BmAt& a, uint4 U) {
  const uint32_t w = a.bit >> 5;
  const uint32_t x = w == 0 ? U.x : w == 1 ? U.y : U.z;
  return (x >> (a.bit & 31u)) & 1u;
}
__device__ __forceinline__ int32_t bm_pos(const BmAt& a, uint4 U) {
  const uint32_t w = a.bit >> 5, below = (1u << (a.bit & 31u)) - 1u;
  const uint32_t r = w == 0 ? __popc(U.x & below)
                   : w == 1 ? __popc(U.x) + __popc(U.y & below)
                            : __popc(U.x) + __popc(U.y) + __popc(U.z & below);
  return (int32_t)(U.w + r);
}

// a unit through a buffer resource over the bitmap
__device__ __forceinline__ uint4 bm_unit(__amdgpu_buffer_rsrc_t r, const BmAt& a) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(a.unit * 16u), 0, 0));
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t bm_rsrc(const uint64_t* bm) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint64_t*>(bm), 0, 0x7FFFFFFF, 0x00020000);
}

}  // namespace yrwi
