// craft_bits.h — sets of grid cells as NW 32-bit words in registers, for the
// bitset BFS of the teacher (craft_teacher.hip) and the connectivity checks of
// the scenario generator (craft_scenarios.hip).
#pragma once
#include <climits>

#include "craft_device.h"

namespace craft {

// A set of cells as NW 32-bit words (cell c = bit c & 31 of word c >> 5).
// Multi-word shifts use v_alignbit_b32 (one funnel shift per word).
template <int NW>
struct Bits {
  uint32_t w[NW];
};

template <int NW>
__device__ __forceinline__ Bits<NW> bzero() {
  Bits<NW> r;
#pragma unroll
  for (int i = 0; i < NW; ++i) r.w[i] = 0u;
  return r;
}
template <int NW>
__device__ __forceinline__ Bits<NW> band(const Bits<NW>& a, const Bits<NW>& b) {
  Bits<NW> r;
#pragma unroll
  for (int i = 0; i < NW; ++i) r.w[i] = a.w[i] & b.w[i];
  return r;
}
template <int NW>
__device__ __forceinline__ Bits<NW> bor(const Bits<NW>& a, const Bits<NW>& b) {
  Bits<NW> r;
#pragma unroll
  for (int i = 0; i < NW; ++i) r.w[i] = a.w[i] | b.w[i];
  return r;
}
template <int NW>
__device__ __forceinline__ Bits<NW> bandn(const Bits<NW>& a, const Bits<NW>& b) {
  Bits<NW> r;
#pragma unroll
  for (int i = 0; i < NW; ++i) r.w[i] = a.w[i] & ~b.w[i];
  return r;
}
template <int NW>
__device__ __forceinline__ bool bany(const Bits<NW>& a) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) x |= a.w[i];
  return x != 0u;
}
template <int NW>
__device__ __forceinline__ bool btest(const Bits<NW>& a, int p) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) x |= (i == (p >> 5)) ? a.w[i] : 0u;
  return (x >> (p & 31)) & 1u;
}
template <int NW>
__device__ __forceinline__ Bits<NW> bbit(int p) {
  Bits<NW> r;
#pragma unroll
  for (int i = 0; i < NW; ++i) r.w[i] = (i == (p >> 5)) ? (1u << (p & 31)) : 0u;
  return r;
}
template <int NW>
__device__ __forceinline__ int blowest(const Bits<NW>& a) {   // INT_MAX if empty
  int r = INT_MAX;
#pragma unroll
  for (int i = NW - 1; i >= 0; --i)
    if (a.w[i]) r = i * 32 + __ffs(a.w[i]) - 1;
  return r;
}
template <int NW>
__device__ __forceinline__ int bhighest(const Bits<NW>& a) {  // -1 if empty
  int r = -1;
#pragma unroll
  for (int i = 0; i < NW; ++i)
    if (a.w[i]) r = i * 32 + 31 - __clz(a.w[i]);
  return r;
}
// The cells [lo, hi) as a set (0 <= lo <= hi <= 32 * NW).
template <int NW>
__device__ __forceinline__ Bits<NW> brange(int lo, int hi) {
  Bits<NW> r;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const int a = max(lo - 32 * i, 0), b = min(hi - 32 * i, 32);
    r.w[i] = b <= a ? 0u : ((b - a >= 32 ? ~0u : ((1u << (b - a)) - 1u)) << a);
  }
  return r;
}
template <int NW>
__device__ __forceinline__ int bcount(const Bits<NW>& a) {
  int c = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) c += __popc(a.w[i]);
  return c;
}

// p -> p + d for every member (0 < |d| < 32); members shifted past either end drop out.
template <int NW>
__device__ __forceinline__ Bits<NW> bshift(const Bits<NW>& a, int d) {
  Bits<NW> r;
  if (d > 0) {
    r.w[0] = a.w[0] << d;
#pragma unroll
    for (int i = 1; i < NW; ++i) r.w[i] = __builtin_amdgcn_alignbit(a.w[i], a.w[i - 1], 32 - d);
  } else {
    const int s = -d;
#pragma unroll
    for (int i = 0; i + 1 < NW; ++i) r.w[i] = __builtin_amdgcn_alignbit(a.w[i + 1], a.w[i], s);
    r.w[NW - 1] = a.w[NW - 1] >> s;
  }
  return r;
}
// bshift for a shift amount known only at run time, which may differ between the
// lanes of a wave (the quad-parallel teacher): branch-free, so lanes shifting up and
// lanes shifting down do not diverge.  Word i of the result is the funnel shift of the
// pair (sel[i+1], sel[i]), sel[j] = a[j-1] for an upward shift (amount 32 - d) and a[j]
// for a downward one (amount -d).
template <int NW>
__device__ __forceinline__ Bits<NW> bshift_var(const Bits<NW>& a, int d) {
  const bool up = d > 0;
  const uint32_t t = up ? (uint32_t)(32 - d) : (uint32_t)(-d);
  uint32_t sel[NW + 1];
#pragma unroll
  for (int j = 0; j <= NW; ++j) {
    const uint32_t lo = j >= 1 ? a.w[j - 1] : 0u, hi = j < NW ? a.w[j] : 0u;
    sel[j] = up ? lo : hi;
  }
  Bits<NW> r;
#pragma unroll
  for (int i = 0; i < NW; ++i) r.w[i] = __builtin_amdgcn_alignbit(sel[i + 1], sel[i], t);
  return r;
}

}  // namespace craft
