// craft_obs.h — the observation half of a tick, shared by the tick kernel
// (craft_tile.hip) and the multi-tick rollout kernel (craft_rollout.hip):
// D scatters CraftState.features() (craft.py:296-330) of each env of a tile into
// u8 rows in LDS, E streams the rows to HBM in the handle's observation format.
#pragma once
#include "craft_device.h"

namespace craft {

typedef unsigned int obs_vec __attribute__((ext_vector_type(4)));

// 16 bytes of output from the tile's u8 feature rows: 4 fp32 (v_cvt_f32_ubyte),
// 8 bf16 (the high half of the exact fp32 value of a byte) or 16 u8.
template <int FMT>
__device__ __forceinline__ obs_vec pack16(const uint8_t* s_obs, int sidx) {
  if (FMT == CRAFT_OBS_F32) {
    const uint32_t w = reinterpret_cast<const uint32_t*>(s_obs)[sidx];
    return obs_vec{__float_as_uint((float)(w & 0xff)), __float_as_uint((float)((w >> 8) & 0xff)),
                   __float_as_uint((float)((w >> 16) & 0xff)), __float_as_uint((float)(w >> 24))};
  } else if (FMT == CRAFT_OBS_BF16) {
    const uint2 w = reinterpret_cast<const uint2*>(s_obs)[sidx];
    auto bf = [](uint32_t b) { return __float_as_uint((float)b) >> 16; };
    auto two = [&](uint32_t x) { return bf(x & 0xff) | (bf((x >> 8) & 0xff) << 16); };
    return obs_vec{two(w.x), two(w.x >> 16), two(w.y), two(w.y >> 16)};
  } else {
    const uint4 w = reinterpret_cast<const uint4*>(s_obs)[sidx];
    return obs_vec{w.x, w.y, w.z, w.w};
  }
}

// Phase E: the tile's rows are contiguous in the output, so the whole tile is one
// flat stream of 16-byte buffer stores (32-bit offsets off one wave-uniform
// descriptor); the cache policy is a tuning knob (craft_sim_tune).  NTHR threads
// (tid in [0, NTHR)) share the stream; with ZERO they also clear every byte they
// read, leaving the rows zeroed for the next scatter.
template <int FMT, int NTHR = kThreads, bool ZERO = false, int U = 4>
__device__ __forceinline__ void stream_obs(uint8_t* s_obs, void* obs, int64_t env0, int F, int nE,
                                           int policy, int tid) {
  constexpr int ESZ = FMT == CRAFT_OBS_F32 ? 4 : (FMT == CRAFT_OBS_BF16 ? 2 : 1);
  constexpr int PER = 16 / ESZ;                // values per 16-byte store
  const int total = nE * F;
  const int nv = total / PER;
  uint8_t* tile_out = static_cast<uint8_t*>(obs) + env0 * (int64_t)F * ESZ;
  const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(tile_out, 0, total * ESZ, 0x00020000);
  // U: independent 16-byte stores in flight per lane
  for (int base = tid; base < nv; base += U * NTHR) {
    obs_vec o[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int sidx = base + u * NTHR;
      if (sidx < nv) {
#ifdef CRAFT_ABL_NOLDS
        o[u] = obs_vec{(unsigned)sidx, 0u, 0u, 0u};
        if (false) {
#else
        o[u] = pack16<FMT>(s_obs, sidx);
        if (ZERO) {
#endif
          if (FMT == CRAFT_OBS_F32) reinterpret_cast<uint32_t*>(s_obs)[sidx] = 0u;
          else if (FMT == CRAFT_OBS_BF16) reinterpret_cast<uint2*>(s_obs)[sidx] = make_uint2(0u, 0u);
          else reinterpret_cast<uint4*>(s_obs)[sidx] = make_uint4(0u, 0u, 0u, 0u);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int sidx = base + u * NTHR;
      if (sidx < nv) {
        if (policy == 1) __builtin_amdgcn_raw_buffer_store_b128(o[u], rsrc, sidx * 16, 0, 2);         // nt
        else if (policy == 2) __builtin_amdgcn_raw_buffer_store_b128(o[u], rsrc, sidx * 16, 0, 16);   // sc1
        else __builtin_amdgcn_raw_buffer_store_b128(o[u], rsrc, sidx * 16, 0, 0);
      }
    }
  }
  for (int f = nv * PER + tid; f < total; f += NTHR) {       // the last few values of the tile
    const uint32_t b = s_obs[f];
    if (ZERO) s_obs[f] = 0;
    if (FMT == CRAFT_OBS_F32) reinterpret_cast<float*>(tile_out)[f] = (float)b;
    else if (FMT == CRAFT_OBS_BF16) reinterpret_cast<uint16_t*>(tile_out)[f] = (uint16_t)(__float_as_uint((float)b) >> 16);
    else tile_out[f] = (uint8_t)b;
  }
}

// Phase D for one env, split over P lanes (right after the envs' transitions, no
// workgroup barrier): the features() row (craft.py:296-330) as work units, unit 0 =
// local one-hot + inventory + dir one-hot, and part p of the env does units p, p + P,
// ...  `ag` = x | y<<8 | dir<<16; `row` is zeroed.  The block-max-pooled one-hots
// (cells outside the grid are pad_slice's zero padding, misc/array.py:3-25):
//   3x3 windows: unit 1 + bi = block row bi, its 27 cells read back to back and
//     OR-ed into one kind mask per block, one byte per kind present;
//   5x5 and 7x7: unit 1 + c = grid column c of the window.  The blocks tile the
//     window without overlap, so each in-grid cell sets the byte of its kind in its
//     own block: one read per grid cell (144 at 12x12), not one per block cell (625).
// (tools/ab.sh: per column is 4 % faster than per block row for w = 5 and 2 % slower
// for w = 3, where the window holds 81 cells and the masks save writes.)
// RUN: the local one-hot's writes at a running offset (see below; off for 3x3 windows and in the
// teacher rollout kernel, whose registers are capped anyway: 973-975 against 981 us there).
template <int WIN, int P, bool RUN = (WIN > 3)>
__device__ __forceinline__ void scatter_env_part(const SimView& v, const uint8_t* g, const uint8_t* iv,
                                                 uint32_t ag, uint8_t* row, int part) {
  const int x = ag & 0xff, y = (ag >> 8) & 0xff, dir = (ag >> 16) & 3;
  const int W = v.W, H = v.H, K = v.K;
  constexpr int W2 = WIN * WIN, hw = WIN / 2, bh = W2 / 2;
  constexpr int NR = W2 < CRAFT_MAX_DIM ? W2 : CRAFT_MAX_DIM;       // window rows inside a grid
  const int L = W2 * K;
  const int cxa = max(x - bh, 0), cxb = min(x - bh + W2 - 1, W - 1);
  const int cya = max(y - bh, 0), cyb = min(y - bh + W2 - 1, H - 1);
  const int nc = WIN == 3 ? WIN : cxb - cxa + 1;                    // pooled units
#pragma unroll 1
  for (int unit = part; unit <= nc; unit += P) {
    if (unit == 0) {
      // every read is unconditional (clamped index, result masked), so the compiler issues
      // them back to back instead of one LDS round trip per predicated cell
      int kk[WIN * WIN];
#pragma unroll
      for (int i = 0; i < WIN; ++i)                                 // local one-hot
#pragma unroll
        for (int j = 0; j < WIN; ++j) {
          const int cx = x - hw + i, cy = y - hw + j;
          const bool ok = (unsigned)cx < (unsigned)W && (unsigned)cy < (unsigned)H;
          const int k = g[min(max(cx, 0), W - 1) * H + min(max(cy, 0), H - 1)];
          kk[i * WIN + j] = ok ? k : 0;
        }
      if constexpr (!RUN) {
#pragma unroll
        for (int c = 0; c < WIN * WIN; ++c)
          if (kk[c]) row[c * K + kk[c]] = 1;
      } else {
        // a running 32-bit offset: at 5x5 / 7x7 the c * K products, hoisted out of the unit loop as
        // 64-bit pointers, held 2 * WIN * WIN registers through every unit (tile_kernel<5>: 108 -> 95
        // VGPRs, rollout_kernel<5>: 204 -> 156; 1018-1028 -> 1004-1015 us per 20 ticks)
        uint32_t off = 0;
#pragma unroll
        for (int c = 0; c < WIN * WIN; ++c) {
          if (kk[c]) row[off + kk[c]] = 1;
          off += K;
          asm volatile("" : "+v"(off));
        }
      }
      {                                                             // inventory counts
        const uint32_t* ivw = reinterpret_cast<const uint32_t*>(iv);   // 8 independent reads
        uint32_t w[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) w[q] = ivw[q];
        uint8_t* irow = row + 2 * L;                                  // the row is zeroed: only the
        uint32_t nz = 0;                                              // nonzero counts are written
#pragma unroll
        for (int q = 0; q < 8; ++q) nz |= byte_tops(nonzero_bytes(w[q])) << (4 * q);
        nz &= K >= 32 ? ~0u : ((1u << K) - 1u);
        while (nz) {
          const int k = __ffs(nz) - 1;
          uint32_t wk = 0;
#pragma unroll
          for (int q = 0; q < 8; ++q) wk = (q == (k >> 2)) ? w[q] : wk;
          irow[k] = (uint8_t)(wk >> (8 * (k & 3)));
          nz &= nz - 1;
        }
      }
      row[2 * L + K + dir] = 1;                                     // dir one-hot
    } else if (WIN == 3) {
      const int bi = unit - 1;                                      // block row bi
      uint32_t m[WIN];
#pragma unroll
      for (int bj = 0; bj < WIN; ++bj) m[bj] = 0;
      const int x0 = x - bh + bi * WIN;
#pragma unroll
      for (int ii = 0; ii < WIN; ++ii) {
        const int cx = x0 + ii;
        const bool okx = (unsigned)cx < (unsigned)W;
        const uint8_t* col = g + min(max(cx, 0), W - 1) * H;
#pragma unroll
        for (int bj = 0; bj < WIN; ++bj)
#pragma unroll
          for (int jj = 0; jj < WIN; ++jj) {
            const int cy = y - bh + bj * WIN + jj;
            const uint32_t k = col[min(max(cy, 0), H - 1)];          // unconditional read
            m[bj] |= (okx && (unsigned)cy < (unsigned)H) ? (1u << k) : 0u;
          }
      }
#pragma unroll
      for (int bj = 0; bj < WIN; ++bj) {
        uint32_t msk = m[bj] & ~1u;                                 // kind 0 = empty
        uint8_t* brow = row + L + (bi * WIN + bj) * K;
        while (msk) {
          brow[__ffs(msk) - 1] = 1;
          msk &= msk - 1;
        }
      }
    } else {
      // column cx of the window, block row bi; its cells' reads are issued back to back
      // (clamped, masked), then each non-empty cell sets its byte
      const int cx = cxa + unit - 1;
      const int bi = (cx - x + bh) / WIN;
      const uint8_t* col = g + cx * H;
      uint8_t* brow = row + L + bi * WIN * K;
      int kk[NR];
#pragma unroll
      for (int j = 0; j < NR; ++j) kk[j] = col[min(cya + j, H - 1)];
#pragma unroll
      for (int j = 0; j < NR; ++j) {
        const int cy = cya + j;
        if (cy <= cyb && kk[j]) brow[((cy - y + bh) / WIN) * K + kk[j]] = 1;   // kind 0 = empty
      }
    }
  }
}

// Phase D: all threads scatter the non-zero bytes of each env's features() row
// into the zeroed u8 rows s_obs[TILE][F] (scatter_env_part, NTHR / TILE threads per
// env).  s_agent[e] = x | y<<8 | dir<<16 | 1<<24 for a live env (0 = skip).
template <int WIN, int TILE, int NTHR = kThreads>
__device__ __forceinline__ void scatter_features(const SimView& v, const uint8_t* s_grid,
                                                 const uint8_t* s_inv, const uint32_t* s_agent,
                                                 uint8_t* s_obs, int nE, int tid) {
  constexpr int kParts = NTHR / TILE;            // threads per env
  const int e = tid % TILE, part = tid / TILE;
  const uint32_t ag = s_agent[e];
  if (e < nE && (ag >> 24))
    scatter_env_part<WIN, kParts>(v, s_grid + e * v.GS, s_inv + e * kInvStride, ag, s_obs + e * v.F, part);
}

}  // namespace craft
