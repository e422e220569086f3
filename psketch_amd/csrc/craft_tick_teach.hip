// craft_tick_teach.hip — craft_step_teach: one rollout tick fused with the
// DemonstrationTeacher on every env's new state (config 5: a DAgger label per
// tick).  The tile kernel (craft_tile.h) with TILE * TL teacher threads beside
// its 256: the tick's waves stream the observations while the teacher waves run
// teach_env on the grid rows the tick left in LDS, so the teacher reads no grid
// from HBM and needs no launch of its own.  For 3x3 windows the two-tile tick
// kernel (craft_tick2.h) serves craft_step_teach.
#include "craft_tick2.h"
#include "craft_tile.h"

namespace craft {

template <int WIN, int TL, int NW, int TILE>
static hipError_t launch_tt(const SimView& v, const TileArgs& a, size_t lds, hipStream_t st) {
  const int64_t tiles = (a.n + TILE - 1) / TILE;
  if (tiles == 0) return hipSuccess;
  // 5x5 / 7x7 windows, 64-env tiles: rows past 64 KiB
  const hipError_t e = ensure_lds<&tile_kernel<WIN, MODE_TICK, TILE, TL, NW>>(lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((tile_kernel<WIN, MODE_TICK, TILE, TL, NW>), dim3((unsigned)tiles),
                     dim3(tile_tick_threads(TILE, TL) + TILE * TL), lds, st, v, a);
  return hipGetLastError();
}

// 3x3 windows: 64-env tiles; wider ones 32 (the handle's default tile) or 64
template <int TL, int NW>
static hipError_t launch_tt_win(int win, int tile, const SimView& v, const TileArgs& a, size_t lds, hipStream_t st) {
  switch (win) {
    case 3: return launch_tt<3, TL, NW, kMaxTileEnvs>(v, a, lds, st);
    case 5: return tile == 32 ? launch_tt<5, TL, NW, 32>(v, a, lds, st) : launch_tt<5, TL, NW, kMaxTileEnvs>(v, a, lds, st);
    default: return tile == 32 ? launch_tt<7, TL, NW, 32>(v, a, lds, st) : launch_tt<7, TL, NW, kMaxTileEnvs>(v, a, lds, st);
  }
}

template <int TL>
static hipError_t launch_tt_nw(int nw, int win, int tile, const SimView& v, const TileArgs& a, size_t lds, hipStream_t st) {
  // nw = 32-bit words per BFS cell set (craft_teach.h: the band of columns 1 .. W-2):
  // 8x8 -> 2, 10x10 -> 3 (run as 4), 12x12 -> 4, 16x16 -> 7 (run as 8)
  if (nw <= 2) return launch_tt_win<TL, 2>(win, tile, v, a, lds, st);
  if (nw <= 4) return launch_tt_win<TL, 4>(win, tile, v, a, lds, st);
  if (nw <= 5) return launch_tt_win<TL, 5>(win, tile, v, a, lds, st);
  return launch_tt_win<TL, 8>(win, tile, v, a, lds, st);
}

// tl = teacher lanes per env: 2 (a pair per env, 2 teacher waves), 4 (a quad, 4 waves) or
// 1 (one wave).
hipError_t launch_tick_teach(int tl, int nw, int win, int tile, const SimView& v, const TileArgs& a, size_t lds,
                             hipStream_t st) {
  if (tl == 1) return launch_tt_nw<1>(nw, win, tile, v, a, lds, st);
  if (tl == 4) return launch_tt_nw<4>(nw, win, tile, v, a, lds, st);
  return launch_tt_nw<2>(nw, win, tile, v, a, lds, st);
}

// The two-tile tick kernel (craft_tick2.h) for craft_step_teach, 3x3 windows: 2 or 4 teacher
// lanes per env, 4 tick waves (8 would leave the BFS too few registers at 2 workgroups per CU).
constexpr int kTick2Tiles = 2, kTick2TickWaves = 4;

size_t tick2_lds_bytes(int tl, int nw, int GS, int F) {
  // as launch_t2_nw rounds nw up to the instantiated NW
  const int NW = nw <= 2 ? 2 : nw <= 4 ? 4 : nw <= 5 ? 5 : 8;
  const int nbuf = tick2_share(tl, NW) ? kTick2TickWaves + kTick2Tiles * tl : kTick2TickWaves;
  return (size_t)tick2_lds(kTick2Tiles, kTick2TickWaves, GS, F, nbuf).bytes;
}

template <int TL, int NW>
static hipError_t launch_t2(const SimView& v, const TileArgs& a, size_t lds, hipStream_t st) {
  constexpr int TW = kTick2TickWaves;
  const int64_t per = (int64_t)kTick2Tiles * kTick2Tile;
  const int64_t blocks = (a.n + per - 1) / per;
  if (blocks == 0) return hipSuccess;
  // the teacher waves' own rows (tick2_share) pass 64 KiB
  const hipError_t e = ensure_lds<&tick2_kernel<3, kTick2Tiles, TW, TL, NW>>(lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((tick2_kernel<3, kTick2Tiles, TW, TL, NW>), dim3((unsigned)blocks),
                     dim3(64 * TW + kTick2Tiles * kTick2Tile * TL), lds, st, v, a);
  return hipGetLastError();
}

template <int TL>
static hipError_t launch_t2_nw(int nw, const SimView& v, const TileArgs& a, size_t lds, hipStream_t st) {
  if (nw <= 2) return launch_t2<TL, 2>(v, a, lds, st);
  if (nw <= 4) return launch_t2<TL, 4>(v, a, lds, st);
  if (nw <= 5) return launch_t2<TL, 5>(v, a, lds, st);
  return launch_t2<TL, 8>(v, a, lds, st);
}

hipError_t launch_tick2(int tl, int nw, const SimView& v, const TileArgs& a, size_t lds, hipStream_t st) {
  if (tl == 4) return launch_t2_nw<4>(nw, v, a, lds, st);
  return launch_t2_nw<2>(nw, v, a, lds, st);
}

}  // namespace craft
