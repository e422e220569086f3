// craft_tile.hip — launchers of the tile kernel (craft_tile.h) for the tick,
// transition, observe and reset entry points.
#include "craft_tile.h"

namespace craft {

template <int WIN, int MODE, int TILE>
static hipError_t launch_one(const SimView& v, const TileArgs& a, size_t lds, hipStream_t st) {
  const int64_t tiles = (a.n + TILE - 1) / TILE;
  if (tiles == 0) return hipSuccess;
  // u8 rows of 5x5 / 7x7 windows on large tiles
  const hipError_t e = ensure_lds<&tile_kernel<WIN, MODE, TILE>>(lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((tile_kernel<WIN, MODE, TILE>), dim3((unsigned)tiles), dim3(kThreads), lds, st, v, a);
  return hipGetLastError();
}

template <int MODE, int TILE>
static hipError_t launch_win(int win, const SimView& v, const TileArgs& a, size_t lds, hipStream_t st) {
  switch (win) {
    case 3: return launch_one<3, MODE, TILE>(v, a, lds, st);
    case 5: return launch_one<5, MODE, TILE>(v, a, lds, st);
    default: return launch_one<7, MODE, TILE>(v, a, lds, st);
  }
}

template <int MODE>
static hipError_t launch_tiled(int tile, int win, const SimView& v, const TileArgs& a, size_t lds,
                               hipStream_t st) {
  switch (tile) {
    case 16: return launch_win<MODE, 16>(win, v, a, lds, st);
    case 32: return launch_win<MODE, 32>(win, v, a, lds, st);
    default: return launch_win<MODE, 64>(win, v, a, lds, st);
  }
}

hipError_t launch_tile(int mode, int win, int tile, const SimView& v, const TileArgs& a, size_t lds,
                       hipStream_t st) {
  switch (mode) {
    case MODE_TICK: return launch_tiled<MODE_TICK>(tile, win, v, a, lds, st);
    case MODE_OBSERVE: return launch_tiled<MODE_OBSERVE>(tile, win, v, a, lds, st);
    case MODE_TRANSITION: return launch_tiled<MODE_TRANSITION>(tile, win, v, a, lds, st);
    default: return launch_tiled<MODE_RESET>(tile, win, v, a, lds, st);
  }
}

}  // namespace craft
