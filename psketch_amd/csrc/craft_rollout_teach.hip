// craft_rollout_teach.hip — launches of the teacher-labelled K-tick rollout kernel
// (craft_rollout_teach.h), one instantiation per window and BFS word count.
#include <algorithm>

#include "craft_rollout_teach.h"

namespace craft {

template <int WIN, int NW, bool LA>
static hipError_t launch_rt_one(const SimView& v, const RolloutArgs& a, hipStream_t st) {
  constexpr int TILE = rt_tile(WIN);
  const int64_t tiles = (v.n_envs + TILE - 1) / TILE;
  if (tiles == 0 || a.n_ticks == 0) return hipSuccess;
#ifdef CRAFT_STAMPS
  const size_t lds = (size_t)rt_lds(TILE, v.GS, v.F, NW).bytes + 512;     // + the stamp sums
#else
  const size_t lds = (size_t)rt_lds(TILE, v.GS, v.F, NW).bytes;
#endif
  auto kern = rollout_teach_kernel<WIN, TILE, NW, LA>;
  {
    const hipError_t e = ensure_lds<&rollout_teach_kernel<WIN, TILE, NW, LA>>(lds);
    if (e != hipSuccess) return e;
  }
  // persistent workgroups: what the chip holds at once, spread so that every workgroup runs the
  // same number of tiles
  const int resident = resident_workgroups<&rollout_teach_kernel<WIN, TILE, NW, LA>>(kRtThreads, lds);
  const int64_t rounds = (tiles + resident - 1) / resident;
  const int64_t rows = (v.n_envs + kMinTileEnvs - 1) / kMinTileEnvs;   // stats_part rows
  const int64_t grid = std::min<int64_t>((tiles + rounds - 1) / rounds, rows);
  if (a.grid_out) *a.grid_out = grid;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kRtThreads), lds, st, v, a);
  return hipGetLastError();
}

template <int WIN, bool LA>
static hipError_t launch_rt_nw(int nw, const SimView& v, const RolloutArgs& a, hipStream_t st) {
  // nw = 32-bit words per BFS cell set (the band of columns 1 .. W-2): 8x8 -> 2, 10x10 -> 3 (run
  // as 4), 12x12 -> 4, up to 15x15 -> 7 (run as 8)
  if (nw <= 2) return launch_rt_one<WIN, 2, LA>(v, a, st);
  if (nw <= 4) return launch_rt_one<WIN, 4, LA>(v, a, st);
  return launch_rt_one<WIN, 8, LA>(v, a, st);
}

template <int WIN>
static hipError_t launch_rt_win(int nw, const SimView& v, const RolloutArgs& a, hipStream_t st) {
  // labels feeding actions, the transition wave looking them up (lsync 2): the LA kernel
  if (a.lsync == 2) return launch_rt_nw<WIN, true>(nw, v, a, st);
  return launch_rt_nw<WIN, false>(nw, v, a, st);
}

hipError_t launch_rollout_teach(int win, int nw, const SimView& v, const RolloutArgs& a, hipStream_t st) {
  switch (win) {
    case 3: return launch_rt_win<3>(nw, v, a, st);
    case 5: return launch_rt_win<5>(nw, v, a, st);
    default: return launch_rt_win<7>(nw, v, a, st);
  }
}

}  // namespace craft
