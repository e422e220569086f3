// craft_step_teach.hip — craft_step_teach on the one-launch-per-tick kernel (craft_step.h) for
// 3x3 windows: 2 teacher lanes per env (a pair; craft_teach.h) beside the 4 tick waves.  Wider
// windows keep the one-tile kernel (craft_tick_teach.hip): their scatter needs the registers
// the BFS lanes would take.
#include "craft_step_launch.h"

namespace craft {

// nw = 32-bit words per cell set: 8x8 -> 2, 10x10 -> 4, 12x12 -> 5, 16x16 -> 8
hipError_t launch_step_teach(int epw, int nw, size_t lds_min, const SimView& v, const TileArgs& a, hipStream_t st) {
  if (nw <= 2) return launch_s_epw<3, 2, 2>(epw, v, a, lds_min, st);
  if (nw <= 4) return launch_s_epw<3, 2, 4>(epw, v, a, lds_min, st);
  if (nw <= 5) return launch_s_epw<3, 2, 5>(epw, v, a, lds_min, st);
  return launch_s_epw<3, 2, 8>(epw, v, a, lds_min, st);
}

}  // namespace craft
