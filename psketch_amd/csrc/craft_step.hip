// craft_step.hip — launchers of the one-launch-per-tick kernel (craft_step.h) for craft_step /
// craft_step_ex (TL = 0); craft_step_teach.hip instantiates it with teacher lanes.
#include "craft_step_launch.h"

namespace craft {

size_t step_lds_bytes(int win, int epw, int tl, int GS, int F) {
  const int sub = win == 3 ? 16 : (win == 5 ? 8 : 4);
  return (size_t)step_lds(epw, sub, tl, GS, F).bytes;
}

// the plain tick (craft_step, craft_step_ex): epw envs per tick wave (16, 32 or 64)
hipError_t launch_step(int win, int epw, size_t lds_min, const SimView& v, const TileArgs& a, hipStream_t st) {
  switch (win) {
    case 3: return launch_s_epw<3, 0, 1>(epw, v, a, lds_min, st);
    case 5: return launch_s_epw<5, 0, 1>(epw, v, a, lds_min, st);
    default: return launch_s_epw<7, 0, 1>(epw, v, a, lds_min, st);
  }
}

}  // namespace craft
