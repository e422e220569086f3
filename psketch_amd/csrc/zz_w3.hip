// craft_rollout_w3.hip — rollout_kernel instantiations for 3x3 windows
// (one translation unit per window so the build compiles them in parallel).
#define CRAFT_SPLIT_WPE 1
#include "zz_rollout.h"

namespace craft {

hipError_t launch_rollout_w3(int tile, int threads, const SimView& v, const RolloutArgs& a, size_t lds,
                             hipStream_t st) {
  return launch_rollout_win<3>(tile, threads, v, a, lds, st);
}

hipError_t launch_rollout(int win, int tile, int threads, const SimView& v, const RolloutArgs& a,
                          size_t lds, hipStream_t st) {
  switch (win) {
    case 3: return launch_rollout_w3(tile, threads, v, a, lds, st);
    case 5: return launch_rollout_w5(tile, threads, v, a, lds, st);
    default: return launch_rollout_w7(tile, threads, v, a, lds, st);
  }
}

}  // namespace craft
