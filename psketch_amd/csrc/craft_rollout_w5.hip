// craft_rollout_w5.hip — rollout_kernel instantiations for 5x5 windows
// (one translation unit per window so the build compiles them in parallel).
#include "craft_rollout.h"

namespace craft {

hipError_t launch_rollout_w5(int tile, int threads, const SimView& v, const RolloutArgs& a, size_t lds,
                             hipStream_t st) {
  return launch_rollout_win<5>(tile, threads, v, a, lds, st);
}

}  // namespace craft
