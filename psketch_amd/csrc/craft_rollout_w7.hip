// craft_rollout_w7.hip — rollout_kernel instantiations for 7x7 windows
// (one translation unit per window so the build compiles them in parallel).
#include "craft_rollout.h"

namespace craft {

hipError_t launch_rollout_w7(int tile, int threads, const SimView& v, const RolloutArgs& a, size_t lds,
                             hipStream_t st) {
  return launch_rollout_win<7>(tile, threads, v, a, lds, st);
}

}  // namespace craft
