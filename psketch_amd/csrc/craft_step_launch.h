// craft_step_launch.h — launch templates of the one-launch-per-tick kernel (craft_step.h),
// shared by craft_step.hip (the plain tick) and craft_step_teach.hip (the tick + teacher).
#pragma once
#include <cstdlib>

#include "craft_step.h"

namespace craft {

// envs per D + E sub-chunk: 64 / SUB lanes per env cover the WIN + 1 scatter items, SUB * F
// bytes stay within ~8.6 KB of LDS per wave, and a sub-chunk's output starts 16-byte aligned in
// every observation format (SUB * F is a multiple of 16)
template <int WIN> struct StepSub { static constexpr int value = WIN == 3 ? 16 : (WIN == 5 ? 8 : 4); };

// lds_min pads the workgroup's LDS request (a residency cap: 160 KiB / lds_min workgroups per CU)
template <int WIN, int EPW, int TL, int NW, int NS>
hipError_t launch_s_ns(const SimView& v, const TileArgs& a, size_t lds_min, hipStream_t st) {
  constexpr int SUB = StepSub<WIN>::value;
  const int64_t per = (int64_t)kStepTick * EPW;
  const int64_t blocks = (a.n + per - 1) / per;
  if (blocks == 0) return hipSuccess;
  const size_t lds = std::max((size_t)step_lds(EPW, SUB, TL, v.GS, v.F).bytes, lds_min);
  if (lds > 163840) return hipErrorInvalidValue;
  auto kern = step_kernel<WIN, EPW, SUB, TL, NW, NS>;
  if (lds > 65536) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(64 * (kStepTick + NS) + kStepTick * EPW * TL),
                     lds, st, v, a);
  return hipGetLastError();
}

// CRAFT_STEP_STREAM=8 (diagnostic): one stream wave per row buffer instead of one per pair
template <int WIN, int EPW, int TL, int NW>
hipError_t launch_s(const SimView& v, const TileArgs& a, size_t lds_min, hipStream_t st) {
  static const bool ns8 = getenv("CRAFT_STEP_STREAM") && atoi(getenv("CRAFT_STEP_STREAM")) == 8;
  if (TL == 0 && ns8) return launch_s_ns<WIN, EPW, TL, NW, 2 * kStepTick>(v, a, lds_min, st);
  return launch_s_ns<WIN, EPW, TL, NW, kStepStream>(v, a, lds_min, st);
}

template <int WIN, int TL, int NW>
hipError_t launch_s_epw(int epw, const SimView& v, const TileArgs& a, size_t lds_min, hipStream_t st) {
  switch (epw) {
    case 16: return launch_s<WIN, 16, TL, NW>(v, a, lds_min, st);
    case 32: return launch_s<WIN, 32, TL, NW>(v, a, lds_min, st);
    default: return launch_s<WIN, 64, TL, NW>(v, a, lds_min, st);
  }
}

}  // namespace craft
