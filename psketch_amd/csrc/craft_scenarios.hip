// craft_scenarios.hip — make_data.sample_scenario on the GPU (craft_pool_generate).
//
// One lane per scenario writes its grid straight into the simulator's pool.
// The algorithm is make_data.py:105-144: a boundary ring, N_PRIMITIVES of each
// primitive, then the workshops, then the initial position, each cell drawn by
// random_free (make_data.py:74-103): rejection-sample (x, y) uniformly, skip
// occupied cells, tentatively occupy the cell and keep it only if
//   (1) the free cells stay one 4-connected component
//       (all_free_cells_reachable from the first free cell, make_data.py:27-72), and
//   (2) every occupied interior cell still has a free 4-neighbour
//       (all_free_cells_reachable started from that cell, make_data.py:88-97:
//        given (1), it reaches every free cell iff it can step into one).
// Both checks run on the occupancy as NW-word bitsets in registers: (1) is a
// flood fill by shifts (+-1, +-H) masked by the free set, (2) one shifted OR.
//
// The random source is the only difference from make_data.py: numpy's single
// sequential MT19937 stream cannot be split across lanes, so each scenario gets
// its own splitmix64 stream keyed by its global id (seed ^ id * 0xD1B5...),
// with randint by Lemire's unbiased multiply-shift.  The results are identical
// for any sharding of the ids.  oracle_generate_scenarios restates the same
// algorithm with either source; with MT19937 it reproduces the reference's own
// scenario stream bit for bit (tests/test_oracle_golden.py), with splitmix64 it
// is the parity check of this kernel.
#include "craft_bits.h"

namespace craft {

struct SplitMix {
  uint64_t s;
  __device__ __forceinline__ uint32_t next32() {
    s += 0x9E3779B97F4A7C15ull;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return (uint32_t)((z ^ (z >> 31)) >> 32);
  }
  __device__ __forceinline__ int randint(uint32_t n) {      // uniform in [0, n), unbiased
    uint64_t m = (uint64_t)next32() * n;
    uint32_t l = (uint32_t)m;
    if (l < n) {
      const uint32_t t = (0u - n) % n;
      while (l < t) {
        m = (uint64_t)next32() * n;
        l = (uint32_t)m;
      }
    }
    return (int)(m >> 32);
  }
};

template <int NW>
__global__ __launch_bounds__(256) void scenario_kernel(SimView v, ScenarioArgs a) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= a.count) return;
  const int W = v.W, H = v.H, C = v.C;
  SplitMix rng{a.seed ^ ((uint64_t)(a.id0 + s) * 0xD1B54A32D192ED03ull)};
  uint8_t* row = const_cast<uint8_t*>(v.pool) + (size_t)(a.first + s) * v.CS;

  Bits<NW> valid = bzero<NW>(), border = bzero<NW>();
  for (int c = 0; c < C; ++c) {
    const int x = c / H, y = c - x * H;
    valid = bor(valid, bbit<NW>(c));
    if (x == 0 || y == 0 || x == W - 1 || y == H - 1) border = bor(border, bbit<NW>(c));
  }
  const Bits<NW> interior = bandn(valid, border);
  // the boundary ring (make_data.py:108-112), everything else empty
  for (int q = 0; q < (v.CS >> 2); ++q) {
    uint32_t w = 0;
    for (int b = 0; b < 4; ++b) {
      const int c = 4 * q + b;
      if (c < C && btest(border, c)) w |= (uint32_t)a.boundary << (8 * b);
    }
    reinterpret_cast<uint32_t*>(row)[q] = w;
  }

  // random_free's acceptance test for the occupancy `occ` (the candidate included)
  auto acceptable = [&](const Bits<NW>& occ) -> bool {
    const Bits<NW> fr = bandn(valid, occ);
    const int p0 = blowest(fr);
    if (p0 == INT_MAX) return true;
    Bits<NW> reach = bbit<NW>(p0);
    for (int it = 0; it < CRAFT_MAX_CELLS; ++it) {            // flood fill, <= C rounds
      const Bits<NW> grow = bor(bor(bshift(reach, 1), bshift(reach, -1)),
                                bor(bshift(reach, H), bshift(reach, -H)));
      const Bits<NW> nxt = bor(reach, band(grow, fr));
      bool same = true;
#pragma unroll
      for (int i = 0; i < NW; ++i) same = same && nxt.w[i] == reach.w[i];
      reach = nxt;
      if (same) break;
    }
    if (bany(bandn(fr, reach))) return false;                 // (1) free cells connected
    const Bits<NW> touch = bor(bor(bshift(fr, 1), bshift(fr, -1)), bor(bshift(fr, H), bshift(fr, -H)));
    return !bany(bandn(band(occ, interior), touch));          // (2) objects stay accessible
  };
  Bits<NW> occ = border;
  bool failed = false;
  auto random_free = [&](int& cell) -> bool {
    for (int draws = 0; draws < (1 << 20); ++draws) {
      const int x = rng.randint((uint32_t)W), y = rng.randint((uint32_t)H);
      const int c = x * H + y;
      if (btest(occ, c)) continue;
      if (acceptable(bor(occ, bbit<NW>(c)))) {
        cell = c;
        return true;
      }
    }
    return false;
  };
  int c = 0;
  for (int p = 0; p < a.n_prim && !failed; ++p)               // ingredients (make_data.py:128-134)
    for (int i = 0; i < a.n_per && !failed; ++i) {
      if (!random_free(c)) { failed = true; break; }
      occ = bor(occ, bbit<NW>(c));
      row[c] = (uint8_t)a.prim[p];
    }
  for (int i = 0; i < a.n_ws && !failed; ++i) {               // workshops (make_data.py:137-139)
    if (!random_free(c)) { failed = true; break; }
    occ = bor(occ, bbit<NW>(c));
    row[c] = (uint8_t)a.ws[i];
  }
  if (!failed && !random_free(c)) failed = true;              // init pos (make_data.py:142)
  if (failed) {
    latch_error(v.err, CRAFT_EINVARIANT, a.id0 + s);
    c = 0;
  }
  // every accepted placement kept the free cells one component (acceptance test (1))
  const_cast<uint8_t*>(v.pool_conn)[a.first + s] = failed ? 0 : 1;
  if (a.init_out) {
    a.init_out[2 * s] = c / H;
    a.init_out[2 * s + 1] = c % H;
  }
}

hipError_t launch_scenarios(const SimView& v, const ScenarioArgs& a, hipStream_t st) {
  if (a.count == 0) return hipSuccess;
  const unsigned blocks = (unsigned)((a.count + 255) / 256);
  const int nw = (v.C + 31) / 32;
  if (nw <= 2) hipLaunchKernelGGL(scenario_kernel<2>, dim3(blocks), dim3(256), 0, st, v, a);
  else if (nw <= 4) hipLaunchKernelGGL(scenario_kernel<4>, dim3(blocks), dim3(256), 0, st, v, a);
  else if (nw <= 5) hipLaunchKernelGGL(scenario_kernel<5>, dim3(blocks), dim3(256), 0, st, v, a);
  else hipLaunchKernelGGL(scenario_kernel<8>, dim3(blocks), dim3(256), 0, st, v, a);
  return hipGetLastError();
}

}  // namespace craft
