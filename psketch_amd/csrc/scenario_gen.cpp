// scenario_gen.cpp — host-side scenario generator of the batched CraftWorld.
//
// Restates make_data.py:27-144 (all_free_cells_reachable, random_free,
// sample_scenario) over numpy's legacy RandomState stream, so a pool generated
// here with seed s is bit-identical to the worlds the reference's generator
// draws from np.random.RandomState(s).  The stream pieces reproduced are:
//   RandomState(int)   -> MT19937 init_genrand(seed)      (numpy _legacy_seeding)
//   randint(high)      -> masked rejection on 32-bit draws (random_bounded_uint64,
//                         use_masked=True, rng = high - 1 <= 0xFFFFFFFF)
// Scenario generation is input preparation (never timed); it runs on the host
// because it is a rejection-sampling loop over a few hundred cells.
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/craft.h"

namespace {

struct Mt19937 {
  uint32_t key[624];
  int pos;
  void seed(uint32_t s) {
    for (int i = 0; i < 624; ++i) {
      key[i] = s;
      s = 1812433253u * (s ^ (s >> 30)) + (uint32_t)(i + 1);
    }
    pos = 624;
  }
  void twist() {
    for (int i = 0; i < 624; ++i) {
      uint32_t y = (key[i] & 0x80000000u) | (key[(i + 1) % 624] & 0x7fffffffu);
      uint32_t v = key[(i + 397) % 624] ^ (y >> 1);
      if (y & 1u) v ^= 0x9908b0dfu;
      key[i] = v;
    }
    pos = 0;
  }
  uint32_t next32() {
    if (pos >= 624) twist();
    uint32_t y = key[pos++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }
  // RandomState.randint(high) for 1 <= high <= 2**32.
  int32_t randint(int32_t high) {
    uint32_t rng = (uint32_t)(high - 1);
    if (rng == 0) return 0;
    uint32_t mask = rng;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v;
    while ((v = next32() & mask) > rng) {}
    return (int32_t)v;
  }
};

const int kDX[4] = {0, 0, -1, 1};   // DOWN, UP, LEFT, RIGHT coord_change (craft.py:77-91)
const int kDY[4] = {-1, 1, 0, 0};

// all_free_cells_reachable, make_data.py:27-72.  nav: W*H occupancy (x-major).
// Returns 1/0, or -1 where the reference would raise (no free cell to start from).
int all_free_cells_reachable(const std::vector<uint8_t>& nav, int W, int H, int sx, int sy) {
  if (sx < 0) {
    for (int i = 0; i < W && sx < 0; ++i)
      for (int j = 0; j < H; ++j)
        if (nav[i * H + j] == 0) { sx = i; sy = j; break; }
    if (sx < 0) return -1;
  }
  std::vector<uint8_t> seen(W * H, 0);
  std::vector<int> queue;
  queue.reserve(W * H);
  queue.push_back(sx * H + sy);
  seen[sx * H + sy] = 1;
  for (size_t head = 0; head < queue.size(); ++head) {
    int p = queue[head], px = p / H, py = p % H;
    for (int a = 0; a < 4; ++a) {
      int nx = px + kDX[a], ny = py + kDY[a];
      if (nav[nx * H + ny]) { nx = px; ny = py; }    // blocked: stay (make_data.py:59-60)
      int q = nx * H + ny;
      if (!seen[q]) { seen[q] = 1; queue.push_back(q); }
    }
  }
  for (int c = 0; c < W * H; ++c)
    if (nav[c] == 0 && !seen[c]) return 0;
  return 1;
}

// random_free(keep_connected=True), make_data.py:74-103.
int random_free(const std::vector<uint8_t>& grid, int W, int H, Mt19937& rs, int* ox, int* oy) {
  std::vector<uint8_t> nav(W * H);
  for (int c = 0; c < W * H; ++c) nav[c] = grid[c] != 0;
  for (;;) {
    int x = rs.randint(W);
    int y = rs.randint(H);
    if (nav[x * H + y]) continue;
    bool good = true;
    nav[x * H + y] = 1;
    int r = all_free_cells_reachable(nav, W, H, -1, -1);
    if (r < 0) return CRAFT_EINVARIANT;
    if (!r) {
      good = false;
    } else {
      for (int i = 0; i < W && good; ++i)
        for (int j = 0; j < H; ++j)
          if (nav[i * H + j] == 1 && i > 0 && i < W - 1 && j > 0 && j < H - 1) {
            int rr = all_free_cells_reachable(nav, W, H, i, j);
            if (rr < 0) return CRAFT_EINVARIANT;
            if (!rr) { good = false; break; }
          }
    }
    if (good) { *ox = x; *oy = y; return CRAFT_OK; }
    nav[x * H + y] = 0;
  }
}

}  // namespace

extern "C" int craft_sample_scenarios(int32_t width, int32_t height, int32_t boundary_kind,
                                      const int32_t* primitives, int32_t n_primitive_kinds,
                                      int32_t n_per_primitive, const int32_t* workshop_kind,
                                      int32_t n_workshops, uint32_t seed, int32_t count,
                                      int32_t dedup, uint8_t* grids_out, int32_t* init_pos_out,
                                      uint32_t* mt_state_out) {
  const int W = width, H = height;
  if (W < 3 || H < 3 || W > CRAFT_MAX_DIM || H > CRAFT_MAX_DIM || count < 0 || !grids_out ||
      (n_primitive_kinds > 0 && !primitives) || (n_workshops > 0 && !workshop_kind) ||
      boundary_kind <= 0 || boundary_kind > 255)
    return CRAFT_EINVAL;
  Mt19937 rs;
  rs.seed(seed);
  const int C = W * H;
  std::vector<uint8_t> grid(C);
  for (int s = 0; s < count; ++s) {
    int ix = 0, iy = 0;
    for (;;) {
      // sample_scenario, make_data.py:105-144
      std::fill(grid.begin(), grid.end(), 0);
      for (int y = 0; y < H; ++y) { grid[0 * H + y] = (uint8_t)boundary_kind; grid[(W - 1) * H + y] = (uint8_t)boundary_kind; }
      for (int x = 0; x < W; ++x) { grid[x * H + 0] = (uint8_t)boundary_kind; grid[x * H + H - 1] = (uint8_t)boundary_kind; }
      for (int p = 0; p < n_primitive_kinds; ++p)
        for (int i = 0; i < n_per_primitive; ++i) {
          int x, y;
          int rc = random_free(grid, W, H, rs, &x, &y);
          if (rc) return rc;
          grid[x * H + y] = (uint8_t)primitives[p];
        }
      for (int w = 0; w < n_workshops; ++w) {
        int x, y;
        int rc = random_free(grid, W, H, rs, &x, &y);
        if (rc) return rc;
        grid[x * H + y] = (uint8_t)workshop_kind[w];
      }
      int rc = random_free(grid, W, H, rs, &ix, &iy);
      if (rc) return rc;
      if (!dedup) break;
      bool duplicate = false;                                  // make_data.py:170-176
      for (int q = 0; q < s && !duplicate; ++q)
        if (std::memcmp(grids_out + (size_t)q * C, grid.data(), C) == 0) duplicate = true;
      if (!duplicate) break;
    }
    std::memcpy(grids_out + (size_t)s * C, grid.data(), C);
    if (init_pos_out) { init_pos_out[2 * s] = ix; init_pos_out[2 * s + 1] = iy; }
  }
  if (mt_state_out) {
    std::memcpy(mt_state_out, rs.key, sizeof(rs.key));
    mt_state_out[624] = (uint32_t)rs.pos;
  }
  return CRAFT_OK;
}
