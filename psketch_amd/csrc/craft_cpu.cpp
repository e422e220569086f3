// craft_cpu.cpp — the CPU variant of the C ABI (include/craft.h), SURVEY.md §8(b): "a CPU variant
// with the same signatures (host pointers)".  libpsketch_craft_cpu.so exports every entry point
// of the HIP library (libpsketch_craft.so) under the same names and signatures, over host
// memory: every pointer documented "device" is a host pointer here, `stream` is ignored and
// every call is synchronous.  It is a separate library a GPU-less caller loads on purpose
// (psketch_amd.CraftSim(device="cpu")); the HIP library never falls back to it.
//
// The state layout is the HIP library's (include/craft.h, craft_device.h): per slot a packed u64
// state word, the restart word, 32 u8 inventory counts and a 256-bit cleared-cell mask over the
// scenario's pool row; configuration, pool and task-table checks come from craft_host.h, so
// both libraries accept and refuse the same inputs.  Work is split over host threads by
// contiguous slot ranges (craft_sim_tune_host; default: the hardware's threads).  Results equal the HIP
// library's bit for bit (tests/test_cpu_variant.py against the oracle here, tests/test_gpu_cpu_variant.py
// against the HIP library on the GPU box).
//
// Each function cites the reference code it restates: worlds/craft.py:285-437 (satisfies,
// features, step), trainers/imitation.py:43-91 (the rollout tick and its summary),
// teachers/base.py:10-87 + teachers/demonstration.py:9-30 (the DemonstrationTeacher),
// make_data.py:27-144 (scenario generation, with the HIP library's per-scenario splitmix64 stream).
#include <algorithm>
#include <atomic>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "craft_host.h"

namespace {

// ---- cell sets: 256 cells (x-major index), 4 words ------------------------------------------
struct Bits {
  uint64_t w[4];
};
inline Bits bzero() { return Bits{{0, 0, 0, 0}}; }
inline Bits bbit(int p) {
  Bits r = bzero();
  if (p >= 0 && p < 256) r.w[p >> 6] = 1ull << (p & 63);
  return r;
}
inline Bits band(const Bits& a, const Bits& b) { Bits r; for (int i = 0; i < 4; ++i) r.w[i] = a.w[i] & b.w[i]; return r; }
inline Bits bor(const Bits& a, const Bits& b) { Bits r; for (int i = 0; i < 4; ++i) r.w[i] = a.w[i] | b.w[i]; return r; }
inline Bits bandn(const Bits& a, const Bits& b) { Bits r; for (int i = 0; i < 4; ++i) r.w[i] = a.w[i] & ~b.w[i]; return r; }
inline bool bany(const Bits& a) { return (a.w[0] | a.w[1] | a.w[2] | a.w[3]) != 0; }
inline bool btest(const Bits& a, int p) { return p >= 0 && p < 256 && ((a.w[p >> 6] >> (p & 63)) & 1u); }
inline bool beq(const Bits& a, const Bits& b) {
  return a.w[0] == b.w[0] && a.w[1] == b.w[1] && a.w[2] == b.w[2] && a.w[3] == b.w[3];
}
inline int blowest(const Bits& a) {
  for (int i = 0; i < 4; ++i)
    if (a.w[i]) return 64 * i + __builtin_ctzll(a.w[i]);
  return INT_MAX;
}
inline int bhighest(const Bits& a) {
  for (int i = 3; i >= 0; --i)
    if (a.w[i]) return 64 * i + 63 - __builtin_clzll(a.w[i]);
  return -1;
}
// r[p] = a[p - k]: cells move up by k (down for k < 0), |k| < 64
inline Bits bshift(const Bits& a, int k) {
  Bits r = bzero();
  if (k >= 0) {
    for (int i = 3; i >= 0; --i) r.w[i] = (a.w[i] << k) | (k && i ? a.w[i - 1] >> (64 - k) : 0);
  } else {
    const int s = -k;
    for (int i = 0; i < 4; ++i) r.w[i] = (a.w[i] >> s) | (i < 3 ? a.w[i + 1] << (64 - s) : 0);
  }
  return r;
}
inline Bits brange(int lo, int hi) {   // cells [lo, hi)
  Bits r = bzero();
  for (int p = std::max(lo, 0); p < std::min(hi, 256); ++p) r.w[p >> 6] |= 1ull << (p & 63);
  return r;
}

uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

struct Agent {
  int x, y, dir, frozen, timer, scen, task;
};
Agent unpack_state(uint64_t s) {
  Agent a;
  const uint32_t lo = (uint32_t)s, hi = (uint32_t)(s >> 32);
  a.x = lo & 0xff; a.y = (lo >> 8) & 0xff; a.dir = (lo >> 16) & 3; a.frozen = (lo >> 18) & 1; a.timer = lo >> 24;
  a.scen = hi & 0xffffff; a.task = hi >> 24;
  return a;
}
uint64_t pack_state(const Agent& a) {
  const uint32_t lo = (uint32_t)a.x | ((uint32_t)a.y << 8) | ((uint32_t)a.dir << 16) | ((uint32_t)a.frozen << 18) |
                      ((uint32_t)a.timer << 24);
  const uint32_t hi = ((uint32_t)a.scen & 0xffffff) | ((uint32_t)a.task << 24);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}
inline int dir_dx(int d) { return d == CRAFT_LEFT ? -1 : (d == CRAFT_RIGHT ? 1 : 0); }
inline int dir_dy(int d) { return d == CRAFT_DOWN ? -1 : (d == CRAFT_UP ? 1 : 0); }

int default_tile(int win) { return win == 3 ? 64 : 32; }     // as the HIP library's (u8 rows)

}  // namespace

struct craft_sim {
  craft_config_t cfg{};
  int64_t n_envs = 0, env_base = 0;
  int32_t pool_capacity = 0, pool_count = 0;
  int W = 0, H = 0, C = 0, K = 0, F = 0, win = 0;
  std::vector<uint8_t> pool, pool_conn;   // [P][C], [P]
  std::vector<uint64_t> state;
  std::vector<uint32_t> init;             // x0 | y0 << 8 | dir0 << 16
  std::vector<uint8_t> inv;               // [n][32]
  std::vector<uint32_t> mask;             // [n][8]: cells cleared this episode
  uint16_t task_tab[CRAFT_MAX_TASKS] = {};
  int32_t task_sub[CRAFT_MAX_TASKS * CRAFT_MAX_SUBTASKS] = {};
  std::atomic<int64_t> stats[3];
  std::atomic<int32_t> err_code{0};
  std::atomic<int64_t> err_slot{-1};
  int obs_fmt = CRAFT_OBS_F32;
  int tile = 64, obs_store = 2, resident_cap = 0, rollout_chunk = 0, rollout_threads = 0, teach_kernel = 0;
  int teach_lanes = 0, teach_table = 0;
  int threads = 1;
  std::string last_error;
};

namespace {

int fail(craft_sim* s, int code, const std::string& msg) {
  if (s) s->last_error = msg;
  return code;
}

void latch(craft_sim* s, int code, int64_t slot) {
  int32_t z = 0;
  if (s->err_code.compare_exchange_strong(z, code)) s->err_slot.store(slot);
}

// the machine's hardware threads (craft_sim_tune_host's default)
int hw_threads() {
  const int hw = (int)std::thread::hardware_concurrency();
  return hw > 0 ? hw : 1;
}

// fn(lo, hi) over [0, n) in contiguous ranges on the handle's threads
template <class Fn>
void parallel_for(const craft_sim* s, int64_t n, Fn fn) {
  const int64_t per = 2048;
  const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(s->threads, (n + per - 1) / per));
  if (nt <= 1) {
    fn((int64_t)0, n);
    return;
  }
  std::vector<std::thread> pool;
  for (int t = 0; t < nt; ++t) {
    const int64_t lo = n * t / nt, hi = n * (t + 1) / nt;
    pool.emplace_back([=] { fn(lo, hi); });
  }
  for (auto& th : pool) th.join();
}

int esize(int fmt) { return fmt == CRAFT_OBS_F32 ? 4 : (fmt == CRAFT_OBS_BF16 ? 2 : 1); }

// The slot's current grid: its scenario's pool row minus the cells cleared this episode.
void env_grid(const craft_sim* s, int64_t slot, int scen, uint8_t* g) {
  std::memcpy(g, s->pool.data() + (size_t)scen * s->C, s->C);
  const uint32_t* m = s->mask.data() + 8 * slot;
  for (int w = 0; w < 8; ++w)
    for (uint32_t mm = m[w]; mm; mm &= mm - 1) g[32 * w + __builtin_ctz(mm)] = 0;
}

// CraftState.satisfies (craft.py:285-294): 1 / 0, -1 for None.
int satisfies(const craft_sim* s, const uint8_t* g, const uint8_t* iv, const Agent& a, int task) {
  const uint32_t tt = s->task_tab[task];
  const int goal = tt & 0xf, arg = (tt >> 4) & 0xff;
  if (goal == CRAFT_GOAL_GET || goal == CRAFT_GOAL_MAKE) return iv[arg] > 0;
  if (goal == CRAFT_GOAL_GO) return g[(a.x + dir_dx(a.dir)) * s->H + (a.y + dir_dy(a.dir))] == arg;
  return -1;
}

// CraftState.step (craft.py:332-424) on grid g and inventory iv; m: the cleared-cell mask.
void transition(craft_sim* s, uint8_t* g, uint8_t* iv, Agent& a, uint32_t* m, int act, bool& inv_changed,
                bool& mask_changed, int64_t slot) {
  const int H = s->H;
  int dx = 0, dy = 0, ndir = a.dir;
  if (act < CRAFT_USE) {                             // moves always turn (craft.py:341-352)
    dx = dir_dx(act);
    dy = dir_dy(act);
    ndir = act;
  } else if (act == CRAFT_USE) {                     // craft.py:356-412
    const int d = a.dir;
    const bool ok = (d == CRAFT_LEFT && a.x > 0) || (d == CRAFT_DOWN && a.y > 0) ||
                    (d == CRAFT_RIGHT && a.x < s->W - 1) || (d == CRAFT_UP && a.y < H - 1);
    if (ok) {
      const int c = (a.x + dir_dx(d)) * H + (a.y + dir_dy(d));
      const int thing = g[c];
      if (thing != 0) {
        const int cls = s->cfg.kind_class[thing];
        if (cls == CRAFT_KIND_GRABBABLE) {           // craft.py:383-386
          if (iv[thing] == 255) latch(s, CRAFT_ERANGE, slot);   // u8 count would wrap
          else iv[thing] = (uint8_t)(iv[thing] + 1);
          g[c] = 0;
          m[c >> 5] |= 1u << (c & 31);
          inv_changed = mask_changed = true;
        } else if (cls == CRAFT_KIND_WORKSHOP) {     // recipes in dict order, chaining (craft.py:388-401)
          for (int r = 0; r < s->cfg.n_recipes; ++r) {
            const craft_recipe_t& rc = s->cfg.recipe[r];
            if (rc.workshop != thing) continue;
            bool have = true;
            for (int q = 0; q < rc.n_inputs; ++q) have = have && iv[rc.input_kind[q]] >= rc.input_count[q];
            if (!have) continue;
            const int made = iv[rc.output] + rc.yield;      // `_yield` (craft.py:394), 1..255
            if (made > 255) latch(s, CRAFT_ERANGE, slot);   // u8 count would wrap: saturate
            iv[rc.output] = (uint8_t)std::min(made, 255);
            for (int q = 0; q < rc.n_inputs; ++q) iv[rc.input_kind[q]] = (uint8_t)(iv[rc.input_kind[q]] - rc.input_count[q]);
            inv_changed = true;
          }
        } else if (cls == CRAFT_KIND_WATER) {        // craft.py:403-406
          if (iv[s->cfg.bridge_kind] > 0) {
            g[c] = 0;
            m[c >> 5] |= 1u << (c & 31);
            iv[s->cfg.bridge_kind] = (uint8_t)(iv[s->cfg.bridge_kind] - 1);
            inv_changed = mask_changed = true;
          }
        } else if (cls == CRAFT_KIND_STONE) {        // craft.py:408-410 (axe kept)
          if (iv[s->cfg.axe_kind] > 0) {
            g[c] = 0;
            m[c >> 5] |= 1u << (c & 31);
            mask_changed = true;
          }
        }
      }
    }
  }
  if (dx | dy) {                                     // collision, craft.py:418-421
    const int nx = a.x + dx, ny = a.y + dy;
    if (g[nx * H + ny] == 0) { a.x = nx; a.y = ny; }
  }
  a.dir = ndir;
}

int transition_code(int ox, int oy, const Agent& a, bool inv_changed) {
  const int dx = a.x - ox, dy = a.y - oy;
  if (dx == 0 && dy == 0) return inv_changed ? 4 : 5;
  return dy < 0 ? CRAFT_DOWN : dy > 0 ? CRAFT_UP : dx < 0 ? CRAFT_LEFT : CRAFT_RIGHT;
}

// CraftState.features (craft.py:296-330) as u8 values into row[F] (pad_slice's zero padding
// outside the grid, misc/array.py:3-25; block_reduce(max) of the w^2 x w^2 window).
void features(const craft_sim* s, const uint8_t* g, const uint8_t* iv, const Agent& a, uint8_t* row) {
  const int W = s->W, H = s->H, K = s->K, w = s->win, hw = w / 2, W2 = w * w, bh = W2 / 2, L = W2 * K;
  std::memset(row, 0, s->F);
  for (int i = 0; i < w; ++i)
    for (int j = 0; j < w; ++j) {
      const int cx = a.x - hw + i, cy = a.y - hw + j;
      if (cx < 0 || cx >= W || cy < 0 || cy >= H) continue;
      const int k = g[cx * H + cy];
      if (k) row[(i * w + j) * K + k] = 1;
    }
  for (int cx = std::max(a.x - bh, 0); cx <= std::min(a.x + bh, W - 1); ++cx)
    for (int cy = std::max(a.y - bh, 0); cy <= std::min(a.y + bh, H - 1); ++cy) {
      const int k = g[cx * H + cy];
      if (k) row[L + (((cx - a.x + bh) / w) * w + (cy - a.y + bh) / w) * K + k] = 1;
    }
  for (int k = 0; k < K; ++k) row[2 * L + k] = iv[k];
  row[2 * L + K + a.dir] = 1;
}

void put_obs(int fmt, void* obs, int64_t i, int F, const uint8_t* row) {
  if (fmt == CRAFT_OBS_F32) {
    float* o = static_cast<float*>(obs) + i * F;
    for (int f = 0; f < F; ++f) o[f] = (float)row[f];
  } else if (fmt == CRAFT_OBS_BF16) {
    uint16_t* o = static_cast<uint16_t*>(obs) + i * F;
    for (int f = 0; f < F; ++f) {
      const float v = (float)row[f];
      uint32_t u;
      std::memcpy(&u, &v, 4);
      o[f] = (uint16_t)(u >> 16);                  // exact: a byte's value has <= 8 significant bits
    }
  } else {
    std::memcpy(static_cast<uint8_t*>(obs) + i * F, row, F);
  }
}

// ---- the DemonstrationTeacher (teachers/demonstration.py:9-30, teachers/base.py:10-87) ---------
// find_closest_resources over shortest_path, as one forward BFS over (position, direction)
// states held as per-direction cell sets, then a backward BFS for the chosen target's first
// action (the HIP library's algorithm, craft_teach.h, scalar, on the whole grid).  Returns false
// where the reference raises (a reachable target before an unreachable one, base.py:31).
bool closest(const craft_sim* s, const uint8_t* g, int kind, int p0, int d0, int& first_action, int& path_len,
             bool want_action) {
  const int H = s->H, C = s->C;
  const int dl[4] = {-1, 1, -H, H};                 // DOWN, UP, LEFT, RIGHT in x-major cell index
  const Bits valid = brange(0, C);
  Bits occ = bzero(), tgt = bzero();
  for (int c = 0; c < C; ++c) {
    if (g[c]) occ.w[c >> 6] |= 1ull << (c & 63);
    if (kind > 0 && g[c] == kind) tgt.w[c >> 6] |= 1ull << (c & 63);
  }
  const Bits fr = bandn(valid, occ);
  Bits blk[4], fa[4];
  for (int a = 0; a < 4; ++a) {
    blk[a] = band(bshift(occ, -dl[a]), valid);       // blk[a][p] = occ[p + dl[a]]
    fa[a] = band(bshift(tgt, -dl[a]), valid);        // fa[a][p] = tgt[p + dl[a]]
  }
  first_action = -1;
  path_len = -1;
  Bits claimed = bzero();
  int L = -1, chosen = -1;
  const int f0 = p0 + dl[d0];                        // the start state already faces a target: []
  if (btest(tgt, f0)) {
    L = 0;
    chosen = f0;
    claimed = bbit(f0);
  }
  Bits V[4];
  for (int a = 0; a < 4; ++a) V[a] = a == d0 ? bbit(p0) : bzero();
  Bits U = bbit(p0);
  const bool open = bany(bandn(tgt, claimed));
  for (int depth = 1; open && L < 0; ++depth) {
    Bits nU = bzero(), nx[4];
    bool face = false;
    for (int a = 0; a < 4; ++a) {
      nx[a] = bandn(bor(band(band(bshift(U, dl[a]), valid), fr), band(U, blk[a])), V[a]);
      V[a] = bor(V[a], nx[a]);
      nU = bor(nU, nx[a]);
      face = face || bany(band(nx[a], fa[a]));
    }
    if (!bany(nU)) break;                            // every reachable state visited
    if (face) {
      Bits hit = bzero();
      for (int a = 0; a < 4; ++a) hit = bor(hit, band(bshift(nx[a], dl[a]), tgt));
      hit = bandn(hit, claimed);
      if (bany(hit)) {
        claimed = bor(claimed, hit);
        L = depth;
        chosen = blowest(hit);                       // first in np.nonzero (x-major) order
        break;
      }
    }
    U = nU;
  }
  if (L < 0) return true;                            // no target, or none reachable: None
  path_len = L;
  if (bany(bandn(tgt, claimed))) {
    // which other targets are reachable at all: faced from any reachable cell next to them
    Bits R = bor(bor(bor(V[0], V[1]), bor(V[2], V[3])), bbit(p0));
    for (;;) {
      Bits adj = bzero();
      for (int a = 0; a < 4; ++a) adj = bor(adj, band(bshift(R, dl[a]), valid));
      claimed = bor(claimed, band(adj, tgt));
      if (!bany(bandn(tgt, claimed))) break;
      const Bits grow = bandn(band(adj, fr), R);
      if (!bany(grow)) break;
      R = bor(R, grow);
    }
    const Bits unreached = bandn(tgt, claimed);
    if (bany(unreached) && blowest(claimed) < bhighest(unreached)) return false;
  }
  if (L == 0 || !want_action) return true;
  Bits G[4];                                         // reverse BFS from the states facing `chosen`
  for (int a = 0; a < 4; ++a) {
    G[a] = band(bbit(chosen - dl[a]), fr);
    V[a] = G[a];
  }
  for (int k = 1; k < L; ++k) {
    Bits P = bzero();                                // predecessors: moved here, or turned in place
    for (int a = 0; a < 4; ++a) P = bor(P, bor(band(bshift(G[a], -dl[a]), fr), band(G[a], blk[a])));
    for (int a = 0; a < 4; ++a) {
      G[a] = bandn(P, V[a]);
      V[a] = bor(V[a], G[a]);
    }
  }
  for (int a = 3; a >= 0; --a) {                     // the smallest qualifying first action
    const int q0 = p0 + dl[a];
    const int q = btest(fr, q0) ? q0 : p0;
    if (!(q == p0 && a == d0) && btest(V[a], q)) first_action = a;
  }
  return true;
}

// DemonstrationTeacher.__call__ for one env (its grid g, inventory iv, agent a, task): the
// action, or -2 where the reference raises (err = CRAFT_ETEACHER); with want_len, len_out =
// len(find_closest_resources(task.arg)) (-1: no target, -2: the reference raises).
int teach(const craft_sim* s, const uint8_t* g, const uint8_t* iv, const Agent& a, int task, bool want_len,
          int& len_out, int& err_out) {
  const int H = s->H;
  const int facing = g[(a.x + dir_dx(a.dir)) * H + (a.y + dir_dy(a.dir))];
  auto sat = [&](int t) -> int {
    const uint32_t tt = s->task_tab[t];
    const int goal = tt & 0xf, arg = (tt >> 4) & 0xff;
    if (goal == CRAFT_GOAL_GET || goal == CRAFT_GOAL_MAKE) return iv[arg] > 0;
    if (goal == CRAFT_GOAL_GO) return facing == arg;
    return -1;
  };
  const int p0 = a.x * H + a.y;
  int leaf_kind = -1, leaf_fa = -1, leaf_len = -1;
  bool leaf_ok = true;
  int action = CRAFT_STOP, err = 0;
  int node = task;
  if (sat(node) != 1) {                              // find_incomplete_subtask, base.py:10-25
    for (int guard = 0; guard < CRAFT_MAX_TASKS; ++guard) {
      const int nsub = (s->task_tab[node] >> 12) & 0xf;
      if (nsub == 0) break;
      const int32_t* sub = s->task_sub + CRAFT_MAX_SUBTASKS * node;
      int chosen = sub[nsub - 1];
      bool last = true;
      for (int q = 0; q + 1 < nsub; ++q)
        if (sat(sub[q]) != 1) { chosen = sub[q]; last = false; break; }
      if (last && sat(chosen) == 1) { err = CRAFT_ETEACHER; break; }   // base.py:24 assert
      node = chosen;
    }
    if (!err) {
      const uint32_t lt = s->task_tab[node];
      const int goal = lt & 0xf, arg = (lt >> 4) & 0xff;
      if (goal == CRAFT_GOAL_USE) {
        action = CRAFT_USE;
      } else if (goal == CRAFT_GOAL_GO) {
        int fa = -1, len = -1;
        leaf_ok = closest(s, g, arg, p0, a.dir, fa, len, true);
        leaf_kind = arg; leaf_fa = fa; leaf_len = len;
        if (!leaf_ok) err = CRAFT_ETEACHER;
        else if (len < 0) action = CRAFT_STOP;                         // demonstration.py:25-26
        else if (len == 0) err = CRAFT_ETEACHER;                       // [][0]
        else action = fa;
      } else {
        err = CRAFT_ETEACHER;                                          // demonstration.py:18
      }
    }
  }
  if (err) action = -2;
  err_out = err;
  if (want_len) {
    const int arg = (s->task_tab[task] >> 4) & 0xff;
    int fa = leaf_fa, len = leaf_len;
    bool ok = leaf_ok;
    if (arg != leaf_kind) {
      len = -1;
      ok = arg > 0 ? closest(s, g, arg, p0, a.dir, fa, len, false) : true;
    }
    len_out = ok ? len : -2;
  }
  return action;
}

// ---- one do_rollout tick of one slot (trainers/imitation.py:43-73), fused with features ------
struct TickIn {
  const int32_t* actions;     // [n] or null: the hashed draw
  const int32_t* ref;
  const uint8_t* bc;
  uint64_t seed;
  int64_t tick;
  uint32_t flags;
  void* obs;                  // [n][F] or null
  float* reward;
  uint8_t* done;
  int8_t* sat;
  int32_t* rec;
  int8_t* code;
  int32_t* label;             // craft_step_teach
};

struct TickAcc {
  int64_t succ = 0, ended = 0, steps = 0;
  bool any_live = false;
};

void tick_slot(craft_sim* s, int64_t i, const TickIn& in, TickAcc& acc, uint8_t* g, uint8_t* row) {
  const int64_t slot = i;
  Agent a = unpack_state(s->state[slot]);
  bool live = !(a.x < 1 || a.x > s->W - 2 || a.y < 1 || a.y > s->H - 2 || a.scen >= s->pool_count);
  int act = 0;
  if (live) {
    act = in.actions ? in.actions[slot]
                     : (int)((uint32_t)(splitmix64(in.seed ^ ((uint64_t)(s->env_base + slot) << 20) ^
                                                   (uint64_t)in.tick) >> 32) % 6u);
    if (in.bc && in.bc[slot]) act = in.ref[slot];    // behaviour cloning, imitation.py:56-57
  } else {
    latch(s, CRAFT_EINVAL, slot);                    // never initialised by reset / set_state
  }
  uint8_t* iv = s->inv.data() + 32 * slot;
  uint32_t* m = s->mask.data() + 8 * slot;
  int d = 0, succ = -1, counted = 0, code = -1;
  if (live) {
    env_grid(s, slot, a.scen, g);
    bool restart = false;
    if (a.frozen) {
      d = 1;
    } else {
      counted = 1;
      a.timer -= 1;
      d = (act == CRAFT_STOP) || a.timer <= 0;
      restart = d && (in.flags & CRAFT_STEP_AUTORESET);
    }
    if (d) succ = satisfies(s, g, iv, a, a.task);   // on the pre-step state
    if (restart) {                                   // CraftScenario.init, craft.py:268-273
      const uint32_t iw = s->init[slot];
      a.x = iw & 0xff; a.y = (iw >> 8) & 0xff; a.dir = (iw >> 16) & 3;
      a.timer = s->cfg.max_timesteps;
      std::memset(iv, 0, 32);
      std::memset(m, 0, 32);
      std::memcpy(g, s->pool.data() + (size_t)a.scen * s->C, s->C);
    } else if (d && !a.frozen) {
      a.frozen = 1;
      a.timer = std::max(a.timer, 0);
    } else if (!d) {
      if (act < 0 || act >= CRAFT_N_ACTIONS) {
        latch(s, CRAFT_EBADACTION, slot);
      } else {
        const int ox = a.x, oy = a.y;
        bool ic = false, mc = false;
        transition(s, g, iv, a, m, act, ic, mc, slot);
        code = transition_code(ox, oy, a, ic);
      }
    }
    s->state[slot] = pack_state(a);
    if (in.done) in.done[i] = (uint8_t)d;
    if (in.sat) in.sat[i] = (int8_t)succ;
    if (in.reward) in.reward[i] = (counted && d && succ == 1) ? 1.0f : 0.0f;
    if (in.rec) in.rec[i] = counted ? act : -1;      // action_seqs, imitation.py:59-61
    acc.succ += counted && d && succ == 1;
    acc.ended += counted && d;
    acc.steps += counted;
    acc.any_live = acc.any_live || (counted && !d);
  }
  if (in.code) in.code[i] = (int8_t)code;
  if (in.obs) {
    if (live) features(s, g, iv, a, row);
    else std::memset(row, 0, s->F);
    put_obs(s->obs_fmt, in.obs, i, s->F, row);
  }
  if (in.label) {                                    // the teacher's label of the new state
    int action = -2;
    if (live && a.frozen) {
      action = -1;                                   // imitation.py:50-51
    } else if (live) {
      int len = -1, err = 0;
      action = teach(s, g, iv, a, a.task, false, len, err);
      if (err) latch(s, err, i);
    }
    in.label[i] = action;
  }
}

int run_ticks(craft_sim* s, const TickIn& in, int32_t* any_live) {
  TickAcc tot;
  std::atomic<int64_t> succ{0}, ended{0}, steps{0};
  std::atomic<bool> live{false};
  parallel_for(s, s->n_envs, [&](int64_t lo, int64_t hi) {
    TickAcc acc;
    std::vector<uint8_t> g(CRAFT_MAX_CELLS), row(s->F);
    for (int64_t i = lo; i < hi; ++i) tick_slot(s, i, in, acc, g.data(), row.data());
    succ += acc.succ; ended += acc.ended; steps += acc.steps;
    if (acc.any_live) live = true;
  });
  s->stats[0] += succ.load();
  s->stats[1] += ended.load();
  s->stats[2] += steps.load();
  if (any_live && live.load()) *any_live = 1;        // only ever set to 1 (craft.h)
  return CRAFT_OK;
}

// The checks craft_step_ex / craft_step_teach make before any work (craft_sim.hip step_args).
int step_check(craft_sim* s, const craft_step_args_t* x) {
  if (x->obs && (reinterpret_cast<uintptr_t>(x->obs) & 15u))
    return fail(s, CRAFT_EINVAL, "craft_step: obs must be 16-byte aligned");
  if (x->behavior_clone && !x->ref_actions)
    return fail(s, CRAFT_EINVAL, "craft_step_ex: behavior_clone needs ref_actions");
  return CRAFT_OK;
}

TickIn tick_in(const craft_step_args_t* x) {
  TickIn in{};
  in.actions = x->actions; in.ref = x->ref_actions; in.bc = x->behavior_clone;
  in.seed = x->action_seed; in.tick = x->tick; in.flags = x->flags;
  in.obs = x->obs; in.reward = x->reward; in.done = x->done; in.sat = x->success;
  in.rec = x->action_record; in.code = x->transition_code;
  return in;
}

// the per-scenario stream of craft_pool_generate (craft_scenarios.hip SplitMix)
struct SplitMix {
  uint64_t s;
  uint32_t next32() {
    s += 0x9E3779B97F4A7C15ull;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return (uint32_t)((z ^ (z >> 31)) >> 32);
  }
  int randint(uint32_t n) {                          // Lemire's unbiased multiply-shift
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

}  // namespace

extern "C" {

const char* craft_strerror(int status) { return craft_host::status_text(status); }

int craft_host_flag_pointer(void* host, int32_t** device_out) {
  if (!host || !device_out) return CRAFT_EINVAL;
  *device_out = static_cast<int32_t*>(host);          // host memory is the CPU variant's own
  return CRAFT_OK;
}

int craft_sim_create(const craft_config_t* cfg, int device, int64_t n_envs, int64_t env_id_base,
                     int32_t pool_capacity, craft_sim_t** out) {
  (void)device;
  if (!cfg || !out || n_envs <= 0 || pool_capacity <= 0 || pool_capacity > (1 << 24) || env_id_base < 0)
    return CRAFT_EINVAL;
  *out = nullptr;
  std::string msg;
  const int rc = craft_host::validate_config(cfg, msg);
  if (rc) {
    fprintf(stderr, "craft_sim_create: %s\n", msg.c_str());
    return rc;
  }
  craft_sim* s = new (std::nothrow) craft_sim();
  if (!s) return CRAFT_ENOMEM;
  s->cfg = *cfg;
  s->n_envs = n_envs;
  s->env_base = env_id_base;
  s->pool_capacity = pool_capacity;
  s->W = cfg->width; s->H = cfg->height; s->C = s->W * s->H; s->K = cfg->n_kinds; s->F = cfg->n_features;
  s->win = cfg->window_width;
  s->tile = default_tile(s->win);
  for (auto& x : s->stats) x = 0;
  try {
    s->pool.assign((size_t)pool_capacity * s->C, 0);
    s->pool_conn.assign((size_t)pool_capacity, 0);
    s->state.assign(n_envs, 0);
    s->init.assign(n_envs, 0);
    s->inv.assign((size_t)n_envs * 32, 0);
    s->mask.assign((size_t)n_envs * 8, 0);
  } catch (const std::bad_alloc&) {
    delete s;
    return CRAFT_ENOMEM;
  }
  craft_host::task_tables(*cfg, s->task_tab, s->task_sub);
  s->threads = hw_threads();
  *out = s;
  return CRAFT_OK;
}

int craft_sim_destroy(craft_sim_t* s) {
  delete s;
  return CRAFT_OK;
}

const char* craft_sim_last_error(const craft_sim_t* s) { return s ? s->last_error.c_str() : "null handle"; }

int craft_sim_info(const craft_sim_t* s, int64_t* n_envs, int32_t* pool_capacity, int32_t* n_features) {
  if (!s) return CRAFT_EINVAL;
  if (n_envs) *n_envs = s->n_envs;
  if (pool_capacity) *pool_capacity = s->pool_capacity;
  if (n_features) *n_features = s->cfg.n_features;
  return CRAFT_OK;
}

// The tuning knobs are validated as the HIP library validates them and reported back by the
// shape queries; they change nothing here (there are no workgroups).
int craft_sim_tune(craft_sim_t* s, int32_t tile_envs, int32_t max_resident_per_cu, int32_t obs_store) {
  if (!s) return CRAFT_EINVAL;
  if (tile_envs == 0) tile_envs = default_tile(s->win);
  if (tile_envs != 16 && tile_envs != 32 && tile_envs != 64)
    return fail(s, CRAFT_EINVAL, "craft_sim_tune: tile_envs must be 16, 32 or 64");
  if (max_resident_per_cu != 0 && (max_resident_per_cu < 3 || max_resident_per_cu > 32))
    return fail(s, CRAFT_EINVAL, "craft_sim_tune: max_resident_per_cu must be 0 or 3..32");
  if (obs_store < 0 || obs_store > 2)
    return fail(s, CRAFT_EINVAL, "craft_sim_tune: obs_store must be 0 (write-back), 1 (nontemporal) or 2 (write-through)");
  s->tile = tile_envs;
  s->resident_cap = max_resident_per_cu;
  s->obs_store = obs_store;
  return CRAFT_OK;
}

int craft_sim_tune_rollout(craft_sim_t* s, int32_t chunk_ticks, int32_t threads) {
  if (!s) return CRAFT_EINVAL;
  if (chunk_ticks < -1 || chunk_ticks > 4096)
    return fail(s, CRAFT_EINVAL, "craft_sim_tune_rollout: chunk_ticks must be -1..4096");
  if (threads != 0 && threads != 128 && threads != 256 && threads != 320 && threads != 384 && threads != 512)
    return fail(s, CRAFT_EINVAL, "craft_sim_tune_rollout: threads must be 0, 128, 256, 320, 384 or 512");
  s->rollout_chunk = chunk_ticks;
  s->rollout_threads = threads;
  return CRAFT_OK;
}

int craft_sim_tune_teach(craft_sim_t* s, int32_t kernel, int32_t lanes, int32_t table) {
  if (!s) return CRAFT_EINVAL;
  if (kernel < 0 || kernel > 2)
    return fail(s, CRAFT_EINVAL, "craft_sim_tune_teach: kernel must be 0 (auto), 1 (one-tile) or 2 (two-tile)");
  if (lanes != 0 && lanes != 1 && lanes != 2 && lanes != 4)
    return fail(s, CRAFT_EINVAL, "craft_sim_tune_teach: lanes must be 0 (default), 1, 2 or 4");
  if (table < 0 || table > 2)
    return fail(s, CRAFT_EINVAL, "craft_sim_tune_teach: table must be 0 (auto), 1 (always) or 2 (never)");
  s->teach_kernel = kernel;
  s->teach_lanes = lanes;
  s->teach_table = table;      // (this variant keeps no table: every query runs the BFS)
  return CRAFT_OK;
}

int craft_abi_version(void) { return CRAFT_ABI_VERSION; }

int craft_sim_tune_host(craft_sim_t* s, int32_t threads) {
  if (!s) return CRAFT_EINVAL;
  if (threads < 0 || threads > 1024)
    return fail(s, CRAFT_EINVAL, "craft_sim_tune_host: threads must be 0 (the machine's) or 1..1024");
  s->threads = threads ? threads : hw_threads();
  return CRAFT_OK;
}

int craft_sim_sync_table(craft_sim_t* s, void* /*stream*/) {
  return s ? CRAFT_OK : CRAFT_EINVAL;      // (this variant keeps no table)
}

int craft_sim_step_shape(const craft_sim_t* s, int32_t teach, int32_t* kernel, int32_t* envs, int32_t* lanes) {
  if (!s) return CRAFT_EINVAL;
  if (kernel) *kernel = CRAFT_KERNEL_TILE;
  if (envs) *envs = s->tile;
  if (lanes) *lanes = teach ? 1 : 0;
  return CRAFT_OK;
}

int craft_sim_rollout_shape(const craft_sim_t* s, int32_t* tile_envs, int32_t* threads, int32_t* split) {
  if (!s) return CRAFT_EINVAL;
  if (tile_envs) *tile_envs = s->tile;
  if (threads) *threads = s->rollout_threads;
  if (split) *split = 0;
  return CRAFT_OK;
}

int craft_sim_tile_shape(const craft_sim_t* s, int32_t* tile_envs, int32_t* obs_store) {
  if (!s) return CRAFT_EINVAL;
  if (tile_envs) *tile_envs = s->tile;
  if (obs_store) *obs_store = s->obs_store;
  return CRAFT_OK;
}

int craft_sim_set_obs_format(craft_sim_t* s, int32_t format) {
  if (!s) return CRAFT_EINVAL;
  if (format != CRAFT_OBS_F32 && format != CRAFT_OBS_BF16 && format != CRAFT_OBS_U8)
    return fail(s, CRAFT_EINVAL, "craft_sim_set_obs_format: format must be 0 (fp32), 1 (bf16) or 2 (u8)");
  s->obs_fmt = format;
  return CRAFT_OK;
}

int craft_sim_check(craft_sim_t* s, int64_t* env_out, void* /*stream*/) {
  if (!s) return CRAFT_EINVAL;
  const int code = s->err_code.exchange(0);
  const int64_t slot = s->err_slot.exchange(-1);
  if (code) {
    if (env_out) *env_out = slot;
    return fail(s, code, std::string(craft_strerror(code)) + " (slot/item " + std::to_string(slot) + ")");
  }
  if (env_out) *env_out = -1;
  return CRAFT_OK;
}

int craft_sim_error_word(craft_sim_t* s, int32_t* out, void* /*stream*/) {
  if (!s || !out) return CRAFT_EINVAL;
  const int code = s->err_code.load();
  const int64_t slot = code ? s->err_slot.load() : 0;
  out[0] = code;
  out[1] = 0;
  out[2] = (int32_t)(slot & 0xffffffff);
  out[3] = (int32_t)(slot >> 32);
  return CRAFT_OK;
}

int craft_pool_load(craft_sim_t* s, const uint8_t* grids, int32_t first, int32_t count) {
  if (!s || !grids || first < 0 || count < 0) return fail(s, CRAFT_EINVAL, "craft_pool_load: bad argument");
  if ((int64_t)first + count > s->pool_capacity) return fail(s, CRAFT_ERANGE, "craft_pool_load: beyond pool capacity");
  std::vector<uint8_t> conn((size_t)count, 0);
  for (int p = 0; p < count; ++p) {             // every row is checked before any is written
    std::string msg;
    const int rc = craft_host::check_pool_grid(s->cfg, grids + (size_t)p * s->C, (int64_t)first + p, msg, &conn[p]);
    if (rc) return fail(s, rc, msg);
  }
  std::memcpy(s->pool.data() + (size_t)first * s->C, grids, (size_t)count * s->C);
  std::memcpy(s->pool_conn.data() + first, conn.data(), count);
  if (first + count > s->pool_count) s->pool_count = first + count;
  return CRAFT_OK;
}

// make_data.sample_scenario (make_data.py:105-144) per scenario with its own splitmix64 stream,
// exactly craft_scenarios.hip: boundary ring, primitives, workshops, init position, each cell
// drawn by random_free with the acceptance test (free cells one component, every occupied
// interior cell next to a free one), at most 2^20 draws per placement.
int craft_pool_generate(craft_sim_t* s, uint64_t seed, int64_t scenario_id0, int32_t first, int32_t count,
                        int32_t boundary_kind, const int32_t* primitives, int32_t n_primitive_kinds,
                        int32_t n_per_primitive, const int32_t* workshop_kind, int32_t n_workshops,
                        int32_t* init_pos_out, void* /*stream*/) {
  if (!s || first < 0 || count < 0 || n_primitive_kinds < 0 || n_primitive_kinds > 8 || n_per_primitive < 0 ||
      n_workshops < 0 || n_workshops > 8 || (n_primitive_kinds && !primitives) || (n_workshops && !workshop_kind))
    return fail(s, CRAFT_EINVAL, "craft_pool_generate: bad argument");
  if ((int64_t)first + count > s->pool_capacity) return fail(s, CRAFT_ERANGE, "craft_pool_generate: beyond pool capacity");
  const int K = s->K, W = s->W, H = s->H, C = s->C;
  auto bad_kind = [&](int k) { return k <= 0 || k >= K; };
  if (bad_kind(boundary_kind)) return fail(s, CRAFT_EINVAL, "craft_pool_generate: bad boundary kind");
  for (int i = 0; i < n_primitive_kinds; ++i)
    if (bad_kind(primitives[i])) return fail(s, CRAFT_EINVAL, "craft_pool_generate: bad primitive kind");
  for (int i = 0; i < n_workshops; ++i)
    if (bad_kind(workshop_kind[i])) return fail(s, CRAFT_EINVAL, "craft_pool_generate: bad workshop kind");
  if ((int64_t)n_primitive_kinds * n_per_primitive + n_workshops + 1 > (int64_t)(W - 2) * (H - 2))
    return fail(s, CRAFT_EINVAL, "craft_pool_generate: more objects than interior cells");
  const Bits valid = brange(0, C);
  Bits border = bzero();
  for (int c = 0; c < C; ++c) {
    const int x = c / H, y = c % H;
    if (x == 0 || y == 0 || x == W - 1 || y == H - 1) border = bor(border, bbit(c));
  }
  const Bits interior = bandn(valid, border);
  auto nbrs = [&](const Bits& b) {
    return band(bor(bor(bshift(b, 1), bshift(b, -1)), bor(bshift(b, H), bshift(b, -H))), valid);
  };
  auto acceptable = [&](const Bits& occ) -> bool {
    const Bits fr = bandn(valid, occ);
    const int p0 = blowest(fr);
    if (p0 == INT_MAX) return true;
    Bits reach = bbit(p0);
    for (int it = 0; it < CRAFT_MAX_CELLS; ++it) {   // flood fill of the free cells
      const Bits nxt = bor(reach, band(nbrs(reach), fr));
      const bool same = beq(nxt, reach);
      reach = nxt;
      if (same) break;
    }
    if (bany(bandn(fr, reach))) return false;       // (1) free cells connected
    return !bany(bandn(band(occ, interior), nbrs(fr)));   // (2) objects stay accessible
  };
  parallel_for(s, count, [&](int64_t lo, int64_t hi) {
    for (int64_t sc = lo; sc < hi; ++sc) {
      SplitMix rng{seed ^ ((uint64_t)(scenario_id0 + sc) * 0xD1B54A32D192ED03ull)};
      uint8_t* row = s->pool.data() + (size_t)(first + sc) * C;
      for (int c = 0; c < C; ++c) row[c] = btest(border, c) ? (uint8_t)boundary_kind : 0;
      Bits occ = border;
      bool failed = false;
      int cell = 0;
      auto random_free = [&](int& out) -> bool {
        for (int draws = 0; draws < (1 << 20); ++draws) {
          const int x = rng.randint((uint32_t)W), y = rng.randint((uint32_t)H);
          const int c = x * H + y;
          if (btest(occ, c)) continue;
          if (acceptable(bor(occ, bbit(c)))) {
            out = c;
            return true;
          }
        }
        return false;
      };
      for (int p = 0; p < n_primitive_kinds && !failed; ++p)
        for (int i = 0; i < n_per_primitive && !failed; ++i) {
          if (!random_free(cell)) { failed = true; break; }
          occ = bor(occ, bbit(cell));
          row[cell] = (uint8_t)primitives[p];
        }
      for (int i = 0; i < n_workshops && !failed; ++i) {
        if (!random_free(cell)) { failed = true; break; }
        occ = bor(occ, bbit(cell));
        row[cell] = (uint8_t)workshop_kind[i];
      }
      if (!failed && !random_free(cell)) failed = true;
      if (failed) {
        latch(s, CRAFT_EINVARIANT, scenario_id0 + sc);
        cell = 0;
      }
      s->pool_conn[first + sc] = failed ? 0 : 1;
      if (init_pos_out) {
        init_pos_out[2 * sc] = cell / H;
        init_pos_out[2 * sc + 1] = cell % H;
      }
    }
  });
  if (first + count > s->pool_count) s->pool_count = first + count;
  return CRAFT_OK;
}

int craft_reset(craft_sim_t* s, const int32_t* scenario, const int32_t* pos_x, const int32_t* pos_y,
                const int32_t* dir, const int32_t* task, void* obs, void* /*stream*/) {
  if (!s || !scenario || !pos_x || !pos_y || !dir || !task) return fail(s, CRAFT_EINVAL, "craft_reset: null input");
  if (obs && (reinterpret_cast<uintptr_t>(obs) & 15u)) return fail(s, CRAFT_EINVAL, "craft_reset: obs must be 16-byte aligned");
  parallel_for(s, s->n_envs, [&](int64_t lo, int64_t hi) {
    std::vector<uint8_t> g(CRAFT_MAX_CELLS), row(s->F);
    for (int64_t i = lo; i < hi; ++i) {             // CraftScenario.init, craft.py:262-273
      const int sc = scenario[i], x0 = pos_x[i], y0 = pos_y[i], d0 = dir[i], tk = task[i];
      const bool ok = !(sc < 0 || sc >= s->pool_count || x0 < 1 || x0 > s->W - 2 || y0 < 1 || y0 > s->H - 2 ||
                        d0 < 0 || d0 > 3 || tk < 0 || tk >= s->cfg.n_tasks);
      if (!ok) {
        latch(s, CRAFT_EINVAL, i);
      } else {
        Agent a{x0, y0, d0, 0, s->cfg.max_timesteps, sc, tk};
        s->state[i] = pack_state(a);
        s->init[i] = (uint32_t)x0 | ((uint32_t)y0 << 8) | ((uint32_t)d0 << 16);
        std::memset(s->inv.data() + 32 * i, 0, 32);
        std::memset(s->mask.data() + 8 * i, 0, 32);
      }
      if (obs) {
        if (ok) {
          std::memcpy(g.data(), s->pool.data() + (size_t)sc * s->C, s->C);
          features(s, g.data(), s->inv.data() + 32 * i, unpack_state(s->state[i]), row.data());
        } else {
          std::memset(row.data(), 0, s->F);
        }
        put_obs(s->obs_fmt, obs, i, s->F, row.data());
      }
    }
  });
  for (auto& x : s->stats) x = 0;
  return CRAFT_OK;
}

int craft_step_ex(craft_sim_t* s, const craft_step_args_t* x, void* /*stream*/) {
  if (!s || !x) return CRAFT_EINVAL;
  const int rc = step_check(s, x);
  if (rc) return rc;
  return run_ticks(s, tick_in(x), x->any_live);
}

int craft_step(craft_sim_t* s, const int32_t* actions, uint64_t action_seed, int64_t tick, uint32_t flags,
               void* obs, float* reward, uint8_t* done, int8_t* success, void* stream) {
  craft_step_args_t x{};
  x.actions = actions; x.action_seed = action_seed; x.tick = tick; x.flags = flags;
  x.obs = obs; x.reward = reward; x.done = done; x.success = success;
  return craft_step_ex(s, &x, stream);
}

int craft_step_teach(craft_sim_t* s, const craft_step_args_t* x, int32_t* label_out, void* /*stream*/) {
  if (!s || !x || !label_out) return CRAFT_EINVAL;
  if (4 * s->C > 1000)
    return fail(s, CRAFT_EINVAL, "craft_step_teach: 4*W*H > 1000 overflows the reference's BFS queue (teachers/base.py:42)");
  const int rc = step_check(s, x);
  if (rc) return rc;
  TickIn in = tick_in(x);
  in.label = label_out;
  return run_ticks(s, in, x->any_live);
}

int craft_rollout(craft_sim_t* s, const int32_t* actions, uint64_t action_seed, int64_t tick0, int32_t n_ticks,
                  uint32_t flags, void* obs, int32_t ring, float* reward, uint8_t* done, int8_t* success,
                  void* /*stream*/) {
  if (!s) return CRAFT_EINVAL;
  if (n_ticks < 0 || ring < 1 || tick0 < 0)
    return fail(s, CRAFT_EINVAL, "craft_rollout: need n_ticks >= 0, ring >= 1, tick0 >= 0");
  const int esz = esize(s->obs_fmt);
  if (obs && ((reinterpret_cast<uintptr_t>(obs) & 15u) || (ring > 1 && (s->n_envs * (int64_t)s->F * esz) % 16 != 0)))
    return fail(s, CRAFT_EINVAL, "craft_rollout: every obs ring slot must be 16-byte aligned");
  const int64_t n = s->n_envs;
  for (int32_t k = 0; k < n_ticks; ++k) {
    const int64_t r = (tick0 + k) % ring;            // tick t writes ring slot t % ring
    TickIn in{};
    in.actions = actions ? actions + (int64_t)k * n : nullptr;
    in.seed = action_seed;
    in.tick = tick0 + k;
    in.flags = flags;
    in.obs = obs ? static_cast<uint8_t*>(obs) + r * n * s->F * esz : nullptr;
    in.reward = reward ? reward + r * n : nullptr;
    in.done = done ? done + r * n : nullptr;
    in.sat = success ? success + r * n : nullptr;
    run_ticks(s, in, nullptr);
  }
  return CRAFT_OK;
}

// craft_rollout_teach: tick by tick, the labels of each tick's new states carried to the next
// tick's label-source slots (make_data.get_reference_actions, imitation.py:47-57)
int craft_rollout_teach(craft_sim_t* s, const craft_rollout_teach_args_t* x, void* /*stream*/) {
  if (!s || !x) return CRAFT_EINVAL;
  if (x->n_ticks < 0 || x->ring < 1 || x->tick0 < 0)
    return fail(s, CRAFT_EINVAL, "craft_rollout_teach: need n_ticks >= 0, ring >= 1, tick0 >= 0");
  if (4 * s->C > 1000)
    return fail(s, CRAFT_EINVAL, "craft_rollout_teach: 4*W*H > 1000 overflows the reference's BFS queue (teachers/base.py:42)");
  const bool lsync = x->label_actions != 0 || x->behavior_clone != nullptr;
  if (lsync && !x->label_in)
    return fail(s, CRAFT_EINVAL, "craft_rollout_teach: label_actions / behavior_clone need label_in");
  const int esz = esize(s->obs_fmt);
  if (x->obs && ((reinterpret_cast<uintptr_t>(x->obs) & 15u) ||
                 (x->ring > 1 && (s->n_envs * (int64_t)s->F * esz) % 16 != 0)))
    return fail(s, CRAFT_EINVAL, "craft_rollout_teach: every obs ring slot must be 16-byte aligned");
  const int64_t n = s->n_envs;
  std::vector<int32_t> cur(n, 0), lab(n, 0);
  std::vector<uint8_t> src(n, 0);                    // 1: the slot acts on its label
  for (int64_t i = 0; i < n; ++i) {
    src[i] = x->label_actions ? 1 : (x->behavior_clone && x->behavior_clone[i] ? 1 : 0);
    if (lsync) cur[i] = x->label_in[i];
  }
  for (int32_t k = 0; k < x->n_ticks; ++k) {
    const int64_t r = (x->tick0 + k) % x->ring;
    TickIn in{};
    in.actions = x->actions ? x->actions + (int64_t)k * n : nullptr;
    in.ref = cur.data();
    in.bc = lsync ? src.data() : nullptr;
    in.seed = x->action_seed;
    in.tick = x->tick0 + k;
    in.flags = x->flags;
    in.obs = x->obs ? static_cast<uint8_t*>(x->obs) + r * n * s->F * esz : nullptr;
    in.reward = x->reward ? x->reward + r * n : nullptr;
    in.done = x->done ? x->done + r * n : nullptr;
    in.sat = x->success ? x->success + r * n : nullptr;
    in.rec = x->action_record ? x->action_record + r * n : nullptr;
    in.label = lab.data();
    run_ticks(s, in, nullptr);
    if (x->labels) std::memcpy(x->labels + r * n, lab.data(), sizeof(int32_t) * n);
    cur.swap(lab);
  }
  return CRAFT_OK;
}

int craft_stats(craft_sim_t* s, int64_t* stats_out, int32_t reset, void* /*stream*/) {
  if (!s || !stats_out) return CRAFT_EINVAL;
  for (int j = 0; j < 3; ++j) stats_out[j] = reset ? s->stats[j].exchange(0) : s->stats[j].load();
  return CRAFT_OK;
}

int craft_transition(craft_sim_t* s, const int32_t* src, const int32_t* dst, const int32_t* actions, int64_t n,
                     int8_t* code_out, void* /*stream*/) {
  if (!s) return CRAFT_EINVAL;
  if (n == 0) return CRAFT_OK;
  if (!actions || n < 0) return fail(s, CRAFT_EINVAL, "craft_transition: bad argument");
  if (!src && n > s->n_envs) return fail(s, CRAFT_ERANGE, "craft_transition: n > n_envs");
  parallel_for(s, n, [&](int64_t lo, int64_t hi) {
    std::vector<uint8_t> g(CRAFT_MAX_CELLS);
    for (int64_t i = lo; i < hi; ++i) {              // CraftState.step, craft.py:332-424
      const int64_t slot = src ? (int64_t)src[i] : i, dslot = dst ? (int64_t)dst[i] : slot;
      int code = -1;
      if (slot < 0 || slot >= s->n_envs || dslot < 0 || dslot >= s->n_envs) {
        latch(s, CRAFT_ERANGE, i);
      } else {
        Agent a = unpack_state(s->state[slot]);
        if (a.x < 1 || a.x > s->W - 2 || a.y < 1 || a.y > s->H - 2 || a.scen >= s->pool_count) {
          latch(s, CRAFT_EINVAL, slot);
        } else {
          uint8_t iv[32];
          uint32_t m[8];
          std::memcpy(iv, s->inv.data() + 32 * slot, 32);
          std::memcpy(m, s->mask.data() + 8 * slot, 32);
          env_grid(s, slot, a.scen, g.data());
          const int act = actions[i];
          if (act >= CRAFT_N_ACTIONS) {
            latch(s, CRAFT_EBADACTION, slot);
          } else if (act >= 0) {
            const int ox = a.x, oy = a.y;
            bool ic = false, mc = false;
            transition(s, g.data(), iv, a, m, act, ic, mc, slot);
            code = transition_code(ox, oy, a, ic);
          }
          s->state[dslot] = pack_state(a);
          if (dslot != slot) s->init[dslot] = s->init[slot];
          std::memcpy(s->inv.data() + 32 * dslot, iv, 32);
          std::memcpy(s->mask.data() + 8 * dslot, m, 32);
        }
      }
      if (code_out) code_out[i] = (int8_t)code;
    }
  });
  return CRAFT_OK;
}

int craft_observe(craft_sim_t* s, const int32_t* slots, int64_t n, const int32_t* tasks, void* obs, int8_t* sat,
                  void* /*stream*/) {
  if (!s) return CRAFT_EINVAL;
  if (n == 0) return CRAFT_OK;
  if (n < 0) return fail(s, CRAFT_EINVAL, "craft_observe: bad argument");
  if (!slots && n > s->n_envs) return fail(s, CRAFT_ERANGE, "craft_observe: n > n_envs");
  if (obs && (reinterpret_cast<uintptr_t>(obs) & 15u)) return fail(s, CRAFT_EINVAL, "craft_observe: obs must be 16-byte aligned");
  parallel_for(s, n, [&](int64_t lo, int64_t hi) {
    std::vector<uint8_t> g(CRAFT_MAX_CELLS), row(s->F);
    for (int64_t i = lo; i < hi; ++i) {              // features() / satisfies(), craft.py:285-330
      const int64_t slot = slots ? (int64_t)slots[i] : i;
      bool live = slot >= 0 && slot < s->n_envs;
      Agent a{};
      if (!live) {
        latch(s, CRAFT_ERANGE, i);
      } else {
        a = unpack_state(s->state[slot]);
        if (a.x < 1 || a.x > s->W - 2 || a.y < 1 || a.y > s->H - 2 || a.scen >= s->pool_count) {
          latch(s, CRAFT_EINVAL, slot);
          live = false;
        }
      }
      if (live) {
        env_grid(s, slot, a.scen, g.data());
        const uint8_t* iv = s->inv.data() + 32 * slot;
        if (sat) {
          const int tk = tasks ? tasks[i] : a.task;
          if (tk < 0 || tk >= s->cfg.n_tasks) {
            latch(s, CRAFT_ERANGE, i);
            sat[i] = -1;
          } else {
            sat[i] = (int8_t)satisfies(s, g.data(), iv, a, tk);
          }
        }
        if (obs) features(s, g.data(), iv, a, row.data());
      } else if (obs) {
        std::memset(row.data(), 0, s->F);
      }
      if (obs) put_obs(s->obs_fmt, obs, i, s->F, row.data());
    }
  });
  return CRAFT_OK;
}

int craft_rollout_distances(craft_sim_t* s, const int32_t* tasks, const int8_t* success, const int32_t* action_seqs,
                            int32_t ticks, int32_t* distances_out, uint8_t* is_get_out, int32_t* n_actions_out,
                            int32_t* flags_out, void* /*stream*/) {
  if (!s) return CRAFT_EINVAL;
  if (!tasks || !success || !distances_out || !is_get_out || !n_actions_out || !flags_out || ticks < 0 ||
      (ticks > 0 && !action_seqs))
    return fail(s, CRAFT_EINVAL, "craft_rollout_distances: bad argument");
  if (4 * s->C > 1000)
    return fail(s, CRAFT_EINVAL, "craft_rollout_distances: 4*W*H > 1000 overflows the reference's BFS queue (teachers/base.py:42)");
  std::atomic<int32_t> f0{0}, f1{0};
  parallel_for(s, s->n_envs, [&](int64_t lo, int64_t hi) {
    for (int64_t i = lo; i < hi; ++i) {              // trainers/imitation.py:79-91
      const int task = tasks[i], succ = success[i];
      int na = 0;
      for (int t = 0; t < ticks; ++t) na += action_seqs[(int64_t)t * s->n_envs + i] >= 0;
      n_actions_out[i] = na;
      if (task < 0 || task >= s->cfg.n_tasks) {
        latch(s, CRAFT_ERANGE, i);
        distances_out[i] = -2;
        is_get_out[i] = 0;
        n_actions_out[i] = 0;
        continue;
      }
      const uint32_t tt = s->task_tab[task];
      const bool is_get = (tt & 0xf) == CRAFT_GOAL_GET;
      const int arg = (tt >> 4) & 0xff;
      int d = is_get ? 0 : -1;
      if (is_get && succ == 0 && arg == 0) {
        d = -1;
      } else if (is_get && succ == 0) {
        const Agent a = unpack_state(s->state[i]);
        if (a.x < 1 || a.x > s->W - 2 || a.y < 1 || a.y > s->H - 2 || a.scen >= s->pool_count) {
          latch(s, CRAFT_EINVAL, i);
          d = -2;
        } else {                                     // world.init_state(grid, pos, dir): the pool row
          int fa = -1, len = -1;
          const bool ok = closest(s, s->pool.data() + (size_t)a.scen * s->C, arg, a.x * s->H + a.y, a.dir, fa,
                                  len, false);
          d = ok ? len : -2;
        }
      }
      distances_out[i] = d;
      is_get_out[i] = is_get;
      if (succ < 0) f0 = 1;
      if ((d == -1 || d == -2) && is_get && succ == 0) f1 = 1;   // len(None), imitation.py:88-89
    }
  });
  flags_out[0] = f0.load();
  flags_out[1] = f1.load();
  return CRAFT_OK;
}

int craft_teacher(craft_sim_t* s, const int32_t* slots, int64_t n, const int32_t* tasks, int32_t* action_out,
                  int32_t* path_len_out, void* /*stream*/) {
  if (!s) return CRAFT_EINVAL;
  if (n == 0) return CRAFT_OK;
  if (!action_out || n < 0) return fail(s, CRAFT_EINVAL, "craft_teacher: bad argument");
  if (!slots && n > s->n_envs) return fail(s, CRAFT_ERANGE, "craft_teacher: n > n_envs");
  if (4 * s->C > 1000)
    return fail(s, CRAFT_EINVAL, "craft_teacher: 4*W*H > 1000 overflows the reference's BFS queue (teachers/base.py:42)");
  parallel_for(s, n, [&](int64_t lo, int64_t hi) {
    std::vector<uint8_t> g(CRAFT_MAX_CELLS);
    for (int64_t i = lo; i < hi; ++i) {              // DemonstrationTeacher.__call__
      const int64_t slot = slots ? (int64_t)slots[i] : i;
      auto put = [&](int act, int len) {
        action_out[i] = act;
        if (path_len_out) path_len_out[i] = len;
      };
      if (slot == -1) { put(-1, -1); continue; }     // skipped item: a done env's ref_action
      if (slot < 0 || slot >= s->n_envs) { latch(s, CRAFT_ERANGE, i); put(-2, -2); continue; }
      const Agent a = unpack_state(s->state[slot]);
      if (a.frozen) { put(-1, -1); continue; }       // imitation.py:50-51
      const int task = tasks ? tasks[i] : a.task;
      if (task < 0 || task >= s->cfg.n_tasks || a.x < 1 || a.x > s->W - 2 || a.y < 1 || a.y > s->H - 2 ||
          a.scen >= s->pool_count) {
        latch(s, task < 0 || task >= s->cfg.n_tasks ? CRAFT_ERANGE : CRAFT_EINVAL, i);
        put(-2, -2);
        continue;
      }
      env_grid(s, slot, a.scen, g.data());
      int len = -1, err = 0;
      const int act = teach(s, g.data(), s->inv.data() + 32 * slot, a, task, path_len_out != nullptr, len, err);
      if (err) latch(s, err, slot);
      if (path_len_out && len == -2) latch(s, CRAFT_ETEACHER, slot);
      put(act, len);
    }
  });
  return CRAFT_OK;
}

int craft_get_state(craft_sim_t* s, const int32_t* slots, int64_t n, int32_t* agent, int32_t* inventory,
                    uint8_t* grid, int32_t* spec, void* /*stream*/) {
  if (!s) return CRAFT_EINVAL;
  if (n == 0) return CRAFT_OK;
  if (n < 0) return fail(s, CRAFT_EINVAL, "craft_get_state: bad argument");
  if (!slots && n > s->n_envs) return fail(s, CRAFT_ERANGE, "craft_get_state: n > n_envs");
  for (int64_t i = 0; i < n; ++i) {
    const int64_t slot = slots ? (int64_t)slots[i] : i;
    if (slot < 0 || slot >= s->n_envs) { latch(s, CRAFT_ERANGE, i); continue; }
    const Agent a = unpack_state(s->state[slot]);
    if (agent) { agent[4 * i] = a.x; agent[4 * i + 1] = a.y; agent[4 * i + 2] = a.dir; agent[4 * i + 3] = a.timer; }
    if (inventory)
      for (int k = 0; k < s->K; ++k) inventory[i * s->K + k] = s->inv[32 * slot + k];
    if (grid) {
      if (a.scen < s->pool_count) env_grid(s, slot, a.scen, grid + i * s->C);
      else std::memset(grid + i * s->C, 0, s->C);
    }
    if (spec) {
      const uint32_t in = s->init[slot];
      spec[5 * i] = a.scen; spec[5 * i + 1] = in & 0xff; spec[5 * i + 2] = (in >> 8) & 0xff;
      spec[5 * i + 3] = (in >> 16) & 3; spec[5 * i + 4] = a.task;
    }
  }
  return CRAFT_OK;
}

int craft_set_state(craft_sim_t* s, const int32_t* slots, int64_t n, const int32_t* spec, const int32_t* agent,
                    const int32_t* inventory, void* /*stream*/) {
  if (!s) return CRAFT_EINVAL;
  if (n == 0) return CRAFT_OK;
  if (n < 0 || !spec || !agent) return fail(s, CRAFT_EINVAL, "craft_set_state: bad argument");
  if (!slots && n > s->n_envs) return fail(s, CRAFT_ERANGE, "craft_set_state: n > n_envs");
  for (int64_t i = 0; i < n; ++i) {
    const int64_t slot = slots ? (int64_t)slots[i] : i;
    if (slot < 0 || slot >= s->n_envs) { latch(s, CRAFT_ERANGE, i); continue; }
    const int sc = spec[5 * i], x0 = spec[5 * i + 1], y0 = spec[5 * i + 2], d0 = spec[5 * i + 3], tk = spec[5 * i + 4];
    const int x = agent[4 * i], y = agent[4 * i + 1], d = agent[4 * i + 2], tm = agent[4 * i + 3];
    bool ok = sc >= 0 && sc < s->pool_count && tk >= 0 && tk < s->cfg.n_tasks && x0 >= 1 && x0 <= s->W - 2 &&
              y0 >= 1 && y0 <= s->H - 2 && d0 >= 0 && d0 < 4 && x >= 1 && x <= s->W - 2 && y >= 1 &&
              y <= s->H - 2 && d >= 0 && d < 4 && tm >= 0 && tm <= 255;
    uint8_t iv[32] = {};
    for (int k = 0; k < s->K; ++k) {
      const int c = inventory ? inventory[i * s->K + k] : 0;
      if (c < 0 || c > 255) ok = false;
      iv[k] = (uint8_t)(c & 0xff);
    }
    if (!ok) { latch(s, CRAFT_EINVAL, i); continue; }
    Agent a{x, y, d, 0, tm, sc, tk};
    s->state[slot] = pack_state(a);
    s->init[slot] = (uint32_t)x0 | ((uint32_t)y0 << 8) | ((uint32_t)d0 << 16);
    std::memcpy(s->inv.data() + 32 * slot, iv, 32);
    std::memset(s->mask.data() + 8 * slot, 0, 32);
  }
  return CRAFT_OK;
}

// Test hook, not part of include/craft.h: craft_host::hint_tables for a configuration, exactly as
// the HIP library builds them at craft_sim_create for the teacher-labelled rollout's walk
// (tests/test_hint_tables.py checks every leaf against the reference's find_incomplete_subtask).
int craft_debug_hint_tables(const craft_config_t* cfg, uint32_t* desc, uint8_t* leaf, int32_t cap,
                            int32_t* n_leaf) {
  if (!cfg || !desc || cap < 0) return CRAFT_EINVAL;
  std::string msg;
  if (craft_host::validate_config(cfg, msg) != CRAFT_OK) return CRAFT_EINVAL;
  std::vector<uint16_t> tab(CRAFT_MAX_TASKS, 0);
  std::vector<int32_t> sub(CRAFT_MAX_TASKS * CRAFT_MAX_SUBTASKS, 0);
  craft_host::task_tables(*cfg, tab.data(), sub.data());
  std::vector<uint8_t> lv;
  craft_host::hint_tables(*cfg, tab.data(), sub.data(), desc, lv);
  if (n_leaf) *n_leaf = (int32_t)lv.size();
  if (leaf && !lv.empty()) std::memcpy(leaf, lv.data(), std::min<size_t>((size_t)cap, lv.size()));
  return CRAFT_OK;
}

}  // extern "C"
