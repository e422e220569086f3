// craft_sim.hip — MI355X (gfx950) kernels and C ABI of the batched CraftWorld.
//
// Data layout in HBM (struct-of-arrays, one entry per environment slot):
//   agent  u32[N]     x | y<<8 | dir<<16 | frozen<<20 | timer<<24
//   spec   int4[N]    {scenario, x0|y0<<8|dir0<<16, task, 0}  (CraftScenario)
//   inv    uint4[N][2] 32 inventory counts, u8 (CraftState.inventory)
//   mask   uint4[N][2] 256-bit set of cells cleared since reset
//   pool   u8[P][CS]  initial grids as kind ids, x-major, CS = roundup(W*H,16)
// A slot's grid is pool[scenario] minus its mask: the reference only ever
// clears cells (grab, bridge, axe: craft.py:383-410), so the per-env grid
// never needs its own copy and a reset is a mask clear.  The pool (147 KB for
// 1024 12x12 worlds) stays L2-resident; per env-step the kernel moves ~100 B of
// state and the F*4-byte fp32 observation row, which dominates.
//
// Hot kernel (tile_kernel<WIN, MODE_TICK>): a 256-thread workgroup owns a tile
// of 64 consecutive envs.
//   phase 0  all threads stage the 64 pool grids into LDS (coalesced dwords)
//   phase 1  wave 0, one lane per env: clear masked cells, run the rollout
//            protocol + transition on the LDS grid, write the state back, and
//            build the observation as a bit image in LDS (one-hot sections)
//   phase 2  all threads stream the tile's 64*F floats to HBM as contiguous
//            16-byte stores, expanding bits (and inventory counts) to fp32
// No MFMA: this is integer/indexing work bounded by the HBM write of the
// observation (see DESIGN.md for the roofline).
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/craft.h"

namespace {

constexpr int kTileEnvs = 64;     // envs per workgroup = one wavefront in phase 1
constexpr int kThreads = 256;     // threads per workgroup
constexpr int kInvStride = 36;    // LDS bytes per inventory row (9 dwords: bank-spread)

enum Mode { MODE_TICK = 0, MODE_TRANSITION = 1, MODE_OBSERVE = 2, MODE_RESET = 3 };

struct SimView {
  const craft_config_t* cfg;  // device copy of the static tables
  const uint8_t* pool;
  uint32_t* agent;
  int4* spec;
  uint4* inv;
  uint4* mask;
  int64_t* stats_part;        // [n_tiles][4]
  int32_t* err;               // [4] {code, pad, slot lo, slot hi}
  int64_t n_envs, env_base;
  int32_t pool_count;
  int32_t W, H, K, F, C, CS, GS, maxT, INV0, NB;
  int32_t lds_bits, lds_inv, lds_scen;   // dynamic-LDS offsets
  uint64_t kc_lo, kc_hi;                  // kind class, 4 bits per kind id
  uint32_t magicQ;                        // floor(2^32 / (F/4)) + 1
};

struct TileArgs {
  const int32_t* src;
  const int32_t* dst;
  const int32_t* actions;
  const int32_t* tasks;
  const int32_t* r_scen;   // MODE_RESET inputs
  const int32_t* r_x;
  const int32_t* r_y;
  const int32_t* r_dir;
  const int32_t* r_task;
  uint64_t seed;
  int64_t tick;
  int64_t n;
  uint32_t flags;
  float* obs;
  float* reward;
  uint8_t* done;
  int8_t* sat;
};

__device__ __forceinline__ void latch_error(int32_t* err, int code, int64_t slot) {
  if (atomicCAS(err, 0, code) == 0) {
    err[2] = (int32_t)(slot & 0xffffffff);
    err[3] = (int32_t)(slot >> 32);
  }
}

__device__ __forceinline__ int kind_class(const SimView& v, int k) {
  return (int)(((k < 16) ? (v.kc_lo >> (4 * k)) : (v.kc_hi >> (4 * (k - 16)))) & 0xf);
}

__device__ __forceinline__ uint32_t pack_agent(int x, int y, int dir, int frozen, int timer) {
  return (uint32_t)x | ((uint32_t)y << 8) | ((uint32_t)dir << 16) | ((uint32_t)frozen << 20) |
         ((uint32_t)timer << 24);
}

__device__ __forceinline__ int dir_dx(int d) { return d == CRAFT_LEFT ? -1 : (d == CRAFT_RIGHT ? 1 : 0); }
__device__ __forceinline__ int dir_dy(int d) { return d == CRAFT_DOWN ? -1 : (d == CRAFT_UP ? 1 : 0); }

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Sets mask bit c in a register-resident 8-word mask (static indices only).
__device__ __forceinline__ void mask_set(uint32_t (&m)[8], int c) {
  const int w = c >> 5;
  const uint32_t b = 1u << (c & 31);
#pragma unroll
  for (int i = 0; i < 8; ++i) m[i] |= (i == w) ? b : 0u;
}

// CraftState.step (craft.py:332-424) on an LDS-resident grid row `g` and
// inventory row `iv`.  Returns true when inventory or grid changed.
__device__ __forceinline__ void transition(const SimView& v, uint8_t* g, uint8_t* iv, int& x,
                                           int& y, int& dir, uint32_t (&m)[8], int a,
                                           bool& inv_changed, bool& mask_changed) {
  const int H = v.H;
  int dx = 0, dy = 0, ndir = dir;
  if (a < CRAFT_USE) {                               // moves always turn (craft.py:341-352)
    dx = dir_dx(a);
    dy = dir_dy(a);
    ndir = a;
  } else if (a == CRAFT_USE) {                       // craft.py:356-412
    const bool ok = (dir == CRAFT_LEFT && x > 0) || (dir == CRAFT_DOWN && y > 0) ||
                    (dir == CRAFT_RIGHT && x < v.W - 1) || (dir == CRAFT_UP && y < H - 1);
    if (ok) {
      const int c = (x + dir_dx(dir)) * H + (y + dir_dy(dir));
      const int thing = g[c];
      if (thing != 0) {
        const int cls = kind_class(v, thing);
        if (cls == CRAFT_KIND_GRABBABLE) {           // craft.py:383-386
          iv[thing] = (uint8_t)(iv[thing] + 1);
          g[c] = 0;
          mask_set(m, c);
          inv_changed = mask_changed = true;
        } else if (cls == CRAFT_KIND_WORKSHOP) {     // recipes in dict order, craft.py:388-401
          const craft_recipe_t* rc = v.cfg->recipe;
          for (int r = 0; r < v.cfg->n_recipes; ++r) {
            if (rc[r].workshop != thing) continue;
            bool have = true;
            for (int i = 0; i < rc[r].n_inputs; ++i)
              have = have && iv[rc[r].input_kind[i]] >= rc[r].input_count[i];
            if (!have) continue;
            iv[rc[r].output] = (uint8_t)(iv[rc[r].output] + rc[r].yield);
            for (int i = 0; i < rc[r].n_inputs; ++i)
              iv[rc[r].input_kind[i]] = (uint8_t)(iv[rc[r].input_kind[i]] - rc[r].input_count[i]);
            inv_changed = true;
          }
        } else if (cls == CRAFT_KIND_WATER) {        // craft.py:403-406
          const int b = v.cfg->bridge_kind;
          if (iv[b] > 0) {
            g[c] = 0;
            mask_set(m, c);
            iv[b] = (uint8_t)(iv[b] - 1);
            inv_changed = mask_changed = true;
          }
        } else if (cls == CRAFT_KIND_STONE) {        // craft.py:408-410 (axe kept)
          if (iv[v.cfg->axe_kind] > 0) {
            g[c] = 0;
            mask_set(m, c);
            mask_changed = true;
          }
        }
      }
    }
  }
  // Collision against the pre-action grid (craft.py:418-421); USE/STOP do not move.
  if (dx | dy) {
    const int nx = x + dx, ny = y + dy;
    if (g[nx * H + ny] == 0) { x = nx; y = ny; }
  }
  dir = ndir;
}

// CraftState.satisfies (craft.py:285-294): 1/0, -1 for None.
__device__ __forceinline__ int satisfies(const SimView& v, const uint8_t* g, const uint8_t* iv,
                                         int x, int y, int dir, int task) {
  const craft_task_t& t = v.cfg->task[task];
  if (t.goal == CRAFT_GOAL_GET || t.goal == CRAFT_GOAL_MAKE) return iv[t.arg_kind] > 0;
  if (t.goal == CRAFT_GOAL_GO) return g[(x + dir_dx(dir)) * v.H + (y + dir_dy(dir))] == t.arg_kind;
  return -1;
}

__device__ __forceinline__ void set_bits(uint32_t* col, int f, uint32_t bits) {
  // col = s_bits + e, word w lives at col[w * kTileEnvs]; bits may straddle two words
  const int w = f >> 5, o = f & 31;
  col[w * kTileEnvs] |= bits << o;
  if (o) {
    const uint32_t hi = bits >> (32 - o);
    if (hi) col[(w + 1) * kTileEnvs] |= hi;
  }
}

// features() (craft.py:296-330) of the state in LDS, as a bit image: local
// window one-hot, block-max-pooled big window one-hot, dir one-hot.  The
// inventory section's bits stay 0; phase 2 substitutes the counts.
template <int WIN>
__device__ __forceinline__ void build_obs_bits(const SimView& v, const uint8_t* g, uint32_t* col,
                                               int x, int y, int dir) {
  const int W = v.W, H = v.H, K = v.K;
  for (int w = 0; w < v.NB; ++w) col[w * kTileEnvs] = 0u;
  constexpr int hw = WIN / 2;
#pragma unroll
  for (int i = 0; i < WIN; ++i) {
    const int cx = x - hw + i;
    if (cx < 0 || cx >= W) continue;
#pragma unroll
    for (int j = 0; j < WIN; ++j) {
      const int cy = y - hw + j;
      if (cy < 0 || cy >= H) continue;
      const int c = g[cx * H + cy];
      if (c) set_bits(col, (i * WIN + j) * K + c, 1u);
    }
  }
  constexpr int bh = (WIN * WIN) / 2;
  const int L = WIN * WIN * K;
#pragma unroll
  for (int bi = 0; bi < WIN; ++bi) {
    const int x0 = x - bh + bi * WIN;
    const int xa = max(x0, 0), xb = min(x0 + WIN, W);
#pragma unroll
    for (int bj = 0; bj < WIN; ++bj) {
      const int y0 = y - bh + bj * WIN;
      const int ya = max(y0, 0), yb = min(y0 + WIN, H);
      uint32_t m = 0;
      for (int cx = xa; cx < xb; ++cx)
        for (int cy = ya; cy < yb; ++cy) m |= 1u << g[cx * H + cy];
      m &= ~1u;   // kind 0 = empty cell, never a feature
      if (m) set_bits(col, L + (bi * WIN + bj) * K, m);
    }
  }
  set_bits(col, 2 * L + K + dir, 1u);
}

template <int WIN, int MODE>
__global__ __launch_bounds__(kThreads) void tile_kernel(SimView v, TileArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* s_grid = smem;
  uint32_t* s_bits = reinterpret_cast<uint32_t*>(smem + v.lds_bits);
  uint8_t* s_inv = smem + v.lds_inv;
  int32_t* s_scen = reinterpret_cast<int32_t*>(smem + v.lds_scen);

  const int tid = threadIdx.x;
  const int64_t env0 = (int64_t)blockIdx.x * kTileEnvs;
  const int nE = (int)min((int64_t)kTileEnvs, a.n - env0);

  // ---- phase 0: scenario ids, then the tile's pool grids into LDS --------------
  int64_t slot = 0, dslot = 0;
  int4 sp = make_int4(0, 0, 0, 0);
  bool live = tid < nE;
  if (live) {
    const int64_t i = env0 + tid;
    if (MODE == MODE_TICK || MODE == MODE_RESET) {
      slot = i;
    } else {
      slot = a.src ? (int64_t)a.src[i] : i;
    }
    dslot = (MODE == MODE_TRANSITION && a.dst) ? (int64_t)a.dst[i] : slot;
    if (slot < 0 || slot >= v.n_envs || dslot < 0 || dslot >= v.n_envs) {
      latch_error(v.err, CRAFT_ERANGE, i);
      live = false;
    }
  }
  if (live) {
    if (MODE == MODE_RESET) {
      const int64_t i = env0 + tid;
      int sc = a.r_scen[i], x0 = a.r_x[i], y0 = a.r_y[i], d0 = a.r_dir[i], tk = a.r_task[i];
      if (sc < 0 || sc >= v.pool_count || x0 < 1 || x0 > v.W - 2 || y0 < 1 || y0 > v.H - 2 ||
          d0 < 0 || d0 > 3 || tk < 0 || tk >= v.cfg->n_tasks) {
        latch_error(v.err, CRAFT_EINVAL, i);
        sc = 0; x0 = 1; y0 = 1; d0 = 0; tk = 0;
      }
      sp = make_int4(sc, x0 | (y0 << 8) | (d0 << 16), tk, 0);
    } else {
      sp = v.spec[slot];
    }
  }
  if (tid < kTileEnvs) s_scen[tid] = live ? sp.x : 0;
  __syncthreads();
  {
    const int nd = v.CS >> 2;   // dwords per pool grid
    const int total = nE * nd;
    const uint32_t* pool32 = reinterpret_cast<const uint32_t*>(v.pool);
    for (int i = tid; i < total; i += kThreads) {
      const int e = i / nd, w = i - e * nd;
      *reinterpret_cast<uint32_t*>(s_grid + e * v.GS + 4 * w) = pool32[(size_t)s_scen[e] * nd + w];
    }
  }
  __syncthreads();

  // ---- phase 1: one lane per env ----------------------------------------------
  if (tid < kTileEnvs) {
    uint8_t* g = s_grid + tid * v.GS;
    uint8_t* iv = s_inv + tid * kInvStride;
    int x = 0, y = 0, dir = 0, frozen = 0, timer = 0;
    uint32_t m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    bool inv_changed = false, mask_changed = false, agent_changed = false;
    int d = 0, succ = -1, counted = 0;
    if (live) {
      if (MODE == MODE_RESET) {
        for (int w = 0; w < 8; ++w) reinterpret_cast<uint32_t*>(iv)[w] = 0u;
        x = sp.y & 0xff; y = (sp.y >> 8) & 0xff; dir = (sp.y >> 16) & 0xf;
        timer = v.maxT;
        inv_changed = mask_changed = agent_changed = true;
      } else {
        const uint32_t ag = v.agent[slot];
        x = ag & 0xff; y = (ag >> 8) & 0xff; dir = (ag >> 16) & 0xf; frozen = (ag >> 20) & 1;
        timer = ag >> 24;
        if (x < 1 || x > v.W - 2 || y < 1 || y > v.H - 2 || dir > 3) {
          // never initialised by craft_reset / craft_set_state
          latch_error(v.err, CRAFT_EINVAL, slot);
          live = false;
        }
      }
    }
    if (!live && a.obs) {
      for (int w = 0; w < v.NB; ++w) s_bits[w * kTileEnvs + tid] = 0u;
      for (int w = 0; w < 8; ++w) reinterpret_cast<uint32_t*>(iv)[w] = 0u;
    }
    if (live) {
      if (MODE != MODE_RESET) {
        const uint4 i0 = v.inv[2 * slot], i1 = v.inv[2 * slot + 1];
        uint32_t* ivw = reinterpret_cast<uint32_t*>(iv);
        ivw[0] = i0.x; ivw[1] = i0.y; ivw[2] = i0.z; ivw[3] = i0.w;
        ivw[4] = i1.x; ivw[5] = i1.y; ivw[6] = i1.z; ivw[7] = i1.w;
        const uint4 m0 = v.mask[2 * slot], m1 = v.mask[2 * slot + 1];
        m[0] = m0.x; m[1] = m0.y; m[2] = m0.z; m[3] = m0.w;
        m[4] = m1.x; m[5] = m1.y; m[6] = m1.z; m[7] = m1.w;
#pragma unroll
        for (int w = 0; w < 8; ++w) {            // cells cleared since reset
          uint32_t mm = m[w];
          while (mm) {
            const int b = __ffs(mm) - 1;
            g[w * 32 + b] = 0;
            mm &= mm - 1;
          }
        }
      }

      if (MODE == MODE_TICK) {
        // per-env body of ImitationTrainer.do_rollout, trainers/imitation.py:59-73
        const int64_t gid = v.env_base + slot;
        int act;
        if (a.actions) {
          act = a.actions[slot];
        } else {
          const uint64_t h = splitmix64(a.seed ^ ((uint64_t)gid << 20) ^ (uint64_t)a.tick);
          act = (int)((uint32_t)(h >> 32) % 6u);
        }
        if (frozen) {
          d = 1;
          succ = satisfies(v, g, iv, x, y, dir, sp.z);
        } else {
          counted = 1;
          agent_changed = true;
          timer -= 1;
          d = (act == CRAFT_STOP) || timer <= 0;
          if (d) {
            succ = satisfies(v, g, iv, x, y, dir, sp.z);
            if (a.flags & CRAFT_STEP_AUTORESET) {     // CraftScenario.init, craft.py:268-273
              x = sp.y & 0xff; y = (sp.y >> 8) & 0xff; dir = (sp.y >> 16) & 0xf;
              timer = v.maxT;
              for (int w = 0; w < 8; ++w) { reinterpret_cast<uint32_t*>(iv)[w] = 0u; m[w] = 0u; }
              const uint32_t* src = reinterpret_cast<const uint32_t*>(v.pool + (size_t)sp.x * v.CS);
              for (int w = 0; w < (v.CS >> 2); ++w) reinterpret_cast<uint32_t*>(g)[w] = src[w];
              inv_changed = mask_changed = true;
            } else {
              frozen = 1;
              timer = max(timer, 0);
            }
          } else if (act < 0 || act >= CRAFT_N_ACTIONS) {
            latch_error(v.err, CRAFT_EBADACTION, slot);
          } else {
            transition(v, g, iv, x, y, dir, m, act, inv_changed, mask_changed);
          }
        }
      } else if (MODE == MODE_TRANSITION) {
        const int act = a.actions[env0 + tid];
        agent_changed = true;
        if (act >= CRAFT_N_ACTIONS) {
          latch_error(v.err, CRAFT_EBADACTION, slot);
        } else if (act >= 0) {
          transition(v, g, iv, x, y, dir, m, act, inv_changed, mask_changed);
        }
        if (dslot != slot) inv_changed = mask_changed = true;   // copy-on-step
      } else if (MODE == MODE_OBSERVE) {
        if (a.sat) {
          const int tk = a.tasks ? a.tasks[env0 + tid] : sp.z;
          if (tk < 0 || tk >= v.cfg->n_tasks) {
            latch_error(v.err, CRAFT_ERANGE, env0 + tid);
            a.sat[env0 + tid] = -1;
          } else {
            a.sat[env0 + tid] = (int8_t)satisfies(v, g, iv, x, y, dir, tk);
          }
        }
      }

      // ---- write back ----
      if (agent_changed) v.agent[dslot] = pack_agent(x, y, dir, frozen, timer);
      if (MODE == MODE_RESET || (MODE == MODE_TRANSITION && dslot != slot)) v.spec[dslot] = sp;
      if (inv_changed) {
        const uint32_t* ivw = reinterpret_cast<const uint32_t*>(iv);
        v.inv[2 * dslot] = make_uint4(ivw[0], ivw[1], ivw[2], ivw[3]);
        v.inv[2 * dslot + 1] = make_uint4(ivw[4], ivw[5], ivw[6], ivw[7]);
      }
      if (mask_changed) {
        v.mask[2 * dslot] = make_uint4(m[0], m[1], m[2], m[3]);
        v.mask[2 * dslot + 1] = make_uint4(m[4], m[5], m[6], m[7]);
      }
      if (MODE == MODE_TICK) {
        const int64_t i = env0 + tid;
        if (a.done) a.done[i] = (uint8_t)d;
        if (a.sat) a.sat[i] = (int8_t)succ;
        if (a.reward) a.reward[i] = (d && succ == 1) ? 1.0f : 0.0f;
      }
      if (a.obs) build_obs_bits<WIN>(v, g, s_bits + tid, x, y, dir);
    }
    if (MODE == MODE_TICK) {
      // episode statistics: the workgroup owns its partial-sum row (no atomics)
      const uint64_t bs = __ballot(live && d && succ == 1 && counted);
      const uint64_t be = __ballot(live && d && counted);
      const uint64_t bt = __ballot(live && counted);
      if (tid == 0) {
        int64_t* row = v.stats_part + 4 * (int64_t)blockIdx.x;
        row[0] += __popcll(bs);
        row[1] += __popcll(be);
        row[2] += __popcll(bt);
      }
    }
  }
  if (!a.obs) return;
  __syncthreads();

  // ---- phase 2: stream the tile's observation rows ------------------------------
  const int F = v.F, K = v.K, INV0 = v.INV0;
  float* tile = a.obs + env0 * (int64_t)F;
  if ((F & 3) == 0) {
    const int Q = F >> 2;
    const int nslots = nE * Q;
    float4* out4 = reinterpret_cast<float4*>(tile);
    for (int s = tid; s < nslots; s += kThreads) {
      const int e = (int)__umulhi((uint32_t)s, v.magicQ);
      const int f = (s - e * Q) << 2;
      const uint32_t w = s_bits[(f >> 5) * kTileEnvs + e] >> (f & 31);
      float4 o = make_float4((float)(w & 1u), (float)((w >> 1) & 1u), (float)((w >> 2) & 1u),
                             (float)((w >> 3) & 1u));
      if (f + 3 >= INV0 && f < INV0 + K) {
        const uint8_t* iv = s_inv + e * kInvStride;
        if (f + 0 >= INV0 && f + 0 < INV0 + K) o.x = (float)iv[f + 0 - INV0];
        if (f + 1 >= INV0 && f + 1 < INV0 + K) o.y = (float)iv[f + 1 - INV0];
        if (f + 2 >= INV0 && f + 2 < INV0 + K) o.z = (float)iv[f + 2 - INV0];
        if (f + 3 >= INV0 && f + 3 < INV0 + K) o.w = (float)iv[f + 3 - INV0];
      }
      out4[s] = o;
    }
  } else {
    const int total = nE * F;
    for (int s = tid; s < total; s += kThreads) {
      const int e = s / F, f = s - e * F;
      float val;
      if (f >= INV0 && f < INV0 + K) val = (float)s_inv[e * kInvStride + f - INV0];
      else val = (float)((s_bits[(f >> 5) * kTileEnvs + e] >> (f & 31)) & 1u);
      tile[s] = val;
    }
  }
}

// ---- teacher: bitset BFS ---------------------------------------------------------
template <int NW>
struct Bits {
  uint64_t w[NW];
};

template <int NW>
__device__ __forceinline__ Bits<NW> bzero() {
  Bits<NW> r;
#pragma unroll
  for (int i = 0; i < NW; ++i) r.w[i] = 0;
  return r;
}
template <int NW>
__device__ __forceinline__ Bits<NW> band(const Bits<NW>& a, const Bits<NW>& b) {
  Bits<NW> r;
#pragma unroll
  for (int i = 0; i < NW; ++i) r.w[i] = a.w[i] & b.w[i];
  return r;
}
template <int NW>
__device__ __forceinline__ Bits<NW> bor(const Bits<NW>& a, const Bits<NW>& b) {
  Bits<NW> r;
#pragma unroll
  for (int i = 0; i < NW; ++i) r.w[i] = a.w[i] | b.w[i];
  return r;
}
template <int NW>
__device__ __forceinline__ Bits<NW> bandn(const Bits<NW>& a, const Bits<NW>& b) {
  Bits<NW> r;
#pragma unroll
  for (int i = 0; i < NW; ++i) r.w[i] = a.w[i] & ~b.w[i];
  return r;
}
template <int NW>
__device__ __forceinline__ bool bany(const Bits<NW>& a) {
  uint64_t x = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) x |= a.w[i];
  return x != 0;
}
template <int NW>
__device__ __forceinline__ bool btest(const Bits<NW>& a, int p) {
  uint64_t x = 0;
#pragma unroll
  for (int i = 0; i < NW; ++i) x |= (i == (p >> 6)) ? a.w[i] : 0ull;
  return (x >> (p & 63)) & 1ull;
}
template <int NW>
__device__ __forceinline__ Bits<NW> bbit(int p) {
  Bits<NW> r;
#pragma unroll
  for (int i = 0; i < NW; ++i) r.w[i] = (i == (p >> 6)) ? (1ull << (p & 63)) : 0ull;
  return r;
}
template <int NW>
__device__ __forceinline__ int blowest(const Bits<NW>& a) {   // INT_MAX if empty
  int r = INT_MAX;
#pragma unroll
  for (int i = NW - 1; i >= 0; --i)
    if (a.w[i]) r = i * 64 + __ffsll((unsigned long long)a.w[i]) - 1;
  return r;
}
template <int NW>
__device__ __forceinline__ int bhighest(const Bits<NW>& a) {  // -1 if empty
  int r = -1;
#pragma unroll
  for (int i = 0; i < NW; ++i)
    if (a.w[i]) r = i * 64 + 63 - __clzll((long long)a.w[i]);
  return r;
}
// p -> p + d for every member (|d| < 64); members shifted past either end drop out.
template <int NW>
__device__ __forceinline__ Bits<NW> bshift(const Bits<NW>& a, int d) {
  Bits<NW> r;
  if (d > 0) {
#pragma unroll
    for (int i = 0; i < NW; ++i) r.w[i] = (a.w[i] << d) | (i > 0 ? a.w[i - 1] >> (64 - d) : 0ull);
  } else {
    const int s = -d;
#pragma unroll
    for (int i = 0; i < NW; ++i)
      r.w[i] = (a.w[i] >> s) | (i + 1 < NW ? a.w[i + 1] << (64 - s) : 0ull);
  }
  return r;
}

// find_closest_resources (teachers/base.py:27-34) over shortest_path
// (teachers/base.py:36-87) as ONE level-synchronous BFS over (pos, dir) states
// held as per-direction position bitsets.  FIFO order within a level is
// sorted by the path's first action (induction: level 1 is enqueued in action
// order DOWN, UP, LEFT, RIGHT, and children keep their first-dequeued parent's
// label), so tracking the level's states per first action (a "label")
// reproduces exactly which state the reference dequeues first:
//   a target's path length = the first level at which a state faces it,
//   its first action = the smallest label among that level's facing states,
//   the chosen target = the first in np.nonzero (x-major) order with the
//   minimal length (strict `<`, base.py:31).
// Returns false where the reference raises (len(None) on an unreachable
// target after a reachable one, base.py:31).
template <int NW>
__device__ bool bfs_closest(const Bits<NW>& occ, const Bits<NW>& tgt, const Bits<NW>& valid,
                            int H, int p0, int d0, int& first_action, int& path_len) {
  const int dl[4] = {-1, 1, -H, H};   // DOWN, UP, LEFT, RIGHT in x-major cell index
  const Bits<NW> fr = bandn(valid, occ);
  Bits<NW> V[4], cur[4], fc[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) V[a] = bzero<NW>();
#pragma unroll
  for (int a = 0; a < 4; ++a) V[a] = (a == d0) ? bbit<NW>(p0) : V[a];
  Bits<NW> claimed = bzero<NW>();
  bool found = false;
  first_action = -1;
  path_len = -1;
  {
    const int f0 = p0 + dl[d0];            // start state already faces a target: []
    if (f0 >= 0 && btest(tgt, f0)) {
      found = true;
      path_len = 0;
      claimed = bbit<NW>(f0);
    }
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int q0 = p0 + dl[a];
    const int q = btest(fr, q0) ? q0 : p0;
    if (!btest(V[a], q)) {
      V[a] = bor(V[a], bbit<NW>(q));
      cur[a] = bbit<NW>(q);
      fc[a] = band(bshift(cur[a], dl[a]), valid);
    } else {
      cur[a] = bzero<NW>();
      fc[a] = bzero<NW>();
    }
  }
  Bits<NW> blk[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) blk[a] = bshift(occ, -dl[a]);   // blk[a][p] = occ[p + dl[a]]
  int depth = 1;
  while (bany(bor(bor(cur[0], cur[1]), bor(cur[2], cur[3])))) {
    int bp = INT_MAX, bl = -1;
#pragma unroll
    for (int lab = 0; lab < 4; ++lab) {
      const Bits<NW> hit = bandn(band(fc[lab], tgt), claimed);
      if (bany(hit)) {
        claimed = bor(claimed, hit);
        const int p = blowest(hit);
        if (p < bp) { bp = p; bl = lab; }
      }
    }
    if (!found && bl >= 0) {
      found = true;
      path_len = depth;
      first_action = bl;
    }
    if (!bany(bandn(tgt, claimed))) break;
    Bits<NW> nc[4], nf[4];
#pragma unroll
    for (int lab = 0; lab < 4; ++lab) {
      nc[lab] = bzero<NW>();
      nf[lab] = bzero<NW>();
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const Bits<NW> moved = bor(band(bshift(cur[lab], dl[a]), fr), band(cur[lab], blk[a]));
        const Bits<NW> fresh = bandn(moved, V[a]);
        V[a] = bor(V[a], fresh);
        nc[lab] = bor(nc[lab], fresh);
        nf[lab] = bor(nf[lab], band(bshift(fresh, dl[a]), valid));
      }
    }
#pragma unroll
    for (int lab = 0; lab < 4; ++lab) { cur[lab] = nc[lab]; fc[lab] = nf[lab]; }
    ++depth;
  }
  if (found) {
    const Bits<NW> unreached = bandn(tgt, claimed);
    if (bany(unreached) && blowest(claimed) < bhighest(unreached)) return false;
  }
  return true;
}

struct TeachArgs {
  const int32_t* slots;
  const int32_t* tasks;
  int64_t n;
  int32_t* act_out;
  int32_t* len_out;
};

template <int NW>
__device__ __forceinline__ int grid_kind(const SimView& v, int scen, const uint32_t (&m)[8], int c) {
  const int k = v.pool[(size_t)scen * v.CS + c];
  uint32_t mw = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) mw |= (i == (c >> 5)) ? m[i] : 0u;
  return ((mw >> (c & 31)) & 1u) ? 0 : k;
}

// DemonstrationTeacher.__call__ (teachers/demonstration.py:9-30), one lane per slot.
template <int NW>
__global__ __launch_bounds__(256) void teacher_kernel(SimView v, TeachArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  const int64_t slot = a.slots ? (int64_t)a.slots[i] : i;
  if (slot < 0 || slot >= v.n_envs) {
    latch_error(v.err, CRAFT_ERANGE, i);
    a.act_out[i] = CRAFT_STOP;
    if (a.len_out) a.len_out[i] = -1;
    return;
  }
  const int4 sp = v.spec[slot];
  const int task = a.tasks ? a.tasks[i] : sp.z;
  if (task < 0 || task >= v.cfg->n_tasks) {
    latch_error(v.err, CRAFT_ERANGE, i);
    a.act_out[i] = CRAFT_STOP;
    if (a.len_out) a.len_out[i] = -1;
    return;
  }
  const uint32_t ag = v.agent[slot];
  const int x = ag & 0xff, y = (ag >> 8) & 0xff, dir = (ag >> 16) & 0xf;
  if (x < 1 || x > v.W - 2 || y < 1 || y > v.H - 2 || dir > 3) {
    latch_error(v.err, CRAFT_EINVAL, slot);
    a.act_out[i] = -2;
    if (a.len_out) a.len_out[i] = -2;
    return;
  }
  uint32_t m[8];
  {
    const uint4 m0 = v.mask[2 * slot], m1 = v.mask[2 * slot + 1];
    m[0] = m0.x; m[1] = m0.y; m[2] = m0.z; m[3] = m0.w;
    m[4] = m1.x; m[5] = m1.y; m[6] = m1.z; m[7] = m1.w;
  }
  const uint8_t* iv = reinterpret_cast<const uint8_t*>(v.inv + 2 * slot);
  const int H = v.H, C = v.C;
  const int facing = grid_kind<NW>(v, sp.x, m, (x + dir_dx(dir)) * H + (y + dir_dy(dir)));

  auto sat = [&](int t) -> int {
    const craft_task_t& tt = v.cfg->task[t];
    if (tt.goal == CRAFT_GOAL_GET || tt.goal == CRAFT_GOAL_MAKE) return iv[tt.arg_kind] > 0;
    if (tt.goal == CRAFT_GOAL_GO) return facing == tt.arg_kind;
    return -1;
  };

  Bits<NW> valid = bzero<NW>();
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const int lo = w * 64;
    const int nb = min(64, max(0, C - lo));
    valid.w[w] = nb >= 64 ? ~0ull : ((1ull << nb) - 1ull);
  }
  auto closest = [&](int kind, int& fa, int& len) -> bool {
    Bits<NW> occ = bzero<NW>(), tgt = bzero<NW>();
    for (int c = 0; c < C; ++c) {
      const int k = grid_kind<NW>(v, sp.x, m, c);
      if (k) {
#pragma unroll
        for (int w = 0; w < NW; ++w) {
          const uint64_t b = (w == (c >> 6)) ? (1ull << (c & 63)) : 0ull;
          occ.w[w] |= b;
          if (k == kind) tgt.w[w] |= b;
        }
      }
    }
    return bfs_closest<NW>(occ, tgt, valid, H, x * H + y, dir, fa, len);
  };

  int action = CRAFT_STOP;
  int err = 0;
  // find_incomplete_subtask, teachers/base.py:10-25
  int node = task;
  if (sat(node) != 1) {
    for (int guard = 0; guard < CRAFT_MAX_TASKS; ++guard) {
      const craft_task_t& t = v.cfg->task[node];
      if (t.n_subtasks == 0) break;
      int chosen = t.subtask[t.n_subtasks - 1];
      bool last = true;
      for (int s = 0; s + 1 < t.n_subtasks; ++s)
        if (sat(t.subtask[s]) != 1) { chosen = t.subtask[s]; last = false; break; }
      if (last && sat(chosen) == 1) { err = CRAFT_ETEACHER; break; }   // base.py:24 assert
      node = chosen;
    }
    if (!err) {
      const craft_task_t& leaf = v.cfg->task[node];
      if (leaf.goal == CRAFT_GOAL_USE) {
        action = CRAFT_USE;
      } else if (leaf.goal == CRAFT_GOAL_GO) {
        int fa = -1, len = -1;
        if (!closest(leaf.arg_kind, fa, len)) err = CRAFT_ETEACHER;
        else if (len < 0) action = CRAFT_STOP;                           // demonstration.py:25-26
        else if (len == 0) err = CRAFT_ETEACHER;                         // [][0]
        else action = fa;
      } else {
        err = CRAFT_ETEACHER;                                            // demonstration.py:18
      }
    }
  }
  if (err) {
    latch_error(v.err, err, slot);
    action = -2;                       // where the reference raises
  }
  a.act_out[i] = action;
  if (a.len_out) {
    const craft_task_t& t = v.cfg->task[task];
    int fa = -1, len = -1;
    if (t.arg_kind > 0 && !closest(t.arg_kind, fa, len)) {
      latch_error(v.err, CRAFT_ETEACHER, slot);
      len = -2;
    }
    a.len_out[i] = len;
  }
}

// ---- state I/O, stats ------------------------------------------------------------
__global__ void get_state_kernel(SimView v, const int32_t* slots, int64_t n, int32_t* agent_out,
                                 int32_t* inv_out, uint8_t* grid_out, int32_t* spec_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t slot = slots ? (int64_t)slots[i] : i;
  if (slot < 0 || slot >= v.n_envs) { latch_error(v.err, CRAFT_ERANGE, i); return; }
  const uint32_t ag = v.agent[slot];
  const int4 sp = v.spec[slot];
  if (agent_out) {
    agent_out[4 * i + 0] = ag & 0xff;
    agent_out[4 * i + 1] = (ag >> 8) & 0xff;
    agent_out[4 * i + 2] = (ag >> 16) & 0xf;
    agent_out[4 * i + 3] = ag >> 24;
  }
  if (inv_out) {
    const uint8_t* iv = reinterpret_cast<const uint8_t*>(v.inv + 2 * slot);
    for (int k = 0; k < v.K; ++k) inv_out[i * v.K + k] = iv[k];
  }
  if (grid_out) {
    const uint32_t* m = reinterpret_cast<const uint32_t*>(v.mask + 2 * slot);
    for (int c = 0; c < v.C; ++c) {
      const int k = v.pool[(size_t)sp.x * v.CS + c];
      grid_out[i * v.C + c] = ((m[c >> 5] >> (c & 31)) & 1u) ? 0 : (uint8_t)k;
    }
  }
  if (spec_out) {
    spec_out[5 * i + 0] = sp.x;
    spec_out[5 * i + 1] = sp.y & 0xff;
    spec_out[5 * i + 2] = (sp.y >> 8) & 0xff;
    spec_out[5 * i + 3] = (sp.y >> 16) & 0xf;
    spec_out[5 * i + 4] = sp.z;
  }
}

__global__ void set_state_kernel(SimView v, const int32_t* slots, int64_t n, const int32_t* spec_in,
                                 const int32_t* agent_in, const int32_t* inv_in) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t slot = slots ? (int64_t)slots[i] : i;
  if (slot < 0 || slot >= v.n_envs) { latch_error(v.err, CRAFT_ERANGE, i); return; }
  const int sc = spec_in[5 * i], x0 = spec_in[5 * i + 1], y0 = spec_in[5 * i + 2],
            d0 = spec_in[5 * i + 3], tk = spec_in[5 * i + 4];
  const int x = agent_in[4 * i], y = agent_in[4 * i + 1], d = agent_in[4 * i + 2],
            tm = agent_in[4 * i + 3];
  bool ok = sc >= 0 && sc < v.pool_count && tk >= 0 && tk < v.cfg->n_tasks && x0 >= 1 &&
            x0 <= v.W - 2 && y0 >= 1 && y0 <= v.H - 2 && d0 >= 0 && d0 < 4 && x >= 1 &&
            x <= v.W - 2 && y >= 1 && y <= v.H - 2 && d >= 0 && d < 4 && tm >= 0 && tm <= 255;
  uint32_t ivw[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int k = 0; k < v.K; ++k) {
    const int c = inv_in ? inv_in[i * v.K + k] : 0;
    if (c < 0 || c > 255) ok = false;
    ivw[k >> 2] |= (uint32_t)(c & 0xff) << (8 * (k & 3));
  }
  if (!ok) { latch_error(v.err, CRAFT_EINVAL, i); return; }
  v.spec[slot] = make_int4(sc, x0 | (y0 << 8) | (d0 << 16), tk, 0);
  v.agent[slot] = pack_agent(x, y, d, 0, tm);
  v.inv[2 * slot] = make_uint4(ivw[0], ivw[1], ivw[2], ivw[3]);
  v.inv[2 * slot + 1] = make_uint4(ivw[4], ivw[5], ivw[6], ivw[7]);
  v.mask[2 * slot] = make_uint4(0, 0, 0, 0);
  v.mask[2 * slot + 1] = make_uint4(0, 0, 0, 0);
}

__global__ void stats_kernel(int64_t* part, int64_t n_rows, int64_t* out, int reset) {
  __shared__ long long acc[3][256];
  long long s0 = 0, s1 = 0, s2 = 0;
  for (int64_t r = threadIdx.x; r < n_rows; r += blockDim.x) {
    s0 += part[4 * r]; s1 += part[4 * r + 1]; s2 += part[4 * r + 2];
    if (reset) { part[4 * r] = 0; part[4 * r + 1] = 0; part[4 * r + 2] = 0; }
  }
  acc[0][threadIdx.x] = s0; acc[1][threadIdx.x] = s1; acc[2][threadIdx.x] = s2;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
      for (int j = 0; j < 3; ++j) acc[j][threadIdx.x] += acc[j][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) { out[0] = acc[0][0]; out[1] = acc[1][0]; out[2] = acc[2][0]; }
}

}  // namespace

// ===================================== host side =====================================

struct craft_sim {
  int device = 0;
  craft_config_t cfg{};
  craft_config_t* d_cfg = nullptr;
  int64_t n_envs = 0, env_base = 0, n_tiles = 0;
  int32_t pool_capacity = 0, pool_count = 0;
  uint8_t* d_pool = nullptr;
  uint32_t* d_agent = nullptr;
  int4* d_spec = nullptr;
  uint4* d_inv = nullptr;
  uint4* d_mask = nullptr;
  int64_t* d_stats = nullptr;
  int32_t* d_err = nullptr;
  SimView view{};
  size_t lds_bytes = 0;
  std::string last_error;
};

namespace {

int fail(craft_sim* sim, int code, const std::string& msg) {
  if (sim) sim->last_error = msg;
  return code;
}

int hip_fail(craft_sim* sim, hipError_t e, const char* what) {
  return fail(sim, CRAFT_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(sim, expr)                                   \
  do {                                                       \
    hipError_t _e = (expr);                                  \
    if (_e != hipSuccess) return hip_fail((sim), _e, #expr); \
  } while (0)

int validate_config(const craft_config_t* c, std::string& msg) {
  if (c->abi_version != CRAFT_ABI_VERSION) { msg = "abi_version mismatch"; return CRAFT_EINVAL; }
  if (c->width < 3 || c->height < 3 || c->width > CRAFT_MAX_DIM || c->height > CRAFT_MAX_DIM ||
      c->width * c->height > CRAFT_MAX_CELLS) { msg = "WIDTH/HEIGHT out of range (3..16)"; return CRAFT_EINVAL; }
  if (c->window_width != c->window_height ||
      (c->window_width != 3 && c->window_width != 5 && c->window_width != 7)) {
    msg = "WINDOW_WIDTH == WINDOW_HEIGHT in {3,5,7} required"; return CRAFT_EINVAL;
  }
  if (c->n_kinds < 2 || c->n_kinds > CRAFT_MAX_KINDS) { msg = "n_kinds out of range"; return CRAFT_EINVAL; }
  const int ww = c->window_width;
  if (c->n_features != 2 * ww * ww * c->n_kinds + c->n_kinds + 5) {
    msg = "n_features != 2*ww*wh*n_kinds + n_kinds + 5 (craft.py:69-75)"; return CRAFT_EINVAL;
  }
  if (c->max_timesteps < 1 || c->max_timesteps > 255) { msg = "max_timesteps must be 1..255"; return CRAFT_EINVAL; }
  if (c->bridge_kind <= 0 || c->bridge_kind >= c->n_kinds || c->axe_kind <= 0 || c->axe_kind >= c->n_kinds) {
    msg = "bridge/axe kind out of range"; return CRAFT_EINVAL;
  }
  for (int k = 0; k < CRAFT_MAX_KINDS; ++k)
    if (c->kind_class[k] > CRAFT_KIND_STONE) { msg = "bad kind_class"; return CRAFT_EINVAL; }
  if (c->n_recipes < 0 || c->n_recipes > CRAFT_MAX_RECIPES) { msg = "n_recipes out of range"; return CRAFT_EINVAL; }
  for (int r = 0; r < c->n_recipes; ++r) {
    const craft_recipe_t& rc = c->recipe[r];
    if (rc.output <= 0 || rc.output >= c->n_kinds || rc.workshop <= 0 || rc.workshop >= c->n_kinds ||
        rc.n_inputs < 1 || rc.n_inputs > CRAFT_MAX_INGREDIENTS) { msg = "bad recipe"; return CRAFT_EINVAL; }
    if (rc.yield != 1) { msg = "_yield != 1 is not supported (u8 inventory counts)"; return CRAFT_EINVAL; }
    for (int i = 0; i < rc.n_inputs; ++i)
      if (rc.input_kind[i] <= 0 || rc.input_kind[i] >= c->n_kinds || rc.input_count[i] < 1 ||
          rc.input_count[i] > 255) { msg = "bad recipe input"; return CRAFT_EINVAL; }
  }
  if (c->n_tasks < 1 || c->n_tasks > CRAFT_MAX_TASKS) { msg = "n_tasks out of range"; return CRAFT_EINVAL; }
  for (int t = 0; t < c->n_tasks; ++t) {
    const craft_task_t& tk = c->task[t];
    if (tk.goal < CRAFT_GOAL_OTHER || tk.goal > CRAFT_GOAL_USE || tk.arg_kind < 0 ||
        tk.arg_kind >= c->n_kinds || tk.n_subtasks < 0 || tk.n_subtasks > CRAFT_MAX_SUBTASKS) {
      msg = "bad task"; return CRAFT_EINVAL;
    }
    if ((tk.goal == CRAFT_GOAL_GET || tk.goal == CRAFT_GOAL_MAKE || tk.goal == CRAFT_GOAL_GO) && tk.arg_kind == 0) {
      msg = "get/make/go task without a kind argument"; return CRAFT_EINVAL;
    }
    for (int s = 0; s < tk.n_subtasks; ++s)
      if (tk.subtask[s] < 0 || tk.subtask[s] >= c->n_tasks) { msg = "bad subtask id"; return CRAFT_EINVAL; }
  }
  return CRAFT_OK;
}

template <int WIN, int MODE>
hipError_t launch_tile(craft_sim* s, const TileArgs& a, hipStream_t st) {
  const int64_t tiles = (a.n + kTileEnvs - 1) / kTileEnvs;
  if (tiles == 0) return hipSuccess;
  hipLaunchKernelGGL((tile_kernel<WIN, MODE>), dim3((unsigned)tiles), dim3(kThreads),
                     s->lds_bytes, st, s->view, a);
  return hipGetLastError();
}

template <int MODE>
hipError_t dispatch_tile(craft_sim* s, const TileArgs& a, hipStream_t st) {
  switch (s->cfg.window_width) {
    case 3: return launch_tile<3, MODE>(s, a, st);
    case 5: return launch_tile<5, MODE>(s, a, st);
    default: return launch_tile<7, MODE>(s, a, st);
  }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

}  // namespace

extern "C" {

const char* craft_strerror(int status) {
  switch (status) {
    case CRAFT_OK: return "ok";
    case CRAFT_EINVAL: return "invalid argument";
    case CRAFT_EBADACTION: return "Unexpected action";
    case CRAFT_EINVARIANT: return "impossible world configuration";
    case CRAFT_ETEACHER: return "teacher assertion";
    case CRAFT_EHIP: return "HIP runtime error";
    case CRAFT_ENOMEM: return "out of memory";
    case CRAFT_ERANGE: return "index out of range";
    default: return "unknown status";
  }
}

int craft_sim_create(const craft_config_t* cfg, int device, int64_t n_envs, int64_t env_id_base,
                     int32_t pool_capacity, craft_sim_t** out) {
  if (!cfg || !out || n_envs <= 0 || pool_capacity <= 0 || env_id_base < 0) return CRAFT_EINVAL;
  *out = nullptr;
  std::string msg;
  int rc = validate_config(cfg, msg);
  if (rc) {
    fprintf(stderr, "craft_sim_create: %s\n", msg.c_str());
    return rc;
  }
  craft_sim* s = new craft_sim();
  s->device = device;
  s->cfg = *cfg;
  s->n_envs = n_envs;
  s->env_base = env_id_base;
  s->pool_capacity = pool_capacity;
  s->n_tiles = (n_envs + kTileEnvs - 1) / kTileEnvs;
  const int W = cfg->width, H = cfg->height, K = cfg->n_kinds, F = cfg->n_features;
  const int C = W * H, CS = (C + 15) & ~15;
  const int GS = CS + 4;                  // odd dword stride: lane-private rows hit distinct banks
  const int ww = cfg->window_width;
  const int NB = (F + 31) / 32 + 1;
  auto cleanup = [&](hipError_t e, const char* what) {
    fprintf(stderr, "craft_sim_create: %s: %s\n", what, hipGetErrorString(e));
    craft_sim_destroy(s);
    return CRAFT_EHIP;
  };
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return cleanup(e, "hipSetDevice");
  if ((e = hipMalloc(&s->d_cfg, sizeof(craft_config_t))) != hipSuccess) return cleanup(e, "hipMalloc cfg");
  if ((e = hipMemcpy(s->d_cfg, cfg, sizeof(craft_config_t), hipMemcpyHostToDevice)) != hipSuccess)
    return cleanup(e, "hipMemcpy cfg");
  if ((e = hipMalloc(&s->d_pool, (size_t)pool_capacity * CS)) != hipSuccess) return cleanup(e, "hipMalloc pool");
  if ((e = hipMemset(s->d_pool, 0, (size_t)pool_capacity * CS)) != hipSuccess) return cleanup(e, "hipMemset pool");
  if ((e = hipMalloc(&s->d_agent, sizeof(uint32_t) * n_envs)) != hipSuccess) return cleanup(e, "hipMalloc agent");
  if ((e = hipMalloc(&s->d_spec, sizeof(int4) * n_envs)) != hipSuccess) return cleanup(e, "hipMalloc spec");
  if ((e = hipMalloc(&s->d_inv, 2 * sizeof(uint4) * n_envs)) != hipSuccess) return cleanup(e, "hipMalloc inv");
  if ((e = hipMalloc(&s->d_mask, 2 * sizeof(uint4) * n_envs)) != hipSuccess) return cleanup(e, "hipMalloc mask");
  if ((e = hipMalloc(&s->d_stats, 4 * sizeof(int64_t) * s->n_tiles)) != hipSuccess) return cleanup(e, "hipMalloc stats");
  if ((e = hipMalloc(&s->d_err, 4 * sizeof(int32_t))) != hipSuccess) return cleanup(e, "hipMalloc err");
  // A never-reset slot is a valid all-zero state: scenario 0, agent (0,0) — rejected
  // by nothing but meaningless; craft_reset / craft_set_state define real states.
  if ((e = hipMemset(s->d_agent, 0, sizeof(uint32_t) * n_envs)) != hipSuccess) return cleanup(e, "memset");
  if ((e = hipMemset(s->d_spec, 0, sizeof(int4) * n_envs)) != hipSuccess) return cleanup(e, "memset");
  if ((e = hipMemset(s->d_inv, 0, 2 * sizeof(uint4) * n_envs)) != hipSuccess) return cleanup(e, "memset");
  if ((e = hipMemset(s->d_mask, 0, 2 * sizeof(uint4) * n_envs)) != hipSuccess) return cleanup(e, "memset");
  if ((e = hipMemset(s->d_stats, 0, 4 * sizeof(int64_t) * s->n_tiles)) != hipSuccess) return cleanup(e, "memset");
  if ((e = hipMemset(s->d_err, 0, 4 * sizeof(int32_t))) != hipSuccess) return cleanup(e, "memset");

  SimView& v = s->view;
  v.cfg = s->d_cfg;
  v.pool = s->d_pool;
  v.agent = s->d_agent;
  v.spec = s->d_spec;
  v.inv = s->d_inv;
  v.mask = s->d_mask;
  v.stats_part = s->d_stats;
  v.err = s->d_err;
  v.n_envs = n_envs;
  v.env_base = env_id_base;
  v.pool_count = 0;
  v.W = W; v.H = H; v.K = K; v.F = F; v.C = C; v.CS = CS; v.GS = GS;
  v.maxT = cfg->max_timesteps;
  v.INV0 = 2 * ww * ww * K;
  v.NB = NB;
  v.kc_lo = v.kc_hi = 0;
  for (int k = 0; k < CRAFT_MAX_KINDS; ++k) {
    const uint64_t cls = cfg->kind_class[k] & 0xf;
    if (k < 16) v.kc_lo |= cls << (4 * k);
    else v.kc_hi |= cls << (4 * (k - 16));
  }
  v.magicQ = (uint32_t)((1ull << 32) / (uint64_t)(F / 4 > 0 ? F / 4 : 1)) + 1u;
  size_t off = (size_t)kTileEnvs * GS;
  off = (off + 15) & ~size_t(15);
  v.lds_bits = (int32_t)off;
  off += (size_t)NB * kTileEnvs * 4;
  off = (off + 15) & ~size_t(15);
  v.lds_inv = (int32_t)off;
  off += (size_t)kTileEnvs * kInvStride;
  off = (off + 15) & ~size_t(15);
  v.lds_scen = (int32_t)off;
  off += (size_t)kTileEnvs * 4;
  s->lds_bytes = (off + 15) & ~size_t(15);
  *out = s;
  return CRAFT_OK;
}

int craft_sim_destroy(craft_sim_t* s) {
  if (!s) return CRAFT_OK;
  (void)hipSetDevice(s->device);
  (void)hipFree(s->d_cfg);
  (void)hipFree(s->d_pool);
  (void)hipFree(s->d_agent);
  (void)hipFree(s->d_spec);
  (void)hipFree(s->d_inv);
  (void)hipFree(s->d_mask);
  (void)hipFree(s->d_stats);
  (void)hipFree(s->d_err);
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

int craft_sim_check(craft_sim_t* s, int64_t* env_out, void* stream) {
  if (!s) return CRAFT_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int32_t h[4] = {0, 0, 0, 0};
  HIP_TRY(s, hipMemcpyAsync(h, s->d_err, sizeof(h), hipMemcpyDeviceToHost, st));
  HIP_TRY(s, hipStreamSynchronize(st));
  if (h[0]) {
    HIP_TRY(s, hipMemsetAsync(s->d_err, 0, sizeof(h), st));
    HIP_TRY(s, hipStreamSynchronize(st));
    const int64_t slot = (int64_t)(uint32_t)h[2] | ((int64_t)h[3] << 32);
    if (env_out) *env_out = slot;
    return fail(s, h[0], std::string(craft_strerror(h[0])) + " (slot/item " + std::to_string(slot) + ")");
  }
  if (env_out) *env_out = -1;
  return CRAFT_OK;
}

int craft_pool_load(craft_sim_t* s, const uint8_t* grids, int32_t first, int32_t count) {
  if (!s || !grids || first < 0 || count < 0) return fail(s, CRAFT_EINVAL, "craft_pool_load: bad argument");
  if ((int64_t)first + count > s->pool_capacity) return fail(s, CRAFT_ERANGE, "craft_pool_load: beyond pool capacity");
  const int W = s->cfg.width, H = s->cfg.height, C = W * H, CS = s->view.CS;
  std::vector<uint8_t> staged((size_t)count * CS, 0);
  for (int p = 0; p < count; ++p) {
    const uint8_t* g = grids + (size_t)p * C;
    for (int c = 0; c < C; ++c) {
      if (g[c] >= s->cfg.n_kinds)
        return fail(s, CRAFT_EINVARIANT, "craft_pool_load: kind id out of range in grid " + std::to_string(first + p));
      const int x = c / H, y = c % H;
      if ((x == 0 || y == 0 || x == W - 1 || y == H - 1) && g[c] == 0)
        return fail(s, CRAFT_EINVARIANT, "craft_pool_load: grid " + std::to_string(first + p) +
                                             " has an open border cell (make_data.py:108-112 builds a boundary ring)");
    }
    std::memcpy(staged.data() + (size_t)p * CS, g, C);
  }
  HIP_TRY(s, hipSetDevice(s->device));
  if (count)
    HIP_TRY(s, hipMemcpy(s->d_pool + (size_t)first * CS, staged.data(), staged.size(), hipMemcpyHostToDevice));
  if (first + count > s->pool_count) s->pool_count = first + count;
  s->view.pool_count = s->pool_count;
  return CRAFT_OK;
}

int craft_reset(craft_sim_t* s, const int32_t* scenario, const int32_t* pos_x, const int32_t* pos_y,
                const int32_t* dir, const int32_t* task, float* obs, void* stream) {
  if (!s || !scenario || !pos_x || !pos_y || !dir || !task) return fail(s, CRAFT_EINVAL, "craft_reset: null input");
  if (obs && !aligned16(obs)) return fail(s, CRAFT_EINVAL, "craft_reset: obs must be 16-byte aligned");
  TileArgs a{};
  a.r_scen = scenario; a.r_x = pos_x; a.r_y = pos_y; a.r_dir = dir; a.r_task = task;
  a.n = s->n_envs;
  a.obs = obs;
  hipError_t e = dispatch_tile<MODE_RESET>(s, a, reinterpret_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(s, e, "craft_reset launch");
  e = hipMemsetAsync(s->d_stats, 0, 4 * sizeof(int64_t) * s->n_tiles, reinterpret_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(s, e, "craft_reset stats memset");
  return CRAFT_OK;
}

int craft_step(craft_sim_t* s, const int32_t* actions, uint64_t action_seed, int64_t tick, uint32_t flags,
               float* obs, float* reward, uint8_t* done, int8_t* success, void* stream) {
  if (!s) return CRAFT_EINVAL;
  if (obs && !aligned16(obs)) return fail(s, CRAFT_EINVAL, "craft_step: obs must be 16-byte aligned");
  TileArgs a{};
  a.actions = actions;
  a.seed = action_seed;
  a.tick = tick;
  a.flags = flags;
  a.n = s->n_envs;
  a.obs = obs;
  a.reward = reward;
  a.done = done;
  a.sat = success;
  hipError_t e = dispatch_tile<MODE_TICK>(s, a, reinterpret_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(s, e, "craft_step launch");
  return CRAFT_OK;
}

int craft_stats(craft_sim_t* s, int64_t* stats_out, int32_t reset, void* stream) {
  if (!s || !stats_out) return CRAFT_EINVAL;
  hipLaunchKernelGGL(stats_kernel, dim3(1), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     s->d_stats, s->n_tiles, stats_out, (int)reset);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(s, e, "craft_stats launch");
  return CRAFT_OK;
}

int craft_transition(craft_sim_t* s, const int32_t* src, const int32_t* dst, const int32_t* actions,
                     int64_t n, void* stream) {
  if (!s || !actions || n < 0) return fail(s, CRAFT_EINVAL, "craft_transition: bad argument");
  if (!src && n > s->n_envs) return fail(s, CRAFT_ERANGE, "craft_transition: n > n_envs");
  TileArgs a{};
  a.src = src;
  a.dst = dst ? dst : src;
  a.actions = actions;
  a.n = n;
  hipError_t e = dispatch_tile<MODE_TRANSITION>(s, a, reinterpret_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(s, e, "craft_transition launch");
  return CRAFT_OK;
}

int craft_observe(craft_sim_t* s, const int32_t* slots, int64_t n, const int32_t* tasks, float* obs,
                  int8_t* sat, void* stream) {
  if (!s || n < 0) return fail(s, CRAFT_EINVAL, "craft_observe: bad argument");
  if (!slots && n > s->n_envs) return fail(s, CRAFT_ERANGE, "craft_observe: n > n_envs");
  if (obs && !aligned16(obs)) return fail(s, CRAFT_EINVAL, "craft_observe: obs must be 16-byte aligned");
  TileArgs a{};
  a.src = slots;
  a.tasks = tasks;
  a.n = n;
  a.obs = obs;
  a.sat = sat;
  hipError_t e = dispatch_tile<MODE_OBSERVE>(s, a, reinterpret_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(s, e, "craft_observe launch");
  return CRAFT_OK;
}

int craft_teacher(craft_sim_t* s, const int32_t* slots, int64_t n, const int32_t* tasks, int32_t* action_out,
                  int32_t* path_len_out, void* stream) {
  if (!s || !action_out || n < 0) return fail(s, CRAFT_EINVAL, "craft_teacher: bad argument");
  if (!slots && n > s->n_envs) return fail(s, CRAFT_ERANGE, "craft_teacher: n > n_envs");
  if (4 * s->view.C > 1000)
    return fail(s, CRAFT_EINVAL, "craft_teacher: 4*W*H > 1000 overflows the reference's BFS queue (teachers/base.py:42)");
  if (n == 0) return CRAFT_OK;
  TeachArgs a{slots, tasks, n, action_out, path_len_out};
  const unsigned blocks = (unsigned)((n + 255) / 256);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int nw = (s->view.C + 63) / 64;
  switch (nw) {
    case 1: hipLaunchKernelGGL(teacher_kernel<1>, dim3(blocks), dim3(256), 0, st, s->view, a); break;
    case 2: hipLaunchKernelGGL(teacher_kernel<2>, dim3(blocks), dim3(256), 0, st, s->view, a); break;
    case 3: hipLaunchKernelGGL(teacher_kernel<3>, dim3(blocks), dim3(256), 0, st, s->view, a); break;
    default: hipLaunchKernelGGL(teacher_kernel<4>, dim3(blocks), dim3(256), 0, st, s->view, a); break;
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(s, e, "craft_teacher launch");
  return CRAFT_OK;
}

int craft_get_state(craft_sim_t* s, const int32_t* slots, int64_t n, int32_t* agent, int32_t* inventory,
                    uint8_t* grid, int32_t* spec, void* stream) {
  if (!s || n < 0) return fail(s, CRAFT_EINVAL, "craft_get_state: bad argument");
  if (!slots && n > s->n_envs) return fail(s, CRAFT_ERANGE, "craft_get_state: n > n_envs");
  if (n == 0) return CRAFT_OK;
  hipLaunchKernelGGL(get_state_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), s->view, slots, n, agent, inventory, grid, spec);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(s, e, "craft_get_state launch");
  return CRAFT_OK;
}

int craft_set_state(craft_sim_t* s, const int32_t* slots, int64_t n, const int32_t* spec, const int32_t* agent,
                    const int32_t* inventory, void* stream) {
  if (!s || n < 0 || !spec || !agent) return fail(s, CRAFT_EINVAL, "craft_set_state: bad argument");
  if (!slots && n > s->n_envs) return fail(s, CRAFT_ERANGE, "craft_set_state: n > n_envs");
  if (n == 0) return CRAFT_OK;
  hipLaunchKernelGGL(set_state_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), s->view, slots, n, spec, agent, inventory);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(s, e, "craft_set_state launch");
  return CRAFT_OK;
}

}  // extern "C"
