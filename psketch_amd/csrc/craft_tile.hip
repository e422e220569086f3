// craft_tile.hip — the hot kernel: one rollout tick (or transition / observe /
// reset) for a tile of 64 consecutive envs per 256-thread workgroup.
//
//   A  lanes 0..63 load their env's packed state, inventory and cleared-cell
//      mask (one HBM round trip); the other waves stage the feature LUT and
//      the task table into LDS.
//   B  all threads copy the tile's 64 scenario grids from the (L2-resident)
//      pool into LDS with coalesced dword loads.
//   C  wave 0, one lane per env: clear masked cells, run the rollout protocol
//      and CraftState.step on the LDS grid, write the state back, and leave
//      inventory / dir / agent position in the env's LDS descriptor row.
//   D  all 256 threads build the observation descriptor: local-window cell
//      one-hots and block-max-pooled kind masks (independent LDS reads).
//   E  all threads stream the tile's 64 x F fp32 observation rows to HBM as
//      contiguous 16-byte stores; each value is one LDS word, shift and mask
//      through the per-feature LUT (no branches).
// The kernel is bound by E's HBM writes (F*4 = 1616 B per env at w=3); A-D
// are a short latency chain.
#include "craft_device.h"

namespace craft {

#ifdef CRAFT_STAMPS
// Diagnostic build only (never the product): wave 0 of every workgroup records
// s_memrealtime (100 MHz) at phase boundaries into v.stamps[block][8].
#define STAMP(k)                                                                         \
  do {                                                                                   \
    if (threadIdx.x == 0 && v.stamps) v.stamps[8 * (int64_t)blockIdx.x + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define STAMP_END()                                                                      \
  do {                                                                                   \
    __syncthreads();                                                                     \
    if (threadIdx.x == 0 && v.stamps) {                                                  \
      v.stamps[8 * (int64_t)blockIdx.x + 6] = __builtin_amdgcn_s_memrealtime();          \
      uint32_t xcc;                                                                      \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));                 \
      v.stamps[8 * (int64_t)blockIdx.x + 7] = xcc;                                       \
    }                                                                                    \
  } while (0)
#else
#define STAMP(k) do {} while (0)
#define STAMP_END() do {} while (0)
#endif

template <int WIN>
__device__ __forceinline__ uint32_t cell_bit(const uint8_t* g, int W, int H, int cx, int cy) {
  const bool ok = (unsigned)cx < (unsigned)W && (unsigned)cy < (unsigned)H;
  const int xc = min(max(cx, 0), W - 1), yc = min(max(cy, 0), H - 1);
  const int k = g[xc * H + yc];
  return ok ? (1u << k) : 0u;
}

template <int WIN, int MODE, int TILE>
__global__ __launch_bounds__(4 * TILE) void tile_kernel(SimView v, TileArgs a) {
  constexpr int kTileEnvs = TILE;
  constexpr int kThreads = 4 * TILE;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const LdsLayout lay = lds_layout(TILE, v.GS, v.ND, v.F);
  uint8_t* s_grid = smem;
  uint32_t* s_desc = reinterpret_cast<uint32_t*>(smem + lay.desc);
  uint16_t* s_lut = reinterpret_cast<uint16_t*>(smem + lay.lut);
  uint16_t* s_task = reinterpret_cast<uint16_t*>(smem + lay.task);
  uint8_t* s_rc = smem + lay.rc;
  uint32_t* s_agent = reinterpret_cast<uint32_t*>(smem + lay.agent);

  constexpr int kDirWord = desc_dir_word(WIN);
  constexpr int kInvWord = desc_inv_word(WIN);
  const int tid = threadIdx.x;
  const int64_t env0 = (int64_t)blockIdx.x * kTileEnvs;
  const int nE = (int)min((int64_t)kTileEnvs, a.n - env0);
  const bool want_obs = a.obs != nullptr;

  // ---- A+B: wave 0 loads each env's state, then its scenario row, and the static
  //      tables; waves 1-3 stage the feature LUT (needed only in E). No barrier. -----
  int64_t slot = 0, dslot = 0;
  bool live = false;
  uint32_t init_word = 0;
  int act = 0;
  uint4 i0 = make_uint4(0, 0, 0, 0), i1 = i0, m0 = i0, m1 = i0;
  Agent s{};
  STAMP(0);
  if (tid < kTileEnvs) {
    // static tables: task entries and compact recipes (read by phase C)
    if (tid < v.n_tasks) s_task[tid] = v.task_tab[tid];
    if (tid < CRAFT_MAX_RECIPES * kRecipeBytes / 4)
      reinterpret_cast<uint32_t*>(s_rc)[tid] = reinterpret_cast<const uint32_t*>(v.rc)[tid];
    live = tid < nE;
    if (live) {
      const int64_t i = env0 + tid;
      slot = (MODE == MODE_TICK || MODE == MODE_RESET || !a.src) ? i : (int64_t)a.src[i];
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
            d0 < 0 || d0 > 3 || tk < 0 || tk >= v.n_tasks) {
          latch_error(v.err, CRAFT_EINVAL, i);
          live = false;
        } else {
          s.x = x0; s.y = y0; s.dir = d0; s.frozen = 0; s.timer = v.maxT; s.scen = sc; s.task = tk;
        }
      } else {
        const uint64_t st = v.state[slot];
        if (MODE == MODE_TICK || MODE == MODE_TRANSITION) init_word = v.init[slot];
        if (MODE == MODE_TICK) {
          if (a.actions) {
            act = a.actions[slot];
          } else {
            const uint64_t gid = (uint64_t)(v.env_base + slot);
            act = (int)((uint32_t)(splitmix64(a.seed ^ (gid << 20) ^ (uint64_t)a.tick) >> 32) % 6u);
          }
        } else if (MODE == MODE_TRANSITION) {
          act = a.actions[env0 + tid];
        }
        i0 = v.inv[2 * slot];
        i1 = v.inv[2 * slot + 1];
        m0 = v.mask[2 * slot];
        m1 = v.mask[2 * slot + 1];
        s = unpack_state(st);
        if (s.x < 1 || s.x > v.W - 2 || s.y < 1 || s.y > v.H - 2 || s.scen >= v.pool_count) {
          latch_error(v.err, CRAFT_EINVAL, slot);   // never initialised by reset / set_state
          live = false;
        }
      }
    }
    if (live) {
      // the env's scenario grid: CS/16 independent 16-byte loads (L2-resident pool)
      const uint4* src = reinterpret_cast<const uint4*>(v.pool + (size_t)s.scen * v.CS);
      uint32_t* dst = reinterpret_cast<uint32_t*>(s_grid + tid * v.GS);
      const int nchunk = v.CS >> 4;
      uint4 c[CRAFT_MAX_CELLS / 16];
#pragma unroll
      for (int q = 0; q < CRAFT_MAX_CELLS / 16; ++q)
        if (q < nchunk) c[q] = src[q];
#pragma unroll
      for (int q = 0; q < CRAFT_MAX_CELLS / 16; ++q)
        if (q < nchunk) {
          dst[4 * q + 0] = c[q].x; dst[4 * q + 1] = c[q].y; dst[4 * q + 2] = c[q].z; dst[4 * q + 3] = c[q].w;
        }
    }
    // LDS written above is read below only by the same lane or, for the tables, by
    // lanes of this same wave: order the wave's LDS accesses, no workgroup barrier.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  } else if (want_obs) {
    const uint32_t* lut32 = reinterpret_cast<const uint32_t*>(v.lut);
    uint32_t* s_lut32 = reinterpret_cast<uint32_t*>(s_lut);
    for (int w = tid - kTileEnvs; w < (v.F + 1) / 2; w += kThreads - kTileEnvs) s_lut32[w] = lut32[w];
  }
  STAMP(2);

  // ---- C: one lane per env -------------------------------------------------------------
  if (tid < kTileEnvs) {
    uint8_t* g = s_grid + tid * v.GS;
    uint32_t* row = s_desc + tid * v.ND;
    uint8_t* iv = reinterpret_cast<uint8_t*>(row + kInvWord);
    uint32_t m[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
    row[kInvWord + 0] = i0.x; row[kInvWord + 1] = i0.y; row[kInvWord + 2] = i0.z; row[kInvWord + 3] = i0.w;
    row[kInvWord + 4] = i1.x; row[kInvWord + 5] = i1.y; row[kInvWord + 6] = i1.z; row[kInvWord + 7] = i1.w;
    bool inv_changed = false, mask_changed = false;
    int d = 0, succ = -1, counted = 0;
    if (live) {
      // The LDS row holds pool[scenario]; cells cleared this episode are applied
      // lazily so that an auto-reset (which restores exactly that row) needs no
      // global reload.
      bool restart = false;
      if (MODE == MODE_TICK) {
        // per-env body of ImitationTrainer.do_rollout, trainers/imitation.py:59-73
        if (s.frozen) {
          d = 1;
        } else {
          counted = 1;
          s.timer -= 1;
          d = (act == CRAFT_STOP) || s.timer <= 0;
          restart = d && (a.flags & CRAFT_STEP_AUTORESET);
        }
        if (d) {
          // satisfies() on the pre-step state: only the facing cell and the inventory matter
          const uint32_t tt = s_task[s.task];
          const int fc = (s.x + dir_dx(s.dir)) * v.H + (s.y + dir_dy(s.dir));
          uint32_t mw = 0;
#pragma unroll
          for (int w = 0; w < 8; ++w) mw |= (w == (fc >> 5)) ? m[w] : 0u;
          const int goal = tt & 0xf, arg = (tt >> 4) & 0xff;
          if (goal == CRAFT_GOAL_GET || goal == CRAFT_GOAL_MAKE) succ = iv[arg] > 0;
          else if (goal == CRAFT_GOAL_GO) succ = (((mw >> (fc & 31)) & 1u) ? 0 : (int)g[fc]) == arg;
          else succ = -1;
        }
      }
      if (!restart) {
#pragma unroll
        for (int w = 0; w < 8; ++w) {                     // cells cleared this episode
          uint32_t mm = m[w];
          while (mm) {
            g[w * 32 + __ffs(mm) - 1] = 0;
            mm &= mm - 1;
          }
        }
      }
      if (MODE == MODE_RESET) {
        inv_changed = mask_changed = true;
      } else if (MODE == MODE_TICK) {
        if (restart) {                                    // CraftScenario.init, craft.py:268-273
          s.x = init_word & 0xff; s.y = (init_word >> 8) & 0xff; s.dir = (init_word >> 16) & 3;
          s.timer = v.maxT;
#pragma unroll
          for (int w = 0; w < 8; ++w) { row[kInvWord + w] = 0u; m[w] = 0u; }
          inv_changed = mask_changed = true;
        } else if (d && !s.frozen) {
          s.frozen = 1;
          s.timer = max(s.timer, 0);
        } else if (!d) {
          if (act < 0 || act >= CRAFT_N_ACTIONS) latch_error(v.err, CRAFT_EBADACTION, slot);
          else transition(v, s_rc, g, iv, s, m, act, inv_changed, mask_changed);
        }
      } else if (MODE == MODE_TRANSITION) {
        if (act >= CRAFT_N_ACTIONS) latch_error(v.err, CRAFT_EBADACTION, slot);
        else if (act >= 0) transition(v, s_rc, g, iv, s, m, act, inv_changed, mask_changed);
        if (dslot != slot) inv_changed = mask_changed = true;   // copy-on-step
      } else if (MODE == MODE_OBSERVE) {
        if (a.sat) {
          const int tk = a.tasks ? a.tasks[env0 + tid] : s.task;
          if (tk < 0 || tk >= v.n_tasks) {
            latch_error(v.err, CRAFT_ERANGE, env0 + tid);
            a.sat[env0 + tid] = -1;
          } else {
            a.sat[env0 + tid] = (int8_t)satisfies(v, g, iv, s, s_task[tk]);
          }
        }
      }
      // write back
      if (MODE != MODE_OBSERVE) v.state[dslot] = pack_state(s);
      if (MODE == MODE_RESET) v.init[dslot] = (uint32_t)s.x | ((uint32_t)s.y << 8) | ((uint32_t)s.dir << 16);
      if (MODE == MODE_TRANSITION && dslot != slot) v.init[dslot] = init_word;
      if (inv_changed) {
        v.inv[2 * dslot] = make_uint4(row[kInvWord], row[kInvWord + 1], row[kInvWord + 2], row[kInvWord + 3]);
        v.inv[2 * dslot + 1] = make_uint4(row[kInvWord + 4], row[kInvWord + 5], row[kInvWord + 6], row[kInvWord + 7]);
      }
      if (mask_changed) {
        v.mask[2 * dslot] = make_uint4(m[0], m[1], m[2], m[3]);
        v.mask[2 * dslot + 1] = make_uint4(m[4], m[5], m[6], m[7]);
      }
      if (MODE == MODE_TICK) {
        const int64_t i = env0 + tid;
        if (a.done) a.done[i] = (uint8_t)d;
        if (a.sat) a.sat[i] = (int8_t)succ;
        if (a.reward) a.reward[i] = (counted && d && succ == 1) ? 1.0f : 0.0f;
      }
    } else if (want_obs) {
#pragma unroll
      for (int w = 0; w < 8; ++w) row[kInvWord + w] = 0u;
    }
    row[kDirWord] = live ? (1u << s.dir) : 0u;
    row[kDirWord + 1] = 0u;
    s_agent[tid] = live ? ((uint32_t)s.x | ((uint32_t)s.y << 8) | (1u << 16)) : 0u;
    if (MODE == MODE_TICK) {
      // episode statistics: one partial-sum row per workgroup (uncontended)
      const uint64_t bs = __ballot(live && counted && d && succ == 1);
      const uint64_t be = __ballot(live && counted && d);
      const uint64_t bt = __ballot(live && counted);
      if (tid == 0) {   // no-return atomics: the wave does not wait for them
        unsigned long long* r = reinterpret_cast<unsigned long long*>(v.stats_part + 4 * (int64_t)blockIdx.x);
        atomicAdd(r + 0, (unsigned long long)__popcll(bs));
        atomicAdd(r + 1, (unsigned long long)__popcll(be));
        atomicAdd(r + 2, (unsigned long long)__popcll(bt));
      }
    }
  }
  STAMP(3);
  if (!want_obs) {
    STAMP_END();
    return;
  }
  __syncthreads();
  STAMP(4);

  // ---- D: descriptors (local one-hots, pooled kind masks), all threads -----------------
  {
    const int e = tid & (kTileEnvs - 1), part = tid / kTileEnvs;
    const uint32_t ag = s_agent[e];
    uint32_t* row = s_desc + e * v.ND;
    const uint8_t* g = s_grid + e * v.GS;
    const int W = v.W, H = v.H;
    const int x = ag & 0xff, y = (ag >> 8) & 0xff;
    const bool ok = (ag >> 16) & 1;
    constexpr int W2 = WIN * WIN;
    if (part == 0) {
      constexpr int hw = WIN / 2;
#pragma unroll
      for (int i = 0; i < WIN; ++i)
#pragma unroll
        for (int j = 0; j < WIN; ++j)
          row[i * WIN + j] = ok ? (cell_bit<WIN>(g, W, H, x - hw + i, y - hw + j) & ~1u) : 0u;
    } else {
      constexpr int bh = W2 / 2;
#pragma unroll
      for (int j = 0; j < (W2 + 2) / 3; ++j) {
        const int b = part - 1 + 3 * j;
        if (b >= W2) break;
        const int bi = b / WIN, bj = b - bi * WIN;
        const int x0 = x - bh + bi * WIN, y0 = y - bh + bj * WIN;
        uint32_t msk = 0;
        if (ok && x0 < W && x0 + WIN > 0 && y0 < H && y0 + WIN > 0) {
#pragma unroll
          for (int ii = 0; ii < WIN; ++ii)
#pragma unroll
            for (int jj = 0; jj < WIN; ++jj) msk |= cell_bit<WIN>(g, W, H, x0 + ii, y0 + jj);
        }
        row[W2 + b] = msk & ~1u;
      }
    }
  }
  __syncthreads();
  STAMP(5);

  // ---- E: stream the tile's observation rows --------------------------------------------
  const int F = v.F;
  float* tile = a.obs + env0 * (int64_t)F;
  if ((F & 3) == 0) {
    const int Q = F >> 2;
    const int nslots = nE * Q;
    float4* out4 = reinterpret_cast<float4*>(tile);
    for (int sidx = tid; sidx < nslots; sidx += kThreads) {
      const int e = (int)__umulhi((uint32_t)sidx, v.magicQ);
      const int f = (sidx - e * Q) << 2;
      const uint2 lw = *reinterpret_cast<const uint2*>(s_lut + f);
      const uint32_t* row = s_desc + e * v.ND;
      const uint32_t u0 = lw.x & 0xffff, u1 = lw.x >> 16, u2 = lw.y & 0xffff, u3 = lw.y >> 16;
      float4 o;
      o.x = (float)((row[u0 & 127] >> ((u0 >> 7) & 31)) & ((u0 & 4096) ? 0xffu : 1u));
      o.y = (float)((row[u1 & 127] >> ((u1 >> 7) & 31)) & ((u1 & 4096) ? 0xffu : 1u));
      o.z = (float)((row[u2 & 127] >> ((u2 >> 7) & 31)) & ((u2 & 4096) ? 0xffu : 1u));
      o.w = (float)((row[u3 & 127] >> ((u3 >> 7) & 31)) & ((u3 & 4096) ? 0xffu : 1u));
      out4[sidx] = o;
    }
  } else {
    for (int sidx = tid; sidx < nE * F; sidx += kThreads) {
      const int e = sidx / F, f = sidx - e * F;
      const uint32_t u = s_lut[f];
      tile[sidx] = (float)((s_desc[e * v.ND + (u & 127)] >> ((u >> 7) & 31)) & ((u & 4096) ? 0xffu : 1u));
    }
  }
  STAMP_END();
}

template <int WIN, int MODE, int TILE>
static hipError_t launch_one(const SimView& v, const TileArgs& a, size_t lds, hipStream_t st) {
  const int64_t tiles = (a.n + TILE - 1) / TILE;
  if (tiles == 0) return hipSuccess;
  hipLaunchKernelGGL((tile_kernel<WIN, MODE, TILE>), dim3((unsigned)tiles), dim3(4 * TILE), lds, st, v, a);
  return hipGetLastError();
}

template <int MODE, int TILE>
static hipError_t launch_win(int win, const SimView& v, const TileArgs& a, size_t lds, hipStream_t st) {
  switch (win) {
    case 3: return launch_one<3, MODE, TILE>(v, a, lds, st);
    case 5: return launch_one<5, MODE, TILE>(v, a, lds, st);
    default: return launch_one<7, MODE, TILE>(v, a, lds, st);
  }
}

template <int MODE>
static hipError_t launch_tiled(int tile, int win, const SimView& v, const TileArgs& a, size_t lds,
                               hipStream_t st) {
  switch (tile) {
    case 16: return launch_win<MODE, 16>(win, v, a, lds, st);
    case 32: return launch_win<MODE, 32>(win, v, a, lds, st);
    default: return launch_win<MODE, 64>(win, v, a, lds, st);
  }
}

// The rollout tick and the observation take the tuned tile size; the
// reference-granular transition / reset always run 64-env tiles.
hipError_t launch_tile(int mode, int win, int tile, const SimView& v, const TileArgs& a, size_t lds,
                       hipStream_t st) {
  switch (mode) {
    case MODE_TICK: return launch_tiled<MODE_TICK>(tile, win, v, a, lds, st);
    case MODE_OBSERVE: return launch_tiled<MODE_OBSERVE>(tile, win, v, a, lds, st);
    case MODE_TRANSITION: return launch_win<MODE_TRANSITION, 64>(win, v, a, lds, st);
    default: return launch_win<MODE_RESET, 64>(win, v, a, lds, st);
  }
}

}  // namespace craft
