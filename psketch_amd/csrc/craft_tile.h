// craft_tile.h — the hot kernel: one rollout tick (or transition / observe /
// reset) for a tile of TILE consecutive envs per 256-thread workgroup.
//
//   A  wave 0, one lane per env: load the env's packed state word, inventory,
//      cleared-cell mask, restart spec and action (one HBM round trip), then its
//      scenario row from the L2-resident pool, straight into LDS; the static
//      task / recipe tables come along.  No workgroup barrier.
//   C  same lanes: run the rollout protocol and CraftState.step on the LDS grid,
//      write the state back.  Meanwhile waves 1-3 zero the tile's observation
//      bytes in LDS.
//   D  all threads scatter the observation's non-zero bytes (local-window
//      one-hots, block-max-pooled one-hots, inventory counts, dir one-hot) into
//      the tile's u8 rows [TILE][F] in LDS.
//   E  all threads stream the rows to HBM: flat index s, one LDS read, one
//      contiguous 16-byte store (fp32: ds_read_b32 of 4 feature bytes and 4
//      v_cvt_f32_ubyte; bf16: 8 bytes; u8: 16 bytes as they are).
// The kernel is bound by E's HBM writes (F*4 = 1616 B per env at w=3).  See
// DESIGN.md for the roofline and the phase timings that shaped this layout.
#pragma once
#include "craft_obs.h"
#include "craft_teach.h"

namespace craft {

// TL > 0 (MODE_TICK only): TILE * TL more threads run the DemonstrationTeacher on
// every env's new state (craft_step_teach), TL lanes per env, while the first
// tick threads stream the observations: the BFS reads the grid rows the tick left in
// LDS.  NW = 32-bit words per cell set (teach_env).
#ifndef CRAFT_TT_WPE
#define CRAFT_TT_WPE 4
#endif
#ifndef CRAFT_TILE_U
#define CRAFT_TILE_U 4          // 16-byte stores in flight per lane of E (3x3 windows)
#endif
// 5x5 / 7x7: 2 (alternating on one box, 32-env tiles at 65,536 envs: the bare tick 61.6 -> 60.9 us,
// with the teacher 66.1 -> 64.7-65.6; 8 no better than 4)
#ifndef CRAFT_TILE_U_WIDE
#define CRAFT_TILE_U_WIDE 2
#endif
// Tick threads per workgroup (A + C on the first TILE, then D and E on all): 256, or 192 with a
// teacher on a 32-env tile (craft_step_teach at 5x5 / 7x7), so that with pairs the workgroup is 4
// waves and four of them share a CU, one wave per SIMD each (the LDS allows four; 5-wave
// workgroups stopped at three per CU, 70.6 against 60 us for the bare tick at 5x5).
__host__ __device__ constexpr int tile_tick_threads(int tile, int tl) { return tl > 0 && tile == 32 ? 192 : kThreads; }

template <int WIN, int MODE, int TILE, int TL = 0, int NW = 0>
__global__ __launch_bounds__(tile_tick_threads(TILE, TL) + TILE * TL, TL > 0 ? CRAFT_TT_WPE : 1) void tile_kernel(SimView v, TileArgs a) {
  constexpr int NT = tile_tick_threads(TILE, TL);
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const LdsLayout lay = lds_layout(TILE, v.GS, v.F);
  uint8_t* s_grid = smem;
  uint8_t* s_obs = smem + lay.obs;
  uint8_t* s_inv = smem + lay.inv;
  uint16_t* s_task = reinterpret_cast<uint16_t*>(smem + lay.task);
  uint32_t* s_rc = reinterpret_cast<uint32_t*>(smem + lay.rc);
  uint32_t* s_agent = reinterpret_cast<uint32_t*>(smem + lay.agent);
  // TL > 0, the teacher's words, packed so that a 32-env tile at 5x5 stays within a quarter of the
  // CU's LDS (four workgroups per CU, tile_tt_lds_bytes): each env's teacher info word (task |
  // frozen << 8 | ...) in the 4 pad bytes of its grid row (GS = CS + 4), the deferred BFS
  // queries in the 4 pad bytes of the inventory rows (counts in the first CRAFT_MAX_KINDS), the
  // D sync and the deferred-BFS controls in the control words, task_sub as bytes after the layout.
  static_assert(kInvStride >= CRAFT_MAX_KINDS + 4 && CRAFT_MAX_TASKS <= 127, "teacher words in row padding");
  uint32_t* s_tinfo = reinterpret_cast<uint32_t*>(smem + v.CS);        // [TILE], word stride GS / 4
  const int tis = v.GS >> 2;
  uint32_t* s_work = reinterpret_cast<uint32_t*>(s_inv + CRAFT_MAX_KINDS);   // [TILE], word stride kInvStride / 4
  constexpr int kWs = kInvStride / 4;
  uint32_t* s_dsync = reinterpret_cast<uint32_t*>(smem + lay.ctrl);
  uint32_t* s_wctl = s_dsync + 1;           // {deferred BFS count, teacher arrivals} (craft_teach.h)
  int8_t* s_tsub = reinterpret_cast<int8_t*>(smem + lay.bytes);        // [n_tasks][CRAFT_MAX_SUBTASKS]

  const int tid = threadIdx.x;
  const int64_t env0 = (int64_t)blockIdx.x * TILE;
  const int nE = (int)min((int64_t)TILE, a.n - env0);
  const bool want_obs = a.obs != nullptr;
  const int F = v.F;

  STAMP(0);
  // ---- A + C: wave 0, one lane per env ------------------------------------------------------
  if (tid < TILE) {
    int64_t slot = 0, dslot = 0;
    bool live = tid < nE;
    uint32_t init_word = 0;
    int act = 0, ref = 0;
    uint32_t bc = 0;
    uint64_t st = 0;
    uint4 i0 = make_uint4(0, 0, 0, 0), i1 = i0, m0 = i0, m1 = i0;
    Agent s{};
    if (live) {
      const int64_t i = env0 + tid;
      slot = (MODE == MODE_TICK || MODE == MODE_RESET || !a.src) ? i : (int64_t)a.src[i];
      dslot = (MODE == MODE_TRANSITION && a.dst) ? (int64_t)a.dst[i] : slot;
      if (slot < 0 || slot >= v.n_envs || dslot < 0 || dslot >= v.n_envs) {
        latch_error(v.err, CRAFT_ERANGE, i);
        live = false;
      }
    }
    // Every independent load of the env first, no result used before the last is issued (a
    // wave waits for its loads in issue order): state, inventory, mask, restart spec, action and
    // clone flag + label, then the static tables into registers; one round trip, then the row.
    if (live && MODE != MODE_RESET) {
      st = v.state[slot];
      i0 = v.inv[2 * slot];
      i1 = v.inv[2 * slot + 1];
      m0 = v.mask[2 * slot];
      m1 = v.mask[2 * slot + 1];
      if (MODE == MODE_TICK || MODE == MODE_TRANSITION) init_word = v.init[slot];
      if (MODE == MODE_TICK) {
        if (a.actions) act = a.actions[slot];
        if (a.bc) {
          bc = a.bc[slot];
          ref = a.ref[slot];
        }
      } else if (MODE == MODE_TRANSITION) {
        act = a.actions[env0 + tid];
      }
    }
    constexpr int QT = (CRAFT_MAX_TASKS + TILE - 1) / TILE;
    constexpr int QR = (CRAFT_MAX_RECIPES * 3 + TILE - 1) / TILE;
    constexpr int QS = TL > 0 ? (CRAFT_MAX_TASKS * CRAFT_MAX_SUBTASKS + TILE - 1) / TILE : 1;
    uint32_t tw[QT], rw[QR];
    int32_t sw[QS];
    // (unconditional loads within the tables' allocations: straight-line code, no wait between)
#pragma unroll
    for (int q = 0; q < QT; ++q) tw[q] = v.task_tab[min(tid + q * TILE, CRAFT_MAX_TASKS - 1)];
#pragma unroll
    for (int q = 0; q < QR; ++q) rw[q] = v.rcw[min(tid + q * TILE, CRAFT_MAX_RECIPES * 3 - 1)];
#pragma unroll
    for (int q = 0; q < QS; ++q)
      sw[q] = TL > 0 ? v.task_sub[min(tid + q * TILE, CRAFT_MAX_TASKS * CRAFT_MAX_SUBTASKS - 1)] : 0;
#pragma unroll
    for (int q = 0; q < QT; ++q)
      if (tid + q * TILE < v.n_tasks) s_task[tid + q * TILE] = (uint16_t)tw[q];
#pragma unroll
    for (int q = 0; q < QR; ++q)
      if (tid + q * TILE < CRAFT_MAX_RECIPES * 3) s_rc[tid + q * TILE] = rw[q];
    if (TL > 0) {
#pragma unroll
      for (int q = 0; q < QS; ++q)
        if (tid + q * TILE < v.n_tasks * CRAFT_MAX_SUBTASKS) s_tsub[tid + q * TILE] = (int8_t)sw[q];
      if (tid == 0) { *s_dsync = 0u; s_wctl[0] = 0u; s_wctl[1] = 0u; }
    }
    if (live) {
      if (MODE == MODE_RESET) {
        const int64_t i = env0 + tid;
        const int sc = a.r_scen[i], x0 = a.r_x[i], y0 = a.r_y[i], d0 = a.r_dir[i], tk = a.r_task[i];
        if (sc < 0 || sc >= v.pool_count || x0 < 1 || x0 > v.W - 2 || y0 < 1 || y0 > v.H - 2 ||
            d0 < 0 || d0 > 3 || tk < 0 || tk >= v.n_tasks) {
          latch_error(v.err, CRAFT_EINVAL, i);
          live = false;
        } else {
          s.x = x0; s.y = y0; s.dir = d0; s.frozen = 0; s.timer = v.maxT; s.scen = sc; s.task = tk;
        }
      } else {
        if (MODE == MODE_TICK) {
          if (!a.actions) {
            const uint64_t gid = (uint64_t)(v.env_base + slot);
            act = (int)((uint32_t)(splitmix64(a.seed ^ (gid << 20) ^ (uint64_t)a.tick) >> 32) % 6u);
          }
          asm volatile("" : "+v"(bc), "+v"(ref));                      // (no early wait on the flag)
          if (a.bc && (bc & 0xffu)) act = ref;                         // behaviour cloning, imitation.py:56-57
        }
        s = unpack_state(st);
        if (s.x < 1 || s.x > v.W - 2 || s.y < 1 || s.y > v.H - 2 || s.scen >= v.pool_count) {
          latch_error(v.err, CRAFT_EINVAL, slot);   // never initialised by reset / set_state
          live = false;
        }
      }
    }
    uint8_t* g = s_grid + tid * v.GS;
    uint32_t conn = 0, tcw0 = ~0u, tcw1 = ~0u;           // TL > 0: the scenario's free cells connected,
    if (TL > 0 && live) {                                  // its clearable cells the teacher table lists
      conn = v.pool_conn[s.scen];
      if (v.ttab) {
        tcw0 = v.tt_cells[2 * (size_t)s.scen];
        tcw1 = v.tt_cells[2 * (size_t)s.scen + 1];
      }
    }
    if (live) {
      // the env's scenario grid: CS/16 independent 16-byte loads (L2-resident pool)
      const uint4* src = reinterpret_cast<const uint4*>(v.pool + (size_t)s.scen * v.CS);
      uint32_t* dst = reinterpret_cast<uint32_t*>(g);
      const int nchunk = v.CS >> 4;
      // (two batches of up to 8 loads with the teacher waves beside: 32 VGPRs, not 64)
      constexpr int QB = TL > 0 ? 8 : CRAFT_MAX_CELLS / 16;
#pragma unroll
      for (int b = 0; b < CRAFT_MAX_CELLS / 16; b += QB) {
        uint4 c[QB];
#pragma unroll
        for (int q = 0; q < QB; ++q)
          if (b + q < nchunk) c[q] = src[b + q];
#pragma unroll
        for (int q = 0; q < QB; ++q)
          if (b + q < nchunk) {
            dst[4 * (b + q) + 0] = c[q].x; dst[4 * (b + q) + 1] = c[q].y;
            dst[4 * (b + q) + 2] = c[q].z; dst[4 * (b + q) + 3] = c[q].w;
          }
      }
    }
    // Every LDS word written above is read below by the same lane, or (the
    // tables) by lanes of this same wave: order the wave's LDS accesses.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#ifndef CRAFT_STAMPS_TT
    STAMP(1);
#endif

    // ---- C ----
    uint32_t* ivw = reinterpret_cast<uint32_t*>(s_inv + tid * kInvStride);
    uint8_t* iv = s_inv + tid * kInvStride;
    uint32_t m[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
    ivw[0] = i0.x; ivw[1] = i0.y; ivw[2] = i0.z; ivw[3] = i0.w;
    ivw[4] = i1.x; ivw[5] = i1.y; ivw[6] = i1.z; ivw[7] = i1.w;
    bool inv_changed = false, mask_changed = false;
    int d = 0, succ = -1, counted = 0;
    int code = -1;                                         // transition code (craft.h)
    if (live) {
      // The LDS row holds pool[scenario]; cells cleared this episode are applied
      // lazily, so an auto-reset (which restores exactly that row) needs no reload.
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
          // satisfies() of the pre-step state: only the facing cell and the inventory matter
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
          for (int w = 0; w < 8; ++w) { ivw[w] = 0u; m[w] = 0u; }
          inv_changed = mask_changed = true;
        } else if (d && !s.frozen) {
          s.frozen = 1;
          s.timer = max(s.timer, 0);
        } else if (!d) {
          if (act < 0 || act >= CRAFT_N_ACTIONS) {
            latch_error(v.err, CRAFT_EBADACTION, slot);
          } else {
            const int ox = s.x, oy = s.y;
            transition<TILE == 64>(v, s_rc, g, iv, s, m, act, inv_changed, mask_changed, rw[0], slot);
            code = transition_code(ox, oy, s, inv_changed);
          }
        }
      } else if (MODE == MODE_TRANSITION) {
        if (act >= CRAFT_N_ACTIONS) {
          latch_error(v.err, CRAFT_EBADACTION, slot);
        } else if (act >= 0) {
          const int ox = s.x, oy = s.y;
          transition<TILE == 64>(v, s_rc, g, iv, s, m, act, inv_changed, mask_changed, rw[0], slot);
          code = transition_code(ox, oy, s, inv_changed);
        }
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
        if (a.reward) a.reward[i] = (counted && d && succ == 1) ? 1.0f : 0.0f;
        if (a.rec) a.rec[i] = counted ? act : -1;        // action_seqs, imitation.py:59-61
      }
    }
    if ((MODE == MODE_TICK || MODE == MODE_TRANSITION) && a.code && tid < nE) a.code[env0 + tid] = (int8_t)code;
    s_agent[tid] = live ? ((uint32_t)s.x | ((uint32_t)s.y << 8) | ((uint32_t)s.dir << 16) | (1u << 24)) : 0u;
    // the teacher's inputs: task | frozen << 8 | scenario connected << 9 | the teacher table has
    // this grid (craft_teach.h) << 10 | its table row << 11 (< 2^21 when the table is on)
    if (TL > 0) {
      int ncl = 0;
#pragma unroll
      for (int w = 0; w < 8; ++w) ncl += __popc(m[w]);
      const int trow = live ? tt_index(v, s.scen, tcw0, tcw1, ncl, [&](int c) { return g[c] == 0; }) : -1;
      s_tinfo[tid * tis] = (uint32_t)s.task | ((uint32_t)s.frozen << 8) | (conn << 9) |
                     (trow >= 0 ? (1u << 10) | ((uint32_t)trow << 11) : 0u);
    }
    if (MODE == MODE_TICK) {
      // episode statistics: one partial-sum row per workgroup (uncontended)
      const uint64_t bs = __ballot(live && counted && d && succ == 1);
      const uint64_t be = __ballot(live && counted && d);
      const uint64_t bt = __ballot(live && counted);
      const uint64_t bl = __ballot(live && counted && !d);
      if (tid == 0) {   // no-return atomics: the wave does not wait for them
        unsigned long long* r = reinterpret_cast<unsigned long long*>(v.stats_part + 4 * (int64_t)blockIdx.x);
        atomicAdd(r + 0, (unsigned long long)__popcll(bs));
        atomicAdd(r + 1, (unsigned long long)__popcll(be));
        atomicAdd(r + 2, (unsigned long long)__popcll(bt));
        if (a.any_live && bl) *a.any_live = 1;          // idempotent plain store
      }
    }
  } else if (want_obs && tid < NT) {
    // waves 1-3: zero the tile's observation bytes while wave 0 runs A + C
    uint4* z = reinterpret_cast<uint4*>(s_obs);
    const int n16 = (nE * F + 15) >> 4;
    for (int i = tid - TILE; i < n16; i += NT - TILE) z[i] = make_uint4(0, 0, 0, 0);
  }
  STAMP(3);
  if (TL == 0 && !want_obs) {
    STAMP_END();
    return;
  }
  __syncthreads();
#ifndef CRAFT_STAMPS_TT
  STAMP(4);
#endif

  // ---- D: scatter the observation's non-zero bytes ---------------------------------------------
  if (want_obs && tid < NT) scatter_features<WIN, TILE, NT>(v, s_grid, s_inv, s_agent, s_obs, nE, tid);
  if (TL == 0) {
    if (want_obs) __syncthreads();
  } else if (want_obs && tid < NT) {
    // D -> E among the tick's 4 waves only (an LDS arrival counter), so the teacher waves
    // start right after C instead of waiting out the scatter at a workgroup barrier
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if ((tid & 63) == 0) __hip_atomic_fetch_add(s_dsync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__hip_atomic_load(s_dsync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < (uint32_t)(NT / 64))
      __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  STAMP(5);

  if constexpr (TL > 0) if (tid >= NT) {
    // ---- T: DemonstrationTeacher on the new state (teachers/demonstration.py:9-30) from the
    // grid row the tick left in LDS (cleared cells already applied), overlapping E ----------
    const int u = tid - NT, e = u / TL, ql = u % TL;
    if (e < nE) {
      const int64_t i = env0 + e;
      const uint32_t ag = s_agent[e], ti = s_tinfo[e * tis];
      int action = -2;                                    // a slot C could not run (error latched)
      if (ag && ((ti >> 8) & 1u)) {
        action = -1;                                      // frozen: the trainer's label for a done env
      } else if (ag) {
#ifdef CRAFT_ABL_NOTEACH
        action = CRAFT_STOP;                              // ablation build only: no teacher work
      } else if (false) {
#endif
        Agent s{};
        s.x = ag & 0xff; s.y = (ag >> 8) & 0xff; s.dir = (ag >> 16) & 3; s.task = ti & 0xff;
        const uint32_t m0[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        int len = -1, err = 0, defer = -1;
        // the hint walk (and, with tt_fused, the teacher table for a pristine grid); a BFS left
        // over is deferred to the workgroup's dense pass
        action = teach_env<NW, TL, true>(v, s_task, s_tsub, reinterpret_cast<const uint32_t*>(s_grid + e * v.GS),
                                   m0, s_inv + e * kInvStride, s, s.task, ql, false, len, err,
                                   ((ti >> 9) & 1u) != 0, (v.tt_fused && ((ti >> 10) & 1u)) ? tt_row(v, (int)(ti >> 11)) : nullptr,
                                   &defer, (v.tt_fused && ((ti >> 10) & 1u)) ? tt_row4(v, (int)(ti >> 11)) : nullptr);
        if (err && ql == 0) latch_error(v.err, err, i);
        if (action == kTeachDeferred && ql == 0)
          s_work[kWs * __hip_atomic_fetch_add(&s_wctl[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)] =
              (uint32_t)e | ((uint32_t)defer << 8);
      }
      if (ql == 0 && action != kTeachDeferred) a.label[i] = action;
    }
    // every teacher wave has listed its deferred queries; then all of them run the BFS densely
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if ((tid & 63) == 0) __hip_atomic_fetch_add(&s_wctl[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__hip_atomic_load(&s_wctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < (uint32_t)(TILE * TL / 64))
      __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const uint32_t nw = __hip_atomic_load(&s_wctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#ifdef CRAFT_STAMPS_TT      // diagnostic: 1 the teacher's walks done, 2 its dense pass done, 4 E done
    if (tid == NT && v.stamps) v.stamps[8 * (int64_t)blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
#endif
    teach_deferred_dense<NW, TL>(v, s_work, (int)nw, u, TILE * TL, s_grid, v.GS, s_agent, s_tinfo, a.label + env0,
                                 env0, kWs, tis);
#ifdef CRAFT_STAMPS_TT
    STAMP_MAX(2);
#endif
    STAMP_END();
    return;
  }
  if (!want_obs) {
    STAMP_END();
    return;
  }

  // ---- E: stream the tile's rows to HBM in the handle's observation format ------------------
  constexpr int U = WIN == 3 ? CRAFT_TILE_U : CRAFT_TILE_U_WIDE;
  switch (v.obs_fmt) {
    case CRAFT_OBS_BF16: stream_obs<CRAFT_OBS_BF16, NT, false, U>(s_obs, a.obs, env0, F, nE, v.obs_policy, tid); break;
    case CRAFT_OBS_U8: stream_obs<CRAFT_OBS_U8, NT, false, U>(s_obs, a.obs, env0, F, nE, v.obs_policy, tid); break;
    default: stream_obs<CRAFT_OBS_F32, NT, false, U>(s_obs, a.obs, env0, F, nE, v.obs_policy, tid); break;
  }
#ifdef CRAFT_STAMPS_TT
  STAMP_MAX(4);
#endif
  STAMP_END();
}

}  // namespace craft
