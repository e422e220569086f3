// craft_tick2.h — one rollout tick fused with the DemonstrationTeacher (craft_step_teach) with
// J tiles of 64 envs per workgroup and the observation work split per wave, so that a
// tick's compute overlaps its own stores instead of waiting for them.
//
// Why.  The one-tile tick kernel (craft_tile.h) runs A (state loads), C (transition),
// D (scatter) and E (stores) in order, and every workgroup of the grid is resident at
// once, so the whole chip does A, C and D before the first byte leaves (~8 us
// of a ~26 us tick).  With the teacher fused in, a workgroup also lives until its BFS
// waves finish, and a second round of workgroups starts only then.
//
// Here (WIN = 3, J = 2, 512 workgroups at 65536 envs: one round; TW = 4 tick waves shown):
//   waves 0..J-1  A + C: wave j owns tile j (one lane per env), loads every word it needs
//                 up front (before any store of the workgroup is queued: a load waits for
//                 the wave's older stores) and writes the post-step grid row to LDS;
//   waves J..3    zero the observation rows meanwhile;
//   one workgroup barrier;
//   waves 0..3    wave w scatters envs 16w..16w+15 of tile 0 (D) into its own LDS rows,
//                 streams them (E, clearing the bytes it reads), then does tile 1: no
//                 barrier between tiles or phases, and D of tile 1 runs while E of tile 0
//                 is still in flight;
//   teacher       J*TL teacher waves (TL lanes per env, a tile's envs on TL waves) run the
//                 DemonstrationTeacher on each tile's post-step rows right after the
//                 barrier, overlapping D and E.
// Fused tick + teacher at 65536 envs: 27-31 us instead of 38 (tools/ab_tick2.sh).  Without
// a teacher (TL = 0) the same structure measured 2-3 us slower than the one-tile kernel
// (half the streaming waves per CU), so craft_step keeps that one.
// Results are identical to tile_kernel<WIN, MODE_TICK> + the teacher: the same tests run
// both (craft_sim_tune_teach selects either kernel).
#pragma once
#include "craft_obs.h"
#include "craft_teach.h"

namespace craft {

constexpr int kTick2Tile = 64;          // envs per tile (one lane each in A + C)

// LDS carve: grid rows [J*64][GS] | inventory rows [J*64][kInvStride] | agent words [J*64] |
// teacher info words [J*64] | task table [64] u16 | task_sub [64][4] | recipe words [16][3] |
// observation rows [nbuf waves][up16(64/TW*F)] (nbuf: the tick waves, plus the teacher waves
// when they join D + E, tick2_share)
struct Tick2Lds {
  int inv, agent, tinfo, task, tsub, rc, wsr, work, obs, bytes;
};
// Whether the teacher waves take D + E chunks once their teaching is done (rows of their own):
// pairs (2 teacher waves per tile) and grids up to 12x12, where the rows still leave two
// workgroups per CU.
__host__ __device__ constexpr bool tick2_share(int TL, int NW) { return TL == 2 && NW <= 4; }
__host__ __device__ inline Tick2Lds tick2_lds(int J, int TW, int GS, int F, int nbuf) {
  auto up16 = [](int x) { return (x + 15) & ~15; };
  const int n = J * kTick2Tile;
  Tick2Lds l;
  l.inv = up16(n * GS);
  l.agent = up16(l.inv + n * kInvStride);
  l.tinfo = l.agent + n * 4;
  l.task = l.tinfo + n * 4;
  l.tsub = up16(l.task + CRAFT_MAX_TASKS * 2);
  l.rc = l.tsub + CRAFT_MAX_TASKS * CRAFT_MAX_SUBTASKS * 4;
  l.wsr = up16(l.rc + CRAFT_MAX_RECIPES * 12);    // SimView::wsr [CRAFT_MAX_KINDS][4] uint2
  l.work = l.wsr + CRAFT_MAX_KINDS * 4 * 8;       // deferred BFS list [n] + {count, arrivals, chunk}
  l.obs = up16(l.work + n * 4 + 12);
  l.bytes = l.obs + nbuf * up16(kTick2Tile / TW * F);
  return l;
}

#ifndef CRAFT_T2_WPE
#define CRAFT_T2_WPE 4
#endif
#ifndef CRAFT_T2_U
#define CRAFT_T2_U 4            // 16-byte stores in flight per lane of a tick wave's E
#endif
// TW tick waves (4 or 8): D + E of 64 / TW envs per tile each.
template <int WIN, int J, int TW, int TL, int NW>
__global__ __launch_bounds__(64 * TW + J * kTick2Tile * TL, CRAFT_T2_WPE) void tick2_kernel(SimView v, TileArgs a) {
  constexpr int kTick2Waves = TW, kTick2Sub = kTick2Tile / TW;
  static_assert(J >= 1 && J < TW, "A + C runs on the first J tick waves, the rest zero the rows");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int GS = v.GS, F = v.F;
  constexpr bool SHARE = tick2_share(TL, NW);
  constexpr int NBUF = SHARE ? TW + J * TL : TW;                        // observation row buffers
  const Tick2Lds lay = tick2_lds(J, TW, GS, F, NBUF);
  uint8_t* s_grid = smem;
  uint8_t* s_inv = smem + lay.inv;
  uint32_t* s_agent = reinterpret_cast<uint32_t*>(smem + lay.agent);
  uint32_t* s_tinfo = reinterpret_cast<uint32_t*>(smem + lay.tinfo);   // task | frozen << 8 | conn << 9
  uint16_t* s_task = reinterpret_cast<uint16_t*>(smem + lay.task);
  int32_t* s_tsub = reinterpret_cast<int32_t*>(smem + lay.tsub);
  uint32_t* s_rc = reinterpret_cast<uint32_t*>(smem + lay.rc);
  uint2* s_wsr = reinterpret_cast<uint2*>(smem + lay.wsr);
  uint32_t* s_work = reinterpret_cast<uint32_t*>(smem + lay.work);       // deferred BFS queries
  uint32_t* s_wctl = s_work + J * kTick2Tile;                  // {count, teacher arrivals, D + E chunks}
  const int obs_w = (kTick2Sub * F + 15) & ~15;

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int64_t envw = (int64_t)blockIdx.x * (J * kTick2Tile);          // this workgroup's first env
  // CRAFT_STAMPS builds (tools/tick2_stamps.py): 0 start, 1 wave 0's loads landed, 2 wave 0's C
  // done, 3 past the barrier, 4 wave 0's first store issued, 5 the last tick wave done issuing
  // stores, 6 the last teacher wave done, 7 the XCC.  With CRAFT_STAMPS_C, wave 0's A + C in
  // detail instead: 1 the state word landed, 2 the pool row in LDS, 3 the pre-step tests and
  // cleared cells applied, 4 the transition done, 5 its global stores issued, 6 C done.
  // With CRAFT_STAMPS_T, the teacher in detail instead: 1 the last teacher wave's walk done, 2
  // the last teacher wave into the dense pass, 4 the number of deferred queries (a count).
#ifdef CRAFT_STAMPS_C
#define T2S(k, kc) do { if ((kc) >= 0) STAMP((kc) < 0 ? 0 : (kc)); } while (0)
#define T2SM(k) do {} while (0)
#define T2ST(k) do {} while (0)
#elif defined(CRAFT_STAMPS_T)
#define T2S(k, kc) do { if ((k) == 3) STAMP(3); } while (0)
#define T2SM(k) STAMP_MAX(k)
#define T2ST(k) STAMP_MAX(k)
#else
#define T2ST(k) do {} while (0)
#define T2S(k, kc) do { if ((k) >= 0) STAMP((k) < 0 ? 0 : (k)); } while (0)
#define T2SM(k) STAMP_MAX(k)
#endif
  STAMP(0);
  const bool want_obs = a.obs != nullptr;
  auto tile_envs = [&](int j) { return (int)max((int64_t)0, min((int64_t)kTick2Tile, a.n - envw - j * kTick2Tile)); };

  if (wave < J) {
    // ---- A + C: wave j, one lane per env of tile j (as tile_kernel<MODE_TICK>) -------------------
    const int j = wave;
    const int nE = tile_envs(j);
    const int le = j * kTick2Tile + lane;                                // env index in the workgroup
    const int64_t slot = envw + le;
    bool live = lane < nE;
    uint32_t init_word = 0;
    int act = 0, ref = 0;
    uint32_t bc = 0;
    uint64_t st = 0;
    uint4 i0 = make_uint4(0, 0, 0, 0), i1 = i0, m0 = i0, m1 = i0;
    Agent s{};
    // every independent load first, no result used before the last is issued (a wave waits for
    // its loads in issue order): one round trip, then the scenario row
    if (live) {
      st = v.state[slot];
      i0 = v.inv[2 * slot];
      i1 = v.inv[2 * slot + 1];
      m0 = v.mask[2 * slot];
      m1 = v.mask[2 * slot + 1];
      init_word = v.init[slot];
      if (a.actions) act = a.actions[slot];
      if (a.bc) {
        bc = a.bc[slot];
        ref = a.ref[slot];
      }
    }
    // each of these waves copies the tables it reads (identical values); unconditional loads
    // within the tables' allocations, in the same round trip
    const uint32_t tw = v.task_tab[lane];
    const uint32_t rw = v.rcw[min(lane, CRAFT_MAX_RECIPES * 3 - 1)];
    int32_t sw[CRAFT_MAX_TASKS * CRAFT_MAX_SUBTASKS / 64];
#pragma unroll
    for (int q = 0; q < CRAFT_MAX_TASKS * CRAFT_MAX_SUBTASKS / 64; ++q) sw[q] = TL > 0 ? v.task_sub[lane + 64 * q] : 0;
    if (lane < v.n_tasks) s_task[lane] = (uint16_t)tw;
    if (lane < CRAFT_MAX_RECIPES * 3) s_rc[lane] = rw;
    if (v.wsr) {                                                          // (each A + C wave its own copy)
      const uint2 ww0 = v.wsr[lane], ww1 = v.wsr[lane + 64];
      s_wsr[lane] = ww0;
      s_wsr[lane + 64] = ww1;
    }
    if (j == 0 && lane < 3) s_wctl[lane] = 0u;                            // (before the barrier)
    if (TL > 0) {
#pragma unroll
      for (int q = 0; q < CRAFT_MAX_TASKS * CRAFT_MAX_SUBTASKS / 64; ++q)
        if (lane + 64 * q < v.n_tasks * CRAFT_MAX_SUBTASKS) s_tsub[lane + 64 * q] = sw[q];
    }
    if (live) {
      if (!a.actions) {
        const uint64_t gid = (uint64_t)(v.env_base + slot);
        act = (int)((uint32_t)(splitmix64(a.seed ^ (gid << 20) ^ (uint64_t)a.tick) >> 32) % 6u);
      }
      asm volatile("" : "+v"(bc), "+v"(ref));                          // (no early wait on the flag)
      if (a.bc && (bc & 0xffu)) act = ref;                             // behaviour cloning, imitation.py:56-57
      s = unpack_state(st);
      if (s.x < 1 || s.x > v.W - 2 || s.y < 1 || s.y > v.H - 2 || s.scen >= v.pool_count) {
        latch_error(v.err, CRAFT_EINVAL, slot);                          // never initialised
        live = false;
      }
    }
    if (j == 0) T2S(-1, 1);
    uint8_t* g = s_grid + le * GS;
    uint32_t conn = 0, tcw0 = ~0u, tcw1 = ~0u;   // the teacher: connected row, its listed clearable cells
    if (TL > 0 && live) {
      conn = v.pool_conn[s.scen];
      if (v.ttab) {
        tcw0 = v.tt_cells[2 * (size_t)s.scen];
        tcw1 = v.tt_cells[2 * (size_t)s.scen + 1];
      }
    }
    if (live) {
      const uint4* src = reinterpret_cast<const uint4*>(v.pool + (size_t)s.scen * v.CS);
      uint32_t* dst = reinterpret_cast<uint32_t*>(g);
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
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (j == 0) T2S(1, 2);

    uint32_t* ivw = reinterpret_cast<uint32_t*>(s_inv + le * kInvStride);
    uint8_t* iv = s_inv + le * kInvStride;
    uint32_t m[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
    ivw[0] = i0.x; ivw[1] = i0.y; ivw[2] = i0.z; ivw[3] = i0.w;
    ivw[4] = i1.x; ivw[5] = i1.y; ivw[6] = i1.z; ivw[7] = i1.w;
    bool inv_changed = false, mask_changed = false;
    int d = 0, succ = -1, counted = 0;
    int code = -1;
    if (live) {
      // per-env body of ImitationTrainer.do_rollout, trainers/imitation.py:59-73
      bool restart = false;
      if (s.frozen) {
        d = 1;
      } else {
        counted = 1;
        s.timer -= 1;
        d = (act == CRAFT_STOP) || s.timer <= 0;
        restart = d && (a.flags & CRAFT_STEP_AUTORESET);
      }
      if (d) {                                                           // satisfies() of the pre-step state
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
      if (!restart) {
#pragma unroll
        for (int w = 0; w < 8; ++w) {                                    // cells cleared this episode
          uint32_t mm = m[w];
          while (mm) {
            g[w * 32 + __ffs(mm) - 1] = 0;
            mm &= mm - 1;
          }
        }
      }
      if (j == 0) T2S(-1, 3);
      if (restart) {                                                     // CraftScenario.init, craft.py:268-273
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
          if (v.wsr) transition<true, true>(v, s_rc, g, iv, s, m, act, inv_changed, mask_changed, rw, slot, s_wsr);
          else transition<true>(v, s_rc, g, iv, s, m, act, inv_changed, mask_changed, rw, slot);
          code = transition_code(ox, oy, s, inv_changed);
        }
      }
      if (j == 0) T2S(-1, 4);
      v.state[slot] = pack_state(s);
      if (inv_changed) {
        v.inv[2 * slot] = make_uint4(ivw[0], ivw[1], ivw[2], ivw[3]);
        v.inv[2 * slot + 1] = make_uint4(ivw[4], ivw[5], ivw[6], ivw[7]);
      }
      if (mask_changed) {
        v.mask[2 * slot] = make_uint4(m[0], m[1], m[2], m[3]);
        v.mask[2 * slot + 1] = make_uint4(m[4], m[5], m[6], m[7]);
      }
      if (a.done) a.done[slot] = (uint8_t)d;
      if (a.sat) a.sat[slot] = (int8_t)succ;
      if (a.reward) a.reward[slot] = (counted && d && succ == 1) ? 1.0f : 0.0f;
      if (a.rec) a.rec[slot] = counted ? act : -1;                       // action_seqs, imitation.py:59-61
    }
    if (j == 0) T2S(-1, 5);
    if (a.code && lane < nE) a.code[slot] = (int8_t)code;
    s_agent[le] = live ? ((uint32_t)s.x | ((uint32_t)s.y << 8) | ((uint32_t)s.dir << 16) | (1u << 24)) : 0u;
    // the teacher's inputs: task | frozen << 8 | scenario connected << 9 | the teacher table has
    // this grid (craft_teach.h) << 10 | its table row << 11 (< 2^21 when the table is on).  The row
    // holds this episode's clears (none after a restart): cleared listed cells read 0
    if (TL > 0) {
      int ncl = 0;
#pragma unroll
      for (int w = 0; w < 8; ++w) ncl += __popc(m[w]);
      const int trow = live ? tt_index(v, s.scen, tcw0, tcw1, ncl, [&](int c) { return g[c] == 0; }) : -1;
      s_tinfo[le] = (uint32_t)s.task | ((uint32_t)s.frozen << 8) | (conn << 9) |
                    (trow >= 0 ? (1u << 10) | ((uint32_t)trow << 11) : 0u);
    }
    // episode statistics: the partial-sum row of this 64-env tile (uncontended)
    const uint64_t bs = __ballot(live && counted && d && succ == 1);
    const uint64_t be = __ballot(live && counted && d);
    const uint64_t bt = __ballot(live && counted);
    const uint64_t bl = __ballot(live && counted && !d);
    if (lane == 0 && nE > 0) {   // no-return atomics
      unsigned long long* r =
          reinterpret_cast<unsigned long long*>(v.stats_part + 4 * ((int64_t)blockIdx.x * J + j));
      atomicAdd(r + 0, (unsigned long long)__popcll(bs));
      atomicAdd(r + 1, (unsigned long long)__popcll(be));
      atomicAdd(r + 2, (unsigned long long)__popcll(bt));
      if (a.any_live && bl) *a.any_live = 1;                             // idempotent plain store
    }
    if (j == 0) T2S(2, 6);
  } else if (want_obs && wave < kTick2Waves) {
    // waves J..3: zero the observation rows of every wave that streams
    uint4* z = reinterpret_cast<uint4*>(smem + lay.obs);
    const int n16 = (NBUF * obs_w) >> 4;
    for (int i = tid - 64 * J; i < n16; i += 64 * (kTick2Waves - J)) z[i] = make_uint4(0, 0, 0, 0);
  }
  if (TL == 0 && !want_obs) return;                                      // no barrier follows
  __syncthreads();
  T2S(3, -1);

  // ---- D + E in chunks of 16 envs of a tile (chunk c: tile c / TW, envs (c % TW) * 16 ..),
  // claimed in order from an LDS counter by whichever wave is free, into its own LDS rows
  auto run_chunks = [&](uint8_t* s_obsw) {
#pragma unroll 1
    for (;;) {
      uint32_t c = 0;
      if (lane == 0) c = __hip_atomic_fetch_add(&s_wctl[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      c = __builtin_amdgcn_readfirstlane(c);
      if (c >= (uint32_t)(J * kTick2Waves)) break;
      const int j = (int)c / kTick2Waves, sl = (int)c % kTick2Waves;
      const int e0 = j * kTick2Tile + sl * kTick2Sub;                   // first env (workgroup index)
      const int nEw = min(kTick2Sub, tile_envs(j) - sl * kTick2Sub);
      if (nEw <= 0) continue;
      scatter_features<WIN, kTick2Sub, 64>(v, s_grid + e0 * GS, s_inv + e0 * kInvStride, s_agent + e0,
                                           s_obsw, nEw, lane);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#if defined(CRAFT_STAMPS) && !defined(CRAFT_STAMPS_C) && !defined(CRAFT_STAMPS_T)
      if (c == 0 && lane == 0 && v.stamps)                              // chunk 0's wave, any wave
        v.stamps[8 * (int64_t)blockIdx.x + 4] = __builtin_amdgcn_s_memrealtime();
#endif
      switch (v.obs_fmt) {
        case CRAFT_OBS_BF16: stream_obs<CRAFT_OBS_BF16, 64, true, CRAFT_T2_U>(s_obsw, a.obs, envw + e0, F, nEw, v.obs_policy, lane); break;
        case CRAFT_OBS_U8: stream_obs<CRAFT_OBS_U8, 64, true, CRAFT_T2_U>(s_obsw, a.obs, envw + e0, F, nEw, v.obs_policy, lane); break;
        default: stream_obs<CRAFT_OBS_F32, 64, true, CRAFT_T2_U>(s_obsw, a.obs, envw + e0, F, nEw, v.obs_policy, lane); break;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");             // the cleared rows before the next D
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  };

  if (wave < kTick2Waves) {
    if (!want_obs) return;
    run_chunks(smem + lay.obs + wave * obs_w);
    T2SM(5);
#ifdef CRAFT_STAMPS
    if (tid == 0 && v.stamps) {
      uint32_t xcc;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      v.stamps[8 * (int64_t)blockIdx.x + 7] = xcc;
    }
#endif
    return;
  }

  if constexpr (TL > 0) {
    // ---- T: DemonstrationTeacher on each env's new state (teachers/demonstration.py:9-30) from
    // the rows C left in LDS, TL lanes per env, overlapping D + E -----------------------------------
    const int u = tid - 64 * kTick2Waves;
    const int j = u / (kTick2Tile * TL), e = (u % (kTick2Tile * TL)) / TL, ql = u % TL;
    if (e < tile_envs(j)) {
      const int le = j * kTick2Tile + e;
      const int64_t i = envw + le;
      const uint32_t ag = s_agent[le], ti = s_tinfo[le];
      int action = -2;                                                   // a slot C could not run
      if (ag && ((ti >> 8) & 1u)) {
        action = -1;                                                     // frozen: the label of a done env
      } else if (ag) {
#ifdef CRAFT_ABL_NOTEACH
        action = CRAFT_STOP;                                             // ablation build only
      } else if (false) {
#endif
        Agent s{};
        s.x = ag & 0xff; s.y = (ag >> 8) & 0xff; s.dir = (ag >> 16) & 3; s.task = ti & 0xff;
        const uint32_t m0[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        int len = -1, err = 0, defer = -1;
        // the hint walk (and, with tt_fused, the teacher table for a pristine grid); a BFS left
        // over is deferred to the workgroup's dense pass
        action = teach_env<NW, TL, true>(v, s_task, s_tsub, reinterpret_cast<const uint32_t*>(s_grid + le * GS), m0,
                                   s_inv + le * kInvStride, s, s.task, ql, false, len, err,
                                   ((ti >> 9) & 1u) != 0, (v.tt_fused && ((ti >> 10) & 1u)) ? tt_row(v, (int)(ti >> 11)) : nullptr,
                                   &defer, (v.tt_fused && ((ti >> 10) & 1u)) ? tt_row4(v, (int)(ti >> 11)) : nullptr);
        if (err && ql == 0) latch_error(v.err, err, i);
        if (action == kTeachDeferred && ql == 0)
          s_work[__hip_atomic_fetch_add(&s_wctl[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)] =
              (uint32_t)le | ((uint32_t)defer << 8);
      }
      if (ql == 0 && action != kTeachDeferred) a.label[i] = action;
    }
    // every teacher wave has listed its deferred queries; then all of them run the BFS densely
    T2ST(1);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if ((tid & 63) == 0) __hip_atomic_fetch_add(&s_wctl[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    while (__hip_atomic_load(&s_wctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < (uint32_t)(J * TL))
      __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const uint32_t nw = __hip_atomic_load(&s_wctl[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    T2ST(2);
#ifdef CRAFT_STAMPS_T
    if (u == 0 && v.stamps) v.stamps[8 * (int64_t)blockIdx.x + 4] = nw;
#endif
    teach_deferred_dense<NW, TL>(v, s_work, (int)nw, u, J * kTick2Tile * TL, s_grid, GS, s_agent, s_tinfo,
                                 a.label + envw, envw);
    T2SM(6);
    if constexpr (SHARE) {
      // done teaching: take the D + E chunks no tick wave has claimed yet
      if (want_obs) {
        run_chunks(smem + lay.obs + (kTick2Waves + (u >> 6)) * obs_w);
        T2SM(5);
      }
    }
  }
}
#undef T2S
#undef T2SM
#undef T2ST

}  // namespace craft
