// craft_rollout_split.h — craft_rollout for 16- and 32-env tiles: the producer
// work of a tick split over two waves.
//
// Small tiles need their own transition latency chain each, so one wave doing
// both the transition and the scatter cannot keep up.  Here:
//   wave 0        C(j+1): the transitions (one lane per env);
//   wave 1        D(j):   the observation scatter of the item before (64 / TILE
//                         lanes per env) into LDS row buffer j & 1;
//   waves 2..     E(j-1): stream the rows of the item before that to HBM and
//                         clear them.
// One workgroup barrier per interval.  An "item" is one tick of one tile.
//
// Continuous pipeline.  When a launch is one work unit per tile (the default:
// no chunked hand-offs), a workgroup's items are all ticks of its first tile,
// then all ticks of its next tile, ... (tiles b, b + G, b + 2G for workgroup b
// of G), and the pipeline runs straight through tile changes: in the interval
// where D and E still work on the previous tile's last ticks, wave 0 publishes
// that tile's state, loads the next tile and runs its first tick.  The pipeline
// fills once and drains once per launch instead of once per tile
// (the launch's fixed cost).  Chunked launches (craft_sim_tune_rollout
// chunk > 0) keep one fill and drain per unit, because a unit may have to wait
// for its tile's previous chunk on another workgroup.
//
// Parity.  C(j+1) and D(j) run at the same time, so the env state is
// double-buffered by item parity: grid rows and inventory rows of item j live in
// buffer j & 1.  A tick changes at most one cell per env (grab, bridge, axe) or
// restarts the episode, recorded in `chg`; C(j+1) first brings its buffer (two
// items old) up to date from that record and copies the inventory, then runs the
// tick.  A freshly loaded tile fills only its first item's buffer; its second
// item copies the whole row across.  Everything else (outputs, statistics) is as
// in craft_rollout.h, and the results are identical (the same tests run both
// kernels).
#pragma once
#include <type_traits>

#include "craft_obs.h"

namespace craft {

// LDS carve: grid rows [2][TILE][GS] | pristine rows [TILE][GS] | observation
// rows [2][up16(TILE*F)] | inventory rows [2][TILE][36] | agent words [2][TILE] |
// task table [64] u16 | recipe words [16][3] | control words [4] | item words [4][2] |
// output words [4][TILE] | next-tile staging: state [TILE] u64, init [TILE] u32,
// inventory and mask [TILE][32 B] each, pool rows [TILE][CS].
// (+ the publish outbox: state [TILE] u64, mask [TILE][8] u32)
__host__ __device__ inline int split_stage_bytes(int tile, int CS) { return tile * (8 + 4 + 64) + tile * CS + tile * 40; }
// (the staging area and the outbox are the continuous pipeline's only: `flat`)
__host__ __device__ inline int split_lds_bytes(int tile, int GS, int F, int CS, bool flat) {
  auto up16 = [](int x) { return (x + 15) & ~15; };
  return up16(3 * tile * GS) + 2 * up16(tile * F) + 2 * tile * kInvStride + 2 * tile * 4 +
         CRAFT_MAX_TASKS * 2 + CRAFT_MAX_RECIPES * 12 + 16 + 32 + 4 * tile * 4 +
         (flat ? split_stage_bytes(tile, CS) : 0);
}

// FLAT: the continuous pipeline (one unit per tile, observations on: RolloutArgs.flat);
// otherwise work units from the queue.  Separate instantiations, so that neither path's
// registers count against the other.
template <int WIN, int TILE, int NT, int FMT, int WPE, bool GIVEN, bool FLAT = false>
__global__ __launch_bounds__(NT, WPE) void rollout_split_kernel(SimView v, RolloutArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  static_assert(NT >= 192 && TILE <= 64, "a producer, a scatter wave and at least one streaming wave");
  constexpr int P = 64 / TILE;                            // scatter lanes per env
  auto up16 = [](int x) { return (x + 15) & ~15; };
  const int GS = v.GS, F = v.F;
  // the recipe words in a VGPR (lane w: word w), loaded while every lane is active, for the
  // transition's recipe loop (v_readlane instead of an LDS round trip per recipe)
  const uint32_t rcv = v.rcw[min((int)(threadIdx.x & 63), CRAFT_MAX_RECIPES * 3 - 1)];
  uint8_t* s_grid = smem;                                 // [2][TILE][GS] by item parity
  uint8_t* s_pristine = smem + 2 * TILE * GS;             // [TILE][GS] pool[scenario]
  const int obs_buf = up16(TILE * F);
  uint8_t* s_obs = smem + up16(3 * TILE * GS);            // [2][obs_buf]
  uint8_t* s_inv = s_obs + 2 * obs_buf;                   // [2][TILE][kInvStride]
  uint32_t* s_agent = reinterpret_cast<uint32_t*>(s_inv + 2 * TILE * kInvStride);   // [2][TILE]
  uint16_t* s_task = reinterpret_cast<uint16_t*>(s_agent + 2 * TILE);
  uint32_t* s_rc = reinterpret_cast<uint32_t*>(s_task + CRAFT_MAX_TASKS);
  uint32_t* s_ctrl = s_rc + CRAFT_MAX_RECIPES * 3;
  uint32_t* s_item = s_ctrl + 4;                          // [4][2]: item j -> {tile + 1 (0 = none), tick}
  // [4][TILE] by item & 3: done | success << 8 | reward << 16 | 1 << 24.  Four, not two: the
  // streaming waves store item j's outputs two intervals after C wrote them, while C writes
  // item j + 2's
  uint32_t* s_out = s_item + 8;
  uint8_t* s_stage = reinterpret_cast<uint8_t*>(s_out + 4 * TILE);   // 16-byte aligned (TILE % 4 == 0)

  const int tid = threadIdx.x;
  const int64_t n = v.n_envs;
  const bool want_obs = a.obs != nullptr;
  constexpr int esz = FMT == CRAFT_OBS_F32 ? 4 : (FMT == CRAFT_OBS_BF16 ? 2 : 1);
  const int n_tiles = (int)((n + TILE - 1) / TILE);
  const int n_chunks = (a.n_ticks + a.chunk - 1) / a.chunk;
  const uint32_t n_units = (uint32_t)n_tiles * (uint32_t)n_chunks;

  // wave 0, one lane per env (see craft_rollout.h for st / init_word / task_word / clr)
  Agent s{};
  uint64_t st = 0;
  uint32_t init_word = 0, task_word = 0;
  uint32_t clr = 0;          // cells cleared this episode (<= 3 ids, count, bit 31 = more)
  uint32_t clr_prev = 0;     // the episode's clears before a restart (for the other buffer)
  uint32_t chg = 0;          // what the last C did to its buffer: 0 nothing, 1 + cell cleared, kRestart
  constexpr uint32_t kRestart = 0x80000000u;
  int sync = 0;              // how C brings its buffer up to date: 0 loaded, 1 whole copy, 2 from chg
  bool live = false;
  int64_t slot = 0;
  const uint32_t* pw = reinterpret_cast<const uint32_t*>(s_pristine + tid * GS);
  const uint8_t* pr = s_pristine + tid * GS;
  auto grid_of = [&](int p) __attribute__((always_inline)) { return s_grid + (p & 1) * TILE * GS + tid * GS; };
  auto inv_of = [&](int p) __attribute__((always_inline)) { return s_inv + (p & 1) * TILE * kInvStride + tid * kInvStride; };
  uint32_t n_succ = 0, n_end = 0, n_step = 0;

  // restore the cells of `cl` (or the whole row) of grid row g from the pristine row
  auto restore = [&](uint8_t* g, uint32_t cl) __attribute__((always_inline)) {
    if (cl >> 31) {
      uint32_t* gw = reinterpret_cast<uint32_t*>(g);
      for (int q0 = 0; q0 < (v.CS >> 2); q0 += 12) {
        uint32_t w[12];
#pragma unroll
        for (int j = 0; j < 12; ++j) w[j] = q0 + j < (v.CS >> 2) ? pw[q0 + j] : 0u;
#pragma unroll
        for (int j = 0; j < 12; ++j)
          if (q0 + j < (v.CS >> 2)) gw[q0 + j] = w[j];
      }
    } else {
      const int nc = (cl >> 24) & 3;
#pragma unroll
      for (int i = 0; i < 3; ++i)
        if (i < nc) {
          const int c = (cl >> (8 * i)) & 0xff;
          g[c] = pr[c];
        }
    }
  };

  // ---- C: tick k on buffer p & 1 (trainers/imitation.py:59-73); p = the item index --------------
  auto tick_c = [&](int k, int p, bool lds_out) __attribute__((always_inline)) {
    const int64_t tick = a.tick0 + k;
    const int64_t r = tick % a.ring;
    int d = 0, succ = -1, counted = 0;
    uint8_t* g = grid_of(p);
    uint8_t* iv = inv_of(p);
    s = unpack_state(st);
    if (live) {
      // bring this buffer up to the other buffer's state: whole row after a load, else its last change
      if (sync == 1) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(grid_of(p ^ 1));
        uint32_t* gw = reinterpret_cast<uint32_t*>(g);
        for (int q0 = 0; q0 < (v.CS >> 2); q0 += 12) {
          uint32_t w[12];
#pragma unroll
          for (int j = 0; j < 12; ++j) w[j] = q0 + j < (v.CS >> 2) ? src[q0 + j] : 0u;
#pragma unroll
          for (int j = 0; j < 12; ++j)
            if (q0 + j < (v.CS >> 2)) gw[q0 + j] = w[j];
        }
      } else if (sync == 2) {
        if (chg == kRestart) restore(g, clr_prev);
        else if (chg) g[chg - 1] = 0;
      }
      if (sync) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(inv_of(p ^ 1));
        uint32_t w[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) w[i] = src[i];
#pragma unroll
        for (int i = 0; i < 8; ++i) reinterpret_cast<uint32_t*>(iv)[i] = w[i];
      }
      sync = sync ? 2 : 1;
      chg = 0;
      int act;
      if (GIVEN) {
        act = a.actions[(int64_t)k * n + slot];
      } else {
        const uint64_t gid = (uint64_t)(v.env_base + slot);
        act = (int)((uint32_t)(splitmix64(a.seed ^ (gid << 20) ^ (uint64_t)tick) >> 32) % 6u);
      }
      bool restart = false;
      if (s.frozen) {
        d = 1;
      } else {
        counted = 1;
        s.timer -= 1;
        d = (act == CRAFT_STOP) || s.timer <= 0;
        restart = d && (a.flags & CRAFT_STEP_AUTORESET);
      }
      if (d) {                                          // satisfies() of the pre-step state
        const int goal = task_word & 0xf, arg = (task_word >> 4) & 0xff;
        const int fc = (s.x + dir_dx(s.dir)) * v.H + (s.y + dir_dy(s.dir));
        if (goal == CRAFT_GOAL_GET || goal == CRAFT_GOAL_MAKE) succ = iv[arg] > 0;
        else if (goal == CRAFT_GOAL_GO) succ = (int)g[fc] == arg;
        else succ = -1;
      }
      if (restart) {                                    // CraftScenario.init, craft.py:268-273
        s.x = init_word & 0xff; s.y = (init_word >> 8) & 0xff; s.dir = (init_word >> 16) & 3;
        s.timer = v.maxT;
#pragma unroll
        for (int w = 0; w < 8; ++w) reinterpret_cast<uint32_t*>(iv)[w] = 0u;
        restore(g, clr);
        clr_prev = clr;
        clr = 0;
        chg = kRestart;
      } else if (d && !s.frozen) {
        s.frozen = 1;
        s.timer = max(s.timer, 0);
      }
      if (!d) {
        bool inv_changed = false, mask_changed = false;
        uint32_t m_unused[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const int fc = (s.x + dir_dx(s.dir)) * v.H + (s.y + dir_dy(s.dir));   // what USE clears
#ifndef CRAFT_ABL_NOTRANS
        if (act < 0 || act >= CRAFT_N_ACTIONS) latch_error(v.err, CRAFT_EBADACTION, slot);
        else transition<true>(v, s_rc, g, iv, s, m_unused, act, inv_changed, mask_changed, rcv, slot);
#endif
        if (mask_changed) {
          chg = 1u + (uint32_t)fc;
          const uint32_t nc = (clr >> 24) & 3;
          clr = (clr >> 31) ? clr
              : nc < 3 ? ((clr & 0x00ffffffu) | ((uint32_t)fc << (8 * nc)) | ((nc + 1) << 24)) : (1u << 31);
        }
      }
      st = pack_state(s);
      if (lds_out) {                                    // stored by the streaming waves with E
        s_out[(p & 3) * TILE + tid] = (uint32_t)(uint8_t)d | ((uint32_t)(uint8_t)(int8_t)succ << 8) |
                                      ((uint32_t)(counted && d && succ == 1) << 16) | (1u << 24);
      } else {
        const int64_t o = r * n + slot;
        if (a.done) a.done[o] = (uint8_t)d;
        if (a.sat) a.sat[o] = (int8_t)succ;
        if (a.reward) a.reward[o] = (counted && d && succ == 1) ? 1.0f : 0.0f;
      }
    } else if (lds_out && tid < TILE) {
      s_out[(p & 3) * TILE + tid] = 0u;
    }
    const uint64_t bs = __ballot(live && counted && d && succ == 1);
    const uint64_t be = __ballot(live && counted && d);
    const uint64_t bt = __ballot(live && counted);
    n_succ += (uint32_t)__popcll(bs);
    n_end += (uint32_t)__popcll(be);
    n_step += (uint32_t)__popcll(bt);
    s_agent[(p & 1) * TILE + tid] =
        live ? ((uint32_t)s.x | ((uint32_t)s.y << 8) | ((uint32_t)s.dir << 16) | (1u << 24)) : 0u;
  };

  // ---- A: lanes < TILE of wave 0 take over tile t into buffer p (state, pool row, clears) -----
  // next-tile staging (flat pipeline): state, init, inventory, mask, pool rows, filled by LDS-DMA
  uint64_t* sg_state = reinterpret_cast<uint64_t*>(s_stage);
  uint32_t* sg_init = reinterpret_cast<uint32_t*>(s_stage + TILE * 8);
  uint4* sg_inv = reinterpret_cast<uint4*>(s_stage + TILE * 12);
  uint4* sg_mask = reinterpret_cast<uint4*>(s_stage + TILE * 44);
  uint8_t* sg_pool = s_stage + TILE * 76;
  uint64_t* ob_state = reinterpret_cast<uint64_t*>(sg_pool + TILE * v.CS);   // publish outbox
  uint32_t* ob_mask = reinterpret_cast<uint32_t*>(ob_state + TILE);

  // STAGED (std::true_type / std::false_type): read the tile from the staging area (LDS) or
  // from HBM -- two instantiations, so the compiler emits ds_read or global_load, never a
  // flat load through a selected pointer
  auto load_tile = [&](int t, int p, auto STAGED) __attribute__((always_inline)) {
    constexpr bool staged = decltype(STAGED)::value;
    const int64_t env0 = (int64_t)t * TILE;
    const int nE = (int)min((int64_t)TILE, n - env0);
    slot = env0 + tid;
    live = tid < nE;
    uint32_t m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t ivr[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (live) {
      uint4 i0, i1, m0, m1;
      if constexpr (staged) {
        st = sg_state[tid];
        init_word = sg_init[tid];
        i0 = sg_inv[2 * tid]; i1 = sg_inv[2 * tid + 1];
        m0 = sg_mask[2 * tid]; m1 = sg_mask[2 * tid + 1];
      } else {
        st = v.state[slot];
        init_word = v.init[slot];
        i0 = v.inv[2 * slot]; i1 = v.inv[2 * slot + 1];
        m0 = v.mask[2 * slot]; m1 = v.mask[2 * slot + 1];
      }
      ivr[0] = i0.x; ivr[1] = i0.y; ivr[2] = i0.z; ivr[3] = i0.w;
      ivr[4] = i1.x; ivr[5] = i1.y; ivr[6] = i1.z; ivr[7] = i1.w;
      m[0] = m0.x; m[1] = m0.y; m[2] = m0.z; m[3] = m0.w;
      m[4] = m1.x; m[5] = m1.y; m[6] = m1.z; m[7] = m1.w;
      s = unpack_state(st);
      if (s.x < 1 || s.x > v.W - 2 || s.y < 1 || s.y > v.H - 2 || s.scen >= v.pool_count) {
        latch_error(v.err, CRAFT_EINVAL, slot);
        live = false;
      }
    }
    chg = 0;
    clr = 0;
    clr_prev = 0;
    sync = 0;
    if (live) {
      task_word = s_task[s.task];
      // pool[scenario] -> the pristine row and grid buffer p; inventory -> buffer p
      uint32_t* g0 = reinterpret_cast<uint32_t*>(grid_of(p));
      uint32_t* pwm = reinterpret_cast<uint32_t*>(s_pristine + tid * GS);
      const uint4* gsrc = reinterpret_cast<const uint4*>(v.pool + (size_t)s.scen * v.CS);
      const uint4* lsrc = reinterpret_cast<const uint4*>(sg_pool + tid * v.CS);
      const int nchunk = v.CS >> 4;
      if constexpr (staged) {                           // LDS -> LDS, one 16-byte chunk at a time
        for (int q0 = 0; q0 < nchunk; ++q0) {
          const uint4 c = lsrc[q0];
          const int q = 4 * q0;
          pwm[q + 0] = g0[q + 0] = c.x;
          pwm[q + 1] = g0[q + 1] = c.y;
          pwm[q + 2] = g0[q + 2] = c.z;
          pwm[q + 3] = g0[q + 3] = c.w;
        }
      } else {                                          // HBM / L2: four chunks in flight
        for (int q0 = 0; q0 < nchunk; q0 += 4) {
          uint4 cq[4];
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (q0 + j < nchunk) cq[j] = gsrc[q0 + j];
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (q0 + j < nchunk) {
              const int q = 4 * (q0 + j);
              pwm[q + 0] = g0[q + 0] = cq[j].x;
              pwm[q + 1] = g0[q + 1] = cq[j].y;
              pwm[q + 2] = g0[q + 2] = cq[j].z;
              pwm[q + 3] = g0[q + 3] = cq[j].w;
            }
        }
      }
      uint32_t* iv0 = reinterpret_cast<uint32_t*>(inv_of(p));
#pragma unroll
      for (int i = 0; i < 8; ++i) iv0[i] = ivr[i];
      uint8_t* b0 = grid_of(p);
#pragma unroll
      for (int w = 0; w < 8; ++w) {                     // cells cleared this episode
        uint32_t mm = m[w];
        while (mm) {
          const int cc = w * 32 + __ffs(mm) - 1;
          b0[cc] = 0;
          const uint32_t nc = (clr >> 24) & 3;
          clr = (clr >> 31) ? clr
              : nc < 3 ? ((clr & 0x00ffffffu) | ((uint32_t)cc << (8 * nc)) | ((nc + 1) << 24)) : (1u << 31);
          mm &= mm - 1;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };

  // ---- the tile's state back to HBM from buffer p (its last item); the mask is rebuilt from
  // the rows: cells are only ever cleared, so mask = {c : pristine[c] != 0 and grid[c] == 0} ---
  // cleared = pristine byte nonzero and current byte zero, 4 cells per word (SWAR); fully
  // unrolled so every mask word index is static
  auto cleared_mask = [&](int p, uint32_t (&m)[8]) __attribute__((always_inline)) {
    const uint32_t* gw = reinterpret_cast<const uint32_t*>(grid_of(p));
#pragma unroll
    for (int i = 0; i < 8; ++i) m[i] = 0u;
#pragma unroll
    for (int q = 0; q < CRAFT_MAX_CELLS / 4; ++q)
      if (q < (v.C + 3) >> 2)
        m[q >> 3] |= byte_tops(nonzero_bytes(pw[q]) & zero_bytes(gw[q])) << (4 * (q & 7));
  };
  auto publish = [&](int p, bool sc1) __attribute__((always_inline)) {
    const uint32_t* ivw = reinterpret_cast<const uint32_t*>(inv_of(p));
    uint32_t m[8];
    cleared_mask(p, m);
    if (sc1) {
      // write-through (sc1) stores: the hand-off form of MI355X_MICROARCH.md "Valid forms"
      // ({sc1 stores} -> every storing wave's s_waitcnt vmcnt(0) -> one lane's flag)
      typedef unsigned int u4v __attribute__((ext_vector_type(4)));
      const __amdgpu_buffer_rsrc_t inv_r = __builtin_amdgcn_make_buffer_rsrc(v.inv, 0, 0x7fffffff, 0x00020000);
      const __amdgpu_buffer_rsrc_t msk_r = __builtin_amdgcn_make_buffer_rsrc(v.mask, 0, 0x7fffffff, 0x00020000);
      const int off = (int)(slot * 32);
      __hip_atomic_store((gu64*)(v.state + slot), (unsigned long long)st, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_raw_buffer_store_b128(u4v{ivw[0], ivw[1], ivw[2], ivw[3]}, inv_r, off, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b128(u4v{ivw[4], ivw[5], ivw[6], ivw[7]}, inv_r, off + 16, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b128(u4v{m[0], m[1], m[2], m[3]}, msk_r, off, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b128(u4v{m[4], m[5], m[6], m[7]}, msk_r, off + 16, 0, 16);
    } else {
      v.state[slot] = st;
      v.inv[2 * slot] = make_uint4(ivw[0], ivw[1], ivw[2], ivw[3]);
      v.inv[2 * slot + 1] = make_uint4(ivw[4], ivw[5], ivw[6], ivw[7]);
      v.mask[2 * slot] = make_uint4(m[0], m[1], m[2], m[3]);
      v.mask[2 * slot + 1] = make_uint4(m[4], m[5], m[6], m[7]);
    }
  };

  // ---- D on wave 1: lane l scatters part l / TILE of env l % TILE of the item in buffer p ----
  auto scatter_d = [&](int p, int nE) __attribute__((always_inline)) {
    const int l = tid - 64, e = l % TILE;
    const uint32_t ag = s_agent[(p & 1) * TILE + e];
#ifdef CRAFT_ABL_NOD
    if (false)
#else
    if (e < nE && ag)
#endif
      scatter_env_part<WIN, P>(v, s_grid + (p & 1) * TILE * GS + e * GS,
                               s_inv + (p & 1) * TILE * kInvStride + e * kInvStride, ag,
                               s_obs + (p & 1) * obs_buf + e * F, l / TILE);
  };

  // ---- E on waves 2..: stream tick k of tile t from buffer p to its ring slot ------------------
  auto stream_e = [&](int p, int t, int k, bool outs) __attribute__((always_inline)) {
    const int64_t env0 = (int64_t)t * TILE;
    const int nE = (int)min((int64_t)TILE, n - env0);
    const int64_t r = (a.tick0 + k) % a.ring;
    if (outs && tid - 128 < nE) {                       // the tick's done / success / reward (flat pipeline)
      const uint32_t w = s_out[(p & 3) * TILE + tid - 128];
      if (w >> 24) {
        const int64_t o = r * n + env0 + (tid - 128);
        if (a.done) a.done[o] = (uint8_t)(w & 0xffu);
        if (a.sat) a.sat[o] = (int8_t)((w >> 8) & 0xffu);
        if (a.reward) a.reward[o] = ((w >> 16) & 1u) ? 1.0f : 0.0f;
      }
    }
    void* out = static_cast<uint8_t*>(a.obs) + r * n * (int64_t)F * esz;
#ifndef CRAFT_ABL_NOE
    stream_obs<FMT, NT - 128, true>(s_obs + (p & 1) * obs_buf, out, env0, F, nE, v.obs_policy, tid - 128);
#else
    (void)out;
    (void)nE;
#endif
  };

  // ---- once per workgroup: task table, cleared observation rows --------------------------------
  for (int t = tid; t < v.n_tasks; t += NT) s_task[t] = v.task_tab[t];
  for (int t = tid; t < CRAFT_MAX_RECIPES * 3; t += NT) s_rc[t] = v.rcw[t];
  if (want_obs) {
    uint4* z = reinterpret_cast<uint4*>(s_obs);
    for (int i = tid; i < (2 * obs_buf >> 4); i += NT) z[i] = make_uint4(0, 0, 0, 0);
  }

  if constexpr (FLAT) {
    // ---- continuous pipeline: tiles b, b + G, ... of this workgroup, all ticks each ----------
#ifdef CRAFT_STAMPS
    // diagnostic build only: per-role totals in s_memrealtime ticks (10 ns) -> stamps[block][16]:
    // 0 start, 1 wave 0 in produce, 2 wave 0 at the barrier, 3 wave 1 in D, 4 wave 1 at the
    // barrier, 5 wave 2 in E, 6 end, 7 wave 0 in tile switches, of which 8 the prefetch wait,
    // 9 publish, 10 load; 11 issuing the prefetch
    unsigned long long t_beg = __builtin_amdgcn_s_memrealtime();
#define SPLIT_NOW() __builtin_amdgcn_s_memrealtime()
#else
#define SPLIT_NOW() 0ull
#endif
    unsigned long long acc_work = 0, acc_wait = 0, acc_sw = 0, acc_pub = 0, acc_vm = 0, acc_ld = 0, acc_dma = 0;
    // wave-uniform state of wave 0: the tile in progress (-1 none yet, -2 none left), its next tick
    int cur_t = -1, cur_k = 0;
    // The next tile's state and pool rows are fetched ahead by LDS-DMA into a staging area
    // (wave 0 issues no other global loads or per-tick stores, so its vmcnt counts only these
    // and its tile claims), and a tile switch reads LDS instead of waiting out an HBM round
    // trip behind the write stream (a load waits behind the stores already queued in the CU's
    // memory pipeline).  Partial tiles load directly.
    bool staged = false;                                // the staging area holds the next tile
    auto stage_state = [&](int t2) __attribute__((always_inline)) {
      const int64_t e0 = (int64_t)t2 * TILE;
      const int l = tid;                                // 64 lanes, 16 bytes each
      typedef __attribute__((address_space(1))) void* gp;
      typedef __attribute__((address_space(3))) void* lp;
      if (l < TILE / 2) __builtin_amdgcn_global_load_lds((gp)(v.state + e0 + 2 * l), (lp)sg_state, 16, 0, 0);
      if (l < TILE / 4) __builtin_amdgcn_global_load_lds((gp)(v.init + e0 + 4 * l), (lp)sg_init, 16, 0, 0);
#pragma unroll
      for (int h = 0; h < 2 * TILE; h += 64) {
        __builtin_amdgcn_global_load_lds((gp)(v.inv + 2 * e0 + h + l), (lp)(sg_inv + h), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((gp)(v.mask + 2 * e0 + h + l), (lp)(sg_mask + h), 16, 0, 0);
      }
    };
    auto stage_pool = [&]() __attribute__((always_inline)) {
      typedef __attribute__((address_space(1))) void* gp;
      typedef __attribute__((address_space(3))) void* lp;
      const int per = v.CS >> 4;                        // 16-byte chunks per pool row
      int e = tid / per, c = tid - (tid / per) * per;   // chunk f = f0 + tid is (e, c)
      const int de = 64 / per, dc = 64 - (64 / per) * per;
      for (int f0 = 0; f0 < TILE * per; f0 += 64) {
        const int f = f0 + tid;
        if (f < TILE * per) {
          const int scen = (int)((sg_state[e] >> 32) & 0xffffffu) % max(1, v.pool_count);
          __builtin_amdgcn_global_load_lds((gp)(v.pool + (size_t)scen * v.CS + 16 * c), (lp)(sg_pool + 16 * f0),
                                           16, 0, 0);
        }
        e += de;                                        // advance (e, c) by 64 chunks
        c += dc;
        if (c >= per) { c -= per; ++e; }
      }
    };
    // Tiles come from the queue counter (a.queue - a.qbase = tiles handed out in this launch),
    // so a workgroup that runs slow takes fewer.  The next tile is claimed late, kF = 6 ticks
    // before the switch (claiming it earlier would hand the launch's last tiles to whichever
    // workgroups asked first, not to those that free up first); its id is read two ticks
    // later (an atomic's return waits behind the CU's queued stores), its state words are
    // fetched then, its pool rows one tick after that.  Every workgroup
    // makes exactly one fetch past the last tile, so a launch advances the counter by
    // n_tiles + gridDim.x and the host keeps qbase without re-zeroing the counter.
    auto fetch_now = [&]() __attribute__((always_inline)) -> int {
      unsigned long long r = 0;
      if (tid == 0) r = atomicAdd(a.queue, 1ull);
      const uint32_t d = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)r) - (uint32_t)a.qbase;
      return d < (uint32_t)n_tiles ? (int)d : -1;       // (a launch hands out < 2^32 units: low words)
    };
    const int K = a.n_ticks;
    const int kF = max(0, K - 6), kA = max(0, K - 4), kB = max(0, K - 3);
    uint32_t pend = 0;                                  // lane 0: the claim in flight
    int64_t pub_slot = -1;                              // per lane: a finished env whose state is in the outbox
    int t_next = -1;
    auto produce = [&](int j) __attribute__((always_inline)) {                         // wave 0: item j into buffer j & 1
      if (cur_t != -2 && (cur_t < 0 || cur_k == K)) {
        const unsigned long long s0 = SPLIT_NOW();
        const int t = cur_t == -1 ? fetch_now() : t_next;
        if (staged) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the pool rows have landed
        const unsigned long long s1 = SPLIT_NOW();
        // the finished tile's state goes out AFTER the next one is loaded (its mask, which needs
        // the pristine rows load_tile replaces, waits in an LDS outbox), so that no wait in
        // load_tile also waits out these stores
        const bool pub = cur_t >= 0 && tid < TILE && live;
        const int64_t pslot = slot;
        if (pub) {
          uint32_t m[8];
          cleared_mask((j - 1) & 1, m);
          ob_state[tid] = st;
#pragma unroll
          for (int i = 0; i < 8; ++i) ob_mask[8 * tid + i] = m[i];
        }
        const unsigned long long s2 = SPLIT_NOW();
        if (t >= 0) {
          cur_t = t;
          cur_k = 0;
          if (tid < TILE) {
            if (staged) load_tile(t, j & 1, std::true_type{});
            else load_tile(t, j & 1, std::false_type{});
          }
        } else {
          cur_t = -2;                                   // no tile left: the pipeline drains
        }
        staged = false;
        t_next = -1;
        pub_slot = pub ? pslot : -1;
        const unsigned long long s3 = SPLIT_NOW();
        acc_sw += s3 - s0;
        acc_vm += s1 - s0;
        acc_pub += s2 - s1;
        acc_ld += s3 - s2;
      }
      const bool have = cur_t >= 0;
      if (have) {
        const unsigned long long d0 = SPLIT_NOW();
        if (cur_k == kF && tid == 0) pend = (uint32_t)atomicAdd(a.queue, 1ull);   // claim the next tile
        if (cur_k == kA) {
          const uint32_t d = (uint32_t)__builtin_amdgcn_readfirstlane((int)pend) - (uint32_t)a.qbase;
          t_next = d < (uint32_t)n_tiles ? (int)d : -1;
          if (t_next >= 0 && (int64_t)(t_next + 1) * TILE <= n) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // earlier staging reads are done
            stage_state(t_next);
          }
        }
        if (cur_k == kB && t_next >= 0 && (int64_t)(t_next + 1) * TILE <= n) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the state words have landed
          stage_pool();
          staged = true;
        }
        acc_dma += SPLIT_NOW() - d0;
      }
      if (have && tid < TILE) tick_c(cur_k, j, true);
      if (pub_slot >= 0) {                              // the finished tile's state, last: nothing waits on it
        const uint32_t* ivw = reinterpret_cast<const uint32_t*>(inv_of((j - 1) & 1));
        const uint32_t* mw = ob_mask + 8 * tid;
        v.state[pub_slot] = ob_state[tid];
        v.inv[2 * pub_slot] = make_uint4(ivw[0], ivw[1], ivw[2], ivw[3]);
        v.inv[2 * pub_slot + 1] = make_uint4(ivw[4], ivw[5], ivw[6], ivw[7]);
        v.mask[2 * pub_slot] = make_uint4(mw[0], mw[1], mw[2], mw[3]);
        v.mask[2 * pub_slot + 1] = make_uint4(mw[4], mw[5], mw[6], mw[7]);
        pub_slot = -1;
      }
      if (tid == 0) {
        s_item[2 * (j & 3)] = have ? (uint32_t)cur_t + 1u : 0u;
        s_item[2 * (j & 3) + 1] = (uint32_t)cur_k;
      }
      if (have) ++cur_k;
    };
    // One loop per role with the same barrier count (interval i: C(i+1) | D(i) | E(i-1)), so
    // that each role's loop-carried registers are live in its own loop only.  A plain
    // s_barrier behind each wave's own LDS accesses (the roles hand each other LDS rows
    // only): in a kernel with LDS-DMA the compiler lowers __syncthreads()'s release to
    // s_waitcnt vmcnt(0), so the streaming waves would drain their stores every tick and
    // wave 0 would wait for the next tile's prefetch.
    auto interval_end = [&](int i, unsigned long long w0) __attribute__((always_inline)) -> bool {
      const unsigned long long w1 = SPLIT_NOW();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      acc_work += w1 - w0;
      acc_wait += SPLIT_NOW() - w1;
      return s_item[2 * (i & 3)] == 0;                  // item i does not exist: all work is done
    };
    if (tid < 64) {
      produce(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      for (int i = 0;; ++i) {
        const unsigned long long w0 = SPLIT_NOW();
        produce(i + 1);
        if (interval_end(i, w0)) break;
      }
    } else if (tid < 128) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      for (int i = 0;; ++i) {
        const unsigned long long w0 = SPLIT_NOW();
        const uint32_t t1 = s_item[2 * (i & 3)];
        if (t1) scatter_d(i & 1, (int)min((int64_t)TILE, n - (int64_t)(t1 - 1) * TILE));
        if (interval_end(i, w0)) break;
      }
    } else {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      for (int i = 0;; ++i) {
        const unsigned long long w0 = SPLIT_NOW();
        if (i >= 1) {
          const uint32_t t1 = s_item[2 * ((i - 1) & 3)];
          if (t1) stream_e(i - 1, (int)t1 - 1, (int)s_item[2 * ((i - 1) & 3) + 1], true);
        }
        if (interval_end(i, w0)) break;
      }
    }
#ifdef CRAFT_STAMPS
    if (v.stamps) {
      uint64_t* row = v.stamps + 16 * (int64_t)blockIdx.x;   // 16 words per workgroup
      if (tid == 0) {
        row[0] = t_beg; row[1] = acc_work; row[2] = acc_wait; row[6] = SPLIT_NOW(); row[7] = acc_sw;
        row[8] = acc_vm; row[9] = acc_pub; row[10] = acc_ld; row[11] = acc_dma;
      } else if (tid == 64) {
        row[3] = acc_work; row[4] = acc_wait;
      } else if (tid == 128) {
        row[5] = acc_work;
      }
    }
#endif
    (void)acc_work;
    (void)acc_wait;
    (void)acc_sw;
    (void)acc_pub;
    (void)acc_vm;
    (void)acc_ld;
    (void)acc_dma;
#undef SPLIT_NOW
  } else {
    (void)s_out;
    (void)s_stage;
#ifdef CRAFT_STAMPS
    // diagnostic build only: s_memrealtime (10 ns) per workgroup -> stamps[block][16]: 0 start,
    // 1 + i the claim of its unit i (i < 12), 13 its first unit's first stores issued, 14 units
    // done, 15 end
    uint64_t* srow_t = v.stamps ? v.stamps + 16 * (int64_t)blockIdx.x : nullptr;
    if (tid == 0 && srow_t) srow_t[0] = __builtin_amdgcn_s_memrealtime();
    int n_done = 0;
#endif
    // ---- work units (tile t, chunk c), one pipeline fill and drain each: unit b first (no
    // claim: 512 claims of one counter at the launch's start took up to ~8 us to return),
    // then units gridDim.x + (claims of queue[1]); every workgroup ends with one claim past
    // the last unit, so a launch adds max(units, grid) to queue[1] -------------------------------
    bool first = (uint32_t)blockIdx.x < n_units;
    for (;;) {
      if (tid == 0)
        s_ctrl[0] = first ? (uint32_t)blockIdx.x
                          : (uint32_t)(gridDim.x + (atomicAdd(a.queue + 1, 1ull) - a.qbase1));
      first = false;
      __syncthreads();                                  // also: s_task / rows ready
      const uint32_t u = s_ctrl[0];
#ifdef CRAFT_STAMPS
      if (tid == 0 && srow_t && n_done < 12) srow_t[1 + n_done] = __builtin_amdgcn_s_memrealtime();
#endif
      if (u >= n_units) break;                          // workgroup-uniform exit
      const int t = (int)(u % (uint32_t)n_tiles), c = (int)(u / (uint32_t)n_tiles);
      const int k0 = c * a.chunk, k1 = min(a.n_ticks, k0 + a.chunk);
      const int nq = k1 - k0;
      const int64_t env0 = (int64_t)t * TILE;
      const int nE = (int)min((int64_t)TILE, n - env0);

      // Publishing the tile for the unit (t, c + 1) (as craft_rollout.h).  Without observation
      // ring reuse inside the launch (ring >= n_ticks) only wave 0's state stores are handed
      // over: they go write-through (sc1) and lane 0 raises the flag after the wave's own
      // drain; otherwise every wave drains and lane 0 releases at agent scope first, so a
      // later chunk rewriting the same ring slot from another XCD lands last.
      const bool state_only = a.ring >= a.n_ticks;
      const bool handoff = c + 1 < n_chunks;
      auto full_release = [&]() __attribute__((always_inline)) {   // every wave, the same barrier
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __hip_atomic_store((gu32*)(a.tile_done + t), (uint32_t)(c + 1), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        }
      };
      // Each role's whole unit sits in its own branch (wave 0: take the tile over, C, publish;
      // wave 1: D; the rest: E), with the same barriers in the same order, so that wave 0's env
      // state is not live in the other roles' loops.
      if (tid < 64) {
        // A: wave 0 takes over the tile (after its previous chunk is published)
        if (c > 0) {
          bool ok = true;
          if (tid == 0) {
            const gu32* f = (const gu32*)(a.tile_done + t);
            for (uint32_t spins = 0; __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (uint32_t)c;) {
              __builtin_amdgcn_s_sleep(2);
              if (++spins > (1u << 26)) { ok = false; break; }   // bounded: never hang the GPU
            }
            if (!ok) latch_error(v.err, CRAFT_EINVARIANT, env0);
          }
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        if (tid < TILE) {
          load_tile(t, 0, std::false_type{});
          tick_c(k0, 0, false);                         // C(0) -> buffer 0
        }
        // the pipeline: interval i runs C(i+1) | D(i) | E(i-1), one barrier each
        if (want_obs) {
          __syncthreads();                              // C(0) complete
          for (int i = 0; i <= nq; ++i) {
            if (tid < TILE && i + 1 < nq) tick_c(k0 + i + 1, i + 1, false);
            __syncthreads();
          }
        } else if (tid < TILE) {
          for (int q = 1; q < nq; ++q) tick_c(k0 + q, q, false);
        }
        if (tid < TILE && live) publish(nq - 1, handoff && state_only);
        if (handoff && state_only) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          if (tid == 0)
            __hip_atomic_store((gu32*)(a.tile_done + t), (uint32_t)(c + 1), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        } else if (handoff) {
          full_release();
        }
      } else {
        if (want_obs) {
          __syncthreads();                              // C(0) complete
          if (tid < 128) {
#pragma unroll 1
            for (int i = 0; i <= nq; ++i) {
              if (i < nq) scatter_d(i, nE);
              __syncthreads();
            }
          } else {
            for (int i = 0; i <= nq; ++i) {
              if (i >= 1) stream_e(i - 1, t, k0 + i - 1, false);
#ifdef CRAFT_STAMPS
              if (tid == 128 && srow_t && n_done == 0 && i == 1) srow_t[13] = __builtin_amdgcn_s_memrealtime();
#endif
              __syncthreads();
            }
          }
        }
        if (handoff && !state_only) full_release();
      }
      __syncthreads();                                  // s_ctrl and the LDS rows are reused
#ifdef CRAFT_STAMPS
      ++n_done;
#endif
    }
#ifdef CRAFT_STAMPS
    if (tid == 0 && srow_t) {
      srow_t[14] = (uint64_t)n_done;
      srow_t[15] = __builtin_amdgcn_s_memrealtime();
    }
#endif
  }

  if (tid == 0) {
    unsigned long long* srow = reinterpret_cast<unsigned long long*>(v.stats_part + 4 * (int64_t)blockIdx.x);
    atomicAdd(srow + 0, (unsigned long long)n_succ);
    atomicAdd(srow + 1, (unsigned long long)n_end);
    atomicAdd(srow + 2, (unsigned long long)n_step);
  }
}

}  // namespace craft
