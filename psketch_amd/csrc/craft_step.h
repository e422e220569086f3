// craft_step.h — the one-launch-per-tick kernel: craft_step / craft_step_ex (a rollout tick
// for every env: the do_rollout protocol of trainers/imitation.py:59-73, CraftState.step
// craft.py:332-424, satisfies :285-294 and the features() observation :296-330), and with
// TL > 0 teacher lanes per env craft_step_teach (the DemonstrationTeacher's label of every
// new state, teachers/demonstration.py:9-30, in the same launch).
//
// Why a different shape from the tile kernel (craft_tile.h).  That kernel gives a 64-env tile
// to a 256-thread workgroup that runs A (loads), C (transition), D (scatter) and E (stores) in
// order; its 1024 workgroups are all resident, so every CU does A + C + D at the same time and
// the stores of a CU stop whenever its waves scatter.  Here one workgroup per CU keeps 256 envs
// and splits the tick over wave roles that run at the same time:
//
//   tick wave w (4, one per SIMD)   A: lane e owns env e of the wave's EPW envs and issues every
//      load of the tick (state, restart spec, action, clone flag and label, inventory, cleared-
//      cell mask; then the scenario's pool row) before the wave queues any store.  C: the same
//      lane runs the protocol and the transition on its LDS grid row and writes the state back.
//      D: the wave scatters SUB envs at a time into two LDS row buffers it shares with stream
//      wave w, waiting on a buffer's sequence word only when both are still being streamed.
//   stream wave w (4)   E: streams each published buffer (16-byte buffer stores, clearing the
//      bytes it reads) and hands it back: the CU's stores never wait for a scatter.
//   teacher lanes (TL > 0)   after C, TL lanes per env run teach_env on the grid rows C left in
//      LDS while the other roles scatter and stream.
//
// One s_barrier per launch, after C (LDS-only fences: the tick waves' state stores are not
// waited for).  Results are identical to the tile kernel's MODE_TICK (craft_sim_tune_step
// selects either; tests/test_gpu_step_kernel.py runs both).
#pragma once
#include "craft_obs.h"
#include "craft_teach.h"

namespace craft {

constexpr int kStepTick = 4;       // tick waves per workgroup (one per SIMD)
constexpr int kStepStream = 4;     // stream waves per workgroup: stream wave w serves tick wave w
constexpr int kStepBufs = 2 * kStepTick;   // two row buffers per (tick, stream) pair

// Dynamic-LDS carve of a step workgroup (16-byte aligned pieces): task table [64] u16 | recipe
// words [16][3] | task_sub [64][4] i32 (TL > 0) | buffer sequence words [8] | per tick wave:
// grid rows [EPW][GS], inventory rows [EPW][36], agent words [EPW], teacher info words [EPW] |
// row buffers [8][SUB * F].
struct StepLds {
  int task, rc, tsub, seq, tick0, grid, inv, agent, tinfo, per_tick, buf0, buf, bytes;
};
__host__ __device__ inline StepLds step_lds(int epw, int sub, int tl, int GS, int F) {
  auto up16 = [](int x) { return (x + 15) & ~15; };
  StepLds l;
  l.task = 0;
  l.rc = up16(CRAFT_MAX_TASKS * 2);
  l.tsub = up16(l.rc + CRAFT_MAX_RECIPES * 12);
  l.seq = l.tsub + (tl > 0 ? CRAFT_MAX_TASKS * CRAFT_MAX_SUBTASKS * 4 : 0);
  l.tick0 = up16(l.seq + 4 * kStepBufs);
  l.grid = 0;                                   // offsets inside one tick wave's region
  l.inv = up16(epw * GS);
  l.agent = up16(l.inv + epw * kInvStride);
  l.tinfo = l.agent + epw * 4;
  l.per_tick = up16(l.tinfo + epw * 4);
  l.buf0 = l.tick0 + kStepTick * l.per_tick;
  l.buf = up16(sub * F);
  l.bytes = l.buf0 + kStepBufs * l.buf;
  return l;
}

#ifdef CRAFT_STAMPS
// Diagnostic builds only (never the product): lane 0 of a tick or stream wave records
// s_memrealtime (100 MHz) at phase boundaries into v.stamps[tick wave][8] (tools/step_stamps.py).
#define STEP_STAMP(k)                                                                   \
  do {                                                                                  \
    if (lane == 0 && v.stamps) v.stamps[8 * gw + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define STEP_STAMP(k) do {} while (0)
#endif

__device__ __forceinline__ void lds_release() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local"); }
__device__ __forceinline__ void lds_acquire() { __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local"); }
__device__ __forceinline__ void wave_lds_order() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ void seq_wait(const uint32_t* w, uint32_t want) {
  while (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != want)
    __builtin_amdgcn_s_sleep(1);
  lds_acquire();
}
__device__ __forceinline__ void seq_set(uint32_t* w, uint32_t val, int lane) {
  lds_release();
  if (lane == 0) __hip_atomic_store(w, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

#ifndef CRAFT_STEP_WPE
#define CRAFT_STEP_WPE 2
#endif
// EPW envs per tick wave (16, 32 or 64), SUB envs per scatter sub-chunk (64 / SUB lanes per env
// in D), TL teacher lanes per env (0: craft_step / craft_step_ex), NW 32-bit words per cell set
// (teacher only).
template <int WIN, int EPW, int SUB, int TL, int NW>
__global__ __launch_bounds__(64 * (kStepTick + kStepStream) + kStepTick * EPW * TL, CRAFT_STEP_WPE)
void step_kernel(SimView v, TileArgs a) {
  static_assert(EPW == 16 || EPW == 32 || EPW == 64, "EPW: envs per tick wave");
  static_assert(EPW % SUB == 0 && 64 % SUB == 0, "SUB divides the wave's envs and its 64 lanes");
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int GS = v.GS, F = v.F;
  const StepLds lay = step_lds(EPW, SUB, TL, GS, F);
  uint16_t* s_task = reinterpret_cast<uint16_t*>(smem + lay.task);
  uint32_t* s_rc = reinterpret_cast<uint32_t*>(smem + lay.rc);
  int32_t* s_tsub = reinterpret_cast<int32_t*>(smem + lay.tsub);
  uint32_t* s_seq = reinterpret_cast<uint32_t*>(smem + lay.seq);
  const bool want_obs = a.obs != nullptr;

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int pair = wave < kStepTick ? wave : (wave < kStepTick + kStepStream ? wave - kStepTick : 0);
  const int64_t gw = (int64_t)blockIdx.x * kStepTick + pair;        // global tick-wave index
  const int64_t env0 = gw * EPW;
  const int nE = (int)max((int64_t)0, min((int64_t)EPW, a.n - env0));

  if (wave < kStepTick) {
    // ================================ tick wave ================================================
    uint8_t* base = smem + lay.tick0 + wave * lay.per_tick;
    uint8_t* s_grid = base + lay.grid;
    uint8_t* s_inv = base + lay.inv;
    uint32_t* s_agent = reinterpret_cast<uint32_t*>(base + lay.agent);
    uint32_t* s_tinfo = reinterpret_cast<uint32_t*>(base + lay.tinfo);
    STEP_STAMP(0);

    // ---- A: every load of the tick, issued before this wave queues any store ----------------
    const int64_t slot = env0 + lane;
    bool live = lane < nE;
    uint64_t st = 0;
    uint32_t init_word = 0;
    int act = 0, ref = 0;
    uint8_t bc = 0;
    uint4 i0 = make_uint4(0, 0, 0, 0), i1 = i0, m0 = i0, m1 = i0;
    if (live) {
      st = v.state[slot];
      init_word = v.init[slot];
      if (a.actions) act = a.actions[slot];
      if (a.bc) bc = a.bc[slot];
      if (a.bc) ref = a.ref[slot];
      i0 = v.inv[2 * slot];
      i1 = v.inv[2 * slot + 1];
      m0 = v.mask[2 * slot];
      m1 = v.mask[2 * slot + 1];
    }
    for (int t = lane; t < v.n_tasks; t += 64) s_task[t] = v.task_tab[t];   // identical values
    for (int t = lane; t < CRAFT_MAX_RECIPES * 3; t += 64) s_rc[t] = v.rcw[t];   // from every
    if (TL > 0)                                                              // tick wave
      for (int t = lane; t < v.n_tasks * CRAFT_MAX_SUBTASKS; t += 64) s_tsub[t] = v.task_sub[t];
    Agent s{};
    if (live) {
      if (!a.actions) {
        const uint64_t gid = (uint64_t)(v.env_base + slot);
        act = (int)((uint32_t)(splitmix64(a.seed ^ (gid << 20) ^ (uint64_t)a.tick) >> 32) % 6u);
      }
      if (bc) act = ref;                                               // behaviour cloning, imitation.py:56-57
      s = unpack_state(st);
      if (s.x < 1 || s.x > v.W - 2 || s.y < 1 || s.y > v.H - 2 || s.scen >= v.pool_count) {
        latch_error(v.err, CRAFT_EINVAL, slot);                        // never initialised
        live = false;
      }
    }
    uint8_t* g = s_grid + lane * GS;
    uint32_t conn = 0;
    if (TL > 0 && live) conn = v.pool_conn[s.scen];
    if (live) {
      // the env's scenario row: CS/16 independent 16-byte loads (L2-resident pool)
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
    uint32_t* ivw = reinterpret_cast<uint32_t*>(s_inv + lane * kInvStride);
    uint8_t* iv = s_inv + lane * kInvStride;
    if (lane < EPW) {
      ivw[0] = i0.x; ivw[1] = i0.y; ivw[2] = i0.z; ivw[3] = i0.w;
      ivw[4] = i1.x; ivw[5] = i1.y; ivw[6] = i1.z; ivw[7] = i1.w;
    }
    // every LDS word written above is read below by the same lane, or (the tables) by other
    // lanes of this wave: order the wave's LDS accesses
    wave_lds_order();
    STEP_STAMP(1);

    // ---- C: the per-env body of ImitationTrainer.do_rollout, trainers/imitation.py:59-73 ------
    uint32_t m[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
    bool inv_changed = false, mask_changed = false;
    int d = 0, succ = -1, counted = 0;
    int code = -1;                                                     // transition code (craft.h)
    if (live) {
      // The LDS row holds pool[scenario]; cells cleared this episode are applied lazily, so an
      // auto-reset (which restores exactly that row) needs no reload.
      bool restart = false;
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
      if (!restart) {
#pragma unroll
        for (int w = 0; w < 8; ++w) {                                  // cells cleared this episode
          uint32_t mm = m[w];
          while (mm) {
            g[w * 32 + __ffs(mm) - 1] = 0;
            mm &= mm - 1;
          }
        }
      }
      if (restart) {                                                   // CraftScenario.init, craft.py:268-273
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
          transition(v, s_rc, g, iv, s, m, act, inv_changed, mask_changed);
          code = transition_code(ox, oy, s, inv_changed);
        }
      }
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
      if (a.rec) a.rec[slot] = counted ? act : -1;                    // action_seqs, imitation.py:59-61
    }
    if (a.code && lane < nE) a.code[slot] = (int8_t)code;
    if (lane < EPW) {
      s_agent[lane] = live ? ((uint32_t)s.x | ((uint32_t)s.y << 8) | ((uint32_t)s.dir << 16) | (1u << 24)) : 0u;
      if (TL > 0) s_tinfo[lane] = (uint32_t)s.task | ((uint32_t)s.frozen << 8) | (conn << 9);
    }
    // episode statistics: one partial-sum row per tick wave (uncontended)
    const uint64_t bs = __ballot(live && counted && d && succ == 1);
    const uint64_t be = __ballot(live && counted && d);
    const uint64_t bt = __ballot(live && counted);
    const uint64_t bl = __ballot(live && counted && !d);
    if (lane == 0 && nE > 0) {                                         // no-return atomics
      unsigned long long* r = reinterpret_cast<unsigned long long*>(v.stats_part + 4 * gw);
      atomicAdd(r + 0, (unsigned long long)__popcll(bs));
      atomicAdd(r + 1, (unsigned long long)__popcll(be));
      atomicAdd(r + 2, (unsigned long long)__popcll(bt));
      if (a.any_live && bl) *a.any_live = 1;                           // idempotent plain store
    }
    STEP_STAMP(2);
    // rows, inventories and agent words published to the stream and teacher lanes; the buffers
    // are zeroed and their sequence words cleared (LDS-only fences: no store is waited for)
    lds_release();
    __builtin_amdgcn_s_barrier();
    lds_acquire();
    STEP_STAMP(3);
    if (!want_obs) return;

    // ---- D: SUB envs at a time (64 / SUB lanes per env) into buffer 2w + (k & 1); its sequence
    // word is 2u while free for use u = k >> 1 (0 after the barrier) and 2u + 1 while full ------
    constexpr int P = 64 / SUB;
    const int e_in = lane % SUB, part = lane / SUB;
#pragma unroll 1
    for (int k = 0; k * SUB < nE; ++k) {
      const int b = 2 * wave + (k & 1);
      uint32_t* sq = s_seq + b;
      if (k >= 2) seq_wait(sq, (uint32_t)(k & ~1));                   // use u - 1 streamed, cleared
      uint8_t* buf = smem + lay.buf0 + b * lay.buf;
      const int e = k * SUB + e_in;
      if (e < nE && part <= WIN) {
        const uint32_t ag = s_agent[e];
        if (ag >> 24) scatter_env_part<WIN, P>(v, s_grid + e * GS, s_inv + e * kInvStride, ag, buf + e_in * F, part);
      }
      seq_set(sq, (uint32_t)(k & ~1) + 1u, lane);                     // full
      if (k == 0) STEP_STAMP(4);
    }
    STEP_STAMP(5);
    return;
  }

  if (wave < kStepTick + kStepStream) {
    // ================================ stream wave ==============================================
    const int p = pair;
    if (want_obs) {                                                    // the pair's two buffers, zeroed
      uint4* z = reinterpret_cast<uint4*>(smem + lay.buf0 + 2 * p * lay.buf);
      for (int i = lane; i < (2 * lay.buf) >> 4; i += 64) z[i] = make_uint4(0, 0, 0, 0);
      if (lane < 2) s_seq[2 * p + lane] = 0u;
    }
    lds_release();
    __builtin_amdgcn_s_barrier();
    lds_acquire();
    if (!want_obs) return;
#pragma unroll 1
    for (int k = 0; k * SUB < nE; ++k) {
      const int b = 2 * p + (k & 1);
      uint32_t* sq = s_seq + b;
      seq_wait(sq, (uint32_t)(k & ~1) + 1u);                          // published by tick wave p
      uint8_t* buf = smem + lay.buf0 + b * lay.buf;
      const int nEs = min(SUB, nE - k * SUB);
      switch (v.obs_fmt) {
        case CRAFT_OBS_BF16: stream_obs<CRAFT_OBS_BF16, 64, true>(buf, a.obs, env0 + k * SUB, F, nEs, v.obs_policy, lane); break;
        case CRAFT_OBS_U8: stream_obs<CRAFT_OBS_U8, 64, true>(buf, a.obs, env0 + k * SUB, F, nEs, v.obs_policy, lane); break;
        default: stream_obs<CRAFT_OBS_F32, 64, true>(buf, a.obs, env0 + k * SUB, F, nEs, v.obs_policy, lane); break;
      }
      seq_set(sq, (uint32_t)(k & ~1) + 2u, lane);                     // cleared: free for use u + 1
    }
#ifdef CRAFT_STAMPS
    if (v.stamps) {                                                    // stores drained; hardware ids
      __builtin_amdgcn_s_waitcnt(0);
      STEP_STAMP(6);
      uint32_t xcc, hw;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      if (lane == 0) v.stamps[8 * gw + 7] = ((uint64_t)xcc << 32) | hw;
    }
#endif
    return;
  }

  if constexpr (TL > 0) {
    // ================================ teacher lanes ============================================
    // TL lanes per env; tick wave w's envs are served by teacher lanes [w * EPW * TL, ...):
    // DemonstrationTeacher on each env's new state from the rows C left in LDS
    // (teachers/demonstration.py:9-30), overlapping the scatter and the stores.
    lds_release();
    __builtin_amdgcn_s_barrier();
    lds_acquire();
    const int u = tid - 64 * (kStepTick + kStepStream);
    const int w = u / (EPW * TL), e = (u % (EPW * TL)) / TL, ql = u % TL;
    const int64_t tenv0 = ((int64_t)blockIdx.x * kStepTick + w) * EPW;
    const int tnE = (int)max((int64_t)0, min((int64_t)EPW, a.n - tenv0));
    if (e < tnE) {
      uint8_t* base = smem + lay.tick0 + w * lay.per_tick;
      const uint32_t ag = reinterpret_cast<const uint32_t*>(base + lay.agent)[e];
      const uint32_t ti = reinterpret_cast<const uint32_t*>(base + lay.tinfo)[e];
      const int64_t i = tenv0 + e;
      int action = -2;                                                 // a slot C could not run
      if (ag && ((ti >> 8) & 1u)) {
        action = -1;                                                   // frozen: the label of a done env
      } else if (ag) {
        Agent s{};
        s.x = ag & 0xff; s.y = (ag >> 8) & 0xff; s.dir = (ag >> 16) & 3; s.task = ti & 0xff;
        const uint32_t m0[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        int len = -1, err = 0;
        action = teach_env<NW, TL>(v, s_task, s_tsub, reinterpret_cast<const uint32_t*>(base + lay.grid + e * GS),
                                   m0, base + lay.inv + e * kInvStride, s, s.task, ql, false, len, err,
                                   ((ti >> 9) & 1u) != 0);
        if (err && ql == 0) latch_error(v.err, err, i);
      }
      if (ql == 0) a.label[i] = action;
    }
  }
}

}  // namespace craft
