// craft_step.h — the step kernel: one launch per tick (craft_step / craft_step_ex when
// craft_sim_tune_step selects it; the tile kernel, craft_tile.h, is the default): the do_rollout
// protocol of trainers/imitation.py:59-73, CraftState.step craft.py:332-424, satisfies :285-294
// and the features() observation :296-330 for every env.
//
// The design round 2's review proposed for the tick: one workgroup per CU keeps 256 envs and
// splits the tick over wave roles that run at the same time, so that the CU's stores never
// wait for a scatter:
//
//   tick wave w (4, one per SIMD)   A: lane e owns env e of the wave's EPW envs and issues every
//      load of the tick (state, restart spec, action, clone flag and label, inventory, cleared-
//      cell mask, the static tables; then the scenario rows, loaded cooperatively) before the
//      wave queues any store.  C: the same lane runs the protocol and the transition on its LDS
//      grid row.  D: the wave scatters SUB envs at a time into two LDS row buffers it shares
//      with its stream wave, waiting on a buffer's sequence word only when both are in use.
//      C's results go to HBM after the last scatter.
//   stream wave (4 or 8)   E: streams each published buffer (16-byte buffer stores, clearing
//      the bytes it reads) and hands it back.
//   teacher lanes (TL > 0)   after C, TL lanes per env run teach_env on the grid rows in LDS.
//
// One s_barrier per launch, at its start.  Measured (tools/step_probe.py and the
// phase stamps of tools/step_stamps.py) at 65,536 envs it is slower than the tile kernel: 28.2-
// 29.6 us against 26.1-27.0 with a fresh 106 MB slot per tick, 23.3-28.0 against 20.3 with one
// reused buffer.  The stores run at the write ceiling once going (~18 us); what loses is the
// ~6.5 us before a CU's first store, which is instruction latency of one wave per SIMD (A ~3,
// C ~1.6, the first scatter ~1.6 us) that the tile kernel's 16 waves per CU overlap better.  So
// it stays an option (tests/test_gpu_step_kernel.py keeps it bit-identical to the tile kernel)
// and only TL = 0 is instantiated (with teacher lanes it measured 36 us against the two-tile
// kernel's 31).
#pragma once
#include "craft_obs.h"
#include "craft_teach.h"

namespace craft {

constexpr int kStepTick = 4;       // tick waves per workgroup (one per SIMD)
constexpr int kStepStream = 4;     // stream waves per workgroup: stream wave w serves tick wave w
constexpr int kStepBufs = 2 * kStepTick;   // two row buffers per (tick, stream) pair

// Dynamic-LDS carve of a step workgroup (16-byte aligned pieces): task table [64] u16 | recipe
// words [16][3] | task_sub [64][4] i32 (TL > 0) | buffer sequence words [8] and C-done flags
// [4] | per tick wave:
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
  l.tick0 = up16(l.seq + 4 * (kStepBufs + kStepTick));   // + the tick waves' C-done flags
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
// extra stamps of the same tick wave in row gw + (tick waves of the launch)
#define STEP_STAMP2(k)                                                                  \
  do {                                                                                  \
    if (lane == 0 && v.stamps)                                                          \
      v.stamps[8 * (gw + (int64_t)gridDim.x * kStepTick) + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define STEP_STAMP(k) do {} while (0)
#define STEP_STAMP2(k) do {} while (0)
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
// NS stream waves: 4 (stream wave w serves both buffers of tick wave w) or 8 (one per buffer).
template <int WIN, int EPW, int SUB, int TL, int NW, int NS = kStepStream>
__global__ __launch_bounds__(64 * (kStepTick + NS) + kStepTick * EPW * TL, CRAFT_STEP_WPE)
void step_kernel(SimView v, TileArgs a) {
  static_assert(NS == kStepTick || NS == 2 * kStepTick, "one or two stream waves per tick wave");
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
  const int pair = wave < kStepTick ? wave : (wave < kStepTick + NS ? (wave - kStepTick) % kStepTick : 0);
  const int64_t gw = (int64_t)blockIdx.x * kStepTick + pair;        // global tick-wave index
  // A tick wave's EPW consecutive envs, in EPW / SUB runs of SUB envs (one scatter sub-chunk each).
  // (Interleaving the runs of all waves, so that the chip's stores sweep one region of the
  // buffer at a time, measured 3 % slower: DESIGN.md.)
  auto run0 = [&](int k) -> int64_t { return gw * EPW + (int64_t)k * SUB; };
  auto run_n = [&](int k) -> int { return (int)max((int64_t)0, min((int64_t)SUB, a.n - run0(k))); };

  if (wave < kStepTick) {
    // ================================ tick wave ================================================
    uint8_t* base = smem + lay.tick0 + wave * lay.per_tick;
    uint8_t* s_grid = base + lay.grid;
    uint8_t* s_inv = base + lay.inv;
    uint32_t* s_agent = reinterpret_cast<uint32_t*>(base + lay.agent);
    uint32_t* s_tinfo = reinterpret_cast<uint32_t*>(base + lay.tinfo);
    STEP_STAMP(0);

    // ---- A: every load of the tick, issued before this wave queues any store, and no load
    // result used before the last independent load is issued (one round trip, then the pool row)
    const int64_t slot = run0(lane / SUB) + lane % SUB;
    const bool in_range = lane < EPW && slot < a.n;
    bool live = in_range;
    uint64_t st = 0;
    uint32_t init_word = 0;
    int act = 0, ref = 0;
    uint32_t bc = 0;
    uint4 i0 = make_uint4(0, 0, 0, 0), i1 = i0, m0 = i0, m1 = i0;
    if (live) {
      st = v.state[slot];
      i0 = v.inv[2 * slot];
      i1 = v.inv[2 * slot + 1];
      m0 = v.mask[2 * slot];
      m1 = v.mask[2 * slot + 1];
      init_word = v.init[slot];
      if (a.actions) act = a.actions[slot];
      // the clone flag and label: loaded unconditionally (from slot 0 of the state when there is
      // no cloning), so that no branch waits on the flag before the next load is issued
      const bool cl = a.bc != nullptr;
      const uint8_t* bcp = cl ? a.bc : reinterpret_cast<const uint8_t*>(v.state);
      const int32_t* refp = cl ? a.ref : reinterpret_cast<const int32_t*>(v.state);
      const int64_t cs = cl ? slot : 0;
      bc = bcp[cs];
      ref = refp[cs];
    }
    // the static tables, one round trip with the loads above (copied to LDS below)
    const uint32_t task_w = lane < v.n_tasks ? (uint32_t)v.task_tab[lane] : 0u;
    const uint32_t rc_w = lane < CRAFT_MAX_RECIPES * 3 ? v.rcw[lane] : 0u;
    int32_t tsub_w[CRAFT_MAX_TASKS * CRAFT_MAX_SUBTASKS / 64];
#pragma unroll
    for (int q = 0; q < CRAFT_MAX_TASKS * CRAFT_MAX_SUBTASKS / 64; ++q)
      tsub_w[q] = (TL > 0 && lane + 64 * q < v.n_tasks * CRAFT_MAX_SUBTASKS) ? v.task_sub[lane + 64 * q] : 0;
    // the stream waves have zeroed the row buffers and cleared the sequence words: one barrier,
    // LDS-only fences, the loads above still in flight
    lds_release();
    __builtin_amdgcn_s_barrier();
    lds_acquire();
    Agent s{};
#ifdef CRAFT_STAMPS
    if (v.stamps) { __builtin_amdgcn_s_waitcnt(0); STEP_STAMP2(0); }   // the first loads landed
#endif
    if (live) {
      s = unpack_state(st);
      if (s.x < 1 || s.x > v.W - 2 || s.y < 1 || s.y > v.H - 2 || s.scen >= v.pool_count) {
        latch_error(v.err, CRAFT_EINVAL, slot);                        // never initialised
        live = false;
      }
    }
    uint8_t* g = s_grid + lane * GS;
    uint32_t conn = 0;
    if (TL > 0 && live) conn = v.pool_conn[s.scen];
    // The envs' scenario rows (L2-resident pool), loaded cooperatively: load q of lane l fetches
    // 16-byte chunk j = 64 q + l of the wave's rows laid end to end (env j / nchunk, chunk
    // j % nchunk), so a wave instruction touches ~3 cache lines per row instead of one line per
    // lane.  Every row's scenario comes by one cross-lane read, all issued before any load; the
    // loads are unconditional (row 0 for an env that is not live), so none waits on a branch.
    const int nchunk = v.CS >> 4;
    constexpr int QMAX = CRAFT_MAX_CELLS / 16;
    int sc[QMAX];
    uint32_t off[QMAX], src_off[QMAX];
    {
      const int scen_l = live ? s.scen : -1;
      int e = lane / nchunk, ch = lane - e * nchunk;
      const int de = 64 / nchunk, dch = 64 - de * nchunk;
#pragma unroll
      for (int q = 0; q < QMAX; ++q) {          // straight-line code over every possible chunk:
        off[q] = (uint32_t)(e * GS + ch * 16);   // loads past nchunk read row 0 and are dropped
        src_off[q] = (uint32_t)(ch * 16);
        sc[q] = __shfl(scen_l, min(e, 63));
        e += de;
        ch += dch;
        if (ch >= nchunk) { ch -= nchunk; ++e; }
      }
    }
    // 32-bit offsets off one wave-uniform descriptor (no 64-bit address arithmetic per load)
    const __amdgpu_buffer_rsrc_t prs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(v.pool), 0, -1, 0x00020000);
    obs_vec c[QMAX];
#pragma unroll
    for (int q = 0; q < QMAX; ++q)
      c[q] = __builtin_amdgcn_raw_buffer_load_b128(prs, (uint32_t)max(sc[q], 0) * (uint32_t)v.CS +
                                                            (q < nchunk ? src_off[q] : 0u), 0, 0);
#ifdef CRAFT_STAMPS
    if (v.stamps) STEP_STAMP2(4);                                      // pool rows issued
#endif
    // meanwhile: the tables and the inventory rows to LDS, the hashed action
    if (lane < v.n_tasks) s_task[lane] = (uint16_t)task_w;
    if (lane < CRAFT_MAX_RECIPES * 3) s_rc[lane] = rc_w;
    if (TL > 0) {
#pragma unroll
      for (int q = 0; q < CRAFT_MAX_TASKS * CRAFT_MAX_SUBTASKS / 64; ++q)
        if (lane + 64 * q < v.n_tasks * CRAFT_MAX_SUBTASKS) s_tsub[lane + 64 * q] = tsub_w[q];
    }
    uint32_t* ivw = reinterpret_cast<uint32_t*>(s_inv + lane * kInvStride);
    uint8_t* iv = s_inv + lane * kInvStride;
    if (lane < EPW) {
      ivw[0] = i0.x; ivw[1] = i0.y; ivw[2] = i0.z; ivw[3] = i0.w;
      ivw[4] = i1.x; ivw[5] = i1.y; ivw[6] = i1.z; ivw[7] = i1.w;
    }
    if (live) {
      if (!a.actions) {
        const uint64_t gid = (uint64_t)(v.env_base + slot);
        act = (int)((uint32_t)(splitmix64(a.seed ^ (gid << 20) ^ (uint64_t)a.tick) >> 32) % 6u);
      }
      asm volatile("" : "+v"(bc), "+v"(ref));                          // (keeps the compiler from
      if (a.bc) act = (bc & 0xffu) ? ref : act;                        // waiting on the flag early)
                                                                       // behaviour cloning, imitation.py:56-57
    }
#ifdef CRAFT_STAMPS
    if (v.stamps) { __builtin_amdgcn_s_waitcnt(0); STEP_STAMP2(1); }   // pool rows landed
#endif
#pragma unroll
    for (int q = 0; q < QMAX; ++q)
      if (q < nchunk && sc[q] >= 0) {
        uint32_t* dst = reinterpret_cast<uint32_t*>(s_grid + off[q]);
        dst[0] = c[q].x; dst[1] = c[q].y; dst[2] = c[q].z; dst[3] = c[q].w;
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
    }
    if (lane < EPW) {
      s_agent[lane] = live ? ((uint32_t)s.x | ((uint32_t)s.y << 8) | ((uint32_t)s.dir << 16) | (1u << 24)) : 0u;
      if (TL > 0) s_tinfo[lane] = (uint32_t)s.task | ((uint32_t)s.frozen << 8) | (conn << 9);
    }
    if (TL > 0) seq_set(s_seq + kStepBufs + wave, 1u, lane);          // C done: the teacher may start
    STEP_STAMP(2);

    // ---- D: SUB envs at a time (64 / SUB lanes per env) into buffer 2w + (k & 1); its sequence
    // word is 2u while free for use u = k >> 1 (0 after the barrier) and 2u + 1 while full.  No
    // global store is issued before the scatter (the compiler drains them before it reuses their
    // data registers): C's results are stored after the last sub-chunk is published ---------------
    if (want_obs) {
      constexpr int P = 64 / SUB;
      const int e_in = lane % SUB, part = lane / SUB;
#pragma unroll 1
      for (int k = 0; k * SUB < EPW; ++k) {
        const int nEs = run_n(k);
        if (nEs == 0) break;                                           // and every later run
        const int b = 2 * wave + (k & 1);
        uint32_t* sq = s_seq + b;
        if (k >= 2) seq_wait(sq, (uint32_t)(k & ~1));                 // use u - 1 streamed, cleared
        uint8_t* buf = smem + lay.buf0 + b * lay.buf;
        const int e = k * SUB + e_in;
        if (e_in < nEs) {
          const uint32_t ag = s_agent[e];
          if (ag >> 24) scatter_env_part<WIN, P>(v, s_grid + e * GS, s_inv + e * kInvStride, ag, buf + e_in * F, part);
        }
#ifdef CRAFT_STAMPS
        if (k == 0 && v.stamps) {     // the first scatter again (idempotent): warm-code timing
          lds_release();
          STEP_STAMP2(2);
          if (e_in < nEs) {
            const uint32_t ag = s_agent[e];
            if (ag >> 24) scatter_env_part<WIN, P>(v, s_grid + e * GS, s_inv + e * kInvStride, ag, buf + e_in * F, part);
          }
          lds_release();
          STEP_STAMP2(3);
        }
#endif
        seq_set(sq, (uint32_t)(k & ~1) + 1u, lane);                   // full
        if (k == 0) STEP_STAMP(3);
      }
    }
    STEP_STAMP(4);

    // ---- C's results to HBM ------------------------------------------------------------------
    if (live) {
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
    if (a.code && in_range) a.code[slot] = (int8_t)code;
    // episode statistics: one partial-sum row per tick wave (uncontended)
    const uint64_t bs = __ballot(live && counted && d && succ == 1);
    const uint64_t be = __ballot(live && counted && d);
    const uint64_t bt = __ballot(live && counted);
    const uint64_t bl = __ballot(live && counted && !d);
    if (lane == 0 && run_n(0) > 0) {                                   // no-return atomics
      unsigned long long* r = reinterpret_cast<unsigned long long*>(v.stats_part + 4 * gw);
      atomicAdd(r + 0, (unsigned long long)__popcll(bs));
      atomicAdd(r + 1, (unsigned long long)__popcll(be));
      atomicAdd(r + 2, (unsigned long long)__popcll(bt));
      if (a.any_live && bl) *a.any_live = 1;                           // idempotent plain store
    }
    return;
  }

  if (wave < kStepTick + NS) {
    // ================================ stream wave ==============================================
    const int p = pair;
    const int par = (wave - kStepTick) / kStepTick;                     // NS = 8: the buffer it serves
    const int nb = NS == kStepTick ? 2 : 1;                             // buffers served
    const int b0 = NS == kStepTick ? 2 * p : 2 * p + par;
    if (want_obs) {                                                    // its buffers, zeroed
      uint4* z = reinterpret_cast<uint4*>(smem + lay.buf0 + b0 * lay.buf);
      for (int i = lane; i < (nb * lay.buf) >> 4; i += 64) z[i] = make_uint4(0, 0, 0, 0);
    }
    if (lane < nb) s_seq[b0 + lane] = 0u;
    if (lane == 2 && par == 0) s_seq[kStepBufs + p] = 0u;              // the tick wave's C-done flag
    lds_release();
    __builtin_amdgcn_s_barrier();
    lds_acquire();
    if (!want_obs) return;
#pragma unroll 1
    for (int k = (NS == kStepTick ? 0 : par); k * SUB < EPW; k += (NS == kStepTick ? 1 : 2)) {
      const int nEs = run_n(k);
      if (nEs == 0) break;
      const int b = 2 * p + (k & 1);
      uint32_t* sq = s_seq + b;
      seq_wait(sq, (uint32_t)(k & ~1) + 1u);                          // published by tick wave p
      uint8_t* buf = smem + lay.buf0 + b * lay.buf;
      switch (v.obs_fmt) {
        case CRAFT_OBS_BF16: stream_obs<CRAFT_OBS_BF16, 64, true>(buf, a.obs, run0(k), F, nEs, v.obs_policy, lane); break;
        case CRAFT_OBS_U8: stream_obs<CRAFT_OBS_U8, 64, true>(buf, a.obs, run0(k), F, nEs, v.obs_policy, lane); break;
        default: stream_obs<CRAFT_OBS_F32, 64, true>(buf, a.obs, run0(k), F, nEs, v.obs_policy, lane); break;
      }
      seq_set(sq, (uint32_t)(k & ~1) + 2u, lane);                     // cleared: free for use u + 1
      if (k <= 1) STEP_STAMP(5);
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
    const int u = tid - 64 * (kStepTick + NS);
    const int w = u / (EPW * TL), e = (u % (EPW * TL)) / TL, ql = u % TL;
    const int64_t tgw = (int64_t)blockIdx.x * kStepTick + w;
    const int64_t i = tgw * EPW + e;
    if (tgw * EPW >= a.n) return;                                      // tick wave w has no env
    seq_wait(s_seq + kStepBufs + w, 1u);                               // tick wave w's C is done
    if (i < a.n) {
      uint8_t* base = smem + lay.tick0 + w * lay.per_tick;
      const uint32_t ag = reinterpret_cast<const uint32_t*>(base + lay.agent)[e];
      const uint32_t ti = reinterpret_cast<const uint32_t*>(base + lay.tinfo)[e];
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
