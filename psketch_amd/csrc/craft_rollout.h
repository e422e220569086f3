// craft_rollout.h — K rollout ticks in one launch (craft_rollout): the kernel
// template, instantiated per window by craft_rollout_w{3,5,7}.hip.
//
// craft_step pays, every tick, for a prologue that moves no observation bytes:
// the state/inventory/mask loads, the scenario row from L2, the transition and
// the scatter.  All workgroups of a launch run that prologue together, so HBM
// idles for its duration (phase stamps).  Here a workgroup keeps a
// tile of envs on chip for a chunk of ticks — state in wave 0's registers, grid
// rows, the scenario's pristine rows and inventories in LDS — and pipelines the
// ticks over two LDS observation buffers: wave 0 (the producer) runs the
// transition C(k+1) and scatters the observation D(k+1) into one buffer while
// waves 1.. (the consumers) stream E(k) from the other.
//
// Work distribution.  The launch is cut into units (tile t, chunk c of `chunk`
// ticks), handed out in chunk-major order from a queue counter to persistent
// workgroups; a unit's env state goes back to HBM at its end and the unit
// (t, c+1) may run on any other workgroup.  That hand-off follows
// cdna_hip_programming.md Guideline 16 / MI355X_MICROARCH.md (valid forms,
// plain-store producer): every storing wave drains (s_waitcnt vmcnt(0)), a
// workgroup barrier, one lane's agent-scope release (which also pushes this
// unit's observation stores out of the XCD's L2, so a later unit rewriting the
// same ring slot from another XCD lands last), a second drain, and a relaxed
// agent-scope store tile_done[t] = c + 1; the consumer wave polls that word
// relaxed, then one agent-scope acquire, then plain loads.  Queue and flags are
// zeroed by a memset ahead of every launch.  A unit waits only for its own
// tile's previous chunk, which was handed out earlier and is held by a running
// workgroup, so the queue cannot deadlock; spins are bounded anyway.
//
// Tick k is exactly craft_step(tick0 + k) with the hashed (or given) actions and
// writes its outputs to ring slot (tick0 + k) % ring, as a driver cycling craft_step
// over a ring of R buffers would.  Used where actions do not depend on the
// observations (random rollouts, configs 2 and 4; or replayed action tables).
#pragma once
#include "craft_obs.h"
#include "craft_rollout_split.h"

#ifndef CRAFT_SPLIT_WPE
#define CRAFT_SPLIT_WPE 4
#endif

namespace craft {

// NT threads per workgroup.  Wave 0 is the producer: lanes < TILE own one env
// each and run its transition C(k+1); then all 64 lanes scatter the tile's
// observation rows D(k+1) (64 / TILE lanes per env) into one of two LDS row
// buffers.  Waves 1.. are consumers: they stream E(k) from the other buffer
// and clear it.  One workgroup barrier per tick; the stores never wait for a
// transition or a scatter.  WPE = waves per SIMD the kernel is built for.
//
// GIVEN: actions come from a.actions (one global load per env-tick); otherwise they
// are the hashed draw and the producer's tick loop issues no global load at all — a
// load would make the wave wait for every older store (vmcnt counts loads and stores
// in issue order), i.e. for the previous ticks' done / success / reward stores.
template <int WIN, int TILE, int NT, int FMT, int WPE, bool GIVEN>
__global__ __launch_bounds__(NT, WPE) void rollout_kernel(SimView v, RolloutArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int P = 64 / TILE;                            // producer lanes per env in D
  const LdsLayout lay = lds_layout(TILE, v.GS, v.F, 2, true);
  uint8_t* s_grid = smem;                                 // [TILE][GS] current grids
  uint8_t* s_pristine = smem + TILE * v.GS;               // [TILE][GS] pool[scenario] (restarts)
  uint8_t* s_obs = smem + lay.obs;                        // two buffers of [TILE][F] bytes
  const int obs_buf = (TILE * v.F + 15) & ~15;
  uint8_t* s_inv = smem + lay.inv;
  uint16_t* s_task = reinterpret_cast<uint16_t*>(smem + lay.task);
  uint32_t* s_rc = reinterpret_cast<uint32_t*>(smem + lay.rc);
  uint32_t* s_ctrl = reinterpret_cast<uint32_t*>(smem + lay.ctrl);

  STAMP(0);
#ifdef CRAFT_STAMPS
  // diagnostic build: phase totals of the producer (1 C, 2 D, 3 barrier) and of
  // consumer wave 1 (4 E, 5 barrier), in s_memrealtime ticks (10 ns)
  unsigned long long acc[6] = {0, 0, 0, 0, 0, 0};
#define CRAFT_NOW() __builtin_amdgcn_s_memrealtime()
#ifdef CRAFT_STAMPS_C        // slots 4 / 5: C up to the transition / the transition itself
#define PACC(q, d) do { if ((q) < 4) acc[q] += (d); } while (0)
#define PACC_C(q, d) acc[q] += (d)
#else
#define PACC(q, d) acc[q] += (d)
#define PACC_C(q, d) do {} while (0)
#endif
#else
#define PACC_C(q, d) do {} while (0)
#define CRAFT_NOW() 0ull
#define PACC(q, d) do {} while (0)
#endif
  const int tid = threadIdx.x;
  // the recipe words in a VGPR (lane w: word w), loaded while every lane is active, for the
  // transition's recipe loop (v_readlane instead of an LDS round trip per recipe)
  const uint32_t rcv = v.rcw[min(tid & 63, CRAFT_MAX_RECIPES * 3 - 1)];
  const int64_t n = v.n_envs;
  const bool want_obs = a.obs != nullptr;
  const int F = v.F;
  constexpr int esz = FMT == CRAFT_OBS_F32 ? 4 : (FMT == CRAFT_OBS_BF16 ? 2 : 1);
  const int n_tiles = (int)((n + TILE - 1) / TILE);
  const int n_chunks = (a.n_ticks + a.chunk - 1) / a.chunk;
  const uint32_t n_units = (uint32_t)n_tiles * (uint32_t)n_chunks;

  // Per lane of wave 0, for the current unit: the packed state word and the init
  // word.  The cleared-cell mask is not carried: cells are only ever cleared, so
  // this episode's mask is exactly {c : pristine[c] != 0 and grid[c] == 0} and is
  // rebuilt from the LDS rows when the state goes back to HBM.
  Agent s{};
  uint64_t st = 0;
  uint32_t init_word = 0;
  uint32_t task_word = 0;                                   // s_task[task]: fixed for the env
  // cells cleared this episode, so that a restart restores only those from the pristine row:
  // up to 3 cell ids (bits 0-23), their count (bits 24-25), bit 31 = more (restore the row)
  uint32_t clr = 0;
  bool live = false;
  int64_t slot = 0;
  uint8_t* g = s_grid + tid * v.GS;
  uint32_t* gw = reinterpret_cast<uint32_t*>(g);
  uint32_t* pw = reinterpret_cast<uint32_t*>(s_pristine + tid * v.GS);
  uint8_t* iv = s_inv + tid * kInvStride;
  uint32_t* ivw = reinterpret_cast<uint32_t*>(iv);
  uint32_t n_succ = 0, n_end = 0, n_step = 0;               // wave-uniform running sums

  // ---- C: the do_rollout tick of wave 0's envs (trainers/imitation.py:59-73) ------------------
  auto tick_c = [&](int k) -> uint32_t {
    const int64_t tick = a.tick0 + k;
    const int64_t r = tick % a.ring;
    int d = 0, succ = -1, counted = 0;
    const unsigned long long tc0 = CRAFT_NOW();
    unsigned long long tc1 = tc0;
    s = unpack_state(st);
    if (live) {
      int act;
      if (GIVEN) {
        act = a.actions[(int64_t)k * n + slot];
      } else {
        const uint64_t gid = (uint64_t)(v.env_base + slot);
#ifdef CRAFT_ABL_NOHASH
        act = (int)((gid + (uint64_t)tick) % 6u);
#else
        act = (int)((uint32_t)(splitmix64(a.seed ^ (gid << 20) ^ (uint64_t)tick) >> 32) % 6u);
#endif
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
#ifdef CRAFT_ABL_NOSAT
      if (false) {
#else
      if (d) {
#endif
        // satisfies() of the pre-step state (the LDS row already has this episode's clears)
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
        for (int w = 0; w < 8; ++w) ivw[w] = 0u;
        if (clr >> 31) {
          // more than 3 cells cleared: the whole scenario row, 12 dword reads in flight at a time
          for (int q0 = 0; q0 < (v.CS >> 2); q0 += 12) {
            uint32_t w[12];
#pragma unroll
            for (int j = 0; j < 12; ++j) w[j] = q0 + j < (v.CS >> 2) ? pw[q0 + j] : 0u;
#pragma unroll
            for (int j = 0; j < 12; ++j)
              if (q0 + j < (v.CS >> 2)) gw[q0 + j] = w[j];
          }
        } else {
          const uint8_t* pr = reinterpret_cast<const uint8_t*>(pw);
          const int nc = (clr >> 24) & 3;
#pragma unroll
          for (int i = 0; i < 3; ++i)
            if (i < nc) {
              const int c = (clr >> (8 * i)) & 0xff;
              g[c] = pr[c];
            }
        }
        clr = 0;
      } else if (d && !s.frozen) {
        s.frozen = 1;
        s.timer = max(s.timer, 0);
      }
      tc1 = CRAFT_NOW();
      if (!d) {
        bool inv_changed = false, mask_changed = false;
        uint32_t m_unused[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // the LDS row is the record
        const int fc = (s.x + dir_dx(s.dir)) * v.H + (s.y + dir_dy(s.dir));   // what USE clears
#ifndef CRAFT_ABL_NOTRANS
        if (act < 0 || act >= CRAFT_N_ACTIONS) latch_error(v.err, CRAFT_EBADACTION, slot);
        else transition<true>(v, s_rc, g, iv, s, m_unused, act, inv_changed, mask_changed, rcv, slot);
#endif
        if (mask_changed) {
          const uint32_t nc = (clr >> 24) & 3;
          clr = nc < 3 ? ((clr & 0x00ffffffu) | ((uint32_t)fc << (8 * nc)) | ((nc + 1) << 24)) : (1u << 31);
        }
      }
      const unsigned long long tc2 = CRAFT_NOW();
      PACC_C(4, tc1 - tc0);
      PACC_C(5, tc2 - tc1);
      st = pack_state(s);
      const int64_t o = r * n + slot;
      if (a.done) a.done[o] = (uint8_t)d;
      if (a.sat) a.sat[o] = (int8_t)succ;
      if (a.reward) a.reward[o] = (counted && d && succ == 1) ? 1.0f : 0.0f;
    }
    const uint64_t bs = __ballot(live && counted && d && succ == 1);
    const uint64_t be = __ballot(live && counted && d);
    const uint64_t bt = __ballot(live && counted);
    n_succ += (uint32_t)__popcll(bs);
    n_end += (uint32_t)__popcll(be);
    n_step += (uint32_t)__popcll(bt);
    return live ? ((uint32_t)s.x | ((uint32_t)s.y << 8) | ((uint32_t)s.dir << 16) | (1u << 24)) : 0u;
  };

  // ---- D: the whole producer wave scatters the tile's rows into buffer `buf` ------------------
  // (lane tid works on env tid % TILE, part tid / TILE; `ag` is valid on lanes < TILE)
  auto scatter_d = [&](uint32_t ag, uint8_t* buf) {
    if (P > 1) {                                        // C's LDS writes -> the env's other lanes
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      ag = (uint32_t)__shfl((int)ag, tid % TILE, 64);
    }
    const int e = tid % TILE;
#ifndef CRAFT_ABL_NOD
    if (ag) scatter_env_part<WIN, P>(v, s_grid + e * v.GS, s_inv + e * kInvStride, ag, buf + e * F, tid / TILE);
#endif
  };

  // ---- once per workgroup: static tables, cleared observation rows ------------------------------
  if (tid < TILE) {
    for (int t = tid; t < v.n_tasks; t += TILE) s_task[t] = v.task_tab[t];
    for (int t = tid; t < CRAFT_MAX_RECIPES * 3; t += TILE) s_rc[t] = v.rcw[t];
  }
  if (want_obs) {
    uint4* z = reinterpret_cast<uint4*>(s_obs);
    const int n16 = 2 * obs_buf >> 4;
    for (int i = tid; i < n16; i += NT) z[i] = make_uint4(0, 0, 0, 0);
  }

  for (;;) {
    // ---- next unit ------------------------------------------------------------------------------
    if (tid == 0) s_ctrl[0] = (uint32_t)(atomicAdd(a.queue, 1ull) - a.qbase);
    __syncthreads();
    const uint32_t u = s_ctrl[0];
    if (u >= n_units) break;                            // workgroup-uniform exit
    const int t = (int)(u % (uint32_t)n_tiles), c = (int)(u / (uint32_t)n_tiles);
    const int k0 = c * a.chunk, k1 = min(a.n_ticks, k0 + a.chunk);
    const int64_t env0 = (int64_t)t * TILE;
    const int nE = (int)min((int64_t)TILE, n - env0);

    // ---- A: wave 0 takes over the tile (after the tile's previous chunk is published) -----------
    if (tid < 64) {
      if (c > 0) {
        bool ok = true;
        if (tid == 0) {                                 // ONE lane polls ONE word, relaxed
          const gu32* f = (const gu32*)(a.tile_done + t);
          for (uint32_t spins = 0; __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (uint32_t)c;) {
            __builtin_amdgcn_s_sleep(2);
            if (++spins > (1u << 26)) { ok = false; break; }   // bounded: never hang the GPU
          }
          if (!ok) latch_error(v.err, CRAFT_EINVARIANT, env0);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // after the match: drop stale L1 lines
      }
      uint32_t ag = 0;
      if (tid < TILE) {
        slot = env0 + tid;
        live = tid < nE;
        uint32_t m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (live) {
          st = v.state[slot];
          init_word = v.init[slot];
          const uint4 i0 = v.inv[2 * slot], i1 = v.inv[2 * slot + 1];
          const uint4 m0 = v.mask[2 * slot], m1 = v.mask[2 * slot + 1];
          ivw[0] = i0.x; ivw[1] = i0.y; ivw[2] = i0.z; ivw[3] = i0.w;
          ivw[4] = i1.x; ivw[5] = i1.y; ivw[6] = i1.z; ivw[7] = i1.w;
          m[0] = m0.x; m[1] = m0.y; m[2] = m0.z; m[3] = m0.w;
          m[4] = m1.x; m[5] = m1.y; m[6] = m1.z; m[7] = m1.w;
          s = unpack_state(st);
          if (s.x < 1 || s.x > v.W - 2 || s.y < 1 || s.y > v.H - 2 || s.scen >= v.pool_count) {
            latch_error(v.err, CRAFT_EINVAL, slot);     // never initialised by reset / set_state
            live = false;
          }
        }
        if (live) {
          task_word = s_task[s.task];
          // pool[scenario] (L2-resident) -> the pristine row and the grid row, 4 x 16 B in flight
          const uint4* src = reinterpret_cast<const uint4*>(v.pool + (size_t)s.scen * v.CS);
          const int nchunk = v.CS >> 4;
          for (int q0 = 0; q0 < nchunk; q0 += 4) {
            uint4 cq[4];
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (q0 + j < nchunk) cq[j] = src[q0 + j];
#pragma unroll
            for (int j = 0; j < 4; ++j)
              if (q0 + j < nchunk) {
                const int q = 4 * (q0 + j);
                pw[q + 0] = gw[q + 0] = cq[j].x; pw[q + 1] = gw[q + 1] = cq[j].y;
                pw[q + 2] = gw[q + 2] = cq[j].z; pw[q + 3] = gw[q + 3] = cq[j].w;
              }
          }
          clr = 0;
#pragma unroll
          for (int w = 0; w < 8; ++w) {                 // cells cleared this episode
            uint32_t mm = m[w];
            while (mm) {
              const int c = w * 32 + __ffs(mm) - 1;
              g[c] = 0;
              const uint32_t nc = (clr >> 24) & 3;
              clr = (clr >> 31) ? clr
                  : nc < 3 ? ((clr & 0x00ffffffu) | ((uint32_t)c << (8 * nc)) | ((nc + 1) << 24)) : (1u << 31);
              mm &= mm - 1;
            }
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        ag = tick_c(k0);
      }
      if (want_obs) scatter_d(ag, s_obs);               // D(k0) -> buffer 0
    }

    // ---- the pipeline, one barrier per tick: between barriers k and k+1 the consumers stream
    // E(k) from buffer k and clear it, while the producer runs C(k+1) and D(k+1) into buffer
    // k+1 (cleared by the consumers before barrier k).  Same barrier count on both roles. ------
    if (!want_obs) {                                    // workgroup-uniform: the producer alone
      if (tid < TILE)
        for (int k = k0; k + 1 < k1; ++k) {
          const unsigned long long t0 = CRAFT_NOW();
          tick_c(k + 1);
          PACC(1, CRAFT_NOW() - t0);
        }
    } else if (tid < 64) {
      __syncthreads();                                  // D(k0) complete
      for (int k = k0; k < k1; ++k) {
        const unsigned long long t0 = CRAFT_NOW();
        unsigned long long tb = t0;
        if (k + 1 < k1) {
          uint32_t ag = 0;
          if (tid < TILE) ag = tick_c(k + 1);
          const unsigned long long t1 = CRAFT_NOW();
          PACC(1, t1 - t0);
          scatter_d(ag, s_obs + ((k + 1 - k0) & 1) * obs_buf);
          tb = CRAFT_NOW();
          PACC(2, tb - t1);
        }
        __syncthreads();
        PACC(3, CRAFT_NOW() - tb);
      }
    } else {
      const int et = tid - 64;
      __syncthreads();
      for (int k = k0; k < k1; ++k) {
        const unsigned long long t0 = CRAFT_NOW();
        const int64_t r = (a.tick0 + k) % a.ring;
        void* out = static_cast<uint8_t*>(a.obs) + r * n * (int64_t)F * esz;
#ifndef CRAFT_ABL_NOE
        stream_obs<FMT, NT - 64, true>(s_obs + ((k - k0) & 1) * obs_buf, out, env0, F, nE,
                                       v.obs_policy, et);
#else
        (void)out;
#endif
        const unsigned long long t1 = CRAFT_NOW();
        PACC(4, t1 - t0);
        __syncthreads();
        PACC(5, CRAFT_NOW() - t1);
      }
    }
#ifdef CRAFT_STAMPS
    if ((tid == 0 || tid == 64) && v.stamps)            // per-workgroup phase totals
      for (int q = 1; q <= 5; ++q)
        if (acc[q]) {
          atomicAdd(reinterpret_cast<unsigned long long*>(v.stamps) + 8 * (int64_t)blockIdx.x + q, acc[q]);
          acc[q] = 0;
        }
#endif

    // ---- publish the tile for the unit (t, c + 1): its state, and every output this unit wrote ----
    // (a later unit may rewrite the same ring slots from another XCD, so the release must cover
    // the observation stores of all waves, not only the state)
    // When no ring slot is written twice in this launch (ring >= n_ticks), only the state
    // passes between units: it is stored write-through (sc1) and published with no
    // release fence (Guideline 16 R1), which leaves this XCD's L2 alone.
    const bool state_only = a.ring >= a.n_ticks;
    const bool handoff = c + 1 < n_chunks;
    if (tid < TILE && live) {
      // this episode's cleared cells: non-empty in pool[scenario], empty in the grid row
      uint32_t m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int q = 0; q < (v.CS >> 2); ++q) {
        const uint32_t p = pw[q], cc = gw[q];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const bool cleared = ((p >> (8 * b)) & 0xffu) != 0 && ((cc >> (8 * b)) & 0xffu) == 0;
          const int cell = 4 * q + b;
          if (cleared) m[cell >> 5] |= 1u << (cell & 31);
        }
      }
      if (handoff && state_only) {
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
    }
    if (handoff && state_only) {
      if (tid < 64) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");    // the storing wave drains
        if (tid == 0)
          __hip_atomic_store((gu32*)(a.tile_done + t), (uint32_t)(c + 1), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
    } else if (handoff) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave drains
      __syncthreads();
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");   // write back this XCD's dirty L2 lines
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // keep: the compiler may drop the fence's own
        __hip_atomic_store((gu32*)(a.tile_done + t), (uint32_t)(c + 1), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    __syncthreads();                                    // s_ctrl and the LDS rows are reused
  }
#undef CRAFT_NOW
#undef PACC
#undef PACC_C

  STAMP_END();
  if (tid == 0) {
    unsigned long long* srow = reinterpret_cast<unsigned long long*>(v.stats_part + 4 * (int64_t)blockIdx.x);
    atomicAdd(srow + 0, (unsigned long long)n_succ);
    atomicAdd(srow + 1, (unsigned long long)n_end);
    atomicAdd(srow + 2, (unsigned long long)n_step);
  }
}

// Host side of one window.  Waves per SIMD: the producer wave of w=3 fits 128
// VGPRs; wider windows get more.
template <int WIN, int TILE, int NT, int FMT, bool GIVEN>
static hipError_t launch_rollout_one(const SimView& v, const RolloutArgs& a, size_t lds, hipStream_t st) {
  const int64_t tiles = (v.n_envs + TILE - 1) / TILE;
  if (tiles == 0 || a.n_ticks == 0) return hipSuccess;
  constexpr int WPE = WIN == 3 ? 4 : 2;
  {                        // double-buffered rows past 64 KiB
    const hipError_t e = ensure_lds<&rollout_kernel<WIN, TILE, NT, FMT, WPE, GIVEN>>(lds);
    if (e != hipSuccess) return e;
  }
  // persistent workgroups: what the chip holds at once (occupancy of this kernel at this LDS
  // size), spread so that every workgroup runs the same number of units (no partial last round)
  const int resident = resident_workgroups<&rollout_kernel<WIN, TILE, NT, FMT, WPE, GIVEN>>(NT, lds);
  const int64_t units = tiles * (int64_t)((a.n_ticks + a.chunk - 1) / a.chunk);
  const int64_t rounds = (units + resident - 1) / resident;
  // every workgroup owns one stats_part row; the handle has (n_envs + 15) / 16 of them
  const int64_t rows = (v.n_envs + kMinTileEnvs - 1) / kMinTileEnvs;
  const int64_t grid = std::min<int64_t>((units + rounds - 1) / rounds, rows);
  if (a.grid_out) *a.grid_out = grid;
  hipLaunchKernelGGL((rollout_kernel<WIN, TILE, NT, FMT, WPE, GIVEN>), dim3((unsigned)grid), dim3(NT), lds, st, v, a);
  return hipGetLastError();
}

// The split-producer kernel (craft_rollout_split.h) for 16- and 32-env tiles: NT threads =
// C wave + D wave + NT / 64 - 2 streaming waves, 5 waves per SIMD.
template <int WIN, int TILE, int NT, int FMT, bool GIVEN>
static hipError_t launch_rollout_split_one(const SimView& v, const RolloutArgs& a, hipStream_t st) {
  const int64_t tiles = (v.n_envs + TILE - 1) / TILE;
  if (tiles == 0 || a.n_ticks == 0) return hipSuccess;
  constexpr int WPE = WIN == 3 ? CRAFT_SPLIT_WPE : 2;
  // the continuous-pipeline instantiation exists for the default 3x3 shape only
  constexpr bool kFlatShape = WIN == 3 && TILE == 32 && NT == 512;
  const bool flat = kFlatShape && a.flat;
  const size_t lds = (size_t)split_lds_bytes(TILE, v.GS, v.F, v.CS, flat);
  auto kern = flat ? rollout_split_kernel<WIN, TILE, NT, FMT, WPE, GIVEN, kFlatShape>
                   : rollout_split_kernel<WIN, TILE, NT, FMT, WPE, GIVEN, false>;
  {
    const hipError_t e = flat ? ensure_lds<&rollout_split_kernel<WIN, TILE, NT, FMT, WPE, GIVEN, kFlatShape>>(lds)
                              : ensure_lds<&rollout_split_kernel<WIN, TILE, NT, FMT, WPE, GIVEN, false>>(lds);
    if (e != hipSuccess) return e;
  }
  // persistent workgroups: what the device holds at once (cached per device and LDS size)
  const int resident = flat ? resident_workgroups<&rollout_split_kernel<WIN, TILE, NT, FMT, WPE, GIVEN, kFlatShape>>(NT, lds)
                            : resident_workgroups<&rollout_split_kernel<WIN, TILE, NT, FMT, WPE, GIVEN, false>>(NT, lds);
  const int64_t units = tiles * (int64_t)((a.n_ticks + a.chunk - 1) / a.chunk);
  const int64_t rounds = (units + resident - 1) / resident;
  const int64_t rows = (v.n_envs + kMinTileEnvs - 1) / kMinTileEnvs;
  const int64_t grid = std::min<int64_t>((units + rounds - 1) / rounds, rows);
  if (a.grid_out) *a.grid_out = grid;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(NT), lds, st, v, a);
  return hipGetLastError();
}

template <int WIN, int TILE, int NT>
static hipError_t launch_rollout_split(const SimView& v, const RolloutArgs& a, hipStream_t st) {
  const bool given = a.actions != nullptr;
  switch (v.obs_fmt) {
    case CRAFT_OBS_BF16: return given ? launch_rollout_split_one<WIN, TILE, NT, CRAFT_OBS_BF16, true>(v, a, st)
                                      : launch_rollout_split_one<WIN, TILE, NT, CRAFT_OBS_BF16, false>(v, a, st);
    case CRAFT_OBS_U8: return given ? launch_rollout_split_one<WIN, TILE, NT, CRAFT_OBS_U8, true>(v, a, st)
                                    : launch_rollout_split_one<WIN, TILE, NT, CRAFT_OBS_U8, false>(v, a, st);
    default: return given ? launch_rollout_split_one<WIN, TILE, NT, CRAFT_OBS_F32, true>(v, a, st)
                          : launch_rollout_split_one<WIN, TILE, NT, CRAFT_OBS_F32, false>(v, a, st);
  }
}

template <int WIN, int TILE, int NT>
static hipError_t launch_rollout_fmt(const SimView& v, const RolloutArgs& a, size_t lds, hipStream_t st) {
  const bool given = a.actions != nullptr;
  switch (v.obs_fmt) {
    case CRAFT_OBS_BF16: return given ? launch_rollout_one<WIN, TILE, NT, CRAFT_OBS_BF16, true>(v, a, lds, st)
                                      : launch_rollout_one<WIN, TILE, NT, CRAFT_OBS_BF16, false>(v, a, lds, st);
    case CRAFT_OBS_U8: return given ? launch_rollout_one<WIN, TILE, NT, CRAFT_OBS_U8, true>(v, a, lds, st)
                                    : launch_rollout_one<WIN, TILE, NT, CRAFT_OBS_U8, false>(v, a, lds, st);
    default: return given ? launch_rollout_one<WIN, TILE, NT, CRAFT_OBS_F32, true>(v, a, lds, st)
                          : launch_rollout_one<WIN, TILE, NT, CRAFT_OBS_F32, false>(v, a, lds, st);
  }
}

// threads per tile workgroup: 0 = the default of the tile width, else 128 / 256 / 512.
template <int WIN>
static hipError_t launch_rollout_win(int tile, int threads, const SimView& v, const RolloutArgs& a,
                                     size_t lds, hipStream_t st) {
  switch (tile) {
    case 16: return threads == 128 ? launch_rollout_fmt<WIN, 16, 128>(v, a, lds, st)
                  : threads == 320 ? launch_rollout_split<WIN, 16, 320>(v, a, st)
                  : threads == 384 ? launch_rollout_split<WIN, 16, 384>(v, a, st)
                  : threads == 512 ? launch_rollout_split<WIN, 16, 512>(v, a, st)
                                   : launch_rollout_fmt<WIN, 16, 256>(v, a, lds, st);
    case 32: return threads == 128 ? launch_rollout_fmt<WIN, 32, 128>(v, a, lds, st)
                  : threads == 320 ? launch_rollout_split<WIN, 32, 320>(v, a, st)
                  : threads == 384 ? launch_rollout_split<WIN, 32, 384>(v, a, st)
                  : threads == 512 ? launch_rollout_split<WIN, 32, 512>(v, a, st)
                                   : launch_rollout_fmt<WIN, 32, 256>(v, a, lds, st);
    default: return threads == 256 ? launch_rollout_fmt<WIN, 64, 256>(v, a, lds, st)
                                   : launch_rollout_fmt<WIN, 64, 512>(v, a, lds, st);
  }
}

hipError_t launch_rollout_w3(int tile, int threads, const SimView& v, const RolloutArgs& a, size_t lds, hipStream_t st);
hipError_t launch_rollout_w5(int tile, int threads, const SimView& v, const RolloutArgs& a, size_t lds, hipStream_t st);
hipError_t launch_rollout_w7(int tile, int threads, const SimView& v, const RolloutArgs& a, size_t lds, hipStream_t st);

}  // namespace craft
