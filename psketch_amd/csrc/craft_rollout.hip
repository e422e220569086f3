// craft_rollout.hip — K rollout ticks in one launch (craft_rollout).
//
// craft_step pays, every tick, for a prologue that moves no observation bytes:
// the state/inventory/mask loads, the scenario row from L2, the transition and
// the scatter.  All workgroups of a launch run that prologue together, so HBM
// idles for its duration (phase stamps).  Here a workgroup keeps a
// tile of envs on chip for a chunk of ticks — state in wave 0's registers, grid
// rows and inventories in LDS — and software-pipelines the ticks: the transition
// of tick k+1 (wave 0) runs while the other waves stream tick k's observation.
//
// Work distribution.  Workgroups do not stream at equal speed (per-workgroup
// stamps, tools/rollout_stamps.py: durations from 0.55x to 1x of the launch, odd
// XCDs slower), so a static tile-per-workgroup launch waits for its slowest
// workgroups.  The launch is instead cut into units (tile t, chunk c of `chunk`
// ticks), handed out in chunk-major order from a queue counter; a unit's env
// state goes back to HBM at its end and the unit (t, c+1) may run on any other
// workgroup.  That hand-off follows cdna_hip_programming.md Guideline 16 /
// MI355X_MICROARCH.md (valid forms, plain-store producer): every storing wave
// drains (s_waitcnt vmcnt(0)), a workgroup barrier, one lane's agent-scope
// release (which also pushes this unit's observation stores out of the XCD's L2,
// so a later unit rewriting the same ring slot from another XCD lands last), a
// second drain, and a relaxed agent-scope store tile_done[t] = c + 1; the
// consumer wave polls that word relaxed, then one agent-scope acquire, then
// plain loads.  Queue and flags are zeroed by a memset
// ahead of every launch.  A unit waits only for its own tile's previous chunk,
// which was handed out earlier and is held by a running workgroup, so the queue
// cannot deadlock; spins are bounded anyway.
//
// Tick k is exactly craft_step(tick0 + k) with the hashed (or given) actions and
// writes its outputs to ring slot (tick0 + k) % ring, as a driver cycling craft_step
// over a ring of R buffers would.  Used where actions do not depend on the
// observations (random rollouts, configs 2 and 4; or replayed action tables).
#include "craft_obs.h"

namespace craft {

typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

// NT threads per workgroup: wave 0 runs the transitions, waves 1.. stream.
template <int WIN, int TILE, int NT>
__global__ __launch_bounds__(NT, WIN == 3 ? 4 : 2) void rollout_kernel(SimView v, RolloutArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const LdsLayout lay = lds_layout(TILE, v.GS, v.F);
  uint8_t* s_grid = smem;
  uint8_t* s_obs = smem + lay.obs;
  uint8_t* s_inv = smem + lay.inv;
  uint16_t* s_task = reinterpret_cast<uint16_t*>(smem + lay.task);
  uint8_t* s_rc = smem + lay.rc;
  uint32_t* s_agent = reinterpret_cast<uint32_t*>(smem + lay.agent);
  uint32_t* s_ctrl = reinterpret_cast<uint32_t*>(smem + lay.ctrl);

  STAMP(0);
  const int tid = threadIdx.x;
  const int64_t n = v.n_envs;
  const bool want_obs = a.obs != nullptr;
  const int F = v.F;
  const int esz = v.obs_fmt == CRAFT_OBS_F32 ? 4 : (v.obs_fmt == CRAFT_OBS_BF16 ? 2 : 1);
  const int n_tiles = (int)((n + TILE - 1) / TILE);
  const int n_chunks = (a.n_ticks + a.chunk - 1) / a.chunk;
  const uint32_t n_units = (uint32_t)n_tiles * (uint32_t)n_chunks;

  // Per lane of wave 0, for the current unit: the packed state word and the init
  // word.  The cleared-cell mask is not carried: cells are only ever cleared, so
  // this episode's mask is exactly {c : pool[c] != 0 and grid[c] == 0} and is
  // rebuilt from the LDS row when the state goes back to HBM.
  Agent s{};
  uint64_t st = 0;
  uint32_t init_word = 0;
  bool live = false;
  int64_t slot = 0;
  uint8_t* g = s_grid + tid * v.GS;
  uint8_t* iv = s_inv + tid * kInvStride;
  uint32_t* ivw = reinterpret_cast<uint32_t*>(iv);
  uint32_t n_succ = 0, n_end = 0, n_step = 0;               // wave-uniform running sums
  // pool[scenario] -> the env's LDS row (L2-resident pool), 4 x 16 B in flight at a
  // time: the row is reloaded only on an episode restart, and the registers it
  // would otherwise pin are the occupancy of the whole tick loop.
  auto load_row = [&]() {
    const uint4* src = reinterpret_cast<const uint4*>(v.pool + (size_t)s.scen * v.CS);
    uint32_t* dst = reinterpret_cast<uint32_t*>(g);
    const int nchunk = v.CS >> 4;
    for (int q0 = 0; q0 < nchunk; q0 += 4) {
      uint4 c[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (q0 + j < nchunk) c[j] = src[q0 + j];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (q0 + j < nchunk) {
          const int q = q0 + j;
          dst[4 * q + 0] = c[j].x; dst[4 * q + 1] = c[j].y; dst[4 * q + 2] = c[j].z; dst[4 * q + 3] = c[j].w;
        }
    }
  };

  // ---- C: the do_rollout tick of wave 0's envs (trainers/imitation.py:59-73) ------------------
  auto tick_c = [&](int k) {
    const int64_t tick = a.tick0 + k;
    const int64_t r = tick % a.ring;
    int d = 0, succ = -1, counted = 0;
    s = unpack_state(st);
    if (live) {
      int act;
      if (a.actions) {
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
      if (d) {
        // satisfies() of the pre-step state (the LDS row already has this episode's clears)
        const uint32_t tt = s_task[s.task];
        const int goal = tt & 0xf, arg = (tt >> 4) & 0xff;
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
        load_row();
      } else if (d && !s.frozen) {
        s.frozen = 1;
        s.timer = max(s.timer, 0);
      } else if (!d) {
        bool inv_changed = false, mask_changed = false;
        uint32_t m_unused[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // the LDS row is the record
        if (act < 0 || act >= CRAFT_N_ACTIONS) latch_error(v.err, CRAFT_EBADACTION, slot);
        else transition(v, s_rc, g, iv, s, m_unused, act, inv_changed, mask_changed);
      }
      st = pack_state(s);
      const int64_t o = r * n + slot;
      if (a.done) a.done[o] = (uint8_t)d;
      if (a.sat) a.sat[o] = (int8_t)succ;
      if (a.reward) a.reward[o] = (counted && d && succ == 1) ? 1.0f : 0.0f;
    }
    s_agent[tid] = live ? ((uint32_t)s.x | ((uint32_t)s.y << 8) | ((uint32_t)s.dir << 16) | (1u << 24)) : 0u;
    const uint64_t bs = __ballot(live && counted && d && succ == 1);
    const uint64_t be = __ballot(live && counted && d);
    const uint64_t bt = __ballot(live && counted);
    n_succ += (uint32_t)__popcll(bs);
    n_end += (uint32_t)__popcll(be);
    n_step += (uint32_t)__popcll(bt);
  };

  // ---- once per workgroup: static tables, cleared observation rows ------------------------------
  if (tid < TILE) {
    for (int t = tid; t < v.n_tasks; t += TILE) s_task[t] = v.task_tab[t];
    for (int t = tid; t < CRAFT_MAX_RECIPES * kRecipeBytes / 4; t += TILE)
      reinterpret_cast<uint32_t*>(s_rc)[t] = reinterpret_cast<const uint32_t*>(v.rc)[t];
  }
  if (want_obs) {
    uint4* z = reinterpret_cast<uint4*>(s_obs);
    const int n16 = (TILE * F + 15) >> 4;
    for (int i = tid; i < n16; i += NT) z[i] = make_uint4(0, 0, 0, 0);
  }

  for (;;) {
    // ---- next unit ------------------------------------------------------------------------------
    if (tid == 0) s_ctrl[0] = (uint32_t)atomicAdd(a.queue, 1ull);
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
          load_row();
#pragma unroll
          for (int w = 0; w < 8; ++w) {                 // cells cleared this episode
            uint32_t mm = m[w];
            while (mm) {
              g[w * 32 + __ffs(mm) - 1] = 0;
              mm &= mm - 1;
            }
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        tick_c(k0);
      }
    }

    // ---- software pipeline, two barriers per tick: after the scatter D(k), wave 0 runs the
    // transition C(k+1) while the other waves stream E(k) and clear the rows they read --------
    for (int k = k0; k < k1; ++k) {
      if (!want_obs) {                                  // workgroup-uniform: wave 0 alone
        if (tid < TILE && k + 1 < k1) tick_c(k + 1);
        continue;
      }
      __syncthreads();                                  // C(k) and the cleared rows are visible
      scatter_features<WIN, TILE, NT>(v, s_grid, s_inv, s_agent, s_obs, nE, tid);
      __syncthreads();                                  // rows complete; C(k+1) may change grids
      if (tid < 64) {
        if (tid < TILE && k + 1 < k1) tick_c(k + 1);
      } else {
        const int64_t r = (a.tick0 + k) % a.ring;
        void* out = static_cast<uint8_t*>(a.obs) + r * n * (int64_t)F * esz;
        const int et = tid - 64;
        switch (v.obs_fmt) {
          case CRAFT_OBS_BF16:
            stream_obs<CRAFT_OBS_BF16, NT - 64, true>(s_obs, out, env0, F, nE, v.obs_policy, et); break;
          case CRAFT_OBS_U8:
            stream_obs<CRAFT_OBS_U8, NT - 64, true>(s_obs, out, env0, F, nE, v.obs_policy, et); break;
          default:
            stream_obs<CRAFT_OBS_F32, NT - 64, true>(s_obs, out, env0, F, nE, v.obs_policy, et); break;
        }
      }
    }

    // ---- publish the tile for the unit (t, c + 1): its state, and every output this unit wrote ----
    // (a later unit may rewrite the same ring slots from another XCD, so the release must cover
    // the observation stores of all waves, not only the state)
    // When no ring slot is written twice in this launch (ring >= n_ticks), only the state
    // passes between units: it is stored write-through (sc1) and published with no
    // release fence (Guideline 16 R1), which leaves this XCD's L2 alone.
    const bool state_only = a.ring >= a.n_ticks;
    const bool handoff = c + 1 < n_chunks;
    if (tid < TILE && live) {
      // this episode's cleared cells: non-empty in pool[scenario], empty in the LDS row
      const uint32_t* row = reinterpret_cast<const uint32_t*>(v.pool + (size_t)s.scen * v.CS);
      const uint32_t* cur = reinterpret_cast<const uint32_t*>(g);
      uint32_t m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int q = 0; q < (v.CS >> 2); ++q) {
        const uint32_t p = row[q], cc = cur[q];
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

  STAMP_END();
  if (tid == 0) {
    unsigned long long* srow = reinterpret_cast<unsigned long long*>(v.stats_part + 4 * (int64_t)blockIdx.x);
    atomicAdd(srow + 0, (unsigned long long)n_succ);
    atomicAdd(srow + 1, (unsigned long long)n_end);
    atomicAdd(srow + 2, (unsigned long long)n_step);
  }
}

template <int WIN, int TILE>
static hipError_t launch_rollout_one(const SimView& v, const RolloutArgs& a, size_t lds, hipStream_t st) {
  const int64_t tiles = (v.n_envs + TILE - 1) / TILE;
  if (tiles == 0 || a.n_ticks == 0) return hipSuccess;
  constexpr int NT = TILE == 64 ? 256 : 128;
  // persistent workgroups: at most what the chip holds (8 per CU), never more than the tiles
  const int64_t grid = tiles < 8 * 256 ? tiles : 8 * 256;
  hipLaunchKernelGGL((rollout_kernel<WIN, TILE, NT>), dim3((unsigned)grid), dim3(NT), lds, st, v, a);
  return hipGetLastError();
}

template <int TILE>
static hipError_t launch_rollout_win(int win, const SimView& v, const RolloutArgs& a, size_t lds,
                                     hipStream_t st) {
  switch (win) {
    case 3: return launch_rollout_one<3, TILE>(v, a, lds, st);
    case 5: return launch_rollout_one<5, TILE>(v, a, lds, st);
    default: return launch_rollout_one<7, TILE>(v, a, lds, st);
  }
}

hipError_t launch_rollout(int win, int tile, const SimView& v, const RolloutArgs& a, size_t lds,
                          hipStream_t st) {
  switch (tile) {
    case 16: return launch_rollout_win<16>(win, v, a, lds, st);
    case 32: return launch_rollout_win<32>(win, v, a, lds, st);
    default: return launch_rollout_win<64>(win, v, a, lds, st);
  }
}

}  // namespace craft
