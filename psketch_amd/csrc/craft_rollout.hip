// craft_rollout.hip — K rollout ticks in one launch (craft_rollout).
//
// craft_step pays, every tick, for a prologue that moves no observation bytes:
// the state/inventory/mask loads, the scenario row from L2, the transition and
// the scatter.  All workgroups of a launch run that prologue together, so HBM
// idles for its duration (phase stamps).  Here each workgroup keeps
// its TILE envs on chip for K ticks — state and mask in wave 0's registers, grid
// rows and inventories in LDS — and loops C -> D -> E with no global
// synchronisation, so one workgroup's transition and scatter overlap the
// observation stores of the others on the same CU.  State goes back to HBM once,
// after the last tick.
//
// Tick k is exactly craft_step(tick0 + k) with the hashed (or given) actions and
// writes its outputs to ring slot (tick0 + k) % ring, as a driver cycling craft_step
// over a ring of R buffers would.  Used where actions do not depend on the
// observations (random rollouts, configs 2 and 4; or replayed action tables).
#include "craft_obs.h"

namespace craft {

template <int WIN, int TILE>
__global__ __launch_bounds__(kThreads) void rollout_kernel(SimView v, RolloutArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const LdsLayout lay = lds_layout(TILE, v.GS, v.F);
  uint8_t* s_grid = smem;
  uint8_t* s_obs = smem + lay.obs;
  uint8_t* s_inv = smem + lay.inv;
  uint16_t* s_task = reinterpret_cast<uint16_t*>(smem + lay.task);
  uint8_t* s_rc = smem + lay.rc;
  uint32_t* s_agent = reinterpret_cast<uint32_t*>(smem + lay.agent);

  const int tid = threadIdx.x;
  const int64_t n = v.n_envs;
  const int64_t env0 = (int64_t)blockIdx.x * TILE;
  const int nE = (int)min((int64_t)TILE, n - env0);
  const bool want_obs = a.obs != nullptr;
  const int F = v.F;
  const int esz = v.obs_fmt == CRAFT_OBS_F32 ? 4 : (v.obs_fmt == CRAFT_OBS_BF16 ? 2 : 1);

  // ---- A (once): wave 0 loads its envs -------------------------------------------------------
  // Loop-carried per lane: the packed state word and the init word only.  The
  // cleared-cell mask is not carried: cells are only ever cleared, so this
  // episode's mask is exactly {c : pool[c] != 0 and grid[c] == 0} and is rebuilt
  // from the LDS row when the state goes back to HBM.
  Agent s{};
  uint64_t st = 0;
  uint32_t init_word = 0;
  bool live = false;
  const int64_t slot = env0 + tid;
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
  if (tid < TILE) {
    for (int t = tid; t < v.n_tasks; t += TILE) s_task[t] = v.task_tab[t];
    for (int t = tid; t < CRAFT_MAX_RECIPES * kRecipeBytes / 4; t += TILE)
      reinterpret_cast<uint32_t*>(s_rc)[t] = reinterpret_cast<const uint32_t*>(v.rc)[t];
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
        latch_error(v.err, CRAFT_EINVAL, slot);   // never initialised by reset / set_state
        live = false;
      }
    }
    if (live) {
      load_row();
#pragma unroll
      for (int w = 0; w < 8; ++w) {                         // cells cleared this episode
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
  }

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

  // Software pipeline, two barriers per tick: after the scatter D(k), wave 0 runs
  // the transition C(k+1) while waves 1-3 stream E(k) and clear the rows they
  // read, so the latency-bound transition hides under the observation stores.
  if (tid < TILE) {
    if (a.n_ticks > 0) tick_c(0);
  } else if (want_obs && tid >= 64) {
    uint4* z = reinterpret_cast<uint4*>(s_obs);
    const int n16 = (nE * F + 15) >> 4;
    for (int i = tid - 64; i < n16; i += kThreads - 64) z[i] = make_uint4(0, 0, 0, 0);
  }
  for (int k = 0; k < a.n_ticks; ++k) {
    if (!want_obs) {                 // workgroup-uniform: wave 0 alone runs the ticks
      if (tid < TILE && k + 1 < a.n_ticks) tick_c(k + 1);
      continue;
    }
    __syncthreads();                 // C(k) and the cleared rows are visible
    scatter_features<WIN, TILE>(v, s_grid, s_inv, s_agent, s_obs, nE, tid);
    __syncthreads();                 // rows complete; C(k+1) may now change grids and agents
    if (tid < 64) {
      if (tid < TILE && k + 1 < a.n_ticks) tick_c(k + 1);
    } else {
      const int64_t r = (a.tick0 + k) % a.ring;
      void* out = static_cast<uint8_t*>(a.obs) + r * n * (int64_t)F * esz;
      const int et = tid - 64;
      switch (v.obs_fmt) {
        case CRAFT_OBS_BF16:
          stream_obs<CRAFT_OBS_BF16, kThreads - 64, true>(s_obs, out, env0, F, nE, v.obs_policy, et); break;
        case CRAFT_OBS_U8:
          stream_obs<CRAFT_OBS_U8, kThreads - 64, true>(s_obs, out, env0, F, nE, v.obs_policy, et); break;
        default:
          stream_obs<CRAFT_OBS_F32, kThreads - 64, true>(s_obs, out, env0, F, nE, v.obs_policy, et); break;
      }
    }
  }

  // ---- write back (once) -------------------------------------------------------------------------
  if (tid < TILE) {
    if (live) {
      v.state[slot] = st;
      v.inv[2 * slot] = make_uint4(ivw[0], ivw[1], ivw[2], ivw[3]);
      v.inv[2 * slot + 1] = make_uint4(ivw[4], ivw[5], ivw[6], ivw[7]);
      // this episode's cleared cells: non-empty in pool[scenario], empty in the LDS row
      const uint32_t* row = reinterpret_cast<const uint32_t*>(v.pool + (size_t)s.scen * v.CS);
      const uint32_t* cur = reinterpret_cast<const uint32_t*>(g);
      uint32_t m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int q = 0; q < (v.CS >> 2); ++q) {
        const uint32_t p = row[q], c = cur[q];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const bool cleared = ((p >> (8 * b)) & 0xffu) != 0 && ((c >> (8 * b)) & 0xffu) == 0;
          const int cell = 4 * q + b;
          if (cleared) m[cell >> 5] |= 1u << (cell & 31);
        }
      }
      v.mask[2 * slot] = make_uint4(m[0], m[1], m[2], m[3]);
      v.mask[2 * slot + 1] = make_uint4(m[4], m[5], m[6], m[7]);
    }
    if (tid == 0) {
      unsigned long long* srow = reinterpret_cast<unsigned long long*>(v.stats_part + 4 * (int64_t)blockIdx.x);
      atomicAdd(srow + 0, (unsigned long long)n_succ);
      atomicAdd(srow + 1, (unsigned long long)n_end);
      atomicAdd(srow + 2, (unsigned long long)n_step);
    }
  }
}

template <int WIN, int TILE>
static hipError_t launch_rollout_one(const SimView& v, const RolloutArgs& a, size_t lds, hipStream_t st) {
  const int64_t tiles = (v.n_envs + TILE - 1) / TILE;
  if (tiles == 0 || a.n_ticks == 0) return hipSuccess;
  hipLaunchKernelGGL((rollout_kernel<WIN, TILE>), dim3((unsigned)tiles), dim3(kThreads), lds, st, v, a);
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
