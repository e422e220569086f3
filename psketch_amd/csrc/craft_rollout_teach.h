// craft_rollout_teach.h — K rollout ticks in one launch with the DemonstrationTeacher's label of
// every env's new state every tick (craft_rollout_teach): config 5's DAgger labels
// (trainers/imitation.py:43-57) and make_data.get_reference_actions' demonstrations
// (make_data.py:146-152, the actions ARE the labels), without a launch per tick.
//
// One launch per tick (craft_step_teach) pays the tick's prologue every tick: the loads, the
// transition and the scatter run on every workgroup before the first observation byte leaves
// (~7 us of ~29 at 65,536 envs).  Here a persistent workgroup keeps a tile of envs on
// chip for all K ticks, as the split rollout kernel does (craft_rollout_split.h), with one more
// wave for the teacher.  512 threads, one barrier per interval; interval i of a tile runs
//   wave 0       C(i+1): the transitions (one lane per env) into grid / inventory buffer (i+1) & 1;
//   wave 1       D(i):   the observation scatter of item i from buffer i & 1;
//   waves 2..6   E(i-1): the observation stream of the item before, to HBM; wave 2 also stores the
//                        teacher's finished label rows, in item order, waves 3..6 item i's done,
//                        success, reward and action record (one array each);
//   wave 7       T(i):   the teacher on item i's post-step rows (buffer i & 1, which C(i+2)
//                        overwrites one interval later).
//
// The teacher wave.  Its walk (find_incomplete_subtask, one lane per env) must finish inside the
// interval, but a BFS chain (~30 dependent levels) is longer than an interval (~4 us), so the
// BFS is decoupled from the item:
//   * the hint walk (find_incomplete_subtask) is a table lookup: the leaf as a function of the
//     task's satisfies() predicates (craft_host.h hint_tables), three rounds of LDS loads;
//   * a go[X] leaf on a grid the teacher table lists (the pool row minus a subset of its listed
//     clearable cells) issues the table's answer load (LDS-DMA) and decodes it kRtLag walks later
//     (policy actions) or right away (label actions);
//   * any other go[X] leaf becomes a BFS job: the leaf lane builds the band bitsets of its grid
//     row while the row is still current and queues them in LDS;
//   * between its own duties the wave runs the queued jobs, one BFS level per step on 16 quads
//     (lane q of a quad: the states entered by action q, as bfs_closest<NW, 4>), each quad a
//     small state machine (forward, reachability flood, backward), taking a new job as soon as
//     its last one ends.  Before every barrier, with jobs queued, it steps until all other waves
//     have arrived (an LDS arrival counter), so the BFS fills the interval's slack and never
//     holds the barrier for more than one level; with none it goes straight to the barrier.
// Labels go into LDS label rows (item g -> row g & 7, with a count of labels still pending); the
// teacher wave issues no global store at all (a store would make its next table load wait:
// vmcnt counts loads and stores in issue order).  Wave 2 stores each row once complete, strictly
// in item order (ring slots may repeat within a launch), and keeps storing while it waits for the
// teacher at each barrier, so a teacher waiting for a free row always gets one.
//
// Action sources, per env: the policy (the hashed draw or given actions) or the label of the
// env's current state (label_actions: every env, make_data's demonstrations; behavior_clone[i]:
// DAgger's mix, imitation.py:56-57).  When labels feed actions, C(i+1) waits for item i's labels,
// and the teacher completes each item inside its interval.
//
// Results are identical to n_ticks craft_step_teach calls with the same action sources (tests:
// tests/test_gpu_rollout_teach.py, tick by tick at 65,536 envs and against the oracle).
#pragma once
#include "craft_host.h"
#include "craft_obs.h"
#include "craft_teach.h"

namespace craft {

constexpr int kRtThreads = 512;        // C, D, 5 streaming waves, the teacher
constexpr int kRtRows = 8;       // label rows in flight: item g -> row g & (kRtRows - 1)
constexpr int kRtQueue = 32;           // BFS jobs waiting for a quad
// Table answers are fetched kRtLag walks ahead of their decode: a load from the table (hundreds of
// MB, random rows) takes longer than an interval while the store stream saturates HBM.
constexpr int kRtLag = 4;
static_assert(kRtRows <= 16 && (kRtRows & (kRtRows - 1)) == 0 && (kRtLag & (kRtLag - 1)) == 0 && kRtLag < kRtRows,
              "rows and lag: powers of two, a fetched item's row still held when it is decoded");
// label row control word: 0 free; kRowFill | pending labels while the teacher fills it (== kRowFill:
// complete); kRowStoring while wave 2 copies it out
constexpr uint32_t kRowFill = 1u << 30, kRowStoring = 1u << 29;
// Every wait in the kernel is bounded (a few hundred ms): past the bound CRAFT_EINVARIANT latches
// and the wave stops waiting, so a broken invariant can never hang the GPU.
constexpr uint32_t kRtSpinCap = 1u << 22;

// LDS carve: table words [kRtLag][64] (the LDS-DMA targets, first, so that their M0 base stays
// below 64 KiB for every window) | grid rows [2][TILE][GS] | pristine rows [TILE][GS] | observation rows
// [2][up16(TILE*F)] | inventory rows [2][TILE][36] | agent words [2][TILE] | teacher info words
// [2][TILE] | the tick's outputs [2][TILE][2] | task table [64] u16 | subtasks [64][4] | recipe
// words [16][3] | control words [8] | label rows [8][4 + TILE] | BFS job queue [32][2 NW + 1] |
// table requests [4][TILE] | their rows [4] | clearable cells [TILE][2] | hint table:
// descriptors [64][4], leaf bytes [2048] | nibble positions [4][TILE] | workshop recipes
// [CRAFT_MAX_KINDS][4] uint2 (SimView::wsr) | the transition wave's labels [2][TILE]
struct RtLds {
  int grid, pristine, obs, inv, agent, tinfo, cout, task, tsub, rc, ctrl, rows, jobs, treq, tval, tpend, tcell, hint,
      tnib, wsr, clab, bytes;
};
__host__ __device__ inline RtLds rt_lds(int tile, int GS, int F, int NW) {
  auto up16 = [](int x) { return (x + 15) & ~15; };
  RtLds l;
  l.tval = 0;                                              // [kRtLag][64] the words fetched (LDS-DMA)
  l.grid = kRtLag * 64 * 4;
  l.pristine = l.grid + 2 * tile * GS;
  l.obs = up16(l.grid + 3 * tile * GS);
  l.inv = l.obs + 2 * up16(tile * F);
  l.agent = up16(l.inv + 2 * tile * kInvStride);
  l.tinfo = l.agent + 2 * tile * 4;
  l.cout = l.tinfo + 2 * tile * 4;                         // [2][TILE][2] C's outputs: flags, action
  l.task = l.cout + 2 * tile * 8;
  l.tsub = up16(l.task + CRAFT_MAX_TASKS * 2);
  l.rc = l.tsub + CRAFT_MAX_TASKS * CRAFT_MAX_SUBTASKS * 4;
  l.ctrl = l.rc + CRAFT_MAX_RECIPES * 12;
  l.rows = up16(l.ctrl + 32);
  l.jobs = up16(l.rows + kRtRows * (4 + tile) * 4);
  l.treq = up16(l.jobs + kRtQueue * (2 * NW + 1) * 4);   // [kRtLag][tile] table-entry requests
  l.tpend = l.treq + kRtLag * tile * 4;                    // [kRtLag] their label rows (~0: none)
  l.tcell = l.tpend + kRtLag * 4;                          // [tile][2] each env's listed clearable cells
  l.hint = up16(l.tcell + tile * 8);                       // craft_host.h hint_tables
  l.tnib = l.hint + CRAFT_MAX_TASKS * 16 + craft_host::kHintLeafCap;   // [kRtLag][tile] nibble in the word
  l.wsr = up16(l.tnib + kRtLag * tile);
  l.clab = l.wsr + CRAFT_MAX_KINDS * 4 * 8;               // [2][tile] the transition wave's labels
  l.bytes = l.clab + 2 * tile * 4;
  return l;
}
// envs per tile: 32 for 3x3 windows (as the split rollout kernel), 16 for wider ones (their
// observation rows: 2 x 34 KB at 5x5)
__host__ __device__ constexpr int rt_tile(int win) { return rt_tile_of(win); }

// The barriers of a unit (one tile, all ticks): the claim, C(0) done, one per interval, the end.
enum { kBClaim = 0, kBC0 = 1, kBTick = 2, kBEnd = 3 };

// ---- the teacher wave's BFS: bfs_closest<NW, 4>'s passes as a per-quad state machine ----------
enum { kQIdle = 0, kQFwd = 1, kQReach = 2, kQBwd = 3 };

// (Only what cannot be recomputed cheaply stays live: the blocked masks and facing sets are
// rebuilt from fr / tgt per level, the start and direction come from the job word.)
template <int NW>
struct QuadBfs {
  int ph = kQIdle;
  int L = -1, chosen = -1, k = 0;
  uint32_t meta = 0;                   // the job's meta word (row, env, start, dir, conn)
  Bits<NW> fr, tgt, V, U, claimed;
};

// Where a bounded wait gave up, for the latched error's slot field (CRAFT_EINVARIANT): bits 60-63
// the wait (1 C's label wait, 2 the stores wave's barrier, 3 its last rows, 4 the teacher idle,
// 5 its BFS), 32-59 the item, 0-31 a state word.
__device__ __forceinline__ int64_t rt_where(uint32_t wait, uint32_t item, uint32_t state) {
  return (int64_t)(((uint64_t)wait << 60) | ((uint64_t)(item & 0xfffffffu) << 32) | state);
}

// Set bits of a wave mask below this lane (v_mbcnt).
__device__ __forceinline__ uint32_t lane_rank(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Job meta word: band start cell p0 (bits 0-7), dir (8-9), connected (10), label row (11-14),
// env in the tile (15-20).
__device__ __forceinline__ uint32_t rt_job_meta(int p0, int d0, int conn, int row, int env) {
  return (uint32_t)p0 | ((uint32_t)d0 << 8) | ((uint32_t)conn << 10) | ((uint32_t)row << 11) |
         ((uint32_t)env << 15);
}

// Byte k (per lane) of an inventory row held in 8 registers.  Written as byte permutes, not as
// r[k >> 2]: hipcc turns an indexed (or index-compared) word into a scratch array.
__device__ __forceinline__ int rbyte(const uint32_t (&r)[8], int k) {
  const uint32_t sel = 0x0c0c0c00u | (uint32_t)(k & 7);             // byte k & 7 of a word pair
  const uint32_t p0 = __builtin_amdgcn_perm(r[1], r[0], sel), p1 = __builtin_amdgcn_perm(r[3], r[2], sel);
  const uint32_t p2 = __builtin_amdgcn_perm(r[5], r[4], sel), p3 = __builtin_amdgcn_perm(r[7], r[6], sel);
  const uint32_t q0 = (k & 8) ? p1 : p0, q1 = (k & 8) ? p3 : p2;
  return (int)((k & 16) ? q1 : q0);
}

// LA: labels feed some env's actions (label_actions or behaviour cloning, the transition wave
// looking them up): it looks every lane's label up, cloning or not, publishes what it decodes,
// and the teacher wave takes those instead of walking (a separate instantiation, so that the
// policy launches keep their register allocation: the shared VGPR budget is tight).
template <int WIN, int TILE, int NW, bool LA>
__global__ __launch_bounds__(kRtThreads, 4) void rollout_teach_kernel(SimView v, RolloutArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr int NT = kRtThreads, NWAVE = NT / 64, TW = NWAVE - 1;   // the teacher is the last wave
  constexpr int NE = NT - 192;                                        // streaming threads (waves 2..6)
  constexpr int P = 64 / TILE;                                        // scatter lanes per env
  constexpr int RW = 4 + TILE;                                        // label row words
  constexpr int JW = 2 * NW + 1;                                      // job words
  static_assert(TILE <= 32 && 64 % TILE == 0, "the teacher's walk: one lane per env");
  auto up16 = [](int x) { return (x + 15) & ~15; };
  const int GS = v.GS, F = v.F, H = v.H, C = v.C;
  const RtLds lay = rt_lds(TILE, GS, F, NW);
  // the recipe words in a VGPR (lane w: word w), loaded while every lane is active (v_readlane)
  const uint32_t rcv = v.rcw[min((int)(threadIdx.x & 63), CRAFT_MAX_RECIPES * 3 - 1)];
  uint8_t* s_grid = smem + lay.grid;                                  // [2][TILE][GS] by item parity
  uint8_t* s_pristine = smem + lay.pristine;                          // [TILE][GS]
  const int obs_buf = up16(TILE * F);
  uint8_t* s_obs = smem + lay.obs;                                    // [2][obs_buf]
  uint8_t* s_inv = smem + lay.inv;                                    // [2][TILE][kInvStride]
  // [2][TILE] x | y<<8 | dir<<16 | live<<24 | frozen<<25 | cells cleared this episode (63 = more) << 26
  uint32_t* s_agent = reinterpret_cast<uint32_t*>(smem + lay.agent);
  uint32_t* s_tinfo = reinterpret_cast<uint32_t*>(smem + lay.tinfo);  // [2][TILE] task|conn<<8|scen<<10
  // [2][TILE] done | (succ + 1) << 1 | counted << 3, and the recorded action: stored by waves 3-6
  uint2* s_cout = reinterpret_cast<uint2*>(smem + lay.cout);
  uint32_t* s_treq = reinterpret_cast<uint32_t*>(smem + lay.treq);    // [kRtLag][TILE] ttab index, ~0 = none
  uint32_t* s_tval = reinterpret_cast<uint32_t*>(smem + lay.tval);    // [kRtLag][64] fetched table words
  uint32_t* s_tpend = reinterpret_cast<uint32_t*>(smem + lay.tpend);  // [kRtLag] their label rows, ~0 none
  uint32_t* s_tcell = reinterpret_cast<uint32_t*>(smem + lay.tcell);  // [TILE][2] tt_cells of the env's row
  uint8_t* s_tnib = smem + lay.tnib;                                  // [kRtLag][TILE] the answer's nibble
  uint16_t* s_task = reinterpret_cast<uint16_t*>(smem + lay.task);
  int32_t* s_tsub = reinterpret_cast<int32_t*>(smem + lay.tsub);
  uint32_t* s_rc = reinterpret_cast<uint32_t*>(smem + lay.rc);
  uint2* s_wsr = reinterpret_cast<uint2*>(smem + lay.wsr);               // SimView::wsr (when set)
  // (label actions) item g's labels as the transition wave decoded them: [g & 1][TILE], 0x100 |
  // label, or 0 where it has none (a BFS answer: the teacher's own walk)
  uint32_t* s_clab = reinterpret_cast<uint32_t*>(smem + lay.clab);
  const uint4* s_hdesc = reinterpret_cast<const uint4*>(smem + lay.hint);   // [task]: predicates, leaf offset
  const uint8_t* s_hleaf = smem + lay.hint + CRAFT_MAX_TASKS * 16;
  // [0] the claimed unit, [1] barrier arrivals, [2] items whose labels are complete (label actions),
  // [3] barriers the teacher has arrived at, [4] items whose labels the transition wave has
  // published in s_clab (label actions)
  uint32_t* s_ctrl = reinterpret_cast<uint32_t*>(smem + lay.ctrl);
  uint32_t* s_rows = reinterpret_cast<uint32_t*>(smem + lay.rows);    // [8][RW]: ctrl, tag = g + 1, tile, ring slot, labels
  uint32_t* s_jobs = reinterpret_cast<uint32_t*>(smem + lay.jobs);    // [32][JW]

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int64_t n = v.n_envs;
#ifdef CRAFT_STAMPS
  // diagnostic builds (tools/rt_stamps.py): per wave 8 shader-clock sums, v.stamps[wg][wave][8]:
  // [0] the hardware barrier, [1] wave 2's wait for the teacher, [2] the role's work (C tick,
  // D scatter, E stream; T walk), T: [3] decode, [4] jobs, [5] BFS steps, [6] idle, [7] steps;
  // wave 0 [6] the workgroup's s_memrealtime span, [7] its shader-clock span
  // (sums in LDS past the carve, so that the stamps cost the waves no registers)
  unsigned long long* stt = reinterpret_cast<unsigned long long*>(smem + lay.bytes) + wave * 8;
  if (lane < 8) stt[lane] = 0ull;
  const uint64_t st_c0 = __builtin_amdgcn_s_memtime(), st_r0 = __builtin_amdgcn_s_memrealtime();
#define RT_CLK() __builtin_amdgcn_s_memtime()
#define RT_ACC(k, t0)                                                                              \
  do {                                                                                             \
    const unsigned long long dt_ = __builtin_amdgcn_s_memtime() - (t0);                            \
    if (lane == 0) __hip_atomic_fetch_add(&stt[k], dt_, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); \
  } while (0)
#else
#define RT_CLK() 0ull
#define RT_ACC(k, t0) ((void)(t0))
#endif
  const bool want_obs = a.obs != nullptr;
  // labels feed some env's actions: (1) each item's row completes inside its interval, before the
  // tick that acts on it; (2) the transition wave looks its labels up itself (hint table, nibble
  // table) and waits only for the row's BFS answers, the teacher's table answers keep their lag
  const int lmode = a.lsync == 2 && !(v.ttab && a.use_table && !v.ttab4) ? 2 : a.lsync ? 1 : 0;
  const bool lsync = lmode != 0;
  const int n_tiles = (int)((n + TILE - 1) / TILE);
  const uint32_t n_units = (uint32_t)n_tiles;                          // one unit per tile: all K ticks

  // ---- once per workgroup: tables, zeroed observation rows, control words ---------------------
  for (int t = tid; t < CRAFT_MAX_TASKS; t += NT) s_task[t] = t < v.n_tasks ? v.task_tab[t] : 0;
  for (int t = tid; t < CRAFT_MAX_TASKS * CRAFT_MAX_SUBTASKS; t += NT)
    s_tsub[t] = t < v.n_tasks * CRAFT_MAX_SUBTASKS ? v.task_sub[t] : 0;
  for (int t = tid; t < CRAFT_MAX_RECIPES * 3; t += NT) s_rc[t] = v.rcw[t];
  if (v.wsr)
    for (int t = tid; t < CRAFT_MAX_KINDS * 4; t += NT) s_wsr[t] = v.wsr[t];
  for (int t = tid; t < CRAFT_MAX_TASKS * 4 + ((v.hint_bytes + 3) >> 2); t += NT)
    reinterpret_cast<uint32_t*>(smem + lay.hint)[t] = v.hint[t];
  {
    uint4* z = reinterpret_cast<uint4*>(s_obs);
    for (int i = tid; i < (2 * obs_buf >> 4); i += NT) z[i] = make_uint4(0, 0, 0, 0);
  }
  if (tid < 8) s_ctrl[tid] = 0u;
  for (int i = tid; i < kRtRows * RW; i += NT) s_rows[i] = 0u;
  if (tid < kRtLag) s_tpend[tid] = ~0u;
  __syncthreads();                                                    // (not counted: nb starts at 0)

  // Barriers.  Every wave adds one arrival per barrier before s_barrier; the teacher wave first
  // runs its queued BFS steps until every other wave has arrived; wave 2 stores label rows until
  // the teacher has (s_ctrl[3]).  (A plain s_barrier behind the wave's own LDS accesses: nothing else is handed over.)
  uint32_t nb = 0;                                                    // barriers passed
  auto arrive = [&]() __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add(&s_ctrl[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  };
  auto arrivals = [&]() __attribute__((always_inline)) -> uint32_t {
    return __builtin_amdgcn_readfirstlane(
        __hip_atomic_load(&s_ctrl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
  };
  auto hw_barrier = [&]() __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint64_t tb = RT_CLK();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    RT_ACC(0, tb);
    ++nb;
  };

  uint32_t n_succ = 0, n_end = 0, n_step = 0;                        // wave 0's episode sums

  if (wave == 0) {
    // =============================== C: the transitions ========================================
    Agent s{};
    uint64_t st = 0;
    uint32_t init_word = 0, task_word = 0, conn = 0;
    uint32_t clr = 0, clr_prev = 0, chg = 0;
    uint32_t clk = 0, clk_prev = 0;   // the kinds of clr's (up to 3) cells before they were cleared
    constexpr uint32_t kRestart = 0x80000000u;
    int sync = 0, lab0 = 0;
    // (label actions) the label of the state the last tick made, looked up by this wave itself:
    // a label byte, kCNib | the nibble's position in c_word (the nibble table's dword, loaded at
    // the end of the last tick), or kCRow: the teacher's row (the walk fallback, BFS answers, errors)
    constexpr uint32_t kCRow = 0x80000000u, kCNib = 0x40000000u;
    uint32_t c_tag = kCRow, c_word = 0;
    uint3 c_hd = make_uint3(0u, 0u, 0u);                               // the task's hint descriptor
    uint2 c_cw = make_uint2(~0u, ~0u);                                 // the row's listed clearable cells
    int ncl = 0;                                                       // cells cleared this episode
    // the inventory row after the last tick, read at its end (its latency behind the barrier, or
    // shared with the label lookup) and written into the next tick's buffer, instead of a read of
    // the other buffer at the tick's start
    uint32_t ivn[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // the kinds of the agent's four neighbour cells after the last tick (transition NB, byte d:
    // one step in direction d), read with ivn: the tick's facing cell / move target and the label
    // lookup's facing cell without a grid read on the tick's path
    uint32_t nbw = 0;
    bool live = false, lsrc = false;
    int64_t slot = 0;
    const uint32_t* pw = reinterpret_cast<const uint32_t*>(s_pristine + lane * GS);
    const uint8_t* pr = s_pristine + lane * GS;
    auto grid_of = [&](int p) __attribute__((always_inline)) { return s_grid + (p & 1) * TILE * GS + lane * GS; };
    auto read_nb = [&](const uint8_t* g) __attribute__((always_inline)) {
      const int p = s.x * H + s.y;                                    // DOWN, UP, LEFT, RIGHT (craft.py:77-91)
      nbw = (uint32_t)g[p - 1] | ((uint32_t)g[p + 1] << 8) | ((uint32_t)g[p - H] << 16) | ((uint32_t)g[p + H] << 24);
    };
    auto inv_of = [&](int p) __attribute__((always_inline)) { return s_inv + (p & 1) * TILE * kInvStride + lane * kInvStride; };
    auto restore = [&](uint8_t* g, uint32_t cl, uint32_t ck) __attribute__((always_inline)) {
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
            g[c] = (uint8_t)(ck >> (8 * i));                         // (no read of the pristine row)
          }
      }
    };
    // ---- A: take over tile t into buffer 0 ----
    auto load_tile = [&](int t) __attribute__((always_inline)) {
      const int64_t env0 = (int64_t)t * TILE;
      const int nE = (int)min((int64_t)TILE, n - env0);
      slot = env0 + lane;
      live = lane < nE;
      lsrc = false;
      uint32_t m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      uint32_t ivr[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if (live) {
        st = v.state[slot];
        init_word = v.init[slot];
        const uint4 i0 = v.inv[2 * slot], i1 = v.inv[2 * slot + 1];
        const uint4 m0 = v.mask[2 * slot], m1 = v.mask[2 * slot + 1];
        uint32_t bcw = 0;
        if (a.bc) bcw = a.bc[slot];
        if (lsync) lab0 = a.label_in[slot];
        ivr[0] = i0.x; ivr[1] = i0.y; ivr[2] = i0.z; ivr[3] = i0.w;
        ivr[4] = i1.x; ivr[5] = i1.y; ivr[6] = i1.z; ivr[7] = i1.w;
        m[0] = m0.x; m[1] = m0.y; m[2] = m0.z; m[3] = m0.w;
        m[4] = m1.x; m[5] = m1.y; m[6] = m1.z; m[7] = m1.w;
        lsrc = a.label_actions || (bcw & 0xffu);
        s = unpack_state(st);
        if (s.x < 1 || s.x > v.W - 2 || s.y < 1 || s.y > v.H - 2 || s.scen >= v.pool_count) {
          latch_error(v.err, CRAFT_EINVAL, slot);
          live = false;
        }
      }
      chg = 0;
      clr = 0;
      clr_prev = 0;
      clk = 0;
      clk_prev = 0;
      sync = 0;
      if (live) {
        task_word = s_task[s.task];
        conn = v.pool_conn[s.scen];
        if (v.ttab) {                                                  // the row's clearable cells the table lists
          c_cw = make_uint2(v.tt_cells[2 * (size_t)s.scen], v.tt_cells[2 * (size_t)s.scen + 1]);
          s_tcell[2 * lane] = c_cw.x;
          s_tcell[2 * lane + 1] = c_cw.y;
        }
        if (lsync) {
          const uint4 hd = s_hdesc[s.task];
          c_hd = make_uint3(hd.x, hd.y, hd.z);
        }
        ncl = 0;
#pragma unroll
        for (int w = 0; w < 8; ++w) ncl += __popc(m[w]);
        uint32_t* g0 = reinterpret_cast<uint32_t*>(grid_of(0));
        uint32_t* pwm = reinterpret_cast<uint32_t*>(s_pristine + lane * GS);
        const uint4* gsrc = reinterpret_cast<const uint4*>(v.pool + (size_t)s.scen * v.CS);
        const int nchunk = v.CS >> 4;
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
        uint32_t* iv0 = reinterpret_cast<uint32_t*>(inv_of(0));
#pragma unroll
        for (int i = 0; i < 8; ++i) iv0[i] = ivn[i] = ivr[i];
        uint8_t* b0 = grid_of(0);
#pragma unroll
        for (int w = 0; w < 8; ++w) {                                  // cells cleared this episode
          uint32_t mm = m[w];
          while (mm) {
            const int cc = w * 32 + __ffs(mm) - 1;
            b0[cc] = 0;
            const uint32_t nc = (clr >> 24) & 3;
            if (!(clr >> 31) && nc < 3) clk |= (uint32_t)pr[cc] << (8 * nc);
            clr = (clr >> 31) ? clr
                : nc < 3 ? ((clr & 0x00ffffffu) | ((uint32_t)cc << (8 * nc)) | ((nc + 1) << 24)) : (1u << 31);
            mm &= mm - 1;
          }
        }
        read_nb(b0);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    // ---- (label actions) the teacher's decision for this lane's new state, as the teacher wave's
    // walk makes it (D_WALK below: hint table leaf, then the nibble table's entry), or kCRow ----
    const bool c_tab = v.ttab4 != nullptr && v.ttab != nullptr && a.use_table;
    auto c_label = [&](const uint8_t* gr, const uint32_t (&ivw)[8]) __attribute__((always_inline)) -> uint32_t {
      if (s.frozen) return 0xffu;                                      // -1: the label of a done env
      const int facing = (int)((nbw >> (8 * s.dir)) & 0xffu);
      const uint4 hd = make_uint4(c_hd.x, c_hd.y, c_hd.z, 0u);
      uint32_t have = 0;
#pragma unroll
      for (int w = 0; w < 8; ++w) have |= byte_tops(nonzero_bytes(ivw[w])) << (4 * w);
      // the listed cells cleared: from the episode's cleared-cell list (clr), or the grid past 3
      uint32_t cleared = 0;
      if (!(clr >> 31)) {
        const uint32_t nc = (clr >> 24) & 3;
        const uint32_t k0 = nc > 0 ? (clr & 0xffu) : 0x100u, k1 = nc > 1 ? ((clr >> 8) & 0xffu) : 0x100u,
                       k2 = nc > 2 ? ((clr >> 16) & 0xffu) : 0x100u;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t c = ((j < 4 ? c_cw.x : c_cw.y) >> (8 * (j & 3))) & 0xffu;
          cleared |= (uint32_t)(c != 0xffu && (c == k0 || c == k1 || c == k2)) << j;
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t c = ((j < 4 ? c_cw.x : c_cw.y) >> (8 * (j & 3))) & 0xffu;
          cleared |= (uint32_t)(c != 0xffu && gr[c != 0xffu ? c : 0u] == 0) << j;
        }
      }
      if (hd.z & craft_host::kHintWalk) {                              // (the host picks mode 1 for these)
        if (lmode == 2) latch_error(v.err, CRAFT_EINVARIANT, slot);
        return kCRow;
      }
      uint32_t bits = 0;
#pragma unroll
      for (int j = 0; j < craft_host::kHintPreds; ++j) {
        const uint32_t b = ((j < 4 ? hd.x : hd.y) >> (8 * (j & 3))) & 0xffu;
        const uint32_t kd = b & 0x3fu;
        const uint32_t t = (b & 0x40u) ? (uint32_t)(facing == (int)kd) : (have >> (kd & 31u)) & 1u;
        bits |= ((b >> 7) & t) << j;
      }
      const uint32_t lf = s_hleaf[hd.z + bits];
      if (lf == craft_host::kHintErr) {                                // the reference raises (as the teacher latches)
        latch_error(v.err, CRAFT_ETEACHER, slot);
        return 0xfeu;                                                  // -2
      }
      if (lf == craft_host::kHintStop) return (uint32_t)CRAFT_STOP;
      if (lf == craft_host::kHintUse) return (uint32_t)CRAFT_USE;
      const int trow = c_tab && ncl == __popc(cleared) ? (int)s.scen * v.tt_nsub + (int)cleared : -1;
      const int sl = trow >= 0 ? tt_slot_of(v, (int)lf) : -1;
      if (sl < 0) return kCRow;
      const uint32_t idx = (uint32_t)(s.dir * C + s.x * H + s.y);
      const uint32_t req = ((uint32_t)trow * (uint32_t)v.tt_slots + (uint32_t)sl) * (uint32_t)(v.tt_blk >> 2) + (idx >> 3);
      c_word = reinterpret_cast<const uint32_t*>(v.ttab4)[req];       // decoded next tick
      return kCNib | (idx & 7u);
    };
    // ---- C: tick k (item g) into buffer k & 1 (trainers/imitation.py:43-73) ----
    auto tick_c = [&](int k, uint32_t g) __attribute__((always_inline)) {
      const int64_t tick = a.tick0 + k;
      int d = 0, succ = -1, counted = 0, act = 0;
      uint8_t* gr = grid_of(k);
      uint8_t* iv = inv_of(k);
      // the label of this env's current state: label_in (the unit's first tick), this wave's own
      // lookup, or the teacher's row of item g - 1 once complete (the teacher finishes each item
      // inside its interval)
      int clab = 0;
      bool use_row = false, unknown = false;
      // (LA: every lane's label is looked up and published, the cloning lanes' and the others')
      if (k > 0 && live && (lsrc || LA)) {
        if (c_tag & kCNib) {
          const uint32_t code = (c_word >> (4 * (c_tag & 7u))) & 0xfu;
          clab = code < 4 ? (int)code : code == 4 ? CRAFT_STOP : -2;
          if (code > 4)                                                // raises / no entry (as the teacher's decode)
            latch_error(v.err, code == 5 ? CRAFT_ETEACHER : CRAFT_EINVARIANT, slot);
        } else if (c_tag & kCRow) {
          use_row = lsrc;                                              // (a lane on the policy needs no wait)
          unknown = true;
        } else {
          clab = (int)(int8_t)(c_tag & 0xffu);
        }
      }
      // (LA) item g - 1's labels published for the teacher wave, which then needs no walk of its
      // own for them: before the wait below, which waits for the teacher
      if (LA && k > 0 && lmode == 2) {
        if (lane < TILE)
          s_clab[((g - 1) & 1) * TILE + lane] = (live && !unknown) ? 0x100u | ((uint32_t)clab & 0xffu) : 0u;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_store(&s_ctrl[4], g, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      // mode 1: the row complete; mode 2: the row's BFS answers in (after its walk: s_ctrl[2])
      if (k > 0 && __ballot(live && lsrc && use_row)) {
        const uint32_t* R = s_rows + ((g - 1) & (kRtRows - 1)) * RW;
        for (uint32_t spins = 0;;) {
          bool ready = __builtin_amdgcn_readfirstlane(
                           __hip_atomic_load(&s_ctrl[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) >= g;
          if (ready && lmode == 2) {
            const uint32_t rc = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(&R[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
            ready = !(rc & kRowFill) || ((rc >> 8) & 0xffu) == 0;       // (0 / storing: complete)
          }
          if (ready) break;
          __builtin_amdgcn_s_sleep(1);
          if (++spins > kRtSpinCap) { latch_error(v.err, CRAFT_EINVARIANT, rt_where(1, g, 0)); break; }   // never hang
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      }
      s = unpack_state(st);
      const uint64_t tc0 = RT_CLK();
      if (live) {
        if (sync == 1) {                                               // bring the buffer up to date
          const uint32_t* src = reinterpret_cast<const uint32_t*>(grid_of(k + 1));
          uint32_t* gw = reinterpret_cast<uint32_t*>(gr);
          for (int q0 = 0; q0 < (v.CS >> 2); q0 += 12) {
            uint32_t w[12];
#pragma unroll
            for (int j = 0; j < 12; ++j) w[j] = q0 + j < (v.CS >> 2) ? src[q0 + j] : 0u;
#pragma unroll
            for (int j = 0; j < 12; ++j)
              if (q0 + j < (v.CS >> 2)) gw[q0 + j] = w[j];
          }
        } else if (sync == 2) {
          if (chg == kRestart) restore(gr, clr_prev, clk_prev);
          else if (chg) gr[chg - 1] = 0;
        }
        if (sync) {
#pragma unroll
          for (int i = 0; i < 8; ++i) reinterpret_cast<uint32_t*>(iv)[i] = ivn[i];
        }
        sync = sync ? 2 : 1;
        chg = 0;
        RT_ACC(4, tc0);
        const uint64_t tc1 = RT_CLK();
        if (a.actions) {
          act = a.actions[(int64_t)k * n + slot];
        } else {
          const uint64_t gid = (uint64_t)(v.env_base + slot);
          act = (int)((uint32_t)(splitmix64(a.seed ^ (gid << 20) ^ (uint64_t)tick) >> 32) % 6u);
        }
        if (lsrc) act = k == 0 ? lab0 : use_row ? (int)s_rows[((g - 1) & (kRtRows - 1)) * RW + 4 + lane] : clab;
        bool restart = false;
        if (s.frozen) {
          d = 1;
        } else {
          counted = 1;
          s.timer -= 1;
          d = (act == CRAFT_STOP) || s.timer <= 0;
          restart = d && (a.flags & CRAFT_STEP_AUTORESET);
        }
        if (d) {                                                       // satisfies() of the pre-step state
          const int goal = task_word & 0xf, arg = (task_word >> 4) & 0xff;
          const int fc = (s.x + dir_dx(s.dir)) * H + (s.y + dir_dy(s.dir));
          if (goal == CRAFT_GOAL_GET || goal == CRAFT_GOAL_MAKE) succ = rbyte(ivn, arg) > 0;
          else if (goal == CRAFT_GOAL_GO) succ = (int)gr[fc] == arg;
          else succ = -1;
        }
        if (restart) {                                                 // CraftScenario.init, craft.py:268-273
          s.x = init_word & 0xff; s.y = (init_word >> 8) & 0xff; s.dir = (init_word >> 16) & 3;
          s.timer = v.maxT;
#pragma unroll
          for (int w = 0; w < 8; ++w) reinterpret_cast<uint32_t*>(iv)[w] = 0u;
          restore(gr, clr, clk);
          clr_prev = clr;
          clk_prev = clk;
          clr = 0;
          clk = 0;
          chg = kRestart;
          ncl = 0;
        } else if (d && !s.frozen) {
          s.frozen = 1;
          s.timer = max(s.timer, 0);
        }
        RT_ACC(5, tc1);
        const uint64_t tc2 = RT_CLK();
        if (!d) {
          bool inv_changed = false, mask_changed = false;
          const int fc = (s.x + dir_dx(s.dir)) * H + (s.y + dir_dy(s.dir));   // what USE clears
          uint32_t m_unused[8] = {0, 0, 0, 0, 0, 0, 0, 0};
          if (act < 0 || act >= CRAFT_N_ACTIONS) latch_error(v.err, CRAFT_EBADACTION, slot);
          else if (v.wsr) transition<true, true, true>(v, s_rc, gr, iv, s, m_unused, act, inv_changed, mask_changed, rcv, slot, s_wsr, nbw);
          else transition<true, false, true>(v, s_rc, gr, iv, s, m_unused, act, inv_changed, mask_changed, rcv, slot, nullptr, nbw);
          if (mask_changed) {
            ++ncl;
            chg = 1u + (uint32_t)fc;
            const uint32_t nc = (clr >> 24) & 3;
            if (!(clr >> 31) && nc < 3) clk |= ((nbw >> (8 * s.dir)) & 0xffu) << (8 * nc);   // USE cleared the facing cell
            clr = (clr >> 31) ? clr
                : nc < 3 ? ((clr & 0x00ffffffu) | ((uint32_t)fc << (8 * nc)) | ((nc + 1) << 24)) : (1u << 31);
          }
        }
        st = pack_state(s);
        RT_ACC(3, tc2);
        const uint64_t tc3 = RT_CLK();
#pragma unroll
        for (int i = 0; i < 8; ++i) ivn[i] = reinterpret_cast<const uint32_t*>(iv)[i];
        read_nb(gr);
        if (lsync && (lsrc || LA) && k + 1 < a.n_ticks) c_tag = c_label(gr, ivn);
        // done, success, reward and the recorded action (action_seqs, imitation.py:59-61) leave
        // from the streaming waves, one array each
        s_cout[(k & 1) * TILE + lane] = make_uint2((uint32_t)d | ((uint32_t)(succ + 1) << 1) | ((uint32_t)counted << 3) |
                                                       (1u << 4),                          // (stored)
                                                   (uint32_t)(counted ? act : -1));
        RT_ACC(1, tc3);
      }
      const uint64_t bs = __ballot(live && counted && d && succ == 1);
      const uint64_t be = __ballot(live && counted && d);
      const uint64_t bt = __ballot(live && counted);
      n_succ += (uint32_t)__popcll(bs);
      n_end += (uint32_t)__popcll(be);
      n_step += (uint32_t)__popcll(bt);
      if (lane < TILE) {
        if (!live) s_cout[(k & 1) * TILE + lane] = make_uint2(0u, 0u);
        s_agent[(k & 1) * TILE + lane] =
            live ? ((uint32_t)s.x | ((uint32_t)s.y << 8) | ((uint32_t)s.dir << 16) | (1u << 24) |
                    ((uint32_t)s.frozen << 25) | ((uint32_t)min(ncl, 63) << 26))
                 : 0u;
        s_tinfo[(k & 1) * TILE + lane] = (uint32_t)s.task | (conn << 8) | ((uint32_t)s.scen << 10);
      }
    };
    // ---- the tile's state back to HBM from buffer p (the mask rebuilt from the rows) ----
    auto publish = [&](int p) __attribute__((always_inline)) {
      const uint32_t* ivw = reinterpret_cast<const uint32_t*>(inv_of(p));
      const uint32_t* gw = reinterpret_cast<const uint32_t*>(grid_of(p));
      uint32_t m[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) m[i] = 0u;
#pragma unroll
      for (int q = 0; q < CRAFT_MAX_CELLS / 4; ++q)
        if (q < (C + 3) >> 2) m[q >> 3] |= byte_tops(nonzero_bytes(pw[q]) & zero_bytes(gw[q])) << (4 * (q & 7));
      v.state[slot] = st;
      v.inv[2 * slot] = make_uint4(ivw[0], ivw[1], ivw[2], ivw[3]);
      v.inv[2 * slot + 1] = make_uint4(ivw[4], ivw[5], ivw[6], ivw[7]);
      v.mask[2 * slot] = make_uint4(m[0], m[1], m[2], m[3]);
      v.mask[2 * slot + 1] = make_uint4(m[4], m[5], m[6], m[7]);
    };
    bool first = (uint32_t)blockIdx.x < n_units;
    uint32_t gbase = 0;
    for (;;) {
      if (lane == 0)
        s_ctrl[0] = first ? (uint32_t)blockIdx.x
                          : (uint32_t)(gridDim.x + (atomicAdd(a.queue + 1, 1ull) - a.qbase1));
      first = false;
      arrive();
      hw_barrier();                                                   // claim
      const uint32_t u = s_ctrl[0];
      if (u >= n_units) break;
      const int nq = a.n_ticks;
      if (lane < TILE) {
        load_tile((int)u);
        tick_c(0, gbase);
      }
      arrive();
      hw_barrier();                                                   // C(0) done
      for (int i = 0; i <= nq; ++i) {
        const uint64_t tc = RT_CLK();
        if (lane < TILE && i + 1 < nq) tick_c(i + 1, gbase + i + 1);
        RT_ACC(2, tc);
        arrive();
        hw_barrier();
      }
      if (lane < TILE && live) publish(nq - 1);
      arrive();
      hw_barrier();                                                   // unit end
      gbase += nq;
    }
  } else if (wave == 1) {
    // =============================== D: the scatter ============================================
    for (;;) {
      arrive();
      hw_barrier();
      const uint32_t u = s_ctrl[0];
      if (u >= n_units) break;
      const int nq = a.n_ticks;
      const int64_t env0 = (int64_t)u * TILE;
      const int nE = (int)min((int64_t)TILE, n - env0);
      arrive();
      hw_barrier();
#pragma unroll 1
      for (int i = 0; i <= nq; ++i) {
        const uint64_t td = RT_CLK();
        if (i < nq && want_obs) {
          const int e = lane % TILE;
          const uint32_t ag = s_agent[(i & 1) * TILE + e];
          if (e < nE && ((ag >> 24) & 1u))
            scatter_env_part<WIN, P, false>(v, s_grid + (i & 1) * TILE * GS + e * GS,
                                     s_inv + (i & 1) * TILE * kInvStride + e * kInvStride, ag,
                                     s_obs + (i & 1) * obs_buf + e * F, lane / TILE);
        }
        RT_ACC(2, td);
        arrive();
        hw_barrier();
      }
      arrive();
      hw_barrier();
    }
  } else if (wave < TW) {
    // =============================== E: the stores =============================================
    const int et = tid - 128;
    uint32_t h = 0;                                                    // wave 2: the next item to store
    // wave 2: store the label rows that are complete, in item order (at most `reps` now)
    auto store_rows = [&](int reps) __attribute__((always_inline)) {
      for (int rep = 0; rep < reps; ++rep) {
        uint32_t* R = s_rows + (h & (kRtRows - 1)) * RW;
        const uint32_t c = __builtin_amdgcn_readfirstlane(
            __hip_atomic_load(&R[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        const uint32_t tag = __builtin_amdgcn_readfirstlane(R[1]);
        if (tag == h + 1 && c == kRowFill) {
          uint32_t won = 0;
          if (lane == 0) {
            uint32_t exp = kRowFill;
            won = __hip_atomic_compare_exchange_strong(&R[0], &exp, kRowStoring, __ATOMIC_ACQUIRE,
                                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) ? 1u : 0u;
          }
          if (!__builtin_amdgcn_readfirstlane(won)) break;
          const int t = (int)R[2];
          const int64_t r = (int64_t)R[3];
          const int nE = (int)min((int64_t)TILE, n - (int64_t)t * TILE);
          const int lab = lane < TILE ? (int)R[4 + lane] : 0;
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          if (lane == 0) __hip_atomic_store(&R[0], 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (a.labels && lane < nE) a.labels[r * n + (int64_t)t * TILE + lane] = lab;
          ++h;
        } else if (tag > h + 1) {
          ++h;                                                         // (not expected: rows are stored here)
        } else {
          break;
        }
      }
    };
    auto e_barrier = [&]() __attribute__((always_inline)) {
      arrive();
      const uint64_t tw = RT_CLK();
      if (wave == 2) {
        // keep storing until the teacher has arrived too (it may wait for a free row)
        for (uint32_t spins = 0; __builtin_amdgcn_readfirstlane(__hip_atomic_load(
                                     &s_ctrl[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < nb + 1; ++spins) {
          store_rows(1);
          __builtin_amdgcn_s_sleep(1);
          if (spins > kRtSpinCap) {                                    // never hang
            latch_error(v.err, CRAFT_EINVARIANT, rt_where(2, h, s_rows[(h & (kRtRows - 1)) * RW]));
            break;
          }
        }
      }
      RT_ACC(1, tw);
      hw_barrier();
    };
    uint32_t gbase = 0;
    for (;;) {
      e_barrier();
      const uint32_t u = s_ctrl[0];
      if (u >= n_units) break;
      const int nq = a.n_ticks;
      gbase += nq;
      const int64_t env0 = (int64_t)u * TILE;
      const int nE = (int)min((int64_t)TILE, n - env0);
      e_barrier();
      for (int i = 0; i <= nq; ++i) {
        const uint64_t te = RT_CLK();
        if (i >= 1 && want_obs) {
          const int64_t r = (a.tick0 + i - 1) % a.ring;
          void* out = static_cast<uint8_t*>(a.obs) + r * n * (int64_t)F * (v.obs_fmt == CRAFT_OBS_F32 ? 4 : v.obs_fmt == CRAFT_OBS_BF16 ? 2 : 1);
          uint8_t* rows = s_obs + ((i - 1) & 1) * obs_buf;
          switch (v.obs_fmt) {
            case CRAFT_OBS_BF16: stream_obs<CRAFT_OBS_BF16, NE, true>(rows, out, env0, F, nE, v.obs_policy, et); break;
            case CRAFT_OBS_U8: stream_obs<CRAFT_OBS_U8, NE, true>(rows, out, env0, F, nE, v.obs_policy, et); break;
            default: stream_obs<CRAFT_OBS_F32, NE, true>(rows, out, env0, F, nE, v.obs_policy, et); break;
          }
        }
        if (wave == 2) store_rows(2);
        if (i < nq && wave >= 3 && lane < nE) {                       // tick i's outputs: one array per wave
          const uint2 c = s_cout[(i & 1) * TILE + lane];
          const int64_t o = ((a.tick0 + i) % a.ring) * n + env0 + lane;
          const int d = (int)(c.x & 1u), succ = (int)((c.x >> 1) & 3u) - 1, counted = (int)((c.x >> 3) & 1u);
          if (c.x & (1u << 4)) {
            if (wave == 3 && a.done) a.done[o] = (uint8_t)d;
            if (wave == 4 && a.sat) a.sat[o] = (int8_t)succ;
            if (wave == 5 && a.reward) a.reward[o] = (counted && d && succ == 1) ? 1.0f : 0.0f;
            if (wave == 6 && a.rec) a.rec[o] = (int32_t)c.y;
          }
        }
        RT_ACC(2, te);
        e_barrier();
      }
      e_barrier();
    }
    // after the last barrier the teacher finishes the BFS jobs left; every label row is stored
    // here, in item order (the teacher stores nothing)
    if (wave == 2)
      for (uint32_t spins = 0; h < gbase; ++spins) {
        store_rows(kRtRows);
        __builtin_amdgcn_s_sleep(1);
        if (spins > kRtSpinCap) {                                      // never hang
          latch_error(v.err, CRAFT_EINVARIANT, rt_where(3, h, s_rows[(h & (kRtRows - 1)) * RW]));
          break;
        }
      }
  } else {
    // =============================== T: the teacher ============================================
    const int ql = lane & 3;
    const Bits<NW> valid = brange<NW>(0, C - 2 * H);                  // the band of columns 1 .. W-2
    QuadBfs<NW> q;
    uint32_t jhead = 0, jtail = 0;                                     // the job queue (wave-uniform)
    // ---- one BFS level for every quad (a new job for an idle quad first) ----
    auto finish = [&](int label, int err) __attribute__((always_inline)) {
      // lane 0 of the quad: the label into its row, one pending label fewer
      if (ql == 0) {
        const int row = (q.meta >> 11) & (kRtRows - 1), env = (q.meta >> 15) & 63;
        uint32_t* R = s_rows + row * RW;
        R[4 + env] = (uint32_t)label;
        if (err) latch_error(v.err, err, (int64_t)R[2] * TILE + env);
        __hip_atomic_fetch_add(&R[0], 0u - 0x101u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);   // (and a BFS one)
      }
      q.ph = kQIdle;
    };
    auto done_go = [&](bool ok, int fa, int len) __attribute__((always_inline)) {
      int err = 0;
      const int label = go_leaf_action(ok, fa, len, err);
      finish(label, err);
    };
    const int dla = ql == 0 ? -1 : ql == 1 ? 1 : ql == 2 ? -H : H;    // this lane's action: cell shift
    auto qp0 = [&]() __attribute__((always_inline)) -> int { return (int)(q.meta & 0xffu); };
    auto qd0 = [&]() __attribute__((always_inline)) -> int { return (int)((q.meta >> 8) & 3u); };
    auto blocked = [&]() __attribute__((always_inline)) -> Bits<NW> {   // blk[p] = occ[p + dla]
      Bits<NW> b = bshift_var(bandn(valid, q.fr), -dla);
      if (ql == 2) b = bor(b, band_edge_lo<NW>(valid, H));           // the border columns left out
      if (ql == 3) b = bor(b, band_edge_hi<NW>(valid, H));           // of the band
      return b;
    };
    auto raises = [&]() __attribute__((always_inline)) -> bool {   // base.py:31: unreachable after reachable
      const Bits<NW> unreached = bandn(q.tgt, q.claimed);
      return bany(unreached) && blowest(q.claimed) < bhighest(unreached);
    };
    auto bwd_final = [&]() __attribute__((always_inline)) {
      const int p0 = qp0();
      const int q0 = p0 + dla;
      const int qq = btest(q.fr, q0) ? q0 : p0;
      const bool ok = !(qq == p0 && ql == qd0()) && btest(q.V, qq);
      const uint32_t quad = (uint32_t)(__ballot(ok) >> (lane & ~3)) & 0xfu;
      done_go(true, quad ? __ffs(quad) - 1 : -1, q.L);
    };
    auto bwd_init = [&]() __attribute__((always_inline)) {
      if (q.L == 0) { done_go(true, -1, 0); return; }
      const int qc = q.chosen - dla;
      q.U = (qc >= 0) ? band(bbit<NW>(qc), q.fr) : bzero<NW>();
      q.V = q.U;
      q.k = 1;
      if (q.k < q.L) q.ph = kQBwd;
      else bwd_final();
    };
    auto after_fwd = [&]() __attribute__((always_inline)) {
      if (q.L < 0) { done_go(true, -1, -1); return; }                 // no target reachable: None
      if (bany(bandn(q.tgt, q.claimed))) {
        if (((q.meta >> 10) & 1u) && btest(q.fr, qp0())) {
          // connected free cells: a target is reachable iff it has a free neighbour
          q.claimed = bor(q.claimed, band(quad_or(bshift_var(q.fr, dla)), q.tgt));
          if (raises()) { done_go(false, -1, -1); return; }
          bwd_init();
        } else {
          q.U = bor(quad_or(q.V), bbit<NW>(qp0()));                    // flood from the visited cells
          q.ph = kQReach;
        }
      } else {
        bwd_init();
      }
    };
    auto take_jobs = [&]() __attribute__((always_inline)) {
      const uint32_t avail = jtail - jhead;
      if (avail == 0) return;
      const uint64_t idle = __ballot(q.ph == kQIdle && ql == 0);
      if (!idle) return;
      // idle quads below this lane's quad (LA: v_mbcnt at the quad's first lane, broadcast to the
      // quad: no per-lane 64-bit mask, which hipcc keeps live for the whole kernel and spilled there)
      uint32_t rank;
      if constexpr (LA) rank = (uint32_t)__builtin_amdgcn_mov_dpp((int)lane_rank(idle), 0x00, 0xf, 0xf, false);
      else rank = (uint32_t)__popcll(idle & ((1ull << (lane & ~3)) - 1ull));
      const uint32_t taken = min(avail, (uint32_t)__popcll(idle));
      if (q.ph == kQIdle && rank < avail) {
        const uint32_t* J = s_jobs + ((jhead + rank) % kRtQueue) * JW;
        Bits<NW> occ;
#pragma unroll
        for (int i = 0; i < NW; ++i) { occ.w[i] = J[i]; q.tgt.w[i] = J[NW + i]; }
        q.meta = J[2 * NW];
        q.fr = bandn(valid, occ);
        const int d0 = qd0(), p0 = qp0();
        const int dl0 = d0 == 0 ? -1 : d0 == 1 ? 1 : d0 == 2 ? -H : H;
        q.claimed = bzero<NW>();
        q.L = -1;
        q.chosen = -1;
        const int f0 = p0 + dl0;                                       // the start already faces a target
        if (f0 >= 0 && btest(q.tgt, f0)) {
          q.L = 0;
          q.chosen = f0;
          q.claimed = bbit<NW>(f0);
        }
        q.V = (ql == d0) ? bbit<NW>(p0) : bzero<NW>();
        q.U = bbit<NW>(p0);
        q.k = 1;
        if (bany(bandn(q.tgt, q.claimed)) && q.L < 0) q.ph = kQFwd;
        else after_fwd();
      }
      jhead += taken;
    };
    auto step = [&]() __attribute__((always_inline)) {
      take_jobs();
      if (q.ph == kQFwd) {
        const Bits<NW> nxt = bandn(bor(band(bshift_var(q.U, dla), q.fr), band(q.U, blocked())), q.V);
        q.V = bor(q.V, nxt);
        const Bits<NW> nU = quad_or(nxt);
        if (!bany(nU)) {
          after_fwd();                                                 // every reachable state visited
        } else {
          uint32_t face = 0;
          const Bits<NW> fa = bshift_var(q.tgt, -dla);                 // fa[p] = tgt[p + dla]
#pragma unroll
          for (int i = 0; i < NW; ++i) face |= nxt.w[i] & fa.w[i];
          bool hitany = false;
          if ((uint32_t)(__ballot(face != 0) >> (lane & ~3)) & 0xfu) {
            const Bits<NW> hit = bandn(quad_or(band(bshift_var(nxt, dla), q.tgt)), q.claimed);
            if (bany(hit)) {
              q.claimed = bor(q.claimed, hit);
              q.L = q.k;
              q.chosen = blowest(hit);
              hitany = true;
            }
          }
          if (hitany) {
            after_fwd();
          } else {
            q.U = nU;
            ++q.k;
          }
        }
      }
      if (q.ph == kQReach) {
        const Bits<NW> adj = quad_or(bshift_var(q.U, dla));          // cells next to the reached set
        q.claimed = bor(q.claimed, band(adj, q.tgt));
        if (!bany(bandn(q.tgt, q.claimed))) {
          bwd_init();
        } else {
          const Bits<NW> grow = bandn(band(adj, q.fr), q.U);
          if (!bany(grow)) {
            if (raises()) done_go(false, -1, -1);
            else bwd_init();
          } else {
            q.U = bor(q.U, grow);
          }
        }
      }
      if (q.ph == kQBwd) {
        // predecessors, any direction: moved here or turned in place (blocked)
        const Bits<NW> P2 = quad_or(bor(band(bshift_var(q.U, -dla), q.fr), band(q.U, blocked())));
        q.U = bandn(P2, q.V);
        q.V = bor(q.V, q.U);
        ++q.k;
        if (q.k >= q.L) bwd_final();
      }
    };
    auto busy = [&]() __attribute__((always_inline)) -> bool {
      return jtail != jhead || __ballot(q.ph != kQIdle) != 0;
    };
    // Policy actions: each walk fetches its items' table words with one LDS-DMA
    // (global_load_lds_dword), a dummy one when the item asks for none, so that the fetch of the
    // item kRtLag walks back is exactly the one vmcnt(kRtLag - 1) leaves waiting for (loads
    // complete in order; any other VMEM op of this wave, a latched error, only makes the wait
    // stricter).  One inline-asm statement that saves M0, points it at the slot, issues the DMA and
    // restores M0: M0 is compiler-reserved, so no compiler-held M0 value may be lost across it
    // (round 5's statement set M0 without restoring it).  Not __builtin_amdgcn_global_load_lds:
    // hipcc cannot tell the DMA's target from the rest of the dynamic LDS, so it waits vmcnt(0)
    // before the wave's next LDS access (28 more vmcnt(0) in rollout_teach_kernel<3, 32, 4>), which
    // undoes the lag: config 5 402.5-405.6 against 393.2-395.4 us per 20-tick launch on one box
    // (profiles/r06/ab_dma).  The "memory" clobber orders it against the slot's reads (decode_slot).
    // (the answers as 4-bit labels, SimView::ttab4: a quarter of the u16 table's footprint, so
    // more of the lines the gather touches are L2 hits; req is then the dword index)
    const bool nib = v.ttab4 != nullptr;
    const uint32_t* tbase = reinterpret_cast<const uint32_t*>(
        nib ? (const void*)v.ttab4 : v.ttab ? (const void*)v.ttab : (const void*)v.task_tab);
    auto fetch = [&](int q, uint32_t req) __attribute__((always_inline)) {
      const uint32_t* gp = tbase + (req == ~0u ? 0u : nib ? req : req >> 1);
      const uint32_t lds = __builtin_amdgcn_readfirstlane(
          (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)(s_tval + q * 64));
      uint32_t keep;
      // (lgkmcnt(0): the slot's last reads are done)
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
                   "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(gp), "s"(lds) : "memory");
    };
    // decode slot q's words (fetched kRtLag walks ago, or at the end: wait_all) into their label row
    auto decode_slot = [&](int q, bool wait_all) __attribute__((always_inline)) {
      const uint64_t tq = RT_CLK();
      const uint32_t prow = __builtin_amdgcn_readfirstlane(s_tpend[q]);
      if (prow == ~0u) { RT_ACC(3, tq); return; }
      if (wait_all) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kRtLag - 1) : "memory");
      uint32_t* R = s_rows + prow * RW;
      const uint32_t req = lane < TILE ? s_treq[q * TILE + lane] : ~0u;
      if (req != ~0u) {
        const uint32_t word = s_tval[q * 64 + lane];
        int err = 0, label = -2;
        if (nib) {
          const uint32_t code = (word >> (4 * (uint32_t)s_tnib[q * TILE + lane])) & 0xfu;
          if (code < 4) label = (int)code;
          else if (code == 4) label = CRAFT_STOP;
          else err = code == 5 ? CRAFT_ETEACHER : CRAFT_EINVARIANT;  // the reference raises; 15: no entry
        } else {
          const uint32_t val = (req & 1u) ? word >> 16 : word & 0xffffu;
          if (val & 0x8000u) label = go_leaf_action((val & 0x4000u) != 0, (int)((val >> 10) & 7u) - 1,
                                                    (int)(val & 0x3ffu) - 1, err);
          else err = CRAFT_EINVARIANT;                                 // (a reachable grid has its entry)
        }
        R[4 + lane] = (uint32_t)label;
        if (err) latch_error(v.err, err, (int64_t)R[2] * TILE + lane);
      }
      const uint32_t cnt = (uint32_t)__popcll(__ballot(req != ~0u));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lane == 0) {
        __hip_atomic_fetch_add(&R[0], 0u - cnt, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        s_tpend[q] = ~0u;
      }
      RT_ACC(3, tq);
    };
    auto row_ctrl = [&](int row) __attribute__((always_inline)) -> uint32_t {
      return __builtin_amdgcn_readfirstlane(
          __hip_atomic_load(&s_rows[row * RW], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
    };
    // queue n jobs: lanes with `mine` write theirs (band bitsets of `row32` for `kind`) in lane order
    auto push_jobs = [&](uint64_t mask, bool mine, const uint8_t* row8, int kind, int p0, int d0, int cn,
                         int row) __attribute__((always_inline)) {
      if (mine) {
        const uint32_t rank = LA ? lane_rank(mask) : (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
        uint32_t* J = s_jobs + ((jtail + rank) % kRtQueue) * JW;
        const uint32_t m0[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        Bits<NW> occ, tgt;
        band_bits<NW, 1>(reinterpret_cast<const uint32_t*>(row8), (C + 3) >> 2, C, H, m0, (uint32_t)kind, 0, occ, tgt);
#pragma unroll
        for (int i = 0; i < NW; ++i) { J[i] = occ.w[i]; J[NW + i] = tgt.w[i]; }
        J[2 * NW] = rt_job_meta(p0, d0, cn, row, lane);
      }
      jtail += (uint32_t)__popcll(mask);
    };

    // The teacher's schedule is a sequence of duties, each run once its condition holds; whenever
    // the next duty has to wait, the wave runs one BFS level (the single step() site: the BFS
    // state stays in registers instead of being spilled around several inlined copies).
    enum { D_BAR, D_WALK, D_WALK_JOBS, D_SYNC, D_DRAIN, D_EXIT };
    enum { B_CLAIM, B_C0, B_TICK, B_END };
    int duty = D_BAR, bkind = B_CLAIM;
    int i = 0, nq = 0, nE = 0;
    uint32_t u = 0, gbase = 0;
    // the walk's per-lane results between its two duties
    int w_label = 0, w_need = 0;
    uint32_t w_key = 0;                                                // p0 | dir<<8 | kind<<12 | conn<<20
    auto next_in_tick = [&]() __attribute__((always_inline)) -> int {   // after the barrier opening interval i
      return i < nq ? D_WALK : D_BAR;
    };
    uint32_t steps_run = 0;                                            // BFS levels in the current wait
    for (uint32_t idle_spins = 0;;) {
      bool wait = false;
      const uint64_t tt = RT_CLK();
      const int duty0 = duty;
      switch (duty) {
        case D_BAR: {
          // with BFS work queued, run it until every other wave has arrived; without, go straight
          // to the barrier
          if (busy() && arrivals() < (uint32_t)NWAVE * nb + (NWAVE - 1)) { wait = true; break; }
          if (lane == 0) __hip_atomic_store(&s_ctrl[3], nb + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          arrive();
          hw_barrier();
          if (bkind == B_CLAIM) {
            u = s_ctrl[0];
            if (u >= n_units) { duty = D_DRAIN; break; }
            nq = a.n_ticks;
            nE = (int)min((int64_t)TILE, n - (int64_t)u * TILE);
            bkind = B_C0;
          } else if (bkind == B_C0) {
            i = 0;
            bkind = B_TICK;
            duty = next_in_tick();
          } else if (bkind == B_TICK) {
            if (++i > nq) bkind = B_END;
            else duty = next_in_tick();
          } else {
            gbase += nq;
            bkind = B_CLAIM;
          }
          break;
        }
        case D_WALK: {                                                 // item g = gbase + i, buffer i & 1
          const uint32_t g = gbase + (uint32_t)i;
          const int row = (int)(g & (kRtRows - 1));
          if (row_ctrl(row) != 0u) { wait = true; break; }             // wave 2 frees it at the latest at the barrier
          uint32_t* R = s_rows + row * RW;
          const int p = i & 1;
          w_label = -2;
          w_need = 0;                                                  // 1: a table answer, 2: a BFS job
          uint32_t req = ~0u;                                          // (policy actions) the ttab index asked
          uint32_t w_nib = 0;                                          // (nibble table) the nibble in that word
          // (every env on its label) the transition wave decoded this item's labels at the start
          // of its next tick (all but BFS answers): taken as they are, no walk for those lanes
          uint32_t clw = 0;
          if (LA && lmode == 2 && i + 1 < nq) {
            if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&s_ctrl[4], __ATOMIC_ACQUIRE,
                                                                 __HIP_MEMORY_SCOPE_WORKGROUP)) < g + 1) {
              wait = true;
              break;
            }
            clw = lane < TILE ? s_clab[(g & 1) * TILE + lane] : 0u;
          }
          if (lane < nE && (clw & 0x100u)) {
            w_label = (int)(int8_t)(clw & 0xffu);
          } else if (lane < nE) {
            // the walk's loads in three rounds, each issued together: the agent and task words and
            // the row's listed clearable cells; the facing cell, the hint descriptor, the inventory
            // and the listed cells' kinds now; the hint leaf
            const uint32_t ag = s_agent[p * TILE + lane];
            const uint32_t ti = s_tinfo[p * TILE + lane];
            const uint32_t cw0 = s_tcell[2 * lane], cw1 = s_tcell[2 * lane + 1];
            const bool live_env = (ag >> 24) & 1u;
            const int x = ag & 0xff, y = (ag >> 8) & 0xff, dir = (ag >> 16) & 3;
            const uint8_t* gr = s_grid + p * TILE * GS + lane * GS;
            const int facing = gr[live_env ? (x + dir_dx(dir)) * H + (y + dir_dy(dir)) : 0];
            const uint8_t* ivb = s_inv + p * TILE * kInvStride + lane * kInvStride;
            const uint4 hd = s_hdesc[ti & 0xff];
            const uint32_t* ivw = reinterpret_cast<const uint32_t*>(ivb);
            uint32_t have = 0;                                         // bit k: inventory[k] > 0
#pragma unroll
            for (int w = 0; w < 8; ++w) have |= byte_tops(nonzero_bytes(ivw[w])) << (4 * w);
            uint32_t cleared = 0;                                      // bit j: listed cell j cleared
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const uint32_t c = ((j < 4 ? cw0 : cw1) >> (8 * (j & 3))) & 0xffu;
              cleared |= (uint32_t)(c != 0xffu && gr[c != 0xffu ? c : 0u] == 0) << j;
            }
            if (live_env && ((ag >> 25) & 1u)) {
              w_label = -1;                                            // frozen: the label of a done env
            } else if (live_env) {
              int err = 0, kind = 0;
              // the hint walk (find_incomplete_subtask): its table, the leaf for this task's
              // predicate values (craft_host.h hint_tables), or the walk itself
              if (hd.z & craft_host::kHintWalk) {
                w_label = hint_leaf(s_task, s_tsub, ivb, facing, (int)(ti & 0xff), err, kind);
              } else {
                uint32_t bits = 0;
#pragma unroll
                for (int j = 0; j < craft_host::kHintPreds; ++j) {
                  const uint32_t b = ((j < 4 ? hd.x : hd.y) >> (8 * (j & 3))) & 0xffu;
                  const uint32_t kd = b & 0x3fu;
                  const uint32_t t = (b & 0x40u) ? (uint32_t)(facing == (int)kd) : (have >> (kd & 31u)) & 1u;
                  bits |= ((b >> 7) & t) << j;
                }
                const uint32_t lf = s_hleaf[hd.z + bits];
                if (lf == craft_host::kHintErr) { w_label = -2; err = CRAFT_ETEACHER; }
                else if (lf == craft_host::kHintStop) w_label = CRAFT_STOP;
                else if (lf == craft_host::kHintUse) w_label = CRAFT_USE;
                else { w_label = kTeachGo; kind = (int)lf; }
              }
              if (err) latch_error(v.err, err, (int64_t)u * TILE + lane);
              w_key = (uint32_t)(x * H + y - H) | ((uint32_t)dir << 8) | ((uint32_t)(kind & 0xff) << 12) |
                      (((ti >> 8) & 1u) << 20);
              if (w_label == kTeachGo) {
                // the table's row for this grid: the pool row minus the listed cells it cleared
                // (tt_index), when those are all the cells it cleared
                const int ncl = (int)(ag >> 26);
                const int trow = v.ttab && a.use_table && ncl == __popc(cleared)
                                     ? (int)(ti >> 10) * v.tt_nsub + (int)cleared : -1;
                const int sl = trow >= 0 ? tt_slot_of(v, kind) : -1;
                w_need = sl >= 0 ? 1 : 2;
                if (w_need == 1) {
                  if (nib) {                                           // the dword holding the nibble
                    const uint32_t idx = (uint32_t)(dir * C + x * H + y);
                    req = ((uint32_t)trow * (uint32_t)v.tt_slots + (uint32_t)sl) * (uint32_t)(v.tt_blk >> 2) + (idx >> 3);
                    w_nib = idx & 7u;
                  } else {
                    req = (uint32_t)(((size_t)trow * v.tt_slots + sl) * 4 + dir) * C + x * H + y;
                  }
                }
              }
            }
          }
          if (lane < TILE) R[4 + lane] = w_need ? 0u : (uint32_t)w_label;
          if (lane == 0) {
            R[1] = g + 1;
            R[2] = u;
            R[3] = (uint32_t)((a.tick0 + i) % a.ring);
          }
          {
            // decode the item fetched kRtLag walks ago (its slot; with label actions every item is
            // decoded in its own interval), then fetch this one's
            const int q = (int)(g & (kRtLag - 1));
            if (lmode != 1) decode_slot(q, false);
            const bool any_req = __ballot(req != ~0u) != 0;          // (the whole wave votes)
            if (lane < TILE) {
              s_treq[q * TILE + lane] = req;
              s_tnib[q * TILE + lane] = (uint8_t)w_nib;
            }
            if (lane == 0) s_tpend[q] = any_req ? (uint32_t)row : ~0u;
            const uint64_t tf = RT_CLK();
            fetch(q, req);
            RT_ACC(1, tf);
          }
          duty = D_WALK_JOBS;
          break;
        }
        case D_WALK_JOBS: {
          const uint64_t bj = __ballot(w_need == 2);
          if (jtail - jhead + (uint32_t)__popcll(bj) > (uint32_t)kRtQueue) { wait = true; break; }
          const int row = (int)((gbase + (uint32_t)i) & (kRtRows - 1));
          push_jobs(bj, w_need == 2, s_grid + (i & 1) * TILE * GS + lane * GS, (w_key >> 12) & 0xff, w_key & 0xff,
                    (w_key >> 8) & 3, (w_key >> 20) & 1, row);
          // the row's control word last: the labels still pending (0 = complete), the BFS ones
          // among them in bits 8-15
          const uint32_t pending = (uint32_t)__popcll(__ballot(w_need != 0)) | ((uint32_t)__popcll(bj) << 8);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          if (lane == 0) {
            __hip_atomic_store(&s_rows[row * RW], kRowFill | pending, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (lmode == 2)                                            // item i walked: its BFS count is out
              __hip_atomic_store(&s_ctrl[2], gbase + (uint32_t)i + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
          duty = lmode == 1 ? D_SYNC : D_BAR;
          if (lmode == 1) decode_slot((int)((gbase + (uint32_t)i) & (kRtLag - 1)), true);   // (after the row's count)
          break;
        }
        case D_SYNC: {                                                 // label actions: item i complete
          const int row = (int)((gbase + (uint32_t)i) & (kRtRows - 1));
          if ((row_ctrl(row) & ~kRowFill) != 0u) { wait = true; break; }
          if (lane == 0)
            __hip_atomic_store(&s_ctrl[2], gbase + (uint32_t)i + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
          duty = D_BAR;
          break;
        }
        case D_DRAIN:                                                  // after the last barrier: the fetches
          if (lmode != 1)                                              // and the BFS jobs left
            for (int q = 0; q < kRtLag; ++q) decode_slot(q, true);
          if (busy()) wait = true;
          else duty = D_EXIT;
          break;
        default:
          break;
      }
      if (!wait) {                                                     // progress: the bounds below are per wait
        idle_spins = 0;
        steps_run = 0;
      }
      if (!wait && duty0 == D_WALK) RT_ACC(2, tt);
      if (!wait && duty0 == D_WALK_JOBS) RT_ACC(4, tt);
      if (duty == D_EXIT) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                // no LDS-DMA outlives the wave
        break;
      }
      if (wait) {
        const uint64_t ts = RT_CLK();
        const bool was_busy = busy();
        if (was_busy) {
          step();
          RT_ACC(5, ts);
#ifdef CRAFT_STAMPS
          if (lane == 0) __hip_atomic_fetch_add(&stt[7], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
          idle_spins = 0;
          if (++steps_run > kRtSpinCap) {                              // never hang the GPU (~2 s)
            latch_error(v.err, CRAFT_EINVARIANT, rt_where(5, gbase + (uint32_t)i, (uint32_t)duty));
            break;
          }
        } else {
          __builtin_amdgcn_s_sleep(1);
          RT_ACC(6, ts);
          if (++idle_spins > kRtSpinCap) {                             // never hang the GPU
            latch_error(v.err, CRAFT_EINVARIANT,
                        rt_where(4, gbase + (uint32_t)i, ((uint32_t)duty << 24) | s_rows[((gbase + i) & (kRtRows - 1)) * RW]));
            break;
          }
        }
      }
    }
  }

#ifdef CRAFT_STAMPS
  if (wave == 0 && lane == 0) {
    stt[6] = __builtin_amdgcn_s_memrealtime() - st_r0;
    stt[7] = __builtin_amdgcn_s_memtime() - st_c0;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  if (lane < 8 && v.stamps) v.stamps[(int64_t)blockIdx.x * 64 + wave * 8 + lane] = stt[lane];
#endif
#undef RT_CLK
#undef RT_ACC
  if (tid == 0) {
    unsigned long long* srow = reinterpret_cast<unsigned long long*>(v.stats_part + 4 * (int64_t)blockIdx.x);
    atomicAdd(srow + 0, (unsigned long long)n_succ);
    atomicAdd(srow + 1, (unsigned long long)n_end);
    atomicAdd(srow + 2, (unsigned long long)n_step);
  }
}

}  // namespace craft
