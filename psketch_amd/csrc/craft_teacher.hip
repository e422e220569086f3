// craft_teacher.hip — DemonstrationTeacher on the GPU over slot lists
// (craft_teacher): one lane or one quad of lanes per item, each env's grid
// rebuilt from its pool row and cleared-cell mask; the per-env body is
// teach_env (craft_teach.h).
#include <cstdlib>

#include "craft_teach.h"

namespace craft {

// Batches up to this many items run 4 lanes per item, larger ones 2 (profiles/r03/teacher_band,
// the band-layout BFS: 4096 items 11.4 / 14.6 / 23.0 us with 4 / 2 / 1 lanes, 16384 items
// 12.0 / 13.7 / 21.9, 65536 items 19.8 / 17.9 / 22.6; round 2, 32768 items: 16.2 / 15.0 / 22.9).
constexpr int64_t kTeacherQuadMaxItems = 16384;

struct TeachArgs {
  const int32_t* slots;
  const int32_t* tasks;
  int64_t n;
  int32_t* act_out;
  int32_t* len_out;
};

// DemonstrationTeacher.__call__ (teachers/demonstration.py:9-30) for item i, LANES lanes per
// item.  Writes the item's outputs and returns -1, or with DEFER (no path lengths asked) returns
// the target kind of a go[X] leaf the teacher table cannot answer, its BFS left to the
// workgroup's dense pass (teacher_kernel).
template <int NW, int LANES, bool DEFER>
__device__ __forceinline__ int teach_item(const SimView& v, const TeachArgs& a, int64_t i, int ql,
                                          const uint16_t* s_tab, const int32_t* s_sub) {
  const bool lead = ql == 0;             // the lane that writes the outputs and latches errors
  const int64_t slot = a.slots ? (int64_t)a.slots[i] : i;
  if (slot == -1) {                    // skipped item: the trainer's ref_action for a done env
    if (lead) {
      a.act_out[i] = -1;
      if (a.len_out) a.len_out[i] = -1;
    }
    return -1;
  }
  if (slot < 0 || slot >= v.n_envs) {
    if (lead) {
      latch_error(v.err, CRAFT_ERANGE, i);
      a.act_out[i] = -2;
      if (a.len_out) a.len_out[i] = -2;
    }
    return -1;
  }
  const Agent s = unpack_state(v.state[slot]);
  if (s.frozen) {                      // done env: its label is -1 (imitation.py:50-51)
    if (lead) {
      a.act_out[i] = -1;
      if (a.len_out) a.len_out[i] = -1;
    }
    return -1;
  }
  const int task = a.tasks ? a.tasks[i] : s.task;
  if (task < 0 || task >= v.n_tasks || s.x < 1 || s.x > v.W - 2 || s.y < 1 || s.y > v.H - 2 ||
      s.scen >= v.pool_count) {
    if (lead) {
      latch_error(v.err, task < 0 || task >= v.n_tasks ? CRAFT_ERANGE : CRAFT_EINVAL, i);
      a.act_out[i] = -2;
      if (a.len_out) a.len_out[i] = -2;
    }
    return -1;
  }
  uint32_t m[8];
  {
    const uint4 m0 = v.mask[2 * slot], m1 = v.mask[2 * slot + 1];
    m[0] = m0.x; m[1] = m0.y; m[2] = m0.z; m[3] = m0.w;
    m[4] = m1.x; m[5] = m1.y; m[6] = m1.z; m[7] = m1.w;
  }
  const uint8_t* iv = reinterpret_cast<const uint8_t*>(v.inv + 2 * slot);
  const uint32_t* row32 = reinterpret_cast<const uint32_t*>(v.pool + (size_t)s.scen * v.CS);
  // the teacher table's row for this grid (the pool row minus the cells it cleared), if it has one
  const int trow = v.ttab ? tt_index_mask(v, s.scen, v.tt_cells[2 * (size_t)s.scen], v.tt_cells[2 * (size_t)s.scen + 1], m)
                          : -1;
  int len = -1, err = 0, defer = -1;
  const int action = teach_env<NW, LANES, DEFER>(v, s_tab, s_sub, row32, m, iv, s, task, ql, a.len_out != nullptr,
                                                 len, err, v.pool_conn[s.scen] != 0,
                                                 trow >= 0 ? tt_row(v, trow) : nullptr, &defer,
                                                 DEFER && trow >= 0 ? tt_row4(v, trow) : nullptr);
  if (DEFER && action == kTeachDeferred) return defer;
  if (lead) {
    if (err) latch_error(v.err, err, slot);
    a.act_out[i] = action;
    if (a.len_out) {
      if (len == -2) latch_error(v.err, CRAFT_ETEACHER, slot);
      a.len_out[i] = len;
    }
  }
  return -1;
}

// One deferred item of the teacher kernel's dense pass (lane group g of L lanes takes list entry
// g): its go[X] BFS on the env's current grid, read from HBM as teach_item does.
template <int NW, int L>
__device__ __forceinline__ void dense_item(const SimView& v, const TeachArgs& a, const uint32_t* s_work, int n, int g,
                                           int ql, int ipb) {
  if (g >= n) return;
  const uint32_t wk = s_work[g];
  const int64_t ii = (int64_t)blockIdx.x * ipb + (wk & 0xffu);
  const int64_t slot = a.slots ? (int64_t)a.slots[ii] : ii;
  const Agent s = unpack_state(v.state[slot]);
  const uint4 m0 = v.mask[2 * slot], m1 = v.mask[2 * slot + 1];
  const uint32_t m[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
  const int C = v.C, H = v.H;
  const Bits<NW> valid = brange<NW>(0, C - 2 * H);
  Bits<NW> occ, tgt;
  band_bits<NW, L>(reinterpret_cast<const uint32_t*>(v.pool + (size_t)s.scen * v.CS), (C + 3) >> 2, C, H, m,
                   (wk >> 8) & 0xffu, ql, occ, tgt);
  int fa = -1, len = -1, err = 0;
  const bool ok = bfs_closest<NW, L>(occ, tgt, valid, H, s.x * H + s.y - H, s.dir, ql, fa, len, true,
                                     v.pool_conn[s.scen] != 0);
  const int action = go_leaf_action(ok, fa, len, err);
  if (ql == 0) {
    if (err) latch_error(v.err, err, slot);
    a.act_out[ii] = action;
  }
}

// The teacher over a slot list, LANES lanes per item: 4 (quad-parallel BFS) gives each query
// the shortest dependent chain, which is what bounds a small batch; 2 (a pair, one shift
// amount per lane) does about half the instructions per query at nearly the same chain
// length, which is what bounds a large one; 1 does the least work but the longest chain
// (launch_teacher picks by batch size).  DEFER (no path lengths asked): the items whose
// answer the teacher table holds finish in the walk; the rest are listed in LDS and searched
// by the workgroup's lane groups densely, one query each, so a wave's BFS instructions serve
// items that need them.
template <int NW, int LANES, bool DEFER>
__global__ __launch_bounds__(256) void teacher_kernel(SimView v, TeachArgs a) {
  // the task tables in LDS: the hint-tree walk reads them in a dependent chain
  __shared__ uint16_t s_tab[CRAFT_MAX_TASKS];
  __shared__ int32_t s_sub[CRAFT_MAX_TASKS * CRAFT_MAX_SUBTASKS];
  __shared__ uint32_t s_work[256 / LANES];
  __shared__ uint32_t s_nwork;
  for (int t = threadIdx.x; t < v.n_tasks * CRAFT_MAX_SUBTASKS; t += blockDim.x) {
    if (t < v.n_tasks) s_tab[t] = v.task_tab[t];
    s_sub[t] = v.task_sub[t];
  }
  if (DEFER && threadIdx.x == 0) s_nwork = 0u;
  __syncthreads();
  constexpr int IPB = 256 / LANES;       // items per workgroup
  const int g = (int)threadIdx.x / LANES, ql = (int)(threadIdx.x % LANES);
  const int64_t i = (int64_t)blockIdx.x * IPB + g;
  int kind = -1;
  if (i < a.n) kind = teach_item<NW, LANES, DEFER>(v, a, i, ql, s_tab, s_sub);   // group-uniform
  if constexpr (DEFER) {
    if (kind >= 0 && ql == 0)
      s_work[__hip_atomic_fetch_add(&s_nwork, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)] =
          (uint32_t)g | ((uint32_t)kind << 8);
    __syncthreads();
    const int nwk = (int)s_nwork;
    // quads (the shortest BFS chain) when every deferred item fits one per quad
    if (LANES < 4 && nwk <= 64) dense_item<NW, 4>(v, a, s_work, nwk, (int)threadIdx.x >> 2, (int)threadIdx.x & 3, IPB);
    else dense_item<NW, LANES>(v, a, s_work, nwk, g, ql, IPB);
  }
}

// ---- the rollout's per-env summary (craft_rollout_distances) ----------------------------------
struct DistArgs {
  const int32_t* tasks;
  const int8_t* success;
  const int32_t* seqs;       // [ticks][n] action record, -1 where the env did not act
  int32_t ticks;
  int64_t n;
  int32_t* dist_out;
  uint8_t* is_get_out;
  int32_t* n_actions_out;
  int32_t* flags;            // [2]: a None success, an unreachable target (plain stores of 1)
};

// trainers/imitation.py:79-91 for env i, LANES lanes per env: is_get = task i's goal is `get`;
// distances[i] = -1 for other goals, 0 for a success, else len(find_closest_resources(task.arg))
// on world.init_state(grid_i, pos, dir): the env's initial grid (its pool row: no cleared cells)
// at the final pose.  Only that BFS runs, as the reference calls only find_closest_resources.
// n_actions[i] counts the action record (len(action_seqs[i])).
template <int NW, int LANES>
__global__ __launch_bounds__(256) void distances_kernel(SimView v, DistArgs a) {
  __shared__ uint16_t s_tab[CRAFT_MAX_TASKS];
  for (int t = threadIdx.x; t < v.n_tasks; t += blockDim.x) s_tab[t] = v.task_tab[t];
  __syncthreads();
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / LANES;
  const int ql = (int)(threadIdx.x % LANES);
  if (i >= a.n) return;                  // lane-group-uniform
  const bool lead = ql == 0;
  const int task = a.tasks[i];
  const int succ = a.success[i];
  if (task < 0 || task >= v.n_tasks) {
    if (lead) {
      latch_error(v.err, CRAFT_ERANGE, i);
      a.dist_out[i] = -2;
      a.is_get_out[i] = 0;
      a.n_actions_out[i] = 0;
    }
    return;
  }
  const uint32_t tt = s_tab[task];
  const bool is_get = (tt & 0xf) == CRAFT_GOAL_GET;
  int d = is_get ? 0 : -1;
  if (is_get && succ == 0 && ((tt >> 4) & 0xffu) == 0) {
    d = -1;                              // kind 0 is never a target (as teach_env)
  } else if (is_get && succ == 0) {
    const Agent s = unpack_state(v.state[i]);
    if (s.x < 1 || s.x > v.W - 2 || s.y < 1 || s.y > v.H - 2 || s.scen >= v.pool_count) {
      if (lead) latch_error(v.err, CRAFT_EINVAL, i);
      d = -2;
    } else {
      const int C = v.C, nq = (C + 3) >> 2;
      const int kind = (tt >> 4) & 0xffu, slot = v.ttab ? tt_slot_of(v, kind) : -1;
      const uint32_t e = slot >= 0 ? tt_row(v, s.scen * v.tt_nsub)[(slot * 4 + s.dir) * C + s.x * v.H + s.y] : 0u;
      int fa = -1, len = -1;
      bool ok;
      if (e & 0x8000u) {                 // the initial grid is the pool row: the teacher table's
        len = (int)(e & 0x3ffu) - 1;     // answer (craft_teach.h)
        ok = (e & 0x4000u) != 0;
      } else {
        const Bits<NW> valid = brange<NW>(0, C - 2 * v.H);  // the band of columns 1 .. W-2
        const uint32_t m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const uint32_t* row32 = reinterpret_cast<const uint32_t*>(v.pool + (size_t)s.scen * v.CS);
        Bits<NW> occ, tgt;
        band_bits<NW, LANES>(row32, nq, C, v.H, m, kind, ql, occ, tgt);
        ok = bfs_closest<NW, LANES>(occ, tgt, valid, v.H, s.x * v.H + s.y - v.H, s.dir, ql, fa, len, false,
                                    v.pool_conn[s.scen] != 0);
      }
      // !ok: a target the BFS cannot reach.  The reference raises the same TypeError, len(None),
      // whether no target exists or none (or a later one, base.py:31) is reachable, so both
      // report through flags[1] below and nothing latches
      d = ok ? len : -2;
    }
  }
  if (lead) {
    int na = 0;                          // (8 loads in flight at a time, not one)
#pragma unroll 8
    for (int t = 0; t < a.ticks; ++t) na += a.seqs[(int64_t)t * a.n + i] >= 0;
    a.dist_out[i] = d;
    a.is_get_out[i] = is_get;
    a.n_actions_out[i] = na;
    if (succ < 0) a.flags[0] = 1;
    if ((d == -1 || d == -2) && is_get && succ == 0) a.flags[1] = 1;
  }
}

// ---- the teacher table (craft_teach.h): bfs_closest for every grid an env of pool rows
// [first, first + count) can reach -- the row with any subset of its first tt_m clearable cells
// cleared -- for every target-kind slot, direction and free interior start cell, LANES lanes per
// key.  Keys no env reaches get 0 (never read): occupied and border start cells, and subsets naming
// a cell the row does not have. ---------------------------------------------------------------------
struct TableArgs {
  int32_t first, count;
  int32_t kinds[16];         // slot -> target kind
};

// Each row's clearable cells (a kind grab, bridge or axe can clear: craft.py:383-410) in x-major
// order, the first tt_m of them, one byte each in tt_cells[row][2] (0xff = none).
__global__ __launch_bounds__(256) void tt_cells_kernel(SimView v, TableArgs a) {
  const int r = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (r >= a.count) return;
  const int row = a.first + r;
  const uint8_t* g = v.pool + (size_t)row * v.CS;
  const int m = 31 - __clz((unsigned)v.tt_nsub);                         // tt_m (tt_nsub = 1 << tt_m)
  uint32_t w[2] = {0xffffffffu, 0xffffffffu};
  int j = 0;
  for (int c = 0; c < v.C && j < m; ++c) {
    const int k = g[c], cls = kind_class(v, k);
    if (k != 0 && (cls == CRAFT_KIND_GRABBABLE || cls == CRAFT_KIND_WATER || cls == CRAFT_KIND_STONE)) {
      w[j >> 2] = (w[j >> 2] & ~(0xffu << (8 * (j & 3)))) | ((uint32_t)c << (8 * (j & 3)));
      ++j;
    }
  }
  uint32_t* out = const_cast<uint32_t*>(v.tt_cells) + 2 * (size_t)row;
  out[0] = w[0];
  out[1] = w[1];
}

template <int NW, int LANES>
__global__ __launch_bounds__(256) void teach_table_kernel(SimView v, TableArgs a) {
  const int C = v.C, H = v.H, S = v.tt_slots;
  const int64_t per_sub = (int64_t)S * 4 * C, per_row = (int64_t)v.tt_nsub * per_sub;
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / LANES;
  const int ql = (int)(threadIdx.x % LANES);
  if (i >= (int64_t)a.count * per_row) return;          // lane-group-uniform
  const int r = (int)(i / per_row);
  const int64_t k = i - (int64_t)r * per_row;
  const int sub = (int)(k / per_sub);
  const int k2 = (int)(k - (int64_t)sub * per_sub);
  const int slot = k2 / (4 * C), dir = (k2 / C) & 3, cell = k2 % C;
  const int row = a.first + r;
  const uint8_t* g = v.pool + (size_t)row * v.CS;
  const uint32_t cw[2] = {v.tt_cells[2 * (size_t)row], v.tt_cells[2 * (size_t)row + 1]};
  uint32_t m[8] = {0, 0, 0, 0, 0, 0, 0, 0};              // the subset's cleared cells
  bool valid = true, here = false;
#pragma unroll
  for (int j = 0; j < 8; ++j)
    if ((sub >> j) & 1) {
      const uint32_t c = (cw[j >> 2] >> (8 * (j & 3))) & 0xffu;
      if (c == 0xffu) valid = false;
      else {
        mask_set(m, (int)c);
        here = here || (int)c == cell;
      }
    }
  const int x = cell / H, y = cell - x * H;
  uint16_t e = 0;
  if (valid && x >= 1 && x <= v.W - 2 && y >= 1 && y <= H - 2 && (g[cell] == 0 || here)) {
    const Bits<NW> vb = brange<NW>(0, C - 2 * H);
    Bits<NW> occ, tgt;
    band_bits<NW, LANES>(reinterpret_cast<const uint32_t*>(g), (C + 3) >> 2, C, H, m, (uint32_t)a.kinds[slot], ql,
                         occ, tgt);
    int fa = -1, len = -1;
    // the row's free cells are one component (pool_conn); a subset grid may not be (its cleared
    // cells need not border a free one), so those run the exact flood instead of the shortcut
    const bool conn = sub == 0 && v.pool_conn[row] != 0;
    const bool ok = bfs_closest<NW, LANES>(occ, tgt, vb, H, cell - H, dir, ql, fa, len, true, conn);
    e = tt_encode(ok, fa, len);
  }
  if (ql == 0) const_cast<uint16_t*>(v.ttab)[(size_t)row * per_row + k] = e;
}

// The rows' answers again as the label each gives (go_leaf_action), 4 bits per (dir, cell), one
// tt_blk-byte block per (trow, slot): what craft_rollout_teach caches per env in LDS.
__global__ __launch_bounds__(256) void tt_nibble_kernel(SimView v, TableArgs a) {
  const int C = v.C, S = v.tt_slots, blk = v.tt_blk;
  const int64_t per_row = (int64_t)v.tt_nsub * S * blk;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)a.count * per_row) return;
  const int64_t r = i / per_row, k = i - r * per_row;
  const int64_t b = k / blk;                                          // sub * S + slot
  const int j = (int)(k - b * blk);
  const int64_t row = a.first + r;
  const uint16_t* e = v.ttab + (row * v.tt_nsub * S + b) * 4 * C;
  auto code = [&](int idx) -> uint32_t {
    if (idx >= 4 * C) return 15u;
    const uint32_t x = e[idx];
    if (!(x & 0x8000u)) return 15u;                                   // not computed
    const int fa = (int)((x >> 10) & 7u) - 1, len = (int)(x & 0x3ffu) - 1;
    if (!(x & 0x4000u) || len == 0) return 5u;                         // the reference raises
    if (len < 0) return 4u;                                            // no target: STOP
    return (uint32_t)fa;
  };
  const_cast<uint8_t*>(v.ttab4)[(row * v.tt_nsub * S + b) * blk + j] = (uint8_t)(code(2 * j) | (code(2 * j + 1) << 4));
}

hipError_t launch_teach_table(int nw, const SimView& v, int32_t first, int32_t count, const int32_t* kinds,
                              hipStream_t st) {
  if (!v.ttab || count <= 0 || v.tt_slots <= 0) return hipSuccess;
  TableArgs a{};
  a.first = first;
  a.count = count;
  for (int s = 0; s < v.tt_slots && s < 16; ++s) a.kinds[s] = kinds[s];
  hipLaunchKernelGGL(tt_cells_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, st, v, a);
  constexpr int LANES = 2;
  const int64_t items = (int64_t)count * v.tt_nsub * v.tt_slots * 4 * v.C;
  const int64_t blocks = (LANES * items + 255) / 256;
  if (blocks > 0x7fffffffLL) return hipErrorInvalidValue;
#define CRAFT_TT(NWV) hipLaunchKernelGGL((teach_table_kernel<NWV, LANES>), dim3((unsigned)blocks), dim3(256), 0, st, v, a)
  if (nw <= 2) CRAFT_TT(2);
  else if (nw <= 4) CRAFT_TT(4);
  else if (nw <= 5) CRAFT_TT(5);
  else CRAFT_TT(8);
#undef CRAFT_TT
  if (v.ttab4) {
    const int64_t bytes = (int64_t)count * v.tt_nsub * v.tt_slots * v.tt_blk;
    if ((bytes + 255) / 256 > 0x7fffffffLL) return hipErrorInvalidValue;
    hipLaunchKernelGGL(tt_nibble_kernel, dim3((unsigned)((bytes + 255) / 256)), dim3(256), 0, st, v, a);
  }
  return hipGetLastError();
}

hipError_t launch_distances(int nw, const SimView& v, const int32_t* tasks, const int8_t* success,
                            const int32_t* seqs, int32_t ticks, int64_t n, int32_t* dist_out,
                            uint8_t* is_get_out, int32_t* n_actions_out, int32_t* flags, hipStream_t st) {
  DistArgs a{tasks, success, seqs, ticks, n, dist_out, is_get_out, n_actions_out, flags};
  const int lanes = n <= kTeacherQuadMaxItems ? 4 : 2;
  const unsigned blocks = (unsigned)((lanes * n + 255) / 256);
#define CRAFT_DIST(NWV)                                                                                 \
  do {                                                                                                  \
    if (lanes == 4) hipLaunchKernelGGL((distances_kernel<NWV, 4>), dim3(blocks), dim3(256), 0, st, v, a); \
    else hipLaunchKernelGGL((distances_kernel<NWV, 2>), dim3(blocks), dim3(256), 0, st, v, a);          \
  } while (0)
  if (nw <= 2) CRAFT_DIST(2);
  else if (nw <= 4) CRAFT_DIST(4);
  else if (nw <= 5) CRAFT_DIST(5);
  else CRAFT_DIST(8);
#undef CRAFT_DIST
  return hipGetLastError();
}

hipError_t launch_teacher(int nw, int forced, const SimView& v, const int32_t* slots, const int32_t* tasks,
                          int64_t n, int32_t* act_out, int32_t* len_out, hipStream_t st) {
  TeachArgs a{slots, tasks, n, act_out, len_out};
  // nw = 32-bit words per BFS cell set (craft_teach.h: the band of columns 1 .. W-2):
  // 8x8 -> 2, 10x10 -> 3 (run as 4), 12x12 -> 4, 16x16 -> 7 (run as 8)
  // forced: craft_sim_tune_teach's lanes per query (1, 2 or 4), else 0: quads for small batches,
  // pairs above
  const int lanes = (forced == 1 || forced == 2 || forced == 4) ? forced : (n <= kTeacherQuadMaxItems ? 4 : 2);
  const unsigned blocks = (unsigned)((lanes * n + 255) / 256);
  // without path lengths the table's answers finish in the walk and the rest run densely
#define CRAFT_TEACH_D(NWV, D)                                                                             \
  do {                                                                                                    \
    if (lanes == 4) hipLaunchKernelGGL((teacher_kernel<NWV, 4, D>), dim3(blocks), dim3(256), 0, st, v, a); \
    else if (lanes == 2) hipLaunchKernelGGL((teacher_kernel<NWV, 2, D>), dim3(blocks), dim3(256), 0, st, v, a); \
    else hipLaunchKernelGGL((teacher_kernel<NWV, 1, D>), dim3(blocks), dim3(256), 0, st, v, a);           \
  } while (0)
#define CRAFT_TEACH(NWV)                         \
  do {                                           \
    if (len_out) CRAFT_TEACH_D(NWV, false);      \
    else CRAFT_TEACH_D(NWV, true);               \
  } while (0)
  if (nw <= 2) CRAFT_TEACH(2);
  else if (nw <= 4) CRAFT_TEACH(4);
  else if (nw <= 5) CRAFT_TEACH(5);
  else CRAFT_TEACH(8);
#undef CRAFT_TEACH
#undef CRAFT_TEACH_D
  return hipGetLastError();
}

}  // namespace craft
