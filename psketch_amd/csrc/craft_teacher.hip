// craft_teacher.hip — DemonstrationTeacher on the GPU: the hint-tree walk of
// BaseTeacher.find_incomplete_subtask and find_closest_resources' BFS, one lane
// per env, the BFS held as per-direction position bitsets in registers.
#include "craft_bits.h"

namespace craft {

// find_closest_resources (teachers/base.py:27-34) over shortest_path
// (teachers/base.py:36-87) as ONE level-synchronous BFS over (pos, dir) states
// held as per-direction position bitsets.  FIFO order within a level is
// sorted by the path's first action (induction: level 1 is enqueued in action
// order DOWN, UP, LEFT, RIGHT, and children keep their first-dequeued parent's
// label), so tracking the level's states per first action (a "label")
// reproduces exactly which state the reference dequeues first:
//   a target's path length = the first level at which a state faces it,
//   its first action = the smallest label among that level's facing states,
//   the chosen target = the first in np.nonzero (x-major) order with the
//   minimal length (strict `<`, base.py:31).
// Returns false where the reference raises (len(None) on an unreachable
// target after a reachable one, base.py:31).
template <int NW>
__device__ bool bfs_closest(const Bits<NW>& occ, const Bits<NW>& tgt, const Bits<NW>& valid,
                            int H, int p0, int d0, int& first_action, int& path_len) {
  const int dl[4] = {-1, 1, -H, H};   // DOWN, UP, LEFT, RIGHT in x-major cell index
  const Bits<NW> fr = bandn(valid, occ);
  Bits<NW> V[4], cur[4], fc[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) V[a] = bzero<NW>();
#pragma unroll
  for (int a = 0; a < 4; ++a) V[a] = (a == d0) ? bbit<NW>(p0) : V[a];
  Bits<NW> claimed = bzero<NW>();
  bool found = false;
  first_action = -1;
  path_len = -1;
  {
    const int f0 = p0 + dl[d0];            // start state already faces a target: []
    if (f0 >= 0 && btest(tgt, f0)) {
      found = true;
      path_len = 0;
      claimed = bbit<NW>(f0);
    }
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int q0 = p0 + dl[a];
    const int q = btest(fr, q0) ? q0 : p0;
    if (!btest(V[a], q)) {
      V[a] = bor(V[a], bbit<NW>(q));
      cur[a] = bbit<NW>(q);
      fc[a] = band(bshift(cur[a], dl[a]), valid);
    } else {
      cur[a] = bzero<NW>();
      fc[a] = bzero<NW>();
    }
  }
  Bits<NW> blk[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) blk[a] = bshift(occ, -dl[a]);   // blk[a][p] = occ[p + dl[a]]
  int depth = 1;
  while (bany(bor(bor(cur[0], cur[1]), bor(cur[2], cur[3])))) {
    int bp = INT_MAX, bl = -1;
#pragma unroll
    for (int lab = 0; lab < 4; ++lab) {
      const Bits<NW> hit = bandn(band(fc[lab], tgt), claimed);
      if (bany(hit)) {
        claimed = bor(claimed, hit);
        const int p = blowest(hit);
        if (p < bp) { bp = p; bl = lab; }
      }
    }
    if (!found && bl >= 0) {
      found = true;
      path_len = depth;
      first_action = bl;
    }
    if (!bany(bandn(tgt, claimed))) break;
    // Expand label by label, in place: a label's current set is only needed for
    // its own expansion, and V[a] (updated immediately) gives smaller labels priority.
#pragma unroll
    for (int lab = 0; lab < 4; ++lab) {
      Bits<NW> nc = bzero<NW>(), nf = bzero<NW>();
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const Bits<NW> moved = bor(band(bshift(cur[lab], dl[a]), fr), band(cur[lab], blk[a]));
        const Bits<NW> fresh = bandn(moved, V[a]);
        V[a] = bor(V[a], fresh);
        nc = bor(nc, fresh);
        nf = bor(nf, band(bshift(fresh, dl[a]), valid));
      }
      cur[lab] = nc;
      fc[lab] = nf;
    }
    ++depth;
  }
  if (found) {
    const Bits<NW> unreached = bandn(tgt, claimed);
    if (bany(unreached) && blowest(claimed) < bhighest(unreached)) return false;
  }
  return true;
}


struct TeachArgs {
  const int32_t* slots;
  const int32_t* tasks;
  int64_t n;
  int32_t* act_out;
  int32_t* len_out;
};

__device__ __forceinline__ int grid_kind(const SimView& v, int scen, const uint32_t (&m)[8], int c) {
  const int k = v.pool[(size_t)scen * v.CS + c];
  uint32_t mw = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) mw |= (i == (c >> 5)) ? m[i] : 0u;
  return ((mw >> (c & 31)) & 1u) ? 0 : k;
}

// DemonstrationTeacher.__call__ (teachers/demonstration.py:9-30), one lane per slot.
template <int NW>
__global__ __launch_bounds__(256) void teacher_kernel(SimView v, TeachArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  const int64_t slot = a.slots ? (int64_t)a.slots[i] : i;
  if (slot == -1) {                    // skipped item: the trainer's ref_action for a done env
    a.act_out[i] = -1;
    if (a.len_out) a.len_out[i] = -1;
    return;
  }
  if (slot < 0 || slot >= v.n_envs) {
    latch_error(v.err, CRAFT_ERANGE, i);
    a.act_out[i] = -2;
    if (a.len_out) a.len_out[i] = -2;
    return;
  }
  const Agent s = unpack_state(v.state[slot]);
  if (s.frozen) {                      // done env: its label is -1 (imitation.py:50-51)
    a.act_out[i] = -1;
    if (a.len_out) a.len_out[i] = -1;
    return;
  }
  const int task = a.tasks ? a.tasks[i] : s.task;
  if (task < 0 || task >= v.n_tasks || s.x < 1 || s.x > v.W - 2 || s.y < 1 || s.y > v.H - 2 ||
      s.scen >= v.pool_count) {
    latch_error(v.err, task < 0 || task >= v.n_tasks ? CRAFT_ERANGE : CRAFT_EINVAL, i);
    a.act_out[i] = -2;
    if (a.len_out) a.len_out[i] = -2;
    return;
  }
  uint32_t m[8];
  {
    const uint4 m0 = v.mask[2 * slot], m1 = v.mask[2 * slot + 1];
    m[0] = m0.x; m[1] = m0.y; m[2] = m0.z; m[3] = m0.w;
    m[4] = m1.x; m[5] = m1.y; m[6] = m1.z; m[7] = m1.w;
  }
  const uint8_t* iv = reinterpret_cast<const uint8_t*>(v.inv + 2 * slot);
  const int H = v.H, C = v.C;
  const int facing = grid_kind(v, s.scen, m, (s.x + dir_dx(s.dir)) * H + (s.y + dir_dy(s.dir)));

  auto sat = [&](int t) -> int {       // satisfies(), craft.py:285-294
    const uint32_t tt = v.task_tab[t];
    const int goal = tt & 0xf, arg = (tt >> 4) & 0xff;
    if (goal == CRAFT_GOAL_GET || goal == CRAFT_GOAL_MAKE) return iv[arg] > 0;
    if (goal == CRAFT_GOAL_GO) return facing == arg;
    return -1;
  };

  Bits<NW> valid = bzero<NW>();
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    const int nb = min(32, max(0, C - w * 32));
    valid.w[w] = nb >= 32 ? ~0u : ((1u << nb) - 1u);
  }
  // Occupancy and per-kind target bitsets of the current grid (pool row minus the
  // cleared-cell mask): the row is read as dwords in a fully unrolled loop so every
  // bit position is static (no per-cell dependent loads, no dynamic indexing).
  const uint32_t* row32 = reinterpret_cast<const uint32_t*>(v.pool + (size_t)s.scen * v.CS);
  const int nq = (C + 3) >> 2;
  auto grids = [&](int kind, Bits<NW>& occ, Bits<NW>& tgt) {
    occ = bzero<NW>();
    tgt = bzero<NW>();
#pragma unroll
    for (int q = 0; q < NW * 8; ++q) {
      if (q < nq) {
        const uint32_t w = row32[q];
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int c = 4 * q + b;
          const uint32_t k = (w >> (8 * b)) & 0xffu;
          const bool cleared = (m[c >> 5] >> (c & 31)) & 1u;
          const uint32_t bit = (k != 0 && !cleared) ? (1u << (c & 31)) : 0u;
          occ.w[c >> 5] |= bit;
          tgt.w[c >> 5] |= (k == (uint32_t)kind) ? bit : 0u;
        }
      }
    }
  };
  auto closest = [&](int kind, int& fa, int& len) -> bool {
    Bits<NW> occ, tgt;
    grids(kind, occ, tgt);
    return bfs_closest<NW>(occ, tgt, valid, H, s.x * H + s.y, s.dir, fa, len);
  };
  int leaf_kind = -1, leaf_fa = -1, leaf_len = -1;
  bool leaf_ok = true;

  int action = CRAFT_STOP;
  int err = 0;
  // find_incomplete_subtask, teachers/base.py:10-25
  int node = task;
  if (sat(node) != 1) {
    for (int guard = 0; guard < CRAFT_MAX_TASKS; ++guard) {
      const int nsub = (v.task_tab[node] >> 12) & 0xf;
      if (nsub == 0) break;
      const int32_t* sub = v.task_sub + CRAFT_MAX_SUBTASKS * node;
      int chosen = sub[nsub - 1];
      bool last = true;
      for (int q = 0; q + 1 < nsub; ++q)
        if (sat(sub[q]) != 1) { chosen = sub[q]; last = false; break; }
      if (last && sat(chosen) == 1) { err = CRAFT_ETEACHER; break; }   // base.py:24 assert
      node = chosen;
    }
    if (!err) {
      const uint32_t lt = v.task_tab[node];
      const int goal = lt & 0xf, arg = (lt >> 4) & 0xff;
      if (goal == CRAFT_GOAL_USE) {
        action = CRAFT_USE;
      } else if (goal == CRAFT_GOAL_GO) {
        int fa = -1, len = -1;
        leaf_ok = closest(arg, fa, len);
        leaf_kind = arg; leaf_fa = fa; leaf_len = len;
        if (!leaf_ok) err = CRAFT_ETEACHER;
        else if (len < 0) action = CRAFT_STOP;                           // demonstration.py:25-26
        else if (len == 0) err = CRAFT_ETEACHER;                         // [][0]
        else action = fa;
      } else {
        err = CRAFT_ETEACHER;                                            // demonstration.py:18
      }
    }
  }
  if (err) {
    latch_error(v.err, err, slot);
    action = -2;                       // where the reference raises
  }
  a.act_out[i] = action;
  if (a.len_out) {
    const int arg = (v.task_tab[task] >> 4) & 0xff;
    int fa = leaf_fa, len = leaf_len;
    bool ok = leaf_ok;
    if (arg != leaf_kind) {               // the teacher's BFS already answered get[X]'s go[X]
      len = -1;
      ok = arg > 0 ? closest(arg, fa, len) : true;
    }
    if (!ok) {
      latch_error(v.err, CRAFT_ETEACHER, slot);
      len = -2;
    }
    a.len_out[i] = len;
  }
}

hipError_t launch_teacher(int nw, const SimView& v, const int32_t* slots, const int32_t* tasks,
                          int64_t n, int32_t* act_out, int32_t* len_out, hipStream_t st) {
  TeachArgs a{slots, tasks, n, act_out, len_out};
  const unsigned blocks = (unsigned)((n + 255) / 256);
  // nw = 32-bit words per cell set: 8x8 -> 2, 10x10 -> 4, 12x12 -> 5, 16x16 -> 8
  if (nw <= 2) hipLaunchKernelGGL(teacher_kernel<2>, dim3(blocks), dim3(256), 0, st, v, a);
  else if (nw <= 4) hipLaunchKernelGGL(teacher_kernel<4>, dim3(blocks), dim3(256), 0, st, v, a);
  else if (nw <= 5) hipLaunchKernelGGL(teacher_kernel<5>, dim3(blocks), dim3(256), 0, st, v, a);
  else hipLaunchKernelGGL(teacher_kernel<8>, dim3(blocks), dim3(256), 0, st, v, a);
  return hipGetLastError();
}

}  // namespace craft
