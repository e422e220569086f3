// craft_teach.h — DemonstrationTeacher (teachers/demonstration.py:9-30) for one
// env: the hint-tree walk of BaseTeacher.find_incomplete_subtask and
// find_closest_resources' BFS (teachers/base.py:10-87), the BFS held as
// per-direction position bitsets in registers.  Shared by the standalone
// teacher kernel (craft_teacher.hip: grid rebuilt from the pool row and the
// cleared-cell mask in HBM) and the fused tick + teacher kernel
// (craft_tick_teach.hip: the post-step grid row already in LDS).
#pragma once
#include "craft_bits.h"

namespace craft {

// find_closest_resources (teachers/base.py:27-34) over shortest_path
// (teachers/base.py:36-87), exactly, with one forward and one backward BFS over
// (pos, dir) states held as per-direction position bitsets.
//
// What the reference returns.  Each target's own FIFO BFS dequeues level by level,
// and within a level in order of the path's first action (level 1 is enqueued in
// action order DOWN, UP, LEFT, RIGHT; a child keeps its first-dequeued parent's
// label).  So a target's path length L is the first level at which a state faces
// it, and its first action is the smallest first action over all shortest paths
// to a state facing it.  The chosen target is the first in np.nonzero (x-major)
// order with the minimal L (strict `<`, base.py:31).
//
// How it is computed here.
//  * Forward: a move's result does not depend on the current direction, so level
//    k+1 in direction a is (shift(U_k, d_a) & free | U_k & blocked_a) minus the
//    visited set of direction a, U_k being the positions of level k.  A level's
//    facing cells are its states shifted once more.  This gives every target's L
//    and the chosen target, in ~40 bitset operations per level.
//  * Backward, for the chosen target only: reverse BFS from the states facing it
//    for L-1 levels; the first action is the smallest a whose level-1 state
//    step(start, a) is within reverse distance L-1 (then exactly L-1).
// Returns false where the reference raises (len(None) on an unreachable target
// after a reachable one, base.py:31): the forward BFS then runs until its
// frontier is empty, so `claimed` holds every reachable target.
// One lane per query (LANES = 1): the same forward and backward passes, the four
// actions of a level in one lane.
template <int NW>
__device__ bool bfs_closest_1(const Bits<NW>& occ, const Bits<NW>& tgt, const Bits<NW>& valid,
                              int H, int p0, int d0, int& first_action, int& path_len,
                              bool want_action) {
  const int dl[4] = {-1, 1, -H, H};   // DOWN, UP, LEFT, RIGHT in x-major cell index
  const Bits<NW> fr = bandn(valid, occ);
  Bits<NW> blk[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) blk[a] = bshift(occ, -dl[a]);   // blk[a][p] = occ[p + dl[a]]
  first_action = -1;
  path_len = -1;
  Bits<NW> claimed = bzero<NW>();
  int L = -1, chosen = -1;
  {
    const int f0 = p0 + dl[d0];            // the start state already faces a target: []
    if (f0 >= 0 && btest(tgt, f0)) {
      L = 0;
      chosen = f0;
      claimed = bbit<NW>(f0);
    }
  }
  Bits<NW> V[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) V[a] = (a == d0) ? bbit<NW>(p0) : bzero<NW>();
  Bits<NW> U = bbit<NW>(p0);
  for (int depth = 1; bany(bandn(tgt, claimed)); ++depth) {
    Bits<NW> nU = bzero<NW>(), hit = bzero<NW>();
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const Bits<NW> nxt = bandn(bor(band(bshift(U, dl[a]), fr), band(U, blk[a])), V[a]);
      V[a] = bor(V[a], nxt);
      nU = bor(nU, nxt);
      hit = bor(hit, band(bshift(nxt, dl[a]), tgt));
    }
    if (!bany(nU)) break;                  // every reachable state visited
    hit = bandn(hit, claimed);
    if (bany(hit)) {
      claimed = bor(claimed, hit);
      if (L < 0) {
        L = depth;
        chosen = blowest(hit);
      }
    }
    U = nU;
  }
  if (L < 0) return true;                  // no target at all, or none reachable: None
  path_len = L;
  const Bits<NW> unreached = bandn(tgt, claimed);
  if (bany(unreached) && blowest(claimed) < bhighest(unreached)) return false;
  if (L == 0 || !want_action) return true;
  Bits<NW> G[4];                           // reverse BFS from the states facing `chosen`
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int q = chosen - dl[a];
    G[a] = (q >= 0) ? band(bbit<NW>(q), fr) : bzero<NW>();
    V[a] = G[a];
  }
  for (int k = 1; k < L; ++k) {
    Bits<NW> P = bzero<NW>();              // predecessors: any direction at these positions
#pragma unroll
    for (int a = 0; a < 4; ++a) P = bor(P, bor(band(bshift(G[a], -dl[a]), fr), band(G[a], blk[a])));
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      G[a] = bandn(P, V[a]);
      V[a] = bor(V[a], G[a]);
    }
  }
#pragma unroll
  for (int a = 3; a >= 0; --a) {           // the smallest qualifying action wins
    const int q0 = p0 + dl[a];
    const int q = btest(fr, q0) ? q0 : p0;
    if (!(q == p0 && a == d0) && btest(V[a], q)) first_action = a;
  }
  return true;
}

// OR over the 4 lanes of a quad (DPP quad_perm [1,0,3,2] then [2,3,0,1]).
__device__ __forceinline__ uint32_t quad_or(uint32_t x) {
  x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);
  x |= (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, false);
  return x;
}
template <int NW>
__device__ __forceinline__ Bits<NW> quad_or(const Bits<NW>& a) {
  Bits<NW> r;
#pragma unroll
  for (int i = 0; i < NW; ++i) r.w[i] = quad_or(a.w[i]);
  return r;
}

// LANES = 4: the four lanes of a quad run one query together, lane ql handling the states
// entered by action ql (its direction's visited set and blocked mask): each
// level is then one action's worth of bitset work plus two quad ORs, instead of
// four actions' worth in one lane.  Every quantity that steers control flow is
// quad-uniform.
template <int NW, int LANES>
__device__ bool bfs_closest(const Bits<NW>& occ, const Bits<NW>& tgt, const Bits<NW>& valid,
                            int H, int p0, int d0, int ql, int& first_action, int& path_len,
                            bool want_action = true) {
  if (LANES == 1) return bfs_closest_1<NW>(occ, tgt, valid, H, p0, d0, first_action, path_len, want_action);
  const int dla = ql == 0 ? -1 : ql == 1 ? 1 : ql == 2 ? -H : H;   // this lane's action
  const Bits<NW> fr = bandn(valid, occ);
  const Bits<NW> blk = bshift_var(occ, -dla);                         // blk[p] = occ[p + dla]
  const int dl0 = d0 == 0 ? -1 : d0 == 1 ? 1 : d0 == 2 ? -H : H;
  first_action = -1;
  path_len = -1;
  Bits<NW> claimed = bzero<NW>();
  int L = -1, chosen = -1;
  {
    const int f0 = p0 + dl0;               // the start state already faces a target: []
    if (f0 >= 0 && btest(tgt, f0)) {
      L = 0;
      chosen = f0;
      claimed = bbit<NW>(f0);
    }
  }
  Bits<NW> V = (ql == d0) ? bbit<NW>(p0) : bzero<NW>();   // visited states of direction ql
  Bits<NW> U = bbit<NW>(p0);
  for (int depth = 1; bany(bandn(tgt, claimed)); ++depth) {
    const Bits<NW> nxt = bandn(bor(band(bshift_var(U, dla), fr), band(U, blk)), V);
    V = bor(V, nxt);
    const Bits<NW> nU = quad_or(nxt);
    Bits<NW> hit = quad_or(band(bshift_var(nxt, dla), tgt));
    if (!bany(nU)) break;                  // every reachable state visited
    hit = bandn(hit, claimed);
    if (bany(hit)) {
      claimed = bor(claimed, hit);
      if (L < 0) {
        L = depth;
        chosen = blowest(hit);
      }
    }
    U = nU;
  }
  if (L < 0) return true;                  // no target at all, or none reachable: None
  path_len = L;
  const Bits<NW> unreached = bandn(tgt, claimed);
  if (bany(unreached) && blowest(claimed) < bhighest(unreached)) return false;
  if (L == 0 || !want_action) return true;
  // reverse BFS from the states facing `chosen`; G = this level's states of direction
  // ql, V reused as the reverse-visited set
  Bits<NW> G;
  {
    const int q = chosen - dla;
    G = (q >= 0) ? band(bbit<NW>(q), fr) : bzero<NW>();
    V = G;
  }
  for (int k = 1; k < L; ++k) {
    // predecessors, any direction, at these positions: moved here or turned in place
    const Bits<NW> P = quad_or(bor(band(bshift_var(G, -dla), fr), band(G, blk)));
    G = bandn(P, V);
    V = bor(V, G);
  }
  // the smallest action whose level-1 state lies within reverse distance L-1
  const int q0 = p0 + dla;
  const int q = btest(fr, q0) ? q0 : p0;
  const bool ok = !(q == p0 && ql == d0) && btest(V, q);
  const uint64_t b = __ballot(ok);
  const uint32_t quad = (uint32_t)(b >> (__lane_id() & ~3u)) & 0xfu;
  first_action = quad ? __ffs(quad) - 1 : -1;
  return true;
}

// DemonstrationTeacher.__call__ (teachers/demonstration.py:9-30) for one env, LANES
// lanes of a quad-aligned group (lane ql of the group).  Its current grid is row32
// (kind ids, x-major, as 32-bit words; NW*8 words at most) minus the cells set in m
// (cleared this episode; all zero when the row is already current), its inventory
// iv, its agent s, the task `task`.  Returns the action, or -2 where the reference
// raises (err_out = CRAFT_ETEACHER).  With want_len, len_out receives
// len(find_closest_resources(task.arg)) (-1: no target, -2: the reference raises).
template <int NW, int LANES>
__device__ __forceinline__ int teach_env(const SimView& v, const uint32_t* row32, const uint32_t (&m)[8],
                                         const uint8_t* iv, const Agent& s, int task, int ql,
                                         bool want_len, int& len_out, int& err_out) {
  const int H = v.H, C = v.C;
  auto kind_at = [&](int c) -> int {
    const uint32_t w = row32[c >> 2];
    const bool cleared = (m[c >> 5] >> (c & 31)) & 1u;
    return cleared ? 0 : (int)((w >> (8 * (c & 3))) & 0xffu);
  };
  const int facing = kind_at((s.x + dir_dx(s.dir)) * H + (s.y + dir_dy(s.dir)));

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
  // Occupancy and per-kind target bitsets of the current grid: the row is read as
  // dwords in a fully unrolled loop so every bit position is static (no per-cell
  // dependent loads, no dynamic indexing).
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
  auto closest = [&](int kind, int& fa, int& len, bool want_action) -> bool {
    Bits<NW> occ, tgt;
    grids(kind, occ, tgt);
    return bfs_closest<NW, LANES>(occ, tgt, valid, H, s.x * H + s.y, s.dir, ql, fa, len, want_action);
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
        leaf_ok = closest(arg, fa, len, true);
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
  if (err) action = -2;                // where the reference raises
  err_out = err;
  if (want_len) {
    const int arg = (v.task_tab[task] >> 4) & 0xff;
    int fa = leaf_fa, len = leaf_len;
    bool ok = leaf_ok;
    if (arg != leaf_kind) {               // the teacher's BFS already answered get[X]'s go[X]
      len = -1;
      ok = arg > 0 ? closest(arg, fa, len, false) : true;
    }
    len_out = ok ? len : -2;
  }
  return action;
}

}  // namespace craft
