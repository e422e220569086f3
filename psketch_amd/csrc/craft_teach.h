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
// A level's states face a target where they stand on F_a = shift(tgt, -d_a) (the
// cell ahead in their direction a is a target), so the level loop only tests
// nxt_a & F_a; the faced targets themselves are formed on the rare levels that
// have any.
// The cell sets are kept over the band of columns 1 .. W-2 only (bit p = cell p + H of the
// x-major grid): columns 0 and W-1 are the border, always occupied, never entered, so they are
// left out (12x12: 120 bits = 4 words instead of 5).  What they contributed is that a LEFT move
// from column 1 and a RIGHT move from column W-2 are blocked: these edge sets say so.  Rows 0
// and H-1 stay in the band, so moves along a column need nothing.  Cell order is unchanged,
// so `first in x-major order` comparisons are too.
template <int NW>
__device__ __forceinline__ Bits<NW> band_edge_lo(const Bits<NW>& valid, int H) {   // column 1
  return brange<NW>(0, H);
}
template <int NW>
__device__ __forceinline__ Bits<NW> band_edge_hi(const Bits<NW>& valid, int H) {   // column W-2
  const int cb = bcount(valid);
  return brange<NW>(cb - H, cb);
}

// One lane per query (LANES = 1): the same forward and backward passes, the four
// actions of a level in one lane.
template <int NW>
__device__ bool bfs_closest_1(const Bits<NW>& occ, const Bits<NW>& tgt, const Bits<NW>& valid,
                              int H, int p0, int d0, int& first_action, int& path_len,
                              bool want_action, bool conn) {
  const int dl[4] = {-1, 1, -H, H};   // DOWN, UP, LEFT, RIGHT in x-major cell index
  const Bits<NW> fr = bandn(valid, occ);
  Bits<NW> blk[4], fa[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    blk[a] = bshift(occ, -dl[a]);     // blk[a][p] = occ[p + dl[a]]
    fa[a] = bshift(tgt, -dl[a]);      // fa[a][p] = tgt[p + dl[a]]
  }
  blk[2] = bor(blk[2], band_edge_lo<NW>(valid, H));   // the border columns left out of the band
  blk[3] = bor(blk[3], band_edge_hi<NW>(valid, H));
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
  const bool open = bany(bandn(tgt, claimed));   // some target not yet claimed
  for (int depth = 1; open && L < 0; ++depth) {
    Bits<NW> nU = bzero<NW>(), nx[4];
    uint32_t face = 0;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      nx[a] = bandn(bor(band(bshift(U, dl[a]), fr), band(U, blk[a])), V[a]);
      V[a] = bor(V[a], nx[a]);
      nU = bor(nU, nx[a]);
#pragma unroll
      for (int i = 0; i < NW; ++i) face |= nx[a].w[i] & fa[a].w[i];
    }
    if (!bany(nU)) break;                  // every reachable state visited
    if (face) {
      Bits<NW> hit = bzero<NW>();
#pragma unroll
      for (int a = 0; a < 4; ++a) hit = bor(hit, band(bshift(nx[a], dl[a]), tgt));
      hit = bandn(hit, claimed);
      if (bany(hit)) {
        claimed = bor(claimed, hit);
        L = depth;
        chosen = blowest(hit);
        break;                             // L and the chosen target are known
      }
    }
    U = nU;
  }
  if (L < 0) return true;                  // no target at all, or none reachable: None
  path_len = L;
  if (bany(bandn(tgt, claimed)) && conn && btest(fr, p0)) {
    // every free cell is reachable (bfs_closest below): the targets next to one
    Bits<NW> adj = bzero<NW>();
#pragma unroll
    for (int a = 0; a < 4; ++a) adj = bor(adj, bshift(fr, dl[a]));
    claimed = bor(claimed, band(adj, tgt));
    const Bits<NW> unreached = bandn(tgt, claimed);
    if (bany(unreached) && blowest(claimed) < bhighest(unreached)) return false;
  } else if (bany(bandn(tgt, claimed))) {
    // reachability of the other targets (base.py:31), as in bfs_closest below
    Bits<NW> R = bor(bor(bor(V[0], V[1]), bor(V[2], V[3])), bbit<NW>(p0));
    for (;;) {
      Bits<NW> adj = bzero<NW>();
#pragma unroll
      for (int a = 0; a < 4; ++a) adj = bor(adj, bshift(R, dl[a]));
      claimed = bor(claimed, band(adj, tgt));
      if (!bany(bandn(tgt, claimed))) break;
      const Bits<NW> grow = bandn(band(adj, fr), R);
      if (!bany(grow)) break;
      R = bor(R, grow);
    }
    const Bits<NW> unreached = bandn(tgt, claimed);
    if (bany(unreached) && blowest(claimed) < bhighest(unreached)) return false;
  }
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

// OR over the 2 lanes of a pair (DPP quad_perm [1,0,3,2]).
__device__ __forceinline__ uint32_t pair_or(uint32_t x) {
  return x | (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);
}
template <int NW>
__device__ __forceinline__ Bits<NW> pair_or(const Bits<NW>& a) {
  Bits<NW> r;
#pragma unroll
  for (int i = 0; i < NW; ++i) r.w[i] = pair_or(a.w[i]);
  return r;
}

// LANES = 2: the two lanes of a pair run one query together, lane pl handling the
// states entered by actions 2pl and 2pl + 1 (DOWN/UP: cell shifts -1/+1; LEFT/RIGHT:
// -H/+H).  Each lane's two shifts are by the same amount s in opposite directions, so
// they are plain funnel shifts by a per-lane amount (no per-lane direction select), and a
// level costs one pair OR instead of two quad steps: about half the instructions per
// query of LANES = 4, at the same dependent-chain length.  The same forward, reachability
// and backward passes as bfs_closest_1; everything that steers control flow is
// pair-uniform.
template <int NW>
__device__ __forceinline__ Bits<NW> bshift_up(const Bits<NW>& a, uint32_t s) {   // p -> p + s
  Bits<NW> r;
  r.w[0] = a.w[0] << s;
#pragma unroll
  for (int i = 1; i < NW; ++i) r.w[i] = __builtin_amdgcn_alignbit(a.w[i], a.w[i - 1], 32u - s);
  return r;
}
template <int NW>
__device__ __forceinline__ Bits<NW> bshift_dn(const Bits<NW>& a, uint32_t s) {   // p -> p - s
  Bits<NW> r;
#pragma unroll
  for (int i = 0; i + 1 < NW; ++i) r.w[i] = __builtin_amdgcn_alignbit(a.w[i + 1], a.w[i], s);
  r.w[NW - 1] = a.w[NW - 1] >> s;
  return r;
}
template <int NW>
__device__ bool bfs_closest_2(const Bits<NW>& occ, const Bits<NW>& tgt, const Bits<NW>& valid,
                              int H, int p0, int d0, int pl, int& first_action, int& path_len,
                              bool want_action, bool conn) {
  const uint32_t s = pl ? (uint32_t)H : 1u;     // lo action 2pl moves by -s, hi action 2pl + 1 by +s
  const int alo = 2 * pl;
  const Bits<NW> fr = bandn(valid, occ);
  Bits<NW> blk_lo = bshift_up(occ, s), blk_hi = bshift_dn(occ, s);         // blk[p] = occ[p + d]
  if (pl) {                              // LEFT / RIGHT: the border columns left out of the band
    blk_lo = bor(blk_lo, band_edge_lo<NW>(valid, H));
    blk_hi = bor(blk_hi, band_edge_hi<NW>(valid, H));
  }
  const Bits<NW> fa_lo = bshift_up(tgt, s), fa_hi = bshift_dn(tgt, s);     // fa[p] = tgt[p + d]
  const int dl0 = d0 == 0 ? -1 : d0 == 1 ? 1 : d0 == 2 ? -H : H;
  const uint32_t psh = __lane_id() & ~1u;                                  // this pair's lanes in a ballot
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
  Bits<NW> Vlo = (alo == d0) ? bbit<NW>(p0) : bzero<NW>();
  Bits<NW> Vhi = (alo + 1 == d0) ? bbit<NW>(p0) : bzero<NW>();
  Bits<NW> U = bbit<NW>(p0);
  const bool open = bany(bandn(tgt, claimed));
  for (int depth = 1; open && L < 0; ++depth) {
    const Bits<NW> nlo = bandn(bor(band(bshift_dn(U, s), fr), band(U, blk_lo)), Vlo);
    const Bits<NW> nhi = bandn(bor(band(bshift_up(U, s), fr), band(U, blk_hi)), Vhi);
    Vlo = bor(Vlo, nlo);
    Vhi = bor(Vhi, nhi);
    const Bits<NW> nU = pair_or(bor(nlo, nhi));
    if (!bany(nU)) break;                  // every reachable state visited
    uint32_t face = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) face |= (nlo.w[i] & fa_lo.w[i]) | (nhi.w[i] & fa_hi.w[i]);
    if ((uint32_t)(__ballot(face != 0) >> psh) & 0x3u) {   // some lane of the pair faces a target
      const Bits<NW> hit = bandn(pair_or(band(bor(bshift_dn(nlo, s), bshift_up(nhi, s)), tgt)), claimed);
      if (bany(hit)) {
        claimed = bor(claimed, hit);
        L = depth;
        chosen = blowest(hit);
        break;
      }
    }
    U = nU;
  }
  if (L < 0) return true;                  // no target at all, or none reachable: None
  path_len = L;
  if (bany(bandn(tgt, claimed)) && conn && btest(fr, p0)) {
    // connected free cells (see bfs_closest): a target is reachable iff it has a free neighbour
    claimed = bor(claimed, band(pair_or(bor(bshift_dn(fr, s), bshift_up(fr, s))), tgt));
    const Bits<NW> unreached = bandn(tgt, claimed);
    if (bany(unreached) && blowest(claimed) < bhighest(unreached)) return false;
  } else if (bany(bandn(tgt, claimed))) {
    Bits<NW> R = bor(pair_or(bor(Vlo, Vhi)), bbit<NW>(p0));
    for (;;) {
      const Bits<NW> adj = pair_or(bor(bshift_dn(R, s), bshift_up(R, s)));   // cells next to R
      claimed = bor(claimed, band(adj, tgt));
      if (!bany(bandn(tgt, claimed))) break;
      const Bits<NW> grow = bandn(band(adj, fr), R);
      if (!bany(grow)) break;
      R = bor(R, grow);
    }
    const Bits<NW> unreached = bandn(tgt, claimed);
    if (bany(unreached) && blowest(claimed) < bhighest(unreached)) return false;
  }
  if (L == 0 || !want_action) return true;
  // reverse BFS from the states facing `chosen` (direction a stands at chosen - d_a)
  Bits<NW> Glo, Ghi;
  {
    const int qlo = chosen + (int)s, qhi = chosen - (int)s;
    Glo = band(bbit<NW>(qlo), fr);
    Ghi = (qhi >= 0) ? band(bbit<NW>(qhi), fr) : bzero<NW>();
    Vlo = Glo;
    Vhi = Ghi;
  }
  for (int k = 1; k < L; ++k) {
    // predecessors, any direction: moved here (from p - d) or turned in place (blocked)
    const Bits<NW> P = pair_or(bor(bor(band(bshift_up(Glo, s), fr), band(Glo, blk_lo)),
                                   bor(band(bshift_dn(Ghi, s), fr), band(Ghi, blk_hi))));
    Glo = bandn(P, Vlo);
    Ghi = bandn(P, Vhi);
    Vlo = bor(Vlo, Glo);
    Vhi = bor(Vhi, Ghi);
  }
  // the smallest action whose level-1 state lies within reverse distance L-1
  const int qlo0 = p0 - (int)s, qhi0 = p0 + (int)s;
  const int qlo = btest(fr, qlo0) ? qlo0 : p0, qhi = btest(fr, qhi0) ? qhi0 : p0;
  const bool ok_lo = !(qlo == p0 && alo == d0) && btest(Vlo, qlo);
  const bool ok_hi = !(qhi == p0 && alo + 1 == d0) && btest(Vhi, qhi);
  const uint32_t blo = (uint32_t)(__ballot(ok_lo) >> psh) & 0x3u, bhi = (uint32_t)(__ballot(ok_hi) >> psh) & 0x3u;
  // actions 0, 1 (lane 0 of the pair) and 2, 3 (lane 1)
  const uint32_t acts = (blo & 1u) | ((bhi & 1u) << 1) | ((blo >> 1) << 2) | ((bhi >> 1) << 3);
  first_action = acts ? __ffs(acts) - 1 : -1;
  return true;
}

// LANES = 4: the four lanes of a quad run one query together, lane ql handling the states
// entered by action ql (its direction's visited set and blocked mask): each
// level is then one action's worth of bitset work plus two quad ORs, instead of
// four actions' worth in one lane.  Every quantity that steers control flow is
// quad-uniform.
template <int NW, int LANES>
__device__ bool bfs_closest(const Bits<NW>& occ, const Bits<NW>& tgt, const Bits<NW>& valid,
                            int H, int p0, int d0, int ql, int& first_action, int& path_len,
                            bool want_action, bool conn) {
  if (LANES == 1)
    return bfs_closest_1<NW>(occ, tgt, valid, H, p0, d0, first_action, path_len, want_action, conn);
  if (LANES == 2)
    return bfs_closest_2<NW>(occ, tgt, valid, H, p0, d0, ql, first_action, path_len, want_action, conn);
  const int dla = ql == 0 ? -1 : ql == 1 ? 1 : ql == 2 ? -H : H;   // this lane's action
  const Bits<NW> fr = bandn(valid, occ);
  Bits<NW> blk = bshift_var(occ, -dla);                               // blk[p] = occ[p + dla]
  if (ql == 2) blk = bor(blk, band_edge_lo<NW>(valid, H));            // the border columns left
  if (ql == 3) blk = bor(blk, band_edge_hi<NW>(valid, H));            // out of the band
  const Bits<NW> fa = bshift_var(tgt, -dla);                          // fa[p] = tgt[p + dla]
  const int dl0 = d0 == 0 ? -1 : d0 == 1 ? 1 : d0 == 2 ? -H : H;
  const uint32_t qsh = __lane_id() & ~3u;                             // this quad's lanes in a ballot
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
  const bool open = bany(bandn(tgt, claimed));   // some target not yet claimed (quad-uniform)
  for (int depth = 1; open && L < 0; ++depth) {
    const Bits<NW> nxt = bandn(bor(band(bshift_var(U, dla), fr), band(U, blk)), V);
    V = bor(V, nxt);
    const Bits<NW> nU = quad_or(nxt);
    if (!bany(nU)) break;                  // every reachable state visited
    uint32_t face = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) face |= nxt.w[i] & fa.w[i];
    if ((uint32_t)(__ballot(face != 0) >> qsh) & 0xfu) {   // some lane of the quad faces a target
      const Bits<NW> hit = bandn(quad_or(band(bshift_var(nxt, dla), tgt)), claimed);
      if (bany(hit)) {
        claimed = bor(claimed, hit);
        L = depth;
        chosen = blowest(hit);
        break;                             // L and the chosen target are known
      }
    }
    U = nU;
  }
  if (L < 0) return true;                  // no target at all, or none reachable: None
  path_len = L;
  if (bany(bandn(tgt, claimed)) && conn && btest(fr, p0)) {
    // The free cells are one component (the scenario's are, and cells are only ever cleared
    // next to the agent): every free cell is reachable, so a target is reachable iff it has
    // a free neighbour -- no flood fill.
    claimed = bor(claimed, band(quad_or(bshift_var(fr, dla)), tgt));
    const Bits<NW> unreached = bandn(tgt, claimed);
    if (bany(unreached) && blowest(claimed) < bhighest(unreached)) return false;
  } else if (bany(bandn(tgt, claimed))) {
    // Which of the other targets are reachable at all (base.py:31 raises on an unreachable
    // target after a reachable one): a target is faced from any reachable position next
    // to it (a blocked move turns in place), so flood the free cells from the positions
    // visited so far until every target is claimed or nothing new is reached.
    Bits<NW> R = bor(quad_or(V), bbit<NW>(p0));
    for (;;) {
      const Bits<NW> adj = quad_or(bshift_var(R, dla));          // cells next to R
      claimed = bor(claimed, band(adj, tgt));
      if (!bany(bandn(tgt, claimed))) break;
      const Bits<NW> grow = bandn(band(adj, fr), R);
      if (!bany(grow)) break;
      R = bor(R, grow);
    }
    const Bits<NW> unreached = bandn(tgt, claimed);
    if (bany(unreached) && blowest(claimed) < bhighest(unreached)) return false;
  }
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

// Lane s of the quad's value, in every lane of the quad (DPP quad_perm [s,s,s,s]).
__device__ __forceinline__ uint32_t quad_bcast(uint32_t x, int s) {
  switch (s) {
    case 0: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x00, 0xF, 0xF, false);
    case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x55, 0xF, 0xF, false);
    case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xAA, 0xF, 0xF, false);
    default: return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xFF, 0xF, 0xF, false);
  }
}


// Lane s of the pair's value, in both lanes of the pair (DPP quad_perm [s,s,2+s,2+s]).
__device__ __forceinline__ uint32_t pair_bcast(uint32_t x, int s) {
  return s == 0 ? (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xA0, 0xF, 0xF, false)
                : (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xF5, 0xF, 0xF, false);
}

// Occupancy and `kind` target sets of a grid row (kind ids, 4 cells per 32-bit word
// of row32, nq words) minus the cells set in m: SWAR byte tests on whole words
// (nonzero byte: ((w & 0x7f..) + 0x7f..) | w has bit 7 set; equal byte: the same on
// w ^ kind), 32 cells per result word, no per-cell work.  With LANES = 4 the quad
// splits the words (lane ql builds words ql, ql + 4, ...) and broadcasts them; LANES = 2
// likewise over a pair.
template <int NW, int LANES>
__device__ __forceinline__ void grid_bits(const uint32_t* row32, int nq, const uint32_t (&m)[8],
                                          uint32_t kind, int ql, const Bits<NW>& valid,
                                          Bits<NW>& occ, Bits<NW>& tgt) {
  constexpr int PER = (NW + LANES - 1) / LANES;   // result words per lane
  const uint32_t k4 = kind * 0x01010101u;
  uint32_t po[PER], pt[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int w = ql + j * LANES;
    uint32_t o = 0u, t = 0u;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int q = 8 * w + k;
      const uint32_t d = (w < NW && q < nq) ? row32[q] : 0u;
      const uint32_t nz = nonzero_bytes(d);
      const uint32_t eq = zero_bytes(d ^ k4);
      o |= byte_tops(nz) << (4 * k);
      t |= byte_tops(eq) << (4 * k);
    }
    uint32_t clr = 0u;
#pragma unroll
    for (int i = 0; i < NW; ++i) clr = (i == w) ? m[i] : clr;
    po[j] = o & ~clr;
    pt[j] = t & ~clr;
  }
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const uint32_t oi = LANES == 1 ? po[i / LANES]
                      : LANES == 2 ? pair_bcast(po[i / LANES], i % LANES) : quad_bcast(po[i / LANES], i % LANES);
    const uint32_t ti = LANES == 1 ? pt[i / LANES]
                      : LANES == 2 ? pair_bcast(pt[i / LANES], i % LANES) : quad_bcast(pt[i / LANES], i % LANES);
    occ.w[i] = oi & valid.w[i];
    tgt.w[i] = ti & oi & valid.w[i];
  }
}

// grid_bits over the whole grid (C cells), then the band of columns 1 .. W-2 (bits H ..
// C-H-1 moved down by H): NW band words from at most NW + 1 grid words.
template <int NW, int LANES>
__device__ __forceinline__ void band_bits(const uint32_t* row32, int nq, int C, int H, const uint32_t (&m)[8],
                                          uint32_t kind, int ql, Bits<NW>& occ, Bits<NW>& tgt) {
  constexpr int NF = NW + 1 < 8 ? NW + 1 : 8;
  Bits<NF> of, tf;
  grid_bits<NF, LANES>(row32, nq, m, kind, ql, brange<NF>(0, C), of, tf);
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    const uint32_t o1 = i + 1 < NF ? of.w[i + 1] : 0u, t1 = i + 1 < NF ? tf.w[i + 1] : 0u;
    occ.w[i] = __builtin_amdgcn_alignbit(o1, of.w[i], (uint32_t)H);
    tgt.w[i] = __builtin_amdgcn_alignbit(t1, tf.w[i], (uint32_t)H);
  }
  const Bits<NW> vb = brange<NW>(0, C - 2 * H);
  occ = band(occ, vb);
  tgt = band(tgt, vb);
}

// ---- the teacher table: find_closest_resources answered ahead of time on pristine grids ----------
// Every env of a scenario starts from the same pool row, and until it clears a cell (grab,
// bridge, axe) its grid IS that row, so the BFS result depends only on (row, target kind, dir,
// cell).  teach_table_kernel (craft_teacher.hip) evaluates bfs_closest for every such key when
// rows are loaded; a query on an env whose cleared-cell mask is empty reads its answer instead
// of running the BFS (the same function, evaluated earlier: bit-identical by construction).
// Entry: bit 15 set = computed; bit 14 = ok (false: the reference raises, base.py:31);
// bits 10-12 = first action + 1; bits 0-9 = path length + 1 (-1: no target).
__device__ __forceinline__ int tt_slot_of(const SimView& v, int kind) {
  if (kind < 0 || kind >= 32) return -1;
  // (a select, not v.tt_slot[kind >> 4]: a per-lane index into the kernel argument would be a
  // vector load, and its vmcnt(0) would wait for every load the wave has in flight)
  const uint64_t w = (kind >> 4) ? v.tt_slot[1] : v.tt_slot[0];
  const int s = (int)((w >> (4 * (kind & 15))) & 0xfu);
  return s == 0xf ? -1 : s;
}
__device__ __forceinline__ uint16_t tt_encode(bool ok, int fa, int len) {
  return (uint16_t)(0x8000u | (ok ? 0x4000u : 0u) | ((uint32_t)(fa + 1) << 10) | (uint32_t)(len + 1));
}
// The table block of table row trow = pool row * tt_nsub + subset (null when there is no table).
__device__ __forceinline__ const uint16_t* tt_row(const SimView& v, int trow) {
  return v.ttab ? v.ttab + (size_t)trow * v.tt_slots * 4 * v.C : nullptr;
}
// The same row as 4-bit labels (SimView::ttab4), or null.
__device__ __forceinline__ const uint8_t* tt_row4(const SimView& v, int trow) {
  return v.ttab4 ? v.ttab4 + (size_t)trow * v.tt_slots * v.tt_blk : nullptr;
}
// The table row of an env of pool row `scen` that has cleared `ncl` cells this episode, cleared(c)
// telling which: scen * tt_nsub + the subset of the row's listed clearable cells it cleared (w0,
// w1 = tt_cells[scen]), or -1 when it cleared a cell the table does not list (or there is no
// table).  Every grid an env can reach is its pool row minus some of the row's clearable cells
// (grab, bridge and axe only ever clear a cell, craft.py:383-410).
template <class Cleared>
__device__ __forceinline__ int tt_index(const SimView& v, int scen, uint32_t w0, uint32_t w1, int ncl,
                                        Cleared cleared) {
  if (!v.ttab) return -1;
  // (cleared() of every slot unconditionally, an unused slot asking cell 0: reads of the grid are
  // then issued together instead of one round trip each)
  int sub = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const uint32_t c = ((j < 4 ? w0 : w1) >> (8 * (j & 3))) & 0xffu;
    const bool cl = cleared((int)(c != 0xffu ? c : 0u));
    sub |= (c != 0xffu && cl) ? 1 << j : 0;
  }
  return __popc((uint32_t)sub) == ncl ? scen * v.tt_nsub + sub : -1;
}
// tt_index over a cleared-cell mask m (8 words, 256 cells).
__device__ __forceinline__ int tt_index_mask(const SimView& v, int scen, uint32_t w0, uint32_t w1,
                                             const uint32_t (&m)[8]) {
  int ncl = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) ncl += __popc(m[i]);
  return tt_index(v, scen, w0, w1, ncl, [&](int c) {
    uint32_t w = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) w = (i == (c >> 5)) ? m[i] : w;
    return ((w >> (c & 31)) & 1u) != 0;
  });
}

// DemonstrationTeacher.__call__ (teachers/demonstration.py:9-30) for one env, LANES
// lanes of a quad-aligned group (lane ql of the group).  Its current grid is row32
// (kind ids, x-major, as 32-bit words; NW*8 words at most) minus the cells set in m
// (cleared this episode; all zero when the row is already current), its inventory
// iv, its agent s, the task `task`; conn: the scenario's free cells are one component
// (pool_conn); task_tab / task_sub are the handle's task tables
// (v.task_tab / v.task_sub, or copies in LDS).  Returns the action, or -2 where the reference
// raises (err_out = CRAFT_ETEACHER).  With want_len, len_out receives
// len(find_closest_resources(task.arg)) (-1: no target, -2: the reference raises).  ttab: the
// teacher-table block of the env's scenario when its grid is pristine (no cell cleared), else
// null: a target kind with a table slot is then read off the table instead of searched.
// The action for a go[X] leaf from find_closest_resources' answer (demonstration.py:23-30).
__device__ __forceinline__ int go_leaf_action(bool ok, int fa, int len, int& err) {
  if (!ok) err = CRAFT_ETEACHER;                    // base.py:31 len(None)
  else if (len < 0) return CRAFT_STOP;              // demonstration.py:25-26
  else if (len == 0) err = CRAFT_ETEACHER;          // [][0]
  else return fa;
  return -2;
}

// DEFER (the fused kernels; no want_len): no BFS here at all.  A go[X] leaf the table cannot
// answer returns kTeachDeferred with *defer = X, for a later dense pass (teach_deferred).
constexpr int kTeachDeferred = -3;

// The hint-tree half of DemonstrationTeacher.__call__ alone (the K-tick teacher rollout,
// craft_rollout_teach.h, resolves go[X] leaves later, from the table or a BFS job):
// find_incomplete_subtask (teachers/base.py:10-25) from `task` with satisfies() read off the
// inventory iv and the facing cell's kind.  Returns CRAFT_STOP when the task is already
// satisfied (demonstration.py:12-13), CRAFT_USE for a use leaf, kTeachGo with go_kind = X for a
// go[X] leaf, or -2 with err = CRAFT_ETEACHER where the reference raises (base.py:24's assert,
// demonstration.py:18's).  The same decisions as teach_env's walk.
constexpr int kTeachGo = -4;
__device__ __forceinline__ int hint_leaf(const uint16_t* task_tab, const int32_t* task_sub, const uint8_t* iv,
                                         int facing, int task, int& err, int& go_kind) {
  auto sat = [&](int t) -> int {       // satisfies(), craft.py:285-294
    const uint32_t tt = task_tab[t];
    const int goal = tt & 0xf, arg = (tt >> 4) & 0xff;
    if (goal == CRAFT_GOAL_GET || goal == CRAFT_GOAL_MAKE) return iv[arg] > 0;
    if (goal == CRAFT_GOAL_GO) return facing == arg;
    return -1;
  };
  err = 0;
  go_kind = -1;
  if (sat(task) == 1) return CRAFT_STOP;
  int node = task;
  for (int guard = 0; guard < CRAFT_MAX_TASKS; ++guard) {
    const int nsub = (task_tab[node] >> 12) & 0xf;
    if (nsub == 0) break;
    const int32_t* sub = task_sub + CRAFT_MAX_SUBTASKS * node;
    int chosen = sub[nsub - 1];
    bool last = true;
    for (int q = 0; q + 1 < nsub; ++q)
      if (sat(sub[q]) != 1) { chosen = sub[q]; last = false; break; }
    if (last && sat(chosen) == 1) { err = CRAFT_ETEACHER; return -2; }   // base.py:24 assert
    node = chosen;
  }
  const uint32_t lt = task_tab[node];
  const int goal = lt & 0xf;
  if (goal == CRAFT_GOAL_USE) return CRAFT_USE;
  if (goal == CRAFT_GOAL_GO) {
    go_kind = (lt >> 4) & 0xff;
    return kTeachGo;
  }
  err = CRAFT_ETEACHER;                                                  // demonstration.py:18
  return -2;
}

template <int NW, int LANES, bool DEFER = false, typename TS = int32_t>
__device__ __forceinline__ int teach_env(const SimView& v, const uint16_t* task_tab, const TS* task_sub,
                                         const uint32_t* row32, const uint32_t (&m)[8],
                                         const uint8_t* iv, const Agent& s, int task, int ql,
                                         bool want_len, int& len_out, int& err_out, bool conn,
                                         const uint16_t* ttab = nullptr, int* defer = nullptr,
                                         const uint8_t* t4 = nullptr) {
  const int H = v.H, C = v.C;
  auto kind_at = [&](int c) -> int {
    const uint32_t w = row32[c >> 2];
    const bool cleared = (m[c >> 5] >> (c & 31)) & 1u;
    return cleared ? 0 : (int)((w >> (8 * (c & 3))) & 0xffu);
  };
  const int facing = kind_at((s.x + dir_dx(s.dir)) * H + (s.y + dir_dy(s.dir)));

  auto sat = [&](int t) -> int {       // satisfies(), craft.py:285-294
    const uint32_t tt = task_tab[t];
    const int goal = tt & 0xf, arg = (tt >> 4) & 0xff;
    if (goal == CRAFT_GOAL_GET || goal == CRAFT_GOAL_MAKE) return iv[arg] > 0;
    if (goal == CRAFT_GOAL_GO) return facing == arg;
    return -1;
  };

  const Bits<NW> valid = brange<NW>(0, C - 2 * H);      // the band of columns 1 .. W-2
  const int nq = (C + 3) >> 2;
  auto closest = [&](int kind, int& fa, int& len, bool want_action) -> bool {
    const int slot = ttab ? tt_slot_of(v, kind) : -1;
    if (slot >= 0) {                                      // group-uniform: one load per lane
      const uint32_t e = ttab[(slot * 4 + s.dir) * C + s.x * H + s.y];
      if (e & 0x8000u) {
        fa = want_action ? (int)((e >> 10) & 7u) - 1 : -1;
        len = (int)(e & 0x3ffu) - 1;
        return (e & 0x4000u) != 0;
      }
    }
    Bits<NW> occ, tgt;
    band_bits<NW, LANES>(row32, nq, C, H, m, (uint32_t)kind, ql, occ, tgt);
#ifdef CRAFT_ABL_NOBFS
    fa = (int)(occ.w[0] ^ tgt.w[NW - 1]) & 3;             // ablation build only: no BFS
    len = 1;
    return true;
#endif
    return bfs_closest<NW, LANES>(occ, tgt, valid, H, s.x * H + s.y - H, s.dir, ql, fa, len, want_action, conn);
  };
  int leaf_kind = -1, leaf_fa = -1, leaf_len = -1;
  bool leaf_ok = true;

  int action = CRAFT_STOP;
  int err = 0;
  // find_incomplete_subtask, teachers/base.py:10-25
  int node = task;
  if (sat(node) != 1) {
    for (int guard = 0; guard < CRAFT_MAX_TASKS; ++guard) {
      const int nsub = (task_tab[node] >> 12) & 0xf;
      if (nsub == 0) break;
      const TS* sub = task_sub + CRAFT_MAX_SUBTASKS * node;
      int chosen = sub[nsub - 1];
      bool last = true;
      for (int q = 0; q + 1 < nsub; ++q)
        if (sat(sub[q]) != 1) { chosen = sub[q]; last = false; break; }
      if (last && sat(chosen) == 1) { err = CRAFT_ETEACHER; break; }   // base.py:24 assert
      node = chosen;
    }
    if (!err) {
      const uint32_t lt = task_tab[node];
      const int goal = lt & 0xf, arg = (lt >> 4) & 0xff;
      if (goal == CRAFT_GOAL_USE) {
        action = CRAFT_USE;
      } else if (goal == CRAFT_GOAL_GO) {
        if constexpr (DEFER) {
          const int slot = ttab ? tt_slot_of(v, arg) : -1;
          if (t4 && slot >= 0) {                                         // the label, 4 bits (ttab4)
            const int idx = s.dir * C + s.x * H + s.y;
            const uint32_t code = (t4[slot * v.tt_blk + (idx >> 1)] >> (4 * (idx & 1))) & 0xfu;
            if (code == 15u) {
              *defer = arg;                                              // not in the table: a BFS later
              err_out = 0;
              return kTeachDeferred;
            }
            if (code < 4u) action = (int)code;
            else if (code == 4u) action = CRAFT_STOP;
            else err = CRAFT_ETEACHER;                                   // the reference raises
          } else {
          const uint32_t e = slot >= 0 ? ttab[(slot * 4 + s.dir) * C + s.x * H + s.y] : 0u;
          if (!(e & 0x8000u)) {
            *defer = arg;                                                // a BFS, done densely later
            err_out = 0;
            return kTeachDeferred;
          }
          action = go_leaf_action((e & 0x4000u) != 0, (int)((e >> 10) & 7u) - 1, (int)(e & 0x3ffu) - 1, err);
          }
        } else {
          int fa = -1, len = -1;
          leaf_ok = closest(arg, fa, len, true);
          leaf_kind = arg; leaf_fa = fa; leaf_len = len;
          action = go_leaf_action(leaf_ok, fa, len, err);
        }
      } else {
        err = CRAFT_ETEACHER;                                            // demonstration.py:18
      }
    }
  }
  if (err) action = -2;                // where the reference raises
  err_out = err;
  if (!DEFER && want_len) {
    const int arg = (task_tab[task] >> 4) & 0xff;
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


// The deferred BFS queries of a workgroup, densely: work[k] = env index | target kind << 8 for
// k < n, answered by the workgroup's teacher lane groups in order (group g takes k = g; every env
// defers at most one query and there is one group per env, so n <= G), so a wave spends its BFS
// instructions on envs that need one instead of on the few of its own.  grid / agent / info as the fused kernels keep them in LDS (info: task |
// frozen << 8 | connected << 9); label: the label row of the workgroup's first env; ws / is: the
// word strides of work and info (1: arrays; the one-tile kernel keeps them in row padding).
template <int NW, int LANES>
__device__ __forceinline__ void teach_deferred(const SimView& v, const uint32_t* work, int n, int g, int G, int ql,
                                               const uint8_t* s_grid, int GS, const uint32_t* s_agent,
                                               const uint32_t* s_info, int32_t* label, int64_t env0, int ws = 1,
                                               int is = 1) {
  const int H = v.H, C = v.C, nq = (C + 3) >> 2;
  const Bits<NW> valid = brange<NW>(0, C - 2 * H);
  const uint32_t m0[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (g < n) {
    const uint32_t wk = work[g * ws];
    const int e = wk & 0xff, kind = (wk >> 8) & 0xff;
    const uint32_t ag = s_agent[e], ti = s_info[e * is];
    const int x = ag & 0xff, y = (ag >> 8) & 0xff, dir = (ag >> 16) & 3;
    Bits<NW> occ, tgt;
    band_bits<NW, LANES>(reinterpret_cast<const uint32_t*>(s_grid + e * GS), nq, C, H, m0, (uint32_t)kind, ql,
                         occ, tgt);
    int fa = -1, len = -1, err = 0;
    const bool ok = bfs_closest<NW, LANES>(occ, tgt, valid, H, x * H + y - H, dir, ql, fa, len, true,
                                           ((ti >> 9) & 1u) != 0);
    const int action = go_leaf_action(ok, fa, len, err);
    if (ql == 0) {
      if (err) latch_error(v.err, err, env0 + e);
      label[e] = action;
    }
  }
}

// The dense pass over NT teacher threads (thread u of them) with the widest lane groups the count
// allows: quads, the BFS's shortest dependent chain, when the n queries fit one per quad, else
// the kernel's own LANES (n is workgroup-uniform, so is the branch).
template <int NW, int LANES>
__device__ __forceinline__ void teach_deferred_dense(const SimView& v, const uint32_t* work, int n, int u, int NT,
                                                     const uint8_t* s_grid, int GS, const uint32_t* s_agent,
                                                     const uint32_t* s_info, int32_t* label, int64_t env0,
                                                     int ws = 1, int is = 1) {
  if (LANES < 4 && n <= NT / 4)
    teach_deferred<NW, 4>(v, work, n, u >> 2, NT / 4, u & 3, s_grid, GS, s_agent, s_info, label, env0, ws, is);
  else
    teach_deferred<NW, LANES>(v, work, n, u / LANES, NT / LANES, u % LANES, s_grid, GS, s_agent, s_info, label, env0,
                              ws, is);
}

}  // namespace craft
