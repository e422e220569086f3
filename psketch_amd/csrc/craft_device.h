// craft_device.h — device-side data layout and helpers shared by the kernels.
//
// Per-environment state in HBM (struct-of-arrays, slot = env index on this GPU):
//   state u64[N]      x:8 | y:8 | dir:2 | frozen:1 | . | timer:8 | scenario:24 | task:8
//                     (one 8-byte load gives everything a tick needs to start)
//   init  u32[N]      x0 | y0<<8 | dir0<<16   (read only when an episode restarts)
//   inv   uint4[N][2] 32 inventory counts, u8  (CraftState.inventory)
//   mask  uint4[N][2] 256-bit set of cells cleared since the episode started
//   pool  u8[P][CS]   initial grids as kind ids, x-major, CS = roundup(W*H, 16)
// A slot's grid is pool[scenario] minus its mask: the reference only ever clears
// cells (grab, bridge, axe: craft.py:383-410), so an episode restart is a mask
// clear and no per-env grid copy exists.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <cstdint>

#include "../../include/craft.h"

namespace craft {

typedef __attribute__((address_space(1))) uint32_t gu32;      // global-memory words for
typedef __attribute__((address_space(1))) unsigned long long gu64;   // scoped atomics

constexpr int kThreads = 256;      // threads per tile workgroup
constexpr int kMaxTileEnvs = 64;   // envs per workgroup tile: 16, 32 or 64
constexpr int kMinTileEnvs = 16;
constexpr int kInvStride = 36;     // LDS bytes per inventory row (9 dwords: bank-spread)

enum Mode { MODE_TICK = 0, MODE_TRANSITION = 1, MODE_OBSERVE = 2, MODE_RESET = 3 };

struct SimView {
  const uint8_t* pool;
  const uint8_t* pool_conn;   // [P]: 1 = the free cells of pool row p form one 4-connected component
  uint64_t* state;
  uint32_t* init;
  uint4* inv;
  uint4* mask;
  const uint16_t* task_tab;   // [n_tasks]: goal | arg_kind<<4 | n_subtasks<<12
  const int32_t* task_sub;    // [n_tasks][4] subtask ids
  // the hint walk tabulated (craft_host.h hint_tables): [CRAFT_MAX_TASKS][4] descriptor words,
  // then hint_bytes leaf bytes
  const uint32_t* hint;
  int32_t hint_bytes;
  int64_t* stats_part;        // [n_tiles][4]
  int32_t* err;               // [4] {code, pad, slot lo, slot hi}
  int64_t n_envs, env_base;
  int32_t pool_count, n_tasks, n_recipes;
  int32_t W, H, K, F, C, CS, GS, maxT;
  int32_t bridge, axe;
  int32_t obs_policy;         // observation stores: 0 write-back, 1 nontemporal, 2 write-through (sc1)
  int32_t obs_fmt;            // craft_obs_format_t: 0 fp32, 1 bf16, 2 u8
  // The teacher's BFS answers (craft_teach.h teacher table) for every pool row's grid with any
  // subset of its first tt_m clearable cells cleared:
  //   ttab[((trow * tt_slots + slot) * 4 + dir) * C + cell],  trow = row * tt_nsub + subset,
  // slot = the target kind's slot (tt_slot: 4 bits per kind id, 0xf = none), subset bit j = the
  // row's clearable cell tt_cells[row] byte j cleared (0xff = no such cell); null when off
  const uint16_t* ttab;
  // the same answers as the label they give (go_leaf_action), 4 bits each, one tt_blk-byte block
  // per (trow, slot): entry dir * C + cell in the low (even) / high (odd) nibble of byte >> 1;
  // 0-3 the first action, 4 STOP (no target), 5 the reference raises, 15 not computed
  const uint8_t* ttab4;
  int32_t tt_blk;             // bytes per block: 2 C rounded up to 16
  const uint32_t* tt_cells;   // [P][2]: each row's first tt_m clearable cells, a byte each
  int32_t tt_slots;
  int32_t tt_nsub;            // 1 << tt_m
  int32_t tt_fused;           // 1: the fused tick + teacher kernels read the table too (set per
                              // launch by craft_step_teach from craft_sim_tune_teach's table mode;
                              // 0: they defer every go[X] BFS instead)
  uint64_t tt_slot[2];
  uint64_t kc_lo, kc_hi;      // kind class, 4 bits per kind id
  // compact recipes, 3 words each: out | ws<<8 | n_in<<16 | kind0<<24, count0 | kind1<<8 |
  // count1<<16 | kind2<<24, count2 | kind3<<8 | count3<<16 | yield<<24.  Kernels copy the table to LDS.
  // (As kernel-argument words they cost ~50 scalar registers, which spilled.)
  const uint32_t* rcw;
  // the same recipes grouped by workshop, compact: [CRAFT_MAX_KINDS][4] uint2, slot j < kWsSlots
  // of kind k = the j-th recipe made at workshop k in dict order, {out | ws << 8 | in0 << 16 |
  // in1 << 24, count0 | count1 << 8 | yield << 16} (an absent ingredient: kind 0, count 0), all
  // zero past the last; null when a workshop has more than kWsSlots recipes or a recipe more
  // than two ingredients (recipes.yaml: three per workshop, one or two ingredients)
  const uint2* wsr;
  uint64_t* stamps;           // diagnostic builds only (CRAFT_STAMPS); null otherwise
};

// Dynamic-LDS carve of a tile workgroup (16-byte aligned pieces, Guideline 17):
// grid rows [tile][GS] (the rollout kernel adds the scenario's pristine rows
// [tile][GS]) | observation bytes [tile * F] (contiguous rows; the rollout
// kernel double-buffers them, each buffer 16-byte aligned) |
// inventory rows [tile][36] | task table [64] u16 | recipe words [16][3] |
// agent words [tile] u32.
#ifdef CRAFT_STAMPS
// Diagnostic build only (never the product): thread 0 of every workgroup
// records s_memrealtime (100 MHz) at phase boundaries into v.stamps[block][8].
#define STAMP(k)                                                                         \
  do {                                                                                   \
    if (threadIdx.x == 0 && v.stamps)                                                    \
      v.stamps[8 * (int64_t)blockIdx.x + (k)] = __builtin_amdgcn_s_memrealtime();        \
  } while (0)
#define STAMP_END()                                                                      \
  do {                                                                                   \
    __syncthreads();                                                                     \
    if (threadIdx.x == 0 && v.stamps) {                                                  \
      v.stamps[8 * (int64_t)blockIdx.x + 6] = __builtin_amdgcn_s_memrealtime();          \
      uint32_t xcc;                                                                      \
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));                 \
      v.stamps[8 * (int64_t)blockIdx.x + 7] = xcc;                                       \
    }                                                                                    \
  } while (0)
// The latest time any wave reaches a point (lane 0 of each wave, a vector atomic max).
#define STAMP_MAX(k)                                                                     \
  do {                                                                                   \
    if ((threadIdx.x & 63) == 0 && v.stamps)                                             \
      atomicMax(reinterpret_cast<unsigned long long*>(v.stamps + 8 * (int64_t)blockIdx.x + (k)), \
                (unsigned long long)__builtin_amdgcn_s_memrealtime());                   \
  } while (0)
#else
#define STAMP(k) do {} while (0)
#define STAMP_END() do {} while (0)
#define STAMP_MAX(k) do {} while (0)
#endif

// The launchers' caches are per device (a process may drive several) and thread-safe (atomics).
constexpr int kCacheDevices = 64;

// Raises a kernel's dynamic-LDS limit past the default 64 KiB (gfx950 allows 160 KiB per
// workgroup) once per kernel, device and size, not per launch: a host runtime call per launch
// costs every tick of a trainer's loop, and a launch captured into a HIP graph is replayed without
// this code.
template <auto KERNEL>
inline hipError_t ensure_lds(size_t lds) {
  static std::atomic<size_t> granted[kCacheDevices];                 // 0: the default 64 KiB
  if (lds <= 65536) return hipSuccess;
  if (lds > 163840) return hipErrorInvalidValue;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  const bool cached = dev >= 0 && dev < kCacheDevices;
  if (cached && lds <= granted[dev].load(std::memory_order_relaxed)) return hipSuccess;
  e = hipFuncSetAttribute(reinterpret_cast<const void*>(KERNEL), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e == hipSuccess && cached) {
    size_t cur = granted[dev].load(std::memory_order_relaxed);
    while (cur < lds && !granted[dev].compare_exchange_weak(cur, lds, std::memory_order_relaxed)) {
    }
  }
  return e;
}

// Workgroups of KERNEL (`threads` threads, `lds` dynamic LDS bytes) the current device holds at
// once: occupancy per CU x CUs, cached per device and LDS size (a persistent launch's grid).
template <auto KERNEL>
inline int resident_workgroups(int threads, size_t lds) {
  static std::atomic<uint64_t> cache[kCacheDevices];                 // lds << 32 | workgroups
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  const bool cached = dev >= 0 && dev < kCacheDevices;
  if (cached) {
    const uint64_t c = cache[dev].load(std::memory_order_relaxed);
    if ((uint32_t)c != 0 && (c >> 32) == (uint64_t)lds) return (int)(uint32_t)c;
  }
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, KERNEL, threads, lds) != hipSuccess || per_cu < 1) per_cu = 1;
  if (dev < 0 || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
    cus = 256;
  const int r = per_cu * cus;
  if (cached) cache[dev].store(((uint64_t)lds << 32) | (uint32_t)r, std::memory_order_relaxed);
  return r;
}

// envs per tile of the teacher-labelled K-tick rollout (craft_rollout_teach.h rt_tile): 32 for
// 3x3 windows, 16 for wider ones
__host__ __device__ constexpr int rt_tile_of(int win) { return win == 3 ? 32 : 16; }

// 32-bit words per cell set of the teacher's BFS (craft_teach.h: the band of grid columns
// 1 .. W-2, the border columns left out); the kernels' NW template argument.
__host__ __device__ inline int teach_words(int W, int H) { return ((W - 2) * H + 31) / 32; }

struct LdsLayout {
  int obs, inv, task, rc, agent, ctrl, bytes;
};
__host__ __device__ inline LdsLayout lds_layout(int tile, int GS, int F, int obs_bufs = 1,
                                                 bool pristine = false) {
  auto up16 = [](int x) { return (x + 15) & ~15; };
  LdsLayout l;
  l.obs = up16(tile * GS * (pristine ? 2 : 1));
  l.inv = up16(l.obs + obs_bufs * up16(tile * F));
  l.task = up16(l.inv + tile * kInvStride);
  l.rc = up16(l.task + CRAFT_MAX_TASKS * 2);
  l.agent = up16(l.rc + CRAFT_MAX_RECIPES * 12);
  l.ctrl = up16(l.agent + tile * 4);         // workgroup-uniform control words (rollout queue)
  l.bytes = l.ctrl + 16;
  return l;
}

struct TileArgs {
  const int32_t* src;
  const int32_t* dst;
  const int32_t* actions;
  const int32_t* tasks;
  const int32_t* r_scen;   // MODE_RESET inputs
  const int32_t* r_x;
  const int32_t* r_y;
  const int32_t* r_dir;
  const int32_t* r_task;
  uint64_t seed;
  int64_t tick;
  int64_t n;
  uint32_t flags;
  void* obs;
  float* reward;
  uint8_t* done;
  int8_t* sat;
  const int32_t* ref;      // MODE_TICK rollout fusion (craft_step_ex)
  const uint8_t* bc;
  int32_t* rec;
  int32_t* any_live;
  int8_t* code;            // transition codes (craft_step_ex, craft_transition)
  int32_t* label;          // craft_step_teach: teacher label of every env's new state
};

struct RolloutArgs {       // craft_rollout: n_ticks ticks in one launch
  const int32_t* actions;  // [n_ticks][n_envs] or null (hashed draw)
  uint64_t seed;
  int64_t tick0;
  int32_t n_ticks;
  int32_t ring;            // outputs of tick t go to ring slot t % ring
  uint32_t flags;
  void* obs;               // [ring][n_envs][F] in the obs format, or null
  float* reward;           // [ring][n_envs] each, or null
  uint8_t* done;
  int8_t* sat;
  int32_t chunk;           // ticks per work unit
  unsigned long long* queue;   // work-unit counter: unit = the value fetched - qbase
  unsigned long long qbase;    // the counter's value at the launch (kept by the host)
  // split kernel, per-unit path: workgroup b takes unit b without a claim, later units come
  // from queue[1] (its value at the launch: qbase1); a launch adds max(units, grid) to it
  unsigned long long qbase1;
  int64_t* grid_out;       // host side only: the launch reports its grid size here
  uint32_t* tile_done;     // per tile: chunks completed in this launch, zeroed before the launch
  int32_t flat;            // split kernel, one unit per tile: one continuous pipeline (no queue)
  // craft_rollout_teach (craft_rollout_teach.h)
  const int32_t* label_in; // [n_envs] the teacher's label of each slot's state before tick0
  const uint8_t* bc;       // [n_envs] behaviour cloning: the slot acts on its label, or null
  int32_t label_actions;   // 1: every slot acts on its label (make_data.get_reference_actions)
  int32_t lsync;           // labels feed some slot's actions (label_actions or bc): 1 row sync, 2 C looks up
  int32_t use_table;       // the teacher reads the teacher table for pristine grids
  int32_t* labels;         // [ring][n_envs] the label of every slot's new state, or null
  int32_t* rec;            // [ring][n_envs] the action taken (-1: none), or null
};

struct ScenarioArgs {      // craft_pool_generate
  uint64_t seed;
  int64_t id0;             // global id of scenario 0 of this launch
  int32_t count;
  int32_t first;           // pool row of scenario 0
  int32_t boundary;
  int32_t n_prim, n_per, n_ws;
  int32_t prim[8];
  int32_t ws[8];
  int32_t* init_out;       // [count][2] or null
};

struct Agent {
  int x, y, dir, frozen, timer, scen, task;
};

__device__ __forceinline__ Agent unpack_state(uint64_t s) {
  Agent a;
  const uint32_t lo = (uint32_t)s, hi = (uint32_t)(s >> 32);
  a.x = lo & 0xff;
  a.y = (lo >> 8) & 0xff;
  a.dir = (lo >> 16) & 3;
  a.frozen = (lo >> 18) & 1;
  a.timer = lo >> 24;
  a.scen = hi & 0xffffff;
  a.task = hi >> 24;
  return a;
}

__device__ __forceinline__ uint64_t pack_state(const Agent& a) {
  const uint32_t lo = (uint32_t)a.x | ((uint32_t)a.y << 8) | ((uint32_t)a.dir << 16) |
                      ((uint32_t)a.frozen << 18) | ((uint32_t)a.timer << 24);
  const uint32_t hi = ((uint32_t)a.scen & 0xffffff) | ((uint32_t)a.task << 24);
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

__device__ __forceinline__ void latch_error(int32_t* err, int code, int64_t slot) {
  if (atomicCAS(err, 0, code) == 0) {
    err[2] = (int32_t)(slot & 0xffffffff);
    err[3] = (int32_t)(slot >> 32);
  }
}

// SWAR byte tests on a 32-bit word of 4 kind-id cells: bit 7 of each byte set where that
// byte is nonzero / zero ((b & 0x7f) + 0x7f carries into bit 7 for any nonzero low bits).
__device__ __forceinline__ uint32_t nonzero_bytes(uint32_t w) {
  return (((w & 0x7f7f7f7fu) + 0x7f7f7f7fu) | w) & 0x80808080u;
}
__device__ __forceinline__ uint32_t zero_bytes(uint32_t w) { return ~nonzero_bytes(w) & 0x80808080u; }
// The top bits of the 4 bytes of m (bits 7, 15, 23, 31) as a nibble.
__device__ __forceinline__ uint32_t byte_tops(uint32_t m) {
  return ((m >> 7) | (m >> 14) | (m >> 21) | (m >> 28)) & 0xfu;
}

__device__ __forceinline__ int kind_class(const SimView& v, int k) {
  return (int)(((k < 16) ? (v.kc_lo >> (4 * k)) : (v.kc_hi >> (4 * (k - 16)))) & 0xf);
}

__device__ __forceinline__ int dir_dx(int d) { return d == CRAFT_LEFT ? -1 : (d == CRAFT_RIGHT ? 1 : 0); }
__device__ __forceinline__ int dir_dy(int d) { return d == CRAFT_DOWN ? -1 : (d == CRAFT_UP ? 1 : 0); }

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Sets bit c of a register-resident 8-word mask (static indices only).
__device__ __forceinline__ void mask_set(uint32_t (&m)[8], int c) {
  const int w = c >> 5;
  const uint32_t b = 1u << (c & 31);
#pragma unroll
  for (int i = 0; i < 8; ++i) m[i] |= (i == w) ? b : 0u;
}

// CraftState.step (craft.py:332-424) on an LDS grid row `g` and inventory
// bytes `iv`; `rc` is the recipe table (LDS copy of v.rcw).  Records whether inventory / mask changed.
// What PrimitiveLanguageTeacher.describe reads off a (state, next state) pair
// (teachers/primitive_language.py:61-85): 0..3 = moved by the coord_change of
// DOWN / UP / LEFT / RIGHT, 4 = did not move and the inventory changed, 5 = neither.
__device__ __forceinline__ int transition_code(int ox, int oy, const Agent& s, bool inv_changed) {
  const int dx = s.x - ox, dy = s.y - oy;
  if (dx == 0 && dy == 0) return inv_changed ? 4 : 5;
  return dy < 0 ? CRAFT_DOWN : dy > 0 ? CRAFT_UP : dx < 0 ? CRAFT_LEFT : CRAFT_RIGHT;
}

// Recipe slots per workshop kind in SimView::wsr (recipes.yaml: 3 per workshop).
constexpr int kWsSlots = 3;

// RCV: the recipe words also sit in a VGPR, lane w holding word w (w < 3 * CRAFT_MAX_RECIPES,
// loaded while every lane of the wave was active); the recipe loop reads them with v_readlane
// instead of one LDS round trip per recipe.
// WSR: `wsr` is SimView::wsr copied to LDS (non-null): a lane at a workshop runs only that
// workshop's recipes, in two LDS round trips whatever the recipe count (the slots' words, then
// every slot's output and ingredient counts), the updates applied in registers in the
// reference's order (an applied recipe's new counts forwarded to the later slots that name the
// same kinds) and written once; instead of every recipe of every workshop some lane of the wave
// faces, one or two round trips each.
// NB: `nbw` holds the kinds of the agent's four neighbour cells (byte d: the cell one step in
// direction d, DOWN UP LEFT RIGHT), read before the tick: the facing cell and a move's target
// without a grid read.
template <bool RCV = false, bool WSR = false, bool NB = false>
__device__ __forceinline__ void transition(const SimView& v, const uint32_t* rc, uint8_t* g, uint8_t* iv, Agent& s,
                                           uint32_t (&m)[8], int a, bool& inv_changed,
                                           bool& mask_changed, uint32_t rcv = 0u, int64_t slot = -1,
                                           const uint2* wsr = nullptr, uint32_t nbw = 0u) {
  auto rword = [&](int w) -> uint32_t {
    if constexpr (RCV) return __builtin_amdgcn_readlane(rcv, w);
    else return __builtin_amdgcn_readfirstlane(rc[w]);
  };
  const int H = v.H;
  int dx = 0, dy = 0, ndir = s.dir;
  if (a < CRAFT_USE) {                               // moves always turn (craft.py:341-352)
    dx = dir_dx(a);
    dy = dir_dy(a);
    ndir = a;
  } else if (a == CRAFT_USE) {                       // craft.py:356-412
    const int d = s.dir;
    const bool ok = (d == CRAFT_LEFT && s.x > 0) || (d == CRAFT_DOWN && s.y > 0) ||
                    (d == CRAFT_RIGHT && s.x < v.W - 1) || (d == CRAFT_UP && s.y < H - 1);
    if (ok) {
      const int c = (s.x + dir_dx(d)) * H + (s.y + dir_dy(d));
      const int thing = NB ? (int)((nbw >> (8 * d)) & 0xffu) : g[c];
      if (thing != 0) {
        const int cls = kind_class(v, thing);
        if (cls == CRAFT_KIND_GRABBABLE) {           // craft.py:383-386
          if (iv[thing] == 255) latch_error(v.err, CRAFT_ERANGE, slot);   // u8 count would wrap
          else iv[thing] = (uint8_t)(iv[thing] + 1);
          g[c] = 0;
          mask_set(m, c);
          inv_changed = mask_changed = true;
        } else if (WSR && cls == CRAFT_KIND_WORKSHOP) {   // recipes in dict order, craft.py:388-401
          uint2 w[kWsSlots];
#pragma unroll
          for (int j = 0; j < kWsSlots; ++j) w[j] = wsr[thing * 4 + j];
          int h[kWsSlots][3];                                    // counts of out, in0, in1 (kind 0: absent)
#pragma unroll
          for (int j = 0; j < kWsSlots; ++j) {
            h[j][0] = iv[w[j].x & 0xff];
            h[j][1] = iv[(w[j].x >> 16) & 0xff];
            h[j][2] = iv[w[j].x >> 24];
          }
#pragma unroll
          for (int j = 0; j < kWsSlots; ++j) {
            if ((int)((w[j].x >> 8) & 0xff) != thing) continue;   // (the valid slots are a prefix)
            const int out = w[j].x & 0xff, ka = (w[j].x >> 16) & 0xff, kb = w[j].x >> 24;
            const int ca = w[j].y & 0xff, cb = (w[j].y >> 8) & 0xff;
            int ho = h[j][0], ha = h[j][1], hb = h[j][2];
            if (ha < ca || hb < cb) continue;
            // n_inventory[output] += yld, then each ingredient -= its count (craft.py:396-399), on
            // register copies; copies of one kind are kept equal after every update
            const int made = ho + (int)((w[j].y >> 16) & 0xff);
            if (made > 255) latch_error(v.err, CRAFT_ERANGE, slot);   // u8 count would wrap: saturate
            ho = made > 255 ? 255 : made;
            ha = ka == out ? ho : ha;
            hb = kb == out ? ho : hb;
            ha = (ha - ca) & 0xff;
            ho = out == ka ? ha : ho;
            hb = kb == ka ? ha : hb;
            hb = (hb - cb) & 0xff;
            ho = out == kb ? hb : ho;
            ha = ka == kb ? hb : ha;
            iv[out] = (uint8_t)ho;
            iv[ka] = (uint8_t)ha;                                // (kind 0 absent: its own unchanged 0)
            iv[kb] = (uint8_t)hb;
            inv_changed = true;
#pragma unroll
            for (int j2 = j + 1; j2 < kWsSlots; ++j2)            // forward the new counts
#pragma unroll
              for (int q = 0; q < 3; ++q) {
                const int kq = q == 0 ? (int)(w[j2].x & 0xff) : q == 1 ? (int)((w[j2].x >> 16) & 0xff) : (int)(w[j2].x >> 24);
                h[j2][q] = kq == out ? ho : kq == ka ? ha : kq == kb ? hb : h[j2][q];
              }
          }
        } else if (cls == CRAFT_KIND_WORKSHOP) {     // recipes in dict order, craft.py:388-401
          // Recipe words are wave-uniform (LDS broadcast reads or v_readlane, kept in scalar
          // registers); a recipe's ingredient counts are read together, so a matching recipe
          // costs one or two LDS round trips.  Recipes chain (a product may be the next one's ingredient): each reads
          // the inventory after the previous one's writes (LDS is in order).
          for (int r = 0; r < v.n_recipes; ++r) {
            const uint32_t a0 = rword(3 * r);
            if ((int)((a0 >> 8) & 0xff) != thing) continue;     // the recipe's workshop
            const uint32_t a1 = rword(3 * r + 1);
            const uint32_t a2 = rword(3 * r + 2);
            const int n_in = (a0 >> 16) & 0xff;
            const int k0 = a0 >> 24, k1 = (a1 >> 8) & 0xff, k2 = a1 >> 24, k3 = (a2 >> 8) & 0xff;
            const int c0 = a1 & 0xff, c1 = (a1 >> 16) & 0xff, c2 = a2 & 0xff, c3 = (a2 >> 16) & 0xff;
            const int h0 = iv[k0], h1 = iv[k1], h2 = iv[k2], h3 = iv[k3];   // unused slots read kind 0
            const bool have = (n_in < 1 || h0 >= c0) && (n_in < 2 || h1 >= c1) &&
                              (n_in < 3 || h2 >= c2) && (n_in < 4 || h3 >= c3);
            if (!have) continue;
            const int out = a0 & 0xff;
            const int made = iv[out] + (int)(a2 >> 24);      // `_yield` (craft.py:394), 1..255
            if (made > 255) latch_error(v.err, CRAFT_ERANGE, slot);   // u8 count would wrap: saturate
            iv[out] = (uint8_t)(made > 255 ? 255 : made);
            if (n_in > 0) iv[k0] = (uint8_t)(iv[k0] - c0);
            if (n_in > 1) iv[k1] = (uint8_t)(iv[k1] - c1);
            if (n_in > 2) iv[k2] = (uint8_t)(iv[k2] - c2);
            if (n_in > 3) iv[k3] = (uint8_t)(iv[k3] - c3);
            inv_changed = true;
          }
        } else if (cls == CRAFT_KIND_WATER) {        // craft.py:403-406
          if (iv[v.bridge] > 0) {
            g[c] = 0;
            mask_set(m, c);
            iv[v.bridge] = (uint8_t)(iv[v.bridge] - 1);
            inv_changed = mask_changed = true;
          }
        } else if (cls == CRAFT_KIND_STONE) {        // craft.py:408-410 (axe kept)
          if (iv[v.axe] > 0) {
            g[c] = 0;
            mask_set(m, c);
            mask_changed = true;
          }
        }
      }
    }
  }
  // Collision against the pre-action grid (craft.py:418-421); USE/STOP do not move.
  if (dx | dy) {
    const int nx = s.x + dx, ny = s.y + dy;
    if ((NB ? (nbw >> (8 * a)) & 0xffu : g[nx * H + ny]) == 0) { s.x = nx; s.y = ny; }
  }
  s.dir = ndir;
}

// CraftState.satisfies (craft.py:285-294): 1/0, -1 for None.  `tt` is the
// task-table entry goal | arg<<4.
__device__ __forceinline__ int satisfies(const SimView& v, const uint8_t* g, const uint8_t* iv,
                                         const Agent& s, uint32_t tt) {
  const int goal = tt & 0xf, arg = (tt >> 4) & 0xff;
  if (goal == CRAFT_GOAL_GET || goal == CRAFT_GOAL_MAKE) return iv[arg] > 0;
  if (goal == CRAFT_GOAL_GO) return g[(s.x + dir_dx(s.dir)) * v.H + (s.y + dir_dy(s.dir))] == arg;
  return -1;
}

}  // namespace craft
