// craft_sim.hip — host side of the C ABI (include/craft.h): handle lifetime,
// scenario pool, launches, state I/O and episode statistics.
// Kernels: craft_tile.hip (tick / transition / observe / reset), craft_rollout.hip
// (multi-tick), craft_teacher.hip, craft_scenarios.hip (pool generation).
#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "craft_device.h"
#include "craft_host.h"

namespace craft {
hipError_t launch_tile(int mode, int win, int tile, const SimView& v, const TileArgs& a, size_t lds,
                       hipStream_t st);
hipError_t launch_teacher(int nw, int lanes, const SimView& v, const int32_t* slots, const int32_t* tasks,
                          int64_t n, int32_t* act_out, int32_t* len_out, hipStream_t st);
hipError_t launch_rollout_teach(int win, int nw, const SimView& v, const RolloutArgs& a, hipStream_t st);
hipError_t launch_distances(int nw, const SimView& v, const int32_t* tasks, const int8_t* success,
                            const int32_t* seqs, int32_t ticks, int64_t n, int32_t* dist_out,
                            uint8_t* is_get_out, int32_t* n_actions_out, int32_t* flags, hipStream_t st);
hipError_t launch_rollout(int win, int tile, int threads, const SimView& v, const RolloutArgs& a, size_t lds,
                          hipStream_t st);
hipError_t launch_scenarios(const SimView& v, const ScenarioArgs& a, hipStream_t st);
hipError_t launch_tick_teach(int tl, int nw, int win, int tile, const SimView& v, const TileArgs& a, size_t lds,
                             hipStream_t st);
hipError_t launch_tick2(int tl, int nw, const SimView& v, const TileArgs& a, size_t lds, hipStream_t st);
size_t tick2_lds_bytes(int tl, int nw, int GS, int F);
hipError_t launch_teach_table(int nw, const SimView& v, int32_t first, int32_t count, const int32_t* kinds,
                              hipStream_t st);

namespace {

__global__ void get_state_kernel(SimView v, const int32_t* slots, int64_t n, int32_t* agent_out,
                                 int32_t* inv_out, uint8_t* grid_out, int32_t* spec_out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t slot = slots ? (int64_t)slots[i] : i;
  if (slot < 0 || slot >= v.n_envs) { latch_error(v.err, CRAFT_ERANGE, i); return; }
  const Agent s = unpack_state(v.state[slot]);
  if (agent_out) {
    agent_out[4 * i + 0] = s.x;
    agent_out[4 * i + 1] = s.y;
    agent_out[4 * i + 2] = s.dir;
    agent_out[4 * i + 3] = s.timer;
  }
  if (inv_out) {
    const uint8_t* iv = reinterpret_cast<const uint8_t*>(v.inv + 2 * slot);
    for (int k = 0; k < v.K; ++k) inv_out[i * v.K + k] = iv[k];
  }
  if (grid_out) {
    const uint32_t* m = reinterpret_cast<const uint32_t*>(v.mask + 2 * slot);
    const bool ok = s.scen < v.pool_count;
    if ((v.C & 3) == 0) {               // whole dwords: 4 cells per load and per store
      const uint32_t* row = reinterpret_cast<const uint32_t*>(v.pool + (size_t)s.scen * v.CS);
      uint32_t* out = reinterpret_cast<uint32_t*>(grid_out + i * v.C);
      for (int q = 0; q < (v.C >> 2); ++q) {
        uint32_t w = ok ? row[q] : 0u;
        const uint32_t cleared = (m[q >> 3] >> ((q & 7) * 4)) & 0xfu;   // cells 4q..4q+3
        for (int b = 0; b < 4; ++b)
          if ((cleared >> b) & 1u) w &= ~(0xffu << (8 * b));
        out[q] = w;
      }
    } else {
      for (int c = 0; c < v.C; ++c) {
        const int k = ok ? v.pool[(size_t)s.scen * v.CS + c] : 0;
        grid_out[i * v.C + c] = ((m[c >> 5] >> (c & 31)) & 1u) ? 0 : (uint8_t)k;
      }
    }
  }
  if (spec_out) {
    const uint32_t in = v.init[slot];
    spec_out[5 * i + 0] = s.scen;
    spec_out[5 * i + 1] = in & 0xff;
    spec_out[5 * i + 2] = (in >> 8) & 0xff;
    spec_out[5 * i + 3] = (in >> 16) & 3;
    spec_out[5 * i + 4] = s.task;
  }
}

__global__ void set_state_kernel(SimView v, const int32_t* slots, int64_t n, const int32_t* spec_in,
                                 const int32_t* agent_in, const int32_t* inv_in) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t slot = slots ? (int64_t)slots[i] : i;
  if (slot < 0 || slot >= v.n_envs) { latch_error(v.err, CRAFT_ERANGE, i); return; }
  const int sc = spec_in[5 * i], x0 = spec_in[5 * i + 1], y0 = spec_in[5 * i + 2],
            d0 = spec_in[5 * i + 3], tk = spec_in[5 * i + 4];
  const int x = agent_in[4 * i], y = agent_in[4 * i + 1], d = agent_in[4 * i + 2],
            tm = agent_in[4 * i + 3];
  bool ok = sc >= 0 && sc < v.pool_count && tk >= 0 && tk < v.n_tasks && x0 >= 1 &&
            x0 <= v.W - 2 && y0 >= 1 && y0 <= v.H - 2 && d0 >= 0 && d0 < 4 && x >= 1 &&
            x <= v.W - 2 && y >= 1 && y <= v.H - 2 && d >= 0 && d < 4 && tm >= 0 && tm <= 255;
  uint32_t ivw[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int k = 0; k < v.K; ++k) {
    const int c = inv_in ? inv_in[i * v.K + k] : 0;
    if (c < 0 || c > 255) ok = false;
    ivw[k >> 2] |= (uint32_t)(c & 0xff) << (8 * (k & 3));
  }
  if (!ok) { latch_error(v.err, CRAFT_EINVAL, i); return; }
  Agent s;
  s.x = x; s.y = y; s.dir = d; s.frozen = 0; s.timer = tm; s.scen = sc; s.task = tk;
  v.state[slot] = pack_state(s);
  v.init[slot] = (uint32_t)x0 | ((uint32_t)y0 << 8) | ((uint32_t)d0 << 16);
  v.inv[2 * slot] = make_uint4(ivw[0], ivw[1], ivw[2], ivw[3]);
  v.inv[2 * slot + 1] = make_uint4(ivw[4], ivw[5], ivw[6], ivw[7]);
  v.mask[2 * slot] = make_uint4(0, 0, 0, 0);
  v.mask[2 * slot + 1] = make_uint4(0, 0, 0, 0);
}

__global__ void stats_kernel(int64_t* part, int64_t n_rows, int64_t* out, int reset) {
  __shared__ long long acc[3][256];
  long long s0 = 0, s1 = 0, s2 = 0;
  for (int64_t r = threadIdx.x; r < n_rows; r += blockDim.x) {
    s0 += part[4 * r]; s1 += part[4 * r + 1]; s2 += part[4 * r + 2];
    if (reset) { part[4 * r] = 0; part[4 * r + 1] = 0; part[4 * r + 2] = 0; }
  }
  acc[0][threadIdx.x] = s0; acc[1][threadIdx.x] = s1; acc[2][threadIdx.x] = s2;
  __syncthreads();
  for (int w = blockDim.x / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w)
      for (int j = 0; j < 3; ++j) acc[j][threadIdx.x] += acc[j][threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) { out[0] = acc[0][0]; out[1] = acc[1][0]; out[2] = acc[2][0]; }
}

}  // namespace
}  // namespace craft

using craft::SimView;
using craft::TileArgs;

struct craft_sim {
  int device = 0;
  craft_config_t cfg{};
  int64_t n_envs = 0, env_base = 0, n_tiles = 0;
  int32_t pool_capacity = 0, pool_count = 0;
  uint8_t* d_pool = nullptr;
  uint8_t* d_pool_conn = nullptr;   // per pool row: free cells 4-connected (teacher shortcut)
  uint32_t* d_rcw = nullptr;
  uint2* d_wsr = nullptr;           // SimView::wsr: the recipes grouped by workshop, or null
  uint64_t* d_state = nullptr;
  uint32_t* d_init = nullptr;
  uint4* d_inv = nullptr;
  uint4* d_mask = nullptr;
  uint16_t* d_task = nullptr;
  int32_t* d_task_sub = nullptr;
  uint32_t* d_hint = nullptr;       // hint_tables: descriptors + leaf bytes
  int64_t* d_stats = nullptr;
  int32_t* d_err = nullptr;
  uint16_t* d_ttab = nullptr;       // the teacher table (craft_teach.h), or null
  uint8_t* d_ttab4 = nullptr;       // its answers as 4-bit labels (SimView::ttab4)
  uint32_t* d_ttcells = nullptr;    // [pool_capacity][2]: each row's listed clearable cells
  int tt_nslot = 0;                 // target-kind slots of the table
  bool tt_decided = false;          // its size is fixed at the first pool load (ensure_table)
  // pool rows loaded since the table was last built: craft_pool_load only records them, and the
  // next launch that reads the table builds their entries first, on its own stream
  std::vector<std::pair<int32_t, int32_t>> tt_dirty;
  // craft_sim_tune_teach: which teacher reads the table (0 auto: craft_step_teach when the launch
  // rewrites the previous launch's observation buffer, as a trainer's loop does, every other
  // teacher always; 1 always; 2 never), and teacher lanes per query (0 = each kernel's default)
  int teach_table = 0;
  bool hint_walk = false;           // some task keeps the hint walk (no hint table: craft_host.h)
  int teach_lanes = 0;
  int32_t tt_kinds[16] = {};        // its slots' target kinds
  SimView view{};
  int tile = craft::kMaxTileEnvs;   // envs per tile workgroup
  int tile_knob = 0;                // craft_sim_tune's tile_envs (0 = each kernel's default)
  int resident_cap = 0;             // 0: no cap on tile workgroups per CU
  int rollout_chunk = 0;            // craft_rollout ticks per work unit (0: the whole launch)
  int rollout_threads = 0;          // craft_rollout threads per tile workgroup (0: 8 per env)
  uint8_t* d_sync = nullptr;        // craft_rollout: work-unit counter + per-tile chunk flags
  uint8_t* d_sync_graph = nullptr;  // the same for launches captured into a HIP graph
  size_t sync_bytes = 0;
  bool sync_zeroed = false;         // d_sync zeroed once; then the counter only grows
  int rollout_obs_policy = 2;       // craft_rollout's observation stores until craft_sim_tune sets one:
                                    // write-through, 1.5 % faster than write-back (tools/ab_store.sh)
  bool obs_store_tuned = false;     // craft_sim_tune chose the store policy for every kernel
  int teach_kernel = 0;             // craft_sim_tune_teach: 0 auto, 1 one-tile, 2 two-tile
  uint64_t queue1_next = 0;         // queue[1] (the split kernel's per-unit path) at the next launch
  uint64_t queue_next = 0;          // the counter's value at the next launch (every launch adds
                                    // its units + its grid: one fetch past the end per workgroup)
  std::string last_error;
};

namespace {

int fail(craft_sim* sim, int code, const std::string& msg) {
  if (sim) sim->last_error = msg;
  return code;
}

int hip_fail(craft_sim* sim, hipError_t e, const char* what) {
  return fail(sim, CRAFT_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(sim, expr)                                   \
  do {                                                       \
    hipError_t _e = (expr);                                  \
    if (_e != hipSuccess) return hip_fail((sim), _e, #expr); \
  } while (0)

using craft_host::validate_config;

// The tile kernel's default envs per workgroup (craft_sim_create, craft_sim_tune(0, ...)).
int default_tile(int win) {
  // 3x3: 64-env tiles; 5x5: 32 (35 KB of rows); 7x7: 32 (67 KB), 3 % faster than 16 at 16x16
  return win == 3 ? 64 : 32;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// LDS bytes per tile workgroup; a residency cap R pads the request to 160 KiB / R
// so that at most R tile workgroups share a CU and later tiles' prologues overlap
// earlier tiles' observation stores.
size_t lds_bytes(const craft_sim* s, int tile, int obs_bufs = 1, bool pristine = false) {
  const SimView& v = s->view;
  size_t b = (size_t)craft::lds_layout(tile, v.GS, v.F, obs_bufs, pristine).bytes;
  if (s->resident_cap > 0) {
    const size_t capped = ((size_t)163840 / s->resident_cap) & ~size_t(15);
    if (capped > b) b = capped;
  }
  return b;
}

// The tile kernel's (craft_tile.h).
size_t tile_lds_bytes(const craft_sim* s, int tile) {
  const SimView& v = s->view;
  size_t b = (size_t)craft::lds_layout(tile, v.GS, v.F).bytes;
  if (s->resident_cap > 0) {
    const size_t capped = ((size_t)163840 / s->resident_cap) & ~size_t(15);
    if (capped > b) b = capped;
  }
  return b;
}

// The workgroup shape craft_rollout launches with (craft_sim_rollout_shape).  Default
// (threads 0): for 3x3 windows the split-producer kernel on 32-env tiles with 6
// streaming waves (7-15 % faster than 64-env tiles at 65536 envs);
// otherwise the handle's tile with 256 threads (512 for 64-env tiles).
void rollout_shape(const craft_sim* s, int* tile, int* threads, int* split) {
  // the rollout kernels stage u8 rows (double-buffered): their default tile keeps ~40 KB per buffer
  const int win = s->cfg.window_width;
  int t = s->tile_knob ? s->tile_knob : (win == 3 ? 64 : (win == 5 ? 32 : 16)), nt = s->rollout_threads;
  if (nt == 0 && s->cfg.window_width == 3) {
    t = 32;
    nt = 512;
  }
  // what launch_rollout_win (craft_rollout.h) instantiates for (t, nt): 64-env tiles run 256
  // or 512 threads, smaller tiles 128, the split kernel at 320 / 384 / 512, else 256
  if (t == 64) nt = (nt == 256) ? 256 : 512;
  else if (nt != 128 && nt != 320 && nt != 384 && nt != 512) nt = 256;
  *tile = t;
  *threads = nt;
  *split = (t <= 32 && nt >= 320) ? 1 : 0;
}

// The one-tile teacher kernel's envs per tile: 64 for 3x3 windows; the handle's tile (default 32)
// for wider ones, whose 64-env observation rows (69 KB at 5x5) leave one workgroup per CU.
int teach_tile(const craft_sim* s) {
  return s->cfg.window_width == 3 || s->tile != 32 ? craft::kMaxTileEnvs : 32;
}

// What craft_step / craft_step_ex (teach = false) or craft_step_teach (teach = true) launches:
// CRAFT_KERNEL_TILE (craft_tile.h) or CRAFT_KERNEL_TICK2 (craft_tick2.h), with its envs per
// tile / workgroup and teacher lanes per env.
void step_shape(const craft_sim* s, bool teach, int* kernel, int* envs, int* lanes) {
  if (!teach) {
    *kernel = CRAFT_KERNEL_TILE;
    *envs = s->tile;
    *lanes = 0;
    return;
  }
  const bool w3 = s->cfg.window_width == 3;
  int k = s->teach_kernel;
  // auto: the two-tile kernel for 3x3 windows at the default tile from 32768 envs, where its
  // 128-env workgroups fill the chip, else the one-tile kernel
  if (k == 0) k = (w3 && s->tile == craft::kMaxTileEnvs && s->resident_cap == 0 && s->n_envs >= 32768) ? 2 : 1;
  if (k == 2 && !(w3 && s->tile == craft::kMaxTileEnvs && s->resident_cap == 0)) k = 1;
  // teacher lanes per env (craft_sim_tune_teach): the two-tile kernel runs pairs (or quads), the
  // one-tile kernel quads (or pairs, or one lane)
  const int tl2 = s->teach_lanes == 4 ? 4 : 2;
  // (the 32-env tile of wider windows: pairs by default, 76.5 against 78.5 us with quads at 5x5)
  const int tl1 = (s->teach_lanes == 1 || s->teach_lanes == 2) ? s->teach_lanes
                  : s->teach_lanes == 0 && teach_tile(s) == 32 ? 2 : 4;
  if (k == 2) { *kernel = 2; *envs = 128; *lanes = tl2; }
  else { *kernel = 1; *envs = teach_tile(s); *lanes = tl1; }
}

// Builds the teacher-table entries (and listed clearable cells) of the rows loaded since the last
// build, ahead of the launch (`what`) about to read them: on that launch's stream, then a host
// wait, so that a reader on any other stream finds the rows finished too (one wait per batch of
// pool loads, not per launch).  Refused while the stream is being captured into a HIP graph: the
// build would be captured with the launch (rebuilt on every replay, or never run if the capture
// is dropped), so the caller runs one eager launch (or craft_sim_sync_table) first.  Until built,
// a row's entries read as "not computed" (ensure_table's fill), which latches CRAFT_EINVARIANT
// instead of a wrong label.
int flush_table(craft_sim* s, void* stream, const char* what) {
  if (s->tt_dirty.empty()) return CRAFT_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (s->d_ttab) {
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    HIP_TRY(s, hipStreamIsCapturing(st, &cap));
    if (cap != hipStreamCaptureStatusNone)
      return fail(s, CRAFT_EINVAL, std::string(what) +
                                       ": pool rows loaded since the last eager teacher launch have no teacher-table "
                                       "entries yet; run craft_sim_sync_table (or one eager launch) before capturing");
    for (const auto& r : s->tt_dirty) {
      const hipError_t e = craft::launch_teach_table(craft::teach_words(s->view.W, s->view.H), s->view, r.first,
                                                     r.second, s->tt_kinds, st);
      if (e != hipSuccess) return hip_fail(s, e, "teacher table build");
    }
    HIP_TRY(s, hipStreamSynchronize(st));
  }
  s->tt_dirty.clear();
  return CRAFT_OK;
}

// The view a teacher launch gets: the table hidden when craft_sim_tune_teach says never.
SimView teach_view(const craft_sim* s) {
  SimView v = s->view;
  if (s->teach_table == 2) {
    v.ttab = nullptr;
    v.ttab4 = nullptr;
    v.tt_slots = 0;
  }
  return v;
}

int launch(craft_sim* s, int mode, const TileArgs& a, void* stream, const char* what) {
  hipError_t e = craft::launch_tile(mode, s->cfg.window_width, s->tile, s->view, a, tile_lds_bytes(s, s->tile),
                                    reinterpret_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(s, e, what);
  return CRAFT_OK;
}

// The cells of a grid that grab, bridge or axe can clear (craft.py:383-410): non-empty cells of a
// grabbable, water or stone kind.
int clearable_cells(const craft_config_t& cfg, const uint8_t* g, int C) {
  int m = 0;
  for (int c = 0; c < C; ++c) {
    const int k = g[c], cls = k < CRAFT_MAX_KINDS ? cfg.kind_class[k] : CRAFT_KIND_INERT;
    m += k != 0 && (cls == CRAFT_KIND_GRABBABLE || cls == CRAFT_KIND_WATER || cls == CRAFT_KIND_STONE);
  }
  return m;
}

// The teacher table's size, fixed at the first pool load from the most clearable cells any row of
// that load has (every grid an env of a row can reach is the row minus a subset of them): tt_m =
// that many (at most 8), fewer while pool_capacity rows x 2^tt_m subsets x slots x 4 directions x C
// cells of u16 exceed 1 GiB or 2^21 table rows (the kernels pack a table row into 21 bits).  12x12
// craft_medium: 6 clearable cells per row, 6 slots: 442 KB per row, 453 MB for 1024 rows.  A row
// with more clearable cells lists its first tt_m; an env that clears another one has no table row
// and its queries run the BFS.  Without room for even the pristine grids (tt_m 0) the table is off.
void ensure_table(craft_sim* s, int max_clearable) {
  if (s->tt_decided) return;
  s->tt_decided = true;
  const int C = s->view.C;
  if (s->tt_nslot == 0) return;
  const size_t budget = (size_t)1 << 30;
  int m = std::min(8, std::max(0, max_clearable));
  const size_t blk = ((size_t)2 * C + 15) & ~(size_t)15;      // SimView::tt_blk
  auto bytes = [&](int mm) { return ((size_t)s->pool_capacity << mm) * s->tt_nslot * 4 * C * sizeof(uint16_t); };
  auto bytes4 = [&](int mm) { return ((size_t)s->pool_capacity << mm) * s->tt_nslot * blk; };
  while (m >= 0 && (bytes(m) + bytes4(m) > budget || ((int64_t)s->pool_capacity << m) >= ((int64_t)1 << 21))) --m;
  if (m < 0) return;
  if (hipMalloc(&s->d_ttab, bytes(m)) != hipSuccess || hipMalloc(&s->d_ttab4, bytes4(m)) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipFree(s->d_ttab);
    s->d_ttab = nullptr;                  // no table: every query runs the BFS (same results)
    s->d_ttab4 = nullptr;
    return;
  }
  // every entry "not computed" until its row is built (flush_table): u16 0 and nibble 15 latch
  // CRAFT_EINVARIANT in every reader instead of decoding as a label
  if (hipMemset(s->d_ttab, 0, bytes(m)) != hipSuccess || hipMemset(s->d_ttab4, 0xff, bytes4(m)) != hipSuccess) {
    (void)hipGetLastError();
    (void)hipFree(s->d_ttab);
    (void)hipFree(s->d_ttab4);
    s->d_ttab = nullptr;
    s->d_ttab4 = nullptr;
    return;
  }
  s->view.ttab4 = s->d_ttab4;
  s->view.tt_blk = (int32_t)blk;
  s->view.ttab = s->d_ttab;
  s->view.tt_slots = s->tt_nslot;
  s->view.tt_nsub = 1 << m;
}

}  // namespace

extern "C" {

const char* craft_strerror(int status) { return craft_host::status_text(status); }

int craft_host_flag_pointer(void* host, int32_t** device_out) {
  if (!host || !device_out) return CRAFT_EINVAL;
  *device_out = nullptr;
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, host, 0) != hipSuccess || !d) {
    (void)hipGetLastError();
    return CRAFT_EINVAL;                    // not page-locked host memory HIP knows
  }
  *device_out = static_cast<int32_t*>(d);
  return CRAFT_OK;
}

int craft_sim_create(const craft_config_t* cfg, int device, int64_t n_envs, int64_t env_id_base,
                     int32_t pool_capacity, craft_sim_t** out) {
  if (!cfg || !out || n_envs <= 0 || pool_capacity <= 0 || pool_capacity > (1 << 24) || env_id_base < 0)
    return CRAFT_EINVAL;
  *out = nullptr;
  std::string msg;
  int rc = validate_config(cfg, msg);
  if (rc) {
    fprintf(stderr, "craft_sim_create: %s\n", msg.c_str());
    return rc;
  }
  craft_sim* s = new craft_sim();
  s->device = device;
  s->cfg = *cfg;
  s->n_envs = n_envs;
  s->env_base = env_id_base;
  s->pool_capacity = pool_capacity;
  // stats rows: one per 16-env tile, plus the step kernel's last workgroup's tick waves (its
  // wave count is rounded up to the workgroup's 4)
  s->n_tiles = (n_envs + craft::kMinTileEnvs - 1) / craft::kMinTileEnvs + 4;
  s->tile = default_tile(cfg->window_width);
  const int W = cfg->width, H = cfg->height, K = cfg->n_kinds, F = cfg->n_features;
  const int C = W * H, CS = (C + 15) & ~15;
  const int GS = CS + 4;                  // odd dword stride: lane-private rows hit distinct banks
  uint32_t rcw[CRAFT_MAX_RECIPES * 3] = {};          // SimView::rcw packing (craft_device.h)
  for (int r = 0; r < cfg->n_recipes; ++r) {
    const craft_recipe_t& rc = cfg->recipe[r];
    uint8_t b[12] = {};
    b[0] = (uint8_t)rc.output;
    b[1] = (uint8_t)rc.workshop;
    b[2] = (uint8_t)rc.n_inputs;
    for (int i = 0; i < rc.n_inputs; ++i) {
      b[3 + 2 * i] = (uint8_t)rc.input_kind[i];
      b[4 + 2 * i] = (uint8_t)rc.input_count[i];
    }
    b[11] = (uint8_t)rc.yield;                       // 1..255 (validated)
    for (int q = 0; q < 3; ++q)
      rcw[3 * r + q] = (uint32_t)b[4 * q] | ((uint32_t)b[4 * q + 1] << 8) | ((uint32_t)b[4 * q + 2] << 16) |
                       ((uint32_t)b[4 * q + 3] << 24);
  }
  // SimView::wsr: workshop k's recipes in dict order, compact, kWsSlots slots per kind (the
  // fourth of each kind's 4 stays zero)
  std::vector<uint2> wsr((size_t)CRAFT_MAX_KINDS * 4, make_uint2(0, 0));
  bool wsr_ok = true;
  {
    int used[CRAFT_MAX_KINDS] = {};
    for (int r = 0; r < cfg->n_recipes; ++r) {
      const craft_recipe_t& rc = cfg->recipe[r];
      const int k = rc.workshop;
      if (k <= 0 || k >= CRAFT_MAX_KINDS || used[k] >= craft::kWsSlots || rc.n_inputs > 2) {
        wsr_ok = false;
        continue;
      }
      const uint32_t k0 = rc.n_inputs > 0 ? (uint32_t)rc.input_kind[0] : 0u, c0 = rc.n_inputs > 0 ? (uint32_t)rc.input_count[0] : 0u;
      const uint32_t k1 = rc.n_inputs > 1 ? (uint32_t)rc.input_kind[1] : 0u, c1 = rc.n_inputs > 1 ? (uint32_t)rc.input_count[1] : 0u;
      wsr[(size_t)k * 4 + used[k]++] = make_uint2((uint32_t)rc.output | ((uint32_t)k << 8) | (k0 << 16) | (k1 << 24),
                                                  c0 | (c1 << 8) | ((uint32_t)rc.yield << 16));
    }
  }
  std::vector<uint16_t> task_tab(CRAFT_MAX_TASKS, 0);
  std::vector<int32_t> task_sub(CRAFT_MAX_TASKS * CRAFT_MAX_SUBTASKS, 0);
  craft_host::task_tables(*cfg, task_tab.data(), task_sub.data());
  std::vector<uint32_t> hint(CRAFT_MAX_TASKS * 4, 0);
  std::vector<uint8_t> hint_leaf;
  craft_host::hint_tables(*cfg, task_tab.data(), task_sub.data(), hint.data(), hint_leaf);
  const size_t hint_bytes = hint.size() * 4 + ((hint_leaf.size() + 15) & ~size_t(15));
  hint.resize(hint_bytes / 4, 0u);
  if (!hint_leaf.empty()) memcpy(hint.data() + CRAFT_MAX_TASKS * 4, hint_leaf.data(), hint_leaf.size());
  auto cleanup = [&](hipError_t e, const char* what) {
    fprintf(stderr, "craft_sim_create: %s: %s\n", what, hipGetErrorString(e));
    craft_sim_destroy(s);
    return CRAFT_EHIP;
  };
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return cleanup(e, "hipSetDevice");
#define ALLOC(ptr, bytes)                                                          \
  do {                                                                             \
    if ((e = hipMalloc(&(ptr), (bytes))) != hipSuccess) return cleanup(e, #ptr);   \
    if ((e = hipMemset((ptr), 0, (bytes))) != hipSuccess) return cleanup(e, #ptr); \
  } while (0)
  ALLOC(s->d_pool, (size_t)pool_capacity * CS);
  ALLOC(s->d_pool_conn, (size_t)pool_capacity + 16);
  ALLOC(s->d_state, sizeof(uint64_t) * n_envs);
  ALLOC(s->d_init, sizeof(uint32_t) * n_envs);
  ALLOC(s->d_inv, 2 * sizeof(uint4) * n_envs);
  ALLOC(s->d_mask, 2 * sizeof(uint4) * n_envs);
  ALLOC(s->d_task, sizeof(uint16_t) * task_tab.size());
  ALLOC(s->d_rcw, sizeof(rcw));
  if (wsr_ok) ALLOC(s->d_wsr, sizeof(uint2) * wsr.size());
  ALLOC(s->d_task_sub, sizeof(int32_t) * task_sub.size());
  ALLOC(s->d_hint, hint_bytes);
  ALLOC(s->d_stats, 4 * sizeof(int64_t) * s->n_tiles);
  ALLOC(s->d_err, 4 * sizeof(int32_t));
  s->sync_bytes = (16 + 4 * (size_t)((n_envs + 15) / 16) + 15) & ~size_t(15);   // queue + tile_done
  ALLOC(s->d_sync, s->sync_bytes);
  ALLOC(s->d_sync_graph, s->sync_bytes);      // craft_rollout launches captured into a graph
  // The teacher table: one slot per kind some go[] or get[] task targets (teach_env's BFS kinds
  // and the rollout summary's); its size is fixed at the first pool load (ensure_table).
  // craft_sim_tune_teach(.., table 2) stops every teacher reading it (the parity switch).
  ALLOC(s->d_ttcells, (size_t)pool_capacity * 2 * sizeof(uint32_t));
  {
    int nslot = 0;
    uint64_t smap[2] = {~0ull, ~0ull};
    for (int t = 0; t < cfg->n_tasks; ++t) {
      const craft_task_t& tk = cfg->task[t];
      const int k = tk.arg_kind;
      if ((tk.goal != CRAFT_GOAL_GO && tk.goal != CRAFT_GOAL_GET) || k <= 0 || k >= 32) continue;
      if (((smap[k >> 4] >> (4 * (k & 15))) & 0xfull) != 0xfull) continue;      // has a slot
      if (nslot >= 15) continue;                                                    // no room: BFS
      smap[k >> 4] &= ~(0xfull << (4 * (k & 15)));
      smap[k >> 4] |= (uint64_t)nslot << (4 * (k & 15));
      s->tt_kinds[nslot++] = k;
    }
    s->tt_nslot = nslot;
    s->view.tt_slot[0] = smap[0];
    s->view.tt_slot[1] = smap[1];
  }
#undef ALLOC
  if ((e = hipMemcpy(s->d_task, task_tab.data(), sizeof(uint16_t) * task_tab.size(), hipMemcpyHostToDevice)) != hipSuccess)
    return cleanup(e, "task table");
  if ((e = hipMemcpy(s->d_rcw, rcw, sizeof(rcw), hipMemcpyHostToDevice)) != hipSuccess)
    return cleanup(e, "recipe table");
  if (s->d_wsr && (e = hipMemcpy(s->d_wsr, wsr.data(), sizeof(uint2) * wsr.size(), hipMemcpyHostToDevice)) != hipSuccess)
    return cleanup(e, "workshop recipe table");
  if ((e = hipMemcpy(s->d_task_sub, task_sub.data(), sizeof(int32_t) * task_sub.size(), hipMemcpyHostToDevice)) != hipSuccess)
    return cleanup(e, "subtask table");
  if ((e = hipMemcpy(s->d_hint, hint.data(), hint_bytes, hipMemcpyHostToDevice)) != hipSuccess)
    return cleanup(e, "hint table");

  SimView& v = s->view;
  v.pool = s->d_pool;
  v.pool_conn = s->d_pool_conn;
  v.state = s->d_state;
  v.init = s->d_init;
  v.inv = s->d_inv;
  v.mask = s->d_mask;
  v.task_tab = s->d_task;
  v.task_sub = s->d_task_sub;
  v.hint = s->d_hint;
  v.hint_bytes = (int32_t)hint_leaf.size();
  for (int t = 0; t < cfg->n_tasks; ++t) s->hint_walk |= (hint[4 * t + 2] & craft_host::kHintWalk) != 0;
  v.stats_part = s->d_stats;
  v.err = s->d_err;
  v.ttab = nullptr;                       // (until the first pool load: ensure_table)
  v.ttab4 = nullptr;
  v.tt_blk = 0;
  v.tt_cells = s->d_ttcells;
  v.tt_nsub = 1;
  v.n_envs = n_envs;
  v.env_base = env_id_base;
  v.pool_count = 0;
  v.n_tasks = cfg->n_tasks;
  v.n_recipes = cfg->n_recipes;
  v.W = W; v.H = H; v.K = K; v.F = F; v.C = C; v.CS = CS; v.GS = GS;
  v.maxT = cfg->max_timesteps;
  v.bridge = cfg->bridge_kind;
  // write-through (sc1) observation stores: with one observation buffer rewritten every tick (a
  // trainer's, do_rollout's) the tick kernel takes 20.3 us against 26.4 with nontemporal stores,
  // and 27.0 against 26.5 when every tick writes a fresh slot of a 1.7 GB ring (tools/step_probe.py)
  v.obs_policy = 2;
  v.obs_fmt = CRAFT_OBS_F32;
  v.axe = cfg->axe_kind;
  v.kc_lo = v.kc_hi = 0;
  for (int k = 0; k < CRAFT_MAX_KINDS; ++k) {
    const uint64_t cls = cfg->kind_class[k] & 0xf;
    if (k < 16) v.kc_lo |= cls << (4 * k);
    else v.kc_hi |= cls << (4 * (k - 16));
  }
  v.rcw = s->d_rcw;
  v.wsr = s->d_wsr;
  *out = s;
  return CRAFT_OK;
}

int craft_sim_tune(craft_sim_t* s, int32_t tile_envs, int32_t max_resident_per_cu, int32_t obs_store) {
  if (!s) return CRAFT_EINVAL;
  s->tile_knob = tile_envs;
  if (tile_envs == 0) tile_envs = default_tile(s->cfg.window_width);
  if (tile_envs != 16 && tile_envs != 32 && tile_envs != 64)
    return fail(s, CRAFT_EINVAL, "craft_sim_tune: tile_envs must be 16, 32 or 64");
  if (max_resident_per_cu != 0 && (max_resident_per_cu < 3 || max_resident_per_cu > 32))
    return fail(s, CRAFT_EINVAL, "craft_sim_tune: max_resident_per_cu must be 0 or 3..32");
  if (obs_store < 0 || obs_store > 2)
    return fail(s, CRAFT_EINVAL, "craft_sim_tune: obs_store must be 0 (write-back), 1 (nontemporal) or 2 (write-through)");
  s->tile = tile_envs;
  s->resident_cap = max_resident_per_cu;
  s->view.obs_policy = obs_store;
  s->rollout_obs_policy = obs_store;
  s->obs_store_tuned = true;
  return CRAFT_OK;
}

int craft_sim_tune_teach(craft_sim_t* s, int32_t kernel, int32_t lanes, int32_t table) {
  if (!s) return CRAFT_EINVAL;
  if (kernel < 0 || kernel > 2)
    return fail(s, CRAFT_EINVAL, "craft_sim_tune_teach: kernel must be 0 (auto), 1 (one-tile) or 2 (two-tile)");
  if (lanes != 0 && lanes != 1 && lanes != 2 && lanes != 4)
    return fail(s, CRAFT_EINVAL, "craft_sim_tune_teach: lanes must be 0 (default), 1, 2 or 4");
  if (table < 0 || table > 2)
    return fail(s, CRAFT_EINVAL, "craft_sim_tune_teach: table must be 0 (auto), 1 (always) or 2 (never)");
  s->teach_kernel = kernel;
  s->teach_lanes = lanes;
  s->teach_table = table;
  return CRAFT_OK;
}

int craft_abi_version(void) { return CRAFT_ABI_VERSION; }

int craft_sim_tune_host(craft_sim_t* s, int32_t threads) {
  if (!s) return CRAFT_EINVAL;
  if (threads < 0 || threads > 1024)
    return fail(s, CRAFT_EINVAL, "craft_sim_tune_host: threads must be 0 (the machine's) or 1..1024");
  return CRAFT_OK;                          // (no host workers in this library)
}

int craft_sim_sync_table(craft_sim_t* s, void* stream) {
  if (!s) return CRAFT_EINVAL;
  HIP_TRY(s, hipSetDevice(s->device));
  return flush_table(s, stream, "craft_sim_sync_table");
}

int craft_sim_step_shape(const craft_sim_t* s, int32_t teach, int32_t* kernel, int32_t* envs, int32_t* lanes) {
  if (!s) return CRAFT_EINVAL;
  int k = 0, e = 0, l = 0;
  step_shape(s, teach != 0, &k, &e, &l);
  if (kernel) *kernel = k;
  if (envs) *envs = e;
  if (lanes) *lanes = l;
  return CRAFT_OK;
}

int craft_sim_tune_rollout(craft_sim_t* s, int32_t chunk_ticks, int32_t threads) {
  if (!s) return CRAFT_EINVAL;
  if (chunk_ticks < -1 || chunk_ticks > 4096)
    return fail(s, CRAFT_EINVAL, "craft_sim_tune_rollout: chunk_ticks must be -1..4096");
  if (threads != 0 && threads != 128 && threads != 256 && threads != 320 && threads != 384 && threads != 512)
    return fail(s, CRAFT_EINVAL, "craft_sim_tune_rollout: threads must be 0, 128, 256, 320, 384 or 512");
  s->rollout_chunk = chunk_ticks;
  s->rollout_threads = threads;
  return CRAFT_OK;
}

int craft_sim_set_obs_format(craft_sim_t* s, int32_t format) {
  if (!s) return CRAFT_EINVAL;
  if (format != CRAFT_OBS_F32 && format != CRAFT_OBS_BF16 && format != CRAFT_OBS_U8)
    return fail(s, CRAFT_EINVAL, "craft_sim_set_obs_format: format must be 0 (fp32), 1 (bf16) or 2 (u8)");
  s->view.obs_fmt = format;
  return CRAFT_OK;
}

int craft_sim_destroy(craft_sim_t* s) {
  if (!s) return CRAFT_OK;
  (void)hipSetDevice(s->device);
  (void)hipFree(s->d_pool);
  (void)hipFree(s->d_pool_conn);
  (void)hipFree(s->d_state);
  (void)hipFree(s->d_init);
  (void)hipFree(s->d_inv);
  (void)hipFree(s->d_mask);
  (void)hipFree(s->d_task);
  (void)hipFree(s->d_rcw);
  (void)hipFree(s->d_wsr);
  (void)hipFree(s->d_task_sub);
  (void)hipFree(s->d_hint);
  (void)hipFree(s->d_stats);
  (void)hipFree(s->d_err);
  (void)hipFree(s->d_sync);
  (void)hipFree(s->d_sync_graph);
  (void)hipFree(s->d_ttab);
  (void)hipFree(s->d_ttab4);
  (void)hipFree(s->d_ttcells);
  delete s;
  return CRAFT_OK;
}

const char* craft_sim_last_error(const craft_sim_t* s) { return s ? s->last_error.c_str() : "null handle"; }

int craft_sim_info(const craft_sim_t* s, int64_t* n_envs, int32_t* pool_capacity, int32_t* n_features) {
  if (!s) return CRAFT_EINVAL;
  if (n_envs) *n_envs = s->n_envs;
  if (pool_capacity) *pool_capacity = s->pool_capacity;
  if (n_features) *n_features = s->cfg.n_features;
  return CRAFT_OK;
}

int craft_sim_rollout_shape(const craft_sim_t* s, int32_t* tile_envs, int32_t* threads, int32_t* split) {
  if (!s) return CRAFT_EINVAL;
  int t = 0, nt = 0, sp = 0;
  rollout_shape(s, &t, &nt, &sp);
  if (tile_envs) *tile_envs = t;
  if (threads) *threads = nt;
  if (split) *split = sp;
  return CRAFT_OK;
}

int craft_sim_tile_shape(const craft_sim_t* s, int32_t* tile_envs, int32_t* obs_store) {
  if (!s) return CRAFT_EINVAL;
  if (tile_envs) *tile_envs = s->tile;
  if (obs_store) *obs_store = s->view.obs_policy;
  return CRAFT_OK;
}

int craft_sim_check(craft_sim_t* s, int64_t* env_out, void* stream) {
  if (!s) return CRAFT_EINVAL;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  int32_t h[4] = {0, 0, 0, 0};
  HIP_TRY(s, hipMemcpyAsync(h, s->d_err, sizeof(h), hipMemcpyDeviceToHost, st));
  HIP_TRY(s, hipStreamSynchronize(st));
  if (h[0]) {
    HIP_TRY(s, hipMemsetAsync(s->d_err, 0, sizeof(h), st));
    HIP_TRY(s, hipStreamSynchronize(st));
    const int64_t slot = (int64_t)(uint32_t)h[2] | ((int64_t)h[3] << 32);
    if (env_out) *env_out = slot;
    return fail(s, h[0], std::string(craft_strerror(h[0])) + " (slot/item " + std::to_string(slot) + ")");
  }
  if (env_out) *env_out = -1;
  return CRAFT_OK;
}

int craft_sim_error_word(craft_sim_t* s, int32_t* out, void* stream) {
  if (!s || !out) return CRAFT_EINVAL;
  HIP_TRY(s, hipMemcpyAsync(out, s->d_err, 4 * sizeof(int32_t), hipMemcpyDeviceToDevice,
                            reinterpret_cast<hipStream_t>(stream)));
  return CRAFT_OK;
}

int craft_pool_load(craft_sim_t* s, const uint8_t* grids, int32_t first, int32_t count) {
  if (!s || !grids || first < 0 || count < 0) return fail(s, CRAFT_EINVAL, "craft_pool_load: bad argument");
  if ((int64_t)first + count > s->pool_capacity) return fail(s, CRAFT_ERANGE, "craft_pool_load: beyond pool capacity");
  const int C = s->cfg.width * s->cfg.height, CS = s->view.CS;
  std::vector<uint8_t> staged((size_t)count * CS, 0);
  std::vector<uint8_t> conn((size_t)count, 0);
  for (int p = 0; p < count; ++p) {
    const uint8_t* g = grids + (size_t)p * C;
    std::string msg;
    const int rc = craft_host::check_pool_grid(s->cfg, g, (int64_t)first + p, msg, &conn[p]);
    if (rc) return fail(s, rc, msg);
    std::memcpy(staged.data() + (size_t)p * CS, g, C);
  }
  HIP_TRY(s, hipSetDevice(s->device));
  if (count) {
    int maxm = 0;
    for (int p = 0; p < count; ++p) maxm = std::max(maxm, clearable_cells(s->cfg, grids + (size_t)p * C, C));
    ensure_table(s, maxm);
    HIP_TRY(s, hipMemcpy(s->d_pool + (size_t)first * CS, staged.data(), staged.size(), hipMemcpyHostToDevice));
    HIP_TRY(s, hipMemcpy(s->d_pool_conn + first, conn.data(), count, hipMemcpyHostToDevice));
    // the rows' teacher-table entries: built by the next launch that reads the table (flush_table)
    if (!s->tt_dirty.empty() && s->tt_dirty.back().first + s->tt_dirty.back().second == first)
      s->tt_dirty.back().second += count;
    else
      s->tt_dirty.emplace_back(first, count);
  }
  if (first + count > s->pool_count) s->pool_count = first + count;
  s->view.pool_count = s->pool_count;
  return CRAFT_OK;
}

int craft_pool_generate(craft_sim_t* s, uint64_t seed, int64_t scenario_id0, int32_t first, int32_t count,
                        int32_t boundary_kind, const int32_t* primitives, int32_t n_primitive_kinds,
                        int32_t n_per_primitive, const int32_t* workshop_kind, int32_t n_workshops,
                        int32_t* init_pos_out, void* stream) {
  if (!s || first < 0 || count < 0 || n_primitive_kinds < 0 || n_primitive_kinds > 8 || n_per_primitive < 0 ||
      n_workshops < 0 || n_workshops > 8 || (n_primitive_kinds && !primitives) || (n_workshops && !workshop_kind))
    return fail(s, CRAFT_EINVAL, "craft_pool_generate: bad argument");
  if ((int64_t)first + count > s->pool_capacity) return fail(s, CRAFT_ERANGE, "craft_pool_generate: beyond pool capacity");
  const int K = s->cfg.n_kinds, W = s->cfg.width, H = s->cfg.height;
  auto bad_kind = [&](int k) { return k <= 0 || k >= K; };
  if (bad_kind(boundary_kind)) return fail(s, CRAFT_EINVAL, "craft_pool_generate: bad boundary kind");
  for (int i = 0; i < n_primitive_kinds; ++i)
    if (bad_kind(primitives[i])) return fail(s, CRAFT_EINVAL, "craft_pool_generate: bad primitive kind");
  for (int i = 0; i < n_workshops; ++i)
    if (bad_kind(workshop_kind[i])) return fail(s, CRAFT_EINVAL, "craft_pool_generate: bad workshop kind");
  if ((int64_t)n_primitive_kinds * n_per_primitive + n_workshops + 1 > (int64_t)(W - 2) * (H - 2))
    return fail(s, CRAFT_EINVAL, "craft_pool_generate: more objects than interior cells");
  craft::ScenarioArgs a{};
  a.seed = seed;
  a.id0 = scenario_id0;
  a.count = count;
  a.first = first;
  a.boundary = boundary_kind;
  a.n_prim = n_primitive_kinds;
  a.n_per = n_per_primitive;
  a.n_ws = n_workshops;
  for (int i = 0; i < n_primitive_kinds; ++i) a.prim[i] = primitives[i];
  for (int i = 0; i < n_workshops; ++i) a.ws[i] = workshop_kind[i];
  a.init_out = init_pos_out;
  HIP_TRY(s, hipSetDevice(s->device));
  {
    // the generated rows' clearable cells: n_per_primitive of each clearable primitive kind, and
    // the clearable workshop kinds
    auto clearable = [&](int k) {
      const int cls = s->cfg.kind_class[k];
      return cls == CRAFT_KIND_GRABBABLE || cls == CRAFT_KIND_WATER || cls == CRAFT_KIND_STONE;
    };
    int maxm = 0;
    for (int i = 0; i < n_primitive_kinds; ++i) maxm += clearable(primitives[i]) ? n_per_primitive : 0;
    for (int i = 0; i < n_workshops; ++i) maxm += clearable(workshop_kind[i]) ? 1 : 0;
    if (count) ensure_table(s, maxm);
  }
  hipError_t e = craft::launch_scenarios(s->view, a, reinterpret_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(s, e, "craft_pool_generate launch");
  e = craft::launch_teach_table(craft::teach_words(s->view.W, s->view.H), s->view, first, count, s->tt_kinds,
                                reinterpret_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(s, e, "craft_pool_generate teacher table");
  if (first + count > s->pool_count) s->pool_count = first + count;
  s->view.pool_count = s->pool_count;
  return CRAFT_OK;
}

int craft_reset(craft_sim_t* s, const int32_t* scenario, const int32_t* pos_x, const int32_t* pos_y,
                const int32_t* dir, const int32_t* task, void* obs, void* stream) {
  if (!s || !scenario || !pos_x || !pos_y || !dir || !task) return fail(s, CRAFT_EINVAL, "craft_reset: null input");
  if (obs && !aligned16(obs)) return fail(s, CRAFT_EINVAL, "craft_reset: obs must be 16-byte aligned");
  TileArgs a{};
  a.r_scen = scenario; a.r_x = pos_x; a.r_y = pos_y; a.r_dir = dir; a.r_task = task;
  a.n = s->n_envs;
  a.obs = obs;
  int rc = launch(s, craft::MODE_RESET, a, stream, "craft_reset launch");
  if (rc) return rc;
  HIP_TRY(s, hipMemsetAsync(s->d_stats, 0, 4 * sizeof(int64_t) * s->n_tiles, reinterpret_cast<hipStream_t>(stream)));
  return CRAFT_OK;
}

int craft_step(craft_sim_t* s, const int32_t* actions, uint64_t action_seed, int64_t tick, uint32_t flags,
               void* obs, float* reward, uint8_t* done, int8_t* success, void* stream) {
  craft_step_args_t x{};
  x.actions = actions;
  x.action_seed = action_seed;
  x.tick = tick;
  x.flags = flags;
  x.obs = obs;
  x.reward = reward;
  x.done = done;
  x.success = success;
  return craft_step_ex(s, &x, stream);
}

namespace {
int step_args(craft_sim_t* s, const craft_step_args_t* x, TileArgs& a) {
  if (x->obs && !aligned16(x->obs)) return fail(s, CRAFT_EINVAL, "craft_step: obs must be 16-byte aligned");
  if (x->behavior_clone && !x->ref_actions)
    return fail(s, CRAFT_EINVAL, "craft_step_ex: behavior_clone needs ref_actions");
  a = TileArgs{};
  a.actions = x->actions;
  a.seed = x->action_seed;
  a.tick = x->tick;
  a.flags = x->flags;
  a.n = s->n_envs;
  a.obs = x->obs;
  a.reward = x->reward;
  a.done = x->done;
  a.sat = x->success;
  a.ref = x->ref_actions;
  a.bc = x->behavior_clone;
  a.rec = x->action_record;
  a.any_live = x->any_live;
  a.code = x->transition_code;
  return CRAFT_OK;
}
}  // namespace

int craft_step_teach(craft_sim_t* s, const craft_step_args_t* x, int32_t* label_out, void* stream) {
  if (!s || !x || !label_out) return CRAFT_EINVAL;
  if (4 * s->view.C > 1000)
    return fail(s, CRAFT_EINVAL, "craft_step_teach: 4*W*H > 1000 overflows the reference's BFS queue (teachers/base.py:42)");
  TileArgs a;
  const int rc = step_args(s, x, a);
  if (rc != CRAFT_OK) return rc;
  a.label = label_out;
  int kernel = 0, envs = 0, tl = 0;
  step_shape(s, true, &kernel, &envs, &tl);
  const int nw = craft::teach_words(s->view.W, s->view.H);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipError_t e;
  // Teacher-table reads in the fused kernel (its 4-bit copy since round 5): -2.5 us per tick when
  // the launch rewrites the previous launch's observation buffer (a trainer's loop, ring 1), and
  // -0.9 us (30.1 -> 29.2) when every launch writes a fresh slot of a 16-slot ring (round 6,
  // profiles/r06/teach_table_k1; round 4's u16 reads cost +0.5 us there), so auto reads it always.
  {
    const int frc = flush_table(s, stream, "craft_step_teach");
    if (frc != CRAFT_OK) return frc;
  }
  SimView v = teach_view(s);
  v.tt_fused = s->teach_table != 2;
  if (kernel == 2) {
    e = craft::launch_tick2(tl, nw, v, a, craft::tick2_lds_bytes(tl, nw, s->view.GS, s->view.F), st);
  } else {
    const int tile = teach_tile(s);
    // + task_sub as bytes (the teacher's other words live in row padding and the control words,
    // craft_tile.h): 40,888 bytes for a 32-env tile at 12x12, 5x5, so four workgroups share a CU
    const size_t lds = (size_t)craft::lds_layout(tile, s->view.GS, s->view.F).bytes +
                       (((size_t)s->view.n_tasks * CRAFT_MAX_SUBTASKS + 15) & ~size_t(15));
    e = craft::launch_tick_teach(tl, nw, s->cfg.window_width, tile, v, a, lds, st);
  }
  if (e != hipSuccess) return hip_fail(s, e, "craft_step_teach launch");
  return CRAFT_OK;
}

int craft_step_ex(craft_sim_t* s, const craft_step_args_t* x, void* stream) {
  if (!s || !x) return CRAFT_EINVAL;
  TileArgs a;
  const int rc = step_args(s, x, a);
  if (rc != CRAFT_OK) return rc;
  return launch(s, craft::MODE_TICK, a, stream, "craft_step launch");
}

int craft_rollout(craft_sim_t* s, const int32_t* actions, uint64_t action_seed, int64_t tick0,
                  int32_t n_ticks, uint32_t flags, void* obs, int32_t ring, float* reward,
                  uint8_t* done, int8_t* success, void* stream) {
  if (!s) return CRAFT_EINVAL;
  if (n_ticks < 0 || ring < 1 || tick0 < 0)
    return fail(s, CRAFT_EINVAL, "craft_rollout: need n_ticks >= 0, ring >= 1, tick0 >= 0");
  const int esz = s->view.obs_fmt == CRAFT_OBS_F32 ? 4 : (s->view.obs_fmt == CRAFT_OBS_BF16 ? 2 : 1);
  if (obs && (!aligned16(obs) || (ring > 1 && (s->n_envs * (int64_t)s->view.F * esz) % 16 != 0)))
    return fail(s, CRAFT_EINVAL, "craft_rollout: every obs ring slot must be 16-byte aligned");
  craft::RolloutArgs a{};
  a.actions = actions;
  a.seed = action_seed;
  a.tick0 = tick0;
  a.n_ticks = n_ticks;
  a.ring = ring;
  a.flags = flags;
  a.obs = obs;
  a.reward = reward;
  a.done = done;
  a.sat = success;
  a.chunk = s->rollout_chunk > 0 ? s->rollout_chunk : (n_ticks > 0 ? n_ticks : 1);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // A launch captured into a HIP graph (torch.cuda.graph) is replayed without this host code, so
  // it cannot use the eager launches' running counter: it gets its own sync area, zeroed by a
  // memset captured with it, so every replay starts from zero and never touches the eager one.
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  HIP_TRY(s, hipStreamIsCapturing(st, &cap));
  const bool captured = cap != hipStreamCaptureStatusNone;
  uint8_t* sync = captured ? s->d_sync_graph : s->d_sync;
  a.queue = reinterpret_cast<unsigned long long*>(sync);
  a.tile_done = reinterpret_cast<uint32_t*>(sync + 16);
  int tile = 0, threads = 0, split = 0;
  rollout_shape(s, &tile, &threads, &split);
  // chunk_ticks -1: the split kernel's continuous pipeline (its 3x3 default shape, observations
  // on; otherwise one unit per tile)
  const bool flat = s->rollout_chunk == -1 && split && tile == 32 && threads == 512 &&
                    s->cfg.window_width == 3 && obs != nullptr;
  a.flat = flat ? 1 : 0;
  // The work-unit counter is zeroed once and then only grows: a launch hands out units
  // counter - qbase and ends having added its units + its grid.  Chunked launches (tiles
  // handed between workgroups) also need zeroed per-tile flags: those zero the whole area.
  const int64_t n_chunks = n_ticks > 0 ? (n_ticks + a.chunk - 1) / a.chunk : 0;
  const int64_t units = ((s->n_envs + tile - 1) / tile) * n_chunks;
  if (captured) {
    if (n_ticks > 0) HIP_TRY(s, hipMemsetAsync(sync, 0, s->sync_bytes, st));
    a.qbase = 0;
    a.qbase1 = 0;
  } else {
    if (n_ticks > 0 && (n_chunks > 1 || !s->sync_zeroed)) {
      HIP_TRY(s, hipMemsetAsync(s->d_sync, 0, s->sync_bytes, st));
      s->sync_zeroed = true;
      s->queue_next = 0;
      s->queue1_next = 0;
    }
    a.qbase = s->queue_next;
    a.qbase1 = s->queue1_next;
  }
  int64_t grid = 0;
  a.grid_out = &grid;
  SimView view = s->view;
  view.obs_policy = s->rollout_obs_policy;
  hipError_t e = craft::launch_rollout(s->cfg.window_width, tile, threads, view, a, lds_bytes(s, tile, 2, true), st);
  if (e != hipSuccess) return hip_fail(s, e, "craft_rollout launch");
  // the split kernel's per-unit path counts on queue[1] (craft_rollout_split.h), the others on
  // queue[0]
  if (captured) return CRAFT_OK;
  if (grid > 0 && split && !flat) s->queue1_next += (uint64_t)std::max<int64_t>(units, grid);
  else if (grid > 0) s->queue_next += (uint64_t)(units + grid);
  return CRAFT_OK;
}

int craft_rollout_teach(craft_sim_t* s, const craft_rollout_teach_args_t* x, void* stream) {
  if (!s || !x) return CRAFT_EINVAL;
  if (x->n_ticks < 0 || x->ring < 1 || x->tick0 < 0)
    return fail(s, CRAFT_EINVAL, "craft_rollout_teach: need n_ticks >= 0, ring >= 1, tick0 >= 0");
  if (4 * s->view.C > 1000)
    return fail(s, CRAFT_EINVAL, "craft_rollout_teach: 4*W*H > 1000 overflows the reference's BFS queue (teachers/base.py:42)");
  const bool lsync = x->label_actions != 0 || x->behavior_clone != nullptr;
  if (lsync && !x->label_in)
    return fail(s, CRAFT_EINVAL, "craft_rollout_teach: label_actions / behavior_clone need label_in");
  const int esz = s->view.obs_fmt == CRAFT_OBS_F32 ? 4 : (s->view.obs_fmt == CRAFT_OBS_BF16 ? 2 : 1);
  if (x->obs && (!aligned16(x->obs) || (x->ring > 1 && (s->n_envs * (int64_t)s->view.F * esz) % 16 != 0)))
    return fail(s, CRAFT_EINVAL, "craft_rollout_teach: every obs ring slot must be 16-byte aligned");
  if (x->n_ticks == 0) return CRAFT_OK;
  craft::RolloutArgs a{};
  a.actions = x->actions;
  a.seed = x->action_seed;
  a.tick0 = x->tick0;
  a.n_ticks = x->n_ticks;
  a.ring = x->ring;
  a.flags = x->flags;
  a.obs = x->obs;
  a.reward = x->reward;
  a.done = x->done;
  a.sat = x->success;
  a.chunk = x->n_ticks;                           // one unit per tile: all n_ticks ticks
  a.label_in = x->label_in;
  a.bc = x->behavior_clone;
  a.label_actions = x->label_actions != 0;
  // 2: the transition wave looks labels up itself and waits only for BFS answers; 1: it waits
  // for each item's whole row (a task without a hint table: the walk stays with the teacher)
  a.lsync = lsync ? (s->hint_walk ? 1 : 2) : 0;
  a.use_table = s->teach_table != 2;              // auto = always: the reads overlap the stream
  a.labels = x->labels;
  a.rec = x->action_record;
  {
    const int frc = flush_table(s, stream, "craft_rollout_teach");
    if (frc != CRAFT_OK) return frc;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // the work-unit counter as craft_rollout's split kernel uses it (queue[1], one claim past the
  // last unit per workgroup); a captured launch gets the graph's own zeroed counter
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  HIP_TRY(s, hipStreamIsCapturing(st, &cap));
  const bool captured = cap != hipStreamCaptureStatusNone;
  uint8_t* sync = captured ? s->d_sync_graph : s->d_sync;
  a.queue = reinterpret_cast<unsigned long long*>(sync);
  a.tile_done = reinterpret_cast<uint32_t*>(sync + 16);
  if (captured) {
    HIP_TRY(s, hipMemsetAsync(sync, 0, s->sync_bytes, st));
    a.qbase = 0;
    a.qbase1 = 0;
  } else {
    if (!s->sync_zeroed) {
      HIP_TRY(s, hipMemsetAsync(s->d_sync, 0, s->sync_bytes, st));
      s->sync_zeroed = true;
      s->queue_next = 0;
      s->queue1_next = 0;
    }
    a.qbase = s->queue_next;
    a.qbase1 = s->queue1_next;
  }
  int64_t grid = 0;
  a.grid_out = &grid;
  SimView v = teach_view(s);
  // nontemporal observation stores unless tuned: they keep the table's gathered lines in L2
  // (65,536 envs, 20 ticks: 417 -> 388 us with hashed actions, 539 -> 467 us with label actions)
  v.obs_policy = s->obs_store_tuned ? s->rollout_obs_policy : 1;
  const int64_t units = (s->n_envs + craft::rt_tile_of(s->cfg.window_width) - 1) / craft::rt_tile_of(s->cfg.window_width);
  hipError_t e = craft::launch_rollout_teach(s->cfg.window_width, craft::teach_words(s->view.W, s->view.H), v, a, st);
  if (e != hipSuccess) return hip_fail(s, e, "craft_rollout_teach launch");
  if (!captured && grid > 0) s->queue1_next += (uint64_t)std::max<int64_t>(units, grid);
  return CRAFT_OK;
}

int craft_stats(craft_sim_t* s, int64_t* stats_out, int32_t reset, void* stream) {
  if (!s || !stats_out) return CRAFT_EINVAL;
  hipLaunchKernelGGL(craft::stats_kernel, dim3(1), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     s->d_stats, s->n_tiles, stats_out, (int)reset);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(s, e, "craft_stats launch");
  return CRAFT_OK;
}

int craft_transition(craft_sim_t* s, const int32_t* src, const int32_t* dst, const int32_t* actions,
                     int64_t n, int8_t* code_out, void* stream) {
  if (!s) return CRAFT_EINVAL;
  if (n == 0) return CRAFT_OK;
  if (!actions || n < 0) return fail(s, CRAFT_EINVAL, "craft_transition: bad argument");
  if (!src && n > s->n_envs) return fail(s, CRAFT_ERANGE, "craft_transition: n > n_envs");
  TileArgs a{};
  a.src = src;
  a.dst = dst;
  a.actions = actions;
  a.n = n;
  a.code = code_out;
  return launch(s, craft::MODE_TRANSITION, a, stream, "craft_transition launch");
}

int craft_observe(craft_sim_t* s, const int32_t* slots, int64_t n, const int32_t* tasks, void* obs,
                  int8_t* sat, void* stream) {
  if (!s) return CRAFT_EINVAL;
  if (n == 0) return CRAFT_OK;
  if (n < 0) return fail(s, CRAFT_EINVAL, "craft_observe: bad argument");
  if (!slots && n > s->n_envs) return fail(s, CRAFT_ERANGE, "craft_observe: n > n_envs");
  if (obs && !aligned16(obs)) return fail(s, CRAFT_EINVAL, "craft_observe: obs must be 16-byte aligned");
  TileArgs a{};
  a.src = slots;
  a.tasks = tasks;
  a.n = n;
  a.obs = obs;
  a.sat = sat;
  return launch(s, craft::MODE_OBSERVE, a, stream, "craft_observe launch");
}

int craft_rollout_distances(craft_sim_t* s, const int32_t* tasks, const int8_t* success,
                            const int32_t* action_seqs, int32_t ticks, int32_t* distances_out,
                            uint8_t* is_get_out, int32_t* n_actions_out, int32_t* flags_out, void* stream) {
  if (!s) return CRAFT_EINVAL;
  if (!tasks || !success || !distances_out || !is_get_out || !n_actions_out || !flags_out || ticks < 0 ||
      (ticks > 0 && !action_seqs))
    return fail(s, CRAFT_EINVAL, "craft_rollout_distances: bad argument");
  if (4 * s->view.C > 1000)
    return fail(s, CRAFT_EINVAL, "craft_rollout_distances: 4*W*H > 1000 overflows the reference's BFS queue (teachers/base.py:42)");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  HIP_TRY(s, hipMemsetAsync(flags_out, 0, 2 * sizeof(int32_t), st));
  if (s->n_envs == 0) return CRAFT_OK;
  {
    const int frc = flush_table(s, stream, "craft_rollout_distances");
    if (frc != CRAFT_OK) return frc;
  }
  hipError_t e = craft::launch_distances(craft::teach_words(s->view.W, s->view.H), teach_view(s), tasks, success, action_seqs, ticks,
                                         s->n_envs, distances_out, is_get_out, n_actions_out, flags_out, st);
  if (e != hipSuccess) return hip_fail(s, e, "craft_rollout_distances launch");
  return CRAFT_OK;
}

int craft_teacher(craft_sim_t* s, const int32_t* slots, int64_t n, const int32_t* tasks, int32_t* action_out,
                  int32_t* path_len_out, void* stream) {
  if (!s) return CRAFT_EINVAL;
  if (n == 0) return CRAFT_OK;
  if (!action_out || n < 0) return fail(s, CRAFT_EINVAL, "craft_teacher: bad argument");
  if (!slots && n > s->n_envs) return fail(s, CRAFT_ERANGE, "craft_teacher: n > n_envs");
  if (4 * s->view.C > 1000)
    return fail(s, CRAFT_EINVAL, "craft_teacher: 4*W*H > 1000 overflows the reference's BFS queue (teachers/base.py:42)");
  if (n == 0) return CRAFT_OK;
  {
    const int frc = flush_table(s, stream, "craft_teacher");
    if (frc != CRAFT_OK) return frc;
  }
  hipError_t e = craft::launch_teacher(craft::teach_words(s->view.W, s->view.H), s->teach_lanes, teach_view(s), slots, tasks, n, action_out,
                                       path_len_out, reinterpret_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(s, e, "craft_teacher launch");
  return CRAFT_OK;
}

int craft_get_state(craft_sim_t* s, const int32_t* slots, int64_t n, int32_t* agent, int32_t* inventory,
                    uint8_t* grid, int32_t* spec, void* stream) {
  if (!s) return CRAFT_EINVAL;
  if (n == 0) return CRAFT_OK;
  if (n < 0) return fail(s, CRAFT_EINVAL, "craft_get_state: bad argument");
  if (!slots && n > s->n_envs) return fail(s, CRAFT_ERANGE, "craft_get_state: n > n_envs");
  if (n == 0) return CRAFT_OK;
  hipLaunchKernelGGL(craft::get_state_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), s->view, slots, n, agent, inventory, grid, spec);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(s, e, "craft_get_state launch");
  return CRAFT_OK;
}

int craft_set_state(craft_sim_t* s, const int32_t* slots, int64_t n, const int32_t* spec, const int32_t* agent,
                    const int32_t* inventory, void* stream) {
  if (!s) return CRAFT_EINVAL;
  if (n == 0) return CRAFT_OK;
  if (n < 0 || !spec || !agent) return fail(s, CRAFT_EINVAL, "craft_set_state: bad argument");
  if (!slots && n > s->n_envs) return fail(s, CRAFT_ERANGE, "craft_set_state: n > n_envs");
  if (n == 0) return CRAFT_OK;
  hipLaunchKernelGGL(craft::set_state_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), s->view, slots, n, spec, agent, inventory);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return hip_fail(s, e, "craft_set_state launch");
  return CRAFT_OK;
}

}  // extern "C"

#ifdef CRAFT_STAMPS
// Diagnostic builds only: route phase timestamps of the tile kernel into a
// device buffer of 8 u64 per workgroup (tools/phase_stamps.py).
extern "C" int craft_debug_set_stamps(craft_sim_t* s, uint64_t* stamps) {
  if (!s) return CRAFT_EINVAL;
  s->view.stamps = stamps;
  return CRAFT_OK;
}
#endif
