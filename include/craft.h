/*
 * craft.h — C ABI of the MI355X-native batched CraftWorld simulator.
 *
 * The reference (khanhptnk/psketch) has no FFI: its boundary is the Python
 * duck-typed world protocol selected by name in worlds/__init__.py:5-11
 * (`globals()[config.world.name](config)`).  Every entry point below replaces
 * one piece of that protocol, batched over N environments that live as
 * struct-of-arrays in HBM.  The Python host side (psketch_amd/) binds these
 * with ctypes; INTEGRATION.md shows the binding a maintainer adds to the
 * reference.
 *
 * Conventions
 *   - Plain C types only.  `stream` is a hipStream_t passed as void* (NULL =
 *     the null stream).  Pointers documented "device" are HBM pointers owned by
 *     the caller; "host" pointers are host memory owned by the caller.
 *   - Every function returns a craft_status (0 = CRAFT_OK).  A failing call
 *     stores a message retrievable with craft_sim_last_error().
 *   - Kernel-side errors (an out-of-range action, a teacher assertion) cannot
 *     be returned synchronously; they latch in a device error word that
 *     craft_sim_check() reads (it synchronises the stream).
 *   - A handle is not thread-safe; calls are stream-ordered.  No allocation
 *     happens on the step path.
 *
 * Grid convention: cell (x, y) of a W x H world is index x*H + y (x-major),
 * exactly the order of `grid[x, y, :]` in worlds/craft.py and of
 * `np.nonzero` in CraftState.find_resource_positions (craft.py:453-455).
 * A cell holds one kind id (0 = empty); the reference's one-hot W x H x K
 * float64 grid maps 1:1 onto it (its one-kind-per-cell invariant is asserted
 * at craft.py:365-371 and checked when a grid is loaded).
 */
#ifndef PSKETCH_CRAFT_H
#define PSKETCH_CRAFT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: craft_sim_tune_teach takes (kernel, lanes, table) (was (kernel)); craft_sim_tune_host,
 * craft_sim_sync_table and craft_abi_version added. */
#define CRAFT_ABI_VERSION 2

#define CRAFT_MAX_KINDS 32       /* len(cookbook.index) incl. reserved 0 (21 for recipes.yaml) */
#define CRAFT_MAX_RECIPES 16     /* recipes.yaml has 9 */
#define CRAFT_MAX_INGREDIENTS 4
#define CRAFT_MAX_TASKS 64       /* hints.hierarchy.yaml has 26 */
#define CRAFT_MAX_SUBTASKS 4
#define CRAFT_MAX_DIM 16         /* W, H <= 16 */
#define CRAFT_MAX_CELLS 256      /* W * H <= 256 */

/* status codes */
typedef enum craft_status {
  CRAFT_OK = 0,
  CRAFT_EINVAL = 1,       /* bad argument / configuration */
  CRAFT_EBADACTION = 2,   /* action outside 0..5: craft.py:415-416 `Exception("Unexpected action")` */
  CRAFT_EINVARIANT = 3,   /* grid breaks an invariant: craft.py:365-371 AssertionError */
  CRAFT_ETEACHER = 4,     /* teacher assertion / crash: teachers/base.py:24,31; demonstration.py:18 */
  CRAFT_EHIP = 5,         /* HIP runtime failure */
  CRAFT_ENOMEM = 6,
  CRAFT_ERANGE = 7        /* slot / scenario index out of range */
} craft_status;

/* Actions, craft.py:25-31.  Moves use world.actions.*.coord_change, craft.py:77-91. */
enum {
  CRAFT_DOWN = 0,   /* (0, -1) */
  CRAFT_UP = 1,     /* (0, +1) */
  CRAFT_LEFT = 2,   /* (-1, 0) */
  CRAFT_RIGHT = 3,  /* (+1, 0) */
  CRAFT_USE = 4,
  CRAFT_STOP = 5,
  CRAFT_N_ACTIONS = 6
};

/* What USE does to a facing cell holding a kind (craft.py:373-410, 101-107). */
enum {
  CRAFT_KIND_INERT = 0,      /* boundary, or a workshop index >= N_WORKSHOPS: USE is a no-op */
  CRAFT_KIND_GRABBABLE = 1,  /* not in cookbook.environment: inventory += 1, cell cleared */
  CRAFT_KIND_WORKSHOP = 2,   /* workshop0..N_WORKSHOPS-1: apply its recipes in dict order */
  CRAFT_KIND_WATER = 3,      /* with bridge > 0: cell cleared, bridge -= 1 */
  CRAFT_KIND_STONE = 4       /* with axe > 0: cell cleared, axe kept */
};

/* Task.goal_name values (data/task.py:11) that CraftState.satisfies and the
 * DemonstrationTeacher distinguish (craft.py:285-294, teachers/demonstration.py:18-21). */
enum {
  CRAFT_GOAL_OTHER = 0,   /* left/right/up/down/stop/makeat: satisfies() -> None */
  CRAFT_GOAL_GET = 1,     /* inventory[arg] > 0 */
  CRAFT_GOAL_MAKE = 2,    /* inventory[arg] > 0 */
  CRAFT_GOAL_GO = 3,      /* facing cell holds arg */
  CRAFT_GOAL_USE = 4      /* satisfies() -> None; teacher leaf -> USE */
};

typedef struct craft_recipe {
  int32_t output;        /* kind id produced */
  int32_t workshop;      /* kind id of its `_at` workshop */
  int32_t yield;         /* `_yield`, default 1, 1..255 (craft.py:394); a u8 count that would pass
                            255 saturates and latches CRAFT_ERANGE */
  int32_t n_inputs;
  int32_t input_kind[CRAFT_MAX_INGREDIENTS];
  int32_t input_count[CRAFT_MAX_INGREDIENTS];
} craft_recipe_t;

typedef struct craft_task {
  int32_t goal;          /* CRAFT_GOAL_* */
  int32_t arg_kind;      /* cookbook.index[goal_arg]; 0 when the arg is not a kind */
  int32_t n_subtasks;    /* 0 = leaf (data/task.py:13-15) */
  int32_t subtask[CRAFT_MAX_SUBTASKS];   /* task ids, in hint order */
} craft_task_t;

/* Static world tables: CraftWorld.__init__ (craft.py:59-109), Cookbook
 * (worlds/cookbook.py:8-26), TaskManager (data/task.py:32-75). */
typedef struct craft_config {
  int32_t abi_version;       /* = CRAFT_ABI_VERSION */
  int32_t width, height;     /* WIDTH, HEIGHT */
  int32_t window_width, window_height;   /* WINDOW_WIDTH, WINDOW_HEIGHT (odd, equal, 3..7) */
  int32_t n_kinds;           /* len(cookbook.index) */
  int32_t n_features;        /* must equal 2*ww*wh*n_kinds + n_kinds + 5 (craft.py:69-75) */
  int32_t max_timesteps;     /* trainer.max_timesteps (configs/experiments/imitation.yaml:21) */
  int32_t bridge_kind, axe_kind;
  uint8_t kind_class[CRAFT_MAX_KINDS];   /* CRAFT_KIND_* per kind id */
  int32_t n_recipes;
  craft_recipe_t recipe[CRAFT_MAX_RECIPES];   /* cookbook.recipes in dict (YAML) order */
  int32_t n_tasks;
  craft_task_t task[CRAFT_MAX_TASKS];         /* TaskManager.tasks order */
} craft_config_t;

typedef struct craft_sim craft_sim_t;

/* ---- handle lifetime ------------------------------------------------------ */

/* CRAFT_ABI_VERSION of the loaded library: a caller that binds the symbols at run time (dlsym,
 * ctypes) checks it before calling anything whose signature changed between versions. */
int craft_abi_version(void);

/* Replaces CraftWorld.__init__ (craft.py:59-109) for a batch of `n_envs`
 * environment slots on `device`.  `env_id_base` is the global id of slot 0
 * (rank * n_envs when sharded): per-env randomness is keyed by global id so
 * results do not depend on the number of GPUs.  `pool_capacity` scenario
 * grids can be loaded. */
int craft_sim_create(const craft_config_t* cfg, int device, int64_t n_envs,
                     int64_t env_id_base, int32_t pool_capacity, craft_sim_t** out);
int craft_sim_destroy(craft_sim_t* sim);
const char* craft_sim_last_error(const craft_sim_t* sim);
const char* craft_strerror(int status);
int craft_sim_info(const craft_sim_t* sim, int64_t* n_envs, int32_t* pool_capacity,
                   int32_t* n_features);

/* Performance knobs of the tile kernels (results are identical for every
 * setting): envs per workgroup tile (16, 32 or 64; 0 = default for the
 * window), the most tile workgroups that may share a CU (0 = no cap, else
 * 3..32), and the cache policy of the observation stores (0 write-back,
 * 1 nontemporal, 2 write-through) for every entry point.  Until it is called,
 * every kernel stores write-through (sc1; the measured best for craft_rollout and for a
 * tick that rewrites one buffer) except craft_rollout_teach, which stores nontemporal (its
 * teacher-table gathers keep their L2 lines: 7-15 % faster at 65,536 envs).
 * Note: craft_sim_tune(.., 0, 0, 0) selects write-back. */
int craft_sim_tune(craft_sim_t* sim, int32_t tile_envs, int32_t max_resident_per_cu,
                   int32_t obs_store);

/* craft_rollout scheduling knobs (results are identical for every setting).
 * chunk_ticks: work-unit length.  The launch is cut into (tile, chunk of
 * chunk_ticks ticks) units handed out dynamically to the workgroups, a tile's
 * state passing between workgroups at chunk boundaries, so slow workgroups do
 * fewer units.  0 (default) = one unit per tile for the whole launch, which
 * measured fastest at 65536 envs (the balance gained does not pay for the
 * hand-offs).  -1 = one continuous pipeline per workgroup across
 * the tiles it claims (no pipeline fill and drain per tile, the next tile
 * prefetched by LDS-DMA; the split kernel's 3x3 default shape only): measured
 * level with 0.  threads: threads per tile workgroup on the tile
 * set by craft_sim_tune.  128 or 256: one producer wave, the rest stream; 64-env
 * tiles also take 512.  16- and 32-env tiles with 320, 384 or 512: the
 * split-producer kernel (transition and scatter on two waves, the other 3-6
 * stream).  0 (default) = the measured best: 32-env tiles x 512 threads (split)
 * for 3x3 windows, else the handle's tile with 256 threads (512 for 64-env tiles). */
int craft_sim_tune_rollout(craft_sim_t* sim, int32_t chunk_ticks, int32_t threads);

/* The teacher's knobs (results are identical for every setting; a tuning knob like
 * craft_sim_tune, replacing nothing in the reference):
 *   kernel  which kernel craft_step_teach launches: 0 (default) = the measured best (the two-tile
 *           kernel with 2 teacher lanes per env for 3x3 windows at >= 32768 envs, else the
 *           one-tile kernel: 64-env tiles with 4 lanes for 3x3 windows, the handle's tile (32
 *           by default) with 2 for wider ones), 1 = the one-tile kernel, 2 = the two-tile
 *           kernel (3x3 windows and the default tile only; otherwise the one-tile kernel);
 *   lanes   teacher lanes per query: 0 (default) = each kernel's measured best; 1, 2 or 4 for
 *           craft_teacher and the one-tile kernel, 2 or 4 for the two-tile kernel (others: 2);
 *   table   which teachers read the teacher table (find_closest_resources answered ahead of
 *           time for every grid an env can reach: its pool row minus any subset of the row's
 *           first m clearable cells (m <= 8), for every go/get target kind, start cell and
 *           direction; 4*W*H u16 entries per kind per (row, subset), allocated at the first pool
 *           load for pool_capacity rows with m chosen to fit 1 GiB (12x12 craft_medium: m = 6,
 *           453 MB for 1024 rows); a loaded row's entries are built by the next launch that reads
 *           the table, on its stream, which then waits for them (craft_sim_sync_table)), for envs
 *           whose grid it lists: 0 (default) = auto (every teacher: measured faster in every
 *           launch shape since the 4-bit copy), 1 = always, 2 = never (every query runs the BFS). */
int craft_sim_tune_teach(craft_sim_t* sim, int32_t kernel, int32_t lanes, int32_t table);

/* Host worker threads of the CPU variant of this ABI (libpsketch_craft_cpu.so), which splits
 * every batched call over contiguous slot ranges: 0 = the machine's hardware threads (the
 * default), else 1..1024.  Results are identical for every setting.  The HIP library runs no
 * host workers: it validates the argument and keeps nothing. */
int craft_sim_tune_host(craft_sim_t* sim, int32_t threads);

/* Builds, on `stream`, the teacher-table entries of the pool rows craft_pool_load has loaded since
 * the last build, and waits for them.  Every launch that reads the table (craft_step_teach,
 * craft_rollout_teach, craft_teacher, craft_rollout_distances) does this first, so a caller needs
 * it only before capturing such a launch into a HIP graph right after a pool load: a launch
 * being captured refuses (CRAFT_EINVAL) to build them.  No-op when nothing is pending. */
int craft_sim_sync_table(craft_sim_t* sim, void* stream);

/* The kernel craft_step / craft_step_ex (teach == 0) or craft_step_teach (teach != 0) will
 * launch, resolved from the knobs above: *kernel = CRAFT_KERNEL_TILE / _TICK2, *envs =
 * envs per tile (tile kernel) or per workgroup (two-tile kernel),
 * *lanes = teacher lanes per env (0 without a teacher).  Lets a caller (bench.py) name the
 * kernel it times instead of mirroring the library's defaults. */
#define CRAFT_KERNEL_TILE 1
#define CRAFT_KERNEL_TICK2 2
int craft_sim_step_shape(const craft_sim_t* sim, int32_t teach, int32_t* kernel, int32_t* envs,
                         int32_t* lanes);

/* The launch shape the next craft_rollout will use, resolved from the knobs above:
 * envs per tile workgroup, threads per workgroup, and split = 1 for the
 * split-producer kernel (rollout_split_kernel), 0 for rollout_kernel.  Lets a
 * caller (bench.py) name the kernel it times instead of mirroring the defaults. */
int craft_sim_rollout_shape(const craft_sim_t* sim, int32_t* tile_envs, int32_t* threads,
                            int32_t* split);

/* The tile kernel's current envs per workgroup and observation store policy
 * (craft_sim_tune), for the same purpose on the craft_step path. */
int craft_sim_tile_shape(const craft_sim_t* sim, int32_t* tile_envs, int32_t* obs_store);

/* Element type of every observation buffer this handle writes (craft_reset,
 * craft_step, craft_step_ex, craft_observe).  The features are small
 * non-negative integers (one-hots, block maxima, inventory counts < 256), so
 * all three formats hold exactly the reference's values; bf16 and u8 cut the
 * observation stream (the kernel's dominant HBM traffic) by 2x and 4x for a
 * student that consumes them directly.  Default CRAFT_OBS_F32. */
typedef enum {
  CRAFT_OBS_F32 = 0,
  CRAFT_OBS_BF16 = 1,
  CRAFT_OBS_U8 = 2
} craft_obs_format_t;
int craft_sim_set_obs_format(craft_sim_t* sim, int32_t format);

/* Synchronises `stream` and returns the first kernel-side error latched since
 * the last call (then clears it); *env_out receives the offending slot. */
int craft_sim_check(craft_sim_t* sim, int64_t* env_out, void* stream);

/* Without synchronising: queues a copy of the latched-error record into device int32[4]
 * `out` on `stream` ({status, 0, slot low, slot high}; status 0 = no error), so a caller can
 * read it back together with its own results and call craft_sim_check only when it is set. */
int craft_sim_error_word(craft_sim_t* sim, int32_t* out, void* stream);

/* ---- scenario pool ---------------------------------------------------------- */

/* Uploads `count` initial grids (host, count * W*H kind ids, x-major) into pool
 * entries [first, first+count).  Replaces the `grid` handed to
 * CraftWorld.init_state (craft.py:258-259).  Rejects (CRAFT_EINVARIANT) kind ids
 * >= n_kinds and worlds whose border ring holds a cell that is empty, not inert
 * (CRAFT_KIND_INERT: USE could clear it) or some task's target kind: every
 * make_data.py world has the boundary ring (make_data.py:108-112), and the
 * teacher's BFS and the kernels rely on it. Synchronous. */
int craft_pool_load(craft_sim_t* sim, const uint8_t* grids, int32_t first, int32_t count);

/* ---- episodes ---------------------------------------------------------------- */

/* CraftScenario.init (craft.py:262-273) for every slot: inventory zeroed,
 * grid = pool[scenario], pos/dir given, timer = max_timesteps.  The spec is
 * kept so that an auto-reset returns the slot to the same initial state.
 * Device arrays of n_envs int32 each; `obs` (n_envs x n_features, obs format) may be
 * NULL, else receives features() of the initial states. */
int craft_reset(craft_sim_t* sim, const int32_t* scenario, const int32_t* pos_x,
                const int32_t* pos_y, const int32_t* dir, const int32_t* task,
                void* obs, void* stream);

#define CRAFT_STEP_AUTORESET 1u   /* done slots restart from their spec next tick */

/* One tick of the imitation-trainer rollout for every slot, fused with the
 * observation: the per-env body of ImitationTrainer.do_rollout
 * (trainers/imitation.py:59-73) followed by CraftState.features() of the new
 * state (craft.py:296-330).
 *   timer -= 1; done = (a == STOP) or timer <= 0
 *   done  -> success = satisfies(task) on the pre-step state, no step
 *            (auto-reset: the slot restarts; else it stays frozen)
 *   !done -> state = step(state, a)            (craft.py:332-424)
 * `actions` (device int32[n_envs]) may be NULL: actions are then drawn in the
 * kernel as splitmix64(action_seed ^ (gid << 20) ^ tick) >> 32 mod 6.
 * Outputs (device, each may be NULL): obs [n_envs][n_features] (obs format);
 * reward fp32 (1 on a tick that ends an episode with satisfies() true, else 0 —
 * step() itself always returns 0, craft.py:338); done uint8; success int8
 * (-1 not terminal, else satisfies()).  Episode statistics accumulate inside
 * the handle (per-workgroup partial sums, no atomics); read them with
 * craft_stats. */
int craft_step(craft_sim_t* sim, const int32_t* actions, uint64_t action_seed, int64_t tick,
               uint32_t flags, void* obs, float* reward, uint8_t* done, int8_t* success,
               void* stream);

/* craft_step with the rest of a do_rollout tick fused in (trainers/imitation.py:43-73):
 *   a = behavior_clone[i] ? ref_actions[i] : actions[i]     (imitation.py:56-57)
 *   action_record[i] = a, or -1 for a slot already done     (action_seqs, :59-61)
 *   *any_live = 1 if some slot is still running after this tick (all(done), :42)
 * then the craft_step tick.  ref_actions is craft_teacher's output for the same
 * slots (a done slot's label is -1 and is never used).  Every pointer may be
 * NULL: actions NULL = the hashed draw; ref_actions/behavior_clone NULL = no
 * cloning.  any_live is a device int32 the kernel only ever sets to 1 (plain
 * stores, no atomics: point it at element t of a zeroed per-tick array).  The
 * rollout counters come from craft_stats: num_interactions (:54) = env-steps,
 * num_steps (:71) = env-steps - episodes ended.  obs has the handle's obs format. */
typedef struct {
  const int32_t* actions;          /* int32[n_envs] student actions */
  const int32_t* ref_actions;      /* int32[n_envs] teacher labels */
  const uint8_t* behavior_clone;   /* uint8[n_envs] 0/1 */
  uint64_t action_seed;
  int64_t tick;
  uint32_t flags;                  /* CRAFT_STEP_AUTORESET */
  void* obs;                       /* [n_envs][n_features] in the obs format */
  float* reward;
  uint8_t* done;
  int8_t* success;
  int32_t* action_record;          /* int32[n_envs] */
  int32_t* any_live;               /* int32 scalar flag */
  int8_t* transition_code;         /* int8[n_envs]: see craft_transition; -1 if no step */
} craft_step_args_t;
int craft_step_ex(craft_sim_t* sim, const craft_step_args_t* args, void* stream);

/* The device address of page-locked host memory (hipHostGetDevicePointer), e.g. for an
 * any_live flag array the host polls after an event instead of copying each tick's flag
 * back (the kernel's plain stores of 1 are visible to the host once the launch has
 * completed).  CRAFT_EINVAL if `host` is not page-locked memory HIP maps. */
int craft_host_flag_pointer(void* host, int32_t** device_out);

/* craft_step_ex fused with craft_teacher on every slot's NEW state (its own task),
 * in one launch: label_out (device int32[n_envs]) receives
 * DemonstrationTeacher.__call__ (teachers/demonstration.py:9-30) of each slot
 * after the tick — the ref_actions of the next tick of ImitationTrainer.do_rollout
 * (trainers/imitation.py:47-55): -1 for a slot the tick left frozen, -2 (and
 * CRAFT_ETEACHER latched) where the reference raises.  Identical to craft_step_ex
 * followed by craft_teacher(slots NULL, tasks NULL), but the teacher reads the
 * grid rows the tick holds on chip instead of rebuilding them from HBM, and its
 * BFS overlaps the observation stores (config 5: a teacher label every tick). */
int craft_step_teach(craft_sim_t* sim, const craft_step_args_t* args, int32_t* label_out, void* stream);

/* n_ticks consecutive craft_step ticks (tick0, tick0+1, ...) in one launch, with
 * results identical to n_ticks craft_step calls: each workgroup keeps its envs
 * on chip between ticks, so the per-tick prologue overlaps other workgroups'
 * observation stores.  For rollouts whose actions do not depend on the
 * observations: `actions` is device int32[n_ticks][n_envs] or NULL for the
 * hashed draw.  Tick t writes ring slot t % ring of each output: obs
 * [ring][n_envs][n_features] (obs format; each slot 16-byte aligned), reward /
 * done / success [ring][n_envs]; each may be NULL.
 * Ordering: one handle's craft_rollout launches must run in issue order, i.e. on one stream (or
 * streams the caller orders): the work-unit counter they share is advanced by each launch, not
 * re-zeroed.  A launch captured into a HIP graph (hipStreamIsCapturing) uses a separate counter
 * that a memset captured with it zeroes, so a graph may be replayed any number of times, in
 * order with each other and with eager launches.  Every captured launch of one handle shares
 * that one counter: two captured graphs, or one graph replayed on two streams, must never run
 * concurrently (unsupported: their work units would be skipped or repeated, undetected). */
int craft_rollout(craft_sim_t* sim, const int32_t* actions, uint64_t action_seed, int64_t tick0,
                  int32_t n_ticks, uint32_t flags, void* obs, int32_t ring, float* reward,
                  uint8_t* done, int8_t* success, void* stream);

/* craft_rollout with the DemonstrationTeacher in the same launch: n_ticks ticks, and after each
 * one DemonstrationTeacher.__call__ (teachers/demonstration.py:9-30) of every slot's new state,
 * as n_ticks craft_step_teach calls would give, with each tick's action taken per slot from
 *   - its label (the teacher's action for its current state): every slot when label_actions
 *     (make_data.get_reference_actions, make_data.py:146-152: the demonstrations), or the slots
 *     with behavior_clone[i] set (DAgger's mix, trainers/imitation.py:47-57);
 *   - otherwise the policy: actions[k][i] (device int32[n_ticks][n_envs]) or the hashed draw.
 * The label of a slot's state before tick0 comes from label_in (device int32[n_envs]: craft_teacher's
 * answer, or the last labels ring slot of the previous launch); required when labels feed actions.
 * Tick k = tick0 + k writes ring slot k % ring of each output (each may be NULL): obs
 * [ring][n_envs][n_features] (obs format), reward / done / success as craft_rollout, labels
 * int32 [ring][n_envs] (the label of the slot's state after the tick: -1 for a slot the tick left
 * frozen, -2 and CRAFT_ETEACHER latched where the reference raises), action_record int32
 * [ring][n_envs] (the action taken, -1 for a slot already done: action_seqs).  Episode statistics
 * accumulate as for craft_step.  Ordering as craft_rollout (one stream; a captured launch uses the
 * graph's own counter).  Replaces the per-tick loop of trainers/imitation.py:43-73 with the
 * teacher queried every tick, and make_data.get_reference_actions. */
typedef struct {
  const int32_t* actions;          /* int32[n_ticks][n_envs] policy actions, or NULL: the hashed draw */
  const uint8_t* behavior_clone;   /* uint8[n_envs] 0/1: the slot acts on its label, or NULL */
  int32_t label_actions;           /* 1: every slot acts on its label */
  const int32_t* label_in;         /* int32[n_envs] labels of the states before tick0 */
  uint64_t action_seed;
  int64_t tick0;
  int32_t n_ticks;
  uint32_t flags;                  /* CRAFT_STEP_AUTORESET */
  int32_t ring;                    /* ring slots of every output (>= 1) */
  void* obs;
  float* reward;
  uint8_t* done;
  int8_t* success;
  int32_t* labels;
  int32_t* action_record;
} craft_rollout_teach_args_t;
int craft_rollout_teach(craft_sim_t* sim, const craft_rollout_teach_args_t* args, void* stream);

/* Sums the episode statistics accumulated by craft_step into stats_out
 * (device int64[3] = {successes, episodes ended, env-steps}) — the scalar
 * summary a multi-GPU run all-reduces over RCCL.  reset != 0 zeroes the
 * partial sums afterwards. */
int craft_stats(craft_sim_t* sim, int64_t* stats_out, int32_t reset, void* stream);

/* ---- reference-granular surface (CraftState methods), over slot lists ----
 * For every call below, n == 0 is a no-op that returns CRAFT_OK (pointers unused). */

/* CraftState.step (craft.py:332-424) as a pure transition: slot dst[i] becomes
 * step(slot src[i], actions[i]) — src == dst updates in place, src != dst keeps
 * the old state (the reference's states are immutable).  actions[i] < 0 is a
 * no-op copy.  src/dst NULL = identity over n slots.  Device int32 arrays.
 * code_out (int8[n], may be NULL) receives what PrimitiveLanguageTeacher.describe
 * reads off the (state, next state) pair (teachers/primitive_language.py:61-85):
 * 0..3 = moved by the coord_change of DOWN/UP/LEFT/RIGHT, 4 = did not move and
 * the inventory changed, 5 = neither, -1 = no step (action < 0). */
int craft_transition(craft_sim_t* sim, const int32_t* src, const int32_t* dst,
                     const int32_t* actions, int64_t n, int8_t* code_out, void* stream);

/* CraftState.features() (craft.py:296-330) and satisfies() (craft.py:285-294)
 * for n slots (NULL = identity).  obs: [n][n_features] (obs format) or NULL; sat: int8[n]
 * (-1 = None, 0/1) for task tasks[i] (NULL = the slot's own task) or NULL. */
int craft_observe(craft_sim_t* sim, const int32_t* slots, int64_t n, const int32_t* tasks,
                  void* obs, int8_t* sat, void* stream);

/* The per-env part of the rollout's summary (trainers/imitation.py:79-91), one launch over
 * every slot after a do_rollout: tasks int32[n] (each slot's task), success int8[n]
 * (1 / 0 / -1 for None), action_seqs int32[ticks][n] (the action record, -1 where the env did
 * not act).  Per slot: is_get_out = the task's goal is `get`; distances_out = -1 for other
 * goals, 0 for a success, else len(find_closest_resources(task.arg)) on world.init_state(
 * grid, pos, dir): the slot's initial grid (its pool row, nothing cleared) at its current pose
 * (-1 where the grid holds no target, -2 where a target is unreachable: base.py:31); n_actions_out
 * = the action record's non-negative entries (len(action_seqs[i])).  flags_out int32[2] (zeroed
 * here): [0] some success is None (imitation.py:68 asserts), [1] a failed get task has no
 * reachable target, in either case (the reference raises one TypeError, len(None), at
 * imitation.py:88-89 or base.py:31).  The env states are not modified.
 * Replaces trainers/imitation.py:79-91's per-env loop. */
int craft_rollout_distances(craft_sim_t* sim, const int32_t* tasks, const int8_t* success,
                            const int32_t* action_seqs, int32_t ticks, int32_t* distances_out,
                            uint8_t* is_get_out, int32_t* n_actions_out, int32_t* flags_out,
                            void* stream);

/* DemonstrationTeacher.__call__ (teachers/demonstration.py:9-30) for n slots:
 * find_incomplete_subtask over the hint tree then the BFS of
 * find_closest_resources/shortest_path (teachers/base.py:10-87).
 * action_out int32[n]; path_len_out int32[n] (may be NULL) receives
 * len(best_action_seq) of find_closest_resources for the task's own goal_arg
 * (the trainer's `distances`, trainers/imitation.py:79-91), -1 if no target.
 * Where the reference raises (base.py:24 assert, base.py:31 len(None),
 * demonstration.py:18 assert) the item gets -2 and CRAFT_ETEACHER latches.
 * slots[i] == -1 skips item i, and a frozen slot (an episode craft_step ended
 * without auto-reset) yields action -1 (path length -1, no error): the
 * trainer's ref_actions[i] = -1 for a done env (trainers/imitation.py:50-51). */
int craft_teacher(craft_sim_t* sim, const int32_t* slots, int64_t n, const int32_t* tasks,
                  int32_t* action_out, int32_t* path_len_out, void* stream);

/* State I/O for the Python CraftState shim and for parity tests (device
 * arrays, n slots, NULL slot list = identity).  grid: uint8[n][W*H] current
 * kind ids; inventory: int32[n][n_kinds]; agent: int32[n][4] = {x, y, dir, timer};
 * spec: int32[n][5] = {scenario, x0, y0, dir0, task}. */
int craft_get_state(craft_sim_t* sim, const int32_t* slots, int64_t n, int32_t* agent,
                    int32_t* inventory, uint8_t* grid, int32_t* spec, void* stream);
/* Sets slots to (scenario grid with no removals, agent, inventory); spec as above. */
int craft_set_state(craft_sim_t* sim, const int32_t* slots, int64_t n, const int32_t* spec,
                    const int32_t* agent, const int32_t* inventory, void* stream);

/* make_data.sample_scenario (make_data.py:105-144) on the GPU, straight into pool
 * rows [first, first + count): boundary ring, n_per_primitive of each primitive,
 * then the workshops, each placed by random_free with its connectivity checks,
 * then the initial position (init_pos_out: device int32[count][2], may be NULL).
 * Scenario s draws from its own splitmix64 stream keyed by seed and its global
 * id scenario_id0 + s (numpy's sequential MT19937 stream cannot be split across
 * lanes), so results do not depend on how ids are sharded; otherwise the
 * algorithm and acceptance tests are make_data.py's.  No de-duplication.  Where
 * a placement finds no valid cell in 2^20 draws, CRAFT_EINVARIANT latches. */
int craft_pool_generate(craft_sim_t* sim, uint64_t seed, int64_t scenario_id0, int32_t first,
                        int32_t count, int32_t boundary_kind, const int32_t* primitives,
                        int32_t n_primitive_kinds, int32_t n_per_primitive,
                        const int32_t* workshop_kind, int32_t n_workshops, int32_t* init_pos_out,
                        void* stream);

/* ---- host-side scenario generation ------------------------------------------ */

/* make_data.sample_scenario (make_data.py:105-144) with `random_free`
 * (make_data.py:74-103) and `all_free_cells_reachable` (make_data.py:27-72),
 * drawing from numpy's legacy RandomState(seed) MT19937 stream bit-exactly.
 * Generates `count` scenarios (each rejected and redrawn while it duplicates an
 * earlier one when `dedup`, make_data.py:167-177).  grids_out: host
 * uint8[count][W*H]; init_pos_out: host int32[count][2].  `primitives` lists the
 * primitive kind ids in the iteration order of cookbook.primitives with gold/gem
 * already removed (make_data.py:128-134); workshops are kinds workshop_kind[0..n_ws).
 * The MT19937 state after the last draw is written to mt_state_out (625 uint32,
 * may be NULL) so a caller can continue numpy's stream. */
int craft_sample_scenarios(int32_t width, int32_t height, int32_t boundary_kind,
                           const int32_t* primitives, int32_t n_primitive_kinds,
                           int32_t n_per_primitive, const int32_t* workshop_kind,
                           int32_t n_workshops, uint32_t seed, int32_t count, int32_t dedup,
                           uint8_t* grids_out, int32_t* init_pos_out, uint32_t* mt_state_out);

#ifdef __cplusplus
}
#endif
#endif /* PSKETCH_CRAFT_H */
