/*
 * craft_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * Scalar CPU restatement of psketch's CraftWorld hot path (worlds/craft.py) and
 * DemonstrationTeacher (teachers/base.py, teachers/demonstration.py), used as
 * the parity checker for the HIP path.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product (psketch_amd/)
 * never does.
 *
 * Pinned against the reference: tests/test_oracle_golden.py replays the
 * reference's own data/craft_medium_{dev,test}.json (4400 teacher
 * demonstrations) and the fixtures in tests/golden/ that
 * tests/golden/make_golden.py produced by running the reference's Python code.
 */
#ifndef PSKETCH_CRAFT_ORACLE_H
#define PSKETCH_CRAFT_ORACLE_H

#include <stdint.h>
#include "../include/craft.h"

#ifdef __cplusplus
extern "C" {
#endif

/* One environment, reference semantics (a CraftState plus the trainer's
 * per-env episode bookkeeping). Plain host memory. */
typedef struct oracle_env {
  int32_t scenario, x0, y0, dir0, task;   /* spec (CraftScenario, craft.py:262-273) */
  int32_t x, y, dir;                      /* CraftState.pos / .dir */
  int32_t timer;                          /* do_rollout `timer` (trainers/imitation.py:30) */
  int32_t frozen;                         /* done and not auto-reset */
  int32_t inv[CRAFT_MAX_KINDS];           /* CraftState.inventory (float64 of small ints) */
  uint8_t grid[CRAFT_MAX_CELLS];          /* CraftState.grid as kind ids, x-major */
} oracle_env_t;

int oracle_sizeof_env(void);
int oracle_sizeof_config(void);

/* CraftState.step (craft.py:332-424); returns CRAFT_OK or CRAFT_EBADACTION. */
int oracle_step(const craft_config_t* cfg, oracle_env_t* s, int32_t action);

/* CraftState.features (craft.py:296-330): out[cfg->n_features]. */
void oracle_features(const craft_config_t* cfg, const oracle_env_t* s, float* out);

/* CraftState.satisfies (craft.py:285-294): 1/0, or -1 for None. */
int oracle_satisfies(const craft_config_t* cfg, const oracle_env_t* s, int32_t task);

/* BaseTeacher.find_closest_resources (teachers/base.py:27-34) over per-target
 * shortest_path BFS runs (teachers/base.py:36-87), literally: one FIFO BFS with
 * prev pointers per target.  *first_action = best_action_seq[0] (-1 if the
 * sequence is empty), *path_len = len(best_action_seq) (-1 if None).
 * Returns CRAFT_ETEACHER where the reference raises (len(None), base.py:31). */
int oracle_closest_resource(const craft_config_t* cfg, const oracle_env_t* s, int32_t kind,
                            int32_t* first_action, int32_t* path_len);

/* DemonstrationTeacher.__call__ (teachers/demonstration.py:9-30). */
int oracle_teacher(const craft_config_t* cfg, const oracle_env_t* s, int32_t task,
                   int32_t* action);

/* Action drawn for synthetic rollouts: splitmix64(seed ^ (gid << 20) ^ tick) >> 32 mod 6. */
int32_t oracle_hash_action(uint64_t seed, int64_t gid, int64_t tick);

/* Reset env to its spec from pool (P entries of W*H kind ids). */
void oracle_reset(const craft_config_t* cfg, const uint8_t* pool, oracle_env_t* s);

/* One tick of the rollout protocol of craft_step (include/craft.h) for n envs:
 * the per-env body of ImitationTrainer.do_rollout (trainers/imitation.py:59-73)
 * then features() of the resulting state.  actions NULL = hashed actions.
 * Any output may be NULL.  stats[3] accumulates {successes, episodes, steps}. */
int oracle_batch_tick(const craft_config_t* cfg, const uint8_t* pool, oracle_env_t* envs,
                      int64_t n, int64_t env_id_base, const int32_t* actions, uint64_t seed,
                      int64_t tick, uint32_t flags, float* obs, float* reward, uint8_t* done,
                      int8_t* success, int64_t* stats);

/* Timing helper for bench.py's cpu_baseline: `ticks` ticks (tick0, tick0+1, ...)
 * of oracle_batch_tick over n envs with global ids env_id_base.. and hashed
 * actions, auto-reset, each tick writing obs [n][F] / reward / done / success
 * (own row per env, as the GPU does).  Returns env-steps run, -1 on error. */
int64_t oracle_bench(const craft_config_t* cfg, const uint8_t* pool, oracle_env_t* envs,
                     int64_t n, int64_t env_id_base, int64_t tick0, int64_t ticks, uint64_t seed,
                     float* obs, int32_t ring, float* reward, uint8_t* done, int8_t* success,
                     int32_t* labels, int64_t* stats);

/* make_data.sample_scenario (make_data.py:105-144) with random_free
 * (make_data.py:74-103) and all_free_cells_reachable (make_data.py:27-72),
 * literally (one FIFO BFS per connectivity check), for `count` scenarios.
 * rng_kind 1: ONE stream, numpy's legacy RandomState(seed) (MT19937,
 *   init_genrand; randint by masked rejection), scenarios drawn in order and, with
 *   dedup, redrawn while equal to an earlier one (make_data.py:166-178);
 *   mt_state_out (625 words: key[624], pos) receives the final state.
 * rng_kind 0: one splitmix64 stream per scenario, keyed by its global id
 *   (scenario_id0 + s): the stream of craft_pool_generate (include/craft.h).
 * grids_out: uint8[count][W*H] kind ids, x-major; init_out: int32[count][2].
 * Returns 0, or -1 if a placement found no valid cell in 2^20 draws. */
int oracle_generate_scenarios(int32_t width, int32_t height, int32_t boundary_kind,
                              const int32_t* primitives, int32_t n_primitive_kinds,
                              int32_t n_per_primitive, const int32_t* workshop_kind,
                              int32_t n_workshops, int32_t rng_kind, uint64_t seed,
                              int64_t scenario_id0, int32_t count, int32_t dedup,
                              uint8_t* grids_out, int32_t* init_out, uint32_t* mt_state_out);

#ifdef __cplusplus
}
#endif
#endif
