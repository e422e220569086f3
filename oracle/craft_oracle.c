/*
 * craft_oracle.c — TEST INFRASTRUCTURE ONLY (see craft_oracle.h).
 *
 * A deliberately literal, scalar restatement of the reference algorithms, one
 * environment at a time, kept structurally close to the Python so that each
 * function can be read side by side with the file:line it cites.  It is the
 * parity checker for the HIP kernels and the CPU baseline timed by bench.py —
 * never part of the product path.
 */
#include "craft_oracle.h"

#include <stdlib.h>
#include <string.h>

static const int DX[4] = {0, 0, -1, 1};   /* craft.py:77-91 coord_change of DOWN, UP, LEFT, RIGHT */
static const int DY[4] = {-1, 1, 0, 0};

int oracle_sizeof_env(void) { return (int)sizeof(oracle_env_t); }

static inline int cell(const craft_config_t* cfg, const oracle_env_t* s, int x, int y) {
  return s->grid[x * cfg->height + y];
}

/* CraftState.step, craft.py:332-424. */
int oracle_step(const craft_config_t* cfg, oracle_env_t* s, int32_t action) {
  const int W = cfg->width, H = cfg->height;
  int x = s->x, y = s->y, dx = 0, dy = 0, n_dir = s->dir;
  if (action >= CRAFT_DOWN && action <= CRAFT_RIGHT) {         /* craft.py:341-352 */
    dx = DX[action];
    dy = DY[action];
    n_dir = action;
  } else if (action == CRAFT_STOP) {                           /* craft.py:353-354 */
  } else if (action == CRAFT_USE) {                            /* craft.py:356-412 */
    /* neighbors(pos, dir) yields only the facing cell, if inside the grid (craft.py:426-437) */
    int ok = 0, nx = x, ny = y;
    if (s->dir == CRAFT_LEFT && x > 0) { ok = 1; nx = x - 1; }
    if (s->dir == CRAFT_DOWN && y > 0) { ok = 1; ny = y - 1; }
    if (s->dir == CRAFT_RIGHT && x < W - 1) { ok = 1; nx = x + 1; }
    if (s->dir == CRAFT_UP && y < H - 1) { ok = 1; ny = y + 1; }
    if (ok) {
      int thing = cell(cfg, s, nx, ny);
      if (thing != 0) {                                        /* craft.py:362-363 */
        int cls = cfg->kind_class[thing];
        if (cls == CRAFT_KIND_GRABBABLE) {                     /* craft.py:383-386 */
          s->inv[thing] += 1;
          s->grid[nx * H + ny] = 0;
        } else if (cls == CRAFT_KIND_WORKSHOP) {               /* craft.py:388-401 */
          for (int r = 0; r < cfg->n_recipes; ++r) {
            const craft_recipe_t* rc = &cfg->recipe[r];
            if (rc->workshop != thing) continue;
            int have = 1;
            for (int i = 0; i < rc->n_inputs; ++i)
              if (s->inv[rc->input_kind[i]] < rc->input_count[i]) have = 0;
            if (!have) continue;
            s->inv[rc->output] += rc->yield;
            for (int i = 0; i < rc->n_inputs; ++i) s->inv[rc->input_kind[i]] -= rc->input_count[i];
          }
        } else if (cls == CRAFT_KIND_WATER) {                  /* craft.py:403-406 */
          if (s->inv[cfg->bridge_kind] > 0) {
            s->grid[nx * H + ny] = 0;
            s->inv[cfg->bridge_kind] -= 1;
          }
        } else if (cls == CRAFT_KIND_STONE) {                  /* craft.py:408-410 */
          if (s->inv[cfg->axe_kind] > 0) s->grid[nx * H + ny] = 0;
        }
        /* CRAFT_KIND_INERT: craft.py:374-378 `continue` */
      }
    }
  } else {
    return CRAFT_EBADACTION;                                   /* craft.py:415-416 */
  }
  /* Collision against the grid before the action (craft.py:418-421). A USE
   * only edits the facing cell and has dx = dy = 0, so the own cell is read. */
  int n_x = x + dx, n_y = y + dy;
  if (!(action == CRAFT_USE) && cell(cfg, s, n_x, n_y) != 0) { n_x = x; n_y = y; }
  s->x = n_x;
  s->y = n_y;
  s->dir = n_dir;
  return CRAFT_OK;
}

/* CraftState.features, craft.py:296-330, with misc/array.py:3-25 pad_slice and
 * skimage.measure.block_reduce(func=np.max) (pad to a block multiple, reduce
 * each block; the windows here divide evenly so no padding is added). */
void oracle_features(const craft_config_t* cfg, const oracle_env_t* s, float* out) {
  const int W = cfg->width, H = cfg->height, K = cfg->n_kinds;
  const int ww = cfg->window_width, wh = cfg->window_height;
  const int hw = ww / 2, hh = wh / 2;
  const int bhw = (ww * ww) / 2, bhh = (wh * wh) / 2;
  const int L = ww * wh * K;
  memset(out, 0, sizeof(float) * (size_t)cfg->n_features);
  for (int i = 0; i < ww; ++i)
    for (int j = 0; j < wh; ++j) {
      int cx = s->x - hw + i, cy = s->y - hh + j;
      if (cx < 0 || cy < 0 || cx >= W || cy >= H) continue;   /* zero padding */
      int c = cell(cfg, s, cx, cy);
      if (c) out[(i * wh + j) * K + c] = 1.0f;
    }
  for (int bi = 0; bi < ww; ++bi)
    for (int bj = 0; bj < wh; ++bj)
      for (int ii = 0; ii < ww; ++ii)
        for (int jj = 0; jj < wh; ++jj) {
          int cx = s->x - bhw + bi * ww + ii, cy = s->y - bhh + bj * wh + jj;
          if (cx < 0 || cy < 0 || cx >= W || cy >= H) continue;
          int c = cell(cfg, s, cx, cy);
          if (c) out[L + (bi * wh + bj) * K + c] = 1.0f;
        }
  for (int k = 0; k < K; ++k) out[2 * L + k] = (float)s->inv[k];
  out[2 * L + K + s->dir] = 1.0f;
  /* pos_feats (craft.py:316-319) is computed and dropped; last entry stays 0. */
}

/* CraftState.satisfies, craft.py:285-294. */
int oracle_satisfies(const craft_config_t* cfg, const oracle_env_t* s, int32_t task) {
  const craft_task_t* t = &cfg->task[task];
  if (t->goal == CRAFT_GOAL_GET || t->goal == CRAFT_GOAL_MAKE) return s->inv[t->arg_kind] > 0;
  if (t->goal == CRAFT_GOAL_GO) {
    int fx = s->x + DX[s->dir], fy = s->y + DY[s->dir];
    return cell(cfg, s, fx, fy) == t->arg_kind;
  }
  return -1;
}

/* shortest_path, teachers/base.py:36-87: FIFO BFS over (pos, dir) with a
 * 1000-slot queue; stops at the first dequeued state that faces goal. */
static int shortest_path(const craft_config_t* cfg, const oracle_env_t* s, int gx, int gy,
                         int* first_action, int* len, int* overflow) {
  const int H = cfg->height, NS = 4 * cfg->width * cfg->height;
  int* prev_state = (int*)malloc(sizeof(int) * NS);   /* -2 unseen, -1 root */
  int* prev_action = (int*)malloc(sizeof(int) * NS);
  int queue[1000];
  for (int i = 0; i < NS; ++i) prev_state[i] = -2;
  int start = 0, end = 0, found = -1;
  int item0 = (s->x * H + s->y) * 4 + s->dir;
  queue[end++] = item0;
  prev_state[item0] = -1;
  *overflow = 0;
  while (start < end) {
    int item = queue[start++];
    int p = item / 4, dir = item % 4, px = p / H, py = p % H;
    if (px + DX[dir] == gx && py + DY[dir] == gy) { found = item; break; }
    for (int a = 0; a < 4; ++a) {                     /* action_space order, USE/STOP skipped */
      int nx = px + DX[a], ny = py + DY[a];
      if (cell(cfg, s, nx, ny)) { nx = px; ny = py; }  /* make_navigation_grid, craft.py:450 */
      int ni = (nx * H + ny) * 4 + a;
      if (prev_state[ni] == -2) {
        if (end == 1000) { *overflow = 1; break; }    /* queue[end] IndexError */
        queue[end++] = ni;
        prev_state[ni] = item;
        prev_action[ni] = a;
      }
    }
    if (*overflow) break;
  }
  int rc = 0;
  if (found >= 0) {
    int n = 0, first = -1, it = found;
    while (prev_state[it] != -1) { first = prev_action[it]; it = prev_state[it]; ++n; }
    *first_action = first;
    *len = n;
    rc = 1;
  }
  free(prev_state);
  free(prev_action);
  return rc;
}

/* find_closest_resources, teachers/base.py:27-34 with find_resource_positions
 * (craft.py:453-455: np.nonzero order, x-major). */
int oracle_closest_resource(const craft_config_t* cfg, const oracle_env_t* s, int32_t kind,
                            int32_t* first_action, int32_t* path_len) {
  int have_best = 0, best_len = -1, best_first = -1;
  for (int x = 0; x < cfg->width; ++x)
    for (int y = 0; y < cfg->height; ++y) {
      if (cell(cfg, s, x, y) != kind) continue;
      int fa = -1, len = -1, overflow = 0;
      int ok = shortest_path(cfg, s, x, y, &fa, &len, &overflow);
      if (overflow) return CRAFT_ETEACHER;
      if (!have_best) {            /* best_goal[1] is None: take it, even a None path */
        if (ok) { have_best = 1; best_len = len; best_first = fa; }
      } else {
        if (!ok) return CRAFT_ETEACHER;          /* len(None): TypeError */
        if (len < best_len) { best_len = len; best_first = fa; }
      }
    }
  *first_action = have_best ? best_first : -1;
  *path_len = have_best ? best_len : -1;
  return CRAFT_OK;
}

/* BaseTeacher.find_incomplete_subtask, teachers/base.py:10-25.  Returns the
 * task id, -1 for None, -2 for the assertion at base.py:24. */
static int find_incomplete_subtask(const craft_config_t* cfg, const oracle_env_t* s, int task) {
  if (oracle_satisfies(cfg, s, task) == 1) return -1;
  const craft_task_t* t = &cfg->task[task];
  if (t->n_subtasks == 0) return task;
  for (int i = 0; i + 1 < t->n_subtasks; ++i) {
    int r = find_incomplete_subtask(cfg, s, t->subtask[i]);
    if (r == -2) return -2;
    if (r >= 0) return r;
  }
  int r = find_incomplete_subtask(cfg, s, t->subtask[t->n_subtasks - 1]);
  if (r == -1) return -2;
  return r;
}

/* DemonstrationTeacher.__call__, teachers/demonstration.py:9-30. */
int oracle_teacher(const craft_config_t* cfg, const oracle_env_t* s, int32_t task,
                   int32_t* action) {
  int sub = find_incomplete_subtask(cfg, s, task);
  if (sub == -2) return CRAFT_ETEACHER;
  if (sub == -1) { *action = CRAFT_STOP; return CRAFT_OK; }
  const craft_task_t* t = &cfg->task[sub];
  if (t->goal == CRAFT_GOAL_USE) { *action = CRAFT_USE; return CRAFT_OK; }
  if (t->goal != CRAFT_GOAL_GO) return CRAFT_ETEACHER;     /* demonstration.py:18 assert */
  int fa = -1, len = -1;
  int rc = oracle_closest_resource(cfg, s, t->arg_kind, &fa, &len);
  if (rc) return rc;
  if (len < 0) { *action = CRAFT_STOP; return CRAFT_OK; }  /* demonstration.py:25-26 */
  if (len == 0) return CRAFT_ETEACHER;                     /* best_action_seq[0] on [] */
  *action = fa;
  return CRAFT_OK;
}

static inline uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

int32_t oracle_hash_action(uint64_t seed, int64_t gid, int64_t tick) {
  uint64_t h = splitmix64(seed ^ ((uint64_t)gid << 20) ^ (uint64_t)tick);
  return (int32_t)((uint32_t)(h >> 32) % 6u);
}

/* CraftScenario.init, craft.py:268-273 (+ the trainer's timer reset). */
void oracle_reset(const craft_config_t* cfg, const uint8_t* pool, oracle_env_t* s) {
  const int C = cfg->width * cfg->height;
  memcpy(s->grid, pool + (size_t)s->scenario * C, (size_t)C);
  memset(s->inv, 0, sizeof(s->inv));
  s->x = s->x0;
  s->y = s->y0;
  s->dir = s->dir0;
  s->timer = cfg->max_timesteps;
  s->frozen = 0;
}

int oracle_batch_tick(const craft_config_t* cfg, const uint8_t* pool, oracle_env_t* envs,
                      int64_t n, int64_t env_id_base, const int32_t* actions, uint64_t seed,
                      int64_t tick, uint32_t flags, float* obs, float* reward, uint8_t* done,
                      int8_t* success, int64_t* stats) {
  int status = CRAFT_OK;
  for (int64_t e = 0; e < n; ++e) {
    oracle_env_t* s = &envs[e];
    int32_t a = actions ? actions[e] : oracle_hash_action(seed, env_id_base + e, tick);
    int d, succ = -1;
    float r = 0.0f;
    if (s->frozen) {                         /* done envs are not stepped (imitation.py:66-70) */
      d = 1;
      succ = oracle_satisfies(cfg, s, s->task);
    } else {
      s->timer -= 1;                                           /* imitation.py:63 */
      d = (a == CRAFT_STOP) || s->timer <= 0;                  /* imitation.py:64-65 */
      if (d) {
        succ = oracle_satisfies(cfg, s, s->task);              /* imitation.py:68-70 */
        r = succ == 1 ? 1.0f : 0.0f;
        if (stats) { stats[0] += succ == 1; stats[1] += 1; }
        if (flags & CRAFT_STEP_AUTORESET) oracle_reset(cfg, pool, s);
        else s->frozen = 1;
      } else {
        int rc = oracle_step(cfg, s, a);                       /* imitation.py:71-73 */
        if (rc && !status) status = rc;
      }
      if (stats) stats[2] += 1;
    }
    if (obs) oracle_features(cfg, s, obs + e * (int64_t)cfg->n_features);
    if (reward) reward[e] = r;
    if (done) done[e] = (uint8_t)d;
    if (success) success[e] = (int8_t)succ;
  }
  return status;
}

int64_t oracle_bench(const craft_config_t* cfg, const uint8_t* pool, oracle_env_t* envs,
                     int64_t n, int64_t env_id_base, int64_t tick0, int64_t ticks, uint64_t seed,
                     float* obs, int32_t ring, float* reward, uint8_t* done, int8_t* success,
                     int32_t* labels, int64_t* stats) {
  /* The GPU bench's work, tick for tick: the do_rollout protocol with hashed
   * actions keyed by global id, auto-reset, and every output written to its own
   * row (obs [n][F] in ring slot tick % ring, reward/done/success [n]) — the same
   * stores the GPU is charged for; with `labels`, the DemonstrationTeacher
   * (teachers/demonstration.py:9-30) of every env's new state too (config 5:
   * craft_step_teach), -1 for a frozen env, -2 where the reference raises. */
  const int64_t slot = n * (int64_t)cfg->n_features;
  for (int64_t t = 0; t < ticks; ++t) {
    float* o = obs ? obs + ((tick0 + t) % (ring > 0 ? ring : 1)) * slot : NULL;
    if (oracle_batch_tick(cfg, pool, envs, n, env_id_base, NULL, seed, tick0 + t,
                          CRAFT_STEP_AUTORESET, o, reward, done, success, stats))
      return -1;
    if (labels)
      for (int64_t e = 0; e < n; ++e) {
        int32_t a = -1;
        if (!envs[e].frozen && oracle_teacher(cfg, &envs[e], envs[e].task, &a)) a = -2;
        labels[e] = a;
      }
  }
  return n * ticks;
}

int oracle_sizeof_config(void) { return (int)sizeof(craft_config_t); }

/* ---- scenario generation (make_data.py:27-144) ------------------------------------------ */

typedef struct {
  int kind;               /* 0 splitmix64 per scenario, 1 numpy legacy MT19937 */
  uint64_t sm;
  uint32_t mt[624];
  int mti;
} gen_rng_t;

static void mt_seed(gen_rng_t* r, uint32_t s) {         /* init_genrand, as RandomState(int) */
  r->mt[0] = s;
  for (int i = 1; i < 624; ++i) r->mt[i] = 1812433253u * (r->mt[i - 1] ^ (r->mt[i - 1] >> 30)) + (uint32_t)i;
  r->mti = 624;
}

static uint32_t mt_next(gen_rng_t* r) {
  if (r->mti >= 624) {
    for (int i = 0; i < 624; ++i) {
      const uint32_t y = (r->mt[i] & 0x80000000u) | (r->mt[(i + 1) % 624] & 0x7fffffffu);
      r->mt[i] = r->mt[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
    r->mti = 0;
  }
  uint32_t y = r->mt[r->mti++];
  y ^= y >> 11;
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= y >> 18;
  return y;
}

static uint32_t sm_next32(gen_rng_t* r) {                /* the splitmix64 sequence, high half */
  r->sm += 0x9E3779B97F4A7C15ull;
  uint64_t z = r->sm;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return (uint32_t)((z ^ (z >> 31)) >> 32);
}

/* random.randint(n) */
static int gen_randint(gen_rng_t* r, int n) {
  if (r->kind == 1) {                                    /* numpy legacy: masked rejection */
    const uint32_t max = (uint32_t)(n - 1);
    if (max == 0) return 0;
    uint32_t mask = max;
    mask |= mask >> 1; mask |= mask >> 2; mask |= mask >> 4; mask |= mask >> 8; mask |= mask >> 16;
    uint32_t v;
    while ((v = mt_next(r) & mask) > max) {}
    return (int)v;
  }
  uint64_t m = (uint64_t)sm_next32(r) * (uint32_t)n;     /* Lemire: unbiased multiply-shift */
  uint32_t l = (uint32_t)m;
  if (l < (uint32_t)n) {
    const uint32_t t = (uint32_t)(-(uint32_t)n) % (uint32_t)n;
    while (l < t) {
      m = (uint64_t)sm_next32(r) * (uint32_t)n;
      l = (uint32_t)m;
    }
  }
  return (int)(m >> 32);
}

/* all_free_cells_reachable (make_data.py:27-72): FIFO BFS from init (or the first free cell,
 * x-major), moves into occupied cells blocked; every free cell reached? */
static int all_free_cells_reachable(const uint8_t* nav, int W, int H, int ix, int iy) {
  uint8_t seen[CRAFT_MAX_CELLS];
  int queue[1000];
  if (ix < 0) {
    for (int c = 0; c < W * H && ix < 0; ++c)
      if (!nav[c]) { ix = c / H; iy = c % H; }
  }
  memset(seen, 0, sizeof(seen));
  int start = 0, end = 0;
  queue[end++] = ix * H + iy;
  seen[ix * H + iy] = 1;
  while (start < end) {
    const int p = queue[start++];
    const int x = p / H, y = p % H;
    for (int a = 0; a < 4; ++a) {
      int nx = x + DX[a], ny = y + DY[a];
      if (nav[nx * H + ny]) { nx = x; ny = y; }
      const int q = nx * H + ny;
      if (!seen[q]) { seen[q] = 1; queue[end++] = q; }
    }
  }
  for (int c = 0; c < W * H; ++c)
    if (!nav[c] && !seen[c]) return 0;
  return 1;
}

/* random_free (make_data.py:74-103), keep_connected=True; nav is the occupancy image. */
static int random_free(gen_rng_t* r, uint8_t* nav, int W, int H, int* ox, int* oy) {
  for (int draws = 0; draws < (1 << 20); ++draws) {
    const int x = gen_randint(r, W), y = gen_randint(r, H);
    if (nav[x * H + y]) continue;
    nav[x * H + y] = 1;
    int good = all_free_cells_reachable(nav, W, H, -1, -1);
    for (int i = 0; good && i < W; ++i)
      for (int j = 0; good && j < H; ++j)
        if (nav[i * H + j] && 0 < i && i < W - 1 && 0 < j && j < H - 1 &&
            !all_free_cells_reachable(nav, W, H, i, j))
          good = 0;
    nav[x * H + y] = 0;
    if (good) { *ox = x; *oy = y; return 0; }
  }
  return -1;
}

static int sample_scenario(gen_rng_t* r, int W, int H, int boundary, const int32_t* prims, int n_prim,
                           int n_per, const int32_t* ws, int n_ws, uint8_t* grid, int32_t* init) {
  memset(grid, 0, (size_t)W * H);
  for (int x = 0; x < W; ++x)
    for (int y = 0; y < H; ++y)
      if (x == 0 || y == 0 || x == W - 1 || y == H - 1) grid[x * H + y] = (uint8_t)boundary;
  uint8_t nav[CRAFT_MAX_CELLS];
  int x, y;
  for (int c = 0; c < W * H; ++c) nav[c] = grid[c] != 0;
  for (int p = 0; p < n_prim; ++p)                                 /* ingredients */
    for (int i = 0; i < n_per; ++i) {
      if (random_free(r, nav, W, H, &x, &y)) return -1;
      grid[x * H + y] = (uint8_t)prims[p];
      nav[x * H + y] = 1;
    }
  for (int i = 0; i < n_ws; ++i) {                                 /* crafting stations */
    if (random_free(r, nav, W, H, &x, &y)) return -1;
    grid[x * H + y] = (uint8_t)ws[i];
    nav[x * H + y] = 1;
  }
  if (random_free(r, nav, W, H, &x, &y)) return -1;               /* init pos */
  init[0] = x;
  init[1] = y;
  return 0;
}

int oracle_generate_scenarios(int32_t W, int32_t H, int32_t boundary, const int32_t* prims,
                              int32_t n_prim, int32_t n_per, const int32_t* ws, int32_t n_ws,
                              int32_t rng_kind, uint64_t seed, int64_t id0, int32_t count,
                              int32_t dedup, uint8_t* grids_out, int32_t* init_out,
                              uint32_t* mt_state_out) {
  const int C = W * H;
  gen_rng_t r;
  memset(&r, 0, sizeof(r));
  r.kind = rng_kind;
  if (rng_kind == 1) mt_seed(&r, (uint32_t)seed);
  for (int s = 0; s < count; ++s) {
    uint8_t* g = grids_out + (size_t)s * C;
    if (rng_kind == 0) r.sm = seed ^ ((uint64_t)(id0 + s) * 0xD1B54A32D192ED03ull);
    for (;;) {
      if (sample_scenario(&r, W, H, boundary, prims, n_prim, n_per, ws, n_ws, g, init_out + 2 * s))
        return -1;
      int dup = 0;
      for (int t = 0; dedup && rng_kind == 1 && t < s && !dup; ++t)
        dup = memcmp(g, grids_out + (size_t)t * C, (size_t)C) == 0;
      if (!dup) break;
    }
  }
  if (mt_state_out && rng_kind == 1) {
    memcpy(mt_state_out, r.mt, sizeof(r.mt));
    mt_state_out[624] = (uint32_t)r.mti;
  }
  return 0;
}
