// craft_host.h — host-side pieces shared by the two implementations of include/craft.h: the
// HIP library (craft_sim.hip, libpsketch_craft.so) and its CPU variant (craft_cpu.cpp,
// libpsketch_craft_cpu.so, host pointers).  Plain C++: configuration checks, the packed task
// table, the scenario-grid checks of craft_pool_load and the status strings, so both libraries
// accept and refuse exactly the same inputs with the same messages.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/craft.h"

namespace craft_host {

// craft_sim_create's checks of a compiled craft_config_t (craft.py:59-109 tables).
inline int validate_config(const craft_config_t* c, std::string& msg) {
  if (c->abi_version != CRAFT_ABI_VERSION) { msg = "abi_version mismatch"; return CRAFT_EINVAL; }
  if (c->width < 3 || c->height < 3 || c->width > CRAFT_MAX_DIM || c->height > CRAFT_MAX_DIM ||
      c->width * c->height > CRAFT_MAX_CELLS) { msg = "WIDTH/HEIGHT out of range (3..16)"; return CRAFT_EINVAL; }
  if (c->window_width != c->window_height ||
      (c->window_width != 3 && c->window_width != 5 && c->window_width != 7)) {
    msg = "WINDOW_WIDTH == WINDOW_HEIGHT in {3,5,7} required"; return CRAFT_EINVAL;
  }
  if (c->n_kinds < 2 || c->n_kinds > CRAFT_MAX_KINDS) { msg = "n_kinds out of range"; return CRAFT_EINVAL; }
  const int ww = c->window_width;
  if (c->n_features != 2 * ww * ww * c->n_kinds + c->n_kinds + 5) {
    msg = "n_features != 2*ww*wh*n_kinds + n_kinds + 5 (craft.py:69-75)"; return CRAFT_EINVAL;
  }
  if (c->max_timesteps < 1 || c->max_timesteps > 255) { msg = "max_timesteps must be 1..255"; return CRAFT_EINVAL; }
  if (c->bridge_kind <= 0 || c->bridge_kind >= c->n_kinds || c->axe_kind <= 0 || c->axe_kind >= c->n_kinds) {
    msg = "bridge/axe kind out of range"; return CRAFT_EINVAL;
  }
  for (int k = 0; k < CRAFT_MAX_KINDS; ++k)
    if (c->kind_class[k] > CRAFT_KIND_STONE) { msg = "bad kind_class"; return CRAFT_EINVAL; }
  if (c->n_recipes < 0 || c->n_recipes > CRAFT_MAX_RECIPES) { msg = "n_recipes out of range"; return CRAFT_EINVAL; }
  for (int r = 0; r < c->n_recipes; ++r) {
    const craft_recipe_t& rc = c->recipe[r];
    if (rc.output <= 0 || rc.output >= c->n_kinds || rc.workshop <= 0 || rc.workshop >= c->n_kinds ||
        rc.n_inputs < 1 || rc.n_inputs > CRAFT_MAX_INGREDIENTS) { msg = "bad recipe"; return CRAFT_EINVAL; }
    if (rc.yield < 1 || rc.yield > 255) { msg = "recipe _yield outside 1..255"; return CRAFT_EINVAL; }
    for (int i = 0; i < rc.n_inputs; ++i)
      if (rc.input_kind[i] <= 0 || rc.input_kind[i] >= c->n_kinds || rc.input_count[i] < 1 ||
          rc.input_count[i] > 255) { msg = "bad recipe input"; return CRAFT_EINVAL; }
  }
  if (c->n_tasks < 1 || c->n_tasks > CRAFT_MAX_TASKS) { msg = "n_tasks out of range"; return CRAFT_EINVAL; }
  for (int t = 0; t < c->n_tasks; ++t) {
    const craft_task_t& tk = c->task[t];
    if (tk.goal < CRAFT_GOAL_OTHER || tk.goal > CRAFT_GOAL_USE || tk.arg_kind < 0 ||
        tk.arg_kind >= c->n_kinds || tk.n_subtasks < 0 || tk.n_subtasks > CRAFT_MAX_SUBTASKS) {
      msg = "bad task"; return CRAFT_EINVAL;
    }
    if ((tk.goal == CRAFT_GOAL_GET || tk.goal == CRAFT_GOAL_MAKE || tk.goal == CRAFT_GOAL_GO) && tk.arg_kind == 0) {
      msg = "get/make/go task without a kind argument"; return CRAFT_EINVAL;
    }
    for (int s = 0; s < tk.n_subtasks; ++s)
      if (tk.subtask[s] < 0 || tk.subtask[s] >= c->n_tasks) { msg = "bad subtask id"; return CRAFT_EINVAL; }
  }
  return CRAFT_OK;
}

// craft_strerror's text for each status.
inline const char* status_text(int status) {
  switch (status) {
    case CRAFT_OK: return "ok";
    case CRAFT_EINVAL: return "invalid argument";
    case CRAFT_EBADACTION: return "Unexpected action";
    case CRAFT_EINVARIANT: return "impossible world configuration";
    case CRAFT_ETEACHER: return "teacher assertion";
    case CRAFT_EHIP: return "HIP runtime error";
    case CRAFT_ENOMEM: return "out of memory";
    case CRAFT_ERANGE: return "index out of range";
    default: return "unknown status";
  }
}

// The task table both libraries' kernels read: tab[t] = goal | arg_kind << 4 | n_subtasks << 12,
// sub[t][q] = subtask ids in hint order (data/task.py:32-75).
inline void task_tables(const craft_config_t& cfg, uint16_t* tab, int32_t* sub) {
  for (int t = 0; t < CRAFT_MAX_TASKS; ++t) {
    tab[t] = 0;
    for (int q = 0; q < CRAFT_MAX_SUBTASKS; ++q) sub[CRAFT_MAX_SUBTASKS * t + q] = 0;
  }
  for (int t = 0; t < cfg.n_tasks; ++t) {
    const craft_task_t& tk = cfg.task[t];
    tab[t] = (uint16_t)(tk.goal | (tk.arg_kind << 4) | (tk.n_subtasks << 12));
    for (int q = 0; q < tk.n_subtasks; ++q) sub[CRAFT_MAX_SUBTASKS * t + q] = tk.subtask[q];
  }
}

// ---- the hint walk, tabulated (craft_rollout_teach's teacher wave) ---------------------------
// hint_leaf (craft_teach.h: find_incomplete_subtask, teachers/base.py:10-25, and the leaf's
// action, demonstration.py:12-30) reads satisfies() (craft.py:285-294) of nodes reachable from the
// task, and each node's is one predicate: get/make X -> inventory[X] > 0, go X -> the facing cell
// is X, any other goal -> never satisfied.  For a task with at most kHintPreds distinct predicates
// the leaf is a function of their truth values alone; hint_tables evaluates hint_leaf's walk for
// every combination.  desc[4t], desc[4t+1]: predicate j in byte j (bit 7 used, bit 6 a facing
// test, else an inventory test, bits 0-5 the kind); desc[4t+2]: the byte offset of the task's
// 2^P leaves, or kHintWalk (more predicates, or past kHintLeafCap bytes: the kernel walks).
// Leaf byte: a go[] kind, kHintStop, kHintUse or kHintErr (the reference raises).
constexpr int kHintPreds = 8, kHintLeafCap = 2048;
constexpr uint8_t kHintErr = 0xff, kHintStop = 0xfe, kHintUse = 0xfd;
constexpr uint32_t kHintWalk = 1u << 31;
inline void hint_tables(const craft_config_t& cfg, const uint16_t* tab, const int32_t* sub, uint32_t* desc,
                        std::vector<uint8_t>& leaf) {
  leaf.clear();
  auto key = [&](int t) -> int {                 // the node's predicate: kind | 0x40 facing; -1 none
    const int goal = tab[t] & 0xf, arg = (tab[t] >> 4) & 0xff;
    if (goal == CRAFT_GOAL_GET || goal == CRAFT_GOAL_MAKE) return arg & 0x3f;
    if (goal == CRAFT_GOAL_GO) return 0x40 | (arg & 0x3f);
    return -1;
  };
  for (int t = 0; t < CRAFT_MAX_TASKS; ++t) {
    desc[4 * t] = desc[4 * t + 1] = desc[4 * t + 3] = 0;
    desc[4 * t + 2] = kHintWalk;
    if (t >= cfg.n_tasks) continue;
    int keys[CRAFT_MAX_TASKS], nk = 0;
    bool seen[CRAFT_MAX_TASKS] = {};
    int stack[CRAFT_MAX_TASKS], top = 0;
    stack[top++] = t;
    seen[t] = true;
    while (top) {                                // every node reachable from t
      const int node = stack[--top];
      const int k = key(node);
      bool have = k < 0;
      for (int i = 0; i < nk && !have; ++i) have = keys[i] == k;
      if (!have) keys[nk++] = k;
      const int ns = (tab[node] >> 12) & 0xf;
      for (int q = 0; q < ns && q < CRAFT_MAX_SUBTASKS; ++q) {
        const int c = sub[CRAFT_MAX_SUBTASKS * node + q];
        if (c >= 0 && c < CRAFT_MAX_TASKS && !seen[c]) { seen[c] = true; stack[top++] = c; }
      }
    }
    if (nk > kHintPreds || leaf.size() + ((size_t)1 << nk) > (size_t)kHintLeafCap) continue;
    for (int j = 0; j < nk; ++j) desc[4 * t + (j >> 2)] |= (0x80u | (uint32_t)keys[j]) << (8 * (j & 3));
    desc[4 * t + 2] = (uint32_t)leaf.size();
    for (uint32_t bits = 0; bits < (1u << nk); ++bits) {
      auto sat = [&](int node) -> int {
        const int k = key(node);
        if (k < 0) return -1;
        for (int j = 0; j < nk; ++j)
          if (keys[j] == k) return (int)((bits >> j) & 1u);
        return -1;
      };
      // hint_leaf's walk, statement for statement
      uint8_t out;
      if (sat(t) == 1) {
        out = kHintStop;
      } else {
        int node = t;
        bool raised = false;
        for (int guard = 0; guard < CRAFT_MAX_TASKS; ++guard) {
          const int ns = (tab[node] >> 12) & 0xf;
          if (ns == 0) break;
          const int32_t* sb = sub + CRAFT_MAX_SUBTASKS * node;
          int chosen = sb[ns - 1];
          bool last = true;
          for (int q = 0; q + 1 < ns; ++q)
            if (sat(sb[q]) != 1) { chosen = sb[q]; last = false; break; }
          if (last && sat(chosen) == 1) { raised = true; break; }
          node = chosen;
        }
        const int goal = tab[node] & 0xf;
        out = raised ? kHintErr
            : goal == CRAFT_GOAL_USE ? kHintUse
            : goal == CRAFT_GOAL_GO ? (uint8_t)((tab[node] >> 4) & 0xff)
            : kHintErr;
      }
      leaf.push_back(out);
    }
  }
}

// craft_pool_load's checks of one scenario grid g (W*H kind ids, x-major), pool row `index`:
// kind ids in range, and a border ring of inert, non-target kinds (make_data.py:108-112 fills
// it with `boundary`; the kernels never index past it, and the teacher's band-layout BFS leaves
// columns 0 and W-1 out).  *conn = 1 when the free cells form one 4-connected component (cells
// are only ever cleared next to the agent, so every env grid of the scenario keeps that, and
// the teacher reads reachability off the grid instead of flooding it).
inline int check_pool_grid(const craft_config_t& cfg, const uint8_t* g, int64_t index, std::string& msg,
                           uint8_t* conn) {
  const int W = cfg.width, H = cfg.height, C = W * H;
  uint32_t border_ok = 0;
  for (int k = 1; k < cfg.n_kinds && k < 32; ++k)
    if (cfg.kind_class[k] == CRAFT_KIND_INERT) border_ok |= 1u << k;
  for (int t = 0; t < cfg.n_tasks; ++t)
    if (cfg.task[t].arg_kind > 0 && cfg.task[t].arg_kind < 32) border_ok &= ~(1u << cfg.task[t].arg_kind);
  for (int c = 0; c < C; ++c) {
    if (g[c] >= cfg.n_kinds) {
      msg = "craft_pool_load: kind id out of range in grid " + std::to_string(index);
      return CRAFT_EINVARIANT;
    }
    const int x = c / H, y = c % H;
    if ((x == 0 || y == 0 || x == W - 1 || y == H - 1) && !((border_ok >> g[c]) & 1u)) {
      msg = "craft_pool_load: grid " + std::to_string(index) + " border cell (" + std::to_string(x) + ", " +
            std::to_string(y) + ") holds kind " + std::to_string(g[c]) +
            ": the ring must be occupied by inert, non-target kinds (make_data.py:108-112 builds a boundary ring)";
      return CRAFT_EINVARIANT;
    }
  }
  std::vector<int> stack;
  std::vector<uint8_t> seen(C, 0);
  int n_free = 0, first_free = -1;
  for (int c = 0; c < C; ++c)
    if (g[c] == 0) { ++n_free; if (first_free < 0) first_free = c; }
  int n_seen = 0;
  if (first_free >= 0) { stack.push_back(first_free); seen[first_free] = 1; }
  while (!stack.empty()) {
    const int c = stack.back();
    stack.pop_back();
    ++n_seen;
    const int x = c / H, y = c % H;
    const int nb[4][2] = {{x, y - 1}, {x, y + 1}, {x - 1, y}, {x + 1, y}};
    for (auto& q : nb) {
      if (q[0] < 0 || q[0] >= W || q[1] < 0 || q[1] >= H) continue;
      const int d = q[0] * H + q[1];
      if (!seen[d] && g[d] == 0) { seen[d] = 1; stack.push_back(d); }
    }
  }
  *conn = n_seen == n_free ? 1 : 0;
  return CRAFT_OK;
}

}  // namespace craft_host
