"""TEST INFRASTRUCTURE ONLY — ImitationTrainer.do_rollout restated over the C oracle.

trainers/imitation.py:18-101, one env at a time, with the oracle's
CraftState.step / satisfies / features (craft_oracle.c) and its
DemonstrationTeacher (oracle_teacher, oracle_closest_resource).  The student is
a callable `act(obs, t) -> actions` over the stacked features (the reference's
student.act(states) stacks state.features(), students/imitation.py); the
behaviour-cloning draw (imitation.py:39-41) is passed in as `bc_mask`.

Pinned by tests/golden/imitation_rollout.npz, which the reference's own
do_rollout produced (tests/golden/make_golden.py gen_imitation).
"""
import numpy as np

GOAL_GET = 1          # include/craft.h CRAFT_GOAL_GET
STOP = 5


class ReferenceError_(Exception):
    """Raised where the reference raises (teacher assertion, len(None), bad action)."""


def do_rollout(oracle, spec, act, is_eval, bc_mask=None, max_timesteps=40):
    """spec: int32 [n, 5] (scenario, x0, y0, dir0, task) over oracle.pool.
    Returns the reference's info dict plus 'received' (student.receive calls)."""
    spec = np.asarray(spec, dtype=np.int32)
    n = len(spec)
    cfg = oracle.cfg
    envs = oracle.init_envs(spec[:, 0], spec[:, 1], spec[:, 2], spec[:, 3], spec[:, 4])
    tasks = [int(t) for t in spec[:, 4]]
    timer = [max_timesteps] * n                                   # imitation.py:29
    done = [False] * n
    success = [False] * n
    action_seqs = [[] for _ in range(n)]
    num_interactions = num_steps = 0
    received = []
    t = 0
    while not all(done):                                          # imitation.py:42
        obs = np.stack([oracle.features(envs[i:i + 1]) for i in range(n)])
        actions = [int(a) for a in act(obs, t)]
        ref_actions = [None] * n
        for i in range(n):
            e = envs[i:i + 1]
            if not is_eval:                                       # imitation.py:49-57
                if done[i]:
                    ref_actions[i] = -1
                else:
                    rc, a = oracle.teacher(e, tasks[i])
                    if rc:
                        raise ReferenceError_(f"teacher raises for env {i}")
                    ref_actions[i] = a
                    num_interactions += 1
                if bc_mask[i]:
                    actions[i] = ref_actions[i]
            if not done[i]:
                action_seqs[i].append(actions[i])
            timer[i] -= 1
            done[i] |= actions[i] == STOP or timer[i] <= 0
            if done[i]:                                           # imitation.py:66-73
                s = oracle.satisfies(e, tasks[i])
                if s < 0:
                    raise ReferenceError_("satisfies() is None")
                success[i] = bool(s)
            else:
                if oracle.step(e, actions[i]):
                    raise ReferenceError_(f"Unexpected action {actions[i]}")
                num_steps += (not is_eval)
        if not is_eval:
            received.append(ref_actions)
        t += 1
    distances = []                                                # imitation.py:79-91
    for i in range(n):
        task = cfg.task[tasks[i]]
        if task.goal != GOAL_GET:
            continue
        if success[i]:
            distances.append(0)
            continue
        sc, x0, y0, d0, tk = spec[i]
        probe = oracle.env(oracle.pool[sc], envs["x"][i], envs["y"][i], envs["dir"][i], task=tk)
        rc, _, ln = oracle.closest_resource(probe, task.arg_kind)
        if rc or ln < 0:
            raise ReferenceError_("find_closest_resources: len(None)")
        distances.append(ln)
    return {"action_seqs": action_seqs, "success": success, "distances": distances,
            "num_interactions": num_interactions, "num_steps": num_steps, "received": received}


def fake_policy(W, bias):
    """The deterministic integer student of tests/golden/imitation_rollout.npz."""
    W = np.asarray(W, dtype=np.int64)
    bias = np.asarray(bias, dtype=np.int64)

    def act(obs, t):
        scores = np.asarray(obs).astype(np.int64) @ W[t % len(W)] * 8 + bias
        return scores.argmax(axis=1)
    return act


def teach_rollout(oracle, envs, gids, n_ticks, seed=0, tick0=0, actions=None, autoreset=True,
                  label_in=None, label_src=None, want_obs=False):
    """craft_rollout_teach restated over the C oracle, one env at a time: each tick the action of
    env i is its current label when label_src[i] (make_data.get_reference_actions,
    make_data.py:146-152; behaviour cloning, trainers/imitation.py:56-57), else actions[k][i] or
    the hashed draw of its global id gids[i]; then the tick (oracle_batch_tick) and the
    DemonstrationTeacher of the new state (-1 for a frozen env, -2 where the reference raises).
    envs: oracle envs (modified in place).  Returns per-tick arrays [n_ticks, n]: labels,
    action_record (-1 for an env already done), done, success; with want_obs also obs
    [n_ticks, n, F] (float32, features() of each env's state after the tick)."""
    import oracle as O
    n = len(envs)
    gids = np.asarray(gids, dtype=np.int64)
    src = np.zeros(n, dtype=bool) if label_src is None else np.asarray(label_src, dtype=bool)
    cur = np.zeros(n, dtype=np.int32) if label_in is None else np.asarray(label_in, dtype=np.int32).copy()
    out = {k: np.zeros((n_ticks, n), dtype=dt) for k, dt in
           (("labels", np.int32), ("action_record", np.int32), ("done", np.uint8), ("success", np.int8))}
    obs = [] if want_obs else None
    for k in range(n_ticks):
        t = tick0 + k
        a = np.empty(n, dtype=np.int32)
        for i in range(n):
            if src[i]:
                a[i] = cur[i]
            elif actions is not None:
                a[i] = actions[k][i]
            else:
                a[i] = O.hash_action(seed, int(gids[i]), t)
        frozen = envs["frozen"].copy()
        rows = []
        for i in range(n):
            rc, ob, _, d, s = oracle.batch_tick(envs[i:i + 1], int(gids[i]), a[i:i + 1], seed, t, autoreset,
                                               want_obs=want_obs)
            if rc:
                raise ReferenceError_(f"step raises for env {i} at tick {t}")
            out["done"][k, i] = d[0]
            out["success"][k, i] = s[0]
            if want_obs:
                rows.append(np.asarray(ob, dtype=np.float32).reshape(-1))
        if want_obs:
            obs.append(np.stack(rows))
        out["action_record"][k] = np.where(frozen != 0, -1, a)
        for i in range(n):
            if envs["frozen"][i]:
                cur[i] = -1
            else:
                rc, lab = oracle.teacher(envs[i:i + 1], int(envs["task"][i]))
                cur[i] = -2 if rc else lab
        out["labels"][k] = cur
    if want_obs:
        out["obs"] = np.stack(obs)
    return out
