"""Batched ImitationTrainer.do_rollout on the GPU (trainers/imitation.py:18-101).

The reference rolls a batch out one env at a time in Python: per tick,
student.act(states) over stacked features(), the DemonstrationTeacher for each
live env, the behaviour-cloning substitution, the timer/STOP protocol, step.
Here the whole batch lives in CraftSim slots and every per-env part of a tick is
a kernel on the current stream:

  craft_teacher           ref_actions, -1 for done (frozen) envs      (imitation.py:47-55)
  craft_step_ex           bc ? ref : student (imitation.py:56-57), action_seqs row
                          (:59-61), timer/STOP/satisfies/step + features (:63-73),
                          and an any-env-still-running flag (:42)

The student sees the features as a device tensor and returns device actions;
nothing crosses PCIe inside the loop except the all(done) test (imitation.py:42):
the step kernels store each tick's any-live flag straight into page-locked host
memory, which the host reads once the tick's event has completed.  After the loop, one
launch (craft_rollout_distances) computes every env's `distances` entry (imitation.py:79-91:
failed get tasks search their initial grid from their final pose with
find_closest_resources' BFS), is_get and action count, and the summary comes back in one
transfer.
"""
import ctypes
import inspect
import time
import weakref

import numpy as np
import torch

from . import _native as N
from .sim import CraftSim



class RolloutError(Exception):
    """Raised where the reference's do_rollout raises (TypeError/AssertionError)."""


class RolloutInfo:
    """do_rollout's `info` as device tensors.

    action_seqs int32 [T, n] (-1 after an env's last action), n_actions int32 [n],
    success int8 [n], distances int32 [n] (-1 where the task is not a get task),
    is_get bool [n], num_interactions / num_steps ints, ticks, and obs
    ([T+1, n, F], every observation the student saw) when kept."""

    def __init__(self, **kw):
        self.__dict__.update(kw)

    def to_reference(self):
        """The reference's info dict (python lists, trainers/imitation.py:93-99)."""
        A = self.action_seqs.t().cpu().numpy()
        L = self.n_actions.cpu().numpy()
        succ = self.success.cpu().numpy()
        dist = self.distances.cpu().numpy()
        is_get = self.is_get.cpu().numpy()
        return {
            "action_seqs": [[int(a) for a in A[i, :L[i]]] for i in range(len(L))],
            "success": [bool(s) for s in succ],
            "distances": [int(d) for d, g in zip(dist, is_get) if g],
            "num_interactions": int(self.num_interactions),
            "num_steps": int(self.num_steps),
        }


def do_rollout(sim, spec, act, is_eval, behavior_clone=None, receive=None, keep_obs=False,
               timing=None, fused_teacher=True, lookahead=False, graph=0, graph_key=None):
    """One rollout of sim.n_envs episodes.

    spec: (scenario, x, y, dir, task), each n_envs ints (device or host).
    act(obs, t) -> int device tensor [n]: the student (students/imitation.py act);
      obs is [n, F] on the device in the simulator's obs format (fp32 unless
      sim.set_obs_format) and is overwritten by the next step unless keep_obs.
    behavior_clone: [n] 0/1 (config.random.binomial(1, policy_mix_rate, n),
      imitation.py:39-41); ignored when is_eval.
    receive(ref_actions) is called once per tick when not is_eval
      (student.receive, imitation.py:75-77) with the int32 device tensor.
    timing: optional dict; receives host wall seconds of the setup, the tick
      loop and the distances/summary phases (each ends at a device sync).
    fused_teacher: when not is_eval, each tick's step also labels the new states
      (craft_step_teach: the next tick's ref_actions, in the same launch);
      False runs craft_teacher on a side stream, overlapping the student (with graph=G the
      fork and join are captured in the graphs: the teacher of tick t's states beside act(t),
      then craft_step_ex).
    lookahead: the all(done) test of tick t (imitation.py:42) no longer blocks the
      host before tick t + 1 is queued: tick t + 1 (act and step) is queued behind tick
      t's event, and only then is tick t's any-live flag read.  When tick t ended every episode the queued tick is discarded: its step
      is a no-op on frozen envs (no state, counter, success or action-record change that
      the result keeps), but act was called once more than the reference calls it, so
      lookahead is for side-effect-free students (a fixed or deterministic policy);
      receive() is still called exactly once per real tick.  Needs is_eval or the fused
      teacher.
    graph: G > 0 runs the ticks as HIP graphs of G ticks each (act + step per tick, captured
      with torch.cuda.graph on the first call for this simulator and this `act`, replayed by
      later calls), so the per-tick host work (the student's launches, the step's ctypes call)
      leaves the loop.  The conditions of lookahead apply, and more: act only queues device work
      on the current stream, with fixed shapes and no host synchronisation, and its device
      inputs stay where they were at capture (weights may change in place).  Chunk c + 1 is
      queued before chunk c's flags are read; ticks after the one that ended every episode are
      no-ops and are discarded.  The rollout's buffers are the simulator's own: the results are
      copies, and receive() is called once per real tick after the loop, in tick order, with
      rows of a copy of the labels.  Not with keep_obs.
    graph_key: a hashable naming what the captured graphs read besides the simulator (the
      student's state); the graphs are reused only while act is the same callable and the key is
      equal, and captured anew otherwise.  A student that re-allocates a tensor act reads (a
      new weight tensor instead of an in-place update) must change the key, e.g.
      tuple(p.data_ptr() for p in model.parameters()), or call drop_graphs(sim): a replay would
      read the old allocation.
    """
    if graph:
        return _graph_rollout(sim, spec, act, is_eval, behavior_clone, receive, keep_obs, timing,
                              fused_teacher, int(graph), graph_key)
    t_start = time.perf_counter()
    n, dev, T = sim.n_envs, sim.device, sim.config.max_timesteps
    if T <= 0:
        raise ValueError("max_timesteps must be positive")
    spec = [sim._i32(a, n) for a in spec]
    task = spec[4]
    obs_hist = (torch.empty((T + 1, n, sim.n_features), dtype=sim.obs_dtype, device=dev)
                if keep_obs else None)
    obs = obs_hist[0] if keep_obs else sim.empty_obs()
    sim.reset(*spec, obs=obs)
    success = torch.zeros(n, dtype=torch.int8, device=dev)
    seqs = torch.full((T, n), -1, dtype=torch.int32, device=dev)
    # any-live flags (1: some env still running after tick t), one per tick: page-locked host
    # memory the kernel stores into directly where HIP maps it (read after the tick's event),
    # else a device array copied back per tick
    flags, flag_dev, events = _live_flags(sim, T)
    live = None if flag_dev else torch.zeros(T + 1, dtype=torch.int32, device=dev)
    # ref_actions of every tick: tick t reads refs[t] and (fused) labels refs[t + 1]; receive()
    # gets the row itself (no copy), which no later tick or rollout overwrites
    refs = None if is_eval else torch.empty((T + 1, n), dtype=torch.int32, device=dev)
    bc = None if is_eval else _bc_mask(behavior_clone, n, dev)
    fused = not is_eval and fused_teacher
    if lookahead and not is_eval and not fused_teacher:
        raise ValueError("lookahead needs is_eval or fused_teacher")
    # The teacher reads only the env states, so without the fused teacher tick t's labels are
    # computed on a side stream while the student's act(t) runs on the main stream.
    main = torch.cuda.current_stream(dev)
    side = None
    if not is_eval and not fused_teacher:
        side = getattr(sim, "_teacher_stream", None)
        if side is None:                         # created once per simulator (costly)
            side = sim._teacher_stream = torch.cuda.Stream(dev)
    labels_ready = getattr(sim, "_teacher_event", None)
    if labels_ready is None:
        labels_ready = sim._teacher_event = torch.cuda.Event()

    def launch_teacher(t):
        side.wait_stream(main)                   # after the previous step
        with torch.cuda.stream(side):
            sim.teacher(action_out=refs[t])      # done (frozen) envs get -1
        labels_ready.record(side)

    step = _stepper(sim, fused, bc, success)
    cur = {"obs": obs}

    def issue(t):
        """Tick t on the stream: the student's act, then one step launch (behaviour cloning, the
        action record, the any-live flag and, fused, the next tick's labels), then the flag's
        event (after the flag's copy to the host where it is not mapped)."""
        actions = act(cur["obs"], t)
        if not torch.is_tensor(actions):
            actions = torch.as_tensor(np.asarray(actions), device=dev)
        actions = actions.to(device=dev, dtype=torch.int32).reshape(n).contiguous()
        if side is not None:
            main.wait_event(labels_ready)
        if keep_obs:
            cur["obs"] = obs_hist[t + 1]
        step(t, actions, cur["obs"], None if is_eval else refs[t], seqs[t],
             flag_dev + 4 * t if flag_dev else live[t].data_ptr(), refs[t + 1] if fused else None)
        if side is not None and t + 1 < T:
            launch_teacher(t + 1)                # speculative: all -1 if every env is done
        if not flag_dev:
            flags[t:t + 1].copy_(live[t:t + 1], non_blocking=True)
        events[t].record()

    if not is_eval:
        if fused_teacher:
            sim.teacher(action_out=refs[0])      # the initial states' labels; then every step's
        else:
            launch_teacher(0)
    t_loop = time.perf_counter()
    # every env is done once its timer reaches 0 (imitation.py:42, 62-63): tick t's flag is read
    # after its event; with lookahead, tick t + 1 is queued first (and discarded if every
    # episode ended at tick t)
    issue(0)
    t = 0
    while True:
        if lookahead and t + 1 < T:
            issue(t + 1)
        events[t].synchronize()
        if not is_eval and receive is not None:
            receive(refs[t])                     # tick t is real
        t += 1
        if t >= T or int(flags[t - 1]) == 0:
            break
        if not lookahead:
            issue(t)
    if side is not None:
        main.wait_stream(side)
    t_end_loop = time.perf_counter()
    return _finish(sim, task, success, seqs, t, is_eval, keep_obs, obs_hist, timing, t_start,
                   t_loop, t_end_loop, dev)


def _stepper(sim, teach, bc, success):
    """do_rollout's per-tick craft_step_ex / craft_step_teach (include/craft.h) with the argument
    struct built once: a tick sets only its pointers and the tick number (every buffer is one
    do_rollout allocated and shaped itself, or the student's int32 [n] actions)."""
    args = N.craft_step_args_t()
    args.flags = 0                                         # no auto-reset: done envs freeze
    if bc is not None:
        args.behavior_clone = bc.data_ptr()
    args.success = success.data_ptr()
    lib = N.lib()
    fn = lib.craft_step_teach if teach else lib.craft_step_ex
    h, pargs, di = sim._h, ctypes.byref(args), sim.device.index
    raw = torch._C._cuda_getCurrentRawStream

    def step(t, actions, obs, ref, rec, live_ptr, labels):
        args.actions = actions.data_ptr()
        args.tick = t
        args.obs = obs.data_ptr()
        args.ref_actions = None if ref is None else ref.data_ptr()
        args.action_record = rec.data_ptr()
        args.any_live = live_ptr
        st = fn(h, pargs, labels.data_ptr(), raw(di)) if teach else fn(h, pargs, raw(di))
        if st:
            N.check(st, h, "craft_step_teach" if teach else "craft_step_ex")
    return step


def _bc_mask(behavior_clone, n, dev):
    if behavior_clone is None:
        raise ValueError("behavior_clone is required when not is_eval")
    bc = torch.as_tensor(np.asarray(behavior_clone) if not torch.is_tensor(behavior_clone)
                         else behavior_clone, device=dev)
    if bc.numel() != n:
        raise ValueError(f"behavior_clone has {bc.numel()} entries, expected {n}")
    return (bc.reshape(n) != 0).to(torch.uint8).contiguous()


def drop_graphs(sim):
    """Forget the HIP graphs do_rollout(graph=G) captured for `sim` (the next graph rollout
    captures again): after the student re-allocated a tensor its act reads."""
    sim._graph_state = None


def _graph_rollout(sim, spec, act, is_eval, behavior_clone, receive, keep_obs, timing,
                   fused_teacher, G, graph_key=None):
    """do_rollout(graph=G): see do_rollout."""
    t_start = time.perf_counter()
    n, dev, T = sim.n_envs, sim.device, sim.config.max_timesteps
    if keep_obs:
        raise ValueError("graph mode does not keep observations (keep_obs)")
    if G < 1:
        raise ValueError("graph: ticks per graph must be positive")
    if T <= 0:
        raise ValueError("max_timesteps must be positive")
    spec = [sim._i32(a, n) for a in spec]
    task = spec[4]
    flags, flag_dev, events = _live_flags(sim, T)
    if not flag_dev:
        raise RuntimeError("graph mode needs the any-live flags in mapped host memory")
    gs = getattr(sim, "_graph_state", None)
    side_teacher = not is_eval and not fused_teacher
    key = (is_eval, G, T, graph_key, side_teacher)
    if gs is None or not _same_act(gs["act"], act) or gs["key"] != key:
        sim._graph_state = None                  # drop the old graphs before capturing new ones
        gs = sim._graph_state = {
            "act": _weak_act(act), "key": key, "graphs": [],
            "obs": sim.empty_obs(), "success": torch.zeros(n, dtype=torch.int8, device=dev),
            "seqs": torch.full((T, n), -1, dtype=torch.int32, device=dev),
            "refs": None if is_eval else torch.empty((T + 1, n), dtype=torch.int32, device=dev),
            "bc": None if is_eval else torch.zeros(n, dtype=torch.uint8, device=dev)}
    obs, success, seqs, refs = gs["obs"], gs["success"], gs["seqs"], gs["refs"]
    sim.reset(*spec, obs=obs)
    success.zero_()
    # (every tick writes its whole action-record row; rows past the last tick are filled after
    # the loop, usually none)
    if not is_eval:
        gs["bc"].copy_(_bc_mask(behavior_clone, n, dev))
        sim.teacher(action_out=refs[0])          # the initial states' labels; then every step's
    nch = (T + G - 1) // G
    if not gs["graphs"]:
        step = _stepper(sim, not is_eval and not side_teacher, gs["bc"], success)
        main = torch.cuda.current_stream(dev)
        side = None
        if side_teacher:                         # created once per simulator (costly)
            side = getattr(sim, "_teacher_stream", None)
            if side is None:
                side = sim._teacher_stream = torch.cuda.Stream(dev)

        def issue(t):
            # (side teacher) tick t's ref_actions, the labels of the states tick t - 1 left, on a
            # forked stream beside the student's act(t); the step joins it (tick 0's come from
            # the eager call before the loop)
            cur = torch.cuda.current_stream(dev)    # (the capture's stream)
            if side is not None and t > 0:
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    sim.teacher(action_out=refs[t])
            actions = act(obs, t)
            actions = actions.to(device=dev, dtype=torch.int32).reshape(n).contiguous()
            if side is not None and t > 0:
                cur.wait_stream(side)
            step(t, actions, obs, None if is_eval else refs[t], seqs[t], flag_dev + 4 * t,
                 None if is_eval or side is not None else refs[t + 1])

        warm = torch.cuda.Stream(dev)            # the student's libraries warmed off the capture
        warm.wait_stream(main)
        with torch.cuda.stream(warm):
            act(obs, 0)
        main.wait_stream(warm)
        pool = None
        graphs = []                              # cached only once every chunk is captured
        try:
            for c in range(nch):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, pool=pool):
                    for t in range(c * G, min(T, (c + 1) * G)):
                        issue(t)
                pool = g.pool()
                graphs.append(g)
        except BaseException:
            sim._graph_state = None              # a failed capture leaves nothing behind
            raise
        gs["graphs"] = graphs
    graphs = gs["graphs"]
    t_loop = time.perf_counter()
    graphs[0].replay()
    events[0].record()
    ticks = None
    c = 0
    while ticks is None:
        if c + 1 < nch:                          # queued before chunk c's flags are read
            graphs[c + 1].replay()
            events[c + 1].record()
        events[c].synchronize()
        for t in range(c * G, min(T, (c + 1) * G)):
            if int(flags[t]) == 0:               # every episode ended at tick t (imitation.py:42)
                ticks = t + 1
                break
        c += 1
        if ticks is None and c >= nch:
            ticks = T
    if ticks < T:
        seqs[ticks:].fill_(-1)
    if not is_eval and receive is not None:
        labels = refs[:ticks].clone()
        for t in range(ticks):
            receive(labels[t])
    t_end_loop = time.perf_counter()
    return _finish(sim, task, success.clone(), seqs.clone(), ticks, is_eval, False, None, timing,
                   t_start, t_loop, t_end_loop, dev)


def _weak_act(act):
    """A weak reference to the student's act for the graph cache, so the cache does not keep the
    model alive (WeakMethod for a bound method: `student.act` is a new object on every access;
    a plain strong reference for callables that take no weak references)."""
    try:
        return weakref.WeakMethod(act) if inspect.ismethod(act) else weakref.ref(act)
    except TypeError:
        return lambda: act


def _same_act(ref, act):
    """Whether the cached graphs were captured for this act: equality, which bound methods
    define as the same function on the same object."""
    cached = ref()
    return cached is not None and cached == act


def _live_flags(sim, T):
    """The per-tick any-live flags of do_rollout: a page-locked host int32 array (zeroed here,
    reused across rollouts: the previous rollout's ticks have completed when it returned), its
    device address (craft_host_flag_pointer) or 0 where HIP does not map it, and one event per
    tick."""
    flags = getattr(sim, "_live_host", None)
    if flags is None or flags.numel() < T + 1:
        flags = sim._live_host = torch.zeros(max(T + 1, 64), dtype=torch.int32, pin_memory=True)
        sim._live_events = [torch.cuda.Event() for _ in range(flags.numel())]
        p = ctypes.c_void_p()
        ok = N.lib().craft_host_flag_pointer(flags.data_ptr(), ctypes.byref(p)) == 0
        sim._live_dev = p.value if ok and p.value else 0
    flags[:T + 1].zero_()
    return flags, sim._live_dev, sim._live_events


def _finish(sim, task, success, seqs, t, is_eval, keep_obs, obs_hist, timing, t_start, t_loop,
            t_end_loop, dev):
    """The rollout's summary (imitation.py:79-99) with one read-back: one launch computes every
    env's distance (failed get tasks: find_closest_resources' length on the initial grid at the
    final pose), is_get and action count (craft_rollout_distances); then the episode counters,
    the None-success and unreachable-target flags and the latched-error word come back in one
    transfer."""
    n = sim.n_envs
    task = task.contiguous()
    buf = getattr(sim, "_summary_buf", None)
    if buf is None:   # int64 [0:3] stats, [3] the two flags (int32), [4:6] the error word (int32[4])
        buf = sim._summary_buf = torch.zeros(6, dtype=torch.int64, device=dev)
    distances = torch.empty(n, dtype=torch.int32, device=dev)
    is_get = torch.empty(n, dtype=torch.uint8, device=dev)
    n_actions = torch.empty(n, dtype=torch.int32, device=dev)
    sim._check(N.lib().craft_rollout_distances(
        sim._h, task.data_ptr(), success.data_ptr(), seqs.data_ptr(), seqs.shape[0],
        distances.data_ptr(), is_get.data_ptr(), n_actions.data_ptr(), buf[3:4].data_ptr(),
        sim._stream()), "craft_rollout_distances")
    sim.stats(out=buf[0:3])
    sim.error_word(out=buf[4:6].view(torch.int32))
    summary = buf.cpu()
    flags = summary[3:4].view(torch.int32).tolist()
    _, ended, env_steps = summary[:3].tolist()
    bad_success, unreachable = flags
    err = int(summary[4:6].view(torch.int32)[0])
    if err:
        sim.check()                              # raises: an error latched in the loop or the probe
    if bad_success:
        raise RolloutError("satisfies() returned None for a finished episode (imitation.py:68)")
    if unreachable:
        raise RolloutError("find_closest_resources found no target: len(None) (imitation.py:88-89)")
    is_get = is_get.view(torch.bool)
    num_interactions = 0 if is_eval else env_steps
    num_steps = 0 if is_eval else env_steps - ended
    if timing is not None:
        t_done = time.perf_counter()
        for k, v in (("setup", t_loop - t_start), ("loop", t_end_loop - t_loop),
                     ("summary", t_done - t_end_loop), ("ticks", t)):
            timing[k] = timing.get(k, 0) + v
    return RolloutInfo(action_seqs=seqs[:t], n_actions=n_actions, success=success,
                       distances=distances, is_get=is_get, num_interactions=num_interactions,
                       num_steps=num_steps, ticks=t,
                       obs=obs_hist[:t + 1] if keep_obs else None)


class ImitationRollout:
    """ImitationTrainer.do_rollout(batch, world, student, teacher, is_eval) over
    dataset batches (psketch_amd.dataset.Dataset items): one CraftSim per batch
    size, sharing the dataset's scenario pool.

    policy_mix_rate / random: the behaviour-cloning draw of imitation.py:39-41
    (config.trainer.policy_mix, config.random)."""

    def __init__(self, world, pool, device=None, recipes=None, hints=None,
                 max_timesteps=40, policy_mix_rate=1.0, random=None, obs_format="f32"):
        self.obs_format = obs_format
        self.world, self.device = world, device
        self.recipes, self.hints, self.max_timesteps = recipes, hints, max_timesteps
        self.pool = np.asarray(pool, dtype=np.uint8)
        self.policy_mix_rate = policy_mix_rate
        self.random = random
        self._sims = {}

    def sim(self, n):
        s = self._sims.get(n)
        if s is None:
            s = CraftSim(self.world, n_envs=n, device=self.device,
                         pool_capacity=max(1, len(self.pool)), recipes=self.recipes,
                         hints=self.hints, max_timesteps=self.max_timesteps)
            s.load_pool(self.pool)
            s.set_obs_format(self.obs_format)
            self._sims[n] = s
        return s

    def do_rollout(self, batch, act, is_eval, receive=None, keep_obs=False):
        from .dataset import Dataset
        sim = self.sim(len(batch))
        spec = Dataset.specs(batch)
        bc = None
        if not is_eval:
            bc = self.random.binomial(1, self.policy_mix_rate, size=len(batch))
        return do_rollout(sim, spec, act, is_eval, behavior_clone=bc, receive=receive,
                          keep_obs=keep_obs)
