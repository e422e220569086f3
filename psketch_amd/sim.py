"""Batched CraftWorld simulator on one MI355X: the Python face of the C ABI.

`CraftSim` owns N environment slots in HBM (struct-of-arrays, see
csrc/craft_sim.hip) and exposes the reference's CraftWorld/CraftState surface
batched over torch device tensors:

  reset(...)         CraftScenario.init           craft.py:262-273
  step(actions)      do_rollout tick + features    trainers/imitation.py:59-73, craft.py:296-424
  transition(a)      CraftState.step               craft.py:332-424
  observe()          CraftState.features/satisfies craft.py:285-330
  teacher()          DemonstrationTeacher.__call__ teachers/demonstration.py:9-30

All work runs in HIP kernels on the caller's current torch stream; outputs are
device tensors the trainer consumes in place (no host round trip).
"""
import ctypes
import weakref

import numpy as np
import torch

from . import _native as N
from .cookbook import Cookbook, TaskManager, compile_config, world_params, generator_primitives
from . import gamedef


def _ptr(t):
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


class CraftSim:
    """N CraftWorld environments on one GPU.

    world: a gamedef.WORLDS name ("craft_medium_12x12" is the benchmark world),
    a configs/worlds YAML path or a dict.  recipes / hints: YAML paths or None
    for the built-in tables.  env_id_base: global id of slot 0 (rank * N when
    sharded), which keys every per-env random draw.  device: a GPU index (default:
    the current one) runs the HIP library; device="cpu" runs the CPU variant of the
    same ABI (libpsketch_craft_cpu.so) on host tensors, the same results bit for bit.
    """

    def __init__(self, world="craft_medium_12x12", n_envs=4096, device=None, env_id_base=0,
                 pool_capacity=1024, recipes=None, hints=None,
                 max_timesteps=gamedef.MAX_TIMESTEPS):
        if device is None:
            device = torch.cuda.current_device()
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        if self.device.type not in ("cuda", "cpu"):
            raise ValueError(f"device {self.device}: a GPU index or 'cpu'")
        self._cpu = self.device.type == "cpu"
        self._L = N.lib(cpu=self._cpu)
        self.params = world_params(world)
        self.cookbook = Cookbook(recipes)
        self.task_manager = TaskManager(hints)
        self.config = compile_config(self.params, self.cookbook, self.task_manager, max_timesteps)
        self.width, self.height = self.params["WIDTH"], self.params["HEIGHT"]
        self.n_kinds = self.cookbook.n_kinds
        self.n_features = self.config.n_features
        self.n_envs = int(n_envs)
        self.env_id_base = int(env_id_base)
        self.pool_capacity = int(pool_capacity)
        self.pool_count = 0
        handle = ctypes.c_void_p()
        N.check(self._L.craft_sim_create(ctypes.byref(self.config), self.device.index or 0, self.n_envs,
                                         self.env_id_base, self.pool_capacity,
                                         ctypes.byref(handle)), what="craft_sim_create", L=self._L)
        self._h = handle
        self.obs_format, self.obs_dtype = "f32", torch.float32
        self._rollout_cache = None
        self._teach_cache = None

    # ---- lifetime ---------------------------------------------------------------
    def close(self):
        self._rollout_cache = None
        self._teach_cache = None
        if getattr(self, "_h", None):
            self._L.craft_sim_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def tune(self, tile_envs=0, max_resident_per_cu=0, obs_store=0):
        """Tile-kernel geometry and observation-store cache policy (0 write-back,
        1 nontemporal, 2 write-through); results are identical for every setting."""
        self._check(self._L.craft_sim_tune(self._h, int(tile_envs), int(max_resident_per_cu),
                                           int(obs_store)), "craft_sim_tune")

    def tune_rollout(self, chunk_ticks=0, threads=0):
        """Ticks per dynamically scheduled work unit of rollout() (0 = the whole
        launch, the default; -1 = one continuous pipeline per workgroup across
        its tiles) and threads per tile workgroup (0 = the library's default
        shape); results are identical for every setting."""
        self._check(self._L.craft_sim_tune_rollout(self._h, int(chunk_ticks), int(threads)),
                    "craft_sim_tune_rollout")

    def tune_teach(self, kernel=0, lanes=0, table=0):
        """The teacher's knobs (craft_sim_tune_teach; results are identical for every
        setting): kernel = which kernel step(..., labels=) launches (0 the measured best, 1 the
        one-tile kernel, 2 the two-tile kernel, 3x3 windows); lanes = teacher lanes per query
        (0 default, 1, 2 or 4); table = which teachers read the teacher table (0 auto, 1 always,
        2 never: every query runs the BFS)."""
        self._check(self._L.craft_sim_tune_teach(self._h, int(kernel), int(lanes), int(table)),
                    "craft_sim_tune_teach")

    def tune_host(self, threads=0):
        """Host worker threads of the CPU variant (craft_sim_tune_host: 0 = the machine's);
        validated and ignored by the HIP library. Results are identical for every setting."""
        self._check(self._L.craft_sim_tune_host(self._h, int(threads)), "craft_sim_tune_host")

    def sync_table(self):
        """Build the teacher-table rows of pools loaded since the last teacher launch, on the
        current stream, and wait (craft_sim_sync_table): needed only before capturing a teacher
        launch into a graph right after load_pool (the capture refuses to build them)."""
        self._check(self._L.craft_sim_sync_table(self._h, self._stream()), "craft_sim_sync_table")

    def step_shape(self, teach=False):
        """(kernel name, envs per tile / workgroup, teacher lanes per env) that step()
        launches, without (teach=False) or with labels= (craft_sim_step_shape)."""
        k, e, l = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        self._check(self._L.craft_sim_step_shape(self._h, int(bool(teach)), ctypes.byref(k),
                                                 ctypes.byref(e), ctypes.byref(l)),
                    "craft_sim_step_shape")
        return N.KERNEL_NAMES[k.value], e.value, l.value

    def rollout_shape(self):
        """(tile_envs, threads, split) the next rollout() launches with, as the
        library resolves its knobs (craft_sim_rollout_shape)."""
        t, nt, sp = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        self._check(self._L.craft_sim_rollout_shape(self._h, ctypes.byref(t), ctypes.byref(nt),
                                                    ctypes.byref(sp)), "craft_sim_rollout_shape")
        return t.value, nt.value, bool(sp.value)

    def teach_words(self):
        """32-bit words per cell set of the teacher's BFS as the kernels are instantiated (the
        band of columns 1 .. W-2: 8x8 -> 2, 10x10 and 12x12 -> 4, up to 15x15 -> 8)."""
        nw = ((self.width - 2) * self.height + 31) // 32
        return 2 if nw <= 2 else 4 if nw <= 4 else 8

    def tile_shape(self):
        """(tile_envs, obs_store) of the tick kernel (craft_sim_tile_shape)."""
        t, st = ctypes.c_int32(), ctypes.c_int32()
        self._check(self._L.craft_sim_tile_shape(self._h, ctypes.byref(t), ctypes.byref(st)),
                    "craft_sim_tile_shape")
        return t.value, st.value

    _OBS_FORMATS = {"f32": (N.OBS_F32, torch.float32), "bf16": (N.OBS_BF16, torch.bfloat16),
                    "u8": (N.OBS_U8, torch.uint8)}

    def set_obs_format(self, fmt):
        """Element type of every observation this simulator writes: "f32"
        (default), "bf16" or "u8" — the same exact integer values in each."""
        code, dtype = self._OBS_FORMATS[fmt]
        self._check(self._L.craft_sim_set_obs_format(self._h, code), "craft_sim_set_obs_format")
        self.obs_format, self.obs_dtype = fmt, dtype
        self._rollout_cache = None
        self._teach_cache = None

    def _stream(self):
        # the raw hipStream_t of the caller's current stream on this device (an int; the C ABI's
        # argtypes take it as void*): ~5x cheaper than building a torch.cuda.Stream object.  The
        # CPU variant ignores it.
        if self._cpu:
            return None
        return torch._C._cuda_getCurrentRawStream(self.device.index)

    def _check(self, status, what):
        N.check(status, self._h, what, L=self._L)

    def check(self):
        """Synchronises and raises if a kernel latched an error (bad action,
        teacher assertion, out-of-range slot)."""
        slot = ctypes.c_int64(-1)
        self._check(self._L.craft_sim_check(self._h, ctypes.byref(slot), self._stream()),
                    "kernel error")

    def error_word(self, out=None):
        """Device int32[4] copy of the latched-error record ({status, 0, slot lo, slot hi}),
        queued on the current stream without synchronising (craft_sim_error_word)."""
        if out is None:
            out = torch.empty(4, dtype=torch.int32, device=self.device)
        self._buf("out", out, torch.int32, (4,))
        self._check(self._L.craft_sim_error_word(self._h, _ptr(out), self._stream()),
                    "craft_sim_error_word")
        return out

    # ---- helpers --------------------------------------------------------------------
    def _i32(self, x, n=None):
        if x is None:
            return None
        t = torch.as_tensor(x, device=self.device)
        if t.dtype != torch.int32:
            t = t.to(torch.int32)
        t = t.contiguous()
        if n is not None and t.numel() != n:
            raise ValueError(f"expected {n} entries, got {t.numel()}")
        return t

    def _buf(self, name, t, dtype, shape):
        """Checks a caller-owned output (or input) tensor before its pointer goes
        to the C ABI: dtype, contiguity, exact shape and device.  A wrong buffer
        raises here instead of letting a kernel write out of bounds."""
        if t is None:
            return None
        if not isinstance(t, torch.Tensor):
            raise TypeError(f"{name} must be a torch tensor")
        if t.dtype != dtype:
            raise TypeError(f"{name} is {t.dtype}, expected {dtype}")
        if t.device != self.device:
            raise ValueError(f"{name} is on {t.device}, the simulator is on {self.device}")
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")
        if tuple(t.shape) != tuple(shape):
            raise ValueError(f"{name} has shape {tuple(t.shape)}, expected {tuple(shape)}")
        return t

    def empty_obs(self, n=None):
        n = self.n_envs if n is None else n
        return torch.empty((n, self.n_features), dtype=self.obs_dtype, device=self.device)

    def _obs(self, obs, n=None):
        """An [n, F] observation buffer in the handle's format (n = n_envs)."""
        n = self.n_envs if n is None else n
        return _ptr(self._buf("obs", obs, self.obs_dtype, (n, self.n_features)))

    # ---- scenario pool -----------------------------------------------------------------
    def load_pool(self, grids, first=0):
        """grids: uint8 [P, W, H] or [P, W*H] kind ids (x-major), host or device."""
        g = np.ascontiguousarray(np.asarray(torch.as_tensor(grids).cpu(), dtype=np.uint8))
        g = g.reshape(g.shape[0], self.width * self.height)
        self._check(self._L.craft_pool_load(self._h, g.ctypes.data_as(ctypes.c_void_p), int(first),
                                            int(g.shape[0])), "craft_pool_load")
        self.pool_count = max(self.pool_count, first + g.shape[0])

    def sample_pool(self, count, seed=123, dedup=True):
        """Generates `count` scenarios with the make_data.py generator
        (RandomState(seed) stream) and loads them; returns (grids, init_pos)."""
        grids, init_pos, _ = sample_scenarios(self.params, self.cookbook, seed, count, dedup)
        self.load_pool(grids)
        return grids, init_pos

    def generate_pool(self, count, seed=0, first=0, scenario_id0=None, init_pos=False):
        """make_data.sample_scenario x count on the GPU, straight into pool rows
        [first, first + count) (include/craft.h craft_pool_generate); scenario s
        draws from a stream keyed by its global id (scenario_id0 + s, default
        first + s).  Returns the device int32 [count, 2] initial positions if
        init_pos, else None."""
        prims = np.ascontiguousarray(generator_primitives(self.cookbook), dtype=np.int32)
        ws = np.asarray([self.cookbook.index["workshop%d" % i] for i in range(self.params["N_WORKSHOPS"])],
                        dtype=np.int32)
        out = torch.empty((count, 2), dtype=torch.int32, device=self.device) if init_pos else None
        sid0 = first if scenario_id0 is None else scenario_id0
        self._check(self._L.craft_pool_generate(
            self._h, ctypes.c_uint64(seed & (2**64 - 1)), int(sid0), int(first), int(count),
            self.cookbook.index["boundary"], prims.ctypes.data_as(ctypes.c_void_p), len(prims),
            self.params["N_PRIMITIVES"], ws.ctypes.data_as(ctypes.c_void_p), len(ws), _ptr(out),
            self._stream()), "craft_pool_generate")
        self.pool_count = max(self.pool_count, first + count)
        return out

    # ---- episodes -----------------------------------------------------------------------
    def reset(self, scenario, pos_x, pos_y, dir, task, obs=None):
        n = self.n_envs
        args = [self._i32(a, n) for a in (scenario, pos_x, pos_y, dir, task)]
        self._args_keepalive = args
        self._check(self._L.craft_reset(self._h, *[_ptr(a) for a in args], self._obs(obs), self._stream()),
                    "craft_reset")
        return obs

    def step(self, actions=None, seed=0, tick=0, autoreset=True, obs=None, reward=None, done=None,
             success=None, ref_actions=None, behavior_clone=None, action_record=None,
             any_live=None, transition_code=None, labels=None):
        """One rollout tick for every slot (include/craft.h craft_step / craft_step_ex).
        actions: int32 device tensor [N] or None for the in-kernel hashed draw;
        ref_actions + behavior_clone (uint8 [N]): cloned actions; action_record
        (int32 [N]) receives the action taken (-1 for done slots); any_live (a
        one-element int32 device tensor) is set to 1 if a slot is still running.
        labels (int32 [N]): the DemonstrationTeacher's action for every slot's NEW
        state, computed in the same launch (craft_step_teach) — what teacher()
        would return right after this step."""
        n = self.n_envs
        flags = N.STEP_AUTORESET if autoreset else 0
        if ref_actions is None and behavior_clone is None and action_record is None \
                and any_live is None and transition_code is None and labels is None:
            # plain tick: the short craft_step entry (least host overhead per launch)
            a = self._i32(actions, n) if actions is not None else None
            r = self._buf("reward", reward, torch.float32, (n,))
            d = self._buf("done", done, torch.uint8, (n,))
            sc = self._buf("success", success, torch.int8, (n,))
            self._check(self._L.craft_step(self._h, _ptr(a), ctypes.c_uint64(seed & (2**64 - 1)),
                                           int(tick), flags, self._obs(obs), _ptr(r),
                                           _ptr(d), _ptr(sc), self._stream()), "craft_step")
            return obs
        args = N.craft_step_args_t()
        keep = []

        def put(field, t):
            if t is not None:
                keep.append(t)
                setattr(args, field, t.data_ptr())

        put("actions", self._i32(actions, n) if actions is not None else None)
        put("ref_actions", self._i32(ref_actions, n) if ref_actions is not None else None)
        if behavior_clone is not None:
            bc = torch.as_tensor(behavior_clone, device=self.device)
            bc = (bc != 0).to(torch.uint8).contiguous() if bc.dtype != torch.uint8 else bc.contiguous()
            if bc.numel() != n:
                raise ValueError(f"behavior_clone: expected {n} entries")
            put("behavior_clone", bc)
        for name, t, dt, shape in (("reward", reward, torch.float32, (n,)),
                                   ("done", done, torch.uint8, (n,)),
                                   ("success", success, torch.int8, (n,)),
                                   ("action_record", action_record, torch.int32, (n,)),
                                   ("any_live", any_live, torch.int32, (1,)),
                                   ("transition_code", transition_code, torch.int8, (n,))):
            put(name, self._buf(name, t, dt, shape))
        self._obs(obs)
        put("obs", obs)
        args.action_seed = seed & (2**64 - 1)
        args.tick = int(tick)
        args.flags = flags
        if labels is not None:
            self._buf("labels", labels, torch.int32, (n,))
            self._check(self._L.craft_step_teach(self._h, ctypes.byref(args), _ptr(labels),
                                                 self._stream()), "craft_step_teach")
        else:
            self._check(self._L.craft_step_ex(self._h, ctypes.byref(args), self._stream()),
                        "craft_step")
        return obs

    def rollout(self, n_ticks, seed=0, tick0=0, actions=None, autoreset=True, obs=None,
                reward=None, done=None, success=None):
        """n_ticks craft_step ticks in one launch (include/craft.h craft_rollout),
        identical to calling step(tick=tick0 + k) n_ticks times.  actions: int32
        [n_ticks, N] or None (hashed); obs: [R, N, F] ring in the obs format
        (tick t writes obs[t % R]); reward / done / success: [R, N] rings."""
        n = self.n_envs
        if n_ticks < 0:
            raise ValueError("n_ticks must be >= 0")
        if actions is None:
            # the same output tensors as the last call (a benchmark or trainer loop): their checks
            # still hold, so only the launch arguments change
            c = self._rollout_cache
            if c is not None and all((r is None and t is None) or (r is not None and r() is t)
                                     for r, t in zip(c[0], (obs, reward, done, success))) \
                    and c[1] == self._ring_sig(obs, reward, done, success):
                self._check(self._rollout_fn(self._h, None, seed & 0xFFFFFFFFFFFFFFFF,
                                             int(tick0), int(n_ticks),
                                             N.STEP_AUTORESET if autoreset else 0, *c[2],
                                             self._stream()), "craft_rollout")
                return obs
        ring = None
        for name, t in (("obs", obs), ("reward", reward), ("done", done), ("success", success)):
            if t is not None:
                if t.dim() < 1 or t.shape[0] < 1:
                    raise ValueError(f"{name} must be a ring [R >= 1, {n}, ...]")
                if ring is not None and t.shape[0] != ring:
                    raise ValueError(f"{name} ring {t.shape[0]} != ring {ring} of the other outputs")
                ring = t.shape[0]
        if obs is not None:
            self._buf("obs", obs, self.obs_dtype, (ring, n, self.n_features))
        for name, t, dt in (("reward", reward, torch.float32), ("done", done, torch.uint8),
                            ("success", success, torch.int8)):
            self._buf(name, t, dt, (ring, n) if t is not None else ())
        a = None
        if actions is not None:
            a = self._i32(actions, n * n_ticks)
        self._rollout_fn = self._L.craft_rollout
        self._check(self._rollout_fn(self._h, _ptr(a), ctypes.c_uint64(seed & (2**64 - 1)),
                                     int(tick0), int(n_ticks),
                                     N.STEP_AUTORESET if autoreset else 0, _ptr(obs),
                                     int(ring or 1), _ptr(reward), _ptr(done), _ptr(success),
                                     self._stream()), "craft_rollout")
        if a is None:                   # weak references: the cache keeps no output alive
            self._rollout_cache = (
                tuple(None if t is None else weakref.ref(t) for t in (obs, reward, done, success)),
                self._ring_sig(obs, reward, done, success),
                (_ptr(obs), int(ring or 1), _ptr(reward), _ptr(done), _ptr(success)))
        return obs

    def rollout_teach(self, n_ticks, seed=0, tick0=0, actions=None, autoreset=True, obs=None,
                      reward=None, done=None, success=None, labels=None, action_record=None,
                      label_in=None, behavior_clone=None, label_actions=False):
        """n_ticks ticks with the DemonstrationTeacher's label of every slot's new state after
        each one, in one launch (include/craft.h craft_rollout_teach): identical to n_ticks
        step(..., labels=) calls.  Each tick's action per slot: its current state's label when
        label_actions (every slot: make_data's demonstrations) or behavior_clone[i] (uint8 [N]),
        else actions[k] (int32 [n_ticks, N]) or the hashed draw.  label_in (int32 [N]): the
        labels of the states before tick0, needed when labels feed actions (teacher() of the
        reset states, or the previous launch's last labels slot).  Outputs are [R, ...] rings
        (tick t writes slot t % R): obs, reward, done, success, labels (int32), action_record
        (int32, -1 for done slots)."""
        n = self.n_envs
        if n_ticks < 0:
            raise ValueError("n_ticks must be >= 0")
        outs_t = (obs, reward, done, success, labels, action_record)
        if actions is None and label_in is None and behavior_clone is None and not label_actions:
            # the same output rings as the last call (a benchmark loop): their checks still hold
            c = self._teach_cache
            if c is not None and c[1] == self._ring_sig(*outs_t) and all(
                    (r is None and t is None) or (r is not None and r() is t) for r, t in zip(c[0], outs_t)):
                args = c[2]
                args.action_seed = seed & (2**64 - 1)
                args.tick0 = int(tick0)
                args.n_ticks = int(n_ticks)
                args.flags = N.STEP_AUTORESET if autoreset else 0
                self._check(self._L.craft_rollout_teach(self._h, ctypes.byref(args), self._stream()),
                            "craft_rollout_teach")
                return labels
        args = N.craft_rollout_teach_args_t()
        keep = []

        def put(field, t):
            if t is not None:
                keep.append(t)
                setattr(args, field, t.data_ptr())

        ring = None
        outs = (("obs", obs), ("reward", reward), ("done", done), ("success", success),
                ("labels", labels), ("action_record", action_record))
        for name, t in outs:
            if t is not None:
                if t.dim() < 1 or t.shape[0] < 1:
                    raise ValueError(f"{name} must be a ring [R >= 1, {n}, ...]")
                if ring is not None and t.shape[0] != ring:
                    raise ValueError(f"{name} ring {t.shape[0]} != ring {ring} of the other outputs")
                ring = t.shape[0]
        ring = ring or 1
        if obs is not None:
            self._buf("obs", obs, self.obs_dtype, (ring, n, self.n_features))
        for name, t, dt in (("reward", reward, torch.float32), ("done", done, torch.uint8),
                            ("success", success, torch.int8), ("labels", labels, torch.int32),
                            ("action_record", action_record, torch.int32)):
            self._buf(name, t, dt, (ring, n) if t is not None else ())
        for name, t in outs:
            put(name, t)
        if actions is not None:
            put("actions", self._i32(actions, n * n_ticks))
        if label_in is not None:
            put("label_in", self._i32(label_in, n))
        if behavior_clone is not None:
            bc = torch.as_tensor(behavior_clone, device=self.device)
            bc = (bc != 0).to(torch.uint8).contiguous() if bc.dtype != torch.uint8 else bc.contiguous()
            if bc.numel() != n:
                raise ValueError(f"behavior_clone: expected {n} entries")
            put("behavior_clone", bc)
        args.label_actions = 1 if label_actions else 0
        args.action_seed = seed & (2**64 - 1)
        args.tick0 = int(tick0)
        args.n_ticks = int(n_ticks)
        args.flags = N.STEP_AUTORESET if autoreset else 0
        args.ring = int(ring)
        self._check(self._L.craft_rollout_teach(self._h, ctypes.byref(args), self._stream()),
                    "craft_rollout_teach")
        if actions is None and label_in is None and behavior_clone is None and not label_actions:
            # weak references: the cache keeps no output alive
            self._teach_cache = (tuple(None if t is None else weakref.ref(t) for t in outs_t),
                                 self._ring_sig(*outs_t), args)
        return labels

    @staticmethod
    def _ring_sig(*ts):
        """Storage, shape, strides, dtype and device of each output ring (a tensor resized,
        re-strided or re-pointed in place since the last call no longer matches)."""
        return tuple((t.data_ptr(), tuple(t.shape), t.stride(), t.dtype, t.device)
                     if t is not None else None for t in ts)

    def stats(self, reset=False, out=None):
        """Device int64[3] {successes, episodes ended, env-steps}."""
        if out is None:
            out = torch.zeros(3, dtype=torch.int64, device=self.device)
        self._check(self._L.craft_stats(self._h, _ptr(out), int(bool(reset)), self._stream()),
                    "craft_stats")
        return out

    # ---- reference-granular surface ----------------------------------------------------
    def transition(self, actions, src=None, dst=None, codes=None):
        """CraftState.step per item (craft_transition); codes: int8 [n] device
        tensor receiving the describe() transition code of each item."""
        a = self._i32(actions)
        n = a.numel()
        s, d = self._i32(src, n), self._i32(dst, n)
        self._buf("codes", codes, torch.int8, (n,))
        self._check(self._L.craft_transition(self._h, _ptr(s), _ptr(d), _ptr(a), n, _ptr(codes),
                                             self._stream()), "craft_transition")
        return codes

    def observe(self, slots=None, tasks=None, obs=None, sat=None, n=None):
        s = self._i32(slots)
        n = s.numel() if s is not None else (self.n_envs if n is None else n)
        t = self._i32(tasks, n)
        self._buf("sat", sat, torch.int8, (n,))
        self._check(self._L.craft_observe(self._h, _ptr(s), n, _ptr(t), self._obs(obs, n), _ptr(sat),
                                          self._stream()), "craft_observe")
        return obs, sat

    def teacher(self, slots=None, tasks=None, action_out=None, path_len_out=None, n=None):
        s = self._i32(slots)
        n = s.numel() if s is not None else (self.n_envs if n is None else n)
        t = self._i32(tasks, n)
        if action_out is None:
            action_out = torch.empty(n, dtype=torch.int32, device=self.device)
        self._buf("action_out", action_out, torch.int32, (n,))
        self._buf("path_len_out", path_len_out, torch.int32, (n,))
        self._check(self._L.craft_teacher(self._h, _ptr(s), n, _ptr(t), _ptr(action_out),
                                          _ptr(path_len_out), self._stream()), "craft_teacher")
        return action_out, path_len_out

    def get_state(self, slots=None, n=None, fields=("agent", "inventory", "grid", "spec")):
        """Device copies of the requested fields: agent int32 [n, 4] (x, y, dir,
        timer), inventory int32 [n, K], grid uint8 [n, W*H], spec int32 [n, 5]."""
        s = self._i32(slots)
        n = s.numel() if s is not None else (self.n_envs if n is None else n)
        dev = self.device
        shapes = {"agent": ((n, 4), torch.int32), "inventory": ((n, self.n_kinds), torch.int32),
                  "grid": ((n, self.width * self.height), torch.uint8), "spec": ((n, 5), torch.int32)}
        out = {f: torch.empty(shapes[f][0], dtype=shapes[f][1], device=dev) for f in fields}
        self._check(self._L.craft_get_state(self._h, _ptr(s), n, _ptr(out.get("agent")),
                                            _ptr(out.get("inventory")), _ptr(out.get("grid")),
                                            _ptr(out.get("spec")), self._stream()), "craft_get_state")
        return out

    def set_state(self, spec, agent, inventory=None, slots=None):
        sp = self._i32(spec)
        n = sp.shape[0]
        ag = self._i32(agent)
        iv = self._i32(inventory)
        s = self._i32(slots, n)
        self._check(self._L.craft_set_state(self._h, _ptr(s), n, _ptr(sp), _ptr(ag), _ptr(iv),
                                            self._stream()), "craft_set_state")


# ---- host-side inputs ---------------------------------------------------------------------

def sample_scenarios(params, cookbook, seed, count, dedup=True):
    """make_data.sample_scenario (make_data.py:105-144) x count, native and
    bit-exact against numpy's RandomState(seed).  Returns (grids uint8
    [count, W*H], init_pos int32 [count, 2], mt_state uint32[625])."""
    W, H = params["WIDTH"], params["HEIGHT"]
    prims = np.asarray(generator_primitives(cookbook), dtype=np.int32)
    ws = np.asarray([cookbook.index["workshop%d" % i] for i in range(params["N_WORKSHOPS"])],
                    dtype=np.int32)
    grids = np.zeros((count, W * H), dtype=np.uint8)
    init_pos = np.zeros((count, 2), dtype=np.int32)
    mt = np.zeros(625, dtype=np.uint32)
    st = N.lib().craft_sample_scenarios(
        W, H, cookbook.index["boundary"], prims.ctypes.data_as(ctypes.c_void_p), len(prims),
        params["N_PRIMITIVES"], ws.ctypes.data_as(ctypes.c_void_p), len(ws), seed, count,
        int(bool(dedup)), grids.ctypes.data_as(ctypes.c_void_p),
        init_pos.ctypes.data_as(ctypes.c_void_p), mt.ctypes.data_as(ctypes.c_void_p))
    N.check(st, what="craft_sample_scenarios")
    return grids, init_pos, mt


_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def hash_actions(seed, gids, tick):
    """The in-kernel action draw of craft_step: splitmix64(seed ^ (gid<<20) ^ tick) >> 32 mod 6."""
    g = np.asarray(gids, dtype=np.uint64)
    key = np.uint64(seed) ^ (g << np.uint64(20)) ^ np.uint64(tick)
    return ((splitmix64(key) >> np.uint64(32)) % np.uint64(6)).astype(np.int32)


def synthetic_specs(grids, width, height, n_envs, env_id_base=0, seed=0, task_ids=None):
    """Per-env initial states for synthetic rollouts, keyed by global env id:
    scenario gid mod P, an interior free cell picked by splitmix64, dir 0
    (init_state's default, craft.py:258), task task_ids[gid mod len].
    Returns int32 arrays (scenario, x, y, dir, task)."""
    grids = np.asarray(grids, dtype=np.uint8).reshape(len(grids), width * height)
    P = len(grids)
    gid = np.arange(env_id_base, env_id_base + n_envs, dtype=np.int64)
    scen = (gid % P).astype(np.int64)
    cells = np.arange(width * height)
    cx, cy = cells // height, cells % height
    interior = (cx > 0) & (cx < width - 1) & (cy > 0) & (cy < height - 1)
    free = (grids == 0) & interior[None, :]
    n_free = free.sum(axis=1)
    if (n_free == 0).any():
        raise ValueError("a scenario has no free interior cell")
    # rank of each free cell within its scenario, x-major
    order = np.cumsum(free, axis=1) - 1
    key = (np.uint64(seed) << np.uint64(32)) ^ gid.astype(np.uint64) ^ np.uint64(0xA5A5A5A5A5A5A5A5)
    k = ((splitmix64(key) >> np.uint64(32)) % n_free[scen].astype(np.uint64)).astype(np.int64)
    # cell index of the k-th free cell of each env's scenario
    pick = np.argmax((order[scen] == k[:, None]) & free[scen], axis=1)
    x = (pick // height).astype(np.int32)
    y = (pick % height).astype(np.int32)
    if task_ids is None:
        task_ids = np.arange(1, dtype=np.int32)
    task_ids = np.asarray(task_ids, dtype=np.int32)
    task = task_ids[gid % len(task_ids)].astype(np.int32)
    return scen.astype(np.int32), x, y, np.zeros(n_envs, dtype=np.int32), task
