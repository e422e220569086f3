"""ctypes binding of the C ABI in include/craft.h (libpsketch_craft.so).

The HIP library is the product: every simulator call on a GPU goes through it and there is
no CPU fallback; using it without the built library raises.  The CPU variant of the same ABI
(libpsketch_craft_cpu.so, host pointers) is a separate library that only
CraftSim(device="cpu") loads, on purpose.
"""
import ctypes
import os

import torch  # noqa: F401  (load torch's HIP runtime first so the library shares it)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libpsketch_craft.so")
# diagnostic builds (tools/) may point at another in-tree build of the same ABI
LIB_PATH = os.environ.get("PSKETCH_CRAFT_LIB", LIB_PATH)
CPU_LIB_PATH = os.path.join(_HERE, "lib", "libpsketch_craft_cpu.so")

ABI_VERSION = 2
MAX_KINDS = 32
MAX_RECIPES = 16
MAX_INGREDIENTS = 4
MAX_TASKS = 64
MAX_SUBTASKS = 4
MAX_DIM = 16
MAX_CELLS = 256

OK, EINVAL, EBADACTION, EINVARIANT, ETEACHER, EHIP, ENOMEM, ERANGE = range(8)

DOWN, UP, LEFT, RIGHT, USE, STOP = range(6)
N_ACTIONS = 6

KIND_INERT, KIND_GRABBABLE, KIND_WORKSHOP, KIND_WATER, KIND_STONE = range(5)
GOAL_OTHER, GOAL_GET, GOAL_MAKE, GOAL_GO, GOAL_USE = range(5)

STEP_AUTORESET = 1

KERNEL_TILE, KERNEL_TICK2 = 1, 2
KERNEL_NAMES = {KERNEL_TILE: "tile_kernel", KERNEL_TICK2: "tick2_kernel"}


class craft_recipe_t(ctypes.Structure):
    _fields_ = [
        ("output", ctypes.c_int32),
        ("workshop", ctypes.c_int32),
        ("yield_", ctypes.c_int32),
        ("n_inputs", ctypes.c_int32),
        ("input_kind", ctypes.c_int32 * MAX_INGREDIENTS),
        ("input_count", ctypes.c_int32 * MAX_INGREDIENTS),
    ]


class craft_task_t(ctypes.Structure):
    _fields_ = [
        ("goal", ctypes.c_int32),
        ("arg_kind", ctypes.c_int32),
        ("n_subtasks", ctypes.c_int32),
        ("subtask", ctypes.c_int32 * MAX_SUBTASKS),
    ]


class craft_config_t(ctypes.Structure):
    _fields_ = [
        ("abi_version", ctypes.c_int32),
        ("width", ctypes.c_int32),
        ("height", ctypes.c_int32),
        ("window_width", ctypes.c_int32),
        ("window_height", ctypes.c_int32),
        ("n_kinds", ctypes.c_int32),
        ("n_features", ctypes.c_int32),
        ("max_timesteps", ctypes.c_int32),
        ("bridge_kind", ctypes.c_int32),
        ("axe_kind", ctypes.c_int32),
        ("kind_class", ctypes.c_uint8 * MAX_KINDS),
        ("n_recipes", ctypes.c_int32),
        ("recipe", craft_recipe_t * MAX_RECIPES),
        ("n_tasks", ctypes.c_int32),
        ("task", craft_task_t * MAX_TASKS),
    ]


class craft_step_args_t(ctypes.Structure):
    _fields_ = [
        ("actions", ctypes.c_void_p),
        ("ref_actions", ctypes.c_void_p),
        ("behavior_clone", ctypes.c_void_p),
        ("action_seed", ctypes.c_uint64),
        ("tick", ctypes.c_int64),
        ("flags", ctypes.c_uint32),
        ("obs", ctypes.c_void_p),
        ("reward", ctypes.c_void_p),
        ("done", ctypes.c_void_p),
        ("success", ctypes.c_void_p),
        ("action_record", ctypes.c_void_p),
        ("any_live", ctypes.c_void_p),
        ("transition_code", ctypes.c_void_p),
    ]


class craft_rollout_teach_args_t(ctypes.Structure):
    _fields_ = [
        ("actions", ctypes.c_void_p),
        ("behavior_clone", ctypes.c_void_p),
        ("label_actions", ctypes.c_int32),
        ("label_in", ctypes.c_void_p),
        ("action_seed", ctypes.c_uint64),
        ("tick0", ctypes.c_int64),
        ("n_ticks", ctypes.c_int32),
        ("flags", ctypes.c_uint32),
        ("ring", ctypes.c_int32),
        ("obs", ctypes.c_void_p),
        ("reward", ctypes.c_void_p),
        ("done", ctypes.c_void_p),
        ("success", ctypes.c_void_p),
        ("labels", ctypes.c_void_p),
        ("action_record", ctypes.c_void_p),
    ]


OBS_F32, OBS_BF16, OBS_U8 = 0, 1, 2

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_u32 = ctypes.c_uint32
_u64 = ctypes.c_uint64

# name -> (restype, argtypes); exactly the functions include/craft.h declares
SIGNATURES = {
    "craft_sim_create": (_i32, [ctypes.POINTER(craft_config_t), _i32, _i64, _i64, _i32,
                                ctypes.POINTER(_vp)]),
    "craft_sim_destroy": (_i32, [_vp]),
    "craft_sim_last_error": (ctypes.c_char_p, [_vp]),
    "craft_strerror": (ctypes.c_char_p, [_i32]),
    "craft_host_flag_pointer": (_i32, [_vp, ctypes.POINTER(_vp)]),
    "craft_sim_info": (_i32, [_vp, ctypes.POINTER(_i64), ctypes.POINTER(_i32),
                              ctypes.POINTER(_i32)]),
    "craft_sim_check": (_i32, [_vp, ctypes.POINTER(_i64), _vp]),
    "craft_sim_error_word": (_i32, [_vp, _vp, _vp]),
    "craft_sim_tune": (_i32, [_vp, _i32, _i32, _i32]),
    "craft_sim_set_obs_format": (_i32, [_vp, _i32]),
    "craft_sim_tune_rollout": (_i32, [_vp, _i32, _i32]),
    "craft_sim_tune_teach": (_i32, [_vp, _i32, _i32, _i32]),
    "craft_abi_version": (_i32, []),
    "craft_sim_tune_host": (_i32, [_vp, _i32]),
    "craft_sim_sync_table": (_i32, [_vp, _vp]),
    "craft_sim_step_shape": (_i32, [_vp, _i32, ctypes.POINTER(_i32), ctypes.POINTER(_i32),
                                    ctypes.POINTER(_i32)]),
    "craft_sim_rollout_shape": (_i32, [_vp, ctypes.POINTER(_i32), ctypes.POINTER(_i32),
                                       ctypes.POINTER(_i32)]),
    "craft_sim_tile_shape": (_i32, [_vp, ctypes.POINTER(_i32), ctypes.POINTER(_i32)]),
    "craft_pool_load": (_i32, [_vp, _vp, _i32, _i32]),
    "craft_pool_generate": (_i32, [_vp, _u64, _i64, _i32, _i32, _i32, _vp, _i32, _i32, _vp, _i32,
                                   _vp, _vp]),
    "craft_reset": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "craft_step": (_i32, [_vp, _vp, _u64, _i64, _u32, _vp, _vp, _vp, _vp, _vp]),
    "craft_step_ex": (_i32, [_vp, ctypes.POINTER(craft_step_args_t), _vp]),
    "craft_step_teach": (_i32, [_vp, ctypes.POINTER(craft_step_args_t), _vp, _vp]),
    "craft_rollout": (_i32, [_vp, _vp, _u64, _i64, _i32, _u32, _vp, _i32, _vp, _vp, _vp, _vp]),
    "craft_rollout_teach": (_i32, [_vp, ctypes.POINTER(craft_rollout_teach_args_t), _vp]),
    "craft_stats": (_i32, [_vp, _vp, _i32, _vp]),
    "craft_transition": (_i32, [_vp, _vp, _vp, _vp, _i64, _vp, _vp]),
    "craft_observe": (_i32, [_vp, _vp, _i64, _vp, _vp, _vp, _vp]),
    "craft_teacher": (_i32, [_vp, _vp, _i64, _vp, _vp, _vp, _vp]),
    "craft_rollout_distances": (_i32, [_vp, _vp, _vp, _vp, _i32, _vp, _vp, _vp, _vp, _vp]),
    "craft_get_state": (_i32, [_vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp]),
    "craft_set_state": (_i32, [_vp, _vp, _i64, _vp, _vp, _vp, _vp]),
    "craft_sample_scenarios": (_i32, [_i32, _i32, _i32, _vp, _i32, _i32, _vp, _i32, _u32,
                                      _i32, _i32, _vp, _vp, _vp]),
}


class CraftError(RuntimeError):
    def __init__(self, status, message):
        super().__init__(message)
        self.status = status


_libs = {}


def lib(cpu=False):
    """The loaded HIP library (cpu=False) or the CPU variant of the same ABI (cpu=True); raises
    if it has not been built (neither falls back to the other)."""
    l = _libs.get(cpu)
    if l is None:
        path = CPU_LIB_PATH if cpu else LIB_PATH
        if not os.path.exists(path):
            raise ImportError(
                f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; "
                "g.build()'` (hipcc --offload-arch=gfx950; g++ for the CPU variant). There is no "
                "fallback.")
        l = ctypes.CDLL(path)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(l, name)
            fn.restype = res
            fn.argtypes = args
        if l.craft_abi_version() != ABI_VERSION:
            raise ImportError(f"{path}: ABI version {l.craft_abi_version()}, this binding is "
                              f"{ABI_VERSION} (include/craft.h CRAFT_ABI_VERSION); rebuild it")
        _libs[cpu] = l
    return l


def strerror(status, L=None):
    return (L or lib()).craft_strerror(status).decode()


def check(status, handle=None, what="", L=None):
    """Raise CraftError for a non-zero status; L: the library the handle belongs to."""
    if status != OK:
        L = L or lib()
        msg = strerror(status, L)
        if handle:
            detail = L.craft_sim_last_error(handle)
            if detail:
                msg = detail.decode()
        raise CraftError(status, f"{what}: {msg}" if what else msg)
