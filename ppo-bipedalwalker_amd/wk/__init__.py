"""ctypes binding of libwk.so (include/wk_api.h) -- the MI355X batched walker engine.

This is plumbing for tests and bench.py: every call goes straight to the C ABI and
from there to HIP kernels on gfx950.  There is no CPU fallback: if libwk.so is
missing or no GPU is visible, construction raises.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# WK_LIB selects an alternative in-tree build (kernel A/B experiments)
LIB_PATH = os.environ.get("WK_LIB") or os.path.join(os.path.dirname(_HERE), "libwk.so")

STATE_FLOATS = 112
NPARAM = 6149
NPARAM_CRITIC = 897
NPAIRS = 9
NEV = 16  # WK_NEV event counters (wk_count_events)
IPC_HANDLE_BYTES = 128  # WK_IPC_HANDLE_BYTES: IPC handle + the device's PCI bus id
EVENTS = ["joint", "aabb_ll", "aabb_lf", "aabb_bf", "sat_ll", "sat_lf", "sat_bf", "imp_ll",
          "imp_lf", "imp_bf", "contacts", "substeps", "env_steps", "resets", "steps_lf", "steps_satll"]
ST_TORQUE, ST_POS, ST_PREV, ST_STEPS, ST_POSTRESET, ST_TERMINAL, ST_EPISODES = (
    100, 104, 106, 108, 109, 110, 111)
MATERIALS = {"Carpet": 0, "Ice": 1, "Rubber": 2, "Metal": 3, "Wood": 4, "Paper": 5,
             "Titanium": 6, "SuperRubber": 7}

# every symbol include/wk_api.h declares (checked by tests/test_boundary.py)
EXPORTS = [
    "wk_config_defaults", "wk_version", "wk_create", "wk_destroy", "wk_last_error", "wk_sync",
    "wk_num_envs", "wk_reset", "wk_set_materials", "wk_set_offsets", "wk_step",
    "wk_step_device", "wk_step_sampled", "wk_step_traced", "wk_get_obs", "wk_get_state", "wk_set_state",
    "wk_get_body_view", "wk_set_scene", "wk_get_prop_view", "wk_get_weights", "wk_set_weights", "wk_get_adam", "wk_set_adam",
    "wk_policy_sample", "wk_value", "wk_rollout", "wk_rollout_stats_get", "wk_get_trajectory",
    "wk_set_trajectory", "wk_compute_returns", "wk_ppo_update", "wk_train_batch",
    "wk_minibatch_gradient", "wk_save_weights", "wk_load_weights", "wk_format_weights",
    "wk_parse_weights", "wk_checkpoint_save", "wk_checkpoint_load",
    "wk_host_settings_defaults", "wk_config_to_json", "wk_config_from_json",
    "wk_config_save_json", "wk_config_load_json", "wk_collect_data", "wk_episode_log_count",
    "wk_episode_log_drain", "wk_loss_log_drain", "wk_write_data_file",
    "wk_comm_unique_id", "wk_comm_init", "wk_comm_init_host", "wk_allreduce_test", "wk_profile_enable",
    "wk_profile_get", "wk_profile_reset", "wk_count_events", "wk_snapshot", "wk_time_gradient",
    "wk_time_gradient_ex", "wk_grad_kernel", "wk_rollout_mapping",
    "wk_comm_ipc_handle", "wk_comm_init_ipc", "wk_comm_info", "wk_comm_set_timeout",
    "wk_comm_xch_profile", "wk_comm_xch_stamps", "wk_check_state", "wk_take_actions",
    "wk_object_update", "wk_joint_step", "wk_body_order",
]


def check_state(state):
    """wk_check_state (host only, no device): (ok, first bad walker, first bad record body)"""
    import numpy as np
    st = np.ascontiguousarray(state, dtype=np.float32)
    be, bb = C.c_int(), C.c_int()
    lib = load_library()
    r = lib.wk_check_state(st.ctypes.data, int(st.size // STATE_FLOATS), C.byref(be), C.byref(bb))
    return r == 0, be.value, bb.value


class WkConfig(C.Structure):
    """wk_config: Hyperparameters.cs:80-121 names and defaults + batched extensions."""
    _fields_ = [
        ("GameSpeed", C.c_int), ("Iterations", C.c_int), ("MaxTimesteps", C.c_int),
        ("RoughFloor", C.c_int), ("Epochs", C.c_int), ("BatchSize", C.c_int),
        ("UseGAE", C.c_int), ("NormalizeAdvantages", C.c_int), ("Gamma", C.c_float),
        ("Lambda", C.c_float), ("Epsilon", C.c_float), ("LogStandardDeviation", C.c_float),
        ("Alpha", C.c_float), ("Beta1", C.c_float), ("Beta2", C.c_float),
        ("AdamEpsilon", C.c_float), ("CriticNeuralNetwork", C.c_char_p),
        ("ActorNeuralNetwork", C.c_char_p), ("DeltaTime", C.c_float), ("Horizon", C.c_int),
        ("Minibatch", C.c_int), ("MinibatchGlobal", C.c_int), ("EnvOffset", C.c_int),
        ("RandomizeStart", C.c_int), ("RandomizeMaterial", C.c_int),
        ("LanesPerWalker", C.c_int),
    ]


class HostSettings(C.Structure):
    """wk_host_settings: SerializableHyperparameters' host-only fields (Hyperparameters.cs:11-77)."""
    _fields_ = [
        ("CollectData", C.c_int), ("SaveWeights", C.c_int),
        ("CriticNeuralNetwork", C.c_char * 256), ("ActorNeuralNetwork", C.c_char * 256),
        ("CriticWeightFileName", C.c_char * 256), ("ActorWeightFileName", C.c_char * 256),
        ("FilePath", C.c_char * 1024),
    ]


class EpisodeRec(C.Structure):
    _fields_ = [("total_reward", C.c_float), ("env", C.c_int32), ("length", C.c_int32),
                ("step", C.c_uint32)]


EPISODE_DTYPE = np.dtype([("total_reward", np.float32), ("env", np.int32), ("length", np.int32),
                          ("step", np.uint32)])


class PairTrace(C.Structure):
    _fields_ = [("aabb_hit", C.c_uint8 * 9), ("sat_hit", C.c_uint8 * 9),
                ("n_contacts", C.c_uint8 * 9), ("pad", C.c_uint8 * 5),
                ("normal", (C.c_float * 2) * 9), ("depth", C.c_float * 9),
                ("contact", ((C.c_float * 2) * 2) * 9), ("impulse", (C.c_float * 2) * 9),
                ("joint_depth", C.c_float * 4), ("joint_impulse", C.c_float * 4)]


TRACE_DTYPE = np.dtype([("aabb_hit", np.uint8, 9), ("sat_hit", np.uint8, 9),
                        ("n_contacts", np.uint8, 9), ("pad", np.uint8, 5),
                        ("normal", np.float32, (9, 2)), ("depth", np.float32, 9),
                        ("contact", np.float32, (9, 2, 2)), ("impulse", np.float32, (9, 2)),
                        ("joint_depth", np.float32, 4), ("joint_impulse", np.float32, 4)])
assert TRACE_DTYPE.itemsize == C.sizeof(PairTrace) == 140 + 144 + 72 + 32


class BodyView(C.Structure):
    _fields_ = [("n_vertices", C.c_int), ("vertices", (C.c_float * 2) * 6),
                ("centroid", C.c_float * 2), ("linear_velocity", C.c_float * 2),
                ("angular_velocity", C.c_float), ("angle", C.c_float), ("collided", C.c_int),
                ("is_static", C.c_int)]


SHAPES = {"Square": 0, "Triangle": 1, "Hexagon": 2}
MAX_PROPS, PROP_MAXV, SCENE_MAX_VERTS = 4, 24, 32


class Prop(C.Structure):
    """wk_prop: <Shape>.FromSize + SmoothCorners + velocities + acceleration (include/wk_api.h)"""
    _fields_ = [("shape", C.c_int32), ("smooth", C.c_int32), ("material", C.c_int32),
                ("is_static", C.c_int32), ("cx", C.c_float), ("cy", C.c_float),
                ("size", C.c_float), ("vx", C.c_float), ("vy", C.c_float), ("w", C.c_float),
                ("ax", C.c_float), ("ay", C.c_float)]


def make_prop(shape="Square", smooth=0, material="Wood", is_static=False, cx=0.0, cy=0.0,
              size=40.0, vx=0.0, vy=0.0, w=0.0, ax=0.0, ay=0.0):
    return Prop(SHAPES.get(shape, shape), int(smooth), MATERIALS.get(material, material),
                int(bool(is_static)), cx, cy, size, vx, vy, w, ax, ay)


class PropView(C.Structure):
    _fields_ = [("n_vertices", C.c_int), ("vertices", (C.c_float * 2) * PROP_MAXV),
                ("centroid", C.c_float * 2), ("linear_velocity", C.c_float * 2),
                ("angular_velocity", C.c_float), ("angle", C.c_float), ("is_static", C.c_int)]

    def vertex_array(self):
        return np.array(self.vertices, np.float32)[:self.n_vertices]


class PpoArgs(C.Structure):
    _fields_ = [("epochs", C.c_int), ("minibatch", C.c_int), ("minibatch_global", C.c_int),
                ("update_index", C.c_uint32)]


class RolloutStats(C.Structure):
    _fields_ = [("reward_sum", C.c_double), ("episodes", C.c_int64), ("env_steps", C.c_int64),
                ("fault_or", C.c_uint32), ("pad", C.c_int32)]


class Profile(C.Structure):
    _fields_ = [("physics_ms", C.c_double), ("physics_launches", C.c_int64),
                ("physics_env_steps", C.c_int64), ("grad_ms", C.c_double),
                ("grad_launches", C.c_int64), ("reduce_ms", C.c_double),
                ("reduce_launches", C.c_int64), ("adam_ms", C.c_double),
                ("adam_launches", C.c_int64), ("allreduce_ms", C.c_double),
                ("allreduce_calls", C.c_int64), ("returns_ms", C.c_double),
                ("returns_launches", C.c_int64), ("update_ms", C.c_double),
                ("update_calls", C.c_int64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib = None
# wk_host_allreduce_fn: int (*)(float* buf, int n, void* user)
HOST_ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_float), C.c_int, C.c_void_p)


def load_library(path=None):
    """Load libwk.so (raises OSError if it was not built)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise OSError(f"libwk.so not built at {p}: run __graft_entry__.build() "
                      "(or make -C ppo-bipedalwalker_amd)")
    # PyTorch-ROCm ships its own libamdhip64 / libhsa-runtime64 / librccl with the same
    # SONAMEs as /opt/rocm.  Loading torch first makes libwk.so bind to those copies, so
    # one process has exactly one HIP runtime (torch.cuda.synchronize() then also covers
    # libwk's stream).  Loading libwk first would pull in a second runtime under torch.
    try:
        import torch  # noqa: F401
    except Exception:  # torch is plumbing only; libwk.so stands alone without it
        pass
    lib = C.CDLL(p)
    P, I, F, U32, U64 = C.c_void_p, C.c_int, C.c_float, C.c_uint32, C.c_uint64
    fp = C.POINTER(C.c_float)
    sig = {
        "wk_config_defaults": (None, [C.POINTER(WkConfig)]),
        "wk_version": (C.c_char_p, []),
        "wk_create": (I, [C.POINTER(WkConfig), I, I, U64, C.POINTER(P)]),
        "wk_destroy": (I, [P]),
        "wk_last_error": (C.c_char_p, [P]),
        "wk_sync": (I, [P]),
        "wk_num_envs": (I, [P]),
        "wk_reset": (I, [P, P]),
        "wk_set_materials": (I, [P, P]),
        "wk_set_offsets": (I, [P, P]),
        "wk_step": (I, [P, P, I, P, P, P, P]),
        "wk_step_device": (I, [P, P, I, P, P, P, P]),
        "wk_step_traced": (I, [P, P, P]),
        "wk_step_sampled": (I, [P, I, P, P, P, P, P, P, P, P, P]),
        "wk_get_obs": (I, [P, P]),
        "wk_get_state": (I, [P, P]),
        "wk_set_state": (I, [P, P]),
        "wk_get_body_view": (I, [P, I, I, C.POINTER(BodyView)]),
        "wk_set_scene": (I, [P, P, I]),
        "wk_get_prop_view": (I, [P, I, I, C.POINTER(PropView)]),
        "wk_get_weights": (I, [P, P]),
        "wk_set_weights": (I, [P, P]),
        "wk_get_adam": (I, [P, P, P, C.POINTER(C.c_int)]),
        "wk_set_adam": (I, [P, P, P, I]),
        "wk_policy_sample": (I, [P, I, P, P, P, P, P, P]),
        "wk_value": (I, [P, I, P, P]),
        "wk_rollout": (I, [P, I]),
        "wk_rollout_stats_get": (I, [P, C.POINTER(RolloutStats)]),
        "wk_get_trajectory": (I, [P, P, P, P, P, P, P, P, P]),
        "wk_set_trajectory": (I, [P, I, P, P, P, P, P, P]),
        "wk_compute_returns": (I, [P]),
        "wk_ppo_update": (I, [P, C.POINTER(PpoArgs), fp, fp]),
        "wk_train_batch": (I, [P, I, F, P, P, P, P, P, fp, fp, P, I, C.POINTER(C.c_int)]),
        "wk_minibatch_gradient": (I, [P, I, F, P, P, P, P, P, fp, fp, P, C.POINTER(C.c_int)]),
        "wk_save_weights": (I, [P, C.c_char_p, C.c_char_p]),
        "wk_load_weights": (I, [P, C.c_char_p, C.c_char_p]),
        "wk_format_weights": (I, [P, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t]),
        "wk_parse_weights": (I, [C.c_char_p, C.c_char_p, P]),
        "wk_checkpoint_save": (I, [P, C.c_char_p]),
        "wk_checkpoint_load": (I, [P, C.c_char_p]),
        "wk_host_settings_defaults": (None, [C.POINTER(HostSettings)]),
        "wk_config_to_json": (I, [C.POINTER(WkConfig), C.POINTER(HostSettings), C.c_char_p, C.c_size_t]),
        "wk_config_from_json": (I, [C.c_char_p, C.POINTER(WkConfig), C.POINTER(HostSettings)]),
        "wk_config_save_json": (I, [C.c_char_p, C.POINTER(WkConfig), C.POINTER(HostSettings)]),
        "wk_config_load_json": (I, [C.c_char_p, C.POINTER(WkConfig), C.POINTER(HostSettings)]),
        "wk_collect_data": (I, [P, I]),
        "wk_episode_log_count": (I, [P, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
        "wk_episode_log_drain": (I, [P, P, C.c_int64, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
        "wk_loss_log_drain": (I, [P, P, P, C.c_int64, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
        "wk_write_data_file": (I, [C.c_char_p, P, C.c_int64, P, C.c_int64, P, C.c_int64]),
        "wk_comm_unique_id": (I, [P]),
        "wk_comm_init": (I, [P, I, I, P]),
        "wk_allreduce_test": (I, [P, P, I]),
        "wk_comm_init_host": (I, [P, I, I, HOST_ALLREDUCE_FN, P]),
        "wk_time_gradient": (I, [P, I, I, C.POINTER(C.c_double)]),
        "wk_time_gradient_ex": (I, [P, I, I, I, C.POINTER(C.c_double)]),
        "wk_rollout_mapping": (I, [P, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int64),
                                   C.POINTER(C.c_int64)]),
        "wk_comm_info": (I, [P, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
        "wk_grad_kernel": (I, [P, I]),
        "wk_comm_ipc_handle": (I, [P, P]),
        "wk_comm_init_ipc": (I, [P, I, I, P]),
        "wk_comm_set_timeout": (I, [P, C.c_double]),
        "wk_comm_xch_profile": (I, [P, I]),
        "wk_check_state": (I, [P, I, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
        "wk_take_actions": (I, [P, I, P]),
        "wk_object_update": (I, [P, I, C.c_float]),
        "wk_joint_step": (I, [P]),
        "wk_body_order": (I, [P, I, P, C.POINTER(C.c_int)]),
        "wk_comm_xch_stamps": (I, [P, P, I, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
        "wk_profile_enable": (I, [P, I]),
        "wk_profile_get": (I, [P, C.POINTER(Profile)]),
        "wk_profile_reset": (I, [P]),
        "wk_count_events": (I, [P, I, P]),
        "wk_snapshot": (I, [P, I]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _ = U32
    if path is None:
        _lib = lib
    return lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _f32(a, shape=None):
    a = np.ascontiguousarray(a, dtype=np.float32)
    if shape is not None:
        a = a.reshape(shape)
    return a


WK_ERR_COMM = -4  # enum wk_status (include/wk_api.h)


class WkError(RuntimeError):
    pass


def default_config(**overrides):
    lib = load_library()
    c = WkConfig()
    lib.wk_config_defaults(C.byref(c))
    for k, v in overrides.items():
        if not hasattr(c, k):
            raise KeyError(f"unknown wk_config field {k}")
        if isinstance(v, str):
            v = v.encode()
        setattr(c, k, v)
    return c


def default_host_settings():
    h = HostSettings()
    load_library().wk_host_settings_defaults(C.byref(h))
    return h


def config_to_json(cfg=None, host=None):
    """Hyperparameters.SerializeJson (Hyperparameters.cs:124-131): the indented JSON text."""
    lib = load_library()
    cp = None if cfg is None else C.byref(cfg)
    hp = None if host is None else C.byref(host)
    need = -lib.wk_config_to_json(cp, hp, None, 0)
    if need <= 0:
        raise WkError(f"wk_config_to_json: {lib.wk_last_error(None).decode()}")
    buf = C.create_string_buffer(need)
    rc = lib.wk_config_to_json(cp, hp, buf, need)
    if rc != 0:
        raise WkError(f"wk_config_to_json failed ({rc}): {lib.wk_last_error(None).decode()}")
    return buf.value.decode()


def config_from_json(text, cfg=None, host=None):
    """Hyperparameters.DeserializeJson (Hyperparameters.cs:135-187) applied to (cfg, host)
    (defaults when None).  Returns (cfg, host, corrections): corrections lists the
    ValidateVariables messages (values reset to defaults).  Raises WkError when the
    document is malformed or a value is out of range (nothing is changed then)."""
    lib = load_library()
    cfg = default_config() if cfg is None else cfg
    host = default_host_settings() if host is None else host
    raw = text.encode() if isinstance(text, str) else bytes(text)
    rc = lib.wk_config_from_json(raw, C.byref(cfg), C.byref(host))
    msg = lib.wk_last_error(None).decode()
    if rc < 0:
        raise WkError(f"wk_config_from_json failed ({rc}): {msg}")
    cfg._host = host  # cfg's network strings point into host's buffers
    return cfg, host, (msg.split("\n") if rc > 0 else [])


def write_data_file(path, total_rewards, critic_losses, actor_losses):
    """ConsoleRenderer.CreateDataFile (ConsoleRenderer.cs:124-135)."""
    lib = load_library()
    r, c, a = (np.ascontiguousarray(x, np.float32) for x in (total_rewards, critic_losses, actor_losses))
    rc = lib.wk_write_data_file(os.fsencode(path), _ptr(r), r.size, _ptr(c), c.size, _ptr(a), a.size)
    if rc != 0:
        raise WkError(f"wk_write_data_file failed ({rc}): {lib.wk_last_error(None).decode()}")


def format_weights(params):
    """(critic_text, actor_text) of a WK_NPARAM vector in the reference's weights-file format
    (NeuralNetwork.Save NeuralNetwork.cs:159-176; one line per entry, newline-terminated)."""
    lib = load_library()
    p = _f32(params, (NPARAM,))
    need = -lib.wk_format_weights(_ptr(p), None, 0, None, 0)
    if need <= 0:
        raise WkError("wk_format_weights: size query failed")
    cb, ab = C.create_string_buffer(need), C.create_string_buffer(need)
    rc = lib.wk_format_weights(_ptr(p), cb, need, ab, need)
    if rc != 0:
        raise WkError(f"wk_format_weights failed ({rc})")
    return cb.value.decode(), ab.value.decode()


def parse_weights(critic_text, actor_text):
    """WK_NPARAM vector from weights-file texts (NeuralNetwork.Load NeuralNetwork.cs:94-115)."""
    lib = load_library()
    p = np.empty(NPARAM, np.float32)
    rc = lib.wk_parse_weights(critic_text.encode(), actor_text.encode(), _ptr(p))
    if rc != 0:
        raise WkError(f"wk_parse_weights failed ({rc}): {lib.wk_last_error(None).decode()}")
    return p


class Engine:
    """One wk_ctx: n_env walkers on one GPU."""

    def __init__(self, n_env, seed=20250905, device=0, **cfg):
        self.lib = load_library()
        self.cfg = default_config(**cfg)
        self.n = int(n_env)
        self.seed = int(seed)
        h = C.c_void_p()
        rc = self.lib.wk_create(C.byref(self.cfg), int(device), self.n, self.seed, C.byref(h))
        if rc != 0:
            raise WkError(f"wk_create failed ({rc}): {self.lib.wk_last_error(None).decode()}")
        self.h = h

    # -- plumbing --
    def _chk(self, rc, what):
        if rc != 0:
            msg = f"{what} failed ({rc}): {self.lib.wk_last_error(self.h).decode()}"
            if rc == WK_ERR_COMM and getattr(self, "_host_ar_error", None):
                msg += f" [host all-reduce callback raised {self._host_ar_error}; fatal for the job]"
                self._host_ar_error = None
            raise WkError(msg)

    def close(self):
        if getattr(self, "h", None):
            self.lib.wk_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def sync(self):
        self._chk(self.lib.wk_sync(self.h), "wk_sync")

    # -- environment --
    def reset(self, mask=None):
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        self._chk(self.lib.wk_reset(self.h, _ptr(m)), "wk_reset")

    def set_materials(self, mat):
        m = np.ascontiguousarray(mat, dtype=np.int32)
        self._chk(self.lib.wk_set_materials(self.h, _ptr(m)), "wk_set_materials")

    def set_offsets(self, dx):
        d = _f32(dx)
        self._chk(self.lib.wk_set_offsets(self.h, _ptr(d)), "wk_set_offsets")

    def step(self, actions=None, k=1):
        """k env-steps; actions [k, n, 4] (unclipped) or None to sample from the policy."""
        a = None if actions is None else _f32(actions, (k, self.n, 4))
        obs = np.empty((k, self.n, 12), np.float32)
        rew = np.empty((k, self.n), np.float32)
        done = np.empty((k, self.n), np.uint8)
        fault = np.empty(self.n, np.uint32)
        self._chk(self.lib.wk_step(self.h, _ptr(a), int(k), _ptr(obs), _ptr(rew), _ptr(done),
                                   _ptr(fault)), "wk_step")
        return obs, rew, done, fault

    def step_sampled(self, k=1):
        """Environment.Update with the agent's sampling (wk_step_sampled): the Trajectory
        entries of Environment.cs:70-89 -- states before each step, unclipped actions,
        per-dimension log-probabilities, values, rewards, dones -- the next states, and the
        torso position after each step before any auto-reset (Environment.cs:113-119)."""
        n = self.n
        out = dict(states=np.empty((k, n, 12), np.float32), actions=np.empty((k, n, 4), np.float32),
                   logp=np.empty((k, n, 4), np.float32), values=np.empty((k, n), np.float32),
                   rewards=np.empty((k, n), np.float32), dones=np.empty((k, n), np.uint8),
                   next_obs=np.empty((k, n, 12), np.float32), fault=np.empty(n, np.uint32),
                   position=np.empty((k, n, 2), np.float32))
        self._chk(self.lib.wk_step_sampled(
            self.h, int(k), _ptr(out["states"]), _ptr(out["actions"]), _ptr(out["logp"]),
            _ptr(out["values"]), _ptr(out["rewards"]), _ptr(out["dones"]), _ptr(out["next_obs"]),
            _ptr(out["fault"]), _ptr(out["position"])), "wk_step_sampled")
        return out

    def step_device(self, d_actions, k, d_obs, d_rew, d_done, d_fault):
        """Device-pointer variant (ints or None) on the context's stream; no sync."""
        self._chk(self.lib.wk_step_device(self.h, d_actions, int(k), d_obs, d_rew, d_done,
                                          d_fault), "wk_step_device")

    def step_traced(self, actions):
        a = _f32(actions, (self.n, 4))
        tr = np.zeros((self.n, self.cfg.Iterations), TRACE_DTYPE)
        self._chk(self.lib.wk_step_traced(self.h, _ptr(a), _ptr(tr)), "wk_step_traced")
        return tr

    def get_obs(self):
        o = np.empty((self.n, 12), np.float32)
        self._chk(self.lib.wk_get_obs(self.h, _ptr(o)), "wk_get_obs")
        return o

    def get_state(self):
        s = np.empty((self.n, STATE_FLOATS), np.float32)
        self._chk(self.lib.wk_get_state(self.h, _ptr(s)), "wk_get_state")
        return s

    def set_state(self, s):
        s = _f32(s, (self.n, STATE_FLOATS))
        self._chk(self.lib.wk_set_state(self.h, _ptr(s)), "wk_set_state")

    def body_view(self, env, body):
        v = BodyView()
        self._chk(self.lib.wk_get_body_view(self.h, int(env), int(body), C.byref(v)),
                  "wk_get_body_view")
        return v

    def set_scene(self, props):
        """scene props for every walker (Prop structures / make_prop(...)); [] removes them"""
        arr = (Prop * max(1, len(props)))(*props)
        self._chk(self.lib.wk_set_scene(self.h, C.cast(arr, C.c_void_p), len(props)),
                  "wk_set_scene")

    def prop_view(self, env, k):
        v = PropView()
        self._chk(self.lib.wk_get_prop_view(self.h, int(env), int(k), C.byref(v)),
                  "wk_get_prop_view")
        return v

    # -- policy --
    def get_weights(self):
        p = np.empty(NPARAM, np.float32)
        self._chk(self.lib.wk_get_weights(self.h, _ptr(p)), "wk_get_weights")
        return p

    def set_weights(self, p):
        p = _f32(p, (NPARAM,))
        self._chk(self.lib.wk_set_weights(self.h, _ptr(p)), "wk_set_weights")

    def get_adam(self):
        m = np.empty(NPARAM, np.float32)
        v = np.empty(NPARAM, np.float32)
        t = C.c_int()
        self._chk(self.lib.wk_get_adam(self.h, _ptr(m), _ptr(v), C.byref(t)), "wk_get_adam")
        return m, v, t.value

    def set_adam(self, m, v, t):
        m = _f32(m, (NPARAM,))
        v = _f32(v, (NPARAM,))
        self._chk(self.lib.wk_set_adam(self.h, _ptr(m), _ptr(v), int(t)), "wk_set_adam")

    def save_weights(self, critic_path, actor_path):
        """PPOAgent.Save (PPOAgent.cs:192-213): critic / actor weights text files."""
        self._chk(self.lib.wk_save_weights(self.h, os.fsencode(critic_path), os.fsencode(actor_path)),
                  "wk_save_weights")

    def load_weights(self, critic_path, actor_path):
        """PPOAgent.Load over NeuralNetwork.Load (NeuralNetwork.cs:94-115), strict errors."""
        self._chk(self.lib.wk_load_weights(self.h, os.fsencode(critic_path), os.fsencode(actor_path)),
                  "wk_load_weights")

    def checkpoint_save(self, path):
        """Binary checkpoint: weights, Adam state, walker records and Philox counters."""
        self._chk(self.lib.wk_checkpoint_save(self.h, os.fsencode(path)), "wk_checkpoint_save")

    def checkpoint_load(self, path):
        self._chk(self.lib.wk_checkpoint_load(self.h, os.fsencode(path)), "wk_checkpoint_load")

    # -- data collection (ConsoleRenderer.AddTotalEpisodeReward / AddCriticLoss / AddActorLoss) --
    def collect_data(self, on=True):
        self._chk(self.lib.wk_collect_data(self.h, int(bool(on))), "wk_collect_data")

    def episode_log_count(self):
        e, u = C.c_int64(), C.c_int64()
        self._chk(self.lib.wk_episode_log_count(self.h, C.byref(e), C.byref(u)), "wk_episode_log_count")
        return e.value, u.value

    def drain_episodes(self):
        """finished episodes since the last drain (structured array EPISODE_DTYPE) and the
        number dropped by overflow"""
        cnt, _ = self.episode_log_count()
        out = np.empty(cnt, EPISODE_DTYPE)
        n, dropped = C.c_int64(), C.c_int64()
        self._chk(self.lib.wk_episode_log_drain(self.h, _ptr(out) if cnt else None, cnt, C.byref(n),
                                                C.byref(dropped)), "wk_episode_log_drain")
        return out[:n.value], dropped.value

    def drain_losses(self):
        """(critic, actor) diagnostics of each PPO update since the last drain"""
        _, cnt = self.episode_log_count()
        cap = min(cnt, 1 << 16)
        c, a = np.empty(cap, np.float32), np.empty(cap, np.float32)
        n, dropped = C.c_int64(), C.c_int64()
        self._chk(self.lib.wk_loss_log_drain(self.h, _ptr(c) if cap else None, _ptr(a) if cap else None,
                                             cap, C.byref(n), C.byref(dropped)), "wk_loss_log_drain")
        return c[:n.value], a[:n.value]

    def policy_sample(self, obs, env_ids=None, steps=None):
        obs = _f32(obs)
        n = obs.shape[0]
        ids = None if env_ids is None else np.ascontiguousarray(env_ids, np.int32)
        st = None if steps is None else np.ascontiguousarray(steps, np.uint32)
        mean = np.empty((n, 4), np.float32)
        act = np.empty((n, 4), np.float32)
        lp = np.empty((n, 4), np.float32)
        self._chk(self.lib.wk_policy_sample(self.h, n, _ptr(obs), _ptr(ids), _ptr(st), _ptr(mean),
                                            _ptr(act), _ptr(lp)), "wk_policy_sample")
        return mean, act, lp

    def value(self, obs):
        obs = _f32(obs)
        v = np.empty(obs.shape[0], np.float32)
        self._chk(self.lib.wk_value(self.h, obs.shape[0], _ptr(obs), _ptr(v)), "wk_value")
        return v

    # -- rollout / PPO --
    def rollout(self, horizon=0):
        self._chk(self.lib.wk_rollout(self.h, int(horizon)), "wk_rollout")

    def rollout_stats(self):
        s = RolloutStats()
        self._chk(self.lib.wk_rollout_stats_get(self.h, C.byref(s)), "wk_rollout_stats_get")
        return s

    def get_trajectory(self, horizon):
        n = self.n * horizon
        out = dict(states=np.empty((horizon, self.n, 12), np.float32),
                   actions=np.empty((horizon, self.n, 4), np.float32),
                   logp=np.empty((horizon, self.n, 4), np.float32),
                   rewards=np.empty((horizon, self.n), np.float32),
                   dones=np.empty((horizon, self.n), np.uint8),
                   values=np.empty((horizon, self.n), np.float32),
                   returns=np.empty((horizon, self.n), np.float32),
                   advantages=np.empty((horizon, self.n), np.float32))
        assert n == out["rewards"].size
        self._chk(self.lib.wk_get_trajectory(
            self.h, _ptr(out["states"]), _ptr(out["actions"]), _ptr(out["logp"]),
            _ptr(out["rewards"]), _ptr(out["dones"]), _ptr(out["values"]), _ptr(out["returns"]),
            _ptr(out["advantages"])), "wk_get_trajectory")
        return out

    def set_trajectory(self, states, actions, logp, rewards, dones, values):
        T = rewards.shape[0]
        args = [_f32(states), _f32(actions), _f32(logp), _f32(rewards),
                np.ascontiguousarray(dones, np.uint8), _f32(values)]
        self._chk(self.lib.wk_set_trajectory(self.h, int(T), *[_ptr(a) for a in args]),
                  "wk_set_trajectory")

    def compute_returns(self):
        self._chk(self.lib.wk_compute_returns(self.h), "wk_compute_returns")

    def ppo_update(self, epochs=0, minibatch=0, minibatch_global=0, update_index=0, sync=True):
        """Whole PPO update; returns the last minibatch's (critic, actor) diagnostics, or
        (None, None) with sync=False (then nothing waits on the stream)."""
        a = PpoArgs(int(epochs), int(minibatch), int(minibatch_global), int(update_index))
        if not sync:
            self._chk(self.lib.wk_ppo_update(self.h, C.byref(a), None, None), "wk_ppo_update")
            return None, None
        cd, ad = C.c_float(), C.c_float()
        self._chk(self.lib.wk_ppo_update(self.h, C.byref(a), C.byref(cd), C.byref(ad)),
                  "wk_ppo_update")
        return cd.value, ad.value

    def train_batch(self, states, actions, logp_old, returns, adv, b_div=None, apply_adam=True):
        s, a, l, r, v = (_f32(states), _f32(actions), _f32(logp_old), _f32(returns), _f32(adv))
        B = r.shape[0]
        grads = np.empty(NPARAM, np.float32)
        cd, ad, sk = C.c_float(), C.c_float(), C.c_int()
        self._chk(self.lib.wk_train_batch(
            self.h, int(B), float(B if b_div is None else b_div), _ptr(s), _ptr(a), _ptr(l),
            _ptr(r), _ptr(v), C.byref(cd), C.byref(ad), _ptr(grads), int(bool(apply_adam)),
            C.byref(sk)), "wk_train_batch")
        return grads, cd.value, ad.value, sk.value

    def minibatch_gradient(self, states, actions, logp_old, returns, adv, b_div=None):
        """The matrix-core minibatch gradient wk_ppo_update applies (no Adam)."""
        s, a, l, r, v = (_f32(states), _f32(actions), _f32(logp_old), _f32(returns), _f32(adv))
        B = r.shape[0]
        grads = np.empty(NPARAM, np.float32)
        cd, ad, sk = C.c_float(), C.c_float(), C.c_int()
        self._chk(self.lib.wk_minibatch_gradient(
            self.h, int(B), float(B if b_div is None else b_div), _ptr(s), _ptr(a), _ptr(l),
            _ptr(r), _ptr(v), C.byref(cd), C.byref(ad), _ptr(grads), C.byref(sk)),
            "wk_minibatch_gradient")
        return grads, cd.value, ad.value, sk.value

    # -- multi-GPU --
    @staticmethod
    def comm_unique_id():
        lib = load_library()
        buf = (C.c_uint8 * 128)()
        rc = lib.wk_comm_unique_id(buf)
        if rc != 0:
            raise WkError(f"wk_comm_unique_id failed: {lib.wk_last_error(None).decode()}")
        return bytes(buf)

    def comm_init(self, rank, nranks, uid):
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        self._chk(self.lib.wk_comm_init(self.h, int(rank), int(nranks), buf), "wk_comm_init")

    def comm_init_host(self, rank, nranks, allreduce):
        """wk_comm_init_host: `allreduce(np.ndarray float32 view)` sums the slab over ranks in
        place (e.g. torch.distributed over gloo); the callback object is kept alive here.
        A callback that raises fails this rank's wk_ppo_update with WK_ERR_COMM while the
        peers wait inside their own all-reduce: the WkError carries the exception's text and
        must be treated as fatal for the whole job (let it propagate so the launcher tears the
        process group down; the ranks' replicas have diverged)."""
        self._host_ar_error = None

        def _cb(buf, n, user):
            try:
                allreduce(np.ctypeslib.as_array(buf, shape=(n,)))
                return 0
            except Exception as ex:  # noqa: BLE001 -- reported as WK_ERR_COMM by the library
                self._host_ar_error = f"{type(ex).__name__}: {ex}"
                return 1
        self._host_ar = HOST_ALLREDUCE_FN(_cb)
        self._chk(self.lib.wk_comm_init_host(self.h, int(rank), int(nranks), self._host_ar, None),
                  "wk_comm_init_host")

    def comm_ipc_handle(self):
        """wk_comm_ipc_handle: this rank's IPC_HANDLE_BYTES exchange record"""
        h = (C.c_uint8 * IPC_HANDLE_BYTES)()
        self._chk(self.lib.wk_comm_ipc_handle(self.h, h), "wk_comm_ipc_handle")
        return bytes(h)

    def comm_init_ipc_records(self, rank, nranks, records):
        """wk_comm_init_ipc with every rank's record (rank order)"""
        if len(records) != nranks or any(len(x) != IPC_HANDLE_BYTES for x in records):
            raise WkError(f"wk_comm_init_ipc: need one {IPC_HANDLE_BYTES}-byte record per rank")
        buf = (C.c_uint8 * (IPC_HANDLE_BYTES * nranks)).from_buffer_copy(b"".join(records))
        self._chk(self.lib.wk_comm_init_ipc(self.h, int(rank), int(nranks), buf),
                  "wk_comm_init_ipc")

    def comm_init_ipc(self, rank, nranks, allgather):
        """wk_comm_ipc_handle + wk_comm_init_ipc: the one-shot exchange over peer-mapped memory.
        `allgather(bytes) -> list of bytes` (rank order) exchanges the records over any control
        plane (e.g. torch.distributed.all_gather_object over gloo).  Every rank joins the
        all-gather even when its own handle failed (it sends b""), so the ranks' collectives
        stay paired; then every rank raises."""
        try:
            rec, why = self.comm_ipc_handle(), None
        except WkError as ex:
            rec, why = b"", str(ex)
        records = allgather(rec)
        if why is not None:
            raise WkError(why)
        bad = [r for r, x in enumerate(records) if len(x) != IPC_HANDLE_BYTES]
        if bad:
            raise WkError(f"wk_comm_init_ipc: rank(s) {bad} have no exchange record")
        self.comm_init_ipc_records(rank, nranks, records)

    def comm_set_timeout(self, seconds):
        """wk_comm_set_timeout: the IPC exchange's bounded peer wait (default 30 s, or
        WK_XCH_TIMEOUT_S at the mapping)"""
        self._chk(self.lib.wk_comm_set_timeout(self.h, float(seconds)), "wk_comm_set_timeout")

    COMM_KINDS = {0: "none", 1: "rccl", 2: "host", 3: "ipc"}

    def comm_info(self):
        """wk_comm_info: (exchange kind, whether the IPC region is uncached device memory)"""
        k, f = C.c_int(), C.c_int()
        self._chk(self.lib.wk_comm_info(self.h, C.byref(k), C.byref(f)), "wk_comm_info")
        return self.COMM_KINDS[k.value], bool(f.value & 1)

    # the reference's per-body call shape (Environment.StepObjects, Environment.cs:126-143)
    def take_actions(self, env, actions):
        """wk_take_actions: Walker.TakeActions for walker env (the next frame's torques)"""
        a = _f32(actions).reshape(4).copy()
        self._chk(self.lib.wk_take_actions(self.h, int(env), _ptr(a)), "wk_take_actions")

    def object_update(self, list_count, delta_time):
        """wk_object_update: one IObject.Update call; True when this call ran the frame's step"""
        r = self.lib.wk_object_update(self.h, int(list_count), float(delta_time))
        self._chk(min(r, 0), "wk_object_update")
        return r == 1

    def joint_step(self):
        self._chk(self.lib.wk_joint_step(self.h), "wk_joint_step")

    def body_order(self, env):
        """wk_body_order: walker env's body list as part ids (floor last in episode 0, first after
        a reset)"""
        parts, n = (C.c_int * 15)(), C.c_int()
        self._chk(self.lib.wk_body_order(self.h, int(env), parts, C.byref(n)), "wk_body_order")
        return list(parts[: n.value])

    def xch_profile(self, minibatches):
        """wk_comm_xch_profile: stamp the next exchange launches (a ring of `minibatches`; 0 off)"""
        self._chk(self.lib.wk_comm_xch_profile(self.h, int(minibatches)), "wk_comm_xch_profile")

    def xch_stamps(self, max_launches=1 << 16):
        """wk_comm_xch_stamps: uint64 [launches, blocks, 4] constant-clock ticks (10 ns) per block
        -- entry, slab published, peers' flags seen, exit -- for the last stamped launches"""
        import numpy as np
        n, b = C.c_int(), C.c_int()
        self._chk(self.lib.wk_comm_xch_stamps(self.h, None, 0, C.byref(n), C.byref(b)),
                  "wk_comm_xch_stamps")
        buf = np.zeros((max_launches, b.value, 4), np.uint64)
        self._chk(self.lib.wk_comm_xch_stamps(self.h, buf.ctypes.data, max_launches, C.byref(n),
                                              C.byref(b)), "wk_comm_xch_stamps")
        return buf[: n.value]

    def allreduce_test(self, x):
        x = _f32(x).copy()
        self._chk(self.lib.wk_allreduce_test(self.h, _ptr(x), x.size), "wk_allreduce_test")
        return x

    GRAD_KERNELS = {0: "k_ppo_grad_ws", 1: "k_ppo_grad_tp", 2: "k_ppo_grad_tp1",
                    3: "k_ppo_grad_mfma"}

    def grad_kernel(self, minibatch=0):
        """wk_grad_kernel: the name of the gradient kernel the update launches at this per-GPU
        minibatch (0 = config Minibatch)"""
        k = self.lib.wk_grad_kernel(self.h, int(minibatch))
        self._chk(k if k < 0 else 0, "wk_grad_kernel")
        return self.GRAD_KERNELS[k]

    def time_gradient(self, minibatch=0, reps=64, per_launch_events=False):
        """wk_time_gradient_ex: mean ms of the update's gradient kernel over `reps` back-to-back
        launches on minibatch 0 of the current trajectory -- one event pair around the burst,
        or (per_launch_events) one around every launch, as profile level 2 times the update"""
        ms = C.c_double()
        self._chk(self.lib.wk_time_gradient_ex(self.h, int(minibatch), int(reps),
                                               int(bool(per_launch_events)), C.byref(ms)),
                  "wk_time_gradient_ex")
        return ms.value

    def rollout_mapping(self):
        """wk_rollout_mapping: {lanes_per_walker, walkers_per_wave, waves (holding walkers),
        waves_launched (the grid, whole 4-wave blocks for the split kernels)} of a rollout launch"""
        L, w = C.c_int(), C.c_int()
        n, nl = C.c_int64(), C.c_int64()
        self._chk(self.lib.wk_rollout_mapping(self.h, C.byref(L), C.byref(w), C.byref(n),
                                              C.byref(nl)), "wk_rollout_mapping")
        return {"lanes_per_walker": L.value, "walkers_per_wave": w.value, "waves": n.value,
                "waves_launched": nl.value}

    # -- counting replay / snapshots --
    def count_events(self, k):
        """wk_count_events: replay the last rollout's first k action rows through the
        counting kernel; returns the WK_NEV event totals (see include/wk_api.h)."""
        c = np.zeros(NEV, np.uint64)
        self._chk(self.lib.wk_count_events(self.h, int(k), _ptr(c)), "wk_count_events")
        return c

    def snapshot(self):
        self._chk(self.lib.wk_snapshot(self.h, 0), "wk_snapshot")

    def restore(self):
        self._chk(self.lib.wk_snapshot(self.h, 1), "wk_snapshot")

    # -- profiling --
    def profile_enable(self, on=True):
        """on: False/0 off, True/1 per rollout / update, 2 per kernel launch as well"""
        self._chk(self.lib.wk_profile_enable(self.h, int(on)), "wk_profile_enable")

    def profile_reset(self):
        self._chk(self.lib.wk_profile_reset(self.h), "wk_profile_reset")

    def profile(self):
        p = Profile()
        self._chk(self.lib.wk_profile_get(self.h, C.byref(p)), "wk_profile_get")
        return p.as_dict()
