"""ctypes mirror of include/rmx.h and the loader of the in-tree HIP library ``librmx.so``.

The library is built by ``__graft_entry__.build()`` (hipcc --offload-arch=gfx950) next to this file.
There is no fallback: if the library is missing or fails to load, every engine entry point raises.
"""
from __future__ import annotations

import ctypes as C
import importlib.util
import os

from .tables import CompiledTables

LIB_NAME = "librmx.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)

RMX_OK, RMX_E_INVALID, RMX_E_HIP, RMX_E_ACTION, RMX_E_STATE = 0, -1, -2, -3, -4
F_ACTIVE, F_FAIL, F_TERM, F_TRUNC, F_ENV_TERM, F_RM_TERM, F_ENV_DONE = 0x01, 0x02, 0x04, 0x08, 0x10, 0x20, 0x40
F_STEPS_SHIFT = 16
NSTATS = 4
STAT_SUM_RETURN, STAT_EPISODES, STAT_SUCCESSES, STAT_SUM_LENGTH = 0, 1, 2, 3

# every symbol include/rmx.h declares (checked by tests/test_capi.py)
EXPORTS = (
    "rmx_abi_version", "rmx_last_error", "rmx_build_info", "rmx_create", "rmx_destroy", "rmx_bind", "rmx_reset",
    "rmx_step", "rmx_step_hashed", "rmx_fill_actions", "rmx_rollout", "rmx_stats_device", "rmx_stats_host",
    "rmx_stats_clear", "rmx_check_errors", "rmx_mdp_states", "rmx_mdp", "rmx_step_variant", "rmx_state_bytes",
    "rmx_get_state", "rmx_set_state", "rmx_step_report", "rmx_step_report_fused", "rmx_reset_sync", "rmx_step_sync",
    "rmx_step_sync_begin", "rmx_sync_wait", "rmx_sync_end", "rmx_step_seq", "rmx_queue_counters", "rmx_queue_info",
    "rmx_code_object_check", "rmx_device_count", "rmx_queue_timing", "rmx_queue_times",
)
SYNC_MAX_ENVS = 256  # RMX_SYNC_MAX_ENVS
QUEUE_INFO_N = 7  # RMX_QUEUE_INFO_N
QUEUE_STATES = ("unused", "ready", "unavailable", "retired")  # RMX_QUEUE_*
SEQ_DISPATCH = ("none", "queue", "stream:kernel", "stream:disabled", "stream:queue", "host")  # RMX_SEQ_*
VARIANT_GENERIC, VARIANT_LANE_PER_AGENT, VARIANT_FAST, VARIANT_FAST_LANE_PER_AGENT, VARIANT_HOST = 0, 1, 2, 3, 4
DEVICE_HOST = -1  # RMX_DEVICE_HOST: rmx_config.device of a host handle (the CPU path, csrc/rmx_hoststep.cpp)


ABI_VERSION = 11  # include/rmx.h RMX_ABI_VERSION

# The sources whose SHA-256 (concatenated in this order) librmx.so reports through rmx_build_info(): the same
# list as RMX_HASHED in csrc/Makefile (tests/test_capi.py checks that they agree).
CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")
HASHED_SOURCES = ("rmx_kernels.hip", "rmx_fast.hip", "rmx_sync.hip", "rmx_capi.cpp", "rmx_queue.cpp", "rmx_tables.cpp",
                  "rmx_comd.cpp", "rmx_build_info.cpp", "rmx_internal.h", "rmx_layout.h", "rmx_host.h", "rmx_device.h",
                  "rmx_generic.h", "rmx_comd.h", "rmx_hoststep.cpp", "rmx_hoststep.h", "../../include/rmx.h",
                  "Makefile")


def source_hash(csrc: str = CSRC) -> str:
    """First 16 hex digits of the SHA-256 of the engine sources in the tree (the Makefile's digest)."""
    import hashlib

    h = hashlib.sha256()
    for f in HASHED_SOURCES:
        with open(os.path.join(csrc, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_info(lib=None) -> dict:
    """rmx_build_info() of the loaded library as a dict (src, abi, arch)."""
    lib = lib or load_library(check_source=False)
    return dict(kv.split("=", 1) for kv in lib.rmx_build_info().decode().split())


class RmxConfig(C.Structure):
    _fields_ = [
        ("kind", C.c_int32), ("width", C.c_int32), ("height", C.c_int32), ("n_agents", C.c_int32),
        ("n_rm_states", C.c_int32), ("n_events", C.c_int32), ("max_t", C.c_int32), ("device", C.c_int32),
        ("n_envs", C.c_int64), ("env_offset", C.c_int64), ("n_envs_global", C.c_int64),
        ("hazard_penalty", C.c_float), ("wall_penalty", C.c_float), ("hazard_fail", C.c_int32),
        ("wall_fail", C.c_int32), ("gamma", C.c_float), ("has_shaping", C.c_int32),
        ("reward_modifier", C.c_float), ("n_qrm_max", C.c_int32),
        ("stochastic", C.c_int32), ("slip_n", C.c_int32 * 4), ("slip_out", (C.c_int32 * 4) * 4),
        ("slip_cdf", (C.c_double * 4) * 4), ("seed_scale", C.c_uint64), ("seed_env_stride", C.c_uint64),
        ("seed_episode_stride", C.c_uint64), ("random_starts", C.c_int32),
        ("cell", C.c_void_p), ("cell_event", C.c_void_p), ("next_q", C.c_void_p), ("rm_reward", C.c_void_p),
        ("shape", C.c_void_p), ("init_q", C.c_void_p), ("final_q", C.c_void_p), ("start_xy", C.c_void_p),
        ("n_qrm", C.c_void_p), ("qrm_states", C.c_void_p), ("enc_nq", C.c_void_p),
    ]


class RmxBuffers(C.Structure):
    _fields_ = [(n, C.c_void_p) for n in
                ("pos_x", "pos_y", "rm_q", "flags", "ep_ret", "t", "reward", "shaping", "env_done", "renv",
                 "qrm_s", "qrm_sn", "qrm_rq", "qrm_done", "rng", "episode", "enc_state")]


def make_config(tab: CompiledTables, n_envs: int, env_offset: int = 0, n_envs_global: int = None,
                device: int = 0):
    """Build an RmxConfig; returns (config, keepalive) — keep ``keepalive`` referenced while the
    config's host pointers are in use (rmx_create copies the tables)."""
    import numpy as np

    arrays = {
        "cell": np.ascontiguousarray(tab.cell, np.uint16),
        "cell_event": np.ascontiguousarray(tab.cell_event, np.uint8),
        "next_q": np.ascontiguousarray(tab.next_q, np.uint8),
        "rm_reward": np.ascontiguousarray(tab.rm_reward, np.float32),
        "init_q": np.ascontiguousarray(tab.init_q, np.int32),
        "final_q": np.ascontiguousarray(tab.final_q, np.int32),
        "start_xy": np.ascontiguousarray(tab.start_xy, np.int32),
    }
    if tab.shape is not None:
        arrays["shape"] = np.ascontiguousarray(tab.shape, np.float32)
    if tab.n_qrm is not None:
        arrays["n_qrm"] = np.ascontiguousarray(tab.n_qrm, np.int32)
        arrays["qrm_states"] = np.ascontiguousarray(tab.qrm_states, np.uint8)
    if tab.enc_nq is not None:  # state-encoder strides (QRM outputs, enc_state, get_mdp)
        arrays["enc_nq"] = np.ascontiguousarray(tab.enc_nq, np.int32)
    cfg = RmxConfig()
    cfg.kind, cfg.width, cfg.height = tab.kind, tab.width, tab.height
    cfg.n_agents, cfg.n_rm_states, cfg.n_events = tab.n_agents, tab.n_rm_states, tab.n_events
    cfg.max_t, cfg.device = tab.max_t, device
    cfg.n_envs, cfg.env_offset = int(n_envs), int(env_offset)
    cfg.n_envs_global = int(n_envs if n_envs_global is None else n_envs_global)
    cfg.hazard_penalty, cfg.wall_penalty = tab.hazard_penalty, tab.wall_penalty
    cfg.hazard_fail, cfg.wall_fail, cfg.gamma = tab.hazard_fail, tab.wall_fail, tab.gamma
    cfg.has_shaping = int(tab.shape is not None)
    cfg.reward_modifier = float(tab.reward_modifier)
    cfg.n_qrm_max = int(tab.qrm_states.shape[1]) if tab.n_qrm is not None and int(tab.n_qrm.max()) > 0 else 0
    cfg.stochastic = int(tab.stochastic)
    if tab.stochastic:
        for i in range(4):
            cfg.slip_n[i] = int(tab.slip_n[i])
            for j in range(4):
                cfg.slip_out[i][j] = int(tab.slip_out[i, j])
                cfg.slip_cdf[i][j] = float(tab.slip_cdf[i, j])
    cfg.seed_scale, cfg.seed_env_stride, cfg.seed_episode_stride = (int(v) & (2**64 - 1) for v in tab.seed_schedule)
    cfg.random_starts = int(tab.random_starts)
    for k, v in arrays.items():
        setattr(cfg, k, v.ctypes.data)
    return cfg, arrays


_LIB = None
_RUNTIME = []  # the HIP / HSA runtime files preloaded for librmx.so (keeps their handles alive)


def torch_hip_runtime():
    """The HIP and HSA runtime files bundled with PyTorch-ROCm, located without importing torch ([] without torch).

    torch's libraries ask for ``libamdhip64.so`` / ``libhsa-runtime64.so`` by file name, librmx.so for the SONAMEs
    ``libamdhip64.so.7`` / ``libhsa-runtime64.so.1`` (RUNPATH /opt/rocm), which torch's copies also carry.  Loaded
    AFTER torch, librmx.so therefore binds torch's runtime; loaded BEFORE it (a host-path user, or
    rmx.compat.default_device() counting devices) it would map /opt/rocm's, and a later ``import torch`` a second
    copy: two HIP runtimes in one process, the engine's unable to see the device that torch's holds."""
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return []
    d = os.path.join(os.path.dirname(spec.origin), "lib")
    return [os.path.join(d, n) for n in ("libhsa-runtime64.so", "libamdhip64.so") if os.path.exists(os.path.join(d, n))]


def load_library(path: str = None, check_source: bool = True):
    """Load librmx.so (fail loudly: there is no CPU fallback for the step engine).  RMX_LIB may point at
    a diagnostic build of the same ABI (scripts only).  The in-tree library must report the digest of the
    sources in this tree (rmx_build_info): a stale build is refused instead of silently run."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = path or os.environ.get("RMX_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise RuntimeError(f"rmx HIP library not built: {path} is missing (run __graft_entry__.build())")
    # one HIP runtime per process, whatever the import order: torch's when torch is installed (a no-op when torch is
    # already imported: the loader finds the same files mapped), so librmx.so's SONAME lookups resolve to it
    for rt in torch_hip_runtime():
        try:
            _RUNTIME.append(C.CDLL(rt, mode=os.RTLD_NOW | os.RTLD_GLOBAL))
        except OSError:  # a torch install whose runtime cannot load: librmx.so takes /opt/rocm's (torch would fail)
            break
    lib = C.CDLL(path)
    vp, i32, i64, u64 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64
    sig = {
        "rmx_abi_version": (C.c_int, []),
        "rmx_device_count": (C.c_int, [C.POINTER(C.c_int32)]),
        "rmx_last_error": (C.c_char_p, []),
        "rmx_build_info": (C.c_char_p, []),
        "rmx_state_bytes": (C.c_int, [vp, C.POINTER(C.c_size_t)]),
        "rmx_get_state": (C.c_int, [vp, vp, C.c_size_t]),
        "rmx_set_state": (C.c_int, [vp, vp, C.c_size_t]),
        "rmx_create": (C.c_int, [C.POINTER(RmxConfig), C.POINTER(vp)]),
        "rmx_destroy": (None, [vp]),
        "rmx_bind": (C.c_int, [vp, C.POINTER(RmxBuffers)]),
        "rmx_reset": (C.c_int, [vp, vp, u64, vp]),
        "rmx_step": (C.c_int, [vp, vp, C.c_int, vp]),
        "rmx_step_hashed": (C.c_int, [vp, u64, i64, C.c_int, vp]),
        "rmx_fill_actions": (C.c_int, [vp, u64, i64, i32, vp, vp]),
        "rmx_rollout": (C.c_int, [vp, u64, i64, i32, vp, vp]),
        "rmx_stats_device": (C.c_int, [vp, vp, vp]),
        "rmx_stats_host": (C.c_int, [vp, C.POINTER(C.c_double)]),
        "rmx_stats_clear": (C.c_int, [vp, vp]),
        "rmx_check_errors": (C.c_int, [vp]),
        "rmx_step_variant": (C.c_int, [vp]),
        "rmx_step_report": (C.c_int, [vp, vp, C.c_int, vp, vp]),
        "rmx_step_report_fused": (C.c_int, [vp]),
        "rmx_step_seq": (C.c_int, [vp, vp, C.c_int64, C.c_int32, C.c_int, vp, vp]),
        "rmx_queue_timing": (C.c_int, [vp, C.c_int]),
        "rmx_queue_times": (C.c_int, [vp, vp, C.c_int64, C.POINTER(C.c_int64)]),
        "rmx_queue_counters": (C.c_int, [vp, vp]),
        "rmx_queue_info": (C.c_int, [vp, vp, i32]),
        "rmx_code_object_check": (C.c_int, [vp, C.c_size_t, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.c_char_p,
                                            C.c_size_t]),
        "rmx_mdp_states": (C.c_int, [vp, i32, C.POINTER(C.c_int64)]),
        "rmx_mdp": (C.c_int, [vp, i32, i32, vp, vp, vp, vp]),
        "rmx_reset_sync": (C.c_int, [vp, u64, C.POINTER(RmxBuffers), vp]),
        "rmx_step_sync": (C.c_int, [vp, vp, C.c_int, C.POINTER(RmxBuffers), vp]),
        "rmx_step_sync_begin": (C.c_int, [vp, vp, C.c_int, vp]),
        "rmx_sync_wait": (C.c_int, [vp, C.POINTER(RmxBuffers)]),
        "rmx_sync_end": (C.c_int, [vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    if lib.rmx_abi_version() != ABI_VERSION:  # the ctypes structs below mirror include/rmx.h of that version
        raise RuntimeError(f"{path}: ABI {lib.rmx_abi_version()}, these bindings need {ABI_VERSION} (rebuild)")
    if check_source and os.path.exists(os.path.join(CSRC, "Makefile")) and \
            os.path.abspath(path) == os.path.abspath(LIB_PATH):
        got, want = build_info(lib).get("src"), source_hash()
        if got != want:
            raise RuntimeError(f"{path} was built from other sources (src={got}, tree={want}): rebuild it "
                               "(__graft_entry__.build())")
    _LIB = lib
    return lib


def device_count(lib=None) -> int:
    """HIP devices visible to this process (rmx_device_count; 0 without a driver or a device)."""
    lib = lib or load_library()
    n = C.c_int32()
    check(lib.rmx_device_count(C.byref(n)), "rmx_device_count")
    return n.value


def check(rc: int, what: str = "rmx"):
    if rc == RMX_OK:
        return
    msg = (_LIB.rmx_last_error() or b"").decode() if _LIB is not None else ""
    if rc in (RMX_E_INVALID, RMX_E_ACTION):
        raise ValueError(f"{what}: {msg} (rc={rc})")
    raise RuntimeError(f"{what}: {msg} (rc={rc})")
