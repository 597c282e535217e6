"""``VecRMEnv`` — N environments x A agents stepped by the gfx950 kernels behind include/rmx.h.

The batched equivalent of ``RMEnvironmentWrapper(env, agents)`` (rm_environment_wrapper.py:15-107)
over ``MultiAgentFrozenLake`` / ``MultiAgentOfficeWorld``: state lives in torch tensors on the GPU
(agent-major ``[A, N]`` columns), every call enqueues on torch's current HIP stream and returns
immediately; only ``stats()`` / ``check_errors()`` synchronise.

There is no silent CPU fallback: without ``librmx.so`` or without a GPU construction raises.  ``HostRMEnv``
below is the engine's explicit host path (a host handle of the same C ABI, ``device="cpu"``).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from . import _capi
from .tables import CompiledTables


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _mdp_dicts(A, arrays):
    """(all_P, all_num_states, all_num_actions) of get_mdp from each agent's (next, reward, done) host arrays."""
    all_P, all_ns, all_na = {}, {}, {}
    for a in range(A):
        nxt, rew, done = arrays(a)
        P = {}
        for s in range(nxt.shape[0]):
            P[s] = {k: ([] if done[s, k] == 255 else [(1.0, int(nxt[s, k]), float(rew[s, k]), bool(done[s, k]))])
                    for k in range(4)}
        all_P[a], all_ns[a], all_na[a] = P, nxt.shape[0], 4
    return all_P, all_ns, all_na


class VecRMEnv:
    """Batched RM environment on one GPU (one shard of a possibly multi-GPU job)."""

    def __init__(self, tables: CompiledTables, n_envs: int, device: int = 0, env_offset: int = 0,
                 n_envs_global: Optional[int] = None, with_renv: bool = True, with_env_done: bool = True,
                 with_qrm: bool = False, with_enc_state: bool = False):
        import torch

        if not torch.cuda.is_available():
            raise RuntimeError("VecRMEnv needs a ROCm GPU (the step engine has no CPU path)")
        self.torch = torch
        self.lib = _capi.load_library()
        self.tables = tables
        self.N, self.A = int(n_envs), tables.n_agents
        self.device = torch.device("cuda", device)
        self.cfg, self._keep = _capi.make_config(tables, n_envs, env_offset, n_envs_global, device)
        self.env_offset = int(env_offset)
        self.n_envs_global = int(self.cfg.n_envs_global)
        A, N, dev = self.A, self.N, self.device
        z = lambda shape, dt: torch.zeros(shape, dtype=dt, device=dev)  # noqa: E731
        self.pos_x = z((A, N), torch.int32)
        self.pos_y = z((A, N), torch.int32)
        self.rm_q = z((A, N), torch.int32)
        self.flags = z((A, N), torch.int32)  # uint32 bit layout (bit 31 never set)
        self.ep_ret = z((A, N), torch.float32)
        self.t = z((N,), torch.int32)
        self.reward = z((A, N), torch.float32)
        self.shaping = z((A, N), torch.float32) if tables.shape is not None else None
        self.env_done = z((N,), torch.uint8) if with_env_done else None
        self.renv = z((A, N), torch.float32) if with_renv else None
        # QRM counterfactual experiences [A][Qx][N] (rm_environment_wrapper.py:122-183)
        Qx = int(self.cfg.n_qrm_max)
        self.n_qrm_max = Qx
        q_on = with_qrm and Qx > 0
        self.qrm_s = z((A, Qx, N), torch.int32) if q_on else None
        self.qrm_sn = z((A, Qx, N), torch.int32) if q_on else None
        self.qrm_rq = z((A, Qx, N), torch.float32) if q_on else None
        self.qrm_done = z((A, Qx, N), torch.uint8) if q_on else None
        # stochastic slip / random starts: per-env numpy-PCG64 state [4][N] and episode counter (reset-seed
        # schedule)
        rng_on = bool(tables.stochastic or tables.random_starts)
        self.rng = z((4, N), torch.int64) if rng_on else None  # uint64 bit patterns
        self.episode = z((N,), torch.int32) if rng_on else None
        # learner input: the new observation encoded as state_encoder_*.encode does, (y*W + x)*nQ + q
        self.enc_state = z((A, N), torch.int32) if with_enc_state else None
        h = C.c_void_p()
        _capi.check(self.lib.rmx_create(C.byref(self.cfg), C.byref(h)), "rmx_create")
        self._h = h
        self._buf = _capi.RmxBuffers(*[_ptr(x) for x in (self.pos_x, self.pos_y, self.rm_q, self.flags, self.ep_ret,
                                                         self.t, self.reward, self.shaping, self.env_done, self.renv,
                                                         self.qrm_s, self.qrm_sn, self.qrm_rq, self.qrm_done,
                                                         self.rng, self.episode, self.enc_state)])
        _capi.check(self.lib.rmx_bind(self._h, C.byref(self._buf)), "rmx_bind")
        self._stats_dev = z((_capi.NSTATS,), torch.float64)
        self.reset()

    # -- stream plumbing --------------------------------------------------------------------------
    def _stream(self):
        # torch's current HIP stream on the engine's device as a raw pointer (the private getter skips building a
        # torch.cuda.Stream object: ~2 us of the host time of a short step window)
        raw = getattr(self.torch._C, "_cuda_getCurrentRawStream", None)
        if raw is not None:
            return C.c_void_p(raw(self.device.index))
        return C.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    # -- reference API --------------------------------------------------------------------------
    def reset(self, mask=None, seed: int = 123):
        """RMEnvironmentWrapper.reset for all envs (or those with mask[e] != 0)."""
        m = None
        if mask is not None:
            m = self.torch.as_tensor(mask, device=self.device).to(self.torch.uint8).contiguous()
            if m.numel() != self.N:
                raise ValueError("mask must have n_envs entries")
        _capi.check(self.lib.rmx_reset(self._h, _ptr(m), int(seed), self._stream()), "rmx_reset")

    def step(self, actions, autoreset: bool = True):
        """One wrapper step with caller-provided actions (int32 [A, N] device tensor, 0..4)."""
        a = actions
        if a.dtype is not self.torch.int32 or a.get_device() != self.device.index or not a.is_contiguous():
            a = a.to(device=self.device, dtype=self.torch.int32).contiguous()
        if a.numel() != self.A * self.N:
            raise ValueError(f"actions must be [A={self.A}, N={self.N}]")
        rc = self.lib.rmx_step(self._h, a.data_ptr(), 1 if autoreset else 0, self._stream())
        if rc:
            _capi.check(rc, "rmx_step")

    def step_report(self, actions, autoreset: bool = True, out=None):
        """step(actions) then the statistics report into `out` (device float64[4], default: the handle's
        stats tensor), as one launch where the handle's step kernel allows it (rmx_step_report)."""
        a = actions
        if a.dtype != self.torch.int32 or a.device != self.device or not a.is_contiguous():
            a = a.to(device=self.device, dtype=self.torch.int32).contiguous()
        if a.numel() != self.A * self.N:
            raise ValueError(f"actions must be [A={self.A}, N={self.N}]")
        o = self._stats_dev if out is None else out
        if o.dtype != self.torch.float64 or o.device != self.device or o.numel() != 4 or not o.is_contiguous():
            raise ValueError("out must be a contiguous float64[4] tensor on the engine's device")
        _capi.check(self.lib.rmx_step_report(self._h, _ptr(a), int(autoreset), _ptr(o), self._stream()),
                    "rmx_step_report")
        return o

    def step_seq(self, actions, autoreset: bool = True, out=None):
        """K steps in one submission (rmx_step_seq): actions is an int32 [K, A, N] device tensor, step k reads
        actions[k]; with `out` (device float64[4]) the K-th step is step_report's.  Results identical to K calls of
        step (and step_report); BLOCKING: returns once the steps are complete on the device.  The launches go to the
        engine's own AQL queue where the handle's step is the thread-per-env fast kernel."""
        a, t = actions, self.torch
        if a.dtype is not t.int32 or a.get_device() != self.device.index or not a.is_contiguous():
            raise ValueError("actions must be a contiguous int32 tensor on the engine's device")
        if a.dim() != 3 or a.numel() != a.shape[0] * self.A * self.N or a.shape[0] < 1:
            raise ValueError(f"actions must be [K >= 1, A={self.A}, N={self.N}]")
        if out is not None and (out.dtype is not t.float64 or out.get_device() != self.device.index
                                or out.numel() != 4 or not out.is_contiguous()):
            raise ValueError("out must be a contiguous float64[4] tensor on the engine's device")
        rc = self.lib.rmx_step_seq(self._h, a.data_ptr(), self.A * self.N, a.shape[0], 1 if autoreset else 0,
                                   None if out is None else out.data_ptr(), self._stream())
        if rc:
            _capi.check(rc, "rmx_step_seq")
        return out

    def seq_window(self, actions, autoreset: bool = True, out=None):
        """step_seq(actions, autoreset, out) checked once and bound: returns a callable that runs that window (the
        same K steps on the same buffers, whatever they hold when it is called) with no per-call argument work.
        The tensors must stay alive and in place while the callable is used."""
        a = actions
        if a.dtype is not self.torch.int32 or a.get_device() != self.device.index or not a.is_contiguous() \
                or a.dim() != 3 or a.shape[0] < 1 or a.numel() != a.shape[0] * self.A * self.N:
            raise ValueError(f"actions must be a contiguous int32 [K >= 1, A={self.A}, N={self.N}] tensor on the "
                             "engine's device")
        if out is not None and (out.dtype is not self.torch.float64 or out.get_device() != self.device.index
                                or out.numel() != 4 or not out.is_contiguous()):
            raise ValueError("out must be a contiguous float64[4] tensor on the engine's device")
        fn, h = self.lib.rmx_step_seq, self._h
        raw, index = getattr(self.torch._C, "_cuda_getCurrentRawStream", None), self.device.index
        stream = (lambda: raw(index)) if raw is not None else self._stream
        args = (a.data_ptr(), self.A * self.N, a.shape[0], 1 if autoreset else 0,
                None if out is None else out.data_ptr())
        keep = (a, out)

        def run():
            rc = fn(h, *args, stream())
            if rc:
                _capi.check(rc, "rmx_step_seq")
            return keep[1]
        return run

    def queue_counters(self) -> dict:
        """The device's step queue so far: windows submitted, kernel-argument uploads, packets, windows of the device
        served on a stream instead, and this handle's window recordings (all counts)."""
        i = self.queue_info()
        return {k: i[k] for k in ("windows", "uploads", "packets", "stream_windows", "recordings")}

    def queue_info(self) -> dict:
        """rmx_queue_info: the counters, the device queue's state ("unused", "ready", "unavailable", "retired") and
        how this handle's last step_seq ran ("none", "queue", "stream:kernel" (not the fast kernel),
        "stream:disabled" (RMX_QUEUE=0), "stream:queue" (the queue could not serve it))."""
        v = (C.c_int64 * _capi.QUEUE_INFO_N)()
        _capi.check(self.lib.rmx_queue_info(self._h, v, _capi.QUEUE_INFO_N), "rmx_queue_info")
        return {"windows": v[0], "uploads": v[1], "packets": v[2], "stream_windows": v[3],
                "state": _capi.QUEUE_STATES[v[4]], "dispatch": _capi.SEQ_DISPATCH[v[5]], "recordings": v[6]}

    def queue_timing(self, every: int = 1):
        """Dispatch timing on the device's queue from the next window on (rmx_queue_timing): packets 0, every,
        2*every, ... and each window's last one stamped by the command processor (start, end), the packets still back
        to back; 0 turns it off.  A stamped packet costs ~1.2 us more, so a sparse stride keeps the cadence."""
        _capi.check(self.lib.rmx_queue_timing(self._h, int(every)), "rmx_queue_timing")

    def queue_times(self):
        """The last timed window's stamps [n, 3] (packet index, start ns, end ns), dispatch order (rmx_queue_times);
        [0, 3] when the last window was not timed or ran on the stream."""
        n = C.c_int64()
        _capi.check(self.lib.rmx_queue_times(self._h, None, 0, C.byref(n)), "rmx_queue_times")
        out = np.zeros((n.value, 3), np.uint64)
        if n.value:
            _capi.check(self.lib.rmx_queue_times(self._h, out.ctypes.data, n.value, C.byref(n)), "rmx_queue_times")
        return out[: n.value]

    @property
    def report_fused(self) -> bool:
        """True if step_report computes the report inside the step launch for this handle."""
        return bool(self.lib.rmx_step_report_fused(self._h))

    def step_hashed(self, seed: int, t_global: int, autoreset: bool = True):
        """One step with actions from the SURVEY §8(d) counter hash, generated in-kernel."""
        _capi.check(self.lib.rmx_step_hashed(self._h, int(seed), int(t_global), int(autoreset), self._stream()),
                    "rmx_step_hashed")

    def fill_actions(self, seed: int, t0: int, T: int, out=None):
        """[T, A, N] int32 device tensor of hashed actions for global steps t0..t0+T-1."""
        if out is None:
            out = self.torch.empty((T, self.A, self.N), dtype=self.torch.int32, device=self.device)
        elif out.dtype is not self.torch.int32 or out.get_device() != self.device.index or not out.is_contiguous() \
                or out.numel() < max(int(T), 0) * self.A * self.N:  # the kernel writes T*A*N words at out's address
            raise ValueError("out must be a contiguous int32 tensor of >= T*A*N entries on the engine's device")
        _capi.check(self.lib.rmx_fill_actions(self._h, int(seed), int(t0), int(T), _ptr(out), self._stream()),
                    "rmx_fill_actions")
        return out

    def rollout(self, seed: int, t0: int, T: int, record_rewards: bool = False):
        """T fused autoreset steps with hashed actions; optionally returns the [T, A, N] reward trace."""
        trace = None
        if record_rewards:
            trace = self.torch.empty((T, self.A, self.N), dtype=self.torch.float32, device=self.device)
        _capi.check(self.lib.rmx_rollout(self._h, int(seed), int(t0), int(T), _ptr(trace), self._stream()),
                    "rmx_rollout")
        return trace

    # -- model construction ---------------------------------------------------------------------
    def mdp_arrays(self, agent: int, fix_frozen_lake: bool = False):
        """get_mdp of one agent as device arrays (next [S,4] int32, reward [S,4] f32, done [S,4] u8;
        done 255 / next -1 = no entry) — one launch over S*4 (state, action) pairs."""
        S = C.c_int64()
        _capi.check(self.lib.rmx_mdp_states(self._h, int(agent), C.byref(S)), "rmx_mdp_states")
        S = S.value
        t = self.torch
        nxt = t.empty((S, 4), dtype=t.int32, device=self.device)
        rew = t.empty((S, 4), dtype=t.float32, device=self.device)
        done = t.empty((S, 4), dtype=t.uint8, device=self.device)
        _capi.check(self.lib.rmx_mdp(self._h, int(agent), int(fix_frozen_lake), _ptr(nxt), _ptr(rew), _ptr(done),
                                     self._stream()), "rmx_mdp")
        return nxt, rew, done

    def get_mdp(self, fix_frozen_lake: bool = False):
        """(all_P, all_num_states, all_num_actions) keyed by agent index, in the reference's format
        P[s][a] = [(1.0, s', reward, done)] (rm_environment_wrapper.py:206-283)."""
        return _mdp_dicts(self.A, lambda a: (x.cpu().numpy() for x in self.mdp_arrays(a, fix_frozen_lake)))

    # -- statistics -------------------------------------------------------------------------------
    def stats_tensor(self):
        """Device float64[4] (sum return, episodes, successes, sum length), enqueued on the stream."""
        _capi.check(self.lib.rmx_stats_device(self._h, _ptr(self._stats_dev), self._stream()), "rmx_stats_device")
        return self._stats_dev

    def stats(self) -> np.ndarray:
        return self.stats_tensor().cpu().numpy().copy()

    def clear_stats(self):
        _capi.check(self.lib.rmx_stats_clear(self._h, self._stream()), "rmx_stats_clear")

    @property
    def step_variant(self) -> str:
        """Which step kernel this handle launches: "fast", "fast_lpe", "generic" or "lane_per_agent"."""
        v = self.lib.rmx_step_variant(self._h)
        return {_capi.VARIANT_FAST: "fast", _capi.VARIANT_FAST_LANE_PER_AGENT: "fast_lpe",
                _capi.VARIANT_GENERIC: "generic", _capi.VARIANT_LANE_PER_AGENT: "lane_per_agent"}[v]

    def check_errors(self):
        _capi.check(self.lib.rmx_check_errors(self._h), "rmx_check_errors")

    # -- views ----------------------------------------------------------------------------------
    def observations(self):
        """(pos_x, pos_y, rm_q) device tensors, [A, N] each (the reference obs dict + RM index).  Ends a resident
        synchronous workgroup first: it holds the env state in registers until it exits."""
        self.sync_end()
        return self.pos_x, self.pos_y, self.rm_q

    def flag(self, bit):
        self.sync_end()
        return (self.flags & bit) != 0

    # -- synchronous host-boundary calls (rmx_reset_sync / rmx_step_sync): the reference's per-call API --------
    def sync_end(self):
        """End the resident workgroup of the synchronous calls (rmx_sync_end): afterwards the device columns
        (and torch reads of them) are current.  Every asynchronous method of this class does it implicitly."""
        _capi.check(self.lib.rmx_sync_end(self._h), "rmx_sync_end")

    def _sync_out(self):
        """Host arrays (numpy) for every column a synchronous call returns, and their rmx_buffers."""
        if getattr(self, "_sy", None) is None:
            A, N = self.A, self.N
            out = {"pos_x": np.zeros((A, N), np.int32), "pos_y": np.zeros((A, N), np.int32),
                   "rm_q": np.zeros((A, N), np.int32), "flags": np.zeros((A, N), np.uint32),
                   "ep_ret": np.zeros((A, N), np.float32), "t": np.zeros(N, np.int32),
                   "reward": np.zeros((A, N), np.float32), "env_done": np.zeros(N, np.uint8),
                   "renv": np.zeros((A, N), np.float32)}
            if self.shaping is not None:
                out["shaping"] = np.zeros((A, N), np.float32)
            if self.tables.enc_nq is not None:
                out["enc_state"] = np.zeros((A, N), np.int32)
            if self.qrm_s is not None:
                Qx = self.n_qrm_max
                out.update({"qrm_s": np.zeros((A, Qx, N), np.int32), "qrm_sn": np.zeros((A, Qx, N), np.int32),
                            "qrm_rq": np.zeros((A, Qx, N), np.float32), "qrm_done": np.zeros((A, Qx, N), np.uint8)})
            b = _capi.RmxBuffers()
            for k, v in out.items():
                setattr(b, k, v.ctypes.data)
            self._sy = (out, b)
        return self._sy

    def reset_sync(self, seed: int = 123):
        """rmx_reset_sync: reset every env (seed = base of the reset-seed schedule) and return the columns after
        it as host numpy arrays (views reused by the next synchronous call).  N <= rmx._capi.SYNC_MAX_ENVS."""
        out, b = self._sync_out()
        _capi.check(self.lib.rmx_reset_sync(self._h, int(seed) & (2**64 - 1), C.byref(b), self._stream()),
                    "rmx_reset_sync")
        return out

    def step_sync(self, actions, autoreset: bool = False):
        """rmx_step_sync: one step with host actions (int32 [A, N], 0..4); returns the columns after the step as
        host numpy arrays (views reused by the next synchronous call).  No device tensor is touched."""
        a = np.ascontiguousarray(actions, dtype=np.int32)
        if a.size != self.A * self.N:
            raise ValueError(f"actions must be [A={self.A}, N={self.N}]")
        out, b = self._sync_out()
        _capi.check(self.lib.rmx_step_sync(self._h, a.ctypes.data, int(autoreset), C.byref(b), self._stream()),
                    "rmx_step_sync")
        return out

    def snapshot(self):
        """Host copy of every column (checkpoint: save with np.savez, restore with load_snapshot)."""
        self.sync_end()
        names = ("pos_x", "pos_y", "rm_q", "flags", "ep_ret", "t", "reward", "shaping", "env_done", "renv", "rng",
                 "episode", "enc_state")
        return {n: getattr(self, n).cpu().numpy().copy() for n in names if getattr(self, n) is not None}

    def load_snapshot(self, snap):
        self.sync_end()
        for n, v in snap.items():
            dst = getattr(self, n, None)
            if dst is not None:
                dst.copy_(self.torch.as_tensor(v).to(dst.dtype))

    # -- checkpoint / resume through the C ABI (rmx_get_state / rmx_set_state) ---------------------
    def save_state(self) -> bytes:
        """The resumable state of this shard (state columns, rng / episode columns, reset seed, episode
        statistics) as one opaque blob; synchronises.  Write it to disk as bytes / np.frombuffer."""
        n = C.c_size_t()
        _capi.check(self.lib.rmx_state_bytes(self._h, C.byref(n)), "rmx_state_bytes")
        buf = (C.c_ubyte * n.value)()
        _capi.check(self.lib.rmx_get_state(self._h, buf, n), "rmx_get_state")
        return bytes(buf)

    def load_state(self, blob: bytes):
        """Restore a save_state() blob of an engine with the same agents / envs / rng columns."""
        raw = (C.c_ubyte * len(blob)).from_buffer_copy(blob)
        _capi.check(self.lib.rmx_set_state(self._h, raw, len(blob)), "rmx_set_state")

    def close(self):
        if getattr(self, "_h", None):
            self.lib.rmx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HostRMEnv:
    """``VecRMEnv``'s interface on the CPU: a host handle of the same C ABI (rmx_config.device = RMX_DEVICE_HOST;
    csrc/rmx_hoststep.cpp steps the envs over the same compiled tables).  Columns are numpy arrays, ``[A, N]``
    agent-major; every call completes before it returns.  This is the engine's path for the reference's own CPU case
    (BASELINE config 1: one env behind the dict API, rmx.compat with ``device="cpu"``) and for machines without a GPU;
    no torch is imported."""

    device = "cpu"

    def __init__(self, tables: CompiledTables, n_envs: int, device="cpu", env_offset: int = 0,
                 n_envs_global: Optional[int] = None, with_renv: bool = True, with_env_done: bool = True,
                 with_qrm: bool = False, with_enc_state: bool = False):
        self.lib = _capi.load_library()
        self.tables = tables
        self.N, self.A = int(n_envs), tables.n_agents
        self.cfg, self._keep = _capi.make_config(tables, n_envs, env_offset, n_envs_global, _capi.DEVICE_HOST)
        self.env_offset = int(env_offset)
        self.n_envs_global = int(self.cfg.n_envs_global)
        A, N = self.A, self.N
        z = lambda shape, dt: np.zeros(shape, dtype=dt)  # noqa: E731
        self.pos_x, self.pos_y, self.rm_q = z((A, N), np.int32), z((A, N), np.int32), z((A, N), np.int32)
        self.flags = z((A, N), np.uint32)
        self.ep_ret = z((A, N), np.float32)
        self.t = z((N,), np.int32)
        self.reward = z((A, N), np.float32)
        self.shaping = z((A, N), np.float32) if tables.shape is not None else None
        self.env_done = z((N,), np.uint8) if with_env_done else None
        self.renv = z((A, N), np.float32) if with_renv else None
        Qx = int(self.cfg.n_qrm_max)
        self.n_qrm_max = Qx
        q_on = with_qrm and Qx > 0
        self.qrm_s = z((A, Qx, N), np.int32) if q_on else None
        self.qrm_sn = z((A, Qx, N), np.int32) if q_on else None
        self.qrm_rq = z((A, Qx, N), np.float32) if q_on else None
        self.qrm_done = z((A, Qx, N), np.uint8) if q_on else None
        rng_on = bool(tables.stochastic or tables.random_starts)
        self.rng = z((4, N), np.uint64) if rng_on else None
        self.episode = z((N,), np.int32) if rng_on else None
        self.enc_state = z((A, N), np.int32) if with_enc_state else None
        h = C.c_void_p()
        _capi.check(self.lib.rmx_create(C.byref(self.cfg), C.byref(h)), "rmx_create")
        self._h = h
        cols = (self.pos_x, self.pos_y, self.rm_q, self.flags, self.ep_ret, self.t, self.reward, self.shaping,
                self.env_done, self.renv, self.qrm_s, self.qrm_sn, self.qrm_rq, self.qrm_done, self.rng, self.episode,
                self.enc_state)
        self._buf = _capi.RmxBuffers(*[None if x is None else x.ctypes.data for x in cols])
        _capi.check(self.lib.rmx_bind(self._h, C.byref(self._buf)), "rmx_bind")
        self._stats = np.zeros(_capi.NSTATS, np.float64)
        self.reset()

    def reset(self, mask=None, seed: int = 123):
        m = None
        if mask is not None:
            m = np.ascontiguousarray(mask, dtype=np.uint8)
            if m.size != self.N:
                raise ValueError("mask must have n_envs entries")
        _capi.check(self.lib.rmx_reset(self._h, None if m is None else m.ctypes.data, int(seed) & (2**64 - 1), None),
                    "rmx_reset")

    def _acts(self, actions):
        a = np.ascontiguousarray(actions, dtype=np.int32)
        if a.size != self.A * self.N:
            raise ValueError(f"actions must be [A={self.A}, N={self.N}]")
        return a

    def step(self, actions, autoreset: bool = True):
        a = self._acts(actions)
        _capi.check(self.lib.rmx_step(self._h, a.ctypes.data, 1 if autoreset else 0, None), "rmx_step")

    @staticmethod
    def _out(out, dtype, n, what):
        """A caller's output array, checked before its address goes to C: the dtype, C order and >= n entries."""
        if not isinstance(out, np.ndarray) or out.dtype != dtype or not out.flags.c_contiguous or \
                not out.flags.writeable or out.size < n:
            raise ValueError(f"{what} must be a writeable C-contiguous {np.dtype(dtype).name} array of >= {n} entries")
        return out

    def step_report(self, actions, autoreset: bool = True, out=None):
        a = self._acts(actions)
        o = self._stats if out is None else self._out(out, np.float64, _capi.NSTATS, "out")
        _capi.check(self.lib.rmx_step_report(self._h, a.ctypes.data, int(autoreset), o.ctypes.data, None),
                    "rmx_step_report")
        return o

    def step_seq(self, actions, autoreset: bool = True, out=None):
        a = np.ascontiguousarray(actions, dtype=np.int32)
        if a.ndim != 3 or a.shape[0] < 1 or a.size != a.shape[0] * self.A * self.N:
            raise ValueError(f"actions must be [K >= 1, A={self.A}, N={self.N}]")
        if out is not None:
            self._out(out, np.float64, _capi.NSTATS, "out")
        _capi.check(self.lib.rmx_step_seq(self._h, a.ctypes.data, self.A * self.N, a.shape[0], 1 if autoreset else 0,
                                          None if out is None else out.ctypes.data, None), "rmx_step_seq")
        return out

    def step_hashed(self, seed: int, t_global: int, autoreset: bool = True):
        _capi.check(self.lib.rmx_step_hashed(self._h, int(seed), int(t_global), int(autoreset), None), "rmx_step_hashed")

    def fill_actions(self, seed: int, t0: int, T: int, out=None):
        if out is None:
            out = np.empty((T, self.A, self.N), np.int32)
        self._out(out, np.int32, max(int(T), 0) * self.A * self.N, "out")
        _capi.check(self.lib.rmx_fill_actions(self._h, int(seed), int(t0), int(T), out.ctypes.data, None),
                    "rmx_fill_actions")
        return out

    def rollout(self, seed: int, t0: int, T: int, record_rewards: bool = False):
        trace = np.empty((T, self.A, self.N), np.float32) if record_rewards else None
        _capi.check(self.lib.rmx_rollout(self._h, int(seed), int(t0), int(T), None if trace is None else trace.ctypes.data,
                                         None), "rmx_rollout")
        return trace

    def mdp_arrays(self, agent: int, fix_frozen_lake: bool = False):
        S = C.c_int64()
        _capi.check(self.lib.rmx_mdp_states(self._h, int(agent), C.byref(S)), "rmx_mdp_states")
        nxt = np.empty((S.value, 4), np.int32)
        rew = np.empty((S.value, 4), np.float32)
        done = np.empty((S.value, 4), np.uint8)
        _capi.check(self.lib.rmx_mdp(self._h, int(agent), int(fix_frozen_lake), nxt.ctypes.data, rew.ctypes.data,
                                     done.ctypes.data, None), "rmx_mdp")
        return nxt, rew, done

    def get_mdp(self, fix_frozen_lake: bool = False):
        return _mdp_dicts(self.A, lambda a: self.mdp_arrays(a, fix_frozen_lake))

    def stats_tensor(self):
        _capi.check(self.lib.rmx_stats_host(self._h, self._stats.ctypes.data_as(C.POINTER(C.c_double))), "rmx_stats_host")
        return self._stats

    def stats(self) -> np.ndarray:
        return self.stats_tensor().copy()

    def clear_stats(self):
        _capi.check(self.lib.rmx_stats_clear(self._h, None), "rmx_stats_clear")

    @property
    def step_variant(self) -> str:
        return {_capi.VARIANT_HOST: "host"}[self.lib.rmx_step_variant(self._h)]

    def check_errors(self):
        _capi.check(self.lib.rmx_check_errors(self._h), "rmx_check_errors")

    def observations(self):
        return self.pos_x, self.pos_y, self.rm_q

    def flag(self, bit):
        return (self.flags & bit) != 0

    def sync_end(self):
        _capi.check(self.lib.rmx_sync_end(self._h), "rmx_sync_end")

    _sync_out = VecRMEnv._sync_out

    def reset_sync(self, seed: int = 123):
        out, b = self._sync_out()
        _capi.check(self.lib.rmx_reset_sync(self._h, int(seed) & (2**64 - 1), C.byref(b), None), "rmx_reset_sync")
        return out

    def step_sync(self, actions, autoreset: bool = False):
        a = self._acts(actions)
        out, b = self._sync_out()
        _capi.check(self.lib.rmx_step_sync(self._h, a.ctypes.data, int(autoreset), C.byref(b), None), "rmx_step_sync")
        return out

    def snapshot(self):
        names = ("pos_x", "pos_y", "rm_q", "flags", "ep_ret", "t", "reward", "shaping", "env_done", "renv", "rng",
                 "episode", "enc_state")
        return {n: getattr(self, n).copy() for n in names if getattr(self, n) is not None}

    def load_snapshot(self, snap):
        for n, v in snap.items():
            dst = getattr(self, n, None)
            if dst is not None:
                dst[...] = np.asarray(v).view(dst.dtype) if np.asarray(v).dtype.itemsize == dst.dtype.itemsize \
                    else np.asarray(v).astype(dst.dtype)

    queue_info = VecRMEnv.queue_info  # (a host handle has no device queue: "unused"; step_seq reports "host")
    queue_timing = VecRMEnv.queue_timing  # (no-op on a host handle; queue_times is then empty)
    queue_times = VecRMEnv.queue_times
    queue_counters = VecRMEnv.queue_counters
    save_state = VecRMEnv.save_state
    load_state = VecRMEnv.load_state
    close = VecRMEnv.close
    __del__ = VecRMEnv.__del__


def make_env(tables: CompiledTables, n_envs: int, device=0, **kw):
    """A VecRMEnv on GPU `device`, or a HostRMEnv for device="cpu"."""
    if device == "cpu":
        return HostRMEnv(tables, n_envs, **kw)
    return VecRMEnv(tables, n_envs, device=device, **kw)
