"""The C ABI driven from plain ctypes + the HIP runtime, with no torch anywhere: device
columns from hipMalloc, rmx_create / bind / reset / fill_actions / step / step_report / stats / get_state, the
results copied back with hipMemcpy and checked against the CPU oracle.  This is how a caller that is not torch
(the reference's numpy loop, a C host) binds the engine."""
import ctypes as C

import numpy as np
import pytest

import oracle as O
from rmx import _capi
from rmx import tables as T

pytestmark = pytest.mark.gpu

H2D, D2H = 1, 2  # hipMemcpyHostToDevice, hipMemcpyDeviceToHost


class Hip:
    def __init__(self):
        self.lib = C.CDLL("libamdhip64.so")
        self.lib.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
        self.lib.hipFree.argtypes = [C.c_void_p]
        self.lib.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        self.lib.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
        self.lib.hipDeviceSynchronize.argtypes = []
        self.ptrs = []

    def alloc(self, nbytes):
        p = C.c_void_p()
        assert self.lib.hipMalloc(C.byref(p), nbytes) == 0
        assert self.lib.hipMemset(p, 0, nbytes) == 0
        self.ptrs.append(p)
        return p

    def get(self, p, shape, dtype):
        out = np.empty(shape, dtype)
        assert self.lib.hipMemcpy(out.ctypes.data_as(C.c_void_p), p, out.nbytes, D2H) == 0
        return out

    def free(self):
        for p in self.ptrs:
            self.lib.hipFree(p)


@pytest.mark.parametrize("mode", ["steps", "seq"])
@pytest.mark.parametrize("cfg_id", [2, 5])
def test_raw_ctypes_caller_matches_oracle(cfg_id, mode):
    """mode "seq": the same steps as rmx_step_seq windows of 25 (the engine's own queue), the last one reporting."""
    hip = Hip()
    lib = _capi.load_library()
    tab = T.compile_scenario(T.baseline_scenario(cfg_id))
    N, A, Tn, seed = 8192, tab.n_agents, 300, 31
    cfg, keep = _capi.make_config(tab, N)
    h = C.c_void_p()
    assert lib.rmx_create(C.byref(cfg), C.byref(h)) == 0, lib.rmx_last_error()
    try:
        b = _capi.RmxBuffers()
        cols = {}
        for name, nbytes in (("pos_x", 4 * A * N), ("pos_y", 4 * A * N), ("rm_q", 4 * A * N), ("flags", 4 * A * N),
                             ("ep_ret", 4 * A * N), ("t", 4 * N), ("reward", 4 * A * N), ("env_done", N)):
            cols[name] = hip.alloc(nbytes)
            setattr(b, name, cols[name])
        if tab.shape is not None:
            cols["shaping"] = hip.alloc(4 * A * N)
            b.shaping = cols["shaping"]
        assert lib.rmx_bind(h, C.byref(b)) == 0, lib.rmx_last_error()
        assert lib.rmx_reset(h, None, 0, None) == 0
        acts = hip.alloc(4 * Tn * A * N)
        assert lib.rmx_fill_actions(h, seed, 0, Tn, acts, None) == 0
        stats_dev = hip.alloc(8 * 4)
        orc = O.OracleEnv(tab, N)
        host = O.hash_actions(seed, 0, Tn, N, 0, N, A)
        K = 25
        for s in range(Tn):
            ptr = C.c_void_p(acts.value + 4 * s * A * N)
            if mode == "seq":
                if s % K == 0:
                    last = s + K >= Tn
                    assert lib.rmx_step_seq(h, ptr, A * N, K, 1, stats_dev if last else None, None) == 0, \
                        lib.rmx_last_error()
            elif s == Tn - 1:
                assert lib.rmx_step_report(h, ptr, 1, stats_dev, None) == 0, lib.rmx_last_error()
            else:
                assert lib.rmx_step(h, ptr, 1, None) == 0, lib.rmx_last_error()
            orc.step(host[s])
        if mode == "seq":
            q = (C.c_int64 * 3)()
            assert lib.rmx_queue_counters(h, q) == 0 and q[2] >= Tn
        assert lib.rmx_check_errors(h) == 0, lib.rmx_last_error()
        for name, ref in (("pos_x", orc.pos_x), ("pos_y", orc.pos_y), ("rm_q", orc.rm_q)):
            np.testing.assert_array_equal(hip.get(cols[name], (A, N), np.int32), ref, err_msg=name)
        np.testing.assert_array_equal(hip.get(cols["flags"], (A, N), np.uint32), orc.flags)
        np.testing.assert_array_equal(hip.get(cols["t"], (N,), np.int32), orc.t)
        np.testing.assert_array_equal(hip.get(cols["env_done"], (N,), np.uint8), orc.env_done)
        np.testing.assert_array_equal(hip.get(cols["reward"], (A, N), np.float32), orc.reward)
        rep = hip.get(stats_dev, (4,), np.float64)
        host_stats = np.zeros(4, np.float64)
        assert lib.rmx_stats_host(h, host_stats.ctypes.data_as(C.POINTER(C.c_double))) == 0
        want = orc.stats
        for got in (rep, host_stats):
            assert got[1] == want[1] and got[2] == want[2] and got[3] == want[3], (got, want)
            np.testing.assert_allclose(got[0], want[0], rtol=1e-6, atol=1e-6)
        n = C.c_size_t()
        assert lib.rmx_state_bytes(h, C.byref(n)) == 0 and n.value > 0
        blob = C.create_string_buffer(n.value)
        assert lib.rmx_get_state(h, blob, n) == 0, lib.rmx_last_error()
        assert blob.raw[:8] == b"RMXSTATE"
    finally:
        lib.rmx_destroy(h)
        hip.free()
