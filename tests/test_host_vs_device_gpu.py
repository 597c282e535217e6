"""The engine's two paths agree: the host handle (csrc/rmx_hoststep.cpp) and the gfx950 kernels, on the same inputs.

- The dict API (BASELINE config 1's path) on every golden scenario: rmx.compat with device="cpu" (the host step) and
  device=0 (the resident workgroup behind rmx_step_sync) return the same five dicts step for step.
- The batched path at BASELINE shapes: HostRMEnv and VecRMEnv (the default fast kernel) from the same reset with the
  same hashed actions hold the same columns, statistics and rng columns.
Bar: integers and booleans identical, rewards within 1e-6 (the device may fuse the reward's multiply-add)."""
import os

import numpy as np
import pytest

from rmx import compat as CP
from rmx import engine as E
from rmx import tables as T
from test_compat_cpu import _golden_seed, _strip, _wrapper as _cpu_wrapper
from test_engine_gpu import RS_DERIVED

pytestmark = pytest.mark.gpu

SCENARIOS = [("fl2", 0), ("fl2_quirks", 3), ("ow2_final", 1), ("ow2_fail", 0), ("fl2_slip", 2), ("ow2_allslip", 1),
             ("fl2_delay", 5), ("fl2_randstart", 4), ("fl2_randstart_slip", 7), ("fl4", 1), ("ow1", 2), ("ow3", 0),
             ("ow1_map3", 1), ("fl2_initfinal", 0), ("fl2_finalnt", 3), ("fl2_open", 1), ("ow1_slip", 3),
             ("ow2_delay", 0), ("ow3_slip", 2), ("fl4_randstart_open", 5)]


def _dict_wrapper(desc, device):
    w, env, agents = _cpu_wrapper(desc, False)
    w.device = device
    w._build()
    assert isinstance(w._engine, E.HostRMEnv if device == "cpu" else E.VecRMEnv)
    return w, env, agents


def _close(a, b):
    return all(abs(a[k] - b[k]) <= 1e-6 for k in a) and set(a) == set(b)


@pytest.mark.parametrize("name,env_index", SCENARIOS)
def test_host_step_equals_resident_workgroup_on_golden(name, env_index, configs, golden_dir):
    g = dict(np.load(os.path.join(golden_dir, f"traj_{name}.npz")))
    desc = configs[name]
    (wh, envh, agh), (wg, envg, agg) = _dict_wrapper(desc, "cpu"), _dict_wrapper(desc, 0)
    base, episode = int(g["seed"]), 0
    rh = wh.reset(seed=_golden_seed(desc, base, env_index, episode))
    rg = wg.reset(seed=_golden_seed(desc, base, env_index, episode))
    assert rh[0] == rg[0]
    names = ["up", "down", "left", "right"]
    for s in range(g["actions"].shape[0]):
        outs = []
        for w, agents in ((wh, agh), (wg, agg)):
            outs.append(w.step({ag.name: CP.ActionRL(names[int(g["actions"][s, i, env_index])])
                                for i, ag in enumerate(agents)}))
        (oh, rwh, th, uh, ih), (og, rwg, tg, ug, ig) = outs
        assert oh == og and th == tg and uh == ug, s
        assert _close(rwh, rwg), (s, rwh, rwg)
        sh, sg = _strip(ih), _strip(ig)
        for n in sh:  # info dicts: same keys in the same order, floats within 1e-6, everything else equal
            assert [k for k, _ in sh[n]] == [k for k, _ in sg[n]], s
            for (k, vh), (_, vg) in zip(sh[n], sg[n]):
                assert (abs(vh - vg) <= 1e-6) if isinstance(vh, float) else vh == vg, (s, n, k)
        assert envh.timestep == envg.timestep and envh.agent_steps == envg.agent_steps
        assert envh.active_agents == envg.active_agents and envh.agent_fail == envg.agent_fail
        if g["env_done"][s, env_index]:
            episode += 1
            assert wh.reset(seed=_golden_seed(desc, base, env_index, episode))[0] == \
                wg.reset(seed=_golden_seed(desc, base, env_index, episode))[0]


@pytest.mark.parametrize("name", ["cfg2", "cfg3", "cfg4", "cfg5", "fl2_slip", "ow3_slip", "fl2_randstart_slip",
                                  "fl4_randstart_open"] + RS_DERIVED)
def test_batched_host_equals_fast_kernel(name, configs):
    tab = T.compile_scenario(T.baseline_scenario(int(name[3])) if name.startswith("cfg") else configs[name])
    N, Tn, seed, base = 65536 if name.startswith("cfg") else 8192, 300, 23, 9
    h, d = E.HostRMEnv(tab, N, with_enc_state=True), E.VecRMEnv(tab, N, with_enc_state=True)
    assert d.step_variant == "fast"
    h.reset(seed=base)
    d.reset(seed=base)
    for s in range(Tn):
        h.step_hashed(seed, s)
        d.step_hashed(seed, s)
        if s % 100 == 99 or s == Tn - 1:
            for k in ("pos_x", "pos_y", "rm_q", "t", "env_done", "enc_state") + (("rng", "episode") if h.rng is not None
                                                                                 else ()):
                np.testing.assert_array_equal(getattr(h, k), getattr(d, k).cpu().numpy().view(getattr(h, k).dtype),
                                              err_msg=k)
            np.testing.assert_array_equal(h.flags, d.flags.cpu().numpy().view(np.uint32))
            np.testing.assert_allclose(h.reward, d.reward.cpu().numpy(), rtol=0, atol=1e-6)
            np.testing.assert_allclose(h.ep_ret, d.ep_ret.cpu().numpy(), rtol=1e-6, atol=1e-6)
    sh, sd = h.stats(), d.stats()
    np.testing.assert_array_equal(sh[1:], sd[1:])
    np.testing.assert_allclose(sh[0], sd[0], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("name", ["fl2", "fl2_randstart_slip", "ow3_slip"])
def test_checkpoint_moves_between_host_and_device(name, configs):
    """A blob written by the host path resumes on the GPU and the other way round (the same versioned layout): the
    continued runs equal one uninterrupted run on either path."""
    tab = T.compile_scenario(configs[name])
    N, seed = 4096, 31
    h, d = E.HostRMEnv(tab, N), E.VecRMEnv(tab, N)
    h.reset(seed=7)
    for s in range(250):
        h.step_hashed(seed, s)
    d.load_state(h.save_state())  # host -> device
    for s in range(250, 500):
        h.step_hashed(seed, s)
        d.step_hashed(seed, s)
    h2 = E.HostRMEnv(tab, N)
    h2.load_state(d.save_state())  # device -> host
    for s in range(500, 700):
        h.step_hashed(seed, s)
        h2.step_hashed(seed, s)
    for k in ("pos_x", "pos_y", "rm_q", "flags", "t") + (("rng", "episode") if h.rng is not None else ()):
        np.testing.assert_array_equal(getattr(h, k), getattr(h2, k), err_msg=k)
    np.testing.assert_allclose(h.ep_ret, h2.ep_ret, rtol=1e-6, atol=1e-6)
    a, b = h.stats(), h2.stats()
    np.testing.assert_array_equal(a[1:], b[1:])
    np.testing.assert_allclose(a[0], b[0], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("name", ["cfg2", "cfg3", "cfg5", "fl2_slip", "ow3_slip", "fl4_randstart_open"])
def test_qrm_columns_host_equal_device(name, configs):
    """The QRM counterfactual columns (rm_environment_wrapper.py:140-183) of the host step and of the device step
    from the same state and actions: qrm_s / qrm_sn / qrm_done identical, qrm_rq within 1e-6."""
    tab = T.compile_scenario(T.baseline_scenario(int(name[3])) if name.startswith("cfg") else configs[name])
    N, seed = 4096, 17
    h, d = E.HostRMEnv(tab, N, with_qrm=True), E.VecRMEnv(tab, N, with_qrm=True)
    assert h.qrm_s is not None and d.qrm_s is not None
    h.reset(seed=3)
    d.reset(seed=3)
    for s in range(120):
        h.step_hashed(seed, s)
        d.step_hashed(seed, s)
        if s % 40 == 39:
            for k in ("qrm_s", "qrm_sn", "qrm_done", "pos_x", "rm_q"):
                np.testing.assert_array_equal(getattr(h, k), getattr(d, k).cpu().numpy(), err_msg=f"{s} {k}")
            np.testing.assert_allclose(h.qrm_rq, d.qrm_rq.cpu().numpy(), rtol=0, atol=1e-6)
    d.check_errors()
    h.check_errors()


@pytest.mark.parametrize("fix", [False, True])
@pytest.mark.parametrize("name", ["fl2", "fl2_quirks", "ow1", "ow3", "ow2_fail", "ow1_map3", "fl4"])
def test_mdp_host_equals_device(name, fix, configs):
    """get_mdp's arrays (rm_environment_wrapper.py:185-283) from the host handle and from mdp_kernel: identical."""
    tab = T.compile_scenario(configs[name])
    h, d = E.HostRMEnv(tab, 1), E.VecRMEnv(tab, 1)
    for a in range(tab.n_agents):
        hn, hr, hd = h.mdp_arrays(a, fix)
        dn, dr, dd = (x.cpu().numpy() for x in d.mdp_arrays(a, fix))
        np.testing.assert_array_equal(hn, dn)
        np.testing.assert_array_equal(hd, dd)
        np.testing.assert_allclose(hr, dr, rtol=0, atol=1e-6)


def test_host_handle_first_then_device_handle_in_a_fresh_process():
    """The order a CPU-path user meets: librmx.so loaded for a host handle (no torch yet; rmx.compat's
    default_device() counts devices the same way), then a device handle.  One HIP runtime serves both (rmx._capi
    preloads torch's), and the two paths agree.  Before that preload the device handle failed: 'hipSetDevice: no
    ROCm-capable device is detected'."""
    import subprocess
    import sys
    import textwrap

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {os.path.join(root, "multiagent-rl-rm_amd")!r})
        import numpy as np
        from rmx import _capi, engine as E, tables as T
        assert "torch" not in sys.modules
        tab = T.compile_scenario(T.baseline_scenario(2))
        h = E.HostRMEnv(tab, 4096)
        assert _capi.device_count() >= 1
        d = E.VecRMEnv(tab, 4096)
        for s in range(50):
            h.step_hashed(5, s)
            d.step_hashed(5, s)
        for k in ("pos_x", "pos_y", "rm_q", "t"):
            np.testing.assert_array_equal(getattr(h, k), getattr(d, k).cpu().numpy(), err_msg=k)
        d.check_errors()
        print("ok")
    """)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-3000:]
