"""CPU-side checks of the C ABI: librmx.so loads (no GPU needed) and exports every symbol that
include/rmx.h declares; the ctypes signature table covers exactly that set."""
import json
import os
import re
import subprocess

import pytest

from rmx import _capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "rmx.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rmx_[a-z_]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    assert header_functions() == sorted(_capi.EXPORTS)


def test_library_exports_every_header_symbol():
    if not os.path.exists(_capi.LIB_PATH):
        pytest.skip("librmx.so not built (run __graft_entry__.build())")
    out = subprocess.run(["nm", "-D", "--defined-only", _capi.LIB_PATH], capture_output=True, text=True, check=True)
    syms = {ln.split()[-1] for ln in out.stdout.splitlines() if ln.strip()}
    missing = [f for f in header_functions() if f not in syms]
    assert not missing, missing


def test_library_loads_without_gpu():
    if not os.path.exists(_capi.LIB_PATH):
        pytest.skip("librmx.so not built")
    lib = _capi.load_library()
    assert lib.rmx_abi_version() == _capi.ABI_VERSION == 11
    for f in header_functions():
        assert hasattr(lib, f)


def test_hashed_source_list_matches_makefile():
    """rmx/_capi.py recomputes the library's source digest over the same files, in the same order, as the
    Makefile's RMX_HASHED."""
    mk = open(os.path.join(_capi.CSRC, "Makefile")).read()
    m = re.search(r"^RMX_HASHED := (.*?)(?<!\\)\n", mk, flags=re.S | re.M)
    files = tuple(m.group(1).replace("\\\n", " ").split())
    assert files == _capi.HASHED_SOURCES


def test_library_built_from_this_tree():
    """Provenance: the in-tree librmx.so reports the SHA-256 digest of exactly the sources in this tree
    (load_library refuses anything else), so a green GPU run can only come from a HEAD build."""
    if not os.path.exists(_capi.LIB_PATH):
        pytest.skip("librmx.so not built")
    info = _capi.build_info(_capi.load_library())
    assert info["src"] == _capi.source_hash()
    assert info["abi"] == str(_capi.ABI_VERSION) and info["arch"] == "gfx950"


def test_create_rejects_bad_config_without_touching_gpu():
    """Validation happens before any HIP call: a bad config fails with RMX_E_INVALID and a message."""
    import ctypes as C
    if not os.path.exists(_capi.LIB_PATH):
        pytest.skip("librmx.so not built")
    from rmx import tables as T
    lib = _capi.load_library()
    tab = T.compile_scenario(T.baseline_scenario(2))
    cfg, keep = _capi.make_config(tab, 16)
    cfg.n_agents = 9
    h = C.c_void_p()
    assert lib.rmx_create(C.byref(cfg), C.byref(h)) == _capi.RMX_E_INVALID
    assert b"n_agents" in lib.rmx_last_error()
    cfg.n_agents = 2
    tab.start_xy[0, 0] = 99
    cfg2, keep2 = _capi.make_config(tab, 16)
    assert lib.rmx_create(C.byref(cfg2), C.byref(h)) == _capi.RMX_E_INVALID
    assert b"start" in lib.rmx_last_error()


def test_engine_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from rmx import tables as T
    from rmx.engine import VecRMEnv
    with pytest.raises(RuntimeError):
        VecRMEnv(T.compile_scenario(T.baseline_scenario(2)), 8)


def test_entry_points_reject_null_handles_without_touching_gpu():
    """Every device entry point checks its handle and arguments before any HIP call."""
    if not os.path.exists(_capi.LIB_PATH):
        pytest.skip("librmx.so not built")
    lib = _capi.load_library()
    assert lib.rmx_step(None, None, 1, None) == _capi.RMX_E_INVALID
    assert lib.rmx_step_report(None, None, 1, None, None) == _capi.RMX_E_INVALID
    assert lib.rmx_step_report_fused(None) == 0
    assert lib.rmx_step_seq(None, None, 0, 1, 1, None, None) == _capi.RMX_E_INVALID
    assert lib.rmx_step_seq(None, None, 0, (1 << 20) + 1, 1, None, None) == _capi.RMX_E_INVALID
    assert b"window" in lib.rmx_last_error()
    assert lib.rmx_queue_counters(None, None) == _capi.RMX_E_INVALID
    assert lib.rmx_queue_info(None, None, 0) == _capi.RMX_E_INVALID
    assert lib.rmx_stats_device(None, None, None) == _capi.RMX_E_INVALID
    assert lib.rmx_step_hashed(None, 0, 0, 1, None) == _capi.RMX_E_INVALID


def test_step_code_object_symbols_follow_the_queue_mangling():
    """rmx_step_seq's queue finds each step_fast_kernel instantiation by a symbol it spells from the template
    arguments (go_step, rmx_fast.hip); every step kernel symbol in the embedded code object has that spelling."""
    import re
    import subprocess
    co = os.path.join(_capi.CSRC, "build", "rmx_fast.co")
    readelf = "/opt/rocm/lib/llvm/bin/llvm-readelf"
    if not (os.path.exists(co) and os.path.exists(readelf)):
        pytest.skip("build/rmx_fast.co not built")
    syms = set(re.findall(r"(_ZN3rmx16step_fast_kernel\S*\.kd)",
                          subprocess.run([readelf, "--symbols", co], capture_output=True, text=True, check=True).stdout))
    pat = re.compile(r"_ZN3rmx16step_fast_kernelILi(\d+)ELi(\d+)ELb([01])ELi(\d+)ELi(\d+)ELi(\d+)ELb([01])ELi(\d+)EEE"
                     r"viiPKiS2_S2_PKjS2_S2_NS_10FastParamsE\.kd")
    assert 100 < len(syms) <= 320  # round 5: 528 -> 256, then +48 fused-report forms of the slip / random-start steps
    assert all(pat.fullmatch(s) for s in syms)
    # only the table modes (global 1, merged 4, merged4 7) and store modes (none 0, rare 2, rare-nt 3) that won their
    # A/Bs remain (round 5 pruned the rest); kSkipNone only with QRM outputs
    for s in syms:
        kind, a, hashed, tbl, qxb, skip, rpt, slip = pat.fullmatch(s).groups()
        assert tbl in ("1", "4", "7") and skip in ("0", "2", "3"), s
        assert (skip == "0") == (qxb != "0"), s
    # the default step of BASELINE config 2 and its fused-report form
    assert "_ZN3rmx16step_fast_kernelILi0ELi2ELb0ELi7ELi0ELi2ELb0ELi0EEEviiPKiS2_S2_PKjS2_S2_NS_10FastParamsE.kd" in syms
    assert "_ZN3rmx16step_fast_kernelILi0ELi2ELb0ELi7ELi0ELi2ELb1ELi0EEEviiPKiS2_S2_PKjS2_S2_NS_10FastParamsE.kd" in syms
    # config 2 with random starts under the runner's seed schedule (kRngStarts | kRngFixedSeed), plain and reported
    for rpt in "01":
        assert f"_ZN3rmx16step_fast_kernelILi0ELi2ELb0ELi7ELi0ELi2ELb{rpt}ELi6EEEviiPKiS2_S2_PKjS2_S2_NS_10FastParamsE.kd" in syms


@pytest.mark.parametrize("torch_first", [False, True])
def test_one_hip_runtime_whatever_the_import_order(torch_first):
    """librmx.so loaded before or after torch: the process maps ONE HIP and ONE HSA runtime (torch's, when torch is
    installed).  Without rmx._capi's preload, loading librmx.so first mapped /opt/rocm's libamdhip64 and torch then
    its own, and the engine's runtime could not see the GPU torch held (a host handle, then a device handle)."""
    import sys
    import textwrap

    code = textwrap.dedent(f"""
        import json, sys
        sys.path.insert(0, {os.path.join(ROOT, "multiagent-rl-rm_amd")!r})
        if {torch_first}:
            import torch
        from rmx import _capi
        _capi.load_library()
        import torch
        m = sorted({{l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l or "libhsa-runtime64" in l}})
        print(json.dumps({{"maps": m, "expect": _capi.torch_hip_runtime()}}))
    """)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    hip = [p for p in out["maps"] if "libamdhip64" in p]
    hsa = [p for p in out["maps"] if "libhsa-runtime64" in p]
    assert len(hip) == 1 and len(hsa) == 1, out["maps"]
    if out["expect"]:
        assert sorted(os.path.realpath(p) for p in out["expect"]) == sorted(os.path.realpath(p) for p in hip + hsa)
