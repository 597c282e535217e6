"""Driver of tests/test_sanitizers.py (runs in a child process under LD_PRELOAD=libasan; not collected).

Runs the AddressSanitizer + UBSan builds (oracle/Makefile `asan`) of the CPU oracle, of the engine's host path
(csrc/rmx_hoststep.cpp: the RMX_DEVICE_HOST handles' stepper, on every config below) and of the engine's
host-side table builders (csrc/rmx_tables.cpp: validation, generic blob, fast blob, merged / compact tables, free
cells) over every BASELINE config, every golden scenario, the randomised worlds of
test_random_maps_gpu.py and a set of corrupted configs that validation must reject; and of the engine queue's code-object metadata reader
(csrc/rmx_comd.cpp) over build/rmx_fast.co and 1,500 corruptions of it.  Any sanitizer report aborts the process.
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "multiagent-rl-rm_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import oracle as O  # noqa: E402  (RMX_ORACLE_LIB points it at the sanitizer build)
from rmx import _capi, tables as T  # noqa: E402
from test_random_maps_gpu import CASES, random_tables  # noqa: E402

assert O.LIB_PATH.endswith(os.path.join("_asan", "liboracle.so")), O.LIB_PATH
HOST = C.CDLL(os.path.join(ROOT, "oracle", "_asan", "librmxhost.so"))
HOST.rmxh_build.restype = C.c_int
HOST.rmxh_build.argtypes = [C.c_void_p, C.POINTER(C.c_longlong)]
HOST.rmxh_host_run.restype = C.c_int
HOST.rmxh_host_run.argtypes = [C.c_void_p, C.c_longlong, C.c_ulonglong, C.POINTER(C.c_double)]
HOST.rmxh_co_check.restype = C.c_int
HOST.rmxh_co_check.argtypes = [C.c_void_p, C.c_size_t, C.c_ulonglong, C.c_ulonglong, C.c_ulonglong,
                               C.POINTER(C.c_longlong), C.POINTER(C.c_longlong)]


def build(tab, n=64, expect_ok=True, mutate=None):
    cfg, keep = _capi.make_config(tab, n)
    if mutate:
        mutate(cfg, keep)
    out = (C.c_longlong * 8)()
    rc = HOST.rmxh_build(C.byref(cfg), out)
    assert (rc == 0) == expect_ok, (rc, list(out))
    return list(out)


HOST_N, HOST_STEPS, HOST_SEED = 37, 250, 12345


def drive_host(tab):
    """The engine's host path (rmx_hoststep.cpp) under the sanitizers: one rmxh_host_run (every HostEngine entry point
    on exactly-sized columns); returns its statistics, state digest and invalid-action flag for the parent test to
    compare with librmx.so's host handle (tests/test_sanitizers.py host_run_reference)."""
    cfg, keep = _capi.make_config(tab, HOST_N, device=_capi.DEVICE_HOST)
    out = (C.c_double * 6)()
    rc = HOST.rmxh_host_run(C.byref(cfg), HOST_STEPS, HOST_SEED, out)
    assert rc == 0, rc
    return list(out)


def drive_oracle(tab, n=64, steps=300):
    env = O.OracleEnv(tab, n)
    env.reset(seed=11)
    rng = np.random.default_rng(n)
    for s in range(steps):
        acts = rng.integers(0, 5 if not tab.stochastic else 4, size=(tab.n_agents, n)).astype(np.int32)
        env.step(acts)
    env2 = O.OracleEnv(tab, n)
    env2.rollout(3, 0, steps, n_threads=2)
    for a in range(tab.n_agents):
        O.mdp(tab, a)
        O.mdp(tab, a, fix_fl=True)


def control():
    """Negative control: a cell tile two cells short of W*H (a caller bug the C ABI cannot see).  The
    validation pass reads past it, and the sanitizer must abort the process with a report."""
    tab = T.compile_scenario(T.baseline_scenario(2))

    def short_tile(cfg, keep):
        keep["short"] = np.ascontiguousarray(keep["cell"][:-2]).copy()
        cfg.cell = keep["short"].ctypes.data

    build(tab, mutate=short_tile)
    print("CONTROL_NOT_CAUGHT")


def co_check(blob, layout):
    """One metadata read of `blob` in its own heap allocation (exactly len(blob) bytes: a read past it lands in the
    sanitizer's redzone)."""
    # (libc malloc, not a numpy array: numpy serves small arrays from its own cache of larger blocks, which has no
    # redzone at the array's end)
    libc = C.CDLL(None)
    libc.malloc.restype, libc.malloc.argtypes = C.c_void_p, [C.c_size_t]
    libc.free.argtypes = [C.c_void_p]
    buf = libc.malloc(max(len(blob), 1))
    C.memmove(buf, blob, len(blob))
    n, r = C.c_longlong(), C.c_longlong()
    try:
        rc = HOST.rmxh_co_check(buf if len(blob) else None, len(blob), *layout, C.byref(n), C.byref(r))
    finally:
        libc.free(buf)
    return rc, n.value, r.value


def drive_co_reader(iters=1500):
    """The queue's metadata reader (rmx_comd.cpp) over build/rmx_fast.co and corruptions of it: byte flips in the
    metadata note, MessagePack length prefixes blown up, truncations, a scribbled ELF section table."""
    import random
    import struct

    # a note section that is the object's last bytes, its descriptor odd-sized and unpadded: the walk must stop at the
    # section end instead of stepping to the padded offset past the buffer
    ehdr = bytearray(64)
    ehdr[0:4], ehdr[4], ehdr[5], ehdr[6] = b"\x7fELF", 2, 1, 1
    struct.pack_into("<QIHHHHHH", ehdr, 0x28, 64, 0, 64, 0, 0, 64, 1, 0)  # e_shoff, e_flags, e_ehsize .. e_shnum, e_shstrndx
    note = struct.pack("<III", 3, 5, 1) + b"AB\0\0" + b"\x01\x02\x03\x04\x05"
    shdr = bytearray(64)
    struct.pack_into("<IIQQQQ", shdr, 0, 0, 7, 0, 0, 128, len(note))  # sh_name, SHT_NOTE, flags, addr, offset, size
    tail = bytes(ehdr + shdr) + note
    assert co_check(tail, (56, 1000, 1056))[0] == -1  # read whole, no metadata: refused
    for cut in range(1, len(note)):  # and every truncation of it
        co_check(tail[:len(tail) - cut], (56, 1000, 1056))
    co = os.path.join(_capi.CSRC, "build", "rmx_fast.co")
    if not os.path.exists(co):
        print("co reader: build/rmx_fast.co not built, skipped", flush=True)
        return
    blob = open(co, "rb").read()
    # the layout the metadata declares (StepArgs: 56 B of leading arguments, then FastParams)
    import test_queue_meta as QM
    ks = QM.step_kernels(QM.amdgpu_metadata(blob))
    fp = next(iter(ks.values()))[8][".size"]
    layout = (56, fp, (56 + fp + 7) & ~7)
    rc, n, r = co_check(blob, layout)
    assert rc == 0 and n == len(ks) and r == 0, (rc, n, r)
    shoff = struct.unpack_from("<Q", blob, 0x28)[0]
    shentsize, shnum = struct.unpack_from("<HH", blob, 0x3A)
    notes = [struct.unpack_from("<QQ", blob, shoff + i * shentsize + 24) for i in range(shnum)
             if struct.unpack_from("<I", blob, shoff + i * shentsize + 4)[0] == 7]
    off, size = max(notes, key=lambda t: t[1])
    rng = random.Random(99)
    seen = set()
    for it in range(iters):
        b = bytearray(blob)
        kind = it % 4
        if kind == 0:
            for _ in range(rng.randint(1, 8)):
                b[off + rng.randrange(size)] ^= 1 << rng.randrange(8)
        elif kind == 1:
            p = off + rng.randrange(size)
            b[p] = rng.choice([0xDC, 0xDD, 0xDE, 0xDF, 0xDB, 0xC6, 0xC9])
            b[p + 1:p + 5] = b"\xff\xff\xff\xff"
        elif kind == 2:
            b = b[:rng.randrange(0, len(b))]
        else:
            for _ in range(rng.randint(1, 4)):
                p = rng.choice([0x28, 0x3A, 0x3C, shoff + rng.randrange(shnum * shentsize)])
                if p < len(b):
                    b[p] = rng.randrange(256)
        seen.add(co_check(bytes(b), layout)[0])
    assert seen == {0, -1}, seen
    print("co reader", iters, "corruptions", flush=True)


def main():
    if "--control" in sys.argv:
        return control()
    drive_co_reader()
    print("HOSTRUN_PARAMS", HOST_N, HOST_STEPS, HOST_SEED, flush=True)
    tabs = {f"baseline{c}": T.compile_scenario(T.baseline_scenario(c)) for c in (2, 3, 4, 5)}
    with open(os.path.join(ROOT, "tests", "golden", "configs.json")) as f:
        for name, desc in json.load(f).items():
            tabs[name] = T.compile_scenario(desc)
    for name, args in CASES.items():
        tabs[name] = random_tables(*args)
    for name, tab in tabs.items():
        sizes = build(tab)
        assert sizes[0] > 0 and sizes[1] == tab.max_t + 2, (name, sizes)
        drive_oracle(tab, steps=120 if tab.width * tab.height > 500 else 300)
        print(name, sizes, flush=True)
        print("HOSTRUN", name, json.dumps(drive_host(tab)), flush=True)
    # corrupted configs: validation rejects them before any table index is formed
    tab = tabs["baseline5"]
    bad = {
        "n_agents": lambda c, k: setattr(c, "n_agents", 9),
        "grid": lambda c, k: setattr(c, "width", 5000),
        "events": lambda c, k: k["cell_event"].__setitem__((0, 3), 200),
        "next_q": lambda c, k: k["next_q"].__setitem__((1, 2, 3), 77),
        "start": lambda c, k: k["start_xy"].__setitem__((2, 1), -3),
        "final": lambda c, k: k["final_q"].__setitem__(0, 40),
        "tile_off_grid": lambda c, k: k["cell"].__setitem__(0, k["cell"][0] | 0xF),
        "qrm": lambda c, k: k["qrm_states"].__setitem__((0, 0), 99),
        "random_starts_ow": lambda c, k: setattr(c, "random_starts", 1),
    }
    for name, mut in bad.items():
        build(tab, expect_ok=False, mutate=mut)
        print("rejected", name, flush=True)
    print("ASAN_DRIVER_OK")


if __name__ == "__main__":
    main()
