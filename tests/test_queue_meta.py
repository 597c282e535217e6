"""CPU checks of the engine queue's code-object metadata guard (csrc/rmx_queue.cpp).

rmx_step_seq writes each step_fast_kernel's kernel arguments itself: StepArgs, then the code object v5 hidden
arguments a 1-D HIP launch carries (block counts, group sizes, remainders, global offsets, grid dims, dynamic LDS).
A kernel whose metadata lists any other hidden argument (a debugging printf adds hidden_hostcall_buffer) would read
zeros there under the queue, so the queue refuses it and runs that window on the caller's stream.

- this file parses build/rmx_fast.co's NT_AMDGPU_METADATA note itself (ELF + MessagePack, independent of the C++
  parser) and checks every step kernel against the layout the queue writes;
- rmx_code_object_check (the C++ parser the queue uses) agrees on the embedded object, finds nothing to refuse there,
  and refuses the negative controls of tests/data/step_kernel_variants.hip (compiled here with hipcc).
"""
import ctypes as C
import os
import struct
import subprocess

import pytest

from rmx import _capi

CO = os.path.join(_capi.CSRC, "build", "rmx_fast.co")
HIPCC = "/opt/rocm/bin/hipcc"
# StepArgs: N, blk, six column pointers at 0..56, then FastParams by value (its size read from the metadata: every step
# kernel must agree on it); the hidden arguments start at the next 8-aligned offset
# what write_kernargs (rmx_queue.cpp) writes: offset from the hidden base, size
QUEUE_HIDDEN = {
    "hidden_block_count_x": (0, 4), "hidden_block_count_y": (4, 4), "hidden_block_count_z": (8, 4),
    "hidden_group_size_x": (12, 2), "hidden_group_size_y": (14, 2), "hidden_group_size_z": (16, 2),
    "hidden_remainder_x": (18, 2), "hidden_remainder_y": (20, 2), "hidden_remainder_z": (22, 2),
    "hidden_global_offset_x": (40, 8), "hidden_global_offset_y": (48, 8), "hidden_global_offset_z": (56, 8),
    "hidden_grid_dims": (64, 2), "hidden_dynamic_lds_size": (120, 4),
}
LEADING = [(0, 4), (4, 4)] + [(8 + 8 * i, 8) for i in range(6)]


def amdgpu_metadata(blob: bytes) -> dict:
    """The NT_AMDGPU_METADATA note of a 64-bit ELF code object, decoded."""
    import msgpack

    assert blob[:4] == b"\x7fELF" and blob[4] == 2
    shoff = struct.unpack_from("<Q", blob, 0x28)[0]
    shentsize, shnum = struct.unpack_from("<HH", blob, 0x3A)
    for i in range(shnum):
        sh = shoff + i * shentsize
        sh_type = struct.unpack_from("<I", blob, sh + 4)[0]
        off, size = struct.unpack_from("<QQ", blob, sh + 24)
        if sh_type != 7:  # SHT_NOTE
            continue
        o, end = off, off + size
        while end - o >= 12:
            namesz, descsz, ntype = struct.unpack_from("<III", blob, o)
            name_at = o + 12
            desc_at = name_at + ((namesz + 3) & ~3)
            if ntype == 32 and blob[name_at:name_at + namesz] == b"AMDGPU\0":
                return msgpack.unpackb(blob[desc_at:desc_at + descsz], raw=False)
            o = desc_at + ((descsz + 3) & ~3)
    raise AssertionError("no AMDGPU metadata note")


def step_kernels(meta: dict) -> dict:
    return {k[".symbol"]: k[".args"] for k in meta["amdhsa.kernels"] if "step_fast_kernel" in k[".symbol"]}


def why_refused(args, fp_bytes) -> str:
    """'' when the queue's kernel-argument image is exactly what this kernel reads (Python restatement of
    check_step_args; fp_bytes = sizeof(FastParams))."""
    explicit = [(a[".offset"], a[".size"]) for a in args if not a[".value_kind"].startswith("hidden_")]
    if explicit != LEADING + [(56, fp_bytes)]:
        return "explicit"
    hidden_base = (56 + fp_bytes + 7) & ~7
    for a in args:
        kind = a[".value_kind"]
        if not kind.startswith("hidden_") or kind == "hidden_none":
            continue
        if kind not in QUEUE_HIDDEN:
            return kind
        off, size = QUEUE_HIDDEN[kind]
        if (a[".offset"], a[".size"]) != (hidden_base + off, size):
            return kind + "@offset"
    return ""


def c_check(lib, blob):
    n, r = C.c_int64(), C.c_int64()
    rep = C.create_string_buffer(1024)
    rc = lib.rmx_code_object_check(blob, len(blob) if blob else 0, C.byref(n), C.byref(r), rep, 1024)
    return rc, n.value, r.value, rep.value.decode(errors="replace")


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_capi.LIB_PATH):
        pytest.skip("librmx.so not built")
    return _capi.load_library()


def test_embedded_step_kernels_take_only_the_queues_hidden_arguments():
    if not os.path.exists(CO):
        pytest.skip("build/rmx_fast.co not built")
    ks = step_kernels(amdgpu_metadata(open(CO, "rb").read()))
    assert len(ks) > 0
    fp = {a[8][".size"] for a in ks.values()}
    assert len(fp) == 1 and next(iter(fp)) % 8 == 0, fp  # one FastParams layout, 8-B multiple (no tail padding)
    fp_bytes = fp.pop()
    bad = {s: w for s, w in ((s, why_refused(a, fp_bytes)) for s, a in ks.items()) if w}
    assert not bad, bad
    # every kernel carries the group sizes / block counts the queue writes (the kernels read blockDim through them)
    for args in ks.values():
        kinds = {a[".value_kind"] for a in args}
        assert {"hidden_block_count_x", "hidden_group_size_x"} <= kinds


def test_c_check_agrees_on_the_embedded_object(lib):
    rc, n, r, rep = c_check(lib, None)
    assert rc == 0 and r == 0 and rep == "", rep
    if os.path.exists(CO):
        blob = open(CO, "rb").read()
        assert n == len(step_kernels(amdgpu_metadata(blob)))
        assert c_check(lib, blob)[:3] == (0, n, 0)  # the embedded object is build/rmx_fast.co


def test_c_check_rejects_a_non_elf_blob(lib):
    rc, n, r, rep = c_check(lib, b"\0" * 256)
    assert rc == _capi.RMX_E_INVALID and "ELF" in rep


def test_printf_and_foreign_layouts_are_refused(lib, tmp_path):
    """Negative controls: the same parameter list plus a printf (hidden_hostcall_buffer) is refused, a kernel of
    another explicit layout is refused, the plain one is accepted; the Python restatement agrees."""
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    src = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "step_kernel_variants.hip")
    out = tmp_path / "variants.co"
    subprocess.run([HIPCC, "-std=c++17", "-O1", "--offload-arch=gfx950", "--offload-device-only",
                    "--no-gpu-bundle-output", "-I", _capi.CSRC, src, "-o", str(out)], check=True,
                   capture_output=True, timeout=300)
    blob = out.read_bytes()
    ks = step_kernels(amdgpu_metadata(blob))
    assert len(ks) == 3
    plain = [s for s in ks if "ILi0EE" in s]
    fp_bytes = ks[plain[0]][8][".size"]
    why = {s: why_refused(a, fp_bytes) for s, a in ks.items()}
    assert len(plain) == 1 and why[plain[0]] == ""
    assert sorted(w for w in why.values() if w) == ["explicit", "hidden_hostcall_buffer"]
    rc, n, r, rep = c_check(lib, blob)
    assert (rc, n, r) == (0, 3, 2)
    assert "not written by the queue" in rep or "StepArgs" in rep


def test_c_check_survives_corrupted_objects(lib):
    """rmx_code_object_check reads caller-supplied bytes: every corruption of the metadata note (random byte flips,
    truncations, a length field blown up) must end in a verdict — the object refused or read — never a crash or a
    read past the buffer (the ELF and MessagePack readers bound every length against the buffer)."""
    import random

    if not os.path.exists(CO):
        pytest.skip("build/rmx_fast.co not built")
    blob = open(CO, "rb").read()
    # the metadata note's extent, to aim most mutations there
    shoff = struct.unpack_from("<Q", blob, 0x28)[0]
    shentsize, shnum = struct.unpack_from("<HH", blob, 0x3A)
    notes = []
    for i in range(shnum):
        sh = shoff + i * shentsize
        if struct.unpack_from("<I", blob, sh + 4)[0] == 7:
            off, size = struct.unpack_from("<QQ", blob, sh + 24)
            notes.append((off, size))
    assert notes
    off, size = max(notes, key=lambda t: t[1])
    rng = random.Random(1234)
    verdicts = set()
    for it in range(600):
        b = bytearray(blob)
        kind = it % 4
        if kind == 0:  # byte flips inside the note
            for _ in range(rng.randint(1, 8)):
                b[off + rng.randrange(size)] ^= 1 << rng.randrange(8)
        elif kind == 1:  # a MessagePack length prefix blown up
            p = off + rng.randrange(size)
            b[p] = rng.choice([0xDC, 0xDD, 0xDE, 0xDF, 0xDB, 0xC6, 0xC9])
            if p + 5 <= len(b):
                b[p + 1:p + 5] = b"\xff\xff\xff\xff"
        elif kind == 2:  # truncated anywhere
            b = b[:rng.randrange(64, len(b))]
        else:  # the ELF header / section table scribbled
            for _ in range(rng.randint(1, 4)):
                p = rng.choice([0x28, 0x3A, 0x3C, shoff + rng.randrange(shnum * shentsize)])
                if p < len(b):
                    b[p] = rng.randrange(256)
        rc, n, r, rep = c_check(lib, bytes(b))
        assert rc in (0, _capi.RMX_E_INVALID), rc
        verdicts.add(rc)
    assert _capi.RMX_E_INVALID in verdicts
