"""CPU checks of the arithmetic the fast kernels' random starts rest on (rmx_fast.hip rs_*):

- numpy's untyped Generator.shuffle is Fisher-Yates from the end with j_i = random_interval(i) over 32-bit draws,
  low half of each 64-bit PCG64 output first (restated here from numpy's bit stream and compared with numpy itself);
- undoing the swaps for the first A slots in reverse order (shuffle_slots / rs_undo_full) gives the shuffled list's
  first A entries;
- the first-occurrence rows and their chain walk (rs_take<true> / rs_undo_chain) give the same slots;
- the wave-cooperative jump (rs_coop_finish): state after j steps = M^j s + (1 + M + ... + M^(j-1)) c mod 2^128,
  checked against numpy's PCG64 state after j outputs.
No GPU: these pin the math; the GPU tests pin the kernels against the oracle and the reference goldens."""
import numpy as np
import pytest

M128 = (0x2360ED051FC65DA4 << 64) | 0x4385DF649FCCF645
MOD = 1 << 128


def draws_of(seed):
    """numpy's 32-bit draw stream of a fresh default_rng(seed): each 64-bit output split, low half first."""
    bg = np.random.PCG64(seed)
    while True:
        o = int(bg.random_raw())
        yield o & 0xFFFFFFFF
        yield o >> 32


def shuffle_js(seed, n):
    """j_i for i = n-1 .. 1 as numpy's Generator.shuffle of a Python list draws them (random_interval)."""
    d = draws_of(seed)
    js = {}
    for i in range(n - 1, 0, -1):
        mask = i
        for s in (1, 2, 4, 8, 16):
            mask |= mask >> s
        while True:
            v = next(d) & mask
            if v <= i:
                break
        js[i] = v
    return js


def undo_full(js, n, p):
    pos = p
    for i in range(1, n):
        if pos == i:
            pos = js[i]
        elif pos == js[i]:
            pos = i
    return pos


def undo_chain(js, n, p, A):
    F = [0] * (n + 8)
    ini = {}
    for i in range(n - 1, 0, -1):  # drawing order
        v = js[i]
        if (i >= A) if v < A else (v < i):
            F[v] = i
        if i < A:
            ini[i] = v
    pos = p
    for k in range(1, A):
        jk = ini[k]
        pos = jk if pos == k else (k if pos == jk else pos)
    while F[pos] != 0:
        pos = F[pos]
    return pos


@pytest.mark.parametrize("n", [2, 3, 5, 17, 64, 89, 100, 183])
def test_shuffle_restatement_matches_numpy(n):
    for seed in range(25):
        js = shuffle_js(seed, n)
        lst = list(range(n))
        for i in range(n - 1, 0, -1):
            lst[i], lst[js[i]] = lst[js[i]], lst[i]
        ref = list(range(n))
        np.random.default_rng(seed).shuffle(ref)
        assert lst == ref, (n, seed)


@pytest.mark.parametrize("n", [2, 4, 9, 89, 100, 183])
@pytest.mark.parametrize("A", [1, 2, 3, 4])
def test_undo_full_and_chain_give_the_first_slots(n, A):
    if A > n:
        pytest.skip("fewer cells than agents")
    for seed in range(40):
        ref = list(range(n))
        np.random.default_rng(seed).shuffle(ref)
        js = shuffle_js(seed, n)
        for p in range(A):
            assert undo_full(js, n, p) == ref[p], (n, A, seed, p)
            assert undo_chain(js, n, p, A) == ref[p], (n, A, seed, p)


def test_jump_ahead_matches_numpy_state():
    """rs_jump: M^j and the geometric sum, as the host builds them (rmx_capi.cpp RsJumpTable), for j = 1..64."""
    mj, sj, table = 1, 0, []
    for _ in range(64):
        sj = (sj + mj) % MOD
        mj = (mj * M128) % MOD
        table.append((mj, sj))
    for seed in (0, 1, 12345, 2**40 + 7):
        bg = np.random.PCG64(seed)
        st = bg.state["state"]
        s0, c = int(st["state"]), int(st["inc"])
        for j in range(1, 65):
            bg.random_raw()
            mj, sj = table[j - 1]
            assert int(bg.state["state"]["state"]) == (mj * s0 + sj * c) % MOD, (seed, j)
