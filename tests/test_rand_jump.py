"""CPU: the glibc rand() jump-ahead identity the device RANSAC draws by (csrc/ransac.hip): with the
TYPE_3 state s_j = ring[(front + j) % 31] (the 31 newest words, oldest first), the k-th next word
is x_{i+k} = Σ_j C[k][j]·s_j (mod 2^32) for the fixed integer rows C[m−31] = e_m, C[k] = C[k−31] +
C[k−3]; a hypothesis draws rand() = x >> 1, and committing `used` draws rebuilds the ring as
ring'[(front + used + j) % 31] = x_{i+used−31+j}, front' = front + used, rear' = rear + used.
Checked against the oracle's restated glibc rand() (itself pinned to libc's, tests/test_oracle.py)."""
import numpy as np
import pytest

import oracle_ctypes as oc

M32 = 1 << 32


def _jump_table(k_max):
    T = [[0] * 31 for _ in range(k_max + 31)]
    for j in range(31):
        T[j][j] = 1
    for k in range(k_max):
        T[k + 31] = [(T[k][j] + T[k + 28][j]) % M32 for j in range(31)]
    return T[31:]


def _words(st):
    f = int(st[31])
    return [int(st[(f + j) % 31]) % M32 for j in range(31)]


@pytest.mark.parametrize("seed", [1, 7, 12345, 0xFFFFFFFF])
def test_draws_by_jump_table(seed):
    C = _jump_table(400)
    st = oc.rand_state(seed)
    s = _words(st)
    seq = oc.rand_sequence(seed, 400)
    got = [(sum(C[k][j] * s[j] for j in range(31)) % M32) >> 1 for k in range(400)]
    assert got == [int(v) for v in seq]


@pytest.mark.parametrize("used", [1, 3, 16, 30, 31, 32, 100, 272])
def test_commit_rebuilds_the_ring(used):
    C = _jump_table(300)
    st = oc.rand_state(99)
    s = _words(st)
    f, r = int(st[31]), int(st[32])
    ring = [int(v) % M32 for v in st[:31]]
    for j in range(31):
        idx = used - 31 + j
        ring[(f + used + j) % 31] = s[used + j] if idx < 0 else sum(C[idx][q] * s[q] for q in range(31)) % M32
    want = oc.rand_state(99)
    for _ in range(used):
        oc.lib().oracle_rand_next(oc._ptr(want))
    assert [int(v) % M32 for v in want[:31]] == ring
    assert (int(want[31]), int(want[32])) == ((f + used) % 31, (r + used) % 31)
