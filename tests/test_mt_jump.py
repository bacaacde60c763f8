"""The jump-ahead of the parallel torch-parity stream (csrc/mt_poly.cpp),
on the CPU: the host-computed coefficients of x^(g*J - 1) mod P, applied to
the raw MT19937 stream of a seeded state, must give exactly the 624-word
window at draw position g*J of the serial stream (the window every parallel
generator of gc_mt19937_generate_jumped starts from).  The serial stream is a
numpy restatement of at::mt19937, itself checked against the oracle's MT."""
import ctypes as C

import numpy as np
import pytest

from gcodec import _lib
from gcodec import codec
from oracle import oracle as O

J = _lib.GC_MT_JUMP_DRAWS
N, M = 624, 397


def _mix(a, b):
    y = (a & np.uint32(0x80000000)) | (b & np.uint32(0x7FFFFFFF))
    return (y >> np.uint32(1)) ^ np.where(y & np.uint32(1), np.uint32(0x9908B0DF), np.uint32(0))


def raw_stream(state, total):
    """x_0 .. x_{total-1}: the state array, then the MT recurrence
    x_t = x_{t-227} ^ twist(x_{t-624}, x_{t-623}), one block in three phases."""
    blocks = -(-total // N)
    x = np.zeros(blocks * N, dtype=np.uint32)
    x[:N] = state[:N]
    for k in range(N, blocks * N, N):
        for lo, hi in ((0, N - M), (N - M, 2 * (N - M)), (2 * (N - M), N)):
            t = np.arange(k + lo, k + hi)
            x[t] = x[t - (N - M)] ^ _mix(x[t - N], x[t - N + 1])
    return x[:total]


def temper(y):
    y = y ^ (y >> np.uint32(11))
    y = y ^ ((y << np.uint32(7)) & np.uint32(0x9D2C5680))
    y = y ^ ((y << np.uint32(15)) & np.uint32(0xEFC60000))
    return y ^ (y >> np.uint32(18))


def jump_table(first, count, j=None):
    out = np.empty(count * 624, dtype=np.uint32)
    lib = _lib.load()
    if j is None:
        _lib.check(lib.gc_mt19937_jump_table(first, count, out.ctypes.data_as(C.c_void_p)), "jump_table")
    else:
        _lib.check(lib.gc_mt19937_jump_table_j(j, first, count, out.ctypes.data_as(C.c_void_p)), "jump_table")
    return out.reshape(count, 624)


def window_from_table(x, coef):
    bits = np.unpackbits(coef.view(np.uint8), bitorder="little")[:19937]
    acc = np.zeros(624, dtype=np.uint32)
    for k in np.flatnonzero(bits):
        acc ^= x[k + 1:k + 625]
    return acc


def test_numpy_stream_matches_oracle_mt():
    st = codec.mt19937_seed_state(42)
    x = raw_stream(st, 5 * N)
    assert np.array_equal(temper(x[N:]), O.MT19937(42).draws(4 * N))


@pytest.mark.parametrize("seed", [42, 7])
def test_jump_windows_match_serial_stream(seed):
    st = codec.mt19937_seed_state(seed)
    tab = jump_table(1, 2)
    x = raw_stream(st, 2 * J + 2 * N)
    for g in (1, 2):
        assert np.array_equal(window_from_table(x, tab[g - 1]), x[g * J:g * J + 624]), g


def test_jump_table_offsets_agree():
    """generator g's row does not depend on where the table starts"""
    a = jump_table(1, 3)
    assert np.array_equal(jump_table(2, 2), a[1:])
    assert np.array_equal(jump_table(3, 1), a[2:])
    assert np.any(a[0] != a[1])


@pytest.mark.parametrize("j", [624, 1872, 624 * 627])
def test_jump_windows_any_generator_length(j):
    """gc_mt19937_jump_table_j: generators of any multiple of 624 draws (the
    package picks J per count)"""
    st = codec.mt19937_seed_state(11)
    tab = jump_table(1, 3, j)
    x = raw_stream(st, 3 * j + 2 * N)
    for g in (1, 2, 3):
        assert np.array_equal(window_from_table(x, tab[g - 1]), x[g * j:g * j + 624]), g
    assert np.array_equal(jump_table(1, 2, J), jump_table(1, 2))


def test_jump_table_rejects_bad_lengths():
    out = np.empty(624, dtype=np.uint32)
    lib = _lib.load()
    for j in (0, 625, 1000):
        assert lib.gc_mt19937_jump_table_j(j, 1, 1, out.ctypes.data_as(C.c_void_p)) != 0


def test_generator_length_choice():
    """J: a multiple of 624, generators bounded, balanced near sqrt(count)"""
    for n in (1, 1000, 10 ** 6, 10 ** 7, 10 ** 8, 10 ** 9):
        j = codec.mt_generator_draws(n)
        assert j % 624 == 0 and j > 0
        assert -(-n // j) <= codec.MT_MAX_GENERATORS
    assert -(-10 ** 8 // codec.mt_generator_draws(10 ** 8)) == 383
