"""The CPU baseline's timing path (bench.py cpu_baseline) precomputes the reference-cell shape tables
as deal.II's FEValues does (gls_oracle_set_fast_tables); it must produce bit-identical element
matrices and vectors to the oracle's per-cell tabulation (oracle/gls_oracle.c tab_fill)."""
import ctypes as C

import numpy as np
import pytest

from oracle.oracle import Oracle, StructuredProblem, _dp, lib


@pytest.mark.parametrize("dim,k,kp", [(3, 2, 2), (3, 1, 1), (2, 2, 1)])
def test_fast_tables_bit_identical(dim, k, kp):
    p = StructuredProblem(dim, 3, k=k, kp=kp, viscosity=0.01, scheme="bdf2", time_steps=(0.01, 0.012, 0.01, 0.01))
    u = np.random.default_rng(20200200).uniform(-1, 1, p.n_dofs)
    P = p.struct()
    L = lib()
    L.gls_oracle_set_fast_tables.argtypes = [C.c_int]
    L.gls_oracle_time_local_systems.restype = C.c_double
    out = []
    for fast in (0, 1):
        L.gls_oracle_set_fast_tables(fast)
        out.append([L.gls_oracle_time_local_systems(C.byref(P), _dp(u), _dp(u), _dp(u), _dp(u), c, 1, 1, 1)
                    for c in range(p.n_cells)])
    # full element systems through the oracle's assembly (it tabulates through the same tab_fill)
    full = []
    for fast in (0, 1):
        L.gls_oracle_set_fast_tables(fast)
        A, b = Oracle(p).matrix_and_rhs(u, u, u, None)
        full.append((A.tocsr(), b))
    L.gls_oracle_set_fast_tables(0)
    assert out[0] == out[1]
    assert np.array_equal(full[0][1], full[1][1])
    assert (full[0][0] != full[1][0]).nnz == 0
