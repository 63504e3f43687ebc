"""Property tests of the scan algebra the HIP KKT kernels are built on.

The chunked wave-scan (csrc/kkt_scan_impl.h, modelled lane by lane in tests/kernel_model.py)
is correct only if
  * the element combine is associative (phase 2 reorders it into a Sklansky tree),
  * the identity element is exact (idle / masked lanes combine with it, and an empty chunk of a
    horizon shorter than the lane count is the identity),
  * splitting a run of stages anywhere gives the same element (phase 1 chunks the horizon at
    lane-count-dependent boundaries),
  * the chunked solve equals the sequential Riccati solve for every horizon / lane count.
Hypothesis draws the shapes, horizons, split points and lane counts; the stages come from the
seeded generator the parity tests use (tests/lq_cases.py).  CPU only; the oracle is the checker.
"""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings, strategies as st

import kernel_model as KM
from lq_cases import rand_lq

SETTINGS = settings(max_examples=60, deadline=None, derandomize=True, database=None,
                    suppress_health_check=[HealthCheck.too_slow])


@st.composite
def shapes(draw, max_nx=4):
    # any nu <= nx <= 4, and the c4 shapes nx = 8 with nu = 1 / 4
    if draw(st.integers(0, 4)) == 0:
        return draw(st.sampled_from([(8, 1), (8, 4)]))
    nx = draw(st.integers(1, max_nx))
    nu = draw(st.integers(1, nx))
    return nx, nu


def _identity(nx):
    return (np.eye(nx), np.zeros(nx), np.zeros((nx, nx)), np.zeros(nx), np.zeros((nx, nx)))


def _run(case, lo, hi):
    """Element of stages lo..hi-1 by Riccati-form prepends onto the identity (phase 1)."""
    nx = case["A"].shape[-1]
    acc = _identity(nx)
    reg = case["reg"][0]
    for s in range(hi - 1, lo - 1, -1):
        g = lambda k: case[k][0, s]
        acc = KM.prepend(acc, g("A"), g("B"), g("Q"), g("R") + reg * np.eye(g("R").shape[0]),
                         g("M"), g("r"), g("q"), g("c"))
    return _sym(acc)


def _sym(e):
    A, b, C, nu, J = e
    return (A, b, 0.5 * (C + C.T), nu, 0.5 * (J + J.T))


def _close(e1, e2, rtol=1e-9):
    for a, b in zip(e1, e2):
        scale = max(1.0, float(np.max(np.abs(a))))
        assert np.max(np.abs(a - b)) <= rtol * scale, (a, b)


@SETTINGS
@given(shp=shapes(), seed=st.integers(0, 2**31 - 1), n=st.tuples(*[st.integers(1, 4)] * 3))
def test_combine_is_associative(shp, seed, n):
    nx, nu = shp
    case = rand_lq(seed, 1, sum(n), nx, nu, affine=True)
    e1, e2, e3 = _run(case, 0, n[0]), _run(case, n[0], n[0] + n[1]), _run(case, n[0] + n[1], sum(n))
    _close(KM.combine(KM.combine(e1, e2), e3), KM.combine(e1, KM.combine(e2, e3)))


@SETTINGS
@given(shp=shapes(), seed=st.integers(0, 2**31 - 1), n=st.integers(1, 6))
def test_identity_element_is_exact(shp, seed, n):
    """Combining with the identity on either side returns the element bit for bit."""
    nx, nu = shp
    e = _run(rand_lq(seed, 1, n, nx, nu, affine=True), 0, n)
    I = _identity(nx)
    for got in (KM.combine(e, I), KM.combine(I, e)):
        for a, b in zip(got, e):
            assert np.array_equal(a, b)


@SETTINGS
@given(shp=shapes(), seed=st.integers(0, 2**31 - 1), N=st.integers(2, 24), data=st.data())
def test_split_anywhere_gives_the_same_element(shp, seed, N, data):
    nx, nu = shp
    case = rand_lq(seed, 1, N, nx, nu, affine=True)
    m = data.draw(st.integers(1, N - 1))
    _close(KM.combine(_run(case, 0, m), _run(case, m, N)), _run(case, 0, N), rtol=1e-8)


def _suffixes_sequential(elems):
    out = list(elems)
    for l in range(len(elems) - 2, -1, -1):
        out[l] = KM.combine(elems[l], out[l + 1])
    return out


def _suffixes_hillis_steele(elems):
    cur, L, d = list(elems), len(elems), 1
    while d < L:
        cur = [KM.combine(cur[l], cur[l + d]) if l + d < L else cur[l] for l in range(L)]
        d *= 2
    return cur


def _suffixes_sklansky(elems):
    """The device's phase-2 tree: at distance d the lanes of each lower half-block take the
    whole upper half-block's suffix, held by its first lane (kkt_scan_impl.h rev_scan_sklansky)."""
    cur, L, d = list(elems), len(elems), 1
    while d < L:
        nxt = list(cur)
        for l in range(L):
            p = (l & ~(2 * d - 1)) + d
            if not (l & d) and p < L:
                nxt[l] = KM.combine(cur[l], cur[p])
        cur, d = nxt, d * 2
    return cur


@SETTINGS
@given(shp=shapes(), seed=st.integers(0, 2**31 - 1), L=st.sampled_from([2, 4, 8, 16, 32]))
def test_scan_trees_agree(shp, seed, L):
    nx, nu = shp
    case = rand_lq(seed, 1, L, nx, nu, affine=True)
    elems = [_run(case, l, l + 1) for l in range(L)]
    seq = _suffixes_sequential(elems)
    for tree in (_suffixes_hillis_steele(elems), _suffixes_sklansky(elems)):
        for a, b in zip(tree, seq):
            _close(a, b, rtol=1e-8)


@SETTINGS
@given(shp=shapes(), seed=st.integers(0, 2**31 - 1), N=st.integers(1, 48),
       L=st.sampled_from([1, 2, 4, 8, 16, 32, 64]))
def test_chunked_solve_equals_sequential_riccati(shp, seed, N, L):
    """Any horizon against any lane count, including N < L (empty chunks) and ragged chunks."""
    from oracle import noc_oracle as O
    nx, nu = shp
    c = {k: v[0] for k, v in rand_lq(seed, 1, N, nx, nu, affine=True).items()}
    args = (c["A"], c["B"], c["Q"], c["R"], c["M"], c["r"], c["P"], c["reg"])
    dx, du, pred, _, K, d, S, v = KM.model_kkt(*args, x0=c["x0"], q=c["q"], c=c["c"], p=c["p"], L=L)
    ref = O.kkt_solve(*args, c["x0"], c["q"], c["c"], c["p"], symmetrize=True)
    for got, want in ((dx, ref[0]), (du, ref[1]), (K, ref[4]), (d, ref[5]), (S, ref[6]), (v, ref[7])):
        want = np.asarray(want)
        assert np.max(np.abs(got - want)) <= 1e-8 * max(1.0, float(np.max(np.abs(want))))
    assert pred == pytest.approx(float(ref[2]), rel=1e-8, abs=1e-8)
