"""CPU checks of the interior-point engine's workspace carving (noc/ipm.py: carve_zeros): one
zero-filled allocation per dtype, every field 256 bytes aligned within it, no two fields overlapping."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ip-parallel-optimal-control_amd"))

from noc.ipm import carve_zeros  # noqa: E402


def _check(spec, dtype):
    views, buf = carve_zeros(spec, device="cpu", dtype=dtype)
    assert set(views) == set(spec)
    spans = []
    for k, s in spec.items():
        v = views[k]
        assert tuple(v.shape) == tuple(s) and v.dtype == dtype and v.is_contiguous()
        assert (v.data_ptr() - buf.data_ptr()) % 256 == 0  # the HIP allocator's base is 512-aligned
        assert bool((v == 0).all())
        lo = v.data_ptr()
        spans.append((lo, lo + v.numel() * v.element_size()))
        assert buf.data_ptr() <= lo and spans[-1][1] <= buf.data_ptr() + buf.numel() * buf.element_size()
    spans.sort()
    for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
        assert a1 <= b0  # disjoint
    return views


def test_carve_f64_fields_of_a_b1_engine():
    N, nx, nu = 200, 4, 1
    spec = dict(x=(1, N + 1, nx), u=(1, N, nu), x0=(1, nx), A=(3203,), pred=(1,), cost=(1,),
                P=(1, nx, nx), lam=(1, N + 1, nx))
    views = _check(spec, torch.float64)
    views["u"].fill_(1.0)  # writes stay inside the field
    assert bool((views["x"] == 0).all()) and bool((views["x0"] == 0).all())


def test_carve_int_fields_and_odd_sizes():
    _check({k: (n,) for k, n in zip("abcdef", (1, 7, 63, 64, 65, 4096))}, torch.int32)
