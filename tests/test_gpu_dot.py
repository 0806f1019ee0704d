"""The solver's ordered dot (dev_common.hip k_reduce_ordered, the order of
linalg.c:17-25 dotprod: one running sum, i = 0 .. n-1) against that serial
sum on the host, bit for bit: the kernel adds only the non-zero products
(zero products leave the sum unchanged: it starts at +0 and never becomes
-0), so vectors with zeros, -0 entries, a product that is exactly zero from
two non-zero operands' underflow, and chunk boundaries (4,096) are
covered."""
import numpy as np
import pytest

import ipo_amd

pytestmark = pytest.mark.gpu


def serial(a, b):
    s = 0.0
    for x in (a * b).tolist():
        s += x
    return s


@pytest.mark.parametrize("n", [0, 1, 17, 4095, 4096, 4097, 12230, 100_003])
@pytest.mark.parametrize("density", [1.0, 0.5, 0.1, 0.0])
def test_ordered_dot_bitwise(n, density):
    rng = np.random.default_rng(n * 7 + int(density * 10))
    a = rng.standard_normal(n) * np.exp(rng.uniform(-20, 20, n))
    b = rng.standard_normal(n)
    a[rng.uniform(size=n) >= density] = 0.0
    if n > 3:
        a[1] = -0.0                     # a -0 product
        a[2], b[2] = 1e-200, 1e-200     # a product that underflows to +0
    got = ipo_amd.dot_ordered(a, b)
    want = serial(a, b)
    assert np.float64(got).tobytes() == np.float64(want).tobytes(), (got, want)
