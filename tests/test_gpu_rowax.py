"""Column-sliced row products A x (RowAxPlan, row_ax.h / dev_common.hip).

When x exceeds one L2 slice (kAxSliceBytes) the HSD residuals take A x from
passes over column slices of x, each slice's entries stored by jagged
diagonals; every row still adds its entries in ascending column order, the
order of sparse_dot in the residual kernel, so a solve with the sliced
products is bitwise the solve without them.  IPO_HIP_AX_BLOCKS forces the
slice count on problems whose x fits one slice."""
import numpy as np
import pytest

import ipo_amd
from conftest import mps_path

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,blocks", [("afiro", 2), ("25fv47", 3), ("dfl001", 5), ("ken-07", 7)])
def test_sliced_row_products_bitwise(monkeypatch, name, blocks):
    monkeypatch.setenv("IPO_HIP_AX_BLOCKS", "1")
    _, t1, s1 = ipo_amd.run_mps(mps_path(name), "hsd")
    monkeypatch.setenv("IPO_HIP_AX_BLOCKS", str(blocks))
    _, t2, s2 = ipo_amd.run_mps(mps_path(name), "hsd")
    assert t1 == t2
    assert s1["iters"] == s2["iters"] and s1["final_mu"] == s2["final_mu"]


def test_sliced_row_products_synthetic(monkeypatch):
    """A banded LP (rows of up to 40 entries, empty slices for most rows)."""
    p = ipo_amd.synth_random(20000, 100000, 4, 64)
    out = []
    for blocks in ("1", "6"):
        monkeypatch.setenv("IPO_HIP_AX_BLOCKS", blocks)
        r = ipo_amd.solver(p, "hsd")
        out.append(r)
    assert out[0]["status"] == out[1]["status"] == 0
    assert out[0]["stats"]["iters"] == out[1]["stats"]["iters"]
    for k in ("x", "y", "w", "z"):
        assert np.array_equal(out[0][k], out[1][k]), k
