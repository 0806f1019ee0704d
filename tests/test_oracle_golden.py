"""Pin the CPU oracle: its stdout must equal the reference's captured traces
(evaluate/v1-cf4d5ba/netlib/ipo/<name>.mps.sol, copied to tests/golden/netlib)
byte for byte -- banner, dimension lines, every iteration line, status."""
import pytest

import oracle_lib
from conftest import available_problems, golden_trace, mps_path

SLOW = {"pilot", "greenbea", "d2q06c", "pilot87", "pds-06", "dfl001"}
FAST = [p for p in available_problems() if p not in SLOW]


@pytest.mark.parametrize("name", FAST)
def test_oracle_reproduces_golden_trace(name):
    out = oracle_lib.run_cli(mps_path(name), "hsd", timeout=600)
    assert out == golden_trace(name)


@pytest.mark.slow
@pytest.mark.parametrize("name", sorted(SLOW))
def test_oracle_reproduces_golden_trace_slow(name):
    out = oracle_lib.run_cli(mps_path(name), "hsd", timeout=3600)
    assert out == golden_trace(name)


def test_golden_inventory():
    # 97 replayable problems (12 logged ones have no MPS input in the reference)
    assert len(available_problems()) == 97
