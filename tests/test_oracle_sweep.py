"""configs[4] golden (tests/golden/sweep.json, written by tests/golden/make_sweep.py): three
grid points re-derived by the oracle here, so the committed totals the GPU sweep test checks
are the oracle's (CACHE_SIZE 1/4/16 hit cacheIndex = blockIndex % CACHE_SIZE, ref :188)."""
import json
import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tests" / "golden"))
GOLD = json.loads((ROOT / "tests" / "golden" / "sweep.json").read_text())


def test_sweep_golden_covers_the_grid():
    grid = {(p["cache_size"], p["locality"]) for p in GOLD["points"]}
    assert grid == {(cs, q) for cs in (1, 2, 4, 8, 16) for q in (0.0, 0.25, 0.5, 0.75, 1.0)}
    for p in GOLD["points"]:
        assert p["instructions"] == GOLD["systems"] * 8 * GOLD["instr_per_node"]
        assert sum(p["hist"][:2]) > 0


@pytest.mark.parametrize("cs,q", [(1, 0.0), (4, 0.5), (16, 1.0)])
def test_sweep_points_rederived(cs, q):
    import make_sweep
    got = make_sweep.point(cs, q, threads=8)
    want = next(p for p in GOLD["points"] if p["cache_size"] == cs and p["locality"] == q)
    assert got == want
