"""The committed GPU evidence against the oracle's full-size run (CPU only, no GPU needed).

tests/golden/full_size.json holds the oracle's totals over ALL 2^20 systems of BASELINE
configs[2] (uniform) and [3] (contention), made by tests/golden/make_full_size.py. The
bench lines committed under profiles/r01/ were measured on an MI355X over exactly those
workloads, and so is the round-2 headline line profiles/r02/bench_headline.json (its
uniform totals and its `contention` object); their per-type histograms, round totals and
error-system counts must equal the oracle's (bit-exact), and the round-2 line's digest
checksum too, so every committed headline number is a run with the reference's results. The live GPU check of the same fixture is
test_gpu_parity.py::test_full_size_sampled_parity (adds the digest checksum).
"""
import json
import pathlib

import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
GOLD = json.loads((ROOT / "tests" / "golden" / "full_size.json").read_text())
BENCH = {"uniform": "v19_bench_uniform_final.json", "contention": "v19_bench_contention.json"}


def test_fixture_shape():
    assert GOLD["systems"] == 1 << 20 and GOLD["num_procs"] == 8 and GOLD["instr_per_node"] == 4096
    for kind in BENCH:
        g = GOLD[kind]
        assert g["instructions"] == (1 << 20) * 8 * 4096  # every instruction issued
        assert len(g["hist"]) == 13 and len(g["digest_sum"]) == 2


@pytest.mark.parametrize("kind", list(BENCH))
def test_committed_gpu_bench_matches_oracle(kind):
    line = json.loads((ROOT / "profiles" / "r01" / BENCH[kind]).read_text())
    assert line["config"]["systems_per_gpu"] == GOLD["systems"] and line["n_gpus"] == 1
    assert line["config"]["trace"] == kind and line["config"]["cache_size"] == GOLD["cache_size"]
    tot, g = line["totals"], GOLD[kind]
    assert tot["hist"] == g["hist"]
    assert tot["instructions_per_step"] == g["instructions"]
    assert tot["rounds_total"] == g["rounds_total"]
    assert tot["err_systems"] == g["err_systems"]


@pytest.mark.parametrize("kind", list(BENCH))
def test_round2_headline_line_matches_oracle(kind):
    line = json.loads((ROOT / "profiles" / "r02" / "bench_headline.json").read_text())
    assert line["config"]["systems_per_gpu"] == GOLD["systems"] and line["n_gpus"] == 1
    assert line["config"]["trace"] == "uniform" and line["config"]["cache_size"] == GOLD["cache_size"]
    tot = line["totals"] if kind == "uniform" else line["contention"]["totals"]
    g = GOLD[kind]
    assert tot["hist"] == g["hist"]
    assert tot["instructions_per_step"] == g["instructions"]
    assert tot["rounds_total"] == g["rounds_total"]
    assert tot["err_systems"] == g["err_systems"]
    assert tot["digest_sum"] == g["digest_sum"]


SWEEP_GOLD = json.loads((ROOT / "tests" / "golden" / "sweep_full.json").read_text())


def _sweep_points(path):
    line = json.loads(path.read_text())
    sw = line["sweep"]
    return sw["points"] if isinstance(sw, dict) else sw


@pytest.mark.parametrize("path", ["profiles/r03/final/sweep.json", "profiles/r04/bench_headline.json",
                                  "profiles/r05/ev5_b/bench_detail.json",
                                  "profiles/r05/ev5_c/bench_detail.json",
                                  "profiles/r05/ev5_d/bench_detail.json",
                                  "profiles/r05/ev5_e/bench_detail.json"])
def test_committed_sweep_points_match_oracle_full_size(path):
    """configs[4] at full size: three grid points of the committed GPU lines --
    round 3's `bench.py --sweep`, round 4's default headline line and round 5's side file of the
    driver's command (the line itself carries the compact rows), whose `sweep` object the
    driver now times -- equal the oracle's run over all 2^20 systems (tests/golden/sweep_full.json,
    make_sweep_full.py): histograms, instructions, rounds, error systems, digest checksum."""
    f = ROOT / path
    if not f.exists():
        pytest.skip(f"{path} not committed yet")
    assert SWEEP_GOLD["systems"] == 1 << 20 and SWEEP_GOLD["instr_per_node"] == 4096
    pts = {(p["cache_size"], p["locality"]): p for p in _sweep_points(f)}
    assert len(pts) == 25
    for gp in SWEEP_GOLD["points"]:
        p = pts[(gp["cache_size"], gp["locality"])]
        for k in ("hist", "instructions", "rounds_total", "err_systems", "digest_sum"):
            assert p[k] == gp[k], (path, gp["cache_size"], gp["locality"], k)
