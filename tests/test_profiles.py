"""The committed profiler evidence describes the code object that is built (CPU only).

VERDICT r2 (next #2): bench.py reads roofline.traffic and the issue figures from committed
rocprofv3 summaries (profiles/pmc_<kind>.json) and the static opcode mix from
profiles/isa_table.json. Each records the fingerprint of sim_kernel<8,4,16,0> (named
sim_kernel<8,4,16,false> before round 3's MODE split; same bytes) in the library it was
measured on (tools/kernel_fingerprint.py: sha256 of the kernel's code and descriptor); they
must match the library built from this tree -- which ties this CPU test to the toolchain that
built the committed profiles -- and the headline's traffic must re-derive from the one file's
counters.
"""
import csv
import json
import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
import kernel_fingerprint as kf  # noqa: E402

PROFILES = ROOT / "profiles"
LIB = ROOT / "ue22cs343bb1-openmp-assignment_amd" / "libdash.so"


@pytest.fixture(scope="module")
def built_fp(dash):
    return kf.fingerprint(LIB)


@pytest.mark.parametrize("name", ["pmc_uniform.json", "pmc_contention.json", "isa_table.json"])
def test_profile_is_of_the_built_kernel(built_fp, name):
    prof = json.loads((PROFILES / name).read_text())
    assert prof.get("kernel_fingerprint") == built_fp, \
        f"{name} was measured on {prof.get('kernel_fingerprint')}, the built kernel is {built_fp}: refresh it"


SWEEP = sorted(p.name for p in PROFILES.glob("pmc_sweep_cs*_p*.json"))


@pytest.mark.parametrize("name", SWEEP)
def test_sweep_profile_is_of_the_built_kernel(dash, name):
    """The configs[4] point summaries (tools/evidence_sweep_pmc.sh) are bound to the first-tier kernel
    of their CACHE_SIZE, sim_kernel<8, CS, 16, 0>: bench.py fills a sweep row's traffic only when
    they match the library it runs."""
    import re
    cs = int(re.match(r"pmc_sweep_cs(\d+)_p", name).group(1))
    prof = json.loads((PROFILES / name).read_text())
    sym = f"_ZN4dash10sim_kernelILi8ELi{cs}ELj16ELi0EEEvNS_7SimArgsE"
    assert prof["kernel_fingerprint"] == kf.fingerprint(LIB, sym), f"{name}: refresh it"
    assert f"sim_kernel<8, {cs}, 16u, 0>" == prof["kernel"]
    read = prof["tcc_ea0_rdreq_128b_sum"] * 128 + prof["tcc_ea0_rdreq_64b_sum"] * 64 + prof["tcc_ea0_rdreq_32b_sum"] * 32
    assert read + prof["write_size"] * 1024 == pytest.approx(prof["hbm_bytes_per_launch"])
    assert 8 < prof["waves_per_cu"] <= 18.05 and prof["wave_rounds"] > 0


def test_sweep_covers_the_four_accounted_points():
    assert {"pmc_sweep_cs1_p0.json", "pmc_sweep_cs4_p0.json", "pmc_sweep_cs8_p0.json",
            "pmc_sweep_cs16_p0.json"} <= set(SWEEP)


@pytest.mark.parametrize("kind", ["uniform", "contention"])
def test_traffic_rederives_from_the_committed_counters(kind):
    p = json.loads((PROFILES / f"pmc_{kind}.json").read_text())
    # MI355X_MICROARCH.md HBM section: every L2->fabric read is counted by request size
    read = p["tcc_ea0_rdreq_128b_sum"] * 128 + p["tcc_ea0_rdreq_64b_sum"] * 64 + p["tcc_ea0_rdreq_32b_sum"] * 32
    assert read == pytest.approx(p["read_bytes_per_launch"])
    assert p["write_size"] * 1024 == pytest.approx(p["write_bytes_per_launch"])
    assert read + p["write_size"] * 1024 == pytest.approx(p["hbm_bytes_per_launch"])


def test_uniform_kernel_stats_agree_with_the_pmc_run():
    """profiles/r05/ev5_d/kernel_stats_uniform.csv: rocprofv3 --kernel-trace --stats of the bench
    command with the contention leg off (tools/evidence_r5.sh), so its sim_kernel<8,4,16,0> average
    is the headline kernel's, on the library the PMC summary measured."""
    rows = list(csv.DictReader((PROFILES / "r05" / "ev5_d" / "kernel_stats_uniform.csv").open()))
    row = next(r for r in rows if any(k in r["Name"] for k in ("sim_kernel<8, 4, 16u, false>", "sim_kernel<8, 4, 16u, 0>")))
    avg_ms = float(row["AverageNs"]) / 1e6
    pmc = json.loads((PROFILES / "pmc_uniform.json").read_text())
    assert avg_ms == pytest.approx(pmc["kernel_ms"], rel=0.03)
