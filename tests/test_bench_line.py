"""The bench line the driver reads (CPU only, no GPU).

VERDICT r4: the round-4 default line was 52 KB and the driver, which keeps a ~10 KB tail of
stdout + stderr, could not parse it. bench.py now writes the full record to a side file and
prints `compact_headline()` of it. These tests build that line from a synthetic worst case --
25 sweep points with every optional field present, 8 GPUs, maximal string lengths, digits that
do not round away -- and check it stays within LINE_BUDGET (4 KB) and keeps the fields the
driver and the judge check."""
import json
import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def _cpu(kind="reference", instances=16):
    return {"value": 512345.678901, "unit": "instr/s", "cores": 16, "host_cpus_visible": 256, "kind": kind,
            "mode": "A", "batches": {"n": 12, "min": 441234.5678, "median": 525678.1234, "max": 639876.54321},
            "instances": instances, "threads_per_instance": 8, "hung_instances_killed": 3,
            "stalled": {"n": 3, "explained": 3, "causes": {"ctz0_send": 3}, "systems": {"5": [3, 12]},
                        "oracle_ctz0": 3, "basis": "q" * 200},
            "cpu_model": "AMD EPYC 9575F 64-Core Processor with a very long model name string",
            "sample": "x" * 600}


def _roof(traffic=True):
    return {"bound": "hbm", "achieved": 111.72345678901, "peak": 8000.0, "unit": "GB/s",
            "frac": 0.013965432198765, "traffic": 356987495008.123 if traffic else None,
            "traffic_source": "y" * 300, "traffic_note": "z" * 300}


def synthetic_detail(world=8, with_all=True):
    M = 1 << 20
    pts = []
    for cs, p in bench.SWEEP_GRID:
        pts.append({"cache_size": cs, "locality": p, "value": 123456789012.345 * world,
                    "ms_per_step": 745.123456789, "steps": 1, "warmup": 1, "kernel_ms_avg": 744.98765,
                    "kernel_ms_steps": [744.987], "roofline": _roof(), "valu_issue": None,
                    "rounds_per_system": 23456.789, "wave_rounds": 3108572216, "hist": [15438985135] * 13,
                    "instructions": 34359738368 * world, "rounds_total": 24731883018 * world,
                    "err_systems": 224302 * world, "dropped": 210077 * world,
                    "digest_sum": [2251634405826991 * world, 2249834063518710 * world],
                    "ub_frac": 0.2139053344726562, "tier_systems": [M, 12345, 67], "ub_systems": 224302 * world,
                    "err_frac": 0.2139053344726562, "golden_slice": True,
                    "samples": {"checked": 32 * world, "mismatched": 0, "ranks": world, "world": world,
                                "slices_golden": 1, "slices_equal": 1},
                    "cpu_baseline": _cpu(), "vs_baseline": 68371.23456789, "cpu_baseline_note": None})
    per_cs = {cs: {"points": 5, "batches": 15, "hung": 11, "hung_explained": 11, "oracle_ctz0": 11}
              for cs in (1, 2, 4, 8, 16)}
    smp = {"checked": 48 * world, "mismatched": 0, "ranks": world, "world": world, "slices_golden": world,
           "slices_equal": world}
    tot = {"hist": [15438985135] * 13, "instructions_per_step": 34359738368 * world,
           "rounds_total": 23801163240 * world, "err_systems": 51391 * world, "dropped": 60000 * world,
           "digest_sum": [2251634405826991 * world, 2249834063518710 * world], "ub_systems": 51391 * world}
    probe = {"probe_ms": 163.759, "probe_valu_per_s": 839274538336.1628, "sclk_mhz": 1976.6,
             "sclk_min_mhz": 1853.2, "sclk_max_mhz": 2100.9, "sysfs": {"pci": "0000:dc:00.0", "power_w": 937.0}}
    return {
        "metric": "simulated instr/sec (whole node), 8-core DASH systems; % HBM roofline",
        "value": 5.58123456789e10 * world, "unit": "instr/s", "n_gpus": world, "steps": 20, "warmup": 5,
        "ms_per_step": 615.654321987, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": 109876.54321, "vs_baseline_basis": "b" * 200, "vs_baseline_mode_b": 117654.321,
        "dtype": "u8", "data": "synthetic (on-device counter-based generator, seed keyed by global system id)",
        "config": {"workload": f"{M} systems/GPU x 8 nodes x 4096 uniform RD/WR per node, CACHE_SIZE=4",
                   "systems_per_gpu": M, "num_procs": 8, "instr_per_node": 4096, "cache_size": 4,
                   "trace": "uniform", "parallelism": f"systems sharded over {world} GPU(s)"},
        "roofline": _roof(), "valu_issue": {"frac": 0.5012345, "issue_slots": {"busy_frac": 0.855069},
                                            "lds_bank_conflict_frac": 0.266098, "waves_per_cu": 17.61846},
        "valu_issue_note": None,
        "kernel_fingerprint": "da9f04138f4f822f",
        "cpu_baseline": _cpu(), "cpu_baseline_mode_b": _cpu(instances=1),
        "cpu_baseline_note": "n" * 400 if with_all else None, "cpu_port": _cpu("port"),
        "kernel_ms_avg": 615.06543210, "kernel_ms_rank": [614.98765432, 617.12345678],
        "kernel_ms_steps": [615.123] * 20, "rccl_world": world, "backend": "nccl",
        "tier_systems": [M, 3, 0], "wave_rounds": 3018808080, "totals": tot, "ub_frac": 0.0490102767944336,
        "parity_note": "p" * 300,
        "contention": {"value": 6.78123456789e10 * world, "ms_per_step": 503.123456789, "roofline": _roof(),
                       "totals": tot, "samples": smp, "kernel_ms_avg": 503.0, "golden_slice": True},
        "sweep": {"steps": 1, "warmup": 1, "cpu_per_cache_size": per_cs, "notes": bench.SWEEP_NOTES,
                  "golden": bench.sweep_golden_summary(pts, M), "points": pts},
        "next": {"events": {"slowdown": 1.10987654, "parity_same_digests_as_fast": True,
                            "parity_events_logged": True},
                 "seeded": {"slowdown": 1.48123456, "parity_all_issued": True, "parity_reproducible": True}},
        "box": {"probe_before": probe, "probe_after": probe, "device": {"name": "AMD Instinct MI355X"}},
    } | {"samples": smp, "golden": bench.golden_record(True, {"samples": smp, "golden_slice": True}, pts,
                                       tot["hist"] + [0] * 6 + [51391 * world, 48 * world, 0, world, world, world],
                                       world, M)}


@pytest.mark.parametrize("world", [1, 8])
def test_worst_case_line_fits_the_budget(world, tmp_path, capsys):
    d = synthetic_detail(world)
    long_dir = tmp_path / ("d" * 80)
    bench.emit(d, str(long_dir / "bench_detail.json"))
    out = capsys.readouterr().out
    assert out.count("\n") == 1
    assert len(out.encode()) <= bench.LINE_BUDGET, len(out)
    line = json.loads(out)
    # nothing was dropped to make it fit
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "contention", "sweep", "next",
              "box", "rccl_world", "backend", "kernel_ms_rank", "ub_frac", "issue", "detail"):
        assert k in line, k
    assert set(line["roofline"]) == {"bound", "achieved", "peak", "unit", "frac", "traffic"}
    assert {"value", "unit", "cores", "kind", "sample"} <= set(line["cpu_baseline"])
    assert len(line["sweep"]["rows"]) == 25 and len(line["sweep"]["rows"][0]) == len(line["sweep"]["cols"])
    # the line certifies its own results at any N -- rank 0's slice against the
    # full-size goldens, every rank's sampled ids -- and each sweep row says which point it checked
    g = line["golden"]
    assert g["slice"] == [0, 1 << 20] and g["headline"] is True and g["contention"] is True
    assert g["sweep"][:3] == [25, 25, 25] and g["samples"][1] == 0 and g["samples"][2] == g["samples"][3] == world
    assert g["ranks"] == [[world, world], [world, world]]  # every rank's whole slice, both workloads
    cols = line["sweep"]["cols"]
    assert all(dict(zip(cols, r))["golden"] is True and dict(zip(cols, r))["smp_bad"] == 0
               for r in line["sweep"]["rows"])
    assert all(v[1] >= 15 and v[3] == v[2] for v in line["sweep"]["cpu"].values())
    assert line["cpu_baseline"]["hung_explained"] == line["cpu_baseline"]["hung"]
    assert "8.5x" in line["sweep"]["notes"]["8"]
    # the side file holds the full record
    assert json.loads((long_dir / "bench_detail.json").read_text()) == json.loads(json.dumps(d))


def test_line_values_round_trip():
    d = synthetic_detail(1)
    line = bench.compact_headline(d, "gpurun_out/bench_detail.json")
    assert line["value"] == pytest.approx(d["value"], rel=1e-4)
    assert line["ms_per_step"] == pytest.approx(d["ms_per_step"], rel=1e-4)
    assert line["roofline"]["frac"] == pytest.approx(d["roofline"]["frac"], rel=1e-3)
    assert line["cpu_baseline"]["value"] == pytest.approx(d["cpu_baseline"]["value"], rel=1e-3)
    row = line["sweep"]["rows"][0]
    assert row[:2] == [1, 0.0] and row[6] == pytest.approx(d["sweep"]["points"][0]["ub_frac"], rel=1e-2)
    assert line["ub_frac"] == pytest.approx(d["totals"]["ub_systems"] / (1 << 20), rel=1e-2)


def test_sig_keeps_types():
    assert bench.sig(None) is None and bench.sig(7) == 7 and bench.sig(True) is True
    assert bench.sig(0.0) == 0.0 and bench.sig(123456.789) == 123500.0 and bench.sig(1.23456e-5, 3) == 1.23e-5


def test_oversized_line_drops_summaries_not_the_headline(capsys, tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "LINE_BUDGET", 2500)
    bench.emit(synthetic_detail(8), str(tmp_path / "d.json"))
    line = json.loads(capsys.readouterr().out)
    assert {"value", "roofline", "cpu_baseline", "sweep"} <= set(line)
    # a budget the sweep rows cannot fit: they stay in the side file, the line says so and still fits
    monkeypatch.setattr(bench, "LINE_BUDGET", 1800)
    bench.emit(synthetic_detail(8), str(tmp_path / "d.json"))
    out = capsys.readouterr().out
    line = json.loads(out)
    assert len(out.strip()) <= 1800 and line["sweep"]["rows"] == 25 and "sweep" in line["dropped_for_size"]
    assert {"value", "ms_per_step", "roofline", "cpu_baseline", "detail"} <= set(line)


GOLD = json.loads((ROOT / "tests" / "golden" / "full_size.json").read_text())


@pytest.mark.parametrize("path", ["profiles/r05/bench_headline.json"])
def test_committed_line_ub_frac_matches_the_oracle(path):
    """the committed round-5 driver-command line reports the share of systems
    that hit the reference's undefined behaviour; the oracle's full-size run pins the count."""
    f = ROOT / path
    if not f.exists():
        pytest.skip(f"{path} not committed yet")
    line = json.loads([x for x in f.read_text().splitlines() if x.startswith("{")][-1])
    assert len(json.dumps(line, separators=(",", ":"))) <= bench.LINE_BUDGET
    assert line["ub_frac"] == pytest.approx(GOLD["uniform"]["err_systems"] / GOLD["systems"], rel=1e-2)
    assert line["contention"]["err_systems"] == GOLD["contention"]["err_systems"]
    assert line["contention"]["digest_sum"] == GOLD["contention"]["digest_sum"]


def test_committed_line_has_every_row_measured():
    """The committed round-5 line (the driver's command on the final library): every sweep row with
    its value, roofline fraction, HBM traffic from that point's committed PMC passes, the reference
    per CACHE_SIZE with at least three batches, and the three full-size golden points bit-exact."""
    f = ROOT / "profiles" / "r05" / "bench_headline.json"
    if not f.exists():
        pytest.skip("not committed yet")
    line = json.loads([x for x in f.read_text().splitlines() if x.startswith("{")][-1])
    sw = line["sweep"]
    cols = sw["cols"]
    assert len(sw["rows"]) == 25
    for row in sw["rows"]:
        r = dict(zip(cols, row))
        assert r["value_G"] > 0 and 0 < r["frac"] < 1 and r["traffic_GB"] and r["vs_baseline"], row
    assert all(v[0] >= 3 for v in sw["cpu"].values())
    assert len(sw["golden_bit_exact"]) >= 3 and all(sw["golden_bit_exact"])
    assert line["roofline"]["traffic"] and line["issue"]["waves_per_cu"] > 17


@pytest.mark.parametrize("path,world", [("profiles/r06/ev6_a/bench.json", 1), ("profiles/r06/ev6_c/bench.json", 1),
                                        ("profiles/r06/ev6_d/bench.json", 1), ("profiles/r06/ev6_e/bench.json", 1),
                                        ("profiles/r06/two_rank_full/bench.json", 2),
                                        ("profiles/r06/two_rank_full_b/bench.json", 2),
                                        ("profiles/r06/two_rank_full_c/bench.json", 2),
                                        ("profiles/r06/four_rank_full/bench.json", 4)])
def test_committed_r06_lines_certify_themselves(path, world):
    """VERDICT r5 next #1 / #3 on the committed round-6 lines (the driver's command on one GPU, and
    the same at N = 2 with both ranks on the box's GPU): rank 0's slice equals the full-size goldens
    for the headline, contention and all 25 sweep points, every rank checked its sampled ids with no
    mismatch, every stalled reference instance has a cause, and the line fits the driver's budget."""
    f = ROOT / path
    if not f.exists():
        pytest.skip(f"{path} not committed yet")
    text = [x for x in f.read_text().splitlines() if x.startswith("{")][-1]
    assert len(text) <= bench.LINE_BUDGET
    line = json.loads(text)
    assert line["n_gpus"] == world
    g = line["golden"]
    assert g["slice"] == [0, 1 << 20] and g["headline"] is True and g["contention"] is True
    assert g["sweep"][:3] == [25, 25, 25]
    checked, bad, ranks, w = g["samples"]
    assert checked > 0 and bad == 0 and ranks == w == world
    cols = line["sweep"]["cols"]
    for row in line["sweep"]["rows"]:
        r = dict(zip(cols, row))
        assert r["golden"] is True and r["smp_bad"] == 0 and r["vs_baseline"] > 0, row
    for cs, (points, batches, hung, explained) in line["sweep"]["cpu"].items():
        assert points == 5 and batches >= 15 and explained == hung, cs
    assert line["cpu_baseline"]["hung_explained"] == line["cpu_baseline"]["hung"]
    assert line["ub_frac"] == pytest.approx(GOLD["uniform"]["err_systems"] / GOLD["systems"], rel=1e-2)
    if "ranks" in g:  # since the whole-slice goldens of every rank (full_slices.json)
        assert g["ranks"] == [[world, world], [world, world]]
    if len(g["sweep"]) == 5:  # slice 1 of every configs[4] point is committed, slices 2.. are not
        assert g["sweep"][3:] == [25 * min(world, 2)] * 2
