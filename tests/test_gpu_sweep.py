"""configs[4] on the GPU: every CACHE_SIZE x locality grid point of bench.py --sweep (the
driver's sweep path: on-device locality generator, all queue tiers, totals all-reduced over
the ranks) against the oracle's golden totals (tests/golden/sweep.json): per-type histogram,
instructions, rounds, error systems and the digest checksum, bit-exact. Also with the
systems sharded over two ranks that bench.py starts itself (gloo, both on the one GPU)."""
import json
import os
import pathlib
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = pathlib.Path(__file__).resolve().parent.parent
GOLD = json.loads((ROOT / "tests" / "golden" / "sweep.json").read_text())


def _sweep(gpus):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    per_rank = GOLD["systems"] // gpus
    # one rank: the reference baseline per point too (2 concurrent instances to keep it short)
    cpu = ["--ref-instances", "2", "--sweep-cpu-seconds", "0.2"] if gpus == 1 else ["--no-cpu-baseline"]
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--sweep", "--gpus", str(gpus),
                        "--dist-backend", "gloo", "--systems", str(per_rank), "--len", str(GOLD["instr_per_node"]),
                        "--steps", "1", "--warmup", "0", "--seed", str(GOLD["seed"])] + cpu,
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    d = json.loads((ROOT / line["detail"]).read_text())  # the full record (side file)
    assert len(line["sweep"]["rows"]) == 25
    return d


@pytest.mark.parametrize("gpus", [1, 2])
def test_sweep_grid_matches_oracle(gpus):
    line = _sweep(gpus)
    assert line["n_gpus"] == gpus
    got = {(p["cache_size"], p["locality"]): p for p in line["sweep"]["points"]}
    assert len(got) == 25
    for want in GOLD["points"]:
        p = got[(want["cache_size"], want["locality"])]
        for k in ("hist", "instructions", "rounds_total", "err_systems", "digest_sum"):
            assert p[k] == want[k], (want["cache_size"], want["locality"], k)
        # a complete measured line per point: the kernel average over the
        # timed steps (never above the step time), its roofline, and the reference per point
        assert p["kernel_ms_avg"] <= p["ms_per_step"] and len(p["kernel_ms_steps"]) == line["steps"]
        assert p["roofline"]["bound"] == "hbm" and 0 < p["roofline"]["frac"] < 1
        if gpus == 1:
            # the reference per CACHE_SIZE, >= 3 batches
            assert p["cpu_baseline"]["kind"] == "reference", p["cpu_baseline_note"]
            assert f"CS={p['cache_size']}" in p["cpu_baseline"]["sample"]
            assert p["cpu_baseline"]["batches"]["n"] >= 3
            assert f"locality {p['locality']:g}" in p["cpu_baseline"]["sample"]  # its own traces
            assert abs(p["vs_baseline"] - p["value"] / p["cpu_baseline"]["value"]) < 1e-9 * p["vs_baseline"]


def test_headline_line_carries_the_sweep():
    """The default bench.py line's `sweep` object (configs[4] driver-observed):
    forced on at 4096 systems, its 25 points equal the oracle's golden totals, each with its
    kernel average, roofline, one reference batch per point and the golden check (n/a here)."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--systems", str(GOLD["systems"]),
                        "--len", str(GOLD["instr_per_node"]), "--seed", str(GOLD["seed"]), "--steps", "1",
                        "--warmup", "0", "--contention-steps", "0", "--line-sweep", "on", "--cpu-seconds", "0.2",
                        "--ref-instances", "2", "--line-next", "on", "--next-event-systems", "256"],
                       capture_output=True, text=True, timeout=400, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    # what the driver keeps of a run is a ~10 KB tail of stdout + stderr:
    # the line is the last stdout line, <= 4 KB, and stderr stays quiet
    last = r.stdout.rstrip("\n").splitlines()[-1]
    assert len(last.encode()) <= 4096 and len(last.encode()) + len(r.stderr.encode()) <= 5120, \
        (len(last), r.stderr[-2000:])
    compact = json.loads(last)
    assert len(compact["sweep"]["rows"]) == 25 and compact["roofline"]["bound"] == "hbm"
    assert compact["cpu_baseline"]["kind"] == "reference" and compact["next"]["parity"]
    line = json.loads((ROOT / compact["detail"]).read_text())
    sw = line["sweep"]
    assert sw["steps"] == 1 and sw["warmup"] == 1 and len(sw["points"]) == 25
    got = {(p["cache_size"], p["locality"]): p for p in sw["points"]}
    for want in GOLD["points"]:
        p = got[(want["cache_size"], want["locality"])]
        for k in ("hist", "instructions", "rounds_total", "err_systems", "digest_sum"):
            assert p[k] == want[k], (want["cache_size"], want["locality"], k)
        assert p["kernel_ms_avg"] <= p["ms_per_step"] and 0 < p["roofline"]["frac"] < 1
        assert p["cpu_baseline"]["kind"] == "reference", p["cpu_baseline_note"]
        assert p["cpu_baseline"]["batches"]["n"] >= 3 and p["err_frac"] == p["err_systems"] / GOLD["systems"]
        # ub_frac counts only the reference's undefined sends (DASH_ERR_OOB / CTZ0)
        assert p["ub_frac"] == p["ub_systems"] / GOLD["systems"] and p["ub_systems"] <= p["err_systems"]
        # the reference on this point's own traces, every stalled instance explained or counted
        assert f"locality {p['locality']:g}" in p["cpu_baseline"]["sample"]
        st = p["cpu_baseline"]["stalled"]
        assert st["n"] == p["cpu_baseline"]["hung_instances_killed"] and 0 <= st["explained"] <= st["n"]
    box = line["box"]
    assert box["device"]["compute_units"] > 0 and box["device"]["clock_khz"] > 0
    for k in ("probe_before", "probe_after"):
        pb = box[k]
        assert pb["probe_ms"] > 0 and 300 < pb["sclk_mhz"] <= box["device"]["clock_khz"] / 1e3 * 1.05, pb
    cb = line["cpu_baseline"]["batches"]
    assert cb["min"] <= cb["median"] <= cb["max"]
    nx = line["next"]  # the event-log and seeded-schedule rows, each with its parity property
    assert nx["events"]["parity_same_digests_as_fast"] and nx["events"]["parity_events_logged"]
    assert nx["seeded"]["parity_all_issued"] and nx["seeded"]["parity_reproducible"]


FULL = ROOT / "tests" / "golden" / "sweep_full.json"


@pytest.mark.skipif(not FULL.exists(), reason="tests/golden/sweep_full.json not generated")
def test_full_size_sweep_points_match_oracle():
    """Three configs[4] points at the full 2^20 systems x 8 nodes x 4096 instructions (CACHE_SIZE 1 /
    locality 0, 4 / 0.5, 16 / 1) bit-exact against the oracle's full-size run (make_sweep_full.py)."""
    sys.path.insert(0, str(ROOT))
    import bench
    dash = bench.load_dash()
    gold = json.loads(FULL.read_text())
    for gp in gold["points"]:
        with dash.Engine(gold["systems"], num_procs=8, cache_size=gp["cache_size"],
                         max_instr=gold["instr_per_node"]) as eng:
            eng.generate(gold["seed"], gold["instr_per_node"], kind=dash.GEN_LOCALITY,
                         locality=int(round(gp["locality"] * 65536)))
            st = eng.run()
            dsum = bench.digest_sum(eng.read_results()[0])
        assert st["hist"] == gp["hist"] and st["instructions"] == gp["instructions"], gp["cache_size"]
        assert st["rounds_total"] == gp["rounds_total"] and st["err_systems"] == gp["err_systems"]
        assert dsum == gp["digest_sum"]
