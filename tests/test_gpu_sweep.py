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
    return json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])


@pytest.mark.parametrize("gpus", [1, 2])
def test_sweep_grid_matches_oracle(gpus):
    line = _sweep(gpus)
    assert line["n_gpus"] == gpus
    got = {(p["cache_size"], p["locality"]): p for p in line["sweep"]}
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
            assert p["cpu_baseline"]["kind"] == "reference", p["cpu_baseline_note"]
            assert f"CS={p['cache_size']}" in p["cpu_baseline"]["sample"]
            assert abs(p["vs_baseline"] - p["value"] / p["cpu_baseline"]["value"]) < 1e-9 * p["vs_baseline"]
