"""The distributed bench path on real hardware, rehearsed on one GPU: bench.py under
torchrun with 2 ranks (both on the box's one GPU, gloo collectives; on an 8-GPU node
the same code runs one rank per GPU over RCCL). Sharding by global system id, the
MAX-over-ranks timing and the SUM of the per-type histograms must reproduce a single
process running all the systems: results do not depend on the GPU count."""
import json
import os
import pathlib
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = pathlib.Path(__file__).resolve().parent.parent
ARGS = ["--systems", "2048", "--len", "4096", "--steps", "1", "--warmup", "0", "--no-cpu-baseline"]
# the torchrun rehearsal keeps the headline workload only


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _line(out):
    """The full record of a bench run: the side file its printed line names (read right after the
    run, before another run overwrites it), with the printed line itself under "_line"."""
    line = json.loads([x for x in out.splitlines() if x.startswith("{")][-1])
    assert len(json.dumps(line, separators=(",", ":"))) <= 4096
    d = json.loads((ROOT / line["detail"]).read_text())
    d["_line"] = line
    return d


def test_two_ranks_match_one_process():
    env = dict(os.environ)
    two = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                          "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
                          str(ROOT / "bench.py"), "--gpus", "2", "--dist-backend", "gloo", "--contention-steps", "0"] + ARGS,
                         capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert two.returncode == 0, two.stderr[-3000:]
    d2 = _line(two.stdout)
    one = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--contention-steps", "0"] + ARGS[:1] + ["4096"]
                         + ARGS[2:], capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert one.returncode == 0, one.stderr[-3000:]
    d1 = _line(one.stdout)
    assert d2["n_gpus"] == 2 and d2["scaling"] == "weak"
    # the group torchrun's ranks actually formed, per-rank kernel spread
    assert d2["_line"]["rccl_world"] == 2 and d2["_line"]["backend"] == "gloo"
    lo, hi = d2["_line"]["kernel_ms_rank"]
    assert 0 < lo <= hi
    assert d2["totals"]["instructions_per_step"] == d1["totals"]["instructions_per_step"] == 4096 * 8 * 4096
    assert d2["totals"]["hist"] == d1["totals"]["hist"]
    assert d2["totals"]["rounds_total"] == d1["totals"]["rounds_total"]
    assert d2["totals"]["err_systems"] == d1["totals"]["err_systems"]
    assert d2["totals"]["digest_sum"] == d1["totals"]["digest_sum"]  # final states, order-free
    # both ranks checked their own sampled ids against the oracle's per-system results
    g = d2["_line"]["golden"]
    assert g["samples"][1] == 0 and g["samples"][2] == g["samples"][3] == 2 and g["samples"][0] > 0, g
    assert d2["samples"]["checked"] == d1["samples"]["checked"] > 0 and d2["samples"]["ranks"] == 2
    # value = all ranks' instructions / max-over-ranks time
    assert abs(d2["value"] - 4096 * 8 * 4096 / (d2["ms_per_step"] / 1e3)) < 1e-6 * d2["value"]


def test_bench_spawns_two_ranks_without_torchrun():
    """`bench.py --gpus 2` starts its own two ranks (no torchrun): same totals as one process."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    two = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                          "--contention-steps", "1"] + ARGS,
                         capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert two.returncode == 0, two.stderr[-3000:]
    d2 = _line(two.stdout)
    one = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--contention-steps", "1"] + ARGS[:1] + ["4096"]
                         + ARGS[2:], capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert one.returncode == 0, one.stderr[-3000:]
    d1 = _line(one.stdout)
    assert d2["n_gpus"] == 2 and d1["n_gpus"] == 1
    assert d2["rccl_world"] == 2 and d1["rccl_world"] == 1 and d1["backend"] is None
    assert d2["totals"] == d1["totals"]
    assert d2["contention"]["totals"] == d1["contention"]["totals"]
    assert d2["contention"]["totals"]["instructions_per_step"] == 4096 * 8 * 4096


def test_multi_gpu_line_carries_the_reference_baseline():
    """the --gpus N line (the one north_star's 8-GPU target is read from)
    carries the reference baseline in both BASELINE.md modes and the ratio to it. Two ranks
    here (gloo, the one GPU); the CPU legs run on rank 0 after the process group is gone."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                        "--contention-steps", "0", "--cpu-seconds", "0.5"] + ARGS[:-1],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2
    a, b = d["cpu_baseline"], d["cpu_baseline_mode_b"]
    assert a["kind"] == b["kind"] == "reference", d["cpu_baseline_note"]
    assert a["mode"] == "A" and a["instances"] == a["cores"] and b["mode"] == "B" and b["instances"] == 1
    assert a["host_cpus_visible"] >= a["cores"]
    assert abs(d["vs_baseline"] - d["value"] / a["value"]) < 1e-9 * d["vs_baseline"]
    assert abs(d["vs_baseline_mode_b"] - d["value"] / b["value"]) < 1e-9 * d["vs_baseline_mode_b"]
    assert d["cpu_port"]["kind"] == "port"


def test_rccl_collectives_one_rank():
    """The RCCL path itself (backend nccl: init_process_group with the device, barriers and the
    MAX / SUM all-reduces of reduce_totals) on the box's one GPU, as a one-rank group: the
    totals equal a run without a process group (the 8-GPU node runs this code per rank)."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK",
                                                            "MASTER_ADDR", "MASTER_PORT")}
    pg = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--process-group", "--dist-backend", "nccl",
                         "--contention-steps", "1"] + ARGS,
                        capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert pg.returncode == 0, pg.stderr[-3000:]
    dp = _line(pg.stdout)
    one = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--contention-steps", "1"] + ARGS,
                         capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert one.returncode == 0, one.stderr[-3000:]
    d1 = _line(one.stdout)
    assert dp["n_gpus"] == 1 and dp["rccl_world"] == 1 and dp["backend"] == "nccl"
    assert dp["totals"] == d1["totals"] and dp["contention"]["totals"] == d1["contention"]["totals"]


def test_two_rank_line_sweep_matches_one_process():
    """The configs[4] grid inside the headline line (`sweep`) under two ranks, as the driver's
    N-GPU runs produce it at full size: every point's totals (all-reduced per point) equal one
    process running all the systems, and `value` counts both ranks' instructions."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    small = ["--len", "256", "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--contention-steps", "0",
             "--line-sweep", "on", "--line-sweep-warmup", "0"]
    two = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
                          "--systems", "512"] + small, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert two.returncode == 0, two.stderr[-3000:]
    one = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--systems", "1024"] + small,
                         capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert one.returncode == 0, one.stderr[-3000:]
    s2, s1 = _line(two.stdout)["sweep"], _line(one.stdout)["sweep"]
    assert len(s2["points"]) == len(s1["points"]) == 25
    keys = ("hist", "instructions", "rounds_total", "err_systems", "dropped", "digest_sum")
    for p2, p1 in zip(s2["points"], s1["points"]):
        assert (p2["cache_size"], p2["locality"]) == (p1["cache_size"], p1["locality"])
        assert {k: p2[k] for k in keys} == {k: p1[k] for k in keys}, (p2["cache_size"], p2["locality"])
        assert p2["instructions"] == 1024 * 8 * 256
        assert abs(p2["value"] - 1024 * 8 * 256 / (p2["ms_per_step"] / 1e3)) < 1e-6 * p2["value"]
    # no full-size golden covers 512 systems per rank: every point's slice flag is null, not false
    assert [p["bit_exact"] for p in s2["golden"]["points"]] == [None] * 25


def test_four_ranks_line_is_the_driver_shape():
    """The 1/2/4/8-GPU lines the driver reads (SCALE) at four ranks, rehearsed on the box's one GPU
    over gloo: the printed line stays within 4 KB with the sweep rows in it, records the world the
    ranks formed and the per-rank kernel spread, and its totals (headline and every sweep point)
    equal one process running all the systems."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    # 4096 instructions per node: the length the golden fixtures hold, so every rank checks its
    # sampled ids (tests/golden/rank_samples.json) in every workload
    small = ["--len", "4096", "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--contention-steps", "1",
             "--line-sweep", "on", "--line-sweep-warmup", "0"]
    four = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "4", "--dist-backend", "gloo",
                           "--systems", "256"] + small, capture_output=True, text=True, timeout=400, env=env, cwd=ROOT)
    assert four.returncode == 0, four.stderr[-3000:]
    d4 = _line(four.stdout)
    one = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--systems", "1024"] + small,
                         capture_output=True, text=True, timeout=400, env=env, cwd=ROOT)
    assert one.returncode == 0, one.stderr[-3000:]
    d1 = _line(one.stdout)
    line = d4["_line"]
    assert line["n_gpus"] == 4 and line["rccl_world"] == 4 and line["backend"] == "gloo"
    lo, hi = line["kernel_ms_rank"]
    assert 0 < lo <= hi and len(line["sweep"]["rows"]) == 25
    assert d4["totals"] == d1["totals"] and d4["contention"]["totals"] == d1["contention"]["totals"]
    keys = ("hist", "instructions", "rounds_total", "err_systems", "dropped", "digest_sum")
    for p4, p1 in zip(d4["sweep"]["points"], d1["sweep"]["points"]):
        assert {k: p4[k] for k in keys} == {k: p1[k] for k in keys}, (p4["cache_size"], p4["locality"])
    # the line certifies itself: all four ranks held sampled ids in all 27 workloads, none differ
    # from the oracle; no full-size slice golden covers 256 systems per rank (null, not false)
    g = line["golden"]
    assert g["samples"][0] >= 27 * 4 and g["samples"][1] == 0 and g["samples"][2] == g["samples"][3] == 4, g
    assert g["headline"] is None and g["contention"] is None and g["sweep"][:3] == [0, 0, 25]
    assert all(r[line["sweep"]["cols"].index("smp_bad")] == 0 for r in line["sweep"]["rows"])


def test_eight_ranks_line_certifies_itself():
    """The driver's N = 8 line shape, rehearsed with eight ranks on the box's one GPU over gloo (256
    systems per rank, the golden fixtures' 4096 instructions, the sweep in the line): all eight ranks
    hold sampled ids in all 27 workloads and none differs from the oracle; the line fits 4 KB."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    small = ["--len", "4096", "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--contention-steps", "1",
             "--line-sweep", "on", "--line-sweep-warmup", "0", "--systems", "256"]
    eight = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "8", "--dist-backend", "gloo"] + small,
                           capture_output=True, text=True, timeout=500, env=env, cwd=ROOT)
    assert eight.returncode == 0, eight.stderr[-3000:]
    d8 = _line(eight.stdout)
    line = d8["_line"]
    assert line["n_gpus"] == 8 and line["rccl_world"] == 8
    g = line["golden"]
    assert g["samples"][1] == 0 and g["samples"][2] == g["samples"][3] == 8, g
    assert g["samples"][0] >= 27 * 8
    assert d8["totals"]["instructions_per_step"] == 8 * 256 * 8 * 4096
