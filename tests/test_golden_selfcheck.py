"""The bench line's self-certification, on the CPU: the fixtures it checks
against and the checks themselves.

* tests/golden/rank_samples.json (make_rank_samples.py) is pinned here against the oracle on a
  spread of its ids and workloads, and its ids give every rank samples at the driver's 1/2/4/8-GPU
  layout (2^20 systems per rank) and at the GPU rehearsals' small layouts;
* bench.slice_golden() accepts rank 0's slice totals exactly when they equal full_size.json /
  sweep_full.json, and says null (not false) when no golden covers the workload;
* bench.sample_check() counts the rank's sampled ids and flags a single wrong digest, round count
  or error bit;
* bench.stall_cause() reads the reference's patch-5 stderr notes (oracle/patch_ref.py).
"""
import argparse
import json
import pathlib
import sys

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import bench  # noqa: E402
import oracle_ctypes as oc  # noqa: E402

SAMPLES = json.loads((ROOT / "tests" / "golden" / "rank_samples.json").read_text())
FULL = json.loads((ROOT / "tests" / "golden" / "full_size.json").read_text())
SWEEP_FULL = json.loads((ROOT / "tests" / "golden" / "sweep_full.json").read_text())
ARGS = argparse.Namespace(len=4096, seed=0x5EED)


def test_samples_cover_all_workloads():
    want = {"uniform", "contention"} | {bench.golden_key("locality", cs, p) for cs, p in bench.SWEEP_GRID}
    assert set(SAMPLES["workloads"]) == want
    n = len(SAMPLES["ids"])
    for w in SAMPLES["workloads"].values():
        assert len(w["digest"]) == len(w["rounds"]) == len(w["errors"]) == n


@pytest.mark.parametrize("world,per_rank", [(1, 1 << 20), (2, 1 << 20), (4, 1 << 20), (8, 1 << 20),
                                            (2, 2048), (4, 256)])
def test_every_rank_holds_samples(world, per_rank):
    ids = SAMPLES["ids"]
    for r in range(world):
        assert sum(r * per_rank <= g < (r + 1) * per_rank for g in ids) >= 4, (world, per_rank, r)


@pytest.mark.parametrize("key", ["uniform", "contention", "locality:16:0", "locality:1:1", "locality:8:0.25"])
def test_samples_pinned_by_the_oracle(key):
    w = SAMPLES["workloads"][key]
    kind = {"uniform": 0, "contention": 1}.get(key, 2)
    loc = 0 if kind != 2 else int(round(float(key.split(":")[2]) * 65536))
    picks = [0, 7, len(SAMPLES["ids"]) // 2, len(SAMPLES["ids"]) - 1]  # includes rank 7's last id
    for i in picks:
        g = SAMPLES["ids"][i]
        r = oc.run_batch(SAMPLES["seed"], g, 1, num_procs=8, cache_size=w["cache_size"],
                         length=SAMPLES["instr_per_node"], kind=kind, locality=loc)
        assert f"{int(r['digests'][0]):016x}" == w["digest"][i], (key, g)
        assert int(r["rounds"][0]) == w["rounds"][i] and int(r["errors"][0]) == w["errors"][i]


def _rank_arrays(key, base, M):
    """Per-system results of a rank owning [base, base + M): the fixture's values at its sampled
    ids, filler elsewhere (sample_check reads only the sampled positions)."""
    w = SAMPLES["workloads"][key]
    d = np.zeros(M, dtype=np.uint64)
    r = np.zeros(M, dtype=np.uint32)
    e = np.zeros(M, dtype=np.uint32)
    for i, g in enumerate(SAMPLES["ids"]):
        if base <= g < base + M:
            d[g - base], r[g - base], e[g - base] = int(w["digest"][i], 16), w["rounds"][i], w["errors"][i]
    return d, r, e


@pytest.mark.parametrize("rank", [0, 3, 7])
def test_sample_check_counts_and_flags(rank):
    M, key = 1 << 20, "locality:4:0.5"
    base = rank * M
    d, r, e = _rank_arrays(key, base, M)
    held = sum(base <= g < base + M for g in SAMPLES["ids"])
    assert bench.sample_check(key, 4, base, M, ARGS, d, r, e) == (held, 0)
    j = next(g - base for g in SAMPLES["ids"] if base <= g < base + M)
    for arr, bump in ((d, 1), (r, 1), (e, 2)):
        arr[j] += bump
        assert bench.sample_check(key, 4, base, M, ARGS, d, r, e) == (held, 1)
        arr[j] -= bump
    # another CACHE_SIZE, length or seed than the fixture's: nothing is checked
    assert bench.sample_check(key, 8, base, M, ARGS, d, r, e) == (0, 0)
    assert bench.sample_check(key, 4, base, M, argparse.Namespace(len=512, seed=0x5EED), d, r, e) == (0, 0)


def _local(g):
    return {k: g[k] for k in ("hist", "instructions", "rounds_total", "err_systems", "digest_sum")}


def test_slice_golden_headline_and_contention():
    M = 1 << 20
    for key in ("uniform", "contention"):
        loc = _local(FULL[key])
        assert bench.slice_golden(key, 4, loc, 0, M, ARGS) is True
        bad = dict(loc, digest_sum=[loc["digest_sum"][0] + 1, loc["digest_sum"][1]])
        assert bench.slice_golden(key, 4, bad, 0, M, ARGS) is False
        bad = dict(loc, hist=[loc["hist"][0] - 1] + loc["hist"][1:])
        assert bench.slice_golden(key, 4, bad, 0, M, ARGS) is False
        # rank 1's slice has its own golden (full_slices.json), which slice 0's totals do not match;
        # another size, another CACHE_SIZE: no golden applies
        assert bench.slice_golden(key, 4, loc, M, M, ARGS) is (False if (ROOT / "tests" / "golden" /
                                                                          "full_slices.json").exists() else None)
        assert bench.slice_golden(key, 4, loc, 0, M // 2, ARGS) is None
        assert bench.slice_golden(key, 8, loc, 0, M, ARGS) is None


def test_slice_golden_sweep_points():
    M = 1 << 20
    for gp in SWEEP_FULL["points"]:
        key = bench.golden_key("locality", gp["cache_size"], gp["locality"])
        assert bench.slice_golden(key, gp["cache_size"], _local(gp), 0, M, ARGS) is True
        bad = dict(_local(gp), rounds_total=gp["rounds_total"] + 1)
        assert bench.slice_golden(key, gp["cache_size"], bad, 0, M, ARGS) is False


def test_golden_record_summarises_every_workload():
    pts = [{"golden_slice": True, "samples": {"checked": 3, "mismatched": 0, "ranks": 8, "world": 8}}] * 24 + \
          [{"golden_slice": None, "samples": {"checked": 3, "mismatched": 1, "ranks": 7, "world": 8}}]
    tot = [0] * 20 + [5, 0, 8, 8, 7]
    cont = {"samples": {"checked": 5, "mismatched": 0, "ranks": 8, "world": 8, "slices_golden": 1,
                        "slices_equal": 1}, "golden_slice": True}
    g = bench.golden_record(True, cont, pts, tot, 8, 1 << 20)
    assert g["headline"] is True and g["contention"] is True and g["sweep"][:3] == [24, 24, 25]
    assert g["samples"] == [5 + 5 + 75, 1, 7, 8]
    assert g["ranks"] == {"headline": [7, 8, 8], "contention": [1, 1, 8]}


def test_stall_cause_reads_the_patch_notes():
    assert bench.stall_cause("") == "no_snapshot"
    assert bench.stall_cause("bench: dropped 12 to node 15\nbench: dropped 8 to node 32\n") == "ctz0_send"
    assert bench.stall_cause("bench: dropped 7 to node 32\n") == "ctz0_send"
    assert bench.stall_cause("bench: queue full at node 0, dropped 9\n") == "queue_full"


SNAP = "bench: snapshot done {d} inflight {f} q0:{q0} q1:{q1}\n"


def test_stall_cause_reads_the_snapshots():
    """patch 6: the last SIGUSR1 snapshot says what a stalled instance was doing (2 nodes here)."""
    idle = SNAP.format(d=1, f=0, q0="5,5,0", q1="9,9,0")
    assert bench.stall_cause("bench: dropped 11 to node 15\n" + idle * 2, 2) == "waits_with_nothing_in_flight"
    assert bench.stall_cause(SNAP.format(d=1, f=256, q0="7,7,256", q1="1,1,0") * 2, 2) == "queue_full"
    assert bench.stall_cause(SNAP.format(d=0, f=3, q0="1,3,2", q1="4,5,1") * 2, 2) == "stuck_with_messages"
    assert not bench.still_moving(idle * 2) and not bench.still_moving(idle)
    moved = idle + SNAP.format(d=1, f=1, q0="5,6,1", q1="9,9,0")
    assert bench.stall_cause(moved, 2) == "still_moving_at_timeout"
    assert bench.still_moving(idle + SNAP.format(d=1, f=1, q0="5,6,1", q1="9,9,0"))
    assert bench.snapshots(idle)[0] == {"done": 1, "inflight": 0, "queues": [(5, 5, 0), (9, 9, 0)]}


def test_patch_ref_has_the_drop_notes():
    """The benchmark binaries note the sends they drop (patch 5), the only stall evidence a
    killed instance leaves."""
    src = (ROOT / "oracle" / "patch_ref.py").read_text()
    assert "bench_note_drop( receiver, msg.type, 0 )" in src and "bench_note_drop( receiver, msg.type, 1 )" in src
    assert 'bench: dropped %d to node %d' in src and 'bench: queue full at node %d, dropped %d' in src
    assert "signal( SIGUSR1, bench_snapshot )" in src and "bench: snapshot done " in src


def test_probe_sees_a_running_reference_move(tmp_path):
    """patch 6 end to end on the real benchmark binary: a reference instance probed while it runs
    answers both SIGUSR1s with snapshots that differ, so bench.py would wait for it, not kill it."""
    import subprocess
    import time
    exe = bench.ref_exe(4)
    if not exe.exists():
        pytest.skip("oracle/_ref not built (no /root/reference here)")
    tr = oc.gen_system(0x5EED, 3, num_procs=8, length=4096, kind=0)
    (tmp_path / "tests" / "b").mkdir(parents=True)
    for n in range(8):
        (tmp_path / "tests" / "b" / f"core_{n}.txt").write_text("".join(
            f"WR {(w >> 8) & 0x7F:02X} {w & 0xFF}\n" if w & 0x8000 else f"RD {(w >> 8) & 0x7F:02X}\n"
            for w in tr[n].tolist()))
    with open(tmp_path / "stderr.txt", "w") as f:
        p = subprocess.Popen([str(exe), "b"], cwd=tmp_path, stdout=subprocess.DEVNULL, stderr=f)
        time.sleep(0.05)
        moving = bench.probe_late([p], [0], [tmp_path], gap=0.1)
        running = p.poll() is None
        p.wait(timeout=120)
    assert p.returncode == 0  # the handler returns; the run completes and dumps
    snaps = bench.snapshots((tmp_path / "stderr.txt").read_text())
    if not running or len(snaps) < 2:
        pytest.skip("the instance finished before the second snapshot")
    assert moving == [0] and len(snaps[0]["queues"]) == 8


def test_slice_golden_of_every_rank(monkeypatch):
    """Slices r >= 1 of the 8-GPU layout (tests/golden/full_slices.json, make_full_slices.py): a rank
    owning [r * 2^20, (r + 1) * 2^20) is checked against slice r's totals; a rank whose slice has no
    golden, or whose size is not 2^20, is null."""
    M = 1 << 20
    tot = _local(FULL["uniform"])
    fake = {"systems_per_slice": M, "instr_per_node": 4096, "seed": 0x5EED, "cache_size": 4,
            "uniform": {"3": dict(tot)}, "contention": {}}
    monkeypatch.setitem(bench._golden_cache, "full_slices.json", fake)
    assert bench.slice_golden("uniform", 4, tot, 3 * M, M, ARGS) is True
    assert bench.slice_golden("uniform", 4, dict(tot, err_systems=tot["err_systems"] + 1), 3 * M, M, ARGS) is False
    assert bench.slice_golden("uniform", 4, tot, 4 * M, M, ARGS) is None
    assert bench.slice_golden("contention", 4, tot, 3 * M, M, ARGS) is None
    assert bench.slice_golden("locality:4:0.5", 4, tot, 3 * M, M, ARGS) is None
    assert bench.slice_golden("uniform", 4, tot, 3 * 4096, 4096, ARGS) is None


def test_full_slices_fixture_is_consistent():
    """Whatever part of tests/golden/full_slices.json is committed: each slice ran every instruction of
    its 2^20 systems, and no two slices (nor slice 0) share a digest checksum."""
    f = ROOT / "tests" / "golden" / "full_slices.json"
    if not f.exists():
        pytest.skip("full_slices.json not generated")
    g = json.loads(f.read_text())
    assert sorted(g["uniform"]) == sorted(g["contention"]) == [str(r) for r in range(1, 8)]
    sweep0 = {bench.golden_key("locality", q["cache_size"], q["locality"]): q for q in SWEEP_FULL["points"]}
    for kind in [k for k in g if k in ("uniform", "contention") or k.startswith("locality:")]:
        sums = {tuple((FULL[kind] if kind in FULL else sweep0[kind])["digest_sum"])}
        for r, t in g[kind].items():
            assert 1 <= int(r) <= 7 and t["instructions"] == (1 << 20) * 8 * 4096
            assert 0 <= t["err_systems"] < 1 << 20 and sum(t["hist"]) > 0
            assert tuple(t["digest_sum"]) not in sums
            sums.add(tuple(t["digest_sum"]))
