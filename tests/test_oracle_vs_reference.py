"""Pin the oracle against the reference binary itself (CPU only).

oracle/_ref/cache_simulator is /root/reference/assignment.c compiled
unmodified by oracle/build_ref.sh. The reference never exits and its queue
`count` is racy across threads (SURVEY.md §0 finding 1), so it is only a
trustworthy oracle where every message is a self-message: traces in which
each node touches only its own home addresses (like test_1/test_2). There
each node's queue has a single producer/consumer thread and the outcome is
schedule-independent. The binary is run under `timeout` from a scratch CWD
holding tests/<dir>/core_<n>.txt; its last dumps are compared byte-for-byte
with the oracle's. Skipped when the binary was not built (no reference).
"""
import pathlib
import subprocess

import numpy as np
import pytest

from oracle_ctypes import ROOT, dump_node, pack, run_system

REF = ROOT / "oracle" / "_ref" / "cache_simulator"
pytestmark = pytest.mark.skipif(not REF.exists(), reason="reference binary not built")


def write_trace(d: pathlib.Path, rows):
    d.mkdir(parents=True)
    for n, row in enumerate(rows):
        lines = []
        for w in row:
            addr, val = (w >> 8) & 0x7F, w & 0xFF
            lines.append(f"WR 0x{addr:02X} {val}" if w & 0x8000 else f"RD 0x{addr:02X}")
        (d / f"core_{n}.txt").write_text("".join(l + "\n" for l in lines))


@pytest.mark.parametrize("seed", range(6))
def test_self_home_traces_match_reference_binary(tmp_path, seed):
    rng = np.random.default_rng(seed)
    rows = []
    for n in range(4):  # NUM_PROCS is 4 in the reference binary
        k = int(rng.integers(1, 33))
        rows.append([pack("W" if rng.random() < 0.5 else "R", (n << 4) | int(rng.integers(0, 16)),
                          int(rng.integers(0, 256))) for _ in range(k)])
        rows[-1] = [w if w & 0x8000 else (w & 0xFF00) for w in rows[-1]]
    write_trace(tmp_path / "tests" / "t", rows)
    subprocess.run(["timeout", "0.6", str(REF), "t"], cwd=tmp_path, capture_output=True)
    L = max(len(r) for r in rows)
    tr = np.zeros((4, L), np.uint16)
    for n, r in enumerate(rows):
        tr[n, :len(r)] = r
    res = run_system(tr, np.array([len(r) for r in rows], np.uint32), num_procs=4, cache_size=4,
                     ring_depth=256)
    for n in range(4):
        assert (tmp_path / f"core_{n}_output.txt").read_text() == dump_node(res, n, 4), f"node {n}"


BENCH = ROOT / "oracle" / "_ref" / "cache_simulator_bench"


@pytest.mark.skipif(not BENCH.exists(), reason="benchmark reference binary not built")
@pytest.mark.parametrize("seed", range(4))
def test_benchmark_build_of_reference_matches_oracle(tmp_path, seed):
    """oracle/_ref/cache_simulator_bench (the reference + the benchmark patch of
    oracle/patch_ref.py: 8 nodes, 4096 instructions, atomic counts, termination) is
    bench.py's `--cpu-kind reference` baseline. On self-homed 8-node traces of up to 4096
    instructions it must terminate by itself and dump exactly the oracle's final state."""
    rng = np.random.default_rng(100 + seed)
    rows = []
    for n in range(8):
        k = int(rng.integers(1, 4097))
        ws = rng.random(k) < 0.5
        rows.append([pack("W" if w else "R", (n << 4) | int(b), int(v) if w else 0)
                     for w, b, v in zip(ws, rng.integers(0, 16, k), rng.integers(0, 256, k))])
    write_trace(tmp_path / "tests" / "t", rows)
    p = subprocess.run(["timeout", "60", str(BENCH), "t"], cwd=tmp_path, capture_output=True)
    assert p.returncode == 0, p.stderr  # exits on its own (patch 4)
    L = max(len(r) for r in rows)
    tr = np.zeros((8, L), np.uint16)
    for n, r in enumerate(rows):
        tr[n, :len(r)] = r
    res = run_system(tr, np.array([len(r) for r in rows], np.uint32), num_procs=8, cache_size=4,
                     ring_depth=256)
    for n in range(8):
        assert (tmp_path / f"core_{n}_output.txt").read_text() == dump_node(res, n, 4), f"node {n}"
