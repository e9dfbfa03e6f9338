"""GPU parity: libdash on an MI355X vs the CPU oracle, through the C-ABI.

Bar: bit-exact (integer/byte work). Compared per system: full final state of
every node, per-type message histogram, lockstep round count, error bits and
the 64-bit digest.
"""
import json
import os
import pathlib
import shutil
import subprocess

import numpy as np
import pytest

import bench
from oracle_ctypes import GOLDEN, load_test_dir, run_batch, run_system
import oracle_ctypes

pytestmark = pytest.mark.gpu
ROOT = pathlib.Path(__file__).resolve().parent.parent
TESTS = ["sample", "test_1", "test_2", "test_3", "test_4"]
EXPECT_SET = {"sample": "sample", "test_1": "test_1", "test_2": "test_2", "test_3": "run_1",
              "test_4": "run_1"}


def expected_dir(test):
    return GOLDEN / test if EXPECT_SET[test] == test else GOLDEN / test / EXPECT_SET[test]


def random_batch(rng, nsys, N, maxlen, block_span=16, hot_frac=0.0, fixed_len=False):
    if fixed_len:
        lens = np.full((nsys, N), maxlen, dtype=np.uint32)
    else:
        lens = rng.integers(0, maxlen + 1, size=(nsys, N)).astype(np.uint32)
    shape = (nsys, N, max(maxlen, 1))
    is_w = rng.random(shape) < 0.5
    node = rng.integers(0, N, size=shape)
    blk = rng.integers(0, block_span, size=shape)
    if hot_frac > 0:  # contention: a share of writes to 0x00..0x03
        hot = rng.random(shape) < hot_frac
        is_w |= hot
        node = np.where(hot, 0, node)
        blk = np.where(hot, blk & 3, blk)
    val = np.where(is_w, rng.integers(0, 256, size=shape), 0)
    packed = (is_w.astype(np.uint32) << 15) | (((node << 4) | blk).astype(np.uint32) << 8) | val
    idx = np.arange(shape[2])[None, None, :]
    packed = np.where(idx < lens[:, :, None], packed, 0).astype(np.uint16)
    return packed, lens


def state_arrays(nodes, N, CS):
    out = []
    for n in range(N):
        s = nodes[n]
        out.append((bytes(s.memory), bytes(s.dir_bitvector), bytes(s.dir_state),
                    bytes(s.cache_addr)[:CS], bytes(s.cache_value)[:CS], bytes(s.cache_state)[:CS]))
    return out


def check_batch(dash, packed, lens, N, CS, max_rounds=0, flags=0, seed=0, sched=None):
    nsys = packed.shape[0]
    with dash.Engine(nsys, num_procs=N, cache_size=CS, max_instr=packed.shape[2], keep_state=True,
                     max_rounds=max_rounds, flags=flags, schedule_seed=seed) as eng:
        if sched is not None:
            eng.set_schedule(sched)
        eng.load_traces(packed, lens)
        stats = eng.run()
        dig, rnd, err = eng.read_results()
        hist_total = np.zeros(13, dtype=np.uint64)
        rounds_total = 0
        instr_total = 0
        for s in range(nsys):
            res = run_system(packed[s], lens[s], num_procs=N, cache_size=CS, ring_depth=256,
                             max_rounds=max_rounds or (1024 + 256 * packed.shape[2]), arb_seed=seed,
                             sched=sched)
            gpu_nodes = eng.read_state(s)
            assert state_arrays(gpu_nodes, N, CS) == state_arrays(res.node, N, CS), f"system {s}"
            assert int(rnd[s]) == res.rounds, f"system {s} rounds"
            assert int(err[s]) == res.errors, f"system {s} errors"
            assert int(dig[s]) == res.digest, f"system {s} digest"
            assert eng.read_hist(s).tolist() == list(res.hist), f"system {s} hist"
            hist_total += np.array(list(res.hist), dtype=np.uint64)
            rounds_total += res.rounds
            instr_total += res.instructions
        assert stats["hist"] == hist_total.tolist()
        assert stats["rounds_total"] == rounds_total
        assert stats["systems"] == nsys
        assert stats["instructions"] == instr_total
        if not max_rounds:
            assert instr_total == int(lens.sum())
    return stats


@pytest.mark.parametrize("test", TESTS)
def test_golden_through_simulate_dir(dash, test, tmp_path):
    stats = dash.simulate_dir(GOLDEN / test, out_dir=tmp_path)
    exp = expected_dir(test)
    for n in range(4):
        assert (tmp_path / f"core_{n}_output.txt").read_bytes() == \
            (exp / f"core_{n}_output.txt").read_bytes(), f"{test} core_{n}"
    assert stats["err_bits"] == 0


def test_cli_reference_argv_contract(dash, tmp_path):
    exe = dash.PKG / "cache_simulator"
    (tmp_path / "tests").mkdir()
    shutil.copytree(GOLDEN / "test_4", tmp_path / "tests" / "test_4")
    p = subprocess.run([str(exe), "test_4"], cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    assert p.stdout.splitlines() == [f"Processor {n} initialized" for n in range(4)]
    for n in range(4):
        assert (tmp_path / f"core_{n}_output.txt").read_bytes() == \
            (GOLDEN / "test_4" / "run_1" / f"core_{n}_output.txt").read_bytes()
    p = subprocess.run([str(exe)], cwd=tmp_path, capture_output=True, text=True, timeout=60)
    assert p.returncode == 1 and "Usage:" in p.stderr


@pytest.mark.parametrize("N,CS", [(4, 4), (8, 4), (4, 1), (8, 2), (8, 8), (8, 16), (2, 4),
                                  (3, 4), (5, 2), (1, 4), (6, 4), (7, 8), (8, 1), (4, 16)])
def test_random_traces_bit_exact(dash, N, CS):
    rng = np.random.default_rng(1000 * N + CS)
    packed, lens = random_batch(rng, 160, N, 40)
    check_batch(dash, packed, lens, N, CS)


@pytest.mark.parametrize("N", [4, 8])
def test_contention_and_small_address_space(dash, N):
    rng = np.random.default_rng(77 + N)
    packed, lens = random_batch(rng, 128, N, 48, block_span=4, hot_frac=0.7)
    check_batch(dash, packed, lens, N, 4)


# contention systems (generator seed 0x5EED, 4096 instr/node) whose queues exceed 16 (oracle)
DEEP_SYSTEMS = [16, 67, 105, 199, 230, 236, 285, 309, 332]


@pytest.mark.parametrize("flags", [0, 2, 4])
def test_queue_depth_tiers(dash, flags):
    """Deep queues: systems that would fill a shallow LDS ring are handed to the
    next depth (16 -> 32 -> 256) and re-simulated from scratch; every
    tier's kernel must give the oracle's result (queue capacity 256), and the
    hand-offs must be exactly the systems whose unbounded queues exceed each depth."""
    ids = DEEP_SYSTEMS + [0, 1, 2, 3, 4, 5, 6]
    L = 4096
    packed = np.stack([oracle_ctypes.gen_system(0x5EED, s, 8, L, kind=1) for s in ids])
    lens = np.full((len(ids), 8), L, np.uint32)
    depth = [run_system(packed[i], lens[i], num_procs=8, cache_size=4, ring_depth=256).max_depth
             for i in range(len(ids))]
    stats = check_batch(dash, packed, lens, 8, 4, flags=flags)
    first = {0: 0, 2: 1, 4: 2}[flags]
    tiers = [16, 32, 256]
    expect = [0] * 3
    expect[first] = len(ids)
    for k in range(first + 1, 3):
        expect[k] = sum(d > tiers[k - 1] for d in depth)
    assert stats["tier_systems"] == expect
    assert stats["max_depth"] > 16
    assert sum(d > 16 for d in depth) == len(DEEP_SYSTEMS)


def test_adaptive_first_tier(dash):
    """Without a TIER flag, a run in which > 1/32 of the systems overflowed the
    first depth makes the next run start one depth deeper; results are unchanged."""
    L, nsys = 4096, 64
    with dash.Engine(nsys, num_procs=8, cache_size=1, max_instr=L) as eng:
        eng.generate(0x5EED, L, kind=dash.GEN_CONTENTION)
        s1 = eng.run()
        d1 = eng.read_results()[0].copy()
        s2 = eng.run()
        d2 = eng.read_results()[0]
    assert s1["tier_systems"][0] == nsys and s1["tier_systems"][1] * 32 > nsys
    assert s2["tier_systems"][0] == 0 and s2["tier_systems"][1] == nsys
    assert np.array_equal(d1, d2) and s1["hist"] == s2["hist"]


def test_long_traces_window_refill(dash):
    """Traces far longer than the 3-chunk LDS window, ragged lengths."""
    rng = np.random.default_rng(5)
    packed, lens = random_batch(rng, 24, 8, 777)
    check_batch(dash, packed, lens, 8, 4)


def test_edge_cases(dash):
    rng = np.random.default_rng(9)
    # empty traces, a single system, lengths not a multiple of 8
    packed, lens = random_batch(rng, 1, 4, 13)
    lens[0, :] = [0, 13, 1, 7]
    check_batch(dash, packed, lens, 4, 4)
    packed = np.zeros((3, 8, 8), np.uint16)
    lens = np.zeros((3, 8), np.uint32)
    stats = check_batch(dash, packed, lens, 8, 4)
    assert stats["rounds_total"] == 0


def test_error_paths_match_oracle(dash):
    """Uniform random traces hit the reference's undefined behaviour (stale
    EVICT_SHARED turns the empty 0xFF line EXCLUSIVE; evicting it targets
    node 15). The engine and the oracle must flag and drop identically."""
    rng = np.random.default_rng(123)
    packed, lens = random_batch(rng, 400, 8, 64, fixed_len=True)
    stats = check_batch(dash, packed, lens, 8, 4)
    assert stats["err_bits"] & dash.ERR_OOB  # the path was exercised


def test_round_cap(dash):
    rng = np.random.default_rng(11)
    packed, lens = random_batch(rng, 40, 4, 32, fixed_len=True)
    check_batch(dash, packed, lens, 4, 4, max_rounds=20)
    check_batch(dash, packed, lens, 4, 4, max_rounds=21)  # rounded up to 24 by both
    # clamped to 2^31 - 4 before rounding up ((2^64 - 1 + 3) & ~3 used to wrap to 0)
    check_batch(dash, packed[:8], lens[:8], 4, 4, max_rounds=(1 << 64) - 1)


@pytest.mark.parametrize("kind,loc", [(0, 0), (1, 0), (2, 49152), (2, 0), (2, 65536)])
def test_device_generator_matches_host(dash, kind, loc):
    """dash_generate (on-device, counter-based) == the oracle's host twin."""
    N, CS, L, nsys, seed, base = 8, 4, 96, 200, 0x5EED, 12345
    with dash.Engine(nsys, num_procs=N, cache_size=CS, max_instr=L) as eng:
        eng.generate(seed, L, kind=kind, locality=loc, sys_base=base)
        stats = eng.run()
        dig, rnd, err = eng.read_results()
    ref = run_batch(seed, base, nsys, num_procs=N, cache_size=CS, length=L, kind=kind,
                    locality=loc, threads=4)
    assert np.array_equal(dig, ref["digests"])
    assert np.array_equal(rnd, ref["rounds"])
    assert np.array_equal(err, ref["errors"])
    assert stats["hist"] == ref["hist"].tolist()
    assert stats["instructions"] == ref["instructions"]


@pytest.mark.parametrize("test", TESTS)
def test_debug_trace_matches_oracle(dash, test):
    """DEBUG_MSG / DEBUG_INSTR emission (ref :179-182, :649-652) for a batch of one:
    the engine's event log, formatted, equals the oracle's lockstep log; tracing
    does not change the result."""
    tr, lens = load_test_dir(GOLDEN / test)
    _, log = run_system(tr, lens, log=True, log_msgs=True)
    with dash.Engine(1, num_procs=4, cache_size=4, max_instr=32, keep_state=True, trace_events=256) as eng:
        eng.load_traces(tr[None], lens[None])
        eng.run()
        ev = eng.read_events(0)
        assert dash.format_events(ev) == log
        assert dash.format_events(ev, kinds=(dash.EV_INSTR,)) == run_system(tr, lens, log=True)[1]
        dig = eng.read_results()[0][0]
    assert int(dig) == run_system(tr, lens).digest


def test_debug_trace_random_batch(dash):
    rng = np.random.default_rng(21)
    packed, lens = random_batch(rng, 24, 8, 40)
    with dash.Engine(24, num_procs=8, cache_size=2, max_instr=40, trace_events=512) as eng:
        eng.load_traces(packed, lens)
        eng.run()
        for s in range(24):
            _, log = run_system(packed[s], lens[s], num_procs=8, cache_size=2, log=True, log_msgs=True)
            assert dash.format_events(eng.read_events(s)) == log, s


@pytest.mark.parametrize("seed", [87, 0x5EED5EED])
def test_debug_trace_under_seeded_schedule(dash, seed):
    """The event-log kernel (MODE 2) with a seeded schedule switched on at run time: every
    system's formatted DEBUG_MSG / DEBUG_INSTR log equals the oracle's log of the same seeded
    schedule, and the digests equal those of the seeded kernel without the log (MODE 1)."""
    rng = np.random.default_rng(seed & 0xFFFF)
    packed, lens = random_batch(rng, 24, 8, 40, block_span=4, hot_frac=0.5)
    with dash.Engine(24, num_procs=8, cache_size=2, max_instr=40, trace_events=512, schedule_seed=seed) as eng:
        eng.load_traces(packed, lens)
        eng.run()
        dig_log = eng.read_results()[0]
        for s in range(24):
            _, log = run_system(packed[s], lens[s], num_procs=8, cache_size=2, log=True, log_msgs=True,
                                arb_seed=seed)
            assert dash.format_events(eng.read_events(s)) == log, s
    with dash.Engine(24, num_procs=8, cache_size=2, max_instr=40, schedule_seed=seed) as eng:
        eng.load_traces(packed, lens)
        eng.run()
        assert np.array_equal(eng.read_results()[0], dig_log)


@pytest.mark.parametrize("runs", [1, 2])
def test_debug_trace_through_queue_depth_tiers(dash, runs):
    """The round-major event log of systems that overflow the first queue depth and are re-run
    from scratch at the next one (16 -> 32 -> 256; on the second run of a handle the adaptive
    first tier starts deeper): each system's log is the final run's, equal to the oracle's
    (queue capacity 256), with nothing left over from the shallower run."""
    ids = DEEP_SYSTEMS[:5] + [0, 1, 2]
    L = 4096
    packed = np.stack([oracle_ctypes.gen_system(0x5EED, s, 8, L, kind=1) for s in ids])
    lens = np.full((len(ids), 8), L, np.uint32)
    with dash.Engine(len(ids), num_procs=8, cache_size=4, max_instr=L, trace_events=1 << 16) as eng:
        eng.load_traces(packed, lens)
        for _ in range(runs):
            st = eng.run()
        assert st["tier_systems"][1] > 0  # some systems were re-run deeper
        for i in range(len(ids)):
            _, log = run_system(packed[i], lens[i], num_procs=8, cache_size=4, log=True, log_msgs=True,
                                log_bytes=1 << 26)
            assert dash.format_events(eng.read_events(i)) == log, ids[i]


@pytest.mark.parametrize("N,CS,seed", [(1, 3, 0), (3, 16, 0), (5, 5, 0x5EED5EED), (7, 1, 87), (2, 8, 0)])
def test_debug_trace_other_shapes(dash, N, CS, seed):
    """The round-major event log of the other kernel instantiations (1..7 nodes, generic and
    power-of-two cache sizes, lockstep and seeded): every system's log equals the oracle's
    (tools/diag/event_fuzz.py runs the same check over 512 random configurations)."""
    rng = np.random.default_rng(31 * N + CS)
    packed, lens = random_batch(rng, 48, N, 60, block_span=4, hot_frac=0.3)
    with dash.Engine(48, num_procs=N, cache_size=CS, max_instr=60, trace_events=4096, schedule_seed=seed) as eng:
        eng.load_traces(packed, lens)
        eng.run()
        for s in range(48):
            _, log = run_system(packed[s], lens[s], num_procs=N, cache_size=CS, log=True, log_msgs=True,
                                arb_seed=seed)
            assert dash.format_events(eng.read_events(s)) == log, s


def test_event_log_capacity_is_counted_in_rounds(dash):
    """dash_cfg.trace_events counts rounds (include/dash.h): a log of exactly the run's rounds
    holds every event; one whose capacity (rounded up to 4) ends before the last active round
    reports DASH_ETRUNC."""
    tr, lens = load_test_dir(GOLDEN / "test_4")
    _, log = run_system(tr, lens, log=True, log_msgs=True)
    with dash.Engine(1, num_procs=4, cache_size=4, max_instr=32, trace_events=4096) as eng:
        eng.load_traces(tr[None], lens[None])
        rounds = eng.run()["rounds_max"]
    with dash.Engine(1, num_procs=4, cache_size=4, max_instr=32, trace_events=rounds) as eng:
        eng.load_traces(tr[None], lens[None])
        eng.run()
        assert dash.format_events(eng.read_events(0)) == log
    short = (rounds - 1) // 4 * 4
    assert 0 < short < rounds
    with dash.Engine(1, num_procs=4, cache_size=4, max_instr=32, trace_events=short) as eng:
        eng.load_traces(tr[None], lens[None])
        eng.run()
        with pytest.raises(dash.DashError):
            eng.read_events(0)


def test_event_log_ignores_rows_of_an_earlier_run(dash):
    """the round-major log is never cleared, and the kernel writes rows only up to its
    wave's last trip. A long run followed by a short one on the same handle must read back only
    the short run's events (dash_read_events reads rounds < rounds[sys]), exactly the oracle's."""
    rng = np.random.default_rng(77)
    long_tr, long_lens = random_batch(rng, 16, 8, 120, block_span=4, hot_frac=0.3)
    short_tr, short_lens = random_batch(rng, 16, 8, 120, block_span=4, hot_frac=0.3)
    short_lens = np.minimum(short_lens, 6).astype(np.uint32)
    with dash.Engine(16, num_procs=8, cache_size=4, max_instr=120, trace_events=4096) as eng:
        eng.load_traces(long_tr, long_lens)
        eng.run()
        assert sum(len(eng.read_events(s)) for s in range(16)) > 0
        eng.load_traces(short_tr, short_lens)
        eng.run()
        for s in range(16):
            _, log = run_system(short_tr[s], short_lens[s], num_procs=8, cache_size=4, log=True, log_msgs=True)
            assert dash.format_events(eng.read_events(s)) == log, s


def test_micro_schedule_stepping_a_node_with_held_sends_is_flagged(dash):
    """a micro-step schedule that steps a node whose outbox still holds sends is not a
    reference interleaving and would overrun the 8-entry outbox. The system stops with
    DASH_ERR_SCHEDULE (and the launch ends); a system of the same batch that holds nothing at
    that point is untouched."""
    tr, lens = load_test_dir(GOLDEN / "test_4")
    tr2, lens2 = tr.copy(), lens.copy()
    lens2[0] = 0  # node 0 has nothing to issue, so it never holds a send
    acts = np.full((40, 4), dash.SIT_OUT, np.uint8)
    acts[0:12, 0] = dash.MICRO_STEP  # node 0 steps again and again without delivering
    with dash.Engine(2, num_procs=4, cache_size=4, max_instr=32, schedule_seed=1) as eng:
        eng.set_micro_schedule(acts)
        eng.load_traces(np.stack([tr, tr2]), np.stack([lens, lens2]))
        st = eng.run()
        _, _, err = eng.read_results()
    assert err[0] & dash.ERR_SCHEDULE and not err[1] & dash.ERR_SCHEDULE
    assert st["err_bits"] & dash.ERR_SCHEDULE


def test_event_count_only_call(dash):
    """dash_read_events(h, sys, NULL, 0, &n) counts without copying the log's rows when
    the log holds every round the system ran -- the same count as a full read and as the oracle's
    log -- and still reports DASH_ETRUNC (with the full count) when it does not."""
    import ctypes
    tr, lens = load_test_dir(GOLDEN / "test_4")
    _, log = run_system(tr, lens, log=True, log_msgs=True)
    lib = dash.lib()
    n = ctypes.c_uint32()
    with dash.Engine(1, num_procs=4, cache_size=4, max_instr=32, trace_events=4096) as eng:
        eng.load_traces(tr[None], lens[None])
        eng.run()
        assert lib.dash_read_events(eng.h, 0, None, 0, ctypes.byref(n)) == dash.OK
        assert n.value == len(eng.read_events(0)) == len(log.splitlines())
        total = n.value
    with dash.Engine(1, num_procs=4, cache_size=4, max_instr=32, trace_events=4) as eng:
        eng.load_traces(tr[None], lens[None])
        eng.run()
        assert lib.dash_read_events(eng.h, 0, None, 0, ctypes.byref(n)) == dash.ETRUNC
        assert n.value == total


def test_debug_trace_truncation_is_reported(dash):
    tr, lens = load_test_dir(GOLDEN / "test_4")
    with dash.Engine(1, num_procs=4, cache_size=4, max_instr=32, trace_events=4) as eng:
        eng.load_traces(tr[None], lens[None])
        eng.run()
        with pytest.raises(dash.DashError):
            eng.read_events(0)


def test_cli_debug_flags(dash, tmp_path):
    exe = dash.PKG / "cache_simulator"
    (tmp_path / "tests").mkdir()
    shutil.copytree(GOLDEN / "sample", tmp_path / "tests" / "sample")
    p = subprocess.run([str(exe), "sample", "--debug-instr", "--debug-msg"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    tr, lens = load_test_dir(GOLDEN / "sample")
    _, log = run_system(tr, lens, log=True, log_msgs=True)
    lines = p.stdout.splitlines()
    assert lines[:4] == [f"Processor {n} initialized" for n in range(4)]
    assert "\n".join(lines[4:]) + "\n" == log
    assert [l for l in lines if "instr type" in l] == \
        [l for l in (GOLDEN / "sample" / "instruction_order.txt").read_text().splitlines() if l.strip()]
    for n in range(4):
        assert (tmp_path / f"core_{n}_output.txt").read_bytes() == \
            (GOLDEN / "sample" / f"core_{n}_output.txt").read_bytes()


def test_cli_schedule_seed(dash, tmp_path):
    """`cache_simulator test_4 --schedule 87`: the drop-in CLI with a seeded legal schedule lands
    on the accepted run_2 (test4.sh); without the option it gives run_1 (lockstep)."""
    exe = dash.PKG / "cache_simulator"
    (tmp_path / "tests").mkdir()
    shutil.copytree(GOLDEN / "test_4", tmp_path / "tests" / "test_4")
    for args, run in (([], "run_1"), (["--schedule", "87"], "run_2")):
        p = subprocess.run([str(exe), "test_4"] + args, cwd=tmp_path, capture_output=True, text=True, timeout=120)
        assert p.returncode == 0, p.stderr
        for n in range(4):
            assert (tmp_path / f"core_{n}_output.txt").read_bytes() == \
                (GOLDEN / "test_4" / run / f"core_{n}_output.txt").read_bytes(), (run, n)


def test_bulk_dirs_ingest_and_dump(dash, tmp_path):
    """Trace-directory ingest at scale (ref :822-850 per directory) and bulk
    printProcessorState emission: 40 directories in one batch."""
    dirs = [GOLDEN / TESTS[k % 5] for k in range(40)]
    with dash.Engine(40, num_procs=4, cache_size=4, max_instr=32, keep_state=True) as eng:
        eng.load_dirs(dirs)
        eng.run()
        for k in (0, 1, 2, 3, 4, 37, 39):
            eng.dump_system(k, tmp_path / str(k))
            exp = expected_dir(TESTS[k % 5])
            for n in range(4):
                assert (tmp_path / str(k) / f"core_{n}_output.txt").read_bytes() == \
                    (exp / f"core_{n}_output.txt").read_bytes(), (k, n)
        eng.write_digests(tmp_path / "digests.txt")
    rows = (tmp_path / "digests.txt").read_text().split("\n")
    for k in range(40):
        tr, lens = load_test_dir(GOLDEN / TESTS[k % 5])
        sysid, dig, rounds, err = rows[k].split()
        assert int(sysid) == k and int(dig, 16) == run_system(tr, lens).digest


def test_digest_file_is_the_results_formatted(dash, tmp_path):
    """dash_write_digests (parallel hand-formatted chunks) writes exactly the lines
    "%llu %016llx %u %x" of dash_read_results for every system, across chunk boundaries
    (65,536 lines) and with nonzero error words (uniform traces send to node 15, ref :772)."""
    n = 70_000
    with dash.Engine(n, num_procs=8, cache_size=4, max_instr=48) as eng:
        eng.generate(0x5EED, 48, kind=dash.GEN_UNIFORM)
        eng.run()
        dig, rnd, err = eng.read_results()
        eng.write_digests(tmp_path / "d.txt")
    assert int((err != 0).sum()) > 0
    exp = "".join(f"{k} {int(dig[k]):016x} {int(rnd[k])} {int(err[k]):x}\n" for k in range(n))
    assert (tmp_path / "d.txt").read_text() == exp


def test_cli_batch_and_synthetic(dash, tmp_path):
    exe = dash.PKG / "cache_simulator"
    lst = tmp_path / "dirs.txt"
    lst.write_text("\n".join(str(GOLDEN / t) for t in TESTS) + "\n")
    p = subprocess.run([str(exe), "--batch", str(lst), "-o", str(tmp_path / "out"), "--digests",
                        str(tmp_path / "d.txt")], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    for k, t in enumerate(TESTS):
        for n in range(4):
            assert (tmp_path / "out" / str(k) / f"core_{n}_output.txt").read_bytes() == \
                (expected_dir(t) / f"core_{n}_output.txt").read_bytes()
    p = subprocess.run([str(exe), "--synthetic", "96", "--len", "64", "--kind", "contention", "--digests",
                        str(tmp_path / "s.txt"), "--dump", "3,95", "-o", str(tmp_path / "syn")],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    ref = run_batch(0x5EED, 0, 96, num_procs=8, cache_size=4, length=64, kind=1, threads=4)
    got = [int(r.split()[1], 16) for r in (tmp_path / "s.txt").read_text().split("\n") if r]
    assert got == [int(x) for x in ref["digests"]]
    assert (tmp_path / "syn" / "95" / "core_7_output.txt").exists()


@pytest.mark.parametrize("seed,N,CS", [(1, 8, 4), (87, 4, 4), (0xABCDEF, 8, 2), (5, 3, 1)])
def test_seeded_schedule_bit_exact(dash, seed, N, CS):
    """Seeded legal schedules (stalls + seeded sender order): bit-exact vs the
    oracle's twin (orc_arb_stall / orc_arb_prio), including contention."""
    rng = np.random.default_rng(seed)
    packed, lens = random_batch(rng, 96, N, 48, hot_frac=0.3)
    check_batch(dash, packed, lens, N, CS, seed=seed)


def test_seeded_schedule_past_the_round_table(dash):
    """The seeded schedule's per-round words come from a table built at dash_create; rounds past
    its end hash their key in the kernel. With the table cut to 8 rounds (the test-only flag
    DASH_TEST_SHORT_ARB) most rounds take that path: still bit-exact vs the oracle's twin."""
    rng = np.random.default_rng(44)
    packed, lens = random_batch(rng, 64, 8, 48, hot_frac=0.3)
    check_batch(dash, packed, lens, 8, 4, seed=0xABCDEF, flags=dash.TEST_SHORT_ARB)


def test_seeded_schedule_reaches_other_accepted_run(dash, tmp_path):
    """test_4 accepts run_1..run_4 (test4.sh); lockstep gives run_1, the seeded
    schedule 87 gives run_2 -- both legal serialisations."""
    tr, lens = load_test_dir(GOLDEN / "test_4")
    with dash.Engine(2, num_procs=4, cache_size=4, max_instr=32, keep_state=True, schedule_seed=87) as eng:
        eng.load_traces(np.stack([tr, tr]), np.stack([lens, lens]))
        eng.run()
        eng.dump_system(1, tmp_path)
    for n in range(4):
        assert (tmp_path / f"core_{n}_output.txt").read_bytes() == \
            (GOLDEN / "test_4" / "run_2" / f"core_{n}_output.txt").read_bytes()


SCHED_DIR = ROOT / "tests" / "golden" / "schedules"


@pytest.mark.parametrize("name", sorted(p.stem for p in SCHED_DIR.glob("test_*_run_*.json")))
def test_engine_reproduces_every_accepted_run(dash, name, tmp_path):
    """every accepted output of the racy tests -- test_3/run_1..2 and
    test_4/run_1..4 (test3.sh / test4.sh) -- comes out of the engine byte-exactly. The committed
    round schedule (tests/golden/schedules/, classified legal race-free in tests/test_legality.py)
    goes in through dash_set_schedule; 64 copies of the system run in one batch (a whole wave
    and more) and all of them dump run_k; the event-log kernel under the same schedule logs
    exactly the oracle twin's DEBUG_MSG / DEBUG_INSTR lines."""
    from test_legality import rounds_array
    rec = json.loads((SCHED_DIR / f"{name}.json").read_text())
    test, run = rec["test"], rec["run"]
    tr, lens = load_test_dir(GOLDEN / test)
    sched = rounds_array(rec["rounds"])
    n = 64
    with dash.Engine(n, num_procs=4, cache_size=4, max_instr=32, keep_state=True, schedule_seed=1) as eng:
        eng.set_schedule(sched)
        eng.load_traces(np.stack([tr] * n), np.stack([lens] * n))
        eng.run()
        dig = eng.read_results()[0]
        assert (dig == dig[0]).all()
        eng.dump_system(n - 1, tmp_path)
    assert int(dig[0]) == int(rec["digest"], 16)
    for k in range(4):
        assert (tmp_path / f"core_{k}_output.txt").read_bytes() == \
            (GOLDEN / test / run / f"core_{k}_output.txt").read_bytes(), (run, k)
    _, log = run_system(tr, lens, log=True, log_msgs=True, sched=sched)
    with dash.Engine(1, num_procs=4, cache_size=4, max_instr=32, trace_events=256, schedule_seed=1) as eng:
        eng.set_schedule(sched)
        eng.load_traces(tr[None], lens[None])
        eng.run()
        assert dash.format_events(eng.read_events(0)) == log


def test_cli_round_schedule_file(dash, tmp_path):
    """`cache_simulator test_4 --rounds tests/golden/schedules/test_4_run_k.json`: the drop-in CLI
    with an explicit round schedule writes each accepted run_k of test4.sh, byte-exact."""
    exe = dash.PKG / "cache_simulator"
    (tmp_path / "tests").mkdir()
    shutil.copytree(GOLDEN / "test_4", tmp_path / "tests" / "test_4")
    for run in ("run_1", "run_2", "run_3", "run_4"):
        p = subprocess.run([str(exe), "test_4", "--rounds", str(SCHED_DIR / f"test_4_{run}.json")], cwd=tmp_path,
                           capture_output=True, text=True, timeout=120)
        assert p.returncode == 0, p.stderr
        for n in range(4):
            assert (tmp_path / f"core_{n}_output.txt").read_bytes() == \
                (GOLDEN / "test_4" / run / f"core_{n}_output.txt").read_bytes(), (run, n)


@pytest.mark.parametrize("n", [4, 8])
def test_cli_micro_schedule_file(dash, n, tmp_path):
    """`cache_simulator DIR --micro CASE.json --debug-instr --debug-msg`: the drop-in CLI driven by
    a micro-step schedule prints the reference run's DEBUG lines (thread by thread) and writes its
    dumps, for the first non-round-model reference runs of tests/golden/ref_runs/micro{n}.json."""
    import ref_pin
    exe = dash.PKG / "cache_simulator"
    for i, (c, cs, tr, lens, acts, _) in enumerate(ref_pin.micro_cases(n)):
        if i == 4:
            break
        d = tmp_path / str(i)
        rows = [[tr[t, j] for j in range(lens[t])] for t in range(n)]
        ref_pin.write_trace(d / "tests" / "t", rows)
        (d / "case.json").write_text(json.dumps(c))
        p = subprocess.run([str(exe), "t", "-n", str(n), "-c", str(cs), "--micro", "case.json", "--debug-instr",
                            "--debug-msg"], cwd=d, capture_output=True, text=True, timeout=120)
        assert p.returncode in (0, 2), p.stderr  # 2: a reference UB flag, reported as in any run
        assert ref_pin.log_tokens(p.stdout, n) == c["log"], c["seed"]
        dumps = [(d / f"core_{k}_output.txt").read_text() for k in range(n)]
        assert oracle_ctypes.dumps_digest(dumps, cs) == int(c["digest"], 16), c["seed"]


@pytest.mark.parametrize("N,CS", [(8, 4), (5, 2), (4, 1)])
def test_explicit_schedule_bit_exact(dash, N, CS):
    """dash_set_schedule with random round tables (each node sits a round out with its own
    probability, random delivery positions among all P lanes, 300 rounds, then lockstep):
    every system bit-exact against the oracle's twin (orc_cfg.sched), contention included."""
    rng = np.random.default_rng(1000 + N)
    packed, lens = random_batch(rng, 96, N, 48, hot_frac=0.3)
    P = 1 << (N - 1).bit_length()
    R = 300
    p = rng.uniform(0, 0.8, size=N)
    pos = np.argsort(rng.random((R, P)), axis=1)[:, :N].astype(np.uint8)  # distinct, < P
    sched = np.where(rng.random((R, N)) < p, dash.SIT_OUT, pos).astype(np.uint8)
    check_batch(dash, packed, lens, N, CS, seed=1, sched=sched)


@pytest.mark.parametrize("n", [4, 8])
def test_engine_reenacts_reference_runs(dash, n):
    """The GPU engine against the reference itself, not the oracle: 40 runs per node count of the
    reference binary (tests/golden/ref_runs/, past complete exploration) whose own DEBUG logs
    define an engine round schedule (make_ref_replays.py). Driven by that schedule through
    dash_set_schedule, the engine's event log equals the reference's DEBUG_MSG / DEBUG_INSTR
    lines thread by thread, and its final state is the reference's dumps (digest)."""
    import ref_pin
    k = 0
    for c, cs, tr, lens, sched in ref_pin.replay_cases(n):
        with dash.Engine(1, num_procs=n, cache_size=cs, max_instr=32, trace_events=512, schedule_seed=1) as eng:
            eng.set_schedule(sched)
            eng.load_traces(tr[None], lens[None])
            eng.run()
            dig = int(eng.read_results()[0][0])
            ev = eng.read_events(0)
        assert dig == int(c["digest"], 16), c["seed"]
        got = ref_pin.event_tokens([(e.node, e.kind == dash.EV_INSTR, e.word) for e in ev], n)
        assert got == c["log"], c["seed"]
        k += 1
    assert k == 40


def reenact_micro(dash, n, name, want_err=0):
    import ref_pin
    k = 0
    for c, cs, tr, lens, acts, _ in ref_pin.micro_cases(n, name):
        with dash.Engine(1, num_procs=n, cache_size=cs, max_instr=32, trace_events=4096, schedule_seed=1) as eng:
            eng.set_micro_schedule(acts)
            eng.load_traces(tr[None], lens[None])
            st = eng.run()
            dig = int(eng.read_results()[0][0])
            ev = eng.read_events(0)
        assert not st["err_bits"] & (dash.ERR_ROUNDCAP | dash.ERR_DEADLOCK), c["seed"]  # ran to quiescence
        assert st["err_bits"] & want_err == want_err, c["seed"]
        assert dig == int(c["digest"], 16), c["seed"]
        got = ref_pin.event_tokens([(e.node, e.kind == dash.EV_INSTR, e.word) for e in ev], n)
        assert got == c["log"], c["seed"]
        k += 1
    return k


@pytest.mark.parametrize("n", [4, 8])
def test_engine_reenacts_every_logged_reference_run(dash, n):
    """No selection: one reference run of each of the first 160 guided-pin traces per node count
    (tests/golden/ref_runs/all{n}.json), round-model executions or not, re-enacted through the
    micro-step schedule the oracle recovered from its logs: the engine's event log equals the
    reference's thread by thread and its final state equals the reference's dumps, every run."""
    assert reenact_micro(dash, n, "all") == 160


@pytest.mark.parametrize("n", [4, 8])
def test_engine_reenacts_non_round_model_runs(dash, n):
    """The reference runs the round model cannot express (tests/golden/ref_runs/micro{n}.json: a
    thread interleaved between its own sendMessage calls, 40 per node count): driven through the
    interleaving the oracle recovered from each run's logs, as a micro-step schedule
    (dash_set_micro_schedule, sim_kernel MODE 4: steps hold their sends in an LDS outbox, sends
    are delivered one per round), the engine's event log equals the reference's DEBUG_MSG /
    DEBUG_INSTR lines thread by thread, and its final state is the reference's dumps (digest)."""
    assert reenact_micro(dash, n, "micro") == 40


@pytest.mark.parametrize("n", [4, 8])
def test_engine_reenacts_reference_runs_through_the_undefined_send(dash, n):
    """The reference's undefined send pinned on the reference itself: 40 runs
    per node count of the reference pin binary that evicted a never-filled 0xFF line to node 15
    (assignment.c:772,786; its own stderr shows the receiver guard dropping it,
    tests/golden/ref_runs/ub{n}.json, make_ref_ub.py), re-enacted through the interleaving the
    oracle recovered from their logs: the engine drops and flags the same send (DASH_ERR_OOB), its
    event log equals the reference's thread by thread and its final state is the reference's
    dumps."""
    assert reenact_micro(dash, n, "ub", want_err=dash.ERR_OOB) == 40


@pytest.mark.parametrize("N,CS", [(2, 1), (3, 3), (4, 4), (5, 16), (8, 2), (8, 4)])
def test_micro_schedule_random_interleavings(dash, N, CS):
    """MODE 4 beyond the reference's runs: random legal interleavings of the oracle's STRICT
    micro-step model (tests/micro_fuzz.py: random traces, random node weights, run to
    quiescence) drive the engine through dash_set_micro_schedule; every system ends in the
    walk's final state with the walk's per-node sequence of pops and issues."""
    import micro_fuzz
    rng = np.random.default_rng(1000 + 10 * N + CS)
    bad, skipped = micro_fuzz.one_config(dash, rng, N, CS, 16, 40, random_batch)
    assert bad == [] and len(skipped) < 4


def test_set_micro_schedule_checks_its_input(dash):
    tr, lens = load_test_dir(GOLDEN / "test_4")
    with dash.Engine(1, num_procs=4, cache_size=4, max_instr=32, schedule_seed=1) as eng:
        two = np.full((3, 4), dash.SIT_OUT, np.uint8)
        two[1, 0] = two[1, 2] = dash.MICRO_STEP
        with pytest.raises(dash.DashError):
            eng.set_micro_schedule(two)
        bad = np.full((3, 4), dash.SIT_OUT, np.uint8)
        bad[0, 1] = 5
        with pytest.raises(dash.DashError):
            eng.set_micro_schedule(bad)
    with dash.Engine(1, num_procs=4, cache_size=4, max_instr=32) as eng:
        with pytest.raises(dash.DashError):
            eng.set_micro_schedule(np.full((2, 4), dash.SIT_OUT, np.uint8))


def test_set_schedule_checks_its_input(dash):
    tr, lens = load_test_dir(GOLDEN / "test_4")
    with dash.Engine(1, num_procs=4, cache_size=4, max_instr=32) as eng:
        with pytest.raises(dash.DashError) as e:
            eng.set_schedule(np.zeros((1, 4), np.uint8))
        assert e.value.code == dash.ESTATE
    with dash.Engine(1, num_procs=4, cache_size=4, max_instr=32, schedule_seed=3) as eng:
        for bad in ([[0, 0, 1, 2]], [[0, 1, 2, 4]]):  # repeated position; position >= P
            with pytest.raises(dash.DashError) as e:
                eng.set_schedule(np.array(bad, np.uint8))
            assert e.value.code == dash.EINVAL
        eng.set_schedule(np.zeros((0, 4), np.uint8))  # all lockstep: run_1
        eng.load_traces(tr[None], lens[None])
        eng.run()
        assert int(eng.read_results()[0][0]) == run_system(tr, lens).digest
    with dash.Engine(1, num_procs=4, cache_size=4, max_instr=32, schedule_seed=3,
                     flags=dash.TEST_SHORT_ARB) as eng:  # the table does not hold the whole run
        with pytest.raises(dash.DashError) as e:
            eng.set_schedule(np.zeros((1, 4), np.uint8))
        assert e.value.code == dash.EINVAL


@pytest.mark.parametrize("kind", [0, 1])
def test_full_size_sampled_parity(dash, kind):
    """BASELINE configs[2] (uniform) and [3] (contention) at full size: 1M systems x
    8 nodes x 4096 instructions, CACHE_SIZE 4 (64 GiB of trace). Size-independent
    properties: every instruction issued, per-system statistics consistent with the
    totals, a run started one queue-depth tier deeper gives the same digest of every
    system (checksum of checksums), and 48 sampled systems are bit-exact (digest,
    rounds, error bits) against the oracle. The whole run is bit-exact against the oracle's
    own full-size run (tests/golden/full_size.json, made by tests/golden/make_full_size.py):
    per-type histogram, round and error-system totals, and the order-free sums of all 2^20
    per-system state digests."""
    N, CS, L, nsys, seed = 8, 4, 4096, 1 << 20, 0x5EED
    runs = []
    for flags in (0, dash.TIER_FROM_32):
        with dash.Engine(nsys, num_procs=N, cache_size=CS, max_instr=L, flags=flags) as eng:
            eng.generate(seed, L, kind=kind)
            st = eng.run()
            runs.append((st, eng.read_results()))
    (st, (dig, rnd, err)), (st2, (dig2, rnd2, err2)) = runs
    assert st["systems"] == nsys and st["instructions"] == nsys * N * L
    assert st["rounds_total"] == int(rnd.sum()) and int(rnd.min()) > 0
    assert st["err_systems"] == int(np.count_nonzero(err))
    assert np.array_equal(dig, dig2) and np.array_equal(rnd, rnd2) and np.array_equal(err, err2)
    assert st["hist"] == st2["hist"]
    gold = json.loads((GOLDEN.parent / "full_size.json").read_text())["contention" if kind else "uniform"]
    assert st["hist"] == gold["hist"]
    assert st["instructions"] == gold["instructions"]
    assert st["rounds_total"] == gold["rounds_total"]
    assert st["err_systems"] == gold["err_systems"]
    assert bench.digest_sum(dig) == gold["digest_sum"]
    rng = np.random.default_rng(kind)
    for s in sorted(rng.choice(nsys, 48, replace=False).tolist()):
        ref = run_batch(seed, s, 1, num_procs=N, cache_size=CS, length=L, kind=kind, threads=1)
        assert int(dig[s]) == int(ref["digests"][0]), f"system {s} digest"
        assert int(rnd[s]) == int(ref["rounds"][0]), f"system {s} rounds"
        assert int(err[s]) == int(ref["errors"][0]), f"system {s} errors"


def test_overflow_hint_reruns_match(dash):
    """Repeated runs of the same traces start the systems that overflowed the 16-deep
    rings one tier deeper on a side stream, concurrently with the first tier (which
    skips them): every result and statistic equals the first run's; new traces drop
    the hint (results again equal the oracle's)."""
    N, CS, L, nsys = 8, 4, 1024, 4096
    with dash.Engine(nsys, num_procs=N, cache_size=CS, max_instr=L) as eng:
        eng.generate(0x5EED, L, kind=dash.GEN_CONTENTION)
        runs = []
        for _ in range(3):
            st = eng.run()
            runs.append((st, [x.copy() for x in eng.read_results()]))
        s1, r1 = runs[0]
        assert 0 < s1["tier_systems"][1] and s1["tier_systems"][1] * 32 < nsys  # first tier stays 16
        for st, r in runs[1:]:
            assert all(np.array_equal(a, b) for a, b in zip(r1, r))
            for k in ("hist", "instructions", "rounds_total", "rounds_max", "systems", "err_systems",
                      "dropped", "tier_systems"):
                assert st[k] == s1[k], k
        eng.generate(0xBEEF, L, kind=dash.GEN_CONTENTION)
        st = eng.run()
        dig, rnd, err = eng.read_results()
    ref = run_batch(0xBEEF, 0, nsys, num_procs=N, cache_size=CS, length=L, kind=1, threads=8)
    assert np.array_equal(dig, ref["digests"]) and np.array_equal(rnd, ref["rounds"])
    assert np.array_equal(err, ref["errors"]) and st["hist"] == ref["hist"].tolist()


@pytest.mark.parametrize("N,CS", [(8, 3), (4, 5), (8, 6), (8, 7), (5, 12), (8, 15)])
def test_non_power_of_two_cache_size(dash, N, CS):
    """CACHE_SIZE is a free #define in the reference (cacheIndex = blockIndex % CACHE_SIZE,
    ref :188): non-powers of two run on the generic kernel (runtime modulo, LDS sized for
    16 lines) and match the oracle bit-exactly, including dumps."""
    rng = np.random.default_rng(4000 + 16 * N + CS)
    packed, lens = random_batch(rng, 96, N, 40)
    check_batch(dash, packed, lens, N, CS)
    packed, lens = random_batch(rng, 48, N, 48, block_span=6, hot_frac=0.4)
    check_batch(dash, packed, lens, N, CS)


@pytest.mark.parametrize("N", [8, 5])
def test_rd_value_bits_ignored_at_the_boundary(dash, N):
    """The reference parses every RD with value 0 (ref :839) and later fills REPLY_ID /
    REPLY_WR / FLUSH_INVACK lines with the last issued value (:383,470,531): RD words
    whose bits 7..0 are set must give the results of the clean words (dash.h contract).
    N=8 takes the strided-copy path, N=5 the host re-layout."""
    rng = np.random.default_rng(77 + N)
    clean, lens = random_batch(rng, 96, N, 256, block_span=4)
    dirty = clean.copy()
    rd = (dirty & 0x8000) == 0
    dirty[rd] |= rng.integers(1, 256, size=int(rd.sum())).astype(np.uint16)
    assert (dirty != clean).any()
    with dash.Engine(96, num_procs=N, cache_size=2, max_instr=256, keep_state=True) as eng:
        eng.load_traces(dirty, lens)
        stats = eng.run()
        dig, rnd, err = eng.read_results()
        for s in range(96):
            res = run_system(clean[s], lens[s], num_procs=N, cache_size=2, ring_depth=256)
            assert int(dig[s]) == res.digest and int(rnd[s]) == res.rounds and int(err[s]) == res.errors, s
            assert state_arrays(eng.read_state(s), N, 2) == state_arrays(res.node, N, 2), s
    assert stats["instructions"] == int(lens.sum())


def test_full_queue_is_stuck_like_the_reference(dash):
    """An adversarial 8-node trace (tests/golden/stuck_queue.npy, found by hill-climbing
    queue depth on the oracle) fills a receiver queue to MSG_BUFFER_SIZE = 256. The
    reference then has head == tail and never drains that queue again (:167-170) while
    later sends to it drop (:754-761); the engine models exactly that at its final tier
    (DASH_ERR_STUCK), bit-exact with the oracle."""
    tr = np.load(GOLDEN / ".." / "stuck_queue.npy")
    packed = tr[None, :, :].astype(np.uint16)
    lens = np.full((1, 8), tr.shape[1], dtype=np.uint32)
    # (max_rounds = the default cap, passed explicitly: nodes left waiting never finish their traces)
    stats = check_batch(dash, packed, lens, 8, 1, max_rounds=1024 + 256 * tr.shape[1])
    res = run_system(tr, lens[0], num_procs=8, cache_size=1, ring_depth=256)
    assert res.errors & oracle_ctypes.ERR_STUCK and res.max_depth == 256
    assert stats["err_bits"] & dash.ERR_STUCK
    assert stats["tier_systems"][2] == 1  # handed from the 16- and 32-deep tiers to the reference depth


def test_probe_box_reports_the_device(dash):
    """dash_probe_box: the device's identity and limits, and a probe whose measured shader clock is
    a plausible fraction of the device's maximum (the bench line's `box`)."""
    b = dash.probe_box(0)
    # dash_probe_box itself is arch-agnostic: any AMD GPU the library was built for
    assert b["arch"].startswith("gfx") and b["compute_units"] >= 1, b
    assert b["probe_ms"] > 0 and b["probe_valu_per_s"] > 0
    assert 300 < b["probe_sclk_mhz"] <= b["clock_khz"] / 1e3 * 1.05, b
    assert b["probe_sclk_min_mhz"] <= b["probe_sclk_mhz"] <= b["probe_sclk_max_mhz"]
    with pytest.raises(dash.DashError):
        dash.probe_box(99)


@pytest.mark.parametrize("kind", [0, 1])
def test_every_rank_slice_of_the_eight_gpu_layout(dash, kind):
    """What each rank of the driver's 8-GPU run computes, on one GPU, one slice at a time: global
    systems [r * 2^20, (r + 1) * 2^20) for r = 0..7 (bench.shard; traces keyed by global id), full
    size, uniform / contention. Every slice's sampled systems (tests/golden/rank_samples.json, the
    fixture the bench line checks at any N) equal the oracle's per-system digest, rounds and error
    bits; every slice whose full-size golden is committed (slice 0: full_size.json, slices 1..7:
    full_slices.json) equals it -- the check each rank of the driver's line makes of its own slice."""
    import argparse
    args = argparse.Namespace(len=4096, seed=0x5EED)
    key = ("uniform", "contention")[kind]
    M = 1 << 20
    checked = 0
    with dash.Engine(M, num_procs=8, cache_size=4, max_instr=4096) as eng:
        for r in range(8):
            eng.generate(0x5EED, 4096, kind=kind, sys_base=r * M)
            st = eng.run()
            d, rnd, e = eng.read_results()
            c, bad = bench.sample_check(key, 4, r * M, M, args, d, rnd, e)
            assert c >= 16 and bad == 0, (r, c, bad)
            checked += c
            local = {"hist": st["hist"], "instructions": st["instructions"], "rounds_total": st["rounds_total"],
                     "err_systems": st["err_systems"], "digest_sum": bench.digest_sum(d)}
            ok = bench.slice_golden(key, 4, local, r * M, M, args)
            # slice 0: full_size.json; slices 1..7 where tests/golden/full_slices.json holds them
            assert ok is True if r == 0 else ok is not False, (r, ok)
    assert checked == sum(1 for _ in json.loads((GOLDEN.parent / "rank_samples.json").read_text())["ids"])


def test_sweep_points_on_the_second_slice(dash):
    """configs[4] as rank 1 of the driver's N >= 2 runs computes it: global systems [2^20, 2^21), all
    25 CACHE_SIZE x locality points at full size, each equal to the oracle's run of that slice
    (tests/golden/full_slices.json, make_full_slices.py) -- so an N = 2 line certifies both ranks'
    whole slices at every sweep point."""
    import argparse
    args = argparse.Namespace(len=4096, seed=0x5EED)
    M = 1 << 20
    n = 0
    for cs in (1, 2, 4, 8, 16):
        with dash.Engine(M, num_procs=8, cache_size=cs, max_instr=4096) as eng:
            for p in (0.0, 0.25, 0.5, 0.75, 1.0):
                eng.generate(0x5EED, 4096, kind=dash.GEN_LOCALITY, locality=int(round(p * 65536)), sys_base=M)
                st = eng.run()
                d = eng.read_results()[0]
                local = {"hist": st["hist"], "instructions": st["instructions"], "rounds_total": st["rounds_total"],
                         "err_systems": st["err_systems"], "digest_sum": bench.digest_sum(d)}
                assert bench.slice_golden(bench.golden_key("locality", cs, p), cs, local, M, M, args) is True, (cs, p)
                n += 1
    assert n == 25
