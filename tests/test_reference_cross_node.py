"""The oracle's cross-node handlers pinned against the reference itself (CPU only).

VERDICT r2 (next #3): the round-2 pins ran the reference binary only on self-homed traces,
so the cross-node handlers (WRITEBACK_INT/INV, FLUSH/FLUSH_INVACK, UPGRADE, the
EVICT_SHARED hand-off; ref :257-349, :476-589) rested on three fixture systems. Here
tests/ref_pin.py runs the benchmark-patched reference (4 nodes, 32 instructions, DEBUG_MSG)
on 208 small random cross-node systems, 4 times each, and every dump set it writes must lie
in the oracle explorer's COMPLETE legal outcome set for that trace. Mutation check: seven
oracle builds that each misread one cross-node handler (oracle/Makefile `mutants`) must each
be refuted by the reference's runs. Skipped when the reference binaries were not built.

Round 4 -- the GUIDED pin (tests/ref_pin.py run_guided): 320
traces per node count, 4 and 8 nodes, far past complete exploration (5-10 instructions per node
on 1-4 blocks, up to 8 active nodes), each run twice by the reference built with -DDEBUG_MSG
-DDEBUG_INSTR; every run's per-thread event log is replayed by the oracle's STRICT model
(orc_guided) and must end in the reference's dumps byte for byte. Thirteen mutant oracles
(m1-m7 cross-node handlers; m8-m13 READ_REQUEST's sharer bit, WRITE_REQUEST's EM update,
REPLY_WR's unconditional replacement, INV's missing state check, EVICT_MODIFIED's missing
ownership check, the WR hit on E) are each refuted, at 4 and at 8 nodes, by reference runs kept
as fixtures (tests/golden/ref_logs/, make_ref_logs.py): so the refutations need no reference
binary and do not depend on which interleavings a live run happens to take; m4 is refuted by the
mutant build itself failing to produce the home's logged second FLUSH_INVACK.
"""
import json
import pathlib

import numpy as np
import pytest

import oracle_ctypes as oc
import ref_pin

needs_ref = pytest.mark.skipif(not ref_pin.available(), reason="reference pin binaries not built")


@pytest.fixture(scope="module")
def report():
    return ref_pin.run()


@needs_ref
def test_reference_outcomes_lie_in_the_complete_legal_sets(report):
    assert report["traces"] == ref_pin.COUNT
    assert report["reference_runs"] == ref_pin.COUNT * ref_pin.RUNS
    assert report["violations"] == [], report["violations"][:5]
    assert report["distinct_reference_outcomes_total"] > ref_pin.COUNT  # the reference is racy here


@needs_ref
def test_every_handler_is_exercised_by_the_reference(report):
    cov = report["coverage"]
    assert all(cov[t] > 0 for t in ref_pin.oc.TXN_NAMES), cov
    assert cov["UPGRADE"] >= 10 and cov["REPLY_ID"] >= 10 and cov["INV"] >= 10
    assert cov["WRITEBACK_INV with home == requester"] >= 10
    assert cov["EVICT_SHARED hand-off to a non-home owner"] >= 10


@pytest.mark.skipif(not ref_pin.available(8), reason="8-node reference pin binaries not built")
def test_reference_outcomes_at_eight_nodes():
    """The same pin at the headline's node count: the reference built with NUM_PROCS 8
    (oracle/_ref/cache_simulator_pin8_cs{1,4}) on 160 small random systems whose 2-4 active
    nodes address homes among all 8 nodes, 3 runs each; every dump set lies in the oracle
    explorer's complete legal outcome set, and every handler is exercised."""
    rep = ref_pin.run(ref_pin.COUNT8, ref_pin.RUNS8, n=8)
    assert rep["traces"] == ref_pin.COUNT8
    assert rep["violations"] == [], rep["violations"][:5]
    assert rep["distinct_reference_outcomes_total"] > ref_pin.COUNT8
    assert all(rep["coverage"][t] > 0 for t in ref_pin.oc.TXN_NAMES), rep["coverage"]



@needs_ref
@pytest.mark.parametrize("n", [4, 8])
def test_guided_pin_replays_every_reference_run(n):
    """Every run of the reference on 320 traces past complete exploration, replayed from its own
    event logs by the STRICT race-free model, ends in the reference's dumps byte for byte; each
    thread issued exactly its trace (ingest); every handler is exercised."""
    rep = ref_pin.run_guided(n=n)
    assert rep["traces"] == ref_pin.GUIDED_COUNT
    assert rep["violations"] == [], rep["violations"][:5]
    assert rep["replayed_exact"] == ref_pin.GUIDED_COUNT * ref_pin.GUIDED_RUNS
    cov = rep["coverage"]
    assert all(cov[t] >= 100 for t in oc.TXN_NAMES), cov
    assert cov["WRITEBACK_INV with home == requester"] >= 100
    assert cov["EVICT_SHARED hand-off to a non-home owner"] >= 100


def _fixture_case(c):
    n, cs = c["num_procs"], c["cache_size"]
    rows = [[oc.pack(w[0][0], int(w[1], 16), int(w[2]) if len(w) > 2 else 0)
             for w in (ln.split() for ln in r)] for r in c["trace"]]
    tr, lens = ref_pin.as_arrays(rows)
    ev = [[(1 << 31) if tok == "I" else
           (lambda a: int(a[0]) | int(a[1]) << 8 | int(a[2], 16) << 16)(tok.split("."))
           for tok in line.split()] for line in c["log"]]
    return n, cs, tr, lens, ev


@pytest.mark.parametrize("n", [4, 8])
def test_logged_reference_runs_refute_every_mutant(n):
    """Reference runs kept as fixtures: the real oracle replays each to its dumps exactly, and
    together they refute all thirteen mutants (each listed mutant cannot replay its run)."""
    cases = json.loads((oc.ROOT / "tests" / "golden" / "ref_logs" / f"pin{n}.json").read_text())["cases"]
    refuted = set()
    for c in cases:
        _, cs, tr, lens, ev = _fixture_case(c)
        found, res, _, _ = oc.guided(tr, lens, ev, num_procs=n, cache_size=cs)
        assert found and [oc.dump_node(res, k, cs) for k in range(n)] == c["dumps"], c["seed"]
        for m in c["refutes"]:
            L = oc.bind(ref_pin.MUT_DIR / f"libdash_oracle_{m}.so")
            f, r, _, complete = oc.guided(tr, lens, ev, num_procs=n, cache_size=cs, L=L)
            assert (not f and complete) or [oc.dump_node(r, k, cs, L=L) for k in range(n)] != c["dumps"], (m, c["seed"])
            refuted.add(int(m[1:]))
    assert refuted == set(ref_pin.MUTANTS)


@pytest.mark.parametrize("n", [4, 8])
def test_reference_runs_replay_on_the_round_model(n):
    """Reference runs that are executions of the ENGINE's round model (tests/golden/ref_runs/,
    make_ref_replays.py: 40 per node count, schedules derived from the runs' own logs by
    orc_rounds_from_logs): the oracle's round runner under each schedule prints exactly the
    reference's DEBUG_MSG / DEBUG_INSTR lines, thread by thread, and ends in its dumps (digest).
    tests/test_gpu_parity.py holds the GPU engine to the same runs."""
    k = 0
    for c, cs, tr, lens, sched in ref_pin.replay_cases(n):
        res, log = oc.run_system(tr, lens, num_procs=n, cache_size=cs, sched=sched, log=True, log_msgs=True)
        assert res.digest == int(c["digest"], 16), c["seed"]
        assert ref_pin.log_tokens(log, n) == c["log"], c["seed"]
        k += 1
    assert k == 40


@pytest.mark.parametrize("n", [4, 8])
def test_reference_runs_replay_as_micro_steps(n):
    """Reference runs that are NOT executions of the engine's round model (tests/golden/ref_runs/
    micro{n}.json, make_ref_micro.py: a complete search found no round schedule for their logs --
    a thread was interleaved between its own sendMessage calls): the interleaving of the
    reference's threads that the oracle recovered from each run's logs, re-executed micro-step by
    micro-step (pop / issue / one send), ends quiescent in the reference's dumps (digest).
    tests/test_gpu_parity.py drives the engine through the same interleavings
    (dash_set_micro_schedule)."""
    k = 0
    for c, cs, tr, lens, acts, steps in ref_pin.micro_cases(n):
        out, terminal = oc.replay_steps(tr, lens, steps, num_procs=n, cache_size=cs)
        assert terminal and out.digest == int(c["digest"], 16), c["seed"]
        assert (acts != 0xFF).sum(axis=1).max() == 1  # one acting node per round
        k += 1
    assert k == 40


@pytest.mark.parametrize("n", [4, 8])
def test_every_logged_reference_run_replays_as_micro_steps(n):
    """No selection: one reference run of each of the first 160 guided-pin traces per node count
    (tests/golden/ref_runs/all{n}.json, make_ref_micro.py --all), round-model executions or not,
    replays micro-step by micro-step on the oracle into the reference's dumps."""
    k = 0
    for c, cs, tr, lens, acts, steps in ref_pin.micro_cases(n, "all"):
        out, terminal = oc.replay_steps(tr, lens, steps, num_procs=n, cache_size=cs)
        assert terminal and out.digest == int(c["digest"], 16), c["seed"]
        k += 1
    assert k == 160

