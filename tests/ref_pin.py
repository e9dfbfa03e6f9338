"""TEST INFRASTRUCTURE: the oracle's cross-node handlers checked against the reference itself.

The round-2 pins compared the oracle with the reference binary only on self-homed traces
(every message a self-message). Here the reference runs real cross-node traffic:

  * oracle/_ref/cache_simulator_pin_cs{1,4} is /root/reference/assignment.c with the
    benchmark patch of oracle/patch_ref.py (atomic queue counts, receiver guard, termination)
    at the reference's own NUM_PROCS 4 / MAX_INSTR_NUM 32, built with -DDEBUG_MSG so it
    prints every message it handles (ref :179-182);
  * each trace is a small random 4-node system (2-4 nodes with instructions, 1-4 instructions
    each, addresses on 1-2 cache indices so lines conflict, homes on any node), run
    `RUNS` times from its own scratch directory (dumps land in the CWD, ref :860);
  * the oracle's explorer (orc_explore: every interleaving of the race-free micro-step
    model, pop-first persistent sets) enumerates the trace's COMPLETE legal outcome set;
  * every dump set the reference wrote must be a member of that set.

A handler the oracle restated wrongly changes the outcomes the explorer enumerates, so the
reference's own outcomes fall outside the set. Traces whose exploration does not complete
within MAX_STATES are skipped (deterministically, by seed) until COUNT complete ones ran.

Coverage is counted from the reference's DEBUG_MSG lines: messages handled per
transactionType (ref :30-44), plus
  * WRITEBACK_INV with home == requester: the owner then sends FLUSH_INVACK to the home
    twice (ref :492,498), so per (owner, address) the FLUSH_INVACKs the home handles minus
    the WRITEBACK_INVs the owner handled from it;
  * the EVICT_SHARED hand-off: an EVICT_SHARED handled by a node that is not the address's
    home (sent by the home to the last sharer, ref :569-580).

`python3 tests/ref_pin.py OUT.json` writes the coverage table (profiles/r03/ref_pin_coverage.json);
`--nodes 8` runs the same at the headline's node count (profiles/r03/ref_pin8_coverage.json).

Round 4 -- the GUIDED pin (`run_guided`, `guided_mutant_kills`; `python3 tests/ref_pin.py --guided
[--nodes 8] OUT.json`). The pin binaries also print DEBUG_INSTR (ref :649-652), so every reference
run hands over each thread's whole event log: the messages it popped, in order, and where it
issued. For traces far past complete exploration (5-8 instructions per node on 3-4 blocks, or
6-10 per node hammering 1-2 lines; 2-8 active nodes) the oracle's orc_guided searches the STRICT
race-free micro-step model for an interleaving in which every node pops exactly its logged
messages and issues where it logged an issue, and the final state must then equal the
reference's dumps byte for byte. Each thread's issue log must also equal its trace (the ingest).
A mutant oracle is refuted by the first run it cannot replay (no interleaving exists: the
search is exhaustive) or replays to other dumps -- including m4, whose missing second
FLUSH_INVACK the home's logged pops expose through the mutant build itself.
"""
from __future__ import annotations

import collections
import json
import pathlib
import re
import subprocess
import sys
import tempfile

import numpy as np

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parent))
import oracle_ctypes as oc  # noqa: E402

REF_DIR = oc.ROOT / "oracle" / "_ref"
COUNT = 208
RUNS = 4
# the headline's 8 nodes (oracle/_ref/cache_simulator_pin8_cs{1,4}): 2-4 nodes with instructions
# among 8 homes, fewer runs per trace
COUNT8 = 160
RUNS8 = 3
MAX_STATES = 200_000
THREADS = 6  # explorations in parallel (ctypes drops the GIL)
# oracle/Makefile `mutants`: one misreading of a cross-node handler each (dash_oracle.c ORC_MUTANT)
MUTANTS = {
    1: "WRITEBACK_INT checks the line address before setting SHARED (ref :284 does not)",
    2: "FLUSH clears waitingForReply only at the requester (ref :322 clears it at every receiver)",
    3: "UPGRADE's REPLY_ID carries the whole bitVector, requester included (ref :337-341 removes it)",
    4: "WRITEBACK_INV sends one FLUSH_INVACK when home == requester (ref :492,498 send two)",
    5: "FLUSH_INVACK fills the requester's line with the message value (ref :531: instr.value)",
    6: "EVICT_SHARED at home does not promote the home's own line when it is the last sharer (ref :586)",
    7: "EVICT_SHARED at a non-home node checks the line address before setting EXCLUSIVE (ref :558)",
    8: "READ_REQUEST at S does not add the requester to the sharers (ref :222 does)",
    9: "WRITE_REQUEST at S leaves the directory S (ref :456-457 always set EM / requester)",
    10: "REPLY_WR replaces the line only when it holds another address (ref :467: unconditional)",
    11: "INV invalidates only a SHARED line (ref :396 does not check the state)",
    12: "EVICT_MODIFIED applies only when the sender is the recorded owner (ref :602-616 do not check)",
    13: "a WR hit on EXCLUSIVE keeps the line EXCLUSIVE (ref :706-710 make it MODIFIED)",
}
GUIDED_COUNT = 320  # traces per node count (each run `GUIDED_RUNS` times)
GUIDED_RUNS = 2
MUT_DIR = oc.ROOT / "oracle" / "_mut"
LINE = re.compile(r"Processor (\d+) msg from: (\d+), type: (\d+), address: 0x([0-9A-F]{2})")


def pin_exe(cs, n=4):
    return REF_DIR / (f"cache_simulator_pin_cs{cs}" if n == 4 else f"cache_simulator_pin{n}_cs{cs}")


def available(n=4):
    return all(pin_exe(cs, n).exists() for cs in (1, 4))


def gen_trace(seed, n=4):
    """(cache_size, rows) of one small cross-node n-node system: 2-4 nodes with instructions,
    homes on any of the n nodes."""
    rng = np.random.default_rng(seed)
    cs = (1, 4)[seed % 2]
    act = rng.choice(n, int(rng.integers(2, 5)), replace=False)
    b0 = int(rng.integers(0, 16))
    blocks = [b0] if rng.random() < 0.4 else [b0, (b0 + cs * int(rng.integers(1, 16 // cs))) % 16]
    rows = [[] for _ in range(n)]
    for t in act:
        for _ in range(int(rng.integers(1, 5))):
            a = (int(rng.integers(0, n)) << 4) | int(rng.choice(blocks))
            w = rng.random() < 0.5
            rows[t].append(oc.pack("W" if w else "R", a, int(rng.integers(1, 256)) if w else 0))
    return cs, rows


def gen_trace_large(seed, n=4):
    """(cache_size, rows) of one system past complete exploration, by seed % 3:
      0 'spread': 2-4 active nodes (all 4 at n = 4), 5-8 instructions each on 3-4 blocks homed on
        1-3 nodes;
      1 'hot': 3-6 active nodes (at most n), 6-10 instructions each on 1-2 blocks (a cache index
        apart) homed on 1-2 nodes, so lines bounce between readers and writers (sharers that
        write: m3);
      2 'pairs': 3-5 active nodes, which are also the homes, 6-10 instructions on 2 blocks, half
        of them a read followed by a write of the same line -- a home woken early by a FLUSH for
        another line (ref :322) writes while its read reply is still in flight, so the REPLY_WR
        can land on a line that is valid again (m10)."""
    rng = np.random.default_rng(seed + 10_000)
    cs = (1, 4)[(seed // 3) % 2]
    rows = [[] for _ in range(n)]
    kind = seed % 3
    if kind == 2:
        act = [int(a) for a in rng.choice(n, min(n, int(rng.integers(3, 6))), replace=False)]
        blocks = [int(rng.integers(0, 16))]
        blocks.append((blocks[0] + cs) % 16)
        for t in act:
            prev = None
            for _ in range(int(rng.integers(6, 11))):
                if prev is not None and rng.random() < 0.5:
                    a, w = prev, True
                else:
                    a, w = (int(rng.choice(act)) << 4) | int(rng.choice(blocks)), rng.random() < 0.3
                rows[t].append(oc.pack("W" if w else "R", a, int(rng.integers(1, 256)) if w else 0))
                prev = None if w else a
        return cs, rows
    if kind == 0:
        nb = int(rng.integers(3, 5))
        b0 = int(rng.integers(0, 16))
        blocks = ([(b0 + cs * k) % 16 for k in range(nb)] if rng.random() < 0.5
                  else [int(b) for b in rng.choice(16, nb, replace=False)])
        act = rng.choice(n, int(rng.integers(2, 5)), replace=False) if n > 4 else range(n)
        homes = rng.choice(n, int(rng.integers(1, 4)), replace=False)
        lo, hi = 5, 9
    else:
        blocks = [int(rng.integers(0, 16))]
        if rng.random() < 0.5:
            blocks.append((blocks[0] + cs) % 16)
        homes = rng.choice(n, int(rng.integers(1, 3)), replace=False)
        act = rng.choice(n, min(n, int(rng.integers(3, 7))), replace=False)
        lo, hi = 6, 11
    for t in act:
        for _ in range(int(rng.integers(lo, hi))):
            a = (int(rng.choice(homes)) << 4) | int(rng.choice(blocks))
            w = rng.random() < 0.5
            rows[t].append(oc.pack("W" if w else "R", a, int(rng.integers(1, 256)) if w else 0))
    return cs, rows


def as_arrays(rows):
    L = max(max(len(r) for r in rows), 1)
    tr = np.zeros((len(rows), L), np.uint16)
    for n, r in enumerate(rows):
        tr[n, :len(r)] = r
    return tr, np.array([len(r) for r in rows], np.uint32)


def write_trace(d: pathlib.Path, rows):
    d.mkdir(parents=True, exist_ok=True)
    for n, row in enumerate(rows):
        (d / f"core_{n}.txt").write_text("".join(
            f"WR 0x{(w >> 8) & 0x7F:02X} {w & 0xFF}\n" if w & 0x8000 else f"RD 0x{(w >> 8) & 0x7F:02X}\n"
            for w in row))


def coverage_of(lines, cov):
    """Add one reference run's DEBUG_MSG lines to the coverage counters."""
    fia_home = collections.Counter()  # (home, owner, addr) -> FLUSH_INVACKs handled at the home
    wbinv = collections.Counter()     # (home, owner, addr) -> WRITEBACK_INVs the owner handled
    for m in LINE.finditer(lines):
        rcv, snd, typ, addr = int(m[1]), int(m[2]), int(m[3]), int(m[4], 16)
        home = addr >> 4
        cov[oc.TXN_NAMES[typ]] += 1
        if typ == 10 and rcv == home:
            fia_home[(home, snd, addr)] += 1
        elif typ == 7 and snd == home:
            wbinv[(home, rcv, addr)] += 1
        elif typ == 11 and rcv != home:
            cov["EVICT_SHARED hand-off to a non-home owner"] += 1
    cov["WRITEBACK_INV with home == requester"] += sum(
        max(0, n - wbinv[k]) for k, n in fia_home.items())


def run(count=COUNT, runs=RUNS, max_states=MAX_STATES, n=4):
    """Returns a report: per trace the legal-set size and the reference's outcomes, coverage,
    and the list of violations (reference outcome not in the complete legal set)."""
    cov = collections.Counter()
    cases = []  # (seed, cache_size, rows, the reference's distinct outcomes)
    report = {"traces": 0, "skipped_incomplete": 0, "reference_runs": 0, "violations": [],
              "legal_outcomes_total": 0, "distinct_reference_outcomes_total": 0, "timeouts": 0}
    from concurrent.futures import ThreadPoolExecutor

    def explore(seed):
        cs, rows = gen_trace(seed, n)
        tr, lens = as_arrays(rows)
        # the STRICT model (round 4): a thread's sends complete before its next step, exactly the
        # race-free reference; its complete sets are subsets of the round-3 BUFFERED ones
        outs, _, complete = oc.explore(tr, lens, num_procs=n, cache_size=cs, max_states=max_states,
                                       micro=oc.MICRO_STRICT)
        legal = {tuple(oc.dump_node(o, k, cs) for k in range(n)) for o in outs} if complete else None
        return seed, cs, rows, legal

    with tempfile.TemporaryDirectory() as td, ThreadPoolExecutor(THREADS) as pool:
        nxt = 0
        while report["traces"] < count:
            batch = list(pool.map(explore, range(nxt, nxt + 2 * (count - report["traces"]))))
            nxt += len(batch)
            for seed, cs, rows, legal in batch:
                if report["traces"] >= count:
                    break
                if legal is None:
                    report["skipped_incomplete"] += 1
                    continue
                d = pathlib.Path(td, f"s{seed}")
                write_trace(d / "tests" / "t", rows)
                seen = set()
                for _ in range(runs):
                    p = subprocess.run(["timeout", "10", str(pin_exe(cs, n)), "t"], cwd=d, capture_output=True,
                                       text=True)
                    report["reference_runs"] += 1
                    if p.returncode != 0:
                        report["timeouts"] += 1
                        report["violations"].append({"seed": seed, "why": f"reference exit {p.returncode}"})
                        continue
                    got = tuple((d / f"core_{k}_output.txt").read_text() for k in range(n))
                    seen.add(got)
                    coverage_of(p.stdout, cov)
                    if got not in legal:
                        report["violations"].append({"seed": seed, "cache_size": cs, "why": "outcome not legal"})
                cases.append((seed, cs, rows, seen))
                report["traces"] += 1
                report["legal_outcomes_total"] += len(legal)
                report["distinct_reference_outcomes_total"] += len(seen)
    report["coverage"] = {k: cov[k] for k in oc.TXN_NAMES + ["WRITEBACK_INV with home == requester",
                                                              "EVICT_SHARED hand-off to a non-home owner"]}
    report["cases"] = cases
    return report


def mutant_kills(cases, max_states=MAX_STATES, n=4):
    """For every mutant oracle: the first case (in order) whose COMPLETE legal outcome set under
    the mutant misses an outcome the reference produced, or None if the mutant survives."""
    from concurrent.futures import ThreadPoolExecutor
    if not all((MUT_DIR / f"libdash_oracle_m{k}.so").exists() for k in MUTANTS):
        subprocess.run(["make", "-s", "-C", str(oc.ORACLE_DIR), "mutants"], check=True)
    kills = {}
    for k in MUTANTS:
        L = oc.bind(MUT_DIR / f"libdash_oracle_m{k}.so")

        def killed(case):
            seed, cs, rows, seen = case
            tr, lens = as_arrays(rows)
            outs, _, complete = oc.explore(tr, lens, num_procs=n, cache_size=cs, max_states=max_states, L=L,
                                           micro=oc.MICRO_STRICT)
            if not complete:
                return False
            legal = {tuple(oc.dump_node(o, k, cs, L=L) for k in range(n)) for o in outs}
            return any(got not in legal for got in seen)

        kills[k] = None
        with ThreadPoolExecutor(THREADS) as pool:
            for i in range(0, len(cases), 4 * THREADS):
                chunk = cases[i:i + 4 * THREADS]
                hit = [c for c, dead in zip(chunk, pool.map(killed, chunk)) if dead]
                if hit:
                    kills[k] = hit[0][0]
                    break
    return kills


def run_guided(count=GUIDED_COUNT, runs=GUIDED_RUNS, n=4, threads=THREADS):
    """The guided pin (module docstring): every reference run's event logs replayed by the
    oracle, final dumps compared byte for byte. Returns a report with the runs kept for the
    mutant check."""
    from concurrent.futures import ThreadPoolExecutor
    cov = collections.Counter()
    report = {"traces": 0, "reference_runs": 0, "replayed_exact": 0, "violations": [], "events": 0,
              "instructions": 0, "max_search_states": 0, "timeouts": 0}
    kept = []

    def one(seed):
        cs, rows = gen_trace_large(seed, n)
        tr, lens = as_arrays(rows)
        out = []
        with tempfile.TemporaryDirectory() as td:
            d = pathlib.Path(td)
            write_trace(d / "tests" / "t", rows)
            for _ in range(runs):
                p = subprocess.run(["timeout", "20", str(pin_exe(cs, n)), "t"], cwd=d, capture_output=True,
                                   text=True)
                if p.returncode != 0:
                    out.append((seed, cs, None, None, None, f"reference exit {p.returncode}"))
                    continue
                ev, instr = oc.parse_logs(p.stdout, n)
                dumps = [(d / f"core_{k}_output.txt").read_text() for k in range(n)]
                out.append((seed, cs, p.stdout, ev, (instr, dumps), None))
        return seed, cs, tr, lens, rows, out

    with ThreadPoolExecutor(threads) as pool:
        for seed, cs, tr, lens, rows, out in pool.map(one, range(count)):
            report["traces"] += 1
            for _, _, stdout, ev, extra, err in out:
                report["reference_runs"] += 1
                if err:
                    report["timeouts"] += 1
                    report["violations"].append({"seed": seed, "why": err})
                    continue
                instr, dumps = extra
                coverage_of(stdout, cov)
                report["events"] += sum(len(e) for e in ev)
                report["instructions"] += sum(len(r) for r in rows)
                if instr != rows:
                    report["violations"].append({"seed": seed, "why": "issue log differs from the trace"})
                    continue
                found, res, states, complete = oc.guided(tr, lens, ev, num_procs=n, cache_size=cs)
                report["max_search_states"] = max(report["max_search_states"], states)
                if not found:
                    report["violations"].append({"seed": seed, "why": "no interleaving replays the logs",
                                                 "complete": complete})
                    continue
                if [oc.dump_node(res, k, cs) for k in range(n)] != dumps:
                    report["violations"].append({"seed": seed, "why": "replayed final state differs"})
                    continue
                report["replayed_exact"] += 1
                kept.append((seed, cs, tr, lens, ev, dumps))
    report["coverage"] = {k: cov[k] for k in oc.TXN_NAMES + ["WRITEBACK_INV with home == requester",
                                                              "EVICT_SHARED hand-off to a non-home owner"]}
    report["runs"] = kept
    return report


def guided_mutant_kills(runs, n=4, max_states=2_000_000):
    """For every mutant oracle: (index of the first run it cannot replay, how), or None."""
    if not all((MUT_DIR / f"libdash_oracle_m{k}.so").exists() for k in MUTANTS):
        subprocess.run(["make", "-s", "-C", str(oc.ORACLE_DIR), "mutants"], check=True)
    kills = {}
    for k in MUTANTS:
        L = oc.bind(MUT_DIR / f"libdash_oracle_m{k}.so")
        kills[k] = None
        for i, (seed, cs, tr, lens, ev, dumps) in enumerate(runs):
            found, res, _, complete = oc.guided(tr, lens, ev, num_procs=n, cache_size=cs, L=L,
                                                max_states=max_states)
            if not found and complete:
                kills[k] = (i, seed, "no interleaving of the mutant replays the reference's logs")
                break
            if found and [oc.dump_node(res, q, cs, L=L) for q in range(n)] != dumps:
                kills[k] = (i, seed, "the mutant replays the logs to other final dumps")
                break
    return kills


def replay_cases(n):
    """tests/golden/ref_runs/replay{n}.json (make_ref_replays.py): reference runs with an engine
    round schedule each. Yields (case, cache_size, trace, lens, schedule uint8 [rounds][n])."""
    data = json.loads((oc.ROOT / "tests" / "golden" / "ref_runs" / f"replay{n}.json").read_text())
    for c in data["cases"]:
        rows = [[oc.pack(w[0][0], int(w[1], 16), int(w[2]) if len(w) > 2 else 0)
                 for w in (ln.split() for ln in r)] for r in c["trace"]]
        tr, lens = as_arrays(rows)
        sched = np.array([[0xFF if ch == "-" else int(ch) for ch in row] for row in c["rounds"]],
                         np.uint8).reshape(len(c["rounds"]), n)
        yield c, c["cache_size"], tr, lens, sched


def micro_cases(n, name="micro"):
    """tests/golden/ref_runs/micro{n}.json (make_ref_micro.py): reference runs that are not
    round-model executions (name "all": one run of each of the first 160 traces, none selected),
    with the interleaving of the reference's threads the oracle recovered
    from their logs. Yields (case, cache_size, trace, lens, acts uint8 [rounds][n] in
    dash_set_micro_schedule form, steps uint16 in the oracle's XSTEP form)."""
    data = json.loads((oc.ROOT / "tests" / "golden" / "ref_runs" / f"{name}{n}.json").read_text())
    for c in data["cases"]:
        rows = [[oc.pack(w[0][0], int(w[1], 16), int(w[2]) if len(w) > 2 else 0)
                 for w in (ln.split() for ln in r)] for r in c["trace"]]
        tr, lens = as_arrays(rows)
        toks = c["steps"].split()
        acts = np.full((len(toks), n), 0xFF, np.uint8)
        steps = np.zeros(len(toks), np.uint16)
        for r, tk in enumerate(toks):
            t = int(tk[1:])
            acts[r, t] = 1 if tk[0] == "D" else 0  # MICRO_SEND / MICRO_STEP (a pop or an issue)
            steps[r] = "PID".index(tk[0]) << 8 | t  # the oracle's XSTEP: pop / issue / send
        yield c, c["cache_size"], tr, lens, acts, steps


def log_tokens(text, n):
    """Each thread's DEBUG_MSG / DEBUG_INSTR lines (ref :179-182, :649-652) as tokens, in the
    thread's order: pops "type.sender.ADDR", issues "R.ADDR" / "W.ADDR.value"."""
    out = [[] for _ in range(n)]
    for ln in text.splitlines():
        m = oc.LOG_MSG.match(ln)
        if m:
            out[int(m[1])].append(f"{int(m[3])}.{int(m[2])}.{int(m[4], 16):02X}")
            continue
        m = oc.LOG_INSTR.match(ln)
        if m:
            a = int(m[3], 16)
            out[int(m[1])].append(f"W.{a:02X}.{int(m[4])}" if m[2] == "W" else f"R.{a:02X}")
    return [" ".join(t) for t in out]


def event_tokens(kind_word_node, n):
    """Per-node tokens of (node, is_instr, word) events, as make_ref_replays.py writes them."""
    out = [[] for _ in range(n)]
    for node, instr, w in kind_word_node:
        a = (w >> 8) & 0x7F
        if instr:
            out[node].append(f"W.{a:02X}.{w & 0xFF}" if w & 0x8000 else f"R.{a:02X}")
        else:
            out[node].append(f"{w & 15}.{(w >> 4) & 7}.{a:02X}")
    return [" ".join(t) for t in out]


def explorer_reach(seeds, n, max_states=MAX_STATES):
    """How many of the guided pin's traces the complete explorer (round 3) could not finish."""
    skipped = 0
    for seed in seeds:
        cs, rows = gen_trace_large(seed, n)
        tr, lens = as_arrays(rows)
        _, _, complete = oc.explore(tr, lens, num_procs=n, cache_size=cs, max_states=max_states)
        skipped += not complete
    return skipped


if __name__ == "__main__" and "--guided" in sys.argv:
    args = [a for a in sys.argv[1:] if a != "--guided"]
    n = 4
    if "--nodes" in args:
        n = int(args[args.index("--nodes") + 1])
        del args[args.index("--nodes"):args.index("--nodes") + 2]
    rep = run_guided(n=n)
    runs = rep.pop("runs")
    kills = guided_mutant_kills(runs, n=n)
    rep["mutants"] = {f"m{k}: {MUTANTS[k]}": (f"rejected at reference run {v[0]} (trace seed {v[1]}): {v[2]}"
                                              if v else "NOT REJECTED") for k, v in kills.items()}
    rep["beyond_complete_exploration"] = (f"{explorer_reach(range(rep['traces']), n)} of {rep['traces']} traces "
                                          f"exceed the round-3 explorer's {MAX_STATES} states")
    exe = "cache_simulator_pin_cs{1,4}" if n == 4 else f"cache_simulator_pin{n}_cs{{1,4}}"
    out = json.dumps({"source": f"tests/ref_pin.py --guided (oracle/_ref/{exe}: assignment.c + oracle/patch_ref.py, "
                                f"NUM_PROCS {n}, MAX_INSTR_NUM 32, -DDEBUG_MSG -DDEBUG_INSTR)",
                      "num_procs": n, "count": rep["traces"], "runs_per_trace": GUIDED_RUNS, **rep}, indent=1)
    if args:
        pathlib.Path(args[0]).write_text(out + "\n")
    print(out)
elif __name__ == "__main__":
    args = sys.argv[1:]
    n = 4
    if "--nodes" in args:
        n = int(args[args.index("--nodes") + 1])
        del args[args.index("--nodes"):args.index("--nodes") + 2]
    count, runs = (COUNT, RUNS) if n == 4 else (COUNT8, RUNS8)
    rep = run(count, runs, n=n)
    cases = rep.pop("cases")
    kills = mutant_kills(cases, n=n)
    rep["mutants"] = {f"m{k}: {MUTANTS[k]}": (f"rejected: a reference outcome is not legal under it (trace seed {s})"
                                              if s is not None else "final states do not separate it")
                      for k, s in kills.items()}
    # m4 changes only how many FLUSH_INVACKs the home handles (the second one is idempotent unless
    # another of the home's steps lands between the owner's two sends); the reference's own
    # message stream refutes it: homes handled FLUSH_INVACKs beyond one per WRITEBACK_INV
    dup = rep["coverage"]["WRITEBACK_INV with home == requester"]
    if kills.get(4) is None and dup > 0:
        rep["mutants"][f"m4: {MUTANTS[4]}"] = (f"rejected by the reference's DEBUG_MSG stream: {dup} FLUSH_INVACKs "
                                              f"handled by a home beyond one per WRITEBACK_INV it forwarded")
    exe = "cache_simulator_pin_cs{1,4}" if n == 4 else f"cache_simulator_pin{n}_cs{{1,4}}"
    out = json.dumps({"source": f"tests/ref_pin.py (oracle/_ref/{exe}: assignment.c + "
                                f"oracle/patch_ref.py, NUM_PROCS {n}, MAX_INSTR_NUM 32, -DDEBUG_MSG)",
                      "num_procs": n, "count": count, "runs_per_trace": runs, "max_states": MAX_STATES, **rep},
                     indent=1)
    if args:
        pathlib.Path(args[0]).write_text(out + "\n")
    print(out)
