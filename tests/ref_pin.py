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
}
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
        outs, _, complete = oc.explore(tr, lens, num_procs=n, cache_size=cs, max_states=max_states)
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
            outs, _, complete = oc.explore(tr, lens, num_procs=n, cache_size=cs, max_states=max_states, L=L)
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


if __name__ == "__main__":
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
