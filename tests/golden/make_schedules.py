"""Generate tests/golden/schedules/: a classification of every accepted output of the
reference's racy tests (tests/test_3/run_*, tests/test_4/run_*; test3.sh / test4.sh accept any
one of them) against the oracle's micro-step model, with witnesses.

TEST INFRASTRUCTURE (uses the oracle only). For each run_k:
  * target = the system digest of the reference's own run_k dumps (parsed back into node state);
  * `reach`: oracle orc_reach, a goal-directed DFS over the STRICT race-free micro-step model
    (a thread's sendMessage calls complete before its next pop or issue, as in assignment.c
    :741-765), trying node-priority orders until a terminal state with that digest is found;
    its witness (one token per micro-step: P<t> pop, I<t> issue, S<t> send) is committed and replayed by the tests;
  * `rounds`: an engine round schedule (dash_set_schedule) reaching the same output, found by a
    seeded random search over per-node sit-out probabilities and delivery orders with the
    oracle's twin (orc_run_system with cfg.sched), then minimised (rounds turned back into
    lockstep rounds while the output stays run_k). One string per round, one character per
    node: '-' = sits the round out, else its delivery position.
If no race-free witness existed, the script would search the RACE model (the unlocked count--
of :177 against count++ of :757) next; every accepted run is reached race-free, so it does not.

Run: python tests/golden/make_schedules.py  (a few seconds)
"""
import itertools
import json
import pathlib
import sys

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
import oracle_ctypes as oc  # noqa: E402

N = 4


def accepted(test):
    d = oc.GOLDEN / test
    return {r.name: [(r / f"core_{n}_output.txt").read_text() for n in range(N)] for r in sorted(d.glob("run_*"))}


def find_witness(tr, lens, target):
    for prio in itertools.permutations(range(N)):
        hit, wit, states, _ = oc.reach(tr, lens, [target], prio=list(prio), max_states=5_000_000)
        if hit == 0:
            return list(prio), wit, states
    return None, None, None


def find_rounds(tr, lens, target, seed=0, tries=200_000, R=200):
    if oc.run_system(tr, lens).digest == target:
        return np.zeros((0, N), np.uint8)
    rng = np.random.default_rng(seed)
    for _ in range(tries):
        p = rng.uniform(0, 1, size=N) ** 3 * 0.97
        stall = rng.random((R, N)) < p
        pos = np.argsort(rng.random((R, N)), axis=1).astype(np.uint8)
        sched = np.where(stall, 0xFF, pos).astype(np.uint8)
        if oc.run_system(tr, lens, sched=sched).digest == target:
            return minimise(tr, lens, sched, target)
    return None


def minimise(tr, lens, sched, target):
    lock = np.arange(N, dtype=np.uint8)
    ok = lambda s: oc.run_system(tr, lens, sched=s).digest == target  # noqa: E731
    for r in reversed(range(len(sched))):
        if not (sched[r] == lock).all():
            old = sched[r].copy()
            sched[r] = lock
            if not ok(sched):
                sched[r] = old
    for r in range(len(sched)):
        for t in range(N):
            if sched[r, t] == 0xFF:
                old = sched[r].copy()
                row = old.copy()
                row[t] = 0
                for i, u in enumerate([u for u in range(N) if row[u] != 0xFF]):
                    row[u] = i
                sched[r] = row
                if not ok(sched):
                    sched[r] = old
    keep = [r for r in range(len(sched)) if not (sched[r] == lock).all()]
    return sched[:keep[-1] + 1] if keep else sched[:0]


def rounds_text(sched):
    return ["".join("-" if v == 0xFF else str(int(v)) for v in row) for row in sched]


def main():
    out = HERE / "schedules"
    out.mkdir(exist_ok=True)
    for test in ("test_3", "test_4"):
        tr, lens = oc.load_test_dir(oc.GOLDEN / test)
        for run, dumps in accepted(test).items():
            target = oc.dumps_digest(dumps)
            prio, wit, states = find_witness(tr, lens, target)
            assert wit is not None, f"{test}/{run}: no race-free witness"
            sched = find_rounds(tr, lens, target)
            assert sched is not None, f"{test}/{run}: no round schedule found"
            rec = {
                "test": test, "run": run, "digest": f"{target:016x}",
                "classification": "legal: reached by the race-free reference (STRICT micro-step model)",
                "reach": {"prio": prio, "states": states, "steps": len(wit)},
                "witness": " ".join(oc.step_str(w) for w in wit),
                "rounds": rounds_text(sched),
            }
            (out / f"{test}_{run}.json").write_text(json.dumps(rec, indent=1).replace('\n  ', ' ') + "\n")
            print(test, run, "witness", len(wit), "steps after", states, "states (prio", prio, ");",
                  len(sched), "schedule rounds")


if __name__ == "__main__":
    main()
