"""Generate tests/golden/ref_runs/micro{4,8}.json: reference runs that are NOT executions of the
engine's round model, re-enacted through a micro-step schedule (dash_set_micro_schedule).

TEST INFRASTRUCTURE. For the guided pin's traces (tests/ref_pin.py gen_trace_large, seeds in
order) the reference pin binaries (oracle/_ref/cache_simulator_pin{,8}_cs{1,4}: assignment.c +
the benchmark patch, -DDEBUG_MSG -DDEBUG_INSTR) run each trace. A run is kept when
orc_rounds_from_logs proves (complete search) that no engine round schedule reproduces its logs,
i.e. one of its threads was interleaved between its own sendMessage calls (ref :741-765). The
oracle's log-guided search (orc_guided_witness, STRICT model) then recovers an interleaving of
the reference's threads that meets every thread's log: a sequence of micro-steps (a thread pops
or issues; a thread completes one sendMessage), checked by re-executing it
(orc_replay_steps: the outcome is the reference's dumps). A case holds the trace, that sequence
as "P<t>" / "I<t>" (node t pops / issues: a step) and "D<t>" (node t delivers its oldest held
message) tokens, each
thread's logged events (ref_pin.log_tokens) and the digest of the reference's dumps.

Run: python tests/golden/make_ref_micro.py [--all]   (about a minute; --all writes ref_runs/all{4,8}.json:
one run of each of the first ALL traces, none selected)
"""
import json
import pathlib
import subprocess
import sys
import tempfile

HERE = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
import oracle_ctypes as oc  # noqa: E402
import ref_pin  # noqa: E402

RUNS = 40
ALL = 160  # consecutive traces per node count for ref_runs/all{n}.json: every run kept, none selected


def case_of(seed, n, only_non_round):
    """One reference run of trace `seed` as a micro-step case, or None when only_non_round and a
    round schedule exists for it."""
    cs, rows = ref_pin.gen_trace_large(seed, n)
    tr, lens = ref_pin.as_arrays(rows)
    with tempfile.TemporaryDirectory() as td:
        d = pathlib.Path(td)
        ref_pin.write_trace(d / "tests" / "t", rows)
        p = subprocess.run(["timeout", "20", str(ref_pin.pin_exe(cs, n)), "t"], cwd=d, capture_output=True,
                           text=True, check=True)
        dumps = [(d / f"core_{k}_output.txt").read_text() for k in range(n)]
    ev, _ = oc.parse_logs(p.stdout, n)
    round_model = None
    if only_non_round:
        sched, _ = oc.rounds_from_logs(tr, lens, ev, num_procs=n, cache_size=cs, max_states=10_000_000)
        if sched is not None:
            return None
        round_model = False
    found, out, steps = oc.guided_witness(tr, lens, ev, num_procs=n, cache_size=cs)
    digest = oc.dumps_digest(dumps, cs)
    assert found and out.digest == digest, seed
    rep, term = oc.replay_steps(tr, lens, steps, num_procs=n, cache_size=cs)
    assert term and rep.digest == digest, seed
    c = {"seed": seed, "num_procs": n, "cache_size": cs,
         "trace": [[f"WR 0x{(w >> 8) & 0x7F:02X} {w & 0xFF}" if w & 0x8000 else f"RD 0x{(w >> 8) & 0x7F:02X}"
                    for w in r] for r in rows],
         "steps": " ".join("PID"[int(x) >> 8] + str(int(x) & 15) for x in steps),
         "log": ref_pin.log_tokens(p.stdout, n), "digest": f"{digest:016x}"}
    if round_model is not None:
        c["round_model"] = round_model
    return c


def main_all():
    """ref_runs/all{n}.json: one reference run of each of the first ALL traces, every one kept."""
    for n in (4, 8):
        cases = [case_of(seed, n, False) for seed in range(ALL)]
        (HERE / "ref_runs" / f"all{n}.json").write_text(json.dumps(
            {"source": f"tests/golden/make_ref_micro.py --all (oracle/_ref/cache_simulator_pin{'' if n == 4 else n}_cs{{1,4}})",
             "traces": ALL, "cases": cases}, separators=(",", ":")) + "\n")
        print(n, "nodes:", len(cases), "runs, every one kept")


def main():
    if "--all" in sys.argv:
        return main_all()
    for n in (4, 8):
        cases = []
        seed = 0
        while len(cases) < RUNS:
            c = case_of(seed, n, True)
            if c is not None:
                del c["round_model"]
                cases.append(c)
            seed += 1
        (HERE / "ref_runs" / f"micro{n}.json").write_text(json.dumps(
            {"source": f"tests/golden/make_ref_micro.py (oracle/_ref/cache_simulator_pin{'' if n == 4 else n}_cs{{1,4}})",
             "tried_traces": seed, "cases": cases}, indent=0) + "\n")
        print(n, "nodes:", len(cases), "non-round-model runs kept of", seed, "traces")


if __name__ == "__main__":
    main()
