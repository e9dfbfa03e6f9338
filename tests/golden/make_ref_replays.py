"""Generate tests/golden/ref_runs/replay{4,8}.json: reference runs that the GPU engine re-enacts.

TEST INFRASTRUCTURE. For the guided pin's traces (tests/ref_pin.py gen_trace_large, seeds in
order) the reference pin binaries (oracle/_ref/cache_simulator_pin{,8}_cs{1,4}: assignment.c +
the benchmark patch, -DDEBUG_MSG -DDEBUG_INSTR) run each trace; for each run the oracle's
orc_rounds_from_logs looks for an ENGINE round schedule (dash_set_schedule form) under which
every node pops exactly the messages of its log, in order, and issues where its log says. About
half of the reference's runs are round-model executions; RUNS of them per node count are kept,
each checked first on the oracle's twin: its per-thread DEBUG lines and its final state (digest
of the reference's dumps) equal the reference's. A case holds the trace, the schedule rows, each
thread's logged events -- pops "type.sender.ADDR", issues "R.ADDR" / "W.ADDR.value", in the
thread's order -- and the digest of the dumps the run wrote (printProcessorState, ref :853-905,
parsed back into node state).

Run: python tests/golden/make_ref_replays.py   (under a minute)
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


def main():
    for n in (4, 8):
        cases = []
        seed = 0
        while len(cases) < RUNS:
            cs, rows = ref_pin.gen_trace_large(seed, n)
            tr, lens = ref_pin.as_arrays(rows)
            with tempfile.TemporaryDirectory() as td:
                d = pathlib.Path(td)
                ref_pin.write_trace(d / "tests" / "t", rows)
                p = subprocess.run(["timeout", "20", str(ref_pin.pin_exe(cs, n)), "t"], cwd=d, capture_output=True,
                                   text=True, check=True)
                dumps = [(d / f"core_{k}_output.txt").read_text() for k in range(n)]
            ev, _ = oc.parse_logs(p.stdout, n)
            sched, _ = oc.rounds_from_logs(tr, lens, ev, num_procs=n, cache_size=cs)
            if sched is not None:
                res, log = oc.run_system(tr, lens, num_procs=n, cache_size=cs, sched=sched, log=True, log_msgs=True)
                digest = oc.dumps_digest(dumps, cs)
                assert res.digest == digest and ref_pin.log_tokens(log, n) == ref_pin.log_tokens(p.stdout, n), seed
                cases.append({"seed": seed, "num_procs": n, "cache_size": cs,
                              "trace": [[f"WR 0x{(w >> 8) & 0x7F:02X} {w & 0xFF}" if w & 0x8000 else
                                         f"RD 0x{(w >> 8) & 0x7F:02X}" for w in r] for r in rows],
                              "rounds": ["".join("-" if v == 0xFF else str(int(v)) for v in row) for row in sched],
                              "log": ref_pin.log_tokens(p.stdout, n), "digest": f"{digest:016x}"})
            seed += 1
        (HERE / "ref_runs").mkdir(exist_ok=True)
        (HERE / "ref_runs" / f"replay{n}.json").write_text(json.dumps(
            {"source": f"tests/golden/make_ref_replays.py (oracle/_ref/cache_simulator_pin{'' if n == 4 else n}_cs{{1,4}})",
             "tried_traces": seed, "cases": cases}, indent=0) + "\n")
        print(n, "nodes:", len(cases), "runs kept of", seed, "traces")


if __name__ == "__main__":
    main()
