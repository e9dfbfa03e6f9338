"""Generate tests/golden/ref_logs/pin{4,8}.json: reference runs, with their event logs, that
refute each mutant oracle (tests/ref_pin.py MUTANTS) -- DATA captured from the reference itself.

TEST INFRASTRUCTURE. Needs oracle/_ref/cache_simulator_pin{,8}_cs{1,4} (oracle/patch_ref.py:
assignment.c with the benchmark patch, -DDEBUG_MSG -DDEBUG_INSTR). For the guided pin's traces
(tests/ref_pin.py gen_trace_large) in seed order, each reference run is kept when some mutant not
yet refuted cannot replay it (orc_guided finds no interleaving, or one ending in other dumps),
until all thirteen are refuted. Every kept run is also replayed exactly by the real oracle.
A case holds the trace, each thread's logged events (pops as "type.sender.ADDR", issues as
"I", in the thread's order) and the dumps the run wrote (core_<n>_output.txt, ref :860) --
the reference's outputs, so tests/test_reference_cross_node.py can refute the mutants
deterministically even where the reference is absent.

Run: python tests/golden/make_ref_logs.py  (about a minute)
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


def instr_text(w):
    return f"WR 0x{(w >> 8) & 0x7F:02X} {w & 0xFF}" if w & 0x8000 else f"RD 0x{(w >> 8) & 0x7F:02X}"


def ev_token(e):
    return "I" if e >> 31 else f"{e & 0xFF}.{(e >> 8) & 0xFF}.{(e >> 16) & 0xFF:02X}"


def main(max_seeds=4000, runs=3):
    for n in (4, 8):
        muts = {k: oc.bind(ref_pin.MUT_DIR / f"libdash_oracle_m{k}.so") for k in ref_pin.MUTANTS}
        cases = []
        for seed in range(max_seeds):
            if not muts:
                break
            cs, rows = ref_pin.gen_trace_large(seed, n)
            tr, lens = ref_pin.as_arrays(rows)
            with tempfile.TemporaryDirectory() as td:
                d = pathlib.Path(td)
                ref_pin.write_trace(d / "tests" / "t", rows)
                for _ in range(runs):
                    p = subprocess.run(["timeout", "20", str(ref_pin.pin_exe(cs, n)), "t"], cwd=d,
                                       capture_output=True, text=True, check=True)
                    ev, _ = oc.parse_logs(p.stdout, n)
                    dumps = [(d / f"core_{k}_output.txt").read_text() for k in range(n)]
                    found, res, _, _ = oc.guided(tr, lens, ev, num_procs=n, cache_size=cs)
                    assert found and [oc.dump_node(res, k, cs) for k in range(n)] == dumps, seed
                    refutes = []
                    for k, L in list(muts.items()):
                        f, r, _, complete = oc.guided(tr, lens, ev, num_procs=n, cache_size=cs, L=L)
                        if (not f and complete) or (f and [oc.dump_node(r, q, cs, L=L) for q in range(n)] != dumps):
                            refutes.append(f"m{k}")
                            del muts[k]
                    if refutes:
                        cases.append({"seed": seed, "num_procs": n, "cache_size": cs,
                                      "trace": [[instr_text(w) for w in r] for r in rows],
                                      "log": [" ".join(ev_token(e) for e in evt) for evt in ev],
                                      "dumps": dumps, "refutes": refutes})
                        print(n, "seed", seed, "refutes", refutes, flush=True)
        assert not muts, f"{n} nodes: mutants not refuted: {sorted(muts)}"
        (HERE / "ref_logs").mkdir(exist_ok=True)
        (HERE / "ref_logs" / f"pin{n}.json").write_text(json.dumps(
            {"source": f"tests/golden/make_ref_logs.py (oracle/_ref/cache_simulator_pin{'' if n == 4 else n}_cs{{1,4}})",
             "cases": cases}, indent=0) + "\n")


if __name__ == "__main__":
    main()
