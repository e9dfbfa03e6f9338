"""Generate tests/golden/ref_runs/ub{4,8}.json: reference runs that took the reference's
undefined send -- the eviction of a never-filled 0xFF line, which messageBuffers[15] receives
out of bounds (assignment.c:772,786 into :751) -- so the engine's defined drop-and-flag rule
 is pinned on the reference itself, not only on the oracle.

TEST INFRASTRUCTURE. The reference pin binaries (oracle/_ref/cache_simulator_pin{,8}_cs{1,4}:
assignment.c + oracle/patch_ref.py, whose receiver guard (patch 3) drops exactly that send and,
since round 6, notes it on stderr (patch 5): "bench: dropped 11 to node 15" / "... 12 ...") run
short random systems that the oracle's lockstep run flags DASH_ERR_OOB (the counter-based
generator, 16 instructions per node, uniform addresses, seed 0x5EED). A run is kept only when
its own stderr shows the drop. As in make_ref_micro.py, the oracle's log-guided search
(orc_guided_witness, STRICT model) recovers an interleaving of the reference's threads that meets
every thread's DEBUG_MSG / DEBUG_INSTR log, checked by re-executing it (orc_replay_steps: the
outcome is the reference's dumps, and the replay itself drops and flags the send); a case holds
the trace, that interleaving ("P<t>" / "I<t>" / "D<t>" tokens), each thread's log, the digest of
the reference's dumps and the reference's stderr notes.

Run: python tests/golden/make_ref_ub.py   (seconds)
"""
import json
import pathlib
import subprocess
import sys
import tempfile

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
import oracle_ctypes as oc  # noqa: E402
import ref_pin  # noqa: E402

RUNS = 40        # kept runs per node count
TRIES = 6        # reference runs per candidate trace until one takes the undefined send
LEN = 16
SEED = 0x5EED


def cases_for(n):
    cases, tried = [], 0
    for cs in (4, 1):
        # CACHE_SIZE 1 rarely leaves a 0xFF line to promote: scan more systems for it
        r = oc.run_batch(SEED, 0, 50000 if cs == 4 else 1 << 20, num_procs=n, cache_size=cs, length=LEN, kind=0,
                         threads=4)
        cand = [int(i) for i in np.nonzero(r["errors"] & oc.ERR_OOB)[0]]
        for sid in cand:
            if len(cases) >= (RUNS // 2 if cs == 4 else RUNS):
                break
            tried += 1
            tr = oc.gen_system(SEED, sid, num_procs=n, length=LEN, kind=0)
            lens = np.full(n, LEN, np.uint32)
            rows = [[int(w) for w in tr[k]] for k in range(n)]
            with tempfile.TemporaryDirectory() as td:
                d = pathlib.Path(td)
                ref_pin.write_trace(d / "tests" / "t", rows)
                for _ in range(TRIES):
                    p = subprocess.run(["timeout", "20", str(ref_pin.pin_exe(cs, n)), "t"], cwd=d,
                                       capture_output=True, text=True)
                    if p.returncode == 0 and "to node 15" in p.stderr:
                        break
                else:
                    continue
                dumps = [(d / f"core_{k}_output.txt").read_text() for k in range(n)]
            ev, _ = oc.parse_logs(p.stdout, n)
            found, out, steps = oc.guided_witness(tr, lens, ev, num_procs=n, cache_size=cs)
            digest = oc.dumps_digest(dumps, cs)
            assert found and out.digest == digest, (n, cs, sid)
            rep, term = oc.replay_steps(tr, lens, steps, num_procs=n, cache_size=cs)
            assert term and rep.digest == digest and rep.errors & oc.ERR_OOB, (n, cs, sid)
            cases.append({"seed": sid, "system": sid, "num_procs": n, "cache_size": cs,
                          "trace": [[f"WR 0x{(w >> 8) & 0x7F:02X} {w & 0xFF}" if w & 0x8000
                                     else f"RD 0x{(w >> 8) & 0x7F:02X}" for w in row] for row in rows],
                          "steps": " ".join("PID"[int(x) >> 8] + str(int(x) & 15) for x in steps),
                          "log": ref_pin.log_tokens(p.stdout, n), "digest": f"{digest:016x}",
                          "ref_stderr": [ln for ln in p.stderr.splitlines() if ln.startswith("bench:")],
                          "oracle_errors": int(rep.errors)})
    return cases, tried


def main():
    for n in (4, 8):
        cases, tried = cases_for(n)
        (HERE / "ref_runs" / f"ub{n}.json").write_text(json.dumps(
            {"source": f"tests/golden/make_ref_ub.py (oracle/_ref/cache_simulator_pin{'' if n == 4 else n}_cs{{1,4}}, "
                       f"seed 0x{SEED:X}, {LEN} instructions per node)",
             "tried_traces": tried, "cases": cases}, separators=(",", ":")) + "\n")
        print(n, "nodes:", len(cases), "runs through the undefined send kept of", tried, "traces")


if __name__ == "__main__":
    main()
