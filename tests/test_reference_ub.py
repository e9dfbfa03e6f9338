"""The reference's undefined send, pinned on the reference itself, on the CPU.

tests/golden/ref_runs/ub{4,8}.json (make_ref_ub.py) holds 40 runs per node count of the reference
pin binary (assignment.c + oracle/patch_ref.py, DEBUG_MSG / DEBUG_INSTR) in which a thread evicted
a never-filled 0xFF line -- promoted to EXCLUSIVE by a stale EVICT_SHARED without an address check
(ref :558) -- and so sent EVICT_SHARED to node 15, out of bounds of messageBuffers (ref :772,786,
:751). The binary's receiver guard drops that send, and its stderr says so. Here the oracle
re-executes the interleaving it recovered from each run's logs: it must run to quiescence, drop and
flag that send (DASH_ERR_OOB, the engine's defined rule) and end in the reference's
dumps. tests/test_gpu_parity.py re-enacts the same runs on the GPU engine."""
import json
import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tests"))
import oracle_ctypes as oc  # noqa: E402
import ref_pin  # noqa: E402


@pytest.mark.parametrize("n", [4, 8])
def test_ub_runs_replay_to_the_reference_dumps(n):
    data = json.loads((ROOT / "tests" / "golden" / "ref_runs" / f"ub{n}.json").read_text())
    k = 0
    for (c, cs, tr, lens, _, steps) in ref_pin.micro_cases(n, "ub"):
        # the reference itself took the undefined send in this run (its guard's note, patch 5)
        assert any("to node 15" in ln for ln in c["ref_stderr"]), c["seed"]
        rep, term = oc.replay_steps(tr, lens, steps, num_procs=n, cache_size=cs)
        assert term, c["seed"]
        assert rep.errors & oc.ERR_OOB and not rep.errors & (oc.ERR_DEADLOCK | oc.ERR_ROUNDCAP), c["seed"]
        assert f"{rep.digest:016x}" == c["digest"], c["seed"]
        k += 1
    assert k == len(data["cases"]) == 40
    assert {c["cache_size"] for c in data["cases"]} == {1, 4}


@pytest.mark.parametrize("n,cs,kind,loc", [(8, 4, 0, 0), (8, 16, 2, 0), (4, 1, 1, 0), (8, 2, 2, 49152)])
def test_ctz0_path_is_unreachable(n, cs, kind, loc):
    """an EM directory entry always holds exactly one sharer bit, so the reference's
    __builtin_ctz(0) (ref :209,451) cannot happen and DASH_ERR_CTZ0 is a defensive flag. The oracle
    over 20,000 random systems per configuration never raises it (while OOB does occur)."""
    r = oc.run_batch(0xC720, 0, 20000, num_procs=n, cache_size=cs, length=64, kind=kind,
                     locality=loc, threads=4)
    assert not (r["errors"] & oc.ERR_CTZ0).any()
