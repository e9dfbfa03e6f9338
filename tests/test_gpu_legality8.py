"""The HIP path itself against the complete legal outcome sets at 8 nodes (-m gpu).

tests/ref_pin.py's 8-node systems (2-4 active nodes, homes among all 8, conflicting cache
indices) whose exploration completes: the oracle's explorer (orc_explore, pinned against the
reference binary by tests/test_reference_cross_node.py) enumerates every legal final state,
and the engine's outcome under lockstep and under eight seeded legal schedules,
dumped by printProcessorState (ref :853-905) from the device state, must be one of them.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import oracle_ctypes as oc
import ref_pin

pytestmark = pytest.mark.gpu
N = 8
TRACES = 128
SEEDS = [0, 1, 2, 3, 5, 8, 13, 21, 87]


def complete_cases():
    def one(seed):
        cs, rows = ref_pin.gen_trace(seed, N)
        tr, lens = ref_pin.as_arrays(rows)
        outs, _, complete = oc.explore(tr, lens, num_procs=N, cache_size=cs, max_states=ref_pin.MAX_STATES,
                                       micro=oc.MICRO_STRICT)
        legal = {tuple(oc.dump_node(o, k, cs) for k in range(N)) for o in outs} if complete else None
        return cs, tr, lens, legal
    with ThreadPoolExecutor(8) as pool:
        cases = [c for c in pool.map(one, range(2 * TRACES)) if c[3] is not None]
    return cases[:TRACES]


def test_engine_outcomes_are_legal_at_eight_nodes(dash):
    cases = complete_cases()
    assert len(cases) == TRACES
    L = max(c[1].shape[1] for c in cases)
    checked = 0
    for cs in (1, 4):
        group = [c for c in cases if c[0] == cs]
        packed = np.zeros((len(group), N, L), np.uint16)
        lens = np.zeros((len(group), N), np.uint32)
        for i, (_, tr, ln, _) in enumerate(group):
            packed[i, :, :tr.shape[1]] = tr
            lens[i] = ln
        for seed in SEEDS:
            with dash.Engine(len(group), num_procs=N, cache_size=cs, max_instr=L, keep_state=True,
                             schedule_seed=seed) as eng:
                eng.load_traces(packed, lens)
                eng.run()
                for i, case in enumerate(group):
                    st = eng.read_state(i)
                    got = tuple(dash.dump_node(st[k], k, cs) for k in range(N))
                    assert got in case[3], (cs, seed, i)
                    checked += 1
    assert checked == TRACES * len(SEEDS)
