"""Differential fuzz of micro-step schedules (sim_kernel MODE 4) against the oracle's STRICT
micro-step model (test infrastructure: the oracle is the checker and the schedule source).

For each random system: one weighted random walk of the STRICT model (orc_random_walk: pops,
issues and single sends of the nodes in a random legal order, run to quiescence) gives an
interleaving and its final outcome; the engine, driven by the same interleaving through
dash_set_micro_schedule, must end in the same state (digest) with every instruction issued and
log one event per pop and per issue, in each node's order of the walk. Walks in which a queue of
the micro-step model overflowed (it holds 40 messages; the reference and the engine 256) are
skipped and counted: there the model, not the reference, drops the message."""
import numpy as np

import oracle_ctypes as oc

XK_POP, XK_ISSUE, XK_SEND = 0, 1, 2
ORC_ERR_OVERFLOW = 1  # oracle/dash_oracle.h: a queue of the micro-step model (XQ = 40 messages) overflowed


def acts_of(steps, n):
    acts = np.full((len(steps), n), 0xFF, np.uint8)
    for r, s in enumerate(steps):
        acts[r, s & 15] = 1 if (s >> 8) == XK_SEND else 0
    return acts


def one_config(dash, rng, N, CS, nsys, maxlen, random_batch):
    packed, lens = random_batch(rng, nsys, N, maxlen, block_span=int(rng.choice([2, 4, 16])),
                                hot_frac=float(rng.choice([0.0, 0.5])))
    bad, skipped = [], []
    for s in range(nsys):
        w = rng.integers(1, 16, size=N)
        out, steps = oc.random_walk(packed[s], lens[s], int(rng.integers(1, 1 << 62)), weights=w, num_procs=N,
                                    cache_size=CS)
        if out.errors & ORC_ERR_OVERFLOW:  # the explorer's queues hold 40 messages, the reference's 256
            skipped.append(s)
            continue
        acts = acts_of(steps, N)
        rounds = max(len(steps), 1)
        with dash.Engine(1, num_procs=N, cache_size=CS, max_instr=packed.shape[2], trace_events=rounds + 8,
                         schedule_seed=1, max_rounds=rounds + 64) as eng:
            eng.set_micro_schedule(acts)
            eng.load_traces(packed[s:s + 1], lens[s:s + 1])
            st = eng.run()
            dig = int(eng.read_results()[0][0])
            ev = eng.read_events(0)
        # each node's events in the walk's order: one per pop / issue step of that node
        per_node = [[] for _ in range(N)]
        for x in steps:
            if (x >> 8) in (XK_POP, XK_ISSUE):
                per_node[x & 15].append((x >> 8) == XK_ISSUE)
        got = [[] for _ in range(N)]
        for e in ev:
            got[e.node].append(e.kind == dash.EV_INSTR)
        ok = (dig == out.digest and st["instructions"] == int(lens[s].sum()) and got == per_node
              and not st["err_bits"] & (dash.ERR_ROUNDCAP | dash.ERR_DEADLOCK))
        if not ok:
            bad.append({"system": s, "digest_equal": dig == out.digest, "err_bits": st["err_bits"],
                        "instructions": st["instructions"], "expected_instructions": int(lens[s].sum()),
                        "events_equal": got == per_node, "steps": len(steps)})
    return bad, skipped
