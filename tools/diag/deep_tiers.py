# diagnostic (tools/ only): the deep-queue batch of test_queue_depth_tiers through one library
# (DASH_LIB=tools/variants/libdash_X.so): tier hand-offs and per-system parity with the oracle
import os, sys, pathlib
import numpy as np
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "tests")); sys.path.insert(0, str(ROOT))
import oracle_ctypes as oc
import __graft_entry__ as g
dash = g.load_package()
ids = [16, 67, 105, 199, 230, 236, 285, 309, 332, 0, 1, 2, 3, 4, 5, 6]
L = 4096
packed = np.stack([oc.gen_system(0x5EED, s, 8, L, kind=1) for s in ids])
lens = np.full((len(ids), 8), L, np.uint32)
with dash.Engine(len(ids), num_procs=8, cache_size=4, max_instr=L, keep_state=True) as eng:
    eng.load_traces(packed, lens)
    st = eng.run()
    dig, rnd, err = eng.read_results()
print("tiers", st["tier_systems"], "max_depth", st["max_depth"])
for i, s in enumerate(ids):
    r = oc.run_system(packed[i], lens[i], num_procs=8, cache_size=4, ring_depth=256)
    print(i, s, "ok" if int(dig[i]) == r.digest else "DIFF", "rounds", int(rnd[i]), r.rounds, "err", int(err[i]), r.errors, "depth", r.max_depth)
