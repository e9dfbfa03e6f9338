# diagnostic (tools/ only): system 105 (queue depth 17) alone and beside deep neighbours in one wave;
# caught the cross-system leak of the rejected EMPTY13 variant
import sys, pathlib
import numpy as np
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "tests")); sys.path.insert(0, str(ROOT))
import oracle_ctypes as oc
import __graft_entry__ as g
dash = g.load_package()
L = 4096
for ids in ([105], [0, 105], [16, 105], [105, 16], [67, 105], [199, 105, 1, 2]):
    packed = np.stack([oc.gen_system(0x5EED, s, 8, L, kind=1) for s in ids])
    lens = np.full((len(ids), 8), L, np.uint32)
    with dash.Engine(len(ids), num_procs=8, cache_size=4, max_instr=L, keep_state=True) as eng:
        eng.load_traces(packed, lens)
        st = eng.run()
        dig, rnd, err = eng.read_results()
    out = []
    for i, s in enumerate(ids):
        r = oc.run_system(packed[i], lens[i], num_procs=8, cache_size=4, ring_depth=256)
        out.append(f"{s}:{'ok' if int(dig[i]) == r.digest else 'DIFF'}/{int(rnd[i])}")
    print(ids, "tiers", st["tier_systems"], " ".join(out))
