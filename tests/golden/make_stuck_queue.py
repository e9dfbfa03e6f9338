"""How tests/golden/stuck_queue.npy was found (kept for provenance; the .npy is the fixture).

Hill-climbing on the oracle's max queue depth: 8 nodes, CACHE_SIZE 1, instructions drawn as
60 % WR, the home node 0 w.p. 0.7 (else uniform), blocks 0..3; a candidate mutates 1..39
random instructions and is kept when the depth does not drop. The fixture came from three
climbs of 240 s each (seeds 2, 3 at 2048 instructions per node, then seed 4 after doubling
the best trace to 4096), which raised the depth 168 -> 171 -> 256 = MSG_BUFFER_SIZE (ref
:9): the queue fills, the reference's drain loop (:167-170) stops for good (head == tail)
and DASH_ERR_STUCK is set. Usage: python make_stuck_queue.py SEED [START.npy] [SECONDS].
"""
import pathlib
import sys
import time

import numpy as np

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parents[1]))
import oracle_ctypes as oc  # noqa: E402

N, CS = 8, 1


def main():
    seed = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    start = sys.argv[2] if len(sys.argv) > 2 else None
    budget = float(sys.argv[3]) if len(sys.argv) > 3 else 240.0
    rng = np.random.default_rng(seed)

    def rand_instr():
        node = int(rng.integers(N)) if rng.random() < 0.3 else 0
        w = int(rng.random() < 0.6)
        return (w << 15) | (((node << 4) | int(rng.integers(4))) << 8) | (int(rng.integers(256)) if w else 0)

    tr = np.load(start) if start else np.array([[rand_instr() for _ in range(2048)] for _ in range(N)], np.uint16)
    L = tr.shape[1]
    lens = np.full(N, L, np.uint32)

    def depth(t):
        return oc.run_system(t, lens, num_procs=N, cache_size=CS, ring_depth=256).max_depth

    best, t0 = depth(tr), time.time()
    while time.time() - t0 < budget and best < 256:
        cand = tr.copy()
        for _ in range(int(rng.integers(1, 40))):
            cand[rng.integers(N), rng.integers(L)] = rand_instr()
        d = depth(cand)
        if d >= best:
            if d > best:
                print(f"{time.time() - t0:.0f} s: depth {d}", flush=True)
            best, tr = d, cand
    np.save(f"stuck_queue_seed{seed}.npy", tr)
    print("depth", best)


if __name__ == "__main__":
    main()
