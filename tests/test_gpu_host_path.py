"""The host-buffer boundary as bench.py drives it (--host-traces): traces handed over from host
memory through dash_load_traces every step, unbatched and in batches on two handles driven
by two host threads (copies overlapped with runs). Batching must not change any result:
the per-type histograms of the same host traces are identical for B = 1, 4 and 8, and equal
the oracle's over the same traces."""
import json
import pathlib
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = pathlib.Path(__file__).resolve().parent.parent
ARGS = ["--host-traces", "--systems", "4096", "--len", "512", "--steps", "1", "--warmup", "1"]


def _run(batches):
    r = subprocess.run([sys.executable, str(ROOT / "bench.py")] + ARGS + ["--host-batches", str(batches)],
                       capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])


def test_batched_host_path_matches_unbatched():
    import numpy as np
    import bench
    from oracle_ctypes import run_system
    one = _run(1)
    # the oracle over the same host traces (bench.host_trace_batch, seed 0x5EED, one rank):
    # RD value bits are random there and must be ignored by both (ref :839)
    packed, lens = bench.host_trace_batch(0x5EED, 4096, 512)
    hist = np.zeros(13, dtype=np.int64)
    for s in range(packed.shape[0]):
        hist += np.array(list(run_system(packed[s], lens[s], num_procs=8, cache_size=4).hist), dtype=np.int64)
    assert one["hist_per_step"] == hist.tolist()
    assert sum(one["hist_per_step"]) > 0 and one["config"]["host_batches"] == 1
    assert one["value"] > 0 and one["h2d_GBps"] > 0
    for b in (4, 8):
        d = _run(b)
        assert d["config"]["host_batches"] == b
        assert d["hist_per_step"] == one["hist_per_step"], b
        assert len(d["load_s_steps"]) == b and len(d["kernel_ms_steps"]) == b


@pytest.mark.parametrize("N,batches", [(8, 1), (8, 4), (8, 8), (4, 2), (5, 3)])
def test_run_host_batched_matches_single_run(dash, N, batches):
    """dash_run_host_batched (two handles, two host threads, copies overlapped with runs)
    gives exactly the per-system results and merged statistics of one dash_load_traces +
    dash_run over all systems (N = 5 takes the host re-layout path)."""
    import numpy as np
    from test_gpu_parity import random_batch
    rng = np.random.default_rng(77 + N * 10 + batches)
    packed, lens = random_batch(rng, 96 * batches, N, 120, hot_frac=0.2)
    st, d, r, e = dash.run_host_batched(packed, lens, batches, num_procs=N, cache_size=4)
    with dash.Engine(packed.shape[0], num_procs=N, cache_size=4, max_instr=packed.shape[2]) as eng:
        eng.load_traces(packed, lens)
        st1 = eng.run()
        d1, r1, e1 = eng.read_results()
    assert np.array_equal(d, d1) and np.array_equal(r, r1) and np.array_equal(e, e1)
    from oracle_ctypes import run_system
    for s in range(packed.shape[0]):  # and the oracle, system by system
        o = run_system(packed[s], lens[s], num_procs=N, cache_size=4)
        assert (int(d[s]), int(r[s]), int(e[s])) == (o.digest, o.rounds, o.errors), s
    for k in ("hist", "instructions", "rounds_total", "rounds_max", "systems", "err_systems", "err_bits",
              "dropped", "max_depth"):
        assert st[k] == st1[k], k
    assert st["instructions"] == int(lens.sum())


def test_run_host_batched_error_stops_and_reports(dash):
    """A failing batch (a trace longer than the handles' max_instr) stops both threads and
    its message reaches the caller through dash_last_error(NULL)."""
    import numpy as np
    from test_gpu_parity import random_batch
    rng = np.random.default_rng(5)
    packed, lens = random_batch(rng, 64, 8, 32, fixed_len=True)
    lens[40, 3] = 33  # batch 2 of 4: longer than the stride
    with pytest.raises(dash.DashError) as ei:
        dash.run_host_batched(packed, lens, 4, num_procs=8, cache_size=4)
    assert ei.value.code == dash.EINVAL and "longer" in str(ei.value)
