"""`bench.py --next`: the SURVEY.md §8(f) rows around the hot path, measured on one GPU, each
with a size-independent parity property checked in the same run. One JSON line:

* ingest    -- trace-directory ingest at scale (`dash_load_dirs`: `initializeProcessor`'s
               `core_<n>.txt` format, ref :806-851, parsed on host threads into the packed
               layout, then one H2D copy). Parity: the run from text equals the run of the same
               traces handed over as packed words (`dash_load_traces`), digest for digest.
               Beside it: the single-thread rate of `dash_parse_core_file` (the C restatement
               of the reference's fgets/sscanf parser) on a sample of the same files.
* digests   -- `dash_write_digests` for every system, `dash_dump_system` (`printProcessorState`
               text, ref :853-905) for a sample. Parity: the digest file lists the digests that
               `dash_read_results` returns.
* events    -- DEBUG_MSG / DEBUG_INSTR emission (ref :179-182, :649-652): the SLOW kernel with
               the event log against the fast kernel on the same systems. Parity: every system
               logs exactly one event per issued instruction and per popped message, and its
               digests equal the fast kernel's (the log does not change the run).
* seeded    -- seeded legal schedules on the headline workload (1M systems x 8
               x 4096 uniform, generated on the device): the SLOW kernel's instr/s against the
               lockstep kernel's. Parity: every instruction issues, and a second run with the
               same seed reproduces every digest (checksum of all 2^20 digests).

Inputs are synthetic: numpy's PCG64 raw bits for the text traces (like --host-traces), the
device generator for the seeded workload. Nothing here touches oracle/.
"""
import json
import pathlib
import tempfile
import time

import numpy as np

HEX = np.frombuffer(b"0123456789ABCDEF", dtype=np.uint8)


def trace_text(words):
    """core_<n>.txt bytes for one node's packed u16 words: "WR 0xAA V" / "RD 0xAA" lines, the
    address as two hex digits and the value in decimal, as in the reference's tests."""
    w = words.astype(np.uint32)
    wr = (w >> 15) & 1
    addr = (w >> 8) & 0x7F
    val = w & 0xFF
    n = len(w)
    rows = np.full((n, 12), ord("\n"), dtype=np.uint8)
    rows[:, 0] = np.where(wr == 1, ord("W"), ord("R"))
    rows[:, 1] = np.where(wr == 1, ord("R"), ord("D"))
    rows[:, 2] = ord(" ")
    rows[:, 3] = ord("0")
    rows[:, 4] = ord("x")
    rows[:, 5] = HEX[addr >> 4]
    rows[:, 6] = HEX[addr & 15]
    nd = 1 + (val >= 10) + (val >= 100)
    d = [val // 100, (val // 10) % 10, val % 10]
    for k in range(3):  # digit k of the value (most significant first) sits at column 8 + k - (3 - nd)
        col = 8 + k - (3 - nd)
        ok = (wr == 1) & (col >= 8)
        rows[ok, col[ok]] = ord("0") + d[k][ok]
    rows[:, 7] = np.where(wr == 1, ord(" "), ord("\n"))
    length = np.where(wr == 1, 9 + nd, 8)
    return rows[np.arange(12)[None, :] < length[:, None]].tobytes()


def write_dirs(root, packed):
    dirs = []
    for s in range(packed.shape[0]):
        d = pathlib.Path(root, f"s{s}")
        d.mkdir()
        for n in range(packed.shape[1]):
            (d / f"core_{n}.txt").write_bytes(trace_text(packed[s, n]))
        dirs.append(d)
    return dirs


def ingest_rows(dash, dev, seed, systems, L, workdir):
    rng = np.random.default_rng(seed)
    packed = rng.bit_generator.random_raw(systems * 8 * L // 4).view(np.uint16).reshape(systems, 8, L).copy()
    lens = np.full((systems, 8), L, dtype=np.uint32)
    t0 = time.perf_counter()
    dirs = write_dirs(workdir, packed)
    t_write = time.perf_counter() - t0
    text_bytes = sum(f.stat().st_size for d in dirs for f in d.iterdir())
    out = {}
    with dash.Engine(systems, num_procs=8, cache_size=4, max_instr=L, keep_state=True, device=dev) as eng:
        eng.load_dirs(dirs)  # warm: page cache, host threads, device buffers
        t0 = time.perf_counter()
        eng.load_dirs(dirs)
        t_ingest = time.perf_counter() - t0
        st = eng.run()
        dig_text, rnd_text, err_text = eng.read_results()
        # bulk digests and dumps
        dpath = pathlib.Path(workdir, "digests.txt")
        t0 = time.perf_counter()
        eng.write_digests(dpath)
        t_dig = time.perf_counter() - t0
        listed = np.array([int(line.split()[1], 16) for line in dpath.read_text().splitlines()], dtype=np.uint64)
        K = min(64, systems)
        pathlib.Path(workdir, "dump").mkdir()
        t0 = time.perf_counter()
        for k in range(K):
            eng.dump_system(k, pathlib.Path(workdir, "dump", str(k)))
        t_dump = time.perf_counter() - t0
        dump_bytes = sum(f.stat().st_size for f in pathlib.Path(workdir, "dump").rglob("*.txt"))
    with dash.Engine(systems, num_procs=8, cache_size=4, max_instr=L, device=dev) as eng:
        eng.load_traces(packed, lens)
        eng.run()
        dig_bin, rnd_bin, err_bin = eng.read_results()
    # single-thread parser rate (the reference's initializeProcessor restated in C)
    sample = [d / f"core_{n}.txt" for d in dirs[:32] for n in range(8)]
    t0 = time.perf_counter()
    for f in sample:
        dash.parse_core_file(f, num_procs=8, max_instr=L)
    t_parse1 = time.perf_counter() - t0
    lines = systems * 8 * L
    out["ingest"] = {
        "workload": f"{systems} trace directories x 8 core_<n>.txt x {L} lines ({text_bytes / 1e6:.0f} MB of text)",
        "seconds": t_ingest, "lines_per_s": lines / t_ingest, "MB_per_s": text_bytes / t_ingest / 1e6,
        "host_threads": "min(16, hardware_concurrency)",
        "single_thread_parse": {"lines_per_s": len(sample) * L / t_parse1, "files": len(sample),
                                "kind": "port (dash_parse_core_file, the reference's fgets + sscanf rules)"},
        "write_seconds": t_write,
        "run_kernel_ms": st["kernel_ms"],
        "parity_text_equals_packed": bool(np.array_equal(dig_text, dig_bin) and np.array_equal(rnd_text, rnd_bin)
                                          and np.array_equal(err_text, err_bin)),
    }
    out["digests"] = {
        "systems": systems, "write_digests_seconds": t_dig, "systems_per_s": systems / t_dig,
        "dump_systems": K, "dump_seconds": t_dump, "dump_ms_per_system": t_dump / K * 1e3,
        "dump_bytes": dump_bytes,
        "parity_file_equals_results": bool(np.array_equal(listed, dig_text)),
    }
    return out, packed, lens


def events_row(dash, dev, seed, systems, L):
    E = 8 * L  # log capacity in rounds: > the rounds of these runs (about 5.5 L)
    with dash.Engine(systems, num_procs=8, cache_size=4, max_instr=L, device=dev) as eng:
        eng.generate(seed, L, kind=dash.GEN_UNIFORM)
        eng.run()
        fast = eng.run()
        dig_fast = eng.read_results()[0]
    with dash.Engine(systems, num_procs=8, cache_size=4, max_instr=L, device=dev, trace_events=E,
                     keep_state=True) as eng:
        eng.generate(seed, L, kind=dash.GEN_UNIFORM)
        eng.run()
        slow = eng.run()
        dig_slow = eng.read_results()[0]
        per_sys_ok = True
        for s in range(min(8, systems)):  # one event per issued instruction and per popped message
            ev = eng.read_events(s)
            per_sys_ok &= len(ev) == 8 * L + int(eng.read_hist(s).sum())
    events = slow["instructions"] + sum(slow["hist"])
    return {
        "workload": f"{systems} systems x 8 nodes x {L} uniform (device generator), event log {E} rounds",
        "events": events, "kernel_ms": slow["kernel_ms"], "events_per_s": events / (slow["kernel_ms"] / 1e3),
        "fast_kernel_ms": fast["kernel_ms"], "slowdown": slow["kernel_ms"] / fast["kernel_ms"],
        "parity_same_digests_as_fast": bool(np.array_equal(dig_fast, dig_slow)),
        "parity_events_logged": bool(per_sys_ok and slow["err_bits"] == fast["err_bits"]),
    }


def seeded_row(dash, dev, seed, systems, L, steps):
    out = {}
    digs = []
    for name, sched in (("lockstep", 0), ("seeded", 0x5EED5EED), ("seeded_again", 0x5EED5EED)):
        with dash.Engine(systems, num_procs=8, cache_size=4, max_instr=L, device=dev, schedule_seed=sched) as eng:
            eng.generate(seed, L, kind=dash.GEN_UNIFORM)
            eng.run()
            t0 = time.perf_counter()
            ks = []
            for _ in range(steps):
                st = eng.run()
                ks.append(st["kernel_ms"])
            el = time.perf_counter() - t0
            d = eng.read_results()[0]
            digs.append((int((d & np.uint64(0xFFFFFFFF)).sum(dtype=np.uint64)), int((d >> np.uint64(32)).sum(dtype=np.uint64))))
            out[name] = {"instr_per_s": st["instructions"] * steps / el, "ms_per_step": el / steps * 1e3,
                         "kernel_ms": ks, "instructions": st["instructions"], "rounds_total": st["rounds_total"],
                         "err_systems": st["err_systems"], "tier_systems": st["tier_systems"],
                         "wave_rounds": st["wave_rounds"]}
    out["workload"] = f"{systems} systems x 8 nodes x {L} uniform (device generator, seed 0x{seed:X}), schedule seed 0x5EED5EED"
    out["slowdown"] = out["lockstep"]["instr_per_s"] / out["seeded"]["instr_per_s"]
    # the slowdown split: rounds the schedule needs, and kernel time per wave-round
    out["rounds_ratio"] = out["seeded"]["rounds_total"] / out["lockstep"]["rounds_total"]
    out["time_per_wave_round_ratio"] = ((sum(out["seeded"]["kernel_ms"]) / out["seeded"]["wave_rounds"])
                                        / (sum(out["lockstep"]["kernel_ms"]) / out["lockstep"]["wave_rounds"]))
    out["parity_all_issued"] = out["seeded"]["instructions"] == systems * 8 * L
    out["parity_reproducible"] = digs[1] == digs[2]
    out["differs_from_lockstep"] = digs[0] != digs[1]
    del out["seeded_again"]
    return out


def digests_at_scale(dash, dev, seed, systems, td):
    """dash_write_digests for a headline-sized batch (every system's digest, rounds and error
    word as text: parity at 1M systems without 19 GB of dumps). Short traces:
    the row times the emitter, not the simulation."""
    L = 64
    with dash.Engine(systems, num_procs=8, cache_size=4, max_instr=L, device=dev) as eng:
        eng.generate(seed, L, kind=dash.GEN_UNIFORM)
        eng.run()
        dig, rnd, err = eng.read_results()
        path = pathlib.Path(td, "digests_1m.txt")
        t0 = time.perf_counter()
        eng.write_digests(path)
        t = time.perf_counter() - t0
    text = path.read_bytes()
    lines = text.split(b"\n")[:-1]
    sample = range(0, systems, max(systems // 4096, 1))
    ok = len(lines) == systems and all(
        lines[k] == f"{k} {int(dig[k]):016x} {int(rnd[k])} {int(err[k]):x}".encode() for k in sample)
    return {"systems": systems, "seconds": t, "systems_per_s": systems / t, "bytes": len(text),
            "parity_lines_equal_results": bool(ok)}


def run(dash, dev, args):
    L = min(args.len, 4096)
    with tempfile.TemporaryDirectory(dir=args.next_dir) as td:
        res, packed, lens = ingest_rows(dash, dev, args.seed, args.next_systems, L, td)
        res["digests"]["at_scale"] = digests_at_scale(dash, dev, args.seed, args.systems, td)
    res["events"] = events_row(dash, dev, args.seed, args.next_event_systems, L)
    res["seeded"] = seeded_row(dash, dev, args.seed, args.systems, args.len, max(args.steps, 1))
    line = {"metric": "SURVEY.md 8(f) rows beside the hot path (ingest, digests/dumps, DEBUG events, seeded schedules)",
            "n_gpus": 1, "data": "synthetic", "rows": res}
    print(json.dumps(line), flush=True)
