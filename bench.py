#!/usr/bin/env python3
"""Headline benchmark: simulated instructions/second of 8-node DASH systems.

Workload (BASELINE.json configs[2], the `metric`'s configuration): 1M (2^20)
independent 8-node systems per GPU, 4096 uniform-random RD/WR per node,
CACHE_SIZE 4. Traces are generated on the device (counter-based, seed keyed
by the GLOBAL system id) before the timed region, so they are resident in
HBM (64 GiB per GPU). One step = one full pass of the hot path: every system
from initial state to quiescence.

Multi-GPU: one process per GPU. `bench.py --gpus N` starts the N ranks itself (a parent
that never touches the GPU spawns N fresh child processes with RANK / LOCAL_RANK /
WORLD_SIZE set); under torchrun the ranks come from the environment and WORLD_SIZE must
equal --gpus. Systems are sharded by global id with no data-path collective (weak
scaling); the single exchange is one RCCL all-reduce of the per-transaction histograms
after the timed region.

The headline line also carries `contention` (BASELINE configs[3], its own timed steps),
`cpu_baseline` (the reference itself, assignment.c + the SURVEY §8(d) benchmark patch,
one instance per host core = BASELINE.md mode (A)) and `cpu_port` (the oracle restatement
on the same host). Every line certifies its own results at any GPU count (`golden`, round 6):
each rank compares its own pre-reduce totals with the full-size golden of its slice where one is
committed (rank 0's slice always: tests/golden/full_size.json, sweep_full.json; slices 1..7:
full_slices.json) and its systems among the sampled ids of tests/golden/rank_samples.json with the
oracle's per-system results; the counts ride in the one all-reduce. These are
fixture files, not the oracle.

Prints ONE JSON line on rank 0 (contract in the task statement), at most LINE_BUDGET (4 KB)
long: the driver keeps only a ~10 KB tail of stdout + stderr, and round 4's 52-KB line was
unreadable to it. The full record (per-point histograms, kernel times, CPU-baseline
samples, box sysfs, next rows) goes to the side file named by the line's `detail` (--detail);
the line itself is `compact_headline()` of that record. Stderr stays quiet: one progress line
per sweep CACHE_SIZE.

Other modes (not the headline): --kind contention (configs[3]); --sweep (configs[4]);
--host-traces [--host-batches B] [--host-native]: traces handed over from host memory every
step (PCIe-inclusive rate of the drop-in boundary); --next: the SURVEY §8(f)
rows beside the hot path (text ingest, digests / dumps, DEBUG event log, seeded schedules),
each with a parity property (bench_next.py); --process-group: run the collectives as a
one-rank group (the RCCL path on a 1-GPU box); --cpu-kind port: the oracle restatement as
the CPU baseline instead of the reference binary.
"""
import argparse
import json
import math
import os
import pathlib
import sys
import time

ROOT = pathlib.Path(__file__).resolve().parent
DETAIL_DEFAULT = ROOT / "gpurun_out" / "bench_detail.json"
LINE_BUDGET = 4096  # bytes of the printed line
PEAK_HBM = 8.0e12  # B/s, MI355X_MICROARCH.md chip table
BYTES_PER_INSTR = 2  # packed trace record read once
# VALU issue ceiling for this kernel's instruction forms (v_cndmask_e64, v_cmp_e64, v_bfe,
# v_or3, v_lshl_or, ...): 1 wave64 instruction per cycle per CU (4 cycles per SIMD),
# measured by tools/micro (profiles/r01/micro); the SIMD-32 issue limit of plain VOP2
# forms in homogeneous streams is 2 per cycle per CU. 256 CUs x 2.4 GHz.
VALU_PEAK = 256 * 2.4e9
# architectural VALU issue limit (MI355X_MICROARCH.md "Wave scheduling": a wave64 VALU
# instruction occupies a SIMD-32 for 2 cycles, 4 SIMDs per CU): 2 per cycle per CU
VALU_PEAK_SIMD32 = 2 * VALU_PEAK


def host_cores():
    """CPUs this process may use: the cgroup CPU quota when one is set (the GPU box shows
    hundreds of CPUs but grants a 16-CPU share), else the affinity mask."""
    try:
        quota, period = pathlib.Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if quota != "max":
            return max(1, int(int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    return len(os.sched_getaffinity(0))


def cpu_model():
    try:
        for ln in pathlib.Path("/proc/cpuinfo").read_text().splitlines():
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def load_dash():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "dash_amd", ROOT / "ue22cs343bb1-openmp-assignment_amd" / "dash.py")
    mod = importlib.util.module_from_spec(spec)
    sys.modules["dash_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def cpu_baseline(args, seed, kind, locality, target_s):
    """The oracle (C port of the reference protocol, OpenMP over systems) on a
    bounded sample of the same workload, on this box's host cores."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_ctypes as oc
    threads = args.cpu_threads
    cal = oc.run_batch(seed, 0, max(threads, 8), num_procs=8, cache_size=args.cache_size,
                       length=args.len, kind=kind, locality=locality, threads=threads)
    rate = cal["instructions"] / max(cal["seconds"], 1e-9)
    per_sys = 8 * args.len
    count = int(max(threads, min(1 << 20, rate * target_s / per_sys)))
    res = oc.run_batch(seed, 0, count, num_procs=8, cache_size=args.cache_size, length=args.len,
                       kind=kind, locality=locality, threads=threads)
    return {"value": res["instructions"] / res["seconds"], "unit": "instr/s", "cores": threads,
            "host_cpus_visible": host_cpus_visible(), "kind": "port", "cpu_model": cpu_model(),
            "sample": f"{count} systems x 8 nodes x {args.len} instr ({args.kind}, CS={args.cache_size}, "
                      f"seed 0x{seed:X}) in {res['seconds']:.1f} s on {threads} threads; "
                      f"oracle/dash_oracle.c lockstep restatement of assignment.c"}


def host_cpus_visible():
    """Logical CPUs the machine exposes (the quota in host_cores() is what a job may use)."""
    return os.cpu_count() or 1


def ref_exe(cache_size):
    """oracle/_ref/cache_simulator_bench (CACHE_SIZE 4) or ..._cs<C> (oracle/patch_ref.py)."""
    name = "cache_simulator_bench" + ("" if cache_size == 4 else f"_cs{cache_size}")
    return ROOT / "oracle" / "_ref" / name


_TRACE_LINES = []


def trace_lines():
    """The reference's trace line (`RD XX` / `WR XX v`, ref :835-845) of every packed 16-bit record,
    as bytes, indexed by the record (an RD's value bits are ignored): a table lookup per instruction
    when bench.py writes the reference's input files (16-128 instances x 8 nodes x 4096 lines per leg)."""
    if not _TRACE_LINES:
        _TRACE_LINES.extend((f"WR {(w >> 8) & 0x7F:02X} {w & 0xFF}\n" if w & 0x8000 else
                             f"RD {(w >> 8) & 0x7F:02X}\n").encode() for w in range(1 << 16))
    return _TRACE_LINES


WRITEBACK_INV, WRITEBACK_INT = 7, 8  # message types whose receiver comes from __builtin_ctz (ref :209,451)
# causes that name the reference rule behind the stall; the others only describe its state
STALL_EXPLAINED = ("ctz0_send", "queue_full")
MSG_BUFFER_SIZE = 256  # ref :9


def snapshots(stderr_text):
    """The instance's SIGUSR1 snapshot lines (oracle/patch_ref.py patch 6), parsed: [{"done",
    "inflight", "queues": [(head, tail, count)] * NUM_PROCS}]."""
    out = []
    for ln in stderr_text.splitlines():
        if not ln.startswith("bench: snapshot "):
            continue
        f = ln.split()
        qs = [tuple(int(x) for x in tok.split(":")[1].split(",")) for tok in f[6:]]
        out.append({"done": int(f[3]), "inflight": int(f[5]), "queues": qs})
    return out


def stall_cause(stderr_text, num_procs=8):
    """Why a killed reference instance stalled, from its own stderr (oracle/patch_ref.py patches 5
    and 6). From its drop notes: "ctz0_send" = it dropped a WRITEBACK_INT / WRITEBACK_INV addressed
    to a node >= NUM_PROCS other than 15 -- the reference's __builtin_ctz(0) (tzcnt gives 32; ref
    :209,451), whose requester then waits forever; "queue_full" = a full queue dropped a message (ref
    :758-762; at 256 the drain loop's head != tail test never pops it again, ref :167-170). Else from
    its last snapshot (taken after a second without any queue moving): a queue at 256 is
    "queue_full"; every queue empty and nothing in flight while a thread is not done is
    "waits_with_nothing_in_flight" (a node waits for a reply no one will send); otherwise
    "stuck_with_messages" (and "no_snapshot" without one; "still_moving_at_timeout" for a slow
    instance killed only at --ref-timeout)."""
    cause = None
    for ln in stderr_text.splitlines():
        f = ln.split()
        if ln.startswith("bench: queue full"):
            return "queue_full"
        if ln.startswith("bench: dropped") and len(f) >= 6:
            t, r = int(f[2]), int(f[5])
            if t in (WRITEBACK_INV, WRITEBACK_INT) and r >= num_procs and r != 15:
                cause = "ctz0_send"
    if cause:
        return cause
    snap = snapshots(stderr_text)
    if not snap:
        return "no_snapshot"
    if len(snap) >= 2 and snap[-1] != snap[-2]:
        return "still_moving_at_timeout"  # slow, killed only at --ref-timeout
    last = snap[-1]
    if any(c >= MSG_BUFFER_SIZE for _, _, c in last["queues"]):
        return "queue_full"
    if last["inflight"] == 0 and all(c == 0 for _, _, c in last["queues"]) and last["done"] < num_procs:
        return "waits_with_nothing_in_flight"
    return "stuck_with_messages"


def still_moving(stderr_text):
    """True when the instance's last two snapshots differ (a queue moved between them)."""
    snap = snapshots(stderr_text)
    return len(snap) >= 2 and snap[-1] != snap[-2]


def probe_late(procs, late, dirs, gap=1.0):
    """Two SIGUSR1 snapshots `gap` s apart of each still-running instance in `late`; returns the
    ones whose queues moved in between (slow, not stalled)."""
    import signal
    for i in late:
        if procs[i].poll() is None:
            procs[i].send_signal(signal.SIGUSR1)
    time.sleep(gap)
    for i in late:
        if procs[i].poll() is None:
            procs[i].send_signal(signal.SIGUSR1)
    time.sleep(0.2)
    return [i for i in late if procs[i].poll() is None and still_moving((dirs[i] / "stderr.txt").read_text())]


def explain_stalls(stalls, seed, kind_id, locality, cache_size, length):
    """every killed instance with its system id and cause (stall_cause), and the
    oracle's lockstep verdict on that system (its error bits: DASH_ERR_CTZ0 = 4, DEADLOCK = 8 ...).
    `explained` counts the stalls whose own log shows a send that leaves a requester waiting forever
    (or a full queue)."""
    from collections import Counter
    if not stalls:
        return {"n": 0, "explained": 0}
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_ctypes as oc
    by_sys = Counter(i for i, _ in stalls)
    flags = {i: int(oc.run_batch(seed, i, 1, num_procs=8, cache_size=cache_size, length=length, kind=kind_id,
                                 locality=locality)["errors"][0]) for i in by_sys}
    return {"n": len(stalls), "explained": sum(c in STALL_EXPLAINED for _, c in stalls),
            "causes": dict(Counter(c for _, c in stalls)),
            # system id -> [times it stalled, the oracle's error bits for it under lockstep]
            "systems": {str(i): [n, flags[i]] for i, n in sorted(by_sys.items())},
            "oracle_ctz0": sum(n for i, n in by_sys.items() if flags[i] & ERR_CTZ0),
            "basis": "killed only after two SIGUSR1 snapshots a second apart showed no queue moving; cause from "
                     "the instance's own stderr (oracle/patch_ref.py patches 5, 6: drop notes, last snapshot); the "
                     "oracle runs the same system under the engine's lockstep schedule"}


def ref_baseline(args, seed, kind_id, target_s, instances=0, cache_size=4, locality=0, kind_name=None,
                 min_batches=1):
    """The reference itself (oracle/_ref/cache_simulator_bench[_cs<C>]: assignment.c with the
    benchmark patch of SURVEY.md §8(d), gcc -O2 -fopenmp, 8 spinning OpenMP threads per
    instance) on systems 0.. of the same synthetic workload, written as the reference's
    tests/<dir>/core_<n>.txt. `instances` processes run concurrently (0 = one per host core,
    BASELINE.md mode (A): the north star's "as many concurrent instances as host cores";
    1 = mode (B), one 8-thread instance); batches repeat until `target_s` has passed and at
    least `min_batches` ran."""
    import subprocess
    import tempfile
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_ctypes as oc
    exe = ref_exe(cache_size)
    if not exe.exists():
        raise RuntimeError(f"{exe.relative_to(ROOT)} missing (built by __graft_entry__.build() / "
                           f"oracle/build_ref.sh where /root/reference exists)")
    # mode (A) is one instance per host core, capped (--ref-max-instances): each instance spins 8
    # threads, and a large node's quota would otherwise start thousands of them at once
    k = instances or min(host_cores(), getattr(args, "ref_max_instances", 64))
    kind_name = kind_name or args.kind
    with tempfile.TemporaryDirectory() as td:
        dirs = []
        for i in range(k):
            d = pathlib.Path(td, f"i{i}")
            (d / "tests" / "b").mkdir(parents=True)
            tr = oc.gen_system(seed, i, num_procs=8, length=args.len, kind=kind_id, locality=locality)
            for n in range(8):
                (d / "tests" / "b" / f"core_{n}.txt").write_bytes(b"".join(map(trace_lines().__getitem__,
                                                                               tr[n].tolist())))
            dirs.append(d)
        # The reference can stall for good under some thread schedules (a queue that reaches 256 is
        # never drained again, ref :167-170). An instance still running well after the batch's
        # others finished (4x the slowest finisher, at least 5 s) is probed: two SIGUSR1 snapshots a
        # second apart (patch 6). If a queue moved it is slow, not stalled, and the batch waits on
        # (until --ref-timeout); if nothing moved it is killed and not counted -- instructions and
        # time are those of the instances that finished -- and its cause is read from its stderr.
        batches, hung, instr, elapsed, t0 = 0, 0, 0, 0.0, time.perf_counter()
        waited_slow = 0  # late instances found still moving and waited for
        rates = []  # per batch: finished instances' instructions / the batch's slowest finisher
        stalls = []  # per killed instance: (system id, cause from its own stderr)
        while True:
            errs = [open(d / "stderr.txt", "w") for d in dirs]
            procs = [subprocess.Popen([str(exe), "b"], cwd=d, stdout=subprocess.DEVNULL, stderr=f)
                     for d, f in zip(dirs, errs)]
            tb = last = time.perf_counter()
            fin = {}
            extend, slow_seen = 0.0, set()
            try:
                while len(fin) < k:
                    time.sleep(0.005)
                    now = time.perf_counter()
                    for i, p in enumerate(procs):
                        if i not in fin and p.poll() is not None:
                            if p.returncode != 0:
                                raise RuntimeError(f"reference instance exited with {p.returncode}")
                            fin[i] = now - tb
                    limit = max(5.0, 4 * max(fin.values())) if fin else args.ref_timeout
                    limit = max(limit, extend)
                    if len(fin) < k and now - tb > min(limit, args.ref_timeout):
                        late = [i for i in range(k) if i not in fin]
                        moving = probe_late(procs, late, dirs) if now - tb < args.ref_timeout else []
                        if moving:  # slow, not stalled: wait another `limit` seconds and look again
                            waited_slow += len(set(moving) - slow_seen)
                            slow_seen |= set(moving)
                            extend = time.perf_counter() - tb + max(5.0, 4 * max(fin.values()) if fin else 5.0)
                            continue
                        hung += sum(1 for i in range(k) if i not in fin)
                        break
                    if now - last > 30:
                        last = now
                        print(f"[ref_baseline] {len(fin)}/{k} instances done, {now - tb:.0f} s", file=sys.stderr,
                              flush=True)
            finally:  # stalled, or another instance failed: none keeps spinning into the next leg
                for i, p in enumerate(procs):
                    if p.poll() is None:
                        p.kill()
                    p.wait()
                for f in errs:
                    f.close()
            stalls += [(i, stall_cause((dirs[i] / "stderr.txt").read_text())) for i in range(k) if i not in fin]
            if not fin:
                raise RuntimeError(f"no reference instance finished within {args.ref_timeout:.0f} s")
            for i in fin:  # the instance reached quiescence and dumped its 8 nodes
                assert all((dirs[i] / f"core_{n}_output.txt").exists() for n in range(8)), dirs[i]
            batches += 1
            instr += len(fin) * 8 * args.len
            elapsed += max(fin.values())
            rates.append(len(fin) * 8 * args.len / max(fin.values()))
            if batches >= min_batches and time.perf_counter() - t0 >= target_s:
                break
    cores = host_cores()
    loc = f", locality {locality / 65536:g}" if kind_name == "locality" else ""
    stalled = explain_stalls(stalls, seed, kind_id, locality, cache_size, args.len)
    return {"value": instr / elapsed, "unit": "instr/s", "cores": cores, "host_cpus_visible": host_cpus_visible(),
            "stalled": stalled, "slow_instances_waited_for": waited_slow,
            "kind": "reference", "mode": "A" if k == cores else ("B" if k == 1 else f"{k} instances"),
            # spread over the batches (the spinning instances vary from batch to batch): instr/s
            "batches": {"n": len(rates), "min": min(rates), "median": sorted(rates)[len(rates) // 2],
                        "max": max(rates)},
            "instances": k, "threads_per_instance": 8, "hung_instances_killed": hung, "cpu_model": cpu_model(),
            "sample": f"{batches} batch(es) x {k} concurrent instance(s) x 8 OpenMP threads, one 8-node system "
                      f"x {args.len} instr each ({kind_name}{loc}, CS={cache_size}, systems 0..{k - 1} of seed "
                      f"0x{seed:X}) in {elapsed:.1f} s ({hung} stalled instance(s) killed, not counted: the "
                      f"figure is over the instances that finished, see `stalled` for why the others stalled); {cores} "
                      f"CPUs of cgroup quota on a host exposing "
                      f"{host_cpus_visible()} logical CPUs ({cpu_model()}); assignment.c + benchmark patch "
                      f"(oracle/patch_ref.py), gcc -O2 -fopenmp"}


def sysfs_gpu(pci_domain, pci_bus):
    """The GPU's current clock levels and power / temperature from sysfs (amdgpu), found by its
    PCI address; None where the files are absent or unreadable (e.g. no GPU)."""
    import glob
    want = f"{pci_domain:04x}:{pci_bus:02x}:"
    for dev in sorted(glob.glob("/sys/class/drm/card*/device")):
        real = os.path.realpath(dev)
        if not os.path.basename(real).lower().startswith(want):
            continue
        out = {"pci": os.path.basename(real)}
        for f in ("pp_dpm_sclk", "pp_dpm_mclk", "pp_dpm_fclk", "power_dpm_force_performance_level"):
            try:
                txt = pathlib.Path(dev, f).read_text()
            except OSError:
                continue
            cur = [ln.strip() for ln in txt.splitlines() if ln.strip().endswith("*")]
            out[f] = cur[0] if cur else txt.strip()
        for hw in sorted(glob.glob(f"{dev}/hwmon/hwmon*")):
            for f, key, scale in (("power1_average", "power_w", 1e-6), ("power1_input", "power_w", 1e-6),
                                  ("temp1_input", "temp_edge_c", 1e-3), ("temp2_input", "temp_hotspot_c", 1e-3),
                                  ("freq1_input", "sclk_mhz", 1e-6)):
                if key in out:
                    continue
                try:
                    out[key] = round(int(pathlib.Path(hw, f).read_text()) * scale, 1)
                except (OSError, ValueError):
                    pass
        return out
    return None


class ClockSampler:
    """Samples the GPU's current shader clock from sysfs (hwmon freq1_input, else the starred
    pp_dpm_sclk level) every `period` s on a thread while the timed region runs (dash_run
    releases the GIL), so a line shows whether the box held its clock under the sustained load."""

    def __init__(self, sysfs_dev, period=0.05):
        import glob
        import threading
        self.files = sorted(glob.glob(f"{sysfs_dev}/hwmon/hwmon*/freq1_input")) if sysfs_dev else []
        self.dpm = f"{sysfs_dev}/pp_dpm_sclk" if sysfs_dev else None
        self.period, self.samples, self.stop_ev = period, [], threading.Event()
        self.th = threading.Thread(target=self._run, daemon=True)

    def _read(self):
        try:
            if self.files:
                return int(pathlib.Path(self.files[0]).read_text()) / 1e6
            for ln in pathlib.Path(self.dpm).read_text().splitlines():
                if ln.strip().endswith("*"):
                    return float(ln.split(":")[1].lower().replace("mhz", "").replace("*", "").strip())
        except (OSError, ValueError, IndexError, TypeError):
            return None
        return None

    def _run(self):
        while not self.stop_ev.wait(self.period):
            v = self._read()
            if v is not None:
                self.samples.append(v)

    def __enter__(self):
        if self.files or self.dpm:
            self.th.start()
        return self

    def __exit__(self, *exc):
        self.stop_ev.set()
        if self.th.is_alive():
            self.th.join()

    def summary(self):
        s = sorted(self.samples)
        if not s:
            return None
        return {"n": len(s), "min_mhz": s[0], "median_mhz": s[len(s) // 2], "max_mhz": s[-1],
                "source": "hwmon freq1_input" if self.files else "pp_dpm_sclk (starred level)"}


def sysfs_dev_path(pci_domain, pci_bus):
    import glob
    want = f"{pci_domain:04x}:{pci_bus:02x}:"
    for dev in sorted(glob.glob("/sys/class/drm/card*/device")):
        if os.path.basename(os.path.realpath(dev)).lower().startswith(want):
            return dev
    return None


def box_probe(dash, dev):
    """dash_probe_box (the device, its clock limits, a fixed VALU probe and the shader clock it
    ran at) plus the sysfs clock levels, sampled around the timed region."""
    try:
        b = dash.probe_box(dev)
    except Exception as e:
        return {"error": str(e)}
    return {"probe_ms": round(b["probe_ms"], 3), "probe_valu_per_s": b["probe_valu_per_s"],
            "sclk_mhz": round(b["probe_sclk_mhz"], 1), "sclk_min_mhz": round(b["probe_sclk_min_mhz"], 1),
            "sclk_max_mhz": round(b["probe_sclk_max_mhz"], 1),
            "sysfs": sysfs_gpu(b["pci_domain"], b["pci_bus"]), "_dev": b}


def box_record(before, after):
    """The line's `box` object: what ran (device identity, limits) and how it ran (the probe and
    clocks before and after the timed regions)."""
    dev = before.pop("_dev", None) if before else None
    if after:
        after.pop("_dev", None)
    out = {"probe_before": before, "probe_after": after,
           "probe_basis": "dash_probe_box: CUs x 8 workgroups x 256 threads, 8 dependent full-rate VALU chains "
                          "per lane, 2^21 trips (~170 ms); sclk = shader-clock cycles (s_memtime) / 100-MHz reference ticks "
                          "(s_memrealtime) over each workgroup's loop"}
    if dev:
        out["device"] = {k: dev[k] for k in ("name", "arch", "compute_units", "clock_khz", "mem_clock_khz",
                                             "pci_domain", "pci_bus", "pci_device", "total_mem")}
    return out


def shard(rank, world, per_gpu):
    """Weak scaling: rank g owns global systems [g*M, (g+1)*M). Traces are keyed
    by global id, so results do not depend on the GPU count."""
    return rank * per_gpu, per_gpu


def reduce_totals(elapsed, counters, device, world):
    """The one collective: MAX of the timed region, SUM of the histograms
    (RCCL over xGMI when backend is nccl; gloo in the CPU tests)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    c = torch.tensor(counters, dtype=torch.int64, device=device)
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
    return float(t.item()), [int(x) for x in c.tolist()]


def digest_sum(digests):
    """[sum of low 32 bits, sum of high 32 bits] of the per-system state digests: exact in
    int64 up to 2^31 systems, and independent of how systems are sharded over ranks."""
    import numpy as np
    d = np.asarray(digests, dtype=np.uint64)
    return [int((d & np.uint64(0xFFFFFFFF)).sum(dtype=np.uint64)), int((d >> np.uint64(32)).sum(dtype=np.uint64))]


GOLDEN = ROOT / "tests" / "golden"
_golden_cache = {}
ERR_OOB, ERR_CTZ0 = 2, 4  # include/dash.h: the reference's undefined sends (ref :772,786 / :209,451)


def golden_file(name):
    """A committed golden fixture (tests/golden/<name>; data, not the oracle), or None."""
    if name not in _golden_cache:
        try:
            _golden_cache[name] = json.loads((GOLDEN / name).read_text())
        except (OSError, ValueError):
            _golden_cache[name] = None
    return _golden_cache[name]


def golden_key(kind_name, cache_size, locality=None):
    """The workload's key in the golden fixtures: "uniform" / "contention" (CACHE_SIZE 4) or
    "locality:<CS>:<p>" (the configs[4] grid)."""
    return kind_name if kind_name in ("uniform", "contention") else f"locality:{cache_size}:{locality:g}"


def slice_golden(key, cache_size, local, sys_base, M, args):
    """This rank's own (pre-reduce) totals against the oracle's full-size totals of its slice. Slice 0
    = global systems [0, 2^20): tests/golden/full_size.json (uniform, contention) and sweep_full.json
    (configs[4]); slices r = 1..7 of the 8-GPU layout, [r * 2^20, (r + 1) * 2^20):
    tests/golden/full_slices.json (uniform, contention; make_full_slices.py). True / False when this
    rank owns exactly such a slice and a golden exists for it, else None. At any GPU count rank 0
    owns slice 0 (shard()), so every driver line is checked; at 2^20 systems per GPU every rank is."""
    if M != 1 << 20 or sys_base % M:
        return None
    r = sys_base // M
    if r:
        g = golden_file("full_slices.json")
        # the headline workloads at the file's CACHE_SIZE; a configs[4] key names its own
        same_cs = key.startswith("locality:") or (g or {}).get("cache_size") == cache_size
        gp = (g or {}).get(key, {}).get(str(r)) if g and same_cs else None
        if not gp or (g["systems_per_slice"], g["instr_per_node"], g["seed"]) != (M, args.len, args.seed):
            return None
        return all(local[k] == gp[k] for k in ("hist", "instructions", "rounds_total", "err_systems", "digest_sum"))
    if key in ("uniform", "contention"):
        g = golden_file("full_size.json")
        gp = g.get(key) if g and g.get("cache_size") == cache_size else None
    else:
        g = golden_file("sweep_full.json")
        gp = next((q for q in (g or {}).get("points", []) if golden_key("locality", q["cache_size"], q["locality"])
                   == key), None)
    if not gp or (g["systems"], g["instr_per_node"], g["seed"]) != (M, args.len, args.seed):
        return None
    return all(local[k] == gp[k] for k in ("hist", "instructions", "rounds_total", "err_systems", "digest_sum"))


def sample_check(key, cache_size, sys_base, M, args, digests, rounds, errors):
    """Every rank: its systems among the sampled global ids of tests/golden/rank_samples.json
    (make_rank_samples.py) against the oracle's per-system digest, rounds and error bits.
    Returns (checked, mismatched)."""
    s = golden_file("rank_samples.json")
    w = (s or {}).get("workloads", {}).get(key)
    if not w or w["cache_size"] != cache_size or (s["seed"], s["instr_per_node"]) != (args.seed, args.len):
        return 0, 0
    checked = bad = 0
    for i, g in enumerate(s["ids"]):
        if sys_base <= g < sys_base + M:
            j = g - sys_base
            checked += 1
            bad += (int(digests[j]) != int(w["digest"][i], 16) or int(rounds[j]) != w["rounds"][i]
                    or int(errors[j]) != w["errors"][i])
    return checked, bad


# the all-reduced counter vector of one workload: hist[13], instructions, rounds_total, err_systems,
# dropped, digest_sum[2], ub_systems, sampled systems checked, sampled mismatches, ranks with samples,
# ranks whose whole slice has a golden, ranks whose slice equals it
N_COUNTERS = 25


def local_totals(eng, stats, key, cache_size, sys_base, M, args):
    """After a timed region: this rank's counter vector (above) and its slice check (slice_golden).
    Reads the per-system results once (digests, rounds, error bits)."""
    d, r, e = eng.read_results()
    dsum = digest_sum(d)
    local = {"hist": stats["hist"], "instructions": stats["instructions"], "rounds_total": stats["rounds_total"],
             "err_systems": stats["err_systems"], "digest_sum": dsum}
    ub = int(((e & (ERR_OOB | ERR_CTZ0)) != 0).sum())
    checked, bad = sample_check(key, cache_size, sys_base, M, args, d, r, e)
    ok = slice_golden(key, cache_size, local, sys_base, M, args)
    vec = (stats["hist"] + [stats["instructions"], stats["rounds_total"], stats["err_systems"], stats["dropped"]]
           + dsum + [ub, checked, bad, 1 if checked else 0, 0 if ok is None else 1, 1 if ok else 0])
    return vec, ok


def samples_obj(totals, world):
    """The sampled-id check summed over the ranks: systems checked, mismatches, ranks that held
    samples (all of them when the ranks' slices are 2^20 systems or a few hundred); and the
    whole-slice check: ranks whose slice has a full-size golden, ranks whose slice equals it."""
    return {"checked": totals[20], "mismatched": totals[21], "ranks": totals[22], "world": world,
            "slices_golden": totals[23], "slices_equal": totals[24]}


def sim_symbol(cache_size):
    """Mangled name of the first-tier lockstep kernel sim_kernel<8, CS, 16, 0> (8-node systems)."""
    return f"_ZN4dash10sim_kernelILi8ELi{cache_size}ELj16ELi0EEEvNS_7SimArgsE"


def kernel_fingerprint(lib_path, sym=None):
    """sha256 prefix of a kernel's code + descriptor in the library being run (default the
    headline sim_kernel<8,4,16,0>; tools/kernel_fingerprint.py), or None if it cannot be read."""
    sys.path.insert(0, str(ROOT / "tools"))
    try:
        import kernel_fingerprint as kf
        return kf.fingerprint(lib_path, sym or kf.HEADLINE_SYM)
    except Exception:
        return None


def read_profile(kind, fp, sym=None):
    """Per-launch counters of the first-tier sim_kernel from the committed rocprofv3
    PMC summary for this workload (tools/pmc_summary.py), only if it was measured on the
    code object being run: (profile or None, note). `fp` = kernel_fingerprint of the
    kernel (`sym`, default the headline's) in the library this process loaded."""
    f = ROOT / "profiles" / f"pmc_{kind}.json"
    if not f.exists():
        return None, f"{f.relative_to(ROOT)} missing"
    try:
        prof = json.loads(f.read_text())
    except Exception as e:
        return None, f"{f.relative_to(ROOT)} unreadable: {e}"
    if fp is None or prof.get("kernel_fingerprint") != fp:
        return None, (f"{f.relative_to(ROOT)} was measured on kernel {prof.get('kernel_fingerprint')}, this run's "
                      f"{sym or 'sim_kernel<8,4,16,0>'} is {fp}: its counters do not describe this binary, so "
                      f"traffic and issue figures are omitted")
    return prof, None


SWEEP_GRID = [(cs, p) for cs in (1, 2, 4, 8, 16) for p in (0.0, 0.25, 0.5, 0.75, 1.0)]


def sweep_gpu(args, dash, rank, world, dev, steps, warmup):
    """configs[4] on the GPU: the CACHE_SIZE x locality grid, args.systems per GPU (sharded by
    global id), `warmup` untimed and `steps` timed steps per point (same barriers as the
    headline); one RCCL all-reduce of the totals per point. One engine per CACHE_SIZE, new
    traces per locality."""
    import torch
    M = args.systems
    sys_base, M = shard(rank, world, M)
    points = []
    a = argparse.Namespace(**vars(args))
    a.steps, a.warmup = steps, warmup
    full = M == 1 << 20 and args.len == 4096  # per GPU: the size the committed PMC passes ran
    for cs in (1, 2, 4, 8, 16):
        eng = dash.Engine(M, num_procs=8, cache_size=cs, max_instr=args.len, device=dev)
        t_cs = time.perf_counter()
        fp = kernel_fingerprint(dash.LIB_PATH, sim_symbol(cs)) if full else None
        try:
            for c2, p in SWEEP_GRID:
                if c2 != cs:
                    continue
                loc = int(round(p * 65536))
                eng.generate(args.seed, args.len, kind=dash.GEN_LOCALITY, locality=loc, sys_base=sys_base)
                elapsed, stats, kms = timed_headline(eng, a, world, dev)
                vec, slice_ok = local_totals(eng, stats, golden_key("locality", cs, p), cs, sys_base, M, args)
                elapsed, totals = reduce_totals(elapsed, vec, torch.device("cuda", dev), world)
                avg_s = sum(kms) / len(kms) / 1e3
                # committed PMC passes of this point (tools/evidence_sweep_pmc.sh), only for the full-size
                # workload and only when measured on this code object
                prof, note = read_profile(f"sweep_cs{cs}_p{p:g}", fp, sim_symbol(cs)) if full else \
                    (None, "committed PMC runs are of the full-size workload")
                points.append({"cache_size": cs, "locality": p,
                               "value": world * M * 8 * args.len * steps / elapsed,
                               "ms_per_step": elapsed / steps * 1e3, "steps": steps, "warmup": warmup,
                               # this rank's launches over the timed steps (HIP events; the step time above
                               # is the max over ranks of the whole timed region)
                               "kernel_ms_avg": avg_s * 1e3, "kernel_ms_steps": [round(x, 3) for x in kms],
                               "roofline": roofline(M, args.len, avg_s, prof, note),
                               "valu_issue": valu_issue(prof, stats["wave_rounds"]) if prof else None,
                               "rounds_per_system": totals[14] / (world * M),
                               "wave_rounds": stats["wave_rounds"],
                               "hist": totals[:13], "instructions": totals[13], "rounds_total": totals[14],
                               "err_systems": totals[15], "dropped": totals[16], "digest_sum": totals[17:19],
                               # systems that hit the reference's undefined behaviour (DASH_ERR_OOB / CTZ0
                               # only): parity there is with the engine's defined drop rule
                               "ub_systems": totals[19], "ub_frac": totals[19] / (world * M),
                               "err_frac": totals[15] / (world * M),
                               # rank 0's slice [0, 2^20) against sweep_full.json; every rank's sampled ids
                               # against rank_samples.json
                               "golden_slice": slice_ok if rank == 0 else None,
                               "samples": samples_obj(totals, world),
                               "tier_systems": stats["tier_systems"]})
        finally:
            eng.close()
        if rank == 0:  # one progress line per CACHE_SIZE (stderr stays well under 1 KB)
            print(f"[sweep] CS {cs}: 5 points in {time.perf_counter() - t_cs:.1f} s", file=sys.stderr, flush=True)
    return points


def sweep_cpu(args, dash, points, target_s, min_batches=3):
    """The reference itself on EACH point's own traces (its speed depends heavily on
    locality, so one figure per CACHE_SIZE misstates the other localities by up to ~45x): mode (A),
    one instance per host core, the binary built for the point's CACHE_SIZE, systems 0.. of that
    point's locality traces, at least `min_batches` batches (and `target_s` seconds). Each point's
    `vs_baseline` is against its own figure. Rank 0, after every GPU point and after the process
    group is gone. Returns {cs: the five points' batches and stalled instances, summed}."""
    per_cs = {}
    for pt in points:
        cs = pt["cache_size"]
        cpu = None
        if not args.no_cpu_baseline:
            try:
                cpu = ref_baseline(args, args.seed, dash.GEN_LOCALITY, target_s, args.ref_instances, cache_size=cs,
                                   locality=int(round(pt["locality"] * 65536)), kind_name="locality",
                                   min_batches=min_batches)
            except Exception as e:  # reported, never substituted by the port
                cpu = {"error": f"reference baseline unavailable: {e}"}
        ok = cpu is not None and "value" in cpu
        pt["cpu_baseline"] = cpu if ok else None
        pt["vs_baseline"] = pt["value"] / cpu["value"] if ok else None
        pt["cpu_baseline_note"] = None if ok else (cpu or {}).get("error", "no CPU baseline (--no-cpu-baseline)")
        agg = per_cs.setdefault(cs, {"points": 0, "batches": 0, "hung": 0, "hung_explained": 0, "oracle_ctz0": 0})
        if ok:
            agg["points"] += 1
            agg["batches"] += cpu["batches"]["n"]
            agg["hung"] += cpu["hung_instances_killed"]
            agg["hung_explained"] += cpu["stalled"]["explained"]
            agg["oracle_ctz0"] += cpu["stalled"].get("oracle_ctz0", 0)
    return per_cs


def sweep(args, dash, rank, world, dev):
    """bench.py --sweep: configs[4] as its own line (--steps / --warmup per point)."""
    import torch.distributed as dist
    M = shard(rank, world, args.systems)[1]
    points = sweep_gpu(args, dash, rank, world, dev, args.steps, args.warmup)
    if dist.is_initialized():
        dist.destroy_process_group()
    if rank == 0:
        per_cs = sweep_cpu(args, dash, points, args.sweep_cpu_seconds, args.sweep_cpu_batches)
        detail = {"metric": "simulated instr/sec (whole node), 8-core DASH systems; sweep",
                  "unit": "instr/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                  "higher_is_better": True, "scaling": "weak", "dtype": "u8",
                  "data": "synthetic locality traces (on-device generator, seed keyed by global id)",
                  "config": {"workload": f"{world * M} systems ({M}/GPU) x 8 nodes x {args.len} "
                                         f"instr, CACHE_SIZE x locality grid (BASELINE configs[4])",
                             "parallelism": f"systems sharded over {world} GPU(s)"},
                  "vs_baseline_basis": SWEEP_CPU_BASIS,
                  "sweep": {"steps": args.steps, "warmup": args.warmup, "cpu_per_cache_size": per_cs, "notes": SWEEP_NOTES,
                            "golden": sweep_golden_summary(points, M), "points": points}}

        def compact(d, shown):
            out = {k: d[k] for k in ("metric", "unit", "n_gpus", "steps", "warmup", "higher_is_better",
                                     "scaling", "dtype", "data", "config")}
            out["sweep"] = compact_sweep(d["sweep"])
            out["detail"] = str(shown)
            return out
        emit(detail, args.detail, compact)


def host_trace_batch(seed, M, L):
    """The --host-traces workload: [M][8][L] packed u16 words from numpy's PCG64 raw bits
    (uniform-like over nodes, blocks, R/W and values); RD words keep their random value bits,
    which the library ignores (ref :839, dash.h). Also used by tests/test_gpu_host_path.py."""
    import numpy as np
    rng = np.random.default_rng(seed)
    packed = rng.bit_generator.random_raw(M * 8 * L // 4).view(np.uint16).reshape(M, 8, L)
    return packed, np.full((M, 8), L, dtype=np.uint32)


def host_traces(args, dash, rank, world, dev):
    """PCIe-inclusive rate of the host-buffer boundary: per step, dash_load_traces (one strided
    H2D copy of the caller's [system][node][instr] u16 array) plus the run. Synthetic uniform
    traces from numpy's generator (node, block, R/W, value uniform; RD value 0). With
    --host-batches B > 1 the systems go in B equal batches through two dash_t handles (each
    with its own HIP stream) on two host threads: batch k+1's copy overlaps batch k's run."""
    import threading

    import numpy as np
    import torch
    import torch.distributed as dist
    M, L = args.systems, args.len
    packed, lens = host_trace_batch(args.seed + rank, M, L)
    B = args.host_batches
    if B < 1 or M % B:
        raise SystemExit("--host-batches must divide --systems")
    Mb = M // B
    engs = [dash.Engine(Mb, num_procs=8, cache_size=args.cache_size, max_instr=L, device=dev)
            for _ in range(min(B, 2))]
    hist = np.zeros(13, dtype=np.uint64)
    load_s, kernel_ms = [], []
    lock = threading.Lock()

    def lane(i):  # host thread i drives handle i over batches i, i+2, ... (ctypes drops the GIL)
        torch.cuda.set_device(dev)
        for b in range(i, B, len(engs)):
            t1 = time.perf_counter()
            engs[i].load_traces(packed[b * Mb:(b + 1) * Mb], lens[b * Mb:(b + 1) * Mb])
            load_s.append(time.perf_counter() - t1)
            st = engs[i].run()
            with lock:
                kernel_ms.append(st["kernel_ms"])
                hist[:] += np.array(st["hist"], dtype=np.uint64)

    def step():
        if args.host_native:
            st = dash.run_host_batched(packed, lens, B, num_procs=8, cache_size=args.cache_size, device=dev)[0]
            with lock:
                kernel_ms.append(st["kernel_ms"])
                hist[:] += np.array(st["hist"], dtype=np.uint64)
            return
        ts = [threading.Thread(target=lane, args=(i,)) for i in range(len(engs))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()

    def barrier():
        if dist.is_initialized():
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    barrier()
    hist[:] = 0
    load_s.clear()
    kernel_ms.clear()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier()
    elapsed, _ = reduce_totals(time.perf_counter() - t0, [0], torch.device("cuda", dev), world)
    instr = world * M * 8 * L * args.steps
    if rank == 0:
        print(json.dumps({"metric": "simulated instr/sec from host trace buffers (PCIe-inclusive), 8-core DASH systems",
                          "value": instr / elapsed, "unit": "instr/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
                          "higher_is_better": True, "scaling": "weak", "dtype": "u8",
                          "data": "synthetic host traces (numpy PCG64 raw bits, uniform-like)",
                          "config": {"workload": f"{M} systems/GPU x 8 nodes x {L} instr, CACHE_SIZE={args.cache_size}, "
                                                 f"traces handed over in host memory every step",
                                     "trace_bytes_per_step": M * 8 * L * 2, "host_batches": B,
                                     "driver": "dash_run_host_batched" if args.host_native else "python threads"},
                          "load_s_steps": [round(x, 4) for x in load_s],
                          "h2d_GBps": M * 8 * L * 2 * args.steps / sum(load_s) / 1e9 if load_s else None,
                          "hist_per_step": [int(x) // args.steps for x in hist],
                          "kernel_ms_steps": [round(x, 3) for x in kernel_ms]}), flush=True)
    for e in engs:
        e.close()
    if dist.is_initialized():
        dist.destroy_process_group()


def free_port():
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(args):
    """`bench.py --gpus N` without torchrun: start N ranks as fresh child processes (this
    parent never initialises HIP, so nothing is exec'd from a GPU process), one per GPU,
    with the torch.distributed environment set; rank 0 prints the line. Any rank failing
    stops the others and fails the launch."""
    import signal
    import subprocess
    port = free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(pathlib.Path(__file__).resolve())] + sys.argv[1:],
                                      env=env, start_new_session=True))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in procs:  # one rank failed: the collectives of the others would hang
                        os.killpg(q.pid, signal.SIGTERM)
            time.sleep(0.05)
    finally:
        for q in procs:
            if q.poll() is None:
                os.killpg(q.pid, signal.SIGKILL)
    return rc


def timed_headline(eng, args, world, dev):
    """W untimed steps, then exactly K timed steps bracketed by barrier + synchronize."""
    import torch
    import torch.distributed as dist

    def barrier():
        if dist.is_initialized():
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        eng.run()
    barrier()
    t0 = time.perf_counter()
    kernel_ms = []
    stats = None
    for _ in range(args.steps):
        stats = eng.run()
        kernel_ms.append(stats["kernel_ms"])
    barrier()
    return time.perf_counter() - t0, stats, kernel_ms


def roofline(M, length, avg_kernel_s, prof, note=None):
    """Algorithmic bytes per launch (2 B per simulated instruction) over the
    launch's average duration (HIP events on the engine's stream), against 8 TB/s;
    `traffic` = HBM bytes per launch of the same kernel from the committed rocprofv3 PMC
    run (profiles/pmc_<kind>.json, tools/pmc_summary.py), not from this process, and only
    when that run's kernel fingerprint is this binary's (else null, `traffic_note` says why)."""
    achieved = M * 8 * length * BYTES_PER_INSTR / avg_kernel_s
    return {"bound": "hbm", "achieved": achieved / 1e9, "peak": PEAK_HBM / 1e9, "unit": "GB/s",
            "frac": achieved / PEAK_HBM, "traffic": prof.get("hbm_bytes_per_launch") if prof else None,
            "traffic_source": (f"{prof.get('source')} (committed rocprofv3 --pmc run of this kernel, "
                               f"per launch; kernel fingerprint {prof.get('kernel_fingerprint')})") if prof else None,
            "traffic_note": note}


def valu_issue(prof, wave_rounds):
    """Issue figures of the first-tier launch from its committed PMC run (count / duration),
    against the architectural 2 wave64 VALU per cycle per CU (so frac <= 1)."""
    if not prof:
        return None
    rate = prof["valu_per_launch"] / (prof["kernel_ms"] / 1e3)
    wr = max(wave_rounds, 1)
    return {"achieved": rate, "peak": VALU_PEAK_SIMD32, "unit": "wave-instr/s", "frac": rate / VALU_PEAK_SIMD32,
            "peak_basis": "2 wave64 VALU/cycle/CU x 256 CUs x 2.4 GHz (MI355X_MICROARCH.md wave scheduling)",
            "valu_per_wave_round": prof["valu_per_launch"] / wr,
            "salu_per_wave_round": prof.get("sq_insts_salu", 0.0) / wr,
            "lds_per_wave_round": prof.get("sq_insts_lds", 0.0) / wr,
            "lds_bank_conflict_frac": (prof["sq_lds_bank_conflict"] / prof["sq_lds_idx_active"]
                                       if prof.get("sq_lds_idx_active") else None),
            "l2_hit_rate": prof.get("l2_hit_rate"),
            # mean resident waves per CU over the launch (SQ_WAVE_CYCLES / SQ_BUSY_CU_CYCLES x 4)
            "waves_per_cu": (prof["sq_wave_cycles"] / prof["sq_busy_cu_cycles"] * 4
                             if prof.get("sq_wave_cycles") and prof.get("sq_busy_cu_cycles") else None),
            "vector_pipe": vector_pipe(prof, wr),
            # measured (SQ_ACTIVE_INST_VALU2, SQ_CYCLES): SIMD quad-cycles that issued one or two
            # VALU / two VALU, and the mean active lanes of a VALU instruction
            "issue_slots": ({"busy_frac": prof["valu_issue_busy_frac"], "dual_frac": prof["valu_dual_issue_frac"],
                             "exec_lanes": prof.get("valu_exec_lanes"),
                             "basis": "(SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2) / SIMD quad-cycles; a SIMD "
                                      "issues at most two VALU per quad-cycle"}
                            if "valu_issue_busy_frac" in prof else None),
            "source": f"{prof.get('source')} (committed rocprofv3 --pmc run, not this process)"}


def vector_pipe(prof, wave_rounds):
    """VALU pipe occupancy model: the PMC VALU count split by the static opcode mix of the
    round loop (tools/isa_table.py --json, committed) into the two measured issue rates of
    tools/micro/valu_ops (simple ops ~2 SIMD cycles per wave64 instruction, three-operand
    ops, selects, compares and bit-field ops ~4), against the SIMD cycles available."""
    path = ROOT / "profiles" / "isa_table.json"
    if not path.exists() or not prof.get("kernel_ms"):
        return None
    isa = json.loads(path.read_text())
    if isa.get("kernel_fingerprint") != prof.get("kernel_fingerprint"):
        return None  # static mix of another code object
    f = isa["valu_full_fraction"]
    cyc = prof["valu_per_launch"] / wave_rounds * (2.0 * f + 4.0 * (1.0 - f))
    avail = prof["kernel_ms"] / 1e3 * 2.4e9 * 1024 / wave_rounds  # 256 CUs x 4 SIMDs at 2.4 GHz
    return {"cycles_per_wave_round": cyc, "available_per_wave_round": avail, "busy_frac": cyc / avail,
            "full_rate_fraction": f, "basis": "model: 2 / 4 SIMD cycles per full / half-rate wave64 VALU "
            "(tools/micro/valu_ops), static mix from profiles/isa_table.json"}


def run_kind(dash, args, kind_name, M, sys_base, world, dev, steps, tier_flag, sampler=None):
    """One workload (uniform / contention / locality): generate on the device, time it (the
    optional ClockSampler samples the clock meanwhile), all-reduce the totals; returns
    (elapsed, totals, stats, kernel_ms)."""
    import torch
    kind = {"uniform": dash.GEN_UNIFORM, "contention": dash.GEN_CONTENTION,
            "locality": dash.GEN_LOCALITY}[kind_name]
    locality = int(round(args.locality * 65536)) if kind_name == "locality" else 0
    eng = dash.Engine(M, num_procs=8, cache_size=args.cache_size, max_instr=args.len,
                      device=dev, flags=tier_flag)
    try:
        eng.generate(args.seed, args.len, kind=kind, locality=locality, sys_base=sys_base)
        a = argparse.Namespace(**vars(args))
        a.steps = steps
        if sampler is not None:
            with sampler:
                elapsed, stats, kernel_ms = timed_headline(eng, a, world, dev)
        else:
            elapsed, stats, kernel_ms = timed_headline(eng, a, world, dev)
        # a checksum of the per-system state digests (sums of their 32-bit
        # halves: order-free, so identical for any GPU count), read back after the timed region,
        # with this rank's golden checks (its slice, its sampled ids)
        key = golden_key(kind_name, args.cache_size, args.locality)
        vec, slice_ok = local_totals(eng, stats, key, args.cache_size, sys_base, M, args)
    finally:
        eng.close()
    elapsed, totals = reduce_totals(elapsed, vec, torch.device("cuda", dev), world)
    return elapsed, totals, stats, kernel_ms, slice_ok


def sweep_golden_summary(points, M):
    """The sweep's golden checks per point (labelled): rank 0's slice against sweep_full.json
    (null where no full-size golden exists for this workload) and the sampled ids of every rank."""
    return {"slice": [0, M], "slice_basis": "rank 0's own totals of global systems [0, M) vs "
                                            "tests/golden/sweep_full.json (oracle, 2^20 systems x 4096 instr)",
            "points": [{"cache_size": p["cache_size"], "locality": p["locality"], "bit_exact": p["golden_slice"],
                        "samples": p["samples"]} for p in points]}


def golden_record(slice_ok, cont, points, totals, world, M):
    """The line's `golden` object: rank 0's slice [0, M) against the full-size goldens (headline,
    contention, and how many of the sweep points that have one are bit-exact: [equal, with a golden,
    points]), and the sampled ids summed over every workload of the run: [checked, mismatched, the
    fewest ranks holding samples in any workload, world]."""
    objs = [samples_obj(totals, world)] + ([cont["samples"]] if cont else []) + \
        [p["samples"] for p in points or []]
    flags = [p["golden_slice"] for p in points] if points else None
    head = samples_obj(totals, world)
    return {"slice": [0, M], "headline": slice_ok, "contention": cont.get("golden_slice") if cont else None,
            # every rank's whole slice: [ranks equal to their slice's golden, ranks with one, world]
            "ranks": {"headline": [head["slices_equal"], head["slices_golden"], world],
                      "contention": ([cont["samples"]["slices_equal"], cont["samples"]["slices_golden"], world]
                                     if cont else None)},
            # [rank 0 equal, rank 0 with a golden, points, all ranks' slices equal, all ranks' slices with one]
            "sweep": ([sum(f is True for f in flags), sum(f is not None for f in flags), len(flags),
                       sum(p["samples"].get("slices_equal", 0) for p in points),
                       sum(p["samples"].get("slices_golden", 0) for p in points)]
                      if flags is not None else None),
            "samples": [sum(o["checked"] for o in objs), sum(o["mismatched"] for o in objs),
                        min(o["ranks"] for o in objs), world],
            "basis": "slice: rank 0's own pre-reduce totals (hist, instructions, rounds, err_systems, digest_sum) vs "
                     "tests/golden/full_size.json / sweep_full.json, null where no golden covers the workload; ranks: "
                     "each rank's totals vs its slice's golden (full_slices.json for slices 1..7); samples: "
                     "each rank's systems among tests/golden/rank_samples.json's ids, per-system digest + rounds + "
                     "error bits"}


def totals_dict(totals):
    """The all-reduced totals (the same for any GPU count; the sampled-id check, whose rank count is
    not, sits beside them as `samples`)."""
    return {"hist": totals[:13], "instructions_per_step": totals[13], "rounds_total": totals[14],
            "err_systems": totals[15], "dropped": totals[16], "digest_sum": totals[17:19],
            "ub_systems": totals[19]}


def rank_spread(x, device):
    """[min, max] of a per-rank figure over the ranks (one MIN and one MAX all-reduce; [x, x]
    without a process group)."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized():
        return [x, x]
    lo = torch.tensor([x], dtype=torch.float64, device=device)
    hi = lo.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    return [float(lo.item()), float(hi.item())]


# the CACHE_SIZE 8 trade, stated in the line rather than re-measured
SWEEP_NOTES = {"8": "2-instr window: 18 not 16 waves/CU, p0 668->655 ms; L2 fills 8.5x algorithmic (CS4 5.1x), <1 TB/s"}
SWEEP_CPU_BASIS = ("per point: the reference built for its CACHE_SIZE, mode (A), >= 3 batches on systems 0.. of "
                   "that point's own locality traces; each point's vs_baseline is against its own figure")


def sig(x, n=4):
    """x rounded to n significant digits (ints, bools and None unchanged): keeps the line short."""
    if x is None or isinstance(x, (bool, int)) or not isinstance(x, float) or x == 0 or not math.isfinite(x):
        return x
    return float(f"{x:.{n - 1}e}")


def compact_cpu(c, sample=True):
    """The line's form of a reference / port CPU baseline: figure, cores, mode, batch spread."""
    if not c or "value" not in c:
        return None
    out = {"value": sig(c["value"]), "unit": c.get("unit", "instr/s"), "cores": c.get("cores"),
           "kind": c.get("kind")}
    if c.get("mode"):
        out["mode"] = c["mode"]
    b = c.get("batches")
    if b:
        out["batches"] = [b["n"], sig(b["min"], 3), sig(b["median"], 3), sig(b["max"], 3)]
    if "hung_instances_killed" in c:
        out["hung"] = c["hung_instances_killed"]
        out["hung_explained"] = (c.get("stalled") or {}).get("explained")
    if sample:
        out["cpu_model"] = (c.get("cpu_model") or "")[:48]
        out["sample"] = ((f"{c['instances']} concurrent instances x 8 OpenMP threads, assignment.c + bench patch, "
                          f"gcc -O2 -fopenmp" if c.get("kind") == "reference" else
                          "oracle/dash_oracle.c restatement, OpenMP over systems") + "; full text in detail")
    return out


def compact_roofline(r):
    return {k: sig(r.get(k)) for k in ("bound", "achieved", "peak", "unit", "frac", "traffic")} if r else None


def compact_headline(d, detail_path):
    """The printed line (<= LINE_BUDGET bytes) from the full record `d`: the contract fields, roofline,
    CPU baselines, and configs[3] / configs[4] / §8(f) / box summaries; everything else stays in
    the side file `detail_path`."""
    line = {k: d.get(k) for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                  "higher_is_better", "scaling", "vs_baseline", "dtype", "data")}
    for k in ("value", "ms_per_step", "vs_baseline"):
        line[k] = sig(line[k], 5)
    line["config"] = {"workload": d["config"]["workload"], "parallelism": d["config"]["parallelism"]}
    line["rccl_world"] = d.get("rccl_world")
    line["backend"] = d.get("backend")
    line["kernel_ms_avg"] = sig(d.get("kernel_ms_avg"), 5)
    line["kernel_ms_rank"] = [sig(x, 5) for x in d.get("kernel_ms_rank") or []]
    line["roofline"] = compact_roofline(d.get("roofline"))
    vi = d.get("valu_issue")
    if vi:  # VALU busy, LDS bank conflicts and occupancy beside the roofline
        line["issue"] = {"valu_frac": sig(vi.get("frac"), 3),
                         "valu_busy": sig((vi.get("issue_slots") or {}).get("busy_frac"), 3),
                         "lds_conflict": sig(vi.get("lds_bank_conflict_frac"), 3),
                         "waves_per_cu": sig(vi.get("waves_per_cu"), 3)}
    line["ub_frac"] = sig(d.get("ub_frac"), 3)
    g = d.get("golden")
    if g:
        line["golden"] = {k: g.get(k) for k in ("slice", "headline", "contention", "sweep", "samples")}
        rk = g.get("ranks") or {}
        # whole slices of all ranks: [[headline equal, with a golden], [contention ...]] (world: samples[3])
        line["golden"]["ranks"] = [(rk.get("headline") or [None, None])[:2], (rk.get("contention") or [None, None])[:2]]
    line["cpu_baseline"] = compact_cpu(d.get("cpu_baseline"))
    if d.get("cpu_baseline_note"):
        line["cpu_baseline_note"] = d["cpu_baseline_note"][:160]
    if d.get("cpu_baseline_mode_b"):
        line["vs_baseline_mode_b"] = sig(d.get("vs_baseline_mode_b"))
        line["cpu_baseline_mode_b"] = compact_cpu(d["cpu_baseline_mode_b"], sample=False)
    if d.get("cpu_port"):
        line["cpu_port"] = sig(d["cpu_port"]["value"])
    c = d.get("contention")
    if c:
        t = c["totals"]
        line["contention"] = {"value": sig(c["value"], 5), "ms_per_step": sig(c["ms_per_step"], 5),
                              "frac": sig(c["roofline"]["frac"]), "traffic": sig(c["roofline"].get("traffic")),
                              "err_systems": t["err_systems"], "digest_sum": t["digest_sum"]}
    if d.get("sweep"):
        line["sweep"] = compact_sweep(d["sweep"])
    nx = d.get("next")
    if nx:
        ev, sd = nx.get("events") or {}, nx.get("seeded") or {}
        line["next"] = {"events_x": sig(ev.get("slowdown"), 3), "seeded_x": sig(sd.get("slowdown"), 3),
                        "parity": bool(ev.get("parity_same_digests_as_fast") and ev.get("parity_events_logged")
                                       and sd.get("parity_all_issued") and sd.get("parity_reproducible"))}
    b = d.get("box") or {}
    pb, pa = b.get("probe_before") or {}, b.get("probe_after") or {}
    if pb or pa:
        line["box"] = {"pci": ((pb.get("sysfs") or {}).get("pci")),
                       "probe_ms": [pb.get("probe_ms"), pa.get("probe_ms")],
                       "sclk_mhz": [pb.get("sclk_mhz"), pa.get("sclk_mhz")]}
    line["kernel_fingerprint"] = d.get("kernel_fingerprint")
    line["detail"] = str(detail_path)
    return line


def compact_sweep(sw):
    """configs[4] in the line: one row per point, the reference per CACHE_SIZE, the golden flags."""
    def giga(x):
        return sig(x / 1e9, 4) if x is not None else None
    rows = [[p["cache_size"], p["locality"], giga(p["value"]), sig(p["ms_per_step"]), sig(p["roofline"]["frac"], 3),
             sig(p.get("vs_baseline"), 3), sig(p["ub_frac"], 3), giga(p["roofline"].get("traffic")),
             p.get("golden_slice"), (p.get("samples") or {}).get("mismatched")]
            for p in sw["points"]]
    cpu = {str(cs): ([c["points"], c["batches"], c["hung"], c["hung_explained"]] if c else None)
           for cs, c in (sw.get("cpu_per_cache_size") or {}).items()}
    return {"cols": ["cs", "p", "value_G", "ms_per_step", "frac", "vs_baseline", "ub_frac", "traffic_GB",
                     "golden", "smp_bad"],
            "rows": rows, "steps": sw["steps"],
            "cpu_cols": ["points", "batches", "hung", "hung_explained"], "cpu": cpu, "notes": sw.get("notes")}


def detail_path_arg(p):
    """--detail PATH (relative paths are taken from the repo root, where the driver runs)."""
    path = pathlib.Path(p) if p else DETAIL_DEFAULT
    return path if path.is_absolute() else ROOT / path


def emit(detail, detail_arg, compact=None):
    """Write the full record to the side file and print the compact line (rank 0)."""
    path = detail_path_arg(detail_arg)
    shown = path.relative_to(ROOT) if path.is_relative_to(ROOT) else path
    try:
        path.parent.mkdir(parents=True, exist_ok=True)
        path.write_text(json.dumps(detail, indent=1))
    except OSError as e:
        shown = f"unwritten ({e})"
    line = (compact or compact_headline)(detail, shown)
    text = json.dumps(line, separators=(",", ":"))
    if len(text) > LINE_BUDGET:  # never silently: drop the least important summaries until it fits
        for k in ("next", "box", "cpu_baseline_mode_b", "contention", "sweep"):
            if k == "sweep" and line.get("sweep"):  # last resort: the rows stay in the side file only
                sw = line["sweep"]
                vals = [r[2] for r in sw["rows"] if r[2] is not None]
                line["sweep"] = {"rows": len(sw["rows"]), "value_G_range": [min(vals), max(vals)] if vals else None,
                                 "golden_not_exact": [[r[0], r[1]] for r in sw["rows"] if r[8] is False]}
            else:
                line.pop(k, None)
            line["dropped_for_size"] = line.get("dropped_for_size", []) + [k]
            text = json.dumps(line, separators=(",", ":"))
            if len(text) <= LINE_BUDGET:
                break
    print(text, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); without torchrun bench.py starts them itself")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--systems", type=int, default=1 << 20, help="systems per GPU")
    ap.add_argument("--len", type=int, default=4096, help="instructions per node")
    ap.add_argument("--cache-size", type=int, default=4)
    ap.add_argument("--kind", choices=["uniform", "contention", "locality"], default="uniform")
    ap.add_argument("--locality", type=float, default=0.5)
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED)
    ap.add_argument("--contention-steps", type=int, default=5,
                    help="timed steps of the contention workload (configs[3]) reported in the headline "
                         "line's `contention` object (0 = skip); its own warmup step precedes them")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="target seconds of each CPU leg (reference mode A, mode B, oracle port)")
    ap.add_argument("--sweep-cpu-seconds", type=float, default=1.0,
                    help="configs[4]: target seconds of the reference baseline per CACHE_SIZE (at least "
                         "--sweep-cpu-batches batches)")
    ap.add_argument("--sweep-cpu-batches", type=int, default=3,
                    help="configs[4]: minimum reference batches per CACHE_SIZE")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--detail", default=None,
                    help="side file for the full record (default gpurun_out/bench_detail.json; relative to the "
                         "repo root); the printed line is its <= 4 KB summary and names it")
    ap.add_argument("--line-sweep", choices=["auto", "on", "off"], default="auto",
                    help="the configs[4] grid inside the headline line (`sweep` object): auto = only with the "
                         "full-size uniform headline workload")
    ap.add_argument("--line-sweep-steps", type=int, default=1, help="timed steps per sweep point in the line")
    ap.add_argument("--line-next", choices=["auto", "on", "off"], default="auto",
                    help="the DEBUG event-log and seeded-schedule rows of --next inside the headline line (`next` "
                         "object): auto = only with the full-size uniform headline on one GPU")
    ap.add_argument("--line-sweep-warmup", type=int, default=1, help="untimed steps per sweep point in the line")
    ap.add_argument("--cpu-kind", choices=["port", "reference"], default="reference",
                    help="headline cpu_baseline: the reference binary itself (oracle/_ref/cache_simulator_bench, "
                         "default; the oracle port is then reported as cpu_port) or only the oracle port")
    ap.add_argument("--ref-instances", type=int, default=0,
                    help="concurrent reference instances (0 = one per host core: BASELINE.md mode (A); "
                         "1 = mode (B))")
    ap.add_argument("--ref-max-instances", type=int, default=64,
                    help="cap on mode (A)'s concurrent instances (8 threads each); a capped run reports "
                         "mode '<k> instances' instead of 'A'")
    ap.add_argument("--ref-timeout", type=float, default=240.0,
                    help="give up on the reference baseline after this many seconds (reported as null)")
    ap.add_argument("--first-depth", type=int, choices=[0, 32, 256], default=0,
                    help="first queue-depth tier (0 = adaptive, starting at 16)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend for N > 1 (nccl = RCCL over xGMI; gloo only for the "
                         "1-GPU rehearsal of the distributed path in tests/test_gpu_distributed.py)")
    ap.add_argument("--process-group", action="store_true",
                    help="initialise the process group and run the collectives even at --gpus 1 (exercises "
                         "the RCCL barrier / all-reduce path on a 1-GPU box; tests/test_gpu_distributed.py)")
    ap.add_argument("--host-traces", action="store_true",
                    help="drop-in host-buffer path: traces built in host memory (numpy, uniform-like) and "
                         "handed over through dash_load_traces inside every timed step (PCIe-inclusive rate; "
                         "DESIGN.md §4); not the headline `value`")
    ap.add_argument("--host-batches", type=int, default=1,
                    help="--host-traces: split the systems into this many batches on two handles driven by two "
                         "host threads, so one batch's H2D copy overlaps another's simulation")
    ap.add_argument("--host-native", action="store_true",
                    help="--host-traces through the library's own batched entry point (dash_run_host_batched: "
                         "C++ threads, handles created per call) instead of Python threads over two engines")
    ap.add_argument("--sweep", action="store_true",
                    help="BASELINE configs[4]: CACHE_SIZE {1,2,4,8,16} x locality {0,.25,.5,.75,1}, "
                         "systems sharded over the ranks, histograms all-reduced per configuration")
    ap.add_argument("--next", action="store_true",
                    help="the SURVEY.md 8(f) rows beside the hot path, measured with a parity property each "
                         "(bench_next.py): text ingest, digests / dumps, DEBUG event log, seeded schedules")
    ap.add_argument("--next-systems", type=int, default=2048, help="--next: trace directories written and ingested")
    ap.add_argument("--next-dir", default=None, help="--next: where the trace directories go (default: $TMPDIR)")
    ap.add_argument("--next-event-systems", type=int, default=32768,
                    help="--next: systems of the DEBUG event-log row (device-generated traces)")
    ap.add_argument("--dist-selftest", action="store_true",
                    help="no GPU: the rank launch plus one gloo all-reduce of the shard table on the CPU "
                         "(tests/test_distributed.py checks the launcher with it)")
    args = ap.parse_args()

    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        raise SystemExit(launch_ranks(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: the rank count must equal --gpus")

    import torch
    import torch.distributed as dist

    if args.dist_selftest:  # CPU only: what each rank owns, summed over the ranks
        if world > 1:
            dist.init_process_group("gloo")
        base, count = shard(rank, world, args.systems)
        owned = torch.zeros(world * args.systems, dtype=torch.int64)
        owned[base:base + count] = 1
        if world > 1:
            dist.all_reduce(owned)
        # the same fields the GPU line records: the group actually formed and a per-rank spread
        # (here of rank + 1, so [1, world])
        rccl_world = dist.get_world_size() if dist.is_initialized() else 1
        backend = str(dist.get_backend()) if dist.is_initialized() else None
        spread = rank_spread(float(rank + 1), torch.device("cpu"))
        if rank == 0:
            print(json.dumps({"world": world, "systems_owned": int(owned.sum()),
                              "each_once": bool((owned == 1).all()), "local_rank": local_rank,
                              "rccl_world": rccl_world, "backend": backend, "kernel_ms_rank": spread}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    dash = load_dash()
    # one rank per GPU; ranks beyond the visible GPUs share them (1-GPU rehearsal, gloo only)
    ndev = torch.cuda.device_count()
    if world > ndev and args.dist_backend == "nccl":
        raise SystemExit(f"bench.py: {world} ranks over nccl need {world} GPUs, {ndev} visible")
    dev = local_rank % max(ndev, 1)
    torch.cuda.set_device(dev)
    if world > 1 or args.process_group:
        if world == 1:  # a one-rank group of its own (env:// rendezvous on the loopback)
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(free_port()))
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo")

    if args.sweep:
        return sweep(args, dash, rank, world, dev)
    if args.next:
        if world != 1:
            raise SystemExit("bench.py --next runs on one GPU")
        import bench_next
        return bench_next.run(dash, dev, args)
    if args.host_traces:
        return host_traces(args, dash, rank, world, dev)

    tier_flag = {0: 0, 32: dash.TIER_FROM_32, 256: dash.TIER_FROM_256}[args.first_depth]
    sys_base, M = shard(rank, world, args.systems)
    probe0 = box_probe(dash, dev)
    pdev = probe0.get("_dev") or {}
    sampler = ClockSampler(sysfs_dev_path(pdev["pci_domain"], pdev["pci_bus"])) if pdev else None
    elapsed, totals, stats, kernel_ms, slice_ok = run_kind(dash, args, args.kind, M, sys_base, world, dev,
                                                 args.steps, tier_flag, sampler)
    probe1 = box_probe(dash, dev)
    instr_per_step = world * M * 8 * args.len
    value = instr_per_step * args.steps / elapsed
    avg_kernel_s = sum(kernel_ms) / len(kernel_ms) / 1e3
    full = M == 1 << 20 and args.len == 4096 and args.cache_size == 4
    fp = kernel_fingerprint(dash.LIB_PATH)
    prof, prof_note = read_profile(args.kind, fp) if full else (None, "committed PMC runs are of the full-size workload")

    # configs[3] beside the headline: its own warmup and timed steps (same barriers)
    cont = None
    if args.contention_steps > 0 and args.kind == "uniform":
        c_el, c_tot, c_stats, c_kms, c_slice_ok = run_kind(dash, args, "contention", M, sys_base, world, dev,
                                               args.contention_steps, tier_flag)
        c_prof, c_note = read_profile("contention", fp) if full else (None, prof_note)
        c_avg = sum(c_kms) / len(c_kms) / 1e3
        cont = {"workload": f"{M} systems/GPU x 8 nodes x {args.len} contention RD/WR per node (90 % WR to "
                            f"0x00-0x03), CACHE_SIZE={args.cache_size} (BASELINE configs[3])",
                "value": instr_per_step * args.contention_steps / c_el, "unit": "instr/s",
                "steps": args.contention_steps, "warmup": args.warmup,
                "ms_per_step": c_el / args.contention_steps * 1e3,
                "kernel_ms_avg": c_avg * 1e3, "kernel_ms_steps": [round(x, 3) for x in c_kms],
                "roofline": roofline(M, args.len, c_avg, c_prof, c_note),
                "valu_issue": valu_issue(c_prof, c_stats["wave_rounds"]),
                "tier_systems": c_stats["tier_systems"], "wave_rounds": c_stats["wave_rounds"],
                "totals": totals_dict(c_tot), "samples": samples_obj(c_tot, world), "golden_slice": c_slice_ok}

    # configs[4] beside the headline: the whole CACHE_SIZE x locality grid at
    # this line's systems per GPU, --line-sweep-warmup untimed and --line-sweep-steps timed steps per
    # point; by default only with the full-size headline workload
    line_sweep = args.line_sweep == "on" or (args.line_sweep == "auto" and full and args.kind == "uniform")
    points = sweep_gpu(args, dash, rank, world, dev, args.line_sweep_steps, args.line_sweep_warmup) \
        if line_sweep else None
    # two SURVEY §8(f) rows beside the hot path, driver-observed on one GPU (bench_next.py): the
    # DEBUG event log against the fast kernel, and the seeded legal schedules at the headline size
    line_next = args.line_next == "on" or (args.line_next == "auto" and full and args.kind == "uniform"
                                           and world == 1)
    next_rows = None
    if line_next:
        import bench_next
        next_rows = {"events": bench_next.events_row(dash, dev, args.seed, args.next_event_systems, args.len),
                     "seeded": bench_next.seeded_row(dash, dev, args.seed, M, args.len, 1)}

    # what the process group actually formed, and the spread of the headline
    # kernel's average launch time over the ranks (one MIN and one MAX all-reduce)
    rccl_world = dist.get_world_size() if dist.is_initialized() else 1
    backend = str(dist.get_backend()) if dist.is_initialized() else None
    k_rank = rank_spread(avg_kernel_s * 1e3, torch.device("cuda", dev))
    # the CPU legs run after the timed regions and after the process group is gone, on rank 0
    # only, for every --gpus N (the ratio north_star states is the 8-GPU one)
    if dist.is_initialized():
        dist.destroy_process_group()
    if rank == 0:
        sweep_obj = None
        if points is not None:
            sweep_cpu_obj = sweep_cpu(args, dash, points, args.sweep_cpu_seconds, args.sweep_cpu_batches)
            sweep_obj = {"workload": f"{world * M} systems ({M}/GPU) x 8 nodes x {args.len} locality RD/WR per "
                                     f"node, CACHE_SIZE {{1,2,4,8,16}} x locality {{0,.25,.5,.75,1}} "
                                     f"(BASELINE configs[4]; seed 0x{args.seed:X}, keyed by global id)",
                         "steps": args.line_sweep_steps, "warmup": args.line_sweep_warmup,
                         "cpu_baseline_basis": SWEEP_CPU_BASIS, "cpu_per_cache_size": sweep_cpu_obj,
                         "notes": SWEEP_NOTES,
                         "golden": sweep_golden_summary(points, M), "points": points}
        cpu, cpu_b, port, note = None, None, None, None
        if not args.no_cpu_baseline:
            kind_id = {"uniform": dash.GEN_UNIFORM, "contention": dash.GEN_CONTENTION,
                       "locality": dash.GEN_LOCALITY}[args.kind]
            locality = int(round(args.locality * 65536)) if args.kind == "locality" else 0
            if args.cpu_kind == "reference":
                try:  # BASELINE.md mode (A): one instance per host core; mode (B): one instance
                    cpu = ref_baseline(args, args.seed, kind_id, args.cpu_seconds, args.ref_instances,
                                       args.cache_size, locality)
                    if not args.ref_instances:
                        cpu_b = ref_baseline(args, args.seed, kind_id, args.cpu_seconds, 1, args.cache_size, locality)
                except Exception as e:  # reported, never substituted by the port
                    note = f"reference baseline unavailable: {e}"
            port = cpu_baseline(args, args.seed, kind_id, locality, args.cpu_seconds)
            if args.cpu_kind == "port":
                cpu, port = port, None
        detail = {
            "metric": "simulated instr/sec (whole node), 8-core DASH systems; % HBM roofline",
            "value": value,
            "unit": "instr/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            # BASELINE.md publishes no number: the ratio is against cpu_baseline measured in this run
            "vs_baseline": value / cpu["value"] if cpu else None,
            "vs_baseline_basis": (f"value / cpu_baseline.value ({cpu['kind']}"
                                  + (f", mode {cpu['mode']}" if cpu.get("mode") else "")
                                  + ", measured on this box's host in this run; BASELINE.md publishes no number)")
            if cpu else None,
            "vs_baseline_mode_b": value / cpu_b["value"] if cpu_b else None,
            "dtype": "u8",
            "data": "synthetic (on-device counter-based generator, seed keyed by global system id)",
            "config": {"workload": f"{M} systems/GPU x 8 nodes x {args.len} {args.kind} RD/WR per node, "
                                   f"CACHE_SIZE={args.cache_size}",
                       "systems_per_gpu": M, "num_procs": 8, "instr_per_node": args.len,
                       "cache_size": args.cache_size, "trace": args.kind,
                       "parallelism": f"systems sharded over {world} GPU(s)"},
            "roofline": roofline(M, args.len, avg_kernel_s, prof, prof_note),
            # what binds this integer state machine: instruction issue
            "valu_issue": valu_issue(prof, stats["wave_rounds"]),
            "valu_issue_note": prof_note,
            "kernel_fingerprint": fp,
            # the first-tier kernel of this run's CACHE_SIZE, as run (tools/pmc_summary.py binds the PMC
            # passes of this process to it, not to whatever library is built when it summarises them)
            "kernel_fingerprint_run": (fp if args.cache_size == 4 else
                                       kernel_fingerprint(dash.LIB_PATH, sim_symbol(args.cache_size))),
            "cpu_baseline": cpu,
            "cpu_baseline_mode_b": cpu_b,
            "cpu_baseline_note": note,
            "cpu_port": port,
            "kernel_ms_avg": avg_kernel_s * 1e3,
            "kernel_ms_rank": k_rank,
            "kernel_ms_steps": [round(x, 3) for x in kernel_ms],
            "rccl_world": rccl_world,
            "backend": backend,
            "tier_systems": stats["tier_systems"],
            "wave_rounds": stats["wave_rounds"],
            # systems whose run hit the reference's undefined send to node 15 (ref :772,786):
            # parity there is with the engine's defined drop-and-flag rule
            "totals": totals_dict(totals),
            "samples": samples_obj(totals, world),
            "ub_frac": totals[19] / (world * M),
            "err_frac": totals[15] / (world * M),
            # the line certifies its own results at any GPU count -- rank 0's
            # own slice (global systems [0, M), the committed full-size goldens when M = 2^20) and
            # every rank's sampled ids (tests/golden/rank_samples.json)
            "golden": golden_record(slice_ok, cont, points, totals, world, M),
            "parity_note": ("totals.ub_systems systems hit the reference's undefined behaviour (mostly the "
                            "send to node 15, assignment.c:772,786: DASH_ERR_OOB; or ctz(0), :209,451: "
                            "DASH_ERR_CTZ0); on them parity is with the engine's defined drop-and-flag rule "
                            "(DESIGN.md §2), the rest with the reference's semantics under the lockstep "
                            "schedule. err_frac also counts systems flagged only DEADLOCK / STUCK etc."),
            "contention": cont,
            "sweep": sweep_obj,
            "next": next_rows,
            "box": dict(box_record(probe0, probe1),
                        sclk_during_timed_steps=sampler.summary() if sampler else None),
        }
        emit(detail, args.detail)


if __name__ == "__main__":
    main()
