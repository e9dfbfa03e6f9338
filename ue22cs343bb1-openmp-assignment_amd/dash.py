"""Python view of libdash (the C-ABI in include/dash.h) -- the host-side mirror
of the reference's interface for the hot path.

The reference (assignment.c) exposes: the CLI `./cache_simulator <dir>`
(:126-131), initializeProcessor (:806-851), the per-thread event loop
(:149-738) and printProcessorState (:853-905). This module maps them onto
libdash:

    parse_core_file(path)          -> initializeProcessor's parse (:822-850)
    Engine(...).load_dir(dir)      -> initializeProcessor per node (:152)
    Engine.run()                   -> the OpenMP parallel region (:149-738)
    Engine.read_state(sys)         -> the nodes' processorNode state
    dump_node(state, node)         -> printProcessorState bytes (:868-902)
    simulate_dir(dir, out_dir)     -> main() end to end

There is no CPU fallback: if libdash.so is missing or no HIP device is
present the calls raise.
"""
from __future__ import annotations

import ctypes
import os
import pathlib
import subprocess

import numpy as np

PKG = pathlib.Path(__file__).resolve().parent
# DASH_LIB: an alternative build of the same library (kernel variant experiments, tools/)
LIB_PATH = pathlib.Path(os.environ["DASH_LIB"]) if os.environ.get("DASH_LIB") else PKG / "libdash.so"

MEM_SIZE = 16
MAX_PROCS = 8
MAX_CACHE = 16
NUM_TXN = 13
TXN_NAMES = ("READ_REQUEST", "WRITE_REQUEST", "REPLY_RD", "REPLY_WR", "REPLY_ID", "INV",
             "UPGRADE", "WRITEBACK_INV", "WRITEBACK_INT", "FLUSH", "FLUSH_INVACK",
             "EVICT_SHARED", "EVICT_MODIFIED")

OK, EINVAL, EIO, EPARSE, EADDR, EDEVICE, ENOMEM, ESTATE, ETRUNC = 0, -1, -2, -3, -4, -5, -6, -7, -8
EV_MSG, EV_INSTR = 0, 1
ERR_OVERFLOW, ERR_OOB, ERR_CTZ0, ERR_DEADLOCK, ERR_ROUNDCAP, ERR_STUCK = 1, 2, 4, 8, 16, 32
ERR_SCHEDULE = 64  # a micro-step schedule stepped a node with held sends (dash.h)
KEEP_STATE = 1
TIER_FROM_32, TIER_FROM_256 = 2, 4
TEST_SHORT_ARB = 8  # testing only (dash.h)
NUM_TIERS = 3
GEN_UNIFORM, GEN_CONTENTION, GEN_LOCALITY = 0, 1, 2

# every symbol include/dash.h declares
EXPORTS = ("dash_create", "dash_destroy", "dash_last_error", "dash_load_traces", "dash_generate",
           "dash_run", "dash_read_state", "dash_read_results", "dash_read_hist", "dash_stream",
           "dash_parse_core_file", "dash_resolve_dir", "dash_load_dir", "dash_init_node_state",
           "dash_dump_node", "dash_dump_file", "dash_digest_node", "dash_simulate_dir",
           "dash_read_events", "dash_format_event", "dash_load_dirs", "dash_dump_system",
           "dash_write_digests", "dash_run_host_batched", "dash_set_schedule", "dash_probe_box",
           "dash_set_micro_schedule")
SIT_OUT = 0xFF
MICRO_STEP, MICRO_SEND = 0, 1  # dash_set_micro_schedule actions


class DashError(RuntimeError):
    def __init__(self, code: int, what: str):
        super().__init__(f"{what} failed with code {code}")
        self.code = code


class Cfg(ctypes.Structure):
    _fields_ = [("num_procs", ctypes.c_uint32), ("cache_size", ctypes.c_uint32),
                ("max_instr", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("num_systems", ctypes.c_uint64), ("max_rounds", ctypes.c_uint64),
                ("device", ctypes.c_int32), ("trace_events", ctypes.c_uint32),
                ("schedule_seed", ctypes.c_uint64)]


class Event(ctypes.Structure):
    _fields_ = [("round", ctypes.c_uint32), ("node", ctypes.c_uint32), ("kind", ctypes.c_uint32),
                ("word", ctypes.c_uint32)]


class NodeState(ctypes.Structure):
    _fields_ = [("memory", ctypes.c_uint8 * MEM_SIZE), ("dir_bitvector", ctypes.c_uint8 * MEM_SIZE),
                ("dir_state", ctypes.c_uint8 * MEM_SIZE), ("cache_addr", ctypes.c_uint8 * MAX_CACHE),
                ("cache_value", ctypes.c_uint8 * MAX_CACHE),
                ("cache_state", ctypes.c_uint8 * MAX_CACHE)]


class Stats(ctypes.Structure):
    _fields_ = [("hist", ctypes.c_uint64 * NUM_TXN), ("instructions", ctypes.c_uint64),
                ("rounds_total", ctypes.c_uint64), ("rounds_max", ctypes.c_uint64),
                ("systems", ctypes.c_uint64), ("err_systems", ctypes.c_uint64),
                ("err_bits", ctypes.c_uint64), ("dropped", ctypes.c_uint64),
                ("max_depth", ctypes.c_uint64), ("kernel_ms", ctypes.c_double),
                ("tier_systems", ctypes.c_uint64 * NUM_TIERS), ("wave_rounds", ctypes.c_uint64)]

    def as_dict(self):
        return {"hist": [int(x) for x in self.hist], "instructions": int(self.instructions),
                "rounds_total": int(self.rounds_total), "rounds_max": int(self.rounds_max),
                "systems": int(self.systems), "err_systems": int(self.err_systems),
                "err_bits": int(self.err_bits), "dropped": int(self.dropped),
                "max_depth": int(self.max_depth), "kernel_ms": float(self.kernel_ms),
                "tier_systems": [int(x) for x in self.tier_systems],
                "wave_rounds": int(self.wave_rounds)}


class BoxProbe(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 64), ("arch", ctypes.c_char * 32), ("compute_units", ctypes.c_int32),
                ("clock_khz", ctypes.c_int32), ("mem_clock_khz", ctypes.c_int32), ("pci_domain", ctypes.c_int32),
                ("pci_bus", ctypes.c_int32), ("pci_device", ctypes.c_int32), ("total_mem", ctypes.c_uint64),
                ("probe_ms", ctypes.c_double), ("probe_valu_per_s", ctypes.c_double),
                ("probe_sclk_mhz", ctypes.c_double), ("probe_sclk_min_mhz", ctypes.c_double),
                ("probe_sclk_max_mhz", ctypes.c_double)]


class Gen(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64), ("sys_base", ctypes.c_uint64), ("kind", ctypes.c_uint32),
                ("locality", ctypes.c_uint32), ("len", ctypes.c_uint32), ("_reserved", ctypes.c_uint32)]


_lib = None


def build():
    """Compile libdash.so + cache_simulator for gfx950 (in-tree)."""
    subprocess.run(["make", "-s", "-C", str(PKG), f"-j{min(8, os.cpu_count() or 1)}"], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise RuntimeError(f"{LIB_PATH} is missing: run build() first (no CPU fallback exists)")
    L = ctypes.CDLL(str(LIB_PATH))
    vp, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    sig = {
        "dash_create": (i32, [ctypes.POINTER(Cfg), ctypes.POINTER(vp)]),
        "dash_destroy": (None, [vp]),
        "dash_last_error": (ctypes.c_char_p, [vp]),
        "dash_load_traces": (i32, [vp, vp, u64, vp, u64]),
        "dash_generate": (i32, [vp, ctypes.POINTER(Gen)]),
        "dash_set_schedule": (i32, [vp, vp, u32]),
        "dash_set_micro_schedule": (i32, [vp, vp, u32]),
        "dash_probe_box": (i32, [i32, ctypes.POINTER(BoxProbe)]),
        "dash_run": (i32, [vp, ctypes.POINTER(Stats)]),
        "dash_read_state": (i32, [vp, u64, ctypes.POINTER(NodeState)]),
        "dash_read_results": (i32, [vp, u64, u64, vp, vp, vp]),
        "dash_read_hist": (i32, [vp, u64, vp]),
        "dash_stream": (vp, [vp]),
        "dash_parse_core_file": (i32, [ctypes.c_char_p, u32, u32, vp, ctypes.POINTER(u32)]),
        "dash_resolve_dir": (i32, [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]),
        "dash_load_dir": (i32, [vp, ctypes.c_char_p, u64]),
        "dash_init_node_state": (None, [ctypes.POINTER(NodeState), u32, u32]),
        "dash_dump_node": (i32, [ctypes.POINTER(NodeState), u32, u32, ctypes.c_char_p, ctypes.c_size_t]),
        "dash_dump_file": (i32, [ctypes.POINTER(NodeState), u32, u32, ctypes.c_char_p]),
        "dash_digest_node": (u64, [ctypes.POINTER(NodeState), u32, u32]),
        "dash_simulate_dir": (i32, [ctypes.c_char_p, u32, u32, u32, ctypes.c_char_p, i32,
                                    ctypes.POINTER(Stats)]),
        "dash_read_events": (i32, [vp, u64, vp, u32, ctypes.POINTER(u32)]),
        "dash_load_dirs": (i32, [vp, ctypes.POINTER(ctypes.c_char_p), u64]),
        "dash_dump_system": (i32, [vp, u64, ctypes.c_char_p]),
        "dash_write_digests": (i32, [vp, ctypes.c_char_p]),
        "dash_format_event": (i32, [ctypes.POINTER(Event), ctypes.c_char_p, ctypes.c_size_t]),
        "dash_run_host_batched": (i32, [ctypes.POINTER(Cfg), vp, u64, vp, u64, u32, ctypes.POINTER(Stats),
                                        vp, vp, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


# handle-less entry points whose failure text dash_last_error(NULL) holds (dash.h)
_GLOBAL_MSG = ("dash_create", "dash_run_host_batched", "dash_simulate_dir", "dash_probe_box")


def _check(rc: int, what: str, handle=None):
    if rc != OK:
        msg = what
        if handle or what in _GLOBAL_MSG:
            detail = lib().dash_last_error(handle)
            if detail:
                msg = f"{what}: {detail.decode(errors='replace')}"
        raise DashError(rc, msg)


# ------------------------------------------------------------------ host boundary

def parse_core_file(path, num_procs=4, max_instr=32) -> np.ndarray:
    """initializeProcessor's parse (assignment.c:822-850) -> packed u16 records."""
    out = np.zeros(max(max_instr, 1), dtype=np.uint16)
    n = ctypes.c_uint32(0)
    _check(lib().dash_parse_core_file(str(path).encode(), num_procs, max_instr,
                                      out.ctypes.data, ctypes.byref(n)), f"parse {path}")
    return out[:n.value].copy()


def init_node_state(node_id: int, cache_size=4) -> NodeState:
    s = NodeState()
    lib().dash_init_node_state(ctypes.byref(s), node_id, cache_size)
    return s


def dump_node(state: NodeState, node_id: int, cache_size=4) -> str:
    """printProcessorState (assignment.c:853-905), byte-exact."""
    buf = ctypes.create_string_buffer(16384)
    n = lib().dash_dump_node(ctypes.byref(state), node_id, cache_size, buf, 16384)
    if n < 0:
        raise DashError(n, "dump_node")
    return buf.raw[:n].decode()


def digest_node(state: NodeState, node_id: int, cache_size=4) -> int:
    return int(lib().dash_digest_node(ctypes.byref(state), node_id, cache_size))


def format_events(events, kinds=(0, 1)) -> str:
    """Lines exactly as the reference prints them under -D DEBUG_MSG / -D DEBUG_INSTR."""
    buf = ctypes.create_string_buffer(128)
    out = []
    for e in events:
        if e.kind in kinds:
            n = lib().dash_format_event(ctypes.byref(e), buf, 128)
            _check(n if n < 0 else OK, "dash_format_event")
            out.append(buf.value.decode())
    return "".join(out)


def probe_box(device=0) -> dict:
    """dash_probe_box: device identity and clock limits, and a fixed VALU probe with the shader
    clock the box held while it ran (a benchmark line's box description)."""
    b = BoxProbe()
    _check(lib().dash_probe_box(device, ctypes.byref(b)), "dash_probe_box")
    d = {f: getattr(b, f) for f, _ in BoxProbe._fields_}
    d["name"], d["arch"] = b.name.decode(errors="replace"), b.arch.decode(errors="replace")
    return d


def simulate_dir(test_dir, out_dir=".", num_procs=4, cache_size=4, max_instr=32, device=0) -> dict:
    """main() end to end for one trace directory (assignment.c:126-739)."""
    st = Stats()
    _check(lib().dash_simulate_dir(str(test_dir).encode(), num_procs, cache_size, max_instr,
                                   str(out_dir).encode(), device, ctypes.byref(st)),
           f"simulate_dir {test_dir}")
    return st.as_dict()


def run_host_batched(packed: np.ndarray, lens: np.ndarray, batches: int, num_procs=8, cache_size=4,
                     max_instr=None, device=0, flags=0):
    """dash_run_host_batched: host traces [systems, num_procs, stride] u16 in `batches` batches
    on two handles, copies overlapped with runs. Returns (stats dict, digests, rounds, errors)."""
    packed = np.ascontiguousarray(packed, dtype=np.uint16)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    nsys = packed.shape[0]
    assert packed.ndim == 3 and packed.shape[1] == num_procs and lens.shape == (nsys, num_procs)
    cfg = Cfg(num_procs, cache_size, max_instr or packed.shape[2], flags, nsys, 0, device, 0, 0)
    st = Stats()
    d = np.zeros(nsys, dtype=np.uint64)
    r = np.zeros(nsys, dtype=np.uint32)
    e = np.zeros(nsys, dtype=np.uint32)
    _check(lib().dash_run_host_batched(ctypes.byref(cfg), packed.ctypes.data, packed.shape[2], lens.ctypes.data,
                                       nsys, batches, ctypes.byref(st), d.ctypes.data, r.ctypes.data,
                                       e.ctypes.data), "dash_run_host_batched")
    return st.as_dict(), d, r, e


# ------------------------------------------------------------------ device engine

class Engine:
    """One batch of independent N-node systems on one GPU (a dash_t handle)."""

    def __init__(self, num_systems, num_procs=8, cache_size=4, max_instr=32, keep_state=False,
                 device=0, max_rounds=0, flags=0, trace_events=0, schedule_seed=0):
        self.cfg = Cfg(num_procs, cache_size, max_instr, (KEEP_STATE if keep_state else 0) | flags,
                       num_systems, max_rounds, device, trace_events, schedule_seed)
        self.h = ctypes.c_void_p()
        _check(lib().dash_create(ctypes.byref(self.cfg), ctypes.byref(self.h)), "dash_create")
        self.num_systems = num_systems
        self.num_procs = num_procs
        self.cache_size = cache_size

    def close(self):
        if self.h:
            lib().dash_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load_traces(self, packed: np.ndarray, lens: np.ndarray):
        """packed: [systems, num_procs, stride] u16; lens: [systems, num_procs] u32."""
        packed = np.ascontiguousarray(packed, dtype=np.uint16)
        lens = np.ascontiguousarray(lens, dtype=np.uint32)
        assert packed.ndim == 3 and packed.shape[:2] == (self.num_systems, self.num_procs)
        assert lens.shape == (self.num_systems, self.num_procs)
        _check(lib().dash_load_traces(self.h, packed.ctypes.data, packed.shape[2], lens.ctypes.data,
                                      self.num_systems), "dash_load_traces", self.h)

    def load_dir(self, test_dir):
        _check(lib().dash_load_dir(self.h, str(test_dir).encode(), 0), "dash_load_dir", self.h)

    def load_dirs(self, dirs):
        """Bulk ingest: system k = trace directory dirs[k]."""
        arr = (ctypes.c_char_p * max(len(dirs), 1))(*[str(d).encode() for d in dirs])
        _check(lib().dash_load_dirs(self.h, arr, len(dirs)), "dash_load_dirs", self.h)

    def dump_system(self, sys: int, out_dir):
        _check(lib().dash_dump_system(self.h, sys, str(out_dir).encode()), "dash_dump_system", self.h)

    def write_digests(self, path):
        _check(lib().dash_write_digests(self.h, str(path).encode()), "dash_write_digests", self.h)

    def generate(self, seed, length, kind=GEN_UNIFORM, locality=0, sys_base=0):
        g = Gen(seed, sys_base, kind, locality, length, 0)
        _check(lib().dash_generate(self.h, ctypes.byref(g)), "dash_generate", self.h)

    def set_schedule(self, sched: np.ndarray):
        """dash_set_schedule: an explicit round schedule, uint8 [rounds][num_procs] (SIT_OUT or
        the node's delivery position); later rounds are lockstep. Needs schedule_seed != 0."""
        sched = np.ascontiguousarray(sched, dtype=np.uint8)
        assert sched.ndim == 2 and sched.shape[1] == self.num_procs
        _check(lib().dash_set_schedule(self.h, sched.ctypes.data, sched.shape[0]), "dash_set_schedule", self.h)

    def set_micro_schedule(self, acts: np.ndarray):
        """dash_set_micro_schedule: uint8 [rounds][num_procs] of SIT_OUT / MICRO_STEP / MICRO_SEND,
        at most one acting node per round (include/dash.h). Needs schedule_seed != 0."""
        acts = np.ascontiguousarray(acts, dtype=np.uint8)
        assert acts.ndim == 2 and acts.shape[1] == self.num_procs
        _check(lib().dash_set_micro_schedule(self.h, acts.ctypes.data, acts.shape[0]), "dash_set_micro_schedule",
               self.h)

    def run(self) -> dict:
        st = Stats()
        _check(lib().dash_run(self.h, ctypes.byref(st)), "dash_run", self.h)
        return st.as_dict()

    def read_state(self, sys: int):
        arr = (NodeState * self.num_procs)()
        _check(lib().dash_read_state(self.h, sys, arr), "dash_read_state", self.h)
        return list(arr)

    def read_hist(self, sys: int) -> np.ndarray:
        h = np.zeros(NUM_TXN, dtype=np.uint32)
        _check(lib().dash_read_hist(self.h, sys, h.ctypes.data), "dash_read_hist", self.h)
        return h

    def read_results(self, first=0, count=None):
        count = self.num_systems - first if count is None else count
        d = np.zeros(count, dtype=np.uint64)
        r = np.zeros(count, dtype=np.uint32)
        e = np.zeros(count, dtype=np.uint32)
        _check(lib().dash_read_results(self.h, first, count, d.ctypes.data, r.ctypes.data,
                                       e.ctypes.data), "dash_read_results", self.h)
        return d, r, e

    def read_events(self, sys: int) -> list:
        """The system's DEBUG_MSG / DEBUG_INSTR events in lockstep order (needs trace_events)."""
        n = ctypes.c_uint32()
        # count first (cap 0), then read exactly that many: the log keeps trace_events rounded up to
        # a multiple of 4 rounds, so trace_events * num_procs can undercount it
        _check(lib().dash_read_events(self.h, sys, None, 0, ctypes.byref(n)), "dash_read_events", self.h)
        cap = n.value
        arr = (Event * max(cap, 1))()
        _check(lib().dash_read_events(self.h, sys, arr, cap, ctypes.byref(n)), "dash_read_events", self.h)
        return list(arr[:min(n.value, cap)])

    def stream(self) -> int:
        return int(lib().dash_stream(self.h) or 0)
