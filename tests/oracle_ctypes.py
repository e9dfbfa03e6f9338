"""ctypes view of the CPU parity oracle (oracle/libdash_oracle.so).

TEST INFRASTRUCTURE: used only by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg. The trace parser here restates
initializeProcessor's accept rules (reference assignment.c:823-849) in Python
so the oracle's inputs never pass through the product's C ingest.
"""
from __future__ import annotations

import ctypes
import pathlib
import subprocess

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent.parent
ORACLE_DIR = ROOT / "oracle"
ORACLE_SO = ORACLE_DIR / "libdash_oracle.so"
GOLDEN = ROOT / "tests" / "golden" / "reference"

MAX_PROCS = 8
MEM = 16
MAX_CACHE = 16
NTXN = 13
ERR_OVERFLOW, ERR_OOB, ERR_CTZ0, ERR_DEADLOCK, ERR_ROUNDCAP, ERR_STUCK = 1, 2, 4, 8, 16, 32
TXN_NAMES = ["READ_REQUEST", "WRITE_REQUEST", "REPLY_RD", "REPLY_WR", "REPLY_ID", "INV",
             "UPGRADE", "WRITEBACK_INV", "WRITEBACK_INT", "FLUSH", "FLUSH_INVACK",
             "EVICT_SHARED", "EVICT_MODIFIED"]


class OrcCfg(ctypes.Structure):
    _fields_ = [("num_procs", ctypes.c_int), ("cache_size", ctypes.c_int),
                ("ring_depth", ctypes.c_int), ("max_rounds", ctypes.c_uint64),
                ("log_msgs", ctypes.c_int), ("_pad", ctypes.c_int), ("arb_seed", ctypes.c_uint64)]


class OrcNodeState(ctypes.Structure):
    _fields_ = [("memory", ctypes.c_uint8 * MEM), ("dir_bitvector", ctypes.c_uint8 * MEM),
                ("dir_state", ctypes.c_uint8 * MEM), ("cache_addr", ctypes.c_uint8 * MAX_CACHE),
                ("cache_value", ctypes.c_uint8 * MAX_CACHE),
                ("cache_state", ctypes.c_uint8 * MAX_CACHE)]


class OrcResult(ctypes.Structure):
    _fields_ = [("node", OrcNodeState * MAX_PROCS), ("hist", ctypes.c_uint64 * NTXN),
                ("rounds", ctypes.c_uint64), ("instructions", ctypes.c_uint64),
                ("errors", ctypes.c_uint32), ("dropped", ctypes.c_uint32),
                ("max_depth", ctypes.c_uint32), ("_pad", ctypes.c_uint32),
                ("digest", ctypes.c_uint64)]


class OrcGen(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64), ("kind", ctypes.c_uint32),
                ("locality", ctypes.c_uint32), ("len", ctypes.c_uint32),
                ("num_procs", ctypes.c_uint32)]


_lib = None


def bind(path):
    """ctypes binding of an oracle build (the checker, or a mutant of oracle/_mut/)."""
    L = ctypes.CDLL(str(path))
    L.orc_run_system.argtypes = [ctypes.POINTER(OrcCfg), ctypes.c_void_p, ctypes.c_uint64,
                                 ctypes.c_void_p, ctypes.POINTER(OrcResult),
                                 ctypes.c_char_p, ctypes.c_uint64]
    L.orc_run_system.restype = ctypes.c_int
    L.orc_gen_instr.argtypes = [ctypes.POINTER(OrcGen), ctypes.c_uint64, ctypes.c_uint32,
                                ctypes.c_uint32]
    L.orc_gen_instr.restype = ctypes.c_uint16
    L.orc_gen_system.argtypes = [ctypes.POINTER(OrcGen), ctypes.c_uint64, ctypes.c_void_p,
                                 ctypes.c_uint64]
    L.orc_run_batch.argtypes = [ctypes.POINTER(OrcCfg), ctypes.POINTER(OrcGen),
                                ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                                ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                ctypes.c_void_p, ctypes.c_void_p]
    L.orc_run_batch.restype = ctypes.c_double
    L.orc_dump_node.argtypes = [ctypes.POINTER(OrcNodeState), ctypes.c_int, ctypes.c_int,
                                ctypes.c_char_p, ctypes.c_int]
    L.orc_dump_node.restype = ctypes.c_int
    V, U64 = ctypes.c_void_p, ctypes.c_uint64
    L.orc_replay_lockstep.argtypes = [ctypes.POINTER(OrcCfg), V, U64, V, V, V]
    L.orc_random_schedule.argtypes = [ctypes.POINTER(OrcCfg), V, U64, V, U64, V]
    L.orc_explore.argtypes = [ctypes.POINTER(OrcCfg), V, U64, V, U64, V, ctypes.c_int, V, V, V]
    for f in (L.orc_replay_lockstep, L.orc_random_schedule, L.orc_explore):
        f.restype = ctypes.c_int
    return L


def lib():
    global _lib
    if _lib is None:
        if not ORACLE_SO.exists():
            subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)
        _lib = bind(ORACLE_SO)
    return _lib


# ---------------------------------------------------------------- traces

def pack(kind: str, address: int, value: int) -> int:
    """Packed instruction: bit15 = WR, bits 14..8 = address, bits 7..0 = value."""
    return ((1 if kind == "W" else 0) << 15) | ((address & 0x7F) << 8) | (value & 0xFF)


def parse_core_file(path, max_instr=32):
    """initializeProcessor's parse loop (assignment.c:831-847) for well-formed
    input: fgets(line[20]) chunks, `RD %hhx` / `WR %hhx %hhu`, at most
    max_instr lines. Lines the reference would turn into an uninitialised
    instruction raise ValueError."""
    data = pathlib.Path(path).read_bytes()
    out = []
    pos = 0
    while pos < len(data) and len(out) < max_instr:
        nl = data.find(b"\n", pos)
        end = len(data) if nl < 0 else nl + 1
        end = min(end, pos + 19)  # fgets(line, 20): at most 19 bytes per call
        line = data[pos:end].decode("ascii")
        pos = end
        toks = line.split()
        if line.startswith("RD") and len(toks) >= 2:
            out.append(pack("R", int(toks[1], 16) & 0xFF, 0))
        elif line.startswith("WR") and len(toks) >= 3:
            out.append(pack("W", int(toks[1], 16) & 0xFF, int(toks[2]) & 0xFF))
        else:
            raise ValueError(f"{path}: line {line!r} is not RD/WR")
    return out


def load_test_dir(d, num_procs=4, max_instr=32):
    rows = [parse_core_file(pathlib.Path(d) / f"core_{n}.txt", max_instr) for n in range(num_procs)]
    L = max([len(r) for r in rows] + [1])
    tr = np.zeros((num_procs, L), dtype=np.uint16)
    lens = np.zeros(num_procs, dtype=np.uint32)
    for n, r in enumerate(rows):
        tr[n, :len(r)] = r
        lens[n] = len(r)
    return tr, lens


# ---------------------------------------------------------------- runs

def run_system(trace, lens, num_procs=4, cache_size=4, ring_depth=256, max_rounds=0, log=False,
               log_msgs=False, arb_seed=0):
    """log=True also returns the DEBUG_INSTR lines (plus DEBUG_MSG lines with
    log_msgs=True) in lockstep order (round, then node)."""
    trace = np.ascontiguousarray(trace, dtype=np.uint16)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    cfg = OrcCfg(num_procs, cache_size, ring_depth, max_rounds, 1 if log_msgs else 0, 0, arb_seed)
    res = OrcResult()
    buf = ctypes.create_string_buffer(1 << 20) if log else None
    rc = lib().orc_run_system(ctypes.byref(cfg), trace.ctypes.data, trace.shape[1],
                              lens.ctypes.data, ctypes.byref(res), buf, (1 << 20) if log else 0)
    if rc != 0:
        raise ValueError("oracle rejected the configuration or trace")
    return (res, buf.value.decode()) if log else res


class OrcOutcome(ctypes.Structure):
    _fields_ = [("node", OrcNodeState * MAX_PROCS), ("digest", ctypes.c_uint64),
                ("errors", ctypes.c_uint32), ("_pad", ctypes.c_uint32)]


def _tr(trace, lens):
    return (np.ascontiguousarray(trace, dtype=np.uint16), np.ascontiguousarray(lens, dtype=np.uint32))


def replay_lockstep(trace, lens, num_procs=4, cache_size=4):
    """The lockstep schedule as race-free micro-steps (legality checker)."""
    trace, lens = _tr(trace, lens)
    cfg = OrcCfg(num_procs, cache_size, 256, 0)
    out = OrcOutcome()
    steps = ctypes.c_uint64()
    rc = lib().orc_replay_lockstep(ctypes.byref(cfg), trace.ctypes.data, trace.shape[1], lens.ctypes.data,
                                   ctypes.addressof(out), ctypes.addressof(steps))
    if rc != 0:
        raise ValueError(f"lockstep replay failed ({rc})")
    return out, int(steps.value)


def random_schedule(trace, lens, seed, num_procs=4, cache_size=4):
    """Final state of one uniformly random legal micro-step schedule."""
    trace, lens = _tr(trace, lens)
    cfg = OrcCfg(num_procs, cache_size, 256, 0)
    out = OrcOutcome()
    if lib().orc_random_schedule(ctypes.byref(cfg), trace.ctypes.data, trace.shape[1], lens.ctypes.data,
                                 seed, ctypes.addressof(out)) != 0:
        raise ValueError("random schedule failed")
    return out


def explore(trace, lens, num_procs=4, cache_size=4, max_states=1_000_000, max_outs=4096, L=None):
    """Exhaustive search of the race-free micro-step model (pop-first persistent
    sets). Returns (distinct outcomes, states visited, complete). `L`: another oracle
    build (bind()), e.g. a mutant."""
    trace, lens = _tr(trace, lens)
    L = L or lib()
    cfg = OrcCfg(num_procs, cache_size, 256, 0)
    outs = (OrcOutcome * max_outs)()
    n = ctypes.c_int()
    states = ctypes.c_uint64()
    full = ctypes.c_int()
    rc = L.orc_explore(ctypes.byref(cfg), trace.ctypes.data, trace.shape[1], lens.ctypes.data,
                           max_states, ctypes.addressof(outs), max_outs, ctypes.addressof(n),
                           ctypes.addressof(states), ctypes.addressof(full))
    if rc != 0:
        raise ValueError("explore failed")
    # more distinct outcomes than max_outs: the list is cut, so the set is not complete
    return [outs[k] for k in range(min(n.value, max_outs))], int(states.value), bool(full.value) and n.value <= max_outs


def dump_node(res, node, cache_size=4, L=None) -> str:
    buf = ctypes.create_string_buffer(8192)
    n = (L or lib()).orc_dump_node(ctypes.byref(res.node[node]), node, cache_size, buf, 8192)
    return buf.raw[:n].decode()


def gen_system(seed, sys, num_procs=8, length=64, kind=0, locality=0):
    g = OrcGen(seed, kind, locality, length, num_procs)
    tr = np.zeros((num_procs, length), dtype=np.uint16)
    lib().orc_gen_system(ctypes.byref(g), sys, tr.ctypes.data, length)
    return tr


def run_batch(seed, first, count, num_procs=8, cache_size=4, length=64, kind=0, locality=0,
              ring_depth=256, threads=1, max_rounds=0):
    cfg = OrcCfg(num_procs, cache_size, ring_depth, max_rounds)
    g = OrcGen(seed, kind, locality, length, num_procs)
    dig = np.zeros(count, dtype=np.uint64)
    rnd = np.zeros(count, dtype=np.uint32)
    err = np.zeros(count, dtype=np.uint32)
    hist = np.zeros(NTXN, dtype=np.uint64)
    instr = np.zeros(1, dtype=np.uint64)
    secs = lib().orc_run_batch(ctypes.byref(cfg), ctypes.byref(g), first, count, threads,
                               dig.ctypes.data, rnd.ctypes.data, err.ctypes.data,
                               hist.ctypes.data, instr.ctypes.data)
    return dict(digests=dig, rounds=rnd, errors=err, hist=hist, instructions=int(instr[0]),
                seconds=secs)
