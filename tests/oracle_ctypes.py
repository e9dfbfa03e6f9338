"""ctypes view of the CPU parity oracle (oracle/libdash_oracle.so).

TEST INFRASTRUCTURE: used only by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg. The trace parser here restates
initializeProcessor's accept rules (reference assignment.c:823-849) in Python
so the oracle's inputs never pass through the product's C ingest.
"""
from __future__ import annotations

import ctypes
import pathlib
import re
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
                ("log_msgs", ctypes.c_int), ("micro", ctypes.c_int), ("arb_seed", ctypes.c_uint64),
                ("sched", ctypes.c_void_p), ("sched_rounds", ctypes.c_uint32), ("count_msgs", ctypes.c_int)]


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
    I = ctypes.c_int
    L.orc_reach.argtypes = [ctypes.POINTER(OrcCfg), V, U64, V, I, V, I, U64, V, U64, V, V,
                            ctypes.c_uint32, V, V, V, V]
    L.orc_random_walk.argtypes = [ctypes.POINTER(OrcCfg), V, U64, V, I, U64, V, V, V, V,
                                  ctypes.c_uint32, V]
    L.orc_replay_steps.argtypes = [ctypes.POINTER(OrcCfg), V, U64, V, I, V, ctypes.c_uint32, V, V]
    L.orc_guided.argtypes = [ctypes.POINTER(OrcCfg), V, U64, V, V, V, U64, V, V, V, V]
    L.orc_guided.restype = ctypes.c_int
    L.orc_guided_witness.argtypes = [ctypes.POINTER(OrcCfg), V, U64, V, V, V, U64, V, V, V, V, ctypes.c_uint32, V]
    L.orc_guided_witness.restype = ctypes.c_int
    L.orc_rounds_from_logs.argtypes = [ctypes.POINTER(OrcCfg), V, U64, V, V, V, U64, V, ctypes.c_uint32, V, V, V]
    L.orc_rounds_from_logs.restype = ctypes.c_int
    L.orc_schedule_witness.argtypes = [ctypes.POINTER(OrcCfg), V, U64, V, V, ctypes.c_uint32, V, V]
    for f in (L.orc_replay_lockstep, L.orc_random_schedule, L.orc_explore, L.orc_reach,
              L.orc_random_walk, L.orc_replay_steps, L.orc_schedule_witness):
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
               log_msgs=False, arb_seed=0, sched=None, log_bytes=1 << 20):
    """log=True also returns the DEBUG_INSTR lines (plus DEBUG_MSG lines with
    log_msgs=True) in lockstep order (round, then node). sched: an explicit round schedule
    (uint8 [rounds][num_procs], 0xFF = sits out, else delivery position), the twin of
    dash_set_schedule."""
    trace = np.ascontiguousarray(trace, dtype=np.uint16)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    cfg = OrcCfg(num_procs, cache_size, ring_depth, max_rounds, 1 if log_msgs else 0, 0, arb_seed)
    if sched is not None:
        sched = np.ascontiguousarray(sched, dtype=np.uint8)
        assert sched.ndim == 2 and sched.shape[1] == num_procs
        cfg.sched, cfg.sched_rounds = sched.ctypes.data, sched.shape[0]
    res = OrcResult()
    buf = ctypes.create_string_buffer(log_bytes) if log else None
    rc = lib().orc_run_system(ctypes.byref(cfg), trace.ctypes.data, trace.shape[1],
                              lens.ctypes.data, ctypes.byref(res), buf, log_bytes if log else 0)
    if rc != 0:
        raise ValueError("oracle rejected the configuration or trace")
    if log and len(buf.value) + 64 >= log_bytes:  # the oracle stops logging 64 B before the end
        raise ValueError(f"oracle log longer than log_bytes={log_bytes}: pass a larger buffer")
    return (res, buf.value.decode()) if log else res


class OrcOutcome(ctypes.Structure):
    _fields_ = [("node", OrcNodeState * MAX_PROCS), ("digest", ctypes.c_uint64),
                ("errors", ctypes.c_uint32), ("_pad", ctypes.c_uint32),
                ("hist", ctypes.c_uint32 * NTXN), ("_pad2", ctypes.c_uint32)]


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


def explore(trace, lens, num_procs=4, cache_size=4, max_states=1_000_000, max_outs=4096, L=None,
            micro=0, count_msgs=False):
    """Exhaustive search of the race-free micro-step model (pop-first persistent
    sets; micro = MICRO_BUFFERED or MICRO_STRICT). Returns (distinct outcomes, states
    visited, complete). `L`: another oracle build (bind()), e.g. a mutant."""
    trace, lens = _tr(trace, lens)
    L = L or lib()
    cfg = OrcCfg(num_procs, cache_size, 256, 0, 0, micro, 0)
    cfg.count_msgs = 1 if count_msgs else 0
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


MICRO_BUFFERED, MICRO_STRICT, MICRO_RACE = 0, 1, 2
STEP_KINDS = ["POP", "ISSUE", "SEND", "RACE"]


def step_str(w: int) -> str:
    """A witness step as a token: P<t> (POP), I<t> (ISSUE), S<t> (SEND), R<s>><t> (RACE: t
    pops while s's append to t loses its count++)."""
    k, aux, t = w >> 8, (w >> 4) & 15, w & 15
    return f"R{aux}>{t}" if k == 3 else f"{STEP_KINDS[k][0]}{t}"


def step_parse(tok: str) -> int:
    k = "PISR".index(tok[0])
    if k == 3:
        a, t = tok[1:].split(">")
        return (3 << 8) | (int(a) << 4) | int(t)
    return (k << 8) | int(tok[1:])


def reach(trace, lens, targets, num_procs=4, cache_size=4, micro=MICRO_STRICT, race_max=0,
          max_states=10_000_000, prio=None, order_seed=0, wit_cap=1 << 16, L=None, count_msgs=False,
          all_targets=False):
    """Goal-directed DFS (orc_reach). Returns (hit index or -1, witness steps, states, complete);
    with all_targets=True the first item is the list of found flags, one per target."""
    trace, lens = _tr(trace, lens)
    L = L or lib()
    cfg = OrcCfg(num_procs, cache_size, 256, 0, 0, micro, 0)
    cfg.count_msgs = 1 if count_msgs else 0
    tg = np.ascontiguousarray(targets, dtype=np.uint64)
    flags = np.zeros(max(len(tg), 1), np.int32) if all_targets else None
    pr = None if prio is None else np.ascontiguousarray(prio, dtype=np.uint8)
    wit = np.zeros(wit_cap, np.uint16)
    hit, wl, states, full = ctypes.c_int(), ctypes.c_uint32(), ctypes.c_uint64(), ctypes.c_int()
    rc = L.orc_reach(ctypes.byref(cfg), trace.ctypes.data, trace.shape[1], lens.ctypes.data, race_max,
                     tg.ctypes.data, len(tg), max_states, None if pr is None else pr.ctypes.data,
                     order_seed, ctypes.addressof(hit), wit.ctypes.data, wit_cap, ctypes.addressof(wl),
                     ctypes.addressof(states), ctypes.addressof(full),
                     None if flags is None else flags.ctypes.data)
    if rc != 0:
        raise ValueError(f"reach failed ({rc})")
    first = [bool(f) for f in flags[:len(tg)]] if all_targets else hit.value
    return first, [int(w) for w in wit[:wl.value]], int(states.value), bool(full.value)


def random_walk(trace, lens, seed, weights=None, num_procs=4, cache_size=4, micro=MICRO_STRICT,
                race_max=0, wit_cap=1 << 16, count_msgs=False, L=None, kind_weights=None):
    """One weighted random legal schedule and its witness: (outcome, steps). weights: per node;
    kind_weights: per step kind (POP, ISSUE, SEND, RACE)."""
    trace, lens = _tr(trace, lens)
    cfg = OrcCfg(num_procs, cache_size, 256, 0, 0, micro, 0)
    cfg.count_msgs = 1 if count_msgs else 0
    w = None if weights is None else np.ascontiguousarray(weights, dtype=np.uint32)
    kw = None if kind_weights is None else np.ascontiguousarray(kind_weights, dtype=np.uint32)
    out = OrcOutcome()
    wit = np.zeros(wit_cap, np.uint16)
    wl = ctypes.c_uint32()
    rc = (L or lib()).orc_random_walk(ctypes.byref(cfg), trace.ctypes.data, trace.shape[1], lens.ctypes.data,
                               race_max, seed, None if w is None else w.ctypes.data,
                               None if kw is None else kw.ctypes.data, ctypes.addressof(out), wit.ctypes.data, wit_cap, ctypes.addressof(wl))
    if rc != 0:
        raise ValueError(f"random walk failed ({rc})")
    return out, [int(x) for x in wit[:wl.value]]


def replay_steps(trace, lens, steps, num_procs=4, cache_size=4, micro=MICRO_STRICT, race_max=0,
                 count_msgs=False):
    """Re-execute a witness: (outcome, terminal). Raises if a step is not enabled."""
    trace, lens = _tr(trace, lens)
    cfg = OrcCfg(num_procs, cache_size, 256, 0, 0, micro, 0)
    cfg.count_msgs = 1 if count_msgs else 0
    st = np.ascontiguousarray(steps, dtype=np.uint16)
    out = OrcOutcome()
    term = ctypes.c_int()
    rc = lib().orc_replay_steps(ctypes.byref(cfg), trace.ctypes.data, trace.shape[1], lens.ctypes.data,
                                race_max, st.ctypes.data, len(st), ctypes.addressof(out),
                                ctypes.addressof(term))
    if rc != 0:
        raise ValueError(f"witness step {-rc - 1} is not enabled" if rc < -1 else "replay failed")
    return out, bool(term.value)


LOG_MSG = re.compile(r"Processor (\d+) msg from: (\d+), type: (\d+), address: 0x([0-9A-Fa-f]{2})")
LOG_INSTR = re.compile(r"Processor (\d+): instr type=([RW]), address=0x([0-9A-Fa-f]{2}), value=(\d+)")


def parse_logs(text: str, num_procs: int):
    """A reference run's -DDEBUG_MSG / -DDEBUG_INSTR lines (assignment.c:179-182, :649-652) as
    per-node event words for orc_guided (each thread's lines keep its program order)."""
    ev = [[] for _ in range(num_procs)]
    instr = [[] for _ in range(num_procs)]
    for line in text.splitlines():
        m = LOG_MSG.match(line)
        if m:
            t, snd, typ, a = int(m[1]), int(m[2]), int(m[3]), int(m[4], 16)
            ev[t].append(typ | (snd << 8) | (a << 16))
            continue
        m = LOG_INSTR.match(line)
        if m:
            t = int(m[1])
            ev[t].append(1 << 31)
            instr[t].append(pack(m[2], int(m[3], 16), int(m[4])))
    return ev, instr


def guided(trace, lens, events, num_procs=4, cache_size=4, max_states=2_000_000, L=None):
    """orc_guided: (found, outcome, states, complete) for per-node event lists."""
    trace, lens = _tr(trace, lens)
    cfg = OrcCfg(num_procs, cache_size, 256, 0, 0, MICRO_STRICT, 0)
    flat = np.ascontiguousarray([w for e in events for w in e] or [0], dtype=np.uint32)
    cnt = np.ascontiguousarray([len(e) for e in events], dtype=np.uint32)
    out = OrcOutcome()
    found, states, full = ctypes.c_int(), ctypes.c_uint64(), ctypes.c_int()
    rc = (L or lib()).orc_guided(ctypes.byref(cfg), trace.ctypes.data, trace.shape[1], lens.ctypes.data,
                                 flat.ctypes.data, cnt.ctypes.data, max_states, ctypes.addressof(found),
                                 ctypes.addressof(out), ctypes.addressof(states), ctypes.addressof(full))
    if rc != 0:
        raise ValueError(f"guided search failed ({rc})")
    return bool(found.value), out, int(states.value), bool(full.value)


def guided_witness(trace, lens, events, num_procs=4, cache_size=4, max_states=2_000_000, cap=1 << 16):
    """orc_guided_witness: (found, outcome, steps uint16) -- the micro-step interleaving (XSTEP
    words: pop / issue / one send of a node) under which the nodes' logs are met."""
    trace, lens = _tr(trace, lens)
    cfg = OrcCfg(num_procs, cache_size, 256, 0, 0, MICRO_STRICT, 0)
    flat = np.ascontiguousarray([w for e in events for w in e] or [0], dtype=np.uint32)
    cnt = np.ascontiguousarray([len(e) for e in events], dtype=np.uint32)
    out = OrcOutcome()
    found, states, n = ctypes.c_int(), ctypes.c_uint64(), ctypes.c_uint32()
    wit = np.zeros(cap, np.uint16)
    rc = lib().orc_guided_witness(ctypes.byref(cfg), trace.ctypes.data, trace.shape[1], lens.ctypes.data,
                                  flat.ctypes.data, cnt.ctypes.data, max_states, ctypes.addressof(found),
                                  ctypes.addressof(out), ctypes.addressof(states), wit.ctypes.data, cap,
                                  ctypes.addressof(n))
    if rc != 0:
        raise ValueError(f"guided witness search failed ({rc})")
    return bool(found.value), out, wit[:n.value].copy()


def rounds_from_logs(trace, lens, events, num_procs=4, cache_size=4, max_states=500_000, cap=4096):
    """orc_rounds_from_logs: (engine round schedule uint8 [rounds][num_procs] or None, states)."""
    trace, lens = _tr(trace, lens)
    cfg = OrcCfg(num_procs, cache_size, 256, 0, 0, MICRO_STRICT, 0)
    flat = np.ascontiguousarray([w for e in events for w in e] or [0], dtype=np.uint32)
    cnt = np.ascontiguousarray([len(e) for e in events], dtype=np.uint32)
    out = np.zeros((cap, num_procs), np.uint8)
    nr, found, states = ctypes.c_uint32(), ctypes.c_int(), ctypes.c_uint64()
    rc = lib().orc_rounds_from_logs(ctypes.byref(cfg), trace.ctypes.data, trace.shape[1], lens.ctypes.data,
                                    flat.ctypes.data, cnt.ctypes.data, max_states, out.ctypes.data, cap,
                                    ctypes.addressof(nr), ctypes.addressof(found), ctypes.addressof(states))
    if rc != 0:
        raise ValueError(f"rounds_from_logs failed ({rc})")
    return (out[:nr.value].copy() if found.value else None), int(states.value)


def schedule_witness(trace, lens, num_procs=4, cache_size=4, arb_seed=0, sched=None,
                     micro=MICRO_STRICT, wit_cap=1 << 16):
    """The engine's schedule (lockstep / seeded / explicit) as a micro-step witness, every step
    checked enabled in `micro`: (outcome, steps)."""
    trace, lens = _tr(trace, lens)
    cfg = OrcCfg(num_procs, cache_size, 256, 0, 0, micro, arb_seed)
    if sched is not None:
        sched = np.ascontiguousarray(sched, dtype=np.uint8)
        cfg.sched, cfg.sched_rounds = sched.ctypes.data, sched.shape[0]
    out = OrcOutcome()
    wit = np.zeros(wit_cap, np.uint16)
    wl = ctypes.c_uint32()
    rc = lib().orc_schedule_witness(ctypes.byref(cfg), trace.ctypes.data, trace.shape[1], lens.ctypes.data,
                                    wit.ctypes.data, wit_cap, ctypes.addressof(wl), ctypes.addressof(out))
    if rc != 0:
        raise ValueError(f"schedule witness failed ({rc})")
    return out, [int(x) for x in wit[:wl.value]]


def dump_node(res, node, cache_size=4, L=None) -> str:
    buf = ctypes.create_string_buffer(8192)
    n = (L or lib()).orc_dump_node(ctypes.byref(res.node[node]), node, cache_size, buf, 8192)
    return buf.raw[:n].decode()


def parse_dump(text: str, node: int, cache_size=4) -> OrcNodeState:
    """A printProcessorState dump (assignment.c:853-905) back into a node state, so the
    reference's own run_k outputs can be targets of the reachability search."""
    st = OrcNodeState()
    dstate = {"EM": 0, "S": 1, "U": 2}
    cstate = {"MODIFIED": 0, "EXCLUSIVE": 1, "SHARED": 2, "INVALID": 3}
    rows = [ln.strip().strip("|").split("|") for ln in text.splitlines()
            if ln.startswith("|  ") and "Index" not in ln]
    if len(rows) != 32 + cache_size:
        raise ValueError(f"dump has {len(rows)} table rows")
    for i, r in enumerate(rows[:16]):
        assert int(r[0]) == i and int(r[1], 16) == (node << 4) + i
        st.memory[i] = int(r[2])
    for i, r in enumerate(rows[16:32]):
        st.dir_state[i] = dstate[r[2].strip()]
        st.dir_bitvector[i] = int(r[3].strip()[2:], 2)
    for i, r in enumerate(rows[32:]):
        st.cache_addr[i] = int(r[1], 16)
        st.cache_value[i] = int(r[2])
        st.cache_state[i] = cstate[r[3].strip()]
    return st


def _fmix(k):
    M = (1 << 64) - 1
    k ^= k >> 33
    k = (k * 0xff51afd7ed558ccd) & M
    k ^= k >> 33
    k = (k * 0xc4ceb9fe1a85ec53) & M
    return k ^ (k >> 33)


def outcome_key(digest: int, hist) -> int:
    """An outcome digest folded with its per-type handled-message counts (cfg.count_msgs)."""
    hk = 0x452821E638D01377
    for k, v in enumerate(hist):
        hk = _fmix(hk ^ ((k << 32) | int(v)))
    return _fmix(digest ^ hk)


def dumps_digest(texts, cache_size=4) -> int:
    """The system digest of a set of per-node dumps."""
    d = 0x9E3779B97F4A7C15
    M = (1 << 64) - 1

    def fmix(k):
        k ^= k >> 33
        k = (k * 0xff51afd7ed558ccd) & M
        k ^= k >> 33
        k = (k * 0xc4ceb9fe1a85ec53) & M
        return k ^ (k >> 33)
    L = lib()
    L.orc_digest_node.argtypes = [ctypes.POINTER(OrcNodeState), ctypes.c_int, ctypes.c_int]
    L.orc_digest_node.restype = ctypes.c_uint64
    for n, t in enumerate(texts):
        st = parse_dump(t, n, cache_size)
        d = fmix(d ^ L.orc_digest_node(ctypes.byref(st), n, cache_size))
    return d


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
