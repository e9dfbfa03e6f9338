"""CPU-only checks of the C-ABI library: it loads, exports every symbol
include/dash.h declares, and its host-side boundary (trace ingest, dump,
digest) agrees with the oracle and the reference's fixtures. No device call
is made here."""
import ctypes
import pathlib
import re
import subprocess

import numpy as np
import pytest

from oracle_ctypes import GOLDEN, dump_node as orc_dump, load_test_dir, parse_core_file, run_system

ROOT = pathlib.Path(__file__).resolve().parent.parent
TESTS = ["sample", "test_1", "test_2", "test_3", "test_4"]


def declared_symbols():
    hdr = (ROOT / "include" / "dash.h").read_text()
    return sorted(set(re.findall(r"^\s*(?:[\w\s\*]+?)\b(dash_\w+)\s*\(", hdr, re.M)))


def test_header_and_module_agree(dash):
    assert declared_symbols() == sorted(dash.EXPORTS)


def test_library_exports_every_symbol(dash):
    lib = dash.lib()
    for name in declared_symbols():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", str(dash.LIB_PATH)], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\sT\s(dash_\w+)", out))
    assert set(declared_symbols()) <= exported


@pytest.mark.parametrize("test", TESTS)
def test_ingest_matches_reference_parse(dash, test):
    for n in range(4):
        path = GOLDEN / test / f"core_{n}.txt"
        got = dash.parse_core_file(path, 4, 32)
        assert got.tolist() == parse_core_file(path, 32)


def test_ingest_rules(dash, tmp_path):
    f = tmp_path / "core_0.txt"
    f.write_text("WR 0x15 300\nRD 17\nWR 0x3f 7\n")
    # %hhu wraps mod 256; %hhx without prefix; lower-case hex
    assert dash.parse_core_file(f, 4, 32).tolist() == [0x8000 | 0x15 << 8 | 44, 0x17 << 8,
                                                       0x8000 | 0x3F << 8 | 7]
    f.write_text("RD 0x05\n\nRD 0x06\n")  # blank line = garbage instruction in the reference
    with pytest.raises(dash.DashError) as e:
        dash.parse_core_file(f, 4, 32)
    assert e.value.code == dash.EPARSE
    f.write_text("RD 0x50\n")  # node 5 does not exist with NUM_PROCS 4
    with pytest.raises(dash.DashError) as e:
        dash.parse_core_file(f, 4, 32)
    assert e.value.code == dash.EADDR
    f.write_text("".join(f"RD 0x{i % 16:02X}\n" for i in range(40)))
    assert len(dash.parse_core_file(f, 4, 32)) == 32  # MAX_INSTR_NUM cap (ref :834)
    with pytest.raises(dash.DashError) as e:
        dash.parse_core_file(tmp_path / "missing.txt", 4, 32)
    assert e.value.code == dash.EIO


def to_dash_state(dash, res, n, cs):
    s = dash.NodeState()
    o = res.node[n]
    for b in range(16):
        s.memory[b] = o.memory[b]
        s.dir_bitvector[b] = o.dir_bitvector[b]
        s.dir_state[b] = o.dir_state[b]
    for i in range(cs):
        s.cache_addr[i] = o.cache_addr[i]
        s.cache_value[i] = o.cache_value[i]
        s.cache_state[i] = o.cache_state[i]
    return s


@pytest.mark.parametrize("test", TESTS)
def test_dump_and_digest_match_oracle(dash, test):
    tr, lens = load_test_dir(GOLDEN / test)
    res = run_system(tr, lens)
    for n in range(4):
        s = to_dash_state(dash, res, n, 4)
        assert dash.dump_node(s, n, 4) == orc_dump(res, n, 4)
    import oracle_ctypes
    lib = oracle_ctypes.lib()
    lib.orc_digest_node.restype = ctypes.c_uint64
    for n in range(4):
        s = to_dash_state(dash, res, n, 4)
        assert dash.digest_node(s, n, 4) == lib.orc_digest_node(ctypes.byref(res.node[n]), n, 4)


def test_initial_state_dump(dash):
    s = dash.init_node_state(2, 4)
    txt = dash.dump_node(s, 2, 4)
    assert "|    5  |  0x25   |     45   |" in txt
    assert txt.count("   INVALID \t|") == 4
    assert txt.count("  U   |   0x00000000   |") == 16


def test_resolve_dir(dash, tmp_path, monkeypatch):
    (tmp_path / "tests" / "t1").mkdir(parents=True)
    (tmp_path / "tests" / "t1" / "core_0.txt").write_text("RD 0x00\n")
    monkeypatch.chdir(tmp_path)
    buf = ctypes.create_string_buffer(256)
    assert dash.lib().dash_resolve_dir(b"t1", buf, 256) == 0 and buf.value == b"tests/t1"
    assert dash.lib().dash_resolve_dir(b"tests/t1", buf, 256) == 0 and buf.value == b"tests/t1"
    assert dash.lib().dash_resolve_dir(b"nope", buf, 256) == dash.EIO


def test_bench_next_trace_text_round_trips(dash, tmp_path):
    """bench.py --next writes its ingest workload as core_<n>.txt text (bench_next.trace_text);
    the library's parser (the reference's fgets + sscanf rules) must read back the same words,
    RD values as 0 (ref :839)."""
    import sys
    sys.path.insert(0, str(pathlib.Path(__file__).resolve().parent.parent))
    import bench_next
    rng = np.random.default_rng(11)
    w = rng.bit_generator.random_raw(1024).view(np.uint16).copy()
    w[:3] = [0x8000, 0x80FF, 0x7F00 | 0x55]  # WR 0x00 0, WR 0x00 255, RD 0x7F (value dropped)
    f = tmp_path / "core_0.txt"
    f.write_bytes(bench_next.trace_text(w))
    assert f.read_text().splitlines()[:3] == ["WR 0x00 0", "WR 0x00 255", "RD 0x7F"]
    got = dash.parse_core_file(f, num_procs=8, max_instr=len(w))
    assert np.array_equal(got, np.where(w & 0x8000, w, w & 0xFF00).astype(np.uint16))


def test_create_error_message_describes_this_call(dash, tmp_path):
    """dash_last_error(NULL) after a failed dash_create names that call's own
    problem, not an older handle-less failure (no device call: num_procs is checked first)."""
    with pytest.raises(dash.DashError):
        dash.simulate_dir(tmp_path / "missing")  # leaves a message behind
    with pytest.raises(dash.DashError) as e:
        dash.Engine(4, num_procs=9)
    assert "num_procs" in str(e.value) and e.value.code == dash.EINVAL
    with pytest.raises(dash.DashError) as e:
        dash.Engine(4, num_procs=8, cache_size=17)
    assert "cache_size" in str(e.value)


def test_cli_refuses_conflicting_or_empty_schedules(dash, tmp_path):
    """`--rounds` with `--micro` is refused (one would be dropped silently), and so is
    an empty micro-step schedule (it would fall through to a plain lockstep run). Both are
    argument errors reported before the GPU is touched."""
    import shutil
    import subprocess
    exe = dash.PKG / "cache_simulator"
    (tmp_path / "tests").mkdir()
    shutil.copytree(GOLDEN / "test_4", tmp_path / "tests" / "test_4")
    (tmp_path / "empty.txt").write_text("\n")
    (tmp_path / "one.txt").write_text("P0\n")
    (tmp_path / "r.txt").write_text("0123\n")
    p = subprocess.run([str(exe), "test_4", "--rounds", "r.txt", "--micro", "one.txt"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=60)
    assert p.returncode == 1 and "exclusive" in p.stderr
    p = subprocess.run([str(exe), "test_4", "--micro", "empty.txt"], cwd=tmp_path, capture_output=True, text=True,
                       timeout=60)
    assert p.returncode == 1 and "empty micro-step schedule" in p.stderr
    assert not (tmp_path / "core_0_output.txt").exists()
