"""Host-code sanitizers (CPU only; GPU sanitizers are not available on this pool):
the C half of the boundary (csrc/dash_host.c: ingest, dump, digest, event
formatting) and the oracle (oracle/dash_oracle.c, including the legality
checker and the threaded batch mode) built with gcc -fsanitize=address,undefined
and driven over the reference's golden directories, 3000 fuzzed core_n.txt files
and 400 random systems (tools/host_sanitize.c). Any sanitizer report or check
failure fails the test."""
import os
import pathlib
import shutil
import subprocess

import pytest

from oracle_ctypes import GOLDEN

ROOT = pathlib.Path(__file__).resolve().parent.parent
DIRS = ["sample", "test_1", "test_2", "test_3", "test_4"]


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_host_code_under_asan_ubsan(tmp_path):
    exe = tmp_path / "host_sanitize"
    cmd = ["gcc", "-O1", "-g", "-std=c11", "-D_POSIX_C_SOURCE=200809L", "-fopenmp",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer",
           "-I", str(ROOT / "include"), "-I", str(ROOT / "oracle"),
           str(ROOT / "tools" / "host_sanitize.c"),
           str(ROOT / "ue22cs343bb1-openmp-assignment_amd" / "csrc" / "dash_host.c"),
           str(ROOT / "oracle" / "dash_oracle.c"), "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1",
               OMP_NUM_THREADS="2")
    scratch = tmp_path / "scratch"
    scratch.mkdir()
    p = subprocess.run([str(exe), str(scratch)] + [str(GOLDEN / d) for d in DIRS], capture_output=True,
                       text=True, timeout=600, env=env)
    assert p.returncode == 0, (p.stdout + p.stderr)[-4000:]
    assert "runtime error" not in p.stderr and "AddressSanitizer" not in p.stderr, p.stderr[-4000:]
    assert "host sanitizer run clean" in p.stdout
