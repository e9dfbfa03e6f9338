"""INTEGRATION.md's code is what a maintainer copies, so it is built and run here.

* CPU: the §1 drop-in main() (assignment.c's main with the OpenMP region replaced, ref
  :126-155, :853-905) and the §2 many-systems snippet compile and link against
  include/dash.h and the built libdash.so with plain gcc; the §3 ctypes stub names an
  exported symbol.
* GPU: the §1 program runs the reference's `sample` fixture with the reference's argv
  contract and writes byte-identical core_<n>_output.txt dumps; the §3 stub writes the same.
"""
import ctypes
import pathlib
import re
import shutil
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
PKG = ROOT / "ue22cs343bb1-openmp-assignment_amd"
LIB = PKG / "libdash.so"
DOC = (ROOT / "INTEGRATION.md").read_text()
GOLDEN = ROOT / "tests" / "golden" / "reference"


def blocks(lang):
    return re.findall(r"```" + lang + r"\n(.*?)```", DOC, flags=re.S)


def build_main(tmp_path):
    if not LIB.exists():
        pytest.skip("libdash.so not built (run __graft_entry__.build())")
    src = tmp_path / "assignment_gpu.c"
    src.write_text(blocks("c")[0])
    exe = tmp_path / "cache_simulator_gpu"
    subprocess.run(["gcc", "-O2", "-Wall", "-Werror", f"-I{ROOT / 'include'}", "-o", str(exe), str(src),
                    f"-L{PKG}", "-ldash", f"-Wl,-rpath,{PKG}"], check=True, capture_output=True, text=True)
    return exe


def test_drop_in_main_compiles_and_links(tmp_path):
    assert build_main(tmp_path).exists()


def test_many_systems_snippet_compiles(tmp_path):
    body = blocks("c")[1]
    src = tmp_path / "batch.c"
    src.write_text("#include <stdint.h>\n#include <stdlib.h>\n#include \"dash.h\"\n"
                   "int main(void) {\n" + body + "    free(dig);\n    dash_destroy(h);\n    return 0;\n}\n")
    subprocess.run(["gcc", "-O2", "-Wall", "-Werror", f"-I{ROOT / 'include'}", "-c", "-o",
                    str(tmp_path / "batch.o"), str(src)], check=True, capture_output=True, text=True)


def test_ctypes_stub_names_an_export():
    if not LIB.exists():
        pytest.skip("libdash.so not built")
    stub = blocks("python")[0]
    names = set(re.findall(r"lib\.(\w+)", stub))
    lib = ctypes.CDLL(str(LIB))
    for n in names:
        assert hasattr(lib, n), n
    assert "dash_simulate_dir" in names


def golden_dir(tmp_path):
    (tmp_path / "tests").mkdir()
    shutil.copytree(GOLDEN / "sample", tmp_path / "tests" / "sample")
    for f in (tmp_path / "tests" / "sample").glob("core_*_output.txt"):
        f.unlink()


def same_dumps(out_dir):
    for n in range(4):
        assert (out_dir / f"core_{n}_output.txt").read_bytes() == \
            (GOLDEN / "sample" / f"core_{n}_output.txt").read_bytes(), n


@pytest.mark.gpu
def test_drop_in_main_reproduces_sample(tmp_path):
    exe = build_main(tmp_path)
    run = tmp_path / "run"
    run.mkdir()
    golden_dir(run)
    p = subprocess.run([str(exe), "sample"], cwd=run, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    assert p.stdout.splitlines() == [f"Processor {n} initialized" for n in range(4)]
    same_dumps(run)


@pytest.mark.gpu
def test_ctypes_stub_reproduces_sample(tmp_path):
    golden_dir(tmp_path)
    stub = blocks("python")[0].replace('"ue22cs343bb1-openmp-assignment_amd/libdash.so"', repr(str(LIB)))
    p = subprocess.run(["python3", "-c", stub + "\nassert rc == 0, rc\n"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    same_dumps(tmp_path)


def test_schedule_snippet_compiles(tmp_path):
    """The §2a snippet (an explicit round schedule through dash_set_schedule) compiles."""
    body = blocks("c")[2]
    assert "dash_set_schedule" in body
    src = tmp_path / "sched.c"
    src.write_text("#include <stdint.h>\n#include \"dash.h\"\nint main(void) {\n" + body +
                   "    dash_destroy(h);\n    return (int)st.err_bits;\n}\n")
    subprocess.run(["gcc", "-O2", "-Wall", "-Werror", f"-I{ROOT / 'include'}", "-c", "-o",
                    str(tmp_path / "sched.o"), str(src)], check=True, capture_output=True, text=True)
