"""Copy the reference's own test fixtures (inputs + accepted dumps) into
tests/golden/reference/ so parity tests run without /root/reference
(the GPU box does not have it). Data only: core_<n>.txt traces,
core_<n>_output.txt dumps, run_<k>/ alternatives and instruction_order.txt
witnesses from /root/reference/tests.

Usage: python tests/golden/make_golden.py [/root/reference]
"""
import pathlib
import shutil
import sys

ref = pathlib.Path(sys.argv[1] if len(sys.argv) > 1 else "/root/reference") / "tests"
dst = pathlib.Path(__file__).resolve().parent / "reference"
if dst.exists():
    shutil.rmtree(dst)
n = 0
for f in sorted(ref.rglob("*.txt")):
    out = dst / f.relative_to(ref)
    out.parent.mkdir(parents=True, exist_ok=True)
    shutil.copyfile(f, out)
    n += 1
print(f"copied {n} fixture files into {dst}")
