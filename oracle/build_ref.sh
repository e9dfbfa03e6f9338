#!/bin/bash
# TEST INFRASTRUCTURE: compile the reference simulator from its own single
# source file, where it lies, into oracle/_ref/ (git-ignored; never vendored).
#   oracle/_ref/cache_simulator      unmodified /root/reference/assignment.c
# Used only by tests/test_oracle_vs_reference.py to pin the oracle on traces
# whose outcome is schedule-independent (every message is a self-message).
set -euo pipefail
REF=${1:-/root/reference}
OUT=$(cd "$(dirname "$0")" && pwd)/_ref
if [ ! -f "$REF/assignment.c" ]; then
    echo "reference not present at $REF; skipping" >&2
    exit 0
fi
mkdir -p "$OUT"
gcc -O0 -fopenmp -w -o "$OUT/cache_simulator" "$REF/assignment.c"
echo "built $OUT/cache_simulator"
# oracle/_ref/cache_simulator_bench: the reference with the benchmark patch of
# SURVEY.md §8(d) (atomic queue counts, receiver guard, termination), 8 nodes,
# 4096 instructions, gcc -O2 -fopenmp -- the CPU baseline bench.py can time
python3 "$(dirname "$0")/patch_ref.py" "$REF"
