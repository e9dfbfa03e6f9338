"""Per-launch durations of one kernel from a rocprofv3 --kernel-trace CSV, for the launches of a
given grid size: the first K of them (e.g. the headline's warmup + timed launches, before a
process's other rows launch the same kernel). Prints a JSON summary.
Usage: python tools/trace_launches.py run_kernel_trace.csv KERNEL_SUBSTRING GRID_SIZE K"""
import csv
import json
import sys

path, kname, grid, k = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
rows = [r for r in csv.DictReader(open(path)) if kname in r["Kernel_Name"] and int(r.get("Grid_Size") or r["Grid_Size_X"]) == grid]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ms = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows[:k]]
print(json.dumps({"source": path, "kernel": rows[0]["Kernel_Name"] if rows else kname, "grid_size": grid,
                  "launches_of_this_grid": len(rows), "first_k": k, "durations_ms": ms,
                  "avg_ms": sum(ms) / len(ms) if ms else None,
                  "avg_ms_timed": sum(ms[1:]) / len(ms[1:]) if len(ms) > 1 else None,
                  "note": "launch 0 is the untimed warmup step"}, indent=1))
