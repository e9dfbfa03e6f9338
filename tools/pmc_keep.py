#!/usr/bin/env python3
"""Copy a tools/evidence_sweep_pmc.sh run into profiles/ and summarise it (measurement tooling).

For every point directory under SRC (cs<CS>_p<P> or pmc_<kind>) and every pass in it, keeps the
pass's line (.log), its side file (.detail.json), its kernel trace and the counter rows of the one
dispatch tools/pmc_summary.py reads (the first launch of the point's first-tier kernel at its
largest grid), then writes the summary profiles/pmc_sweep_cs<CS>_p<P>.json / profiles/pmc_<kind>.json
bound to that kernel's fingerprint in the in-tree library.
Usage: python3 tools/pmc_keep.py SRC DST   (e.g. gpurun_out/sw_r5f profiles/r05/pmc)
"""
import csv
import os
import pathlib
import shutil
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parent.parent
PASSES = ("sq1", "sq2", "sq3", "sq4", "tcc1", "tcc2", "write")


def kernel_of(point):
    if point.startswith("pmc_"):
        return 4, point[4:], "sim_kernel<8, 4, 16u, 0>"
    cs = int(point[2:point.index("_p")])
    p = float(point[point.index("_p") + 2:])
    return cs, f"sweep_cs{cs}_p{p:g}", f"sim_kernel<8, {cs}, 16u, 0>"


def keep_pass(src, dst, kname):
    dst.mkdir(parents=True, exist_ok=True)
    rows = list(csv.DictReader(open(src / "run_counter_collection.csv")))
    mine = [r for r in rows if kname in r["Kernel_Name"]]
    grid = max(int(r["Grid_Size"]) for r in mine)
    first = min(int(r["Dispatch_Id"]) for r in mine if int(r["Grid_Size"]) == grid)
    with open(dst / "run_counter_collection.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        w.writeheader()
        w.writerows(r for r in mine if int(r["Dispatch_Id"]) == first)
    shutil.copy(src / "run_kernel_trace.csv", dst / "run_kernel_trace.csv")


def main():
    src, dst = pathlib.Path(sys.argv[1]).resolve(), pathlib.Path(sys.argv[2]).resolve()
    for pdir in sorted(p for p in src.iterdir() if p.is_dir()):
        cs, kind, kname = kernel_of(pdir.name)
        out = dst / pdir.name
        for ps in PASSES:
            keep_pass(pdir / ps, out / ps, kname)
            for ext in (".log", ".detail.json"):
                shutil.copy(pdir / (ps + ext), out / (ps + ext))
        env = dict(os.environ, DASH_KSYM=f"_ZN4dash10sim_kernelILi8ELi{cs}ELj16ELi0EEEvNS_7SimArgsE")
        dirs = [str((out / ps).relative_to(ROOT)) + "/" for ps in PASSES]
        subprocess.run([sys.executable, str(ROOT / "tools" / "pmc_summary.py"), kind, kname,
                        str(ROOT / "profiles" / f"pmc_{kind}.json")] + dirs, check=True, env=env,
                       stdout=subprocess.DEVNULL, cwd=ROOT)
        print(f"{pdir.name}: profiles/pmc_{kind}.json")


if __name__ == "__main__":
    main()
