"""Per-launch summary of one sim_kernel instantiation from rocprofv3 PMC passes
(tools/evidence.sh: separate --pmc runs), written to profiles/pmc_<kind>.json and
read by bench.py for roofline.traffic and valu_issue.

HBM bytes, corrected as MI355X_MICROARCH.md (§HBM) prescribes: FETCH_SIZE counts
TCC_EA0_RDREQ x 64 B, i.e. half of every 128-B request. When the request-size
counters were collected (tcc1 pass) the read bytes are the size-weighted sum
RDREQ_128B x 128 + RDREQ_64B x 64 + RDREQ_32B x 32 (disjoint on this part: the
uniform launch measured RDREQ 3.038e9 = 128B 3.038e9 + 64B 2.5e4 + 32B 0);
otherwise 2 x FETCH_SIZE. WRITE_SIZE is taken as measured (KiB).
The summary records the fingerprint of the measured kernel in the library the passes ran
(tools/kernel_fingerprint.py; $DASH_LIB or the in-tree libdash.so; $DASH_KSYM names the kernel's
symbol, default the headline sim_kernel<8,4,16,0>): bench.py uses the file only for that code
object. The wave-rounds of the launch (the engine's statistic) come from the pass's bench line.
Usage: python tools/pmc_summary.py KIND KERNEL_SUBSTRING OUT_JSON DIR [DIR ...]"""
import collections
import csv
import glob
import json
import os
import pathlib
import sys

sys.path.insert(0, str(pathlib.Path(__file__).resolve().parent))
import kernel_fingerprint  # noqa: E402

kind, kname, out = sys.argv[1], sys.argv[2], sys.argv[3]
agg = collections.defaultdict(float)
dur = {}
for d in sys.argv[4:]:
    # one dispatch per pass: the first launch of the kernel at its largest grid (the workload's
    # first-tier launch; a pass's process may also launch the same kernel for other rows)
    rows = []
    for f in sorted(glob.glob(f"{d}/**/*.csv", recursive=True)):
        rows += [r for r in csv.DictReader(open(f)) if "Counter_Name" in r and kname in r["Kernel_Name"]]
    if not rows:
        continue
    grid = max(int(r["Grid_Size"]) for r in rows)
    first = min(int(r["Dispatch_Id"]) for r in rows if int(r["Grid_Size"]) == grid)
    for row in rows:
        if int(row["Dispatch_Id"]) != first:
            continue
        agg[row["Counter_Name"]] += float(row["Counter_Value"])
        dur[row["Counter_Name"]] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1e6
res = {"kernel": kname, "workload": kind, "source": " ".join(sys.argv[4:]),
       "kernel_fingerprint": kernel_fingerprint.fingerprint(os.environ.get("DASH_LIB") or kernel_fingerprint.LIB,
                                                     os.environ.get("DASH_KSYM") or kernel_fingerprint.HEADLINE_SYM)}
fp_summarised = res["kernel_fingerprint"]
for k in sorted(agg):
    res[k.lower()] = agg[k]
read = None
if "TCC_EA0_RDREQ_128B_sum" in agg:
    r128, r64, r32 = agg["TCC_EA0_RDREQ_128B_sum"], agg.get("TCC_EA0_RDREQ_64B_sum", 0.0), \
        agg.get("TCC_EA0_RDREQ_32B_sum", 0.0)
    read = r128 * 128 + r64 * 64 + r32 * 32
    res["read_bytes_source"] = "TCC_EA0_RDREQ_{128B,64B,32B} size-weighted"
elif "FETCH_SIZE" in agg:
    read = agg["FETCH_SIZE"] * 1024 * 2
    res["read_bytes_source"] = "2 x FETCH_SIZE (128-B requests counted at 64 B)"
if read is not None:
    res["read_bytes_per_launch"] = read
if "WRITE_SIZE" in agg:
    res["write_bytes_per_launch"] = agg["WRITE_SIZE"] * 1024
if read is not None and "WRITE_SIZE" in agg:
    res["hbm_bytes_per_launch"] = read + agg["WRITE_SIZE"] * 1024
if "TCC_HIT_sum" in agg and "TCC_MISS_sum" in agg:
    res["l2_hit_rate"] = agg["TCC_HIT_sum"] / max(agg["TCC_HIT_sum"] + agg["TCC_MISS_sum"], 1.0)
if "SQ_INSTS_VALU" in agg:
    res["valu_per_launch"] = agg["SQ_INSTS_VALU"]
    res["kernel_ms"] = dur["SQ_INSTS_VALU"]
# VALU issue slots, measured (sq3 pass): SQ_CYCLES is summed over the 32 shader engines
# (8 XCDs x 4), so SIMD quad-cycles = SQ_CYCLES / 32 x 1024 SIMDs / 4. A SIMD issues at most
# two VALU per quad-cycle (SQ_ACTIVE_INST_VALU2 counts the quad-cycles that issued two), so
# quad-cycles with any VALU issue = INSTS_VALU - VALU2
if "SQ_ACTIVE_INST_VALU2" in agg and "SQ_CYCLES" in agg and "SQ_INSTS_VALU" in agg:
    q = agg["SQ_CYCLES"] / 32 * 1024 / 4
    res["simd_quad_cycles"] = q
    res["valu_issue_busy_frac"] = (agg["SQ_INSTS_VALU"] - agg["SQ_ACTIVE_INST_VALU2"]) / q
    res["valu_dual_issue_frac"] = agg["SQ_ACTIVE_INST_VALU2"] / q
if "SQ_THREAD_CYCLES_VALU" in agg and "SQ_INSTS_VALU" in agg:
    res["valu_exec_lanes"] = agg["SQ_THREAD_CYCLES_VALU"] / agg["SQ_INSTS_VALU"]  # of 64


def pass_record(d):
    """The bench record of a pass: its line (DIR.log), or -- since round 5, when the line is the
    compact summary -- the full record in the pass's side file (DIR.detail.json, else the path
    the line names)."""
    log = pathlib.Path(d.rstrip("/") + ".log")
    line = json.loads([x for x in log.read_text().splitlines() if x.startswith("{")][-1])
    if "totals" in line:
        return line
    side = pathlib.Path(d.rstrip("/") + ".detail.json")
    if not side.exists() and line.get("detail"):
        side = pathlib.Path(line["detail"])
        side = side if side.is_absolute() else pathlib.Path(__file__).resolve().parent.parent / side
    return json.loads(side.read_text())


# the box each pass ran on (bench.py's `box` object, round 4), from the pass's own line (DIR.log),
# so a reader can compare the PMC box with the box of the bench line these counters annotate
boxes = []
for d in sys.argv[4:]:
    try:
        line = pass_record(d)
    except (OSError, IndexError, ValueError):
        continue
    b = line.get("box") or {}
    pb, pa = b.get("probe_before") or {}, b.get("probe_after") or {}
    boxes.append({"pass": pathlib.Path(d).name, "device": (b.get("device") or {}).get("name"),
                  "pci_bus": (b.get("device") or {}).get("pci_bus"),
                  "sclk_mhz": [pb.get("sclk_mhz"), pa.get("sclk_mhz")],
                  "probe_ms": [pb.get("probe_ms"), pa.get("probe_ms")], "kernel_ms_avg": line.get("kernel_ms_avg")})
if boxes:
    res["boxes"] = boxes
# per wave-round figures (the engine's wave_rounds statistic of the same launch, from a pass's line):
# what the sweep's CACHE_SIZE points differ in
wr, instr = None, None
for d in sys.argv[4:]:
    try:
        line = pass_record(d)
        wr = line.get("wave_rounds")
        instr = (line.get("totals") or {}).get("instructions_per_step")
    except (OSError, IndexError, ValueError):
        continue
    if wr:
        break
if wr:
    res["wave_rounds"] = wr
    for k, name in (("SQ_INSTS_VALU", "valu"), ("SQ_INSTS_SALU", "salu"), ("SQ_INSTS_LDS", "lds"),
                    ("SQ_INSTS_BRANCH", "branch"), ("SQ_INSTS_SMEM", "smem"), ("SQ_INSTS_VMEM_RD", "vmem_rd")):
        if k in agg:
            res[f"{name}_per_wave_round"] = agg[k] / wr
    if "kernel_ms" in res:
        # CU-cycles at the 2.4-GHz clock limit per wave-round and CU (256 CUs)
        res["ns_per_wave_round_per_cu"] = res["kernel_ms"] * 1e6 * 256 / wr
if "SQ_LDS_BANK_CONFLICT" in agg and agg.get("SQ_LDS_IDX_ACTIVE"):
    res["lds_bank_conflict_frac"] = agg["SQ_LDS_BANK_CONFLICT"] / agg["SQ_LDS_IDX_ACTIVE"]
if "SQ_WAVE_CYCLES" in agg and agg.get("SQ_BUSY_CU_CYCLES"):
    # mean resident waves per CU: wave-cycles over busy CU-cycles (both in quad-cycle units on gfx950)
    res["waves_per_cu"] = agg["SQ_WAVE_CYCLES"] / agg["SQ_BUSY_CU_CYCLES"] * 4
if "read_bytes_per_launch" in res and instr:
    res["fill_bytes_per_algorithmic_byte"] = res["read_bytes_per_launch"] / (2 * instr)  # 2 B per instruction
# round 5: the passes' own records name the kernel they ran (bench.py `kernel_fingerprint_run`); a
# summary of passes measured on another build than the one present now must not take its fingerprint
ran = set()
for d in sys.argv[4:]:
    try:
        fr = pass_record(d).get("kernel_fingerprint_run")
    except (OSError, IndexError, ValueError):
        continue
    if fr:
        ran.add(fr)
if ran:
    if len(ran) > 1:
        sys.exit(f"passes ran different kernels: {sorted(ran)}")
    res["kernel_fingerprint"] = ran.pop()
    res["kernel_fingerprint_source"] = "the passes' bench records (kernel_fingerprint_run)"
    if res["kernel_fingerprint"] != fp_summarised:
        print(f"note: summarised with a library whose kernel is {fp_summarised}", file=sys.stderr)
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
