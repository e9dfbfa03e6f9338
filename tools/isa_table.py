#!/usr/bin/env python3
"""Instruction table of the round loop of the headline kernel.

Disassembles the gfx950 code object inside libdash.so, finds the round loop of
sim_kernel<8, 4, 16, 0> (the tightest backward branch around four arrival exchanges) and counts its
instructions by encoding and unit: VOP1/VOP2/VOPC in their 32-bit forms, VOP3 (64-bit
encodings: three-operand ops, SGPR-mask selects and compares, modifiers), SDWA, SALU, LDS,
VMEM, branches, waits. Counts are static, over one trip of the loop (DASH_QCHECK = 4
rounds, unrolled) and divided by 4 per round; the rare blocks behind wave-uniform tests
(REPLY_ID fan-out, errors) are listed apart. The dynamic per-round counts come from the
PMC run (profiles/pmc_uniform.json) for comparison.

VALU rate classes come from tools/micro/valu_ops.hip (profiles/r01/micro/valu_ops.txt):
"full" ops issue at 1.4-1.7 wave64 per cycle per CU, "half" ops at 0.90-0.96 (left shifts,
selects, compares, bit-field and three-operand ops, SDWA).

Usage: python3 tools/isa_table.py [libdash.so] [kernel-symbol] [--json out.json]
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
SYM = "_ZN4dash10sim_kernelILi8ELi4ELj16ELi0EEEvNS_7SimArgsE"
ROUNDS_PER_TRIP = 4

# measured in tools/micro/valu_ops.hip (32 waves/CU, profiles/r01/micro/valu_ops.txt and
# profiles/r02/valu_ops_r2.txt): wave64 VALU per cycle per CU. Left shifts are slow, right
# shifts fast; bitop3 and the clamped subtract are fast.
FULL = {"v_xor_b32": 1.42, "v_and_b32": 1.70, "v_lshrrev_b32": 1.50, "v_sub_u32": 1.71,
        "v_subrev_u32": 1.48, "v_mov_b32": 1.50, "v_add_u32": 1.46, "v_or_b32": 1.51,
        "v_bitop3_b32": 1.64}
HALF = {"v_max_u32": 0.96, "v_cndmask_b32": 0.94, "v_cmp_eq_u32": 0.96, "v_bfe_u32": 0.95,
        "v_lshl_or_b32": 0.94, "v_or3_b32": 0.94, "v_bcnt_u32_b32": 0.95, "v_pk_add_u16": 0.94,
        "v_bfi_b32": 0.94, "v_ffbl_b32": 0.90, "v_perm_b32": 0.94, "v_lshl_add_u32": 0.94,
        "v_and_or_b32": 0.95, "v_lshlrev_b32": 0.96, "v_add3_u32": 0.93, "v_mad_u32_u24": 0.94,
        "v_cmp_gt_i32": 0.94}
# same datapath as a measured op (assumption, marked in the table)
LIKE_FULL = ("v_not_b32", "v_ashrrev_i32")


def extract(lib):
    tmp = tempfile.mkdtemp(prefix="isa_")
    dst = os.path.join(tmp, "libdash.so")
    with open(lib, "rb") as f, open(dst, "wb") as g:
        g.write(f.read())
    subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", dst], check=True, cwd=tmp,
                   stdout=subprocess.DEVNULL)
    co = [p for p in os.listdir(tmp) if "gfx950" in p]
    if not co:
        sys.exit("no gfx950 code object in " + lib)
    out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", os.path.join(tmp, co[0])],
                         check=True, capture_output=True, text=True).stdout
    return out


def kernel_insns(dis, sym):
    lines = dis.splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(rf"^[0-9a-f]+ <{re.escape(sym)}>:", l))
    insns = []
    for l in lines[start + 1:]:
        if re.match(r"^[0-9a-f]+ <", l):
            break
        m = re.match(r"^\s+(\S+)(.*?)//\s*([0-9A-F]+):((?: [0-9A-F]{8})+)(?:\s*<[^+>]*\+0x([0-9a-f]+)>)?", l)
        if not m:
            continue
        op, args, addr, enc, tgt = m.groups()
        insns.append(dict(op=op, args=args.strip(), addr=int(addr, 16), size=4 * len(enc.split()),
                          tgt=int(tgt, 16) if tgt else None))
    base = insns[0]["addr"]
    for x in insns:
        x["off"] = x["addr"] - base
    return insns


def unit(x):
    op = x["op"]
    if op.startswith("s_waitcnt") or op == "s_nop":
        return "wait/nop"
    if op.startswith("s_cbranch") or op == "s_branch":
        return "branch"
    if op.startswith("s_load") or op.startswith("s_buffer"):
        return "SMEM"
    if op.startswith("s_"):
        return "SALU"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "VMEM"
    if op.startswith("v_"):
        if "_sdwa" in op:
            return "VALU SDWA"
        if "_dpp" in op:
            return "VALU DPP"
        if op.endswith("_e32"):
            return "VALU VOP1/2/C (e32)"
        return "VALU VOP3 (e64)"
    return "other"


def rate(op):
    if op.endswith("_sdwa"):
        return "half"  # SDWA forms measured slow (shift, compare)
    base = re.sub(r"_(e32|e64|sdwa|dpp)$", "", op)
    if base in FULL:
        return "full"
    if base in HALF:
        return "half"
    if base in LIKE_FULL:
        return "full*"
    return "half*"


def main():
    args = [a for i, a in enumerate(sys.argv[1:], 1) if a != "--json" and sys.argv[i - 1] != "--json"]
    lib = args[0] if args else os.path.join(ROOT, "ue22cs343bb1-openmp-assignment_amd", "libdash.so")
    sym = args[1] if len(args) > 1 else SYM
    insns = kernel_insns(extract(lib), sym)
    # the round loop: the tightest backward branch around one trip's ROUNDS_PER_TRIP arrival
    # exchanges (ds_wrxchg, one per round)
    back = [(x["tgt"], x["off"]) for x in insns if x["tgt"] is not None and x["tgt"] <= x["off"]]
    xchg = [x["off"] for x in insns if x["op"].startswith("ds_wrxchg")]
    cands = [b for b in back if sum(b[0] <= o <= b[1] for o in xchg) >= ROUNDS_PER_TRIP]
    lo, hi = min(cands, key=lambda b: b[1] - b[0])
    body = [x for x in insns if lo <= x["off"] <= hi]
    # nested backward branches = the waterfall loops of the rare blocks
    # (other branches back to the loop header are latches of the same loop)
    inner = [(t, s) for t, s in back if lo < t and s <= hi]
    cold = lambda x: any(t <= x["off"] <= s for t, s in inner)
    tab = collections.Counter()
    tab_cold = collections.Counter()
    ops = collections.Counter()
    rates = collections.Counter()
    for x in body:
        u = unit(x)
        if cold(x):
            tab_cold[u] += 1
            continue
        tab[u] += 1
        ops[x["op"]] += 1
        if u.startswith("VALU"):
            rates[rate(x["op"])] += 1
    r = ROUNDS_PER_TRIP
    print(f"kernel {sym}: round loop at +0x{lo:x}..+0x{hi:x}, {len(body)} instructions per trip "
          f"({r} rounds), {sum(tab_cold.values())} of them in {len(inner)} inner (waterfall) loops")
    print(f"\n{'unit / encoding':28s} {'per trip':>9s} {'per round':>10s}")
    order = ["VALU VOP1/2/C (e32)", "VALU VOP3 (e64)", "VALU SDWA", "VALU DPP", "SALU", "SMEM", "LDS", "VMEM",
             "branch", "wait/nop", "other"]
    for k in order:
        if tab[k]:
            print(f"{k:28s} {tab[k]:9d} {tab[k] / r:10.1f}")
    valu = sum(v for k, v in tab.items() if k.startswith("VALU"))
    issued = valu + tab["SALU"] + tab["LDS"]
    print(f"{'VALU total':28s} {valu:9d} {valu / r:10.1f}")
    print(f"{'VALU + SALU + LDS':28s} {issued:9d} {issued / r:10.1f}")
    print(f"\nVALU by measured rate class (tools/micro/valu_ops; * = by analogy, not measured):")
    for k in ("full", "full*", "half", "half*"):
        if rates[k]:
            print(f"  {k:6s} {rates[k]:5d} per trip {rates[k] / r:6.1f} per round")
    # VALU pipe model: wave64 on one SIMD, full-rate ops ~2 cycles, half-rate ops ~4
    nf = rates["full"] + rates["full*"]
    nh = rates["half"] + rates["half*"]
    print(f"  pipe model: {nf / r:.1f} x 2 + {nh / r:.1f} x 4 = {(2 * nf + 4 * nh) / r:.0f} SIMD cycles per round")
    print("\ntop opcodes (per trip):")
    for op, n in ops.most_common(int(os.environ.get("ISA_TOP", "24"))):
        print(f"  {n:4d}  {op:28s} {unit({'op': op}):22s} {rate(op) if op.startswith('v_') else ''}")
    if "--json" in sys.argv:
        import json
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        import kernel_fingerprint
        out = {"kernel": sym, "kernel_fingerprint": kernel_fingerprint.fingerprint(lib, sym), "rounds_per_trip": r, "source": "tools/isa_table.py (static, round loop "
               "without its waterfall loops)", "per_round": {k: tab[k] / r for k in order if tab[k]},
               "valu_rate_class_per_round": {k: rates[k] / r for k in ("full", "full*", "half", "half*")},
               "valu_full_fraction": nf / max(nf + nh, 1),
               "pipe_model_cycles_per_round": (2 * nf + 4 * nh) / r}
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump(out, f, indent=1)
    pmc = os.path.join(ROOT, "profiles", "pmc_uniform.json")
    if os.path.exists(pmc):
        import json
        p = json.load(open(pmc))
        print(f"\ndynamic (PMC, {p.get('source', pmc)}): per launch VALU {p['sq_insts_valu']:.4g}, SALU "
              f"{p['sq_insts_salu']:.4g}, LDS {p['sq_insts_lds']:.4g} (divide by the bench line's wave_rounds)")


if __name__ == "__main__":
    main()
