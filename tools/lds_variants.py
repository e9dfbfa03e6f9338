#!/usr/bin/env python3
"""LDS bank-conflict attribution probe: kernel variants of
csrc/dash_kernels.hip that each take one LDS structure's access pattern out of the bank-conflict
picture, built into tools/var_r6/libdash_lds_<name>.so (experiments only, never shipped; git-ignored, but
not gpurun-ignored, so the probe can load them on the GPU box).

Timing and SQ_LDS_BANK_CONFLICT only: variants marked "results wrong" change what the simulation
does, so their rounds differ from the base's; they are compared per wave-round (tools/lds_probe.py
runs them with a round cap, so a variant whose messages go astray still ends).

  base      the product kernel
  ring      ring placement stores (place() and the INV fan-out) aimed at the SENDER's own ring
            column instead of the receiver's: k senders to one receiver no longer share a bank
            (results wrong: receivers read their own columns)
  arrive    the arrival-mask ORs aimed at the sender's own mask word (results wrong)
  hist      the per-system histogram atomic aimed at a private word per lane (results identical
            except the histogram)
  window    trace-window refill stores removed; the HBM loads stay (results wrong: stale
            instructions are issued)
  swizzle   u16 rows (ENT, CAC, window) unswizzled: lane l at half-word l (results identical)

Usage: python3 tools/lds_variants.py [name ...]   (default: all)
"""
import pathlib
import subprocess
import sys
import tempfile

ROOT = pathlib.Path(__file__).resolve().parent.parent
SRC = ROOT / "ue22cs343bb1-openmp-assignment_amd" / "csrc" / "dash_kernels.hip"

OFF = "const uint32_t off = (q.y + (rank << 8)) & RMASK;"
VARIANTS = {
    "base": [],
    "ring": [(OFF, "const uint32_t off = (((q.y + (rank << 8)) & RMASK) & ~0xFCu) | (lane << 2);", 2)],
    "arrive": [("__hip_atomic_fetch_or(&lds[L::MQM + L::MQS * (seg + xdP)]", "__hip_atomic_fetch_or(&lds[L::MQM + L::MQS * lane]", 1),
               ("__hip_atomic_fetch_or(&lds[L::MQM + L::MQS * (seg + msr)]", "__hip_atomic_fetch_or(&lds[L::MQM + L::MQS * lane]", 1),
               ("__hip_atomic_fetch_or(&lds[L::MQM + L::MQS * (seg + ffbl(im))]", "__hip_atomic_fetch_or(&lds[L::MQM + L::MQS * lane]", 1)],
    "hist": [("__hip_atomic_fetch_add(&lds[L::HST + pty * L::HSTRIDE + lane / P], 1u,",
              "__hip_atomic_fetch_add(&lds[L::HST + lane], 1u + 0u * pty,", 1)],
    "window": [("""            w[0] = (uint16_t)x;
            w[64] = (uint16_t)(x >> 16);
            if constexpr (WCHUNK == 4) {
                w[128] = (uint16_t)y;
                w[192] = (uint16_t)(y >> 16);
            }
            pend = *++pp;""", """            asm volatile("" :: "v"(x), "v"(y), "v"(w));
            pend = *++pp;""", 1)],
    "swizzle": [("const uint32_t sw = ((lane & 31u) << 1) | (lane >> 5);", "const uint32_t sw = lane;", 1)],
}


def build(name):
    src = SRC.read_text()
    for old, new, n in VARIANTS[name]:
        if src.count(old) != n:
            raise SystemExit(f"{name}: anchor found {src.count(old)} times, want {n}: {old[:60]!r}")
        src = src.replace(old, new)
    with tempfile.TemporaryDirectory() as td:
        f = pathlib.Path(td) / "dash_kernels.hip"
        f.write_text(src)
        subprocess.run(["bash", str(ROOT / "tools" / "build_variant.sh"), f"lds_{name}"], check=True,
                       env={**__import__("os").environ, "SRC": str(f), "OUT": str(ROOT / "tools" / "var_r6")})


if __name__ == "__main__":
    for n in sys.argv[1:] or list(VARIANTS):
        build(n)
