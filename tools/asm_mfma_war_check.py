"""Static check: asynchronous loads that overwrite an in-flight MFMA's source VGPRs.

A VMEM (`global_load*`, `buffer_load*`) or LDS (`ds_read*`) load writes its destination
VGPRs when the data returns, asynchronously to the wave's instruction stream.  If such a load
targets a VGPR that a recently issued `v_mfma*` still reads (SrcA / SrcB / SrcC), the return
can land before the matrix core has read the operand: with two workgroups per CU contending
for the XDL pipe, the resident-band kernel lost row 12 of its A fragment this way
("co-residency corruption").  The compiler's hazard recognizer does not model
this write-after-read; the kernels keep a full K step of MFMAs between the last read of a
register slot and the load that refills it.

This tool reports every load whose destination overlaps a source operand of one of the
MFMAs issued within the previous `--window` instructions (in program order of the listing;
a loop back-edge is not followed).

usage: python tools/asm_mfma_war_check.py file.s [--window 8] [--kernel SUBSTR]
"""
import argparse
import re
import sys

VREG = re.compile(r"\b[va]\[(\d+):(\d+)\]|\b[va](\d+)\b")
KERNEL = re.compile(r"^(_Z\S+):")
LOAD = re.compile(r"^(global_load|buffer_load|ds_read|flat_load|scratch_load)")


def regs(text):
    out = set()
    for m in VREG.finditer(text):
        pre = text[m.start()]
        if m.group(3) is not None:
            out.add((pre, int(m.group(3))))
        else:
            out.update((pre, r) for r in range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def check(path, window, ksub=None):
    kern = None
    recent = []  # (instruction index, line no, set of source regs) of the last MFMAs, newest last
    idx = 0
    issues = 0
    seen = set()
    with open(path) as f:
        lines = f.readlines()
    for no, raw in enumerate(lines, 1):
        m = KERNEL.match(raw)
        if m:
            kern = m.group(1)
            recent = []
            continue
        if ksub and (kern is None or ksub not in kern):
            continue
        line = raw.split(";")[0].strip()
        if not line or line.endswith(":") or line.startswith("."):
            continue
        op = line.split()[0]
        idx += 1
        recent = [r for r in recent if idx - r[0] <= window]
        if op.startswith("v_mfma"):
            ops = [o.strip() for o in line[len(op):].split(",")]
            srcs = regs(",".join(ops[1:4]))
            recent.append((idx, no, srcs))
            continue
        if LOAD.match(op) and "lds" not in op.split("_")[-1] and not op.startswith("global_load_lds"):
            dst = regs(line[len(op):].split(",")[0])
            for _i, mno, srcs in recent:
                hit = dst & srcs
                if hit:
                    key = (kern, no)
                    if key not in seen:
                        seen.add(key)
                        issues += 1
                        rr = sorted(r for _, r in hit)
                        print(f"{path}:{no}: {(kern or '?')[:100]}: `{line}` overwrites v{rr[0]}..v{rr[-1]}, "
                              f"a source of the MFMA at line {mno} ({no - mno} lines earlier)")
    print(f"{path}: {issues} loads overwrite a source of an MFMA issued within the previous {window} instructions")
    return issues


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--window", type=int, default=8)
    ap.add_argument("--kernel")
    a = ap.parse_args()
    n = sum(check(f, a.window, a.kernel) for f in a.files)
    sys.exit(1 if n else 0)
