"""Static check of the hand-counted LDS waits in a gfx950 device assembly listing.

The resident-band and band kernels issue their LDS fragment reads as inline asm
(`ds_read_b128` between ;;#ASMSTART/;;#ASMEND) and wait for them with hand-counted
`s_waitcnt lgkmcnt(N)`.  The compiler cannot see those reads as in flight, so any
instruction it places between a read and the wait that covers it and that touches the
read's destination VGPRs (a copy `v_mov`, a spill, a reuse of the register) sees stale
data.  This tool simulates the in-order LGKM queue per basic block and reports every
such access.

Scalar-memory loads (s_load_*, s_buffer_load_*, s_memtime / s_memrealtime) count in
LGKM_CNT too but return OUT OF ORDER.  The tool tracks every one issued since
the last lgkmcnt(0) and reports each hand-counted (inline-asm) `lgkmcnt(N>0)` issued while
one may be in flight.  Whether such a wait is a hazard depends on what it is meant to cover:
for LDS reads counted over LDS reads only it is still exact -- L LDS + K scalar ops
outstanding, waiting until <= N remain forces >= L + K - N completions, >= L - N of them LDS
ones, and LDS ops complete in order -- so the oldest L - N reads are done whatever the scalar
loads do; it would be a hazard only for a wait meant to cover the scalar load itself or
counted with the scalar load in N.  Both counts are printed.

usage: python tools/asm_lgkm_check.py file.s [--verbose]
"""
import re
import sys

VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
SMEM = ("s_load_", "s_buffer_load_", "s_memtime", "s_memrealtime", "s_scratch_load", "s_dcache_")
KERNEL = re.compile(r"^(_Z\S+):")


def regs(text):
    out = set()
    for m in VREG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def split_operands(ins):
    parts = ins.split(None, 1)
    if len(parts) < 2:
        return parts[0], "", ""
    op, rest = parts
    ops = [o.strip() for o in rest.split(",")]
    # first operand is the destination for most VALU / DS-read / MFMA / VMEM-load instructions
    dst_first = not (op.startswith("ds_write") or op.startswith("global_store") or op.startswith("buffer_store")
                     or op.startswith("s_") or op.startswith("ds_store") or op == "global_load_lds_dwordx4"
                     or op.startswith("global_load_lds"))
    if dst_first:
        # v_mfma: dst, srcA, srcB, srcC
        return op, ops[0], ",".join(ops[1:])
    return op, "", ",".join(ops)


def check(path, verbose=False):
    kern = None
    pending = []  # list of (dest regs, line no) of hand-counted asm reads, oldest first
    smem = []  # line numbers of scalar-memory loads possibly in flight (since the last lgkmcnt(0))
    in_asm = False
    issues = 0
    nreads = 0
    smem_waits = 0  # hand-counted lgkmcnt(N > 0) issued while a scalar load may be in flight
    hand_waits = 0
    with open(path) as f:
        lines = f.readlines()
    for no, raw in enumerate(lines, 1):
        line = raw.split(";")[0].strip() if not raw.strip().startswith(";;#ASM") else raw.strip()
        m = KERNEL.match(raw)
        if m:
            kern = m.group(1)
            pending = []
            smem = []
            continue
        if raw.strip() == ";;#ASMSTART":
            in_asm = True
            continue
        if raw.strip() == ";;#ASMEND":
            in_asm = False
            continue
        if not line:
            continue
        if line.endswith(":"):  # a label: conservatively keep the queue (fallthrough)
            continue
        op = line.split()[0]
        if op.startswith(SMEM):
            smem.append(no)
        if in_asm:
            if op.startswith("ds_read"):
                d = regs(line.split(",")[0])
                pending.append((d, no))
                nreads += 1
            elif op == "s_waitcnt":
                mm = re.search(r"lgkmcnt\((\d+)\)", line)
                if mm:
                    n = int(mm.group(1))
                    hand_waits += 1
                    if n > 0 and smem:
                        smem_waits += 1
                        if verbose:
                            print(f"{path}:{no}: {(kern or '')[:90]}: hand-counted lgkmcnt({n}) with scalar loads "
                                  f"possibly in flight (issued at lines {smem[-4:]})")
                    if n == 0:
                        smem = []
                    while len(pending) > n:
                        pending.pop(0)
            continue
        if op == "s_waitcnt":
            mm = re.search(r"lgkmcnt\((\d+)\)", line)
            if mm:
                n = int(mm.group(1))
                if n == 0:
                    smem = []
                while len(pending) > n:
                    pending.pop(0)
            continue
        if op.startswith("s_endpgm") or op.startswith("s_branch") or op.startswith("s_cbranch"):
            if pending and op.startswith("s_endpgm"):
                print(f"{path}:{no}: {kern}: program ends with {len(pending)} reads pending")
            # branches: keep the queue (the loop back-edge re-enters with reads pending only
            # if the wait is after the branch, which the next block's first wait resolves)
            continue
        if not pending:
            continue
        opn, dst, src = split_operands(line)
        touched_dst = regs(dst)
        touched_src = regs(src)
        for d, rno in pending:
            hit_r = d & touched_src
            hit_w = d & touched_dst
            if hit_r or hit_w:
                issues += 1
                kind = "reads" if hit_r else "writes"
                print(f"{path}:{no}: {kern[:90]}: `{line}` {kind} v{sorted(hit_r or hit_w)} of the LDS read at line {rno} before its lgkmcnt wait")
    print(f"checked {nreads} hand-counted LDS reads: {issues} premature accesses; "
          f"{smem_waits} of {hand_waits} hand-counted lgkmcnt waits issued with a scalar load possibly in flight")
    return issues


if __name__ == "__main__":
    sys.exit(1 if check(sys.argv[1], "--verbose" in sys.argv) else 0)
