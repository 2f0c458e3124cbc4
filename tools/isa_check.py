#!/usr/bin/env python3
"""ISA check of the shipped library: no kernel that issues MFMAs also issues packed-FP32 VALU.

Every kernel of libqnn_hip.so that contains a `v_mfma*` must contain no `v_pk_fma_f32`,
`v_pk_mul_f32` or `v_pk_add_f32` ("co-residency corruption": a packed epilogue of
one workgroup beside another workgroup's MFMA loop on the same SIMD returned a wrong low element
now and then; the Makefile builds every MFMA translation unit with `-packed-fp32-ops`).  A new
MFMA source file, a renamed one or a build outside the Makefile would bring the packed ops back
silently; this check reads the code objects actually shipped, so it catches all of those.

The device code objects are read straight from the library's `.hip_fatbin` section (clang
offload bundles: magic, entry count, then (offset, size, triple) per entry), disassembled with
ROCm's llvm-objdump, and split per kernel symbol.

    python tools/isa_check.py [path/to/libqnn_hip.so]     (exit 1 on a violation)
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(HERE, "quantized.pytorch_amd", "qnn", "libqnn_hip.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
PACKED = re.compile(r"\bv_pk_(fma|mul|add)_f32\b")
SMEM = ("s_load_", "s_buffer_load_", "s_memtime", "s_memrealtime", "s_scratch_load")
LGKM = re.compile(r"lgkmcnt\((\d+)\)")


def code_objects(path, arch="gfx950"):
    """Every device ELF for `arch` inside the library's offload bundles."""
    data = open(path, "rb").read()
    out = []
    pos = data.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + len(MAGIC))[0]
        p = pos + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if arch in triple and size:
                out.append((triple, data[pos + off:pos + off + size]))
        pos = data.find(MAGIC, pos + 1)
    return out


def kernels(elf_bytes):
    """{kernel symbol: [instruction lines]} of one device code object."""
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(elf_bytes)
        f.flush()
        txt = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", "--mcpu=gfx950", f.name], check=True,
                             capture_output=True, text=True).stdout
    ks, cur = {}, None
    for line in txt.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            cur = m.group(1)
            ks.setdefault(cur, [])
        elif cur is not None and line.strip():
            ks[cur].append(line.strip())
    return ks


def check(path=LIB):
    """(number of MFMA kernels checked, [(kernel, first packed-FP32 instruction)] violations)."""
    nmfma, bad = 0, []
    objs = code_objects(path)
    if not objs:
        raise RuntimeError(f"{path}: no gfx950 code objects found")
    for _triple, elf in objs:
        for name, ins in kernels(elf).items():
            if not any(i.startswith("v_mfma") for i in ins):
                continue
            nmfma += 1
            hit = next((i for i in ins if PACKED.search(i)), None)
            if hit:
                bad.append((name, hit))
    return nmfma, bad


if __name__ == "__main__":
    n, bad = check(sys.argv[1] if len(sys.argv) > 1 else LIB)
    for name, ins in bad:
        print(f"packed FP32 in an MFMA kernel: {name[:140]}: `{ins}`")
    print(f"{n} MFMA kernels checked, {len(bad)} with packed-FP32 VALU")
    sys.exit(1 if bad else 0)


ADDR = re.compile(r"//\s*([0-9A-Fa-f]+):")


def _cfg(ins):
    """Successor lists of one kernel's instructions (branch targets from the objdump addresses;
    a branch's immediate counts dwords from the next instruction)."""
    addr = []
    for i in ins:
        m = ADDR.search(i)
        addr.append(int(m.group(1), 16) if m else None)
    at = {a: k for k, a in enumerate(addr) if a is not None}
    succ = []
    for k, i in enumerate(ins):
        op = i.split()[0]
        nxt = [k + 1] if k + 1 < len(ins) else []
        if op == "s_endpgm":
            succ.append([])
            continue
        if op == "s_branch" or op.startswith("s_cbranch"):
            imm = int(i.split()[1].split("//")[0].strip(","))
            imm = imm - 65536 if imm >= 32768 else imm
            base = addr[k + 1] if k + 1 < len(ins) else (addr[k] + 4 if addr[k] is not None else None)
            t = at.get(base + 4 * imm) if base is not None else None
            tgt = [t] if t is not None else nxt  # unresolved: fall through (conservative enough)
            succ.append(tgt if op == "s_branch" else nxt + [t for t in tgt if t not in nxt])
            continue
        succ.append(nxt)
    return succ


def lgkm_hazards(ins):
    """The counted LGKM waits of one kernel's instruction lines reachable with a scalar load in
    flight (smem_lgkm_check)."""
    if not ins:
        return []
    succ = _cfg(ins)
    state = [None] * len(ins)  # in-state: a scalar load may be in flight
    state[0] = False
    work = [0]
    while work:
        k = work.pop()
        fl = state[k]
        op = ins[k].split()[0]
        if op.startswith(SMEM):
            fl = True
        elif op == "s_waitcnt":
            m = LGKM.search(ins[k])
            if m and int(m.group(1)) == 0:
                fl = False
        for t in succ[k]:
            if state[t] is None or (fl and not state[t]):
                state[t] = fl or bool(state[t])
                work.append(t)
    out = []
    for k, i in enumerate(ins):
        if state[k] and i.split()[0] == "s_waitcnt":
            m = LGKM.search(i)
            if m and 0 < int(m.group(1)) < 15:  # lgkmcnt(15): no LGKM wait at all
                out.append(i)
    return out


def smem_lgkm_check(path=LIB):
    """(kernels scanned, [(kernel, wait)]): every `s_waitcnt lgkmcnt(N)`, 0 < N < 15, that may be
    reached while a scalar-memory load (out-of-order in LGKM_CNT) is still in flight -- a forward
    dataflow over the kernel's branches (the state clears at lgkmcnt(0)).  The compiler never
    emits such a wait (with a scalar load pending it waits for 0), so one in the shipped code is a
    hand-counted inline-asm wait in a window the compiler put a scalar load into (VERDICT r4:
    the resident-band kernels' band reads)."""
    n, bad = 0, []
    for _triple, elf in code_objects(path):
        for name, ins in kernels(elf).items():
            n += 1
            bad += [(name, i) for i in lgkm_hazards(ins)]
    return n, bad
