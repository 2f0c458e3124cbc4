#!/usr/bin/env python3
"""Per-kernel register / spill / LDS summary of the shipped library's gfx950 code objects
(llvm-readelf --notes of each device ELF in libqnn_hip.so).

    python tools/kres_lib.py [substring of the kernel name] [path/to/libqnn_hip.so]
"""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from isa_check import LIB, code_objects  # noqa: E402

READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def main():
    pat = sys.argv[1] if len(sys.argv) > 1 else ""
    lib = sys.argv[2] if len(sys.argv) > 2 else LIB
    for _triple, co in code_objects(lib):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(co)
            f.flush()
            notes = subprocess.run([READELF, "--notes", f.name], capture_output=True, text=True).stdout
        for blk in notes.split("- .agpr_count:")[1:]:
            def g(k):
                m = re.search(r"\." + k + r":\s+(\S+)", blk)
                return m.group(1) if m else "?"
            name = g("name")
            if pat not in name:
                continue
            agpr = blk.split("\n", 1)[0].strip()
            print(f"{name[:100]:100s} vgpr={g('vgpr_count'):>4} agpr={agpr:>3} sgpr={g('sgpr_count'):>4} "
                  f"spill={g('vgpr_spill_count')}/{g('sgpr_spill_count')} lds={g('group_segment_fixed_size')}")


if __name__ == "__main__":
    main()
