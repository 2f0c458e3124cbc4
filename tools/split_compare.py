#!/usr/bin/env python3
"""Per-block comparison of the fused general-chain epilogue against the split one (the block's
last conv with RangeBN codes only + qnn_chain_epilogue), from two tools/trace_check.py outputs
of the same bench command (QNN_ENGINE_SPLIT_CHAIN=0 / 1).

    python tools/split_compare.py FUSED_TRACECHECK.json SPLIT_TRACECHECK.json
"""
import json
import sys


def main():
    a = json.load(open(sys.argv[1]))["launches"]
    b = json.load(open(sys.argv[2]))["launches"]
    print(f"# fused {sys.argv[1]}: {sum(l['us'] for l in a):.1f} us per forward; "
          f"split {sys.argv[2]}: {sum(l['us'] for l in b):.1f} us")
    j = 0
    for l in a:
        k = l["kernel"]
        if j < len(b) and b[j]["kernel"] == k:
            j += 1
            continue
        conv = b[j]
        j += 1
        chain = b[j] if j < len(b) and "chain" in b[j]["kernel"] else None
        if chain:
            j += 1
        tot = conv["us"] + (chain["us"] if chain else 0.0)
        print(f"{l['i']:3d} fused {l['us']:7.1f} {k[:44]:44s} | split {conv['us']:7.1f} {conv['kernel'][:36]:36s}"
              f" + chain {chain['us'] if chain else 0:6.1f} = {tot:7.1f} ({tot - l['us']:+6.1f})")


if __name__ == "__main__":
    main()
