#!/usr/bin/env python3
"""Cross-check a bench.py line against the rocprofv3 kernel trace of the same command.

    rocprofv3 --kernel-trace --stats --output-format csv -d DIR -o run -- \\
        python3 bench.py --no-cpu-baseline --module-path 0 [ARGS] > BENCH.json
    python tools/trace_check.py DIR/.../run_kernel_trace.csv BENCH.json OUT.json

The bench's timed region is `warmup + steps` back-to-back replays of the engine's hipGraph, so
its dispatches form the longest run of consecutive forwards in the trace (blocks of launches per
forward, each starting at the input quantizer, with the same kernels; the per-kind timing graphs
that follow have fewer launches).  From the
last `steps` blocks of that run this computes, per forward: the kernel-time sum, the busy time
(the union of the launches' intervals: the engine runs each residual block's downsample conv
concurrently with the main path, so launches may overlap), the contraction kernels' busy time, and
the roofline fraction Σ contraction ops / their busy time / peak.  It FAILS (exit 1) when the
trace's per-forward busy time exceeds the bench's own ms_per_step (the trace would then not
describe the benched build), or when the bench's roofline.frac differs from the trace's by more
than 5 % (relative).  Contraction kernels: qconv*/stem_pool*/chain_epilogue*.
"""
import csv
import json
import sys

PEAK_TOPS = 5000.0
CONV_KERNELS = ("qconv", "stem_pool", "chain_epilogue")  # (the split chain epilogue: charged to the contractions)


def forward_blocks(rows, period):
    """(start, n) of the longest run of consecutive forwards in the start-ordered trace: blocks of
    `period` launches, each beginning at the forward's first launch -- the input quantizer, the one
    `quantize` kernel of a forward -- with the same multiset of kernel names.  (Anchoring on the
    quantizer also keeps a rotated run from starting mid-forward; comparing multisets
    rather than sequences admits forwards whose concurrent branches start in either order.)"""
    names = [r["Kernel_Name"] for r in rows]
    anchors = [i for i, nm in enumerate(names) if "quantize" in nm and i + period <= len(names)]
    sig = lambda i: sorted(names[i:i + period])  # noqa: E731
    best = (0, 0)
    k = 0
    while k < len(anchors):
        i, n = anchors[k], 1
        ref = sig(i)
        while (i + n * period < len(names) and "quantize" in names[i + n * period]
               and sig(i + n * period) == ref):
            n += 1
        if n > best[1]:
            best = (i, n)
        k += 1
        while k < len(anchors) and anchors[k] < i + n * period:
            k += 1
    return best


def union_us(rows):
    """Time covered by at least one of the launches (us): concurrent launches count once."""
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
    tot, cur_s, cur_e = 0, None, None
    for s_, e_ in iv:
        if cur_e is None or s_ > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s_, e_
        else:
            cur_e = max(cur_e, e_)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot / 1e3


def main(trace, bench_json, out):
    line = json.loads(open(bench_json).read().strip().splitlines()[-1])
    L = line["engine"]["launches_per_forward"]
    steps = line["steps"]
    rows = sorted((r for r in csv.DictReader(open(trace)) if "qnn" in r["Kernel_Name"]),
                  key=lambda r: int(r["Start_Timestamp"]))
    start, n = forward_blocks(rows, L)
    if n < steps:
        raise SystemExit(f"trace: longest run of {L}-launch forwards is {n} < steps {steps}")
    blocks = [rows[start + (n - steps + f) * L:start + (n - steps + f + 1) * L] for f in range(steps)]
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # noqa: E731 (us)
    is_conv = lambda r: any(k in r["Kernel_Name"] for k in CONV_KERNELS)  # noqa: E731
    tot = sum(sum(dur(r) for r in b) for b in blocks) / steps
    busy = sum(union_us(b) for b in blocks) / steps
    conv_sum = sum(sum(dur(r) for r in b if is_conv(r)) for b in blocks) / steps
    conv = sum(union_us([r for r in b if is_conv(r)]) for b in blocks) / steps
    # per launch: the k-th launch of a kernel name in every forward, in the first forward's order
    def keyed(b):
        seen, out_ = {}, []
        for r in b:
            nm = r["Kernel_Name"]
            seen[nm] = seen.get(nm, 0) + 1
            out_.append(((nm, seen[nm]), r))
        return out_
    order = [k for k, _ in keyed(blocks[0])]
    acc = {k: 0.0 for k in order}
    for b in blocks:
        for k, r in keyed(b):
            acc[k] += dur(r)
    per_launch = [acc[k] / steps for k in order]
    names = [k[0].replace("void qnn::", "").split("(")[0][:80] for k in order]
    ms_step = line["ms_per_step"]
    ops = line["roofline"]["achieved"] * line["roofline"]["kernel_ms_per_forward"] * 1e-3 * 1e12  # Σ conv ops
    frac_trace = ops / (conv * 1e-6) / 1e12 / PEAK_TOPS
    frac_bench = line["roofline"]["frac"]
    res = {"source": f"rocprofv3 kernel trace {trace}: the last {steps} of {n} consecutive graph replays "
                     f"({L} launches each) = bench.py's timed region",
           "bench": bench_json, "ms_per_step": ms_step, "trace_kernel_ms_per_forward": round(tot / 1e3, 4),
           "trace_busy_ms_per_forward": round(busy / 1e3, 4),
           "trace_conv_ms_per_forward": round(conv / 1e3, 4),
           "trace_conv_kernel_sum_ms_per_forward": round(conv_sum / 1e3, 4),
           "bench_conv_ms_per_forward_in_graph": line["roofline"]["kernel_ms_per_forward"],
           "conv_gop_per_forward": round(ops / 1e9, 2), "frac_trace": round(frac_trace, 4),
           "frac_bench": frac_bench, "frac_rel_diff": round(abs(frac_bench - frac_trace) / frac_trace, 4),
           "launches": [{"i": i, "kernel": k, "us": round(u, 2)} for i, (k, u) in enumerate(zip(names, per_launch))]}
    ok_sum = busy / 1e3 <= ms_step
    ok_frac = res["frac_rel_diff"] <= 0.05
    res["checks"] = {"trace_busy_le_ms_per_step": ok_sum, "frac_within_5pct": ok_frac}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "launches"}))
    if not ok_sum:
        print(f"REFUSED: per-forward kernel busy time {busy / 1e3:.4f} ms > ms_per_step {ms_step} ms", file=sys.stderr)
    if not ok_frac:
        print(f"REFUSED: bench frac {frac_bench} vs trace frac {frac_trace:.4f}", file=sys.stderr)
    return 0 if ok_sum and ok_frac else 1


if __name__ == "__main__":
    if len(sys.argv) != 4:
        raise SystemExit(__doc__)
    sys.exit(main(*sys.argv[1:]))
