#!/usr/bin/env python3
"""Cross-check a bench.py line against the rocprofv3 kernel trace of the same command.

    rocprofv3 --kernel-trace --stats --output-format csv -d DIR -o run -- \\
        python3 bench.py --no-cpu-baseline --module-path 0 [ARGS] > BENCH.json
    python tools/trace_check.py DIR/.../run_kernel_trace.csv BENCH.json OUT.json

The bench's timed region is `warmup + steps` back-to-back replays of the engine's hipGraph, so
its dispatches form the longest run of identical consecutive launch blocks in the trace (period
= launches per forward; the per-kind timing graphs that follow have shorter periods).  From the
last `steps` blocks of that run this computes, per forward: the kernel-time sum, the contraction
kernels' time, and the roofline fraction Σ contraction ops / their trace time / peak.  It FAILS
(exit 1) when the trace's per-forward kernel sum exceeds the bench's own ms_per_step (the trace
would then not describe the benched build), or when the bench's roofline.frac differs from the
trace's by more than 5 % (relative).  Contraction kernels: qconv*/stem_pool*.
"""
import csv
import json
import sys

PEAK_TOPS = 5000.0
CONV_KERNELS = ("qconv", "stem_pool")


def forward_blocks(rows, period):
    """(start, n) of the longest run of identical consecutive blocks of `period` names."""
    names = [r["Kernel_Name"] for r in rows]
    best = (0, 0)
    i = 0
    while i + period <= len(names):
        n = 1
        while names[i + n * period:i + (n + 1) * period] == names[i:i + period]:
            n += 1
        if n > best[1]:
            best = (i, n)
        i += period * n if n > 1 else 1
    # A rotation of a periodic launch stream is periodic too, so the run found first may start
    # mid-forward (e.g. at the previous forward's classifier head).  Anchor it on the forward's
    # first launch -- the input quantizer, the one `quantize` kernel of a block -- dropping the
    # then-partial last block.
    s, n = best
    if n:
        q = [k for k in range(period) if "quantize" in names[s + k]]
        if len(q) == 1 and q[0] > 0:
            best = (s + q[0], n - 1)
    return best


def main(trace, bench_json, out):
    line = json.loads(open(bench_json).read().strip().splitlines()[-1])
    L = line["engine"]["launches_per_forward"]
    steps = line["steps"]
    rows = sorted((r for r in csv.DictReader(open(trace)) if "qnn" in r["Kernel_Name"]),
                  key=lambda r: int(r["Start_Timestamp"]))
    start, n = forward_blocks(rows, L)
    if n < steps:
        raise SystemExit(f"trace: longest run of identical {L}-launch blocks is {n} < steps {steps}")
    blocks = [rows[start + (n - steps + f) * L:start + (n - steps + f + 1) * L] for f in range(steps)]
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # noqa: E731 (us)
    tot = sum(sum(dur(r) for r in b) for b in blocks) / steps
    conv = sum(sum(dur(r) for r in b if any(k in r["Kernel_Name"] for k in CONV_KERNELS)) for b in blocks) / steps
    per_launch = [sum(dur(b[i]) for b in blocks) / steps for i in range(L)]
    names = [r["Kernel_Name"].replace("void qnn::", "").split("(")[0][:80] for r in blocks[0]]
    ms_step = line["ms_per_step"]
    ops = line["roofline"]["achieved"] * line["roofline"]["kernel_ms_per_forward"] * 1e-3 * 1e12  # Σ conv ops
    frac_trace = ops / (conv * 1e-6) / 1e12 / PEAK_TOPS
    frac_bench = line["roofline"]["frac"]
    res = {"source": f"rocprofv3 kernel trace {trace}: the last {steps} of {n} consecutive graph replays "
                     f"({L} launches each) = bench.py's timed region",
           "bench": bench_json, "ms_per_step": ms_step, "trace_kernel_ms_per_forward": round(tot / 1e3, 4),
           "trace_conv_ms_per_forward": round(conv / 1e3, 4),
           "bench_conv_ms_per_forward_in_graph": line["roofline"]["kernel_ms_per_forward"],
           "conv_gop_per_forward": round(ops / 1e9, 2), "frac_trace": round(frac_trace, 4),
           "frac_bench": frac_bench, "frac_rel_diff": round(abs(frac_bench - frac_trace) / frac_trace, 4),
           "launches": [{"i": i, "kernel": k, "us": round(u, 2)} for i, (k, u) in enumerate(zip(names, per_launch))]}
    ok_sum = tot / 1e3 <= ms_step
    ok_frac = res["frac_rel_diff"] <= 0.05
    res["checks"] = {"trace_sum_le_ms_per_step": ok_sum, "frac_within_5pct": ok_frac}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "launches"}))
    if not ok_sum:
        print(f"REFUSED: per-forward kernel sum {tot / 1e3:.4f} ms > ms_per_step {ms_step} ms", file=sys.stderr)
    if not ok_frac:
        print(f"REFUSED: bench frac {frac_bench} vs trace frac {frac_trace:.4f}", file=sys.stderr)
    return 0 if ok_sum and ok_frac else 1


if __name__ == "__main__":
    if len(sys.argv) != 4:
        raise SystemExit(__doc__)
    sys.exit(main(*sys.argv[1:]))
