"""tools/trace_check.py (CPU): finds bench.py's timed graph replays in a rocprofv3 kernel trace,
recomputes the roofline fraction from the trace, and refuses a trace that does not describe the
benched build (per-forward kernel sum above ms_per_step) or a frac off by more than 5 %."""
import csv
import json
import os
import sys

from conftest import REPO

sys.path.insert(0, os.path.join(REPO, "tools"))

NAMES = ["void qnn::quantize_s2d_x2_kernel<1, 3>(int)", "void qnn::sp::stem_pool_kernel<4, true>(int)",
         "void qnn::qconv_kernel<qnn::Cfg<1>>(int)", "void qnn::avgpool_quant_kernel(int)"]
DUR = [20_000, 100_000, 50_000, 5_000]  # ns


def _write(tmp, steps=20, warmup=5, conv_frac=None, ms_per_step=None, lead=None):
    rows, t = [], 1_000_000
    def emit(name, dur):
        nonlocal t
        rows.append({"Kernel_Name": name, "Start_Timestamp": t, "End_Timestamp": t + dur})
        t += dur + 1_000
    for _ in range(3):  # autotune: one conv repeated
        emit(NAMES[2], 60_000)
    if lead is not None:  # a launch before the replays with the name of a block's last one
        emit(NAMES[lead], DUR[lead])
    for _ in range(1 + warmup + steps):  # capture warm-up + the replays
        for n, dur in zip(NAMES, DUR):
            emit(n, dur)
        emit("void at::native::copy_kernel(int)", 2_000)  # torch copies are not qnn launches
    for _ in range(steps):  # the conv-only timing graph (period 2)
        emit(NAMES[1], 100_000)
        emit(NAMES[2], 50_000)
    trace = os.path.join(tmp, "run_kernel_trace.csv")
    with open(trace, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        w.writerows(rows)
    conv_ms = 0.152  # in-graph conv time incl. launch gaps (> the 0.150 of kernel time)
    ops = 1e12 * 0.75
    achieved = ops / (conv_ms * 1e-3) / 1e12
    frac = conv_frac if conv_frac is not None else achieved / 5000.0
    line = {"steps": steps, "ms_per_step": ms_per_step or 0.2,
            "engine": {"launches_per_forward": 4},
            "roofline": {"achieved": achieved, "frac": frac, "kernel_ms_per_forward": conv_ms}}
    bj = os.path.join(tmp, "bench.json")
    with open(bj, "w") as f:
        f.write("some log line\n" + json.dumps(line) + "\n")
    return trace, bj


def test_trace_check_accepts_consistent_trace(tmp_path):
    import trace_check
    trace, bj = _write(str(tmp_path))
    out = str(tmp_path / "out.json")
    assert trace_check.main(trace, bj, out) == 0
    r = json.load(open(out))
    assert abs(r["trace_kernel_ms_per_forward"] - 0.175) < 1e-9
    assert abs(r["trace_conv_ms_per_forward"] - 0.150) < 1e-9
    assert r["checks"] == {"trace_busy_le_ms_per_step": True, "frac_within_5pct": True}
    assert [x["us"] for x in r["launches"]] == [20.0, 100.0, 50.0, 5.0]


def test_trace_check_refuses_stale_trace(tmp_path):
    import trace_check
    trace, bj = _write(str(tmp_path), ms_per_step=0.17)  # kernels alone take 0.175 ms
    assert trace_check.main(trace, bj, str(tmp_path / "o.json")) == 1
    trace, bj = _write(str(tmp_path), conv_frac=0.2)  # the bench's frac disagrees with the trace
    assert trace_check.main(trace, bj, str(tmp_path / "o2.json")) == 1


def test_trace_check_anchors_on_the_input_quantizer(tmp_path):
    """A leading launch named like a block's last one makes a rotated run periodic too; the
    blocks must still start at the forward's first launch."""
    import trace_check
    trace, bj = _write(str(tmp_path), lead=3)
    out = str(tmp_path / "out.json")
    assert trace_check.main(trace, bj, out) == 0
    r = json.load(open(out))
    assert r["launches"][0]["kernel"].startswith("quantize_s2d")
    assert [x["us"] for x in r["launches"]] == [20.0, 100.0, 50.0, 5.0]


def test_trace_check_concurrent_branches(tmp_path):
    """Forwards whose two middle launches run concurrently, starting in either order: the blocks
    are still found, each launch is matched by name, and the busy time counts overlap once."""
    import trace_check
    rows, t = [], 1_000_000
    names = [NAMES[0], NAMES[1], "void qnn::qconv_kernel<ds>(int)", NAMES[2], NAMES[3]]
    for f in range(26):
        rows.append({"Kernel_Name": names[0], "Start_Timestamp": t, "End_Timestamp": t + 20_000})
        t += 21_000
        rows.append({"Kernel_Name": names[1], "Start_Timestamp": t, "End_Timestamp": t + 100_000})
        t += 101_000
        a, b = (names[2], names[3]) if f % 2 else (names[3], names[2])
        da, db = (10_000, 50_000) if a == names[2] else (50_000, 10_000)
        rows.append({"Kernel_Name": a, "Start_Timestamp": t, "End_Timestamp": t + da})
        rows.append({"Kernel_Name": b, "Start_Timestamp": t + 500, "End_Timestamp": t + 500 + db})
        t += 51_000
        rows.append({"Kernel_Name": names[4], "Start_Timestamp": t, "End_Timestamp": t + 5_000})
        t += 6_000
    trace = str(tmp_path / "run_kernel_trace.csv")
    with open(trace, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        w.writerows(rows)
    conv_busy_ms = 0.1505  # stem 100 us + the concurrent pair 50.5 us
    ops = 1e12 * 0.75
    line = {"steps": 20, "ms_per_step": 0.19, "engine": {"launches_per_forward": 5},
            "roofline": {"achieved": ops / (conv_busy_ms * 1e-3) / 1e12,
                         "frac": ops / (conv_busy_ms * 1e-3) / 1e12 / 5000.0, "kernel_ms_per_forward": conv_busy_ms}}
    bj = str(tmp_path / "bench.json")
    open(bj, "w").write(json.dumps(line) + "\n")
    out = str(tmp_path / "out.json")
    assert trace_check.main(trace, bj, out) == 0
    r = json.load(open(out))
    assert abs(r["trace_kernel_ms_per_forward"] - 0.185) < 1e-9
    # the pair covers 50.5 us when the short launch starts first, 50 when the long one does
    assert abs(r["trace_busy_ms_per_forward"] - 0.17525) < 1e-4
    assert abs(r["trace_conv_ms_per_forward"] - 0.15025) < 1e-4
    us = {x["kernel"]: x["us"] for x in r["launches"]}
    assert us["qconv_kernel<ds>"] == 10.0 and us["qconv_kernel<qnn::Cfg<1>>"] == 50.0
