"""Lines the hook calls of tools/hook_trace_probe.py up with the rocprofv3 kernel and HIP-runtime trace
of the same run, to show where a slow call under the bulk job spends its time.
For every block-service worker generation (k_block_svc dispatch): the time from its launch call
(hipLaunchKernel / hipExtLaunchKernel, matched by correlation id) to the kernel's start, i.e. how long
it waited for the GPU to start it.  For every hook call over the threshold: whether a worker launch
happened inside it, how long that worker waited, and which bulk kernels were running meanwhile.
usage: python tools/hook_trace_summary.py TRACE_DIR CALLS_CSV [threshold_us]"""
import csv
import glob
import os
import sys


def rows(pattern):
    files = glob.glob(pattern, recursive=True)
    if not files:
        sys.exit(f"no file matches {pattern}")
    with open(files[0]) as f:
        return list(csv.DictReader(f))


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))] if v else float("nan")


def main():
    tdir, calls_csv = sys.argv[1], sys.argv[2]
    thr = float(sys.argv[3]) if len(sys.argv) > 3 else 500.0
    kern = rows(os.path.join(tdir, "**", "*kernel_trace.csv"))
    api = rows(os.path.join(tdir, "**", "*hip_api_trace.csv"))
    with open(calls_csv) as f:
        calls = [(int(r["op"]), int(r["start_us"]) * 1000, int(r["dur_us"]) * 1000) for r in csv.DictReader(f)]
    launch_api = {}
    for a in api:
        if "LaunchKernel" in a["Function"]:
            launch_api[a["Correlation_Id"]] = (int(a["Start_Timestamp"]), int(a["End_Timestamp"]))
    svc, bulk = [], []
    for k in kern:
        s, e = int(k["Start_Timestamp"]), int(k["End_Timestamp"])
        if "k_block_svc" in k["Kernel_Name"]:
            la = launch_api.get(k["Correlation_Id"])
            svc.append((la[1] if la else s, s, e))
        else:
            bulk.append((s, e, k["Kernel_Name"].split("(")[0]))
    # the hook calls' clock (CLOCK_MONOTONIC) against the trace's: report the offset of the first worker
    # launch call from the first hook call, so a mismatch of clock domains shows
    t_first_call = min(c[1] for c in calls)
    t_first_svc = min(x[0] for x in svc) if svc else 0
    print(f"# {len(calls)} hook calls, {len(svc)} worker generations, {len(bulk)} other kernels")
    print(f"# first worker launch - first hook call: {(t_first_svc - t_first_call) / 1e6:.3f} ms "
          "(same clock domain if small)")
    waits = [(st - la) / 1e3 for la, st, _ in svc]
    print(f"worker start after its launch call: p50 {pct(waits, .5):.1f} us, p90 {pct(waits, .9):.1f}, "
          f"max {max(waits) if waits else float('nan'):.1f} us")
    lives = [(e - s) / 1e6 for _, s, e in svc]
    print(f"worker lifetimes: mean {sum(lives) / max(1, len(lives)):.2f} ms, max {max(lives) if lives else 0:.2f} ms")
    for op, name in ((0, "generate"), (1, "recover")):
        d = [c[2] / 1e3 for c in calls if c[0] == op]
        slow = [c for c in calls if c[0] == op and c[2] / 1e3 > thr]
        with_launch = 0
        wait_in = []
        for _, t0, dur in slow:
            ls = [(la, st) for la, st, _ in svc if t0 <= la <= t0 + dur]
            if ls:
                with_launch += 1
                wait_in.append(max((st - la) / 1e3 for la, st in ls))
        print(f"{name}: p50 {pct(d, .5):.0f} p99 {pct(d, .99):.0f} us; {len(slow)} calls over {thr:.0f} us, "
              f"{with_launch} of them launched a worker (its start waited p50 {pct(wait_in, .5):.0f} us)")
    # per slow call: what ran on the GPU during it
    print("# slowest calls: op, duration us, worker launched inside (wait us), kernels overlapping")
    for op, t0, dur in sorted(calls, key=lambda c: -c[2])[:12]:
        ls = [(st - la) / 1e3 for la, st, _ in svc if t0 <= la <= t0 + dur]
        ov = {}
        for s, e, n in bulk:
            if s < t0 + dur and e > t0:
                ov[n] = ov.get(n, 0) + 1
        print(f"{op} {dur / 1e3:8.0f}  launch {'%.0f' % ls[0] if ls else '-':>6}  " +
              ", ".join(f"{n} x{c}" for n, c in ov.items()))


if __name__ == "__main__":
    main()
