#!/usr/bin/env python3
"""Exposed-communication analysis of a rocprofv3 kernel trace (+ optional roctx marker trace).

    python tools/comm_overlap.py <run_kernel_trace.csv> [<run_marker_api_trace.csv>] [--skip-steps N] [--json out]

Communication kernels = RCCL device kernels (names containing 'nccl' / 'rccl') and, because a one-rank RCCL
collective lowers to device copies on RCCL's internal streams (the DS_ZERO_FORCE_PARTITION=1 rehearsal), copy
kernels on any stream other than the main compute stream (the busiest one). For the timed window (from the first
kernel after the warmup steps to the last kernel), it reports
  * comm busy time        = union of the comm kernels' [start, end) intervals,
  * compute busy time     = union of every other kernel's intervals,
  * exposed comm time     = comm busy time NOT covered by any compute kernel (what a perfect overlap would hide),
  * per-stream totals (the compute stream vs the ZeRO all-gather / reduce-scatter side streams),
and, given the marker trace, the total time inside each roctx range name (ZeRO fetch / reduce / step phases).
"""
import argparse
import collections
import csv
import json


def _union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def _length(iv):
    return sum(b - a for a, b in iv)


def _intersect(a, b):
    i = j = 0
    out = []
    while i < len(a) and j < len(b):
        lo, hi = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if lo < hi:
            out.append([lo, hi])
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def is_comm(name):
    n = name.lower()
    return "nccl" in n or "rccl" in n


def analyse(kernel_csv, marker_csv=None, t_from=None):
    rows = list(csv.DictReader(open(kernel_csv)))
    ks = []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        stream = r.get("Stream_Id") or r.get("Queue_Id") or "?"
        ks.append((s, e, r["Kernel_Name"], stream))
    ks.sort()
    if t_from is not None:
        ks = [k for k in ks if k[0] >= t_from]
    if not ks:
        return {}
    t0, t1 = ks[0][0], max(k[1] for k in ks)
    busy = collections.Counter()
    for s, e, n, st in ks:
        busy[st] += e - s
    main = busy.most_common(1)[0][0]

    def comm_k(n, st):
        return is_comm(n) or (st != main and "copyBuffer" in n)

    comm = _union([[s, e] for s, e, n, st in ks if comm_k(n, st)])
    comp = _union([[s, e] for s, e, n, st in ks if not comm_k(n, st)])
    covered = _intersect(comm, comp)
    per_stream = collections.defaultdict(lambda: [0, 0])
    for s, e, n, st in ks:
        per_stream[st][0] += e - s
        per_stream[st][1] += 1
    comm_names = collections.Counter()
    for s, e, n, st in ks:
        if comm_k(n, st):
            comm_names[f"{n.split('(')[0][:60]} (stream {st})"] += e - s
    res = {
        "window_ms": (t1 - t0) / 1e6,
        "main_stream": str(main),
        "compute_busy_ms": _length(comp) / 1e6,
        "comm_busy_ms": _length(comm) / 1e6,
        "comm_overlapped_ms": _length(covered) / 1e6,
        "comm_exposed_ms": (_length(comm) - _length(covered)) / 1e6,
        "idle_ms": ((t1 - t0) - _length(_union(comm + comp))) / 1e6,
        "streams": {str(k): {"busy_ms": v[0] / 1e6, "kernels": v[1]} for k, v in per_stream.items()},
        "comm_kernels_ms": {k: v / 1e6 for k, v in comm_names.most_common(8)},
    }
    if marker_csv:
        mrows = list(csv.DictReader(open(marker_csv)))
        tot = collections.defaultdict(lambda: [0, 0])
        for r in mrows:
            msg = r.get("Function") or r.get("Message") or r.get("Operation") or ""
            try:
                s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            except (KeyError, ValueError):
                continue
            if t_from is not None and s < t_from:
                continue
            tot[msg][0] += e - s
            tot[msg][1] += 1
        res["roctx_ranges_ms"] = {k: {"total_ms": v[0] / 1e6, "count": v[1]}
                                  for k, v in sorted(tot.items(), key=lambda kv: -kv[1][0])[:20]}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernel_csv")
    ap.add_argument("marker_csv", nargs="?")
    ap.add_argument("--from-kernel", default=None, help="start the window at the N-th launch of this kernel name")
    ap.add_argument("--nth", type=int, default=1)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    t_from = None
    if a.from_kernel:
        starts = sorted(int(r["Start_Timestamp"]) for r in csv.DictReader(open(a.kernel_csv))
                        if a.from_kernel in r["Kernel_Name"])
        if len(starts) >= a.nth:
            t_from = starts[a.nth - 1]
    res = analyse(a.kernel_csv, a.marker_csv, t_from)
    txt = json.dumps(res, indent=1)
    print(txt)
    if a.json:
        with open(a.json, "w") as f:
            f.write(txt)


if __name__ == "__main__":
    main()
