#!/usr/bin/env python3
"""Overlap of host<->device copies with compute in a `rocprofv3 --kernel-trace --memory-copy-trace` run.

Reads the `*_kernel_trace.csv` and `*_memory_copy_trace.csv` of one run directory and reports, per copy direction,
the bytes moved, the time the copy engines were busy, and how much of that time at least one compute kernel was
running on the device (the copies of the Twin-Flow offload path are issued on dedicated d2h / h2d streams, so the
overlapped share is the part of the transfer cost that the step does not pay for). Prints one JSON line.
"""
import csv
import glob
import json
import os
import sqlite3
import sys


def _col(row, *names):
    for n in names:
        if n in row and row[n] != "":
            return row[n]
    raise KeyError(names)


def _merge(iv):
    iv.sort()
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def _overlap(a, b):
    """Total length of the intersection of two merged interval lists."""
    i = j = 0
    tot = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            tot += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def _from_db(path, min_bytes):
    """rocprofv3's default output: one sqlite file with `kernels` and `memory_copies` views."""
    c = sqlite3.connect(path)
    # the runtime performs device->pinned-host copies with a blit kernel (`__amd_rocclr_copyBuffer`) on the copy's
    # stream: those dispatches are transfers, not compute
    blit = "name like '__amd_rocclr_copy%'"
    kern = [[s, e] for s, e in c.execute(f"select start, end from kernels where not ({blit})")]
    kstreams = sorted({r[0] for r in c.execute(f"select distinct stream_id from kernels where not ({blit})")})
    per = {}
    for start, end, stream in c.execute(f"select start, end, stream_id from kernels where {blit} and "
                                        "end - start > 20000"):
        d = per.setdefault("BLIT_KERNEL_COPY (device->host staging)", {"iv": [], "bytes": 0, "n": 0,
                                                                        "streams": set()})
        d["iv"].append([start, end])
        d["n"] += 1
        d["streams"].add(stream)
    for name, start, end, size, stream in c.execute("select name, start, end, size, stream_id from memory_copies"):
        if size < min_bytes:
            continue
        d = per.setdefault(name, {"iv": [], "bytes": 0, "n": 0, "streams": set()})
        d["iv"].append([start, end])
        d["bytes"] += size
        d["n"] += 1
        d["streams"].add(stream)
    # the stream that carries most kernel time is the compute stream
    busiest = c.execute(f"select stream_id, sum(end - start) t from kernels where not ({blit}) group by stream_id "
                        "order by t desc limit 1").fetchone()
    return kern, per, {"kernel_streams": kstreams, "compute_stream": busiest[0] if busiest else None}


def main():
    d = sys.argv[1]
    min_bytes = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    kfiles = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    cfiles = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)
    dbs = glob.glob(os.path.join(d, "**", "*.db"), recursive=True)
    extra = {}
    per = {}
    if kfiles and cfiles:
        kern = []
        for f in kfiles:
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    kern.append([int(_col(r, "Start_Timestamp")), int(_col(r, "End_Timestamp"))])
        for f in cfiles:
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    direction = _col(r, "Direction", "Name", "Kind")
                    nbytes = int(float(r.get("Bytes", r.get("Size", 0)) or 0))
                    if nbytes < min_bytes:
                        continue
                    per.setdefault(direction, {"iv": [], "bytes": 0, "n": 0, "streams": set()})
                    per[direction]["iv"].append([int(_col(r, "Start_Timestamp")), int(_col(r, "End_Timestamp"))])
                    per[direction]["bytes"] += nbytes
                    per[direction]["n"] += 1
                    if r.get("Stream_Id"):
                        per[direction]["streams"].add(int(r["Stream_Id"]))
    elif dbs:
        kern, per, extra = _from_db(dbs[0], min_bytes)
    else:
        raise SystemExit(f"no kernel / memory-copy trace under {d}")
    kern = _merge(kern)
    span = (kern[-1][1] - kern[0][0]) if kern else 0
    out = {"kernel_busy_ms": round(sum(e - s for s, e in kern) / 1e6, 1), "trace_span_ms": round(span / 1e6, 1),
           "directions": {}}
    out.update(extra)
    for k, v in per.items():
        iv = _merge(v["iv"])
        busy = sum(e - s for s, e in iv)
        ov = _overlap(iv, kern)
        out["directions"][k] = {"copies": v["n"], "gib": round(v["bytes"] / 2**30, 2),
                                "busy_ms": round(busy / 1e6, 1), "overlapped_with_kernels_ms": round(ov / 1e6, 1),
                                "overlapped_share": round(ov / busy, 3) if busy else None,
                                "gib_per_s": round(v["bytes"] / 2**30 / (busy / 1e9), 1) if busy and v["bytes"] else None,
                                "streams": sorted(v["streams"])}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
