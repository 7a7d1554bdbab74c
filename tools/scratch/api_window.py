#!/usr/bin/env python3
"""Summarise a rocprofv3 --hip-trace run into something small enough to keep.

Prints the HIP API stats table and one steady-state window of the API trace (calls with their
durations), skipping registration noise.  Usage: api_window.py <dir-with-run_*.csv> [n_calls]
"""
import csv
import glob
import os
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 200
SKIP = {"hipGetDevice", "hipSetDevice", "hipThreadExchangeStreamCaptureMode", "__hipPushCallConfiguration",
        "__hipPopCallConfiguration", "hipGetLastError", "hipPeekAtLastError", "hipGetDeviceCount",
        "hipDeviceGetAttribute", "__hipRegisterFunction", "__hipRegisterFatBinary", "__hipRegisterVar",
        "hipStreamGetCaptureInfo"}
stats = glob.glob(os.path.join(d, "**", "*hip_api_stats.csv"), recursive=True)
if stats:
    rows = list(csv.DictReader(open(stats[0])))
    print("## HIP API stats")
    for r in rows[:25]:
        print(f"{r['Name'][:40]:40s} calls={r['Calls']:>7s} total_ns={r['TotalDurationNs']:>12s} avg_ns={float(r['AverageNs']):10.0f}")
tr = glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)
if tr:
    rows = [r for r in csv.DictReader(open(tr[0])) if r["Function"] not in SKIP]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    mid = len(rows) * 3 // 4
    win = rows[mid:mid + n]
    t0 = int(win[0]["Start_Timestamp"])
    print(f"\n## API trace window ({n} calls from 3/4 of the run)")
    for r in win:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"{(s - t0) / 1000:10.1f} {(e - s) / 1000:8.1f} {r['Function']} tid={r['Thread_Id']}")

kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
if kt:
    rows = list(csv.DictReader(open(kt[0])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    mid = len(rows) * 3 // 4
    win = rows[mid:mid + n // 4]
    t0 = int(win[0]["Start_Timestamp"])
    print(f"\n## kernel timeline window ({len(win)} kernels): start_us dur_us gap_us queue name")
    prev = None
    for r in win:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1000 if prev is not None else 0.0
        prev = e
        print(f"{(s - t0) / 1000:10.1f} {(e - s) / 1000:8.1f} {gap:8.1f} q={r.get('Queue_Id', '?')} "
              f"{r['Kernel_Name'][:70]}")
