"""Per-call kernel timeline of tools/latency_probe.py from a rocprofv3
kernel-trace CSV: kernels are grouped into calls by the idle gaps between
them; for every kernel name, the median start and end (ms from the call's
first kernel dispatch) over the calls, and the chain that ends last.

    python tools/critical_path.py DIR/.../lat_kernel_trace.csv [out.json]
"""

import csv
import json
import statistics
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]) for r in rows), key=lambda x: x[0])
    calls, cur, last_end = [], [], None
    for s, e, k in ks:
        if last_end is not None and s - last_end > 5_000_000:  # > 5 ms idle: a new call
            calls.append(cur)
            cur = []
        cur.append((s, e, k))
        last_end = e if last_end is None else max(last_end, e)
    if cur:
        calls.append(cur)
    calls = calls[5:] if len(calls) > 10 else calls  # skip warm-up calls
    per = {}
    spans = []
    for c in calls:
        t0 = c[0][0]
        spans.append((max(e for _, e, _ in c) - t0) / 1e6)
        seen = {}
        for s, e, k in c:
            j = seen.get(k, 0)
            seen[k] = j + 1
            per.setdefault(f"{k}#{j}" if j else k, []).append(((s - t0) / 1e6, (e - t0) / 1e6))
    out = {"calls": len(calls), "device_span_ms_p50": statistics.median(spans), "kernels": {}}
    for k, v in sorted(per.items(), key=lambda kv: statistics.median(x[0] for x in kv[1])):
        st, en = statistics.median(x[0] for x in v), statistics.median(x[1] for x in v)
        out["kernels"][k] = {"start_ms": round(st, 3), "end_ms": round(en, 3), "ms": round(en - st, 3)}
    txt = json.dumps(out, indent=1)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
