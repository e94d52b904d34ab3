"""Per-kernel HBM traffic per launch from a FETCH_SIZE run and a WRITE_SIZE run
of rocprofv3 --pmc (separate passes: the two do not fit one TCC pass).  Both
counters are in KB; on gfx950 FETCH_SIZE reports half the bytes of a wide read
(/opt/skills/guides/MI355X_MICROARCH.md, HBM section), so
bytes = FETCH_SIZE x 2048 + WRITE_SIZE x 1024 (as profiles/pmc_traffic.json).

    python tools/pmc_summary.py FETCH_DIR WRITE_DIR [kernel ...]
"""
import collections
import csv
import json
import os
import sys


def per_launch(d):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    f, w = per_launch(sys.argv[1]), per_launch(sys.argv[2])
    want = sys.argv[3:] or sorted(set(f) | set(w))
    out = {}
    for k in want:
        fb, wb = f.get(k, 0.0) * 2048, w.get(k, 0.0) * 1024
        out[k] = {"fetch_GB": round(fb / 1e9, 3), "write_GB": round(wb / 1e9, 3), "total_GB": round((fb + wb) / 1e9, 3)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
