"""Idle time inside the 131k bench steps from a rocprofv3 kernel-trace CSV.

A step runs from one 131,072-set k_pk_decompress (or k_set_hash_w2 when the
keys come from the table) dispatch to the next; for each step, the union of
kernel intervals, the gaps with no kernel running (> 0.05 ms), and the time
with only small latency kernels running (grid < 16,384 threads).

    python tools/step_gaps.py DIR/run_kernel_trace.csv [first_kernel]
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    first = sys.argv[2] if len(sys.argv) > 2 else "k_pk_decompress"
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0], int(r["Grid_Size_X"])) for r in rows)
    starts = [s for s, e, k, g in ks if k == first and g == 131072]
    for a, b in zip(starts, starts[1:]):
        if (b - a) > 80e6:  # not back-to-back steps
            continue
        inside = [(s, e, k, g) for s, e, k, g in ks if a <= s < b]
        ev = sorted(inside)
        busy, big, gaps, cur_s, cur_e = 0, 0, [], None, None
        for s, e, k, g in ev:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                    if s - cur_e > 50_000:
                        gaps.append((round((cur_e - a) / 1e6, 2), round((s - cur_e) / 1e6, 3), k))
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        # time covered by large kernels only
        iv = sorted((s, e) for s, e, k, g in inside if g >= 16384)
        cs, ce = None, None
        for s, e in iv:
            if ce is None or s > ce:
                if ce is not None:
                    big += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        if ce is not None:
            big += ce - cs
        print(f"step {(b - a) / 1e6:7.3f} ms  busy {busy / 1e6:7.3f}  large kernels {big / 1e6:7.3f}  gaps {gaps}")
        last_big = max(e for s, e, k, g in inside if g >= 16384)
        tail = [(k, round((s - a) / 1e6, 2), round((e - s) / 1e6, 3)) for s, e, k, g in inside if s >= last_big - 1_000_000 or g < 16384]
        print("   small / tail kernels:", tail)


if __name__ == "__main__":
    main()
