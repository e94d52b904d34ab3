"""HBM traffic per kernel launch from rocprofv3 PMC passes.

Reads the counter_collection CSVs of a FETCH_SIZE pass and a WRITE_SIZE pass
(each collected in its own rocprofv3 run, tools/profile_round.sh) and writes
profiles/pmc_traffic.json: per kernel, the average bytes per launch.

Units and corrections (MI355X_MICROARCH.md, HBM section): rocprofv3's
FETCH_SIZE / WRITE_SIZE are kilobytes (TCC_EA0_RDREQ/WRREQ x 64 B / 1024);
on gfx950 FETCH_SIZE counts half the bytes of wide coalesced reads, so it is
doubled here; WRITE_SIZE is taken as is.

python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write profiles/pmc_traffic.json
"""

import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_kernel(d, counter):
    acc = defaultdict(list)
    for path in glob.glob(os.path.join(d, "*counter_collection.csv")):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row["Counter_Name"] != counter:
                    continue
                acc[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main(fetch_dir, write_dir, out):
    fetch = per_kernel(fetch_dir, "FETCH_SIZE")
    write = per_kernel(write_dir, "WRITE_SIZE")
    res = {}
    for k in sorted(set(fetch) | set(write)):
        fb = fetch.get(k, 0.0) * 1024 * 2  # gfx950: FETCH_SIZE is half of the bytes read
        wb = write.get(k, 0.0) * 1024
        res[k] = {"fetch_kb_raw": fetch.get(k), "write_kb_raw": write.get(k), "bytes_per_launch": fb + wb}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res.items():
        print(f"{k[:40]:40s} {v['bytes_per_launch'] / 1e6:12.1f} MB/launch")


if __name__ == "__main__":
    main(*sys.argv[1:4])
