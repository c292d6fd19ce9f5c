"""Build profiles/<round>/pmc_summary.json from two rocprofv3 --pmc CSV passes
(FETCH_SIZE and WRITE_SIZE collected in separate runs, MI355X_MICROARCH.md):

    python tools/pmc_summary.py FETCH.{csv,db} WRITE.{csv,db} FRAMES "bench.py --seconds 256" > profiles/r01/pmc_summary.json

Per kernel: launches, KiB per launch as reported, HBM bytes per launch with
the gfx950 correction (FETCH_SIZE x 2 for wide coalesced reads) and per frame.
"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"^void ", "", name).replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*$", "", name)


def load(path, counter):
    acc = defaultdict(lambda: [0, 0.0])
    if path.endswith(".db"):  # rocpd database (rocprofv3's default output on this image)
        import sqlite3

        c = sqlite3.connect(path)
        for name, value in c.execute("select kernel_name, value from counters_collection where counter_name = ?",
                                     (counter,)):
            k = short(name)
            acc[k][0] += 1
            acc[k][1] += float(value)
        return acc
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            k = short(row["Kernel_Name"])
            acc[k][0] += 1
            acc[k][1] += float(row["Counter_Value"])
    return acc


def main(fetch_csv, write_csv, frames, source):
    frames = int(frames)
    fe, wr = load(fetch_csv, "FETCH_SIZE"), load(write_csv, "WRITE_SIZE")
    out = {"source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), {source}, MI355X",
           "units": "FETCH_SIZE/WRITE_SIZE in KiB as reported; gfx950 correction per MI355X_MICROARCH.md: "
                    "FETCH_SIZE x2 (wide coalesced reads)",
           "frames": frames, "kernels": {}}
    for k in sorted(set(fe) | set(wr)):
        n = max(fe[k][0], wr[k][0], 1)
        f_kib = fe[k][1] / max(fe[k][0], 1)
        w_kib = wr[k][1] / max(wr[k][0], 1)
        b = (2.0 * f_kib + w_kib) * 1024.0
        out["kernels"][k] = {"launches": n, "FETCH_SIZE_KiB_per_launch": f_kib, "WRITE_SIZE_KiB_per_launch": w_kib,
                             "hbm_bytes_per_launch_corrected": b, "hbm_bytes_per_frame_per_launch": b / frames}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(*sys.argv[1:5])
