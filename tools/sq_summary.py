"""profiles/<round>/pmc_sq_summary.json from one rocprofv3 --pmc pass of SQ
counters (SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS
SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAIT_ANY) over a short C2 bench:

    python tools/sq_summary.py SQ.db FRAMES SEARCHES "source" [commit] > profiles/rNN/pmc_sq_summary.json

Per kernel: the counter sums and the summed dispatch duration.  For the scan
kernel: instructions per search and the measured VALU issue fraction = VALU
wave-instructions x 2 cycles (a wave64 VALU instruction occupies a SIMD-32
for 2 cycles, MI355X_MICROARCH.md) / (4 SIMDs x frames (one CU each) x the
launch's duration x 2.4 GHz) -- the share of the SIMDs' issue slots the scan
actually fills, next to the algorithm-equivalent roofline fraction.
"""
import json
import re
import sqlite3
import sys
from collections import defaultdict

CLOCK_HZ = 2.4e9


def short(n):
    n = re.sub(r"^void ", "", n).replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*$", "", n)


def main(db, frames, searches, source, commit=None):
    frames, searches = int(frames), int(searches)
    c = sqlite3.connect(db)
    acc = defaultdict(lambda: defaultdict(float))
    dur = defaultdict(dict)
    for name, ctr, val, disp, s, e in c.execute(
            "select kernel_name, counter_name, value, dispatch_id, start, end from counters_collection"):
        k = short(name)
        acc[k][ctr] += float(val)
        dur[k][disp] = (e - s) * 1e-9
    out = {"source": source, "source_commit": commit, "units": "SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_BUSY_CYCLES as reported (quad-cycles); "
                                      "instruction counts summed over waves; duration_s = summed dispatch durations",
           "kernels": {}}
    for k in sorted(acc):
        out["kernels"][k] = dict(acc[k], duration_s=sum(dur[k].values()), dispatches=len(dur[k]))
    scan = [k for k in acc if k.startswith("gsc::scan_batch_kernel")]
    if scan:
        k = max(scan, key=lambda x: acc[x]["SQ_INSTS_VALU"])
        a, t = acc[k], sum(dur[k].values())
        out["scan_kernel"] = k
        out["scan_per_search"] = {
            "valu_insts": a["SQ_INSTS_VALU"] / searches, "salu_insts": a["SQ_INSTS_SALU"] / searches,
            "lds_insts": a["SQ_INSTS_LDS"] / searches,
            "wait_any_frac_of_wave_cycles": a["SQ_WAIT_ANY"] / a["SQ_WAVE_CYCLES"], "searches": searches,
            "frames": frames}
        out["scan_valu_issue_frac"] = a["SQ_INSTS_VALU"] * 2.0 / (4.0 * frames * t * CLOCK_HZ)
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(*sys.argv[1:6])
