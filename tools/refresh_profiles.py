"""Copy the round's profile set from gpurun_out/prof (tools/gpu_profile.sh) into
profiles/<round>/: kernel stats of the traced bench, PMC CSV exports and
summary (FETCH_SIZE / WRITE_SIZE passes), and the default bench line.

    python tools/refresh_profiles.py r01
"""
import csv
import json
import re
import sqlite3
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PROF = ROOT / "gpurun_out" / "prof"


def short(n):
    n = re.sub(r"^void ", "", n).replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*$", "", n)


def head_commit() -> str:
    """The commit the profiled build came from (+ "-dirty" with uncommitted source changes)."""
    h = subprocess.run(["git", "-C", str(ROOT), "rev-parse", "--short=12", "HEAD"], capture_output=True,
                       text=True).stdout.strip()
    dirty = subprocess.run(["git", "-C", str(ROOT), "status", "--porcelain", "--", "soundchunks_amd", "bench.py"],
                           capture_output=True, text=True).stdout.strip()
    return h + ("-dirty" if dirty else "")


def main(rnd):
    out = ROOT / "profiles" / rnd
    commit = head_commit()
    out.mkdir(parents=True, exist_ok=True)
    stats = subprocess.run([sys.executable, str(ROOT / "tools/rocpd_summary.py"), str(PROF / "trace/run_results.db")],
                           check=True, capture_output=True, text=True).stdout
    (out / "kernel_stats_bench1024.csv").write_text(stats)
    bench_line = [l for l in (PROF / "trace.log").read_text().splitlines() if l.startswith("{")]
    (out / "rocprof_kernel_trace_bench1024.log").write_text(
        "# rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace -o run -- python3 -u bench.py --steps 1 --warmup 0"
        " --no-cpu-baseline   (MI355X)\n# per-kernel summary (tools/rocpd_summary.py of run_results.db):\n" + stats +
        "# bench line of the same run:\n" + "\n".join(bench_line) + "\n")
    for ctr, name in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        c = sqlite3.connect(PROF / name / "run_results.db")
        rows = c.execute("select dispatch_id, kernel_name, counter_name, value, start, end from counters_collection "
                         "where counter_name = ? order by dispatch_id", (ctr,)).fetchall()
        with open(out / f"pmc_{name}_size_256s.csv", "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value", "Duration_ns"])
            for d, k, cn, v, s, e in rows:
                w.writerow([d, short(k), cn, v, e - s])
    summ = subprocess.run([sys.executable, str(ROOT / "tools/pmc_summary.py"), str(PROF / "fetch/run_results.db"),
                           str(PROF / "write/run_results.db"), "64",
                           "bench.py --seconds 256 --steps 1 --warmup 0 (64 frames)"],
                          check=True, capture_output=True, text=True).stdout
    (out / "pmc_summary.json").write_text(summ)
    if (PROF / "sq" / "run_results.db").exists():  # the SQ pass (tools/gpu/profile.sh)
        sql = [l for l in (PROF / "sq.log").read_text().splitlines() if l.startswith("{")][-1]
        sqj = json.loads(sql)
        summ = subprocess.run([sys.executable, str(ROOT / "tools/sq_summary.py"), str(PROF / "sq/run_results.db"),
                               str(sqj["config"]["frames"]), str(sqj["scan"]["searches"]),
                               "rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS "
                               "SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAIT_ANY -- python3 bench.py --seconds 64 --steps 1 "
                               f"--warmup 0 --no-cpu-baseline ({sqj['config']['frames']} C2 frames, MI355X, "
                               "tools/gpu/profile.sh)", commit], check=True, capture_output=True, text=True).stdout
        (out / "pmc_sq_summary.json").write_text(summ)
    if (PROF / "bench_default.log").exists():
        line = [l for l in (PROF / "bench_default.log").read_text().splitlines() if l.startswith("{")][-1]
        d = json.loads(line)
        d["source_commit"] = commit  # recorded here: the GPU box's snapshot has no .git
        (out / "bench_1gpu.json").write_text(json.dumps(d) + "\n")
        print(json.loads(line)["value"])


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
