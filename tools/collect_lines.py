"""Copy bench JSON lines from GPU logs into profiles/<round>/, stamped with the
commit of the build that produced them (the GPU box's snapshot has no .git,
so the stamp is added here, from the same tree that was sent).

    python tools/collect_lines.py r06 gpurun_out/prof/bench_c5_3600.log [...]
    python tools/collect_lines.py r06 --prefix strong_ gpurun_out/prof/strong_c5_r0of8.log [...]

Each log's last line starting with '{' goes to profiles/<round>/<prefix><log stem>.json.
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from refresh_profiles import ROOT, head_commit  # noqa: E402


def main(argv):
    rnd, rest = argv[0], argv[1:]
    prefix = ""
    if rest and rest[0] == "--prefix":
        prefix, rest = rest[1], rest[2:]
    out = ROOT / "profiles" / rnd
    out.mkdir(parents=True, exist_ok=True)
    commit = head_commit()
    for log in rest:
        p = Path(log)
        lines = [ln for ln in p.read_text().splitlines() if ln.startswith("{")]
        if not lines:
            print(f"{p}: no JSON line", file=sys.stderr)
            continue
        d = json.loads(lines[-1])
        d["source_commit"] = commit
        name = p.stem if p.stem.startswith(prefix) else prefix + p.stem
        (out / f"{name}.json").write_text(json.dumps(d) + "\n")
        print(f"{name}: {d.get('ms_per_step')} ms/step, bit_exact {d.get('bit_exact')}")


if __name__ == "__main__":
    main(sys.argv[1:])
