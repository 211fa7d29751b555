"""Per-fit GPU timeline of a rocprofv3 database of ``bench_north.py --config svc_sparse`` (bucket round):
fits are cut at each ``glm_bkt_count_kernel`` that follows a gap (one count pass per trainer), and
for every fit the span (first kernel of the fit → last kernel / copy before the next fit), the busy
kernel time, the idle time between activities, the largest gaps and per-kernel mean durations are
printed as one JSON line. Usage: ``python scripts/fit_timeline.py DB_OR_DIR [max_fits]``."""
import glob
import json
import sqlite3
import sys
from collections import defaultdict


def short(name):
    for p in ("void ", "(anonymous namespace)::"):
        name = name.replace(p, "")
    return name.split("(")[0][:60]


def main():
    path = sys.argv[1]
    db = path if path.endswith(".db") else glob.glob(path + "/**/*.db", recursive=True)[0]
    c = sqlite3.connect(db)
    ev = [(s, e, short(n), "k") for s, e, n in c.execute("select start, end, name from kernels")]
    try:
        ev += [(s, e, "copy:%s" % n, "c") for s, e, n in c.execute("select start, end, name from memory_copies")]
    except sqlite3.Error:
        pass
    ev.sort()
    starts = [i for i, x in enumerate(ev) if x[2] == "glm_bkt_count_kernel"
              and (i == 0 or ev[i - 1][2] != "glm_bkt_count_kernel")]
    out = []
    for j, i0 in enumerate(starts):
        i1 = starts[j + 1] if j + 1 < len(starts) else len(ev)
        seg = ev[i0:i1]
        # a fit ends at the coefficient read-back (the last device→host copy); anything after it
        # belongs to the harness (the next trainer's set-up kernels come before the next count)
        last = max((k for k, x in enumerate(seg) if x[3] == "c"), default=len(seg) - 1)
        seg = seg[:last + 1]
        t0, t1 = seg[0][0], max(x[1] for x in seg)
        busy, gaps, prev = 0, [], t0
        per = defaultdict(list)
        for s, e, n, _ in seg:
            if s > prev:
                gaps.append((s - prev, n))
            busy += max(0, e - max(s, prev))
            prev = max(prev, e)
            per[n].append(e - s)
        gaps.sort(reverse=True)
        out.append({"fit": j, "span_us": round((t1 - t0) / 1e3, 1), "busy_us": round(busy / 1e3, 1),
                    "idle_us": round((t1 - t0 - busy) / 1e3, 1),
                    "top_gaps_us": [[round(g / 1e3, 1), n] for g, n in gaps[:4]],
                    "kernels": {n: [len(v), round(sum(v) / len(v) / 1e3, 2)] for n, v in per.items()}})
    for r in out[:int(sys.argv[2]) if len(sys.argv) > 2 else 99]:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
