"""Per-kernel summary of a rocprofv3 database (``rocprofv3 --kernel-trace -d DIR -o run``):
name, calls, mean / total µs, sorted by total — printed as a table or (``--json``) one JSON line
per kernel."""
import glob
import json
import sqlite3
import sys


def summary(db):
    c = sqlite3.connect(db)
    return c.execute("select name, count(*), avg(end-start)/1000.0, sum(end-start)/1000.0 from kernels "
                     "group by name order by sum(end-start) desc").fetchall()


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    path = args[0]
    dbs = glob.glob(path + "/**/*.db", recursive=True) if not path.endswith(".db") else [path]
    for db in dbs:
        for name, n, mean, tot in summary(db)[:int(args[1]) if len(args) > 1 else 30]:
            if "--json" in sys.argv:
                print(json.dumps({"kernel": name[:160], "calls": n, "mean_us": round(mean, 2), "total_us": round(tot, 1)}))
            else:
                print("%-100s %6d %10.2f %12.1f" % (name[:100], n, mean, tot))


if __name__ == "__main__":
    main()
