"""Per-kernel statistics from a rocprofv3 results database (rocpd SQLite
output, the default of this ROCm's rocprofv3): name, calls, total/avg/min/max
in microseconds, sorted by total time.  Usage: prof_db_stats.py RESULTS.db [--csv OUT]"""
import sqlite3
import sys


def stats(db):
    con = sqlite3.connect(db)
    tabs = [r[0] for r in con.execute("select name from sqlite_master where type in ('table','view')")]
    kd = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
    ks = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
    rows = con.execute(
        f"select s.kernel_name, count(*), sum(d.end - d.start), min(d.end - d.start), "
        f"max(d.end - d.start) from {kd} d join {ks} s on d.kernel_id = s.id "
        f"group by s.kernel_name order by 3 desc").fetchall()
    return rows


if __name__ == "__main__":
    rows = stats(sys.argv[1])
    out = ["name,calls,total_us,avg_us,min_us,max_us"]
    for name, n, tot, mn, mx in rows:
        short = name.split("(")[0][:90]
        out.append(f"\"{short}\",{n},{tot / 1e3:.1f},{tot / n / 1e3:.1f},{mn / 1e3:.1f},{mx / 1e3:.1f}")
    print("\n".join(out))
    if "--csv" in sys.argv:
        open(sys.argv[sys.argv.index("--csv") + 1], "w").write("\n".join(out) + "\n")
