"""Per-kernel count / total / average duration from a rocprofv3 SQLite output (rocpd *.db), for runs
made without --output-format csv.   python tools/rocpd_stats.py <results.db> [name-filter]"""
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    rows = c.execute("select s.display_name, count(*), sum(d.end - d.start), avg(d.end - d.start) "
                     "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id "
                     "group by s.display_name order by 3 desc").fetchall()
    tot = sum(r[2] for r in rows)
    print(f"{'kernel':70s} {'calls':>7s} {'total ms':>10s} {'avg us':>9s} {'%':>6s}")
    for name, n, t, a in rows:
        if pat in name:
            print(f"{name[:70]:70s} {n:7d} {t / 1e6:10.3f} {a / 1e3:9.2f} {100 * t / tot:6.2f}")


if __name__ == "__main__":
    main()
