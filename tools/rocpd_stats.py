"""Per-kernel statistics from a rocprofv3 SQLite database (run_results.db): calls, average and
total duration, sorted by total time.  python tools/rocpd_stats.py <db> [name-substring ...]"""
import sqlite3
import sys


def stats(path, filt=()):
    db = sqlite3.connect(path)
    rows = db.execute("select name, count(*), avg(duration), sum(duration) from kernels group by name "
                      "order by sum(duration) desc").fetchall()
    out = []
    for name, n, avg, tot in rows:
        if filt and not any(f in name for f in filt):
            continue
        out.append((name, n, avg / 1e3, tot / 1e6))
    return out


if __name__ == "__main__":
    for name, n, avg_us, tot_ms in stats(sys.argv[1], sys.argv[2:]):
        print(f"{tot_ms:10.3f} ms {n:6d} x {avg_us:9.2f} us  {name[:110]}")
