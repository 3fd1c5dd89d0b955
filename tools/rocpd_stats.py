"""Per-kernel statistics from a rocprofv3 SQLite database (rocpd *_results.db): name, calls,
total / average / min / max duration in us, share of the total -- the --stats summary, for runs
whose output format was the database."""
import sqlite3
import sys


def main(path, top=40):
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), sum(end - start), min(end - start), max(end - start) "
                     "from kernels group by name order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows)
    print(f"{'kernel':60s} {'calls':>6s} {'total_us':>10s} {'avg_us':>8s} {'min_us':>8s} {'max_us':>8s} {'pct':>6s}")
    for name, n, s, lo, hi in rows[:top]:
        print(f"{name[:60]:60s} {n:6d} {s / 1e3:10.1f} {s / n / 1e3:8.2f} {lo / 1e3:8.2f} {hi / 1e3:8.2f} "
              f"{100 * s / tot:6.2f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40)
