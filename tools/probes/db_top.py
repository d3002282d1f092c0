"""Top kernels from a rocprofv3 rocpd database directory (``--stats`` output in .db form)."""
import glob
import sqlite3
import sys


def top(d, n=20):
    f = glob.glob(f"{d}/**/*.db", recursive=True)[0]
    c = sqlite3.connect(f)
    rows = c.execute("select name, total_calls, average, percentage from top_kernels").fetchall()
    for name, calls, avg, pct in rows[:n]:
        print(f"{avg:9.1f} us x{calls:5d} {pct:5.1f}%  {name[:100]}")


if __name__ == "__main__":
    top(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
