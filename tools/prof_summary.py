"""Summarise a rocprofv3 ``--stats`` kernel_stats.csv into a compact Markdown table."""
import csv
import sys


def main(path, top=15):
    rows = list(csv.DictReader(open(path)))
    print("| kernel | calls | total ms | avg us | % |")
    print("|---|---:|---:|---:|---:|")
    for r in rows[:top]:
        name = r["Name"]
        name = name[:90] + ("..." if len(name) > 90 else "")
        print(f"| `{name}` | {r['Calls']} | {int(r['TotalDurationNs'])/1e6:.3f} | {float(r['AverageNs'])/1e3:.1f} | {float(r['Percentage']):.2f} |")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 15)
