"""Summarise a rocprofv3 --kernel-trace --stats CSV directory into markdown (per step when --steps)."""
import csv
import sys


def main(stats_csv, steps=1, top=15):
    rows = list(csv.DictReader(open(stats_csv)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"| kernel | calls | total ms | ms/step | avg us | % |\n|---|---|---|---|---|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        t = float(r["TotalDurationNs"])
        name = r["Name"].replace("(anonymous namespace)::", "").replace("|", "/")[:70]
        print(f"| `{name}` | {r['Calls']} | {t/1e6:.2f} | {t/1e6/steps:.2f} | {float(r['AverageNs'])/1e3:.1f} | "
              f"{100*t/tot:.1f} |")
    print(f"\ntotal kernel time {tot/1e6:.1f} ms over {steps} step(s) = {tot/1e6/steps:.2f} ms/step")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1)
