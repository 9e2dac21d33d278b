"""Top kernels of a rocprofv3 rocpd database (total / calls / average), optionally divided by a call count.
usage: python tools/kt_top.py run_results.db [divide_by] [top]"""
import collections
import sqlite3
import sys


def main():
    db = sys.argv[1]
    div = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    c = sqlite3.connect(db)
    d = collections.defaultdict(lambda: [0, 0.0])
    for n, s, e in c.execute("select name, start, end from kernels"):
        d[n][0] += 1
        d[n][1] += e - s
    tot = sum(v[1] for v in d.values())
    print(f"total kernel time {tot / 1e6 / div:.2f} ms (/ {div:g})")
    for n, (k, t) in sorted(d.items(), key=lambda x: -x[1][1])[:top]:
        print(f"{t / 1e6 / div:9.2f} ms {k / div:8.1f} calls {t / k / 1e3:9.1f} us  {n[:110]}")


if __name__ == "__main__":
    main()
