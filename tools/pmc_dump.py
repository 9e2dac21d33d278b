"""Per-kernel PMC counter sums from a rocprofv3 --pmc rocpd database (plus kernel-trace VGPR/LDS when
present): usage python tools/pmc_dump.py run_results.db [name-substring]"""
import sqlite3
import sys
from collections import defaultdict


def main(db, sub=""):
    c = sqlite3.connect(db)
    rows = c.execute("select kernel_name, counter_name, value from counters_collection").fetchall()
    agg = defaultdict(lambda: defaultdict(float))
    n = defaultdict(set)
    for k, cn, v in rows:
        if sub in k:
            agg[k[:90]][cn] += v
    for k, d in agg.items():
        print(k)
        for cn in sorted(d):
            print(f"   {cn:32s} {d[cn]:.4g}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
