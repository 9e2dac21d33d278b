"""Summarise a rocprofv3 rocpd database (--kernel-trace; ROCm 7 writes <name>_results.db) of a bench.py run into a
per-kernel stats CSV (the --stats columns) and a markdown report whose per-step figures reconcile with the bench.

usage: python tools/rocpd_summary.py run_results.db out_stats.csv [bench.log W K]

A pfm_run call is delimited by `cif_fire_kernel`, launched exactly once per call (the argmax reduction used before
round 5 is not: it undercounted). bench.py's fast leg makes, in order: W warmup calls, K timed calls (the headline
pass: `ms_per_step`), K calls with live HIP events around the GEMM / attention launches (the roofline pass: one
encoder group, so its kernels are the M = B T launches `roofline.dominant` times), and one more call that prices the
event pairs. The report gives, for the headline and the roofline pass separately, the kernel time per call, the
trace's wall span per call (first kernel start to last kernel end) and the per-kernel table; the headline pass's
wall span is what compares with the bench's ms_per_step (a kernel trace serialises the concurrent encoder-group
streams, so profile the headline with PFM_SUBBATCH=1 PFM_DEC_SUBBATCH=1 for a trace without concurrency: then
the kernel time per call is the step). The dominant kernel's rocprof average over the roofline pass is what compares
with `roofline.dominant.avg_launch_us`.
"""
import csv
import json
import sqlite3
import sys
from collections import defaultdict

MARKER = "cif_fire_kernel"
DOMINANT = "ffn2_kernel<4"


def short(k):
    return k.replace("(anonymous namespace)::", "").replace("|", "/")[:80]


def table(rows, ncalls, title):
    agg = defaultdict(list)
    for name, st, en, dur in rows:
        agg[name].append(dur)
    tot = sum(sum(v) for v in agg.values())
    print(f"\n### {title}\n")
    print("| kernel | calls/step | ms/step | avg us | % |\n|---|---|---|---|---|")
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:20]:
        print(f"| `{short(k)}` | {len(v) / ncalls:.1f} | {sum(v) / 1e6 / ncalls:.3f} | {sum(v) / len(v) / 1e3:.1f} | "
              f"{100 * sum(v) / max(tot, 1):.1f} |")
    return agg


def main(db, out_csv, bench_log=None, warmup=None, ksteps=None):
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, duration from kernels order by start").fetchall()
    agg = defaultdict(list)
    for name, st, en, dur in rows:
        agg[name].append(dur)
    tot = sum(sum(v) for v in agg.values())
    with open(out_csv, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_ALL)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([k, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / tot, min(v), max(v)])
    ends = [en for name, st, en, dur in rows if MARKER in name]
    print(f"pfm_run calls in the trace (launches of {MARKER}): {len(ends)}; total kernel time {tot / 1e6:.2f} ms")
    bench = None
    if bench_log:
        line = [x for x in open(bench_log) if x.startswith("{")][-1]
        bench = json.loads(line)
    if warmup is None or ksteps is None or len(ends) < int(warmup) + 2 * int(ksteps):
        table(rows, max(1, len(ends)), "all kernels of the trace, per pfm_run call")
        return
    W, K = int(warmup), int(ksteps)

    def window(i0, i1):   # kernels of calls i0 .. i1-1: after the end of call i0-1, up to the end of call i1-1
        lo = ends[i0 - 1] if i0 > 0 else -1
        hi = ends[i1 - 1]
        return [r for r in rows if lo < r[1] and r[2] <= hi]

    head, roof = window(W, W + K), window(W + K, W + 2 * K)
    for rws, title in ((head, f"headline pass (calls {W}..{W + K - 1}: the bench's timed steps)"),
                       (roof, f"roofline pass (calls {W + K}..{W + 2 * K - 1}: live HIP events, one encoder group)")):
        kern = sum(r[3] for r in rws) / 1e6 / K
        span = (max(r[2] for r in rws) - min(r[1] for r in rws)) / 1e6 / K
        print(f"\n{title}: kernel time {kern:.3f} ms per call, trace wall span {span:.3f} ms per call")
        table(rws, K, title)
    dom = [r[3] for r in roof if DOMINANT in r[0]]
    if dom:
        gfl = None
        print(f"\ndominant kernel `{DOMINANT}>` over the roofline pass: {len(dom)} launches, rocprof avg "
              f"{sum(dom) / len(dom) / 1e3:.2f} us")
    if bench:
        print(f"\nbench line: ms_per_step {bench['ms_per_step']}, value {bench['value']} {bench['unit']}")
        r = bench.get("roofline", {})
        d = r.get("dominant")
        if d:
            print(f"bench roofline.dominant: {d['kernel']} live HIP-event avg {d['avg_launch_us']} us over "
                  f"{d['launches']} launches, {d['gflop_per_launch']} GFLOP each -> {d['achieved']} TFLOP/s, "
                  f"frac {d['frac']}")
        print(f"bench roofline (GEMM class): avg {r.get('avg_launch_us')} us over {r.get('launches')} launches, "
              f"frac {r.get('frac')}")


if __name__ == "__main__":
    main(*sys.argv[1:])
