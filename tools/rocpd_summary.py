"""Summarise a rocprofv3 rocpd database (--kernel-trace; ROCm 7 writes <name>_results.db) into a
per-kernel stats CSV (the --stats columns) and a markdown table per step.

usage: python tools/rocpd_summary.py run_results.db out_stats.csv [step_marker_kernel [bench.log [W K]]]
With W K (the bench's --warmup / --steps), the GEMM average is also reported over the bench's second
(HIP-event instrumented, roofline) pass alone: the pfm_run calls W+K .. W+2K-1, delimited by the step
marker's end times.
Steps are counted as the number of launches of step_marker_kernel (default: argmax_reduce_kernel,
launched once per pfm_run). GEMM launches are additionally split by grid (= shape) in the markdown.
"""
import csv
import sqlite3
import sys
from collections import defaultdict


def is_gemm(k):
    return ("gemm_bf16_kernel" in k or "gemm_nt_kernelIDF16b" in k or "gemm_nt_kernel<__bf16>" in k
            or "ffn_fused_kernel" in k)


def main(db, out_csv, marker="argmax_reduce_kernel", bench_log=None, warmup=None, ksteps=None):
    c = sqlite3.connect(db)
    rows = c.execute("select name, duration, grid_x, grid_y, grid_z, workgroup_x from kernels").fetchall()
    agg = defaultdict(list)
    shapes = defaultdict(list)
    for name, dur, gx, gy, gz, wx in rows:
        agg[name].append(dur)
        if "gemm" in name:
            shapes[(name.split("(")[0][-60:], gx // max(wx, 1), gy, gz)].append(dur)
    steps = max(1, sum(len(v) for k, v in agg.items() if marker in k))
    tot = sum(sum(v) for v in agg.values())
    with open(out_csv, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_ALL)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([k, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / tot, min(v), max(v)])
    print(f"steps (launches of {marker}): {steps}; total kernel time {tot / 1e6:.2f} ms = "
          f"{tot / 1e6 / steps:.2f} ms/step\n")
    print("| kernel | calls/step | ms/step | avg us | % |\n|---|---|---|---|---|")
    for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1]))[:20]:
        nm = k.replace("(anonymous namespace)::", "").replace("|", "/")[:80]
        print(f"| `{nm}` | {len(v) / steps:.0f} | {sum(v) / 1e6 / steps:.3f} | {sum(v) / len(v) / 1e3:.1f} | "
              f"{100 * sum(v) / tot:.1f} |")
    # roofline cross-check: the bench's dominant-kernel set = every bf16 GEMM launch
    gl = [d for k, v in agg.items() for d in v
          if "gemm_bf16_kernel" in k or "gemm_nt_kernelIDF16b" in k or "gemm_nt_kernel<__bf16>" in k]
    if gl:
        print(f"\nbf16 GEMM launches (bench roofline kernel set): {len(gl)} launches, "
              f"avg {sum(gl) / len(gl) / 1e3:.2f} us (rocprof)")
    if warmup is not None and ksteps is not None:
        W, K = int(warmup), int(ksteps)
        ends = sorted(e for (e,) in c.execute("select end from kernels where name like ?", (f"%{marker}%",)))
        if len(ends) >= W + 2 * K:
            lo, hi = ends[W + K - 1], ends[W + 2 * K - 1]
            g2 = [d for (n, st, en, d) in c.execute("select name, start, end, duration from kernels")
                  if is_gemm(n) and lo < st and en <= hi]
            if g2:
                print(f"bf16 GEMM launches of the bench's roofline pass (pfm_run calls {W + K}..{W + 2 * K - 1}): "
                      f"{len(g2)} launches, avg {sum(g2) / len(g2) / 1e3:.2f} us (rocprof)")
    if bench_log:
        import json
        line = [x for x in open(bench_log) if x.startswith("{")][-1]
        r = json.loads(line)["roofline"]
        print(f"bench live HIP-event avg_launch_us {r['avg_launch_us']} over {r['launches']} launches; "
              f"achieved {r['achieved']} TFLOP/s, frac {r['frac']}")
    print("\n| GEMM kernel / blocks | calls/step | ms/step | avg us |\n|---|---|---|---|")
    for k, v in sorted(shapes.items(), key=lambda kv: -sum(kv[1]))[:20]:
        print(f"| `{k[0]}` {k[1]}x{k[2]}x{k[3]} | {len(v) / steps:.0f} | {sum(v) / 1e6 / steps:.3f} | "
              f"{sum(v) / len(v) / 1e3:.1f} |")


if __name__ == "__main__":
    main(*sys.argv[1:])
