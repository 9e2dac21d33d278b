"""GPU occupancy of the fast step from a rocprofv3 kernel trace (CSV): the window between consecutive
argmax_reduce_kernel launches is one pfm_run; per window, the union of kernel intervals (busy), the sum of kernel
durations (work; > busy when the two utterance-group streams overlap) and the largest idle gaps.
usage: python tools/trace_busy.py <kernel_trace.csv> [marker-kernel-substring]"""
import csv
import sys


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "argmax_reduce_kernel"
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marks = [e for s, e, n in rows if marker in n]
    print(f"{len(rows)} kernels, {len(marks)} '{marker}' markers")
    for w in range(1, len(marks)):
        t0, t1 = marks[w - 1], marks[w]
        ks = [(max(s, t0), min(e, t1), n) for s, e, n in rows if e > t0 and s < t1]
        work = sum(e - s for s, e, _ in ks)
        busy, cur_s, cur_e, gaps = 0, None, None, []
        for s, e, n in sorted(ks):
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                    gaps.append((s - cur_e, n))
                elif s > t0:
                    gaps.append((s - t0, n))
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            busy += cur_e - cur_s
        span = t1 - t0
        gaps.sort(reverse=True)
        print(f"window {w}: span {span / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms ({100 * busy / span:.1f} %), "
              f"work {work / 1e6:.3f} ms (overlap x{work / max(busy, 1):.2f}), {len(gaps)} gaps, "
              f"sum {sum(g for g, _ in gaps) / 1e6:.3f} ms; largest: "
              + ", ".join(f"{g / 1e3:.0f}us before {n[:40]}" for g, n in gaps[:4]))


if __name__ == "__main__":
    main()
