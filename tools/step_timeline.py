"""Wall-clock anatomy of offline pfm_run steps from a rocprofv3 kernel trace (rocpd db).

A step = the kernels from the first launch after the previous step's `argmax_reduce_kernel` up to and
including its own. Per step: wall time, busy time (union of all kernel intervals, any stream), idle
gaps, and per kernel class the wall time during which at least one kernel of that class runs
(classes overlap when streams run concurrently). Phases: encoder (up to the cif_alpha launch),
predictor (to the last copy after cif_fire), decoder (the rest).
usage: python tools/step_timeline.py run_results.db [first_step last_step]"""
import sqlite3
import sys
from collections import defaultdict


def cls(n):
    for key, c in (("ffn_fused", "ffn_fused"), ("gemm_skinny", "gemm_skinny"), ("gemm", "gemm"),
                   ("attn", "attention"), ("layernorm", "layernorm"), ("fsmn", "fsmn"), ("cif", "cif"),
                   ("argmax", "argmax"), ("rocclr", "copy/fill")):
        if key in n:
            return c
    return "other"


def union(iv):
    iv = sorted(iv)
    tot, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main(db, a=None, b=None):
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, stream_id from kernels order by start").fetchall()
    ends = [i for i, r in enumerate(rows) if "argmax_reduce_kernel" in r[0]]
    steps = []
    prev = -1
    for i in ends:
        steps.append(rows[prev + 1:i + 1])
        prev = i
    lo = int(a) if a is not None else 0
    hi = int(b) if b is not None else len(steps) - 1
    print(f"{len(steps)} steps in trace; showing {lo}..{hi}")
    for k in range(lo, hi + 1):
        st = steps[k]
        t0, t1 = st[0][1], max(r[2] for r in st)
        wall = (t1 - t0) / 1e6
        busy = union([(r[1], r[2]) for r in st]) / 1e6
        per = defaultdict(list)
        for r in st:
            per[cls(r[0])].append((r[1], r[2]))
        i_alpha = next((i for i, r in enumerate(st) if "cif_alpha" in r[0]), None)
        i_fire = next((i for i, r in enumerate(st) if "cif_fire" in r[0]), None)
        enc = (st[i_alpha][1] - t0) / 1e6 if i_alpha is not None else float("nan")
        dec_start = None
        if i_fire is not None:
            later = [r for r in st[i_fire + 1:] if "gemm" in r[0] or "layernorm" in r[0]]
            dec_start = later[0][1] if later else None
        pred = (dec_start - st[i_alpha][1]) / 1e6 if dec_start and i_alpha is not None else float("nan")
        dec = (t1 - dec_start) / 1e6 if dec_start else float("nan")
        streams = len(set(r[3] for r in st))
        print(f"step {k}: {len(st)} kernels on {streams} streams, wall {wall:.3f} ms, busy {busy:.3f} ms "
              f"(idle {wall - busy:.3f}); encoder {enc:.3f}, predictor+sync {pred:.3f}, decoder {dec:.3f} ms")
        line = "   " + ", ".join(f"{k2} {union(v) / 1e6:.3f}" for k2, v in sorted(per.items(), key=lambda x: -union(x[1])))
        print(line)


if __name__ == "__main__":
    main(*sys.argv[1:])


def decoder_detail(db, k):
    """Per-kernel-name time inside step k's decoder window (from the first GEMM / LN after cif_fire)."""
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end, stream_id, grid_x, workgroup_x from kernels order by start").fetchall()
    ends = [i for i, r in enumerate(rows) if "argmax_reduce_kernel" in r[0]]
    st = rows[(ends[k - 1] + 1 if k else 0):ends[k] + 1]
    i_fire = next(i for i, r in enumerate(st) if "cif_fire" in r[0])
    win = [r for r in st[i_fire + 1:]]
    d0 = next(r[1] for r in win if "gemm" in r[0] or "layernorm" in r[0])
    agg = defaultdict(list)
    for r in st:
        if r[2] > d0:
            agg[(r[0][:70], r[4] // max(r[5], 1))].append((max(r[1], d0), r[2]))
    tot = (max(r[2] for r in st) - d0) / 1e6
    print(f"decoder window {tot:.3f} ms")
    for key, v in sorted(agg.items(), key=lambda x: -sum(e - s for s, e in x[1])):
        print(f"  {len(v):4d} x {sum(e - s for s, e in v) / len(v) / 1e3:8.1f} us  sum {sum(e - s for s, e in v) / 1e6:.3f} ms"
              f"  grid {key[1]:6d}  {key[0]}")
