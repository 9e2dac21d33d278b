"""Interleaved A/B of bench.py under different environment settings on one GPU box (each arm is a
fresh process; rounds alternate the arms so clock / thermal drift spreads evenly).
usage: python tools/bench_ab.py ROUNDS "A=1 B=0" "A=0" ... [-- bench args]"""
import json
import os
import subprocess
import sys


def main():
    argv = sys.argv[1:]
    extra = []
    if "--" in argv:
        i = argv.index("--")
        argv, extra = argv[:i], argv[i + 1:]
    rounds, arms = int(argv[0]), argv[1:]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = {a: [] for a in arms}
    for r in range(rounds):
        for a in arms:
            env = dict(os.environ)
            for kv in a.split():
                k, _, v = kv.partition("=")
                env[k] = v
            cmd = [sys.executable, os.path.join(root, "bench.py"), "--exact-steps", "0", "--cpu-utts", "0"] + extra
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
            line = [x for x in p.stdout.splitlines() if x.startswith("{")]
            if p.returncode != 0 or not line:
                print(f"arm {a!r} failed rc={p.returncode}\n{p.stderr[-2000:]}", flush=True)
                sys.exit(1)
            d = json.loads(line[-1])
            res[a].append(d["ms_per_step"])
            print(f"round {r} {a!r:40s} {d['ms_per_step']:.3f} ms/step  {d['value']:.0f}", flush=True)
    for a in arms:
        v = sorted(res[a])
        print(f"{a!r:40s} median {v[len(v) // 2]:.3f} ms/step  min {v[0]:.3f}")


if __name__ == "__main__":
    main()
