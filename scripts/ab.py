"""Generic A/B driver: run one timing command under several environment
variants, interleaved over rounds (so drift hits every variant alike), and
print every output line that carries a time, tagged with its variant, plus
the median of each line's first "<float> ms" value per variant.

  python scripts/ab.py --rounds 3 base: la1:GELIM_BIG_LOOKAHEAD=1 -- python scripts/time_solver.py 4096

Replaces the per-knob ab_*.sh drivers of rounds 2-4 (deleted with their knobs
in round 5; the measurements stay in profiles/).
"""
import argparse
import os
import re
import statistics
import subprocess
import sys

MS = re.compile(r"([0-9]+\.[0-9]+) ms")


def main() -> int:
    argv = sys.argv[1:]
    if "--" not in argv:
        print(__doc__)
        return 2
    cut = argv.index("--")
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--timeout", type=int, default=300)
    ap.add_argument("variants", nargs="+", help="NAME:VAR=V,VAR=V (empty after ':' = the default build)")
    a = ap.parse_args(argv[:cut])
    cmd = argv[cut + 1:]
    variants = {}
    for spec in a.variants:
        name, _, kv = spec.partition(":")
        variants[name] = dict(x.split("=", 1) for x in kv.split(",") if x)
    seen: dict[tuple[str, str], list[float]] = {}
    for rnd in range(a.rounds):
        for name, env in variants.items():
            r = subprocess.run(cmd, env=dict(os.environ, **env), capture_output=True, text=True, timeout=a.timeout)
            if r.returncode != 0:
                print(f"[{name}] round {rnd}: exit {r.returncode}\n{r.stderr[-2000:]}", flush=True)
                return r.returncode
            for line in r.stdout.splitlines():
                m = MS.search(line)
                if not m:
                    continue
                print(f"[{name}] {line}", flush=True)
                key = MS.sub("<t> ms", line)
                key = re.sub(r"\(min [^)]*\)", "", key)
                seen.setdefault((name, key), []).append(float(m.group(1)))
    print("== medians")
    for (name, key), v in seen.items():
        print(f"[{name}] {statistics.median(v):.3f} ms  ({len(v)} runs)  {key}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
