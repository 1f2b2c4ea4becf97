#!/usr/bin/env python3
"""Side-by-side view of tools/bench_sweep.py outputs: python tools/sweep_cmp.py NEW.jsonl [OLD.jsonl]"""
import json
import sys


def load(p):
    with open(p) as f:
        return {d["case"]: d for d in (json.loads(line) for line in f if line.strip())}


def main():
    new = load(sys.argv[1])
    old = load(sys.argv[2]) if len(sys.argv) > 2 else {}
    for k, d in new.items():
        was = " (was %8.2f)" % old[k]["kernel_us"] if k in old else ""
        print("%-24s %-8s N=%d F=%2d es=%d %-7s %8.2f us%s %6.1f B %5.1f%%" % (
            k, d["kind"], d["N"], d["F"], d["state_bytes"], d.get("obs", "float32"), d["kernel_us"], was,
            d["bytes_per_env_step"], 100 * d["frac"]))


if __name__ == "__main__":
    main()
