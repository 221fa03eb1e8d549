#!/usr/bin/env python3
"""Per-kernel statistics from a rocprofv3 rocpd database (ROCm 7 default output):
total / mean / count per kernel name, optionally only dispatches after the first
`--skip` of a marker kernel (warmup). Usage: rocpd_stats.py run_results.db [--last N]"""
import argparse
import re
import sqlite3
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--md", action="store_true", help="markdown table")
    ap.add_argument("--timeline", default="", help="print the dispatches from the last "
                    "occurrence of this kernel on (one step's timeline)")
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    rows = db.execute("select name, start, end from kernels order by start").fetchall()
    per = {}
    for name, s, e in rows:
        m = re.search(r"\b(k_\w+(?:<[^()]*?>)?)", name)
        short = m.group(1) if m else name.replace("void ", "").split("(")[0][:60]
        per.setdefault(short, []).append((e - s) / 1e3)
    tot = sum(sum(v) for v in per.values())
    items = sorted(per.items(), key=lambda kv: -sum(kv[1]))[: a.top]
    if a.md:
        print("| kernel | calls | total us | mean us | median us | share |")
        print("|---|---|---|---|---|---|")
    for k, v in items:
        if a.md:
            print(f"| `{k[:70]}` | {len(v)} | {sum(v):.1f} | {sum(v)/len(v):.2f} | "
                  f"{statistics.median(v):.2f} | {100*sum(v)/tot:.1f}% |")
        else:
            print(f"{k[:70]:70s} {len(v):6d} {sum(v):10.1f} {sum(v)/len(v):8.2f} {statistics.median(v):8.2f}")
    print(f"total kernel time {tot:.1f} us over {len(rows)} dispatches")
    if a.timeline:
        idx = [i for i, r in enumerate(rows) if a.timeline in r[0]]
        if idx:
            t0 = rows[idx[-2] if len(idx) > 1 else idx[-1]][1]
            print("| start us | dur us | kernel |")
            print("|---:|---:|---|")
            for name, st, en in rows:
                if st < t0 or st > t0 + 2e6:
                    continue
                m = re.search(r"\b(k_\w+(?:<[^()]*?>)?)", name)
                k = m.group(1) if m else name.replace("void ", "").split("(")[0][:50]
                print(f"| {(st - t0) / 1e3:.1f} | {(en - st) / 1e3:.1f} | `{k}` |")


if __name__ == "__main__":
    main()
