#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace database (rocpd SQLite, ``-d DIR -o NAME`` -> NAME_results.db).

Per kernel name (shortened): dispatches, total / mean / p50 / p99 duration in microseconds, the
resources of its code object (VGPR, AGPR, LDS bytes, workgroup size, grid), and -- with
``--overlap SUBSTR`` -- how the dispatches of every other kernel ran while a kernel whose name
contains SUBSTR was running (e.g. the decode kernels under a GEMM): count and p50 duration of
the dispatches overlapping one, against those that did not.

Usage: python tools/rocpd_summary.py RESULTS.db [--overlap Cijk] [--md OUT.md]
"""
import argparse
import bisect
import re
import sqlite3
import sys


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "")  # its parentheses are not the argument list
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"^void ", "", n)
    if len(n) > 70:
        n = n[:67] + "..."
    return n


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(len(xs) * q))] if xs else 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--overlap", default=None)
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end, vgpr_count, accum_vgpr_count, lds_size, workgroup_x, grid_x, stream "
                     "from kernels order by start").fetchall()
    by = {}
    for name, s, e, vg, ag, lds, wg, grid, stream in rows:
        k = short(name)
        d = by.setdefault(k, {"durs": [], "vgpr": vg, "agpr": ag, "lds": lds, "wg": wg, "grids": set(), "spans": []})
        d["durs"].append((e - s) / 1e3)
        d["grids"].add(grid)
        d["spans"].append((s, e))
    out = ["| kernel | n | total ms | mean us | p50 us | p99 us | VGPR | AGPR | LDS B | WG | grids |",
           "|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---|"]
    for k, d in sorted(by.items(), key=lambda kv: -sum(kv[1]["durs"])):
        ds = d["durs"]
        grids = sorted(d["grids"])
        g = f"{grids[0]}..{grids[-1]}" if len(grids) > 1 else str(grids[0])
        out.append(f"| {k} | {len(ds)} | {sum(ds) / 1e3:.2f} | {sum(ds) / len(ds):.1f} | {pct(ds, .5):.1f} | "
                   f"{pct(ds, .99):.1f} | {d['vgpr']} | {d['agpr']} | {d['lds']} | {d['wg']} | {g} |")
    if a.overlap:
        busy = sorted(sp for k, d in by.items() if a.overlap in k for sp in d["spans"])
        starts = [s for s, _ in busy]
        out += ["", f"Dispatches overlapping a `{a.overlap}` kernel, against the rest:", "",
                "| kernel | n overlapped | p50 us overlapped | n alone | p50 us alone |", "|---|---:|---:|---:|---:|"]

        def overlaps(s, e):
            i = bisect.bisect_right(starts, e)
            for j in range(max(0, i - 4), i):
                if busy[j][0] < e and busy[j][1] > s:
                    return True
            return False

        for k, d in sorted(by.items(), key=lambda kv: -sum(kv[1]["durs"])):
            if a.overlap in k:
                continue
            ov = [(e - s) / 1e3 for s, e in d["spans"] if overlaps(s, e)]
            al = [(e - s) / 1e3 for s, e in d["spans"] if not overlaps(s, e)]
            out.append(f"| {k} | {len(ov)} | {pct(ov, .5):.1f} | {len(al)} | {pct(al, .5):.1f} |")
    text = "\n".join(out)
    print(text)
    if a.md:
        with open(a.md, "w") as f:
            f.write(text + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
