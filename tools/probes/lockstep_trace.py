#!/usr/bin/env python3
"""The RCCL lockstep's agreements in a rocprofv3 kernel trace (rocpd SQLite): the kernels on the
lockstep stream (the stream running words_copy_kernel), grouped per agreement -- words in, RCCL's
all-reduce, words out -- with the device-side span of each agreement, the gaps between its kernels
(dependent launches on one stream), and what else was running on the GPU meanwhile.

Usage: python tools/probes/lockstep_trace.py RESULTS.db
"""
import re
import sqlite3
import sys


def pct(xs, q):
    xs = sorted(xs)
    return round(xs[min(len(xs) - 1, int(len(xs) * q))] / 1e3, 2) if xs else None


def main():
    c = sqlite3.connect(sys.argv[1])
    rows = c.execute("select name, start, end, stream from kernels order by start").fetchall()
    ls_streams = {s for n, _, _, s in rows if "words_copy_kernel" in n}
    if not ls_streams:
        print("no words_copy_kernel in the trace")
        return
    ls = [(n, a, b) for n, a, b, s in rows if s in ls_streams]
    others = [(a, b) for n, a, b, s in rows if s not in ls_streams]
    # agreements: words_copy (in) ... words_copy (out): pairs of words_copy_kernel dispatches
    agreements, cur = [], []
    for k in ls:
        cur.append(k)
        if "words_copy_kernel" in k[0] and len([x for x in cur if "words_copy_kernel" in x[0]]) == 2:
            agreements.append(cur)
            cur = []
    spans = [a[-1][2] - a[0][1] for a in agreements]
    gaps = [a[i + 1][1] - a[i][2] for a in agreements for i in range(len(a) - 1)]
    durs = {}
    for a in agreements:
        for n, s, e in a:
            durs.setdefault(re.sub(r"\(.*", "", n.replace("(anonymous namespace)", ""))[:60], []).append(e - s)
    busy = []
    j = 0
    for a in agreements:
        s0, e0 = a[0][1], a[-1][2]
        busy.append(sum(1 for (s, e) in others if s < e0 and e > s0))
    per = round(sum(len(a) for a in agreements) / max(1, len(agreements)), 2)
    print({"agreements": len(agreements), "kernels_per_agreement": per,
           "span_us_p50": pct(spans, 0.5), "span_us_p90": pct(spans, 0.9), "span_us_p99": pct(spans, 0.99),
           "gap_between_its_kernels_us_p50": pct(gaps, 0.5), "gap_us_p90": pct(gaps, 0.9),
           "other_kernels_overlapping_p50": sorted(busy)[len(busy) // 2] if busy else None})
    for n, d in durs.items():
        print(f"  {n}: n={len(d)} p50 {pct(d, 0.5)} us p99 {pct(d, 0.99)} us")


if __name__ == "__main__":
    main()
