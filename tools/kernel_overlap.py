"""Kernel timeline summary from a rocprofv3 kernel trace: per-queue counts, overlap between
launches, GPU-busy fraction (union of kernel intervals) and mean duration.

Usage: python tools/kernel_overlap.py gpurun_out/<dir>/run_kernel_trace.csv [name-substring]
"""
import collections
import csv
import sys


def main() -> None:
    path = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    rows = [r for r in csv.DictReader(open(path)) if pat in r["Kernel_Name"] and "at::native" not in r["Kernel_Name"]
            and "rocclr" not in r["Kernel_Name"]]
    if not rows:
        print("no kernels")
        return
    print("queues:", dict(collections.Counter(r["Queue_Id"] for r in rows)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
    overlap = sum(1 for i in range(1, len(ks)) if ks[i][0] < ks[i - 1][1])
    span = ks[-1][1] - ks[0][0]
    busy, cur_s, cur_e = 0, ks[0][0], ks[0][1]
    for s, e in ks[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    dur = sum(e - s for s, e in ks)
    print(f"kernels {len(ks)}  overlapping starts {overlap}  window {span / 1e3:.1f} us  "
          f"gpu busy (union) {busy / 1e3:.1f} us = {100 * busy / span:.1f} %  mean {dur / len(ks) / 1e3:.2f} us")


if __name__ == "__main__":
    main()
