#!/usr/bin/env python3
"""Condenses a gpu_run.sh session (gpurun_out/) into a committed profile directory.

Writes ``<dst>/SUMMARY.md`` with:
  * the bench JSON lines (``bench*.log``);
  * per-kernel GPU durations from ``rocprofv3 --kernel-trace`` (grouped by kernel and grid size),
    for the framework's kernels (``tkh::``) and the PyTorch kernels they are compared against;
  * per-kernel PMC counter means from ``--pmc`` passes, with derived HBM bytes per dispatch;
and copies the small raw files (kernel_stats.csv, logs) next to it.

Usage: python tools/prof_summary.py gpurun_out profiles/<name>
"""
from __future__ import annotations

import collections
import csv
import glob
import json
import os
import shutil
import sys

KEEP = ("tkh", "bfloat16_copy", "float8_copy", "index_put", "index_elementwise", "rccl", "ncclDevKernel")


def short(name: str) -> str:
    if name.startswith("_ZN3tkh"):
        # mangled: keep the kernel identifier and template tail
        core = name.split("GLOBAL__N_1", 1)[-1]
        return "tkh::" + core[:60]
    for k in ("fixed_vec_kernel", "varlen_direct_kernel", "varlen_pad_kernel"):
        if k in name and "tkh" in name:
            return "tkh::" + name.split("tkh::(anonymous namespace)::", 1)[-1][:60]
    if "bfloat16_copy" in name:
        return "torch Tensor.to(bf16)"
    if "float8_copy" in name:
        return "torch Tensor.to(fp8)"
    if "index_elementwise" in name or "index_put" in name:
        return "torch index_put (pad)"
    return name[:60]


def kernel_trace_table(path: str) -> list[str]:
    rows = list(csv.DictReader(open(path)))
    d = collections.defaultdict(list)
    for r in rows:
        n = r["Kernel_Name"]
        if not any(k in n for k in KEEP):
            continue
        d[(short(n), int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))].append(
            int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = ["| kernel | grid | wg | calls | mean µs | min µs |", "|---|---:|---:|---:|---:|---:|"]
    for (k, g, wg), v in sorted(d.items()):
        out.append(f"| `{k}` | {g} | {wg} | {len(v)} | {sum(v) / len(v) / 1e3:.2f} | {min(v) / 1e3:.2f} |")
    return out


def pmc_table(paths: list[str]) -> list[str]:
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            n = r["Kernel_Name"]
            if not any(k in n for k in KEEP):
                continue
            d[(short(n), int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
    counters = sorted({c for v in d.values() for c in v})
    out = ["| kernel | grid | " + " | ".join(counters) + " |", "|---|---:|" + "---:|" * len(counters)]
    for (k, g), v in sorted(d.items()):
        cells = []
        for c in counters:
            xs = v.get(c)
            cells.append(f"{sum(xs) / len(xs):.0f}" if xs else "")
        out.append(f"| `{k}` | {g} | " + " | ".join(cells) + " |")
    out.append("")
    out.append("FETCH_SIZE / WRITE_SIZE are KiB per dispatch (TCC); FETCH_SIZE under-counts wide streams "
               "(cdna_hip_programming.md). A zero-copy read from pinned host memory is not an HBM fetch.")
    return out


def main() -> int:
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    md = [f"# Profile summary ({os.path.basename(dst.rstrip('/'))})", ""]
    benches = sorted(glob.glob(os.path.join(src, "bench*.log")) + glob.glob(os.path.join(src, "config*.log")))
    if benches:
        md += ["## Bench lines", ""]
        for b in benches:
            for line in open(b):
                line = line.strip()
                if line.startswith("{"):
                    try:
                        j = json.loads(line)
                    except ValueError:
                        continue
                    md.append(f"- `{os.path.basename(b)}`: `{json.dumps(j)}`")
            shutil.copy(b, dst)
        md.append("")
    for name in ("pytest_gpu.log", "smoke.log", "kernel_bench.log", "host_overhead.log", "lockstep_check.log",
                 "lockstep_rccl.log"):
        p = os.path.join(src, name)
        if os.path.exists(p):
            shutil.copy(p, dst)
    for sub in ("prof", "kprof", "profcopy"):
        tr = os.path.join(src, sub, "run_kernel_trace.csv")
        if os.path.exists(tr):
            md += [f"## Kernel durations: `{sub}` (rocprofv3 --kernel-trace)", ""] + kernel_trace_table(tr) + [""]
            st = os.path.join(src, sub, "run_kernel_stats.csv")
            if os.path.exists(st):
                shutil.copy(st, os.path.join(dst, f"{sub}_kernel_stats.csv"))
    pmcs = sorted(glob.glob(os.path.join(src, "pmc*", "run_counter_collection.csv")))
    if pmcs:
        md += ["## PMC counters (means per dispatch)", ""] + pmc_table(pmcs) + [""]
    open(os.path.join(dst, "SUMMARY.md"), "w").write("\n".join(md) + "\n")
    print(f"wrote {dst}/SUMMARY.md")
    return 0


if __name__ == "__main__":
    sys.exit(main())
