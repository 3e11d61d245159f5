#!/usr/bin/env python
"""Idle gaps between consecutive kernels of a rocprofv3 kernel trace (one bench step, the last complete one
between two launches of the step's last kernel: the SH backward with the fused Adam epilogue, or the
separate Adam kernel of the unfused and the data-parallel steps): prints each kernel's start offset, duration and the gap before it.
    python scripts/trace_gaps.py gpurun_out/prof/bench_kernel_trace.csv [step index]
bench.py's trace holds the warmup steps, the timed steps, then the kernels_ms pass (hipEvents around every launch,
which add ~10 us before each kernel): pass the index of a timed step (e.g. 10 for `--warmup 5`) to see those."""
import csv
import sys


def main(path, which=-1):
    r = sorted(csv.DictReader(open(path)), key=lambda x: int(x["Start_Timestamp"]))
    last = lambda n: ("k_adam" in n or "k_preprocess_bwd_sh_adam" in n  # noqa: E731
                      or ("k_preprocess_bwd_sh_rows" in n and "true>" in n))
    idx = [i for i, x in enumerate(r) if last(x["Kernel_Name"])]
    # which: the step (counted between consecutive last kernels; -1 = the last one in the trace)
    a, b = (idx[-2], idx[-1]) if which < 0 else (idx[which], idx[which + 1])
    t_prev = int(r[a]["End_Timestamp"])
    gaps = busy = 0
    for x in r[a + 1:b + 1]:
        s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
        gap = max(0, s - t_prev)
        gaps += gap
        busy += e - s
        print(f"gap {gap / 1e3:7.1f} us  dur {(e - s) / 1e3:8.1f} us  {x['Kernel_Name'][:70]}")
        t_prev = max(t_prev, e)
    print(f"step: busy {busy / 1e3:.1f} us, gaps {gaps / 1e3:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/bench_kernel_trace.csv",
         int(sys.argv[2]) if len(sys.argv) > 2 else -1)
