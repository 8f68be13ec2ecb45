"""The bench line's dominant kernel in a rocprofv3 kernel trace of the SAME
default command (scripts/gpu_r06final.sh: `rocprofv3 --kernel-trace --stats
-- python3 bench.py`): the trace's averaged stats mix every leg that runs the
same instantiation (spin-up, per-call rows of 16 B .. 1 MiB, the extra
configs), so this picks the timed region itself -- the last 2 x steps
dispatches of the first contiguous run of full-batch launches (no other
dispatch and no gap > 50 ms between them) -- and prints their average next to
the bench line's own hipEvent average (roofline.avg_launch_ms).
  python3 scripts/summarize_bench_trace.py TRACE_CSV BENCH_JSON > summary.json
"""
import csv
import json
import statistics
import sys

KERNEL = "gf_matmul_v16<6, 3, 4, true, 256, 1>"


def main():
    trace, bench = sys.argv[1], sys.argv[2]
    line = next(json.loads(ln) for ln in open(bench) if ln.startswith("{") and '"metric"' in ln)
    n = 2 * line["steps"]
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    run, runs, last_end = [], [], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        full = KERNEL in r["Kernel_Name"] and (e - s) > 1_000_000  # a full 1024-stripe batch: > 1 ms
        gap = last_end is not None and s - last_end > 50_000_000
        if not full or gap:
            if run:
                runs.append(run)
            run = []
        if full:
            run.append((e - s) * 1e-6)
        last_end = e
    if run:
        runs.append(run)
    timed = runs[0][-n:]
    algo = line["roofline"]["algorithmic_bytes_per_launch"]
    avg = statistics.mean(timed)
    print(json.dumps({
        "kernel": KERNEL, "dispatches_in_first_run": len(runs[0]), "timed_region_dispatches": len(timed),
        "avg_ms_trace": round(avg, 4), "median_ms_trace": round(statistics.median(timed), 4),
        "frac_trace": round(algo / (avg * 1e-3) / 8e12, 4),
        "bench_line_avg_launch_ms": line["roofline"]["avg_launch_ms"], "bench_line_frac": line["roofline"]["frac"],
        "bench_line_value_GiBps": line["value"],
        "agreement": round(avg / line["roofline"]["avg_launch_ms"], 4)}, indent=1))


if __name__ == "__main__":
    main()
