"""Per-config roofline evidence in ONE lease (GPU box), for every BASELINE
config: the bench line, the rocprofv3 kernel trace of that same process, and
FETCH_SIZE / WRITE_SIZE in two separate --pmc passes of the same command.

For each config the summary records
  * the bench JSON line printed by the profiled process itself (so its
    ms_per_step and the trace come from the same run),
  * the engine kernel's average duration over the timed region (the last
    launches_per_step x steps dispatches of the trace) and over all launches,
  * launches x average <= ms_per_step (the profile explains the line),
  * frac recomputed from the trace = algorithmic bytes / avg / 8 TB/s,
  * HBM traffic per launch from the PMC passes, corrected per
    MI355X_MICROARCH.md §HBM (FETCH_SIZE KiB x1024 x2 on gfx950 16-B/lane
    streaming reads; WRITE_SIZE KiB x1024).

usage: python3 scripts/profile_configs.py OUTDIR [config ...]
Every GPU step runs under its own `timeout -k 10`; the first failure ends
the script (no GPU step after a failed one).
"""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK = 8.0e12
COMMON = ["--steps", "10", "--warmup", "3", "--spinup", "0.3", "--cpu-seconds", "0", "--host-path", "0",
          "--extra-configs", "0"]  # extra configs run other kernels shapes in the same process
# name -> (bench args, k, m, cell, stripes, launches per step)
CONFIGS = {
    "rs32": (["--k", "3", "--m", "2", "--stripes", "1024"], 3, 2, 1 << 20, 1024, 2),
    "rs63": ([], 6, 3, 1 << 20, 1024, 2),
    "rs63enc": (["--encode-only"], 6, 3, 1 << 20, 1024, 1),
    "rs104": (["--k", "10", "--m", "4", "--global-stripes", "2048"], 10, 4, 1 << 20, 2048, 2),
    "rs104x256": (["--k", "10", "--m", "4", "--stripes", "256"], 10, 4, 1 << 20, 256, 2),
    "c64k": (["--cell", "65536", "--stripes", "65536"], 6, 3, 65536, 65536, 2),
}
KERNEL_RE = "gf_matmul"
# the checksum kernels, from bench.py --crc (RS(6,3) 1 MiB x 1024): the fused
# encode + CRC32C and decode + verify kernels and the CRC-only kernel; per
# kernel name, bytes per launch = the line's TB/s x ms for that leg
CRC_CONFIGS = {"crc63": (["--crc", "--corrupt", ""], 6, 3, 1 << 20, 1024)}
CRC_RE = "gf_fused_crc|checksum_chunks512"
# mixed-pattern decode (bench.py --decode-mode mixed: a random 1..m data
# shards lost per stripe): the gf_decode_mixed kernel alone, its algorithmic
# bytes (k survivors read + the e_s rebuilt cells written per stripe) from the
# bench line's roofline.decode_mixed
MIXED_CONFIGS = {
    "mx104": (["--k", "10", "--m", "4", "--stripes", "256", "--decode-mode", "mixed"], 10, 4, 1 << 20, 256),
    "mx63": (["--decode-mode", "mixed"], 6, 3, 1 << 20, 1024),
}
MIXED_RE = "gf_decode_mixed"


def fused_template_args(name):
    """Template arguments of a gf_fused_crc<K, R, SLABS, SCHEME, KIND, VERIFY,
    WPE, PAIR> dispatch name, as strings ([] for other kernels).  The legs are
    told apart by VERIFY (the 6th argument): matching "false" anywhere in the
    name also caught the decode+verify kernel through its PAIR argument."""
    i = name.find("gf_fused_crc<")
    if i < 0:
        return []
    j = name.index(">", i)
    return [t.strip() for t in name[i + len("gf_fused_crc<"):j].split(",")]


def is_fused(name, k, m, verify):
    t = fused_template_args(name)
    return len(t) >= 6 and t[0] == str(k) and t[1] == str(m) and t[5] == ("true" if verify else "false")


def crc_leg_bytes(leg, k, m, cell, stripes, e=None):
    """Algorithmic HBM bytes of one launch of a checksum leg, the 4-B chunk
    sums included: encode + CRC reads k cells, writes m parity cells and
    (k+m) x nchunks sums; decode + verify reads the k survivors and their
    k x nchunks expected sums and writes the e rebuilt cells (the flags are
    written only on a mismatch); the CRC pass reads k+m cells, writes the sums."""
    nck = (cell + 511) // 512
    e = m if e is None else e
    if leg == "encode_crc":
        return ((k + m) * cell + 4 * nck * (k + m)) * stripes
    if leg == "decode_verify":
        return ((k + e) * cell + 4 * nck * k) * stripes
    return ((k + m) * cell + 4 * nck * (k + m)) * stripes


CRC_LEGS = [  # kernel-name test, leg ms key, leg name for crc_leg_bytes
    (lambda n, k, m: is_fused(n, k, m, verify=False), "encode_crc_ms", "encode_crc"),
    (lambda n, k, m: is_fused(n, k, m, verify=True), "decode_verify_ms", "decode_verify"),
    (lambda n, k, m: "checksum_chunks512" in n, "crc_only_ms", "crc_only"),
]


def run(cmd, log, limit):
    with open(log, "w") as f:
        rc = subprocess.call(["timeout", "-k", "10", str(limit)] + cmd, stdout=f, stderr=subprocess.STDOUT,
                             cwd=ROOT)
    if rc != 0:
        sys.stdout.write(open(log).read()[-3000:])
        raise SystemExit(f"step failed rc={rc}: {' '.join(cmd)}")


def rows(d, pattern):
    out = []
    for path in sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True)):
        with open(path) as f:
            out.extend(csv.DictReader(f))
    return out


def bench_line(log):
    for line in reversed(open(log).read().splitlines()):
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    raise SystemExit(f"no bench line in {log}")


def counter(d, name, match=lambda n: KERNEL_RE in n, last=None):
    """Counter value per dispatch (rows summed per Dispatch_Id: a dispatch may
    report several rows), in dispatch order; `last` = keep only the last N
    dispatches -- the bench's timed region.  The spin-up before it is
    time-based, so a --pmc pass (slower kernels) runs fewer spin-up
    dispatches than the trace pass: only the tail lines up across passes."""
    got = {}
    for r in rows(d, "*counter_collection.csv"):
        if match(r.get("Kernel_Name", "")) and r.get("Counter_Name") == name:
            i = int(r["Dispatch_Id"])
            got[i] = got.get(i, 0.0) + float(r["Counter_Value"])
    vals = [got[i] for i in sorted(got)]
    if not vals:
        raise SystemExit(f"no {name} rows under {d}")
    if last is not None:
        if len(vals) < last:
            raise SystemExit(f"{name}: {len(vals)} dispatches under {d}, the timed region has {last}")
        vals = vals[-last:]
    return vals


def profile(out, name):
    args, k, m, cell, stripes, lps = CONFIGS[name]
    d = os.path.join(out, name)
    os.makedirs(d, exist_ok=True)
    bench = ["python3", "bench.py"] + args + COMMON
    prof = ["rocprofv3", "--kernel-trace", "--stats", "-d", os.path.join(d, "trace"), "-o", "run",
            "--output-format", "csv", "--"]
    run(prof + bench, os.path.join(d, "bench_trace.log"), 400)
    line = bench_line(os.path.join(d, "bench_trace.log"))
    for cnt in ("FETCH_SIZE", "WRITE_SIZE"):
        pmc = ["rocprofv3", "--pmc", cnt, "--kernel-include-regex", KERNEL_RE, "-d",
               os.path.join(d, cnt.lower()), "-o", "run", "--output-format", "csv", "--"]
        run(pmc + bench, os.path.join(d, f"bench_{cnt.lower()}.log"), 400)

    trace = [r for r in rows(os.path.join(d, "trace"), "*kernel_trace.csv") if KERNEL_RE in r.get("Kernel_Name", "")]
    trace.sort(key=lambda r: int(r["Start_Timestamp"]))
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9 for r in trace]
    steps = line["steps"]
    timed = durs[-lps * steps:]
    avg_timed = sum(timed) / len(timed)
    avg_all = sum(durs) / len(durs)
    stats = [r for r in rows(os.path.join(d, "trace"), "*kernel_stats.csv") if KERNEL_RE in r["Name"]]
    algo = (k + m) * cell * stripes  # per launch: k cells read + r = m written (uniform decode: e = m)
    fetch = counter(os.path.join(d, "fetch_size"), "FETCH_SIZE", last=lps * steps)
    write = counter(os.path.join(d, "write_size"), "WRITE_SIZE", last=lps * steps)
    fetch_b = 2.0 * 1024 * sum(fetch) / len(fetch)
    write_b = 1024.0 * sum(write) / len(write)
    res = {
        "config": name, "args": " ".join(args + COMMON),
        "k": k, "m": m, "cell": cell, "stripes": stripes, "launches_per_step": lps,
        "kernel": sorted({r["Name"] for r in stats}),
        "dispatches": len(durs),
        "avg_launch_ms_timed_region": round(avg_timed * 1e3, 4),
        "avg_launch_ms_all": round(avg_all * 1e3, 4),
        "stats_avg_ms": [round(float(r["AverageNs"]) * 1e-6, 4) for r in stats],
        "ms_per_step": line["ms_per_step"],
        "kernel_ms_per_step": round(lps * avg_timed * 1e3, 4),
        "kernel_within_step": lps * avg_timed * 1e3 <= line["ms_per_step"],
        "algorithmic_bytes_per_launch": algo,
        "frac_from_trace": round(algo / avg_timed / PEAK, 4),
        "frac_bench_line": line["roofline"]["frac"],
        "fetch_bytes_per_launch": fetch_b, "write_bytes_per_launch": write_b,
        "hbm_bytes_per_launch": fetch_b + write_b,
        "traffic_over_algorithmic": round((fetch_b + write_b) / algo, 5),
        "pmc_dispatches": {"fetch": len(fetch), "write": len(write)},
        "corrections": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count on 16B/lane streaming reads); WRITE_SIZE KiB x1024",
        "bench_line": line,
    }
    with open(os.path.join(out, "summary.jsonl"), "a") as f:
        f.write(json.dumps(res) + "\n")
    print(f"{name}: line {line['value']} GiB/s ms/step {line['ms_per_step']} | kernel {avg_timed * 1e3:.4f} ms x{lps} "
          f"= {lps * avg_timed * 1e3:.4f} | frac trace {res['frac_from_trace']} line {res['frac_bench_line']} | "
          f"traffic x{res['traffic_over_algorithmic']}", flush=True)


def profile_crc(out, name):
    args, k, m, cell, stripes = CRC_CONFIGS[name]
    d = os.path.join(out, name)
    os.makedirs(d, exist_ok=True)
    bench = ["python3", "bench.py"] + args + COMMON
    prof = ["rocprofv3", "--kernel-trace", "--stats", "-d", os.path.join(d, "trace"), "-o", "run",
            "--output-format", "csv", "--"]
    run(prof + bench, os.path.join(d, "bench_trace.log"), 400)
    line = bench_line(os.path.join(d, "bench_trace.log"))
    crc = line["crc32c"]
    for cnt in ("FETCH_SIZE", "WRITE_SIZE"):
        pmc = ["rocprofv3", "--pmc", cnt, "--kernel-include-regex", CRC_RE, "-d",
               os.path.join(d, cnt.lower()), "-o", "run", "--output-format", "csv", "--"]
        run(pmc + bench, os.path.join(d, f"bench_{cnt.lower()}.log"), 400)
    trace = [r for r in rows(os.path.join(d, "trace"), "*kernel_trace.csv")]
    for match, ms_key, leg in CRC_LEGS:
        mine = sorted((r for r in trace if match(r.get("Kernel_Name", ""), k, m)), key=lambda r: int(r["Dispatch_Id"]))
        if not mine:
            raise SystemExit(f"{name}: no dispatch for {ms_key}")
        algo = crc_leg_bytes(leg, k, m, cell, stripes)

        def per_dispatch(cnt):  # counter value per dispatch, in dispatch order
            got = {}
            for r in rows(os.path.join(d, cnt.lower()), "*counter_collection.csv"):
                if match(r.get("Kernel_Name", ""), k, m) and r.get("Counter_Name") == cnt:
                    got[int(r["Dispatch_Id"])] = got.get(int(r["Dispatch_Id"]), 0.0) + float(r["Counter_Value"])
            return [got[i] for i in sorted(got)]
        fetch_all = [2.0 * 1024 * v for v in per_dispatch("FETCH_SIZE")]
        write_all = [1024.0 * v for v in per_dispatch("WRITE_SIZE")]
        if not (len(fetch_all) == len(write_all) == len(mine)):
            raise SystemExit(f"{name}: {ms_key}: {len(mine)} traced vs {len(fetch_all)}/{len(write_all)} PMC dispatches")
        # the same kernel also runs over other cell sets in other legs (the
        # unfused verify pass checks k cells): keep the dispatches whose HBM
        # bytes are this leg's (same dispatch order in all three runs)
        keep = [i for i in range(len(mine)) if abs(fetch_all[i] + write_all[i] - algo) < 0.03 * algo]
        if not keep:
            raise SystemExit(f"{name}: {ms_key}: no dispatch moves the leg's bytes")
        durs = [(int(mine[i]["End_Timestamp"]) - int(mine[i]["Start_Timestamp"])) * 1e-9 for i in keep]
        avg = sum(durs) / len(durs)
        fetch_b = sum(fetch_all[i] for i in keep) / len(keep)
        write_b = sum(write_all[i] for i in keep) / len(keep)
        fetch = write = keep
        res = {
            "config": f"{name}:{ms_key[:-3]}", "args": " ".join(args + COMMON), "k": k, "m": m, "cell": cell,
            "stripes": stripes, "kernel": sorted({mine[i]["Kernel_Name"] for i in keep}),
            "dispatches": len(durs), "dispatches_of_kernel": len(mine),
            "avg_launch_ms_all": round(avg * 1e3, 4), "leg_ms": crc[ms_key],
            "kernel_within_leg": avg * 1e3 <= crc[ms_key] * 1.02,
            "algorithmic_bytes_per_launch": algo, "frac_from_trace": round(algo / avg / PEAK, 4),
            "fetch_bytes_per_launch": fetch_b, "write_bytes_per_launch": write_b,
            "hbm_bytes_per_launch": fetch_b + write_b,
            "traffic_over_algorithmic": round((fetch_b + write_b) / algo, 5),
            "pmc_dispatches": {"fetch": len(fetch), "write": len(write)},
            "corrections": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count on 16B/lane streaming reads); WRITE_SIZE KiB x1024",
            "crc_leg": crc,
        }
        with open(os.path.join(out, "summary_crc.jsonl"), "a") as f:
            f.write(json.dumps(res) + "\n")
        print(f"{res['config']}: kernel {avg * 1e3:.4f} ms (leg {crc[ms_key]} ms) frac trace {res['frac_from_trace']} "
              f"traffic x{res['traffic_over_algorithmic']}", flush=True)


def profile_mixed(out, name):
    args, k, m, cell, stripes = MIXED_CONFIGS[name]
    d = os.path.join(out, name)
    os.makedirs(d, exist_ok=True)
    bench = ["python3", "bench.py"] + args + COMMON
    prof = ["rocprofv3", "--kernel-trace", "--stats", "-d", os.path.join(d, "trace"), "-o", "run",
            "--output-format", "csv", "--"]
    run(prof + bench, os.path.join(d, "bench_trace.log"), 400)
    line = bench_line(os.path.join(d, "bench_trace.log"))
    dm = line["roofline"]["decode_mixed"]
    for cnt in ("FETCH_SIZE", "WRITE_SIZE"):
        pmc = ["rocprofv3", "--pmc", cnt, "--kernel-include-regex", MIXED_RE, "-d",
               os.path.join(d, cnt.lower()), "-o", "run", "--output-format", "csv", "--"]
        run(pmc + bench, os.path.join(d, f"bench_{cnt.lower()}.log"), 400)
    trace = sorted((r for r in rows(os.path.join(d, "trace"), "*kernel_trace.csv")
                    if MIXED_RE in r.get("Kernel_Name", "")), key=lambda r: int(r["Start_Timestamp"]))
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9 for r in trace]
    timed = durs[-line["steps"]:]
    avg = sum(timed) / len(timed)
    algo = dm["algorithmic_bytes_per_launch"]
    match = lambda n: MIXED_RE in n  # noqa: E731
    # every dispatch of the timed region (the last `steps` decode launches of
    # each pass), each dispatch's rows summed
    fetch = counter(os.path.join(d, "fetch_size"), "FETCH_SIZE", match, last=line["steps"])
    write = counter(os.path.join(d, "write_size"), "WRITE_SIZE", match, last=line["steps"])
    fetch_b = 2.0 * 1024 * sum(fetch) / len(fetch)
    write_b = 1024.0 * sum(write) / len(write)
    per = [2.0 * 1024 * f_ + 1024.0 * w_ for f_, w_ in zip(fetch, write)]
    res = {
        "config": name, "args": " ".join(args + COMMON), "k": k, "m": m, "cell": cell, "stripes": stripes,
        "erased_cells": dm["erased_cells"], "kernel": sorted({r["Kernel_Name"] for r in trace}),
        "dispatches": len(durs), "avg_launch_ms_timed_region": round(avg * 1e3, 4),
        "bench_decode_avg_launch_ms": dm["avg_launch_ms"],
        "algorithmic_bytes_per_launch": algo, "frac_from_trace": round(algo / avg / PEAK, 4),
        "frac_bench_line": dm["frac"], "frac_bench_line_encode_plus_decode": line["roofline"]["frac"],
        "fetch_bytes_per_launch": fetch_b, "write_bytes_per_launch": write_b,
        "hbm_bytes_per_launch": fetch_b + write_b,
        "traffic_over_algorithmic": round((fetch_b + write_b) / algo, 5),
        "pmc_dispatches": {"fetch": len(fetch), "write": len(write), "timed_region": line["steps"]},
        # (max - min) / mean of the per-dispatch corrected HBM bytes: every
        # timed launch decodes the same stripes, so this should be ~0
        "traffic_per_dispatch_spread": round((max(per) - min(per)) / (sum(per) / len(per)), 6),
        "corrections": "FETCH_SIZE KiB x1024 x2 (gfx950 half-count on 16B/lane streaming reads); WRITE_SIZE KiB x1024",
        "bench_line": line,
    }
    with open(os.path.join(out, "summary_mixed.jsonl"), "a") as f:
        f.write(json.dumps(res) + "\n")
    print(f"{name}: mixed decode kernel {avg * 1e3:.4f} ms (line {dm['avg_launch_ms']}) frac trace "
          f"{res['frac_from_trace']} line {dm['frac']} (enc+dec {line['roofline']['frac']}) "
          f"traffic x{res['traffic_over_algorithmic']}", flush=True)


def write_traffic(out, tag):
    """pmc_traffic_configs.json: what bench.py reads for roofline.traffic
    (matched on k, m, cell, stripes and decode mode)."""
    path = os.path.join(out, "summary.jsonl")
    rows = [json.loads(ln) for ln in open(path)] if os.path.exists(path) else []
    cfgs = [{"config": r["config"], "k": r["k"], "m": r["m"], "cell": r["cell"], "stripes": r["stripes"],
             "decode_mode": "uniform", "kernel": r["kernel"],
             "fetch_bytes_per_launch": r["fetch_bytes_per_launch"], "write_bytes_per_launch": r["write_bytes_per_launch"],
             "hbm_bytes_per_launch": r["hbm_bytes_per_launch"],
             "algorithmic_bytes_per_launch": r["algorithmic_bytes_per_launch"],
             "traffic_over_algorithmic": r["traffic_over_algorithmic"]} for r in rows]
    with open(os.path.join(out, "pmc_traffic_configs.json"), "w") as f:
        json.dump({"tag": tag, "corrections": rows[0]["corrections"] if rows else None, "configs": cfgs}, f, indent=1)


def main():
    out = sys.argv[1]
    names = sys.argv[2:] or list(CONFIGS) + list(CRC_CONFIGS) + list(MIXED_CONFIGS)
    os.makedirs(out, exist_ok=True)
    os.environ["TMPDIR"] = "/tmp"
    for n in names:
        (profile_crc if n in CRC_CONFIGS else profile_mixed if n in MIXED_CONFIGS else profile)(out, n)
    write_traffic(out, os.path.basename(os.path.normpath(out)))
    print("profile_configs ok", flush=True)


if __name__ == "__main__":
    main()
