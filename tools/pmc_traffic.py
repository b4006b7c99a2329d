"""Summarise rocprofv3 output per kernel family (for profiles/ and bench.py's roofline).

    python tools/pmc_traffic.py --trace DIR [--fetch DIR] [--write DIR] --steps K \
        --out profiles/rNN_summary.json

--trace  a `rocprofv3 --kernel-trace --stats --output-format csv` directory: average launch
         duration per family (compare with bench.py's live HIP-event numbers).
--fetch / --write  `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE` directories (separate
         passes: the two do not fit one TCC pass on gfx950).  HBM bytes per launch are
         (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE/WRITE_SIZE are in KiB, and on gfx950
         FETCH_SIZE counts half the bytes of a wide coalesced read (MI355X_MICROARCH.md, HBM).
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
from collections import defaultdict

# kernel-name substring -> the engine's probe family (latice/engine.py _launch names)
FAMILIES = [
    ("conv3x3_big_kernel", "conv3x3_fwd"),
    ("conv3x3_small_kernel", "conv3x3_fwd"),
    ("conv3x3_split_kernel", "conv3x3_fwd"),
    ("conv3x3_pipe_kernel", "conv3x3_fwd"),
    ("ev::wgrad_kernel<", "conv3x3_wgrad"),
    ("wgrad_split_kernel", "conv3x3_wgrad"),
    ("wgrad_pipe_kernel", "conv3x3_wgrad"),
    ("pack_wmax", "pack_weight"),
    ("pack_split", "pack_weight"),
    ("pack_conv_weights", "pack_weight"),
    ("wgrad_reduce", "wgrad_reduce"),
    ("in_bwd_edge_kernel", "in_bwd_edge"),
    ("in_bwd_kernel", "in_bwd"),
    ("in_bwd_finalize", "in_bwd"),
    ("in_stats_finalize", "in_stats"),
    ("conv_cout1", "conv_cout1"),
    ("heads_", "heads"),
    ("loss_", "loss"),
    ("adam", "adam"),
    ("pack_conv_weight", "pack_weight"),
]


def family(name: str) -> str:
    for sub, fam in FAMILIES:
        if sub in name:
            return fam
    return "other"


def _csv(d: str, suffix: str):
    hits = glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True)
    if not hits:
        raise SystemExit(f"no *{suffix} under {d}")
    with open(hits[0], newline="") as f:
        return list(csv.DictReader(f))


def _fold(rows):
    fam = defaultdict(lambda: {"launches": 0, "ns": 0.0})
    for r in rows:
        f = fam[family(r["Kernel_Name"])]
        f["launches"] += 1
        f["ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return fam


def trace_summary(d: str, steps: int):
    out = {}
    for k, v in _fold(_csv(d, "kernel_trace.csv")).items():
        out[k] = {"launches": v["launches"], "avg_launch_us": round(v["ns"] / v["launches"] / 1e3, 2),
                  "ms_per_step": round(v["ns"] / 1e6 / steps, 3) if steps else None}
    return out


def probed_summary(d: str, warmup: int, timed: int, every: int):
    """Per-family averages over the steps bench.py probes (timed step i with i % every == 0,
    after `warmup` steps): the launches its HIP events time, for a like-for-like comparison.
    Steps are delimited by their Adam launch (one per training step)."""
    rows = sorted(_csv(d, "kernel_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"]]
    if len(ends) != warmup + timed:
        return {"error": f"{len(ends)} Adam launches in the trace, expected {warmup + timed}"}
    want = {warmup + i for i in range(timed) if i % every == 0}
    sel = []
    for s, e in enumerate(ends):
        if s in want:
            sel += rows[(ends[s - 1] + 1 if s else 0):e + 1]
    out = {}
    for k, v in _fold(sel).items():
        out[k] = {"launches": v["launches"], "avg_launch_us": round(v["ns"] / v["launches"] / 1e3, 2),
                  "ms_per_step": round(v["ns"] / 1e6 / len(want), 3)}
    return {"steps": sorted(want), "families": out}


def counter(d: str, name: str):
    per = defaultdict(list)
    for r in _csv(d, "counter_collection.csv"):
        if r.get("Counter_Name") == name:
            per[family(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trace", required=True)
    ap.add_argument("--fetch")
    ap.add_argument("--write")
    ap.add_argument("--steps", type=int, default=0, help="timed+warmup steps in the profiled run")
    ap.add_argument("--probed", default="",
                    help="WARMUP:TIMED:EVERY of the traced bench run: also average its probed steps")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    res = {"trace": trace_summary(a.trace, a.steps)}
    if a.probed:
        w, t, e = (int(v) for v in a.probed.split(":"))
        res["trace_probed_steps"] = probed_summary(a.trace, w, t, e)
    if a.fetch and a.write:
        fetch, write = counter(a.fetch, "FETCH_SIZE"), counter(a.write, "WRITE_SIZE")
        traffic = {}
        for k in sorted(set(fetch) & set(write)):
            fk = sum(fetch[k]) / len(fetch[k])
            wk = sum(write[k]) / len(write[k])
            traffic[k] = {"launches": len(fetch[k]), "fetch_size_kib": round(fk, 1),
                          "write_size_kib": round(wk, 1),
                          "hbm_bytes_per_launch": round((2.0 * fk + wk) * 1024.0)}
        res["traffic"] = traffic
        res["traffic_formula"] = "(2*FETCH_SIZE + WRITE_SIZE) * 1024 per launch (gfx950 FETCH_SIZE is half)"
        # per training step: the profiled run's steps = its Adam launches (one per step;
        # the "adam" family also holds the step-counter kernel)
        nsteps = sum(1 for r in _csv(a.fetch, "counter_collection.csv")
                     if r.get("Counter_Name") == "FETCH_SIZE" and "adam_kernel" in r["Kernel_Name"]) or None
        if nsteps:
            tot = sum(sum(fetch[k]) * 2.0 + sum(write[k]) for k in set(fetch) & set(write)) * 1024.0
            res["hbm_bytes_per_step"] = round(tot / nsteps)
            res["hbm_bytes_per_step_by_family"] = {
                k: round((2.0 * sum(fetch[k]) + sum(write[k])) * 1024.0 / nsteps)
                for k in sorted(set(fetch) & set(write))}
            res["steps_in_pmc_run"] = nsteps
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print(json.dumps(res, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
