"""Per-layer breakdown of torch.profiler chrome traces by the engine's phase ranges.

Library behind tools/prof.py and the train driver's --debug output (see
deepspeech_amd/utils/trace.py for the phase names). Reference counterpart:
tools/prof.py of yxlao/deepSpeech (TF timeline -> per-layer periods/gaps CSVs).
"""
from __future__ import annotations

import bisect
import csv
import json
import os
import sys
from collections import OrderedDict, defaultdict


def load_events(path):
    with open(path) as f:
        data = json.load(f)
    return data["traceEvents"] if isinstance(data, dict) else data


def _is_launch(ev):
    n = ev.get("name", "")
    return ev.get("cat") in ("cuda_runtime", "hip_runtime", "cuda_driver") and (
        "Launch" in n or "launch" in n or "Memcpy" in n or "Memset" in n)


def analyse(events, threshold_us=50.0):
    ann = defaultdict(list)       # tid -> [(ts, end, name)]
    launches = []
    kernels = []
    cpu_ops = []
    for ev in events:
        if ev.get("ph") != "X":
            continue
        cat = ev.get("cat", "")
        if cat == "user_annotation":
            ann[ev.get("tid")].append((float(ev["ts"]), float(ev["ts"]) + float(ev.get("dur", 0)), ev["name"]))
        elif _is_launch(ev):
            launches.append(ev)
        elif cat in ("kernel", "gpu_memcpy", "gpu_memset"):
            kernels.append(ev)
        elif cat == "cpu_op":
            cpu_ops.append(ev)
    for tid in ann:
        ann[tid].sort()
    starts = {tid: [a[0] for a in v] for tid, v in ann.items()}

    def phase_at(tid, ts):
        v = ann.get(tid)
        if not v:
            return None
        i = bisect.bisect_right(starts[tid], ts)
        best = None
        # innermost enclosing range = the latest-starting one that still covers ts
        for j in range(i - 1, -1, -1):
            s, e, name = v[j]
            if s <= ts <= e:
                best = name
                break
        return best

    if not kernels:
        # CPU-only trace: attribute the top-level CPU ops (not nested in another op) instead
        by_tid = defaultdict(list)
        for ev in cpu_ops:
            by_tid[ev.get("tid")].append(ev)
        for tid, evs in by_tid.items():
            evs.sort(key=lambda e: (float(e["ts"]), -float(e.get("dur", 0))))
            end = -1.0
            for ev in evs:
                ts = float(ev["ts"])
                if ts >= end:
                    ev = dict(ev)
                    ev.setdefault("args", {})
                    ev["args"] = dict(ev["args"], correlation=("cpu", tid, ts))
                    launches.append({"tid": tid, "ts": ts, "args": {"correlation": ("cpu", tid, ts)}})
                    kernels.append(ev)
                    end = ts + float(ev.get("dur", 0))
    corr_phase = {}
    for ev in launches:
        c = (ev.get("args") or {}).get("correlation")
        if c is not None:
            corr_phase[c] = phase_at(ev.get("tid"), float(ev["ts"]))
    per = OrderedDict()
    rows = []
    for k in sorted(kernels, key=lambda e: float(e["ts"])):
        c = (k.get("args") or {}).get("correlation")
        ph = corr_phase.get(c) or "(unattributed)"
        ts, dur = float(k["ts"]), float(k.get("dur", 0))
        d = per.setdefault(ph, {"kernels": 0, "kernel_us": 0.0, "first": ts, "last": ts + dur, "ivals": []})
        d["kernels"] += 1
        d["kernel_us"] += dur
        d["first"] = min(d["first"], ts)
        d["last"] = max(d["last"], ts + dur)
        d["ivals"].append((ts, ts + dur))
        rows.append((ph, k.get("name", ""), ts, dur))
    out = OrderedDict()
    for ph, d in per.items():
        iv = sorted(d["ivals"])
        gaps, gaps_small = 0.0, 0.0
        end = iv[0][1]
        for s, e in iv[1:]:
            if s > end:
                g = s - end
                gaps += g
                if g < threshold_us:
                    gaps_small += g
            end = max(end, e)
        out[ph] = {"kernels": d["kernels"], "kernel_ms": d["kernel_us"] / 1000.0,
                   "span_ms": (d["last"] - d["first"]) / 1000.0, "gap_ms": gaps / 1000.0,
                   "gap_below_threshold_ms": gaps_small / 1000.0}
    return out, rows


def write_outputs(out, rows, folder):
    os.makedirs(folder, exist_ok=True)
    with open(os.path.join(folder, "layers_exeTime.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["layer", "kernels", "kernel_ms", "span_ms"])
        for k, v in out.items():
            w.writerow([k, v["kernels"], "%.4f" % v["kernel_ms"], "%.4f" % v["span_ms"]])
    with open(os.path.join(folder, "layers_gaps.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["layer", "gap_ms", "gap_below_threshold_ms"])
        for k, v in out.items():
            w.writerow([k, "%.4f" % v["gap_ms"], "%.4f" % v["gap_below_threshold_ms"]])
    with open(os.path.join(folder, "kernels.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["layer", "kernel", "ts_us", "dur_us"])
        for r in rows:
            w.writerow([r[0], r[1], "%.3f" % r[2], "%.3f" % r[3]])


def format_table(out):
    tot = sum(v["kernel_ms"] for v in out.values()) or 1.0
    lines = ["%-34s %8s %11s %9s %9s %7s" % ("layer", "kernels", "kernel_ms", "span_ms", "gap_ms", "%")]
    for k, v in sorted(out.items(), key=lambda kv: -kv[1]["kernel_ms"]):
        lines.append("%-34s %8d %11.3f %9.3f %9.3f %6.1f%%" % (k, v["kernels"], v["kernel_ms"], v["span_ms"],
                                                               v["gap_ms"], 100.0 * v["kernel_ms"] / tot))
    return "\n".join(lines)


