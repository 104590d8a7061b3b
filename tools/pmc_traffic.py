"""Parse rocprofv3 PMC passes into per-kernel-INSTANCE figures per launch (medians), stamped with the
kernel sources' sha256 and the bench workload they were measured on, so bench.py only attaches
counters of the same kernel instance, build and workload.

  HBM bytes: FETCH_SIZE / WRITE_SIZE passes; counters in KB (x1024); on gfx950 FETCH_SIZE reports
             half the bytes of wide (16 B/lane) streaming reads -> doubled (MI355X_MICROARCH.md, HBM).
  MFMA:      SQ_VALU_MFMA_BUSY_CYCLES (cycles, summed over SIMDs) and GRBM_GUI_ACTIVE (GPU-busy cycles
             summed over the 8 XCDs): mfma_util = MFMA_BUSY / (SIMDs x GRBM_GUI_ACTIVE / 8).

    python tools/pmc_traffic.py <workload> <out.json> <fetch.csv> <write.csv> [<sq.csv> [<trace.csv> <steps>
                                [<pmc_trace.csv> <schedule>]]]
"""
import csv
import hashlib
import json
import os
import re
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOT_SOURCES = ["mgn_common.h", "mgn_chain.h", "mgn_chain16_dev.h", "mgn_mlp.hip", "mgn_chain16.hip", "mgn_rew.hip",
               "mgn_graph.hip"]
SIMDS = 256 * 4  # MI355X: 256 CUs x 4 SIMDs
XCDS = 8


def sources_sha():
    """sha256 of the training-step kernel sources (graph construction in mgn_build.hip is not in the step)."""
    h = hashlib.sha256()
    for f in HOT_SOURCES:
        h.update(open(os.path.join(ROOT, "graph-physics_amd", "csrc", f), "rb").read())
    return h.hexdigest()[:16]


def kernel_class(name):
    """bench.py / libmgn profiler class of a kernel instance (None: not a training-step class)."""
    # generic MLP kernels, mangled (..._kernelIfLi128ELi32ELi1E...) or demangled (<float, 128, 32, 1>)
    m = re.search(r"mlp_(fwd|bwd)_kernel(?:.*?Li(\d+)ELi(\d+)ELi(\d)E|<[^,<>]+, (\d+), (\d+), (\d)(?:, (?:true|false))?>)", name)
    if m:
        mode = m.group(4) or m.group(7)
        return f"{m.group(1)}_" + {"0": "dense", "1": "edge", "2": "node"}[mode]
    for key, cls in (("chain16_node_fwd_kernel", "fwd_node"), ("chain16_node_bwd_kernel", "bwd_node"),
                     ("chain16_dense_fwd_kernel", "fwd_dense"), ("chain16_dense_bwd_kernel", "bwd_dense"),
                     ("chain16_fwd_kernel", "fwd_edge"), ("chain16_bwd_kernel", "bwd_edge"),
                     ("edge_fwd_f32_chain_kernel", "fwd_edge"), ("edge_bwd_f32_chain_kernel", "bwd_edge"),
                     ("node_fwd_f32_chain_kernel", "fwd_node"), ("node_fwd_f32_split_kernel", "fwd_node"),
                     ("node_bwd_f32_chain_kernel", "bwd_node"),
                     ("mlp_wgrad_kernel", "wgrad_dense"), ("wgrad_ring_kernel", "wgrad"),
                     ("wgrad_ring_f32_kernel", "wgrad"), ("chain16_rew_kernel", "wgrad"),
                     ("wgrad_reduce_kernel", "wgrad_reduce"), ("node_grad_kernel", "combine"),
                     ("node_proj_kernel", "proj"), ("adamw", "adamw"), ("pack_kernel", "pack")):
        if key in name:
            return cls
    return None


def instance_key(r):
    return "%s|grid=%s" % (r["Kernel_Name"], r.get("Grid_Size", r.get("Grid_Size_X", "")))


def load(path):
    """{instance: {counter: [values per launch]}}"""
    per = {}
    if not path or not os.path.exists(path):
        return per
    for r in csv.DictReader(open(path)):
        if kernel_class(r["Kernel_Name"]) is None:
            continue
        per.setdefault(instance_key(r), {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return per


def block_wgrad(name, launches_per_step, mp):
    """The generic kernels' weight-gradient launch of a processor block (block_wgrad_generic: one multi-job
    mlp_wgrad_kernel launch per block, hidden 16/32/64 — Cfg A, Cfg C) is bench.py's class "wgrad", like
    the ring of the h=128 blocks; the encoders' / decoder's mlp_wgrad_kernel launches stay "wgrad_dense".
    Told apart by their count: MP launches per step."""
    return "mlp_wgrad_kernel" in name and mp and abs(launches_per_step - mp) < 1e-9


def _mp(workload):
    m = re.search(r":mp(\d+):", ":" + (workload or "") + ":")
    return int(m.group(1)) if m else None


def replay_classes(trace_csv, steps, workload=None):
    """Per-class device time of the last `steps` REPLAYED steps of a rocprofv3 kernel trace (a step
    starts at its preamble_stats launch, as tools/gap_summary.py): {class: {us_per_step, launches_per_step,
    avg_us}} — what bench.py picks its dominant kernel class from (the replay, not eager steps)."""
    rows = sorted(csv.DictReader(open(trace_csv)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("preamble_stats")]
    seg = rows[starts[-steps]:]
    mp = _mp(workload)
    count = {}
    for r in seg:
        count[instance_key(r)] = count.get(instance_key(r), 0) + 1
    agg = {}
    for r in seg:
        c = kernel_class(r["Kernel_Name"])
        if c is None:
            continue
        if block_wgrad(r["Kernel_Name"], count[instance_key(r)] / steps, mp):
            c = "wgrad"
        agg.setdefault(c, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return {c: {"us_per_step": round(sum(v) / steps, 2), "launches_per_step": len(v) / steps,
                "avg_us": round(sum(v) / len(v), 2)} for c, v in agg.items()}


def trace_durations(trace_csv):
    """{instance: median duration in us} of every training-step kernel launch in a kernel trace."""
    per = {}
    for r in csv.DictReader(open(trace_csv)):
        if kernel_class(r["Kernel_Name"]) is None:
            continue
        key = "%s|grid=%s" % (r["Kernel_Name"], r.get("Grid_Size", r.get("Grid_Size_X", "")))
        per.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return {k: statistics.median(v) for k, v in per.items()}


def main(workload, out, fetch_csv, write_csv, sq_csv=None, trace_csv=None, steps=5, pmc_trace_csv=None,
         schedule=None):
    """pmc_trace_csv: a kernel trace of the bench command run with the SAME schedule as the PMC passes
    (profile_round.sh: one stream, MGN_CONC_WGRAD=0), so every PMC record carries the duration of its own
    launches (`trace_us`) and the clock its GRBM_GUI_ACTIVE implies over them; trace_csv (the default
    schedule) gives the replayed step's per-class times."""
    f, w, q = load(fetch_csv), load(write_csv), load(sq_csv)
    durs = trace_durations(pmc_trace_csv) if pmc_trace_csv else {}
    res = {}
    for key in sorted(set(f) | set(w) | set(q)):
        name = key.split("|grid=")[0]
        d = {"class": kernel_class(name), "kernel": name, "grid": key.split("|grid=")[1]}
        if key in f and "FETCH_SIZE" in f[key]:
            d["fetch_bytes"] = 2.0 * 1024.0 * statistics.median(f[key]["FETCH_SIZE"])
            d["launches"] = len(f[key]["FETCH_SIZE"])
        if key in w and "WRITE_SIZE" in w[key]:
            d["write_bytes"] = 1024.0 * statistics.median(w[key]["WRITE_SIZE"])
        if "fetch_bytes" in d and "write_bytes" in d:
            d["hbm_bytes"] = d["fetch_bytes"] + d["write_bytes"]
        for c, v in q.get(key, {}).items():
            d[c] = statistics.median(v)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in d and d.get("GRBM_GUI_ACTIVE"):
            d["mfma_util"] = d["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * d["GRBM_GUI_ACTIVE"] / XCDS)
        if d.get("GRBM_GUI_ACTIVE"):
            d["grbm_us_at_2400MHz"] = round(d["GRBM_GUI_ACTIVE"] / XCDS / 2400.0, 2)
        if key in durs:
            d["trace_us"] = round(durs[key], 2)
            if d.get("GRBM_GUI_ACTIVE"):
                d["implied_clock_mhz"] = round(d["GRBM_GUI_ACTIVE"] / XCDS / durs[key], 0)
        res[key] = d
    # processor blocks' generic weight-gradient launches: class "wgrad" (block_wgrad); steps profiled =
    # AdamW launches (one per step)
    nsteps = sum(d.get("launches", 0) for d in res.values() if d["class"] == "adamw")
    for d in res.values():
        if nsteps and block_wgrad(d["kernel"], d.get("launches", 0) / nsteps, _mp(workload)):
            d["class"] = "wgrad"
    doc = {"sources_sha": sources_sha(), "workload": workload, "fetch_correction": 2.0,
           "unit": "per launch (median over launches)", "kernels": res,
           "schedule": schedule or "default (MGN_CONC_WGRAD=auto)"}
    if trace_csv:
        doc["replay"] = replay_classes(trace_csv, int(steps), workload)
        doc["replay_source"] = "rocprofv3 --kernel-trace of the same bench command, last %s replayed steps" % steps
    json.dump(doc, open(out, "w"), indent=1)
    for k, d in res.items():
        print(f"{d['class']:12s} {d.get('hbm_bytes', 0) / 1e6:8.1f} MB  mfma_util {d.get('mfma_util', float('nan')):.3f}"
              f"  {d['kernel'][:60]} grid={d['grid']}")


if __name__ == "__main__":
    main(*sys.argv[1:])
