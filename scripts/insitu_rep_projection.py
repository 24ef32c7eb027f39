"""Projection of the configs[2] frame (wavelets64, 1024x1024x8spp, PT) at
N = 2 / 4 / 8 GPUs for the replicated-ray in-situ frame, from MEASURED
per-rank device times and a stated model of the collectives.

    python scripts/insitu_rep_projection.py profiles/r4_rep_rehearse.json \
        [--n1-ms 0.77] [--out profiles/r4_insitu_projection.json]

Inputs
* rehearse.json (scripts/insitu_rep_rehearse.py on one MI355X): for each N
  and partition, every rank's per-phase device time of the frame (HIP events;
  the ranks' device work serialised, so a rank's times are its own kernels'
  times), and the one-rank RCCL all-reduce times of the frame's message
  sizes (the per-call floor).
* the measured N = 1 frame (the bench's fused single-GPU frame, --n1-ms).
* optionally (--kernels) the same runs' per-rank segment times from rocprofv3
  kernel traces (scripts/rehearse_kernel_segments.py): robust against the
  rehearsal's clock drops after its long host-collective gaps, and the
  numbers DESIGN quotes.

Model of one frame at N ranks (every rank runs the same sequence):
  PT: T = max_r(cull + select + film slots + keyed closest hit & shading)
          + AR(4 |C'|) + max_r(list positions + shadow any hit + winners)
          + AR(|C'| + 192) + max_r(film + totals) + RED(12 runs)
          (C' = rays entering the scene box; t bits MIN; the list positions'
          u8 MIN overlaps the shadow any hit; runs = the pixel runs along C')
  AO: T = max_r(route + select + keyed closest hit) + AR(8 |C|) + max_r(publish)
          + AR(16 |C|) + max_r(AO spawn + any hit) + AR(2 fb |C|)
          + max_r(film + totals)  (fb = 2 / 4 / 8 bits for N <= 3 / 15 / 64;
                                   no image reduce: rank 0 films all)
  AR(B)  = alpha + 2 (N - 1) / N * B / bw     (ring all-reduce)
  RED(B) = alpha + (N - 1) / N * B / bw * 2   (reduce to rank 0 as reduce-
           scatter + gather)
The phases are taken per rank and maxed per phase (each phase ends in a
collective every rank waits for).  alpha and bw are NOT measured (no
multi-GPU box): the table gives a conservative and an optimistic pair.
"""
import argparse
import json

LINK = {  # per-collective latency (ms) and ring bus bandwidth (GB/s) at 8 GPUs
    "conservative": {"alpha_ms": 0.030, "bw_GBs": 300.0},
    "optimistic": {"alpha_ms": 0.015, "bw_GBs": 500.0},
}
IMAGE_BYTES = 1024 * 1024 * 16


def ar(b, n, link):
    return link["alpha_ms"] + 2.0 * (n - 1) / n * b / (link["bw_GBs"] * 1e9) * 1e3


def red(b, n, link):
    return link["alpha_ms"] + 2.0 * (n - 1) / n * b / (link["bw_GBs"] * 1e9) * 1e3


def fbits(n):
    return 2 if n <= 3 else (4 if n <= 15 else 8)


SEGMENTS = {  # phases between the frame's collectives, in order
    "pt": [("cull_select", "film_slots", "keyed_shade"), ("list_pos", "shadow_trace", "winners"),
           ("film_totals",)],
    "ao": [("route", "cull_select", "select", "keyed_closest_hit"), ("publish",),
           ("ao_spawn", "ao_trace", "ao_own_trace"), ("film_totals",)],
}


def project(run, link, seg=None):
    n = run["world"]
    ranks = run["ranks"]
    kind = run.get("kind", "pt")
    ph = lambda r, k: r["phases_ms"].get(k, 0.0)  # noqa: E731
    # every segment ends in a collective all ranks wait for: its busiest rank
    # (HIP-event phases, or the kernel traces' segment sums when given)
    if seg is None:
        seg = [max(sum(ph(r, k) for k in names) for r in ranks) for names in SEGMENTS[kind]]
    nc = ranks[0]["nc"]
    if kind == "ao":
        fb = fbits(n)
        comm = ar(8 * nc, n, link) + ar(16 * nc, n, link) + ar(2 * fb * nc, n, link)
    else:
        # t bits MIN, then occlusion bytes + totals SUM (the list positions'
        # MIN runs beside the shadow any hit), the film's run sums to rank 0
        comm = ar(4 * nc, n, link) + ar(nc + 192, n, link) + red(12 * ranks[0]["pixel_runs"], n,
                                                                  link)
    dev = sum(seg)
    return {"device_ms": round(dev, 4), "comm_ms": round(comm, 4),
            "frame_ms": round(dev + comm, 4),
            "busiest_per_segment": [round(x, 4) for x in seg]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("rehearse")
    ap.add_argument("--n1-ms", type=float, default=0.77, help="measured N = 1 PT frame")
    ap.add_argument("--n1-ao-ms", type=float, default=None, help="measured N = 1 AO frame")
    ap.add_argument("--kernels", default=None,
                    help="segments.json of scripts/rehearse_kernel_segments.py (per-rank "
                         "kernel-trace segment times of the same runs)")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    rep = json.load(open(args.rehearse))
    ksegs = {}
    if args.kernels:
        for r in json.load(open(args.kernels))["runs"]:
            ksegs[(r["world"], r["partition"], r["kind"])] = r["busiest_per_segment_ms"]
    rows = []
    for run in rep["runs"]:
        if run.get("kind", "pt") not in ("pt", "ao"):
            continue
        row = {"world": run["world"], "partition": run["partition"],
               "kind": run.get("kind", "pt"),
               "domains_per_rank": [r["domains"] for r in run["ranks"]],
               "rank_device_ms": [round(sum(v for k, v in r["phases_ms"].items()
                                            if k != "collectives"), 4) for r in run["ranks"]]}
        for name, link in LINK.items():
            p = project(run, link)
            base = args.n1_ms if row["kind"] == "pt" else args.n1_ao_ms
            p["speedup_vs_n1"] = round(base / p["frame_ms"], 3) if base else None
            row[name] = p
        key = (run["world"], run["partition"], row["kind"])
        if key in ksegs:  # the same frame from the kernel traces
            for name, link in LINK.items():
                p = project(run, link, ksegs[key])
                base = args.n1_ms if row["kind"] == "pt" else args.n1_ao_ms
                p["speedup_vs_n1"] = round(base / p["frame_ms"], 3) if base else None
                row["kernel_trace_" + name] = p
        rows.append(row)
    out = {"model": __doc__.strip().split("\n\n")[2], "links": LINK, "n1_ms": args.n1_ms,
           "rccl_one_rank_floor": rep.get("rccl_one_rank_floor"), "rows": rows}
    print("| frame | N | partition | busiest rank per segment (ms) | device ms | comm ms (cons.) "
          "| frame ms (cons. / opt.) | x N=1 (cons. / opt.) |")
    print("|---|---|---|---|---|---|---|---|")
    sx = lambda v: "-" if v is None else "%.2f" % v  # noqa: E731
    for r in rows:
        c, o = r["conservative"], r["optimistic"]
        print("| %s | %d | %s | %s | %.3f | %.3f | %.3f / %.3f | %s / %s |" % (
            r["kind"], r["world"], r["partition"],
            " + ".join("%.3f" % x for x in c["busiest_per_segment"]), c["device_ms"],
            c["comm_ms"], c["frame_ms"], o["frame_ms"], sx(c["speedup_vs_n1"]),
            sx(o["speedup_vs_n1"])))
        if "kernel_trace_conservative" in r:
            c, o = r["kernel_trace_conservative"], r["kernel_trace_optimistic"]
            print("| %s (kernel trace) | %d | %s | %s | %.3f | %.3f | %.3f / %.3f | %s / %s |" % (
                r["kind"], r["world"], r["partition"],
                " + ".join("%.3f" % x for x in c["busiest_per_segment"]), c["device_ms"],
                c["comm_ms"], c["frame_ms"], o["frame_ms"], sx(c["speedup_vs_n1"]),
                sx(o["speedup_vs_n1"])))
    if args.out:
        with open(args.out, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
