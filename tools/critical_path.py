"""Critical path of one single c3 registration: device kernel spans (rocprofv3 kernel
trace) merged with phase B's host marks (FCCF_HOST_TRACE=1), VERDICT r3 item 7.

  run:     FCCF_HOST_TRACE=1 rocprofv3 --kernel-trace -f csv -d OUT -o run -- \
               python3 tools/critical_path.py run [reps] 2> host.log
  report:  python3 tools/critical_path.py report OUT host.log [out.txt]

The report takes the last registration of the run: its host marks (microseconds after
the cloud stage was enqueued) and every kernel that overlaps it, and splits the
registration into the segments that follow each other on its critical path.
"""
import csv
import glob
import os
import re
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(reps):
    sys.path.insert(0, os.path.join(ROOT, "fccf-pcr_amd"))
    import fccf_amd as F
    cfg = F.CONFIGS["c3"]
    src, tar, _ = F.synth_pair(cfg["n"], cfg["room"])
    ctx = F.Ctx(0)
    ds, dt = ctx.upload(src), ctx.upload(tar)
    e2e = []
    for i in range(reps + 3):
        a = time.perf_counter()
        ctx.register_device(ds, len(src), dt, len(tar), cfg["leaf"])
        if i >= 3:
            e2e.append((time.perf_counter() - a) * 1e3)
        time.sleep(0.005)  # registrations apart on the trace
    print(f"e2e median {statistics.median(e2e):.3f} ms over {reps}", flush=True)


STAGE = [  # (segment, first kernel, last kernel) by name prefix, in device order
    ("main VoxelGrid (K1)", "k_vg_bbox", "k_vg_centroid"),
    ("driver pass", "k_finite_fix", "k_vg_centroid"),
    ("face stage", "k_block_aggr", "k_compact_planar"),
]


def short(name):
    m = re.search(r"(k_\w+|__amd\w+)", name)
    return m.group(1) if m else name[:40]


def report(trace_dir, host_log, out=None):
    lines = [l for l in open(host_log) if l.startswith("host trace t0_mono_ns=")]
    if not lines:
        raise SystemExit("no host trace lines (FCCF_HOST_TRACE=1?)")
    m = re.match(r"host trace t0_mono_ns=(\d+) boot_minus_mono_ns=(-?\d+):(.*)", lines[-1].strip())
    t0_mono, boff, rest = int(m.group(1)), int(m.group(2)), m.group(3)
    marks = [(k, float(v)) for k, v in re.findall(r"(\w+)=([\d.]+)", rest)]
    rows = []
    for f in glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                         r.get("Stream_Id", r.get("Queue_Id", "?"))))
    rows.sort()
    end_us = max(v for _, v in marks)
    # the trace clock: the conversion under which the registration's first k_vg_bbox
    # starts within 1 ms after the enqueue
    best = None
    for name, t0 in (("monotonic", t0_mono), ("boottime", t0_mono + boff)):
        first = [s for s, e, k, q in rows if k.startswith("k_vg_bbox") and t0 <= s <= t0 + 1_000_000]
        if first and (best is None or first[0] - t0 < best[2]):
            best = (name, t0, first[0] - t0)
    if best is None:
        raise SystemExit("no k_vg_bbox within 1 ms of the last registration's enqueue")
    clock, t0, _ = best
    ks = [((s - t0) / 1e3, (e - t0) / 1e3, k, q) for s, e, k, q in rows if e >= t0 and s <= t0 + end_us * 1e3]
    out_lines = [f"trace clock: {clock}; last registration, times in us after its cloud stage was enqueued", ""]

    def span(pref_a, pref_b, after=0.0):
        a = [x for x in ks if x[2].startswith(pref_a) and x[0] >= after]
        if not a:
            return None
        s = a[0][0]
        b = [x for x in ks if x[2].startswith(pref_b) and x[0] >= s]
        return (s, b[0][1]) if b else None

    segs = []
    cur = 0.0
    for name, a, b in STAGE:
        sp = span(a, b, cur)
        if sp:
            segs.append((name, sp[0], sp[1]))
            cur = sp[1]
    xs = [x for x in ks if x[2].startswith("k_xs") and x[0] < cur]
    mk = dict(marks)
    fv = [x for x in ks if x[2].startswith("k_fv_transform")]
    fine = None
    if fv:  # from the transform to the last k_fv_* kernel after it (k_fv_score / k_fv_mail_err)
        last = [x for x in ks if x[2].startswith("k_fv") and x[0] >= fv[0][0]]
        fine = (fv[0][0], last[-1][1])
    match = [x for x in ks if x[2].startswith("k_match")]
    out_lines.append(f"{'segment':34s} {'start':>8s} {'end':>8s} {'us':>8s}")
    first_k = ks[0][0] if ks else 0.0
    out_lines.append(f"{'enqueue -> first kernel':34s} {0:8.1f} {first_k:8.1f} {first_k:8.1f}")
    prev_end = first_k
    for name, s, e in segs:
        if s - prev_end > 1.0:
            out_lines.append(f"{'  (gap)':34s} {prev_end:8.1f} {s:8.1f} {s - prev_end:8.1f}")
        out_lines.append(f"{name:34s} {s:8.1f} {e:8.1f} {e - s:8.1f}")
        prev_end = e
    if xs:
        out_lines.append(f"{'  side branch: exact centroid sums':34s} {xs[0][0]:8.1f} {xs[-1][1]:8.1f} "
                         f"{xs[-1][1] - xs[0][0]:8.1f}")
    host_prev = prev_end
    for k, v in marks:
        if k == "fine" and fine:
            out_lines.append(f"{'  fine verification (device)':34s} {fine[0]:8.1f} {fine[1]:8.1f} {fine[1] - fine[0]:8.1f}")
        label = {"clouds": "host wakes (clouds done)", "next_enq": "host: next-pair enqueue (batch only)",
                 "grow": "host: region growing", "match": "host+device: matching", "cluster": "host: clustering",
                 "vpairs": "host: quick_verify pairs + scores",
                 "verify": "host: LM (top per type)", "fine_setup": "host: fine setup",
                 "fine_launched": "host: fine launch", "fine": "host wakes (fine scores)"}.get(k, k)
        out_lines.append(f"{label:34s} {host_prev:8.1f} {v:8.1f} {v - host_prev:8.1f}")
        host_prev = v
    if match:
        out_lines.append(f"{'  (matching kernels on the device)':34s} {match[0][0]:8.1f} {match[-1][1]:8.1f} "
                         f"{match[-1][1] - match[0][0]:8.1f}")
    out_lines.append("")
    out_lines.append("kernels of the registration (start, end, stream, name):")
    for s, e, k, q in ks:
        out_lines.append(f"  {s:8.1f} {e:8.1f}  s{q:>3s}  {k}")
    text = "\n".join(out_lines)
    print(text)
    if out:
        open(out, "w").write(text + "\n")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 5)
    else:
        report(sys.argv[2], sys.argv[3], sys.argv[4] if len(sys.argv) > 4 else None)
