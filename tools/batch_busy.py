"""Dev: how busy the GPU is during a pipelined c3 batch (VERDICT r3 item 7 follow-up).

  run:     rocprofv3 --kernel-trace -f csv -d OUT -o run -- python3 tools/batch_busy.py run [pairs]
  report:  python3 tools/batch_busy.py report OUT [out.txt]

The run warms both stage groups, sleeps, then registers one batch; the report takes the
last burst of kernels (separated from the warm-up by the sleep) and prints its wall time,
the union of kernel intervals (busy), the idle gaps longer than 5 us with the kernels on
either side, and busy time per kernel family.
"""
import collections
import csv
import glob
import os
import re
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(pairs):
    sys.path.insert(0, os.path.join(ROOT, "fccf-pcr_amd"))
    import fccf_amd as F
    cfg = F.CONFIGS["c3"]
    src, tar, _ = F.synth_pair(cfg["n"], cfg["room"])
    ctx = F.Ctx(0)
    ds, dt = ctx.upload(src), ctx.upload(tar)
    pair = ((ds, len(src)), (dt, len(tar)))
    for _ in range(2):
        ctx.register_batch([pair] * pairs, cfg["leaf"], on_device=True)
    time.sleep(0.2)
    a = time.perf_counter()
    ctx.register_batch([pair] * pairs, cfg["leaf"], on_device=True)
    print(f"batch of {pairs}: {(time.perf_counter() - a) * 1e3 / pairs:.3f} ms/registration", flush=True)


def short(name):
    m = re.search(r"(k_\w+|__amd\w+)", name)
    return m.group(1) if m else name[:40]


def report(trace_dir, out=None):
    rows = []
    for f in glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                         int(r.get("Queue_Id", 0) or 0), int(r.get("Grid_Size_Y", 1) or 1)))
    rows.sort()
    # last burst: after the last gap of > 50 ms between a kernel's start and the previous end
    cut = 0
    last_end = rows[0][1]
    for i in range(1, len(rows)):
        if rows[i][0] - last_end > 50_000_000:
            cut = i
        last_end = max(last_end, rows[i][1])
    b = rows[cut:]
    t0, t1 = b[0][0], max(x[1] for x in b)
    b3 = [(x[0], x[1], x[2]) for x in b]
    busy, gaps = 0, []
    cs, ce, prev = b[0][0], b[0][1], b[0][2]
    full = b
    b = b3
    for s, e, k in b[1:]:
        if s > ce:
            busy += ce - cs
            gaps.append((s - ce, ce - t0, prev, k))
            cs, ce = s, e
        else:
            ce = max(ce, e)
        if e >= ce:
            prev = k
    busy += ce - cs
    fam = collections.Counter()
    for s, e, k in b:
        fam[k] += e - s
    L = [f"kernels {len(b)}, wall {(t1 - t0) / 1e3:.1f} us, busy (union) {busy / 1e3:.1f} us "
         f"({100.0 * busy / (t1 - t0):.1f} %), idle {(t1 - t0 - busy) / 1e3:.1f} us in {len(gaps)} gaps", ""]
    big = sorted((g for g in gaps if g[0] > 5000), key=lambda g: -g[0])
    L.append(f"idle gaps > 5 us: {len(big)}, total {sum(g[0] for g in big) / 1e3:.1f} us; largest 40 "
             "(length us, at us, kernel before -> after):")
    for g in big[:40]:
        L.append(f"  {g[0] / 1e3:8.1f} {g[1] / 1e3:10.1f}  {g[2]} -> {g[3]}")
    L.append("")
    # the cloud stages: main VoxelGrid's k_is_prep (the sort's first launch) to the stage's
    # k_mail_done (its last kernel before the S1 replay); fill = batch start -> first
    # stage end, drain = last stage end -> batch end
    preps = [s for s, e, k in b if k == "k_is_prep"]
    dones = [e for s, e, k in b if k == "k_mail_done"]
    L.append("stages (us from the batch's first kernel): sort start -> clouds done")
    for i, ps in enumerate(preps):
        de = [d for d in dones if d > ps]
        L.append(f"  stage {i}: {(ps - t0) / 1e3:9.1f} -> {((de[0] if de else ps) - t0) / 1e3:9.1f}"
                 f"  ({((de[0] if de else ps) - ps) / 1e3:.1f} us)")
    if dones:
        L.append(f"  drain after the last stage: {(t1 - max(dones)) / 1e3:.1f} us of {(t1 - t0) / 1e3:.1f}")
        L.append("  the drain's kernels (start, end us from the batch's first kernel, queue, grid y):")
        for s_, e_, k_, q_, y_ in full:
            if e_ > max(dones):
                L.append(f"    {(s_ - t0) / 1e3:9.1f} {(e_ - t0) / 1e3:9.1f}  q{q_} y{y_}  {k_}")
    # between stages: every kernel overlapping [stage i clouds done, stage i+1 sort start]
    for i in range(len(preps) - 1):
        de = [d for d in dones if d > preps[i]]
        if not de:
            continue
        a, z = de[0], preps[i + 1]
        L.append(f"  transition {i} -> {i + 1}: {(a - t0) / 1e3:.1f} -> {(z - t0) / 1e3:.1f} us "
                 f"({(z - a) / 1e3:.1f} us); kernels in it (start, end, queue, grid y):")
        for s_, e_, k_, q_, y_ in full:
            if e_ > a and s_ < z:
                L.append(f"    {(s_ - t0) / 1e3:9.1f} {(e_ - t0) / 1e3:9.1f}  q{q_} y{y_}  {k_}")
    L.append("")
    L.append("kernel time by name (sum of durations, may overlap):")
    for k, v in fam.most_common(30):
        L.append(f"  {k:28s} {v / 1e3:9.1f} us")
    text = "\n".join(L)
    print(text)
    if out:
        open(out, "w").write(text + "\n")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 20)
    else:
        report(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
