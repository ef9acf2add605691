"""Projection of one registration sharded over N GPUs (BASELINE configs[3]/[4]: c4 x 4,
c5 x 8) from quantities measured on ONE GPU:

  * the unsharded registration: e2e latency and its device spans (fccf_stats.dev_ms:
    main VoxelGrid = the sort + centroids, the face stage, fine verification);
  * row D: K1's sort of each cloud's keys unsharded and as each rank r of N would run it
    (FCCF_SHARD_D_SIM=r/N: the replicated first rounds, then only rank r's range), the
    slowest rank taken;
  * the exchange: virtual ranks (fccf_group_create_local, N contexts on the one GPU, the
    product's exchange code with the packed all-gather-v) register the pair once, and
    fccf_group_bytes gives the bytes every rank received per channel;
  * the collectives issued per registration (count from the same run's code path).

Projected N-GPU latency = e2e_1 - (sort_1 - sort_N) - (faces_1 - faces_N) + exchange, with
faces_N = replicated codes pass + (rest of the face stage) / N, and exchange = bytes /
BW + collectives x latency + host round trips.  BW, the per-collective latency and the
face stage's replicated share are ASSUMPTIONS (stated in the output), not measurements:
no multi-GPU run has executed here.

Usage: python tools/group_projection.py [cfg:N ...]  (GPU)  -> one JSON line per config"""
import json
import os
import statistics
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fccf-pcr_amd"), os.path.join(ROOT, "tools")]
import fccf_amd as F  # noqa: E402
from is_bench import leaf_keys  # noqa: E402

BW_GBPS = 300.0          # assumed all-gather receive bandwidth per rank over xGMI (RCCL ring, 7 links)
COLL_LAT_US = 20.0       # assumed latency of one RCCL collective (small messages)
HOST_SYNC_US = 25.0      # assumed host round trip per stream sync on the exchange path (measured ~20 us)
FACE_REPLICATED = 0.15   # share of the face stage every rank repeats (octree bounds + leaf codes), from the stage timeline


def sort_ms(ctx, k, reps=3):
    ts = []
    for _ in range(reps):
        ctx.sort_keys(k)
        ts.append(int(ctx.sort_stats()["raw"][31]) / 1e6)
    return min(ts)


def on_threads(fn, n):
    res, errs = [None] * n, []

    def run(r):
        try:
            res[r] = fn(r)
        except BaseException as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=run, args=(r,)) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    if errs:
        raise errs[0]
    return res


def project(cfg_name, n):
    c = F.CONFIGS[cfg_name]
    src, tar, _ = F.synth_pair(c["n"], c["room"])
    leaf = c["leaf"]
    out = {"config": cfg_name, "ranks": n, "n_points": c["n"]}
    with F.Ctx(0) as ctx:
        d_s, d_t = ctx.upload(src), ctx.upload(tar)
        for _ in range(3):
            ctx.register_device(d_s, len(src), d_t, len(tar), leaf)
        e2e, dev = [], []
        import time
        for _ in range(5):
            a = time.perf_counter()
            _, st = ctx.register_device(d_s, len(src), d_t, len(tar), leaf)
            e2e.append((time.perf_counter() - a) * 1e3)
            dev.append(st.as_dict()["dev_ms"])
        ctx.free(d_s)
        ctx.free(d_t)
        out["one_gpu"] = {"e2e_ms": statistics.median(e2e),
                          "dev_ms": {k: statistics.median(d[k] for d in dev) for k in dev[0]}}
        sorts = {}
        for which, pts in (("src", src), ("tar", tar)):
            k = leaf_keys(pts, leaf)
            os.environ.pop("FCCF_SHARD_D_SIM", None)
            whole = sort_ms(ctx, k)
            per = []
            for r in range(n):
                os.environ["FCCF_SHARD_D_SIM"] = f"{r}/{n}"
                per.append(sort_ms(ctx, k))
            os.environ.pop("FCCF_SHARD_D_SIM", None)
            sorts[which] = {"unsharded_ms": whole, "slowest_rank_ms": max(per), "per_rank_ms": per}
        out["row_D_sort"] = sorts
    # the exchange, by the product's code on virtual ranks
    ctxs = [F.Ctx(0) for _ in range(n)]
    try:
        groups = F.local_groups(ctxs)

        def work(r):
            ctxs[r].register(src, tar, leaf)  # warm (graphs, workspaces)
            b0 = groups[r].rx_bytes()
            _, s = ctxs[r].register(src, tar, leaf)
            b1 = groups[r].rx_bytes()
            return [y - x for x, y in zip(b0, b1)], s.as_dict()["sharded"]

        res = on_threads(work, n)
        for g in groups:
            g.close()
    finally:
        for cx in ctxs:
            cx.close()
    rx = [r[0] for r in res]
    out["exchange_bytes_per_rank"] = {"match": max(x[0] for x in rx), "fine": max(x[1] for x in rx),
                                      "cloud": max(x[2] for x in rx)}
    out["sharded_stages"] = res[0][1]
    one = out["one_gpu"]
    # the two clouds' sorts run in the same launches: the main VoxelGrid span scales with
    # the summed sort time (the centroid passes stay: ~5 % of the span)
    s1 = sorts["src"]["unsharded_ms"] + sorts["tar"]["unsharded_ms"]
    sN = sorts["src"]["slowest_rank_ms"] + sorts["tar"]["slowest_rank_ms"]
    vg1 = one["dev_ms"]["vg_main"]
    vgN = vg1 * sN / s1
    f1 = one["dev_ms"]["faces"]
    fN = f1 * (FACE_REPLICATED + (1 - FACE_REPLICATED) / n)
    tot_bytes = sum(out["exchange_bytes_per_rank"].values())
    # collectives of one registration: D (counts, slices), P (2 count gathers, records),
    # K5 (counts, lists), F (scores); host syncs: D bounds, P counts x2, K5 counts, K5 lists
    n_coll, n_sync = 7, 5
    xch_ms = tot_bytes / (BW_GBPS * 1e9) * 1e3 + n_coll * COLL_LAT_US / 1e3 + n_sync * HOST_SYNC_US / 1e3
    projN = one["e2e_ms"] - (vg1 - vgN) - (f1 - fN) + xch_ms
    out["projection"] = {
        "assumptions": {"allgather_GBps_per_rank": BW_GBPS, "collective_latency_us": COLL_LAT_US,
                        "host_sync_us": HOST_SYNC_US, "face_replicated_share": FACE_REPLICATED},
        "vg_main_ms": [vg1, vgN], "faces_ms": [f1, fN], "exchange_ms": xch_ms,
        "e2e_ms_1gpu": one["e2e_ms"], "e2e_ms_projected": projN, "speedup": one["e2e_ms"] / projN}
    return out


def main():
    for spec in sys.argv[1:] or ["c4:4", "c5:8"]:
        cfg, n = spec.split(":")
        print(json.dumps(project(cfg, int(n))), flush=True)


if __name__ == "__main__":
    main()
