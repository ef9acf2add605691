#!/usr/bin/env python3
"""bench.py — FCCF-PCR registration on MI355X (BASELINE.json metric).

One step = one full registration (both VoxelGrid passes, plane extraction,
coplane-pair correspondence search, transform estimation, clustering,
verification, fusion) of the c3 workload: a synthetic 1M x 1M-point room pair,
voxel 0.05 m (BASELINE.json configs[2]).  Inputs are uploaded to
HBM before the timed region.  value = coplane-pair correspondence tests (K = B1*B2
per registration, FCCF.cpp:1415-1427) processed by all ranks / wall time.

Multi-GPU: registrations are independent objects, so each rank registers its own
pair on its own GPU (weak scaling, no data-path collective); a gloo process group
(CPU) provides only the barrier and the max-over-ranks of the timed span.  libfccf
links the system ROCm HIP runtime, so torch never touches the GPU here.  After that
leg, N > 1 also measures strong scaling as BASELINE configs[3]/[4] name it: ONE c4
pair registered by min(N, 4) ranks and ONE c5 pair by N ranks of an RCCL group inside
libfccf (fccf_group_create: search, fine verification and the VoxelGrid sort sharded),
each rank in a child process with a time limit; reported under "sharded" beside the
replica `value` (sharded_pass).
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "fccf-pcr_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

METRIC = "coplane-pair correspondences/sec + end-to-end registration ms, 1M-pt pair"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md "HBM"); every kernel here is HBM/latency bound
# Kernels with a probe site (fccf-pcr_amd/csrc, FCCF_PROBED) and their algorithmic bytes per launch
# ("Measurement").  The roofline reports the one with the most GPU time per step.
PROBE_KERNELS = ["k_is_count_plan", "k_is_wave", "k_is_scatter", "k_is_block", "k_xs_chain", "k_xs_chunk", "k_oct_sim", "k_rs_scatter",
                 "k_vg_keys", "k_vg_centroid", "k_gather", "k_voxel_fit", "k_fv_counts", "k_match_count",
                 "k_match_emit"]


def stage_roofline(st):
    """algorithmic bytes of the N-proportional stages over their
    device spans (the cloud stage's kernel timestamps, fccf_stats.dev_ms), per
    stage and aggregated.  Per cloud c: D = 12 N_c + 12 M1_c + 12 M1_c + 12 M_c (both
    VoxelGrid passes), P = 12 M_c + 32 V_c (1 m voxel fit, V = occupied leaves),
    F = 12 (S1 + S2) per fine_verify evaluation."""
    N = (st.n_src, st.n_tar)
    M1 = (st.m1_src, st.m1_tar)
    M = (st.m_src, st.m_tar)
    V = (st.leaves1, st.leaves2)
    bytes_ = {"D": sum(12 * N[c] + 24 * M1[c] + 12 * M[c] for c in range(2)),
              "P": sum(12 * M[c] + 32 * V[c] for c in range(2)),
              "F": 12 * (st.res1 + st.res2) * st.fine_evals}
    ms = {"D": st.dev_ms[0] + st.dev_ms[1], "P": st.dev_ms[2], "F": st.dev_ms[3]}
    out = {}
    for k in ("D", "P", "F"):
        gbs = bytes_[k] / (ms[k] * 1e-3) / 1e9 if ms[k] > 0 else None
        out[k] = {"bytes": int(bytes_[k]), "ms": round(ms[k], 4), "achieved_GBps": gbs,
                  "frac": gbs / HBM_PEAK_GBS if gbs else None}
    tb, tm = sum(bytes_.values()), sum(ms.values())
    agg = tb / (tm * 1e-3) / 1e9 if tm > 0 else None
    out["aggregate"] = {"bytes": int(tb), "ms": round(tm, 4), "achieved_GBps": agg,
                        "frac": agg / HBM_PEAK_GBS if agg else None}
    return out


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def spawn_ranks(n, argv):
    """--gpus N > 1 without a launcher: start N rank processes of this script (one per
    GPU, RANK/LOCAL_RANK/WORLD_SIZE set) BEFORE anything touches the GPU, wait for all
    of them and return the worst exit code.  Rank 0 prints the JSON line."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    codes = [p.wait() for p in procs]
    bad = [c for c in codes if c != 0]
    return bad[0] if bad else 0


def dist_setup(gpus):
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={ws}; refusing to report a different n_gpus")
    if ws <= 1:
        return 0, 1, 0, None
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method="env://")
    return dist.get_rank(), ws, int(os.environ.get("LOCAL_RANK", "0")), dist


def barrier(dist):
    if dist is not None:
        dist.barrier()


def allmax(dist, v):
    if dist is None:
        return v
    import torch
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def allsum(dist, v):
    if dist is None:
        return v
    import torch
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def cpu_baseline(src, tar, leaf, budget_s):
    """The oracle (single-threaded C++ restatement of FCCF.cpp, introsort mode =
    the reference's std::sort) on the same workload, repeated within a time budget,
    pinned to one host core (taskset-style pinning, CPU model recorded)."""
    import oracle_py
    times, K, stages, ref_win, T = [], None, None, [], None
    try:
        prev = os.sched_getaffinity(0)
        core = min(prev)
        os.sched_setaffinity(0, {core})
    except (AttributeError, OSError):
        prev, core = None, None
    try:
        t_end = time.time() + budget_s
        while not times or (time.time() < t_end and len(times) < 20):
            t0 = time.perf_counter()
            run = oracle_py.Run(src, tar, leaf, oracle_py.INTROSORT)
            times.append(time.perf_counter() - t0)
            K = int(run.get("counts", np.int64)[0])
            T = run.T.copy()
            stages = run.times()
            ref_win.append(times[-1] * 1e3 - float(run.get("main_vg_ms", np.float64)[0]))
            del run
    finally:
        if prev is not None:
            os.sched_setaffinity(0, prev)
    med = statistics.median(times)
    names = ["downsample", "voxelfit", "grow_select", "match", "cluster", "verify", "fine", "fuse", "total"]
    out = {"value": K / med, "unit": "correspondences/s", "cores": 1, "kind": "port",
           "ms_per_registration": med * 1e3, "K": K, "pinned_cpu": core, "cpu_model": cpu_model(),
           "host_nproc": os.cpu_count(),
           "stage_ms_last": {n: round(float(v), 3) for n, v in zip(names, stages)} if stages is not None else None,
           # the reference's own timer window (FCCF.cpp:1681-1685) excludes main's VoxelGrid
           "ref_window_ms_median": statistics.median(ref_win),
           "sample": f"{len(times)} full registrations of the same c3 pair (median), oracle/ C++ restatement "
                     f"with PCL's structures (std::sort VoxelGrid, pointer octrees with per-leaf index "
                     f"vectors), 1 thread pinned to CPU {core}"}
    return out, T  # T: the oracle's transform (the parity check against the GPU's)


def same_bits(a, b):
    return np.array_equal(np.ascontiguousarray(a, np.float32).view(np.uint32),
                          np.ascontiguousarray(b, np.float32).view(np.uint32))


def parity_pass(F, ctx, configs):
    """Parity of the product against the oracle (introsort order = the reference's
    std::sort VoxelGrid), outside the timed region: per BASELINE config, one GPU
    registration from host arrays (fccf_register) and one oracle registration of the
    same synthetic pair; the 4x4 transforms must be equal bit for bit and the
    correspondence test counts K (FCCF.cpp:1415-1427) equal.  Returns
    {config: verdict}; any mismatch ends the bench without a JSON line."""
    import oracle_py
    out = {}
    for name in configs:
        cfg = F.CONFIGS[name]
        src, tar, _ = F.synth_pair(cfg["n"], cfg["room"])
        Tg, st = ctx.register(src, tar, cfg["leaf"])
        run = oracle_py.Run(src, tar, cfg["leaf"], oracle_py.INTROSORT)
        To, Ko = run.T.copy(), int(run.get("counts", np.int64)[0])
        del run
        if not same_bits(Tg, To) or int(st.K) != Ko:
            raise SystemExit(f"bench.py: parity FAILED at {name}: GPU K {int(st.K)} T\n{Tg}\n"
                             f"oracle K {Ko} T\n{To}")
        out[name] = "bit-exact"
    return out


class _SelftestCtx:
    """--selftest: stands in for fccf_amd.Ctx so the distributed/JSON logic can be
    exercised on CPU (tests/test_dist.py).  Computes nothing; never used for numbers."""

    class _St:
        K, K_pass, graph_captures = 100, 10, 0

        def as_dict(self):
            return {"ms": {"stub": 0.0}}

    def upload(self, a):
        return 0

    def free(self, d):
        pass

    def register_device(self, ds, ns, dt, nt, leaf):
        time.sleep(0.002)
        return np.eye(4, dtype=np.float32), self._St()

    def register(self, src, tar, leaf):
        return self.register_device(0, 0, 0, 0, leaf)


def pmc_traffic(kernel, config, width):
    """HBM bytes per launch of `kernel` at launch width `width` (clouds per launch) from
    the newest committed PMC summary of the same workload and shape
    (profiles/*/pmc_traffic.json, written by tools/pmc_traffic.py from rocprofv3 --pmc
    passes), else None.  Summaries without a width are of single registrations (2)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_traffic.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("config", "c3") != config or int(d.get("width", 2)) != width:
            continue
        # (the probe label names the kernel family: the sort's round kernels have a small-
        # and a large-cloud form, k_is_scatter_s / k_is_scatter, by symbol)
        for name in (kernel, kernel + "_s"):
            if name in d.get("kernels", {}):
                return d["kernels"][name]["hbm_bytes_per_launch"]
    return None


def probe_pass(ctx, run, kernel, reps=1):
    """Every launch of `kernel` during `reps` calls of run() (a pipelined batch, or
    single registrations), timed with HIP events on its own stream.  Returns the totals
    (ms, launches, algorithmic bytes) and the same split by launch width (clouds per
    batched launch: {width: (ms, launches, bytes)})."""
    ctx.set_probe(kernel)
    run()  # one untimed eager warm-up call of the same shape
    ctx.set_probe(kernel)  # resets the totals
    for _ in range(reps):
        run()
    ms, n, b = ctx.probe_read()
    return ms, n, b, ctx.probe_read_widths()


def width_table(widths):
    """{width: {launches, avg_launch_us, algorithmic_bytes_per_launch, achieved_GBps, frac}}"""
    out = {}
    for w, (ms, n, b) in sorted(widths.items()):
        gbs = (b / n) / (ms * 1e-3 / n) / 1e9 if ms > 0 else None
        out[str(w)] = {"launches": n, "avg_launch_us": ms * 1e3 / n, "algorithmic_bytes_per_launch": b / n,
                       "achieved_GBps": gbs, "frac": gbs / HBM_PEAK_GBS if gbs else None}
    return out


PROBE_BATCH = 10  # registrations per pre-pass window: two stage groups of five pairs

SHARDED_PLAN = (("c4", 4), ("c5", 8))  # BASELINE configs[3]/[4]: the pair and its rank count (capped at N)


def _wait_file(path, timeout_s):
    t0 = time.time()
    while not os.path.exists(path):
        if time.time() - t0 > timeout_s:
            raise TimeoutError(f"{path} did not appear within {timeout_s} s")
        time.sleep(0.002)


def sharded_child(args):
    """One rank of the strong-scaling leg (a child process of bench rank `child_rank`,
    so a collective that never completes cannot hang the bench: the parent kills it at
    its time limit).  For each BASELINE multi-GPU config (c4 over min(N, 4) ranks, c5
    over N): the pair is registered collectively by an RCCL group of the ranks
    (fccf_group_create; rows K5, F and D of SURVEY.md §8(e) sharded, FCCF.cpp:1410-1428,
    :785-839, :1668-1678), device-resident inputs, timed as one pipelined batch of
    `steps` registrations and as single registrations; the group's T must equal this
    GPU's unsharded T bit for bit.  Rank 0 first times the unsharded pipelined batch on
    its own GPU (the one-GPU figure the speed-up is taken against).  Results go to
    <dir>/res_<cfg>_<rank>.json; the group id travels through <dir>/id_<cfg>."""
    d, rank, world = args.sharded_child, args.child_rank, args.child_world
    steps = args.steps
    for cfg_name, cap in SHARDED_PLAN:
        ranks = min(world, cap)
        if rank >= ranks:
            continue
        res = {"ranks": ranks}
        outp = os.path.join(d, f"res_{cfg_name}_{rank}.json")
        try:
            if args.selftest:  # CPU stub (tests/test_dist.py): the merge logic only, no numbers
                time.sleep(0.01)
                res.update({"one_gpu_ms_per_registration": 2.0 if rank == 0 else None,
                            "one_gpu_ms_per_registration_pp1": 2.5 if rank == 0 else None, "elapsed_s": 0.001 * steps,
                            "e2e_s": [0.002] * min(steps, 10), "parity": "selftest-stub",
                            "sharded": ["fine", "search", "sort"], "K": 100, "device_ms": {}})
                raise StopIteration
            import fccf_amd as F
            cfg = F.CONFIGS[cfg_name]
            src, tar, _ = F.synth_pair(cfg["n"], cfg["room"])
            leaf = cfg["leaf"]
            with F.Ctx(args.device) as ctx:
                ds, dt = ctx.upload(src), ctx.upload(tar)
                pair = ((ds, src.shape[0]), (dt, tar.shape[0]))
                T0, _ = ctx.register_device(ds, src.shape[0], dt, tar.shape[0], leaf)  # unsharded reference
                if rank == 0:
                    ctx.register_batch([pair] * steps, leaf, on_device=True)  # warm: the timed batch's own shape
                    a = time.perf_counter()
                    ctx.register_batch([pair] * steps, leaf, on_device=True)
                    res["one_gpu_ms_per_registration"] = (time.perf_counter() - a) / steps * 1e3
                    # the same at one pair per cloud stage (round 4's group form), beside it
                    os.environ["FCCF_PAIR_BATCH"] = "1"
                    try:
                        ctx.register_batch([pair] * steps, leaf, on_device=True)
                        a = time.perf_counter()
                        ctx.register_batch([pair] * steps, leaf, on_device=True)
                        res["one_gpu_ms_per_registration_pp1"] = (time.perf_counter() - a) / steps * 1e3
                    finally:
                        del os.environ["FCCF_PAIR_BATCH"]
                    uid = F.group_unique_id()
                    with open(os.path.join(d, f"id_{cfg_name}.tmp"), "wb") as f:
                        f.write(uid)
                    os.replace(os.path.join(d, f"id_{cfg_name}.tmp"), os.path.join(d, f"id_{cfg_name}"))
                else:
                    _wait_file(os.path.join(d, f"id_{cfg_name}"), 120)
                    uid = open(os.path.join(d, f"id_{cfg_name}"), "rb").read()
                g = F.Group(ctx, uid, ranks, rank)
                try:
                    ctx.register_batch([pair] * 2, leaf, on_device=True)  # warm (graphs, communicator buffers)
                    # file barrier, then one collective registration: the ranks start in step
                    open(os.path.join(d, f"ready_{cfg_name}_{rank}"), "w").close()
                    for r in range(ranks):
                        _wait_file(os.path.join(d, f"ready_{cfg_name}_{r}"), 120)
                    ctx.register_device(ds, src.shape[0], dt, tar.shape[0], leaf)
                    a = time.perf_counter()
                    Tb, sb = ctx.register_batch([pair] * steps, leaf, on_device=True)
                    res["elapsed_s"] = time.perf_counter() - a
                    per = []
                    for _ in range(min(steps, 10)):
                        a = time.perf_counter()
                        T1, s1 = ctx.register_device(ds, src.shape[0], dt, tar.shape[0], leaf)
                        per.append(time.perf_counter() - a)
                    res["e2e_s"] = per
                finally:
                    g.close()
                ctx.free(ds)
                ctx.free(dt)
            same = all(same_bits(T, T0) for T in list(Tb) + [T1])
            res.update({"parity": "bit-exact vs this GPU's unsharded T" if same else "MISMATCH",
                        "sharded": s1.as_dict()["sharded"], "K": int(s1.K),
                        "device_ms": {k: round(v, 4) for k, v in s1.as_dict()["dev_ms"].items()}})
        except StopIteration:
            pass
        except Exception as e:  # noqa: BLE001 (reported in the JSON line, never hidden)
            res["error"] = f"{type(e).__name__}: {e}"
        with open(outp + ".tmp", "w") as f:
            json.dump(res, f)
        os.replace(outp + ".tmp", outp)


def sharded_pass(dist, ws, rank, local, args, timeout_s):
    """Strong scaling of ONE registration (BASELINE configs[3]/[4]), run after the
    replica leg: every rank starts a child process (sharded_child) on its GPU and waits
    for it at most timeout_s; rank 0 merges the children's results.  Returns
    {cfg: {...}} on rank 0 (None elsewhere)."""
    import shutil
    import subprocess
    import tempfile
    d = [tempfile.mkdtemp(prefix="fccf_shard_") if rank == 0 else None]
    dist.broadcast_object_list(d, src=0)
    d = d[0]
    cmd = [sys.executable, os.path.abspath(__file__), "--sharded-child", d, "--child-rank", str(rank),
           "--child-world", str(ws), "--device", str(local), "--steps", str(args.steps)] + \
        (["--selftest"] if args.selftest else [])
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE",
                                                           "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.Popen(cmd, env=env, start_new_session=True)
    status = "ok"
    try:
        rc = p.wait(timeout=timeout_s)
        if rc != 0:
            status = f"child exit {rc}"
    except subprocess.TimeoutExpired:
        status = f"child killed at its {timeout_s} s limit"
        import signal
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except OSError:
            pass
        p.wait()
    stats = [None] * ws
    dist.all_gather_object(stats, status)
    out = None
    if rank == 0:
        out = {}
        for cfg_name, cap in SHARDED_PLAN:
            ranks = min(ws, cap)
            rs = []
            for r in range(ranks):
                f = os.path.join(d, f"res_{cfg_name}_{r}.json")
                rs.append(json.load(open(f)) if os.path.exists(f) else {"error": f"rank {r}: {stats[r]}"})
            errs = [x["error"] for x in rs if "error" in x]
            if errs:
                out[cfg_name] = {"ranks": ranks, "error": errs[0]}
                continue
            el = max(x["elapsed_s"] for x in rs)
            e2e = [max(v) for v in zip(*[x["e2e_s"] for x in rs])]
            one = rs[0].get("one_gpu_ms_per_registration")
            one1 = rs[0].get("one_gpu_ms_per_registration_pp1")
            ms = el / args.steps * 1e3
            # both sides batch five pairs per cloud stage (the group form does since round 5);
            # the one-GPU figure at one pair per stage is reported beside it
            out[cfg_name] = {"ranks": ranks, "ms_per_registration": ms,
                             "e2e_ms_median": statistics.median(e2e) * 1e3,
                             "one_gpu_ms_per_registration": one,
                             "one_gpu_ms_per_registration_pp1": one1,
                             "speedup_vs_one_gpu": one / ms if one else None,
                             "correspondences_per_s": rs[0]["K"] / (ms * 1e-3),
                             "sharded_stages": rs[0]["sharded"],
                             "parity": rs[0]["parity"] if all(x["parity"] == rs[0]["parity"] for x in rs)
                             else "MISMATCH between ranks",
                             "device_ms_rank0": rs[0]["device_ms"]}
        shutil.rmtree(d, ignore_errors=True)
    return out


def ingest_pass(F, ctx, src, tar, leaf, T_ref, reps=3):
    """f2, informational: the reference's PLY -> T path
    (FCCF.cpp:1655-1685) with the clouds streamed from PLY files into HBM
    (fccf_ply_load_device: chunked decode overlapped with the upload), and a pipelined
    batch from host arrays (uploads on the copy stream, overlapping the previous
    pair's compute).  Files are written to a scratch directory first (untimed)."""
    import tempfile
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for fmt, binary in (("binary", True), ("ascii", False)):
            ps, pt = os.path.join(td, f"s_{fmt}.ply"), os.path.join(td, f"t_{fmt}.ply")
            F.ply_write(ps, src, binary)
            F.ply_write(pt, tar, binary)
            load, e2e = [], []
            for _ in range(reps):
                a = time.perf_counter()
                ds, ns = ctx.ply_load(ps)
                dt, nt = ctx.ply_load(pt)
                b = time.perf_counter()
                T3, _ = ctx.register_device(ds, ns, dt, nt, leaf)
                c = time.perf_counter()
                ctx.free(ds)
                ctx.free(dt)
                assert np.array_equal(T3.view(np.uint32), np.asarray(T_ref).view(np.uint32)), "PLY-path result differs"
                load.append(b - a)
                e2e.append(c - a)
            nbytes = os.path.getsize(ps) + os.path.getsize(pt)
            out[fmt] = {"file_MB": round(nbytes / 1e6, 2), "load_ms_median": statistics.median(load) * 1e3,
                        "load_GBps": nbytes / statistics.median(load) / 1e9,
                        "ply_to_T_ms_median": statistics.median(e2e) * 1e3}
    k = 8
    a = time.perf_counter()
    Tb, _ = ctx.register_batch([(src, tar)] * k, leaf)
    out["host_input_batch_ms_per_registration"] = (time.perf_counter() - a) / k * 1e3
    assert np.array_equal(Tb[-1].view(np.uint32), np.asarray(T_ref).view(np.uint32)), "host batch result differs"
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--selftest", action="store_true", help="CPU stub registration (tests only)")
    ap.add_argument("--probe-kernel", default="auto", help="kernel for the roofline object (auto = dominant)")
    ap.add_argument("--no-sharded", action="store_true",
                    help="N>1: skip the strong-scaling leg (one c4 / c5 registration by an RCCL group of ranks)")
    ap.add_argument("--sharded-timeout", type=float, default=180.0,
                    help="time limit of a strong-scaling child (normally well under a minute)")
    ap.add_argument("--sharded-child", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--child-rank", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--child-world", type=int, default=1, help=argparse.SUPPRESS)
    ap.add_argument("--device", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--parity-configs", default=None,
                    help="comma-separated BASELINE configs checked bit for bit against the oracle after the "
                         "timed region (default c2,c4,c5 at N=1, none at N>1; the bench's own config is always "
                         "checked on rank 0)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="time K sequential fccf_register_device calls instead of one pipelined batch of K")
    args = ap.parse_args()
    if args.sharded_child:
        sharded_child(args)
        return
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))

    rank, ws, local, dist = dist_setup(args.gpus)
    if os.environ.get("FCCF_BENCH_ONE_DEVICE") == "1":
        local = 0  # dev: every rank on device 0 (rehearsal of the N > 1 plumbing on a one-GPU box)
    if ws > 1 and "FCCF_HOST_THREADS" not in os.environ:
        # each rank's host stages get an equal share of this node's cores (<= 16 each),
        # so N ranks' worker pools do not oversubscribe the host
        lws = int(os.environ.get("LOCAL_WORLD_SIZE", str(ws)))
        try:
            ncpu = len(os.sched_getaffinity(0))
        except AttributeError:
            ncpu = os.cpu_count() or 16
        os.environ["FCCF_HOST_THREADS"] = str(max(2, min(16, ncpu // max(lws, 1))))
    import fccf_amd as F
    cfg = F.CONFIGS[args.config]
    if args.selftest:
        src = tar = np.zeros((cfg["n"], 3), np.float32)
        T_gt = np.eye(4, dtype=np.float32)
        ctx = _SelftestCtx()
        args.no_cpu_baseline = True
    else:
        src, tar, T_gt = F.synth_pair(cfg["n"], cfg["room"])
        ctx = F.Ctx(local)
    leaf = cfg["leaf"]
    d_src, d_tar = ctx.upload(src), ctx.upload(tar)

    def reg():
        return ctx.register_device(d_src, src.shape[0], d_tar, tar.shape[0], leaf)

    def batch(k):  # k pipelined registrations of the pair (fccf_register_batch)
        pair = ((d_src, src.shape[0]), (d_tar, tar.shape[0]))
        return ctx.register_batch([pair] * k, leaf, on_device=True)

    pipelined = not args.no_pipeline and not args.selftest
    # Untimed pre-pass: GPU time per step of every probed kernel (HIP events around
    # each launch; probed calls launch eagerly, see csrc/probe.h), in the timed region's
    # own shape: a pipelined batch (five pairs per cloud stage, ten clouds per launch)
    # of PROBE_BATCH registrations, or single registrations with --no-pipeline.  The
    # roofline kernel is the one with the most GPU time per step (or --probe-kernel).
    table, probe = {}, None
    if not args.selftest:
        pre, pre_steps = ((lambda: batch(PROBE_BATCH)), PROBE_BATCH) if pipelined else (reg, 1)
        for k in PROBE_KERNELS:
            ms, n, b, _ = probe_pass(ctx, pre, k, 1)
            if n:
                table[k] = {"ms_per_step": ms / pre_steps, "launches_per_step": n / pre_steps,
                            "avg_launch_us": ms * 1e3 / n, "algorithmic_bytes_per_launch": b / n,
                            "achieved_GBps": (b / n) / (ms * 1e-3 / n) / 1e9 if ms > 0 else None}
        ctx.set_probe(None)
        probe = max(table, key=lambda k: table[k]["ms_per_step"]) if args.probe_kernel == "auto" else args.probe_kernel
    batch_ms = None
    for _ in range(args.warmup):
        T, st = reg()
    if pipelined and args.warmup:
        # the timed batch's own shape: every stage group of it (up to five pairs per cloud
        # stage, groups on alternating workspaces, a smaller last group) captures its
        # graphs here, not in the timed batch
        batch(args.steps)
    barrier(dist)
    t0 = time.perf_counter()
    Ks = 0
    if pipelined:
        # exactly K registrations, pair i+1's cloud stage overlapping pair i's later stages
        Tb, sts = batch(args.steps)
    else:
        for _ in range(args.steps):
            T, st = reg()  # returns after T is on host
            Ks += st.K
    elapsed = time.perf_counter() - t0
    if pipelined:  # (the per-registration stats are read after the clock stops)
        T, st = Tb[-1], sts[-1]
        Ks = sum(x.K for x in sts)
        batch_ms = {k: statistics.mean(x.as_dict()["ms"][k] for x in sts) for k in sts[0].as_dict()["ms"]}
    barrier(dist)
    # latency: single registrations, one at a time (untimed for `value`)
    per, ref_win, stage_rl = [], [], None
    for _ in range(min(args.steps, 10)):
        a = time.perf_counter()
        T1, st1 = reg()
        per.append(time.perf_counter() - a)
        if not args.selftest:
            # the reference's timer window (FCCF.cpp:1681-1685) excludes main's VoxelGrid
            # pass: the registration minus that pass's device span
            ref_win.append(per[-1] * 1e3 - st1.dev_ms[0])
            stage_rl = stage_roofline(st1)
    if not args.selftest:
        assert np.array_equal(T1.view(np.uint32), np.asarray(T).view(np.uint32)), "pipelined result differs"
        if pipelined:  # every registration of the timed batch (the same pair), not only the last
            assert all(np.array_equal(np.asarray(x).view(np.uint32), T1.view(np.uint32)) for x in Tb), \
                "a pipelined registration's result differs"
    # PCIe-inclusive latency: the same registration from host arrays (fccf_register);
    # informational, never `value`
    per_host, h2d = [], []
    for _ in range(min(args.steps, 5)):
        a = time.perf_counter()
        T2, st2 = ctx.register(src, tar, leaf)
        per_host.append(time.perf_counter() - a)
        if not args.selftest:
            h2d.append(st2.as_dict()["ms"]["h2d"])
    if not args.selftest:
        assert np.array_equal(T2.view(np.uint32), np.asarray(T).view(np.uint32)), "host-input result differs"
    ingest = None if args.selftest or rank != 0 else ingest_pass(F, ctx, src, tar, leaf, T)
    sharded = sharded_pass(dist, ws, rank, local, args, args.sharded_timeout) \
        if ws > 1 and not args.no_sharded else None
    roofline = None
    if probe:
        # Probe window right after the timed region, same inputs and the same shape (one
        # pipelined batch of `steps` registrations, or `steps` single ones with
        # --no-pipeline): every launch of the roofline kernel timed with HIP events on its
        # own stream.  The figure is taken at the timed shape's launch width (the width
        # with the most launches); the other widths, and the two-cloud launches of a single
        # registration, are reported beside it.
        run = (lambda: batch(args.steps)) if pipelined else (lambda: [reg() for _ in range(args.steps)])
        pms, pn, pb, pw = probe_pass(ctx, run, probe, 1)
        sms, sn, sb, sw = probe_pass(ctx, reg, probe, min(args.steps, 10)) if pipelined else (None, 0, None, {})
        ctx.set_probe(None)
        if pn:
            w = max(pw, key=lambda x: pw[x][1])  # the timed shape's launch width
            wms, wn, wb = pw[w]
            avg_s = wms * 1e-3 / wn
            achieved = (wb / wn) / avg_s / 1e9
            roofline = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic(probe, args.config, w),
                        "kernel": probe, "launch_width": w, "avg_launch_us": avg_s * 1e6,
                        "algorithmic_bytes_per_launch": wb / wn, "launches_per_step": pn / args.steps,
                        "shape": "pipelined batch" if pipelined else "single registrations",
                        "by_width": width_table(pw)}
            if sn:
                roofline["single_registration"] = dict(width_table(sw), traffic=pmc_traffic(probe, args.config, 2))
    # parity against the oracle, after every timed or probed run (other sizes re-capture graphs)
    parity = None
    if rank == 0 and not args.selftest:
        pc = args.parity_configs if args.parity_configs is not None else ("c2,c4,c5" if ws == 1 else "")
        parity = parity_pass(F, ctx, [c for c in pc.split(",") if c and c != args.config])
    elapsed = allmax(dist, elapsed)
    Ks_all = allsum(dist, float(Ks))
    ctx.free(d_src)
    ctx.free(d_tar)

    if rank == 0:
        R = T[:3, :3].astype(np.float64).T @ T_gt[:3, :3].astype(np.float64)
        rot_err = float(np.degrees(np.arccos(np.clip((np.trace(R) - 1) / 2, -1, 1))))
        out = {
            "metric": METRIC,
            "value": Ks_all / elapsed,
            "unit": "correspondences/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "selftest-stub" if args.selftest else "synthetic",
            "config": {"workload": f"{args.config}: synthetic {cfg['n']:,}/{cfg['n']:,}-point room pair "
                                   f"R{tuple(cfg['room'])}, voxel {leaf} m, one registration per step per GPU",
                       "n_points": cfg["n"], "leaf": leaf, "room": list(cfg["room"]),
                       "parallelism": f"replicas x{ws}",
                       "pipelined": pipelined,
                       "host_threads_per_rank": int(os.environ.get("FCCF_HOST_THREADS", "0")) or None},
            "e2e_ms_median": statistics.median(per) * 1e3,  # one registration alone (latency)
            "e2e_host_input_ms_median": statistics.median(per_host) * 1e3,  # incl. H2D of both clouds
            "h2d_ms_median": statistics.median(h2d) if h2d else None,  # that copy alone (copy-stream events)
            "ref_window_ms_median": statistics.median(ref_win) if ref_win else None,
            "device_ms": {k: round(v, 4) for k, v in st1.as_dict()["dev_ms"].items()} if not args.selftest else None,
            "K_per_registration": int(st.K),
            "K_pass": int(st.K_pass),
            "graph_captures_last_step": int(st.graph_captures),
            "stage_ms": {k: round(v, 4) for k, v in st.as_dict()["ms"].items()},
            "stage_ms_in_batch": {k: round(v, 4) for k, v in batch_ms.items()} if batch_ms else None,
            "rot_err_deg_vs_gt": rot_err,
            "trans_err_m_vs_gt": float(np.linalg.norm(T[:3, 3] - T_gt[:3, 3])),
        }
        if ingest is not None:
            out["ingest"] = ingest
        if sharded is not None:
            # strong scaling: ONE registration of each multi-GPU BASELINE pair by all ranks
            out["sharded"] = sharded
        if roofline is not None:
            roofline["stage"] = stage_rl
            tr = roofline["traffic"]
            # over-fetch: calibrated L2-miss bytes per launch / algorithmic bytes per launch
            roofline["traffic_over_algorithmic"] = tr / roofline["algorithmic_bytes_per_launch"] if tr else None
            out["roofline"] = roofline
            # the sort's finish kernels beside the dominant one: honest
            # algorithmic bytes (keys, values and, for the elements a kernel finishes, the
            # sorted point gathered and written: DESIGN.md §14) and calibrated traffic, at
            # the pre-pass's width (ten clouds per launch)
            fk = {}
            for k in ("k_is_wave", "k_is_block"):
                if k in table:
                    t = table[k]
                    trk = pmc_traffic(k, args.config, PROBE_BATCH if pipelined else 2)
                    fk[k] = {"avg_launch_us": t["avg_launch_us"],
                             "algorithmic_bytes_per_launch": t["algorithmic_bytes_per_launch"],
                             "achieved_GBps": t["achieved_GBps"],
                             "frac": t["achieved_GBps"] / HBM_PEAK_GBS if t["achieved_GBps"] else None,
                             "traffic": trk,
                             "traffic_over_algorithmic": trk / t["algorithmic_bytes_per_launch"] if trk else None}
            out["finish_kernels"] = fk
            out["kernel_table"] = {k: {a: (round(b, 4) if isinstance(b, float) else b) for a, b in v.items()}
                                   for k, v in table.items()}
        T_oracle = None
        if ws == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"], T_oracle = cpu_baseline(src, tar, leaf, args.cpu_budget)
            # the CPU and GPU runs must do the same work (same plane pairs, same K)
            if out["cpu_baseline"]["K"] != out["K_per_registration"]:
                raise SystemExit(f"bench.py: cpu_baseline K {out['cpu_baseline']['K']} != GPU K "
                                 f"{out['K_per_registration']}")
        if parity is not None:
            if T_oracle is None:  # no CPU baseline leg: one oracle registration of the bench's pair
                import oracle_py
                T_oracle = oracle_py.Run(src, tar, leaf, oracle_py.INTROSORT).T.copy()
            # the timed registrations' T (every step returned the same bits, asserted above)
            if not same_bits(T, T_oracle):
                raise SystemExit(f"bench.py: parity FAILED at {args.config}: GPU T\n{T}\noracle T\n{T_oracle}")
            out["parity"] = dict({args.config: "bit-exact"}, **parity)
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    try:
        main()
    except SystemExit:
        raise
    except BaseException:
        # fail fast: do not let context teardown after a device error hold the process
        import traceback
        traceback.print_exc()
        sys.stderr.flush()
        os._exit(1)
