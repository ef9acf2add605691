"""Rank process of tests/test_gpu_group.py's multi-rank case: one fccf ctx + one RCCL
group rank; registers the c2 pair with the sharded search and prints T's bits as
JSON.  argv: rank n_ranks id_file out_file"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fccf-pcr_amd"))
import fccf_amd as F  # noqa: E402

rank, n, idf, outf = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3], sys.argv[4]
if rank == 0:
    uid = F.group_unique_id()
    with open(idf + ".tmp", "wb") as f:
        f.write(uid)
    os.replace(idf + ".tmp", idf)
else:
    t0 = time.time()
    while not os.path.exists(idf):
        if time.time() - t0 > 60:
            raise SystemExit("no group id")
        time.sleep(0.05)
    uid = open(idf, "rb").read()
c = F.CONFIGS["c2"]
src, tar, _ = F.synth_pair(c["n"], c["room"])
ctx = F.Ctx(0)
try:
    g = F.Group(ctx, uid, n, rank)
except F.FCCFError as e:
    json.dump({"error": e.code, "msg": str(e)}, open(outf, "w"))
    raise SystemExit(0)
T, st = ctx.register(src, tar, c["leaf"])
g.close()
ctx.close()
json.dump({"T": T.view("uint32").ravel().tolist(), "K": st.K, "K_pass": st.K_pass, "cand": list(st.cand)},
          open(outf, "w"))
