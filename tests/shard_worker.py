"""Rank process of tests/test_gpu_stages.py::test_match_sharded_two_ranks_gloo:
sharded coplane-pair search (fccf-pcr_amd/shard.py) with a gloo candidate gather."""
import json
import os
import sys

import numpy as np
import torch.distributed as dist

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fccf-pcr_amd"))
import fccf_amd  # noqa: E402
import shard  # noqa: E402


def main(inp, outp):
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    d = np.load(inp)
    F1, F2 = fccf_amd.planes_from_dump(d["planes1"]), fccf_amd.planes_from_dump(d["planes2"])
    B1, B2 = fccf_amd.bases_from_dump(d["bases1"]), fccf_amd.bases_from_dump(d["bases2"])
    with fccf_amd.Ctx(0) as ctx:
        cands, k_pass = shard.match_sharded(ctx, F1, B1, F2, B2, rank, world, shard.torch_gather())
    if rank == 0:
        np.savez(outp, cand0=cands[0], cand1=cands[1], cand2=cands[2],
                 meta=json.dumps({"world": world, "k_pass": k_pass}))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
