"""One rank of an RCCL world, one GPU per rank (launched by tests/test_gpu_rccl.py through
torch.distributed.run; RCCL rejects two ranks on one device).  Runs the text job of
PageRank.java over RCCL -- ingest replicated, rows dealt, the chunked x' exchange per round --
then the collective outputs: ranks(), topk(k), write_top_page, checkpoint_save.  Not a test.

  python -m torch.distributed.run --nproc-per-node N ... rccl_worker.py OUT_PREFIX ARCS MAPPING
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "page-rank-and-tfidf-using-apache-spark_amd"))

import numpy as np  # noqa: E402
import prmi355x as P  # noqa: E402

P.lib()  # ROCm's HIP + RCCL before torch loads its own copies

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    out, arcs_path, map_path = sys.argv[1], sys.argv[2], sys.argv[3]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = int(os.environ.get("LOCAL_RANK", rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = P.Engine(device=dev, n_ranks=world, rank=rank)
    uid = P.comm_unique_id() if rank == 0 else bytes(128)
    t = torch.tensor(list(uid), dtype=torch.uint8)
    dist.broadcast(t, 0)
    eng.comm_init(bytes(t.tolist()))
    eng.ingest_files(arcs_path, map_path)
    st = eng.run(10)
    r = eng.ranks()
    tops = {k: eng.topk(k) for k in (1, 37, 100, 1000)}
    eng.write_top_page(out + ".topPage")          # collective; rank 0 writes
    eng.checkpoint_save(out + ".ckpt")            # collective; rank 0 writes
    if rank == 0:
        np.save(out + ".ranks.npy", r)
        json.dump({"iterations": st["iterations"],
                   "topk": {str(k): [[int(a), int(b), float(c)] for a, b, c in v]
                            for k, v in tops.items()}}, open(out + ".json", "w"))
    dist.barrier()
    eng.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
