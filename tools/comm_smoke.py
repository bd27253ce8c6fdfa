"""Rendezvous + collectives smoke under ``torch.distributed.run`` (any world size).

``--fake``: the loopback test communicator on CPU (rehearses the torchrun agent-store
rendezvous without GPUs); default: RCCL on ``cuda:LOCAL_RANK``.  Prints one JSON line per
rank with the results of a broadcast, an all-reduce and an object all-gather."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fake", action="store_true")
    a = ap.parse_args()
    import torch

    from flink_tensorflow_amd.parallel import comm

    rank, ws, local = comm.world()
    store = comm.rendezvous_store(rank, ws)
    if a.fake:
        from flink_tensorflow_amd.parallel.fake import FakeCommunicator

        c = FakeCommunicator(rank, ws, "cpu", store)
    else:
        c = comm.RcclCommunicator(rank, ws, torch.device("cuda", comm.local_device(local)), store)
    comm.set_communicator(c)
    x = torch.full((4,), float(rank + 1), device=c.device)
    comm.broadcast_tensors([x], src=0)
    y = torch.full((3,), float(rank + 1), device=c.device)
    c.all_reduce(y)
    objs = comm.all_gather_object({"rank": rank})
    comm.barrier()
    sys.stdout.write(json.dumps({"rank": rank, "ws": ws, "bcast": x.tolist(), "sum": y.tolist(),
                                 "objs": [o["rank"] for o in objs]}) + "\n")  # one write per record
    sys.stdout.flush()
    comm.destroy()


if __name__ == "__main__":
    main()
