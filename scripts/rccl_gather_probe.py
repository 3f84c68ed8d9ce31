#!/usr/bin/env python3
"""The RCCL branch of the germline result gather (distributed.gather_germline on a "cuda:k"
device) in one process: torch.distributed over nccl (= RCCL) at world size 1, so the HIP
device-to-device copy of the library's result image into a torch tensor, the RCCL all-gathers
of counts and sizes, and the image decode all run; the gathered records must equal the
library's own host copy.  Prints one JSON line; exit status 0 iff identical."""
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import torch.distributed as dist
    from guacamole_amd import native, synthetic
    from guacamole_amd.distributed import gather_germline
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    g = synthetic.generate(300_000, 30.0)
    ctx = native.Context(0)
    reads = ctx.upload(g.arrays)
    loci = (np.array([0], np.int32), np.array([0], np.int64), np.array([299_999], np.int64), np.array([0], np.int64))
    want = ctx.germline_threshold(reads, loci, 8).tuples(["20"])
    calls = ctx.germline_threshold_device(reads, loci, 8)
    got = gather_germline(calls, "cuda:0")
    rows = [t for c in got for t in c.tuples(["20"])]
    dist.destroy_process_group()
    ok = rows == want and len(rows) > 100
    print(json.dumps({"backend": "nccl", "world": 1, "records": len(rows), "identical": rows == want}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
