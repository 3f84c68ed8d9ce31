#!/usr/bin/env python3
"""GPU check of the multi-GPU bench's terminal gather with one rank (RCCL, world size 1):
gather_images_to_rank0 moves the device result image into a torch tensor; its bytes must equal
the image copied to the host.  Run: python scripts/check_gather.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist
    from guacamole_amd import native, synthetic
    from guacamole_amd.distributed import gather_images_to_rank0

    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:29533", world_size=1, rank=0,
                            device_id=torch.device("cuda", 0))
    g = synthetic.generate(2_000_000, 30.0)
    ctx = native.Context(0)
    reads = ctx.upload(g.arrays)
    loci = (np.array([0], np.int32), np.array([0], np.int64), np.array([1_999_999], np.int64), np.array([0], np.int64))
    d = ctx.germline_threshold_device(reads, loci, 8)
    parts = gather_images_to_rank0(d, "cuda:0")
    got = parts[0].cpu().numpy()
    host = np.zeros(d.image_bytes, np.uint8)
    import ctypes as C
    hip = C.CDLL("libamdhip64.so.7")  # by SONAME: the HIP runtime already loaded in this process
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    assert hip.hipMemcpy(host.ctypes.data, C.c_void_p(d.image), d.image_bytes, 2) == 0
    assert got.shape == host.shape and np.array_equal(got, host), "gathered image differs"
    h = ctx.germline_threshold(reads, loci, 8)
    print("gather ok: %d bytes, %d records (host API %d)" % (d.image_bytes, len(d), len(h)))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
