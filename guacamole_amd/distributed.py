"""Multi-GPU driver pieces: static LociSet split across ranks + one terminal gather.

Loci ranges shard embarrassingly (each locus depends only on reads overlapping it,
DistributedUtil.scala:585-597 with halfWindowSize = 0), so every rank runs the
pileup engine on its own contiguous loci range with no data-path collective.
The single exchange is the end-of-job gather of the per-rank genotype buffers to
rank 0: sizes are all-gathered, then each rank's packed
buffer goes to rank 0 over RCCL (backend "nccl" on ROCm) — or gloo on CPU tests.
Rank 0 concatenates in rank order = partition order.
"""
from __future__ import annotations

import os
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .loci import LociMapBuilder, LociSet, partition_loci_uniformly


def rank_info() -> Tuple[int, int, int]:
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def split_loci(loci: LociSet, world: int) -> List[LociSet]:
    """Static contiguous split of a LociSet into `world` parts in partition order
    (partitionLociUniformly with tasks = world, DistributedUtil.scala:83-108)."""
    inv = partition_loci_uniformly(world, loci).as_inverse_map()
    return [inv.get(r, LociSet()) for r in range(world)]


def gather_images_to_rank0(calls, device: str):
    # device "cpu": the images are staged in host memory (a gloo rehearsal of the flow)
    """The terminal gather of the multi-GPU bench: every rank's germline result image (left in
    HBM by gq_germline_threshold_device) goes to rank 0's HBM with one RCCL gather over xGMI
    (sizes all-gathered first).  Returns rank 0's list of per-rank uint8 device tensors
    (partition order), None elsewhere."""
    import ctypes as C

    import torch
    import torch.distributed as dist

    calls.check_current()
    world, rank = dist.get_world_size(), dist.get_rank()
    dev = torch.device(device)
    n = torch.tensor([int(calls.image_bytes)], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(x.item()) for x in sizes]
    cap = max(1, max(sizes))
    mine = torch.empty(cap, dtype=torch.uint8, device=dev)
    if calls.image_bytes:
        on_gpu = dev.type == "cuda"
        if on_gpu:
            torch.cuda.synchronize(dev)
        hip = C.CDLL("libamdhip64.so.7")  # by SONAME: the HIP runtime already loaded in this process
        hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        # device to device (RCCL) or device to host (a gloo rehearsal)
        rc = hip.hipMemcpy(C.c_void_p(mine.data_ptr()), C.c_void_p(calls.image), int(calls.image_bytes),
                           3 if on_gpu else 2)
        if rc != 0:
            raise RuntimeError("hipMemcpy of the result image failed (%d)" % rc)
    if rank == 0:
        parts = [torch.empty(cap, dtype=torch.uint8, device=dev) for _ in range(world)]
        dist.gather(mine, gather_list=parts, dst=0)
        return [parts[r][:sizes[r]] for r in range(world)]
    dist.gather(mine, dst=0)
    return None


def gather_to_rank0(buf: np.ndarray, device: Optional[str] = None) -> Optional[List[np.ndarray]]:
    """Variable-size gather of one uint8 buffer per rank to rank 0.

    device: torch device for the collective ("cuda:k" => RCCL over xGMI; None => CPU/gloo)."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size() == 1:
        return [buf]
    world, rank = dist.get_world_size(), dist.get_rank()
    dev = torch.device(device) if device else torch.device("cpu")
    n = torch.tensor([int(buf.size)], dtype=torch.int64, device=dev)
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    cap = max(1, max(sizes))
    mine = torch.zeros(cap, dtype=torch.uint8, device=dev)
    if buf.size:
        mine[:buf.size] = torch.from_numpy(buf).to(dev)
    if rank == 0:
        parts = [torch.empty(cap, dtype=torch.uint8, device=dev) for _ in range(world)]
        dist.gather(mine, gather_list=parts, dst=0)
        return [parts[r][:sizes[r]].cpu().numpy() for r in range(world)]
    dist.gather(mine, dst=0)
    return None
