"""Scene-sharded multi-GPU execution of the render path: one process per GPU, no data-path collective.

The reference renders every object of a batch on its own (core/gs.py:42-93, a Python loop over B) and trains
with accelerate's DDP: objects are split across ranks and only the UNet's parameter gradients are
all-reduced, by DDP, outside this path. So the render path shards by object (scene): rank r owns objects
shard_range(B, r, world); ranks never exchange splats, pixels or per-Gaussian gradients. The only collectives
here are the barrier and the max-over-ranks time reduction of the bench (torch.distributed: RCCL on GPUs,
gloo in the CPU tests).
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import Callable


@dataclass(frozen=True)
class RankInfo:
    rank: int
    world: int
    local: int


def rank_info() -> RankInfo:
    """RANK / WORLD_SIZE / LOCAL_RANK as set by torch.distributed.run (defaults: a single process)."""
    return RankInfo(int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
                    int(os.environ.get("LOCAL_RANK", 0)))


def init(backend: str, info: RankInfo, device=None) -> None:
    """Initialise the default process group when world > 1 (env:// rendezvous; MASTER_ADDR 127.0.0.1 on one node)."""
    if info.world <= 1:
        return
    import torch.distributed as dist
    if not dist.is_initialized():
        kw = {"device_id": device} if (device is not None and backend == "nccl") else {}
        dist.init_process_group(backend, rank=info.rank, world_size=info.world, **kw)


def finalize(info: RankInfo) -> None:
    if info.world > 1:
        import torch.distributed as dist
        if dist.is_initialized():
            dist.destroy_process_group()


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous, balanced split of n objects over world ranks (sizes differ by at most one)."""
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def scene_seed(rank: int, base: int = 1) -> int:
    """Seed of the synthetic scene rank `rank` renders in the weak-scaling bench (one distinct scene per GPU)."""
    return base + rank


def barrier(info: RankInfo) -> None:
    if info.world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x: float, info: RankInfo, device=None) -> float:
    if info.world <= 1:
        return float(x)
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def warm_up(step: Callable[[], None], steps: int, sync: Callable[[], None], info: RankInfo = None, device=None,
            min_seconds: float = 0.05) -> int:
    """Untimed warmup: `steps` calls of step() (at least one), then as many more as bring the warmup to min_seconds of
    wall time at the measured rate -- the same count on every rank (max over ranks), so steps that hold collectives
    stay matched. Returns the number of calls. The GPU's clocks ramp under load: a single-scene step takes ~240 us
    for its first ~60 steps after a pause (253 us after 100 ms idle) and 224-225 us from ~15-20 ms of continuous
    work on (profiles/r04/diag_idle), so a warmup counted only in steps (10 x 0.23 ms) left the whole timed loop on
    the ramp."""
    import math
    import time
    steps = max(1, steps)
    # the first call carries one-time costs (library load, the workspace's first allocation, autograd setup): it is
    # kept out of the rate estimate, else a slow first call makes W steps "long enough" and the timed loop starts
    # on cold clocks (BENCH_r04's pool: 5 warmup steps, timed mean 6.5 % above the same run's median step)
    step()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    el = time.perf_counter() - t0
    extra = math.ceil(max(0.0, min_seconds - el) / (el / steps)) if el > 0 else 0
    if info is not None and info.world > 1:
        extra = int(max_over_ranks(float(extra), info, device))
    for _ in range(extra):
        step()
    sync()
    return 1 + steps + extra


def timed_steps(step: Callable[[], None], steps: int, info: RankInfo, sync: Callable[[], None],
                device=None, stamps: dict | None = None) -> float:
    """Time exactly `steps` calls of step(): barrier + sync on both sides, wall time maxed over ranks (seconds).
    Python's collector is left as it is: a full collection right before the loop made the next few dozen single-scene
    steps ~16 us slower on the GPU (profiles/r04/diag_host: 225 -> 241 us per step, host work unchanged), and pausing
    it for the loop measured slower too (profiles/r04/s3_gc_paused).

    stamps (a dict, CUDA devices only): also records, inside the timed loop, each step's host enqueue time and an
    event after each step on the current stream, and fills stamps with 'host_ms' (per step), 'gpu_ms' (event to
    event; the first span starts at t0, so it holds the first step's launch latency) and 'tail_ms' (last event to
    the end of the final sync, host clock) -- where a slow loop's time went, at the cost of one event record per
    step."""
    evs = None
    if stamps is not None:
        import torch
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
        host = [0.0] * steps
    barrier(info)
    sync()
    t0 = time.perf_counter()
    if evs is None:
        for _ in range(steps):
            step()
    else:
        evs[0].record()
        for i in range(steps):
            h = time.perf_counter()
            step()
            host[i] = time.perf_counter() - h
            evs[i + 1].record()
    sync()
    t1 = time.perf_counter()
    barrier(info)
    el = t1 - t0
    if evs is not None:
        gpu = [evs[i].elapsed_time(evs[i + 1]) for i in range(steps)]
        stamps.update(host_ms=[round(1e3 * h, 4) for h in host], gpu_ms=[round(g, 4) for g in gpu],
                      loop_ms=round(1e3 * el, 4), gpu_sum_ms=round(sum(gpu), 4),
                      tail_ms=round(1e3 * el - sum(gpu), 4))
    return max_over_ranks(el, info, device)


def _spawned_rank(local_rank, world, port, target, args):
    os.environ.update(RANK=str(local_rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    target(*args)


def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(target: Callable, world: int, *args) -> None:
    """One process per rank on this node without an external launcher: each child gets torch.distributed.run's
    environment (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT) and calls target(*args).
    Started with the 'spawn' method, as fresh children: the caller must not have initialised the GPU (no exec of a
    GPU-initialised process). Raises if any rank fails."""
    import torch.multiprocessing as mp
    mp.start_processes(_spawned_rank, args=(world, free_port(), target, args), nprocs=world, start_method="spawn")


def allreduce_scene_grads(grad, info: RankInfo):
    """View-sharded variant: when the V views of ONE scene are split over ranks
    (views shard_range(V, rank, world)), each rank's dL/dgaussians holds only its views' contributions; one
    in-place SUM all-reduce (RCCL over xGMI: 2(G-1)/G x 56 N bytes per GPU) completes the per-scene sum that
    the single-GPU backward does across views."""
    if info.world > 1:
        import torch.distributed as dist
        dist.all_reduce(grad, op=dist.ReduceOp.SUM)
    return grad


def make_ddp(module, device=None, bucket_cap_mb: float = 100.0, bf16_compress: bool = False, **kw):
    """DistributedDataParallel for LGM's training step (main.py:82-109 trains through accelerate's DDP), for one
    node of MI355X over xGMI: RCCL's ring all-reduce is bound by the 7 point-to-point links
    (~153 GB/s each), not by launch count, so the default buckets are larger than DDP's 25 MB (the 'big' UNet's
    1.66 GB of fp32 gradients in ~17 buckets of 100 MB, each still overlapping the backward of the layers before
    it). Gradients are all-reduced in fp32, as the reference's accelerate DDP does; bf16_compress=True opts into
    torch's bf16_compress_hook (half the link bytes, gradients rounded to bf16 on the wire -- a numerics change, off
    by default). The bucket size and the hook are link-bytes arguments, unmeasured on 8 GPUs here (the driver's
    8-GPU run is the measurement). Wraps whenever a process group is initialised (a one-rank group too: DDP's
    reducer and hooks then run on the real communicator); without one the module is returned unchanged."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return module
    from torch.distributed.algorithms.ddp_comm_hooks import default_hooks
    from torch.nn.parallel import DistributedDataParallel as DDP
    ids = None
    if device is not None and getattr(device, "type", str(device)) == "cuda":
        ids = [device]
    ddp = DDP(module, device_ids=ids, bucket_cap_mb=bucket_cap_mb, **kw)
    if bf16_compress:
        ddp.register_comm_hook(None, default_hooks.bf16_compress_hook)
    return ddp


class GradAccumulator:
    """Gradient accumulation over `steps` micro-batches for a make_ddp model, with accelerate's semantics
    (main.py:93 `accelerator.accumulate(model)`, core/options.py:48 gradient_accumulation_steps): the first
    steps - 1 micro-steps run their backward inside DDP's no_sync() (gradients summed locally, no all-reduce), the
    last one all-reduces the summed gradients once; backward() scales the loss by 1 / steps (accelerate.backward)
    and `sync_gradients` says when the clip and the optimizer step apply (accelerate skips both otherwise).
    The last batch of the data forces a sync and restarts the count (accelerate's sync_with_dataloader default:
    an epoch whose length `steps` does not divide neither carries its leftover micro-batch gradients into the next
    epoch nor shifts the next epoch's sync phase); pass last=True for it.
        acc = GradAccumulator(ddp, steps)
        for i, batch in enumerate(loader):
            with acc.accumulate(last=i == len(loader) - 1):
                loss = ...; acc.backward(loss)
                if acc.sync_gradients: clip; opt.step(); opt.zero_grad()"""

    def __init__(self, model, steps: int = 1):
        if steps < 1:
            raise ValueError("gradient accumulation steps must be >= 1")
        self.model, self.steps, self.count, self.sync_gradients = model, int(steps), 0, True

    def accumulate(self, last: bool = False):
        import contextlib
        if last:  # (accelerate GradientState.end_of_dataloader: sync, and the next micro-step counts from 1)
            self.count, self.sync_gradients = 0, True
        else:
            self.count += 1
            self.sync_gradients = self.count % self.steps == 0
        no_sync = getattr(self.model, "no_sync", None)
        return contextlib.nullcontext() if self.sync_gradients or no_sync is None else no_sync()

    def backward(self, loss):
        (loss / self.steps if self.steps > 1 else loss).backward()


def allreduce_bucketed(flat, bucket_elems: int, info: RankInfo, bf16: bool = False):
    """All-reduce (average) of one flat fp32 gradient buffer in buckets, as DDP does at the end of the backward:
    the communication cost of the training step's parameter gradients (bench.py's cfg5 object). fp32 on the wire
    by default (the reference's numerics); bf16=True halves the bytes (make_ddp's bf16_compress)."""
    if info.world <= 1:
        return flat
    import torch
    import torch.distributed as dist
    for b0 in range(0, flat.numel(), bucket_elems):
        seg = flat[b0:b0 + bucket_elems]
        if bf16:
            t = seg.to(torch.bfloat16)
            dist.all_reduce(t)
            seg.copy_(t.float().div_(info.world))
        else:
            dist.all_reduce(seg)
            seg.div_(info.world)
    return flat
