"""Multi-rank paths on CPU (gloo, world_size 2, 127.0.0.1): scene sharding with no data-path collective, the
view-sharded variant with one gradient all-reduce, and the bench's barrier + max-over-ranks timing
(lgm_amd/dist.py). The per-rank render is the CPU oracle (test infrastructure) standing in for the GPU kernels,
which cannot run here; the GPU path shares every line of the sharding logic."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from lgm_amd import dist as D

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scene(B, V, N, seed, H=32):
    from lgm_amd.cameras import orbit_cameras
    from lgm_amd.synthetic import synthetic_gaussians, synthetic_upstream_grads
    g = synthetic_gaussians(B, N, seed=seed)
    cv, cvp, _ = orbit_cameras(V)
    d_img, _, d_alpha, bg = synthetic_upstream_grads(B, V, H, H, seed=seed + 7)
    return g, cv[None].expand(B, V, 4, 4), cvp[None].expand(B, V, 4, 4), d_img, d_alpha, bg


def _render(g, cv, cvp, d_img, d_alpha, bg, H=32):
    from lgm_amd.cameras import tan_half_fov
    from oracle import oracle as O
    t = tan_half_fov(49.1)
    return O.render(g.numpy(), cv.numpy(), cvp.numpy(), t, H, H, bg.numpy(), d_image=d_img.numpy(),
                    d_alpha=d_alpha.numpy(), nthreads=1)


def _worker(rank, port, tmp, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD),
                      LOCAL_RANK=str(rank))
    info = D.rank_info()
    D.init("gloo", info)
    try:
        if mode == "scenes":
            B = 5  # ragged over 2 ranks: 3 + 2 objects
            g, cv, cvp, d_img, d_alpha, bg = _scene(B, 2, 300, seed=11)
            s0, s1 = D.shard_range(B, info.rank, info.world)
            out = _render(g[s0:s1], cv[s0:s1], cvp[s0:s1], d_img[s0:s1], d_alpha[s0:s1], bg)
            np.savez(os.path.join(tmp, f"r{rank}.npz"), image=out["image"], dg=out["d_gaussians"],
                     rng=np.array([s0, s1]))
        elif mode == "views":
            V = 5
            g, cv, cvp, d_img, d_alpha, bg = _scene(1, V, 300, seed=12)
            v0, v1 = D.shard_range(V, info.rank, info.world)
            out = _render(g, cv[:, v0:v1], cvp[:, v0:v1], d_img[:, v0:v1], d_alpha[:, v0:v1], bg)
            dg = torch.from_numpy(out["d_gaussians"].astype(np.float64))
            D.allreduce_scene_grads(dg, info)
            np.savez(os.path.join(tmp, f"r{rank}.npz"), dg=dg.numpy())
        elif mode == "timing":
            import time
            calls = []
            dt = 0.05 * (1 + rank)  # rank 1 is the slow one

            def step():
                calls.append(1)
                time.sleep(dt)

            el = D.timed_steps(step, 3, info, sync=lambda: None)
            np.savez(os.path.join(tmp, f"r{rank}.npz"), el=np.array(el), calls=np.array(len(calls)))
        elif mode == "warmup":
            import time
            import torch.distributed as dist
            dt = 0.004 * (1 + 3 * rank)  # rank 1 is 4x slower: alone it would need fewer calls for the same time

            def step():
                time.sleep(dt)
                t = torch.ones(1)
                dist.all_reduce(t)  # a collective inside the step: the ranks' call counts must match

            n = D.warm_up(step, 2, sync=lambda: None, info=info, min_seconds=0.1)
            np.savez(os.path.join(tmp, f"r{rank}.npz"), n=np.array(n))
    finally:
        D.finalize(info)


def _run(mode, tmp):
    mp.start_processes(_worker, args=(_free_port(), str(tmp), mode), nprocs=WORLD, start_method="spawn")
    return [np.load(os.path.join(tmp, f"r{r}.npz")) for r in range(WORLD)]


def _spawn_target(tmp):
    info = D.rank_info()
    D.init("gloo", info)
    try:
        t = torch.tensor([float(info.rank + 1)])
        import torch.distributed as dist
        dist.all_reduce(t)
        np.savez(os.path.join(tmp, f"s{info.rank}.npz"), rank=info.rank, world=info.world, local=info.local,
                 total=t.numpy(), addr=os.environ["MASTER_ADDR"])
    finally:
        D.finalize(info)


def test_spawn_ranks_sets_launcher_env(tmp_path):
    """bench.py --gpus N without torchrun: dist.spawn_ranks starts N ranks with torchrun's environment."""
    D.spawn_ranks(_spawn_target, WORLD, str(tmp_path))
    res = [np.load(os.path.join(tmp_path, f"s{r}.npz")) for r in range(WORLD)]
    assert [int(r["rank"]) for r in res] == list(range(WORLD))
    assert all(int(r["world"]) == WORLD and int(r["local"]) == int(r["rank"]) for r in res)
    assert all(float(r["total"][0]) == WORLD * (WORLD + 1) / 2 for r in res)
    assert all(str(r["addr"]) == "127.0.0.1" for r in res)


def _ddp_target(tmp, bf16):
    info = D.rank_info()
    D.init("gloo", info)
    try:
        torch.manual_seed(0)  # same init on every rank
        m = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.Tanh(), torch.nn.Linear(32, 14))
        ddp = D.make_ddp(m, bucket_cap_mb=0.001, bf16_compress=bf16)  # tiny buckets: several all-reduces
        x = torch.randn(5, 16, generator=torch.Generator().manual_seed(10 + info.rank))
        ddp(x).pow(2).sum().backward()
        flat = torch.randn(1000, generator=torch.Generator().manual_seed(20 + info.rank))
        D.allreduce_bucketed(flat, 128, info, bf16=False)
        np.savez(os.path.join(tmp, f"d{info.rank}.npz"), g=np.concatenate([p.grad.numpy().ravel() for p in m.parameters()]),
                 flat=flat.numpy())
    finally:
        D.finalize(info)


@pytest.mark.parametrize("bf16", [False, True])
def test_make_ddp_buckets(tmp_path, bf16):
    """DDP through lgm_amd.dist.make_ddp: every rank ends with the same gradients, equal to the mean of the per-rank
    gradients -- in fp32 (the default, as the reference's accelerate DDP) to fp32 rounding, with the opt-in bf16
    compression hook to bf16 rounding; the bucketed all-reduce averages."""
    D.spawn_ranks(_ddp_target, WORLD, str(tmp_path), bf16)
    res = [np.load(os.path.join(tmp_path, f"d{r}.npz")) for r in range(WORLD)]
    np.testing.assert_array_equal(res[0]["g"], res[1]["g"])
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.Tanh(), torch.nn.Linear(32, 14))
    grads = []
    for r in range(WORLD):
        m.zero_grad()
        m(torch.randn(5, 16, generator=torch.Generator().manual_seed(10 + r))).pow(2).sum().backward()
        grads.append(np.concatenate([p.grad.numpy().ravel() for p in m.parameters()]))
    mean = np.mean(grads, 0)
    assert np.abs(res[0]["g"] - mean).max() <= (1e-2 if bf16 else 1e-6) * np.abs(mean).max()
    flats = [torch.randn(1000, generator=torch.Generator().manual_seed(20 + r)).numpy() for r in range(WORLD)]
    np.testing.assert_allclose(res[0]["flat"], np.mean(flats, 0), rtol=1e-6, atol=1e-6)


def _accum_target(tmp):
    """Two ranks, gloo: 3 micro-steps of gradient accumulation (GradAccumulator) through make_ddp, with a comm hook
    counting the buckets DDP all-reduces."""
    info = D.rank_info()
    D.init("gloo", info)
    try:
        torch.manual_seed(0)
        m = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.Tanh(), torch.nn.Linear(32, 14))
        ddp = D.make_ddp(m, bucket_cap_mb=0.001)
        calls = []

        def hook(state, bucket):
            calls.append(len(calls))
            return torch.distributed.algorithms.ddp_comm_hooks.default_hooks.allreduce_hook(None, bucket)

        ddp.register_comm_hook(None, hook)
        acc = D.GradAccumulator(ddp, 3)
        syncs, per_step = [], []
        for k in range(3):
            x = torch.randn(5, 16, generator=torch.Generator().manual_seed(100 * info.rank + k))
            with acc.accumulate():
                acc.backward(ddp(x).pow(2).sum())
                syncs.append(acc.sync_gradients)
                per_step.append(len(calls))
        np.savez(os.path.join(tmp, f"a{info.rank}.npz"), g=np.concatenate([p.grad.numpy().ravel() for p in m.parameters()]),
                 syncs=np.array(syncs), calls=np.array(per_step))
    finally:
        D.finalize(info)


def test_gradient_accumulation_no_sync(tmp_path):
    """accelerate.accumulate's DDP path (main.py:93, gradient_accumulation_steps) through GradAccumulator: the first
    micro-steps all-reduce nothing (no_sync), the last all-reduces once, and every rank ends with the mean over ranks
    of the per-rank sums of loss / steps gradients."""
    D.spawn_ranks(_accum_target, WORLD, str(tmp_path))
    res = [np.load(os.path.join(tmp_path, f"a{r}.npz")) for r in range(WORLD)]
    np.testing.assert_array_equal(res[0]["g"], res[1]["g"])
    for r in res:
        assert r["syncs"].tolist() == [False, False, True]
        assert r["calls"][0] == 0 and r["calls"][1] == 0 and r["calls"][2] > 0
    torch.manual_seed(0)
    m = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.Tanh(), torch.nn.Linear(32, 14))
    grads = []
    for r in range(WORLD):
        m.zero_grad()
        for k in range(3):
            x = torch.randn(5, 16, generator=torch.Generator().manual_seed(100 * r + k))
            (m(x).pow(2).sum() / 3).backward()
        grads.append(np.concatenate([p.grad.numpy().ravel() for p in m.parameters()]))
    mean = np.mean(grads, 0)
    assert np.abs(res[0]["g"] - mean).max() <= 1e-6 * np.abs(mean).max()


def test_shard_range():
    for n in range(0, 20):
        for w in range(1, 9):
            rs = [D.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            sizes = [b - a for a, b in rs]
            assert max(sizes) - min(sizes) <= 1
    assert D.scene_seed(0) != D.scene_seed(1)


def test_scene_sharded_equals_single_process(tmp_path):
    res = _run("scenes", tmp_path)
    g, cv, cvp, d_img, d_alpha, bg = _scene(5, 2, 300, seed=11)
    full = _render(g, cv, cvp, d_img, d_alpha, bg)
    for r in res:
        s0, s1 = r["rng"]
        np.testing.assert_array_equal(r["image"], full["image"][s0:s1])
        np.testing.assert_array_equal(r["dg"], full["d_gaussians"][s0:s1])
    assert sum(int(r["rng"][1] - r["rng"][0]) for r in res) == 5


def test_view_sharded_allreduce(tmp_path):
    res = _run("views", tmp_path)
    g, cv, cvp, d_img, d_alpha, bg = _scene(1, 5, 300, seed=12)
    full = _render(g, cv, cvp, d_img, d_alpha, bg)["d_gaussians"]
    for r in res:
        np.testing.assert_allclose(r["dg"], full, rtol=1e-5, atol=1e-7 * np.abs(full).max())
    np.testing.assert_array_equal(res[0]["dg"], res[1]["dg"])


def test_timed_steps_max_over_ranks(tmp_path):
    res = _run("timing", tmp_path)
    els = [float(r["el"]) for r in res]
    assert els[0] == els[1]  # every rank reports the max
    assert els[0] >= 3 * 0.1 * 0.95  # the slow rank's 3 x 0.1 s
    assert all(int(r["calls"]) == 3 for r in res)


def test_warm_up_matches_call_counts_over_ranks(tmp_path):
    """dist.warm_up tops the W warmup steps up to a minimum wall time (the GPU clocks' ramp) with the same number of
    calls on every rank, so a step holding a collective cannot deadlock."""
    res = _run("warmup", tmp_path)
    ns = [int(r["n"]) for r in res]
    assert ns[0] == ns[1] and ns[0] >= 3  # the untimed first call + W = 2
    assert ns[0] * 0.016 >= 0.1 * 0.8  # the collective paces both ranks at the slow one's 16 ms per step


def test_gradient_accumulation_end_of_data():
    """GradAccumulator at the end of the data (accelerate's sync_with_dataloader): with steps = 3 and 4 batches per
    epoch, the 4th (last) batch syncs and restarts the count, so every epoch syncs at batches 3 and 4 and no
    micro-batch gradient is left unsynced between epochs. Without a process group no_sync does not apply."""
    m = torch.nn.Linear(4, 2)
    acc = D.GradAccumulator(m, 3)
    pattern = []
    for epoch in range(3):
        for i in range(4):
            with acc.accumulate(last=i == 3):
                acc.backward(m(torch.ones(1, 4)).sum())
                pattern.append(acc.sync_gradients)
                if acc.sync_gradients:
                    m.zero_grad()
    assert pattern == [False, False, True, True] * 3
    assert acc.count == 0
