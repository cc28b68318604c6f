"""Data-parallel gradient exchange (hiseg.distributed) on CPU with the gloo backend, world size 2.

The tape / FlatParams / bucket machinery is device-agnostic; here the backward closures are plain torch ops
on CPU tensors that write rank-dependent gradients through TrainState.grad (exactly how the HIP backward
closures reach their gradient pointers).  Checks: the averaged gradients, that the first step learns the
schedule and the second launches buckets during the backward in reverse flat order, and the parameter
broadcast at enable time.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _Toy(nn.Module):
    def __init__(self):
        super().__init__()
        self.a = nn.Conv2d(8, 16, 3)
        self.b = nn.Conv2d(16, 32, 3)
        self.c = nn.Linear(32, 64)
        self.d = nn.BatchNorm2d(64)
        self.e = nn.Linear(64, 4)   # never receives a gradient on the "tape"


def _backward(TE, S, model, rank, step):
    T = TE.Tape(S)
    params = [model.a.weight, model.a.bias, model.b.weight, model.b.bias, model.c.weight, model.c.bias,
              model.d.weight, model.d.bias]
    for j, p in enumerate(params):   # forward order: op j writes params[j]
        def back(p=p, j=j):
            S.grad(p).add_(float((rank + 1) * (j + 1) + step))
        T.push(back)
    S.flat.prepare_backward()
    T.run_backward()


def _worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from hiseg import distributed as HD
        from hiseg import train_engine as TE
        torch.manual_seed(100 + rank)          # different init per rank: the broadcast must unify it
        model = _Toy()
        sync = HD.enable_grad_sync(model, bucket_mb=4 * 300 / (1 << 20))   # ~300-float buckets
        w0 = model.a.weight.detach().clone()
        S = TE.TrainState(model, torch.float32, torch.device("cpu"))
        S.sync = sync
        results = {}
        for step in range(2):
            for p in model.parameters():
                p.grad = None
            _backward(TE, S, model, rank, step)
            results[step] = {n: p.grad.flatten().tolist() for n, p in model.named_parameters() if p.grad is not None}
            results[f"launched{step}"] = list(sync.launched)
        gathered = [None] * world
        dist.all_gather_object(gathered, w0.flatten().tolist())
        q.put((rank, results, len(sync.buckets), dict(sync.launch_after), gathered))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - surfaced by the parent
        q.put((rank, repr(e), None, None, None))


def test_grad_bucket_sync_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    out.sort(key=lambda t: t[0])
    for rank, res, *_ in out:
        assert not isinstance(res, str), res
    _, r0, nb, launch_after, w = out[0]
    assert w[0] == w[1], "parameters were not broadcast from rank 0"
    assert nb >= 3
    names = ["a.weight", "a.bias", "b.weight", "b.bias", "c.weight", "c.bias", "d.weight", "d.bias"]
    for step in range(2):
        for j, n in enumerate(names):
            # mean over ranks of (rank+1)*(j+1)+step
            expect = ((1 + 2) / 2) * (j + 1) + step
            for rank in range(world):
                g = torch.tensor(out[rank][1][step][n])
                assert torch.allclose(g, torch.full_like(g, expect)), (step, n, rank, g[:3])
        # e.* never written: stays zero on every rank
        for rank in range(world):
            assert not any(out[rank][1][step]["e.weight"])
    # step 0 reduces everything at the end; step 1 launches buckets as the tape completes them,
    # last flat bucket first (reverse of the forward order)
    assert sorted(r0["launched0"]) == list(range(nb))
    order = r0["launched1"]
    assert sorted(order) == list(range(nb))
    assert any(k >= 0 for k in launch_after), launch_after
    assert order[0] != 0 and order.index(nb - 1) < order.index(0)


def _count_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from hiseg import distributed as HD
        seen = []

        class _Loss(nn.Module):   # the hook sync_loss_class_weights installs on RefinedHierarchicalLoss
            count_sync = None

        loss = HD.sync_loss_class_weights(_Loss())
        c = torch.tensor([10.0 + rank, 20.0 * (rank + 1), 3.0, 4.0 + 2 * rank], dtype=torch.float64)
        loss.count_sync(c)
        seen.append(c.tolist())
        q.put((rank, seen))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))


def test_loss_class_counts_all_reduced_gloo_world2():
    """sync_loss_class_weights: each rank's 4 class pixel counts become their sum over the ranks before the
    loss's EMA update (the GPU side of the same hook: tests/test_gpu_train.py
    test_loss_class_weights_data_parallel_equal_single_process)."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_count_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
    for rank, res in out:
        assert not isinstance(res, str), res
        assert res[0] == [21.0, 60.0, 6.0, 10.0]


def _state_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        import types
        from hiseg import distributed as HD
        # FusedAdamW's device state (moments, segment bounds, step counts); rank 1 has a different segment count
        # (another unfreeze history): it adopts rank 0's table size
        if rank == 0:
            seg, steps, nseg = torch.tensor([0, 2, 6]), torch.tensor([3, 5, 3, 5], dtype=torch.int32), 2
        else:
            seg, steps, nseg = torch.tensor([0, 1, 4, 6]), torch.tensor([1, 2, 3, 1, 2, 3], dtype=torch.int32), 3
        opt = types.SimpleNamespace(exp_avg=torch.full((6,), float(rank + 1)),
                                    exp_avg_sq=torch.full((6,), 10.0 * (rank + 1)),
                                    _seg_start=seg, _steps=steps, _nseg=nseg)
        loss = types.SimpleNamespace(_state=torch.arange(8, dtype=torch.float64) * (rank + 1))
        HD.broadcast_training_state(opt, loss)
        q.put((rank, [opt.exp_avg.tolist(), opt.exp_avg_sq.tolist(), opt._steps.tolist(), loss._state.tolist(),
                      opt._seg_start.tolist(), opt._nseg]))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e)))


def test_broadcast_training_state_gloo_world2():
    """the DDP bench leg starts from rank 0's optimizer moments, per-parameter step counts and loss
    EMA state, not from each rank's own local-training state."""
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_state_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
    for rank, res in out:
        assert not isinstance(res, str), res
        assert res == [[1.0] * 6, [10.0] * 6, [3, 5, 3, 5], [float(i) for i in range(8)], [0, 2, 6], 2]
