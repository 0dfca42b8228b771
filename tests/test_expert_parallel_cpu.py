"""All-to-all expert parallelism (parallel/expert_parallel.py) over gloo, world 2 and 4:
token-sharded dispatch/combine equals the single-process MoE on every rank's tokens, the TP
engine's replicated form equals the all-reduce form, and a TP=2 engine with
EIA_EP_DISPATCH=all_to_all reproduces TP=1's greedy tokens."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from enterprise_inference_amd.ops import reference as ref


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
        from enterprise_inference_amd.ops import moe
        from enterprise_inference_amd.parallel.expert_parallel import (moe_all_to_all,
                                                                       moe_all_to_all_replicated)
        E, k, H, I = 8, 2, 64, 48
        g = torch.Generator().manual_seed(0)
        w13 = torch.randn(E, 2 * I, H, generator=g) * H ** -0.5
        w2 = torch.randn(E, H, I, generator=g) * I ** -0.5
        e_per = E // world
        lo = rank * e_per
        # token-sharded: every rank has its own tokens (different counts per rank)
        gx = torch.Generator().manual_seed(100 + rank)
        T = 5 + 3 * rank
        x = torch.randn(T, H, generator=gx)
        w, ids = moe.topk_route(torch.randn(T, E, generator=gx), k, True)
        got = moe_all_to_all(x, w, ids, w13[lo:lo + e_per], w2[lo:lo + e_per], lo, e_per)
        want = ref.fused_moe(x, w13, w2, w, ids)
        err1 = (got - want).abs().max().item()
        # padded, host-sync-free exchange (capacity = the largest rank's T * k, equal on every
        # rank): same result; no split sizes are read back (tolist / item would raise)
        cap = (5 + 3 * (world - 1)) * k
        real_tolist, real_item = torch.Tensor.tolist, torch.Tensor.item

        def no_sync(*a, **kw):
            raise AssertionError("host read-back in the padded all-to-all")
        torch.Tensor.tolist, torch.Tensor.item = no_sync, no_sync
        try:
            gotp = moe_all_to_all(x, w, ids, w13[lo:lo + e_per], w2[lo:lo + e_per], lo, e_per,
                                  capacity=cap)
        finally:
            torch.Tensor.tolist, torch.Tensor.item = real_tolist, real_item
        err1 = max(err1, (gotp - want).abs().max().item())
        # replicated tokens (TP engine form) vs the all-reduce EP form
        gr = torch.Generator().manual_seed(7)
        Tr = 11
        xr = torch.randn(Tr, H, generator=gr)
        wr, idr = moe.topk_route(torch.randn(Tr, E, generator=gr), k, True)
        a2a = moe_all_to_all_replicated(xr, wr, idr, w13[lo:lo + e_per], w2[lo:lo + e_per], lo,
                                        e_per)
        part = moe.fused_moe(xr, w13[lo:lo + e_per], w2[lo:lo + e_per], wr, idr,
                             (lo, lo + e_per))
        dist.all_reduce(part)
        err2 = (a2a - part).abs().max().item()
        # the same batch through the exact-split exchange (prefill-sized form)
        from enterprise_inference_amd.parallel import expert_parallel as ep
        saved = ep.PADDED_MAX_TOKENS
        ep.PADDED_MAX_TOKENS = 0
        try:
            exact = moe_all_to_all_replicated(xr, wr, idr, w13[lo:lo + e_per],
                                              w2[lo:lo + e_per], lo, e_per)
        finally:
            ep.PADDED_MAX_TOKENS = saved
        err2 = max(err2, (exact - part).abs().max().item())
        q.put((rank, err1, err2))
    except Exception as e:   # noqa: BLE001
        q.put((rank, repr(e), None))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_all_to_all_moe_matches_single_process(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    for rank, e1, e2 in res:
        assert not isinstance(e1, str), e1
        assert e1 < 1e-4 and e2 < 1e-4, (rank, e1, e2)


def test_tp2_all_to_all_ep_engine_matches_tp1(tmp_path, monkeypatch):
    from tests.test_tensor_parallel_cpu import _ckpt, _run
    from enterprise_inference_amd.models.catalog import tiny_config
    d = tiny_config("MixtralForCausalLM")
    path = _ckpt(tmp_path, d)
    ref_toks = _run(path, d, 1)
    monkeypatch.setenv("EIA_EP_DISPATCH", "all_to_all")
    got = _run(path, d, 2, ep=True)
    assert got == ref_toks


def test_dispatch_layout_slots():
    """Each (token, slot) pair lands in its owner's block, in order, without collisions."""
    from enterprise_inference_amd.parallel.expert_parallel import dispatch_layout
    ids = torch.tensor([[5, 0], [1, 7], [4, 2], [6, 3]], dtype=torch.int32)   # 8 experts
    gids, dest = dispatch_layout(ids, e_per=2, world=4, capacity=8)
    assert gids.tolist() == [5, 0, 1, 7, 4, 2, 6, 3]
    # owners 2,0,0,3,2,1,3,1 -> block * 8 + running position within the block
    assert dest.tolist() == [16, 0, 1, 24, 17, 8, 25, 9]
    assert len(set(dest.tolist())) == len(dest)
