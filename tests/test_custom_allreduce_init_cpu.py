"""Init-time checks of the custom xGMI all-reduce (parallel/custom_allreduce.py) on the CPU:
the self-test against the reference reduction, the agreed fallback when ONE rank's reduction
is wrong (every rank goes back to RCCL, none keeps the custom kernel), the exported status, and
the timing -> threshold rule.  The custom kernel is replaced by a stand-in that reduces over
gloo, so what is tested is the protocol around it."""

import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from enterprise_inference_amd.parallel import custom_allreduce as cam


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _GlooAR:
    """CustomAllReduce stand-in: the same API, sums over gloo; ``wrong`` perturbs its result
    the way a memory-ordering bug would (one element off, nothing hangs)."""

    device = "cpu"

    def __init__(self, rank, world, wrong=False, max_bytes=8 << 20, raise_case=-1,
                 spin_in_tuning=False):
        self.rank, self.world, self.wrong = rank, world, wrong
        self.max_bytes = self.use_max = max_bytes
        self.oneshot_max = 512 * 1024
        self.closed = False
        self.calls = 0
        self.raise_case = raise_case          # this rank's custom call #n raises
        self.spin_in_tuning = spin_in_tuning  # a timing call sets the sticky error flag
        self.err = 0

    def all_reduce(self, x, out=None, kind=None):
        self.calls += 1
        if self.calls == self.raise_case:
            # a local failure: the peers' custom call has no partner (their kernel would spin
            # out); the stand-in does not join their gloo sum, the protocol must not hang
            raise RuntimeError("injected custom kernel failure")
        if self.raise_case > 0:
            # peers of a raising rank: the custom form is local-only here (no cross-rank
            # traffic), so a missing partner cannot deadlock the stand-in
            return x * self.world
        dist.all_reduce(x)
        if self.wrong:
            x.view(-1)[-1] += 1.0
        if self.spin_in_tuning and x.numel() >= (32 << 10) // 2 and x.dtype == torch.bfloat16 \
                and bool((x == self.world).all()):
            self.err = 1                      # torch.ones input: the tuning pass
        return x

    def add_rmsnorm(self, x, residual, weight, eps, twoshot=None):
        from enterprise_inference_amd.ops import norm
        if hasattr(x, "materialize"):   # split-K slabs: the real kernel sums them while staging
            x = x.materialize()
        s = self.all_reduce(x)
        out, _ = norm.fused_add_rms_norm(s, residual, weight, eps)
        return out

    def error_flag(self):
        return self.err

    def close(self):
        self.closed = True


def _worker(rank, world, port, bad_rank, q, mode="wrong"):
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                                world_size=world)
        if mode == "raise":
            # every rank takes the local-only custom form; rank bad_rank's second custom call
            # raises mid self-test
            ar = _GlooAR(rank, world, raise_case=2 if rank == bad_rank else 10 ** 9)
        elif mode == "spin":
            ar = _GlooAR(rank, world, spin_in_tuning=(rank == bad_rank))
        else:
            ar = _GlooAR(rank, world, wrong=(rank == bad_rank))

        def reference(x):
            dist.all_reduce(x)
            return x

        def agree(t, op):
            dist.all_reduce(t, op=op)
            return t

        got = cam.init_custom_allreduce(8 << 20, factory=lambda mb: ar, reference=reference,
                                        agree=agree, tune=(mode == "spin"))
        from enterprise_inference_amd.parallel import comm
        q.put((rank, got is not None, ar.closed, cam.STATUS["reason"],
               comm.get_custom_allreduce() is not None))
        comm.set_custom_allreduce(None)
    except Exception as e:   # noqa: BLE001
        q.put((rank, repr(e), None, None, None))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _run(world, bad_rank, mode="wrong"):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, bad_rank, q, mode))
          for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    return res


@pytest.mark.parametrize("world,bad", [(2, -1), (2, 1), (4, 0)])
def test_self_test_agreed_fallback(world, bad):
    res = _run(world, bad)
    for rank, active, closed, reason, registered in res:
        assert not isinstance(active, str), active
        if bad < 0:
            assert active and registered and not closed and reason == "ok", res
        else:
            # the wrong rank AND its healthy peers all fall back together
            assert not active and not registered and closed, res
            assert reason == "self-test mismatch", res


def test_self_test_cases_are_exact_and_cover_both_forms():
    cases = cam.selftest_cases(16 << 20, 512 << 10)
    kinds = {(op, kind) for op, _, kind in cases}
    assert kinds == {("ar", 0), ("ar", 1), ("norm", 0), ("norm", 1), ("norm_sk", 0),
                     ("norm_sk", 1)}
    # the split-K input: two integer fp32 slabs whose sum is the bf16 x exactly
    case = next(c for c in cases if c[0] == "norm_sk")
    x, _, _, sk = cam.selftest_inputs(case, 3, "cpu")
    assert sk.sk == 2 and torch.equal(sk.part.sum(0).to(torch.bfloat16), x)
    assert torch.equal(sk.materialize(), x)
    assert len({shape for op, shape, _ in cases if op == "ar"}) == 3
    # integer inputs: the sum over 8 ranks is exact in bf16
    for case in cases[:2]:
        xs = [cam.selftest_inputs(case, r, "cpu")[0] for r in range(8)]
        s32 = torch.stack([x.float() for x in xs]).sum(0)
        assert torch.equal(s32.to(torch.bfloat16).float(), s32)
    # shapes beyond the buffer are not tested
    small = cam.selftest_cases(64 << 10, 32 << 10)
    assert all(2 * (s[0] if op == "ar" else s[0] * s[1]) <= 64 << 10 for op, s, _ in small)


def test_tune_thresholds_rule():
    sizes = [32 << 10, 128 << 10, 512 << 10, 1 << 20, 2 << 20, 4 << 20]
    one = [10, 12, 20, 35, 70, 140]
    two = [14, 15, 18, 25, 40, 75]
    rccl = [30, 30, 32, 34, 45, 70]
    o, u = cam.tune_thresholds(sizes, one, two, rccl, 16 << 20)
    assert o == 128 << 10          # one-shot loses to two-shot from 512 KiB on
    assert u == 2 << 20            # RCCL wins at 4 MiB
    o, u = cam.tune_thresholds(sizes, one, two, [1] * 6, 16 << 20)
    assert u == 0                  # RCCL always faster: nothing routed to the custom kernel


def test_status_gauge_rendered():
    from enterprise_inference_amd.metrics import EngineMetrics
    m = EngineMetrics("tiny")
    m.set_custom_allreduce({"active": False, "reason": "self-test mismatch"})
    text = m.render().decode()
    assert 'eia:custom_allreduce_active{model_name="tiny",reason="self-test mismatch"} 0.0' in text


@pytest.mark.parametrize("world,bad", [(2, 0), (4, 2)])
def test_self_test_local_raise_does_not_hang(world, bad):
    """One rank's custom call raises mid self-test: it keeps running the remaining cases'
    reference collectives with its peers, and every rank falls back together (no hang)."""
    res = _run(world, bad, mode="raise")
    assert len(res) == world
    for rank, active, closed, reason, registered in res:
        assert not isinstance(active, str), active
        assert not active and not registered and closed, res
        assert reason == "self-test mismatch", res


def test_tuning_spin_timeout_falls_back_everywhere():
    """A barrier spin limit hit during the timing pass (sticky error flag on ONE rank): every
    rank closes the custom kernel with reason 'tuning spin timeout' instead of starting the
    engine with a set flag."""
    res = _run(2, 1, mode="spin")
    for rank, active, closed, reason, registered in res:
        assert not isinstance(active, str), active
        assert not active and not registered and closed, res
        assert reason == "tuning spin timeout", res
