"""Fused SGD(nesterov) + ModelEMA step (csrc/optim.hip, yolox_amd.optim.FusedStep) vs the
reference's torch path: torch.optim.SGD with the reference parameter groups
(config.py:307-333, foreach) followed by ModelEMA.update (utils/ema.py:46-58), over
three steps with changing gradients, BN statistics and learning rate.  Bar: fp32
element-wise ops in the same order -> within 1 ulp-scale (rel 1e-6) of torch."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a - b).abs().max() / (b.abs().max() + 1e-30))


@pytest.mark.parametrize("name", ["yolox_s", "yolox_nano"])
def test_fused_step_matches_torch_sgd_and_ema(name):
    from yolox_amd.config import named_config
    from yolox_amd.optim import FusedStep
    from yolox_amd.trainer import ModelEMA, get_optimizer

    torch.manual_seed(0)
    ma = named_config(name).get_model().cuda()
    mb = copy.deepcopy(ma)
    oa, ob = get_optimizer(ma, lr=0.01), get_optimizer(mb, lr=0.01)
    ea, eb = ModelEMA(ma, 0.9998), ModelEMA(mb, 0.9998)
    fused = FusedStep(mb, ob, eb)
    g = torch.Generator(device="cuda").manual_seed(1)
    for step in range(3):
        for pa, pb in zip(ma.parameters(), mb.parameters()):
            gr = torch.randn(pa.shape, generator=g, device="cuda") * 1e-2
            pa.grad, pb.grad = gr.clone(), gr.clone()
        for (ka, ba), (kb, bb) in zip(ma.named_buffers(), mb.named_buffers()):
            if ba.dtype.is_floating_point:
                d = torch.rand(ba.shape, generator=g, device="cuda")
                ba.add_(d)
                bb.add_(d)
        for o in (oa, ob):
            for grp in o.param_groups:
                grp["lr"] = 0.01 * (step + 1) / 3  # warm-up style schedule
        oa.step()
        ea.update(ma)
        fused.step()
        torch.cuda.synchronize()
        for (n, pa), pb in zip(ma.named_parameters(), mb.parameters()):
            assert _rel(pb, pa) < 1e-6, (step, n)
            assert _rel(ob.state[pb]["momentum_buffer"], oa.state[pa]["momentum_buffer"]) < 1e-6, (step, n)
        sa, sb = ea.ema.state_dict(), eb.ema.state_dict()
        for k in sa:
            if sa[k].dtype.is_floating_point:
                assert _rel(sb[k], sa[k]) < 1e-6, (step, k)
        assert ea.updates == eb.updates


def test_fused_step_bumps_versions_and_rejects_missing_grads():
    from yolox_amd.config import named_config
    from yolox_amd.optim import FusedStep
    from yolox_amd.trainer import get_optimizer

    m = named_config("yolox_nano").get_model().cuda()
    o = get_optimizer(m, lr=0.01)
    f = FusedStep(m, o)
    with pytest.raises(RuntimeError):
        f.step()  # no gradients yet
    for p in m.parameters():
        p.grad = torch.ones_like(p)
    v = [p._version for p in m.parameters()]
    f.step()
    assert all(p._version > a for p, a in zip(m.parameters(), v))
    assert all("momentum_buffer" in o.state[p] for p in m.parameters())


def test_fused_step_with_grad_scaler_matches_torch():
    """--fp16 step (trainer.py:111-114): torch GradScaler.scale/step/update + SGD + EMA vs
    FusedStep.step(scaler) over 5 steps with growth_interval 2 (the scale grows), an inf
    gradient at step 2 (step skipped, scale backs off, EMA still updates) and a NaN at
    step 4.  Parameters, momentum, EMA, unscaled .grad, scale and growth tracker."""
    from yolox_amd.config import named_config
    from yolox_amd.optim import FusedStep
    from yolox_amd.trainer import ModelEMA, get_optimizer

    torch.manual_seed(0)
    ma = named_config("yolox_nano").get_model().cuda()
    mb = copy.deepcopy(ma)
    oa, ob = get_optimizer(ma, lr=0.01), get_optimizer(mb, lr=0.01)
    ea, eb = ModelEMA(ma, 0.9998), ModelEMA(mb, 0.9998)
    sa = torch.amp.GradScaler("cuda", init_scale=2.0 ** 10, growth_interval=2)
    sb = torch.amp.GradScaler("cuda", init_scale=2.0 ** 10, growth_interval=2)
    fused = FusedStep(mb, ob, eb)
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.ones((), device="cuda", requires_grad=True)
    for step in range(5):
        for s in (sa, sb):
            s.scale(x)  # lazy init of the scale / tracker tensors, as scaler.scale(loss)
        grads = [torch.randn(p.shape, generator=g, device="cuda") * float(sa.get_scale()) * 1e-2
                 for p in ma.parameters()]
        if step == 2:
            grads[3].view(-1)[0] = float("inf")
        if step == 4:
            grads[7].view(-1)[1] = float("nan")
        for pa, pb, gr in zip(ma.parameters(), mb.parameters(), grads):
            pa.grad, pb.grad = gr.clone(), gr.clone()
        sa.step(oa)
        sa.update()
        ea.update(ma)
        fused.step(sb)
        torch.cuda.synchronize()
        assert float(sb.get_scale()) == float(sa.get_scale()), step
        assert int(sb._growth_tracker) == int(sa._growth_tracker), step
        for (n, pa), pb in zip(ma.named_parameters(), mb.parameters()):
            if step in (2, 4):  # skipped step: .grad holds the unscaled gradient on both sides
                # (after a taken step torch's foreach SGD has also added m * buf into the
                # .grad of nesterov params without weight decay -- not part of the contract)
                assert torch.equal(pb.grad.isfinite(), pa.grad.isfinite()), (step, n)
                fin = pa.grad.isfinite()
                assert _rel(pb.grad[fin], pa.grad[fin]) < 1e-6, (step, n)
            assert _rel(pb, pa) < 1e-6, (step, n)
            if "momentum_buffer" in oa.state[pa]:
                assert _rel(ob.state[pb]["momentum_buffer"], oa.state[pa]["momentum_buffer"]) < 1e-6, (step, n)
        ema_a, ema_b = ea.ema.state_dict(), eb.ema.state_dict()
        for k in ema_a:
            if ema_a[k].dtype.is_floating_point:
                assert _rel(ema_b[k], ema_a[k]) < 1e-6, (step, k)
    assert float(sa.get_scale()) != 2.0 ** 10  # grew and backed off along the way
