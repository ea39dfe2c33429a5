"""Fused optimizer step: torch.optim.SGD (nesterov) + ModelEMA.update in one HIP pass.

The reference steps the optimizer through the GradScaler and then updates the EMA
(core/trainer.py:124-127; groups config.py:307-333; EMA utils/ema.py:46-58).  On the
HIP path both are HBM-bound element-wise passes; torch runs them as ~10 foreach kernels
plus one per BN buffer.  ``FusedStep`` keeps the torch optimizer as the source of truth
for hyper-parameters (lr schedules write ``param_groups[i]['lr']`` as usual) and for
checkpoints (its momentum buffers are views of the fused step's flat buffer, stored in
``optimizer.state[p]['momentum_buffer']``), and replaces ``optimizer.step()`` +
``ema.update(model)`` with one ``yxh_sgd_ema_step`` launch (csrc/optim.hip).

``step(scaler)`` is the --fp16 form (trainer.py:111-114, ``scaler.step(optimizer);
scaler.update()`` + EMA): the GradScaler's scale / growth tracker tensors are used in
place, the inf/NaN check, the in-place unscale, the skipped-or-taken SGD update, the EMA
update and ``_amp_update_scale_`` all run on the device in three launches, with no host
synchronisation (torch's GradScaler.step reads found_inf with ``.item()``).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import torch

from . import _native as N


class FusedStep:
    def __init__(self, model: torch.nn.Module, optimizer: torch.optim.Optimizer, ema=None):
        if not isinstance(optimizer, torch.optim.SGD):
            raise TypeError("FusedStep wraps torch.optim.SGD (the reference optimizer)")
        if len(optimizer.param_groups) > 4:
            raise ValueError("at most 4 parameter groups")
        moms = {g["momentum"] for g in optimizer.param_groups}
        nest = {bool(g["nesterov"]) for g in optimizer.param_groups}
        if len(moms) != 1 or len(nest) != 1 or any(g["dampening"] != 0 or g.get("maximize", False)
                                                    for g in optimizer.param_groups):
            raise ValueError("FusedStep: one momentum / nesterov setting, dampening 0, maximize False")
        self.opt, self.ema = optimizer, ema
        self.lib = N.lib()
        self.group = {}
        params = []
        for gi, g in enumerate(optimizer.param_groups):
            for p in g["params"]:
                if p.dtype != torch.float32 or not p.is_contiguous() or p.device.type != "cuda":
                    raise ValueError("FusedStep: fp32 contiguous device parameters only")
                self.group[id(p)] = gi
                params.append(p)
        self.params = params
        self.device = params[0].device
        offs, off = {}, 0
        for p in params:
            offs[id(p)] = off
            off += p.numel()
        self.flat_buf = torch.zeros(off, dtype=torch.float32, device=self.device)
        self.bufs = {id(p): self.flat_buf[offs[id(p)]:offs[id(p)] + p.numel()].view_as(p) for p in params}
        held = [p for p in params if "momentum_buffer" in optimizer.state.get(p, {})
                and optimizer.state[p]["momentum_buffer"] is not None]
        if held and len(held) != len(params):
            raise ValueError("FusedStep: momentum buffers exist for some parameters only")
        for p in held:  # resume: continue from the optimizer's buffers
            self.bufs[id(p)].copy_(optimizer.state[p]["momentum_buffer"])
        self.first = not held
        # EMA pairs (ema tensor, model tensor) over floating state_dict entries (ema.py:50-58)
        self.ema_of, self.ema_only = {}, []
        if ema is not None:
            pid = {p.data_ptr(): p for p in params}
            m = model.module if hasattr(model, "module") else model
            model_sd = m.state_dict()
            for k, e in ema.ema.state_dict().items():
                if not e.dtype.is_floating_point:
                    continue
                s = model_sd[k]
                if e.dtype != torch.float32 or s.dtype != torch.float32 or not e.is_contiguous():
                    raise ValueError(f"FusedStep: EMA entry {k} is not fp32 contiguous")
                if s.data_ptr() in pid:
                    self.ema_of[id(pid[s.data_ptr()])] = e
                else:
                    self.ema_only.append((e, s))
        self._key = None
        self.model = model.module if hasattr(model, "module") else model
        self.chunk = int(self.lib.yxh_opt_chunk_elems())
        self.found_inf = torch.zeros(1, dtype=torch.float32, device=self.device)

    def _table(self):
        grads = [p.grad for p in self.params]
        if any(g is None for g in grads):
            raise RuntimeError("FusedStep: every parameter needs a gradient (the HIP reverse pass writes all)")
        key = tuple(g.data_ptr() for g in grads)
        if key == self._key:
            return
        segs, chunks = [], []
        for p, g in zip(self.params, grads):
            if g.dtype != torch.float32 or not g.is_contiguous():
                raise ValueError("FusedStep: fp32 contiguous gradients only")
            gi = self.group[id(p)]
            e = self.ema_of.get(id(p))
            segs.append(N.OptSeg(p.data_ptr(), g.data_ptr(), self.bufs[id(p)].data_ptr(),
                                 e.data_ptr() if e is not None else None, None, p.numel(),
                                 float(self.opt.param_groups[gi]["weight_decay"]), gi))
        for e, s in self.ema_only:
            segs.append(N.OptSeg(None, None, None, e.data_ptr(), s.data_ptr(), e.numel(), 0.0, 0))
        for i, s in enumerate(segs):
            for c in range((s.n + self.chunk - 1) // self.chunk):
                chunks += [i, c]
        raw = (N.OptSeg * len(segs))(*segs)
        self.d_segs = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.device)
        self.d_chunks = torch.tensor(chunks, dtype=torch.int32).to(self.device)
        self.nchunks = len(chunks) // 2
        self._key = key

    @torch.no_grad()
    def step(self, scaler=None) -> None:
        """optimizer.step() + ema.update(model); with an enabled torch GradScaler whose
        scale() produced the gradients: scaler.step(optimizer) + scaler.update() + EMA."""
        self._table()
        amp = scaler is not None and scaler.is_enabled()
        if amp:
            self._check_scaler(scaler)
            st = N.stream_ptr(self.device)
            N.check(self.lib.yxh_amp_found_inf(self.d_segs.data_ptr(), self.d_chunks.data_ptr(), self.nchunks,
                                               self.found_inf.data_ptr(), st), "amp_found_inf")
            if self.first:  # zero buffers: b*m + g == g exactly, the first step needs no flag
                for p in self.params:
                    self.opt.state[p]["momentum_buffer"] = self.bufs[id(p)]
                self.first = False
        hp = N.OptHparams()
        for gi, g in enumerate(self.opt.param_groups):
            hp.lr[gi] = float(g["lr"])
        hp.momentum = float(self.opt.param_groups[0]["momentum"])
        hp.nesterov = int(bool(self.opt.param_groups[0]["nesterov"]))
        hp.first_step = int(self.first)
        if self.ema is not None:
            self.ema.updates += 1
            d = self.ema.decay(self.ema.updates)
            hp.ema_d, hp.ema_omd, hp.do_ema = float(d), float(1.0 - d), 1
        if amp:
            hp.amp_scale, hp.amp_found_inf = scaler._scale.data_ptr(), self.found_inf.data_ptr()
        N.check(self.lib.yxh_sgd_ema_step(self.d_segs.data_ptr(), self.d_chunks.data_ptr(), self.nchunks,
                                          C.byref(hp), N.stream_ptr(self.device)), "sgd_ema_step")
        if amp:
            N.check(self.lib.yxh_amp_update_scale(
                scaler._scale.data_ptr(), scaler._growth_tracker.data_ptr(), self.found_inf.data_ptr(),
                float(scaler._growth_factor), float(scaler._backoff_factor), int(scaler._growth_interval),
                N.stream_ptr(self.device)), "amp_update_scale")
            torch.autograd.graph.increment_version([scaler._scale, scaler._growth_tracker] +
                                                   [p.grad for p in self.params])
        if self.first:
            for p in self.params:
                self.opt.state[p]["momentum_buffer"] = self.bufs[id(p)]
            self.first = False
        # in-place writes behind torch's back: bump versions (eager plans) and the modules'
        # weights epochs (captured plans) so eval plans repack
        torch.autograd.graph.increment_version(self.params)
        for m in (getattr(self.model, "module", self.model), getattr(self.ema, "ema", None)):
            if hasattr(m, "weights_changed"):
                m.weights_changed()
        if self.ema is not None:
            torch.autograd.graph.increment_version(list(self.ema.ema.parameters()))

    def _check_scaler(self, scaler) -> None:
        from torch.amp.grad_scaler import OptState
        if getattr(scaler, "_scale", None) is None or getattr(scaler, "_growth_tracker", None) is None:
            raise RuntimeError("FusedStep.step(scaler): call scaler.scale(loss) before backward")
        for t, dt in ((scaler._scale, torch.float32), (scaler._growth_tracker, torch.int32)):
            if t.device != self.device or t.dtype != dt or t.numel() != 1:
                raise ValueError("FusedStep.step(scaler): scaler state must be on the parameters' device")
        stage = scaler._per_optimizer_states[id(self.opt)]["stage"]
        if stage is not OptState.READY:
            raise RuntimeError("FusedStep.step(scaler): gradients were already unscaled / stepped by the scaler")
