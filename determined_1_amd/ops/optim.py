"""Fused, arena-based optimizer steps for stock ``torch.optim`` optimizers.

``FusedOptimizer(opt)`` re-homes the optimizer's parameters into arenas (``arena.py``) and
replaces ``opt.step`` with one HIP launch per arena (``libdetkernels.so``: ``det_sgd_step``,
``det_adam_step`` ...).  The optimizer object itself stays a stock ``torch.optim.SGD`` /
``Adam`` / ``AdamW`` / ``RMSprop`` / ``Adagrad`` / ``Adadelta``:

  * ``param_groups`` hyper-parameters are read every step, so LR schedulers keep working;
  * per-parameter state tensors are *views* into flat fp32 state arenas, so
    ``opt.state_dict()`` has exactly the stock layout and checkpoints stay loadable by a plain
    PyTorch program (the reference stores ``optimizers_state_dict`` verbatim,
    ``harness/determined/pytorch/_pytorch_trial.py:741-744``);
  * ``opt.load_state_dict()`` is wrapped to copy loaded state back into the arenas.

The step takes an extra gradient scale (host float x optional device scalar) and an optional
device ``found_inf`` flag; this is where DP averaging, ``aggregation_frequency`` division
(``_pytorch_context.py:470-477``), AMP unscale and the clip coefficient are applied -- all in the
optimizer's single read of the gradient.

Reference optimizer kinds used by the reference's examples: SGD (``pytorch_onevar_model.py:65``),
RMSprop (``cifar10_pytorch/model_def.py:69``), Adadelta (``mnist_pytorch/model_def.py``),
AdamW (``bert_squad_pytorch/model_def.py:63``).
"""
import math
from typing import Any, Callable, Dict, List, Optional, Tuple

import torch

from determined_1_amd.ops import _lib
from determined_1_amd.ops.arena import Arena, build_arenas
from determined_1_amd.ops.functional import _stream_ptr, dtype_code, is_gpu

# state slot names as stored by torch.optim, per kind
_KINDS = {
    torch.optim.SGD: "sgd",
    torch.optim.Adam: "adam",
    torch.optim.AdamW: "adamw",
    torch.optim.RMSprop: "rmsprop",
    torch.optim.Adagrad: "adagrad",
    torch.optim.Adadelta: "adadelta",
}

MASTER_KEY = "det_master_param"


def fused_kind(opt: torch.optim.Optimizer) -> Optional[str]:
    """Return the fused kind for ``opt`` or None if it cannot be fused exactly."""
    kind = _KINDS.get(type(opt))
    if kind is None:
        return None
    for g in opt.param_groups:
        if g.get("maximize", False) or g.get("differentiable", False):
            return None
        if kind in ("adam", "adamw") and isinstance(g.get("lr"), torch.Tensor):
            return None
        if kind == "adagrad" and g.get("lr_decay", 0) != 0 and False:
            return None
    return kind


def _slots(kind: str, group: Dict[str, Any]) -> List[str]:
    """Kernel state slots (in kernel argument order) for a param group."""
    if kind == "sgd":
        return ["momentum_buffer"] if group.get("momentum", 0) != 0 else []
    if kind in ("adam", "adamw"):
        return ["exp_avg", "exp_avg_sq"] + (["max_exp_avg_sq"] if group.get("amsgrad", False) else [])
    if kind == "rmsprop":
        return ["square_avg", "momentum_buffer", "grad_avg"]
    if kind == "adagrad":
        return ["sum"]
    if kind == "adadelta":
        return ["square_avg", "acc_delta"]
    raise ValueError(kind)


def _visible(kind: str, group: Dict[str, Any], slot: str) -> bool:
    """Whether torch.optim would expose ``slot`` in state for this group."""
    if kind == "rmsprop":
        if slot == "momentum_buffer":
            return group.get("momentum", 0) > 0
        if slot == "grad_avg":
            return bool(group.get("centered", False))
    return True


def _has_step(kind: str) -> bool:
    return kind != "sgd"


class _GroupState:
    def __init__(self, arenas: List[Arena]) -> None:
        self.arenas = arenas
        self.slots = {}  # type: Dict[int, Dict[str, torch.Tensor]]  # arena idx -> slot -> flat
        self.initialized = False
        self.step = None  # type: Optional[torch.Tensor]  # shared CPU scalar (torch's layout)
        self.momentum_ready = False  # SGD: torch clones d_p on the first step
        # Adam on the GPU: [lr, 1 - b1^t, sqrt(1 - b2^t)] in device memory, read by the kernel at run
        # time (a hipGraph replays kernel arguments; these change every step)
        self.hyper_dev = None  # type: Optional[torch.Tensor]


class FusedOptimizer:
    """Arena-backed fused step engine attached to a stock torch optimizer."""

    def __init__(self, optimizer: torch.optim.Optimizer, device: torch.device) -> None:
        kind = fused_kind(optimizer)
        if kind is None:
            raise ValueError(f"{type(optimizer).__name__} cannot be fused")
        self.opt = optimizer
        self.kind = kind
        self.device = device
        self.groups = []  # type: List[_GroupState]
        for group in optimizer.param_groups:
            self.groups.append(_GroupState(build_arenas(group["params"], device)))
        # per-step scale inputs, set by the context right before step()
        self.grad_scale = 1.0
        self.grad_scale_dev = None  # type: Optional[torch.Tensor]
        self.found_inf = None  # type: Optional[torch.Tensor]
        self.sink = None  # type: Optional[Any]  # ops.arena.GradSink, attached by the trial context
        self.steps_called = 0
        self._orig_step = optimizer.step
        self._orig_zero_grad = optimizer.zero_grad
        self._orig_load_state_dict = optimizer.load_state_dict
        def _step(closure: Optional[Callable[[], Any]] = None) -> Any:
            optimizer._opt_called = True  # type: ignore  # LR schedulers check this
            return self.step(closure)

        _step._wrapped_by_lr_sched = True  # type: ignore
        optimizer.step = _step  # type: ignore
        optimizer.zero_grad = self.zero_grad  # type: ignore
        optimizer.load_state_dict = self.load_state_dict  # type: ignore
        optimizer._det_fused = self  # type: ignore
        # Adagrad materializes its state eagerly in torch; mirror that.
        if kind == "adagrad":
            for gi in range(len(self.groups)):
                self._bind_state(gi)

    # ------------------------------------------------------------------------------------------
    @property
    def arenas(self) -> List[Arena]:
        return [a for g in self.groups for a in g.arenas]

    def zero_grad(self, set_to_none: bool = True) -> None:  # noqa: ARG002
        if self.sink is not None:
            self.sink.start_window()  # grads -> None; the next backward lands them in one copy
            return
        for a in self.arenas:
            a.zero_grad()

    def ensure_grads(self) -> None:
        if self.sink is not None and self.sink.fresh:
            return
        for a in self.arenas:
            a.ensure_grads()

    def sync_master_from_params(self) -> None:
        for a in self.arenas:
            a.sync_master_from_params()

    # ------------------------------------------------------------------------------------------
    def _bind_state(self, gi: int) -> None:
        gs = self.groups[gi]
        group = self.opt.param_groups[gi]
        st = self.opt.state
        slots = _slots(self.kind, group)
        init_val = float(group.get("initial_accumulator_value", 0.0)) if self.kind == "adagrad" else 0.0
        for ai, a in enumerate(gs.arenas):
            flats = gs.slots.setdefault(ai, {})
            names = slots + ([MASTER_KEY] if a.has_master else [])
            for name in names:
                if name not in flats:
                    if name == MASTER_KEY:
                        flats[name] = a.master
                    else:
                        flats[name] = torch.full((a.numel,), init_val, dtype=torch.float32, device=a.device)
                flat = flats[name]
                for i, p in enumerate(a.params):
                    v = a.view(flat, i)
                    pstate = st.setdefault(p, {})
                    old = pstate.get(name)
                    if old is not None and old is not v:
                        with torch.no_grad():
                            v.copy_(old.to(device=v.device, dtype=v.dtype).view_as(v))
                    if name == MASTER_KEY or _visible(self.kind, group, name):
                        pstate[name] = v
        if _has_step(self.kind):
            step_val = 0.0
            for a in gs.arenas:
                for p in a.params:
                    s = st.get(p, {}).get("step")
                    if s is not None:
                        step_val = float(s.item() if isinstance(s, torch.Tensor) else s)
                        break
            gs.step = torch.tensor(step_val, dtype=torch.float32)
            for a in gs.arenas:
                for p in a.params:
                    st[p]["step"] = gs.step
        if self.kind == "sgd":
            gs.momentum_ready = all(
                "momentum_buffer" in st.get(p, {}) and st[p]["momentum_buffer"] is not None
                for a in gs.arenas
                for p in a.params
            ) and gs.initialized
        gs.initialized = True

    def load_state_dict(self, state_dict: Dict[str, Any]) -> None:
        had = [g.initialized for g in self.groups]
        self._orig_load_state_dict(state_dict)
        # torch casts floating state to its parameter's dtype on load (bf16 for O2 parameters), which
        # would round the fp32 moments and master weights the arenas keep: put the saved values back
        # at their own precision before they are copied into the arenas
        params = [p for g in self.opt.param_groups for p in g["params"]]
        saved = state_dict.get("state", {})
        for k, p in enumerate(params):
            sv = saved.get(k)
            if not sv or p not in self.opt.state:
                continue
            for name, val in sv.items():
                if isinstance(val, torch.Tensor) and val.is_floating_point() and name != "step":
                    self.opt.state[p][name] = val.to(device=p.device)
        # torch replaced our state views with fresh tensors; copy them back into the arenas.
        for gi, gs in enumerate(self.groups):
            group = self.opt.param_groups[gi]
            any_state = any(len(self.opt.state.get(p, {})) > 0 for a in gs.arenas for p in a.params)
            if not any_state and not had[gi] and self.kind != "adagrad":
                continue
            gs.initialized = False
            self._bind_state(gi)
            if self.kind == "sgd":
                gs.momentum_ready = any(
                    "momentum_buffer" in self.opt.state.get(p, {}) for a in gs.arenas for p in a.params
                ) and group.get("momentum", 0) != 0
            if not any(MASTER_KEY in sd for sd in state_dict.get("state", {}).values()):
                for a in gs.arenas:
                    a.sync_master_from_params()

    # ------------------------------------------------------------------------------------------
    # HIP-graph support (pytorch/_graph.py): a captured step replays the kernel launches with the
    # scalar hyper-parameters baked in, so the graph is keyed by the values the NEXT step would
    # pass, and the host-side bookkeeping a replay skips is advanced explicitly.
    def graph_capturable(self) -> bool:
        """Kernel arguments do not change from step to step by themselves (Adagrad's lr decay does;
        Adam's per-step lr and bias corrections are read from device memory, see graph_prepare)."""
        if self.kind == "adagrad":
            return all(float(g.get("lr_decay", 0.0)) == 0.0 for g in self.opt.param_groups)
        return True

    def graph_signature(self) -> Tuple[Any, ...]:
        sig = []
        for gi, gs in enumerate(self.groups):
            group = self.opt.param_groups[gi]
            h = self._hyper(group, gs) if gs.initialized else {"uninitialized": 1}
            if self.kind == "sgd" and gs.initialized:
                h["first"] = int(not gs.momentum_ready)
            if self.kind in ("adam", "adamw"):
                for key in ("lr", "bc1", "bc2s"):  # device-side (graph_prepare)
                    h.pop(key, None)
            sig.append(tuple(sorted(h.items())))
        return tuple(sig)

    def chunk_capturable(self) -> bool:
        """Several steps in one replay: Adam's device-side hyper-parameters hold one step's values."""
        return self.kind not in ("adam", "adamw")

    def capturing(self, on: bool) -> None:
        """Inside a capture the step must not upload its hyper-parameters (the upload would be
        recorded and replayed with stale host data); graph_prepare does it before each replay."""
        self._capturing = on

    def graph_prepare(self, advanced: bool = False) -> None:
        """Before a replay: upload the hyper-parameters of the step it will run -- step count + 1, or
        the count itself right after a capture (which advanced the host bookkeeping already)."""
        if self.kind not in ("adam", "adamw"):
            return
        for gi, gs in enumerate(self.groups):
            if gs.hyper_dev is None:
                continue
            group = self.opt.param_groups[gi]
            t = (float(gs.step.item()) if gs.step is not None else 0.0) + (0.0 if advanced else 1.0)
            b1, b2 = group["betas"]
            self._upload_hyper(gs, float(group["lr"]), 1.0 - float(b1) ** t, math.sqrt(1.0 - float(b2) ** t))

    @staticmethod
    def _upload_hyper(gs: _GroupState, lr: float, bc1: float, bc2s: float) -> None:
        host = torch.tensor([lr, bc1, bc2s], dtype=torch.float32).pin_memory()
        gs.hyper_dev.copy_(host, non_blocking=True)  # the caching host allocator keeps it until copied

    def host_state(self) -> List[Tuple[Optional[float], bool]]:
        return [(float(gs.step) if gs.step is not None else None, gs.momentum_ready) for gs in self.groups]

    def set_host_state(self, state: List[Tuple[Optional[float], bool]]) -> None:
        for gs, (step, ready) in zip(self.groups, state):
            if gs.step is not None and step is not None:
                gs.step.fill_(step)
            gs.momentum_ready = ready

    def graph_replayed(self) -> None:
        """What step() does on the host besides launching kernels."""
        self.opt._opt_called = True  # type: ignore
        for gs in self.groups:
            if gs.step is not None:
                gs.step += 1
            if self.kind == "sgd":
                gs.momentum_ready = True

    # ------------------------------------------------------------------------------------------
    @torch.no_grad()
    def step(self, closure: Optional[Callable[[], Any]] = None) -> Any:
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self.steps_called += 1  # host count of step() calls (a hipGraph capture notes whether it stepped)
        from determined_1_amd.ops.arena import join_side_work

        join_side_work()  # side-stream weight gradients (a loss.backward() outside context.backward)
        for gi, gs in enumerate(self.groups):
            if not gs.initialized:
                self._bind_state(gi)
            group = self.opt.param_groups[gi]
            if gs.step is not None:
                gs.step += 1
            for ai, a in enumerate(gs.arenas):
                self._step_arena(group, gs, ai, a)
            if self.kind == "sgd":
                gs.momentum_ready = True
        return loss

    def _step_arena(self, group: Dict[str, Any], gs: _GroupState, ai: int, a: Arena) -> None:
        flats = gs.slots.get(ai, {})
        slot_names = _slots(self.kind, group)
        s = [flats[n] for n in slot_names] + [None] * (3 - len(slot_names))
        out_model = a.flat_param if a.has_master else None
        gsc = float(self.grad_scale)
        if is_gpu(a.flat_param):
            self._launch(group, gs, a, s, out_model, gsc)
        else:
            self._reference(group, gs, a, s, out_model, gsc)

    def _hyper(self, group: Dict[str, Any], gs: _GroupState) -> Dict[str, float]:
        k = self.kind
        h = {"lr": float(group["lr"]), "wd": float(group.get("weight_decay", 0.0))}
        if k == "sgd":
            h.update(momentum=float(group.get("momentum", 0.0)), dampening=float(group.get("dampening", 0.0)),
                     nesterov=int(bool(group.get("nesterov", False))), first=int(not gs.momentum_ready))
        elif k in ("adam", "adamw"):
            b1, b2 = group["betas"]
            t = float(gs.step.item()) if gs.step is not None else 1.0
            h.update(b1=float(b1), b2=float(b2), eps=float(group["eps"]), amsgrad=int(bool(group.get("amsgrad", False))),
                     bc1=1.0 - float(b1) ** t, bc2s=math.sqrt(1.0 - float(b2) ** t))
        elif k == "rmsprop":
            h.update(alpha=float(group["alpha"]), eps=float(group["eps"]), momentum=float(group.get("momentum", 0.0)),
                     centered=int(bool(group.get("centered", False))))
        elif k == "adagrad":
            t = float(gs.step.item()) if gs.step is not None else 1.0
            h.update(clr=h["lr"] / (1.0 + (t - 1.0) * float(group.get("lr_decay", 0.0))), eps=float(group["eps"]))
        elif k == "adadelta":
            h.update(rho=float(group["rho"]), eps=float(group["eps"]))
        return h

    def _launch(self, group, gs, a: Arena, s, out_model, gsc: float) -> None:
        lib = _lib.get_lib()
        h = self._hyper(group, gs)
        st = _stream_ptr(a.flat_param)
        gd = dtype_code(a.flat_grad.dtype)
        od = dtype_code(a.flat_param.dtype) if out_model is not None else _lib.BF16
        p = a.master.data_ptr()
        g = a.flat_grad.data_ptr()
        ptr = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        om = ptr(out_model)
        gsd = ptr(self.grad_scale_dev)
        fi = ptr(self.found_inf)
        n = a.numel
        k = self.kind
        if k == "sgd":
            rc = lib.det_sgd_step(st, gd, od, p, g, ptr(s[0]), om, n, h["lr"], h["momentum"], h["dampening"], h["wd"],
                                  h["nesterov"], h["first"], gsc, gsd, fi)
        elif k in ("adam", "adamw"):
            if gs.hyper_dev is None:
                if getattr(self, "_capturing", False):
                    raise RuntimeError("first Adam step inside a graph capture (no eager step yet)")
                gs.hyper_dev = torch.zeros(3, dtype=torch.float32, device=a.flat_param.device)
            if not getattr(self, "_capturing", False) and a is gs.arenas[0]:
                self._upload_hyper(gs, h["lr"], h["bc1"], h["bc2s"])
            rc = lib.det_adam_step(st, gd, od, p, g, ptr(s[0]), ptr(s[1]), ptr(s[2]), om, n, h["lr"], h["b1"], h["b2"],
                                   h["eps"], h["wd"], int(k == "adamw"), h["amsgrad"], h["bc1"], h["bc2s"], gsc, gsd, fi,
                                   gs.hyper_dev.data_ptr())
        elif k == "rmsprop":
            rc = lib.det_rmsprop_step(st, gd, od, p, g, ptr(s[0]), ptr(s[1]), ptr(s[2]), om, n, h["lr"], h["alpha"],
                                      h["eps"], h["wd"], h["momentum"], h["centered"], gsc, gsd, fi)
        elif k == "adagrad":
            rc = lib.det_adagrad_step(st, gd, od, p, g, ptr(s[0]), om, n, h["clr"], h["eps"], h["wd"], gsc, gsd, fi)
        else:
            rc = lib.det_adadelta_step(st, gd, od, p, g, ptr(s[0]), ptr(s[1]), om, n, h["lr"], h["rho"], h["eps"],
                                       h["wd"], gsc, gsd, fi)
        _lib.check(rc, f"{k}_step")

    # fp32 PyTorch reference of exactly the kernel math (CPU tests; numerics oracle on GPU tests)
    def _reference(self, group, gs, a: Arena, s, out_model, gsc: float) -> None:
        if self.found_inf is not None and int(self.found_inf.item()) != 0:
            return
        h = self._hyper(group, gs)
        scale = gsc * (float(self.grad_scale_dev.item()) if self.grad_scale_dev is not None else 1.0)
        p = a.master
        g = a.flat_grad.float() * scale
        k = self.kind
        wd = h["wd"]
        if k == "sgd":
            d = g + wd * p if wd else g
            if h["momentum"] != 0:
                buf = s[0]
                if h["first"]:
                    buf.copy_(d)
                else:
                    buf.mul_(h["momentum"]).add_(d, alpha=1 - h["dampening"])
                d = d + h["momentum"] * buf if h["nesterov"] else buf
            p.add_(d, alpha=-h["lr"])
        elif k in ("adam", "adamw"):
            if wd:
                if k == "adamw":
                    p.mul_(1 - h["lr"] * wd)
                else:
                    g = g + wd * p
            m, v, vmax = s[0], s[1], s[2]
            m.lerp_(g, 1 - h["b1"])
            v.mul_(h["b2"]).addcmul_(g, g, value=1 - h["b2"])
            vd = v
            if h["amsgrad"]:
                torch.maximum(vmax, v, out=vmax)
                vd = vmax
            denom = vd.sqrt() / h["bc2s"] + h["eps"]
            p.addcdiv_(m, denom, value=-h["lr"] / h["bc1"])
        elif k == "rmsprop":
            if wd:
                g = g + wd * p
            sq, buf, ga = s
            sq.mul_(h["alpha"]).addcmul_(g, g, value=1 - h["alpha"])
            if h["centered"]:
                ga.lerp_(g, 1 - h["alpha"])
                avg = (sq - ga * ga).sqrt() + h["eps"]
            else:
                avg = sq.sqrt() + h["eps"]
            if h["momentum"] > 0:
                buf.mul_(h["momentum"]).add_(g / avg)
                p.add_(buf, alpha=-h["lr"])
            else:
                p.add_(g / avg, alpha=-h["lr"])
        elif k == "adagrad":
            if wd:
                g = g + wd * p
            sm = s[0]
            sm.addcmul_(g, g)
            p.sub_(h["clr"] * g / (sm.sqrt() + h["eps"]))
        else:
            if wd:
                g = g + wd * p
            sq, acc = s[0], s[1]
            sq.mul_(h["rho"]).addcmul_(g, g, value=1 - h["rho"])
            delta = (acc + h["eps"]).sqrt() / (sq + h["eps"]).sqrt() * g
            acc.mul_(h["rho"]).addcmul_(delta, delta, value=1 - h["rho"])
            p.add_(delta, alpha=-h["lr"])
        if out_model is not None:
            out_model.copy_(p)
