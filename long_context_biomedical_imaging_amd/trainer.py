"""Training step — the hot-path driver of /root/reference/trainer/trainer_base.py (:94-189).

One process per GPU (torchrun), torch.distributed over RCCL (backend "nccl" on ROCm). The model is wrapped
in DDP exactly as the reference does (trainer_base.py:98); its bucketed fp32 gradient all-reduce runs on
RCCL over xGMI, overlapped with backward. Per step (trainer_base.py:157-182): forward under autocast,
loss, backward, optimizer step, zero_grad.

Documented deviations from the reference step:
  * autocast dtype is bf16 on gfx950 (the reference's utils/status.py:50-58 `support_bfloat16` checks for
    "A100"/"H100" in the device name and would pick fp16 here); with bf16 no GradScaler is needed;
  * DDP broadcast_buffers=False: the only buffers are constant index tables (relative_position_index,
    Hyena pos-emb t/deltas), so the per-forward broadcast the reference pays moves nothing that changes;
  * a batch of 1 is duplicated as the reference does (trainer_base.py:160-164) when the model holds a BatchNorm
    (the UperNet heads: a PSP bin-1 map has one value per channel and sample, which BatchNorm cannot train on).
    Without one the duplicate changes nothing — a mean loss over two identical samples has the loss and the
    gradients of one — so it is skipped there (the 3-D ViTUNETR / SwinUNETR benches at one volume per GPU
    would otherwise do twice the work for the same update).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F
from torch.optim.adam import _fused_adam


def init_distributed():
    """Returns (rank, local_rank, world_size); initialises the process group when launched by torchrun."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        # LCI_DIST_BACKEND=gloo: rehearse N ranks on fewer GPUs (gloo moves CUDA tensors through the host)
        backend = os.environ.get("LCI_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
    return rank, local, world


TUNED_GEMMS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tunableop_gfx950.csv")


def use_tuned_gemms(path: str = TUNED_GEMMS) -> bool:
    """Route torch's Linear / matmul GEMMs through PyTorch-ROCm TunableOp with the solutions recorded for this
    package's shapes on MI355X (hipBLASLt / rocBLAS solution ids, written by a tuning run of bench.py with
    PYTORCH_TUNABLEOP_ENABLED=1; e.g. the ViT-small qkv projection at L = 65536: 0.58 -> 0.15 ms). Tuning itself
    stays off (it costs ~2 min per workload on first use); shapes absent from the file keep the default
    heuristics, and a file recorded under another PyTorch / ROCm / hipBLASLt / arch is rejected by TunableOp's
    validators. LCI_TUNED_GEMMS=0 disables. Returns whether the table is active."""
    if os.environ.get("LCI_TUNED_GEMMS", "1") == "0" or not os.path.exists(path) or not torch.cuda.is_available():
        return False
    import torch.cuda.tunable as tunable
    tunable.enable(True)
    tunable.tuning_enable(False)
    # anything TunableOp writes at exit goes to the temp dir, never over the shipped table
    import tempfile
    tunable.set_filename(os.path.join(tempfile.gettempdir(), f"lci_tunableop_{os.getpid()}.csv"))
    return bool(tunable.read_file(path))


class _LciAdamStep:
    """Adam / AdamW whose update runs on csrc/optim.hip (kernels.adam_step). A subclass of torch's optimizer built
    with fused=True, so its state (per-parameter device `step`, `exp_avg`, `exp_avg_sq`), param_groups and
    state_dict are torch's own and checkpoints move between the two; only the arithmetic kernel differs (the same
    formulas: csrc/optim.hip). torch's fused kernel gave each 64-K-element chunk one workgroup (~1000 over a
    SwinUNETR step at ~1 TB/s); this one streams at the HBM rate. Groups with options the reference never sets
    (amsgrad, complex or non-f32 parameters, a tensor lr, differentiable) take torch's fused update.

    torch's fused Adam declares `_step_supports_amp_scaling`, so a GradScaler (the reference's loop,
    trainer_base.py:116,171-182) does not unscale / inf-check for it but hands the optimizer `grad_scale` and
    `found_inf`; while either is set the step runs torch's fused kernel with them (gradients unscaled in the kernel,
    the update skipped on a device-side inf / NaN), exactly what the class it derives from does."""

    _decoupled = False

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        grad_scale, found_inf = getattr(self, "grad_scale", None), getattr(self, "found_inf", None)
        scaled = grad_scale is not None or found_inf is not None
        for group in self.param_groups:
            params, grads, exp_avgs, exp_avg_sqs, max_sqs, steps = [], [], [], [], [], []
            has_complex = self._init_group(group, params, grads, exp_avgs, exp_avg_sqs, max_sqs, steps)
            if not params:
                continue
            beta1, beta2 = group["betas"]
            if (scaled or has_complex or group["amsgrad"] or group.get("differentiable")
                    or isinstance(group["lr"], torch.Tensor)
                    or any(p.dtype != torch.float32 or not p.is_cuda for p in params)
                    or any(g.is_sparse or not g.is_contiguous() for g in grads)):
                _fused_adam(params, grads, exp_avgs, exp_avg_sqs, max_sqs, steps, grad_scale, found_inf,
                                             amsgrad=group["amsgrad"], has_complex=has_complex, beta1=beta1,
                                             beta2=beta2, lr=group["lr"], weight_decay=group["weight_decay"],
                                             eps=group["eps"], maximize=group["maximize"], capturable=True,
                                             differentiable=False, decoupled_weight_decay=self._decoupled)
                continue
            torch._foreach_add_(steps, 1)
            from . import kernels
            kernels.adam_step(params, grads, exp_avgs, exp_avg_sqs, steps, group["lr"], beta1, beta2,
                              group["weight_decay"], group["eps"], self._decoupled, group["maximize"])
        return loss


class LciAdam(_LciAdamStep, torch.optim.Adam):
    def __init__(self, params, **kw):
        torch.optim.Adam.__init__(self, params, fused=True, **kw)


class LciAdamW(_LciAdamStep, torch.optim.AdamW):
    _decoupled = True

    def __init__(self, params, **kw):
        torch.optim.AdamW.__init__(self, params, fused=True, **kw)


def build_optimizer(params, config):
    """The reference's optimizers (optim_base.py:87-93; same hyper-parameters). On the GPU Adam / AdamW update on
    csrc/optim.hip (LciAdam / LciAdamW, torch-compatible state); LCI_HIP_ADAM=0 uses torch's fused kernel,
    LCI_FUSED_ADAM=0 torch's multi-tensor one (~150 launches per SwinUNETR step, 6.4 ms per C3 step)."""
    o = config.optim
    params = list(params)
    fused = all(p.is_cuda for p in params) and os.environ.get("LCI_FUSED_ADAM", "1") != "0"
    hip = fused and os.environ.get("LCI_HIP_ADAM", "1") != "0"
    if config.optim_type == "adam":
        if hip:
            return LciAdam(params, lr=o.lr, betas=(o.beta1, o.beta2), weight_decay=o.weight_decay)
        return torch.optim.Adam(params, lr=o.lr, betas=(o.beta1, o.beta2), weight_decay=o.weight_decay,
                                fused=fused or None)
    if config.optim_type == "adamw":
        if hip:
            return LciAdamW(params, lr=o.lr, betas=(o.beta1, o.beta2), weight_decay=o.weight_decay)
        return torch.optim.AdamW(params, lr=o.lr, betas=(o.beta1, o.beta2), weight_decay=o.weight_decay,
                                 fused=fused or None)
    if config.optim_type == "nadam":
        return torch.optim.NAdam(params, lr=o.lr, betas=(o.beta1, o.beta2), weight_decay=o.weight_decay)
    if config.optim_type == "sgd":   # optim_base.py:90-91: momentum 0.9
        return torch.optim.SGD(params, lr=o.lr, momentum=0.9, weight_decay=o.weight_decay)
    raise NotImplementedError(f"Optimizer not implemented: {config.optim_type}")


def loss_fn(config):
    if config.loss_func == "CrossEntropy":
        return nn.CrossEntropyLoss()
    return nn.MSELoss()


class TrainStep:
    """model (already on device) -> DDP -> step(inputs, targets) returns the loss tensor (no host sync)."""

    def __init__(self, model, config, device, ddp: bool):
        self.device = device
        self.model = model
        if ddp:
            kw = {"device_ids": [device.index]} if device.type == "cuda" else {}
            # gradient_as_bucket_view: the parameters' .grad are views into DDP's all-reduce buckets instead of
            # separate tensors copied in and out of them (C5: 3.29 GB of f32 gradients, 805 M of them the zero
            # pos-embed, held once instead of twice)
            self.model = nn.parallel.DistributedDataParallel(model, find_unused_parameters=False,
                                                             broadcast_buffers=False, gradient_as_bucket_view=True,
                                                             **kw)
        self.optim = build_optimizer(self.model.parameters(), config)
        self.loss_func = loss_fn(config)
        self.use_amp = bool(config.use_amp)
        self.clip = float(getattr(config, "clip_grad_norm", 0.0) or 0.0)
        self.accum = max(1, int(getattr(config, "iters_to_accumulate", 1) or 1))
        self.micro = 0   # micro-batches since the last optimizer step (trainer_base.py:172 `idx`)
        self.dup_batch1 = any(isinstance(m, nn.modules.batchnorm._BatchNorm) for m in model.modules())
        self.optim.zero_grad(set_to_none=True)

    def step(self, inputs, targets, update: bool | None = None):
        """trainer_base.py:160-182: a batch of 1 is duplicated (BatchNorm), autocast forward + loss /
        iters_to_accumulate, backward; the optional grad-norm clip, optimizer step and zero_grad run only at the end
        of an accumulation window, i.e. every `iters_to_accumulate` calls (`update=None`), as the reference's
        `(idx + 1) % iters_to_accumulate == 0`. `update=True` forces the step (the reference's last iteration of an
        epoch, `idx + 1 == total_iters`), `update=False` suppresses it."""
        if inputs.shape[0] == 1 and self.dup_batch1:
            inputs = torch.cat([inputs] * 2, dim=0)
            targets = torch.cat([targets] * 2, dim=0)
        dev = "cuda" if self.device.type == "cuda" else "cpu"
        with torch.autocast(device_type=dev, dtype=torch.bfloat16, enabled=self.use_amp):
            out = self.model(inputs)
            loss = self.loss_func(out, targets) / self.accum
        loss.backward()
        self.micro += 1
        if update is None:
            update = self.micro % self.accum == 0
        if update:
            if self.clip > 0:
                nn.utils.clip_grad_norm_(self.model.parameters(), self.clip)
            self.optim.step()
            self.optim.zero_grad(set_to_none=True)
            self.micro = 0
        return loss.detach()


class GraphedStep:
    """A TrainStep captured once into a HIP graph and replayed (HIP graphs instead of a tracing compiler).

    The step (autocast forward, loss, backward, optimizer step, zero_grad) on static input/target buffers is warmed
    up on a side stream, then captured; `step(x, y)` copies the batch into the static buffers (skipped when they
    are the same tensors) and replays the graph. Every liblci launch goes to torch's current stream, so the
    kernels are captured as graph nodes; the per-op host work of the Python modules and autograd (~2000 launches
    per Swin-tiny step) is paid once at capture. Single process only (no DDP: its all-reduce hooks are not part
    of the capture here); the optimizer runs with capturable=True (fused Adam / AdamW keep their step on device).

    Constructing it TRAINS: the `warmup` side-stream steps and the captured step are real optimizer steps on the
    static batch (warmup + 1 updates before the first replay). If the capture fails, the optimizer's `capturable`
    flags are restored before the error propagates (the weights keep the warm-up updates). Gradient accumulation
    (iters_to_accumulate > 1) is refused: the graph replays one fixed step, always with the optimizer update.
    """

    def __init__(self, trainer: "TrainStep", inputs, targets, warmup: int = 2):
        if not isinstance(trainer.model, nn.Module) or isinstance(trainer.model, nn.parallel.DistributedDataParallel):
            raise ValueError("GraphedStep: single-process TrainStep only")
        if trainer.accum != 1:
            raise ValueError("GraphedStep: iters_to_accumulate > 1 is not supported (the graph always updates)")
        # TrainStep.step's duplication of a batch of 1, once on the static buffers; replays duplicate exactly when
        # the capture did (a BatchNorm model captured at batch 1), never a genuine batch of 2
        self.dup = inputs.shape[0] == 1 and trainer.dup_batch1
        if self.dup:
            inputs, targets = self._dup(inputs), self._dup(targets)
        saved = [(g, g["capturable"]) for g in trainer.optim.param_groups if "capturable" in g]
        for g, _ in saved:
            g["capturable"] = True
        self.trainer = trainer
        self.inputs, self.targets = inputs, targets
        try:
            side = torch.cuda.Stream(device=inputs.device)
            side.wait_stream(torch.cuda.current_stream(inputs.device))
            with torch.cuda.stream(side):
                for _ in range(warmup):
                    trainer.step(inputs, targets, update=True)
            torch.cuda.current_stream(inputs.device).wait_stream(side)
            torch.cuda.synchronize(inputs.device)
            self.graph = torch.cuda.CUDAGraph()
            # relaxed: the kernels' one-time launch attributes (hipFuncSetAttribute) are legal during the capture
            with torch.cuda.graph(self.graph, capture_error_mode="relaxed"):
                self.loss = trainer.step(inputs, targets, update=True)
        except Exception:
            for g, c in saved:
                g["capturable"] = c
            raise

    @staticmethod
    def _dup(t):
        return None if t is None else torch.cat([t] * 2, dim=0)

    def step(self, inputs=None, targets=None):
        if inputs is not None and inputs is not self.inputs:
            if self.dup and inputs.shape[0] == 1:
                inputs = self._dup(inputs)
            self.inputs.copy_(inputs)
        if targets is not None and targets is not self.targets:
            if self.dup and targets.shape[0] == 1:
                targets = self._dup(targets)
            self.targets.copy_(targets)
        self.graph.replay()
        return self.loss


def synthetic_batch(config, batch, device, seed):
    """U[0,1) images (B, C, T, H, W) and targets of the task's shape."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.rand(batch, config.no_in_channel, config.time, config.height, config.width, generator=g)
    if config.task_type == "seg":
        y = torch.randint(0, config.no_out_channel, (batch, config.time, config.height, config.width), generator=g)
    elif config.task_type == "class":
        y = torch.randint(0, config.no_out_channel, (batch,), generator=g)
    else:
        y = torch.randn(batch, config.no_out_channel, config.time, config.height, config.width, generator=g)
    return x.to(device), y.to(device)


__all__ = ["init_distributed", "TrainStep", "synthetic_batch", "LciAdam", "LciAdamW", "F"]
