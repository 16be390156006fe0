"""AVSRTrainer on the HIP engine — drop-in for src/custom_trainer.py:4-102 as script/train.py
uses it (script/train.py:259-308): HF `Trainer` with a separate evaluation collator.

The reference inherits its distributed step from HF Trainer -> accelerate ->
DistributedDataParallel (+ fp16 autocast / GradScaler, torch AdamW, clip_grad_norm_). Here the
same loop (data loading, gradient accumulation, LR schedule, logging, evaluation, checkpoints,
resume) drives the engine instead:

  * the model is NOT wrapped in DDP; `parallel.ArenaDDP` gives the DDP semantics over the flat
    gradient arena (rank-0 broadcast, per-forward BN statistics broadcast, bucketed RCCL
    all-reduce overlapped with the backward, `no_sync()` on non-final GA micro-steps — accelerate
    calls `model.no_sync()` exactly where it would call DDP's);
  * the optimizer is `optim.ArenaAdamW` (torch AdamW arithmetic, one fused launch per
    weight-decay segment; HF's scheduler drives its lr; checkpointed in torch's layout);
  * gradient clipping: the global norm comes from one fused reduction and the clip coefficient
    is applied inside the AdamW kernel;
  * `fp16=True` / `bf16=True` (the reference trains with fp16=True) select the engine's bf16
    compute with fp32 master weights; there is no autocast and no GradScaler (bf16 needs no
    loss scaling). Otherwise the engine computes in fp32.
"""
import copy
import gc
import os
import warnings

import torch
import torch.distributed as dist
from transformers import Trainer

from .engine import prioritize_step_stream
from .optim import ArenaAdamW
from .parallel import ArenaDDP


class AVSRTrainer(Trainer):
    def __init__(self, model=None, args=None, data_collator=None, valid_data_collator=None, train_dataset=None,
                 eval_dataset=None, processing_class=None, model_init=None, compute_loss_func=None,
                 compute_metrics=None, callbacks=None, optimizers=(None, None), optimizer_cls_and_kwargs=None,
                 preprocess_logits_for_metrics=None):
        if model is None or not hasattr(model, "setup_engine"):
            raise TypeError("AVSRTrainer trains an avsr_amd AVHubertAVSR")
        # RCCL's internal streams at high priority like the step stream (parallel.init_from_env);
        # must be set before the process group exists, i.e. before args.device is first read
        if not dist.is_initialized():
            os.environ.setdefault("TORCH_NCCL_HIGH_PRIORITY", "1")
        elif dist.get_world_size() > 1 and os.environ.get("TORCH_NCCL_HIGH_PRIORITY") != "1":
            warnings.warn("process group created without TORCH_NCCL_HIGH_PRIORITY=1: gradient all-reduces "
                          "queue behind the high-priority step stream")
        args = copy.copy(args)
        self.engine_dtype = torch.bfloat16 if (args.fp16 or args.bf16) else torch.float32
        args.fp16 = args.bf16 = False          # precision is the engine's: no autocast / GradScaler
        optim = getattr(args, "optim", "adamw_torch")
        if not str(getattr(optim, "value", optim)).startswith("adamw"):
            raise NotImplementedError(f"optim={args.optim}: the arena optimizer implements AdamW")
        model.setup_engine(args.device, self.engine_dtype)
        prioritize_step_stream(args.device)   # data-grad chain ahead of the side stream's weight-grads
        kw = dict(model=model, args=args, data_collator=data_collator, train_dataset=train_dataset,
                  eval_dataset=eval_dataset, processing_class=processing_class, model_init=model_init,
                  compute_loss_func=compute_loss_func, compute_metrics=compute_metrics, callbacks=callbacks,
                  optimizers=optimizers, preprocess_logits_for_metrics=preprocess_logits_for_metrics)
        if optimizer_cls_and_kwargs is not None:
            kw["optimizer_cls_and_kwargs"] = optimizer_cls_and_kwargs
        super().__init__(**kw)
        self.valid_data_collator = valid_data_collator
        self.ddp = ArenaDDP(self.model, average=True)
        # keep accelerate from wrapping the engine model in DistributedDataParallel
        prepare_model = self.accelerator.prepare_model

        def _prepare_model(m, device_placement=None, evaluation_mode=False):
            if m is self.model:
                return m
            return prepare_model(m, device_placement=device_placement, evaluation_mode=evaluation_mode)

        self.accelerator.prepare_model = _prepare_model
        self._arena_opt = None

    def train(self, *args, **kwargs):
        """HF Trainer.train with the heap alive at its start in the collector's permanent
        generation for the duration of training (a full collection inside a step stalls the
        host for ~0.1 s, profiles/r02_gc_stall_ab.txt); unfrozen again when training ends."""
        gc.collect()
        gc.freeze()
        try:
            return super().train(*args, **kwargs)
        finally:
            gc.unfreeze()

    # ---------------------------------------------------------------- optimizer / clipping
    def create_optimizer(self, model=None):
        if self.optimizer is None:
            a = self.args
            self.optimizer = ArenaAdamW(self.model.avsr.engine().arena, lr=a.learning_rate,
                                        betas=(a.adam_beta1, a.adam_beta2), eps=a.adam_epsilon,
                                        weight_decay=a.weight_decay)
        self._arena_opt = self.optimizer if isinstance(self.optimizer, ArenaAdamW) else None
        return self.optimizer

    def _clip_grad_norm(self, model):
        if self._arena_opt is None:
            return super()._clip_grad_norm(model)
        return self._arena_opt.clip_grad_norm_(self.args.max_grad_norm)

    def _get_grad_norm(self, model, grad_norm=None):
        if grad_norm is None and self._arena_opt is not None:
            return self._arena_opt.grad_norm()
        return super()._get_grad_norm(model, grad_norm=grad_norm)

    # ---------------------------------------------------------------- evaluation collator
    def get_eval_dataloader(self, eval_dataset=None):
        """custom_trainer.py:43-102: evaluation batches use valid_data_collator"""
        if self.valid_data_collator is None:
            return super().get_eval_dataloader(eval_dataset)
        saved = self.data_collator
        self.data_collator = self.valid_data_collator
        try:
            return super().get_eval_dataloader(eval_dataset)
        finally:
            self.data_collator = saved
