"""Pipeline-parallel training/eval engine (1F1B).

Reference parity: runtime/pipe/engine.py ``PipelineEngine`` (:61-1426): ``train_batch`` :338,
``eval_batch`` :429, ``_exec_schedule`` :1409 with ``_INSTRUCTION_MAP`` :1396-1407, loss aggregation and
broadcast to all stages (:569), tied-gradient all-reduce (module.py:454), ZeRO <= 1 restriction.

Differences by design: the instruction stream comes from :mod:`.schedule` (per-stage 1F1B), adjacent
communication instructions are fused into one batched P2P group (:mod:`.p2p`), and gradient
reduction is the flat-shard ZeroOptimizer's: the last micro-batch's backward *holds* its bucket
reductions until the tied-weight gradients have been summed across stages, then releases them as one
burst of DP collectives.
"""
import torch

from ... import comm as dist
from ...utils.logging import log_dist
from ..engine import DeepSpeedEngine
from . import p2p
from . import schedule as S
from .module import PipelineModule


def _as_tuple(x):
    return tuple(x) if isinstance(x, (tuple, list)) else (x, )


class PipelineEngine(DeepSpeedEngine):
    _mb_index = 0

    def __init__(self, has_bool_tensors=False, *args, **kwargs):
        super().__init__(*args, **kwargs)
        assert isinstance(self.module, PipelineModule), "PipelineEngine requires a PipelineModule"
        assert self.zero_optimization_stage() < 2, "ZeRO-2 and ZeRO-3 are incompatible with pipeline parallelism"
        self.grid = self.module._grid
        self.num_stages = self.grid.get_pipe_parallel_world_size()
        self.stage_id = self.grid.get_stage_id()
        self.micro_batches = self.gradient_accumulation_steps()
        self.prev_rank = self.grid.stage_to_global(self.stage_id - 1) if self.stage_id > 0 else None
        self.next_rank = self.grid.stage_to_global(self.stage_id + 1) if self.stage_id < self.num_stages - 1 \
            else None
        self.has_bool_tensors = has_bool_tensors
        self.has_attention_mask = False
        self.data_iterator = None
        self.batch_fn = None
        self.pipe_buffers = {}
        self._send_meta_done = False
        self._recv_meta = None
        self.total_loss = None
        self.agg_train_loss = None
        self.agg_eval_loss = None
        self.agg_additional_losses = None
        self._additional_acc = {}
        self._eval_outputs = None
        self._compute_loss = True
        # tensor parallelism inside a stage: every model-parallel rank holds the same activation, so each sends only
        # its 1/mp slice to the next stage (and its slice of the input gradient back) and the receiver all-gathers
        # over the model-parallel group -- the p2p bytes per link drop by mp (reference engine.py:144-145,720-842)
        pcfg = self._config.pipeline or {}
        mp = self.grid.get_model_parallel_world_size()
        self.is_pipe_partitioned = mp > 1 and bool(pcfg.get("pipe_partitioned", True))
        self.is_grad_partitioned = self.is_pipe_partitioned and bool(pcfg.get("grad_partitioned", True))
        self._mp_group = self.grid.get_model_parallel_group() if mp > 1 else None
        self.p2p_bytes_sent = 0
        if self.num_stages > 1:
            self.module.sync_tied_weights()
            if self.optimizer is not None:
                self.optimizer.refresh_fp32_from_lp()
        log_dist(f"PipelineEngine: stages={self.num_stages} micro_batches={self.micro_batches} "
                 f"partition={self.module.parts}", ranks=[0])

    # ------------------------------------------------------------------------------------
    def is_first_stage(self):
        return self.stage_id == 0

    def is_last_stage(self):
        return self.stage_id == self.num_stages - 1

    def set_dataiterator(self, iterator):
        self.data_iterator = iterator

    def set_batch_fn(self, fn):
        self.batch_fn = fn

    # ---- reference PipelineEngine surface (runtime/pipe/engine.py) -----------------------------------------------
    def set_has_attention_mask(self, value):
        """The first stage's micro-batch inputs carry an attention mask as their last tensor (sent to the next stage
        with the activations: the p2p meta describes every tensor of the tuple, bool ones included)."""
        assert isinstance(value, bool)
        self.has_attention_mask = value

    def reset_activation_shape(self):
        """Forget the cached activation / gradient shapes so the next batch re-sends its meta (variable sequence
        length between batches). Every stage must call it before the same batch."""
        self._send_meta_done = False
        self._recv_meta = None
        self.pipe_buffers = {}

    def set_train_batch_size(self, train_batch_size):
        super().set_train_batch_size(train_batch_size)
        self.micro_batches = self.gradient_accumulation_steps()

    def set_dataloader(self, loader):
        """Data for the stages that read it (first: inputs, last: labels)."""
        if self.is_first_stage() or self.is_last_stage():
            self.training_dataloader = loader
            self.data_iterator = iter(loader)

    def log_for_device(self, *msg):
        """Print on the rank given by ``LOG_STAGE`` / ``DATA_PARALLEL_ID`` (env, default: stage 0, dp rank 0)."""
        import os
        stage = int(os.environ.get("LOG_STAGE", "0"))
        dp_id = int(os.environ.get("DATA_PARALLEL_ID", "0"))
        if self.stage_id == stage and self.grid.get_data_parallel_rank() == dp_id:
            print(f"RANK={dist.get_rank()} PIPE-ID={self.stage_id} DATA-ID={self.grid.get_data_parallel_rank()} "
                  f"MBATCH-ID={self._mb_index} STEP-ID={self.global_steps}", *msg, flush=True)

    def tput_log(self, *msg):
        if dist.get_rank() == 0 and self.global_steps % self.steps_per_print() == 0:
            print(*msg, flush=True)

    def mem_status(self, msg, print_rank=-1, reset_max=False):
        """Allocated / cached / peak device memory on this rank (``print_rank``: only that global rank)."""
        if print_rank >= 0 and dist.get_rank() != print_rank:
            return None
        if not torch.cuda.is_available():
            return None
        if reset_max:
            torch.cuda.reset_peak_memory_stats()
        g = 2**30
        rec = {"allocated_gib": torch.cuda.memory_allocated() / g, "reserved_gib": torch.cuda.memory_reserved() / g,
               "max_allocated_gib": torch.cuda.max_memory_allocated() / g}
        print(f"RANK={dist.get_rank()} STAGE={self.stage_id} STEP={self.global_steps} MEMSTATS {msg} "
              + " ".join(f"{k}={v:.2f}" for k, v in rec.items()), flush=True)
        return rec

    def load_module_state_dict(self, checkpoint, strict=True, custom_load_fn=None, fetch_z3_params=False):
        """A state dict (or ``{"module": ...}``) loads through the engine; a directory of layer files (the
        reference's layer-wise pipeline checkpoint, PipelineModule.save_state_dict) loads per stage."""
        import os
        if isinstance(checkpoint, str) and os.path.isdir(checkpoint):
            self.module.load_state_dir(checkpoint, strict=strict)
            if self.optimizer is not None:
                self.optimizer.refresh_fp32_from_lp()
            return
        super().load_module_state_dict(checkpoint, strict=strict, custom_load_fn=custom_load_fn,
                                       fetch_z3_params=fetch_z3_params)

    def get_additional_losses(self):
        """Extra named losses the last stage's loss function reported (a dict returned next to the loss), averaged
        over the micro-batches of the last batch; None if it reported none."""
        return getattr(self, "agg_additional_losses", None)

    def is_gradient_accumulation_boundary(self):
        return self._mb_index == self.micro_batches - 1

    def forward(self, *args, **kwargs):
        raise RuntimeError("PipelineEngine: use train_batch() / eval_batch() instead of forward()")

    def backward(self, *args, **kwargs):
        raise RuntimeError("PipelineEngine: use train_batch() instead of backward()")

    def step(self, *args, **kwargs):
        raise RuntimeError("PipelineEngine: use train_batch() instead of step()")

    # ------------------------------------------------------------------------------------
    def train_batch(self, data_iter=None):
        """One global batch = ``gradient_accumulation_steps`` micro-batches through the pipeline.
        Returns the mean loss over micro-batches (on every stage)."""
        if data_iter is not None:
            self.set_dataiterator(data_iter)
        self.module.train()
        self.total_loss = None
        self._additional_acc = {}
        self._compute_loss = True
        if getattr(self, "_ac_reset", False):
            from ..activation_checkpointing import checkpointing as _ac
            _ac.reset()  # every micro-batch of the previous batch has finished its backward
        sched = S.TrainSchedule(self.micro_batches, self.num_stages, self.stage_id)
        self._exec_schedule(sched)
        self.agg_train_loss = self._aggregate_loss(self.total_loss)
        self.agg_additional_losses = ({k: v / self.micro_batches for k, v in self._additional_acc.items()}
                                      if self._additional_acc else None)
        return self.agg_train_loss

    def eval_batch(self, data_iter, return_logits=False, compute_loss=True, reduce_output="avg", bcast_loss=True,
                   num_micro_batches=None):
        self.module.eval()
        self.set_dataiterator(data_iter)
        self.total_loss = None
        self._compute_loss = compute_loss
        self._eval_outputs = [] if return_logits else None
        mb = num_micro_batches or self.micro_batches
        with torch.no_grad():
            self._exec_schedule(S.InferenceSchedule(mb, self.num_stages, self.stage_id), train=False, n_micro=mb)
        out = None
        if compute_loss:
            out = self._aggregate_loss(self.total_loss, n_micro=mb, reduce_output=reduce_output,
                                       bcast=bcast_loss)
            self.agg_eval_loss = out
        self.module.train()
        if return_logits:
            return out, self._eval_outputs
        return out

    # ------------------------------------------------------------------------------------
    def _aggregate_loss(self, total, n_micro=None, reduce_output="avg", bcast=True):
        n_micro = n_micro or self.micro_batches
        dev = self.device
        if self.is_last_stage():
            loss = (total if total is not None else torch.zeros((), device=dev)).detach().float()
            if reduce_output == "avg":
                loss = loss / n_micro
            if self.dp_world_size > 1:
                dist.all_reduce(loss, group=self.dp_group)
                loss = loss / self.dp_world_size
        else:
            loss = torch.zeros((), dtype=torch.float32, device=dev)
        if bcast and self.num_stages > 1:
            src = self.grid.stage_to_global(self.num_stages - 1)
            loss = loss.reshape(1).contiguous()
            dist.broadcast(loss, src, group=self.grid.get_pipe_parallel_group())
            loss = loss.reshape(())
        return loss

    def _exec_schedule(self, sched, train=True, n_micro=None):
        self.pipe_buffers = {"inputs": {}, "labels": {}, "outputs": {}, "grads_in": {}}
        self._n_micro = n_micro or self.micro_batches
        self._train = train
        for step in sched.steps():
            comm = []
            for cmd in step:
                if isinstance(cmd, S.COMM_INSTRUCTIONS):
                    comm.append(cmd)
                    continue
                if comm:
                    self._exec_comm(comm)
                    comm = []
                self._INSTRUCTION_MAP[type(cmd)](self, cmd)
            if comm:
                self._exec_comm(comm)

    # ---- instructions -------------------------------------------------------------------
    def _next_batch(self):
        batch = next(self.data_iterator)
        if self.batch_fn is not None:
            batch = self.batch_fn(batch)
        return batch

    def _to_dev(self, x):
        if isinstance(x, torch.Tensor):
            return x.to(self.device, non_blocking=True)
        if isinstance(x, (tuple, list)):
            return type(x)(self._to_dev(t) for t in x)
        return x

    def _exec_load_micro_batch(self, cmd):
        batch = self._next_batch()
        inputs, labels = (batch[0], batch[1]) if isinstance(batch, (tuple, list)) and len(batch) == 2 else (batch,
                                                                                                          None)
        if self.is_first_stage():
            self.pipe_buffers["inputs"][cmd.buffer_id] = self._to_dev(inputs)
        if self.is_last_stage():
            self.pipe_buffers["labels"][cmd.buffer_id] = self._to_dev(labels)

    def _exec_forward_pass(self, cmd):
        mb = cmd.buffer_id
        self._mb_index = mb
        x = self.pipe_buffers["inputs"][mb]
        if self.optimizer is not None:
            self.optimizer.pre_forward()
        out = self.module(x)
        if self.optimizer is not None:
            self.optimizer.post_forward()
        if self.is_last_stage():
            labels = self.pipe_buffers["labels"].pop(mb, None)
            if self._compute_loss and self.module.loss_fn is not None:
                loss = self.module.loss_fn(out, labels)
                if isinstance(loss, (tuple, list)) and len(loss) == 2 and isinstance(loss[1], dict):
                    loss, extra = loss  # (loss, {name: additional loss}) -> get_additional_losses()
                    acc = self._additional_acc
                    for k, v in extra.items():
                        v = v.detach().float() if torch.is_tensor(v) else torch.tensor(float(v))
                        acc[k] = v if k not in acc else acc[k] + v
            else:
                loss = out
            if self._eval_outputs is not None:
                self._eval_outputs.append(out.detach() if isinstance(out, torch.Tensor) else out)
            if isinstance(loss, torch.Tensor) and loss.dim() == 0:
                d = loss.detach()
                self.total_loss = d.clone() if self.total_loss is None else self.total_loss + d
            self.pipe_buffers["outputs"][mb] = loss
        else:
            self.pipe_buffers["outputs"][mb] = out
        if not self._train:
            self.pipe_buffers["inputs"].pop(mb, None)

    def _exec_backward_pass(self, cmd):
        mb = cmd.buffer_id
        self._mb_index = mb
        boundary = mb == self._n_micro - 1
        zopt = self.optimizer
        zopt.prepare_backward(boundary)
        zopt.hold_reduction = boundary and self.num_stages > 1 and bool(self.module._tied_groups)
        out = self.pipe_buffers["outputs"].pop(mb)
        if self.is_last_stage():
            loss = out / self.micro_batches
            zopt.backward(loss)
        else:
            outs = [t for t in _as_tuple(out) if isinstance(t, torch.Tensor) and t.requires_grad]
            grads = self.pipe_buffers["grads_in"].pop(mb)  # already carry the loss scale of the next stage
            torch.autograd.backward(outs, grad_tensors=list(grads[:len(outs)]))
        zopt.finish_backward()
        x = self.pipe_buffers["inputs"].pop(mb, None)
        if not self.is_first_stage():
            self.pipe_buffers["grads_out"] = self.pipe_buffers.get("grads_out", {})
            self.pipe_buffers["grads_out"][mb] = [t.grad if t.grad is not None else torch.zeros_like(t)
                                                  for t in _as_tuple(x) if isinstance(t, torch.Tensor) and
                                                  t.is_floating_point()]

    def _exec_reduce_tied_grads(self, cmd):
        self.module.allreduce_tied_weight_gradients()

    def _exec_reduce_grads(self, cmd):
        zopt = self.optimizer
        if zopt._held:
            zopt.release_held_reductions()
        zopt.hold_reduction = False

    def _exec_optimizer_step(self, cmd):
        ok = self.optimizer.step()
        if ok is False:
            self.skipped_steps += 1
        elif self.lr_scheduler is not None:
            self.lr_scheduler.step()
        self.global_steps += 1
        self.global_samples += self.train_batch_size()
        self.micro_steps += self.micro_batches

    # ---- communication ------------------------------------------------------------------
    def _slice(self, t):
        """This model-parallel rank's 1/mp of ``t`` (flat, zero-padded to a multiple of mp)."""
        mp, r = dist.get_world_size(self._mp_group), dist.get_rank(self._mp_group)
        flat = t.detach().reshape(-1)
        n = -(-flat.numel() // mp)
        part = flat.new_zeros(n)
        lo, hi = min(r * n, flat.numel()), min((r + 1) * n, flat.numel())
        part[:hi - lo] = flat[lo:hi]
        return part

    def _part_buf(self, shape, dtype):
        mp = dist.get_world_size(self._mp_group)
        numel = 1
        for d in shape:
            numel *= d
        return torch.empty(-(-numel // mp), dtype=dtype, device=self.device)

    def _gather_full(self, part, shape):
        mp = dist.get_world_size(self._mp_group)
        full = part.new_empty(part.numel() * mp)
        dist.all_gather_into_tensor(full, part, group=self._mp_group)
        numel = 1
        for d in shape:
            numel *= d
        return full[:numel].view(shape)

    @staticmethod
    def _first_float(ts):
        return next((i for i, t in enumerate(ts) if t.is_floating_point()), None)

    def _exec_comm(self, cmds):
        ops, posts = [], []
        for cmd in cmds:
            mb = cmd.buffer_id
            if isinstance(cmd, S.SendActivation):
                out = self.pipe_buffers["outputs"][mb] if self._train else self.pipe_buffers["outputs"].pop(mb)
                ts = [t for t in _as_tuple(out) if isinstance(t, torch.Tensor)]
                if not self._send_meta_done:
                    p2p.send_meta(ts, self.next_rank, self.device)
                    self._send_meta_done = True
                send = [t.detach() for t in ts]
                i0 = self._first_float(send) if self.is_pipe_partitioned else None
                if i0 is not None:
                    send[i0] = self._slice(send[i0])
                ops += [("send", t, self.next_rank) for t in send]
            elif isinstance(cmd, S.RecvActivation):
                if self._recv_meta is None:
                    self._recv_meta = p2p.recv_meta(self.prev_rank, self.device)
                bufs = p2p.alloc_from_meta(self._recv_meta, self.device)
                i0 = self._first_float(bufs) if self.is_pipe_partitioned else None
                if i0 is not None:
                    bufs[i0] = self._part_buf(self._recv_meta[i0][2], self._recv_meta[i0][0])
                ops += [("recv", t, self.prev_rank) for t in bufs]

                def post(mb=mb, bufs=bufs, i0=i0):
                    xs = []
                    for i, (t, (_, grad, shape)) in enumerate(zip(bufs, self._recv_meta)):
                        if i == i0:
                            t = self._gather_full(t, shape)
                        if t.is_floating_point() and self._train:
                            t.requires_grad_(True)
                        xs.append(t)
                    self.pipe_buffers["inputs"][mb] = xs[0] if len(xs) == 1 else tuple(xs)

                posts.append(post)
            elif isinstance(cmd, S.SendGrad):
                gs = list(self.pipe_buffers["grads_out"].pop(mb))
                if self.is_grad_partitioned and gs:
                    gs[0] = self._slice(gs[0])
                ops += [("send", g, self.prev_rank) for g in gs]
            elif isinstance(cmd, S.RecvGrad):
                out = self.pipe_buffers["outputs"][mb]
                ts = [t for t in _as_tuple(out) if isinstance(t, torch.Tensor) and t.is_floating_point()]
                bufs = [torch.empty_like(t) for t in ts]
                if self.is_grad_partitioned and bufs:
                    bufs[0] = self._part_buf(ts[0].shape, ts[0].dtype)

                    def post(mb=mb, bufs=bufs, shape=ts[0].shape):
                        bufs[0] = self._gather_full(bufs[0], shape)

                    posts.append(post)
                ops += [("recv", g, self.next_rank) for g in bufs]
                self.pipe_buffers["grads_in"][mb] = bufs
        self.p2p_bytes_sent += sum(t.numel() * t.element_size() for kind, t, _ in ops if kind == "send")
        p2p.batch_p2p(ops)
        for post in posts:
            post()

    _INSTRUCTION_MAP = {
        S.OptimizerStep: _exec_optimizer_step,
        S.ReduceGrads: _exec_reduce_grads,
        S.ReduceTiedGrads: _exec_reduce_tied_grads,
        S.LoadMicroBatch: _exec_load_micro_batch,
        S.ForwardPass: _exec_forward_pass,
        S.BackwardPass: _exec_backward_pass,
    }
