"""Trainer: data-parallel bf16 pretraining loop on the gfx950 kernels.

Reference: scripts/train_transformer.py:35-109 (``Trainer``: LR warmup 10 % then
constant, bf16 autocast, GradScaler, DDP with an every-other-step sync toggle,
rank-0-only eval through the DDP wrapper, end-of-run save).

Same semantics where they were intended, fixed where they were defects
(SURVEY.md §8):
* LR: linear warmup over ``warmup_frac`` (0.1) of ``t_train_steps`` then
  constant (``lr_schedule='ref'``); ``'step'`` uses the reference's unused
  ``t_lr_decay_step``/``t_lr_decayed`` keys; ``'cosine'`` decays to ``t_lr_decayed``;
* gradient accumulation syncs once per optimizer step, never skips a sync (D5);
* evaluation runs on ALL ranks on their own shard and the loss is all-reduced (D11);
* logged train loss is the all-reduced mean over the log window (D16);
* periodic atomic checkpoints + resume (model, optimizer incl. fp32 master,
  step, data position, RNG); unwrapped keys (D7), directories created (D8);
* NaN/inf loss guard; tokens/s and MFU in every log line.
"""
from __future__ import annotations

import contextlib
import math
import os
import time
from typing import Optional

import torch
import torch.distributed as dist

from .. import ops
from ..data import TokenLoader, ensure_synthetic_shard
from ..models import GPT, ModelConfig, get_preset
from ..parallel.dp import DataParallelEngine, all_reduce_mean
from ..parallel.model_parallel import (build_dense_shell, gather_dense_state, init_parallel_groups,
                                       parallelize_gpt, sync_replicated_grads)
from ..utils.checkpoint import load_checkpoint, save_checkpoint
from .amp import DynamicLossScaler, autocast_ctx, loss_scaling_default, precision_mode
from ..utils.dist import DistInfo, apply_rccl_env, init_distributed, parse_env_list
from ..utils.metrics import MetricsLogger, mfu, peak_memory_gb
from .optim import FlatAdamW, no_decay_1d


def model_config_from(cfg: dict) -> ModelConfig:
    preset = cfg.get("model_preset")
    dims = {k: cfg[k] for k in ("vocab_size", "context_length", "n_embed", "n_head", "n_blocks") if k in cfg}
    extra = {k: cfg[k] for k in ("n_kv_head", "ffn_hidden", "activation_checkpointing") if cfg.get(k) is not None}
    if preset:
        mc = get_preset(preset)
        over = {k: v for k, v in {**dims, **extra}.items() if cfg.get("override_preset_dims", False) or k in extra}
        return mc.replace(**over) if over else mc
    from ..models.config import _ref
    return _ref(**dims, **extra)


def lr_at(step: int, cfg: dict) -> float:
    total = cfg["t_train_steps"]
    lr = cfg["t_lr"]
    warm = cfg.get("warmup_steps")
    if warm is None:
        warm = total * cfg.get("warmup_frac", 0.1)
    if warm > 0 and step < warm:
        return lr * step / warm
    sched = cfg.get("lr_schedule", "ref")
    if sched == "step":
        return cfg.get("t_lr_decayed", lr) if step >= cfg.get("t_lr_decay_step", total) else lr
    if sched == "cosine":
        lo = cfg.get("t_lr_decayed", 0.1 * lr)
        frac = min(1.0, (step - warm) / max(1.0, total - warm))
        return lo + 0.5 * (lr - lo) * (1 + math.cos(math.pi * frac))
    return lr


class Trainer:
    def __init__(self, cfg: dict, dist_info: Optional[DistInfo] = None, log=print):
        self.cfg = dict(cfg)
        self.log = log
        if dist_info is None:  # RCCL's environment must be in place before the communicator exists
            apply_rccl_env(self.cfg.get("rccl_channels"), parse_env_list(self.cfg.get("rccl_env")))
        self.di = dist_info or init_distributed(self.cfg.get("ddp_backend", "auto"), self.cfg.get("device", "auto"))
        self.device = self.di.device
        seed = int(self.cfg.get("seed", 1337))
        torch.manual_seed(seed)  # identical init on every rank (then broadcast for certainty)
        from ..utils import memory as _mem
        det = bool(self.cfg.get("deterministic", False))
        # workspace budgets (CE chunk rows, attention dQ slabs) decided once, not per call from the
        # free HBM; deterministic: pinned to their fixed caps (utils/memory.py)
        _mem.freeze_budgets(pin_caps=det)
        if det:
            # every hand-written kernel already reduces in a fixed order (attention dQ slabs,
            # split-K wgrad slabs, sorted embedding backward); this pins torch's own ops too
            torch.use_deterministic_algorithms(True, warn_only=True)
        self.mcfg = model_config_from(self.cfg)
        self.seq_len = int(self.cfg.get("seq_len") or self.mcfg.context_length)
        # precision (train/amp.py): bf16 on the HIP kernels; float16 = the reference's bf16 compute
        # + dynamic loss scaling; float16_autocast = fp32 weights + fp16 autocast + loss scaling
        # (opt-in, torch ops); float32 = fp32 through torch
        dtype_name = self.cfg.get("dtype", "bfloat16")
        self.dtype, self.autocast_dtype = precision_mode(dtype_name, self.device, bool(self.cfg.get("cpu_bf16", False)))
        ls = self.cfg.get("loss_scaling")
        self.scaler = DynamicLossScaler(init_scale=float(self.cfg.get("loss_scale_init", 2.0 ** 16)),
                                        growth_interval=int(self.cfg.get("loss_scale_growth_interval", 2000)),
                                        enabled=loss_scaling_default(dtype_name) if ls is None else bool(ls))
        self.tuned_gemms = False
        if self.device.type == "cuda":
            # CUs the persistent fused-epilogue GEMM grid leaves to RCCL kernels (world > 1); 0 = all;
            # persistent grids at world 1 only (train/graph.py gemm_persistent_policy)
            from .graph import gemm_persistent_policy
            ops.gemm_config(reserve_cus=int(self.cfg.get("gemm_reserve_cus", 0)),
                            persistent=gemm_persistent_policy(self.di.world_size, self.cfg.get("gemm_persistent", "auto")))
        if self.device.type == "cuda" and self.cfg.get("tuned_gemms", True):
            # the shipped TunableOp GEMM selections (pretraining_llm_amd/tuning/), as bench.py uses them
            from ..utils.gemm_tuning import enable_tuned_gemms
            self.tuned_gemms = enable_tuned_gemms(self.device.index or 0)
        # model parallelism (parallel/model_parallel.py): a dp x cp x tp mesh; the model is built
        # dense from the shared seed, then sharded, so every layout starts from the same weights.
        # Sharded layouts build and slice the dense model in HOST memory and move only this
        # rank's shards to the GPU: no rank ever holds the dense model in HBM (the point of TP
        # is models that do not fit one device)
        tp, cp = int(self.cfg.get("tp_size", 1)), int(self.cfg.get("cp_size", 1))
        self.pg = init_parallel_groups(tp, cp, bool(self.cfg.get("sequence_parallel", False)),
                                       self.cfg.get("cp_mode", "ring"))
        if self.pg.model_parallel:
            self.model = GPT(self.mcfg)
            parallelize_gpt(self.model, self.pg)
            self.model = self.model.to(device=self.device, dtype=self.dtype)
        else:
            self.model = GPT(self.mcfg).to(device=self.device, dtype=self.dtype)
        decay_filter = None if self.cfg.get("weight_decay_all", True) else no_decay_1d
        okw = dict(lr=self.cfg["t_lr"], betas=tuple(self.cfg.get("betas", (0.9, 0.999))),
                   eps=self.cfg.get("eps", 1e-8), weight_decay=self.cfg.get("weight_decay", 0.01),
                   decay_filter=decay_filter, max_grad_norm=self.cfg.get("max_grad_norm", 0.0))
        bkw = dict(bucket_mb=self.cfg.get("bucket_mb", 64.0), first_bucket_mb=self.cfg.get("first_bucket_mb", 4.0))
        if int(self.cfg.get("zero_stage", 0)) >= 1:
            # ZeRO-1: fp32 master + moments sharded over the DP ranks (parallel/zero.py)
            from ..parallel.zero import ShardedFlatAdamW, ZeroDataParallelEngine
            self.opt = ShardedFlatAdamW(self.model, process_group=self.pg.grad_group, **okw, **bkw)
            self.engine = ZeroDataParallelEngine(self.opt)
        else:
            self.opt = FlatAdamW(self.model, **okw)
            # gradients are averaged over the ranks that hold the same shard: dp x cp
            self.engine = DataParallelEngine(self.opt, process_group=self.pg.grad_group, **bkw)
        if self.pg.tp > 1:
            self.opt.set_tensor_parallel(self.pg.tp_group, self.pg.tp)  # global grad norm over TP shards
        self.accum = int(self.cfg.get("grad_accum_steps", 1))
        self.step = 0
        # TORCH_COMPILE (reference: torch.compile(model) unless the env var is "0", default "1",
        # scripts/train_transformer.py:31-33,118-120).  The hot ops here are hand-written kernels, so
        # what a compiler would still remove is per-launch host cost: on the GPU the whole step
        # (every micro-step's fwd + bwd, bucketed all-reduce, clip, AdamW, zero_grad) is captured
        # once as a hipGraph and replayed (train/graph.py) -- on by default, like the reference's
        # compile.  On the CPU (tests, plumbing) the default is eager; TORCH_COMPILE=1 there runs
        # torch.compile.
        comp = self.cfg.get("compile")
        if comp is None:
            env = os.environ.get("TORCH_COMPILE")
            comp = (env == "1") if env is not None else self.device.type == "cuda"
        self.compile = bool(comp)
        self.gstep = None
        self.use_graph = False
        self.fwd = self.model
        if self.compile:
            # the same policy bench.py applies (train/graph.py): at world > 1 the eager step with
            # hook-launched RCCL buckets (graph_collectives is refused); on the CPU torch.compile
            from . import graph as _graph
            ok, why = _graph.graph_step_policy(
                cuda=self.device.type == "cuda", world=self.di.world_size,
                dist_backend=dist.get_backend() if dist.is_initialized() else None,
                zero=int(self.cfg.get("zero_stage", 0)) >= 1, model_parallel=self.pg.model_parallel,
                loss_scaling=self.scaler.enabled, bf16=self.dtype == torch.bfloat16, hip_ops=self._hip_step_ok(),
                graph_collectives=bool(self.cfg.get("graph_collectives", False)))
            if ok:
                self.use_graph = True
                if self.di.is_master:
                    self.log(f"TORCH_COMPILE: whole training step captured as a hipGraph (grad_accum_steps={self.accum})")
            elif self.device.type != "cuda":
                self.fwd = torch.compile(self.model, backend=self.cfg.get("compile_backend", "inductor"))
            elif self.di.is_master:
                self.log(f"TORCH_COMPILE: hipGraph step disabled for this configuration ({why}); running eagerly")
        self.step_mode = "graph" if self.use_graph else "eager"
        self.metrics = MetricsLogger(self.cfg.get("metrics_path"), enabled=self.di.is_master)
        self.train_loader = self._loader(self.cfg["train_path"], seed, 0)
        vp = self.cfg.get("val_path") or self.cfg.get("dev_path")
        self.val_loader = self._loader(vp, seed + 1, 0, stream=1) if vp else None
        self.flops_per_token = self.mcfg.flops_per_token(self.seq_len)
        if self.cfg.get("resume"):
            self.resume(self.cfg["resume"])

    # ------------------------------------------------------------------
    def _loader(self, path: str, seed: int, start: int, stream: int = 0):
        if self.cfg.get("synthetic_data", False) or not os.path.exists(path):
            if not self.cfg.get("synthetic_data", False) and not self.cfg.get("allow_synthetic", True):
                raise FileNotFoundError(path)
            n = int(self.cfg.get("synthetic_tokens", 2_000_000))
            syn = self.cfg.get("synthetic_dir", "data/synthetic")
            kind = self.cfg.get("synthetic_kind", "auto")
            path = os.path.join(syn, f"{os.path.basename(path) or 'tokens'}.{self.mcfg.vocab_size}.{n}"
                                     f"{'' if kind == 'auto' else '.' + kind}.bin")
            kind = self.cfg.get("synthetic_kind", "auto")  # auto | markov | fast (data/shards.py)
            if self.di.is_master:
                ensure_synthetic_shard(path, n, self.mcfg.vocab_size, seed=int(self.cfg.get("seed", 1337)),
                                       stream=stream, fast=None if kind == "auto" else kind == "fast")
            if dist.is_initialized():
                dist.barrier()
        # every rank of a TP / CP group reads the same batch: shard the data over dp only
        return TokenLoader(path, self.cfg["t_batch_size"], self.seq_len, self.pg.dp_rank,
                           self.pg.dp, seed=seed, start_batch=start, device=self.device)

    def lr(self, step: int) -> float:
        return lr_at(step, self.cfg)

    # ------------------------------------------------------------------
    def train_step(self) -> torch.Tensor:
        """One optimizer step (``grad_accum_steps`` micro-batches). Returns the mean loss (device tensor)."""
        lr = self.lr(self.step)
        if self.use_graph and self.gstep is None and self.device.type == "cuda" and not self._hip_step_ok():
            self.use_graph = False  # the op backend was switched to torch after construction
        if self.use_graph:
            return self._graph_step(lr)
        self.opt.param_groups[0]["lr"] = lr
        total = torch.zeros((), device=self.device, dtype=torch.float32)
        for micro in range(self.accum):
            x, y = self.train_loader.next()
            ctx = self.engine.no_sync() if micro < self.accum - 1 else contextlib.nullcontext()
            with ctx:
                with autocast_ctx(self.device, self.autocast_dtype):
                    _, loss = self.fwd(x, y, return_logits=False)
                self.scaler.scale_loss(loss).backward()
            total += loss.detach().float()
        scale = self.engine.finish_grad_sync()
        if self.pg.sequence_parallel:
            # each TP rank's loss is the mean over its T/tp tokens: replicated parameters hold
            # partial gradients (summed over the TP group here) and every gradient is tp x the
            # gradient of the global mean
            sync_replicated_grads(self.opt, self.pg)
            scale /= self.pg.tp
        if self.scaler.enabled:
            # GradScaler.step/update: an inf/nan gradient skips the optimizer step and backs the
            # scale off; otherwise the unscale rides on the AdamW kernel's grad_scale
            used = self.scaler.scale  # the scale this step's backward ran with
            inf = self.scaler.found_inf(self.opt)
            self.scaler.update(inf)
            if inf:
                self.opt.zero_grad()
                self.step += 1
                return total / self.accum
            scale /= used
        self.opt.step(grad_scale=scale / self.accum)
        self.opt.zero_grad()
        self.step += 1
        return total / self.accum

    def _hip_step_ok(self) -> bool:
        """The captured step replays the HIP kernels, AdamW included."""
        return bool(getattr(self.opt, "use_hip", False)) and ops.get_backend() == "auto"

    def _graph_step(self, lr: float) -> torch.Tensor:
        """hipGraph-replayed step.  The first call runs one real (eager, side-stream) step on its
        batch -- it also teaches the DP engine its bucket order -- then captures the step; every
        later call copies its micro-batches into the static inputs and replays."""
        from . import graph as _graph
        batches = [self.train_loader.next() for _ in range(self.accum)]
        x = torch.stack([b[0] for b in batches])
        y = torch.stack([b[1] for b in batches])
        self.step += 1
        if self.gstep is None:
            _, B, T = x.shape
            self.gstep = _graph.GraphedTrainStep(self.model, self.opt, self.engine, B, T, self.device, warmup=1,
                                                 accum=self.accum)
            self.gstep.capture(x, y, lr)
            return self.gstep.warmup_loss
        return self.gstep(x, y, lr).clone()

    @torch.no_grad()
    def evaluate(self, iters: Optional[int] = None) -> float:
        if self.val_loader is None:
            return float("nan")
        iters = iters or int(self.cfg.get("t_eval_iters", 250))
        self.model.eval()
        acc = torch.zeros((), device=self.device, dtype=torch.float32)
        for _ in range(iters):
            x, y = self.val_loader.next()
            with autocast_ctx(self.device, self.autocast_dtype):
                _, loss = self.fwd(x, y, return_logits=False)
            acc += loss.float()
        self.model.train()
        return float(all_reduce_mean(acc / iters))

    def train(self, steps: Optional[int] = None):
        cfg = self.cfg
        total = steps if steps is not None else cfg["t_train_steps"]
        log_every = int(cfg.get("log_interval", cfg.get("t_eval_steps", 1000)))
        eval_every = int(cfg.get("t_eval_steps", 1000))
        ckpt_every = int(cfg.get("ckpt_interval", 0))
        tokens_per_step = cfg["t_batch_size"] * self.seq_len * self.accum * self.di.world_size
        self.model.train()
        window_loss = torch.zeros((), device=self.device)
        window_n = 0
        t0 = time.perf_counter()
        window_steps = 0
        last_val = float("nan")
        prof = self._profiler()
        while self.step < total:
            step = self.step
            if prof is not None:
                prof.step()
            do_eval = self.val_loader is not None and eval_every > 0 and step % eval_every == 0 and (
                step > 0 or cfg.get("eval_at_start", True))
            if do_eval:
                last_val = self.evaluate()
            loss = self.train_step()
            window_loss += loss
            window_n += 1
            window_steps += 1
            if (step % log_every == 0) or self.step == total:
                if self.device.type == "cuda":
                    torch.cuda.synchronize(self.device)
                dt = time.perf_counter() - t0
                tl = float(all_reduce_mean(window_loss / max(1, window_n)))
                if not math.isfinite(tl):
                    raise FloatingPointError(f"non-finite training loss {tl} at step {step}")
                tps = tokens_per_step * window_steps / max(dt, 1e-9)
                rec = {"step": step, "train_loss": tl, "val_loss": last_val, "lr": self.opt.lr,
                       "step_ms": 1000 * dt / max(1, window_steps), "tokens_per_s": tps,
                       "tokens_per_s_per_gpu": tps / self.di.world_size,
                       "mfu": mfu(tps / self.di.world_size, self.flops_per_token),
                       "peak_mem_gb": peak_memory_gb(self.device)}
                if self.opt.last_grad_norm is not None:
                    rec["grad_norm"] = float(self.opt.last_grad_norm)
                if self.di.is_master:
                    self.log(f"Step {step}: Train Loss={tl:.4f}, Val Loss={last_val:.4f}, LR={self.opt.lr:.2e}, "
                             f"Time={dt * 1000:.2f}ms, tok/s={tps:,.0f}, MFU={rec['mfu'] * 100:.1f}%")
                self.metrics.log(rec)
                window_loss.zero_()
                window_n = 0
                window_steps = 0
                t0 = time.perf_counter()
            if ckpt_every and self.step % ckpt_every == 0 and self.step < total:
                self.save(self._ckpt_path(periodic=True))
        if prof is not None:
            self._finish_profile(prof)
        self.opt.wait_params()  # ZeRO-1: the last step's weight all-gathers
        out = cfg.get("t_out_path")
        if out:
            self.save(out)
        return self

    # ------------------------------------------------------------------
    def _profiler(self):
        """torch.profiler over optimizer steps [start, end) of ``profile_steps`` with ROCm
        (HIP) activity: per-rank chrome trace + a kernel-time table.
        Kernel-level counters come from ``rocprofv3`` (scripts/gpu/prof.sh, profiles/)."""
        d = self.cfg.get("profile_dir")
        if not d:
            return None
        a, b = (int(x) for x in str(self.cfg.get("profile_steps", "3:6")).split(":"))
        acts = [torch.profiler.ProfilerActivity.CPU]
        if self.device.type == "cuda":
            acts.append(torch.profiler.ProfilerActivity.CUDA)
        os.makedirs(d, exist_ok=True)
        prof = torch.profiler.profile(activities=acts, schedule=torch.profiler.schedule(
            wait=max(0, a - 1), warmup=1 if a > 0 else 0, active=max(1, b - a), repeat=1), record_shapes=False)
        prof.start()
        return prof

    def _finish_profile(self, prof):
        prof.stop()
        d = self.cfg["profile_dir"]
        path = os.path.join(d, f"trace_rank{self.di.rank}.json")
        prof.export_chrome_trace(path)
        key = "self_cuda_time_total" if self.device.type == "cuda" else "self_cpu_time_total"
        table = prof.key_averages().table(sort_by=key, row_limit=25)
        with open(os.path.join(d, f"kernels_rank{self.di.rank}.txt"), "w") as f:
            f.write(table)
        if self.di.is_master:
            self.log(f"profile written to {path}")

    # ------------------------------------------------------------------
    def _ckpt_path(self, periodic=False):
        out = self.cfg.get("t_out_path", "models/transformer_B.pt")
        if not periodic:
            return out
        root, ext = os.path.splitext(out)
        return f"{root}.latest{ext or '.pt'}"

    def save(self, path: str):
        data_state = {"train_batches": self.train_loader.batches_consumed,
                      "val_batches": self.val_loader.batches_consumed if self.val_loader else 0}
        if self.pg.tp > 1:
            return self._save_tp(path, data_state)
        # a sharded optimizer consolidates its state collectively (every rank), rank 0 writes it
        osd = self.opt.state_dict() if getattr(self.opt, "collective_state", False) else None
        if self.di.is_master:
            save_checkpoint(path, self.model, self.opt if osd is None else None, step=self.step, config=self.cfg,
                            data_state=data_state, optimizer_state=osd, params=self.opt.params,
                            extra=self._scaler_extra())
            self.log(f"saved checkpoint to {path} (step {self.step})")
        if dist.is_initialized():
            dist.barrier()

    def _scaler_extra(self) -> dict:
        # reference key name for a GradScaler's state; only written when loss scaling is on
        return {"scaler_state_dict": self.scaler.state_dict()} if self.scaler.enabled else {}

    def _save_tp(self, path: str, data_state: dict):
        """Tensor parallelism: each TP rank of replica (dp 0, cp 0) writes its shard with its optimizer
        state to ``path.tp{r}`` (what ``resume`` reads back), and global rank 0 writes the
        consolidated dense fp32 checkpoint in the reference format to ``path`` (generate_text.py
        loads it as usual).  Collective over the TP group of that replica."""
        pg = self.pg
        osd = self.opt.state_dict()  # collective for ZeRO (over the dp x cp group)
        writer = pg.dp_rank == 0 and pg.cp_rank == 0
        if writer:
            save_checkpoint(f"{path}.tp{pg.tp_rank}", self.model, optimizer_state=osd, params=self.opt.params,
                            step=self.step, config=self.cfg, data_state=data_state,
                            extra={"tp_rank": pg.tp_rank, "tp_size": pg.tp, **self._scaler_extra()})
            # fp32 masters in the consolidated file on both optimizer paths: FlatAdamW's own
            # buffer, or (ZeRO) the consolidated state the writer ranks just gathered
            if getattr(self.opt, "collective_state", False):
                st = osd.get("state", {})
                masters = {id(p): st[i]["master"].reshape(p.shape) for i, p in enumerate(self.opt.params)
                           if i in st and "master" in st[i]}
            else:
                masters = {id(p): self.opt.master[self.opt.offsets[i]:self.opt.offsets[i] + p.numel()].view(p.shape)
                           for i, p in enumerate(self.opt.params)}
            # only global rank 0 materialises the dense model, in host memory, from no RNG draw
            # (parallel/model_parallel.py build_dense_shell); the other writers just contribute
            dense = build_dense_shell(self.mcfg) if self.di.is_master else None
            gather_dense_state(self.model, dense, pg, masters)
            if self.di.is_master:
                save_checkpoint(path, dense, step=self.step, config=self.cfg, data_state=data_state,
                                extra={"tp_size": pg.tp, "tp_shards": [f"{path}.tp{r}" for r in range(pg.tp)]})
                self.log(f"saved checkpoint to {path} (+{pg.tp} tensor-parallel shards, step {self.step})")
            del dense
        if dist.is_initialized():
            dist.barrier()

    def resume(self, path: str):
        if path == "auto":
            path = self._ckpt_path(periodic=True)
            if not os.path.exists(path):
                return
        if self.pg.tp > 1:
            path = f"{path}.tp{self.pg.tp_rank}"  # this rank's shard (and its optimizer state)
        ck = load_checkpoint(path, map_location="cpu")
        missing, unexpected = self.model.load_state_dict(ck["model_state_dict"], strict=False)
        missing = [k for k in missing if not k.endswith("pos_idxs")]
        if missing or unexpected:
            raise RuntimeError(f"checkpoint mismatch: missing={missing} unexpected={unexpected}")
        self.opt.sync_master_from_params()
        if "optimizer_state_dict" in ck:
            self.opt.load_state_dict(ck["optimizer_state_dict"])
        self.step = int(ck.get("step", 0))
        if "scaler_state_dict" in ck:
            self.scaler.load_state_dict(ck["scaler_state_dict"])
        ds = ck.get("data_state", {})
        seed = int(self.cfg.get("seed", 1337))
        self.train_loader.close()
        self.train_loader = self._loader(self.cfg["train_path"], seed, int(ds.get("train_batches", 0)))
        if self.val_loader is not None:
            vp = self.cfg.get("val_path") or self.cfg.get("dev_path")
            self.val_loader.close()
            self.val_loader = self._loader(vp, seed + 1, int(ds.get("val_batches", 0)), stream=1)
        if self.di.is_master:
            self.log(f"resumed from {path} at step {self.step}")
