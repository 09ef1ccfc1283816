"""SimCLR contrastive pre-training (the ``main`` entry point).

Reference: ``/root/reference/main.py:61-131,134-180`` (call stacks §3.1-3.2).  Per
step the reference does warmup LR → zero_grad → two DDP forwards (view0, view1) → NT-Xent →
backward (DDP bucket all-reduces, SyncBN collectives) → LARC.step → cosine step; once per epoch
rank 0 logs ``Epoch:{e}/{E} progress:{p:.3f} loss:{l:.3f}, lr:{lr:.7f}`` (last batch's loss) and
saves ``epoch={E}-{name}`` every ``save_model_epoch`` epochs.

MI355X step (``Trainer.step``), identical math:
  augment kernel (both views, on device) → ONE forward of the 2N batch with per-view BN
  statistics (``segments=2``) on the implicit-GEMM / fused-BN kernels → fused NT-Xent →
  backward with gradients written into the flat fp32 buffer and bucketed RCCL all-reduces on a
  comm stream → ``lr_step`` + fused LARS (no host sync anywhere in the step).
By default (``runtime.hip_graph=auto``) the HIP path runs its first ``GRAPH_AFTER`` steps
eagerly, then captures the whole step (fwd + bwd + optimizer, collectives included) once into a
hipGraph and replays it for every later batch — what bench.py measures — to remove per-kernel
launch overhead: by the native multi-stream executor over the captured nodes
(``runtime.replay=streams``, runtime/graph_exec.py) or by ``hipGraphLaunch``
(``runtime.replay=graph``).  ``runtime.hip_graph=false`` issues every step eagerly.
"""
from __future__ import annotations

import json
import logging
import math
import os
import time
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from ..comm.ipc import StepGuard
from ..config import check_pretrain_conf
from ..data.datasets import load_dataset
from ..data.loader import ContrastiveLoader
from ..loss.ntxent import NTXent
from ..models.contrastive import ContrastiveModel
from ..ops import registry
from ..optim.lars import FusedLARS, weight_decay_per_param
from ..optim.schedule import MODE_WARMUP_COSINE, calculate_initial_lr
from ..parallel.flat import FlatParamStore
from ..parallel.invariant import require_replicas
from ..runtime.dist import init_distributed
from ..utils.checkpoint import (checkpoint_name, gather_rng_states, load_resume,
                                save_reference_checkpoint, save_resume)
from ..utils.misc import cfg_get, seed_everything, MetricsWriter, refuse_experiment_knobs

log = logging.getLogger(__name__)


def build_contrastive_model(cfg, device, precision: str):
    model = ContrastiveModel(base_cnn=cfg["experiment"]["base_cnn"], d=cfg["parameter"]["d"],
                             cifar_stem=cfg_get(cfg, "model.cifar_stem", None),
                             stem_padding=cfg_get(cfg, "model.stem_padding", 3))
    model = model.to(device)
    shadow = torch.bfloat16 if (precision == "bf16" and device.type == "cuda") else None
    store = FlatParamStore(model, device, shadow_dtype=shadow,
                           bucket_mb=cfg_get(cfg, "runtime.bucket_mb", 32.0),
                           last_bucket_mb=cfg_get(cfg, "runtime.last_bucket_mb", 2.0))
    store.broadcast_from(0)
    return model, store


class Trainer:
    """Owns model, flat store, optimizer, loss and the (optionally graph-captured) step.

    ``guard`` (comm/ipc.py ``StepGuard``): RCCL statistics + rank-0 tuning table for the first
    eager steps, and the per-step check of the IPC exchange's error flag (``guard.on_error``:
    ``"raise"`` in training, ``"defer"`` in bench.py, which checks collectively)."""

    def __init__(self, cfg, st, dataset_len: int, precision: Optional[str] = None):
        self.cfg = cfg
        self.st = st
        self.device = st.device
        prec = precision or cfg_get(cfg, "runtime.precision", "bf16")
        self.precision = prec if self.device.type == "cuda" else "fp32"
        self.model, self.store = build_contrastive_model(cfg, self.device, self.precision)
        self.store.defer_side_join = True  # _step_body calls store.finish() before the optimizer
        batches = cfg["experiment"]["batches"]
        world = st.world_size
        # reference: int(num_samples / (batches * world)) (main.py:76)
        self.steps_per_epoch = max(1, int(dataset_len / (batches * world)))
        self.total_steps = cfg["parameter"]["epochs"] * self.steps_per_epoch
        self.warmup_steps = cfg["parameter"]["warmup_epochs"] * self.steps_per_epoch
        wds = weight_decay_per_param(self.store, cfg["experiment"]["decay"])
        self.opt = FusedLARS(self.store, wds, lr0=calculate_initial_lr(cfg),
                             momentum=cfg["parameter"]["momentum"], nesterov=False,
                             trust_coefficient=0.001, eps=1e-8, lars=True,
                             schedule_mode=MODE_WARMUP_COSINE, warmup_steps=self.warmup_steps,
                             total_steps=self.total_steps)
        self._early_updates()
        self.loss_fn = NTXent(temperature=cfg["parameter"]["temperature"],
                              gather=cfg_get(cfg, "loss.gather", False))
        # global negatives over RCCL: the fused head gathers z view by view under its GEMM 2
        # (models/head_fused.py _gemm2_pregather)
        zg = self.loss_fn.gather is True and bool(st.comm)
        for m in self.model.modules():
            if hasattr(m, "use_fused") and hasattr(m, "_seq"):
                m._zgather = zg
        self.hip = self.device.type == "cuda" and registry.use_hip(self.store.master) \
            and self.precision == "bf16"
        self.model.train()
        self.graph = None
        # how a captured step is issued: "graph" (hipGraphLaunch) or "streams" (the native
        # multi-stream executor over the same captured nodes, runtime/graph_exec.py)
        self.replay_mode = "graph"
        self.sreplay = None
        self._static_x = None
        self._static_loss = None
        self.guard = StepGuard(st)

    def _early_updates(self) -> None:
        """Single GPU: the fused executor issues the optimizer update of stages 4 (with the
        projection head), 3 and 2 as soon as their gradients are final (FusedLARS.early_step,
        models/fused.py backward).  With a data-parallel group the gradients are final only
        after their bucket's all-reduce, so the update stays in step()."""
        if (self.device.type != "cuda" or self.store.comm
                or os.environ.get("SIMCLR_EARLY_UPDATE", "1") == "0"):
            return
        groups: dict = {}
        for i, n in enumerate(self.store.names):
            parts = n.split(".")
            if parts[0] == "g":
                groups.setdefault(4, []).append(i)
            elif len(parts) > 1 and parts[1] in ("layer2", "layer3", "layer4"):
                groups.setdefault(int(parts[1][5]), []).append(i)
        backbone = getattr(self.model, "f", None)
        if not groups or backbone is None:
            return
        self.opt.set_early_groups(groups)
        backbone.stage_grads_ready = self.opt.early_step

    def prepare(self, x: torch.Tensor) -> torch.Tensor:
        if self.precision == "bf16" and self.device.type == "cuda":
            return x
        x = x.float()
        if x.shape[1] != 3:
            x = x[:, :3]
        return x.contiguous()

    def _step_body(self, x: torch.Tensor) -> torch.Tensor:
        z = self.model(x, segments=2)
        loss = self.loss_fn(z)
        if not self.hip:
            self.store.zero_grad()
        loss.backward()
        self.store.finish()
        self.opt.step()
        return loss.detach()

    def _eager(self, x: torch.Tensor) -> torch.Tensor:
        return self.guard.run(self._step_body, x)

    def step(self, x: torch.Tensor) -> torch.Tensor:
        x = self.prepare(x)
        if self.graph is not None:
            if x.data_ptr() != self._static_x.data_ptr():  # (the loader may write in place)
                self._static_x.copy_(x)
            if self.replay_mode == "streams" and self.sreplay is not None:
                self.sreplay.replay()
            else:
                self.graph.replay()
            self.opt.host_step += 1
            loss = self._static_loss
        else:
            loss = self._eager(x)
        self.guard.check(self.opt.host_step)
        return loss

    def capture(self, x: torch.Tensor, warmup: int = 2, streams: int = -1) -> None:
        """Capture one full training step into a hipGraph (after ``warmup`` eager steps) and
        build the native multi-stream executor over its nodes (``streams`` > 0; kept as
        ``self.sreplay``, selected by ``replay_mode = "streams"``)."""
        x = self.prepare(x)
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._eager(x)
        torch.cuda.current_stream(self.device).wait_stream(s)
        if self.st.comm:
            # the RCCL watchdog polls the end events of the eager warm-up collectives; HIP refuses
            # that query once their stream joins a capture ("event last recorded in a capturing
            # stream").  Let every eager work complete and be reaped (the watchdog polls every
            # ~100 ms) before the capture starts.
            torch.cuda.synchronize(self.device)
            time.sleep(1.0)
        self._static_x = x.clone()
        if self.device.type == "cuda":
            from ..ops import _ext
            if _ext.available():
                # the last-arriver reductions' persistent ticket arrays cannot be allocated
                # inside the capture (a capture with no eager warm-up step reaches them first)
                torch.ops.simclr_amd.bn_tickets_init(self._static_x)
        g = torch.cuda.CUDAGraph(keep_graph=True)
        # with collectives in the step, the RCCL watchdog thread polls work events while the
        # capture is open: thread-local capture mode keeps those queries legal
        mode = "thread_local" if self.st.comm else "global"
        with torch.cuda.graph(g, capture_error_mode=mode):
            self._static_loss = self._step_body(self._static_x)
        self.opt.host_step -= 1  # the captured body incremented it once; replays add per step
        g.instantiate()
        self.graph = g
        self.sreplay = None
        sched = None
        if self.st.comm:
            # with collectives: the capture-order plan, which keeps the gradient all-reduce
            # chain on a stream of its own (a list schedule planned from one timed replay could
            # queue chain kernels behind an all-reduce whose duration depends on the other
            # ranks); single GPU: the list schedule (runtime/graph_exec.py)
            sched = os.environ.get("SIMCLR_REPLAY_SCHED", "capture")
        if streams < 0:
            # N > 1: main chain, weight-gradient stream, downsample branch, all-reduce chain (at
            # most the 4 hardware queues a process gets, GPU_MAX_HW_QUEUES).  N = 1: the list
            # schedule over 2 streams (chain + one side stream) beat 3 by 0.09-0.26 ms (r5 log):
            # side work beyond one stream slows the chain more than it overlaps
            streams = 4 if self.st.comm else 2
        if streams > 0:
            from ..runtime.graph_exec import StreamReplay
            try:
                self.sreplay = StreamReplay(g, max_streams=streams, sched=sched)
            except RuntimeError as e:  # a node type the executor does not issue: graph only
                log.warning("multi-stream replay unavailable: %s", e)
                self.sreplay = None


def pretrain(cfg) -> dict:
    refuse_experiment_knobs("pretrain")
    st = init_distributed(cfg, use_cuda=cfg["parameter"].get("use_cuda", True))
    check_pretrain_conf(cfg)
    registry.set_backend(cfg_get(cfg, "runtime.backend", "auto"))
    seed = cfg["parameter"]["seed"]
    det = bool(cfg_get(cfg, "runtime.deterministic", False))
    seed_everything(seed, deterministic=det)
    if det:
        from ..ops import tuning
        tuning.set_enabled(False)
    if cfg_get(cfg, "runtime.debug", False):
        from ..ops import _ext
        _ext.set_debug(True)
    fault = parse_fault(cfg_get(cfg, "runtime.fault_inject", None)
                        or os.environ.get("SIMCLR_FAULT_INJECT"))
    prof_win = parse_window(cfg_get(cfg, "runtime.profile", None))
    prof = None
    rank = st.rank
    log.info("Using {}".format(st.device))
    ds = load_dataset(cfg["experiment"]["name"], train=True,
                      root=cfg_get(cfg, "data.root", "~/pytorch_datasets"),
                      synthetic=bool(cfg_get(cfg, "data.synthetic", False)),
                      synthetic_size=cfg_get(cfg, "data.synthetic_size", None),
                      synthetic_noise=float(cfg_get(cfg, "data.synthetic_noise", 25.0)),
                      synthetic_colour=bool(cfg_get(cfg, "data.synthetic_colour", True)),
                      synthetic_kind=str(cfg_get(cfg, "data.synthetic_kind", "template")),
                      allow_synthetic_fallback=bool(cfg_get(cfg, "data.synthetic_fallback", False)),
                      seed=seed)
    loader = ContrastiveLoader(ds, cfg["experiment"]["batches"], st.device, rank=rank,
                               world=st.world_size, strength=cfg["experiment"]["strength"],
                               seed=seed, views=2)
    loader.with_labels = False  # SimCLR pre-training uses no labels
    tr = Trainer(cfg, st, len(ds))
    epochs = cfg["parameter"]["epochs"]
    start_epoch = 1
    resume = cfg_get(cfg, "runtime.resume", None)
    if resume:
        blob = load_resume(resume, tr.model, tr.opt, tr.store)
        start_epoch = int(blob["epoch"]) + 1
        loader.counter = int(blob["step"])
    max_steps = cfg_get(cfg, "runtime.max_steps", None)
    log_every = int(cfg_get(cfg, "runtime.log_every", 0) or 0)  # progress lines (syncs the step)
    graph_mode = _graph_mode(cfg_get(cfg, "runtime.hip_graph", "auto"))
    # the captured step cannot hold host (gloo) collectives: a gloo rehearsal stays eager
    use_graph = (graph_mode != "off" and tr.hip
                 and (not st.comm or dist.get_backend(st.group) == "nccl"))
    metrics = MetricsWriter("metrics.jsonl" if rank == 0 else None)
    save_every = cfg["experiment"]["save_model_epoch"]
    step_global = tr.opt.host_step
    loss = torch.zeros(())
    summary = {"epochs_run": 0, "steps": 0}
    t_start = time.time()
    done = False
    for epoch in range(start_epoch, epochs + 1):
        loader.set_epoch(epoch)
        if st.device.type == "cuda":
            torch.cuda.synchronize()
        t0 = time.time()
        nsteps = 0
        for x, _ in loader:
            if fault is not None and fault[0] == rank and fault[1] == step_global:
                log.error("fault injection: rank %d exits with %d at step %d", rank, fault[2],
                          step_global)
                logging.shutdown()
                os._exit(fault[2])
            if prof_win is not None and step_global == prof_win[0] and prof is None:
                prof = _start_profiler()
            if use_graph and tr.graph is None and tr.guard.eager_steps >= GRAPH_AFTER:
                # the first GRAPH_AFTER steps ran eagerly (autotuning, plans, the IPC guard's
                # tuning steps); this batch's step is the captured one, so every batch is
                # trained exactly once, as in the eager loop
                try:
                    tr.capture(x, warmup=0)
                except Exception as e:
                    if graph_mode == "on":
                        raise
                    log.warning("hipGraph capture failed (%r): issuing every step eagerly", e)
                    tr.graph, tr.sreplay, use_graph = None, None, False
                if tr.graph is not None:
                    tr.replay_mode = str(cfg_get(cfg, "runtime.replay", "streams"))
                    loader.out = tr._static_x  # later batches are augmented in place
                    if rank == 0:
                        log.info("step %d: training step captured; replay mode %s", step_global,
                                 "streams" if (tr.replay_mode == "streams"
                                               and tr.sreplay is not None) else "graph")
            loss = tr.step(x)
            nsteps += 1
            step_global += 1
            if log_every and rank == 0 and step_global % log_every == 0:
                log.info("step %d loss %.4f", step_global, float(loss))
            if prof is not None and step_global >= prof_win[1]:
                _stop_profiler(prof, rank)
                prof = None
            if max_steps is not None and step_global >= max_steps:
                done = True
                break
        if st.device.type == "cuda":
            torch.cuda.synchronize()
        dt = max(time.time() - t0, 1e-9)
        tr.guard.flush(step_global)  # the epoch's last step (its flag copy has landed)
        if st.world_size > 1:
            # data-parallel invariant: master, shadow, momentum, step counter and BatchNorm
            # buffers bitwise equal on every rank (a mis-replayed collective or a rank-local
            # statistics error would otherwise surface only as a bad accuracy)
            require_replicas(tr.store, tr.opt, tr.model, group=st.group,
                             where=f"after epoch {epoch}")
        imgs = nsteps * cfg["experiment"]["batches"] * st.world_size
        summary.update(epochs_run=summary["epochs_run"] + 1, steps=step_global)
        if rank == 0:
            lval = float(loss.item())
            lr = tr.opt.logged_lr
            logging.info("Epoch:{}/{} progress:{:.3f} loss:{:.3f}, lr:{:.7f}".format(
                epoch, epochs, epoch / epochs, lval, lr))
            metrics.write(epoch=epoch, step=step_global, loss=lval, lr=lr,
                          images_per_sec=imgs / dt, seconds=dt)
            summary.update(loss=lval, lr=lr, images_per_sec=imgs / dt)
            if epoch % save_every == 0:
                save_reference_checkpoint(tr.model, checkpoint_name(
                    epoch, cfg["experiment"]["output_model_name"]))
                if cfg_get(cfg, "runtime.save_resume", True):
                    save_resume("resume-{}.pt".format(epoch), tr.model, tr.opt, epoch,
                                loader.counter, group=st.group if st.world_size > 1 else None)
        elif epoch % save_every == 0 and cfg_get(cfg, "runtime.save_resume", True):
            gather_rng_states(dst=0, group=st.group)  # rank 0's resume file holds every rank's
        if st.world_size > 1:
            # no rank starts the next epoch's first exchange while rank 0 is still logging /
            # saving (a multi-second save would exceed the IPC exchange's spin bound)
            dist.barrier(group=st.group)
        if done:
            break
    if prof is not None:
        _stop_profiler(prof, rank)
    summary["wall_seconds"] = time.time() - t_start
    metrics.close()
    return summary


# eager steps before the step is captured (runtime.hip_graph auto / true)
GRAPH_AFTER = 2


def _graph_mode(v) -> str:
    """``runtime.hip_graph``: auto (default: capture + native replay on the HIP path, eager if
    the capture fails), true (capture, a failure is an error), false (eager issue)."""
    if isinstance(v, bool):
        return "on" if v else "off"
    v = str(v).strip().lower()
    if v in ("false", "0", "off", "none", "null", "no", "eager"):
        return "off"
    if v in ("true", "1", "on", "yes"):
        return "on"
    if v == "auto":
        return "auto"
    raise ValueError(f"runtime.hip_graph must be auto, true or false, not {v!r}")


def _ints(spec):
    # "A-B-C" (a YAML string; "A:B" would be read as a base-60 integer) or a [A, B, C] list
    if isinstance(spec, (list, tuple)):
        return [int(v) for v in spec]
    return [int(v) for v in str(spec).replace(",", "-").split("-")]


def parse_fault(spec):
    """``"RANK-STEP[-CODE]"`` → (rank, step, exit code) or None (failure-detection tests)."""
    if spec is None or spec == "":
        return None
    parts = _ints(spec)
    return parts[0], parts[1], parts[2] if len(parts) > 2 else 13


def parse_window(spec):
    """``"A-B"`` → the global-step window [A, B) traced by torch.profiler, or None."""
    if spec is None or spec == "":
        return None
    a, b = _ints(spec)[:2]
    return a, b


def _start_profiler():
    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    prof = torch.profiler.profile(activities=acts, record_shapes=False)
    prof.__enter__()
    return prof


def _stop_profiler(prof, rank: int) -> None:
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    prof.__exit__(None, None, None)
    path = f"trace-rank{rank}.json"
    prof.export_chrome_trace(path)
    log.info("torch.profiler trace written to %s", path)
