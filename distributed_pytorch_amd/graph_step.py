"""The training step as a HIP graph (stream capture + replay) instead of ~110 Python-issued launches.

The engine's step is a static schedule over persistent buffers, so once the warm-up steps have
sized every workspace, one capture of forward + backward (both streams: the wgrad stream joins
the capture through its dependency events) + gradient sync + fused SGD replays the whole step with
one host call.  Only the batch fetch runs eagerly: the on-device augmentation writes into the
loader's fixed input buffers, which the graph reads.

Scope (by construction, checked at construction time):
* single-rank communicator: with a real communicator the collectives, their watchdog events and
  the DDP buffer broadcast stay eager (``ValueError``);
* full batches only (a partial last batch runs the eager step);
* the learning rate / momentum / weight decay are baked into the graph: ``recapture()`` after
  changing them.
The first ``warmup`` steps run eagerly (the first SGD step initialises the momentum buffers with
a different kernel argument, and the split-K workspaces are allocated lazily).
"""
from __future__ import annotations

from typing import Iterator, Optional, Tuple

import torch


class GraphedStep:
    def __init__(self, engine, sync, loader=None, warmup: int = 2, fallback: bool = False):
        if engine.device.type != "cuda":
            raise ValueError("GraphedStep needs a GPU engine")
        if sync.active:
            raise ValueError("GraphedStep captures single-rank steps only (collectives run eagerly)")
        self.engine, self.sync, self.loader = engine, sync, loader
        self.warmup = max(1, warmup)
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self._x = self._t = None
        self._it: Optional[Iterator[Tuple[torch.Tensor, torch.Tensor]]] = None
        self.replays = 0
        self.fallback = fallback  # on a failed capture run eagerly instead of raising
        self.failed = False

    def _body(self, x: torch.Tensor, t: torch.Tensor):
        s = self.sync
        s.begin_step()
        self.engine.forward_backward(x, t, grad_ready=s.grad_ready, pre_forward=s.pre_forward,
                                     params_free=s.params_free)
        s.update(s.finish())

    def recapture(self):
        self.graph = None

    def run(self, x: torch.Tensor, t: torch.Tensor):
        """One training step on (x, t); (x, t) must be the loader's persistent buffers."""
        e = self.engine
        full = x.shape[0] == e.max_batch
        if self.graph is not None and full:
            if x.data_ptr() != self._x.data_ptr() or t.data_ptr() != self._t.data_ptr():
                raise ValueError("GraphedStep: the batch must live in the buffers the graph was captured on")
            self.graph.replay()
            self.replays += 1
        elif not full or e.steps_taken < self.warmup:
            self._body(x, t)
        elif self.failed:
            self._body(x, t)
        else:
            torch.cuda.synchronize(e.device)
            g = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(g):
                    self._body(x, t)
            except RuntimeError as err:  # capture refused: keep training eagerly, say so once
                if not self.fallback:
                    raise
                self.failed = True
                print(f"[GraphedStep] stream capture failed ({err}); running the step eagerly", flush=True)
                torch.cuda.synchronize(e.device)
                self._body(x, t)
                e.finish_step()
                return
            self.graph, self._x, self._t = g, x, t
            g.replay()  # capture records only: this replay performs the step
            self.replays += 1
        e.finish_step()

    def _batches(self):
        ep = self.loader.epoch
        while True:
            self.loader.set_epoch(ep)
            yield from self.loader
            ep += 1

    def step(self):
        """Fetch the next batch from the loader (eager augmentation) and run one step."""
        if self._it is None:
            if self.loader is None:
                raise ValueError("GraphedStep.step() needs a loader")
            self._it = self._batches()
        x, t = next(self._it)
        self.run(x, t)
